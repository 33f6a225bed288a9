// wave_ops.h -- wavefront-64 reductions for gfx950 without LDS round trips.
//
// __shfl_xor lowers to ds_bpermute (an LDS-path round trip per 32-bit half); a double
// reduction over 64 lanes then costs ~12 of them.  Here each 16-lane row is reduced with
// DPP lane moves (quad_perm xor1, quad_perm xor2, row_half_mirror, row_mirror: every lane
// of a row ends with the row result, the same bits on every lane), then the four row results
// are combined in a fixed order by DPP row broadcasts into lane 63 and read from there.  The
// combine order is fixed, so the result is bit-identical on every lane and every run.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace twosd {

// DPP controls (GFX9 encoding)
constexpr int kDppXor1 = 0xB1;        // quad_perm(1,0,3,2)
constexpr int kDppXor2 = 0x4E;        // quad_perm(2,3,0,1)
constexpr int kDppHalfMirror = 0x141; // row_half_mirror
constexpr int kDppMirror = 0x140;     // row_mirror

// (the quad permutes and mirrors read a valid lane for every lane: no old value to preset)
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const int lo = dpp_i<CTRL>((int)(uint32_t)u);
    const int hi = dpp_i<CTRL>((int)(uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ double readlane_dbl(double v, int lane) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// sum over the 64 lanes; every lane returns the same bits (uniform)

// arg-reduction: the lane with the largest key (ties: smallest idx); returns the winning
// idx (uniform) and the payload values of that lane.  Lanes without a candidate pass
// key = -inf / idx = INT_MAX.
struct ArgBest {
    double key;
    int idx;
    double p0, p1;
};
template <int CTRL>
__device__ __forceinline__ void arg_step(double &key, int &idx, double &p0, double &p1) {
    const double k2 = dpp_d<CTRL>(key);
    const int i2 = dpp_i<CTRL>(idx);
    const double a2 = dpp_d<CTRL>(p0);
    const double b2 = dpp_d<CTRL>(p1);
    if (k2 > key || (k2 == key && i2 < idx)) { key = k2; idx = i2; p0 = a2; p1 = b2; }
}
__device__ __forceinline__ ArgBest warg_max(double key, int idx, double p0, double p1) {
    arg_step<kDppXor1>(key, idx, p0, p1);
    arg_step<kDppXor2>(key, idx, p0, p1);
    arg_step<kDppHalfMirror>(key, idx, p0, p1);
    arg_step<kDppMirror>(key, idx, p0, p1);
    ArgBest b{readlane_dbl(key, 0), __builtin_amdgcn_readlane(idx, 0), readlane_dbl(p0, 0), readlane_dbl(p1, 0)};
#pragma unroll
    for (int l = 16; l < 64; l += 16) {
        const double k2 = readlane_dbl(key, l);
        const int i2 = __builtin_amdgcn_readlane(idx, l);
        if (k2 > b.key || (k2 == b.key && i2 < b.idx)) {
            b.key = k2; b.idx = i2; b.p0 = readlane_dbl(p0, l); b.p1 = readlane_dbl(p1, l);
        }
    }
    return b;
}

// the same with one payload value
struct ArgBest1 {
    double key;
    int idx;
    double p0;
};
template <int CTRL>
__device__ __forceinline__ void arg_step1(double &key, int &idx, double &p0) {
    const double k2 = dpp_d<CTRL>(key);
    const int i2 = dpp_i<CTRL>(idx);
    const double a2 = dpp_d<CTRL>(p0);
    if (k2 > key || (k2 == key && i2 < idx)) { key = k2; idx = i2; p0 = a2; }
}
// row results carried across rows (GFX9 DPP row_bcast:15 into rows 1 / 3, row_bcast:31 into rows
// 2 / 3; rows outside the row mask keep their own value): lane 63 ends with the wave result
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_bcast_d(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)u, (int)(uint32_t)u, CTRL, ROWS, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(u >> 32), (int)(uint32_t)(u >> 32), CTRL, ROWS, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
// the same with 0 outside the row mask (for sums)
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_bcast0_d(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, ROWS, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, ROWS, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ int dpp_bcast_min_i(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false));
    return min(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false));
}
// sum over the 64 lanes; every lane returns the same bits (uniform).  The row totals meet in
// lane 63 as (r3 + r2) + (r1 + r0) -- the fixed order (r0 + r1) + (r2 + r3) up to commutation,
// which is exact in IEEE arithmetic
__device__ __forceinline__ double wsum(double v) {
    v += dpp_d<kDppXor1>(v);
    v += dpp_d<kDppXor2>(v);
    v += dpp_d<kDppHalfMirror>(v);
    v += dpp_d<kDppMirror>(v);
    v += dpp_bcast0_d<0x142, 0xA>(v);   // rows 1 / 3: + the row 0 / row 2 total
    v += dpp_bcast0_d<0x143, 0xC>(v);   // rows 2 / 3: + lane 31 (rows 0 + 1)
    return readlane_dbl(v, 63);
}

__device__ __forceinline__ double wmin(double v) {
    v = fmin(v, dpp_d<kDppXor1>(v));
    v = fmin(v, dpp_d<kDppXor2>(v));
    v = fmin(v, dpp_d<kDppHalfMirror>(v));
    v = fmin(v, dpp_d<kDppMirror>(v));
    v = fmin(v, dpp_bcast_d<0x142, 0xA>(v));
    v = fmin(v, dpp_bcast_d<0x143, 0xC>(v));
    return readlane_dbl(v, 63);
}

__device__ __forceinline__ double wmax(double v) {
    v = fmax(v, dpp_d<kDppXor1>(v));
    v = fmax(v, dpp_d<kDppXor2>(v));
    v = fmax(v, dpp_d<kDppHalfMirror>(v));
    v = fmax(v, dpp_d<kDppMirror>(v));
    v = fmax(v, dpp_bcast_d<0x142, 0xA>(v));
    v = fmax(v, dpp_bcast_d<0x143, 0xC>(v));
    return readlane_dbl(v, 63);
}

// maximum over the 64 lanes (uniform)
__device__ __forceinline__ double wmax_any(double v) {
    v = fmax(v, dpp_d<kDppXor1>(v));
    v = fmax(v, dpp_d<kDppXor2>(v));
    v = fmax(v, dpp_d<kDppHalfMirror>(v));
    v = fmax(v, dpp_d<kDppMirror>(v));
    v = fmax(v, dpp_bcast_d<0x142, 0xA>(v));
    v = fmax(v, dpp_bcast_d<0x143, 0xC>(v));
    return readlane_dbl(v, 63);
}
// The same selection as the pairwise tree (largest key, ties: smallest idx) from the maximum:
// the lanes holding it by ballot, the lowest such lane, and only when several lanes hold it
// (rare but for the all-zero keys of a finished solve) a minimum over their idx.
__device__ __forceinline__ ArgBest1 warg_max1(double key, int idx, double p0) {
    const double M = wmax_any(key);
    const uint64_t hit = __builtin_amdgcn_ballot_w64(key == M);
    int wl = hit ? (int)__builtin_ctzll(hit) : 0;   // (no hit only for NaN keys)
    int wi = __builtin_amdgcn_readlane(idx, wl);
    if (__builtin_popcountll(hit) > 1) {
        int im = key == M ? idx : 0x7fffffff;
        im = min(im, dpp_i<kDppXor1>(im));   // quad / mirror moves read within the row: old unused
        im = min(im, dpp_i<kDppXor2>(im));
        im = min(im, dpp_i<kDppHalfMirror>(im));
        im = min(im, dpp_i<kDppMirror>(im));
        wi = __builtin_amdgcn_readlane(dpp_bcast_min_i(im), 63);
        const uint64_t h2 = __builtin_amdgcn_ballot_w64((key == M) & (idx == wi));
        wl = h2 ? (int)__builtin_ctzll(h2) : 0;
    }
    return ArgBest1{M, wi, readlane_dbl(p0, wl)};
}

}  // namespace twosd
