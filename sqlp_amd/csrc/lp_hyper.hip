// lp_hyper.hip -- hypersparse batched dual simplex for the stage-2 LPs (gfx950).
//
// Bounded dual simplex for solve_problem! (src/smps/smps_routines.jl:50-62), one
// 64-lane wavefront per scenario, built for what the SMPS recourse matrices look like:
// B0^{-1} of storm is 1.2 % dense (about 6 nonzeros per row/column) and the FTRAN
// columns B^{-1} a_q about 1 %, so dense 64R-wide row operations would be ~99 % zeros.
// Here:
//   * B0^{-1} is stored CSC (column c -> (row i, B0^{-1}[i][c])), shared by all waves;
//   * the eta file of a wave is a sparse arena (row index, value) in HBM (L1/L2 hits in
//     practice), its pivot rows and offsets in the wave's LDS slice;
//   * BTRAN: u = e_r' E_K..E_1 with u dense in LDS, each eta a lane-parallel sparse dot;
//     rho_c = sum_i u_i B0^{-1}[i][c] as lane-parallel gathers over B0^{-1} columns;
//   * reduced costs d_j live in registers of the lane that owns column j (j = 64c+lane,
//     C slots, template parameter) and are updated in place (no dual vector, no pi);
//   * FTRAN: scatter of the sparse B0^{-1} columns of a_q, then the sparse etas;
//   * x_B and dual Devex weights stay in registers (row i: lane i%64, slot i/64).
// Pivot rules (dual Devex leaving row, Harris two-pass ratio test, lowest index on ties)
// are those of the C oracle (oracle/cpu_lp.c), so both follow the same pivot path up to
// rounding.
#include <hip/hip_runtime.h>
#include <math.h>
#include <type_traits>
#include "twosd_internal.h"
#include "wave_ops.h"

namespace twosd {

#define HTOL_P 1e-9
#define HTOL_D 1e-9
#define HTOL_PIV 1e-9
#define HPI_ZERO 1e-12


// Diagnostic build (-DTWOSD_STAMPS, libtwosd_hip_stamps.so): per-phase s_memtime cycle
// totals summed over waves.  Never used for timing claims (stamps perturb the schedule).
#ifdef TWOSD_STAMPS
#define STAMP_DECL unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                                      \
    {                                                                 \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
        st_acc[i] += t_ - st_last;                                    \
        st_last = t_;                                                 \
    }
#define STAMP_FLUSH                                                                         \
    if (lane == 0 && P.stamps)                                                              \
        for (int i_ = 0; i_ < 10; ++i_) atomicAdd(&P.stamps[i_], st_acc[i_]);
#elif defined(TWOSD_ISA_MARK)   // assembly inspection only: phase markers as asm comments
#define STAMP_DECL
#define STAMP(i) asm volatile("; TWOSD_PHASE_END " #i);
#define STAMP_FLUSH
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH
#endif

__device__ __forceinline__ double h_wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double h_wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ void h_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// scatter-add into the wave's own LDS slice: ds_add_f64, no return value, so no read-modify-write
// latency chain.  One wave owns the slice and its LDS instructions execute in program order, so
// every address accumulates its terms in a fixed order (deterministic), each term rounded once
// as a product and once in the sum -- the arithmetic of the C oracle's dot products.
__device__ __forceinline__ void lds_add(double *p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
// inclusive scans over the 64 lanes: DPP row shifts within each 16-lane row (lanes shifted in
// from outside the row read 0, bound_ctrl), then the carries of the rows before (row broadcasts)
template <int K>
__device__ __forceinline__ int h_row_shr(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x110 + K, 0xF, 0xF, true);
}
// the row totals carried across rows (GFX9 DPP row_bcast): lane 15 of rows 0 / 2 into rows 1 / 3,
// then lane 31 into rows 2 and 3; rows outside the row mask read 0
__device__ __forceinline__ int h_bcast15(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false); }
__device__ __forceinline__ int h_bcast31(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false); }
__device__ __forceinline__ int h_scan_add(int v) {
    v += h_row_shr<1>(v);
    v += h_row_shr<2>(v);
    v += h_row_shr<4>(v);
    v += h_row_shr<8>(v);
    v += h_bcast15(v);
    return v + h_bcast31(v);
}
__device__ __forceinline__ int h_scan_max(int v) {   // v >= 0
    v = max(v, h_row_shr<1>(v));
    v = max(v, h_row_shr<2>(v));
    v = max(v, h_row_shr<4>(v));
    v = max(v, h_row_shr<8>(v));
    v = max(v, h_bcast15(v));
    return max(v, h_bcast31(v));
}
// Segmented scatter-add: lane j holds a row (entries p0 .. p0 + len - 1 of cidx / cval) and its
// multiplier v; target[cidx[p]] += v * cval[p] over every entry of every row.  The rows are laid
// end to end and consumed 64 entries per wave step (lane l: entry c0 + l), so a row of a few
// entries does not occupy a whole step.  A lane finds its row as the last row start at or
// before its entry (starts marked in the LDS scratch smark[64], all zero on entry and on exit,
// then a max-scan over lanes).  Rows go in lane order across steps; entries of different rows
// that meet in one address within a step are added by one ds_add_f64 in a fixed hardware order.
// Returns the number of entries.
__device__ __forceinline__ int h_seg_scatter(int p0, int len, double v, const int *__restrict__ cidx,
                                             const double *__restrict__ cval, double *target, int *smark, int lane) {
    const int incl = h_scan_add(len);
    const int excl = incl - len;
    const int T = __builtin_amdgcn_readlane(incl, 63);
    const int dd = p0 - excl;   // entry e of the concatenation sits at cidx[dd_row + e]
    int carry = 0;
    for (int c0 = 0; c0 < T; c0 += 64) {
        if (len > 0 && excl >= c0 && excl < c0 + 64) smark[excl - c0] = lane + 1;
        h_wave_sync();
        int mv = smark[lane];
        smark[lane] = 0;
        mv = h_scan_max(mv);
        mv = mv > carry ? mv : carry;
        carry = __builtin_amdgcn_readlane(mv, 63);
        const int j = mv > 0 ? mv - 1 : 0;
        const int dj = __builtin_amdgcn_ds_bpermute(4 * j, dd);
        const uint64_t vb = (uint64_t)__double_as_longlong(v);
        const uint32_t vlo = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * j, (int)(uint32_t)vb);
        const uint32_t vhi = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * j, (int)(uint32_t)(vb >> 32));
        const double vj = __longlong_as_double((long long)(((uint64_t)vhi << 32) | vlo));
        const int e = c0 + lane;
        if (e < T) {
            int ci = cidx[dj + e];
            double cv = cval[dj + e];
            asm volatile("" : "+v"(ci), "+v"(cv));   // both loads in flight before either is used
            lds_add(&target[ci], vj * cv);
        }
    }
    return T;
}
// sign bit of an fp64 value as a 64-bit mask: flip(v, 1) = -v, exactly
__device__ __forceinline__ double h_flip(double v, uint64_t signmask) {
    return __longlong_as_double(__double_as_longlong(v) ^ (long long)signmask);
}

// a wave-uniform value pinned to SGPRs
__device__ __forceinline__ uint32_t h_uniform(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t h_uniform(uint64_t v) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
// register-array element p = 64 * slot + lane (p uniform)
template <int R>
__device__ __forceinline__ int h_get_row_i(const int (&a)[R], int p) {
    // one readlane per slot and a scalar select: a select chain over a[t] is folded by the
    // compiler into a dynamically indexed load, which sends the whole array to scratch
    const int slot = p >> 6;
    int v = 0;
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const int u = __builtin_amdgcn_readlane(a[t], p & 63);
        v = (t == slot) ? u : v;
    }
    return v;
}

// popcount of the bits of m below this lane (v_mbcnt; no per-lane mask register)
__device__ __forceinline__ int h_prefix_count(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// The kernel's argument block read where a field is used: an s_load through a pointer the
// compiler cannot see through, so the per-scenario (prologue / epilogue) fields are not held in
// registers across the pivot loop.  Held there, they outgrow the 102 SGPRs, spill into VGPR lanes
// and from there to scratch, which the 2048 waves' 55 MB of scratch then re-read from HBM on every
// scenario.
__device__ __forceinline__ const __attribute__((address_space(4))) HyperParams *h_args() {
    uint64_t a = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(a));
    return (const __attribute__((address_space(4))) HyperParams *)a;
}
#define CP (*h_args())

// per-wave LDS slice: a union of {ut, rho} (MP doubles each) and alpha (the pivot row over the
// 64C column slots during pricing; the columns past n + m are never scattered to, so every slot
// can be read and zeroed unconditionally), the scenario deltas (k doubles), the pricing list
// values (64 doubles), the pricing list rows and row-start marks (64 ints each), etap (u16),
// etaoff (int)
static __host__ __device__ inline int hyper_union_doubles(int R, int C) {
    return 128 * R > 64 * C ? 128 * R : 64 * C;
}
static __host__ __device__ inline size_t hyper_slice_bytes(int R, int C, int kmax, int k) {
    const int kmaxp = (kmax + 3) & ~3;
    return 8 * (size_t)hyper_union_doubles(R, C) + 8 * (size_t)((k + 1) & ~1) + 8 * 64 + 4 * 64 + 4 * 64 + 2 * kmaxp +
           4 * (kmaxp + 4);
}
size_t hyper_lds_bytes(int R, int C, int kmax, int k) { return (size_t)kWavesPerBlock * hyper_slice_bytes(R, C, kmax, k); }

// min waves per SIMD (VGPR budget 256 / 168): measured on MI355X, storm (R=9) is fastest
// at 2 waves/SIMD, ssn (R=4) at 3 (tools/lp_speed.py)
// loads in flight per memory round trip: etas per group (BTRAN / FTRAN)
#ifndef TWOSD_ETA_G
#define TWOSD_ETA_G 2
#endif
constexpr int EG = TWOSD_ETA_G;
// unroll of the per-scenario gathers (x_B warm start, vertex recovery): loads in flight
#ifndef TWOSD_REC_UNROLL
#define TWOSD_REC_UNROLL 1
#endif
// ELL columns of the x_B warm start per memory round trip
#ifndef TWOSD_XB_U
#define TWOSD_XB_U 1
#endif
constexpr int XU = TWOSD_XB_U;
#ifndef TWOSD_HYPER_WPE
#define TWOSD_HYPER_WPE(R) ((R) >= 9 ? 2 : 3)
#endif

// Reduced costs are kept SIGN-FOLDED: d'_j = s_j d_j with s_j = -1 for the columns nonbasic at
// their upper bound (the slacks of G rows, [-inf, 0]) and +1 otherwise, and the pricing writes
// alpha'_j = s_j alpha~_j (the structural columns have s_j = +1, so only the slack entry of a G
// row flips).  Sign flips are exact and commute with every rounding, so the ratio test on
// (d', alpha') takes exactly the decisions of the unfolded one (C oracle rules):
//   eligible  <=>  s_j a_j > tol              (a_j = sg alpha~_j; was: at lb a > tol, at ub a < -tol)
//   pass 1    nu = d'_j + tol, de = a'_j      (was: d + tol / tol - d, |a|)
//   pass 2    d'_j <= thmax a'_j              (was: a > 0 ? d <= thmax a : d >= thmax a)
//   theta_D = d'_q / a'_q = d_q / a_q,  d'_j -= theta_D a'_j.
// The dual update runs over every slot: basic columns' d' are never read (candidates exclude
// them, an entering column is set to 0, a leaving one to its new value, the dual key masks
// them), and a nonbasic column with alpha = 0 keeps its value (d + 0).
//
// FULL = false: the main solve of solve_push / solve_batch without pi, y, heads, basis keys or
// eta files -- the vertex recovery and the refresh outputs are compiled out (a smaller kernel:
// fewer registers and instruction-cache lines).
template <int R, int C, bool FULL>
__global__ void __launch_bounds__(256, TWOSD_HYPER_WPE(R)) lp_hyper_kernel(HyperParams P) {
    extern __shared__ double lds_raw[];
    using Mask = typename std::conditional<(C > 32), uint64_t, uint32_t>::type;
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    constexpr int MP = 64 * R;
    constexpr int UD = 128 * R > 64 * C ? 128 * R : 64 * C;
    const int kmaxp = (P.kmax + 3) & ~3;
    const int ncol = P.n + P.m;
    char *slice = reinterpret_cast<char *>(lds_raw) + (size_t)wid * hyper_slice_bytes(R, C, P.kmax, P.k);
    double *ut = reinterpret_cast<double *>(slice);        // dense scratch vector (u, then alpha_q)
    double *rho = ut + MP;                                  // pivot row of B^{-1}
    double *alpha = ut;                                     // pricing: alpha'_j over the same space
    double *dvl = ut + UD;                                  // this scenario's coef_e(x) dv_e
    double *lstv = dvl + ((P.k + 1) & ~1);                  // pricing list: rho values
    int *lsti = reinterpret_cast<int *>(lstv + 64);         // pricing list: rows
    int *smark = lsti + 64;                                 // pricing: row starts within a wave step
    unsigned short *etap = reinterpret_cast<unsigned short *>(smark + 64);
    int *etaoff = reinterpret_cast<int *>(etap + kmaxp);

    const int m = P.m, n = P.n;
    const int slot_id = blockIdx.x * kWavesPerBlock + wid;
    int *eidx = P.eidx + (size_t)slot_id * P.ecap;
    double *evals = P.evals + (size_t)slot_id * P.ecap;
    const uint64_t fixedm = CP.fixedmask[lane];
    const uint64_t ubm = CP.ubmask[lane];

    for (int j = lane; j < UD; j += 64) ut[j] = 0.0;
    smark[lane] = 0;
    h_wave_sync();
    STAMP_DECL

    // XCD-aware work queues: the visiting order is cut into qgroups contiguous ranges, range g
    // served first by the blocks with blockIdx % qgroups == g (one XCD under the round-robin
    // block placement, speed only), so the waves that share a pool basis share one L2.  A wave
    // whose range is exhausted moves on to the next range (never back: exhausted stays exhausted).
    // The claim of the next queue position, its scenario (order) and its pool pick are three
    // dependent global round trips; they are software-pipelined across scenarios: the claim is
    // issued when a scenario starts and resolved after its x_B loads (which it overlaps), the
    // order load is issued then and resolved after the pivot loop, where the pick load is issued.
    const int G = CP.qgroups;
    const int g0 = blockIdx.x % G;
    int gt = 0;
    auto group_of = [&](int gi) { return g0 + gi < G ? g0 + gi : g0 + gi - G; };
    auto claim_sync = [&]() -> int {   // next position, moving on to the next range when one is exhausted
        for (; gt < G; ++gt) {
            const int g = group_of(gt);
            const int lo = (int)(((long long)P.N * g) / G), hi = (int)(((long long)P.N * (g + 1)) / G);
            int t = 0;
            if (lane == 0) t = atomicAdd(CP.queue + g * kQueueStride, 1);
            t = __builtin_amdgcn_readfirstlane(__shfl(t, 0));
            if (lo + t < hi) return lo + t;
        }
        return -1;
    };
    int q_nx = claim_sync();
    int s_nx = q_nx < 0 ? -1 : (CP.order ? __builtin_amdgcn_readfirstlane(CP.order[q_nx]) : q_nx);
    int pb_nx = (s_nx >= 0 && CP.npool > 1) ? __builtin_amdgcn_readfirstlane(CP.pool_pick[s_nx]) : 0;
    // coef_e(x) dv_e of a scenario into LDS (dvl is read by the x_B gathers only).  With k <= 128
    // the next scenario's deltas are loaded when its index is known (after the pivot loop) and
    // written at the end of the epilogue, so the load overlaps the epilogue
    auto dv_fill = [&](int sn) {
        const double *dvs = CP.dv + (size_t)sn * P.k;
        for (int e = lane; e < P.k; e += 64) dvl[e] = CP.kcoef[e] * dvs[e];
    };
    const bool dv_pf = P.k <= 128;
    if (s_nx >= 0 && dv_pf) dv_fill(s_nx);
    for (;;) {
        if (q_nx < 0) break;
        const int qpos = q_nx;
        int s = s_nx;                                    // grouped by pool basis
        int pb = pb_nx;                                  // warm-start basis (pool_select_kernel; 0 without a pool)
        // claim of the following position, resolved after this scenario's x_B loads
        int t_claim = 0;
        if (lane == 0 && gt < G) t_claim = atomicAdd(CP.queue + group_of(gt) * kQueueStride, 1);

        if (!dv_pf) dv_fill(s);
        h_wave_sync();
        // x_B of pool basis p at this scenario: xbase_p + sum_e coef_e B_p^{-1}[i][row_e] dv_e
        // (sliced ELL by row: independent coalesced loads, deltas gathered from LDS).  The slot
        // bounds arrive in one load; the ELL columns are walked for all slots together (column u
        // of every slot that has one), so each round trip carries up to R independent loads.
        int lnx = lane;   // opaque copy: per-lane address terms of the gathers stay inside the scenario loop
        asm volatile("" : "+v"(lnx));
        double xB[R];
        float wd[R];   // dual Devex weights, row 64t + lane (registers: no LDS round trip per update)
        int hb[R];
        double d[C];   // sign-folded reduced costs d'_j, j = 64c + lane
        uint64_t bmask;
        const int *brptr, *bcp;
        int K = 0, it = 0, status = TWOSD_LP_OPTIMAL;
        int eoff = 0;
        unsigned nops = 0;   // entries processed by this solve (< 2^32: at most kmax pivots of <= a few 10^4 each)
        // a pool start that ends non-optimal (numerics, iteration cap) is retried from the
        // primary basis, so the pool never changes which scenarios solve
        for (int attempt = 0; attempt < 2; ++attempt) {
        {
            // one opaque argument pointer per start: the field loads below are shared within it and
            // dead before the pivot loop
            const auto *A = h_args();
            const int ln = lnx;
            brptr = A->brptr + (size_t)pb * (MP + 1);
            bcp = A->bcp + (size_t)pb * (MP + 1);
            const double *xb = A->xbase + (size_t)pb * MP;
            const double *kv = A->kv;
            const int *kix = A->kix;
            const int ksv = ln <= R ? A->kslot[pb * (R + 1) + ln] : 0;
            int eb[R], len[R];
            int w = 0;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                eb[t] = __builtin_amdgcn_readlane(ksv, t);
                len[t] = __builtin_amdgcn_readlane(ksv, t + 1) - eb[t];
                w = len[t] > w ? len[t] : w;
                xB[t] = xb[64 * t + ln];
                hb[t] = A->hb0[(size_t)pb * MP + 64 * t + ln];
                wd[t] = 1.0f;
            }
            nops += (unsigned)(__builtin_amdgcn_readlane(ksv, R) - eb[0]) * 64u;
            // columns u .. u + XU - 1 of every slot per round trip (all their loads issued before the
            // first is used), applied in increasing u per row: the same fma order as a per-row walk
            for (int u0 = 0; u0 < w; u0 += XU) {
                double kvv[XU][R];
                int kiv[XU][R];
#pragma unroll
                for (int uu = 0; uu < XU; ++uu)
#pragma unroll
                    for (int t = 0; t < R; ++t) {
                        const int u = u0 + uu;
                        kvv[uu][t] = 0.0;
                        kiv[uu][t] = 0;
                        if (u < len[t]) {
                            kvv[uu][t] = kv[(size_t)(eb[t] + u) * 64 + ln];
                            kiv[uu][t] = kix[(size_t)(eb[t] + u) * 64 + ln];
                        }
                    }
#pragma unroll
                for (int uu = 0; uu < XU; ++uu)
#pragma unroll
                    for (int t = 0; t < R; ++t)
                        if (u0 + uu < len[t]) xB[t] = fma(kvv[uu][t], dvl[kiv[uu][t]], xB[t]);
            }
            // the per-slot sign masks from an opaque copy of ubm: hoisted out of the scenario loop
            // they would be 28 loop-invariant 64-bit values, spilled and re-read every scenario
            uint64_t ub = ubm;
            asm volatile("" : "+v"(ub));
#pragma unroll
            for (int c = 0; c < C; ++c)
                d[c] = h_flip(A->d0[(size_t)pb * 64 * C + 64 * c + ln], ((ub >> c) & 1) << 63);
            bmask = A->basic0[pb * 64 + ln];
        }
        K = 0; status = TWOSD_LP_OPTIMAL; eoff = 0;
        if (lane == 0) etaoff[0] = 0;
        h_wave_sync();
        if (attempt == 0) {
            // the claim has returned with the x_B loads: the next position (a range exhausted:
            // claim from the next one, rare), then its scenario's order entry in flight
            if (gt < G) {
                const int g = group_of(gt);
                const int hi = (int)(((long long)P.N * (g + 1)) / G), lo = (int)(((long long)P.N * g) / G);
                const int t = __builtin_amdgcn_readfirstlane(__shfl(t_claim, 0));
                if (lo + t < hi) q_nx = lo + t;
                else { ++gt; q_nx = claim_sync(); }
            } else {
                q_nx = -1;
            }
            if (q_nx >= 0) s_nx = CP.order ? CP.order[q_nx] : q_nx;   // resolved after the pivot loop
        }
        STAMP(0)

        // the first-64 entries of etas t0, t0 + dir, ..., t0 + (EG - 1) dir that exist (0 <= t < K).
        // The loads are issued unconditionally (entry 0 of the arena where there is none), so every
        // group issues the same number of them and the wait for a group prefetched one step earlier
        // leaves the newer group's loads in flight
        auto eta_group = [&](int t0, int dir, int (&gi)[EG], double (&gv)[EG], int (&gn)[EG], int (&go)[EG]) {
#pragma unroll
            for (int g = 0; g < EG; ++g) {
                const int tt = t0 + dir * g;
                const bool ok = (tt >= 0) & (tt < K);
                const int tc = ok ? tt : 0;
                const int o0 = etaoff[tc], o1 = etaoff[tc + 1];
                go[g] = ok ? o0 : 0;
                gn[g] = ok ? o1 - o0 : 0;
                const bool mine = lane < gn[g];
                const int at = mine ? go[g] + lane : 0;
                const int ix = eidx[at];
                const double vx = evals[at];
                gi[g] = mine ? ix : 0;
                gv[g] = mine ? vx : 0.0;
            }
        };
        for (;;) {
            // ---- 1. leaving row (dual Devex: max infeas^2 / w, lowest row on ties)
            // within the lane the rows are compared as fractions (dl^2 * w_best > best_num * w:
            // no division per row), one division for the lane's winner
            double bnum = 0.0, bden = 1.0, bdel = 0.0;
            int br = 0x7fffffff;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                // below -tol counts unless the row is G, above +tol only for G / E (bt & 1);
                // padding rows (hb < 0) never
                const int bt = hb[t] & 3;
                const bool inf = (hb[t] >= 0) & (((xB[t] < -HTOL_P) & (bt != BT_G)) | ((xB[t] > HTOL_P) & ((bt & 1) != 0)));
                if (__builtin_amdgcn_ballot_w64(inf) != 0 && inf) {   // most slots hold no infeasible row
                    const double dl = xB[t];
                    const double num = dl * dl, den = (double)wd[t];
                    if (num * bden > bnum * den) { bnum = num; bden = den; br = 64 * t + lane; bdel = dl; }
                }
            }
            const ArgBest1 lr = warg_max1(bnum / bden, br, bdel);
            const int r = lr.idx;
            STAMP(1)
            if (lr.key == 0.0) break;
            if (K >= P.kcap) { status = TWOSD_LP_ITER_LIMIT; break; }
            const double delta = lr.p0;

            // ---- 2. BTRAN: u = e_r' E_K..E_1 (u dense in LDS), rho = u' B0^{-1}
            if (lane == (r & 63)) ut[r] = 1.0;
            h_wave_sync();
            // etas in groups of EG: the group's entries (first 64 of each) are loaded together, and
            // the next group's loads are issued before this group is applied (two register sets,
            // ping-pong), so the memory round trips overlap the sequential steps
            {
                auto apply = [&](int tg, const int (&gi)[EG], const double (&gv)[EG], const int (&gn)[EG], const int (&go)[EG]) {
#pragma unroll
                    for (int g = 0; g < EG; ++g) {
                        const int tt = tg - g;
                        if (tt < 0) break;
                        const double ug = gv[g] != 0.0 ? ut[gi[g]] : 0.0;
                        // a dead eta: u is zero on all its rows (u holds only r and the pivot rows
                        // set so far), so u . eta_t = 0 and u[p_t] -- one of those rows (the pivot
                        // entry 1 / alpha_r is never zero) -- is zero already: nothing to write.
                        // (Skipped, the pivot row keeps its zero instead of being rewritten with a
                        // zero of either sign; every later use tests u != 0.)
                        if (gn[g] <= 64 && __builtin_amdgcn_ballot_w64(ug != 0.0) == 0) {
                            nops += gn[g];
                            continue;
                        }
                        double acc = ug * gv[g];
                        for (int e = 64 + lane; e < gn[g]; e += 64) acc = fma(ut[eidx[go[g] + e]], evals[go[g] + e], acc);
                        acc = wsum(acc);
                        nops += gn[g];
                        if (lane == 0) ut[etap[tt]] = acc;
                        h_wave_sync();
                    }
                };
                int ai[EG], an[EG], ao[EG], bi[EG], bn[EG], bo[EG];
                double av[EG], bv[EG];
                if (K <= 2 * EG) {   // short file (storm: most solves): one group in flight at a time
                    for (int tg = K - 1; tg >= 0; tg -= EG) {
                        eta_group(tg, -1, ai, av, an, ao);
                        apply(tg, ai, av, an, ao);
                    }
                } else {
                    eta_group(K - 1, -1, ai, av, an, ao);
                    for (int tg = K - 1; tg >= 0;) {
                        eta_group(tg - EG, -1, bi, bv, bn, bo);
                        apply(tg, ai, av, an, ao);
                        tg -= EG;
                        if (tg < 0) break;
                        eta_group(tg - EG, -1, ai, av, an, ao);
                        apply(tg, bi, bv, bn, bo);
                        tg -= EG;
                    }
                }
            }
            STAMP(2)
            // rho = u' B0^{-1} as one segmented scatter over the nonzero rows of u, which sit at r
            // and at the eta pivot rows, in the fixed order r, etap[K-1], ..., etap[0] (64 rows per
            // batch; deterministic accumulation order).  A row that appears again later (pivoted
            // more than once) contributes at its first position only; each row is zeroed after.
            for (int b0 = 0; b0 <= K; b0 += 64) {
                const int jj = b0 + lane;
                const int gp = jj <= K ? (jj == 0 ? r : (int)etap[K - jj]) : -1;
                const int nbt = K + 1 - b0 < 64 ? K + 1 - b0 : 64;
                bool dup = false;
                for (int i = 0; i < nbt - 1; ++i) dup |= (i < lane) & (__builtin_amdgcn_readlane(gp, i) == gp);
                double up = 0.0;
                int p0 = 0, len = 0;
                if (gp >= 0 && !dup) {
                    up = ut[gp];
                    if (up != 0.0) {
                        p0 = brptr[gp];
                        len = brptr[gp + 1] - p0;
                    }
                }
                nops += h_seg_scatter(p0, len, up, P.brcol, P.brval, rho, smark, lane);
                h_wave_sync();
                if (gp >= 0) ut[gp] = 0.0;
                h_wave_sync();
            }
            STAMP(3)

            // ---- 3. pricing: alpha'_j = s_j rho' a_j for every column as a scatter over the
            // nonzeros of rho (~6 % of the rows on storm).  alpha lives in LDS over the ut/rho space
            // (both zero here once rho is in registers).  (A column-wise variant -- dot products over
            // [W I]'s columns -- measured no faster even on ssn's denser rho.)
            double rv[R];
#pragma unroll
            for (int t = 0; t < R; ++t) rv[t] = rho[64 * t + lane];
            h_wave_sync();
#pragma unroll
            for (int t = 0; t < R; ++t) rho[64 * t + lane] = 0.0;
            h_wave_sync();
            // the nonzero rows of rho (ascending) are compacted into the LDS list, 64 per batch, and
            // the batch's W rows (CSR) scattered 64 entries per wave step (h_seg_scatter)
            {
                uint64_t mk[R];
                int tot = 0;
#pragma unroll
                for (int t = 0; t < R; ++t) {
                    mk[t] = __ballot(rv[t] != 0.0);
                    tot += __popcll(mk[t]);
                }
                for (int b0 = 0; b0 < tot; b0 += 64) {
                    int base = -b0;
#pragma unroll
                    for (int t = 0; t < R; ++t) {
                        const int pos = base + h_prefix_count(mk[t]);
                        if (rv[t] != 0.0 && pos >= 0 && pos < 64) {
                            lsti[pos] = 64 * t + lane;
                            lstv[pos] = rv[t];
                        }
                        base += __popcll(mk[t]);
                    }
                    h_wave_sync();
                    const int nb = tot - b0 < 64 ? tot - b0 : 64;
                    int p0 = 0, len = 0;
                    double gr = 0.0;
                    if (lane < nb) {
                        const int gi = lsti[lane];
                        gr = lstv[lane];
                        p0 = P.wcp[gi];
                        len = P.wcp[gi + 1] - p0;
                        // slack of row i: entry 1 in row i only, folded by its sign (G row: -1)
                        alpha[n + gi] = P.btype[n + gi] == BT_G ? -gr : gr;
                    }
                    nops += h_seg_scatter(p0, len, gr, P.wcc, P.wcv, alpha, smark, lane) + nb;
                    h_wave_sync();   // the list is rewritten by the next batch
                }
            }
            h_wave_sync();
            STAMP(4)

            // Harris ratio test over the nonbasic columns (d' in registers, alpha' from LDS), branch
            // free per slot; the alpha' of slot c + 1 is read while slot c is tested.
            // pass 1: thmax = min over the eligible columns of (d'_j + tol) / a'_j, compared as
            // fractions within the lane (nu * de_best < nu_best * de), one division per lane
            const uint64_t sgm = delta > 0 ? 0ull : (1ull << 63);   // a = sg alpha
            const Mask cand = (Mask)~(bmask | fixedm);
            // A slot (64 columns) with no eligible column is skipped after its test (wave-uniform
            // branch), and the slots with any nonzero alpha' are noted for the dual update: on
            // storm ~9 of the 28 slots hold an eligible column and ~18 a nonzero alpha' per pivot.
            double bnu = INFINITY, bde = 1.0;
            Mask elm = 0, sel = 0, snz = 0;
            double apf = alpha[lane];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const double av = apf;
                if (c + 1 < C) apf = alpha[64 * (c + 1) + lane];
                const double a = h_flip(av, sgm);
                const bool el = (((cand >> c) & 1) != 0) & (a > HTOL_PIV);
                // folded now (readfirstlane: an SGPR value): deferred, the 28 ballots stay live and spill
                snz = h_uniform(snz | ((Mask)(__builtin_amdgcn_ballot_w64(av != 0.0) != 0) << c));
                if (__builtin_amdgcn_ballot_w64(el) != 0) {
                    sel |= (Mask)1 << c;
                    const double nu = d[c] + HTOL_D;
                    const bool better = el & (nu * bde < bnu * a);
                    bnu = better ? nu : bnu;
                    bde = better ? a : bde;
                    elm |= (Mask)el << c;
                }
                // one slot at a time: unscheduled, the 28 slots' LDS reads are hoisted together and
                // the register pressure spills d[] for the whole pivot loop
                __builtin_amdgcn_sched_barrier(0);
            }
            const double thmax = wmin(bnu / bde);
            if (thmax == INFINITY) {
                status = TWOSD_LP_INFEASIBLE;
                h_wave_sync();
#pragma unroll
                for (int c = 0; c < C; ++c) alpha[64 * c + lane] = 0.0;
                break;
            }
            // pass 2: among the eligible columns with d'_j <= thmax a'_j the largest a'_j (lowest
            // column on ties)
            double bA = 0.0, bD = 0.0;
            int bq = 0x7fffffff;
            apf = alpha[lane];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const double av = apf;
                if (c + 1 < C) apf = alpha[64 * (c + 1) + lane];
                if ((sel >> c) & 1) {
                    const double a = h_flip(av, sgm);
                    const bool ok = (((elm >> c) & 1) != 0) & (d[c] <= thmax * a) & (a > bA);
                    bA = ok ? a : bA;
                    bD = ok ? d[c] : bD;
                    bq = ok ? 64 * c + lane : bq;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            const ArgBest1 eq = warg_max1(bA, bq, bD);
            const int q = eq.idx;
            STAMP(5)
            if (eq.key == 0.0) {
                status = TWOSD_LP_NUMERIC;
                h_wave_sync();
#pragma unroll
                for (int c = 0; c < C; ++c) alpha[64 * c + lane] = 0.0;
                break;
            }
            const double thetaD = eq.p0 / eq.key;   // d'_q / a'_q = d_q / a_q
            // d'_j -= thetaD a'_j over the slots with a nonzero alpha', alpha back to zero (ut / rho
            // all zero after); an all-zero slot would leave d' unchanged but for the sign of a zero
            apf = alpha[lane];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const double av = apf;
                if (c + 1 < C) apf = alpha[64 * (c + 1) + lane];
                if ((snz >> c) & 1) {
                    alpha[64 * c + lane] = 0.0;
                    d[c] = fma(-thetaD, h_flip(av, sgm), d[c]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            h_wave_sync();
            STAMP(6)

            // ---- 4. FTRAN: ut = E_K..E_1 B0^{-1} a_q (ut is all zeros here): the CSC columns of
            // B0^{-1} under the nonzeros of a_q as one segmented scatter (lane j: nonzero np0 + j),
            // 64 nonzeros per batch, then the etas
            {
                const int np0 = q >= n ? 0 : P.colptr[q], np1 = q >= n ? 1 : P.colptr[q + 1];
                for (int pw0 = np0; pw0 < np1; pw0 += 64) {
                    const int pw = pw0 + lane;
                    int p0 = 0, len = 0;
                    double fa = 0.0;
                    if (pw < np1) {
                        const int cc = q >= n ? q - n : P.rowidx[pw];
                        fa = q >= n ? 1.0 : P.val[pw];
                        p0 = bcp[cc];
                        len = bcp[cc + 1] - p0;
                    }
                    nops += h_seg_scatter(p0, len, fa, P.bci, P.bcv, ut, smark, lane);
                }
            }
            h_wave_sync();
            {
                auto apply = [&](int tg, const int (&gi)[EG], const double (&gv)[EG], const int (&gn)[EG], const int (&go)[EG]) {
#pragma unroll
                    for (int g = 0; g < EG; ++g) {
                        const int tt = tg + g;
                        if (tt >= K) break;
                        const int p = etap[tt];
                        const double vp = ut[p];
                        if (vp != 0.0) {
                            // the pivot row p is replaced, the others accumulate (distinct rows)
                            if (lane < gn[g]) {
                                if (gi[g] == p) ut[p] = gv[g] * vp;
                                else lds_add(&ut[gi[g]], gv[g] * vp);
                            }
                            for (int e = 64 + lane; e < gn[g]; e += 64) {
                                const int i = eidx[go[g] + e];
                                const double ev = evals[go[g] + e];
                                if (i == p) ut[p] = ev * vp;
                                else lds_add(&ut[i], ev * vp);
                            }
                            nops += gn[g];
                            h_wave_sync();   // (an eta that wrote nothing needs no ordering)
                        }
                    }
                };
                int ai[EG], an[EG], ao[EG], bi[EG], bn[EG], bo[EG];
                double av[EG], bv[EG];
                if (K <= 2 * EG) {
                    for (int tg = 0; tg < K; tg += EG) {
                        eta_group(tg, 1, ai, av, an, ao);
                        apply(tg, ai, av, an, ao);
                    }
                } else {
                    eta_group(0, 1, ai, av, an, ao);
                    for (int tg = 0; tg < K;) {   // ping-pong: the next group in flight while one is applied
                        eta_group(tg + EG, 1, bi, bv, bn, bo);
                        apply(tg, ai, av, an, ao);
                        tg += EG;
                        if (tg >= K) break;
                        eta_group(tg + EG, 1, ai, av, an, ao);
                        apply(tg, bi, bv, bn, bo);
                        tg += EG;
                    }
                }
            }
            const double arq = ut[r];
            double col[R];
#pragma unroll
            for (int t = 0; t < R; ++t) col[t] = ut[64 * t + lane];
            h_wave_sync();
#pragma unroll
            for (int t = 0; t < R; ++t) ut[64 * t + lane] = 0.0;
            STAMP(7)
            if (fabs(arq) < 1e-12) { status = TWOSD_LP_NUMERIC; h_wave_sync(); break; }

            // ---- 5. updates: primal, Devex, sparse eta, basis, reduced costs of q / leaving
            const double thetaP = delta / arq;
            const double inv_arq = 1.0 / arq;
            float wrr = 0.0f;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const float u = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, wd[t]), r & 63));
                wrr = (t == (r >> 6)) ? u : wrr;
            }
            int cnt = 0;
#pragma unroll
            for (int t = 0; t < R; ++t) cnt += __popcll(__ballot(col[t] != 0.0));
            if (eoff + cnt > P.ecap) { status = TWOSD_LP_ITER_LIMIT; h_wave_sync(); break; }
            // per slot: the eta entry (stores under the nonzero mask), x_B and the Devex weight by
            // selects (row r: thetaP and max(wrr / arq^2, 1); others with col != 0: x_B - thetaP col,
            // max(w, ratio^2 wrr))
            int base = eoff;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const int i = 64 * t + lane;
                const bool nz = col[t] != 0.0;
                const bool isr = i == r;
                const uint64_t bal = __ballot(nz);
                const double ratio = col[t] * inv_arq;
                if (nz) {
                    const int pos = base + h_prefix_count(bal);
                    eidx[pos] = i;
                    evals[pos] = isr ? inv_arq : -ratio;
                }
                const float nw = (float)((double)wrr * inv_arq * inv_arq);
                const float cand = (float)(ratio * ratio * (double)wrr);
                const double xo = fma(-thetaP, col[t], xB[t]);
                xB[t] = isr ? thetaP : (nz ? xo : xB[t]);
                wd[t] = isr ? (nw > 1.0f ? nw : 1.0f) : ((nz & (cand > wd[t])) ? cand : wd[t]);
                base += __popcll(bal);
            }
            eoff += cnt;
            if (lane == 0) {
                etap[K] = (unsigned short)r;
                etaoff[K + 1] = eoff;
            }
            ++K;
            const int lh = h_get_row_i<R>(hb, r);
            const int leaving = lh >> 2;
            // reduced cost of the leaving variable: -sg thetaD, folded by its sign (a G-row
            // slack leaves to its upper bound 0: s = -1); of q: 0
            {
                const int ls = leaving >> 6, qs = q >> 6;
                const double dlv = (delta > 0) == ((lh & 3) == BT_G) ? thetaD : -thetaD;
                const bool lme = lane == (leaving & 63), qme = lane == (q & 63);
                // one slot each (ls, qs uniform): scalar branches, two selects in all
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    if (c == ls) d[c] = lme ? dlv : d[c];
                    if (c == qs) d[c] = qme ? 0.0 : d[c];
                }
                if (lme) bmask &= ~(1ull << ls);
                if (qme) bmask |= 1ull << qs;
                if (lane == (r & 63)) {
                    const int rs = r >> 6;
                    const int nh = q * 4 + (int)P.btype[q];
#pragma unroll
                    for (int t = 0; t < R; ++t) {
                        int v = (t == rs) ? nh : hb[t];
                        asm volatile("" : "+v"(v));   // per-slot select kept: no dynamic store into hb
                        hb[t] = v;
                    }
                }
            }
            ++it;
            h_wave_sync();
            STAMP(8)
        }
        if (attempt == 0 && q_nx >= 0) {   // the next scenario and its pool pick (in flight over the epilogue)
            s_nx = __builtin_amdgcn_readfirstlane(s_nx);
            if (CP.npool > 1) pb_nx = CP.pool_pick[s_nx];
        }
        if (status == TWOSD_LP_OPTIMAL || pb == 0 || !CP.retry) break;
        if (lane == 0 && CP.retries) atomicAdd(CP.retries, 1ull);   // rare: counted for the bench line
        pb = 0;
        }   // attempt
        // the next scenario's coef_e and dv_e, e = lane, lane + 64 (multiplied at the LDS write)
        double dvn0 = 0.0, dvn1 = 0.0, kcn0 = 0.0, kcn1 = 0.0;
        if (dv_pf && q_nx >= 0) {
            const auto *A = h_args();
            const double *dvs = A->dv + (size_t)s_nx * P.k;
            if (lane < P.k) { dvn0 = dvs[lane]; kcn0 = A->kcoef[lane]; }
            if (lane + 64 < P.k) { dvn1 = dvs[lane + 64]; kcn1 = A->kcoef[lane + 64]; }
        }

        // ---- objective, dual-vertex key, vertex recovery pi = c_B' B^{-1}
        double objv = NAN;
        if (status == TWOSD_LP_OPTIMAL) {
            // the q_j of all slots loaded together (one pointer, clamped indices), summed in slot order
            const double *qc = CP.q;
            double qv[R];
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const int j = hb[t] >> 2;
                qv[t] = qc[(hb[t] >= 0 && j < n) ? j : 0];
            }
            double ob = 0.0;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const int j = hb[t] >> 2;
                ob = (hb[t] >= 0 && j < n) ? fma(qv[t], xB[t], ob) : ob;
            }
            objv = wsum(ob);
            if (CP.vkey) {
                // key of the dual: pi_i = -d_{n+i} is the reduced cost of row i's slack, kept
                // current in registers by every pivot (fixed E-row slacks included; unfolded here,
                // basic slacks 0).  Components at or below key_zero (1 + max) are snapped to zero --
                // the threshold of the exact recovery (HPI_ZERO), so a component the recovered pi
                // keeps also separates the keys -- and the rest rounded to 24 significant bits; the
                // key is the order-independent sum of mix64(row, bits).
                // Scenarios with equal keys have duals equal to ~2^-23 relative -- the same vertex
                // up to rounding noise, so their exactly recovered pi push as equal vectors
                // (16-bit rule, dual_set.jl:24-53).  A vertex split over two keys only costs one
                // more re-solved representative; the push dedup still merges it.
                // d_j of row i's slack (nonbasic; basic: 0), unfolded (ub: opaque copy, as at the load)
                uint64_t ub = ubm;
                int lane = threadIdx.x & 63;   // opaque copies: the per-slot column terms of the key are
                asm volatile("" : "+v"(ub), "+v"(lane));   // not hoisted out of the scenario loop (spills)
                auto dk = [&](int c) -> double {
                    const int j = 64 * c + lane;
                    const bool slack = (j >= n) & (j < ncol) & (((bmask >> c) & 1) == 0);
                    return slack ? h_flip(d[c], ((ub >> c) & 1) << 63) : 0.0;
                };
                double pm = 0.0;
#pragma unroll
                for (int c = 0; c < C; ++c) pm = fmax(pm, fabs(dk(c)));
                pm = wmax(pm);
                const double zt = CP.key_zero * (1.0 + pm);
                unsigned long long h = 0;
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const int j = 64 * c + lane;
                    if (j >= n && j < ncol) {
                        const double dc = dk(c);
                        const double v = fabs(dc) <= zt ? 0.0 : dc;
                        // sign, exponent and 23 mantissa bits (35 bits) next to the row (< 2^24)
                        const unsigned long long b = ((unsigned long long)__double_as_longlong(v) + (1ull << 28)) >> 29;
                        h += mix64(((unsigned long long)(j - n) << 35) | b);
                    }
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
                if (lane == 0) CP.vkey[s] = h;
            }
        }
        if constexpr (FULL) {
        if (status == TWOSD_LP_OPTIMAL && (P.pi || P.y)) {
            const double *qc = CP.q;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const int j = hb[t] >> 2;
                const bool bq = hb[t] >= 0 && j < n;
                const double qj = qc[bq ? j : 0];
                ut[64 * t + lane] = bq ? qj : 0.0;
            }
            h_wave_sync();
            for (int tt = K - 1; tt >= 0; --tt) {
                const int off = etaoff[tt], nnz = etaoff[tt + 1] - off;
                double acc = 0.0;
                for (int e = lane; e < nnz; e += 64) acc = fma(ut[eidx[off + e]], evals[off + e], acc);
                acc = wsum(acc);
                nops += nnz;
                if (lane == 0) ut[etap[tt]] = acc;
                h_wave_sync();
            }
            double pv[R];
            double pmax = 0.0;
#pragma unroll
            for (int t = 0; t < R; ++t) {   // lane: column 64t + lane of B^{-1} (CSC, rows ascending)
                const int cc = 64 * t + lane;
                const int e0 = cc < m ? bcp[cc] : 0, e1 = cc < m ? bcp[cc + 1] : 0;
                double a = 0.0;
#pragma unroll TWOSD_REC_UNROLL
                for (int e = e0; e < e1; ++e) a = fma(ut[P.bci[e]], P.bcv[e], a);
                pv[t] = a;
                pmax = fmax(pmax, fabs(a));
            }
            nops += P.bnnz[pb];
            pmax = wmax(pmax);
            const double zt = HPI_ZERO * (1.0 + pmax);
#pragma unroll
            for (int t = 0; t < R; ++t)
                if (fabs(pv[t]) <= zt) pv[t] = 0.0;
            h_wave_sync();
#pragma unroll
            for (int t = 0; t < R; ++t) ut[64 * t + lane] = 0.0;
            if (P.pi) {
                double *po = P.pi + (size_t)(P.pi_by_pos ? qpos : s) * m;
#pragma unroll
                for (int t = 0; t < R; ++t)
                    if (64 * t + lane < m) po[64 * t + lane] = pv[t];
            }
            if (P.y) {
                double *yo = P.y + (size_t)s * n;
                for (int j = lane; j < n; j += 64) yo[j] = 0.0;
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int t = 0; t < R; ++t) {
                    const int j = hb[t] >> 2;
                    if (hb[t] >= 0 && j < n) yo[j] = xB[t];
                }
            }
        } else if (status != TWOSD_LP_OPTIMAL && P.pi) {
            double *po = P.pi + (size_t)(P.pi_by_pos ? qpos : s) * m;
#pragma unroll
            for (int t = 0; t < R; ++t)
                if (64 * t + lane < m) po[64 * t + lane] = NAN;
        }
        if (P.head_out) {
            const size_t ho = (size_t)(P.pi_by_pos ? qpos : s) * m;
#pragma unroll
            for (int t = 0; t < R; ++t)
                if (64 * t + lane < m) P.head_out[ho + 64 * t + lane] = hb[t] >> 2;
        }
        if (P.bkey && status == TWOSD_LP_OPTIMAL) {   // the set of basic columns, order-independent
            unsigned long long h = 0;
#pragma unroll
            for (int t = 0; t < R; ++t)
                if (64 * t + lane < m) h += mix64((unsigned long long)(hb[t] >> 2));
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
            if (lane == 0) P.bkey[s] = h;
        }
        if (P.eo_K) {   // eta file of the solve (pool refresh composes B^{-1} = E_K..E_1 B_pb^{-1} from it)
            const int erow = P.pi_by_pos ? qpos : s;
            // 64-bit claim counter: it keeps counting past the arena (a scenario that does not
            // fit gets K = -1) but cannot wrap into a valid offset; eo_cap <= INT32_MAX
            unsigned long long off64 = 0;
            if (lane == 0 && status == TWOSD_LP_OPTIMAL) off64 = atomicAdd(P.eo_used, (unsigned long long)eoff);
            off64 = __shfl(off64, 0);
            const bool ok = status == TWOSD_LP_OPTIMAL && off64 + (unsigned long long)eoff <= (unsigned long long)P.eo_cap;
            const int off = ok ? (int)off64 : 0;
            if (ok) {
                for (int e = lane; e < eoff; e += 64) {
                    P.eo_eidx[off + e] = eidx[e];
                    P.eo_evals[off + e] = evals[e];
                }
                for (int t = lane; t < K; t += 64) P.eo_etap[(size_t)erow * P.kmax + t] = etap[t];
                for (int t = lane; t <= K; t += 64) P.eo_etaoff[(size_t)erow * (P.kmax + 1) + t] = etaoff[t];
            }
            if (lane == 0) {
                P.eo_K[erow] = ok ? K : -1;
                P.eo_off[erow] = off;
                P.eo_pb[erow] = pb;
            }
        }
        }   // FULL
        if (lane == 0) {
            CP.obj[s] = objv;
            CP.status[s] = status;
            CP.iters[s] = it;
            if (CP.ops) CP.ops[s] = (long long)nops;
            if (CP.etan) CP.etan[s] = eoff;   // the eta-arena entries this solve wrote (12 B each)
            if (CP.npool > 1) CP.pool_pick[s] = pb;   // 0 if the pool start was retried
        }
        if (dv_pf && q_nx >= 0) {
            if (lane < P.k) dvl[lane] = kcn0 * dvn0;
            if (lane + 64 < P.k) dvl[lane + 64] = kcn1 * dvn1;
        }
        h_wave_sync();
        pb_nx = __builtin_amdgcn_readfirstlane(pb_nx);
        STAMP(9)
    }
    STAMP_FLUSH
}

// ---- warm-start selection over the basis pool.  Lane = scenario (64 per block, deltas
// staged transposed in LDS), the pool bases split over the block's 4 waves; the sparse
// structure (active rows of every pool basis, their coef_e B_p^{-1}[i][row_e] entries) is
// wave-uniform, so it streams through scalar loads and the per-lane work is LDS reads +
// FMAs.  Key: total primal infeasibility sum_i |infeas(x_B,i)| at b_w (constant rows
// precomputed in cinf); ties: lowest p.
// The selection is a heuristic (any pool basis is a valid start; the choice only changes
// pivot counts), so it runs in fp32: half the LDS traffic of the staged deltas, 8-byte
// records (code, value) -- deterministic like everything else.
// records are sign-folded by pool_selstream_kernel (x' = -x for Y / L basics, x for G, both
// signs for E), so a row's infeasibility is x' when x' > tol
__device__ __forceinline__ float h_viol_f(float x, float cw) { return x > 1e-9f ? x + cw : 0.0f; }

constexpr int kSelWaves = 16;   // 16 waves share one staged scenario tile (latency hiding)
#ifndef TWOSD_SEL_B
#define TWOSD_SEL_B 16           // records per batch of the selection streams (loads in flight)
#endif
constexpr int kSelB = TWOSD_SEL_B;
// Two scenarios per lane: s0 + lane (.x) and s0 + 64 + lane (.y), 128 per block.  The staged
// deltas are (x, y) pairs, so one ds_read_b64 (2 LDS cycles per wave, as a ds_read_b32) and one
// v_pk_fma_f32 serve both.  The arithmetic per scenario is that of one scenario per lane (same
// fp32 fma and adds, same order), so the picks are identical to it (same pivots per x in the
// bench A/B); measured on storm 1M: 11.2 -> 10.3 ms per step with 16-record batches.  The
// kernels are SALU-bound on the wave-uniform record streams (SALU 2x VALU instructions).
typedef float sel_f2 __attribute__((ext_vector_type(2)));
constexpr int kSelTile = 128;
__device__ __forceinline__ sel_f2 h_viol_f2(sel_f2 x, float cw) {
    sel_f2 r;
    r.x = h_viol_f(x.x, cw);
    r.y = h_viol_f(x.y, cw);
    return r;
}
// stage the k deltas of tile scenarios 0..127 (scenario sl at dv row srow(sl); nv valid) as
// pairs: element e of lane l = (scenario l, scenario 64 + l)
template <typename RowOf>
__device__ __forceinline__ void h_stage_pairs(float *dvt, const double *__restrict__ dv, const double *__restrict__ kcoef,
                                              int k, int nv, RowOf srow) {
    for (int idx = threadIdx.x; idx < kSelTile * k; idx += 64 * kSelWaves) {
        const int sl = idx / k, e = idx - sl * k;
        dvt[2 * (e * 65 + (sl & 63)) + (sl >> 6)] = sl < nv ? (float)(kcoef[e] * dv[(size_t)srow(sl) * k + e]) : 0.0f;
    }
}
// byte address of the staged pair of element `off` (the record's byte offset e * 65 * 8; row starts
// carry -1 and read element 0) for this lane, computed on the VALU: the record streams are
// wave-uniform, so on the scalar unit every record's address would add two SALU instructions to
// a loop that is SALU-bound already
__device__ __forceinline__ const sel_f2 *h_pair_addr(const sel_f2 *dvt2, int off, int lane8) {
    int o;
    asm("v_max_i32 %0, %1, 0" : "=v"(o) : "s"(off));
    return reinterpret_cast<const sel_f2 *>(reinterpret_cast<const char *>(dvt2) + o + lane8);
}
// one basis' record stream for both scenarios of the lane (records (value bits, byte offset); offset
// < 0: row start), pruned once no scenario of the wave can still win (alive2); returns the pair's
// keys (inf when pruned)
template <typename Alive>
__device__ __forceinline__ sel_f2 h_stream2(const int2 *__restrict__ rec, int j0, int j1, float cinf, float cw,
                                            const sel_f2 *dvt2, int lane, Alive alive2) {
    sel_f2 inf = {cinf, cinf}, x = {0.0f, 0.0f};
    const int lane8 = 8 * lane;
    auto step = [&](int code, float v, sel_f2 dl) {
        if (code < 0) {   // next row: close the previous one
            inf += h_viol_f2(x, cw);
            x = (sel_f2){v, v};
        } else {
            x = __builtin_elementwise_fma((sel_f2){v, v}, dl, x);
        }
    };
    int j = (__ballot(alive2(inf)) == 0) ? j1 : j0;
    for (; j + kSelB <= j1; j += kSelB) {   // batches of records: scalar loads and LDS reads in flight together
        int2 rc[kSelB];
        sel_f2 dl[kSelB];
#pragma unroll
        for (int u = 0; u < kSelB; ++u) rc[u] = rec[j + u];
#pragma unroll
        for (int u = 0; u < kSelB; ++u) dl[u] = *h_pair_addr(dvt2, rc[u].y, lane8);
#pragma unroll
        for (int u = 0; u < kSelB; ++u) step(rc[u].y, __int_as_float(rc[u].x), dl[u]);
        // exact pruning: inf only grows, so once no scenario of the wave can still beat its best,
        // this basis cannot win for any of them
        if (__ballot(alive2(inf)) == 0) return (sel_f2){INFINITY, INFINITY};
    }
    for (; j < j1; ++j) {
        const int2 r = rec[j];
        step(r.y, __int_as_float(r.x), *h_pair_addr(dvt2, r.y, lane8));
    }
    inf += h_viol_f2(x, cw);
    return inf;
}

__global__ void __launch_bounds__(64 * kSelWaves) pool_select_kernel(PoolSelParams S) {
    extern __shared__ float dvt[];   // k x 65 pairs
    const sel_f2 *dvt2 = reinterpret_cast<const sel_f2 *>(dvt);
    __shared__ float bsum[kSelWaves][kSelTile];
    __shared__ int bidx[kSelWaves][kSelTile];
    // best key found so far by any wave, per scenario (keys are >= 0, so the uint order of the
    // fp32 bits is the float order): a wave stops a basis once it is strictly worse than
    // another wave's best for every scenario it holds
    __shared__ unsigned sbest[kSelTile];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar stream loads
    const int s0 = blockIdx.x * kSelTile;
    const int ns = min(kSelTile, S.N - s0);
    h_stage_pairs(dvt, S.dv, S.kcoef, S.k, ns, [&](int sl) { return s0 + sl; });
    if (threadIdx.x < kSelTile) sbest[threadIdx.x] = 0x7f800000u;   // +inf
    __syncthreads();
    sel_f2 best = {INFINITY, INFINITY};
    int bpx = 0, bpy = 0;
    // a scenario can still win with key `inf` only if inf < its own best (lower p wins ties within
    // the wave) and inf <= every other wave's best (ties with other waves are settled at the end)
    auto alive2 = [&](sel_f2 inf) {
        const float ox = __uint_as_float(__hip_atomic_load(&sbest[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        const float oy = __uint_as_float(__hip_atomic_load(&sbest[64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        return (inf.x < best.x && inf.x <= ox) || (inf.y < best.y && inf.y <= oy);
    };
    // blockIdx.y: a contiguous chunk of the pool (several chunks per tile when the batch alone
    // would not fill the GPU; pool_select_merge_kernel merges them)
    const int p_lo = (int)((long long)S.npool * blockIdx.y / gridDim.y), p_hi = (int)((long long)S.npool * (blockIdx.y + 1) / gridDim.y);
    bpx = bpy = p_lo;
    for (int p = p_lo + wid; p < p_hi; p += kSelWaves) {
        const sel_f2 inf = h_stream2(S.rec, S.sptr[p], S.send[p], S.cinf[p], S.cw, dvt2, lane, alive2);
        if (inf.x < best.x) {
            best.x = inf.x;
            bpx = p;
            atomicMin(&sbest[lane], __float_as_uint(inf.x));
        }
        if (inf.y < best.y) {
            best.y = inf.y;
            bpy = p;
            atomicMin(&sbest[64 + lane], __float_as_uint(inf.y));
        }
    }
    bsum[wid][lane] = best.x; bidx[wid][lane] = bpx;
    bsum[wid][64 + lane] = best.y; bidx[wid][64 + lane] = bpy;
    __syncthreads();
    if (wid < 2) {   // wave 0: scenarios 0..63, wave 1: 64..127
        const int sl = 64 * wid + lane;
        if (sl < ns) {
            float b = bsum[0][sl];
            int bp = bidx[0][sl];
            for (int w = 1; w < kSelWaves; ++w) {
                const float v = bsum[w][sl];
                const int pw = bidx[w][sl];
                if (v < b || (v == b && pw < bp)) { b = v; bp = pw; }
            }
            if (gridDim.y == 1) {
                S.pick[s0 + sl] = bp;
                if (S.key) S.key[s0 + sl] = b;
            } else {
                S.ppick[(size_t)blockIdx.y * S.N + s0 + sl] = bp;
                S.pkey[(size_t)blockIdx.y * S.N + s0 + sl] = b;
            }
        }
    }
}

// ---- level 2: 128 consecutive entries of `order` (scenarios sorted by their level-1 pick, so a
// tile holds one or two pick groups) per block; the block's 16 waves share the staged deltas
// and split each group's candidate list (candidate ci on wave ci % 16).  Each candidate streams
// its records wave-uniformly, as in level 1.  Result per scenario: least (key, ci) with the
// level-1 pick as ci = -1, i.e. a candidate replaces the pick only with a strictly smaller key,
// and among equal keys the earlier candidate wins (deterministic).
__global__ void __launch_bounds__(64 * kSelWaves) pool_refine_kernel(PoolRefineParams S) {
    extern __shared__ float dvt[];   // k x 65 pairs
    const sel_f2 *dvt2 = reinterpret_cast<const sel_f2 *>(dvt);
    __shared__ float rkey[kSelWaves][kSelTile];
    __shared__ int rci[kSelWaves][kSelTile];
    __shared__ unsigned sbest[kSelTile];   // best key so far over all waves, per scenario (as in level 1)
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware tile remap: consecutive tiles (the same level-1 pick group, the same candidate
    // record streams) go to blocks b, b + 8, ... which share one XCD's L2 under round-robin
    // placement (speed only; any bijection is correct)
    const int nb = gridDim.x, b = blockIdx.x, xq = nb >> 3, xr = nb & 7, xc = b & 7;
    const int tile = xc * xq + min(xc, xr) + (b >> 3);
    const int t0 = tile * kSelTile;
    const int nv = min(kSelTile, S.N - t0);
    h_stage_pairs(dvt, S.dv, S.kcoef, S.k, nv, [&](int sl) { return S.order[t0 + sl]; });
    const bool vx = lane < nv, vy = 64 + lane < nv;
    const int sx = vx ? S.order[t0 + lane] : 0, sy = vy ? S.order[t0 + 64 + lane] : 0;
    const int px = vx ? S.pick[sx] : -1, py = vy ? S.pick[sy] : -1;
    sel_f2 best = {vx ? S.key[sx] : 0.0f, vy ? S.key[sy] : 0.0f};
    int bcx = -1, bcy = -1;
    if (wid == 0) {
        sbest[lane] = __float_as_uint(best.x);
        sbest[64 + lane] = __float_as_uint(best.y);
    }
    __syncthreads();
    // a candidate can still win for a scenario only below its own best (strict: the level-1
    // pick and earlier candidates of this wave win ties) and not above any other wave's best
    // (ties with other waves are settled by candidate index at the end)
    bool mx = false, my = false;
    auto alive2 = [&](sel_f2 inf) {
        const float ox = __uint_as_float(__hip_atomic_load(&sbest[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        const float oy = __uint_as_float(__hip_atomic_load(&sbest[64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        return (mx && inf.x < best.x && inf.x <= ox) || (my && inf.y < best.y && inf.y <= oy);
    };
    // blockIdx.y: a contiguous chunk of the candidate lists (pool_refine_merge_kernel merges)
    const int c_lo = (int)((long long)S.ncand * blockIdx.y / gridDim.y), c_hi = (int)((long long)S.ncand * (blockIdx.y + 1) / gridDim.y);
    uint64_t todx = __ballot(vx), tody = __ballot(vy);
    while (todx | tody) {
        const int g = todx ? __builtin_amdgcn_readlane(px, __builtin_ctzll(todx))
                           : __builtin_amdgcn_readlane(py, __builtin_ctzll(tody));
        mx = vx && px == g;
        my = vy && py == g;
        todx &= ~__ballot(mx);
        tody &= ~__ballot(my);
        for (int ci = c_lo + wid; ci < c_hi; ci += kSelWaves) {
            const int cb = S.cand[(size_t)g * S.ncand + ci];
            if (cb < 0) break;
            const sel_f2 inf = h_stream2(S.rec, S.sptr[cb], S.send[cb], S.cinf[cb], S.cw, dvt2, lane, alive2);
            if (mx && inf.x < best.x) {
                best.x = inf.x;
                bcx = ci;
                atomicMin(&sbest[lane], __float_as_uint(inf.x));
            }
            if (my && inf.y < best.y) {
                best.y = inf.y;
                bcy = ci;
                atomicMin(&sbest[64 + lane], __float_as_uint(inf.y));
            }
        }
    }
    rkey[wid][lane] = best.x; rci[wid][lane] = bcx;
    rkey[wid][64 + lane] = best.y; rci[wid][64 + lane] = bcy;
    __syncthreads();
    if (wid < 2) {
        const int sl = 64 * wid + lane;
        if (sl < nv) {
            float bk = rkey[0][sl];
            int bc = rci[0][sl];
            for (int w = 1; w < kSelWaves; ++w) {
                const float v = rkey[w][sl];
                const int cw = rci[w][sl];
                if (v < bk || (v == bk && cw >= 0 && (bc < 0 ? false : cw < bc))) { bk = v; bc = cw; }
            }
            const int s = S.order[t0 + sl];
            if (gridDim.y > 1) {
                S.pkey[(size_t)blockIdx.y * S.N + s] = bk;
                S.pci[(size_t)blockIdx.y * S.N + s] = bc;
            } else if (bc >= 0) {
                S.pick[s] = S.cand[(size_t)S.pick[s] * S.ncand + bc];
            }
        }
    }
}

// merges of the chunked selections, per scenario in chunk order: the rules of the in-block merges
// (level 1: least (key, basis); level 2: least key, the level-1 pick (-1) keeps ties, then the
// earlier candidate), so the picks equal those of one chunk
__global__ void pool_select_merge_kernel(int N, int G, const float *__restrict__ pkey, const int *__restrict__ ppick, int *pick,
                                         float *key) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= N) return;
    float b = pkey[s];
    int bp = ppick[s];
    for (int y = 1; y < G; ++y) {
        const float v = pkey[(size_t)y * N + s];
        const int p = ppick[(size_t)y * N + s];
        if (v < b || (v == b && p < bp)) { b = v; bp = p; }
    }
    pick[s] = bp;
    if (key) key[s] = b;
}
__global__ void pool_refine_merge_kernel(int N, int G, int ncand, const float *__restrict__ pkey, const int *__restrict__ pci,
                                         const int *__restrict__ cand, int *pick) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= N) return;
    float bk = pkey[s];
    int bc = pci[s];
    for (int y = 1; y < G; ++y) {
        const float v = pkey[(size_t)y * N + s];
        const int c = pci[(size_t)y * N + s];
        if (v < bk || (v == bk && c >= 0 && (bc < 0 ? false : c < bc))) { bk = v; bc = c; }
    }
    if (bc >= 0) pick[s] = cand[(size_t)pick[s] * ncand + bc];
}

// chunks per tile: enough blocks to fill the GPU (~1024) when the batch alone does not, at least
// kSelWaves bases / candidates per chunk, at most 64 chunks (a rank's 2048 training scenarios at
// N = 8 picking over a 4096-basis pool: 16 tiles x 64 chunks)
static int sel_split(int N, int items) {
    if (getenv("TWOSD_SEL_NOSPLIT")) return 1;   // test hook: one chunk (the picks must not change)
    const int nb = (N + kSelTile - 1) / kSelTile;
    int g = (1024 + nb - 1) / nb;
    g = std::min(g, std::max(1, items / kSelWaves));
    return std::max(1, std::min(g, 64));
}
int pool_select_split(int N, int npool) { return sel_split(N, npool); }
int pool_refine_split(int N, int ncand) { return sel_split(N, ncand); }

hipError_t launch_pool_refine(const PoolRefineParams &p, hipStream_t s) {
    if (p.N <= 0 || p.ncand <= 0) return hipSuccess;
    const int G = p.pkey ? pool_refine_split(p.N, p.ncand) : 1;
    hipLaunchKernelGGL(pool_refine_kernel, dim3((p.N + kSelTile - 1) / kSelTile, G), dim3(64 * kSelWaves), pool_select_lds_bytes(p.k), s, p);
    if (G > 1) hipLaunchKernelGGL(pool_refine_merge_kernel, dim3((p.N + 255) / 256), dim3(256), 0, s, p.N, G, p.ncand, p.pkey, p.pci, p.cand, p.pick);
    return hipGetLastError();
}

size_t pool_select_lds_bytes(int k) { return (size_t)4 * 65 * (kSelTile / 64) * (size_t)std::max(k, 1); }

hipError_t launch_pool_select(const PoolSelParams &p, hipStream_t s) {
    if (p.N <= 0) return hipSuccess;
    const int nb = (p.N + kSelTile - 1) / kSelTile;
    const int G = p.pkey ? pool_select_split(p.N, p.npool) : 1;
    hipLaunchKernelGGL(pool_select_kernel, dim3(nb, G), dim3(64 * kSelWaves), pool_select_lds_bytes(p.k), s, p);
    if (G > 1) hipLaunchKernelGGL(pool_select_merge_kernel, dim3((p.N + 255) / 256), dim3(256), 0, s, p.N, G, p.pkey, p.ppick, p.pick, p.key);
    return hipGetLastError();
}

// ---- dispatch: R in {1,2,4,9,16}, C in {2,4,8,16,32,64}
static const int kHR[] = {1, 2, 4, 9, 16};
static const int kHC[] = {2, 4, 8, 14, 16, 28, 32, 64};   // 14 / 28: ssn / storm exactly (fewer d[] registers)

int hyper_rows_per_lane(int m) {
    for (int R : kHR)
        if (m <= 64 * R) return R;
    return -1;
}
int hyper_cols_per_lane(int ncols) {
    for (int C : kHC)
        if (ncols <= 64 * C) return C;
    return -1;
}

template <int R, int C>
static hipError_t hl(const HyperParams &p, int nb, size_t lds, hipStream_t s) {
    // the lean kernel when the launch asks for none of the recovery / refresh outputs
    if (p.pi || p.y || p.head_out || p.bkey || p.eo_K)
        hipLaunchKernelGGL((lp_hyper_kernel<R, C, true>), dim3(nb), dim3(256), lds, s, p);
    else
        hipLaunchKernelGGL((lp_hyper_kernel<R, C, false>), dim3(nb), dim3(256), lds, s, p);
    return hipGetLastError();
}
template <int R, int C>
static int ho(size_t lds) {
    int nb = 0, nb2 = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, lp_hyper_kernel<R, C, true>, 256, lds) != hipSuccess) return 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb2, lp_hyper_kernel<R, C, false>, 256, lds) != hipSuccess) return 1;
    nb = std::min(nb, nb2);   // one grid size for both (the eta arena is sized by it)
    return nb > 0 ? nb : 1;
}

#ifdef HYP_DEV_STORM_ONLY   // development builds: the storm instance (R = 9, C = 28) only
#define HYPER_C_SWITCH(R, FN, ...)                  \
    switch (C) {                                    \
        case 28: if (R == 9) return FN<9, 28>(__VA_ARGS__); \
    }
#else
#define HYPER_C_SWITCH(R, FN, ...)                  \
    switch (C) {                                    \
        case 2: return FN<R, 2>(__VA_ARGS__);       \
        case 4: return FN<R, 4>(__VA_ARGS__);       \
        case 8: return FN<R, 8>(__VA_ARGS__);       \
        case 14: return FN<R, 14>(__VA_ARGS__);     \
        case 16: return FN<R, 16>(__VA_ARGS__);     \
        case 28: return FN<R, 28>(__VA_ARGS__);     \
        case 32: return FN<R, 32>(__VA_ARGS__);     \
        case 64: return FN<R, 64>(__VA_ARGS__);     \
    }
#endif

hipError_t launch_hyper(int R, int C, const HyperParams &p, int nblocks, size_t lds, hipStream_t s) {
    switch (R) {
        case 1: HYPER_C_SWITCH(1, hl, p, nblocks, lds, s); break;
        case 2: HYPER_C_SWITCH(2, hl, p, nblocks, lds, s); break;
        case 4: HYPER_C_SWITCH(4, hl, p, nblocks, lds, s); break;
        case 9: HYPER_C_SWITCH(9, hl, p, nblocks, lds, s); break;
        case 16: HYPER_C_SWITCH(16, hl, p, nblocks, lds, s); break;
    }
    return hipErrorInvalidValue;
}

int hyper_max_blocks_per_cu(int R, int C, int kmax, int k) {
    const size_t lds = hyper_lds_bytes(R, C, kmax, k);
    switch (R) {
        case 1: HYPER_C_SWITCH(1, ho, lds); break;
        case 2: HYPER_C_SWITCH(2, ho, lds); break;
        case 4: HYPER_C_SWITCH(4, ho, lds); break;
        case 9: HYPER_C_SWITCH(9, ho, lds); break;
        case 16: HYPER_C_SWITCH(16, ho, lds); break;
    }
    return 1;
}

}  // namespace twosd
