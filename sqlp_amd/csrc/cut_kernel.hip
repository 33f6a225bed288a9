// cut_kernel.hip -- argmax_procedure + build_sasa_cut on gfx950 (fp64 MFMA).
//
// Reference: argmax_procedure (src/sd_algorithm/subprob.jl:141-169) and build_sasa_cut
// (src/sd_algorithm/epigraph.jl:125-146).  For scenario w (element deltas dv[w,e] at
// rows row_e; coef_e = 1 for an RHS element, -x[col_e] for a T element):
//     score[w,v] = pi_v . (r - T x)  +  sum_e pi_v[row_e] * coef_e * dv[w,e]
//                = base[v]          +  (DR_w . PK_v)           (an N x |V| x k GEMM)
//     a(w)  = lowest v within tie_rel*(1+|max|) of max_v score[w,v]   (tie_rel=0: the
//             reference's strict '>' first maximum)
//     p_w   = weight_w / total_weight
//     alpha = g.r + sum_{e RHS} S_e,   beta = -T' g - sum_{e T} S_e e_{col_e}
// with g = sum_v h_v pi_v,  h_v = sum_{w: a(w)=v} p_w,  S_e = sum_w p_w PK[a(w),e] dv[w,e].
// (Same value as the reference's per-scenario loop, re-associated.)
//
// Kernels:
//   cut_pk_kernel      PK (|V| x k4 row-major) and PKT (k4 x vcap) gathers of new vertices
//   cut_vbase_kernel   base[v] = pi_v . (r - T x)                (8|V|(m+1) bytes)
//   cut_pktc_kernel    PKTc = coef(x) * PKT plus the base row: the chunk source of the argmax
//   cut_argmax2_kernel MFMA score tiles (v_mfma_f64_16x16x4f64: 32 vertices x 32 scenarios
//                      per wave and chunk), vertex chunks DMA'd into LDS, running max/argmax
//                      per scenario in registers; per-wave partial sums; h via uint64
//                      fixed-point atomics (exact and order independent -> identical on any
//                      rank count); the last round's tiles split by vertex range
//   cut_tail_merge_kernel  per-range results of the split tiles merged in vertex order
//   cut_fixup_kernel   scenarios whose running argmax slid within the tolerance band are
//                      re-decided by the exact two-pass rule (sequential fp64)
//   cut_reduce_kernel  deterministic fixed-order sum of the partial slots
//   cut_g_kernel(s)    g = sum_v h_v pi_v (two-level, fixed order)
#include <hip/hip_runtime.h>
#include <math.h>
#include <algorithm>
#include <cstdlib>
#include <vector>
#include "twosd_ctx.h"

namespace twosd {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr double kFix = 4611686018427387904.0;   // 2^62 fixed-point scale of p_w

constexpr int kHistLds = 256;      // |V| up to this: the block histogram lives in LDS

struct CutParams {
    int N, k, k4, nv, vcap, m;
    int hist_lds;          // 1: per-block LDS histogram (nv <= kHistLds), flushed once per block
    double tie_rel, inv_total;
    const double *dv;      // N x k
    const double *w;       // N
    const double *coef;    // k4 (zero padded)
    const double *PK;      // nv x k4
    const double *PKT;     // k4 x vcap
    const double *PKTc;    // 4 KB x vcap32: coef_e(x) * PKT, zero padded (cut_argmax2_kernel's LDS-DMA source)
    int vcap32;            // row stride of PKTc (a multiple of 32 >= nv)
    const double *base;    // nv
    int *arg; double *val; int *flag;   // N
    unsigned long long *hist;           // nv (fixed point)
    unsigned long long *hist_part;      // gridDim.x x nv block histograms (hist_lds mode)
    double *partial;       // slots x (k + 1): [sum p*val, S_0..S_{k-1}]
    // work units of cut_argmax2_kernel: units [0, full_units) are whole scenario tiles; the
    // tiles past them (the last, partial round of the persistent grid) are cut into tail_S
    // vertex ranges each, and such a unit leaves its per-scenario (M, SV, I, F) in tp_* at
    // [(s - 128 full_units) tail_S + range] for cut_tail_merge_kernel
    int full_units, tail_S;
    double *tp_m, *tp_sv;
    int *tp_i, *tp_f;
};

__global__ void cut_pk_kernel(int from, int to, int m, int k, int k4, int vcap, const int *__restrict__ rows,
                              const double *__restrict__ V, double *__restrict__ PK, double *__restrict__ PKT) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = (to - from) * k4;
    if (idx >= total) return;
    const int v = from + idx / k4, e = idx % k4;
    const double x = e < k ? V[(size_t)v * m + rows[e]] : 0.0;
    PK[(size_t)v * k4 + e] = x;
    PKT[(size_t)e * vcap + v] = x;
}

// PKTc[kk][v] = coef_kk * PKT[kk][v] over rows [0, rows) x columns [0, vcap32), zero outside
// [0, k) x [0, nv) (the LDS-DMA source of cut_argmax2_kernel; per x)
// With base != nullptr, row k holds base[v] (-inf for v >= nv): the MFMA then adds the vertex
// base through a constant 1 in the scenarios' delta column k.
__global__ void cut_pktc_kernel(int nv, int k, int rows, int vcap, int vcap32, const double *__restrict__ PKT,
                                const double *__restrict__ coef, const double *__restrict__ base, double *__restrict__ PKTc) {
    const size_t total = (size_t)rows * vcap32;
    for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
        const int kk = (int)(idx / vcap32), v = (int)(idx % vcap32);
        double x = (kk < k && v < nv) ? coef[kk] * PKT[(size_t)kk * vcap + v] : 0.0;
        if (base && kk == k) x = v < nv ? base[v] : -INFINITY;
        PKTc[idx] = x;
    }
}

__global__ void __launch_bounds__(256) cut_vbase_kernel(int nv, int m, const double *__restrict__ V,
                                                        const double *__restrict__ bvec, double *__restrict__ base) {
    const int lane = threadIdx.x & 63;
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    for (int v = gw; v < nv; v += nw) {
        const double *p = V + (size_t)v * m;
        double s = 0.0;
        for (int i = lane; i < m; i += 64) s = fma(p[i], bvec[i], s);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) base[v] = s;
    }
}

__device__ __forceinline__ double tolf(double M, double rel) { return rel * (1.0 + fabs(M)); }

// Running (max, argmax) of one scenario row over the vertices one lane sees, in increasing
// vertex order: M = max so far, I = lowest vertex within tolf(M) of M, SV = its score,
// F = the exact rule cannot be decided from this state (left to cut_fixup_kernel).
struct RowBest { double M, SV; int I, F; };

__device__ __forceinline__ void row_update(RowBest &b, double s, int v, double rel) {
    if (s == -INFINITY) return;
    if (b.M == -INFINITY || s > b.M + tolf(b.M, rel)) {
        // a new max beyond the old band; if the old candidate still lies within the new
        // band the lowest-index rule would keep it -> flag (rare: scores 1e-12 apart)
        if (b.M != -INFINITY && b.SV >= s - tolf(s, rel)) b.F = 1;
        b.M = s; b.I = v; b.SV = s;
    } else if (s > b.M) {
        // max slides up inside the band: the candidate must stay within the new band
        if (!(b.SV >= s - tolf(s, rel))) b.F = 1;
        b.M = s;
    }
    // s within the band but not above M: a later (higher) index never wins
}

// the same update behind its only trigger: every action needs s > M (M = -inf takes any
// finite s), so the common case is one compare
__device__ __forceinline__ void row_update_fast(RowBest &b, double s, int v, double rel) {
    if (__builtin_expect(s > b.M, 0)) row_update(b, s, v, rel);
}

// ---- v2: the score tile transposed -- MFMA A operand = the staged vertex chunk, B operand =
// the scenario deltas -- so the C/D layout puts one SCENARIO per lane column (j) and four
// vertices per lane (rows g + 4r): a lane tracks the running argmax of ONE scenario per A tile
// instead of four, which frees the registers for two scenario tiles per wave (32 scenarios,
// 128 per block) and two vertex tiles per chunk (32 vertices): every chunk staged in LDS
// serves twice the scenarios of v1, and each LDS fragment read feeds two MFMAs.  The deltas
// stay raw in registers (coef_e(x) is folded into the staged chunk), so the S_e sums of the
// cut reuse them instead of re-reading the deltas from HBM.  Chunks are double-buffered.
#ifndef TWOSD_CUT_KG
#define TWOSD_CUT_KG 6                   // k-blocks whose fragments are read ahead together
#endif
#ifndef TWOSD_CUT_SB
#define TWOSD_CUT_SB 1                   // scheduling barrier between the groups
#endif
#ifndef TWOSD_CUT_FASTRU
#define TWOSD_CUT_FASTRU 1               // row updates behind the s > M test
#endif
#if TWOSD_CUT_FASTRU
#define RU2 row_update_fast
#else
#define RU2 row_update
#endif
#ifndef TWOSD_CUT_BASEK
#define TWOSD_CUT_BASEK 1                // vertex base as an extra k-row of the chunk (no VALU add)
#endif
#ifndef TWOSD_CUT_PF
#define TWOSD_CUT_PF 0                   // read the next group's fragments before this group's MFMAs
#endif
constexpr int kVT2 = 32;                 // vertices per LDS chunk (two 16-vertex MFMA tiles)
constexpr int kCutTile2 = 128;           // scenarios per block tile (4 waves x 2 x 16)
constexpr int kLdsRow2 = 32;             // doubles per k-row of a chunk

// LDS position of (k-row kk, vertex vv): odd rows have their 16-double halves swapped, so the
// two k-rows a half-wave reads together (g = 0, 1 / 2, 3) fall on disjoint banks
__device__ __forceinline__ int lds2(int kk, int vv) { return kk * kLdsRow2 + (vv ^ ((kk & 1) << 4)); }

#ifndef TWOSD_CUT_LB3
#define TWOSD_CUT_LB3 1                  // 3 blocks per CU for KB <= 22 (168 VGPRs; ssn: 62 -> 76 % of the roofline)
#endif
template <int KB>
__global__ void __launch_bounds__(256, (TWOSD_CUT_LB3 && KB <= 22) ? 3 : 2) cut_argmax2_kernel(CutParams P) {
    __shared__ double Bs[2][4 * KB * kLdsRow2];     // double-buffered chunk (k-major)
    __shared__ double bs[2][kVT2];
    extern __shared__ unsigned long long hl[];      // nv entries when P.hist_lds
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar staging loop
    if (P.hist_lds)
        for (int v = threadIdx.x; v < P.nv; v += 256) hl[v] = 0ull;
    const int g = lane >> 4, j = lane & 15;
    const int ntiles = (P.N + kCutTile2 - 1) / kCutTile2;
    const int nchunks = (P.nv + kVT2 - 1) / kVT2;
    const int nunits = P.full_units + (ntiles - P.full_units) * P.tail_S;
    double pv_sum = 0.0;
    double Sacc[2] = {0.0, 0.0};   // lane (g, j): e = 4 kb + g for kb = j, j + 16

    for (int unit = blockIdx.x; unit < nunits; unit += gridDim.x) {
        // a whole tile (all vertex chunks), or vertex range `range` of a tail tile
        const bool tail = unit >= P.full_units;
        const int tile = tail ? P.full_units + (unit - P.full_units) / P.tail_S : unit;
        const int range = tail ? (unit - P.full_units) % P.tail_S : 0;
        const int c_lo = tail ? (int)((long long)nchunks * range / P.tail_S) : 0;
        const int c_hi = tail ? (int)((long long)nchunks * (range + 1) / P.tail_S) : nchunks;
        // this wave: scenarios s0 + j (tile 0) and s0 + 16 + j (tile 1); lane (g, j) holds their
        // deltas e = 4 kb + g (the B operand: k = g, column = j)
        const int s0 = tile * kCutTile2 + wid * 32;
        double a0[KB], a1[KB];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            const int e = 4 * kb + g;
            const int sa = s0 + j, sb = s0 + 16 + j;
            a0[kb] = (sa < P.N && e < P.k) ? P.dv[(size_t)sa * P.k + e] : 0.0;
            a1[kb] = (sb < P.N && e < P.k) ? P.dv[(size_t)sb * P.k + e] : 0.0;
            if (TWOSD_CUT_BASEK && e == P.k) a0[kb] = a1[kb] = 1.0;   // x the base row of the chunk
        }
        RowBest rb0, rb1;   // scenario s0 + j / s0 + 16 + j over this lane's vertices v0 + g + 4r (+16)
        rb0.M = -INFINITY; rb0.SV = -INFINITY; rb0.I = -1; rb0.F = 0;
        rb1 = rb0;

        // chunk staging by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip): instruction i
        // of the chunk writes k-rows 4i .. 4i+3 (1 KiB, lane-linear), lane L the 16 bytes of
        // row 4i + L/16 at LDS position 2 (L % 16); the source vertex pair is that position with
        // the row's half swap (lds2) applied, so the image is exactly lds2's layout
        double preb = -INFINITY;
        auto stage = [&](int buf, int v0) {
            for (int i = wid; i < KB; i += 4) {
                const int kk = 4 * i + (lane >> 4);
                const int vv = (2 * (lane & 15)) ^ ((kk & 1) << 4);
                __builtin_amdgcn_global_load_lds((const void *)(P.PKTc + (size_t)kk * P.vcap32 + v0 + vv),
                                                 (__attribute__((address_space(3))) void *)&Bs[buf][i * 4 * kLdsRow2], 16, 0, 0);
            }
            if (!TWOSD_CUT_BASEK && threadIdx.x < kVT2) preb = v0 + (int)threadIdx.x < P.nv ? P.base[v0 + threadIdx.x] : -INFINITY;
        };
        stage(0, c_lo * kVT2);
        if (!TWOSD_CUT_BASEK && threadIdx.x < kVT2) bs[0][threadIdx.x] = preb;
        __syncthreads();            // chunk c_lo landed (the barrier drains the DMA)
        for (int ch = c_lo; ch < c_hi; ++ch) {
            const int buf = (ch - c_lo) & 1;
            const int v0 = ch * kVT2;
            // chunk ch+1 into the other buffer while this one is multiplied (its readers passed
            // the last barrier)
            if (ch + 1 < c_hi) stage(buf ^ 1, v0 + kVT2);
            d4 c00 = {0.0, 0.0, 0.0, 0.0}, c01 = c00, c10 = c00, c11 = c00;   // c[vertex tile][scenario tile]
            // fragments are read in groups of KG k-blocks ahead of their MFMAs; the scheduling
            // barrier keeps the compiler from hoisting every read of the chunk (register spills)
            constexpr int KG = TWOSD_CUT_KG;
            if constexpr (TWOSD_CUT_PF) {
                // software-pipelined: group k0 + KG is read while group k0 is multiplied
                double x0[KG], x1[KG];
#pragma unroll
                for (int u = 0; u < KG; ++u) {
                    x0[u] = Bs[buf][lds2(4 * u + g, j)];
                    x1[u] = Bs[buf][lds2(4 * u + g, 16 + j)];
                }
#pragma unroll
                for (int k0 = 0; k0 < KB; k0 += KG) {
                    double y0[KG], y1[KG];
#pragma unroll
                    for (int u = 0; u < KG; ++u) {
                        if (k0 + KG + u < KB) {
                            y0[u] = Bs[buf][lds2(4 * (k0 + KG + u) + g, j)];
                            y1[u] = Bs[buf][lds2(4 * (k0 + KG + u) + g, 16 + j)];
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int u = 0; u < KG; ++u) {
                        if (k0 + u < KB) {
                            c00 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0[u], a0[k0 + u], c00, 0, 0, 0);
                            c01 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0[u], a1[k0 + u], c01, 0, 0, 0);
                            c10 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1[u], a0[k0 + u], c10, 0, 0, 0);
                            c11 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1[u], a1[k0 + u], c11, 0, 0, 0);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int u = 0; u < KG; ++u) {
                        x0[u] = y0[u];
                        x1[u] = y1[u];
                    }
                }
            } else {
#pragma unroll
            for (int k0 = 0; k0 < KB; k0 += KG) {
                double x0[KG], x1[KG];
#pragma unroll
                for (int u = 0; u < KG; ++u) {
                    if (k0 + u < KB) {
                        x0[u] = Bs[buf][lds2(4 * (k0 + u) + g, j)];
                        x1[u] = Bs[buf][lds2(4 * (k0 + u) + g, 16 + j)];
                    }
                }
#pragma unroll
                for (int u = 0; u < KG; ++u) {
                    if (k0 + u < KB) {
                        c00 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0[u], a0[k0 + u], c00, 0, 0, 0);
                        c01 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0[u], a1[k0 + u], c01, 0, 0, 0);
                        c10 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1[u], a0[k0 + u], c10, 0, 0, 0);
                        c11 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1[u], a1[k0 + u], c11, 0, 0, 0);
                    }
                }
                if (TWOSD_CUT_SB) __builtin_amdgcn_sched_barrier(0);
            }
            }
            // C/D: register r of a tile is vertex row g + 4r, scenario column j; this lane's
            // vertices in increasing order: v0 + g + 4r, then v0 + 16 + g + 4r
            if constexpr (TWOSD_CUT_BASEK) {   // the scores include the base (-inf past nv)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    RU2(rb0, c00[r], v0 + g + 4 * r, P.tie_rel);
                    RU2(rb1, c01[r], v0 + g + 4 * r, P.tie_rel);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    RU2(rb0, c10[r], v0 + 16 + g + 4 * r, P.tie_rel);
                    RU2(rb1, c11[r], v0 + 16 + g + 4 * r, P.tie_rel);
                }
            } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int va = v0 + g + 4 * r;
                const double ba = va < P.nv ? bs[buf][g + 4 * r] : -INFINITY;
                RU2(rb0, ba + c00[r], va, P.tie_rel);
                RU2(rb1, ba + c01[r], va, P.tie_rel);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int vb = v0 + 16 + g + 4 * r;
                const double bb = vb < P.nv ? bs[buf][16 + g + 4 * r] : -INFINITY;
                RU2(rb0, bb + c10[r], vb, P.tie_rel);
                RU2(rb1, bb + c11[r], vb, P.tie_rel);
            }
            }
            if (!TWOSD_CUT_BASEK && ch + 1 < c_hi && threadIdx.x < kVT2) bs[buf ^ 1][threadIdx.x] = preb;
            __syncthreads();
        }
        // combine the 4 lanes (g) of each scenario column: max M, band threshold, lowest candidate
        // inside the band; a lane whose max reaches the band but whose candidate does not (or
        // that flagged) -> exact fixup.  Every lane of the column ends with the result.
        auto combine = [&](RowBest &rb) {
            double M = rb.M;
            M = fmax(M, __shfl_xor(M, 16));
            M = fmax(M, __shfl_xor(M, 32));
            const double thr = M - tolf(M, P.tie_rel);
            const bool reach = rb.M != -INFINITY && rb.M >= thr;
            int it = (reach && rb.SV >= thr) ? rb.I : 0x7fffffff;
            double st = rb.SV;
            int fl = reach && (rb.F || !(rb.SV >= thr));
#pragma unroll
            for (int o = 16; o <= 32; o <<= 1) {
                const int i2 = __shfl_xor(it, o);
                const double s2 = __shfl_xor(st, o);
                fl |= __shfl_xor(fl, o);
                if (i2 < it) { it = i2; st = s2; }
            }
            rb.I = (M == -INFINITY || it == 0x7fffffff) ? -1 : it;
            rb.SV = st;
            rb.F = fl;
            rb.M = M;
        };
        combine(rb0);
        combine(rb1);
        const int sa = s0 + j, sb = s0 + 16 + j;
        if (tail) {   // this vertex range's result; cut_tail_merge_kernel decides and sums
            if (g == 0) {
                const int t0 = P.full_units * kCutTile2;
                if (sa < P.N) {
                    const size_t o = (size_t)(sa - t0) * P.tail_S + range;
                    P.tp_m[o] = rb0.M; P.tp_sv[o] = rb0.SV; P.tp_i[o] = rb0.I; P.tp_f[o] = rb0.F;
                }
                if (sb < P.N) {
                    const size_t o = (size_t)(sb - t0) * P.tail_S + range;
                    P.tp_m[o] = rb1.M; P.tp_sv[o] = rb1.SV; P.tp_i[o] = rb1.I; P.tp_f[o] = rb1.F;
                }
            }
            continue;
        }
        if (g == 0) {
            if (sa < P.N) { P.arg[sa] = rb0.I; P.val[sa] = rb0.SV; P.flag[sa] = rb0.F; }
            if (sb < P.N) { P.arg[sb] = rb1.I; P.val[sb] = rb1.SV; P.flag[sb] = rb1.F; }
        }
        const bool ok0 = sa < P.N && !rb0.F && rb0.I >= 0, ok1 = sb < P.N && !rb1.F && rb1.I >= 0;
        const double p0 = ok0 ? P.w[sa] * P.inv_total : 0.0, p1 = ok1 ? P.w[sb] * P.inv_total : 0.0;
        // sum p * val and the vertex histogram, scenarios in order (lane 0 reads them from lanes 0-15)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const int ok = __shfl(t == 0 ? (int)ok0 : (int)ok1, jj);
                const int ai = __shfl(t == 0 ? rb0.I : rb1.I, jj);
                const double pp = __shfl(t == 0 ? p0 : p1, jj);
                const double vl = __shfl(t == 0 ? rb0.SV : rb1.SV, jj);
                if (lane == 0 && ok) {
                    pv_sum = fma(pp, vl, pv_sum);
                    const unsigned long long hq = (unsigned long long)__double2ull_rn(pp * kFix);
                    if (P.hist_lds) __hip_atomic_fetch_add(&hl[ai], hq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    else atomicAdd(&P.hist[ai], hq);
                }
            }
        }
        // S_e = sum_w p_w PK[a(w), e] dv[w, e] from the delta registers: lane (g, j) holds
        // scenario j's e = 4 kb + g and its pick; the 16 scenarios of a tile are summed by a
        // fixed xor tree, lane (g, kb mod 16) keeps the sum
        auto s_pass = [&](const double (&a)[KB], bool ok, int ai, double pp) {
            const double *pk = P.PK + (size_t)(ok ? ai : 0) * P.k4;
            const double pu = ok ? pp : 0.0;
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                const int e = 4 * kb + g;
                double v = (e < P.k) ? pu * pk[e] * a[kb] : 0.0;
#pragma unroll
                for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o);
                if (j == (kb & 15)) {
                    if (kb < 16) Sacc[0] += v;
                    else Sacc[1] += v;
                }
            }
        };
        s_pass(a0, ok0, rb0.I, p0);
        s_pass(a1, ok1, rb1.I, p1);
    }
    if (P.hist_lds) {
        __syncthreads();
        for (int v = threadIdx.x; v < P.nv; v += 256) P.hist_part[(size_t)blockIdx.x * P.nv + v] = hl[v];
    }
    const int slot = blockIdx.x * 4 + wid;
    double *out = P.partial + (size_t)slot * (P.k + 1);
    if (lane == 0) out[0] = pv_sum;
    // lane (g, j) owns e = 4 j + g (kb = j) and e = 4 (j + 16) + g (kb = j + 16)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int e = 4 * (j + 16 * t) + g;
        if (e < P.k) out[1 + e] = Sacc[t];
    }
}

// hist[v] += sum over blocks of the block histograms (integers: exact in any order)
__global__ void __launch_bounds__(256) cut_hist_reduce_kernel(int nb, int nv, const unsigned long long *__restrict__ part,
                                                              unsigned long long *__restrict__ hist) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nv) return;
    unsigned long long s = 0;
    for (int b = 0; b < nb; ++b) s += part[(size_t)b * nv + v];
    hist[v] += s;
}

// Tail scenarios: merge the per-range results in vertex order -- the same rule as `combine`
// over the 4 lanes of a column: M = max, band threshold, lowest candidate inside the band,
// flag when a range reaches the band but its candidate does not -- then, for a decided
// scenario, its p * val, histogram weight and S_e terms (as cut_fixup_kernel).  One wavefront
// per scenario, lane r = range r.
__global__ void __launch_bounds__(256) cut_tail_merge_kernel(CutParams P, int slot0) {
    const int lane = threadIdx.x & 63;
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    const int t0 = P.full_units * kCutTile2, S = P.tail_S;
    double pv_sum = 0.0, Sacc[2] = {0.0, 0.0};
    for (int ts = gw; ts < P.N - t0; ts += nw) {
        const int s = t0 + ts;
        double m = -INFINITY, sv = -INFINITY;
        int ii = -1, ff = 0;
        if (lane < S) {
            const size_t o = (size_t)ts * S + lane;
            m = P.tp_m[o]; sv = P.tp_sv[o]; ii = P.tp_i[o]; ff = P.tp_f[o];
        }
        double M = m;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) M = fmax(M, __shfl_xor(M, o));
        const double thr = M - tolf(M, P.tie_rel);
        const bool reach = m != -INFINITY && m >= thr;
        int it = (reach && ii >= 0 && sv >= thr) ? ii : 0x7fffffff;
        double st = sv;
        int fl = reach && (ff || ii < 0 || !(sv >= thr));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int i2 = __shfl_xor(it, o);
            const double s2 = __shfl_xor(st, o);
            fl |= __shfl_xor(fl, o);
            if (i2 < it) { it = i2; st = s2; }
        }
        const int I = (M == -INFINITY || it == 0x7fffffff) ? -1 : it;
        if (lane == 0) { P.arg[s] = I; P.val[s] = st; P.flag[s] = fl; }
        if (fl || I < 0) continue;
        const double p = P.w[s] * P.inv_total;
        if (lane == 0) {
            pv_sum = fma(p, st, pv_sum);
            atomicAdd(&P.hist[I], (unsigned long long)__double2ull_rn(p * kFix));
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int e = lane + 64 * t;
            if (e < P.k) Sacc[t] = fma(p * P.PK[(size_t)I * P.k4 + e], P.dv[(size_t)s * P.k + e], Sacc[t]);
        }
    }
    double *out = P.partial + (size_t)(slot0 + gw) * (P.k + 1);
    if (lane == 0) out[0] = pv_sum;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int e = lane + 64 * t;
        if (e < P.k) out[1 + e] = Sacc[t];
    }
}

// exact two-pass rule for flagged scenarios; one wavefront per scenario
__global__ void __launch_bounds__(256) cut_fixup_kernel(CutParams P, int slot0) {
    const int lane = threadIdx.x & 63;
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    double pv_sum = 0.0, Sacc[2] = {0.0, 0.0};
    // the flags are read 64 at a time (one coalesced load per wave step: flagged scenarios are
    // rare, and a flag per dependent load made the scan of 1M flags 0.35 ms); the flagged ones of
    // a step in ascending order
    for (int s0 = gw * 64; s0 < P.N; s0 += nw * 64) {
    uint64_t todo = __ballot(s0 + lane < P.N && P.flag[s0 + lane] != 0);
    while (todo) {
        const int s = s0 + (int)__builtin_ctzll(todo);
        todo &= todo - 1;
        // pass 1: max over v (lanes stride vertices)
        double mx = -INFINITY;
        for (int v = lane; v < P.nv; v += 64) {
            double sc = P.base[v];
            for (int e = 0; e < P.k; ++e) sc = fma(P.PK[(size_t)v * P.k4 + e], P.dv[(size_t)s * P.k + e] * P.coef[e], sc);
            mx = fmax(mx, sc);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
        const double tl = tolf(mx, P.tie_rel);
        int best = 0x7fffffff;
        double bv = -INFINITY;
        for (int v = lane; v < P.nv; v += 64) {
            double sc = P.base[v];
            for (int e = 0; e < P.k; ++e) sc = fma(P.PK[(size_t)v * P.k4 + e], P.dv[(size_t)s * P.k + e] * P.coef[e], sc);
            if (sc >= mx - tl && v < best) { best = v; bv = sc; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int b2 = __shfl_xor(best, o);
            const double v2 = __shfl_xor(bv, o);
            if (b2 < best) { best = b2; bv = v2; }
        }
        const double p = P.w[s] * P.inv_total;
        if (lane == 0) {
            P.arg[s] = best;
            P.val[s] = bv;
            pv_sum = fma(p, bv, pv_sum);
            atomicAdd(&P.hist[best], (unsigned long long)__double2ull_rn(p * kFix));
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int e = lane + 64 * t;
            if (e < P.k) Sacc[t] = fma(p * P.PK[(size_t)best * P.k4 + e], P.dv[(size_t)s * P.k + e], Sacc[t]);
        }
    }
    }
    double *out = P.partial + (size_t)(slot0 + gw) * (P.k + 1);
    if (lane == 0) out[0] = pv_sum;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int e = lane + 64 * t;
        if (e < P.k) out[1 + e] = Sacc[t];
    }
}

// sums[c] = sum over slots of partial[slot][c], c < k+1, in a fixed order: block b sums
// the slot range [b*per, (b+1)*per) with a fixed-shape in-block tree, then the last level
// adds the block results in block order (deterministic, independent of timing).
constexpr int kReduceBlocks = 64;
__global__ void __launch_bounds__(256) cut_reduce1_kernel(int slots, int width, const double *__restrict__ partial,
                                                          double *__restrict__ part2) {
    __shared__ double sh[256];
    const int b = blockIdx.x, c = blockIdx.y;
    const int per = (slots + kReduceBlocks - 1) / kReduceBlocks;
    const int s0 = b * per, s1 = min(slots, s0 + per);
    double s = 0.0;
    for (int i = s0 + threadIdx.x; i < s1; i += 256) s += partial[(size_t)i * width + c];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part2[(size_t)c * kReduceBlocks + b] = sh[0];
}
__global__ void cut_reduce2_kernel(int width, const double *__restrict__ part2, double *__restrict__ sums) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= width) return;
    double s = 0.0;
    for (int b = 0; b < kReduceBlocks; ++b) s += part2[(size_t)c * kReduceBlocks + b];
    sums[c] = s;
}

// gpart[b][i] = sum_{v in chunk b} h_v * 2^-62 * V[v][i]
__global__ void cut_g_partial_kernel(int nv, int m, int chunk, const unsigned long long *__restrict__ hist,
                                     const double *__restrict__ V, double *__restrict__ gpart) {
    const int b = blockIdx.x;
    const int v0 = b * chunk, v1 = min(nv, v0 + chunk);
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        double s = 0.0;
        for (int v = v0; v < v1; ++v) {
            const unsigned long long h = hist[v];
            if (h) s = fma((double)h * (1.0 / kFix), V[(size_t)v * m + i], s);
        }
        gpart[(size_t)b * m + i] = s;
    }
}

__global__ void cut_g_final_kernel(int nb, int m, const double *__restrict__ gpart, double *__restrict__ gout) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double s = 0.0;
    for (int b = 0; b < nb; ++b) s += gpart[(size_t)b * m + i];
    gout[i] = s;
}

// ---------------------------------------------------------------------------------
struct CutWs {
    double *PK = nullptr, *PKT = nullptr;
    double *PKTc = nullptr;
    size_t pktc_cap = 0;
    int pk_count = 0, pk_vcap = 0, pk_k4 = 0;
    size_t pk_cap = 0;
    int *rows = nullptr;
    double *coef = nullptr, *bvec = nullptr, *base = nullptr, *partial = nullptr, *sums = nullptr;
    double *gpart = nullptr, *g = nullptr;
    int *arg = nullptr, *flag = nullptr;
    double *val = nullptr;
    unsigned long long *hist = nullptr, *hist_part = nullptr;
    size_t hpart_cap = 0;
    double *part2 = nullptr;
    double *tp_m = nullptr, *tp_sv = nullptr;
    int *tp_i = nullptr, *tp_f = nullptr;
    size_t tp_cap = 0;
    size_t base_cap = 0, part_cap = 0, n_cap = 0, hist_cap = 0, gpart_cap = 0, sums_cap = 0, part2_cap = 0;
    int m = 0, vec_m = 0;
    std::vector<double> h_coef, h_bvec;   // pinned-lifetime host staging for async uploads
};

static CutWs *cws(twosd_ctx *c) {
    if (!c->cut_ws) c->cut_ws = new CutWs();
    return (CutWs *)c->cut_ws;
}

void cut_free(twosd_ctx *c) {
    if (!c->cut_ws) return;
    CutWs *w = (CutWs *)c->cut_ws;
    hipFree(w->PK); hipFree(w->PKT); hipFree(w->PKTc); hipFree(w->rows); hipFree(w->coef); hipFree(w->bvec); hipFree(w->base);
    hipFree(w->partial); hipFree(w->sums); hipFree(w->gpart); hipFree(w->g); hipFree(w->arg); hipFree(w->flag);
    hipFree(w->val); hipFree(w->hist); hipFree(w->part2); hipFree(w->hist_part);
    hipFree(w->tp_m); hipFree(w->tp_sv); hipFree(w->tp_i); hipFree(w->tp_f);
    delete w;
    c->cut_ws = nullptr;
}

void cut_invalidate_pk(twosd_ctx *c) {
    if (!c->cut_ws) return;
    CutWs *w = (CutWs *)c->cut_ws;
    w->pk_count = 0;
    if (w->rows) hipFree(w->rows);
    w->rows = nullptr;   // forces re-upload of the element rows
}

#define HIPCHK(expr)                                                                               \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) return fail(TWOSD_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

template <typename T>
static int realloc_dev(T **p, size_t n) {
    if (*p) hipFree(*p);
    *p = nullptr;
    hipError_t e = hipMalloc((void **)p, sizeof(T) * std::max<size_t>(n, 1));
    if (e != hipSuccess) return fail(TWOSD_E_DEVICE, "cut workspace hipMalloc(%zu): %s", sizeof(T) * n, hipGetErrorString(e));
    return TWOSD_OK;
}

static int kb_for(int k4) {
    static const int KBs[] = {1, 2, 4, 6, 8, 12, 16, 22, 24, 30, 32};   // 22: ssn (k = 86, + base row)
    for (int kb : KBs)
        if (4 * kb >= k4) return kb;
    return -1;
}

template <int KB>
static void launch_argmax_t(const CutParams &P, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL(cut_argmax2_kernel<KB>, dim3(nblocks), dim3(256), P.hist_lds ? sizeof(unsigned long long) * P.nv : 0, s, P);
}

// resident blocks per CU of one instantiation (registers and LDS): the persistent grid is
// sized to exactly what is resident, so no block starts after the first ones drain (a grid
// of 3 blocks per CU at 2 resident ran its last third with half of every CU idle)
template <int KB>
static int argmax_occupancy_t(size_t dyn_lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cut_argmax2_kernel<KB>, 256, dyn_lds) != hipSuccess) nb = 0;
    return nb;
}

static int argmax_occupancy(int KB, size_t dyn_lds) {
    switch (KB) {
        case 1: return argmax_occupancy_t<1>(dyn_lds);
        case 2: return argmax_occupancy_t<2>(dyn_lds);
        case 4: return argmax_occupancy_t<4>(dyn_lds);
        case 6: return argmax_occupancy_t<6>(dyn_lds);
        case 8: return argmax_occupancy_t<8>(dyn_lds);
        case 12: return argmax_occupancy_t<12>(dyn_lds);
        case 16: return argmax_occupancy_t<16>(dyn_lds);
        case 22: return argmax_occupancy_t<22>(dyn_lds);
        case 24: return argmax_occupancy_t<24>(dyn_lds);
        case 30: return argmax_occupancy_t<30>(dyn_lds);
        case 32: return argmax_occupancy_t<32>(dyn_lds);
    }
    return 0;
}

static void launch_argmax(int KB, const CutParams &P, int nblocks, hipStream_t s) {
    switch (KB) {
        case 1: launch_argmax_t<1>(P, nblocks, s); break;
        case 2: launch_argmax_t<2>(P, nblocks, s); break;
        case 4: launch_argmax_t<4>(P, nblocks, s); break;
        case 6: launch_argmax_t<6>(P, nblocks, s); break;
        case 8: launch_argmax_t<8>(P, nblocks, s); break;
        case 12: launch_argmax_t<12>(P, nblocks, s); break;
        case 16: launch_argmax_t<16>(P, nblocks, s); break;
        case 22: launch_argmax_t<22>(P, nblocks, s); break;
        case 24: launch_argmax_t<24>(P, nblocks, s); break;
        case 30: launch_argmax_t<30>(P, nblocks, s); break;
        case 32: launch_argmax_t<32>(P, nblocks, s); break;
    }
}

// bring PK/PKT up to date with the vertex set
static int update_pk(twosd_ctx *c) {
    CutWs *w = cws(c);
    const int nv = c->dvs.size, k = c->k, k4 = (std::max(k, 1) + 3) & ~3, m = c->L.m;
    int rc;
    if (!w->rows || w->pk_k4 != k4 || w->m != m) {
        if ((rc = realloc_dev(&w->rows, std::max(k, 1)))) return rc;
        if (k) HIPCHK(hipMemcpy(w->rows, c->pos_row.data(), sizeof(int) * k, hipMemcpyHostToDevice));
        w->pk_count = 0;
        w->pk_k4 = k4;
        w->m = m;
    }
    if (nv > w->pk_vcap) {
        const int vcap = std::max(nv, 2 * w->pk_vcap + 256);
        if ((rc = realloc_dev(&w->PK, (size_t)vcap * k4)) || (rc = realloc_dev(&w->PKT, (size_t)vcap * k4))) return rc;
        w->pk_vcap = vcap;
        w->pk_count = 0;
    }
    if (w->pk_count > nv) w->pk_count = 0;
    if (w->pk_count < nv) {
        const int total = (nv - w->pk_count) * k4;
        hipLaunchKernelGGL(cut_pk_kernel, dim3((total + 255) / 256), dim3(256), 0, c->stream, w->pk_count, nv, m, k, k4,
                           w->pk_vcap, w->rows, c->dvs.V, w->PK, w->PKT);
        HIPCHK(hipGetLastError());
        w->pk_count = nv;
    }
    return TWOSD_OK;
}

// argmax + partial sums over scenarios [0, N) of epigraph epi at x.  Fills w->hist (nv),
// w->sums (k+1), w->arg / w->val.  total_weight: global total scenario weight.
static int cut_partial_impl(twosd_ctx *c, int epi, const double *x, double tie_rel, double total_weight,
                            unsigned long long *d_hist, double *d_sums) {
    CutWs *w = cws(c);
    const EpiDevice &E = c->epis[epi];
    const int N = E.count, k = c->k, m = c->L.m, nv = c->dvs.size, n1 = c->n1;
    const int k4 = (std::max(k, 1) + 3) & ~3;
    // v2 with the base row: k + 1 rows of the chunk
    const bool base_row = TWOSD_CUT_BASEK;
    const int KB = kb_for(base_row ? ((k + 1 + 3) & ~3) : k4);
    if (KB < 0) return fail(TWOSD_E_UNSUPPORTED, "k = %d random elements exceeds the cut kernel envelope (127)", k);
    int rc;
    if ((rc = update_pk(c))) return rc;
    // host: bvec = r - T x, coef
    std::vector<double> &bvec = w->h_bvec, &coef = w->h_coef;
    bvec.assign(m, 0.0);
    coef.assign(k4, 0.0);
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (int jj = 0; jj < n1; ++jj) s += c->T[(size_t)i * n1 + jj] * x[jj];
        bvec[i] = c->r[i] - s;
    }
    for (int e = 0; e < k; ++e) coef[e] = c->pos_col[e] < 0 ? 1.0 : -x[c->pos_col[e]];
    if (!w->coef || !w->bvec || !w->g || w->vec_m != m) {
        if ((rc = realloc_dev(&w->coef, 256)) || (rc = realloc_dev(&w->bvec, m)) || (rc = realloc_dev(&w->g, m))) return rc;
        w->vec_m = m;
    }
    if ((size_t)nv > w->base_cap) {
        if ((rc = realloc_dev(&w->base, nv))) return rc;
        w->base_cap = nv;
    }
    if ((size_t)N > w->n_cap) {
        if ((rc = realloc_dev(&w->arg, N)) || (rc = realloc_dev(&w->val, N)) || (rc = realloc_dev(&w->flag, N))) return rc;
        w->n_cap = N;
    }
    HIPCHK(hipMemcpyAsync(w->coef, coef.data(), sizeof(double) * k4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(w->bvec, bvec.data(), sizeof(double) * m, hipMemcpyHostToDevice, c->stream));
    const int ntiles = (N + kCutTile2 - 1) / kCutTile2;
    // blocks per CU: resident occupancy of this instantiation (TWOSD_CUT_BPC overrides; the
    // |V| <= kHistLds case adds the LDS histogram, at most 2 KB)
    static const int bpc_env = getenv("TWOSD_CUT_BPC") ? atoi(getenv("TWOSD_CUT_BPC")) : 0;
    int bpc = bpc_env;
    if (bpc <= 0) bpc = argmax_occupancy(KB, sizeof(unsigned long long) * kHistLds);
    if (bpc <= 0) bpc = 2;
    const int nchunks = (nv + kVT2 - 1) / kVT2;
    // The persistent grid runs whole tiles round after round; the tiles past the last full
    // round are cut into S vertex ranges (at least 4 chunks each) so that the last round is as
    // full as the others.  S minimises the tail's length ceil(T S / B) / S in tile durations.
    const int B = bpc * c->num_cus;
    int full = ntiles, S = 1;
    const bool tail_split = !getenv("TWOSD_CUT_TAIL") || atoi(getenv("TWOSD_CUT_TAIL")) != 0;   // A/B knob
    if (tail_split && nchunks >= 8) {
        const int T = ntiles % B;
        double best = 1.0;
        for (int s_ = 2; T > 0 && s_ <= std::min(64, nchunks / 4); ++s_) {
            const double cost = (double)(((long long)T * s_ + B - 1) / B) / s_;
            if (cost < best - 1e-9) { best = cost; S = s_; }
        }
        if (S > 1) full = ntiles - T;
    }
    const int nunits = full + (ntiles - full) * S;
    const int nblocks = std::max(1, std::min(nunits, B));
    const int fix_blocks = std::max(1, std::min((N + 3) / 4, c->num_cus));
    const int ntail = S > 1 ? N - full * kCutTile2 : 0;
    const int merge_blocks = ntail > 0 ? std::max(1, std::min((ntail + 3) / 4, c->num_cus)) : 0;
    const size_t slots = (size_t)nblocks * 4 + (size_t)fix_blocks * 4 + (size_t)merge_blocks * 4;
    if ((size_t)ntail * S > w->tp_cap) {
        if ((rc = realloc_dev(&w->tp_m, (size_t)ntail * S)) || (rc = realloc_dev(&w->tp_sv, (size_t)ntail * S)) ||
            (rc = realloc_dev(&w->tp_i, (size_t)ntail * S)) || (rc = realloc_dev(&w->tp_f, (size_t)ntail * S)))
            return rc;
        w->tp_cap = (size_t)ntail * S;
    }
    if (slots * (k + 1) > w->part_cap) {
        if ((rc = realloc_dev(&w->partial, slots * (k + 1)))) return rc;
        w->part_cap = slots * (k + 1);
    }
    HIPCHK(hipMemsetAsync(d_hist, 0, sizeof(unsigned long long) * std::max(nv, 1), c->stream));
    hipLaunchKernelGGL(cut_vbase_kernel, dim3(std::max(1, std::min((nv + 3) / 4, 4096))), dim3(256), 0, c->stream, nv, m,
                       c->dvs.V, w->bvec, w->base);
    CutParams P{};
    P.N = N; P.k = k; P.k4 = k4; P.nv = nv; P.vcap = w->pk_vcap; P.m = m;
    static const int hist_lds_max = getenv("TWOSD_HIST_LDS") ? atoi(getenv("TWOSD_HIST_LDS")) : kHistLds;
    P.hist_lds = nv <= hist_lds_max ? 1 : 0;
    if (P.hist_lds && (size_t)nblocks * nv > w->hpart_cap) {
        if ((rc = realloc_dev(&w->hist_part, (size_t)nblocks * nv))) return rc;
        w->hpart_cap = (size_t)nblocks * nv;
    }
    P.hist_part = w->hist_part;
    P.tie_rel = tie_rel; P.inv_total = 1.0 / total_weight;
    P.dv = E.d_dv; P.w = E.d_w; P.coef = w->coef; P.PK = w->PK; P.PKT = w->PKT; P.base = w->base;
    {
        const int vcap32 = (nv + 31) & ~31, rows = 4 * KB;
        if ((size_t)rows * vcap32 > w->pktc_cap) {
            if ((rc = realloc_dev(&w->PKTc, (size_t)rows * vcap32))) return rc;
            w->pktc_cap = (size_t)rows * vcap32;
        }
        const size_t tot = (size_t)rows * vcap32;
        hipLaunchKernelGGL(cut_pktc_kernel, dim3((unsigned)std::min<size_t>(4096, (tot + 255) / 256)), dim3(256), 0, c->stream, nv, k,
                           rows, w->pk_vcap, vcap32, w->PKT, w->coef, base_row ? w->base : nullptr, w->PKTc);
        P.PKTc = w->PKTc;
        P.vcap32 = vcap32;
    }
    P.arg = w->arg; P.val = w->val; P.flag = w->flag; P.hist = d_hist; P.partial = w->partial;
    P.full_units = full; P.tail_S = S;
    P.tp_m = w->tp_m; P.tp_sv = w->tp_sv; P.tp_i = w->tp_i; P.tp_f = w->tp_f;
    launch_argmax(KB, P, nblocks, c->stream);
    if (P.hist_lds)
        hipLaunchKernelGGL(cut_hist_reduce_kernel, dim3((nv + 255) / 256), dim3(256), 0, c->stream, nblocks, nv, w->hist_part,
                           d_hist);
    if (merge_blocks)
        hipLaunchKernelGGL(cut_tail_merge_kernel, dim3(merge_blocks), dim3(256), 0, c->stream, P, nblocks * 4 + fix_blocks * 4);
    hipLaunchKernelGGL(cut_fixup_kernel, dim3(fix_blocks), dim3(256), 0, c->stream, P, nblocks * 4);
    if ((size_t)(k + 1) * kReduceBlocks > w->part2_cap) {
        if ((rc = realloc_dev(&w->part2, (size_t)(k + 1) * kReduceBlocks))) return rc;
        w->part2_cap = (size_t)(k + 1) * kReduceBlocks;
    }
    hipLaunchKernelGGL(cut_reduce1_kernel, dim3(kReduceBlocks, k + 1), dim3(256), 0, c->stream, (int)slots, k + 1,
                       w->partial, w->part2);
    hipLaunchKernelGGL(cut_reduce2_kernel, dim3((k + 1 + 63) / 64), dim3(64), 0, c->stream, k + 1, w->part2, d_sums);
    HIPCHK(hipGetLastError());
    return TWOSD_OK;
}

// g = sum_v h_v pi_v, then alpha / beta on the host
static int cut_finalize_impl(twosd_ctx *c, const double *x, const unsigned long long *d_hist, const double *d_sums,
                             double *alpha, double *beta) {
    CutWs *w = cws(c);
    const int nv = c->dvs.size, m = c->L.m, k = c->k, n1 = c->n1;
    (void)x;
    const int chunk = 256;
    const int nb = std::max(1, (nv + chunk - 1) / chunk);
    int rc;
    if ((size_t)nb * m > w->gpart_cap) {
        if ((rc = realloc_dev(&w->gpart, (size_t)nb * m))) return rc;
        w->gpart_cap = (size_t)nb * m;
    }
    hipLaunchKernelGGL(cut_g_partial_kernel, dim3(nb), dim3(256), 0, c->stream, nv, m, chunk, d_hist, c->dvs.V, w->gpart);
    hipLaunchKernelGGL(cut_g_final_kernel, dim3((m + 255) / 256), dim3(256), 0, c->stream, nb, m, w->gpart, w->g);
    HIPCHK(hipGetLastError());
    std::vector<double> g(m), sums(k + 1);
    HIPCHK(hipMemcpyAsync(g.data(), w->g, sizeof(double) * m, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(sums.data(), d_sums, sizeof(double) * (k + 1), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    double a = 0.0;
    for (int i = 0; i < m; ++i) a += g[i] * c->r[i];
    for (int jj = 0; jj < n1; ++jj) {
        double s = 0.0;
        for (int i = 0; i < m; ++i) s += c->T[(size_t)i * n1 + jj] * g[i];
        beta[jj] = -s;
    }
    for (int e = 0; e < k; ++e) {
        if (c->pos_col[e] < 0) a += sums[1 + e];
        else beta[c->pos_col[e]] -= sums[1 + e];
    }
    *alpha = a;
    return TWOSD_OK;
}

}  // namespace twosd

using namespace twosd;

static int check_cut_args(twosd_ctx *c, int epi, const double *x) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "build_cut: no template");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "build_cut: epigraph %d does not exist", epi);
    if (c->n1 > 0 && !x) return fail(TWOSD_E_ARG, "build_cut: x is NULL");
    if (c->dvs.size == 0)
        return fail(TWOSD_E_STATE, "build_cut: the dual vertex set is empty (UndefRefError in build_sasa_cut, epigraph.jl:140)");
    return TWOSD_OK;
}

extern "C" int twosd_build_cut(twosd_ctx *c, int epi, const double *x, double tie_rel, double *alpha, double *beta,
                               double *weight_mark, double *max_val, int *max_arg) {
    int rc = check_cut_args(c, epi, x);
    if (rc) return rc;
    if (!alpha || (c->n1 > 0 && !beta)) return fail(TWOSD_E_ARG, "build_cut: alpha/beta NULL");
    HIPCHK(hipSetDevice(c->device));
    const EpiDevice &E = c->epis[epi];
    CutWs *w = cws(c);
    const int nv = c->dvs.size;
    if ((size_t)nv > w->hist_cap) {
        if ((rc = realloc_dev(&w->hist, nv))) return rc;
        w->hist_cap = nv;
    }
    if ((size_t)(c->k + 1) > w->sums_cap) {
        if ((rc = realloc_dev(&w->sums, c->k + 1))) return rc;
        w->sums_cap = c->k + 1;
    }
    if (E.count == 0 || E.total_weight <= 0.0) {
        // no scenarios: the reference returns the zero cut with weight_mark = total weight
        *alpha = 0.0;
        for (int j = 0; j < c->n1; ++j) beta[j] = 0.0;
        if (weight_mark) *weight_mark = E.total_weight;
        return TWOSD_OK;
    }
    HIPCHK(hipEventRecord(c->ev[4], c->stream));
    if ((rc = cut_partial_impl(c, epi, x, tie_rel, E.total_weight, w->hist, w->sums))) return rc;
    HIPCHK(hipEventRecord(c->ev[5], c->stream));
    if ((rc = cut_finalize_impl(c, x, w->hist, w->sums, alpha, beta))) return rc;
    HIPCHK(hipEventRecord(c->ev[6], c->stream));
    HIPCHK(hipEventSynchronize(c->ev[6]));
    float ms1 = 0, ms2 = 0;
    hipEventElapsedTime(&ms1, c->ev[4], c->ev[5]);
    hipEventElapsedTime(&ms2, c->ev[5], c->ev[6]);
    c->t_us[2] = 1e3 * ms1;
    c->t_us[3] = 1e3 * ms2;
    if (weight_mark) *weight_mark = E.total_weight;
    if (max_val) HIPCHK(hipMemcpy(max_val, w->val, sizeof(double) * E.count, hipMemcpyDeviceToHost));
    if (max_arg) HIPCHK(hipMemcpy(max_arg, w->arg, sizeof(int) * E.count, hipMemcpyDeviceToHost));
    return TWOSD_OK;
}

extern "C" int twosd_cut_partial_len(twosd_ctx *c, int64_t *n_u64, int64_t *n_f64) {
    if (!c) return fail(TWOSD_E_ARG, "cut_partial_len: NULL");
    if (n_u64) *n_u64 = std::max(c->dvs.size, 1);
    if (n_f64) *n_f64 = c->k + 1;
    return TWOSD_OK;
}

extern "C" int twosd_cut_partial(twosd_ctx *c, int epi, const double *x, double tie_rel, double total_weight,
                                 uint64_t *d_hist, double *d_sums, double *max_val, int *max_arg) {
    int rc = check_cut_args(c, epi, x);
    if (rc) return rc;
    if (!d_hist || !d_sums) return fail(TWOSD_E_ARG, "cut_partial: device buffers NULL");
    if (!(total_weight > 0.0)) return fail(TWOSD_E_ARG, "cut_partial: total_weight must be > 0");
    HIPCHK(hipSetDevice(c->device));
    const EpiDevice &E = c->epis[epi];
    if (E.count == 0) {
        HIPCHK(hipMemsetAsync(d_hist, 0, sizeof(uint64_t) * std::max(c->dvs.size, 1), c->stream));
        HIPCHK(hipMemsetAsync(d_sums, 0, sizeof(double) * (c->k + 1), c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        return TWOSD_OK;
    }
    HIPCHK(hipEventRecord(c->ev[4], c->stream));
    if ((rc = cut_partial_impl(c, epi, x, tie_rel, total_weight, (unsigned long long *)d_hist, d_sums))) return rc;
    HIPCHK(hipEventRecord(c->ev[5], c->stream));
    HIPCHK(hipEventSynchronize(c->ev[5]));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev[4], c->ev[5]);
    c->t_us[2] = 1e3 * ms;
    CutWs *w = cws(c);
    if (max_val) HIPCHK(hipMemcpy(max_val, w->val, sizeof(double) * E.count, hipMemcpyDeviceToHost));
    if (max_arg) HIPCHK(hipMemcpy(max_arg, w->arg, sizeof(int) * E.count, hipMemcpyDeviceToHost));
    return TWOSD_OK;
}

extern "C" int twosd_cut_finalize(twosd_ctx *c, const double *x, const uint64_t *d_hist, const double *d_sums,
                                  double *alpha, double *beta) {
    if (!c || !c->has_template || !d_hist || !d_sums || !alpha || (c->n1 > 0 && !beta))
        return fail(TWOSD_E_ARG, "cut_finalize: bad arguments");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventRecord(c->ev[5], c->stream));
    int rc = cut_finalize_impl(c, x, (const unsigned long long *)d_hist, d_sums, alpha, beta);
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev[6], c->stream));
    HIPCHK(hipEventSynchronize(c->ev[6]));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev[5], c->ev[6]);
    c->t_us[3] = 1e3 * ms;
    return TWOSD_OK;
}
