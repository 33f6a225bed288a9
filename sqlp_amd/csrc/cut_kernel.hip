// cut_kernel.hip -- argmax_procedure + build_sasa_cut on gfx950 (fp64 MFMA).
//
// Reference: argmax_procedure (src/sd_algorithm/subprob.jl:141-169) and build_sasa_cut
// (src/sd_algorithm/epigraph.jl:125-146).  For scenario w (element deltas dv[w,e] at
// rows row_e; coef_e = 1 for an RHS element, -x[col_e] for a T element):
//     score[w,v] = pi_v . (r - T x)  +  sum_e pi_v[row_e] * coef_e * dv[w,e]
//                = base[v]          +  (DR_w . PK_v)           (an N x |V| x k GEMM)
//     a(w)  = lowest v within tie_rel*(1+|max|) of max_v score[w,v]   (tie_rel=0: the
//             reference's strict '>' first maximum)
// The DECISION is made on scores evaluated in the restatement's arithmetic order
// (oracle/cpu_lp.c oracle_build_cut; subprob.jl:147-158 with the dots sequential, no
// contraction): base[v] = sum_i pi_v[i] * bvec[i] in index order, then
// score = base[v] + (sum_e pi_v[row_e] * (coef_e dv[w,e]) in element order).  The MFMA pass
// computes every score to within a bound `band` of that value (both share base[v]; the
// k-term dot differs by at most 2 gamma_{k+4} sum|terms|), so a row whose band around the
// MFMA maximum holds ONE vertex is decided; a row with several (real ties: degenerate
// scenarios whose optimal duals are all in V) is re-decided by cut_fixup_kernel, which
// evaluates the logged in-band candidates in the restatement's order -- the same pick as the
// C port, bit for bit, at any tie.
//   candidate log: while a lane scans its vertices it appends every vertex whose MFMA score
//   reaches the running band [M - tol(M) - band, ...]; the band's floor only rises with M, so
//   the log is a superset of the final band (a jump past the band restarts it).
//     p_w   = weight_w / total_weight
//     alpha = g.r + sum_{e RHS} S_e,   beta = -T' g - sum_{e T} S_e e_{col_e}
// with g = sum_v h_v pi_v,  h_v = sum_{w: a(w)=v} p_w,  S_e = sum_w p_w PK[a(w),e] dv[w,e].
// (Same value as the reference's per-scenario loop, re-associated.)
//
// Kernels:
//   cut_pk_kernel      PK (|V| x k4 row-major), PKT (k4 x vcap) and PKO (PK's columns in the
//                      restated element order) gathers of new vertices
//   cut_vbase_kernel   base[v] = pi_v . (r - T x) in index order (8|V|(m+1) bytes) and the
//                      decision band (max_v |base[v]| + sum_e |PK[v,e] coef_e| dmax_e)
//   cut_pktc_kernel    PKTc = coef(x) * PKT plus the base row: the chunk source of the argmax
//   cut_argmax2_kernel MFMA score tiles (v_mfma_f64_16x16x4f64: 32 vertices x 32 scenarios
//                      per wave and chunk), vertex chunks DMA'd into LDS, running max/argmax
//                      per scenario in registers; per-wave partial sums; h via uint64
//                      fixed-point atomics (exact and order independent -> identical on any
//                      rank count); the last round's tiles split by vertex range
//   cut_tail_merge_kernel  per-range results of the split tiles merged in vertex order
//   cut_fixup_kernel   scenarios with several vertices in the decision band: their logged
//                      candidates re-scored in the restatement's order and decided by its rule
//   cut_rescan_kernel  the few whose candidate log overflowed: every vertex re-scored
//   cut_reduce_kernel  deterministic fixed-order sum of the partial slots
//   cut_g_kernel(s)    g = sum_v h_v pi_v (two-level, fixed order)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <math.h>
#include <algorithm>
#include <cstdlib>
#include <cstring>
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
    const double *PKO;     // nv x k4: PK with its columns in the restated order (PKO[v][q] = PK[v][eord[q]])
    const double *PKTc;    // 4 KB x vcap32: coef_e(x) * PKT over the argmax's vertices, zero padded (cut_argmax2_kernel's LDS-DMA source)
    int vcap32;            // row stride of PKTc (a multiple of 32 >= nv)
    const int *vmap;       // the argmax's vertices (dominated twins left out), ascending: column c of PKTc is vertex vmap[c]
    const int *nvc;        // their count (device: set per x by cut_compact_kernel)
    const double *PKOc;    // PKO rows of the argmax's vertices (row c: vertex vmap[c]), per x
    const double *basec;   // base of the argmax's vertices, per x (vcap32 entries; past nvc unused)
    const double *base;    // nv: pi_v . bvec in index order (the restatement's base dot)
    const int *eord;       // k: elements by ascending row (the restated score's order)
    const unsigned long long *band_bits;   // the ACTIVE band of this cut, as bits (cut_band_select_kernel)
    const unsigned long long *mode;        // 1: this cut's MFMA pass runs in fp32 (cut_argmax3_kernel), 0: fp64 (cut_argmax2_kernel)
    const float *basec32;  // vcap32: basec rounded up to fp32 (-inf past nvc): the fp32 pass's prefilter
    const float *PKTc32;   // KR32 x vcap32: PKTc's element rows rounded to fp32, no base row (cut_argmax3_kernel's LDS-DMA source)
    double band_scale;     // 4 gamma_{k+4}: twice the 2 gamma bound
    int *arg; double *val; int *flag;   // N; flag != 0: re-decide (main rows: 4-bit log counts per lane group)
    int *cand;             // candidate logs of the whole tiles: [(s * 4 + g) * kCandC + i]
    unsigned long long *fstats;   // fixup counters: re-decided scenarios, candidates scored, full re-scans
    int *tcand;            // of the tail ranges: [(((s - t0) * tail_S + range) * 4 + g) * kCandC + i]
    unsigned long long *hist;           // nv (fixed point)
    unsigned long long *hist_part;      // gridDim.x x nv block histograms (hist_lds mode)
    double *partial;       // slots x (k + 1): [sum p*val, S_0..S_{k-1}]
    // work units of cut_argmax2_kernel: units [0, full_units) are whole scenario tiles; the
    // tiles past them (the last, partial round of the persistent grid) are cut into tail_S
    // vertex ranges each, and such a unit leaves its per-scenario (M, I, log counts) in tp_* at
    // [(s - 128 full_units) tail_S + range] for cut_tail_merge_kernel
    int full_units, tail_S;
    int fx_gs;             // cut_fixup_kernel: whole-tile scenarios per wave step (64; 32 / 16 for small batches)
    double *tp_m;
    int *tp_i, *tp_f;
};

constexpr int kCandC = 16;         // logged candidates per (scenario, lane group); count kCandC + 1 = overflow
constexpr int kCandBits = 5;       // bits of one lane group's count in a packed flag (4 groups: 20 bits)
static_assert(4 * kCandC == 64, "one 64-lane step of the fixup's enumeration covers one scenario's log slots");

__global__ void cut_pk_kernel(int from, int to, int m, int k, int k4, int vcap, const int *__restrict__ rows,
                              const int *__restrict__ eord, const double *__restrict__ V, double *__restrict__ PK,
                              double *__restrict__ PKT, double *__restrict__ PKO) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = (to - from) * k4;
    if (idx >= total) return;
    const int v = from + idx / k4, e = idx % k4;
    const double x = e < k ? V[(size_t)v * m + rows[e]] : 0.0;
    PK[(size_t)v * k4 + e] = x;
    PKT[(size_t)e * vcap + v] = x;
    PKO[(size_t)v * k4 + e] = e < k ? V[(size_t)v * m + rows[eord[e]]] : 0.0;   // column q = e in the restated order
}

// Twin vertices.  Two vertices whose PK rows are bit-identical have bit-identical restated dot
// terms t for every scenario, so at an x where their bases are equal too their restated scores
// are equal for every scenario: the lower index wins under both rules (the first strict maximum;
// the lowest index within the tie window), and the higher one can never be picked.  storm's
// duals come in such groups (vertices differing only on rows where r - T x is 0), and each one
// made every scenario it won an exact tie the fixup had to re-decide.  tprev[v] is the previous
// vertex of v's PK-equality group (-1: none), maintained with PK; cut_pktc_kernel drops a vertex
// whose base equals that of an earlier group member at this x (cut_compact_kernel).
__global__ void cut_twin_hash_kernel(int from, int to, int k4, const double *__restrict__ PK, unsigned long long *__restrict__ phash) {
    const int v = from + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= to) return;
    unsigned long long h = 0x9e3779b97f4a7c15ull;
    for (int e = 0; e < k4; ++e) {
        h ^= (unsigned long long)__double_as_longlong(PK[(size_t)v * k4 + e]) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
        h *= 0xff51afd7ed558ccdull;
    }
    phash[v] = h;
}

__global__ void cut_iota_kernel(int *v, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

// tprev[v] = the highest u < v with PK row u bit-identical to PK row v (one wavefront per vertex)
__global__ void __launch_bounds__(256) cut_twin_prev_kernel(int from, int to, int k4, const double *__restrict__ PK,
                                                            const unsigned long long *__restrict__ phash, int *__restrict__ tprev) {
    const int lane = threadIdx.x & 63;
    const int v = from + ((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (v >= to) return;   // wave-uniform
    const unsigned long long hv = phash[v];
    int best = -1;
    for (int u = v - 1 - lane; u >= 0 && best < 0; u -= 64) {
        if (phash[u] != hv) continue;
        bool same = true;
        for (int e = 0; e < k4 && same; ++e)
            same = __double_as_longlong(PK[(size_t)u * k4 + e]) == __double_as_longlong(PK[(size_t)v * k4 + e]);
        if (same) best = u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o));
    if (lane == 0) tprev[v] = best;
}

// The argmax's vertex list at x: every vertex except the dominated twins (v whose base equals
// that of an earlier member of its PK-equality group), ascending, so that the MFMA pass does no
// work for them and "lowest index" keeps its meaning.  One block; tprev == nullptr keeps all.
__global__ void __launch_bounds__(1024) cut_compact_kernel(int nv, const double *__restrict__ base, const int *__restrict__ tprev,
                                                           int *__restrict__ vmap, int *__restrict__ nvc,
                                                           unsigned long long *__restrict__ ntwin) {
    __shared__ int wsum[16];
    __shared__ int off;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) off = 0;
    __syncthreads();
    for (int v0 = 0; v0 < nv; v0 += 1024) {
        const int v = v0 + threadIdx.x;
        bool keep = v < nv;
        if (keep && tprev) {
            const double b = base[v];
            for (int u = tprev[v]; u >= 0; u = tprev[u])   // tprev[u] < u: the walk ends
                if (base[u] == b) { keep = false; break; }
        }
        const unsigned long long bal = __ballot(keep);
        const int pos = __popcll(bal & ((1ull << lane) - 1));
        if (lane == 0) wsum[wid] = __popcll(bal);
        __syncthreads();
        int before = off;
        for (int w = 0; w < wid; ++w) before += wsum[w];
        if (keep) vmap[before + pos] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int w = 0; w < 16; ++w) t += wsum[w];
            off += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *nvc = off;
        if (ntwin) *ntwin = (unsigned long long)(nv - off);
    }
}

// The same links for all vertices at once from the (hash, vertex) pairs sorted by hash (stable:
// vertices ascending within a hash): the previous entry of a run with a bit-identical row is the
// highest lower twin.  O(nv log nv) instead of cut_twin_prev_kernel's O(nv^2) for a rebuild.
__global__ void cut_twin_sorted_kernel(int nv, int k4, const double *__restrict__ PK, const unsigned long long *__restrict__ hs,
                                       const int *__restrict__ vs, int *__restrict__ tprev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const int v = vs[i];
    int prev = -1;
    for (int j = i - 1; j >= 0 && hs[j] == hs[i]; --j) {   // runs are short (twin groups)
        const int u = vs[j];
        bool same = true;
        for (int e = 0; e < k4 && same; ++e)
            same = __double_as_longlong(PK[(size_t)u * k4 + e]) == __double_as_longlong(PK[(size_t)v * k4 + e]);
        if (same) { prev = u; break; }
    }
    tprev[v] = prev;
}

// PKOc[c] = PKO[vmap[c]], basec[c] = base[vmap[c]] for c < nvc: the fixup works on the argmax's
// positions (its logs hold them), so its candidate loads need no translation
__global__ void cut_compact_rows_kernel(int nv, int k4, const int *__restrict__ vmap, const int *__restrict__ nvc_p,
                                        const double *__restrict__ PKO, const double *__restrict__ base,
                                        double *__restrict__ PKOc, double *__restrict__ basec, int vcap32, float *__restrict__ basec32) {
    const int nvc = *nvc_p;
    // basec32[c] = the least float >= base[vmap[c]] (-inf past nvc): an upper bound of the base, so
    // the fp32 prefilter of cut_argmax3_kernel never rejects a score the fp64 test would accept
    if (basec32)
        for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < vcap32; c += gridDim.x * blockDim.x)
            basec32[c] = c < nvc ? __double2float_ru(base[vmap[c]]) : -INFINITY;
    const size_t total = (size_t)nv * k4;
    for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(idx / k4), q = (int)(idx % k4);
        if (c >= nvc) continue;
        const int v = vmap[c];
        PKOc[idx] = PKO[(size_t)v * k4 + q];
        if (q == 0) basec[c] = base[v];
    }
}

// PKTc[kk][c] = coef_kk * PKT[kk][vmap[c]] over rows [0, rows) x columns [0, vcap32), zero
// outside [0, k) x [0, nvc) (the LDS-DMA source of cut_argmax2_kernel; per x).
// With base != nullptr, row k holds base[vmap[c]] (-inf for c >= nvc): the MFMA then adds the
// vertex base through a constant 1 in the scenarios' delta column k.
// PKTc32 (rows32 rows, may be null): the element rows of PKTc rounded to fp32, zero past k (the
// fp32 pass adds the base in fp64 outside the MFMA)
__global__ void cut_pktc_kernel(int k, int rows, int vcap, int vcap32, const double *__restrict__ PKT,
                                const double *__restrict__ coef, const double *__restrict__ base, const int *__restrict__ vmap,
                                const int *__restrict__ nvc_p, double *__restrict__ PKTc, int rows32, float *__restrict__ PKTc32) {
    const int nvc = *nvc_p;
    const size_t total = (size_t)std::max(rows, PKTc32 ? rows32 : 0) * vcap32;
    for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
        const int kk = (int)(idx / vcap32), c = (int)(idx % vcap32);
        const int v = c < nvc ? vmap[c] : 0;
        const double pc = (kk < k && c < nvc) ? coef[kk] * PKT[(size_t)kk * vcap + v] : 0.0;
        double x = pc;
        if (base && kk == k) x = c < nvc ? base[v] : -INFINITY;
        if (kk < rows) PKTc[idx] = x;
        if (PKTc32 && kk < rows32) PKTc32[idx] = (float)pc;
    }
}

// base[v] = sum_i V[v][i] * bvec[i] in index order with every product and sum rounded on its
// own (oracle_build_cut's vb[v]), one wavefront per vertex: the lanes form the products of a
// 512-entry slice in LDS, lane 0 adds them in order.  The wave also folds the vertex's term of
// the decision band: |base[v]| + sum_e |PK[v,e] coef_e| dmax_e (any order: a bound).
constexpr int kVbSlice = 512;
__global__ void __launch_bounds__(256) cut_vbase_kernel(int nv, int m, int k, int k4, const double *__restrict__ V,
                                                        const double *__restrict__ bvec, const double *__restrict__ PK,
                                                        const double *__restrict__ coef, const unsigned long long *__restrict__ dmax,
                                                        double *__restrict__ base, unsigned long long *__restrict__ band_bits,
                                                        double band_scale, double band_scale32) {
#pragma clang fp contract(off)
    __shared__ double prod[4][kVbSlice];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int v0 = blockIdx.x * 4; v0 < nv; v0 += gridDim.x * 4) {   // block-uniform trip count
        const int v = v0 + wid;
        const bool act = v < nv;
        const double *p = V + (size_t)(act ? v : 0) * m;
        double s = 0.0;
        for (int i0 = 0; i0 < m; i0 += kVbSlice) {
            const int n = min(kVbSlice, m - i0);
            if (act)
                for (int i = lane; i < n; i += 64) prod[wid][i] = p[i0 + i] * bvec[i0 + i];
            __syncthreads();
            if (act && lane == 0) {
#pragma unroll 8
                for (int i = 0; i < n; ++i) s = s + prod[wid][i];
            }
            __syncthreads();
        }
        if (!act) continue;
        double a = 0.0, pm = 0.0, dm = 0.0;
        for (int e = lane; e < k; e += 64) {
            const double pc = fabs(PK[(size_t)v * k4 + e] * coef[e]), de = __longlong_as_double((long long)dmax[e]);
            a += pc * de;
            pm = fmax(pm, pc);
            dm = fmax(dm, de);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a += __shfl_xor(a, o);
            pm = fmax(pm, __shfl_xor(pm, o));
            dm = fmax(dm, __shfl_xor(dm, o));
        }
        if (lane == 0) {
            base[v] = s;
            const double t = fabs(s) + a;
            // the band itself (a positive scale keeps the order of the maxima, rounding included)
            const double b64 = isfinite(t) ? band_scale * t : INFINITY;
            atomicMax(band_bits, (unsigned long long)__double_as_longlong(b64));
            // the fp32 pass: the element terms rounded to fp32 and summed by an fmaf chain (the f32
            // MFMA's arithmetic) differ from the exact dot by at most gamma_{k+2}(u32) a, plus
            // 2^-126 (1 + max|PK coef| + max dmax) per term for operands and partial sums below
            // the normal range; scale32 = 4 gamma_{k+4}(u32) doubles that bound as band_scale does.
            // The base stays fp64 (the restatement's own value), so the fp64 band is added.
            const double b32 = b64 + band_scale32 * a + 4.0 * (k + 4) * ldexp(1.0, -126) * (1.0 + pm + dm);
            atomicMax(band_bits + 1, (unsigned long long)__double_as_longlong(isfinite(b32) ? b32 : INFINITY));
            // operands and sums well inside the fp32 range, or the cut runs the fp64 pass
            const double lim = ldexp(1.0, 100);
            if (!(a < lim && pm < lim && dm < lim)) atomicOr(band_bits + 2, 1ull);
        }
    }
}

// the cut's pass: fp32 when asked and every vertex's operands fit (band_bits[2] == 0), else
// fp64; band_bits[3] = that pass's band (what every later kernel of the cut reads), [4] = the pass
__global__ void cut_band_select_kernel(unsigned long long *band_bits, int want32) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const unsigned long long m = (want32 && band_bits[2] == 0) ? 1ull : 0ull;
    band_bits[3] = m ? band_bits[1] : band_bits[0];
    band_bits[4] = m;
}

// dmax[e] = max |dv[s][e]| over scenarios [from, to) folded into the epigraph's running maximum
// (non-negative doubles order as their bit patterns)
__global__ void __launch_bounds__(256) cut_dmax_kernel(int from, int to, int k, const double *__restrict__ dv,
                                                       unsigned long long *__restrict__ dmax) {
    if ((int)threadIdx.x >= k) return;
    const int e = threadIdx.x;
    double mx = 0.0;
    for (int s = from + blockIdx.x; s < to; s += gridDim.x) mx = fmax(mx, fabs(dv[(size_t)s * k + e]));   // NaN ignored: its scores never win
    atomicMax(&dmax[e], (unsigned long long)__double_as_longlong(mx));
}

// the decision band of this cut (written by cut_vbase_kernel) through the scalar cache: a
// wave-uniform value held in SGPRs rather than a VGPR pair (the 3-blocks-per-CU argmax would
// spill it)
__device__ __forceinline__ double cut_band_scalar(const CutParams &P) {
    return __longlong_as_double((long long)((const __attribute__((address_space(4))) unsigned long long *)P.band_bits)[0]);
}

// floor of the decision band around a running maximum M: a vertex below it cannot be the
// restatement's pick (monotone in M for tie_rel < 1)
__device__ __forceinline__ double band_floor(double M, double rel, double band) { return M - (rel * (1.0 + fabs(M)) + band); }

// Running state of one scenario row over the vertices one lane sees, in increasing vertex
// order: M = max so far, thr = band_floor(M), I = the first vertex scoring M, n = entries in
// this lane's candidate log (kCandC + 1: overflowed), f = its first entry.  The first entry
// stays in a register and is stored (log[0]) only for a row the fixup will read: most rows
// just raise their maximum past the band again and again, and each raise restarts the log.
struct RowEx { double M, thr; int I, n, f; float thr32; };

// the fp32 prefilter's floor of a row (cut_argmax3_kernel): a float at or below fl32(y) for every
// y >= pred64(thr).  A score s = fl64(base + t) >= thr has base + t >= pred64(thr); with b32 >= base
// (rounded up) and fp32 addition monotone, fl32(b32 + t) >= fl32(pred64(thr)) >= this floor.
// f = RN32(thr) is within one float step of RD32(pred64(thr)); f - |f| 2^-21 (rounded) lies at least
// three float steps lower, and the 2^-140 covers the subnormal range.  -inf stays -inf; past FLT_MAX
// the floor is FLT_MAX (every y there rounds to +inf)
__device__ __forceinline__ float thr32_of(double thr) {
    const float f = (float)thr;
    if (f == INFINITY) return 3.40282347e38f;
    return fmaf(-fabsf(f), 0x1p-21f, f) - 0x1p-140f;
}

// s >= thr: s enters the band of the running max (or raises it).  HOLD: the first entry is kept
// in b.f (stored at the end of the tile for the rows the fixup reads); otherwise it is stored at
// once (the instantiations at 3 blocks per CU have no register to spare for it)
template <bool HOLD>
__device__ __forceinline__ void row_log(RowEx &b, double s, int v, double rel, double band, int *lbase, unsigned lo) {
    if (s == -INFINITY) return;                  // padding vertices (-inf base row) never enter
    // the 3-blocks build: an opaque copy, so the entry addresses are formed here, on this rare path,
    // instead of being hoisted out of the chunk loop as 64-bit values that would spill
    if (!HOLD) asm volatile("" : "+v"(lo));
    const double tn = band_floor(s, rel, band);
    if (tn > b.M) {                              // every earlier entry is below the band for good
        if (HOLD) b.f = v;
        else lbase[lo] = v;
        b.n = 1;
    } else {
        if (HOLD && b.n == 0) b.f = v;
        else if (b.n < kCandC) lbase[lo + b.n] = v;
        b.n = min(b.n + 1, kCandC + 1);
    }
    if (s > b.M) { b.M = s; b.I = v; b.thr = tn; b.thr32 = thr32_of(tn); }
}

template <bool HOLD>
__device__ __forceinline__ void row_fast(RowEx &b, double s, int v, double rel, double band, int *lbase, unsigned lo) {
    if (__builtin_expect(s >= b.thr, 0)) row_log<HOLD>(b, s, v, rel, band, lbase, lo);
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
constexpr int kVT2 = 32;                 // vertices per LDS chunk (two 16-vertex MFMA tiles)
constexpr int kCutTile2 = 128;           // scenarios per block tile (4 waves x 2 x 16)
constexpr int kLdsRow2 = 32;             // doubles per k-row of a chunk

// LDS position of (k-row kk, vertex vv): odd rows have their 16-double halves swapped, so the
// two k-rows a half-wave reads together (g = 0, 1 / 2, 3) fall on disjoint banks
__device__ __forceinline__ int lds2(int kk, int vv) { return kk * kLdsRow2 + (vv ^ ((kk & 1) << 4)); }

// The value of a decided row in fp64, the same bits in every pass, split and kernel: base[I] + t,
// t = (c_0 + c_1) + (c_2 + c_3), c_g the fma chain over e = g, g + 4, g + 8, ... < k of
// (PK[I,e] coef_e) dv_e from 0.  dec_lane_chain is lane (g, .)'s c_g from its register deltas
// d[kb] (e = 4 kb + g); dec_combine the xor-16 / xor-32 sum that forms t on every lane of the column.
template <int KB, typename D>
__device__ __forceinline__ double dec_lane_chain(const CutParams &P, const double *pk, const D (&d)[KB], int g) {
    double c = 0.0;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
        const int e = 4 * kb + g;
        if (e < P.k) c = fma(pk[e] * P.coef[e], (double)d[kb], c);
    }
    return c;
}
__device__ __forceinline__ double dec_combine(double c) {
    c += __shfl_xor(c, 16);
    return c + __shfl_xor(c, 32);
}

// Combine the 4 lanes (g) of a scenario column: the row maximum M, and for each lane the number
// of its logged entries that can lie in the band of M (0 when the lane's own max is below the
// band floor).  tot == 1: the row is decided, its pick the first vertex of the one lane that
// reaches the band; otherwise the row is re-decided from the logs, whose lengths `pack` holds
// (kCandBits per lane group; kCandC + 1 = overflowed).  Every lane of the column ends with the result.
__device__ __forceinline__ void combine_ex(RowEx &rb, double rel, double band, int g, int &pack, int &tot) {
    double M = rb.M;
    M = fmax(M, __shfl_xor(M, 16));
    M = fmax(M, __shfl_xor(M, 32));
    const double thr = band_floor(M, rel, band);
    const int n = (rb.M != -INFINITY && rb.M >= thr) ? rb.n : 0;
    int pk = n << (kCandBits * g);
    tot = n;
    int it = n ? rb.I : 0x7fffffff;
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
        tot += __shfl_xor(tot, o);
        pk |= __shfl_xor(pk, o);
        it = min(it, __shfl_xor(it, o));
    }
    rb.M = M;
    rb.I = (M == -INFINITY || it == 0x7fffffff) ? -1 : it;
    pack = pk;
}

#ifndef TWOSD_CUT_LB3
#define TWOSD_CUT_LB3 1                  // 3 blocks per CU for KB <= 22 (168 VGPRs; ssn: 62 -> 76 % of the roofline)
#endif
template <int KB>
__global__ void __launch_bounds__(256, (TWOSD_CUT_LB3 && KB <= 22) ? 3 : 2) cut_argmax2_kernel(CutParams P) {
    if (*P.mode != 0) return;                       // the fp32 pass runs this cut (cut_argmax3_kernel)
    __shared__ double Bs[2][4 * KB * kLdsRow2];     // double-buffered chunk (k-major)
    constexpr bool kHold = !(TWOSD_CUT_LB3 && KB <= 22);   // a register for the logs' first entries (2 blocks per CU)
    extern __shared__ unsigned long long hl[];      // nv entries when P.hist_lds
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar staging loop
    if (P.hist_lds)
        for (int v = threadIdx.x; v < P.nv; v += 256) hl[v] = 0ull;
    const int g = lane >> 4, j = lane & 15;
    const int ntiles = (P.N + kCutTile2 - 1) / kCutTile2;
    const int nchunks = (*P.nvc + kVT2 - 1) / kVT2;   // the argmax's vertices (vmap)
    const int nunits = P.full_units + (ntiles - P.full_units) * P.tail_S;
    const double band = kHold ? __longlong_as_double((long long)*P.band_bits) : cut_band_scalar(P);
    const double rel = P.tie_rel;
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
            if (e == P.k) a0[kb] = a1[kb] = 1.0;   // x the base row of the chunk
        }
        RowEx rb0, rb1;   // scenario s0 + j / s0 + 16 + j over this lane's vertices v0 + g + 4r (+16)
        rb0.M = -INFINITY; rb0.thr = -INFINITY; rb0.I = -1; rb0.n = 0; rb0.f = 0; rb0.thr32 = -INFINITY;
        rb1 = rb0;
        // this lane's candidate logs of the two scenarios (rows padded to whole tiles)
        // (a wave-uniform base and a 32-bit element offset: one VGPR per lane instead of a pointer pair)
        int *const lbase = tail ? P.tcand : P.cand;
        const unsigned log0 = tail ? (unsigned)(((((size_t)(s0 + j - P.full_units * kCutTile2)) * P.tail_S + range) * 4 + g) * kCandC)
                                      : (unsigned)((((size_t)(s0 + j)) * 4 + g) * kCandC);
        const unsigned lstep = 16u * (tail ? P.tail_S : 1) * 4 * kCandC;   // scenario + 16

        // chunk staging by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip): instruction i
        // of the chunk writes k-rows 4i .. 4i+3 (1 KiB, lane-linear), lane L the 16 bytes of
        // row 4i + L/16 at LDS position 2 (L % 16); the source vertex pair is that position with
        // the row's half swap (lds2) applied, so the image is exactly lds2's layout
        auto stage = [&](int buf, int v0) {
            for (int i = wid; i < KB; i += 4) {
                const int kk = 4 * i + (lane >> 4);
                const int vv = (2 * (lane & 15)) ^ ((kk & 1) << 4);
                __builtin_amdgcn_global_load_lds((const void *)(P.PKTc + (size_t)kk * P.vcap32 + v0 + vv),
                                                 (__attribute__((address_space(3))) void *)&Bs[buf][i * 4 * kLdsRow2], 16, 0, 0);
            }
        };
        stage(0, c_lo * kVT2);
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
            // C/D: register r of a tile is vertex row g + 4r, scenario column j; this lane's
            // vertices in increasing order: v0 + g + 4r, then v0 + 16 + g + 4r.  The scores
            // include the base (-inf past nv).
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                row_fast<kHold>(rb0, c00[r], v0 + g + 4 * r, rel, band, lbase, log0);
                row_fast<kHold>(rb1, c01[r], v0 + g + 4 * r, rel, band, lbase, log0 + lstep);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                row_fast<kHold>(rb0, c10[r], v0 + 16 + g + 4 * r, rel, band, lbase, log0);
                row_fast<kHold>(rb1, c11[r], v0 + 16 + g + 4 * r, rel, band, lbase, log0 + lstep);
            }
            __syncthreads();
        }
        int pk0, pk1, nt0, nt1;
        combine_ex(rb0, rel, band, g, pk0, nt0);
        combine_ex(rb1, rel, band, g, pk1, nt1);
        // the logs' first entries, for the rows the fixup reads (every tail row: the merge decides)
        if (kHold && rb0.n > 0 && (tail || nt0 >= 2)) lbase[log0] = rb0.f;
        if (kHold && rb1.n > 0 && (tail || nt1 >= 2)) lbase[log0 + lstep] = rb1.f;
        // the picks as vertex indices (the logs keep vmap positions: the fixup translates them)
        rb0.I = rb0.I >= 0 ? P.vmap[rb0.I] : -1;
        rb1.I = rb1.I >= 0 ? P.vmap[rb1.I] : -1;
        const int sa = s0 + j, sb = s0 + 16 + j;
        if (tail) {   // this vertex range's result; cut_tail_merge_kernel decides and sums
            if (g == 0) {
                const int t0 = P.full_units * kCutTile2;
                // the log lengths of the range's band: the merge decides with the band of the row's
                // maximum over all ranges (a range below it contributes nothing)
                if (sa < P.N) {
                    const size_t o = (size_t)(sa - t0) * P.tail_S + range;
                    P.tp_m[o] = rb0.M; P.tp_i[o] = rb0.I; P.tp_f[o] = pk0;
                }
                if (sb < P.N) {
                    const size_t o = (size_t)(sb - t0) * P.tail_S + range;
                    P.tp_m[o] = rb1.M; P.tp_i[o] = rb1.I; P.tp_f[o] = pk1;
                }
            }
            continue;
        }
        if (nt0 < 2) pk0 = 0;   // decided
        if (nt1 < 2) pk1 = 0;
        const bool ok0 = sa < P.N && !pk0 && rb0.I >= 0, ok1 = sb < P.N && !pk1 && rb1.I >= 0;
        const double p0 = ok0 ? P.w[sa] * P.inv_total : 0.0, p1 = ok1 ? P.w[sb] * P.inv_total : 0.0;
        // decided rows: the pick's fp64 value (dec_lane_chain; flagged rows keep the pass's maximum,
        // the fixup writes their restated value)
        const double tv0 = dec_combine(dec_lane_chain<KB>(P, P.PK + (size_t)(rb0.I >= 0 ? rb0.I : 0) * P.k4, a0, g));
        const double tv1 = dec_combine(dec_lane_chain<KB>(P, P.PK + (size_t)(rb1.I >= 0 ? rb1.I : 0) * P.k4, a1, g));
        const double vl0 = ok0 ? P.base[rb0.I] + tv0 : rb0.M, vl1 = ok1 ? P.base[rb1.I] + tv1 : rb1.M;
        if (g == 0) {
            if (sa < P.N) { P.arg[sa] = rb0.I; P.val[sa] = vl0; P.flag[sa] = pk0; }
            if (sb < P.N) { P.arg[sb] = rb1.I; P.val[sb] = vl1; P.flag[sb] = pk1; }
        }
        // sum p * val and the vertex histogram, scenarios in order (lane 0 reads them from lanes 0-15)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const int ok = __shfl(t == 0 ? (int)ok0 : (int)ok1, jj);
                const int ai = __shfl(t == 0 ? rb0.I : rb1.I, jj);
                const double pp = __shfl(t == 0 ? p0 : p1, jj);
                const double vl = __shfl(t == 0 ? vl0 : vl1, jj);
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

// ---- v3: the fp32 MFMA pass (v_mfma_f32_16x16x4f32: twice the fp64 rate on gfx950, an exact
// fmaf chain).  The layout of v2 with fp32 operands: the vertex chunk (coef_e(x) PK rows rounded
// to fp32, no base row) DMA'd into LDS, the scenario deltas rounded to fp32 in registers.  The
// MFMA gives t32 ~ sum_e PK[v,e] coef_e dv[w,e]; the score is base[v] + t32 in fp64 (the base is
// the restatement's own fp64 value), within the fp32 band of the restated score
// (cut_vbase_kernel), and the decisions, logs, tail ranges and fixup are those of v2 with that
// band.  The f32 C/D layout: register r of a tile is vertex row 4g + r, scenario column j.  At the
// end of a tile the two scenarios' fp64 deltas are read again for the S_e sums and the decided
// rows' values (fp64, from the pick's PK row).
constexpr int kLdsRow3 = 32;             // floats per k-row of an fp32 chunk (32 vertices)
// LDS position of (k-row kk, vertex vv): a 128-byte k-row puts rows kk and kk + 2 on the same
// banks, so rows with (kk >> 1) odd have their 16-float halves swapped: the four k-rows a wave
// reads together (g = 0..3) fall on disjoint banks
__device__ __forceinline__ int lds3(int kk, int vv) { return kk * kLdsRow3 + (vv ^ (((kk >> 1) & 1) << 4)); }
// k-rows staged per chunk: KB k-blocks of 4, rounded up to whole 8-row (1 KiB) DMA instructions
__host__ __device__ constexpr int kr32(int KB) { return 8 * ((KB + 1) / 2); }

typedef float f4 __attribute__((ext_vector_type(4)));
#ifndef TWOSD_CUT3_BPC
#define TWOSD_CUT3_BPC 3                 // blocks per CU the fp32 pass is compiled for (2: storm cut 11.0 ms, ssn 4.7; 3: 10.6, 3.6)
#endif

template <int KB>
__global__ void __launch_bounds__(256, TWOSD_CUT3_BPC) cut_argmax3_kernel(CutParams P) {
    if (*P.mode != 1) return;                       // the fp64 pass runs this cut (cut_argmax2_kernel)
    // the logs' first entries held in a register (as cut_argmax2_kernel at 2 blocks per CU): most
    // candidate steps restart a log, and a held entry is stored only for the rows the fixup reads
#ifndef TWOSD_CUT3_HOLD
#define TWOSD_CUT3_HOLD 1                // first log entries in a register (storm argmax 8.28 -> 8.14 ms at 3 blocks per CU)
#endif
    constexpr bool kHold3 = TWOSD_CUT3_HOLD;
    constexpr int KR = kr32(KB);
    __shared__ float Bs[2][KR * kLdsRow3];          // double-buffered chunk (k-major)
    __shared__ double Bb[3][kVT2];                  // the chunks' fp64 bases (ring of 3: finish reads chunk ch - 1)
    extern __shared__ unsigned long long hl[];      // nv entries when P.hist_lds
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (P.hist_lds)
        for (int v = threadIdx.x; v < P.nv; v += 256) hl[v] = 0ull;
    const int g = lane >> 4, j = lane & 15;
    const int ntiles = (P.N + kCutTile2 - 1) / kCutTile2;
    const int nvc = *P.nvc;
    const int nchunks = (nvc + kVT2 - 1) / kVT2;
    const int nunits = P.full_units + (ntiles - P.full_units) * P.tail_S;
    const double band = cut_band_scalar(P);
    const double rel = P.tie_rel;
    double pv_sum = 0.0;
    double Sacc[2] = {0.0, 0.0};   // lane (g, j): e = 4 kb + g for kb = j, j + 16
#ifdef TWOSD_CUT3_COUNT
    unsigned long long cnt_steps = 0, cnt_rare = 0, cnt_lanes = 0;
#endif

    for (int unit = blockIdx.x; unit < nunits; unit += gridDim.x) {
        const bool tail = unit >= P.full_units;
        const int tile = tail ? P.full_units + (unit - P.full_units) / P.tail_S : unit;
        const int range = tail ? (unit - P.full_units) % P.tail_S : 0;
        const int c_lo = tail ? (int)((long long)nchunks * range / P.tail_S) : 0;
        const int c_hi = tail ? (int)((long long)nchunks * (range + 1) / P.tail_S) : nchunks;
        const int s0 = tile * kCutTile2 + wid * 32;
        const int sa = s0 + j, sb = s0 + 16 + j;
        float a0[KB], a1[KB];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            const int e = 4 * kb + g;
            a0[kb] = (sa < P.N && e < P.k) ? (float)P.dv[(size_t)sa * P.k + e] : 0.0f;
            a1[kb] = (sb < P.N && e < P.k) ? (float)P.dv[(size_t)sb * P.k + e] : 0.0f;
        }
        RowEx rb0, rb1;
        rb0.M = -INFINITY; rb0.thr = -INFINITY; rb0.I = -1; rb0.n = 0; rb0.f = 0; rb0.thr32 = -INFINITY;
        rb1 = rb0;
        int *const lbase = tail ? P.tcand : P.cand;
        const unsigned log0 = tail ? (unsigned)(((((size_t)(s0 + j - P.full_units * kCutTile2)) * P.tail_S + range) * 4 + g) * kCandC)
                                      : (unsigned)((((size_t)(s0 + j)) * 4 + g) * kCandC);
        const unsigned lstep = 16u * (tail ? P.tail_S : 1) * 4 * kCandC;

        // LDS-DMA staging (global_load_lds_dwordx4): instruction i writes k-rows 8i .. 8i+7 (1 KiB,
        // lane-linear), lane L the 4 floats at LDS position 4 (L % 8) of row 8i + L/8; the source
        // vertices are that position with lds3's half swap applied
        auto stage = [&](int buf, int bslot, int v0) {
            for (int i = wid; i < KR / 8; i += 4) {
                const int kk = 8 * i + (lane >> 3);
                const int vv = (4 * (lane & 7)) ^ (((kk >> 1) & 1) << 4);
                __builtin_amdgcn_global_load_lds((const void *)(P.PKTc32 + (size_t)kk * P.vcap32 + v0 + vv),
                                                 (__attribute__((address_space(3))) void *)&Bs[buf][i * 8 * kLdsRow3], 16, 0, 0);
            }
            // the 32 fp64 bases (256 bytes: lanes 0..15 of the last wave, 16 bytes each)
            if (wid == 3 && lane < 16)
                __builtin_amdgcn_global_load_lds((const void *)(P.basec + v0 + 2 * lane),
                                                 (__attribute__((address_space(3))) void *)&Bb[bslot][0], 16, 0, 0);
        };
        // this lane's 8 vertices of a chunk (positions v0 + 4g + r, v0 + 16 + 4g + r) as prefilter
        // bases (basec32: rounded up, -inf past the argmax's vertices), two 16-byte loads issued one
        // chunk ahead of their use
        auto load_bases = [&](float (&bq)[8], int v0) {
            const f4 lo = *reinterpret_cast<const f4 *>(P.basec32 + v0 + 4 * g);
            const f4 hi = *reinterpret_cast<const f4 *>(P.basec32 + v0 + 16 + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) { bq[r] = lo[r]; bq[4 + r] = hi[r]; }
        };
        // the chunk's 16 scores of this lane, finished one chunk late (under chunk ch + 1's MFMAs).
        // Prefilter in fp32: b32 + t >= thr32 for every score the fp64 test (base + t >= thr, t the
        // MFMA's fp32 value) accepts (thr32_of); most chunks raise no row's band floor, so one
        // wave-wide test skips the rest.  A lane past it re-scores its 8 vertices exactly (fp64
        // bases) and runs the decisions in vertex order
        auto finish = [&](const f4 &q00, const f4 &q01, const f4 &q10, const f4 &q11, const float (&bb)[8], int vb, int bslot) {
            // per row, the bit mask of this lane's vertices (r = 0..7, increasing vertex order) past
            // the prefilter
            unsigned m0 = 0, m1 = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                m0 |= (unsigned)(bb[r] + q00[r] >= rb0.thr32) << r;
                m1 |= (unsigned)(bb[r] + q01[r] >= rb1.thr32) << r;
                m0 |= (unsigned)(bb[4 + r] + q10[r] >= rb0.thr32) << (4 + r);
                m1 |= (unsigned)(bb[4 + r] + q11[r] >= rb1.thr32) << (4 + r);
            }
#ifdef TWOSD_CUT3_COUNT
            ++cnt_steps;
            if (__builtin_amdgcn_ballot_w64((m0 | m1) != 0) != 0) { ++cnt_rare; cnt_lanes += __popcll(__builtin_amdgcn_ballot_w64((m0 | m1) != 0)); }
#endif
            // the exact steps, one passing vertex per row and lane per round (lowest first: each
            // row still sees its vertices in increasing order), the fp64 base from the chunk's LDS slot
            while (__builtin_amdgcn_ballot_w64((m0 | m1) != 0) != 0) {
                const int r0 = m0 ? __builtin_ctz(m0) : 0, r1 = m1 ? __builtin_ctz(m1) : 0;
                const int o0 = (r0 >> 2) * 16 + 4 * g + (r0 & 3), o1 = (r1 >> 2) * 16 + 4 * g + (r1 & 3);
                const double b0 = Bb[bslot][o0], b1 = Bb[bslot][o1];
                const float t0 = r0 < 4 ? q00[r0 & 3] : q10[r0 & 3];
                const float t1 = r1 < 4 ? q01[r1 & 3] : q11[r1 & 3];
                const double s0 = (vb + o0 < nvc ? b0 : -INFINITY) + (double)t0;
                const double s1 = (vb + o1 < nvc ? b1 : -INFINITY) + (double)t1;
                if (m0) row_fast<kHold3>(rb0, s0, vb + o0, rel, band, lbase, log0);
                if (m1) row_fast<kHold3>(rb1, s1, vb + o1, rel, band, lbase, log0 + lstep);
                m0 &= m0 - 1;
                m1 &= m1 - 1;
            }
        };
        f4 p00 = {0.0f, 0.0f, 0.0f, 0.0f}, p01 = p00, p10 = p00, p11 = p00;
        float bp[8];
        int pv0 = 0;
        stage(0, 0, c_lo * kVT2);
        __syncthreads();
        int bs = 0, bsp = 0;   // base ring slots of chunks ch and ch - 1
        for (int ch = c_lo; ch < c_hi; ++ch) {
            const int buf = (ch - c_lo) & 1;
            const int v0 = ch * kVT2;
            float bq[8];
            load_bases(bq, v0);                     // in flight under the MFMAs
            if (ch + 1 < c_hi) stage(buf ^ 1, bs == 2 ? 0 : bs + 1, v0 + kVT2);
            f4 c00 = {0.0f, 0.0f, 0.0f, 0.0f}, c01 = c00, c10 = c00, c11 = c00;
            constexpr int KG = TWOSD_CUT_KG;
#pragma unroll
            for (int k0 = 0; k0 < KB; k0 += KG) {
                float x0[KG], x1[KG];
#pragma unroll
                for (int u = 0; u < KG; ++u) {
                    if (k0 + u < KB) {
                        x0[u] = Bs[buf][lds3(4 * (k0 + u) + g, j)];
                        x1[u] = Bs[buf][lds3(4 * (k0 + u) + g, 16 + j)];
                    }
                }
#pragma unroll
                for (int u = 0; u < KG; ++u) {
                    if (k0 + u < KB) {
                        c00 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[u], a0[k0 + u], c00, 0, 0, 0);
                        c01 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[u], a1[k0 + u], c01, 0, 0, 0);
                        c10 = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[u], a0[k0 + u], c10, 0, 0, 0);
                        c11 = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[u], a1[k0 + u], c11, 0, 0, 0);
                    }
                }
                if (TWOSD_CUT_SB) __builtin_amdgcn_sched_barrier(0);
            }
            if (ch > c_lo) finish(p00, p01, p10, p11, bp, pv0, bsp);   // the previous chunk, under these MFMAs
            p00 = c00; p01 = c01; p10 = c10; p11 = c11;
#pragma unroll
            for (int r = 0; r < 8; ++r) bp[r] = bq[r];
            pv0 = v0;
            bsp = bs;
            bs = bs == 2 ? 0 : bs + 1;
            __syncthreads();
        }
        if (c_hi > c_lo) finish(p00, p01, p10, p11, bp, pv0, bsp);
        int pk0, pk1, nt0, nt1;
        combine_ex(rb0, rel, band, g, pk0, nt0);
        combine_ex(rb1, rel, band, g, pk1, nt1);
        if (kHold3 && rb0.n > 0 && (tail || nt0 >= 2)) lbase[log0] = rb0.f;
        if (kHold3 && rb1.n > 0 && (tail || nt1 >= 2)) lbase[log0 + lstep] = rb1.f;
        rb0.I = rb0.I >= 0 ? P.vmap[rb0.I] : -1;
        rb1.I = rb1.I >= 0 ? P.vmap[rb1.I] : -1;
        if (tail) {
            if (g == 0) {
                const int t0 = P.full_units * kCutTile2;
                if (sa < P.N) {
                    const size_t o = (size_t)(sa - t0) * P.tail_S + range;
                    P.tp_m[o] = rb0.M; P.tp_i[o] = rb0.I; P.tp_f[o] = pk0;
                }
                if (sb < P.N) {
                    const size_t o = (size_t)(sb - t0) * P.tail_S + range;
                    P.tp_m[o] = rb1.M; P.tp_i[o] = rb1.I; P.tp_f[o] = pk1;
                }
            }
            continue;
        }
        if (nt0 < 2) pk0 = 0;
        if (nt1 < 2) pk1 = 0;
        const bool ok0 = sa < P.N && !pk0 && rb0.I >= 0, ok1 = sb < P.N && !pk1 && rb1.I >= 0;
        const double p0 = ok0 ? P.w[sa] * P.inv_total : 0.0, p1 = ok1 ? P.w[sb] * P.inv_total : 0.0;
        // per scenario of the tile: its fp64 deltas again (this lane's e = 4 kb + g), the S_e terms
        // of its pick (the xor tree of v2's s_pass) and its value base[a] + sum_e PK[a,e] coef_e dv_e
        // in fp64 (the lanes' partial sums combined over g in a fixed order)
        auto fin = [&](int sx, bool ok, int ai, double pp) -> double {
            const double *pk = P.PK + (size_t)(ai >= 0 ? ai : 0) * P.k4;
            const double pu = ok ? pp : 0.0;
            // k-blocks in groups of 6 (their loads in flight together): the S_e terms (v2's xor
            // tree) and dec_lane_chain's chain c_g, in the same order and arithmetic
            constexpr int FG = 6;
            double cg = 0.0;
#pragma unroll
            for (int k0 = 0; k0 < KB; k0 += FG) {
                double d64[FG], pke[FG];
#pragma unroll
                for (int u = 0; u < FG; ++u) {
                    const int e = 4 * (k0 + u) + g;
                    const bool in = k0 + u < KB && e < P.k;
                    d64[u] = (in && sx < P.N) ? P.dv[(size_t)sx * P.k + e] : 0.0;
                    pke[u] = in ? pk[e] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < FG; ++u) {
                    const int kb = k0 + u, e = 4 * kb + g;
                    if (kb >= KB) break;
                    if (e < P.k) cg = fma(pke[u] * P.coef[e], d64[u], cg);
                    double v = (e < P.k) ? pu * pke[u] * d64[u] : 0.0;
#pragma unroll
                    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o);
                    if (j == (kb & 15)) {
                        if (kb < 16) Sacc[0] += v;
                        else Sacc[1] += v;
                    }
                }
            }
            return dec_combine(cg);
        };
        const double tv0 = fin(sa, ok0, rb0.I, p0);
        const double tv1 = fin(sb, ok1, rb1.I, p1);
        // decided rows: the fp64 value of the pick; flagged rows keep the MFMA maximum (the fixup
        // re-scores them and writes the restated value)
        const double vl0 = ok0 ? P.base[rb0.I] + tv0 : rb0.M, vl1 = ok1 ? P.base[rb1.I] + tv1 : rb1.M;
        if (g == 0) {
            if (sa < P.N) { P.arg[sa] = rb0.I; P.val[sa] = vl0; P.flag[sa] = pk0; }
            if (sb < P.N) { P.arg[sb] = rb1.I; P.val[sb] = vl1; P.flag[sb] = pk1; }
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const int ok = __shfl(t == 0 ? (int)ok0 : (int)ok1, jj);
                const int ai = __shfl(t == 0 ? rb0.I : rb1.I, jj);
                const double pp = __shfl(t == 0 ? p0 : p1, jj);
                const double vl = __shfl(t == 0 ? vl0 : vl1, jj);
                if (lane == 0 && ok) {
                    pv_sum = fma(pp, vl, pv_sum);
                    const unsigned long long hq = (unsigned long long)__double2ull_rn(pp * kFix);
                    if (P.hist_lds) __hip_atomic_fetch_add(&hl[ai], hq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    else atomicAdd(&P.hist[ai], hq);
                }
            }
        }
    }
    if (P.hist_lds) {
        __syncthreads();
        for (int v = threadIdx.x; v < P.nv; v += 256) P.hist_part[(size_t)blockIdx.x * P.nv + v] = hl[v];
    }
#ifdef TWOSD_CUT3_COUNT
    if (lane == 0 && P.fstats) {
        atomicAdd(&P.fstats[10], cnt_steps); atomicAdd(&P.fstats[11], cnt_rare);
        atomicAdd(&P.fstats[12], cnt_lanes);
    }
#endif
    const int slot = blockIdx.x * 4 + wid;
    double *out = P.partial + (size_t)slot * (P.k + 1);
    if (lane == 0) out[0] = pv_sum;
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

// Tail scenarios: merge the per-range results -- the same rule as combine_ex over the ranges:
// M = max, a range contributes its log lengths when its maximum reaches the band of M; one
// entry in all: decided (the pick is that range's first maximum), then the scenario's p * val,
// histogram weight and S_e terms (as cut_fixup_kernel); several: flag for the fixup (val = M).
// One wavefront per scenario, lane r = range r.
__device__ __forceinline__ int nib_sum(int pk) {
    return (pk & 31) + ((pk >> kCandBits) & 31) + ((pk >> (2 * kCandBits)) & 31) + ((pk >> (3 * kCandBits)) & 31);
}

__global__ void __launch_bounds__(256) cut_tail_merge_kernel(CutParams P, int slot0) {
    const int lane = threadIdx.x & 63;
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    const int t0 = P.full_units * kCutTile2, S = P.tail_S;
    const double band = __longlong_as_double((long long)*P.band_bits);
    double pv_sum = 0.0, Sacc[2] = {0.0, 0.0};
    for (int ts = gw; ts < P.N - t0; ts += nw) {
        const int s = t0 + ts;
        double m = -INFINITY;
        int ii = -1, pk = 0;
        if (lane < S) {
            const size_t o = (size_t)ts * S + lane;
            m = P.tp_m[o]; ii = P.tp_i[o]; pk = P.tp_f[o];
        }
        double M = m;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) M = fmax(M, __shfl_xor(M, o));
        const double thr = band_floor(M, P.tie_rel, band);
        const int n = (m != -INFINITY && m >= thr) ? nib_sum(pk) : 0;
        int tot = n, it = n ? ii : 0x7fffffff;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            tot += __shfl_xor(tot, o);
            it = min(it, __shfl_xor(it, o));
        }
        const int I = (M == -INFINITY || it == 0x7fffffff) ? -1 : it;
        const int fl = tot >= 2;
        if (lane == 0) { P.arg[s] = I; P.val[s] = M; P.flag[s] = fl; }
        if (fl || I < 0) continue;
        const double p = P.w[s] * P.inv_total;
        // the S_e terms of the pick and its value in fp64, base[I] + sum_e PK[I,e] coef_e dv_e (the
        // lanes' terms summed by a fixed xor tree; the pass's maximum M may be an fp32-MFMA score)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int e = lane + 64 * t;
            if (e < P.k) Sacc[t] = fma(p * P.PK[(size_t)I * P.k4 + e], P.dv[(size_t)s * P.k + e], Sacc[t]);
        }
        // lane g < 4: the chain c_g of dec_lane_chain, then (c_0 + c_1) + (c_2 + c_3) as dec_combine
        double cg = 0.0;
        if (lane < 4) {
            const double *pk = P.PK + (size_t)I * P.k4, *dr = P.dv + (size_t)s * P.k;
            for (int e = lane; e < P.k; e += 4) cg = fma(pk[e] * P.coef[e], dr[e], cg);
        }
        const double c01 = __shfl(cg, 0) + __shfl(cg, 1), c23 = __shfl(cg, 2) + __shfl(cg, 3);
        const double vl = P.base[I] + (c01 + c23);
        if (lane == 0) {
            P.val[s] = vl;
            pv_sum = fma(p, vl, pv_sum);
            atomicAdd(&P.hist[I], (unsigned long long)__double2ull_rn(p * kFix));
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

// score[s, v] in the restatement's order (oracle_build_cut, twosd_ref.argmax_procedure):
// t = sum over the random rows in ascending order of pi_v[row_e] (coef_e dv[s,e]) -- the dense
// dot(pi, dvec) of subprob.jl:155 with its zero rows dropped (adding 0 is exact) -- every
// operation rounded on its own, then base[v] + t
__device__ __forceinline__ double restated_score(const CutParams &P, int v, int s) {
#pragma clang fp contract(off)
    const double *po = P.PKO + (size_t)v * P.k4;
    const double *d = P.dv + (size_t)s * P.k;
    double t = 0.0;
#pragma unroll 4
    for (int q = 0; q < P.k; ++q) {
        const int e = P.eord[q];
        t = t + po[q] * (P.coef[e] * d[e]);
    }
    return P.base[v] + t;
}

// Re-decide the flagged scenarios in the restatement's arithmetic: the logged candidates of the
// lane groups (and tail ranges) that reach the band hold every vertex that can be the pick.
// tie_rel = 0: the first strict maximum (highest score, lowest index among equal scores); > 0:
// the lowest index within tie_rel (1 + |M|) of the maximum M (oracle_build_cut's rule).
// Rows go in batches of up to kFxR flagged whole-tile scenarios per wavefront (a tail scenario,
// whose logs span the vertex ranges, is a batch of its own), so every memory round trip of a
// batch -- the flags, the logs, the staged deltas, the candidates' PK rows, the sums -- serves
// all of its rows:
//   1. the rows' coef_e dv[s,e] in the restated element order (eord) into LDS (dvr);
//   2. the logged candidates compacted into one LDS list, row by row (slot order);
//   3. one lane per candidate adds its products pi_v[row_e] dvr[q] in order (the sequential
//      chain of restated_score; the PK gathers are independent of it and run ahead);
//   4. lane r decides row r over its candidates; then the sums of the decided rows.
// A log that overflowed (or a list past kFxList) re-scans every vertex for that row.
constexpr int kFxR = 8;              // flagged scenarios per batch
constexpr int kFxLd = 129;           // doubles per staged delta row (k <= 128; odd stride)
constexpr int kFxList = 256;         // candidate list capacity per batch (8 rows x 32 log slots)

struct FixWave {                     // one wavefront's LDS
    double dvr[kFxR][kFxLd];
    double cs[kFxList];
    int cvr[kFxList];                // (row << 28) | vertex
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// t = sum_q PKO[v][q] wq[q] in q order, wq[q] = cq[q] dq[q] (the restated k-term dot of one
// candidate; the products past k are 0 and leave t unchanged: t is never -0).  The PKO row is read
// in groups of 32 elements (16 dwordx4 loads), the next group's loads issued before this group's adds.
__device__ __forceinline__ double chain_dot_w(const double2 *__restrict__ po, const double *wq, int k4) {
#pragma clang fp contract(off)
    constexpr int GQ = 8;    // pairs per group (16 elements); k4 <= 128: at most 8 groups
    const int k2 = k4 / 2;
    double t = 0.0;
    double2 a[GQ], b[GQ];
    auto load = [&](double2 (&x)[GQ], int g) {
#pragma unroll
        for (int u = 0; u < GQ; ++u) {
            const int pu = g * GQ + u;
            const double2 ld = po[pu < k2 ? pu : k2 - 1];
            x[u] = pu < k2 ? ld : make_double2(0.0, 0.0);
        }
    };
    auto add = [&](const double2 (&x)[GQ], int g) {
#pragma unroll
        for (int u = 0; u < GQ; ++u) {
            const int q = 2 * (g * GQ + u);
            if (q < k4) {   // uniform
                t = t + x[u].x * wq[q];
                t = t + x[u].y * wq[q + 1];
            }
        }
    };
    const int ng = (k2 + GQ - 1) / GQ;
    load(a, 0);
    for (int g = 0; g < ng; g += 2) {   // ping-pong: group g + 1 in flight while g is added
        if (g + 1 < ng) load(b, g + 1);
        add(a, g);
        if (g + 1 >= ng) break;
        if (g + 2 < ng) load(a, g + 2);
        add(b, g + 1);
    }
    return t;
}

// chain_dot_w with the products cq[q] dq[q] formed in the loop (the rescan's one-row form)
__device__ __forceinline__ double chain_dot(const double2 *__restrict__ po, const double *cq, const double *dq, int k4) {
#pragma clang fp contract(off)
    constexpr int GQ = 8;    // pairs per group (16 elements); k4 <= 128: at most 8 groups
    const int k2 = k4 / 2;
    double t = 0.0;
    double2 a[GQ], b[GQ];
    auto load = [&](double2 (&x)[GQ], int g) {
#pragma unroll
        for (int u = 0; u < GQ; ++u) {
            const int pu = g * GQ + u;
            const double2 ld = po[pu < k2 ? pu : k2 - 1];
            x[u] = pu < k2 ? ld : make_double2(0.0, 0.0);
        }
    };
    auto add = [&](const double2 (&x)[GQ], int g) {
#pragma unroll
        for (int u = 0; u < GQ; ++u) {
            const int q = 2 * (g * GQ + u);
            if (q < k4) {   // uniform
                t = t + x[u].x * (cq[q] * dq[q]);
                t = t + x[u].y * (cq[q + 1] * dq[q + 1]);
            }
        }
    };
    const int ng = (k2 + GQ - 1) / GQ;
    load(a, 0);
    for (int g = 0; g < ng; g += 2) {   // ping-pong: group g + 1 in flight while g is added
        if (g + 1 < ng) load(b, g + 1);
        add(a, g);
        if (g + 1 >= ng) break;
        if (g + 2 < ng) load(a, g + 2);
        add(b, g + 1);
    }
    return t;
}

constexpr int kFlagRescan = 0x40000000;   // flag of a scenario left to cut_rescan_kernel (an overflowed log)

__global__ void __launch_bounds__(256, 3) cut_fixup_kernel(CutParams P, int slot0) {
#pragma clang fp contract(off)
    __shared__ FixWave fw_all[4];
    __shared__ double cq[kFxLd];             // coef_e in the restated order (0 past k)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    FixWave &F = fw_all[wid];
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    const int t0 = P.full_units * kCutTile2, S = P.tail_S;
    const double band = cut_band_scalar(P);
    // this lane's elements in the restated order: q = lane, lane + 64 (-1: padding)
    const int e0 = lane < P.k ? P.eord[lane] : -1, e1 = lane + 64 < P.k ? P.eord[lane + 64] : -1;
    if (threadIdx.x < kFxLd) {
        const int q = threadIdx.x;
        cq[q] = q < P.k ? P.coef[P.eord[q]] : 0.0;
    }
    __syncthreads();
    double pv_sum = 0.0, Sq[2] = {0.0, 0.0};  // S_e of this wave in the restated order: q = lane, lane + 64
    unsigned long long st_rows = 0, st_cands = 0, st_full = 0;
#ifdef TWOSD_FIX_STAMPS
    unsigned long long fst[6] = {0, 0, 0, 0, 0, 0}, fst_t = __builtin_amdgcn_s_memtime();
#define FSTAMP(i) { __builtin_amdgcn_s_waitcnt(0); __builtin_amdgcn_sched_barrier(0); \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); fst[i] += t_ - fst_t; fst_t = t_; }
#else
#define FSTAMP(i)
#endif
    // pass 0: the whole-tile rows, 64 consecutive scenarios per wave step; pass 1: the tail rows
    // (each a batch of its own), spread over all waves (lane L of wave gw: scenario t0 + gw + L nw)
    // so that the waves holding the last scenarios do not run one serial batch per tail row
    for (int pass = 0; pass < 2; ++pass) {
    const int hi = pass ? P.N : min(t0, P.N), lstride = pass ? nw : 1;
    const int gs = pass ? 64 : P.fx_gs;     // a small batch: fewer scenarios per wave step, more waves
    for (int sb0 = pass ? t0 + gw : gw * gs; sb0 < hi; sb0 += nw * gs) {
    const int sl = sb0 + lane * lstride;
    const int myflag = (lane < gs && sl < hi) ? P.flag[sl] : 0;
    uint64_t todo = __ballot(myflag != 0);
    while (todo) {
        // ---- the batch: up to kFxR whole-tile rows, or one tail row
        int nr = 0, srow = 0, frow = 0;     // lane r < nr: its row's scenario and flag
        bool tailb = false;
        while (todo && nr < kFxR) {
            const int bit = (int)__builtin_ctzll(todo);
            const int s = sb0 + bit * lstride;
            if (s >= t0) {                       // a tail row: alone in its batch
                if (nr > 0) break;
                tailb = true;
            }
            todo &= todo - 1;
            const int fl = __shfl(myflag, bit);
            if (lane == nr) { srow = s; frow = fl; }
            ++nr;
            if (tailb) break;
        }
        FSTAMP(0)
        // 1. the rows' deltas in the restated order, all loads in one round trip: the products
        // coef_e dv_e of the restated dot into LDS (zero past k; the same operation the chain would
        // do), the raw deltas kept in registers for the S_e sums
        double d0[kFxR], d1[kFxR];
        {
#pragma unroll
            for (int r = 0; r < kFxR; ++r) {
                const int s = __shfl(srow, r < nr ? r : 0);
                const double *dr = P.dv + (size_t)s * P.k;
                d0[r] = e0 >= 0 ? dr[e0] : 0.0;
                d1[r] = e1 >= 0 ? dr[e1] : 0.0;
            }
            const double c0 = cq[lane], c1 = cq[lane + 64];
#pragma unroll
            for (int r = 0; r < kFxR; ++r) {
                if (r < nr) {
                    F.dvr[r][lane] = c0 * d0[r];
                    F.dvr[r][lane + 64] = c1 * d1[r];
                }
            }
        }
        FSTAMP(1)
        // 2. the candidate list (slot order: rows in batch order, each row's slots contiguous)
        int nc = 0;
        uint32_t rstart = 0, rcount = 0;        // lane r: its row's list range
        uint32_t ovf_rows = 0;                  // rows whose log overflowed (or a list past kFxList)
        if (!tailb) {
            constexpr int NIT = kFxR;         // one step per row (4 kCandC == 64 slots)
            int vv[NIT];
#pragma unroll
            for (int it = 0; it < NIT; ++it) {   // every log entry of the batch in one round trip
                const int g = lane / kCandC, i = lane % kCandC;
                const int fl = __shfl(frow, it);
                const int sr = __shfl(srow, it);
                const int c = (fl >> (kCandBits * g)) & 31;
                const int lv = P.cand[((size_t)sr * 4 + g) * kCandC + i];   // rows past nr: srow = 0, a valid address
                vv[it] = it >= nr ? -1 : (c > kCandC ? -2 : (i < c ? lv : -1));   // log entries: argmax positions (vmap)
            }
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                if (it >= nr) break;
                const int v = vv[it];
                const uint64_t has = __ballot(v >= 0);
                const int na = __popcll(has);
                if (__ballot(v == -2) != 0 || nc + na > kFxList) {   // overflowed log (or a full list): rescan
                    ovf_rows |= 1u << it;
                    continue;
                }
                if (v >= 0) F.cvr[nc + __popcll(has & ((1ull << lane) - 1))] = (it << 28) | v;
                if (lane == it) { rstart = nc; rcount = na; }
                nc += na;
            }
        } else {
            const int s = __shfl(srow, 0);
            const int ts = s - t0;
            const double thr = band_floor(P.val[s], P.tie_rel, band);
            const int nslots = S * 4 * kCandC;
            for (int q0 = 0; q0 < nslots; q0 += 64) {
                const int q = q0 + lane;
                int v = -1;
                if (q < nslots) {
                    const int rg = q / (4 * kCandC), g = (q / kCandC) & 3, i = q % kCandC;
                    const size_t o = (size_t)ts * S + rg;
                    const double mr = P.tp_m[o];
                    const int pk = (mr != -INFINITY && mr >= thr) ? P.tp_f[o] : 0;
                    const int c = (pk >> (kCandBits * g)) & 31;
                    if (c > kCandC) v = -2;
                    else if (i < c) v = P.tcand[(o * 4 + g) * kCandC + i];
                }
                const uint64_t has = __ballot(v >= 0);
                if (__ballot(v == -2)) ovf_rows = 1u;
                if (nc + __popcll(has) > kFxList) { ovf_rows = 1u; break; }
                if (v >= 0) F.cvr[nc + __popcll(has & ((1ull << lane) - 1))] = v;
                nc += __popcll(has);
            }
            if (lane == 0) { rstart = 0; rcount = nc; }
        }
        wave_lds_sync();
        FSTAMP(2)
        st_rows += nr;
        st_cands += nc;
        // 3. restated scores, one lane per candidate: base[v] + chain_dot (restated_score's order);
        // candidates are argmax positions (vertex vmap[c]: PKOc / basec rows)
        for (int cb = 0; cb < nc; cb += 64) {
            const int c = cb + lane;
            const int cr = F.cvr[c < nc ? c : 0];
            const int r = cr >> 28, v = cr & 0x0fffffff;
            const double bvv = P.basec[v];
            const double t = chain_dot_w(reinterpret_cast<const double2 *>(P.PKOc + (size_t)v * P.k4), F.dvr[r], P.k4);
            if (c < nc) F.cs[c] = bvv + t;
        }
        wave_lds_sync();
        FSTAMP(3)
        // 4. lane r decides row r over its candidates (the rule takes the lowest vertex among the
        // qualifying ones, whatever their list order; positions order as the vertices)
        int best = 0x7fffffff;
        double bv = -INFINITY;
        if (lane < nr && !((ovf_rows >> lane) & 1)) {
            double M = -INFINITY;
            for (uint32_t c = rstart; c < rstart + rcount; ++c) M = fmax(M, F.cs[c]);
            if (M != -INFINITY) {
                const double lim = P.tie_rel > 0.0 ? M - P.tie_rel * (1.0 + fabs(M)) : M;
                for (uint32_t c = rstart; c < rstart + rcount; ++c) {
                    const int v = F.cvr[c] & 0x0fffffff;
                    const double sc = F.cs[c];
                    if (sc >= lim && v < best) { best = v; bv = sc; }
                }
            }
        }
        // overflowed rows: left to cut_rescan_kernel (every vertex), which also adds their sums
        const bool resc = lane < nr && ((ovf_rows >> lane) & 1);
        if (resc) P.flag[srow] = kFlagRescan;
        st_full += __popc(ovf_rows);
        FSTAMP(4)
        // 5. outputs and sums, rows in batch (= scenario) order; the picks' vertex indices and PKO
        // rows in one round trip
        const bool mine = lane < nr && best != 0x7fffffff;
        const int bvx = mine ? P.vmap[best] : -1;
        {
            double pa[kFxR], pb[kFxR];
#pragma unroll
            for (int r = 0; r < kFxR; ++r) {
                const int b = __shfl(best, r < nr ? r : 0);
                const double *po = P.PKOc + (size_t)(b == 0x7fffffff ? 0 : b) * P.k4;
                pa[r] = po[lane < P.k4 ? lane : 0];
                pb[r] = po[lane + 64 < P.k4 ? lane + 64 : 0];
            }
            // lane r: its row's p and histogram weight (one load, one atomic instruction for all rows)
            const double pr = lane < nr ? P.w[srow] * P.inv_total : 0.0;
            if (lane < nr && !resc) {
                P.arg[srow] = bvx;
                P.val[srow] = mine ? bv : -INFINITY;
            }
            if (mine) atomicAdd(&P.hist[bvx], (unsigned long long)__double2ull_rn(pr * kFix));
#pragma unroll
            for (int r = 0; r < kFxR; ++r) {
                if (r >= nr) break;
                const int b = __shfl(best, r);
                const double bvr = __shfl(bv, r);
                const double p = __shfl(pr, r);
                if (b == 0x7fffffff) continue;   // no finite score: no pick (as the argmax pass leaves it)
                if (lane == 0) pv_sum = fma(p, bvr, pv_sum);
                if (e0 >= 0) Sq[0] = fma(p * pa[r], d0[r], Sq[0]);
                if (e1 >= 0) Sq[1] = fma(p * pb[r], d1[r], Sq[1]);
            }
        }
        wave_lds_sync();   // the next batch rewrites the LDS lists
        FSTAMP(5)
    }
    }
    }
    double *out = P.partial + (size_t)(slot0 + gw) * (P.k + 1);
    if (lane == 0) out[0] = pv_sum;
    if (e0 >= 0) out[1 + e0] = Sq[0];
    if (e1 >= 0) out[1 + e1] = Sq[1];
    if (P.fstats && lane == 0 && st_rows) {
        atomicAdd(&P.fstats[0], st_rows);
        atomicAdd(&P.fstats[1], st_cands);
        atomicAdd(&P.fstats[2], st_full);
#ifdef TWOSD_FIX_STAMPS
        for (int i_ = 0; i_ < 6; ++i_) atomicAdd(&P.fstats[3 + i_], fst[i_]);
#endif
    }
}

// The scenarios whose candidate log overflowed (cut_fixup_kernel marked them kFlagRescan): the
// restated rule over EVERY vertex, one wavefront per scenario, lanes taking the vertices in
// increasing order (64 per step) with chain_dot; pass 0 the first strict maximum, pass 1
// (tie_rel > 0) the lowest vertex within the tolerance.  Then the scenario's sums, as the fixup.
__global__ void __launch_bounds__(256) cut_rescan_kernel(CutParams P, int slot0) {
#pragma clang fp contract(off)
    __shared__ double dqs[4][kFxLd];
    __shared__ double cq[kFxLd];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double *dq = dqs[wid];
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    const int e0 = lane < P.k ? P.eord[lane] : -1, e1 = lane + 64 < P.k ? P.eord[lane + 64] : -1;
    if (threadIdx.x < kFxLd) {
        const int q = threadIdx.x;
        cq[q] = q < P.k ? P.coef[P.eord[q]] : 0.0;
    }
    __syncthreads();
    double pv_sum = 0.0, Sq[2] = {0.0, 0.0};
    for (int sb0 = gw * 64; sb0 < P.N; sb0 += nw * 64) {
    uint64_t todo = __ballot(sb0 + lane < P.N && P.flag[sb0 + lane] == kFlagRescan);
    while (todo) {
        const int s = sb0 + (int)__builtin_ctzll(todo);
        todo &= todo - 1;
        const double *dr = P.dv + (size_t)s * P.k;
        dq[lane] = e0 >= 0 ? dr[e0] : 0.0;
        dq[lane + 64] = e1 >= 0 ? dr[e1] : 0.0;
        wave_lds_sync();
        double bm = -INFINITY;
        int bi = 0x7fffffff;
        for (int v0 = 0; v0 < P.nv; v0 += 64) {
            const int v = v0 + lane;
            const int vc = v < P.nv ? v : P.nv - 1;
            const double sc = P.base[vc] + chain_dot(reinterpret_cast<const double2 *>(P.PKO + (size_t)vc * P.k4), cq, dq, P.k4);
            if (v < P.nv && sc > bm) { bm = sc; bi = v; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double m2 = __shfl_xor(bm, o);
            const int i2 = __shfl_xor(bi, o);
            if (m2 > bm || (m2 == bm && i2 < bi)) { bm = m2; bi = i2; }
        }
        int best = bi;
        double bv = bm;
        if (P.tie_rel > 0.0 && best != 0x7fffffff) {
            const double lim = bm - P.tie_rel * (1.0 + fabs(bm));
            int lo = 0x7fffffff;
            double lv = -INFINITY;
            for (int v0 = 0; v0 < best; v0 += 64) {
                const int v = v0 + lane;
                const int vc = v < P.nv ? v : P.nv - 1;
                const double sc = P.base[vc] + chain_dot(reinterpret_cast<const double2 *>(P.PKO + (size_t)vc * P.k4), cq, dq, P.k4);
                if (v < best && sc >= lim && v < lo) { lo = v; lv = sc; }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const int i2 = __shfl_xor(lo, o);
                const double v2 = __shfl_xor(lv, o);
                if (i2 < lo) { lo = i2; lv = v2; }
            }
            if (lo < best) { best = lo; bv = lv; }
        }
        if (lane == 0) {
            P.arg[s] = best == 0x7fffffff ? -1 : best;
            P.val[s] = best == 0x7fffffff ? -INFINITY : bv;
        }
        if (best != 0x7fffffff) {
            const double p = P.w[s] * P.inv_total;
            const double *po = P.PKO + (size_t)best * P.k4;
            if (lane == 0) {
                pv_sum = fma(p, bv, pv_sum);
                atomicAdd(&P.hist[best], (unsigned long long)__double2ull_rn(p * kFix));
            }
            if (e0 >= 0) Sq[0] = fma(p * po[lane], dq[lane], Sq[0]);
            if (e1 >= 0) Sq[1] = fma(p * po[lane + 64], dq[lane + 64], Sq[1]);
        }
        wave_lds_sync();
    }
    }
    double *out = P.partial + (size_t)(slot0 + gw) * (P.k + 1);
    if (lane == 0) out[0] = pv_sum;
    if (e0 >= 0) out[1 + e0] = Sq[0];
    if (e1 >= 0) out[1 + e1] = Sq[1];
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
    double *PK = nullptr, *PKT = nullptr, *PKO = nullptr;
    double *PKTc = nullptr;
    size_t pktc_cap = 0;
    float *PKTc32 = nullptr;               // the fp32 pass's chunk source
    size_t pktc32_cap = 0;
    float *basec32 = nullptr;              // the fp32 pass's prefilter bases
    size_t basec32_cap = 0;
    int pk_count = 0, pk_vcap = 0, pk_k4 = 0;
    size_t pk_cap = 0;
    int *rows = nullptr;
    int *eord = nullptr;    // elements by ascending row: the order of the restated score's dot
    unsigned long long *phash = nullptr;   // per vertex: hash of its PK row (bits)
    int *tprev = nullptr;                  // per vertex: previous vertex with a bit-identical PK row, or -1
    unsigned long long *tw_hs = nullptr;   // twin rebuild by sort: sorted hashes, vertex ids in / out, cub scratch
    int *tw_vin = nullptr, *tw_vout = nullptr;
    void *tw_tmp = nullptr;
    size_t tw_cap = 0, tw_tmp_bytes = 0;
    int *vmap = nullptr, *nvc = nullptr;   // per x: the argmax's vertices and their count
    size_t vmap_cap = 0;
    double *PKOc = nullptr, *basec = nullptr;   // per x: their PKO rows and bases (vmap order)
    size_t pkoc_cap = 0;
    double *coef = nullptr, *bvec = nullptr, *base = nullptr, *partial = nullptr, *sums = nullptr;
    double *gpart = nullptr, *g = nullptr;
    int *arg = nullptr, *flag = nullptr;
    double *val = nullptr;
    unsigned long long *hist = nullptr, *hist_part = nullptr;
    size_t hpart_cap = 0;
    double *part2 = nullptr;
    double *tp_m = nullptr;
    int *tp_i = nullptr, *tp_f = nullptr;
    size_t tp_cap = 0;
    int *cand = nullptr, *tcand = nullptr;    // candidate logs (whole tiles / tail ranges)
    unsigned long long *fstats = nullptr;     // fixup counters of the last cut (3)
    size_t cand_cap = 0, tcand_cap = 0;
    unsigned long long *band_bits = nullptr;
    // per epigraph: max |dv[., e]| over its scenarios (bits), the rows folded in so far
    std::vector<unsigned long long *> dmax;
    std::vector<int> dmax_rows, dmax_k;
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
    hipFree(w->PK); hipFree(w->PKT); hipFree(w->PKO); hipFree(w->PKTc); hipFree(w->PKTc32); hipFree(w->basec32); hipFree(w->rows); hipFree(w->eord); hipFree(w->coef); hipFree(w->bvec); hipFree(w->base);
    hipFree(w->partial); hipFree(w->sums); hipFree(w->gpart); hipFree(w->g); hipFree(w->arg); hipFree(w->flag);
    hipFree(w->val); hipFree(w->hist); hipFree(w->part2); hipFree(w->hist_part);
    hipFree(w->tp_m); hipFree(w->tp_i); hipFree(w->tp_f);
    hipFree(w->cand); hipFree(w->tcand); hipFree(w->band_bits); hipFree(w->fstats);
    hipFree(w->phash); hipFree(w->tprev); hipFree(w->tw_hs); hipFree(w->tw_vin); hipFree(w->tw_vout); hipFree(w->tw_tmp); hipFree(w->vmap); hipFree(w->nvc); hipFree(w->PKOc); hipFree(w->basec);
    for (auto *p : w->dmax) hipFree(p);
    delete w;
    c->cut_ws = nullptr;
}

void cut_truncate_pk(twosd_ctx *c, int size) {
    if (!c->cut_ws) return;
    CutWs *w = (CutWs *)c->cut_ws;
    if (w->pk_count > size) w->pk_count = size;   // twin links point to lower vertices: still valid
}

void cut_invalidate_pk(twosd_ctx *c) {
    if (!c->cut_ws) return;
    CutWs *w = (CutWs *)c->cut_ws;
    w->pk_count = 0;
    if (w->rows) hipFree(w->rows);
    w->rows = nullptr;   // forces re-upload of the element rows (and their order)
}

#define HIPCHK(expr)                                                                               \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) return fail(TWOSD_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

// a cut that returns before the argmax (no scenarios) leaves no fixup counters: clear the last
// cut's, so twosd_cut_stats does not report them as this cut's
static int clear_cut_stats(twosd_ctx *c) {
    CutWs *w = c->cut_ws ? (CutWs *)c->cut_ws : nullptr;
    if (w && w->fstats) {
        HIPCHK(hipMemsetAsync(w->fstats, 0, sizeof(unsigned long long) * 16, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return TWOSD_OK;
}

template <typename T>
static int realloc_dev(T **p, size_t n) {
    if (*p) hipFree(*p);
    *p = nullptr;
    hipError_t e = hipMalloc((void **)p, sizeof(T) * std::max<size_t>(n, 1));
    if (e != hipSuccess) return fail(TWOSD_E_DEVICE, "cut workspace hipMalloc(%zu): %s", sizeof(T) * n, hipGetErrorString(e));
    if (poison_byte(4) >= 0) { hipMemset(*p, poison_byte(4), sizeof(T) * std::max<size_t>(n, 1)); hipDeviceSynchronize(); }
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

template <int KB>
static void launch_argmax3_t(const CutParams &P, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL(cut_argmax3_kernel<KB>, dim3(nblocks), dim3(256), P.hist_lds ? sizeof(unsigned long long) * P.nv : 0, s, P);
}
template <int KB>
static int argmax3_occupancy_t(size_t dyn_lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cut_argmax3_kernel<KB>, 256, dyn_lds) != hipSuccess) nb = 0;
    return nb;
}
#define CUT_KB_SWITCH(FN, ...)                          \
    switch (KB) {                                       \
        case 1: return FN<1>(__VA_ARGS__);              \
        case 2: return FN<2>(__VA_ARGS__);              \
        case 4: return FN<4>(__VA_ARGS__);              \
        case 6: return FN<6>(__VA_ARGS__);              \
        case 8: return FN<8>(__VA_ARGS__);              \
        case 12: return FN<12>(__VA_ARGS__);            \
        case 16: return FN<16>(__VA_ARGS__);            \
        case 22: return FN<22>(__VA_ARGS__);            \
        case 24: return FN<24>(__VA_ARGS__);            \
        case 30: return FN<30>(__VA_ARGS__);            \
        case 32: return FN<32>(__VA_ARGS__);            \
    }
static int argmax3_occupancy(int KB, size_t dyn_lds) {
    CUT_KB_SWITCH(argmax3_occupancy_t, dyn_lds)
    return 0;
}
static void launch_argmax3(int KB, const CutParams &P, int nblocks, hipStream_t s) {
    CUT_KB_SWITCH(launch_argmax3_t, P, nblocks, s)
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
        if ((rc = realloc_dev(&w->rows, std::max(k, 1))) || (rc = realloc_dev(&w->eord, std::max(k, 1)))) return rc;
        if (k) HIPCHK(hipMemcpy(w->rows, c->pos_row.data(), sizeof(int) * k, hipMemcpyHostToDevice));
        // the restated score's element order: ascending row (the dense dot over the m rows), element
        // order within a row
        std::vector<int> ord(k);
        for (int e = 0; e < k; ++e) ord[e] = e;
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return c->pos_row[a] < c->pos_row[b]; });
        if (k) HIPCHK(hipMemcpy(w->eord, ord.data(), sizeof(int) * k, hipMemcpyHostToDevice));
        w->pk_count = 0;
        w->pk_k4 = k4;
        w->m = m;
    }
    if (nv > w->pk_vcap) {
        const int vcap = std::max(nv, 2 * w->pk_vcap + 256);
        if ((rc = realloc_dev(&w->PK, (size_t)vcap * k4)) || (rc = realloc_dev(&w->PKT, (size_t)vcap * k4)) ||
            (rc = realloc_dev(&w->PKO, (size_t)vcap * k4)) || (rc = realloc_dev(&w->phash, vcap)) ||
            (rc = realloc_dev(&w->tprev, vcap)))
            return rc;
        w->pk_vcap = vcap;
        w->pk_count = 0;
    }
    if (w->pk_count > nv) w->pk_count = 0;
    if (w->pk_count < nv) {
        const int total = (nv - w->pk_count) * k4;
        hipLaunchKernelGGL(cut_pk_kernel, dim3((total + 255) / 256), dim3(256), 0, c->stream, w->pk_count, nv, m, k, k4,
                           w->pk_vcap, w->rows, w->eord, c->dvs.V, w->PK, w->PKT, w->PKO);
        HIPCHK(hipGetLastError());
        const int nn = nv - w->pk_count;
        hipLaunchKernelGGL(cut_twin_hash_kernel, dim3((nn + 255) / 256), dim3(256), 0, c->stream, w->pk_count, nv, k4, w->PK,
                           w->phash);
        if ((long long)nn * nv <= (1ll << 22)) {   // a few new vertices: scan the earlier ones
            hipLaunchKernelGGL(cut_twin_prev_kernel, dim3((nn + 3) / 4), dim3(256), 0, c->stream, w->pk_count, nv, k4, w->PK,
                               w->phash, w->tprev);
        } else {                                             // a rebuild: sort every vertex by hash
            if ((size_t)nv > w->tw_cap) {
                hipFree(w->tw_hs); hipFree(w->tw_vin); hipFree(w->tw_vout);
                w->tw_hs = nullptr; w->tw_vin = w->tw_vout = nullptr;
                if ((rc = realloc_dev(&w->tw_hs, nv)) || (rc = realloc_dev(&w->tw_vin, nv)) || (rc = realloc_dev(&w->tw_vout, nv))) return rc;
                w->tw_cap = nv;
            }
            size_t need = 0;
            HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, w->phash, w->tw_hs, w->tw_vin, w->tw_vout, nv, 0, 64, c->stream));
            if (need > w->tw_tmp_bytes) {
                hipFree(w->tw_tmp);
                w->tw_tmp = nullptr;
                HIPCHK(hipMalloc(&w->tw_tmp, need));
                w->tw_tmp_bytes = need;
            }
            hipLaunchKernelGGL(cut_iota_kernel, dim3((nv + 255) / 256), dim3(256), 0, c->stream, w->tw_vin, nv);
            // (the earlier vertices' hashes are kept in phash; only the new ones were hashed above)
            HIPCHK(hipcub::DeviceRadixSort::SortPairs(w->tw_tmp, need, w->phash, w->tw_hs, w->tw_vin, w->tw_vout, nv, 0, 64,
                                                      c->stream));
            hipLaunchKernelGGL(cut_twin_sorted_kernel, dim3((nv + 255) / 256), dim3(256), 0, c->stream, nv, k4, w->PK, w->tw_hs,
                               w->tw_vout, w->tprev);
        }
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
    // the chunk's k-rows: k element rows plus the vertex base row
    const int KB = kb_for((k + 1 + 3) & ~3);
    if (KB < 0) return fail(TWOSD_E_UNSUPPORTED, "k = %d random elements exceeds the cut kernel envelope (127)", k);
    // the MFMA pass in fp32 (cut_argmax3_kernel, the element rows only: no base row) unless
    // TWOSD_CUT_F32=0 (A/B and test knob, read per cut); a cut whose operands leave the fp32 range
    // runs the fp64 pass anyway (decided on the device, cut_band_select_kernel)
    const int KB32 = kb_for(k4);
    const bool want32 = KB32 > 0 && (!getenv("TWOSD_CUT_F32") || atoi(getenv("TWOSD_CUT_F32")) != 0);
    int rc;
    if ((rc = update_pk(c))) return rc;
    // host: bvec = r - (T x) as the reference writes it (`coef.rhs - coef.transfer * x`,
    // subprob.jl:147): T x accumulated from zero column by column, as SparseArrays' CSC mat-vec
    // does (tx[i] += T[i][j] * x[j] for j ascending, no contraction), then subtracted from r
    // (oracle_build_cut, twosd_ref._seq_base); coef
    std::vector<double> &bvec = w->h_bvec, &coef = w->h_coef;
    bvec.assign(m, 0.0);
    coef.assign(k4, 0.0);
    for (int i = 0; i < m; ++i) {
#pragma clang fp contract(off)
        double tx = 0.0;
        for (int jj = 0; jj < n1; ++jj) tx = tx + c->T[(size_t)i * n1 + jj] * x[jj];
        bvec[i] = c->r[i] - tx;
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
    if (bpc <= 0)
        bpc = want32 ? argmax3_occupancy(KB32, sizeof(unsigned long long) * kHistLds) : argmax_occupancy(KB, sizeof(unsigned long long) * kHistLds);
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
    // the fixup takes 64 scenarios per wave step: enough waves that every SIMD holds several; 3 blocks
    // per CU = its resident occupancy (launch bounds, LDS), so no block waits for a second round
    // (storm 1M at x_EV: 0.88 ms at 4, 0.69 at 3, 0.86 at 2, 0.82 at 8: profiles/r06/ab_fixup_grid.txt)
    static const int fix_per_cu = getenv("TWOSD_FIX_BPC") ? std::max(1, atoi(getenv("TWOSD_FIX_BPC"))) : 3;
    // scenarios per wave step: 64, or 32 / 16 when 64 would leave fewer waves than 3 resident blocks
    // per CU hold (a 125k shard at N = 8: 1953 waves of one step each, every flagged row's batch
    // latency in series)
    int fx_gs = 64;
    while (fx_gs > 16 && (long long)(N + fx_gs - 1) / fx_gs < 12ll * c->num_cus) fx_gs /= 2;
    const int fix_blocks = std::max(1, std::min((N + 4 * fx_gs - 1) / (4 * fx_gs), fix_per_cu * c->num_cus));
    const int ntail = S > 1 ? N - full * kCutTile2 : 0;
    const int merge_blocks = ntail > 0 ? std::max(1, std::min((ntail + 3) / 4, c->num_cus)) : 0;
    const int resc_blocks = std::max(1, std::min((N + 255) / 256, c->num_cus));
    const size_t slots = (size_t)nblocks * 4 + (size_t)fix_blocks * 4 + (size_t)merge_blocks * 4 + (size_t)resc_blocks * 4;
    if ((size_t)ntail * S > w->tp_cap) {
        if ((rc = realloc_dev(&w->tp_m, (size_t)ntail * S)) || (rc = realloc_dev(&w->tp_i, (size_t)ntail * S)) ||
            (rc = realloc_dev(&w->tp_f, (size_t)ntail * S)))
            return rc;
        w->tp_cap = (size_t)ntail * S;
    }
    // candidate logs: rows padded to whole tiles (the padding scenarios of a tile log too)
    const size_t cand_need = (size_t)full * kCutTile2 * 4 * kCandC;
    const size_t tcand_need = (size_t)(ntiles - full) * kCutTile2 * S * 4 * kCandC;
    // the argmax forms log offsets as 32-bit indices (log0 / lstep): past 2^32 slots (~67M
    // scenarios in one epigraph) they would wrap and the fixup would read slots no kernel wrote
    {
        size_t log_max = UINT32_MAX;
        if (const char *e = getenv("TWOSD_CUT_LOG_MAX")) log_max = (size_t)atoll(e);   // test hook
        if (cand_need > log_max || tcand_need > log_max)
            return fail(TWOSD_E_UNSUPPORTED, "cut: %d scenarios need %zu candidate-log slots (32-bit offsets: at most %zu)", N,
                        std::max(cand_need, tcand_need), log_max);
    }
    if (cand_need > w->cand_cap) {
        if ((rc = realloc_dev(&w->cand, cand_need))) return rc;
        w->cand_cap = cand_need;
    }
    if (tcand_need > w->tcand_cap) {
        if ((rc = realloc_dev(&w->tcand, tcand_need))) return rc;
        w->tcand_cap = tcand_need;
    }
    // band_bits: [0] fp64 band, [1] fp32 band, [2] fp32 operands out of range, [3] the active band, [4] the pass
    if (!w->band_bits && (rc = realloc_dev(&w->band_bits, 8))) return rc;
    if (!w->fstats && (rc = realloc_dev(&w->fstats, 16))) return rc;
    HIPCHK(hipMemsetAsync(w->fstats, 0, sizeof(unsigned long long) * 16, c->stream));
    // the epigraph's max |dv| per element, folded in for the rows added since the last cut
    if ((int)w->dmax.size() <= epi) {
        w->dmax.resize(epi + 1, nullptr);
        w->dmax_rows.resize(epi + 1, 0);
        w->dmax_k.resize(epi + 1, -1);
    }
    // Invariant: an epigraph's scenario rows are append-only (twosd_add_scenarios /
    // twosd_add_sampled_scenarios append; no entry point rewrites or removes rows), so the
    // cached max folds in only rows [dmax_rows, N).  A row count below the cached one can only
    // mean the rows were replaced: fold everything in again (a too-small dmax would narrow the
    // decision band and mark near-tied rows decided without a fixup).
    if (w->dmax_k[epi] != k || w->dmax_rows[epi] > N) {
        if ((rc = realloc_dev(&w->dmax[epi], std::max(k, 1)))) return rc;
        HIPCHK(hipMemsetAsync(w->dmax[epi], 0, sizeof(unsigned long long) * std::max(k, 1), c->stream));
        w->dmax_k[epi] = k;
        w->dmax_rows[epi] = 0;
    }
    if (w->dmax_rows[epi] < N && k > 0) {
        const int rows = N - w->dmax_rows[epi];
        hipLaunchKernelGGL(cut_dmax_kernel, dim3(std::max(1, std::min(rows, 2048))), dim3(256), 0, c->stream, w->dmax_rows[epi], N, k,
                           E.d_dv, w->dmax[epi]);
        w->dmax_rows[epi] = N;
    }
    if (slots * (k + 1) > w->part_cap) {
        if ((rc = realloc_dev(&w->partial, slots * (k + 1)))) return rc;
        w->part_cap = slots * (k + 1);
    }
    HIPCHK(hipMemsetAsync(d_hist, 0, sizeof(unsigned long long) * std::max(nv, 1), c->stream));
    HIPCHK(hipMemsetAsync(w->band_bits, 0, sizeof(unsigned long long) * 8, c->stream));
    // band: the MFMA score and the restated one both add base[v] to a (k + 1)-term dot and differ
    // by at most 2 gamma_{k+4} (|base[v]| + sum_e |PK coef dv|) (one more rounding per T element
    // term, coef folded on the other side); twice that for safety
    double band_scale, band_scale32;
    {
        const double u = ldexp(1.0, -53), u32 = ldexp(1.0, -24), nk = (double)(k + 4);
        band_scale = 2.0 * 2.0 * (nk * u / (1.0 - nk * u));
        band_scale32 = 2.0 * 2.0 * (nk * u32 / (1.0 - nk * u32));
    }
    hipLaunchKernelGGL(cut_vbase_kernel, dim3(std::max(1, std::min((nv + 3) / 4, 4096))), dim3(256), 0, c->stream, nv, m, k, k4,
                       c->dvs.V, w->bvec, w->PK, w->coef, w->dmax[epi], w->base, w->band_bits, band_scale, band_scale32);
    hipLaunchKernelGGL(cut_band_select_kernel, dim3(1), dim3(64), 0, c->stream, w->band_bits, want32 ? 1 : 0);
    CutParams P{};
    P.band_scale = band_scale;
    P.N = N; P.k = k; P.k4 = k4; P.nv = nv; P.vcap = w->pk_vcap; P.m = m;
    static const int hist_lds_max = getenv("TWOSD_HIST_LDS") ? atoi(getenv("TWOSD_HIST_LDS")) : kHistLds;
    P.hist_lds = nv <= hist_lds_max ? 1 : 0;
    if (P.hist_lds && (size_t)nblocks * nv > w->hpart_cap) {
        if ((rc = realloc_dev(&w->hist_part, (size_t)nblocks * nv))) return rc;
        w->hpart_cap = (size_t)nblocks * nv;
    }
    P.hist_part = w->hist_part;
    P.tie_rel = tie_rel; P.inv_total = 1.0 / total_weight;
    P.band_bits = w->band_bits + 3;
    P.mode = w->band_bits + 4;
    P.cand = w->cand; P.tcand = w->tcand; P.eord = w->eord; P.fstats = w->fstats;
    P.dv = E.d_dv; P.w = E.d_w; P.coef = w->coef; P.PK = w->PK; P.PKT = w->PKT; P.PKO = w->PKO; P.base = w->base;
    {
        // test / A-B knob, read per cut: TWOSD_CUT_TWINS=0 keeps dominated twins in the argmax (the
        // same picks; more re-decided rows)
        const bool twins = !getenv("TWOSD_CUT_TWINS") || atoi(getenv("TWOSD_CUT_TWINS")) != 0;
        const int vcap32 = (nv + 31) & ~31, rows = 4 * KB;
        if ((size_t)rows * vcap32 > w->pktc_cap) {
            if ((rc = realloc_dev(&w->PKTc, (size_t)rows * vcap32))) return rc;
            w->pktc_cap = (size_t)rows * vcap32;
        }
        if ((size_t)nv > w->vmap_cap) {
            if ((rc = realloc_dev(&w->vmap, nv))) return rc;
            w->vmap_cap = nv;
        }
        if (!w->nvc && (rc = realloc_dev(&w->nvc, 1))) return rc;
        if ((size_t)nv > w->pkoc_cap) {
            if ((rc = realloc_dev(&w->PKOc, (size_t)nv * k4)) || (rc = realloc_dev(&w->basec, (size_t)vcap32))) return rc;
            w->pkoc_cap = nv;
        }
        hipLaunchKernelGGL(cut_compact_kernel, dim3(1), dim3(1024), 0, c->stream, nv, w->base, twins ? w->tprev : nullptr, w->vmap,
                           w->nvc, w->fstats + 9);
        const int rows32 = want32 ? kr32(KB32) : 0;
        if (want32 && (size_t)rows32 * vcap32 > w->pktc32_cap) {
            if ((rc = realloc_dev(&w->PKTc32, (size_t)rows32 * vcap32))) return rc;
            w->pktc32_cap = (size_t)rows32 * vcap32;
        }
        if (want32 && (size_t)vcap32 > w->basec32_cap) {
            if ((rc = realloc_dev(&w->basec32, (size_t)vcap32))) return rc;
            w->basec32_cap = vcap32;
        }
        const size_t tot2 = (size_t)std::max(rows, rows32) * vcap32;
        hipLaunchKernelGGL(cut_pktc_kernel, dim3((unsigned)std::min<size_t>(4096, (tot2 + 255) / 256)), dim3(256), 0, c->stream, k,
                           rows, w->pk_vcap, vcap32, w->PKT, w->coef, w->base, w->vmap, w->nvc, w->PKTc, rows32,
                           want32 ? w->PKTc32 : nullptr);
        P.PKTc32 = w->PKTc32;
        hipLaunchKernelGGL(cut_compact_rows_kernel, dim3((unsigned)std::min<size_t>(2048, ((size_t)nv * k4 + 255) / 256)), dim3(256), 0,
                           c->stream, nv, k4, w->vmap, w->nvc, w->PKO, w->base, w->PKOc, w->basec, vcap32,
                           want32 ? w->basec32 : nullptr);
        P.basec32 = w->basec32;
        P.PKTc = w->PKTc;
        P.vcap32 = vcap32;
        P.vmap = w->vmap;
        P.nvc = w->nvc;
        P.PKOc = w->PKOc;
        P.basec = w->basec;
    }
    P.arg = w->arg; P.val = w->val; P.flag = w->flag; P.hist = d_hist; P.partial = w->partial;
    P.full_units = full; P.tail_S = S; P.fx_gs = fx_gs;
    P.tp_m = w->tp_m; P.tp_i = w->tp_i; P.tp_f = w->tp_f;
    if (want32) launch_argmax3(KB32, P, nblocks, c->stream);   // each of the two returns at once unless its pass runs
    launch_argmax(KB, P, nblocks, c->stream);
    if (P.hist_lds)
        hipLaunchKernelGGL(cut_hist_reduce_kernel, dim3((nv + 255) / 256), dim3(256), 0, c->stream, nblocks, nv, w->hist_part,
                           d_hist);
    if (merge_blocks)
        hipLaunchKernelGGL(cut_tail_merge_kernel, dim3(merge_blocks), dim3(256), 0, c->stream, P, nblocks * 4 + fix_blocks * 4);
    hipLaunchKernelGGL(cut_fixup_kernel, dim3(fix_blocks), dim3(256), 0, c->stream, P, nblocks * 4);
    hipLaunchKernelGGL(cut_rescan_kernel, dim3(resc_blocks), dim3(256), 0, c->stream, P,
                       nblocks * 4 + fix_blocks * 4 + merge_blocks * 4);
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
    // vertex chunks of 32 or more, at most 512 of them (each block reads its chunk's rows of V once)
    const int chunk = std::max(32, (nv + 511) / 512);
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
        return clear_cut_stats(c);
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

extern "C" int twosd_cut_stats(twosd_ctx *c, int64_t *out) {
    if (!c || !out) return fail(TWOSD_E_ARG, "cut_stats: NULL");
    for (int i = 0; i < 4; ++i) out[i] = 0;
    CutWs *w = c->cut_ws ? (CutWs *)c->cut_ws : nullptr;
    if (!w || !w->fstats) return TWOSD_OK;
    unsigned long long h[16] = {};
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(h, w->fstats, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < 3; ++i) out[i] = (int64_t)h[i];
    out[3] = (int64_t)h[9];
    if (getenv("TWOSD_CUT3_COUNT_PRINT"))   // diagnostic build -DTWOSD_CUT3_COUNT only
        fprintf(stderr, "argmax3: chunk steps %llu, past the prefilter %llu, lanes past it %llu\n", h[10], h[11], h[12]);
    if (getenv("TWOSD_FIX_STAMPS_PRINT"))
        fprintf(stderr, "fixup stamps (cycles summed over waves): rows/setup %llu deltas %llu list %llu chains %llu decide %llu sums %llu\n",
                h[3], h[4], h[5], h[6], h[7], h[8]);
    return TWOSD_OK;
}

extern "C" int twosd_cut_pass(twosd_ctx *c, int *fp32, double *band) {
    if (!c || !fp32) return fail(TWOSD_E_ARG, "cut_pass: NULL");
    *fp32 = 0;
    if (band) *band = 0.0;
    CutWs *w = c->cut_ws ? (CutWs *)c->cut_ws : nullptr;
    if (!w || !w->band_bits) return TWOSD_OK;
    unsigned long long h[8] = {};
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(h, w->band_bits, sizeof(h), hipMemcpyDeviceToHost));
    *fp32 = (int)h[4];
    if (band) memcpy(band, &h[3], sizeof(double));
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
        return clear_cut_stats(c);
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
