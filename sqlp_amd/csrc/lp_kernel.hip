// lp_kernel.hip -- batched second-stage recourse LP on gfx950 (MI355X).
//
// Replaces the per-scenario GLPK solve inside solve_problem! (reference
// src/smps/smps_routines.jl:50-62, called from sd_iteration! algorithm.jl:45-55 and
// evaluate smps_routines.jl:67-82):
//     min q'y  s.t.  W y (G/L/E) b_w,  y >= 0,   b_w = r_w - T_w x.
// Only b_w changes between scenarios, so the optimal basis B0 of one scenario is dual
// feasible for all of them: every scenario runs a dual simplex warm-started at B0.
//
// Execution model (CDNA4-first):
//   * one 64-lane wavefront = one scenario; a persistent grid pulls scenarios from an
//     atomic work queue, so waves never synchronise with each other (no __syncthreads).
//   * row i of every basis-indexed vector (x_B, Devex weights, FTRAN/BTRAN vectors) is
//     held in registers: lane i % 64, slot i / 64 (R slots, template parameter).
//     Wave reductions are xor-butterflies, so every lane ends with identical bits.
//   * B0^{-1} (row-major and transposed, zero-padded to 64R columns) is shared by every
//     wave and stays L2/MALL resident; each pivot touches only (pivots+1) of its rows
//     (BTRAN) and the few columns of the entering variable (FTRAN): product-form update.
//   * the per-wave eta file (kmax x 64R fp64) is the only per-scenario HBM stream.
//   * rho (pivot row of B^{-1}) and the duals pi live in the wave's LDS slice for the
//     gather-heavy pricing pass over the CSC columns of W.
// Pivot rules: dual Devex leaving row (largest infeasibility^2 / weight, lowest row on
// ties), Harris two-pass ratio test (largest |alpha| among ratios <= relaxed bound,
// lowest column on ties).  Vertex recovery at the end: pi = c_B' B^{-1} recomputed
// from the final basis and components below PI_ZERO*(1+max|pi|) snapped to exact 0, so
// the 16-significant-bit dedup of dual_set.jl sees clean vertices.
#include <hip/hip_runtime.h>
#include <math.h>
#include "twosd_internal.h"

namespace twosd {

#define TOL_P 1e-9
#define TOL_D 1e-9
#define TOL_PIV 1e-9
#define PI_ZERO 1e-12

__device__ __forceinline__ double readlane_d(double v, int lane) {
    int2 p = *reinterpret_cast<int2 *>(&v);
    p.x = __builtin_amdgcn_readlane(p.x, lane);
    p.y = __builtin_amdgcn_readlane(p.y, lane);
    return *reinterpret_cast<double *>(&p);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}

// orders LDS traffic between lanes of one wave (hardware executes a wave's DS ops in
// order; this stops the compiler from reordering across it)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int R>
__device__ __forceinline__ double get_row(const double (&a)[R], int p) {
    const int slot = p >> 6;
    double v = a[0];
#pragma unroll
    for (int t = 1; t < R; ++t)
        if (t == slot) v = a[t];
    return readlane_d(v, p & 63);
}
template <int R>
__device__ __forceinline__ int get_row_i(const int (&a)[R], int p) {
    const int slot = p >> 6;
    int v = a[0];
#pragma unroll
    for (int t = 1; t < R; ++t)
        if (t == slot) v = a[t];
    return __builtin_amdgcn_readlane(v, p & 63);
}
template <int R, typename T>
__device__ __forceinline__ void set_row(T (&a)[R], int p, T v, int lane) {
    if (lane == (p & 63)) {
        const int slot = p >> 6;
#pragma unroll
        for (int t = 0; t < R; ++t)
            if (t == slot) a[t] = v;
    }
}

__device__ __forceinline__ int btype_of_hb(int hb) { return hb & 3; }

// Primal infeasibility of basic value x with bound type bt (bounds are 0 / +-inf).
__device__ __forceinline__ double infeas(double x, int bt) {
    if (bt == BT_Y || bt == BT_L) return x < -TOL_P ? x : 0.0;
    if (bt == BT_G) return x > TOL_P ? x : 0.0;
    return fabs(x) > TOL_P ? x : 0.0;   // E
}

template <int R>
__global__ void __launch_bounds__(256) lp_dual_simplex_kernel(LpParams P) {
    extern __shared__ double lds_raw[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int MP = 64 * R;
    const int kmaxp = (P.kmax + 3) & ~3;
    // per-wave LDS slice: rho[MP], pi[MP] (fp64), etap[kmaxp] (uint16)
    char *slice = reinterpret_cast<char *>(lds_raw) + (size_t)wid * (16 * MP + 2 * kmaxp);
    double *rho_l = reinterpret_cast<double *>(slice);
    double *pi_l = rho_l + MP;
    unsigned short *etap = reinterpret_cast<unsigned short *>(pi_l + MP);

    const int m = P.m, n = P.n, k = P.k;
    const int slot_id = blockIdx.x * kWavesPerBlock + wid;
    double *eta = P.eta + (size_t)slot_id * P.kmax * MP;
    const uint64_t fixedm = P.fixedmask[lane];
    const uint64_t ubm = P.ubmask[lane];

    for (;;) {
        int s = 0;
        if (lane == 0) s = atomicAdd(P.queue, 1);
        s = __builtin_amdgcn_readfirstlane(__shfl(s, 0));
        if (s >= P.N) break;

        // ---- warm start at B0: x_B = B0^{-1} (r - T x) + sum_e B0K[e] dv[s,e]
        double xB[R], w[R];
        int hb[R];
#pragma unroll
        for (int t = 0; t < R; ++t) {
            xB[t] = P.xbase[64 * t + lane];
            hb[t] = P.hb0[64 * t + lane];
            w[t] = 1.0;
            pi_l[64 * t + lane] = P.pi0[64 * t + lane];
        }
        const double *dvs = P.dv + (size_t)s * k;
        for (int e = 0; e < k; ++e) {
            const double d = dvs[e];   // wave-uniform -> scalar load
            const double *col = P.B0K + (size_t)e * MP;
#pragma unroll
            for (int t = 0; t < R; ++t) xB[t] = fma(col[64 * t + lane], d, xB[t]);
        }
        uint64_t bmask = P.basic0[lane];
        int K = 0, it = 0, status = TWOSD_LP_OPTIMAL;
        long long nops = k;   // x_B warm start: k rows
        wave_sync();

        for (;;) {
            // ---- 1. leaving row: max infeas^2 / w (lowest row on ties)
            double best = 0.0, bdel = 0.0;
            int br = 0x7fffffff;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                if (hb[t] < 0) continue;
                const double d = infeas(xB[t], btype_of_hb(hb[t]));
                if (d != 0.0) {
                    const double sc = d * d / w[t];
                    if (sc > best) { best = sc; br = 64 * t + lane; bdel = d; }
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double b2 = __shfl_xor(best, o);
                const int r2 = __shfl_xor(br, o);
                const double d2 = __shfl_xor(bdel, o);
                if (b2 > best || (b2 == best && r2 < br)) { best = b2; br = r2; bdel = d2; }
            }
            const int r = __builtin_amdgcn_readfirstlane(br);
            if (best == 0.0) break;   // primal feasible -> optimal
            if (K >= P.kmax) { status = TWOSD_LP_ITER_LIMIT; break; }
            const double delta = bdel;

            // ---- 2. BTRAN: u = e_r' E_K..E_1 (dense, registers), rho = u' B0^{-1}
            double u[R];
#pragma unroll
            for (int t = 0; t < R; ++t) u[t] = (64 * t + lane == r) ? 1.0 : 0.0;
            for (int tt = K - 1; tt >= 0; --tt) {
                const double *e = eta + (size_t)tt * MP;
                double acc = 0.0;
#pragma unroll
                for (int t = 0; t < R; ++t) acc = fma(u[t], e[64 * t + lane], acc);
                acc = wave_sum(acc);
                set_row<R, double>(u, (int)etap[tt], acc, lane);
            }
            double rh[R];
#pragma unroll
            for (int t = 0; t < R; ++t) rh[t] = 0.0;
            // nonzeros of u are at r and at the eta pivot rows; zero each after use
            for (int tt = K; tt >= 0; --tt) {
                const int p = (tt == K) ? r : (int)etap[tt];
                const double up = get_row<R>(u, p);
                if (up != 0.0) {
                    const double *row = P.B0inv + (size_t)p * MP;
#pragma unroll
                    for (int t = 0; t < R; ++t) rh[t] = fma(up, row[64 * t + lane], rh[t]);
                    set_row<R, double>(u, p, 0.0, lane);
                    ++nops;
                }
            }
            nops += K;
#pragma unroll
            for (int t = 0; t < R; ++t) rho_l[64 * t + lane] = rh[t];
            wave_sync();

            // ---- 3. Harris ratio test over nonbasic columns
            const double sg = delta > 0 ? 1.0 : -1.0;
            double thmax = INFINITY;
            for (int c = 0; c < P.C; ++c) {
                const uint64_t bit = 1ull << c;
                if ((bmask | fixedm) & bit) continue;
                const int j = 64 * c + lane;
                double a, d;
                if (j >= n) {
                    a = sg * rho_l[j - n];
                    d = -pi_l[j - n];
                } else {
                    double sa = 0.0, sp = 0.0;
                    for (int p = P.colptr[j]; p < P.colptr[j + 1]; ++p) {
                        const int ri = P.rowidx[p];
                        const double v = P.val[p];
                        sa = fma(rho_l[ri], v, sa);
                        sp = fma(pi_l[ri], v, sp);
                    }
                    a = sg * sa;
                    d = P.q[j] - sp;
                }
                const bool atlb = !(ubm & bit);
                if (atlb ? a > TOL_PIV : a < -TOL_PIV) {
                    const double ratio = (atlb ? d + TOL_D : d - TOL_D) / a;
                    thmax = fmin(thmax, ratio);
                }
            }
            thmax = wave_min(thmax);
            if (thmax == INFINITY) { status = TWOSD_LP_INFEASIBLE; break; }
            double bA = 0.0, bD = 0.0, bAs = 0.0;
            int bq = 0x7fffffff;
            for (int c = 0; c < P.C; ++c) {
                const uint64_t bit = 1ull << c;
                if ((bmask | fixedm) & bit) continue;
                const int j = 64 * c + lane;
                double a, d;
                if (j >= n) {
                    a = sg * rho_l[j - n];
                    d = -pi_l[j - n];
                } else {
                    double sa = 0.0, sp = 0.0;
                    for (int p = P.colptr[j]; p < P.colptr[j + 1]; ++p) {
                        const int ri = P.rowidx[p];
                        const double v = P.val[p];
                        sa = fma(rho_l[ri], v, sa);
                        sp = fma(pi_l[ri], v, sp);
                    }
                    a = sg * sa;
                    d = P.q[j] - sp;
                }
                const bool atlb = !(ubm & bit);
                if (atlb ? a > TOL_PIV : a < -TOL_PIV) {
                    if (d / a <= thmax && fabs(a) > bA) { bA = fabs(a); bq = j; bD = d; bAs = a; }
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double a2 = __shfl_xor(bA, o);
                const int q2 = __shfl_xor(bq, o);
                const double d2 = __shfl_xor(bD, o);
                const double s2 = __shfl_xor(bAs, o);
                if (a2 > bA || (a2 == bA && q2 < bq)) { bA = a2; bq = q2; bD = d2; bAs = s2; }
            }
            const int q = __builtin_amdgcn_readfirstlane(bq);
            if (bA == 0.0) { status = TWOSD_LP_NUMERIC; break; }
            const double thetaD = bD / bAs;

            // ---- 4. FTRAN entering column: col = E_K..E_1 B0^{-1} a_q
            double col[R];
            if (q >= n) {
                const double *cc = P.B0invT + (size_t)(q - n) * MP;
#pragma unroll
                for (int t = 0; t < R; ++t) col[t] = cc[64 * t + lane];
            } else {
#pragma unroll
                for (int t = 0; t < R; ++t) col[t] = 0.0;
                const int p0 = P.colptr[q], p1 = P.colptr[q + 1];
                for (int p = p0; p < p1; ++p) {
                    const double a = P.val[p];
                    const double *cc = P.B0invT + (size_t)P.rowidx[p] * MP;
#pragma unroll
                    for (int t = 0; t < R; ++t) col[t] = fma(a, cc[64 * t + lane], col[t]);
                }
            }
            for (int tt = 0; tt < K; ++tt) {
                const int p = etap[tt];
                const double vp = get_row<R>(col, p);
                if (vp != 0.0) {
                    const double *e = eta + (size_t)tt * MP;
                    const int ps = p >> 6;
#pragma unroll
                    for (int t = 0; t < R; ++t) {
                        const double ev = e[64 * t + lane];
                        col[t] = (t == ps && lane == (p & 63)) ? ev * vp : fma(ev, vp, col[t]);
                    }
                }
            }
            nops += K + (q >= n ? 1 : (P.colptr[q + 1] - P.colptr[q])) + 4;
            const double arq = get_row<R>(col, r);
            if (fabs(arq) < 1e-12) { status = TWOSD_LP_NUMERIC; break; }

            // ---- 5. updates: duals (LDS), primal, Devex weights, eta, basis
#pragma unroll
            for (int t = 0; t < R; ++t) pi_l[64 * t + lane] = fma(sg * thetaD, rh[t], pi_l[64 * t + lane]);
            const double thetaP = delta / arq;
            const double wr = get_row<R>(w, r);
            const double inv_arq = 1.0 / arq;
            double *eK = eta + (size_t)K * MP;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const int i = 64 * t + lane;
                const double ratio = col[t] * inv_arq;
                if (i == r) {
                    xB[t] = thetaP;
                    const double nw = wr * inv_arq * inv_arq;
                    w[t] = nw > 1.0 ? nw : 1.0;
                    eK[i] = inv_arq;
                } else {
                    xB[t] = fma(-thetaP, col[t], xB[t]);
                    const double cand = ratio * ratio * wr;
                    w[t] = cand > w[t] ? cand : w[t];
                    eK[i] = -ratio;
                }
            }
            if (lane == 0) etap[K] = (unsigned short)r;
            ++K;
            const int leaving = get_row_i<R>(hb, r) >> 2;
            if (lane == (leaving & 63)) bmask &= ~(1ull << (leaving >> 6));
            if (lane == (q & 63)) bmask |= 1ull << (q >> 6);
            set_row<R, int>(hb, r, q * 4 + (int)P.btype[q], lane);
            ++it;
            wave_sync();
        }

        // ---- vertex recovery + outputs
        double objv = NAN;
        if (status == TWOSD_LP_OPTIMAL) {
            double u[R];
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const int j = hb[t] >> 2;
                u[t] = (hb[t] >= 0 && j < n) ? P.q[j] : 0.0;
            }
            for (int tt = K - 1; tt >= 0; --tt) {
                const double *e = eta + (size_t)tt * MP;
                double acc = 0.0;
#pragma unroll
                for (int t = 0; t < R; ++t) acc = fma(u[t], e[64 * t + lane], acc);
                acc = wave_sum(acc);
                set_row<R, double>(u, (int)etap[tt], acc, lane);
            }
            double pv[R];
#pragma unroll
            for (int t = 0; t < R; ++t) pv[t] = 0.0;
#pragma unroll
            for (int ts = 0; ts < R; ++ts) {
                for (int l = 0; l < 64; ++l) {
                    const int p = 64 * ts + l;
                    if (p >= m) break;
                    const double up = readlane_d(u[ts], l);
                    if (up == 0.0) continue;
                    const double *row = P.B0inv + (size_t)p * MP;
#pragma unroll
                    for (int t = 0; t < R; ++t) pv[t] = fma(up, row[64 * t + lane], pv[t]);
                }
            }
            double pmax = 0.0;
#pragma unroll
            for (int t = 0; t < R; ++t) pmax = fmax(pmax, fabs(pv[t]));
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) pmax = fmax(pmax, __shfl_xor(pmax, o));
            const double zt = PI_ZERO * (1.0 + pmax);
            double ob = 0.0;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                if (fabs(pv[t]) <= zt) pv[t] = 0.0;
                const int j = hb[t] >> 2;
                if (hb[t] >= 0 && j < n) ob = fma(P.q[j], xB[t], ob);
            }
            objv = wave_sum(ob);
            nops += K + m;
            if (P.pi) {
                double *po = P.pi + (size_t)s * m;
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
        } else if (P.pi) {
            double *po = P.pi + (size_t)s * m;
#pragma unroll
            for (int t = 0; t < R; ++t)
                if (64 * t + lane < m) po[64 * t + lane] = NAN;
        }
        if (lane == 0) {
            P.obj[s] = objv;
            P.status[s] = status;
            P.iters[s] = it;
            if (P.ops) P.ops[s] = nops;
        }
        wave_sync();
    }
}

static const int kSupportedR[] = {1, 2, 3, 4, 6, 9, 12, 16};

int lp_rows_per_lane(int m) {
    for (int R : kSupportedR)
        if (m <= 64 * R) return R;
    return -1;
}

size_t lp_lds_bytes(int R, int kmax) {
    const int kmaxp = (kmax + 3) & ~3;
    return (size_t)kWavesPerBlock * (16 * 64 * R + 2 * kmaxp);
}

template <int R>
static hipError_t launch_R(const LpParams &p, int nblocks, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(lp_dual_simplex_kernel<R>, dim3(nblocks), dim3(256), lds, s, p);
    return hipGetLastError();
}

template <int R>
static int occ_R(size_t lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, lp_dual_simplex_kernel<R>, 256, lds) != hipSuccess) return 1;
    return nb > 0 ? nb : 1;
}

int lp_max_blocks_per_cu(int R, int kmax) {
    const size_t lds = lp_lds_bytes(R, kmax);
    switch (R) {
        case 1: return occ_R<1>(lds);
        case 2: return occ_R<2>(lds);
        case 3: return occ_R<3>(lds);
        case 4: return occ_R<4>(lds);
        case 6: return occ_R<6>(lds);
        case 9: return occ_R<9>(lds);
        case 12: return occ_R<12>(lds);
        case 16: return occ_R<16>(lds);
    }
    return 1;
}

hipError_t launch_lp(int R, const LpParams &p, int nblocks, size_t lds, hipStream_t s) {
    switch (R) {
        case 1: return launch_R<1>(p, nblocks, lds, s);
        case 2: return launch_R<2>(p, nblocks, lds, s);
        case 3: return launch_R<3>(p, nblocks, lds, s);
        case 4: return launch_R<4>(p, nblocks, lds, s);
        case 6: return launch_R<6>(p, nblocks, lds, s);
        case 9: return launch_R<9>(p, nblocks, lds, s);
        case 12: return launch_R<12>(p, nblocks, lds, s);
        case 16: return launch_R<16>(p, nblocks, lds, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace twosd
