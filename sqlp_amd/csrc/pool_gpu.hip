// pool_gpu.hip -- device side of a pool refresh: the B^{-1} of every harvested basis and every
// pool-strided array the LP kernel and the pool selection read, built on the GPU.
//
// The host path of api.hip (compose_binv in host_basis.cpp, then upload_pool and
// prepare_elements) composes B^{-1} = E_K..E_1 B_pb^{-1} by sparse row merges and re-derives
// CSC, element rows, sliced ELL, d0 and the basis words on 16 host threads before a PCIe
// upload -- at 4096 bases ~60 ms of a ~90 ms refresh.  Here every column of B^{-1} is the
// eta sequence applied to the start basis's column (a sparse FTRAN: eta t is skipped when the
// column's entry in its pivot row is zero), one wavefront per column with the column dense in
// LDS, so no HBM round trip of a dense B^{-1}:
//   pg_ftran_kernel<0>  per source: max |.| over B_pb^{-1} and the result (drop threshold
//                       1e-14 max, as compose_binv) and per column the nonzero count;
//                       <0> also keeps each column's nonzeros (rows ascending) in a per-source
//                       scratch of sc_cap entries;
//   pg_gather_kernel    the kept entries of each column copied from that scratch (rows
//                       ascending) into an intermediate CSC at host-prefixed offsets.  Kept:
//                       rows some eta touched |v| > drop, other rows exactly B_pb^{-1}'s
//                       entries -- compose_binv's rule, and its arithmetic: row r <- eta_r x_r,
//                       row i <- fma(eta_i, x_r, row i), so the values are bit-identical;
//   pg_ftran_kernel<1>  the same FTRAN again, writing the kept entries directly: only for the
//                       sources whose nonzeros overflowed the scratch (round 3 ran it for all);
//   pg_count_kernel     per source: row / element-row counts, pi0, the dual-feasibility and
//                       4-probe residual checks of finish_composed, the per-basis totals;
//   pg_fill_kernel      at host-prefixed offsets: CSC (compacted), CSR (columns ascending,
//                       one wave walking the columns), element rows as CSR and sliced ELL (one
//                       wave walking the elements, e ascending), hb0 / basic0 / bnnz / d0 /
//                       selection pointers -- upload_pool's and prepare_elements's layouts and
//                       entry order.
// HBM traffic is O(nnz) per basis (~0.2 MB for storm) instead of the dense m x m.
#include <hip/hip_runtime.h>
#include "twosd_internal.h"

namespace twosd {

namespace {

constexpr int kPgThreads = 256;                  // count / fill kernels
constexpr int kFtThreads = 1024;                 // FTRAN kernels: 16 waves = 16 columns at a time per source
constexpr int kFtWaves = kFtThreads / 64;

struct Src {
    int pb, K, off;
    const int *head, *etap, *etaoff;
};

__device__ inline Src src_of(const PgArgs &A, int a) {
    Src s;
    if (a == 0) {
        s.pb = 0; s.K = 0; s.off = 0; s.head = A.head0; s.etap = nullptr; s.etaoff = nullptr;
        return s;
    }
    const int l = A.src_row[a - 1];
    s.pb = A.eo_pb[l];
    s.K = A.eo_K[l];
    s.off = A.eo_off[l];
    s.head = A.heads + (size_t)l * A.m;
    s.etap = A.eo_etap + (size_t)l * A.kmax;
    s.etaoff = A.eo_etaoff + (size_t)l * (A.kmax + 1);
    return s;
}

__device__ inline bool src_ok(const PgArgs &A, const Src &S) {
    return S.K >= 0 && S.K <= A.kmax && S.pb >= 0 && S.pb < A.npool_old;
}

// exclusive prefix of in[0, n) into out[0, n], out[n] = total (all NT threads of the block)
template <int NT = kPgThreads>
__device__ void block_scan(const int *in, int *out, int n, int *tmp) {
    const int tid = threadIdx.x, per = (n + NT - 1) / NT;
    const int b = min(n, tid * per), e = min(n, b + per);
    int s = 0;
    for (int i = b; i < e; ++i) s += in[i];
    tmp[tid] = s;
    __syncthreads();
    for (int o = 1; o < NT; o <<= 1) {
        const int v = tid >= o ? tmp[tid - o] : 0;
        __syncthreads();
        tmp[tid] += v;
        __syncthreads();
    }
    int run = tid ? tmp[tid - 1] : 0;
    for (int i = b; i < e; ++i) {
        out[i] = run;
        run += in[i];
    }
    if (tid == NT - 1) out[n] = tmp[NT - 1];
    __syncthreads();
}

__device__ inline unsigned long long lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// rows any eta of the source touches (compose_binv re-filters exactly these rows)
template <int NT>
__device__ void mark_touched(const PgArgs &A, const Src &S, unsigned char *touched) {
    for (int i = threadIdx.x; i < A.m; i += NT) touched[i] = 0;
    __syncthreads();
    const int ne = S.K > 0 ? S.etaoff[S.K] : 0;
    for (int e = threadIdx.x; e < ne; e += NT) touched[A.eo_eidx[S.off + e]] = 1;
    __syncthreads();
}

}  // namespace

// ---- 1. FTRAN of every column of B_pb^{-1} through the eta file ----------------------------
template <int PASS>
__global__ __launch_bounds__(kFtThreads) void pg_ftran_kernel(PgArgs A) {
    extern __shared__ double smem[];
    __shared__ int tmp[kFtThreads];
    __shared__ double red[kFtWaves];
    const int a = A.a0 + blockIdx.x, m = A.m, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const Src S = src_of(A, a);
    if (!src_ok(A, S) || (PASS == 1 && !(A.amax[a] >= 0.0))) {   // eta file did not fit: unusable
        if (PASS == 0 && tid == 0) { A.amax[a] = -1.0; A.nztot[a] = 0; }
        return;
    }
    if (PASS == 1 && A.sc_cap > 0 && A.nztot[a] <= A.sc_cap) return;   // pg_gather_kernel's source
    __shared__ int sc_ctr;                                // PASS 0: scratch entries claimed
    if (PASS == 0 && tid == 0) sc_ctr = 0;                // (visible after mark_touched's barriers)
    double *x = smem + (size_t)wv * m;                    // this wave's column, dense
    int *etap = reinterpret_cast<int *>(smem + (size_t)kFtWaves * m);
    int *etaoff = etap + A.kmax;
    int *cstart = etaoff + A.kmax + 1;                    // PASS 1: column offsets (m + 1)
    unsigned char *touched = reinterpret_cast<unsigned char *>(cstart + m + 1);
    for (int t = tid; t < S.K; t += kFtThreads) etap[t] = S.etap[t];
    for (int t = tid; t <= S.K; t += kFtThreads) etaoff[t] = S.K > 0 ? S.etaoff[t] : 0;
    mark_touched<kFtThreads>(A, S, touched);
    // bit 2: the etas' pivot rows (each is also one of its eta's rows, so already marked 1; two etas
    // on one row both write 3)
    for (int t = tid; t < S.K; t += kFtThreads) touched[S.etap[t]] = 3;
    __syncthreads();
    double drop = 0.0;
    int *nzc = A.nzc + (size_t)a * m;
    if (PASS == 1) {
        block_scan<kFtThreads>(nzc, cstart, m, tmp);
        drop = 1e-14 * A.amax[a];
    }
    const int *cp = A.bcp0 + (size_t)S.pb * (A.MP + 1);
    const int *eidx = A.eo_eidx + S.off;
    const double *evals = A.eo_evals + S.off;
    double amax = 0.0;
    int nzsum = 0;   // PASS 0, lane 0: nonzeros of this wave's columns
    for (int c = wv; c < m; c += kFtWaves) {
        // a column of B_pb^{-1} with no entry in any eta's pivot row passes every eta unchanged (each
        // E_t acts only when x at its pivot row is nonzero, and none of them writes it): its entries,
        // rows ascending, are the FTRAN's result as they stand -- the same values and order the dense
        // walk below produces, without it.  (storm: ~6 entries a column against ~8 pivot rows, so
        // most columns; one wave step of up to 64 entries, checked ascending)
        {
            const int q0 = cp[c], q1 = cp[c + 1];
            if (q1 - q0 <= 64) {
                const int q = q0 + lane;
                const bool has = q < q1;
                const int i = has ? A.bci0[q] : 0x7fffffff;
                const double v = has ? A.bcv0[q] : 0.0;
                const int inext = __shfl_down(i, 1);
                const bool bad = has && (((touched[i] & 2) != 0) || (lane < 63 && q + 1 < q1 && inext <= i));
                if (__ballot(bad) == 0) {
                    amax = fmax(amax, fabs(v));
                    const bool nz = has && v != 0.0;
                    const unsigned long long msk = __ballot(nz);
                    const int cnt = __popcll(msk);
                    if (PASS == 0) {
                        if (lane == 0) nzc[c] = cnt;
                        nzsum += cnt;
                        if (A.sc_cap > 0) {
                            int off = 0;
                            if (lane == 0) off = atomicAdd(&sc_ctr, cnt);
                            off = __shfl(off, 0);
                            if ((long long)off + cnt <= A.sc_cap && nz) {
                                const size_t at = (size_t)a * A.sc_cap + off + __popcll(msk & lanemask_lt(lane));
                                A.sc_row[at] = i;
                                A.sc_val[at] = v;
                            }
                            if (lane == 0) A.sc_off[(size_t)a * m + c] = off;
                        }
                    } else {
                        const bool kk = has && (touched[i] ? fabs(v) > drop : v != 0.0);
                        const unsigned long long km = __ballot(kk);
                        if (kk) {
                            const size_t at = (size_t)A.inter_off[a] + cstart[c] + __popcll(km & lanemask_lt(lane));
                            A.inter_row[at] = i;
                            A.inter_val[at] = v;
                        }
                        if (lane == 0) A.keptc[(size_t)a * m + c] = __popcll(km);
                    }
                    __builtin_amdgcn_wave_barrier();
                    continue;
                }
            }
        }
        for (int i = lane; i < m; i += 64) x[i] = 0.0;
        __builtin_amdgcn_wave_barrier();
        for (int q = cp[c] + lane; q < cp[c + 1]; q += 64) {
            const double v = A.bcv0[q];
            x[A.bci0[q]] = v;
            amax = fmax(amax, fabs(v));
        }
        __builtin_amdgcn_wave_barrier();
        for (int t = 0; t < S.K; ++t) {
            const int r = etap[t];
            const double xr = x[r];
            __builtin_amdgcn_wave_barrier();
            if (xr != 0.0) {   // E_t x = x + (eta - e_r) x_r: nothing to do when x_r = 0
                for (int e = etaoff[t] + lane; e < etaoff[t + 1]; e += 64) {   // distinct rows
                    const int i = eidx[e];
                    const double v = evals[e];
                    x[i] = i == r ? v * xr : fma(v, xr, x[i]);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (PASS == 0) {
            int cnt = 0;
            for (int i0 = 0; i0 < m; i0 += 64) {
                const int i = i0 + lane;
                const double v = i < m ? x[i] : 0.0;
                amax = fmax(amax, fabs(v));
                cnt += __popcll(__ballot(v != 0.0));
            }
            if (lane == 0) nzc[c] = cnt;
            nzsum += cnt;
            if (A.sc_cap > 0) {   // keep the nonzeros for the gather (a claim past sc_cap: none kept)
                int off = 0;
                if (lane == 0) off = atomicAdd(&sc_ctr, cnt);
                off = __shfl(off, 0);
                if ((long long)off + cnt <= A.sc_cap) {
                    const size_t base = (size_t)a * A.sc_cap + off;
                    int run = 0;
                    for (int i0 = 0; i0 < m; i0 += 64) {
                        const int i = i0 + lane;
                        const double v = i < m ? x[i] : 0.0;
                        const unsigned long long msk = __ballot(v != 0.0);
                        if (v != 0.0) {
                            const size_t at = base + run + __popcll(msk & lanemask_lt(lane));
                            A.sc_row[at] = i;
                            A.sc_val[at] = v;
                        }
                        run += __popcll(msk);
                    }
                }
                if (lane == 0) A.sc_off[(size_t)a * m + c] = off;
            }
        } else {
            const size_t base = (size_t)A.inter_off[a] + cstart[c];
            int run = 0;
            for (int i0 = 0; i0 < m; i0 += 64) {
                const int i = i0 + lane;
                const double v = i < m ? x[i] : 0.0;
                const bool kk = i < m && (touched[i] ? fabs(v) > drop : v != 0.0);
                const unsigned long long msk = __ballot(kk);
                if (kk) {
                    const size_t at = base + run + __popcll(msk & lanemask_lt(lane));
                    A.inter_row[at] = i;
                    A.inter_val[at] = v;
                }
                run += __popcll(msk);
            }
            if (lane == 0) A.keptc[(size_t)a * m + c] = run;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (PASS == 0) {
        for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
        if (lane == 0) {
            red[wv] = amax;
            tmp[wv] = nzsum;
        }
        __syncthreads();
        if (tid == 0) {   // nztot: read back by the host for the intermediate offsets
            double v = red[0];
            int t = tmp[0];
            for (int w = 1; w < kFtWaves; ++w) {
                v = fmax(v, red[w]);
                t += tmp[w];
            }
            A.amax[a] = v;
            A.nztot[a] = t;
        }
    }
}

// ---- 1b. the kept entries from the first pass's scratch --------------------------------------
// per column the entries of pg_ftran_kernel<1> (same rows, values and order: the scratch holds
// the column's nonzeros rows ascending, v != 0, and the drop rule is applied here)
__global__ __launch_bounds__(kFtThreads) void pg_gather_kernel(PgArgs A) {
    extern __shared__ double smem[];
    __shared__ int tmp[kFtThreads];
    const int a = A.a0 + blockIdx.x, m = A.m, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (!(A.amax[a] >= 0.0) || A.nztot[a] > A.sc_cap) return;   // unusable, or pass 1's source
    const Src S = src_of(A, a);
    int *cstart = reinterpret_cast<int *>(smem);
    int *soff = cstart + m + 1;                           // scratch offsets, staged once
    unsigned char *touched = reinterpret_cast<unsigned char *>(soff + m);
    for (int c = tid; c < m; c += kFtThreads) soff[c] = A.sc_off[(size_t)a * m + c];
    mark_touched<kFtThreads>(A, S, touched);
    block_scan<kFtThreads>(A.nzc + (size_t)a * m, cstart, m, tmp);
    const double drop = 1e-14 * A.amax[a];
    const int *srow = A.sc_row + (size_t)a * A.sc_cap;
    const double *sval = A.sc_val + (size_t)a * A.sc_cap;
    for (int c = wv; c < m; c += kFtWaves) {
        const int n = cstart[c + 1] - cstart[c], off = soff[c];
        const size_t base = (size_t)A.inter_off[a] + cstart[c];
        int run = 0;
        for (int q0 = 0; q0 < n; q0 += 64) {
            const int q = q0 + lane;
            int i = 0;
            double v = 0.0;
            if (q < n) {
                i = srow[off + q];
                v = sval[off + q];
            }
            const bool kk = q < n && (touched[i] ? fabs(v) > drop : true);
            const unsigned long long msk = __ballot(kk);
            if (kk) {
                const size_t at = base + run + __popcll(msk & lanemask_lt(lane));
                A.inter_row[at] = i;
                A.inter_val[at] = v;
            }
            run += __popcll(msk);
        }
        if (lane == 0) A.keptc[(size_t)a * m + c] = run;
    }
}

// ---- 2. counts, pi0, checks --------------------------------------------------------------
__global__ __launch_bounds__(kPgThreads) void pg_count_kernel(PgArgs A) {
    extern __shared__ double smem[];
    __shared__ int s_tot[4], s_bad;
    __shared__ int tmp[kPgThreads];
    const int a = A.a0 + blockIdx.x, m = A.m, n = A.n, k = A.k, tid = threadIdx.x;
    const double amax = A.amax[a];
    if (!(amax >= 0.0)) {
        if (tid < 4) A.tot[(size_t)a * 4 + tid] = 0;
        if (tid == 0) A.valid[a] = 0;
        return;
    }
    const Src S = src_of(A, a);
    double *pi0 = smem, *cbv = smem + m, *y = cbv + m;
    int *rowc = reinterpret_cast<int *>(y + m), *erow = rowc + m, *cstart = erow + m;   // cstart: m + 1
    unsigned char *isb = reinterpret_cast<unsigned char *>(cstart + m + 1);
    if (tid < 4) s_tot[tid] = 0;
    if (tid == 0) s_bad = 0;
    for (int i = tid; i < m; i += kPgThreads) { rowc[i] = 0; erow[i] = 0; }
    for (int j = tid; j < n + m; j += kPgThreads) isb[j] = 0;
    __syncthreads();
    for (int i = tid; i < m; i += kPgThreads) {
        const int j = S.head[i];
        isb[j] = 1;
        cbv[i] = j < n ? A.q[j] : 0.0;
    }
    const int *keptc = A.keptc + (size_t)a * m;
    block_scan(A.nzc + (size_t)a * m, cstart, m, tmp);    // intermediate column starts
    const int *irow = A.inter_row + A.inter_off[a];
    const double *ival = A.inter_val + A.inter_off[a];
    // per column (one thread a column): row counts, pi0 = c_B' B^{-1} (rows ascending)
    for (int c = tid; c < m; c += kPgThreads) {
        double pi = 0.0;
        for (int q = cstart[c]; q < cstart[c] + keptc[c]; ++q) {
            const int i = irow[q];
            atomicAdd(&rowc[i], 1);
            pi += cbv[i] * ival[q];
        }
        pi0[c] = pi;
    }
    // element rows: column row_e of B^{-1} gives element e an entry in each of its rows
    for (int e = tid; e < k; e += kPgThreads) {
        const int c = A.pos_row[e];
        for (int q = cstart[c]; q < cstart[c] + keptc[c]; ++q) atomicAdd(&erow[irow[q]], 1);
    }
    __syncthreads();
    int bad = 0;
    // dual feasibility of the nonbasic columns (sparse_dual_infeasibility, 1e-7)
    for (int j = tid; j < n + m; j += kPgThreads) {
        if (isb[j]) continue;
        const int bt = A.btype[j];
        if (bt == BT_E) continue;
        double s = 0.0;
        if (j >= n) s = pi0[j - n];
        else
            for (int q = A.colptr[j]; q < A.colptr[j + 1]; ++q) s += pi0[A.rowidx[q]] * A.val[q];
        const double d = (j < n ? A.q[j] : 0.0) - s;
        if (!((bt == BT_G ? d : -d) <= 1e-7)) bad = 1;
    }
    // B^{-1} a_{head[i0]} = e_{i0} at the probes of sparse_basis_residual (1e-8): the columns
    // of B^{-1} at a's rows, scaled and accumulated
    for (int probe = 0; probe < 4; ++probe) {
        const int i0 = (int)(((long long)probe * 7919 + 13) % m), j = S.head[i0];
        __syncthreads();
        for (int i = tid; i < m; i += kPgThreads) y[i] = 0.0;
        __syncthreads();
        const int q0 = j >= n ? 0 : A.colptr[j], q1 = j >= n ? 1 : A.colptr[j + 1];
        for (int qa = q0; qa < q1; ++qa) {
            const int r = j >= n ? j - n : A.rowidx[qa];
            const double av = j >= n ? 1.0 : A.val[qa];
            for (int q = cstart[r] + tid; q < cstart[r] + keptc[r]; q += kPgThreads) y[irow[q]] += ival[q] * av;
            __syncthreads();   // rows are distinct within a column; columns one after another
        }
        for (int i = tid; i < m; i += kPgThreads)
            if (!(fabs(y[i] - (i == i0 ? 1.0 : 0.0)) <= 1e-8)) bad = 1;
    }
    if (bad) atomicOr(&s_bad, 1);
    for (int i = tid; i < m; i += kPgThreads) {
        A.rowcnt[(size_t)a * m + i] = rowc[i];
        A.erowcnt[(size_t)a * m + i] = erow[i];
        atomicAdd(&s_tot[0], rowc[i]);
        atomicAdd(&s_tot[1], erow[i]);
        // selection records: every row active, rows of fixed basics twice (prepare_elements)
        atomicAdd(&s_tot[3], (1 + erow[i]) * (A.btype[S.head[i]] == BT_E ? 2 : 1));
    }
    if (tid < A.R9) {   // ELL entry rows: per slot of 64 rows the widest row
        int w = 0;
        for (int l = 0; l < 64 && 64 * tid + l < m; ++l) w = max(w, erow[64 * tid + l]);
        atomicAdd(&s_tot[2], w);
    }
    __syncthreads();
    if (tid < 4) A.tot[(size_t)a * 4 + tid] = s_tot[tid];
    if (tid == 0) A.valid[a] = s_bad ? 0 : 1;
}

// ---- 3. pool-strided outputs --------------------------------------------------------------
__global__ __launch_bounds__(kPgThreads) void pg_fill_kernel(PgArgs A, PgFill F) {
    extern __shared__ double smem[];
    __shared__ int tmp[kPgThreads];
    __shared__ uint64_t bits[64];
    __shared__ int ws[65];   // ELL slot offsets (entry rows)
    const int p = F.P0 + blockIdx.x, a = F.map[p];
    const int m = A.m, n = A.n, k = A.k, MP = A.MP, R9 = A.R9, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // a gathered source table (distributed refresh) carries its heads; otherwise the head row
    // of the source's training scenario
    const int *shead = a == 0 ? A.head0 : (A.gheads ? A.gheads + (size_t)(a - 1) * m : src_of(A, a).head);
    double *pi0 = smem, *cbv = smem + m;
    int *rs = reinterpret_cast<int *>(cbv + m), *cs = rs + (m + 1), *es = cs + (m + 1), *ic = es + (m + 1);
    int *cur = ic + (m + 1), *ecur = cur + m;
    unsigned char *isb = reinterpret_cast<unsigned char *>(ecur + m);
    for (int j = tid; j < n + m; j += kPgThreads) isb[j] = 0;
    for (int i = tid; i < m; i += kPgThreads) { cur[i] = 0; ecur[i] = 0; }
    if (tid < 64) bits[tid] = 0;
    __syncthreads();
    for (int i = tid; i < m; i += kPgThreads) {
        const int j = shead[i];
        isb[j] = 1;
        cbv[i] = j < n ? A.q[j] : 0.0;
        atomicOr(reinterpret_cast<unsigned long long *>(&bits[j & 63]), 1ull << (j >> 6));
    }
    const int *keptc = A.keptc + (size_t)a * m;
    block_scan(A.rowcnt + (size_t)a * m, rs, m, tmp);
    block_scan(keptc, cs, m, tmp);
    block_scan(A.erowcnt + (size_t)a * m, es, m, tmp);
    block_scan(A.nzc + (size_t)a * m, ic, m, tmp);        // intermediate column starts
    if (tid == 0) {   // ELL slots: widest element row of each 64 rows
        int o = F.off[(size_t)p * 4 + 2];
        for (int t = 0; t < R9; ++t) {
            int w = 0;
            for (int l = 0; l < 64 && 64 * t + l < m; ++l) w = max(w, es[64 * t + l + 1] - es[64 * t + l]);
            ws[t] = o;
            F.kslot[(size_t)p * (R9 + 1) + t] = o;
            o += w;
        }
        ws[R9] = o;
        F.kslot[(size_t)p * (R9 + 1) + R9] = o;
    }
    __syncthreads();
    const int nb = F.off[(size_t)p * 4 + 0], eb = F.off[(size_t)p * 4 + 1];
    const int *irow = A.inter_row + A.inter_off[a];
    const double *ival = A.inter_val + A.inter_off[a];
    if (wv == 0) {
        // B^{-1} rows (CSR, columns ascending): walk the columns in order, per-row cursors (a
        // column's rows are distinct, so its entries go in any lane order).  The first 64 entries
        // of column c + 1 are loaded while column c is written: one memory round trip per column
        // hides behind the previous one (column sizes from the LDS scan, cs)
        int ni = 0;
        double nv = 0.0;
        if (m > 0 && lane < cs[1] - cs[0]) { ni = irow[ic[0] + lane]; nv = ival[ic[0] + lane]; }
        for (int c = 0; c < m; ++c) {
            const int kc = cs[c + 1] - cs[c];
            const int i0 = ni;
            const double v0 = nv;
            if (c + 1 < m && lane < cs[c + 2] - cs[c + 1]) { ni = irow[ic[c + 1] + lane]; nv = ival[ic[c + 1] + lane]; }
            if (lane < kc) {
                const int at = nb + rs[i0] + cur[i0]++;
                F.brcol[at] = c;
                F.brval[at] = v0;
            }
            for (int q = ic[c] + 64 + lane; q < ic[c] + kc; q += 64) {   // columns of > 64 rows
                const int i = irow[q];
                const int at = nb + rs[i] + cur[i]++;
                F.brcol[at] = c;
                F.brval[at] = ival[q];
            }
            __builtin_amdgcn_wave_barrier();
        }
    } else if (wv == 1) {
        // element rows (CSR, e ascending) and their sliced ELL: walk the elements in order, the
        // next element's column loaded ahead as above
        auto put = [&](int e, int i, double v) {
            const int j = ecur[i]++;
            F.ke[eb + es[i] + j] = e;
            F.kraw[eb + es[i] + j] = v;
            const size_t at = ((size_t)ws[i >> 6] + j) * 64 + (i & 63);
            F.kix[at] = e;
            F.kv[at] = v;
        };
        int ni = 0, nc = k > 0 ? A.pos_row[0] : 0;
        double nv = 0.0;
        if (k > 0 && lane < cs[nc + 1] - cs[nc]) { ni = irow[ic[nc] + lane]; nv = ival[ic[nc] + lane]; }
        for (int e = 0; e < k; ++e) {
            const int c = nc, i0 = ni;
            const double v0 = nv;
            const int kc = cs[c + 1] - cs[c];
            if (e + 1 < k) {
                nc = A.pos_row[e + 1];
                if (lane < cs[nc + 1] - cs[nc]) { ni = irow[ic[nc] + lane]; nv = ival[ic[nc] + lane]; }
            }
            if (lane < kc) put(e, i0, v0);
            for (int q = ic[c] + 64 + lane; q < ic[c] + kc; q += 64) put(e, irow[q], ival[q]);
            __builtin_amdgcn_wave_barrier();
        }
    } else {
        // B^{-1} columns (CSC, rows ascending, compacted) and pi0 (rows ascending)
        for (int c = tid - 128; c < m; c += kPgThreads - 128) {
            const int base = nb + cs[c];
            double pi = 0.0;
            for (int q = 0; q < keptc[c]; ++q) {
                const int i = irow[ic[c] + q];
                const double v = ival[ic[c] + q];
                F.bci[base + q] = i;
                F.bcv[base + q] = v;
                pi += cbv[i] * v;
            }
            pi0[c] = pi;
        }
        // ELL padding: entries [rows of row i, slot width) of every lane (rows >= m: all)
        for (int i = tid - 128; i < 64 * R9; i += kPgThreads - 128) {
            const int t = i >> 6, l = i & 63, w = ws[t + 1] - ws[t];
            for (int j = i < m ? es[i + 1] - es[i] : 0; j < w; ++j) {
                F.kix[((size_t)ws[t] + j) * 64 + l] = 0;
                F.kv[((size_t)ws[t] + j) * 64 + l] = 0.0;
            }
        }
    }
    for (int i = tid; i <= MP; i += kPgThreads) {
        F.brptr[(size_t)p * (MP + 1) + i] = nb + rs[min(i, m)];
        F.bcp[(size_t)p * (MP + 1) + i] = nb + cs[min(i, m)];
    }
    for (int i = tid; i <= m; i += kPgThreads) F.kp[(size_t)p * (m + 1) + i] = eb + es[i];
    for (int i = tid; i < MP; i += kPgThreads)
        F.hb0[(size_t)p * MP + i] = i < m ? shead[i] * 4 + A.btype[shead[i]] : -1;
    if (tid < 64) F.basic0[(size_t)p * 64 + tid] = bits[tid];
    if (tid == 0) {
        F.bnnz[p] = rs[m];
        F.sel_ptr[p] = F.off[(size_t)p * 4 + 3];
        if (p == F.P - 1) F.sel_ptr[F.P] = F.sel_total;
    }
    __syncthreads();
    // d0 = q - W' pi0 on the nonbasic columns (lane-slot order j < 64 CH); pool[0] keeps its
    // uploaded d0 (pi0 from the dense setup inverse)
    for (int j = tid; j < 64 * A.CH; j += kPgThreads) {
        double d;
        if (p == 0) d = F.d0_primary[j];
        else if (j >= n + m || isb[j]) d = 0.0;
        else if (j >= n) d = 0.0 - pi0[j - n];
        else {
            double s = 0.0;
            for (int q = A.colptr[j]; q < A.colptr[j + 1]; ++q) s += pi0[A.rowidx[q]] * A.val[q];
            d = A.q[j] - s;
        }
        F.d0[(size_t)p * 64 * A.CH + j] = d;
    }
}

static size_t ftran_lds(const PgArgs &A) {
    return sizeof(double) * kFtWaves * A.m + sizeof(int) * (2 * A.kmax + 1 + A.m + 1) + A.m + 16;
}
static size_t gather_lds(const PgArgs &A) { return sizeof(int) * (2 * A.m + 1) + A.m + 16; }
static size_t count_lds(const PgArgs &A) {
    return sizeof(double) * 3 * A.m + sizeof(int) * (3 * A.m + 1) + (A.n + A.m) + 16;
}
static size_t fill_lds(const PgArgs &A) {
    return sizeof(double) * 2 * A.m + sizeof(int) * (4 * (A.m + 1) + 2 * A.m) + (A.n + A.m) + 16;
}

int pg_supported(int m, int n, int kmax) {
    PgArgs A{};
    A.m = m; A.n = n; A.kmax = kmax;
    return ftran_lds(A) <= 96 * 1024 && count_lds(A) <= 64 * 1024 && fill_lds(A) <= 64 * 1024 && (m + 63) / 64 <= 64;
}

template <int PASS>
static hipError_t launch_ftran(const PgArgs &A, int nb, hipStream_t s) {
    hipError_t e = hipFuncSetAttribute((const void *)pg_ftran_kernel<PASS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)ftran_lds(A));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pg_ftran_kernel<PASS>, dim3(nb), dim3(kFtThreads), ftran_lds(A), s, A);
    return hipGetLastError();
}
hipError_t pg_launch_ftran(const PgArgs &A, int pass, int nb, hipStream_t s) {
    return pass == 0 ? launch_ftran<0>(A, nb, s) : launch_ftran<1>(A, nb, s);
}
hipError_t pg_launch_gather(const PgArgs &A, int nb, hipStream_t s) {
    hipLaunchKernelGGL(pg_gather_kernel, dim3(nb), dim3(kFtThreads), gather_lds(A), s, A);
    return hipGetLastError();
}
hipError_t pg_launch_count(const PgArgs &A, int nb, hipStream_t s) {
    hipLaunchKernelGGL(pg_count_kernel, dim3(nb), dim3(kPgThreads), count_lds(A), s, A);
    return hipGetLastError();
}
hipError_t pg_launch_fill(const PgArgs &A, const PgFill &F, int np, hipStream_t s) {
    hipLaunchKernelGGL(pg_fill_kernel, dim3(np), dim3(kPgThreads), fill_lds(A), s, A, F);
    return hipGetLastError();
}

}  // namespace twosd
