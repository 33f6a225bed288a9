// pool_gpu.hip -- device side of a pool refresh: the B^{-1} of every harvested basis and every
// pool-strided array the LP kernel and the pool selection read, built on the GPU.
//
// The host path of api.hip (compose_binv in host_basis.cpp, then upload_pool and
// prepare_elements) composes B^{-1} = E_K..E_1 B_pb^{-1} by sparse row merges and re-derives
// CSC, element rows, sliced ELL, d0 and the basis words on 16 host threads before a PCIe
// upload -- at 4096 bases that is ~60 ms of a ~90 ms refresh.  Here, per source basis (one
// workgroup):
//   pg_dense_kernel  B_pb^{-1} column tile (m x W doubles, all rows, in LDS) <- the start
//                    basis's CSC columns; the K etas applied in order (row r <- eta_r row r,
//                    row i <- fma(eta_i, old row r, row i): the same operations and rounding
//                    as compose_binv); the tile written to a dense scratch D (HBM).
//   pg_count_kernel  the entries kept (rows an eta touched: |v| > 1e-14 max|.|, the others
//                    exactly B_pb^{-1}'s pattern, as compose_binv), per row / column /
//                    element-row counts, pi0, the dual-feasibility and 4-probe residual checks
//                    of finish_composed, and the per-basis totals.
//   pg_fill_kernel   at offsets the host prefix-summed from the totals: B^{-1} CSR (columns
//                    ascending) and CSC (rows ascending), element rows as CSR (e ascending)
//                    and sliced ELL, hb0 / basic0 / bnnz / d0 / selection-record pointers --
//                    the layouts (and entry order) of upload_pool and prepare_elements.
// Bytes: D is written once and read ~3x (2.2 MB per storm basis); the rest is the output.
#include <hip/hip_runtime.h>
#include "twosd_internal.h"

namespace twosd {

namespace {

constexpr int kPgThreads = 256;
constexpr size_t kPgTileBytes = 144 * 1024;   // LDS tile budget (gfx950: 160 KB per workgroup)

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
    const int l = a - 1;
    s.pb = A.eo_pb[l];
    s.K = A.eo_K[l];
    s.off = A.eo_off[l];
    s.head = A.heads + (size_t)l * A.m;
    s.etap = A.eo_etap + (size_t)l * A.kmax;
    s.etaoff = A.eo_etaoff + (size_t)l * (A.kmax + 1);
    return s;
}

// exclusive prefix of in[0, n) into out[0, n], out[n] = total (all threads of the block)
__device__ void block_scan(const int *in, int *out, int n, int *tmp) {
    const int tid = threadIdx.x, per = (n + kPgThreads - 1) / kPgThreads;
    const int b = min(n, tid * per), e = min(n, b + per);
    int s = 0;
    for (int i = b; i < e; ++i) s += in[i];
    tmp[tid] = s;
    __syncthreads();
    for (int o = 1; o < kPgThreads; o <<= 1) {
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
    if (tid == kPgThreads - 1) out[n] = tmp[kPgThreads - 1];
    __syncthreads();
}

__device__ inline bool keep_entry(const unsigned char *touched, int i, double v, double drop) {
    return touched[i] ? fabs(v) > drop : v != 0.0;
}

__device__ inline unsigned long long lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

}  // namespace

int pg_tile_width(int m) {
    for (int W = 32; W >= 8; W >>= 1)
        if ((size_t)m * W * sizeof(double) <= kPgTileBytes) return W;
    return 0;
}

// ---- 1. dense composition ------------------------------------------------------------
__global__ __launch_bounds__(kPgThreads) void pg_dense_kernel(PgArgs A) {
    extern __shared__ double tile[];   // m x W, row-major
    __shared__ double red[kPgThreads / 64];
    const int a = A.a0 + blockIdx.x, m = A.m, W = A.W, tid = threadIdx.x;
    const Src S = src_of(A, a);
    if (S.K < 0 || S.K > A.kmax || S.pb < 0 || S.pb >= A.npool_old) {   // eta file did not fit: unusable
        if (tid == 0) A.amax[a] = -1.0;
        return;
    }
    double *D = A.D + (size_t)blockIdx.x * m * m;
    const int *cp = A.bcp0 + (size_t)S.pb * (A.MP + 1);
    const int G = kPgThreads / W, jj = tid % W, g = tid / W;   // G groups of W columns
    double amax = 0.0;
    for (int cb = 0; cb < m; cb += W) {
        const int wc = min(W, m - cb);
        for (int idx = tid; idx < m * W; idx += kPgThreads) tile[idx] = 0.0;
        __syncthreads();
        if (jj < wc)
            for (int q = cp[cb + jj] + g; q < cp[cb + jj + 1]; q += G) {
                const double v = A.bcv0[q];
                tile[A.bci0[q] * W + jj] = v;
                amax = fmax(amax, fabs(v));
            }
        __syncthreads();
        for (int t = 0; t < S.K; ++t) {
            const int r = S.etap[t];
            const double rr = tile[r * W + jj];   // the old row r, before this eta
            __syncthreads();
            const int e1 = S.etaoff[t + 1];
            for (int e = S.etaoff[t] + g; e < e1; e += G) {   // distinct rows within one eta
                const int i = A.eo_eidx[S.off + e];
                const double v = A.eo_evals[S.off + e];
                double &x = tile[i * W + jj];
                x = i == r ? v * rr : fma(v, rr, x);
            }
            __syncthreads();
        }
        for (int idx = tid; idx < m * W; idx += kPgThreads) {
            const int i = idx / W, j = idx - (idx / W) * W;
            if (j < wc) {
                const double v = tile[idx];
                D[(size_t)i * m + cb + j] = v;
                amax = fmax(amax, fabs(v));
            }
        }
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
    if ((tid & 63) == 0) red[tid >> 6] = amax;
    __syncthreads();
    if (tid == 0) {
        double v = red[0];
        for (int w = 1; w < kPgThreads / 64; ++w) v = fmax(v, red[w]);
        A.amax[a] = v;
    }
}

// ---- 2. counts, pi0, checks ------------------------------------------------------------
__global__ __launch_bounds__(kPgThreads) void pg_count_kernel(PgArgs A) {
    extern __shared__ double smem[];
    __shared__ int s_tot[4], s_bad;
    const int a = A.a0 + blockIdx.x, m = A.m, n = A.n, k = A.k, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const double amax = A.amax[a];
    if (!(amax >= 0.0)) {
        if (tid < 4) A.tot[(size_t)a * 4 + tid] = 0;
        if (tid == 0) A.valid[a] = 0;
        return;
    }
    const Src S = src_of(A, a);
    double *pi0 = smem, *cbv = smem + m;
    int *erow = reinterpret_cast<int *>(cbv + m);
    unsigned char *touched = reinterpret_cast<unsigned char *>(erow + m), *isb = touched + m;
    if (tid < 4) s_tot[tid] = 0;
    if (tid == 0) s_bad = 0;
    for (int i = tid; i < m; i += kPgThreads) touched[i] = 0;
    for (int j = tid; j < n + m; j += kPgThreads) isb[j] = 0;
    __syncthreads();
    const int ne = S.K > 0 ? S.etaoff[S.K] : 0;
    for (int e = tid; e < ne; e += kPgThreads) touched[A.eo_eidx[S.off + e]] = 1;
    for (int i = tid; i < m; i += kPgThreads) {
        const int j = S.head[i];
        isb[j] = 1;
        cbv[i] = j < n ? A.q[j] : 0.0;
    }
    __syncthreads();
    const double drop = 1e-14 * amax;
    const double *D = A.D + (size_t)blockIdx.x * m * m;
    // rows (one wave per row): B^{-1} entries and element entries
    for (int i = wv; i < m; i += kPgThreads / 64) {
        int cnt = 0, ec = 0;
        for (int c0 = 0; c0 < m; c0 += 64) {
            const int c = c0 + lane;
            const bool kk = c < m && keep_entry(touched, i, D[(size_t)i * m + c], drop);
            cnt += __popcll(__ballot(kk));
        }
        for (int e0 = 0; e0 < k; e0 += 64) {
            const int e = e0 + lane;
            const bool kk = e < k && keep_entry(touched, i, D[(size_t)i * m + A.pos_row[e]], drop);
            ec += __popcll(__ballot(kk));
        }
        if (lane == 0) {
            A.rowcnt[(size_t)a * m + i] = cnt;
            A.erowcnt[(size_t)a * m + i] = ec;
            erow[i] = ec;
            atomicAdd(&s_tot[0], cnt);
            atomicAdd(&s_tot[1], ec);
        }
    }
    // columns (one thread per column): counts and pi0 = c_B' B^{-1} over the kept entries
    for (int c = tid; c < m; c += kPgThreads) {
        int cnt = 0;
        double pi = 0.0;
        for (int i = 0; i < m; ++i) {
            const double v = D[(size_t)i * m + c];
            if (keep_entry(touched, i, v, drop)) {
                ++cnt;
                pi += cbv[i] * v;
            }
        }
        A.colcnt[(size_t)a * m + c] = cnt;
        pi0[c] = pi;
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
    // B^{-1} a_{head[i0]} = e_{i0} at the probes of sparse_basis_residual (1e-8)
    for (int probe = 0; probe < 4; ++probe) {
        const int i0 = (int)(((long long)probe * 7919 + 13) % m), j = S.head[i0];
        for (int i = tid; i < m; i += kPgThreads) {
            double v = 0.0;
            if (j >= n) {
                const double d = D[(size_t)i * m + (j - n)];
                if (keep_entry(touched, i, d, drop)) v = d;
            } else {
                for (int q = A.colptr[j]; q < A.colptr[j + 1]; ++q) {
                    const double d = D[(size_t)i * m + A.rowidx[q]];
                    if (keep_entry(touched, i, d, drop)) v += d * A.val[q];
                }
            }
            if (!(fabs(v - (i == i0 ? 1.0 : 0.0)) <= 1e-8)) bad = 1;
        }
    }
    if (bad) atomicOr(&s_bad, 1);
    // ELL entry rows (sum over slots of the widest row) and selection records (every row
    // active; rows of fixed basics twice), as prepare_elements
    if (tid < A.R9) {
        int w = 0;
        for (int l = 0; l < 64 && 64 * tid + l < m; ++l) w = max(w, erow[64 * tid + l]);
        atomicAdd(&s_tot[2], w);
    }
    for (int i = tid; i < m; i += kPgThreads)
        atomicAdd(&s_tot[3], (1 + erow[i]) * (A.btype[S.head[i]] == BT_E ? 2 : 1));
    __syncthreads();
    if (tid < 4) A.tot[(size_t)a * 4 + tid] = s_tot[tid];
    if (tid == 0) A.valid[a] = s_bad ? 0 : 1;
}

// ---- 3. pool-strided outputs ------------------------------------------------------------
__global__ __launch_bounds__(kPgThreads) void pg_fill_kernel(PgArgs A, PgFill F) {
    extern __shared__ double smem[];
    __shared__ int tmp[kPgThreads];
    __shared__ uint64_t bits[64];
    __shared__ int ws[65];   // ELL slot widths, then slot offsets
    const int p = F.P0 + blockIdx.x, a = F.map[p];
    const int m = A.m, n = A.n, k = A.k, MP = A.MP, R9 = A.R9, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const Src S = src_of(A, a);
    const double drop = 1e-14 * A.amax[a];
    const double *D = A.D + (size_t)(a - A.a0) * m * m;
    double *pi0 = smem, *cbv = smem + m;
    int *rs = reinterpret_cast<int *>(cbv + m), *cs = rs + (m + 1), *es = cs + (m + 1);
    unsigned char *touched = reinterpret_cast<unsigned char *>(es + (m + 1)), *isb = touched + m;
    for (int i = tid; i < m; i += kPgThreads) touched[i] = 0;
    for (int j = tid; j < n + m; j += kPgThreads) isb[j] = 0;
    if (tid < 64) bits[tid] = 0;
    __syncthreads();
    const int ne = S.K > 0 ? S.etaoff[S.K] : 0;
    for (int e = tid; e < ne; e += kPgThreads) touched[A.eo_eidx[S.off + e]] = 1;
    for (int i = tid; i < m; i += kPgThreads) {
        const int j = S.head[i];
        isb[j] = 1;
        cbv[i] = j < n ? A.q[j] : 0.0;
        atomicOr(reinterpret_cast<unsigned long long *>(&bits[j & 63]), 1ull << (j >> 6));
    }
    block_scan(A.rowcnt + (size_t)a * m, rs, m, tmp);
    block_scan(A.colcnt + (size_t)a * m, cs, m, tmp);
    block_scan(A.erowcnt + (size_t)a * m, es, m, tmp);
    const int nb = F.off[(size_t)p * 4 + 0], eb = F.off[(size_t)p * 4 + 1];
    // B^{-1} rows (CSR, columns ascending) and element rows (CSR, e ascending): one wave a row
    for (int i = wv; i < m; i += kPgThreads / 64) {
        int run = 0;
        for (int c0 = 0; c0 < m; c0 += 64) {
            const int c = c0 + lane;
            const double v = c < m ? D[(size_t)i * m + c] : 0.0;
            const bool kk = c < m && keep_entry(touched, i, v, drop);
            const unsigned long long msk = __ballot(kk);
            if (kk) {
                const int at = nb + rs[i] + run + __popcll(msk & lanemask_lt(lane));
                F.brcol[at] = c;
                F.brval[at] = v;
            }
            run += __popcll(msk);
        }
        run = 0;
        for (int e0 = 0; e0 < k; e0 += 64) {
            const int e = e0 + lane;
            const double v = e < k ? D[(size_t)i * m + A.pos_row[e]] : 0.0;
            const bool kk = e < k && keep_entry(touched, i, v, drop);
            const unsigned long long msk = __ballot(kk);
            if (kk) {
                const int at = eb + es[i] + run + __popcll(msk & lanemask_lt(lane));
                F.ke[at] = e;
                F.kraw[at] = v;
            }
            run += __popcll(msk);
        }
    }
    for (int i = tid; i <= MP; i += kPgThreads) {
        F.brptr[(size_t)p * (MP + 1) + i] = nb + rs[min(i, m)];
        F.bcp[(size_t)p * (MP + 1) + i] = nb + cs[min(i, m)];
    }
    for (int i = tid; i <= m; i += kPgThreads) F.kp[(size_t)p * (m + 1) + i] = eb + es[i];
    // B^{-1} columns (CSC, rows ascending) and pi0: one thread a column
    for (int c = tid; c < m; c += kPgThreads) {
        const int base = nb + cs[c];
        int cnt = 0;
        double pi = 0.0;
        for (int i = 0; i < m; ++i) {
            const double v = D[(size_t)i * m + c];
            if (keep_entry(touched, i, v, drop)) {
                F.bci[base + cnt] = i;
                F.bcv[base + cnt] = v;
                ++cnt;
                pi += cbv[i] * v;
            }
        }
        pi0[c] = pi;
    }
    // sliced ELL of the element rows: slot t = rows [64t, 64t + 64), width = widest row
    if (tid < R9) {
        int w = 0;
        for (int l = 0; l < 64 && 64 * tid + l < m; ++l) w = max(w, es[64 * tid + l + 1] - es[64 * tid + l]);
        ws[tid] = w;
    }
    __syncthreads();
    if (tid == 0) {
        int o = F.off[(size_t)p * 4 + 2];
        for (int t = 0; t < R9; ++t) {
            const int w = ws[t];
            ws[t] = o;
            F.kslot[(size_t)p * (R9 + 1) + t] = o;
            o += w;
        }
        ws[R9] = o;
        F.kslot[(size_t)p * (R9 + 1) + R9] = o;
    }
    __syncthreads();
    for (int i = tid; i < 64 * R9; i += kPgThreads) {
        const int t = i >> 6, l = i & 63, r0 = ws[t], w = ws[t + 1] - ws[t];
        int j = 0;
        if (i < m)
            for (int e = 0; e < k; ++e) {
                const double v = D[(size_t)i * m + A.pos_row[e]];
                if (keep_entry(touched, i, v, drop)) {
                    F.kix[(size_t)(r0 + j) * 64 + l] = e;
                    F.kv[(size_t)(r0 + j) * 64 + l] = v;
                    ++j;
                }
            }
        for (; j < w; ++j) {
            F.kix[(size_t)(r0 + j) * 64 + l] = 0;
            F.kv[(size_t)(r0 + j) * 64 + l] = 0.0;
        }
    }
    // basis words
    for (int i = tid; i < MP; i += kPgThreads)
        F.hb0[(size_t)p * MP + i] = i < m ? S.head[i] * 4 + A.btype[S.head[i]] : -1;
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

static size_t count_lds(const PgArgs &A) {
    return sizeof(double) * 2 * A.m + sizeof(int) * A.m + A.m + (A.n + A.m) + 16;
}
static size_t fill_lds(const PgArgs &A) {
    return sizeof(double) * 2 * A.m + sizeof(int) * 3 * (A.m + 1) + A.m + (A.n + A.m) + 16;
}

hipError_t pg_launch_dense(const PgArgs &A, int nb, hipStream_t s) {
    const size_t lds = (size_t)A.m * A.W * sizeof(double);
    hipError_t e = hipFuncSetAttribute((const void *)pg_dense_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pg_dense_kernel, dim3(nb), dim3(kPgThreads), lds, s, A);
    return hipGetLastError();
}
hipError_t pg_launch_count(const PgArgs &A, int nb, hipStream_t s) {
    const size_t lds = count_lds(A);
    hipError_t e = hipFuncSetAttribute((const void *)pg_count_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pg_count_kernel, dim3(nb), dim3(kPgThreads), lds, s, A);
    return hipGetLastError();
}
hipError_t pg_launch_fill(const PgArgs &A, const PgFill &F, int np, hipStream_t s) {
    const size_t lds = fill_lds(A);
    hipError_t e = hipFuncSetAttribute((const void *)pg_fill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pg_fill_kernel, dim3(np), dim3(kPgThreads), lds, s, A, F);
    return hipGetLastError();
}

}  // namespace twosd
