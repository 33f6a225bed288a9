// vkey.hip -- first occurrence of every optimal dual vertex of an LP batch (solve_push).
//
// push!(V, pi_s) for s = 0..N-1 in order (dual_set.jl:84-94, driven by algorithm.jl:46-54)
// only ever appends the first scenario's dual of each distinct vertex: a later scenario at the
// same vertex pushes an equal vector.  The LP kernel therefore emits, per scenario, a key of
// its optimal dual (its maintained slack reduced costs at 24 significant bits, lp_hyper.hip)
// instead of pi;
// here the lowest scenario index per key is found (open addressing, CAS on the key + atomicMin
// on the scenario), and the representatives, ascending, are listed for the re-solve that
// recovers their pi.  Pushing those pi in that order is the reference's sequence of pushes
// with the no-op pushes left out.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include "twosd_ctx.h"

namespace twosd {

#define HIPCHK(expr)                                                                               \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) return fail(TWOSD_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

__device__ __forceinline__ unsigned long long vk_norm(unsigned long long k) { return k ? k : 1ull; }   // 0 = empty slot
__device__ __forceinline__ unsigned vk_slot(unsigned long long k, unsigned mask) {
    return (unsigned)((k * 0x9E3779B97F4A7C15ull) >> 32) & mask;
}

__global__ void vkey_clear_kernel(unsigned long long *keys, int *first, int *cnt, unsigned cap) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += gridDim.x * blockDim.x) {
        keys[i] = 0ull;
        first[i] = 0x7fffffff;
        cnt[i] = 0;
    }
}

// Scenarios in blocks of kVkItems: a block first merges its scenarios' keys in an LDS table of
// twice as many slots (never full: load <= 1/2; LDS atomics), then inserts each distinct key once
// into the global table with the block's lowest scenario and count.  Many scenarios share a vertex
// (storm 1M: ~3k distinct keys), so per-scenario global atomics would serialize on the hot slots.
// min and sum are order independent: the result equals per-scenario insertion.
constexpr int kVkItems = 2048;
constexpr int kVkLds = 2 * kVkItems;
__global__ void __launch_bounds__(256) vkey_insert_kernel(int N, const unsigned long long *__restrict__ vkey,
                                                          const int *__restrict__ status, unsigned long long *keys,
                                                          int *first, int *cnt, unsigned mask) {
    __shared__ unsigned long long lk[kVkLds];
    __shared__ int lf[kVkLds], lc[kVkLds];
    for (int i = threadIdx.x; i < kVkLds; i += blockDim.x) {
        lk[i] = 0ull;
        lf[i] = 0x7fffffff;
        lc[i] = 0;
    }
    __syncthreads();
    const int s0 = blockIdx.x * kVkItems, s1 = min(N, s0 + kVkItems);
    for (int s = s0 + threadIdx.x; s < s1; s += blockDim.x) {
        if (status[s] != TWOSD_LP_OPTIMAL) continue;
        const unsigned long long k = vk_norm(vkey[s]);
        unsigned i = vk_slot(k, kVkLds - 1);
        for (;;) {
            const unsigned long long old = atomicCAS(&lk[i], 0ull, k);
            if (old == 0ull || old == k) {
                atomicMin(&lf[i], s);
                atomicAdd(&lc[i], 1);
                break;
            }
            i = (i + 1) & (kVkLds - 1);
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < kVkLds; j += blockDim.x) {
        const unsigned long long k = lk[j];
        if (!k) continue;
        unsigned i = vk_slot(k, mask);
        for (;;) {
            const unsigned long long old = atomicCAS(&keys[i], 0ull, k);
            if (old == 0ull || old == k) {
                atomicMin(&first[i], lf[j]);
                atomicAdd(&cnt[i], lc[j]);
                break;
            }
            i = (i + 1) & mask;
        }
    }
}

// occurrences of the key of each representative (list[0, U))
__global__ void vkey_count_kernel(int U, const int *__restrict__ list, const unsigned long long *__restrict__ vkey,
                                  const unsigned long long *__restrict__ keys, const int *__restrict__ cnt, unsigned mask,
                                  int *out) {
    for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < U; a += gridDim.x * blockDim.x) {
        const unsigned long long k = vk_norm(vkey[list[a]]);
        unsigned i = vk_slot(k, mask);
        while (keys[i] != k) i = (i + 1) & mask;
        out[a] = cnt[i];
    }
}

__global__ void vkey_flag_kernel(int N, const unsigned long long *__restrict__ vkey, const int *__restrict__ status,
                                 const unsigned long long *__restrict__ keys, const int *__restrict__ first,
                                 unsigned mask, char *flag) {
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < N; s += gridDim.x * blockDim.x) {
        char f = 0;
        if (status[s] == TWOSD_LP_OPTIMAL) {
            const unsigned long long k = vk_norm(vkey[s]);
            unsigned i = vk_slot(k, mask);
            while (keys[i] != k) i = (i + 1) & mask;
            f = first[i] == s;
        }
        flag[s] = f;
    }
}

struct VkeyWs {
    unsigned long long *keys = nullptr;
    int *first = nullptr, *cnt = nullptr, *counts = nullptr;
    unsigned cap = 0;
    char *flag = nullptr;
    int *list = nullptr, *nsel = nullptr;
    size_t ncap = 0;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
};

static VkeyWs *vws(twosd_ctx *c) {
    if (!c->vkey_ws) c->vkey_ws = new VkeyWs();
    return static_cast<VkeyWs *>(c->vkey_ws);
}

void vkey_free(twosd_ctx *c) {
    VkeyWs *w = static_cast<VkeyWs *>(c->vkey_ws);
    if (!w) return;
    hipFree(w->keys); hipFree(w->first); hipFree(w->cnt); hipFree(w->counts); hipFree(w->flag); hipFree(w->list);
    hipFree(w->nsel); hipFree(w->tmp);
    delete w;
    c->vkey_ws = nullptr;
}

// representatives (first scenario of every distinct key among the optimal scenarios of
// [0, N)), ascending, into *d_list; their number into *U (host); d_counts (nullable): the
// number of scenarios with each representative's key, into *d_counts
int vkey_first_occurrences(twosd_ctx *c, int N, const unsigned long long *d_vkey, const int *d_status, const int **d_list,
                           int *U, const int **d_counts) {
    VkeyWs *w = vws(c);
    unsigned cap = 1024;
    while (cap < 2u * (unsigned)N) cap <<= 1;
    if (cap > w->cap) {
        hipFree(w->keys); hipFree(w->first); hipFree(w->cnt);
        w->keys = nullptr; w->first = nullptr; w->cnt = nullptr; w->cap = 0;
        HIPCHK(hipMalloc(&w->keys, sizeof(unsigned long long) * cap));
        HIPCHK(hipMalloc(&w->first, sizeof(int) * cap));
        HIPCHK(hipMalloc(&w->cnt, sizeof(int) * cap));
        w->cap = cap;
    }
    if ((size_t)N > w->ncap) {
        hipFree(w->flag); hipFree(w->list); hipFree(w->counts);
        w->flag = nullptr; w->list = nullptr; w->counts = nullptr; w->ncap = 0;
        HIPCHK(hipMalloc(&w->flag, (size_t)N));
        HIPCHK(hipMalloc(&w->list, sizeof(int) * (size_t)N));
        HIPCHK(hipMalloc(&w->counts, sizeof(int) * (size_t)N));
        w->ncap = N;
    }
    if (!w->nsel) HIPCHK(hipMalloc(&w->nsel, sizeof(int)));
    size_t need = 0;
    HIPCHK(hipcub::DeviceSelect::Flagged(nullptr, need, hipcub::CountingInputIterator<int>(0), w->flag, w->list, w->nsel, N,
                                         c->stream));
    if (need > w->tmp_bytes) {
        hipFree(w->tmp);
        w->tmp = nullptr; w->tmp_bytes = 0;
        HIPCHK(hipMalloc(&w->tmp, need));
        w->tmp_bytes = need;
    }
    const unsigned mask = w->cap - 1;
    const int nb = std::max(1, std::min(4096, (N + 255) / 256));
    hipLaunchKernelGGL(vkey_clear_kernel, dim3(std::min(4096u, (w->cap + 255) / 256)), dim3(256), 0, c->stream, w->keys, w->first,
                       w->cnt, w->cap);
    hipLaunchKernelGGL(vkey_insert_kernel, dim3(std::max(1, (N + kVkItems - 1) / kVkItems)), dim3(256), 0, c->stream, N, d_vkey, d_status,
                       w->keys, w->first, w->cnt, mask);
    hipLaunchKernelGGL(vkey_flag_kernel, dim3(nb), dim3(256), 0, c->stream, N, d_vkey, d_status, w->keys, w->first, mask,
                       w->flag);
    HIPCHK(hipGetLastError());
    HIPCHK(hipcub::DeviceSelect::Flagged(w->tmp, need, hipcub::CountingInputIterator<int>(0), w->flag, w->list, w->nsel, N,
                                         c->stream));
    HIPCHK(hipMemcpyAsync(U, w->nsel, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *d_list = w->list;
    if (d_counts) {
        if (*U > 0) {
            hipLaunchKernelGGL(vkey_count_kernel, dim3(std::max(1, std::min(4096, (*U + 255) / 256))), dim3(256), 0, c->stream, *U,
                               w->list, d_vkey, w->keys, w->cnt, mask, w->counts);
            HIPCHK(hipGetLastError());
        }
        *d_counts = w->counts;
    }
    return TWOSD_OK;
}

}  // namespace twosd
