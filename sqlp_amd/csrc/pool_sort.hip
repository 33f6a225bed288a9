// pool_sort.hip -- order the scenarios of an LP batch by their warm-start pool basis.
//
// The LP kernel takes scenarios from an atomic work queue in queue order; visiting them
// grouped by pool basis keeps the waves that run at the same time on a few bases, so the
// B^{-1} data of those bases stays in L2 instead of every wave missing to the MALL on a
// different basis.  Stable radix sort of (pool, scenario) on the pool's bits.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include "twosd_internal.h"

namespace twosd {

__global__ void iota_kernel(int *v, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

// tmp == nullptr: *tmp_bytes receives the workspace size (keys_out, vals_in live in it too)
hipError_t sort_by_pool(const int *pick, int *order, int N, int npool, void *tmp, size_t *tmp_bytes, hipStream_t s) {
    int bits = 1;
    while ((1 << bits) < npool) ++bits;
    const size_t aux = 2 * sizeof(int) * (size_t)((N + 63) & ~63);
    size_t cub = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (const int *)nullptr, (int *)nullptr,
                                                      (const int *)nullptr, (int *)nullptr, N, 0, bits, s);
    if (e != hipSuccess) return e;
    if (!tmp) {
        *tmp_bytes = aux + cub + 256;
        return hipSuccess;
    }
    int *keys_out = reinterpret_cast<int *>(tmp);
    int *vals_in = keys_out + ((N + 63) & ~63);
    void *ctmp = reinterpret_cast<char *>(tmp) + aux;
    hipLaunchKernelGGL(iota_kernel, dim3((N + 255) / 256), dim3(256), 0, s, vals_in, N);
    return hipcub::DeviceRadixSort::SortPairs(ctmp, cub, pick, keys_out, vals_in, order, N, 0, bits, s);
}

}  // namespace twosd
