// Peak probes on gfx950 (MI355X): the measured ceilings the roofline fractions are stated
// against, next to the datasheet peaks (78.6 TF fp64, 8 TB/s HBM).
//   * fp64 MFMA (v_mfma_f64_16x16x4f64): back-to-back MFMAs, NACC independent accumulators per
//     wave, 1/2/4 waves per SIMD, operands varying per iteration (no constant-data clock bonus);
//   * fp64 VALU FMA (v_fma_f64): 8 / 16 independent chains per lane;
//   * MFMA + VALU together: in every block half the waves run the MFMA loop and half the VALU
//     loop -- if the fp64 matrix and vector work share one pipe, the pair takes the sum of the
//     standalone times; if not, the max;
//   * HBM copy (STREAM-like, 2 x 2 GiB read+write, 16-byte accesses, 4 in flight per lane).
// Output: one JSON object per line.  Build:
//   hipcc -O3 --offload-arch=gfx950 -Wno-unused-result tools/mfma_f64_probe.hip -o tools/mfma_f64_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__device__ __forceinline__ double mfma_loop(int iters, double a, double b) {
    d4 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
    double av = a + threadIdx.x * 1e-9, bv = b - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[i], 0, 0, 0);
        av = av * 0.999999 + 1e-7;   // operands change every iteration (one VALU op per NACC MFMAs)
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    return s;
}

template <int NCH>
__device__ __forceinline__ double fma_loop(int iters, double a, double b) {
    double x[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) x[i] = a + (threadIdx.x + i) * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) x[i] = fma(x[i], b, a);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NCH; ++i) s += x[i];
    return s;
}

template <int NACC>
__global__ void __launch_bounds__(256) probe_mfma(double *out, int iters, double a, double b) {
    const double s = mfma_loop<NACC>(iters, a, b);
    if (s == 12345.678) out[threadIdx.x] = s;   // keeps the work alive
}

template <int NCH>
__global__ void __launch_bounds__(256) probe_fma(double *out, int iters, double a, double b) {
    const double s = fma_loop<NCH>(iters, a, b);
    if (s == 12345.678) out[threadIdx.x] = s;
}

// 8 waves per block, placed round-robin on the CU's 4 SIMDs: waves 0-3 run the MFMA loop (mi
// iterations), waves 4-7 the VALU loop (vi iterations), so every SIMD holds one of each
__global__ void __launch_bounds__(512) probe_mixed(double *out, int mi, int vi, double a, double b) {
    const int wid = threadIdx.x >> 6;
    const double s = (wid >= 4) ? fma_loop<16>(vi, a, b) : mfma_loop<4>(mi, a, b);
    if (s == 12345.678) out[threadIdx.x] = s;
}

typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) copy_kernel(const dv2 *__restrict__ src, dv2 *__restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        dv2 v0 = __builtin_nontemporal_load(src + i), v1 = __builtin_nontemporal_load(src + i + stride);
        dv2 v2 = __builtin_nontemporal_load(src + i + 2 * stride), v3 = __builtin_nontemporal_load(src + i + 3 * stride);
        __builtin_nontemporal_store(v0, dst + i);
        __builtin_nontemporal_store(v1, dst + i + stride);
        __builtin_nontemporal_store(v2, dst + i + 2 * stride);
        __builtin_nontemporal_store(v3, dst + i + 3 * stride);
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

template <typename F>
static float time_ms(F launch, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    launch();
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0); hipEventDestroy(e1);
    return ms / reps;
}

template <int NACC>
static double run_mfma(int cus, int wps, double *out, int iters) {
    const int blocks = cus * wps;
    const float ms = time_ms([&] { probe_mfma<NACC><<<blocks, 256>>>(out, iters, 1.0, 1.0); }, 3);
    const double fl = 2.0 * 16 * 16 * 4 * (double)NACC * iters * (blocks * 4.0);
    const double tf = fl / (ms * 1e-3) / 1e12;
    printf("{\"probe\": \"mfma_f64_16x16x4f64\", \"nacc\": %d, \"waves_per_simd\": %d, \"tflops\": %.2f, \"ms\": %.3f}\n",
           NACC, wps, tf, ms);
    return tf;
}

template <int NCH>
static double run_fma(int cus, int wps, double *out, int iters) {
    const int blocks = cus * wps;
    const float ms = time_ms([&] { probe_fma<NCH><<<blocks, 256>>>(out, iters, 1e-3, 0.999); }, 3);
    const double fl = 2.0 * NCH * (double)iters * (blocks * 256.0);
    const double tf = fl / (ms * 1e-3) / 1e12;
    printf("{\"probe\": \"v_fma_f64\", \"chains\": %d, \"waves_per_simd\": %d, \"tflops\": %.2f, \"ms\": %.3f}\n", NCH, wps,
           tf, ms);
    return tf;
}

int main() {
    hipDeviceProp_t pr;
    hipGetDeviceProperties(&pr, 0);
    const int cus = pr.multiProcessorCount;
    double *out;
    hipMalloc(&out, 4096);
    const int it = 20000;
    run_mfma<2>(cus, 1, out, it); run_mfma<4>(cus, 1, out, it); run_mfma<8>(cus, 1, out, it);
    run_mfma<2>(cus, 2, out, it); run_mfma<4>(cus, 2, out, it); run_mfma<8>(cus, 2, out, it);
    run_mfma<4>(cus, 4, out, it);
    for (int wps : {2, 4, 8}) run_fma<8>(cus, wps, out, it);
    run_fma<16>(cus, 2, out, it); run_fma<16>(cus, 4, out, it);
    // mixed: one 512-thread block per CU = one MFMA wave + one VALU wave on every SIMD
    {
        const int blocks = cus;
        const int mi = it, vi = 4 * it;
        const float t_m = time_ms([&] { probe_mixed<<<blocks, 512>>>(out, mi, 0, 1.0, 1.0); }, 3);
        const float t_v = time_ms([&] { probe_mixed<<<blocks, 512>>>(out, 0, vi, 1.0, 1.0); }, 3);
        const float t_b = time_ms([&] { probe_mixed<<<blocks, 512>>>(out, mi, vi, 1.0, 1.0); }, 3);
        const double fm = 2.0 * 16 * 16 * 4 * 4.0 * mi * (blocks * 4.0);
        const double fv = 2.0 * 16 * (double)vi * (blocks * 256.0);
        printf("{\"probe\": \"mixed_mfma_valu_f64\", \"ms_mfma_only\": %.3f, \"ms_valu_only\": %.3f, \"ms_both\": %.3f, "
               "\"tflops_mfma_only\": %.2f, \"tflops_valu_only\": %.2f, \"tflops_both\": %.2f}\n",
               t_m, t_v, t_b, fm / (t_m * 1e-3) / 1e12, fv / (t_v * 1e-3) / 1e12, (fm + fv) / (t_b * 1e-3) / 1e12);
    }
    const size_t n = (size_t)2 << 30 >> 4;   // 2 GiB of double2
    dv2 *s, *d;
    hipMalloc(&s, n * 16); hipMalloc(&d, n * 16);
    hipMemset(s, 0, n * 16); hipMemset(d, 0, n * 16);
    for (int bpc : {4, 8, 16}) {
        const int blocks = cus * bpc;
        const float ms = time_ms([&] { copy_kernel<<<blocks, 256>>>(s, d, n); }, 10);
        printf("{\"probe\": \"hbm_copy\", \"blocks_per_cu\": %d, \"bytes\": %zu, \"gbs\": %.1f}\n", bpc, 2 * n * 16,
               2.0 * n * 16 / (ms * 1e-3) / 1e9);
    }
    hipFree(s); hipFree(d); hipFree(out);
    return 0;
}
