// Peak probes on gfx950 (MI355X), used to state measured roofline peaks next to the spec:
//   * fp64 MFMA (v_mfma_f64_16x16x4f64): back-to-back MFMAs, NACC independent accumulators
//     per wave, 1/2/4 waves per SIMD;
//   * fp64 VALU FMA (v_fma_f64): 8 independent chains per lane;
//   * HBM copy (STREAM-like, 2 x 2 GiB read+write, 16-byte loads).
// Build: hipcc -O3 --offload-arch=gfx950 -Wno-unused-result tools/mfma_f64_probe.hip -o tools/mfma_f64_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void __launch_bounds__(256) probe_mfma(double *out, int iters, double a, double b) {
    d4 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
    double av = a + threadIdx.x * 1e-9, bv = b - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.678) out[threadIdx.x] = s;   // keeps the work alive
}

__global__ void __launch_bounds__(256) probe_fma(double *out, int iters, double a, double b) {
    double x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = a + (threadIdx.x + i) * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = fma(x[i], b, a);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    if (s == 12345.678) out[threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) copy_kernel(const double2 *__restrict__ src, double2 *__restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

static float time_ms(void (*launch)(void *), void *arg, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    launch(arg);
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch(arg);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

struct MArg { double *out; int blocks, iters; };
template <int NACC>
static void lm(void *p) { MArg *a = (MArg *)p; probe_mfma<NACC><<<a->blocks, 256>>>(a->out, a->iters, 1.0, 1.0); }
static void lf(void *p) { MArg *a = (MArg *)p; probe_fma<<<a->blocks, 256>>>(a->out, a->iters, 1e-3, 0.999); }
struct CArg { double2 *s, *d; size_t n; int blocks; };
static void lc(void *p) { CArg *a = (CArg *)p; copy_kernel<<<a->blocks, 256>>>(a->s, a->d, a->n); }

template <int NACC>
static void run_mfma(int cus, int wps, double *out) {
    MArg a{out, cus * wps, 20000};
    const float ms = time_ms(lm<NACC>, &a, 3);
    const double fl = 2.0 * 16 * 16 * 4 * (double)NACC * a.iters * (a.blocks * 4.0);
    printf("{\"probe\": \"mfma_f64_16x16x4f64\", \"nacc\": %d, \"waves_per_simd\": %d, \"tflops\": %.2f}\n", NACC, wps,
           fl / (ms * 1e-3) / 1e12);
}

int main() {
    hipDeviceProp_t pr;
    hipGetDeviceProperties(&pr, 0);
    const int cus = pr.multiProcessorCount;
    double *out;
    hipMalloc(&out, 4096);
    run_mfma<2>(cus, 1, out); run_mfma<4>(cus, 1, out);
    run_mfma<2>(cus, 2, out); run_mfma<4>(cus, 2, out); run_mfma<8>(cus, 2, out);
    run_mfma<2>(cus, 4, out); run_mfma<4>(cus, 4, out);
    for (int wps : {2, 4, 8}) {
        MArg a{out, cus * wps, 20000};
        const float ms = time_ms(lf, &a, 3);
        const double fl = 2.0 * 8 * a.iters * (a.blocks * 256.0);
        printf("{\"probe\": \"v_fma_f64\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", wps, fl / (ms * 1e-3) / 1e12);
    }
    const size_t n = (size_t)2 << 30 >> 4;   // 2 GiB of double2
    double2 *s, *d;
    hipMalloc(&s, n * 16); hipMalloc(&d, n * 16);
    hipMemset(s, 0, n * 16); hipMemset(d, 0, n * 16);
    CArg c{s, d, n, cus * 8};
    const float ms = time_ms(lc, &c, 10);
    printf("{\"probe\": \"hbm_copy\", \"bytes\": %zu, \"gbs\": %.1f}\n", 2 * n * 16, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
    hipFree(s); hipFree(d); hipFree(out);
    return 0;
}
