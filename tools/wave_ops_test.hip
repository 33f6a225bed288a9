// Standalone GPU check of sqlp_amd/csrc/wave_ops.h against a serial reference.
// Build: hipcc --offload-arch=gfx950 -O3 -I sqlp_amd/csrc tools/wave_ops_test.hip -o tools/wave_ops_test
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "wave_ops.h"

using namespace twosd;

__global__ void k(const double *x, const int *flag, double *out, int *iout) {
    const int lane = threadIdx.x;
    const double v = x[blockIdx.x * 64 + lane];
    const double s = wsum(v), mn = wmin(v), mx = wmax(v);
    const double key = flag[blockIdx.x * 64 + lane] ? v : -INFINITY;
    const int idx = flag[blockIdx.x * 64 + lane] ? (lane * 7) % 64 : 0x7fffffff;
    ArgBest b = warg_max(key, idx, v * 2.0, v * 3.0);
    // every lane must agree
    if (lane == 0) {
        out[blockIdx.x * 6 + 0] = s; out[blockIdx.x * 6 + 1] = mn; out[blockIdx.x * 6 + 2] = mx;
        out[blockIdx.x * 6 + 3] = b.key; out[blockIdx.x * 6 + 4] = b.p0; out[blockIdx.x * 6 + 5] = b.p1;
        iout[blockIdx.x] = b.idx;
    }
    const double s63 = __shfl(s, 63);
    if (s63 != s || __shfl(b.idx, 37) != b.idx) iout[blockIdx.x] = -999;
}

int main() {
    const int B = 512;
    double *hx = (double *)malloc(sizeof(double) * B * 64);
    int *hf = (int *)malloc(sizeof(int) * B * 64);
    srand(1);
    for (int i = 0; i < B * 64; ++i) {
        hx[i] = (rand() % 2000 - 1000) / 7.0;
        if ((i / 64) % 3 == 0) hx[i] = (double)(rand() % 5);   // many ties
        hf[i] = rand() % 4 != 0;
    }
    double *dx, *dout; int *df, *diout;
    hipMalloc(&dx, sizeof(double) * B * 64); hipMalloc(&df, sizeof(int) * B * 64);
    hipMalloc(&dout, sizeof(double) * B * 6); hipMalloc(&diout, sizeof(int) * B);
    hipMemcpy(dx, hx, sizeof(double) * B * 64, hipMemcpyHostToDevice);
    hipMemcpy(df, hf, sizeof(int) * B * 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(B), dim3(64), 0, 0, dx, df, dout, diout);
    double *ho = (double *)malloc(sizeof(double) * B * 6); int *hi = (int *)malloc(sizeof(int) * B);
    hipMemcpy(ho, dout, sizeof(double) * B * 6, hipMemcpyDeviceToHost);
    hipMemcpy(hi, diout, sizeof(int) * B, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int b = 0; b < B; ++b) {
        const double *x = hx + b * 64; const int *f = hf + b * 64;
        double s = 0, mn = INFINITY, mx = -INFINITY, bk = -INFINITY, bp0 = 0; int bi = 0x7fffffff;
        for (int l = 0; l < 64; ++l) { s += x[l]; mn = fmin(mn, x[l]); mx = fmax(mx, x[l]); }
        for (int l = 0; l < 64; ++l) {
            if (!f[l]) continue;
            const int idx = (l * 7) % 64;
            if (x[l] > bk || (x[l] == bk && idx < bi)) { bk = x[l]; bi = idx; bp0 = 2 * x[l]; }
        }
        if (fabs(ho[b * 6] - s) > 1e-9 * (1 + fabs(s)) || ho[b * 6 + 1] != mn || ho[b * 6 + 2] != mx || hi[b] != bi ||
            ho[b * 6 + 3] != bk || ho[b * 6 + 4] != bp0) {
            if (bad < 5) printf("block %d: sum %g/%g min %g/%g max %g/%g idx %d/%d key %g/%g\n", b, ho[b * 6], s, ho[b * 6 + 1], mn,
                                ho[b * 6 + 2], mx, hi[b], bi, ho[b * 6 + 3], bk);
            ++bad;
        }
    }
    printf("wave_ops_test: %d / %d blocks wrong\n", bad, B);
    return bad != 0;
}
