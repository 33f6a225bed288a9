// sampler.hip -- on-device scenario sampling: rand(rng, sto) of
// src/smps/smps_sto.jl:117-149, i.i.d. per element, straight into an epigraph's delta
// array in HBM (no host round trip).
//
// Element e of global scenario index g draws from Philox4x32-10 with counter
// (g_lo, g_hi, e, 0) and key (seed_lo, seed_hi) -> (x0, x1, x2, x3); u1 = u01(x0, x1),
// u2 = u01(x2, x3).  Transforms (Distributions 0.25.102 as called by the reference):
//   DISCRETE  DiscreteNonParametric(values, probs): support sorted ascending; i = 1,
//             cp = p_1; while cp <= u1 && i < n: cp += p_{++i}; value = x_i
//   NORMAL    Normal(mean, sqrt(variance)): mean + sd * z, z = sqrt(-2 log(1 - u1)) cos(2 pi u2)
//             (Box-Muller; Julia's randn is a ziggurat -- same distribution, other stream)
//   UNIFORM   Uniform(left, right): left + (right - left) * u1 (two roundings, no fma)
// The stream is a function of (seed, global index, element) only, so any sharding of the
// scenarios over ranks reproduces the same scenarios.
#include <hip/hip_runtime.h>
#include <math.h>
#include "twosd_internal.h"
#include "philox.h"

namespace twosd {

__global__ void __launch_bounds__(256) sample_kernel(SampleParams S) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)S.N * S.k;
    if (idx >= total) return;
    const int s = (int)(idx / S.k), e = (int)(idx - (long long)s * S.k);
    const unsigned long long g = S.first_index + (unsigned long long)s;
    const Philox4 r = philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), (uint32_t)e, 0u, (uint32_t)S.seed,
                                    (uint32_t)(S.seed >> 32));
    const double u1 = u01(r.v[0], r.v[1]);
    const int kind = S.kind[e];
    double v;
    if (kind == 0) {   // DISCRETE
        const int o = S.off[e], n = S.off[e + 1] - o;
        int i = 0;
        double cp = S.prob[o];
        while (cp <= u1 && i < n - 1) cp = __dadd_rn(cp, S.prob[o + (++i)]);
        v = S.val[o + i];
    } else if (kind == 1) {   // NORMAL
        const double u2 = u01(r.v[2], r.v[3]);
        const double z = sqrt(-2.0 * log(1.0 - u1)) * cos(6.283185307179586 * u2);
        v = __dadd_rn(S.p0[e], __dmul_rn(S.p1[e], z));
    } else {   // UNIFORM
        v = __dadd_rn(S.p0[e], __dmul_rn(__dadd_rn(S.p1[e], -S.p0[e]), u1));
    }
    S.out[idx] = __dadd_rn(v, -S.tmpl[e]);   // stored as the delta (value - template value)
}

hipError_t launch_sample(const SampleParams &S, hipStream_t st) {
    const long long total = (long long)S.N * S.k;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(sample_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, S);
    return hipGetLastError();
}

}  // namespace twosd
