// dvs_keys.h -- the reference dedup key of a dual vector (src/sd_algorithm/dual_set.jl),
// shared by the vertex-set kernels and the LP kernel epilogue (which keys its own duals).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace twosd {

__device__ __forceinline__ double round16(double x) {
    // Julia round(x; base=2, sigdigits=16): non-finite -> x; 0 -> x;
    // digits = 16 - (1 + exponent(x)); scale by an exact power of two, ties to even.
    if (!isfinite(x) || x == 0.0) return x;
    int e2;
    frexp(x, &e2);                    // x = f * 2^e2, 0.5 <= |f| < 1 -> exponent(x) = e2 - 1
    const int digits = 16 - e2;
    double r;
    if (digits >= 0) {
        const double sc = ldexp(1.0, digits);
        r = rint(x * sc) / sc;
    } else {
        const double isc = ldexp(1.0, -digits);
        r = rint(x / isc) * isc;
    }
    return isfinite(r) ? r : x;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// key component bits: round16 with -0.0 folded onto +0.0 (Julia: -0.0 != 0.0 is false)
__device__ __forceinline__ uint64_t comp_bits(double x) {
    double r = round16(x);
    if (r == 0.0) r = 0.0;
    return (uint64_t)__double_as_longlong(r);
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, o);
    return v;
}

}  // namespace twosd
