// philox.h -- Philox4x32-10 counter-based generator (Salmon, Moraes, Dror, Shaw, "Parallel
// random numbers: as easy as 1, 2, 3", SC'11) and the scenario-sampling transforms of
// rand(sto) (reference src/smps/smps_sto.jl:117-149 over Distributions 0.25.102).
// Header-only, host + device, so the oracle restatement and the kernel share nothing but
// the published algorithm (oracle/sampler.c restates it independently in C).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define TWOSD_HD __host__ __device__ __forceinline__
#else
#define TWOSD_HD static inline
#endif

namespace twosd {

struct Philox4 { uint32_t v[4]; };

TWOSD_HD void philox_round(uint32_t c[4], const uint32_t k[2]) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c[1] ^ k[0], n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

TWOSD_HD Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    uint32_t c[4] = {c0, c1, c2, c3};
    uint32_t k[2] = {k0, k1};
    for (int r = 0; r < 10; ++r) {
        if (r) { k[0] += 0x9E3779B9u; k[1] += 0xBB67AE85u; }
        philox_round(c, k);
    }
    Philox4 o;
    o.v[0] = c[0]; o.v[1] = c[1]; o.v[2] = c[2]; o.v[3] = c[3];
    return o;
}

// 53-bit uniform double in [0, 1) from two 32-bit words
TWOSD_HD double u01(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

}  // namespace twosd
