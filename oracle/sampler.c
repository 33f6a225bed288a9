/* sampler.c -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): CPU restatement of the
 * on-device scenario sampler, checked against the published Philox4x32-10 known-answer
 * vectors (Random123 kat_vectors) in tests/test_oracle_kat.py.
 *
 * Reference: rand(rng, sto) (src/smps/smps_sto.jl:117-149) over Distributions 0.25.102
 * (Manifest.toml): DiscreteNonParametric inverse CDF with a running cumulative sum,
 * Normal(mean, sqrt(variance)), Uniform(left, right) = left + (right-left)*u.  The random
 * stream itself (Julia's Xoshiro / ziggurat) is not reproducible outside Julia; the build
 * uses Philox4x32-10 (Salmon et al., SC'11): element e of scenario index g takes counter
 * (g_lo, g_hi, e, 0), key (seed_lo, seed_hi); u1 from words (0,1), u2 from (2,3) as
 * 53-bit doubles; NORMAL by Box-Muller sqrt(-2 log(1-u1)) cos(2 pi u2).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

static void philox_ref(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t x0 = ctr_in[0], x1 = ctr_in[1], x2 = ctr_in[2], x3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int round = 0; round < 10; ++round) {
        if (round > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t a = (uint64_t)0xD2511F53u * (uint64_t)x0;
        const uint64_t b = (uint64_t)0xCD9E8D57u * (uint64_t)x2;
        const uint32_t y0 = (uint32_t)(b >> 32) ^ x1 ^ k0;
        const uint32_t y1 = (uint32_t)b;
        const uint32_t y2 = (uint32_t)(a >> 32) ^ x3 ^ k1;
        const uint32_t y3 = (uint32_t)a;
        x0 = y0; x1 = y1; x2 = y2; x3 = y3;
    }
    out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
}

void oracle_philox4x32_10(const uint32_t *ctr, const uint32_t *key, uint32_t *out) { philox_ref(ctr, key, out); }

static double u53(uint32_t hi, uint32_t lo) {
    const uint64_t m = ((uint64_t)(hi >> 5) << 26) | (uint64_t)(lo >> 6);
    return (double)m / 9007199254740992.0;
}

/* kind[k] 0/1/2; off[k+1] into val/prob (support sorted ascending); p0/p1 = mean/sd or
 * left/right; tmpl[k]; out[N*k] = value - template (the stored delta) */
void oracle_sample(int N, int k, uint64_t seed, uint64_t first_index, const int *kind, const int *off,
                   const double *val, const double *prob, const double *p0, const double *p1, const double *tmpl,
                   double *out) {
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int s = 0; s < N; ++s) {
        const uint64_t g = first_index + (uint64_t)s;
        for (int e = 0; e < k; ++e) {
            const uint32_t ctr[4] = {(uint32_t)g, (uint32_t)(g >> 32), (uint32_t)e, 0u};
            uint32_t r[4];
            philox_ref(ctr, key, r);
            const double u1 = u53(r[0], r[1]);
            double v;
            if (kind[e] == 0) {
                const int o = off[e], n = off[e + 1] - off[e];
                int i = 0;
                double cp = prob[o];
                while (cp <= u1 && i < n - 1) {
                    i += 1;
                    cp = cp + prob[o + i];
                }
                v = val[o + i];
            } else if (kind[e] == 1) {
                const double u2 = u53(r[2], r[3]);
                const double z = sqrt(-2.0 * log(1.0 - u1)) * cos(6.283185307179586 * u2);
                const volatile double t = p1[e] * z;
                v = p0[e] + t;
            } else {
                const volatile double w = p1[e] - p0[e];
                const volatile double t = w * u1;
                v = p0[e] + t;
            }
            const volatile double d = v - tmpl[e];
            out[(size_t)s * k + e] = d;
        }
    }
}
