// dvs_kernel.hip -- device-resident sdDualVertexSet with batched push!.
//
// Reference semantics (src/sd_algorithm/dual_set.jl):
//   hash(pi)        = bits of round(sum_i |pi_i| (sequential, i ascending); base=2, sigdigits=16)   :46-53
//   isequal(a, b)   = same length && same hash && forall i round16(a_i) == round16(b_i)            :24-40
//   push!(V, pi)    = linear scan; append iff no equal vertex; insertion order kept                :84-94
// Equality is an equivalence relation on the key (hash, round16 components), so pushing a
// batch sequentially == "candidate c is appended iff no vertex of V and no earlier
// candidate of the batch has its key".  The GPU evaluates that in five data-parallel
// phases (key, lookup in V, batch-internal min-index resolution, scan, append), all
// deterministic: new vertex ids follow candidate order exactly as the sequential loop.
// NaN components never compare equal (r1 != r2), so a vector containing NaN is always
// appended, as in the reference.
//
// Device structures: V (cap x m fp64, row-major), hash/fp (cap uint64), an open-
// addressing table (int32 vertex ids, linear probing on a 64-bit fingerprint of the key).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <math.h>
#include <algorithm>
#include <vector>
#include "twosd_ctx.h"
#include "dvs_keys.h"

namespace twosd {

// Phase 1: one LANE per candidate -> hash (reference, sequential L1 order), fingerprint,
// has-NaN flag.  The sequential sum is a dependent chain per vector, so each lane walks
// its own vector; the block's 256 vectors are staged through LDS 16 columns at a time
// (coalesced 128-byte row segments in, conflict-free stride-17 reads out).
// one wavefront per vector: the lanes load the row coalesced and fold the order-independent
// parts (fingerprint sum, NaN flag); |pi_i| goes through LDS and lane 0 adds it in index order
// (the reference's sequential sum, dual_set.jl:47-50, so the same bits).  Round 3 used one
// thread per vector: a push of ~4k vectors occupied 16 CUs for ~0.26 ms.
constexpr int kKeyWaves = 4;
__global__ void __launch_bounds__(64 * kKeyWaves) dvs_key_kernel(int count, int m, const double *__restrict__ pis,
                                                               uint64_t *__restrict__ hash, uint64_t *__restrict__ fp,
                                                               int *__restrict__ nanflag) {
    extern __shared__ double kabs[];   // kKeyWaves x m
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * kKeyWaves + w;
    if (c >= count) return;            // whole wavefronts; no block barrier below
    double *a = kabs + (size_t)w * m;
    const double *p = pis + (size_t)c * m;
    uint64_t f = 0;
    int hasnan = 0;
    for (int i = lane; i < m; i += 64) {
        const double v = p[i];
        hasnan |= isnan(v);
        f += mix64(comp_bits(v) ^ (0xD6E8FEB86659FD93ull * (uint64_t)(i + 1)));
        a[i] = fabs(v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f += __shfl_xor(f, o);
    hasnan = __any(hasnan);
    __builtin_amdgcn_s_waitcnt(0xc07f);   // this wave's LDS writes done (lgkmcnt 0)
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        double acc = 0.0;
        for (int i = 0; i < m; ++i) acc += a[i];
        const uint64_t h = (uint64_t)__double_as_longlong(round16(acc));
        hash[c] = h;
        fp[c] = mix64(f ^ h);
        nanflag[c] = hasnan;
    }
}

// full key equality of candidate row a (hash ha) and row b (hash hb); one wavefront
__device__ bool key_equal(const double *a, uint64_t ha, const double *b, uint64_t hb, int m, int lane) {
    if (ha != hb) return false;
    int diff = 0;
    for (int i = lane; i < m; i += 64) diff |= (round16(a[i]) != round16(b[i]));
    return !__any(diff);
}

// Phase 2: look every candidate up in the existing set V.  out[c] = id or -1.
__global__ void __launch_bounds__(256) dvs_lookup_kernel(int count, int m, const double *__restrict__ pis,
                                                         const uint64_t *__restrict__ chash,
                                                         const uint64_t *__restrict__ cfp,
                                                         const int *__restrict__ nanflag, const double *__restrict__ V,
                                                         const uint64_t *__restrict__ vhash,
                                                         const uint64_t *__restrict__ vfp,
                                                         const int *__restrict__ table, int tmask, int *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    for (int c = gw; c < count; c += nw) {
        int found = -1;
        if (!nanflag[c]) {
            const uint64_t f = cfp[c];
            for (int pos = (int)(f & (uint64_t)tmask);; pos = (pos + 1) & tmask) {
                const int id = table[pos];
                if (id < 0) break;
                if (vfp[id] == f && key_equal(pis + (size_t)c * m, chash[c], V + (size_t)id * m, vhash[id], m, lane)) {
                    found = id;
                    break;
                }
            }
        }
        if (lane == 0) out[c] = found;
    }
}

// Phase 3: batch-internal duplicates.  Temp table slots hold candidate indices; the first
// CAS winner fixes a slot's key, later equal-key candidates atomicMin into it, so each
// slot ends with the minimum (= first in push order) candidate of its key.
__global__ void __launch_bounds__(256) dvs_batch_kernel(int count, int m, const double *__restrict__ pis,
                                                        const uint64_t *__restrict__ chash,
                                                        const uint64_t *__restrict__ cfp,
                                                        const int *__restrict__ nanflag, const int *__restrict__ out,
                                                        int *__restrict__ tt, int ttmask, int *__restrict__ slot) {
    const int lane = threadIdx.x & 63;
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    for (int c = gw; c < count; c += nw) {
        if (out[c] >= 0 || nanflag[c]) {
            if (lane == 0) slot[c] = -1;
            continue;
        }
        const uint64_t f = cfp[c];
        int pos = (int)(f & (uint64_t)ttmask);
        for (;;) {
            int cur = 0;
            if (lane == 0) {
                cur = __hip_atomic_load(&tt[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (cur < 0) {
                    const int prev = atomicCAS(&tt[pos], -1, c);
                    cur = prev < 0 ? c : prev;
                }
            }
            cur = __shfl(cur, 0);
            if (cur == c) break;
            if (cfp[cur] == f && key_equal(pis + (size_t)c * m, chash[c], pis + (size_t)cur * m, chash[cur], m, lane)) {
                if (lane == 0) atomicMin(&tt[pos], c);
                break;
            }
            pos = (pos + 1) & ttmask;
        }
        if (lane == 0) slot[c] = pos;
    }
}

// Phase 4: is_new[c] = candidate c is the representative of its key (or has NaN)
__global__ void dvs_flag_kernel(int count, const int *__restrict__ out, const int *__restrict__ nanflag,
                                const int *__restrict__ tt, const int *__restrict__ slot, int *__restrict__ isnew) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= count) return;
    int v = 0;
    if (out[c] < 0) v = nanflag[c] ? 1 : (tt[slot[c]] == c);
    isnew[c] = v;
}

__device__ __forceinline__ void table_insert(int *table, int tmask, uint64_t f, int id) {
    for (int pos = (int)(f & (uint64_t)tmask);; pos = (pos + 1) & tmask)
        if (atomicCAS(&table[pos], -1, id) == -1) return;
}

// Phase 5: assign ids (base + exclusive scan), append new rows, insert them into the table.
__global__ void __launch_bounds__(256) dvs_assign_kernel(int count, int m, int base, const double *__restrict__ pis,
                                                         const uint64_t *__restrict__ chash,
                                                         const uint64_t *__restrict__ cfp,
                                                         const int *__restrict__ nanflag, const int *__restrict__ tt,
                                                         const int *__restrict__ slot, const int *__restrict__ scan,
                                                         int *__restrict__ out, double *__restrict__ V,
                                                         uint64_t *__restrict__ vhash, uint64_t *__restrict__ vfp,
                                                         int *__restrict__ table, int tmask) {
    const int lane = threadIdx.x & 63;
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    for (int c = gw; c < count; c += nw) {
        if (out[c] >= 0) continue;
        const int rep = nanflag[c] ? c : tt[slot[c]];
        const int id = base + scan[rep];
        if (lane == 0) out[c] = id;
        if (rep == c) {
            const double *src = pis + (size_t)c * m;
            double *dst = V + (size_t)id * m;
            for (int i = lane; i < m; i += 64) dst[i] = src[i];
            if (lane == 0) {
                vhash[id] = chash[c];
                vfp[id] = cfp[c];
                if (!nanflag[c]) table_insert(table, tmask, cfp[c], id);
            }
        }
    }
}

__global__ void dvs_rebuild_kernel(int size, const uint64_t *__restrict__ vfp, int *__restrict__ table, int tmask) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id < size) table_insert(table, tmask, vfp[id], id);
}

__global__ void dvs_fill_kernel(int *p, int n, int v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// ---------------------------------------------------------------------------------
struct DvsWs {
    uint64_t *chash = nullptr, *cfp = nullptr;
    int *nanflag = nullptr, *out = nullptr, *slot = nullptr, *isnew = nullptr, *scan = nullptr, *tt = nullptr;
    size_t ccap = 0, ttcap = 0;
    void *cub_tmp = nullptr;
    size_t cub_bytes = 0;
    double *pis = nullptr;        // staging for host-provided candidates
    size_t pis_cap = 0;
    int *nanhost = nullptr;
};

static DvsWs *ws_of(twosd_ctx *c) {
    if (!c->dvs_ws) c->dvs_ws = new DvsWs();
    return (DvsWs *)c->dvs_ws;
}

static int nblocks_for(int count) { return std::max(1, std::min((count + 3) / 4, 8192)); }

int dvs_init(twosd_ctx *c) {
    dvs_free(c);
    c->dvs.m = c->L.m;
    c->dvs.size = 0;
    cut_truncate_pk(c, 0);
    return TWOSD_OK;
}

void dvs_free(twosd_ctx *c) {
    DvsDevice &D = c->dvs;
    if (D.V) hipFree(D.V);
    if (D.hash) hipFree(D.hash);
    if (D.fp) hipFree(D.fp);
    if (D.table) hipFree(D.table);
    D = DvsDevice();
    if (c->dvs_ws) {
        DvsWs *w = (DvsWs *)c->dvs_ws;
        hipFree(w->chash); hipFree(w->cfp); hipFree(w->nanflag); hipFree(w->out); hipFree(w->slot);
        hipFree(w->isnew); hipFree(w->scan); hipFree(w->tt); hipFree(w->cub_tmp); hipFree(w->pis);
        delete w;
        c->dvs_ws = nullptr;
    }
}

#define HIPCHK(expr)                                                                               \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) return fail(TWOSD_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

static int ensure_capacity(twosd_ctx *c, int need) {
    DvsDevice &D = c->dvs;
    const int m = D.m;
    if (need > D.cap) {
        size_t ncap = std::max<size_t>((size_t)need, (size_t)D.cap * 2 + 256);
        size_t cap = D.cap;
        int rc;
        size_t c1 = cap, c2 = cap, c3 = cap;
        if ((rc = dgrow(&D.V, &c1, ncap * m, (size_t)D.size * m, c->stream))) return rc;
        if ((rc = dgrow(&D.hash, &c2, ncap, (size_t)D.size, c->stream))) return rc;
        if ((rc = dgrow(&D.fp, &c3, ncap, (size_t)D.size, c->stream))) return rc;
        D.cap = (int)ncap;
    }
    // table load factor <= 1/2
    if ((size_t)D.tcap < 2 * (size_t)need || !D.table) {
        int tc = 1024;
        while ((size_t)tc < 2 * (size_t)need) tc <<= 1;
        if (D.table) hipFree(D.table);
        HIPCHK(hipMalloc(&D.table, sizeof(int) * tc));
        D.tcap = tc;
        hipLaunchKernelGGL(dvs_fill_kernel, dim3((tc + 255) / 256), dim3(256), 0, c->stream, D.table, tc, -1);
        if (D.size)
            hipLaunchKernelGGL(dvs_rebuild_kernel, dim3((D.size + 255) / 256), dim3(256), 0, c->stream, D.size, D.fp,
                               D.table, tc - 1);
        HIPCHK(hipGetLastError());
    }
    return TWOSD_OK;
}

template <typename T>
static int ws_grow(T **p, size_t need) {
    if (*p) hipFree(*p);
    *p = nullptr;
    hipError_t e = hipMalloc((void **)p, sizeof(T) * std::max<size_t>(need, 1));
    if (e != hipSuccess) return fail(TWOSD_E_DEVICE, "dvs workspace hipMalloc: %s", hipGetErrorString(e));
    return TWOSD_OK;
}

// Push `count` candidates already on the device (row-major count x m).  d_out_index
// (nullable, device) receives the vertex index of every candidate.
int dvs_push_device(twosd_ctx *c, int count, const double *d_pis, int *d_out_index, const uint64_t *d_hash,
                    const uint64_t *d_fp, const int *d_nan) {
    if (count <= 0) return TWOSD_OK;
    DvsDevice &D = c->dvs;
    DvsWs *w = ws_of(c);
    const int m = D.m;
    int rc;
    if ((size_t)count > w->ccap) {
        size_t cc = std::max<size_t>(count, 1024);
        if ((rc = ws_grow(&w->chash, cc)) || (rc = ws_grow(&w->cfp, cc)) || (rc = ws_grow(&w->nanflag, cc)) ||
            (rc = ws_grow(&w->out, cc)) || (rc = ws_grow(&w->slot, cc)) || (rc = ws_grow(&w->isnew, cc)) ||
            (rc = ws_grow(&w->scan, cc)))
            return rc;
        w->ccap = cc;
        size_t need = 0;
        hipcub::DeviceScan::ExclusiveSum(nullptr, need, w->isnew, w->scan, (int)cc, c->stream);
        if (need > w->cub_bytes) {
            if (w->cub_tmp) hipFree(w->cub_tmp);
            HIPCHK(hipMalloc(&w->cub_tmp, need));
            w->cub_bytes = need;
        }
    }
    size_t ttneed = 1024;
    while (ttneed < 2 * (size_t)count) ttneed <<= 1;
    if (ttneed > w->ttcap) {
        if ((rc = ws_grow(&w->tt, ttneed))) return rc;
        w->ttcap = ttneed;
    }
    if ((rc = ensure_capacity(c, D.size + count))) return rc;
    const int ttmask = (int)w->ttcap - 1;
    const int nb = nblocks_for(count);
    hipLaunchKernelGGL(dvs_fill_kernel, dim3((w->ttcap + 255) / 256), dim3(256), 0, c->stream, w->tt, (int)w->ttcap, -1);
    if (d_hash) {   // keys computed by the producer (LP kernel epilogue)
        HIPCHK(hipMemcpyAsync(w->chash, d_hash, sizeof(uint64_t) * count, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(w->cfp, d_fp, sizeof(uint64_t) * count, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(w->nanflag, d_nan, sizeof(int) * count, hipMemcpyDeviceToDevice, c->stream));
    } else {
        hipLaunchKernelGGL(dvs_key_kernel, dim3((count + kKeyWaves - 1) / kKeyWaves), dim3(64 * kKeyWaves),
                           sizeof(double) * kKeyWaves * m, c->stream, count, m, d_pis, w->chash, w->cfp, w->nanflag);
    }
    hipLaunchKernelGGL(dvs_lookup_kernel, dim3(nb), dim3(256), 0, c->stream, count, m, d_pis, w->chash, w->cfp,
                       w->nanflag, D.V, D.hash, D.fp, D.table, D.tcap - 1, w->out);
    hipLaunchKernelGGL(dvs_batch_kernel, dim3(nb), dim3(256), 0, c->stream, count, m, d_pis, w->chash, w->cfp,
                       w->nanflag, w->out, w->tt, ttmask, w->slot);
    hipLaunchKernelGGL(dvs_flag_kernel, dim3((count + 255) / 256), dim3(256), 0, c->stream, count, w->out, w->nanflag,
                       w->tt, w->slot, w->isnew);
    size_t tb = w->cub_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(w->cub_tmp, tb, w->isnew, w->scan, count, c->stream));
    hipLaunchKernelGGL(dvs_assign_kernel, dim3(nb), dim3(256), 0, c->stream, count, m, D.size, d_pis, w->chash, w->cfp,
                       w->nanflag, w->tt, w->slot, w->scan, w->out, D.V, D.hash, D.fp, D.table, D.tcap - 1);
    HIPCHK(hipGetLastError());
    int last_scan = 0, last_new = 0;
    HIPCHK(hipMemcpyAsync(&last_scan, w->scan + count - 1, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&last_new, w->isnew + count - 1, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (d_out_index)
        HIPCHK(hipMemcpyAsync(d_out_index, w->out, sizeof(int) * count, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    D.size += last_scan + last_new;
    return TWOSD_OK;
}

}  // namespace twosd

using namespace twosd;

extern "C" int twosd_dvs_push(twosd_ctx *c, int count, const double *pis, int *out_index, int *new_size) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "dvs_push: no template");
    if (count < 0 || (count > 0 && !pis)) return fail(TWOSD_E_ARG, "dvs_push: bad arguments");
    HIPCHK(hipSetDevice(c->device));
    if (count > 0) {
        DvsWs *w = ws_of(c);
        const size_t need = (size_t)count * c->dvs.m;
        if (need > w->pis_cap) {
            int rc = ws_grow(&w->pis, need);
            if (rc) return rc;
            w->pis_cap = need;
        }
        HIPCHK(hipMemcpy(w->pis, pis, sizeof(double) * need, hipMemcpyHostToDevice));
        hipEvent_t e0 = c->ev[2], e1 = c->ev[3];
        HIPCHK(hipEventRecord(e0, c->stream));
        int rc = dvs_push_device(c, count, w->pis, nullptr, nullptr, nullptr, nullptr);
        if (rc) return rc;
        HIPCHK(hipEventRecord(e1, c->stream));
        HIPCHK(hipEventSynchronize(e1));
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        c->t_us[1] = 1e3 * ms;
        if (out_index) HIPCHK(hipMemcpy(out_index, w->out, sizeof(int) * count, hipMemcpyDeviceToHost));
    }
    if (new_size) *new_size = c->dvs.size;
    return TWOSD_OK;
}

extern "C" int twosd_dvs_size(twosd_ctx *c, int *size) {
    if (!c || !size) return fail(TWOSD_E_ARG, "dvs_size: NULL");
    *size = c->dvs.size;
    return TWOSD_OK;
}

extern "C" int twosd_dvs_get(twosd_ctx *c, int first, int count, double *out) {
    if (!c || (count > 0 && !out)) return fail(TWOSD_E_ARG, "dvs_get: NULL");
    if (first < 0 || count < 0 || first + count > c->dvs.size) return fail(TWOSD_E_ARG, "dvs_get: range outside the set");
    if (count == 0) return TWOSD_OK;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(out, c->dvs.V + (size_t)first * c->dvs.m, sizeof(double) * count * c->dvs.m, hipMemcpyDeviceToHost));
    return TWOSD_OK;
}

extern "C" int twosd_dvs_clear(twosd_ctx *c) { return twosd_dvs_truncate(c, 0); }

// Order-dependent digest of the set: size + sum_i fp_i (2i + 1) mod 2^64 over the per-vertex
// 64-bit fingerprints of the rounded components (the dedup keys).  Ranks compare it before an
// all-reduce over vertex indices (sqlp_amd/dist.py).
extern "C" int twosd_dvs_fingerprint(twosd_ctx *c, uint64_t *out) {
    if (!c || !out) return fail(TWOSD_E_ARG, "dvs_fingerprint: NULL");
    const int n = c->dvs.size;
    uint64_t acc = (uint64_t)n * 0x9E3779B97F4A7C15ull;
    if (n > 0) {
        HIPCHK(hipSetDevice(c->device));
        std::vector<uint64_t> fp(n);
        HIPCHK(hipMemcpy(fp.data(), c->dvs.fp, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
        for (int i = 0; i < n; ++i) acc += fp[i] * (2 * (uint64_t)i + 1);
    }
    *out = acc;
    return TWOSD_OK;
}

extern "C" int twosd_dvs_truncate(twosd_ctx *c, int size) {
    if (!c) return fail(TWOSD_E_ARG, "dvs_truncate: NULL");
    if (size < 0 || size > c->dvs.size) return fail(TWOSD_E_ARG, "dvs_truncate: size %d outside [0, %d]", size, c->dvs.size);
    if (size == c->dvs.size) return TWOSD_OK;
    HIPCHK(hipSetDevice(c->device));
    DvsDevice &D = c->dvs;
    D.size = size;
    cut_truncate_pk(c, size);   // the cut's PK rows below size stay valid (V[0, size) is unchanged)
    if (D.table) {
        hipLaunchKernelGGL(dvs_fill_kernel, dim3((D.tcap + 255) / 256), dim3(256), 0, c->stream, D.table, D.tcap, -1);
        if (size)
            hipLaunchKernelGGL(dvs_rebuild_kernel, dim3((size + 255) / 256), dim3(256), 0, c->stream, size, D.fp, D.table,
                               D.tcap - 1);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return TWOSD_OK;
}
