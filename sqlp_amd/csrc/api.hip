// api.hip -- C ABI of libtwosd_hip.so (declared in include/twosd_hip.h).
//
// Owns the device-resident state of the TwoSD hot path on one MI355X:
//   template (W CSC, q, bound types), shared warm-start basis (B0^{-1}, pi0), per-epigraph
//   scenario pools (deltas, weights), the dual vertex set, and the LP/cut workspaces.
// Every call is synchronous on the context's own HIP stream.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <map>
#include <memory>
#include <thread>
#include <chrono>
#include "twosd_internal.h"
#include "twosd_ctx.h"

using namespace twosd;

static thread_local std::string g_err;

int twosd::fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                            \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) return fail(TWOSD_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

// TWOSD_POISON=<byte> (test hook): every new device allocation is filled with that byte, so a
// result that depends on memory no kernel wrote changes with it (the fill completes before the
// allocation returns: the context's streams do not order against the null-stream memset)
int twosd::poison_byte(int family) {
    static const int b = getenv("TWOSD_POISON") ? atoi(getenv("TWOSD_POISON")) : -1;
    static const int fam = getenv("TWOSD_POISON_FAMILY") ? atoi(getenv("TWOSD_POISON_FAMILY")) : -1;
    static const bool said = b >= 0 && fprintf(stderr, "TWOSD_POISON: new device allocations filled with 0x%02x (families %d)\n",
                                               b & 0xff, fam) > 0;
    (void)said;
    return (fam & family) ? b : -1;
}
template <typename T>
static int dalloc(T **p, size_t count) {
    if (*p) { hipFree(*p); *p = nullptr; }
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void **)p, sizeof(T) * count);
    if (e != hipSuccess) return fail(TWOSD_E_DEVICE, "hipMalloc(%zu bytes): %s", sizeof(T) * count, hipGetErrorString(e));
    if (poison_byte(1) >= 0) { hipMemset(*p, poison_byte(1), sizeof(T) * count); hipDeviceSynchronize(); }
    return TWOSD_OK;
}
template <typename T>
static void dfree(T *&p) {
    if (p) hipFree(p);
    p = nullptr;
}

// grow a device array to at least `count` elements, keeping `keep` elements
template <typename T>
int twosd::dgrow(T **p, size_t *cap, size_t count, size_t keep, hipStream_t s) {
    if (count <= *cap && *p) return TWOSD_OK;
    size_t ncap = std::max<size_t>(count, *cap * 2 + 1024);
    T *np = nullptr;
    hipError_t e = hipMalloc((void **)&np, sizeof(T) * ncap);
    if (e != hipSuccess) return fail(TWOSD_E_DEVICE, "hipMalloc(%zu bytes): %s", sizeof(T) * ncap, hipGetErrorString(e));
    if (poison_byte(2) >= 0) { hipMemset(np, poison_byte(2), sizeof(T) * ncap); hipDeviceSynchronize(); }
    if (*p && keep) {
        e = hipMemcpyAsync(np, *p, sizeof(T) * keep, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return fail(TWOSD_E_DEVICE, "grow copy: %s", hipGetErrorString(e));
        hipStreamSynchronize(s);
    }
    if (*p) hipFree(*p);
    *p = np;
    *cap = ncap;
    return TWOSD_OK;
}
template int twosd::dgrow<double>(double **, size_t *, size_t, size_t, hipStream_t);
template int twosd::dgrow<int>(int **, size_t *, size_t, size_t, hipStream_t);
template int twosd::dgrow<uint64_t>(uint64_t **, size_t *, size_t, size_t, hipStream_t);

extern "C" const char *twosd_last_error(void) { return g_err.c_str(); }
extern "C" const char *twosd_version(void) { return "twosd-mi355x 0.1 (gfx950)"; }

extern "C" int twosd_create(int device, twosd_ctx **out) {
    if (!out) return fail(TWOSD_E_ARG, "twosd_create: out is NULL");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(TWOSD_E_ARG, "twosd_create: device %d of %d", device, ndev);
    HIPCHK(hipSetDevice(device));
    twosd_ctx *c = new twosd_ctx();
    c->device = device;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int i = 0; i < 8; ++i) HIPCHK(hipEventCreate(&c->ev[i]));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    c->num_cus = prop.multiProcessorCount;
    const char *km = getenv("TWOSD_KMAX");
    if (km) c->kmax_override = atoi(km);
    *out = c;
    return TWOSD_OK;
}

// Sliced ELL of S*64 columns: column j = 64*s + l gives (row, value) entries via colf.
// Slot s has width E_s = max entries over its 64 columns; entry e of lane l is stored at
// [(slot[s] + e) * 64 + l], padding (row 0, value 0).
template <typename F>
static void build_ell(int S, F colf, std::vector<int> &slot, std::vector<int> &ix, std::vector<double> &v) {
    slot.assign(S + 1, 0);
    std::vector<std::vector<std::pair<int, double>>> cols(64);
    ix.clear(); v.clear();
    for (int s = 0; s < S; ++s) {
        int width = 0;
        for (int l = 0; l < 64; ++l) {
            cols[l].clear();
            colf(64 * s + l, cols[l]);
            width = std::max(width, (int)cols[l].size());
        }
        for (int e = 0; e < width; ++e)
            for (int l = 0; l < 64; ++l) {
                const bool has = e < (int)cols[l].size();
                ix.push_back(has ? cols[l][e].first : 0);
                v.push_back(has ? cols[l][e].second : 0.0);
            }
        slot[s + 1] = slot[s] + width;
    }
}

// pinned host staging buffer `slot` of at least n elements of T (grown, never shrunk)
template <typename T>
static T *stage_buf(twosd_ctx *c, int slot, size_t n) {
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    if (bytes > c->stage_bytes[slot]) {
        if (c->stage[slot]) hipHostFree(c->stage[slot]);
        c->stage[slot] = nullptr;
        c->stage_bytes[slot] = 0;
        if (hipHostMalloc(&c->stage[slot], bytes + bytes / 4) != hipSuccess) return nullptr;
        c->stage_bytes[slot] = bytes + bytes / 4;
    }
    return static_cast<T *>(c->stage[slot]);
}

// the two-level candidate lists (device, or staged for the next selection) refer to pool
// indices: every change of the pool drops them
static void reset_candidates(twosd_ctx *c) {
    c->pool_l1 = c->pool_ncand = 0;
    c->cand_pending = false;
    std::vector<int>().swap(c->cand_p1);
    std::vector<int>().swap(c->cand_pf);
}

// the pool no longer matches the device arrays (a failed build or head read-back): keep only
// the primary basis (a host basis) and refuse solves until a basis is installed again
static int drop_pool(twosd_ctx *c, int code) {
    if (c->pool.size() > 1) c->pool.resize(1);
    c->has_basis = false;
    c->prep_valid = false;
    c->k_valid = false;
    c->pool_hb_valid = false;
    reset_candidates(c);
    return code;
}

// head of pool basis p into *h (materialised from c->pool_hb for a device-built basis on first
// use: a refresh of 4096 bases would otherwise spend ~2 ms building host heads nobody reads).
// A failed device read-back drops the pool (drop_pool) and returns TWOSD_E_DEVICE.
static int head_of(twosd_ctx *c, int p, const std::vector<int> **h) {
    PoolBasis &B = c->pool[p];
    if (B.hb_row >= 0 && !c->pool_hb_valid) {
        // the heads of a device-built pool are fetched on the first host use, not by the refresh
        // (at N = 8 every rank would copy 9 MB per step that only tests and the CPU baseline read)
        const size_t need = c->pool.size() * (size_t)c->MP;
        if (need > c->pool_hb_cap) {
            if (c->pool_hb) hipHostFree(c->pool_hb);
            c->pool_hb = nullptr;
            c->pool_hb_cap = 0;
            if (hipHostMalloc((void **)&c->pool_hb, sizeof(int) * need * 5 / 4) != hipSuccess)
                return drop_pool(c, fail(TWOSD_E_DEVICE, "pool heads: pinned allocation of %zu ints failed", need));
            c->pool_hb_cap = need * 5 / 4;
        }
        hipError_t e = hipMemcpyAsync(c->pool_hb, c->d_hb0, sizeof(int) * need, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return drop_pool(c, fail(TWOSD_E_DEVICE, "pool heads: read-back failed: %s", hipGetErrorString(e)));
        c->pool_hb_valid = true;
    }
    if (B.hb_row >= 0) {
        const int m = c->L.m;
        const int *r = c->pool_hb + (size_t)B.hb_row * c->MP;
        B.head.resize(m);
        for (int i = 0; i < m; ++i) B.head[i] = r[i] >> 2;
        B.hb_row = -1;
    }
    if (h) *h = &B.head;
    return TWOSD_OK;
}
static int materialize_heads(twosd_ctx *c) {
    for (int p = 0; p < (int)c->pool.size(); ++p)
        if (int rc = head_of(c, p, nullptr)) return rc;
    return TWOSD_OK;
}

// f(i) for i in [0, n) on up to 16 host threads (per-basis pool preparation: independent work)
template <typename F>
static void parallel_for(int n, F f) {
    const int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < 64 || nth == 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nth; ++t)
        th.emplace_back([&, t]() {
            for (int i = t; i < n; i += nth) f(i);
        });
    for (auto &t : th) t.join();
}

template <typename T>
static int upload_raw(T **d, const T *h, size_t n) {
    int rc = dalloc(d, std::max<size_t>(n, 1));
    if (rc) return rc;
    if (n) HIPCHK(hipMemcpy(*d, h, sizeof(T) * n, hipMemcpyHostToDevice));
    return TWOSD_OK;
}

// grow-only device array of at least n elements (no hipFree / hipMalloc when they fit;
// contents not kept on growth)
template <typename T>
static int dev_reserve(twosd_ctx *c, T **d, size_t n) {
    size_t &cap = c->dcap[(const void *)d];
    if (!*d || cap < std::max<size_t>(n, 1)) {
        const size_t want = std::max<size_t>(n, 1) + std::max<size_t>(n, 1) / 4;
        int rc = dalloc(d, want);
        if (rc) { cap = 0; return rc; }
        cap = want;
    }
    return TWOSD_OK;
}
template <typename T>
static int upload_big(twosd_ctx *c, T **d, const T *h, size_t n) {
    int rc = dev_reserve(c, d, n);
    if (rc) return rc;
    if (n) HIPCHK(hipMemcpy(*d, h, sizeof(T) * n, hipMemcpyHostToDevice));
    return TWOSD_OK;
}
template <typename T>
static int upload_big(twosd_ctx *c, T **d, const std::vector<T> &h) {
    return upload_big(c, d, h.data(), h.size());
}

// device selection-stream outputs of a pool of P bases with `records` records (prepare_x
// writes them per x)
static int reserve_selection(twosd_ctx *c, int P, int records) {
    int rc;
    if ((size_t)std::max(records, 1) > c->sel_code_cap) {
        dfree(c->d_sel_code);
        if ((rc = dalloc(&c->d_sel_code, 2 * (size_t)std::max(records, 1)))) return rc;
        c->sel_code_cap = std::max(records, 1);
    }
    if ((rc = dev_reserve(c, &c->d_sel_end, (size_t)P)) || (rc = dev_reserve(c, &c->d_sel_cinf, (size_t)P))) return rc;
    c->sel_cap_total = records;
    return TWOSD_OK;
}

template <typename T>
static int upload(T **d, const std::vector<T> &h) {
    int rc = dalloc(d, std::max<size_t>(h.size(), 1));
    if (rc) return rc;
    if (!h.empty()) HIPCHK(hipMemcpy(*d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
    return TWOSD_OK;
}

static void free_template(twosd_ctx *c) {
    dfree(c->d_colptr); dfree(c->d_rowidx); dfree(c->d_val); dfree(c->d_q); dfree(c->d_btype);
    dfree(c->d_fixedmask); dfree(c->d_ubmask);
    dfree(c->d_hb0); dfree(c->d_basic0);
    dfree(c->d_xbase); dfree(c->d_queue); dfree(c->d_lpstats);
    dfree(c->d_obj); dfree(c->d_pi); dfree(c->d_pi_rep); dfree(c->d_y); dfree(c->d_status); dfree(c->d_iters); dfree(c->d_ops); dfree(c->d_etan);
    dfree(c->d_dvtmp);
    dfree(c->d_bnnz); dfree(c->d_sel_cinf); dfree(c->d_sel_ptr); dfree(c->d_sel_code); c->sel_code_cap = 0; dfree(c->d_head_out); dfree(c->d_pool_pick); dfree(c->d_cpick); dfree(c->d_order); dfree(c->d_sort_tmp);
    dfree(c->d_cand); dfree(c->d_sel_key); dfree(c->d_sel_pkey); dfree(c->d_sel_ppick); c->sel_pcap = 0; c->key_cap = 0; c->pool_l1 = c->pool_ncand = 0; c->order_cap = 0; c->sort_tmp_bytes = 0; c->head_cap = 0; c->pick_cap = 0; c->pool.clear();
    dfree(c->d_dist_kind); dfree(c->d_dist_off); dfree(c->d_dist_val); dfree(c->d_dist_prob); dfree(c->d_dist_p0);
    dfree(c->d_dist_p1); dfree(c->d_dist_tmpl); c->has_dist = false;
    dfree(c->d_kslot); dfree(c->d_kix); dfree(c->d_kv); dfree(c->d_kcoef); c->k_valid = false;
    dfree(c->d_sel_end); dfree(c->d_kp); dfree(c->d_ke); dfree(c->d_kraw); dfree(c->d_xaux); c->xaux_cap = 0; c->sel_cap_total = 0;
    dfree(c->d_d0); dfree(c->d_eidx); dfree(c->d_evals); dfree(c->d_stamps);
    dfree(c->d_wcp); dfree(c->d_wcc); dfree(c->d_wcv); dfree(c->d_bcp); dfree(c->d_bci); dfree(c->d_bcv);
    dfree(c->d_brptr); dfree(c->d_brcol); dfree(c->d_brval);
    c->earena_slots = 0; c->earena_cap = 0;
    for (auto &e : c->epis) { dfree(e.d_dv); dfree(e.d_w); }
    c->epis.clear();
    c->out_cap = 0; c->dvtmp_cap = 0;
    dvs_free(c);
    cut_free(c);
    vkey_free(c);
    c->dcap.clear();
    dfree(c->d_vkey); c->vkey_cap = 0;
    dfree(c->d_bkey); c->bkey_cap = 0;
    dfree(c->d_refresh_sel); c->refresh_sel_cap = 0; c->box_epi = -1;
    dfree(c->d_eo_pb); dfree(c->d_eo_K); dfree(c->d_eo_off); dfree(c->d_eo_etap); dfree(c->d_eo_etaoff);
    dfree(c->d_eo_eidx); dfree(c->d_eo_evals); dfree(c->d_eo_used); c->eo_rows = c->eo_cap = 0; c->eo_kmax = 0;
    dfree(c->d_pg_scrow); dfree(c->d_pg_scoff); dfree(c->d_pg_scval); dfree(c->d_pg_ival); dfree(c->d_pg_irow); dfree(c->d_pg_ioff); dfree(c->d_pg_amax); dfree(c->d_pg_d0p); dfree(c->d_pg_cnt); dfree(c->d_pg_tot);
    dfree(c->d_pg_valid); dfree(c->d_pg_head0); dfree(c->d_pg_map); dfree(c->d_pg_off); dfree(c->d_pg_pos);
    dfree(c->d_rt_pack); dfree(c->d_gs_heads); dfree(c->d_gs_cnt); dfree(c->d_gs_tot); dfree(c->d_gs_valid);
    dfree(c->d_gs_irow); dfree(c->d_gs_ioff); dfree(c->d_gs_ival);
    if (c->d_gs_seg) { hipFree(c->d_gs_seg); c->d_gs_seg = nullptr; c->gs_seg_cap = 0; }
    c->rt_epi = -1; c->rt_nown = -1; c->rt_trained = false;
    if (c->pool_hb) { hipHostFree(c->pool_hb); c->pool_hb = nullptr; c->pool_hb_cap = 0; }
    c->has_template = c->has_basis = false;
}

extern "C" int twosd_destroy(twosd_ctx *c) {
    if (!c) return TWOSD_OK;
    hipSetDevice(c->device);
    free_template(c);
    for (int i = 0; i < 8; ++i) hipEventDestroy(c->ev[i]);
    for (int i = 0; i < 16; ++i)
        if (c->stage[i]) hipHostFree(c->stage[i]);
    hipStreamDestroy(c->stream);
    delete c;
    return TWOSD_OK;
}

extern "C" int twosd_set_template(twosd_ctx *c, int m2, int n1, int n2, const int64_t *Tcp, const int64_t *Trv,
                                  const double *Tnz, const int64_t *Wcp, const int64_t *Wrv, const double *Wnz,
                                  const double *q, const double *r, const char *sense, const double *ylb,
                                  const double *yub, int base) {
    if (!c) return fail(TWOSD_E_ARG, "ctx is NULL");
    if (m2 <= 0 || n1 < 0 || n2 <= 0 || !Wcp || !Wrv || !Wnz || !q || !r || !sense || (n1 > 0 && (!Tcp || !Trv || !Tnz)))
        return fail(TWOSD_E_ARG, "twosd_set_template: bad sizes or NULL arrays");
    if (base != 0 && base != 1) return fail(TWOSD_E_ARG, "index_base must be 0 or 1");
    HIPCHK(hipSetDevice(c->device));
    free_template(c);
    HostLP &L = c->L;
    L = HostLP();
    L.m = m2; L.n = n2;
    L.colptr.resize(n2 + 1);
    for (int j = 0; j <= n2; ++j) L.colptr[j] = (int)(Wcp[j] - base);
    const int nnzW = L.colptr[n2];
    if (L.colptr[0] != 0 || nnzW < 0) return fail(TWOSD_E_ARG, "W colptr malformed");
    L.rowidx.resize(nnzW); L.val.resize(nnzW);
    for (int p = 0; p < nnzW; ++p) {
        L.rowidx[p] = (int)(Wrv[p] - base);
        L.val[p] = Wnz[p];
        if (L.rowidx[p] < 0 || L.rowidx[p] >= m2) return fail(TWOSD_E_ARG, "W row index %d out of range", L.rowidx[p] + base);
    }
    L.q.assign(q, q + n2);
    L.sense.assign(sense, sense + m2);
    for (int i = 0; i < m2; ++i)
        if (L.sense[i] != 'G' && L.sense[i] != 'L' && L.sense[i] != 'E')
            return fail(TWOSD_E_ARG, "sense[%d] = '%c' (expected G/L/E)", i, L.sense[i]);
    for (int j = 0; j < n2; ++j) {
        const double lo = ylb ? ylb[j] : 0.0, hi = yub ? yub[j] : INFINITY;
        if (lo != 0.0 || !std::isinf(hi) || hi < 0)
            return fail(TWOSD_E_UNSUPPORTED, "y[%d] bounds [%g, %g]: only [0, +inf) is supported (subprob.jl:19-26 warns on these)", j, lo, hi);
    }
    c->n1 = n1;
    c->r.assign(r, r + m2);
    c->T.assign((size_t)m2 * n1, 0.0);   // dense T (m2 x n1) on the host for per-x setup
    for (int j = 0; j < n1; ++j)
        for (int64_t p = Tcp[j] - base; p < Tcp[j + 1] - base; ++p) {
            const int i = (int)(Trv[p] - base);
            if (i < 0 || i >= m2) return fail(TWOSD_E_ARG, "T row index out of range");
            c->T[(size_t)i * n1 + j] = Tnz[p];
        }
    const int R = hyper_rows_per_lane(m2);
    if (R < 0) return fail(TWOSD_E_UNSUPPORTED, "m2 = %d exceeds the LP kernel envelope (%d rows)", m2, 64 * 16);
    const int C = (n2 + m2 + 63) / 64;
    if (C > kMaxColsPerLane) return fail(TWOSD_E_UNSUPPORTED, "n2 + m2 = %d exceeds %d columns", n2 + m2, 64 * kMaxColsPerLane);
    c->R = R; c->MP = 64 * R; c->C = C;
    c->CH = hyper_cols_per_lane(n2 + m2);
    if (c->CH <= 0) return fail(TWOSD_E_UNSUPPORTED, "n2 + m2 = %d exceeds the LP kernel's column slots", n2 + m2);
    // device template
    int rc;
    if ((rc = dalloc(&c->d_colptr, n2 + 1)) || (rc = dalloc(&c->d_rowidx, nnzW)) || (rc = dalloc(&c->d_val, nnzW)) ||
        (rc = dalloc(&c->d_q, n2)) || (rc = dalloc(&c->d_btype, n2 + m2)) || (rc = dalloc(&c->d_fixedmask, 64)) ||
        (rc = dalloc(&c->d_ubmask, 64)))
        return rc;
    std::vector<int8_t> bt(n2 + m2);
    std::vector<uint64_t> fixedm(64, 0), ubm(64, 0);
    for (int j = 0; j < n2 + m2; ++j) {
        int b = BT_Y;
        if (j >= n2) { char s = L.sense[j - n2]; b = s == 'G' ? BT_G : (s == 'L' ? BT_L : BT_E); }
        bt[j] = (int8_t)b;
    }
    for (int j = 0; j < 64 * 64; ++j) {
        const int lane = j & 63, cs = j >> 6;
        if (j >= n2 + m2 || bt[j] == BT_E) fixedm[lane] |= 1ull << cs;
        else if (bt[j] == BT_G) ubm[lane] |= 1ull << cs;
    }
    HIPCHK(hipMemcpy(c->d_colptr, L.colptr.data(), sizeof(int) * (n2 + 1), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_rowidx, L.rowidx.data(), sizeof(int) * std::max(nnzW, 1), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_val, L.val.data(), sizeof(double) * std::max(nnzW, 1), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_q, L.q.data(), sizeof(double) * n2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_btype, bt.data(), n2 + m2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_fixedmask, fixedm.data(), sizeof(uint64_t) * 64, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_ubmask, ubm.data(), sizeof(uint64_t) * 64, hipMemcpyHostToDevice));
    if (c->CH > 0) {   // W by rows (CSR, columns ascending) for the row-wise pricing scatter
        std::vector<std::vector<std::pair<int, double>>> rows(m2);
        for (int j = 0; j < n2; ++j)
            for (int p = L.colptr[j]; p < L.colptr[j + 1]; ++p) rows[L.rowidx[p]].push_back({j, L.val[p]});
        std::vector<int> cp(m2 + 1, 0), cc;
        std::vector<double> cv;
        for (int i = 0; i < m2; ++i) {
            for (auto &e : rows[i]) { cc.push_back(e.first); cv.push_back(e.second); }
            cp[i + 1] = (int)cc.size();
        }
        if ((rc = upload(&c->d_wcp, cp)) || (rc = upload(&c->d_wcc, cc)) || (rc = upload(&c->d_wcv, cv))) return rc;
    }
    c->has_template = true;
    c->k = 0;
    c->pos_row.clear(); c->pos_col.clear();
    if ((rc = dvs_init(c))) return rc;
    return TWOSD_OK;
}

extern "C" int twosd_set_random_positions(twosd_ctx *c, int k, const int *row, const int *col, int base) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "set_random_positions: no template");
    if (k < 0 || (k > 0 && (!row || !col))) return fail(TWOSD_E_ARG, "set_random_positions: bad arguments");
    for (auto &e : c->epis)
        if (e.count) return fail(TWOSD_E_STATE, "set_random_positions: epigraphs already hold scenarios");
    c->pos_row.resize(k); c->pos_col.resize(k);
    for (int e = 0; e < k; ++e) {
        const int rr = row[e] - base;
        const int cc = col[e] < 0 ? -1 : col[e] - base;
        if (rr < 0 || rr >= c->L.m) return fail(TWOSD_E_ARG, "position %d: row %d out of range", e, row[e]);
        if (cc >= c->n1) return fail(TWOSD_E_ARG, "position %d: column %d is not a first-stage column (KeyError in delta_coefficients, subprob.jl:116)", e, col[e]);
        c->pos_row[e] = rr; c->pos_col[e] = cc;
    }
    c->k = k;
    c->prep_valid = false;
    c->k_valid = false;
    c->has_dist = false;
    cut_invalidate_pk(c);
    return TWOSD_OK;
}

// template value at position e (RHS or T entry)
static double template_value(const twosd_ctx *c, int e) {
    const int rr = c->pos_row[e], cc = c->pos_col[e];
    return cc < 0 ? c->r[rr] : c->T[(size_t)rr * c->n1 + cc];
}

// b = r - T x + effect of the element deltas dv (k)
static void rhs_at(const twosd_ctx *c, const double *x, const double *dv, std::vector<double> &b) {
    const int m = c->L.m, n1 = c->n1;
    b.assign(c->r.begin(), c->r.end());
    if (x)
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int j = 0; j < n1; ++j) s += c->T[(size_t)i * n1 + j] * x[j];
            b[i] -= s;
        }
    if (dv)
        for (int e = 0; e < c->k; ++e) {
            const int cc = c->pos_col[e];
            b[c->pos_row[e]] += cc < 0 ? dv[e] : -dv[e] * (x ? x[cc] : 0.0);
        }
}

// validate a basis head (valid distinct columns, nonsingular, dual feasible for q) and
// compute its inverse; thread-safe, returns nullptr or the reason it was rejected
static const char *compute_pool_basis(const twosd_ctx *c, const std::vector<int> &head, PoolBasis &pb) {
    const HostLP &L = c->L;
    const int m = L.m, n = L.n;
    std::vector<char> seen(n + m, 0);
    for (int i = 0; i < m; ++i) {
        if (head[i] < 0 || head[i] >= n + m || seen[head[i]]) return "basis head has an invalid or duplicate column";
        seen[head[i]] = 1;
    }
    std::vector<double> B;
    basis_matrix(L, head, B);
    if (!dense_inverse(m, B, pb.Binv)) return "basis matrix is singular";
    const double dinf = basis_dual_infeasibility(L, head, pb.Binv, pb.pi0);
    if (dinf > 1e-7) return "basis is not dual feasible";
    pb.head = head;
    double amax = 0.0;
    for (double v : pb.Binv) amax = std::max(amax, std::fabs(v));
    const double drop = 1e-14 * amax;
    pb.rptr.assign(1, 0);
    pb.rcol.clear(); pb.rval.clear();
    for (int i = 0; i < m; ++i) {
        for (int cc = 0; cc < m; ++cc) {
            const double v = pb.Binv[(size_t)i * m + cc];
            if (std::fabs(v) > drop) { pb.rcol.push_back(cc); pb.rval.push_back(v); }
        }
        pb.rptr.push_back((int)pb.rcol.size());
    }
    return nullptr;
}
static int make_pool_basis(twosd_ctx *c, const std::vector<int> &head, PoolBasis &pb) {
    const char *why = compute_pool_basis(c, head, pb);
    return why ? fail(TWOSD_E_ARG, "%s", why) : TWOSD_OK;
}

// pi0 = c_B' B^{-1} from the CSR rows (rows ascending)
static void pi0_from_rows(const twosd_ctx *c, PoolBasis &B) {
    const HostLP &L = c->L;
    const int m = L.m, n = L.n;
    B.pi0.assign(m, 0.0);
    for (int i = 0; i < m; ++i) {
        const int j = B.head[i];
        const double cb = j < n ? L.q[j] : 0.0;
        if (cb == 0.0) continue;
        for (int q = B.rptr[i]; q < B.rptr[i + 1]; ++q) B.pi0[B.rcol[q]] += cb * B.rval[q];
    }
}

// host CSR rows and pi0 of the bases a device refresh built (dev_only), read back from the
// pool arrays: upload_pool, prepare_elements and the host compose work on the host forms
static int ensure_host_pool(twosd_ctx *c) {
    if (int rc = materialize_heads(c)) return rc;
    const int P = (int)c->pool.size(), MP = c->MP, m = c->L.m;
    int last = -1;
    for (int p = 0; p < P; ++p)
        if (c->pool[p].dev_only) last = p;
    if (last < 0) return TWOSD_OK;
    const int Pd = last + 1;
    std::vector<int> rp((size_t)Pd * (MP + 1));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(rp.data(), c->d_brptr, sizeof(int) * rp.size(), hipMemcpyDeviceToHost));
    size_t nz = 0;
    for (int p = 0; p < Pd; ++p) nz = std::max(nz, (size_t)rp[(size_t)p * (MP + 1) + m]);
    std::vector<int> col(std::max<size_t>(nz, 1));
    std::vector<double> val(std::max<size_t>(nz, 1));
    if (nz) {
        HIPCHK(hipMemcpy(col.data(), c->d_brcol, sizeof(int) * nz, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(val.data(), c->d_brval, sizeof(double) * nz, hipMemcpyDeviceToHost));
    }
    parallel_for(Pd, [&](int p) {
        PoolBasis &B = c->pool[p];
        if (!B.dev_only) return;
        const int *r = rp.data() + (size_t)p * (MP + 1);
        B.rptr.resize(m + 1);
        for (int i = 0; i <= m; ++i) B.rptr[i] = r[i] - r[0];
        B.rcol.assign(col.begin() + r[0], col.begin() + r[m]);
        B.rval.assign(val.begin() + r[0], val.begin() + r[m]);
        pi0_from_rows(c, B);
        B.dev_only = false;
    });
    return TWOSD_OK;
}

// Upload the hypersparse-kernel form of every pool basis, pool-strided (pool[0] first, so
// the leading MP / 64 / 64C entries are the primary basis): hb0 (MP), basic0 (64),
// d0 (64C), B^{-1} columns as CSC (bcp absolute into the concatenated bci/bcv),
// B^{-1} rows as CSR (brptr absolute into the concatenated brcol/brval).
static int upload_pool(twosd_ctx *c) {
    const auto t_up0 = std::chrono::steady_clock::now();
    if (int rc0 = ensure_host_pool(c)) return rc0;
    const HostLP &L = c->L;
    const int m = L.m, n = L.n, MP = c->MP, P = (int)c->pool.size();
    std::vector<int8_t> bt(n + m);
    HIPCHK(hipMemcpy(bt.data(), c->d_btype, n + m, hipMemcpyDeviceToHost));
    std::vector<int> hb((size_t)P * MP, -1), bnnz(P, 0);
    std::vector<uint64_t> basic((size_t)P * 64, 0);
    // B^{-1} of every basis by rows (CSR) and by columns (CSC, rows ascending), both at the same
    // per-basis offset ro[p]; offsets are known up front, so every basis fills its part of the
    // concatenated arrays directly (default-initialised buffers, first touch in parallel)
    std::vector<size_t> ro(P + 1, 0);
    for (int p = 0; p < P; ++p) ro[p + 1] = ro[p] + c->pool[p].rcol.size();
    if (ro[P] > INT32_MAX) return fail(TWOSD_E_UNSUPPORTED, "basis pool too large (> 2^31 entries)");
    const size_t nz = std::max<size_t>(ro[P], 1);
    std::vector<int> rp_all((size_t)P * (MP + 1)), cp_all((size_t)P * (MP + 1));
    int *rc_all = stage_buf<int>(c, 0, nz), *ci_all = stage_buf<int>(c, 1, nz);
    double *rv_all = stage_buf<double>(c, 2, nz), *cv_all = stage_buf<double>(c, 3, nz);
    double *d0_all = stage_buf<double>(c, 4, (size_t)P * 64 * std::max(c->CH, 1));
    if (!rc_all || !ci_all || !rv_all || !cv_all || !d0_all) return fail(TWOSD_E_DEVICE, "pool upload: pinned staging allocation failed");
    parallel_for(P, [&](int p) {
        const PoolBasis &B = c->pool[p];
        std::vector<char> isb(n + m, 0);
        for (int i = 0; i < m; ++i) {
            hb[(size_t)p * MP + i] = B.head[i] * 4 + bt[B.head[i]];
            basic[(size_t)p * 64 + (B.head[i] & 63)] |= 1ull << (B.head[i] >> 6);
            isb[B.head[i]] = 1;
        }
        bnnz[p] = (int)B.rcol.size();
        const int base = (int)ro[p];
        for (int i = 0; i <= MP; ++i) rp_all[(size_t)p * (MP + 1) + i] = base + B.rptr[std::min(i, m)];
        std::copy(B.rcol.begin(), B.rcol.end(), rc_all + base);
        std::copy(B.rval.begin(), B.rval.end(), rv_all + base);
        // columns: counting sort of the row CSR (rows ascending within a column)
        std::vector<int> pos(m + 1, 0);
        for (int cc : B.rcol) ++pos[cc + 1];
        for (int cc = 0; cc < m; ++cc) pos[cc + 1] += pos[cc];
        for (int cc = 0; cc <= MP; ++cc) cp_all[(size_t)p * (MP + 1) + cc] = base + pos[std::min(cc, m)];
        for (int i = 0; i < m; ++i)
            for (int q = B.rptr[i]; q < B.rptr[i + 1]; ++q) {
                const int at = base + pos[B.rcol[q]]++;
                ci_all[at] = i;
                cv_all[at] = B.rval[q];
            }
        if (c->CH <= 0) return;
        double *d0 = d0_all + (size_t)p * 64 * c->CH;
        for (int j = 0; j < 64 * c->CH; ++j) {
            if (j >= n + m || isb[j]) { d0[j] = 0.0; continue; }
            double sum = 0.0;
            if (j >= n) sum = B.pi0[j - n];
            else
                for (int q = L.colptr[j]; q < L.colptr[j + 1]; ++q) sum += B.pi0[L.rowidx[q]] * L.val[q];
            d0[j] = (j < n ? L.q[j] : 0.0) - sum;
        }
    });
    const auto tc = std::chrono::steady_clock::now();
    int rc;
    if ((rc = upload_big(c, &c->d_hb0, hb)) || (rc = upload_big(c, &c->d_basic0, basic)) || (rc = upload_big(c, &c->d_bnnz, bnnz))) return rc;
    if (c->CH > 0) {
        if ((rc = upload_big(c, &c->d_bcp, cp_all)) || (rc = upload_big(c, &c->d_bci, ci_all, ro[P])) ||
            (rc = upload_big(c, &c->d_bcv, cv_all, ro[P])) || (rc = upload_big(c, &c->d_brptr, rp_all)) ||
            (rc = upload_big(c, &c->d_brcol, rc_all, ro[P])) || (rc = upload_big(c, &c->d_brval, rv_all, ro[P])) ||
            (rc = upload_big(c, &c->d_d0, d0_all, (size_t)P * 64 * c->CH)))
            return rc;
        c->b0_nnz = bnnz[0];
    }
    if (getenv("TWOSD_DEBUG")) {
        const auto td = std::chrono::steady_clock::now();
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "upload_pool P=%d: build %.1f ms, upload %.1f ms (%.1f MB, %zu nonzeros)\n", P, ms(t_up0, tc), ms(tc, td),
                (ro[P] * 24.0 + (size_t)P * 64 * std::max(c->CH, 0) * 8.0) / 1e6, ro[P]);
    }
    c->prep_valid = false;
    c->k_valid = false;
    reset_candidates(c);   // candidate lists refer to pool indices: rebuild after a change
    return TWOSD_OK;
}

static int install_basis(twosd_ctx *c, const std::vector<int> &head) {
    PoolBasis pb;
    int rc = make_pool_basis(c, head, pb);
    if (rc) return rc;
    c->head0 = head;
    c->pool.clear();
    c->sel_lo.clear();
    c->sel_hi.clear();
    c->box_epi = -1;
    c->pool.push_back(std::move(pb));
    if ((rc = upload_pool(c))) return rc;
    c->has_basis = true;
    return TWOSD_OK;
}

static bool same_basis(const std::vector<int> &a, const std::vector<int> &b) {
    std::vector<int> sa(a), sb(b);
    std::sort(sa.begin(), sa.end());
    std::sort(sb.begin(), sb.end());
    return sa == sb;
}

// append a basis to the pool; returns 1 if added, 0 if already present, < 0 on error
static int pool_add(twosd_ctx *c, const std::vector<int> &head, bool upload_now) {
    if (int rc = materialize_heads(c)) return rc;
    for (const PoolBasis &B : c->pool)
        if (same_basis(B.head, head)) return 0;
    PoolBasis pb;
    int rc = make_pool_basis(c, head, pb);
    if (rc) return rc;
    std::vector<double>().swap(pb.Binv);
    c->pool.push_back(std::move(pb));
    if (upload_now && (rc = upload_pool(c))) return rc;
    return 1;
}

extern "C" int twosd_compute_basis(twosd_ctx *c, const double *x, const double *values) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "compute_basis: no template");
    HIPCHK(hipSetDevice(c->device));
    std::vector<double> dv(c->k, 0.0);
    if (values)
        for (int e = 0; e < c->k; ++e) dv[e] = values[e] - template_value(c, e);
    std::vector<double> b;
    rhs_at(c, x, values ? dv.data() : nullptr, b);
    std::vector<int> head;
    double obj = 0;
    int iters = 0;
    std::string err;
    const int st = setup_solve(c->L, b, head, obj, iters, err);
    if (st != TWOSD_LP_OPTIMAL) return fail(TWOSD_E_LP, "compute_basis: %s (status %d)", err.c_str(), st);
    return install_basis(c, head);
}

extern "C" int twosd_set_basis(twosd_ctx *c, const int *head) {
    if (!c || !c->has_template || !head) return fail(TWOSD_E_STATE, "set_basis: no template / NULL head");
    HIPCHK(hipSetDevice(c->device));
    return install_basis(c, std::vector<int>(head, head + c->L.m));
}

extern "C" int twosd_get_basis(twosd_ctx *c, int *head) {
    if (!c || !c->has_basis || !head) return fail(TWOSD_E_STATE, "get_basis: no basis");
    std::copy(c->head0.begin(), c->head0.end(), head);
    return TWOSD_OK;
}

extern "C" int twosd_pool_add_basis(twosd_ctx *c, const int *head, int *added) {
    if (!c || !c->has_basis || !head) return fail(TWOSD_E_STATE, "pool_add_basis: no primary basis / NULL head");
    HIPCHK(hipSetDevice(c->device));
    const int rc = pool_add(c, std::vector<int>(head, head + c->L.m), true);
    if (rc < 0) return rc;
    if (added) *added = rc;
    return TWOSD_OK;
}

extern "C" int twosd_pool_size(twosd_ctx *c, int *size) {
    if (!c || !size) return fail(TWOSD_E_ARG, "pool_size: NULL argument");
    *size = (int)c->pool.size();
    return TWOSD_OK;
}

extern "C" int twosd_pool_get(twosd_ctx *c, int p, int *head) {
    if (c && !c->has_basis) return fail(TWOSD_E_STATE, "pool_get: no basis");
    if (!c || !head || p < 0 || p >= (int)c->pool.size()) return fail(TWOSD_E_ARG, "pool_get: basis %d of %zu", p, c ? c->pool.size() : 0);
    const std::vector<int> *h = nullptr;
    if (int rc = head_of(c, p, &h)) return rc;
    std::copy(h->begin(), h->end(), head);
    return TWOSD_OK;
}

static int64_t pivots_of_last_lp(twosd_ctx *c, int N) {
    std::vector<int> its(N);
    if (hipMemcpy(its.data(), c->d_iters, sizeof(int) * N, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    int64_t sum = 0;
    for (int v : its) sum += v;
    return sum;
}

// Grow the pool from training scenarios [first, first + count) of epigraph epi at x.  The
// first half harvests: solved from the current pool, its optimal bases are added in order
// of decreasing frequency (ties: first occurrence) up to max_pool bases.  The second half
// validates: the grown pool is kept only if it solves those scenarios in fewer pivots.
extern "C" int twosd_pool_build(twosd_ctx *c, int epi, const double *x, int first, int count, int max_pool,
                                int *pool_size) {
    if (!c || !c->has_basis) return fail(TWOSD_E_STATE, "pool_build: no primary basis");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "pool_build: epigraph %d does not exist", epi);
    const EpiDevice &E = c->epis[epi];
    if (first < 0 || count < 0 || first + count > E.count || max_pool < 1 || (c->n1 > 0 && !x))
        return fail(TWOSD_E_ARG, "pool_build: bad arguments");
    if (pool_select_lds_bytes(c->k) + 17 * 1024 > 160 * 1024)   // + the selection kernels' static LDS
        return fail(TWOSD_E_UNSUPPORTED, "pool_build: k = %d random elements too many for pool selection", c->k);
    HIPCHK(hipSetDevice(c->device));
    const int m = c->L.m;
    const int nh = count / 2, nv = count - nh;
    if (count > 0 && c->k > 0) {   // training box of the deltas (selection row pruning)
        std::vector<double> dv((size_t)count * c->k);
        HIPCHK(hipMemcpy(dv.data(), E.d_dv + (size_t)first * c->k, sizeof(double) * dv.size(), hipMemcpyDeviceToHost));
        c->box_epi = -1;   // the refresh's cached box no longer applies
        c->sel_lo.assign(c->k, INFINITY);
        c->sel_hi.assign(c->k, -INFINITY);
        for (int s = 0; s < count; ++s)
            for (int e = 0; e < c->k; ++e) {
                c->sel_lo[e] = std::min(c->sel_lo[e], dv[(size_t)s * c->k + e]);
                c->sel_hi[e] = std::max(c->sel_hi[e], dv[(size_t)s * c->k + e]);
            }
        c->prep_valid = false;
    }
    if (nh > 0 && (int)c->pool.size() < max_pool) {
        const double *dh = E.d_dv + (size_t)first * c->k, *dval = dh + (size_t)nh * c->k;
        int rc;
        if ((rc = run_lp(c, x, dval, nv, false, false))) return rc;
        const int64_t piv0 = pivots_of_last_lp(c, nv);
        c->want_head = true;
        rc = run_lp(c, x, dh, nh, false, false);
        c->want_head = false;
        if (rc) return rc;
        std::vector<int> heads((size_t)nh * m), st(nh);
        HIPCHK(hipMemcpy(heads.data(), c->d_head_out, sizeof(int) * heads.size(), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(st.data(), c->d_status, sizeof(int) * nh, hipMemcpyDeviceToHost));
        std::map<std::vector<int>, std::pair<int, int>> freq;   // sorted head -> (count, first scenario)
        if ((rc = materialize_heads(c))) return rc;
        for (const PoolBasis &B : c->pool) {
            std::vector<int> key(B.head);
            std::sort(key.begin(), key.end());
            freq[key] = {0, -1};                                 // already in the pool
        }
        for (int s = 0; s < nh; ++s) {
            if (st[s] != TWOSD_LP_OPTIMAL) continue;
            std::vector<int> key(heads.begin() + (size_t)s * m, heads.begin() + (size_t)(s + 1) * m);
            std::sort(key.begin(), key.end());
            auto it = freq.find(key);
            if (it == freq.end()) freq.emplace(std::move(key), std::make_pair(1, s));
            else if (it->second.second >= 0) ++it->second.first;
        }
        std::vector<std::pair<int, int>> order;   // (-count, first scenario)
        for (auto &kv : freq)
            if (kv.second.second >= 0) order.push_back({-kv.second.first, kv.second.second});
        std::sort(order.begin(), order.end());
        const size_t old_size = c->pool.size();
        // candidates are distinct and new; their inverses are computed in parallel, and a
        // candidate that fails validation (numerically singular / dual infeasible) is skipped
        const size_t want = std::min(order.size(), (size_t)max_pool - old_size);
        std::vector<PoolBasis> cand(want);
        std::vector<int> ok(want, 0);
        const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nth; ++t)
            th.emplace_back([&, t]() {
                for (size_t a = t; a < want; a += nth) {
                    const int s = order[a].second;
                    std::vector<int> head(heads.begin() + (size_t)s * m, heads.begin() + (size_t)(s + 1) * m);
                    ok[a] = compute_pool_basis(c, head, cand[a]) == nullptr;
                    std::vector<double>().swap(cand[a].Binv);   // sparse forms kept; dense m x m only for the primary
                }
            });
        for (auto &t : th) t.join();
        for (size_t a = 0; a < want; ++a)
            if (ok[a]) c->pool.push_back(std::move(cand[a]));
        if (c->pool.size() > old_size) {
            if ((rc = upload_pool(c))) return rc;
            if ((rc = run_lp(c, x, dval, nv, false, false))) return rc;
            const int64_t piv1 = pivots_of_last_lp(c, nv);
            std::vector<int> st2(nv);
            HIPCHK(hipMemcpy(st2.data(), c->d_status, sizeof(int) * nv, hipMemcpyDeviceToHost));
            const bool all_ok = std::all_of(st2.begin(), st2.end(), [](int v) { return v == TWOSD_LP_OPTIMAL; });
            if (piv1 < 0 || piv0 < 0 || piv1 >= piv0 || !all_ok) {   // no gain: back to the old pool
                c->pool.resize(old_size);
                if ((rc = upload_pool(c))) return rc;
            }
        }
    }
    if (pool_size) *pool_size = (int)c->pool.size();
    return TWOSD_OK;
}

static int select_pool(twosd_ctx *c, const double *d_dv, int N, int *d_pick, int npool_override);
static int prepare_elements(twosd_ctx *c);

// ---- pool refresh at x: the pool's bases are optimal near the x they were harvested at
// (storm: 8.9 pivots per scenario at the training x, 28-67 at SD candidates 25-37 % away), so a
// new x gets a pool of its own.  B^{-1} of a harvested basis is composed from its start basis
// and the eta file of its solve, B^{-1} = E_K..E_1 B_pb^{-1} (sparse row merges), so no
// refactorisation: the cost is the training solves plus O(K nnz) host work per basis.

// pi0 = c_B' B^{-1} from the composed rows, then the checks of host_basis.cpp; nullptr if the
// basis is usable
static const char *finish_composed(const twosd_ctx *c, PoolBasis &B) {
    const HostLP &L = c->L;
    pi0_from_rows(c, B);
    if (sparse_dual_infeasibility(L, B.head, B.pi0) > 1e-7) return "composed basis is not dual feasible";
    if (sparse_basis_residual(L, B.head, B.rptr, B.rcol, B.rval, 4) > 1e-8) return "composed B^{-1} inconsistent";
    return nullptr;
}

// Device build of the refreshed pool (pool_gpu.hip) from the eta files and heads of the
// training solves (rows = training scenarios in c->d_eo_* / c->d_head_out; the representatives
// in c->d_refresh_sel).  Two phases:
//   pg_compute   sources a = 0 (primary), a = 1..R (eta-file row d_refresh_sel[a - 1]) composed
//                column by column into an intermediate CSC and checked (d_pg_* arrays);
//   pg_assemble  the sources listed in `order` that passed the checks become pool[0..P), in
//                that order: the arrays upload_pool + prepare_elements would produce.
// The single-GPU refresh runs both on one source table; the distributed refresh
// (twosd_refresh_*) runs pg_compute on each rank's own representatives and pg_assemble on the
// table all ranks gathered.

// workspace + PgArgs of a compute over nsrc sources (the template and start-pool fields)
static int pg_args(twosd_ctx *c, int nsrc, PgArgs &A) {
    const HostLP &L = c->L;
    const int m = L.m;
    int rc;
    if ((rc = dev_reserve(c, &c->d_pg_pos, (size_t)std::max(c->k, 1))) || (rc = dev_reserve(c, &c->d_pg_amax, (size_t)nsrc)) ||
        (rc = dev_reserve(c, &c->d_pg_cnt, (size_t)4 * nsrc * m)) || (rc = dev_reserve(c, &c->d_pg_tot, (size_t)5 * nsrc)) ||
        (rc = dev_reserve(c, &c->d_pg_valid, (size_t)nsrc)) || (rc = dev_reserve(c, &c->d_pg_head0, (size_t)m)) ||
        (rc = dev_reserve(c, &c->d_pg_d0p, (size_t)64 * c->CH)) || (rc = dev_reserve(c, &c->d_pg_ioff, (size_t)nsrc)))
        return rc;
    HIPCHK(hipMemcpyAsync(c->d_pg_head0, c->head0.data(), sizeof(int) * m, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_pg_d0p, c->d_d0, sizeof(double) * 64 * c->CH, hipMemcpyDeviceToDevice, c->stream));
    if (c->k) HIPCHK(hipMemcpyAsync(c->d_pg_pos, c->pos_row.data(), sizeof(int) * c->k, hipMemcpyHostToDevice, c->stream));
    A = PgArgs{};
    A.m = m; A.n = L.n; A.MP = c->MP; A.CH = c->CH; A.R9 = c->R; A.k = c->k; A.kmax = c->eo_kmax;
    A.npool_old = (int)c->pool.size();
    A.colptr = c->d_colptr; A.rowidx = c->d_rowidx; A.val = c->d_val; A.q = c->d_q; A.btype = c->d_btype;
    A.pos_row = c->d_pg_pos;
    A.bcp0 = c->d_bcp; A.bci0 = c->d_bci; A.bcv0 = c->d_bcv;
    A.eo_pb = c->d_eo_pb; A.eo_K = c->d_eo_K; A.eo_off = c->d_eo_off; A.eo_etap = c->d_eo_etap;
    A.eo_etaoff = c->d_eo_etaoff; A.eo_eidx = c->d_eo_eidx; A.eo_evals = c->d_eo_evals;
    A.head0 = c->d_pg_head0; A.heads = c->d_head_out; A.src_row = c->d_refresh_sel;
    A.a0 = 0;
    A.amax = c->d_pg_amax;
    A.nzc = c->d_pg_cnt; A.keptc = c->d_pg_cnt + (size_t)nsrc * m;
    A.rowcnt = c->d_pg_cnt + (size_t)2 * nsrc * m; A.erowcnt = c->d_pg_cnt + (size_t)3 * nsrc * m;
    A.tot = c->d_pg_tot; A.nztot = c->d_pg_tot + (size_t)4 * nsrc; A.valid = c->d_pg_valid;
    return TWOSD_OK;
}

// compute phase over sources [0, nsrc): FTRAN passes + counts and checks; the per-source
// totals (4 each), nonzero counts and validity are read back into h_tot / h_nz / h_valid
// (pinned staging), the intermediate offsets prefixed into A.inter_off
static int pg_compute(twosd_ctx *c, int nsrc, PgArgs &A, int **h_tot, int **h_valid, long long *inz_out, bool dbg) {
    int rc;
    if ((rc = pg_args(c, nsrc, A))) return rc;
    // the first pass keeps each source's nonzeros (up to sc_cap entries, sized from the last
    // build's largest source; at most 1.5 GiB in all) for pg_gather_kernel: one FTRAN per
    // column instead of two; a source past sc_cap runs the second FTRAN pass
    const int m = c->L.m;
    long long cap = c->pg_sc_cap > 0 ? c->pg_sc_cap : std::min<long long>((long long)m * m, 16384);
    if (getenv("TWOSD_PG_NOSCRATCH")) cap = 0;   // A/B knob: two FTRAN passes
    if (const char *e = getenv("TWOSD_PG_SCCAP")) cap = atoll(e);   // test hook: sources past it take pass 1
    cap = std::min(cap, ((3LL << 29) / 12) / std::max(nsrc, 1));
    if (cap > 0 && ((rc = dev_reserve(c, &c->d_pg_scrow, (size_t)nsrc * cap)) || (rc = dev_reserve(c, &c->d_pg_scval, (size_t)nsrc * cap)) ||
                    (rc = dev_reserve(c, &c->d_pg_scoff, (size_t)nsrc * m))))
        return rc;
    A.sc_cap = cap; A.sc_row = c->d_pg_scrow; A.sc_val = c->d_pg_scval; A.sc_off = c->d_pg_scoff;
    HIPCHK(pg_launch_ftran(A, 0, nsrc, c->stream));
    int *h_nz = stage_buf<int>(c, 11, (size_t)nsrc);
    long long *h_ioff = stage_buf<long long>(c, 12, (size_t)nsrc);
    if (!h_nz || !h_ioff) return fail(TWOSD_E_DEVICE, "pool refresh: pinned staging allocation failed");
    HIPCHK(hipMemcpyAsync(h_nz, A.nztot, sizeof(int) * nsrc, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    long long inz = 0, nzmax = 0;
    int over = 0;
    for (int a = 0; a < nsrc; ++a) {
        h_ioff[a] = inz;
        inz += h_nz[a];
        nzmax = std::max<long long>(nzmax, h_nz[a]);
        over += h_nz[a] > cap;
    }
    if ((rc = dev_reserve(c, &c->d_pg_irow, (size_t)inz)) || (rc = dev_reserve(c, &c->d_pg_ival, (size_t)inz))) return rc;
    HIPCHK(hipMemcpyAsync(c->d_pg_ioff, h_ioff, sizeof(long long) * nsrc, hipMemcpyHostToDevice, c->stream));
    A.inter_off = c->d_pg_ioff; A.inter_row = c->d_pg_irow; A.inter_val = c->d_pg_ival;
    if (cap > 0) HIPCHK(pg_launch_gather(A, nsrc, c->stream));
    if (over || cap == 0) HIPCHK(pg_launch_ftran(A, 1, nsrc, c->stream));
    c->pg_sc_cap = std::max<long long>(1024, nzmax + nzmax / 2);   // the next build's scratch
    HIPCHK(pg_launch_count(A, nsrc, c->stream));
    int *ht = stage_buf<int>(c, 9, (size_t)5 * nsrc);
    if (!ht) return fail(TWOSD_E_DEVICE, "pool refresh: pinned staging allocation failed");
    HIPCHK(hipMemcpyAsync(ht, c->d_pg_tot, sizeof(int) * 4 * nsrc, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(ht + (size_t)4 * nsrc, c->d_pg_valid, sizeof(int) * nsrc, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (dbg) fprintf(stderr, "pg_compute: %d sources, %lld intermediate entries, largest %lld, %d past the scratch of %lld\n", nsrc, inz,
                     nzmax, over, cap);
    *h_tot = ht;
    *h_valid = ht + (size_t)4 * nsrc;
    *inz_out = inz;
    return TWOSD_OK;
}

// assemble phase: pool = the sources of `order` (order[0] = 0, the primary) that passed, in
// order; A describes the source table (compute output or the gathered table)
static int pg_assemble(twosd_ctx *c, PgArgs &A, const int *h_tot, const int *h_valid, const std::vector<int> &order) {
    const HostLP &L = c->L;
    const int m = L.m, MP = c->MP;
    int rc;
    if (order.empty() || order[0] != 0 || !h_valid[0]) return 1;   // the primary failed the device checks: host path
    std::vector<int> map, off;
    std::vector<int64_t> acc(4, 0);
    for (int a : order) {
        if (!h_valid[a]) continue;
        map.push_back(a);
        for (int f = 0; f < 4; ++f) {
            off.push_back((int)acc[f]);
            acc[f] += h_tot[(size_t)a * 4 + f];
        }
        if (acc[0] > INT32_MAX || acc[1] > INT32_MAX || acc[2] * 64 > INT32_MAX || acc[3] > INT32_MAX)
            return fail(TWOSD_E_UNSUPPORTED, "basis pool too large (> 2^31 entries)");
    }
    const int P = (int)map.size();
    const bool dbg = getenv("TWOSD_DEBUG") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    if ((rc = dev_reserve(c, &c->d_pg_map, (size_t)P)) || (rc = dev_reserve(c, &c->d_pg_off, (size_t)4 * P))) return rc;
    // From here the live pool arrays are grown in place (a grown array does not keep its
    // contents) and then overwritten: a failure past this point leaves c->pool describing
    // arrays that no longer hold it.  The context then drops its basis, so every later solve
    // fails cleanly (TWOSD_E_STATE) until twosd_compute_basis / twosd_set_basis installs one.
    // the device-built bases read their heads lazily from pool_hb, which the failing path may
    // have reallocated or overwritten: keep only the primary (a host basis)
    auto broken = [c](int code) { return drop_pool(c, code); };
    if (const char *inj = getenv("TWOSD_INJECT_FAIL"); inj && !strcmp(inj, "refresh_fill"))   // test hook
        return broken(fail(TWOSD_E_DEVICE, "pool refresh: injected failure after the pool-array reservation"));
    HIPCHK(hipMemcpyAsync(c->d_pg_map, map.data(), sizeof(int) * P, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_pg_off, off.data(), sizeof(int) * 4 * P, hipMemcpyHostToDevice, c->stream));
    const size_t nz = (size_t)acc[0], kz = (size_t)acc[1], ez = (size_t)acc[2] * 64;
    if ((rc = dev_reserve(c, &c->d_brptr, (size_t)P * (MP + 1))) || (rc = dev_reserve(c, &c->d_brcol, nz)) ||
        (rc = dev_reserve(c, &c->d_brval, nz)) || (rc = dev_reserve(c, &c->d_bcp, (size_t)P * (MP + 1))) ||
        (rc = dev_reserve(c, &c->d_bci, nz)) || (rc = dev_reserve(c, &c->d_bcv, nz)) ||
        (rc = dev_reserve(c, &c->d_kp, (size_t)P * (m + 1))) || (rc = dev_reserve(c, &c->d_ke, kz)) ||
        (rc = dev_reserve(c, &c->d_kraw, kz)) || (rc = dev_reserve(c, &c->d_kslot, (size_t)P * (c->R + 1))) ||
        (rc = dev_reserve(c, &c->d_kix, ez)) || (rc = dev_reserve(c, &c->d_kv, ez)) ||
        (rc = dev_reserve(c, &c->d_hb0, (size_t)P * MP)) || (rc = dev_reserve(c, &c->d_basic0, (size_t)P * 64)) ||
        (rc = dev_reserve(c, &c->d_bnnz, (size_t)P)) || (rc = dev_reserve(c, &c->d_d0, (size_t)P * 64 * c->CH)) ||
        (rc = dev_reserve(c, &c->d_sel_ptr, (size_t)P + 1)) || (rc = reserve_selection(c, P, (int)acc[3])))
        return broken(rc);
    // (a grown array is reallocated: the start pool's CSC was read only by the FTRAN passes)
    PgFill F{};
    F.P = P; F.map = c->d_pg_map; F.off = c->d_pg_off; F.sel_total = (int)acc[3]; F.d0_primary = c->d_pg_d0p;
    F.brptr = c->d_brptr; F.brcol = c->d_brcol; F.brval = c->d_brval; F.bcp = c->d_bcp; F.bci = c->d_bci; F.bcv = c->d_bcv;
    F.kp = c->d_kp; F.ke = c->d_ke; F.kraw = c->d_kraw; F.kslot = c->d_kslot; F.kix = c->d_kix; F.kv = c->d_kv;
    F.hb0 = c->d_hb0; F.basic0 = c->d_basic0; F.bnnz = c->d_bnnz; F.d0 = c->d_d0; F.sel_ptr = c->d_sel_ptr;
    F.P0 = 0;
    if (pg_launch_fill(A, F, P, c->stream) != hipSuccess) return broken(fail(TWOSD_E_DEVICE, "pool refresh: fill launch failed"));
    // the pool's heads (hb0 = 4 head + type) stay on the device; a host head is fetched on first
    // use (head_of)
    c->pool_hb_valid = false;
    const auto t1 = std::chrono::steady_clock::now();
    // host pool: the primary keeps its host forms; the new bases refer to their head rows
    std::vector<PoolBasis> keep(P);
    keep[0] = std::move(c->pool[0]);
    for (int p = 1; p < P; ++p) {
        keep[p].hb_row = p;
        keep[p].dev_only = true;
    }
    c->pool.swap(keep);
    std::thread([old = std::move(keep)]() mutable { old.clear(); }).detach();
    c->b0_nnz = h_tot[0];
    c->prep_valid = false;
    c->k_valid = true;
    reset_candidates(c);
    if (dbg) {
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "pg_assemble: P=%d fill + heads %.2f ms, host pool %.2f ms\n", P, ms(t0, t1),
                ms(t1, std::chrono::steady_clock::now()));
    }
    return TWOSD_OK;
}

// Returns 1, with the pool unchanged, when the LDS layouts do not fit or the primary fails the
// device checks (the caller then composes on the host).
static int refresh_build_device(twosd_ctx *c, const std::vector<int> &sel) {
    const int R = (int)sel.size();
    if (!pg_supported(c->L.m, c->L.n, c->eo_kmax)) return 1;
    const bool dbg = getenv("TWOSD_DEBUG") != nullptr;
    PgArgs A;
    int *h_tot = nullptr, *h_valid = nullptr;
    long long inz = 0;
    int rc;
    if ((rc = pg_compute(c, R + 1, A, &h_tot, &h_valid, &inz, dbg))) return rc;
    std::vector<int> order(R + 1);
    for (int a = 0; a <= R; ++a) order[a] = a;
    return pg_assemble(c, A, h_tot, h_valid, order);
}

// pivot cap of the training solves of a refresh.  One wavefront solves one scenario, so a
// training launch lasts as long as its slowest scenario; the scenarios far from the current
// pool (tens of pivots) mostly end at rare bases.  Auto: 3 x the mean pivots of the last large
// batch, at least 32 (storm: 32-33; ssn, ~33 pivots a solve: ~100); none before any batch.
// Storm 1M, 4096-basis pool (profiles/r03/train_kcap_1M.txt): cap 32 vs none -- refresh
// 18.3 vs 25.6 ms, and the next solve 86.6 vs 108.5 ms (fewer pivots from the capped pool).
// The one statement of the rule (twosd_training_cap exposes it to the distributed refresh, which
// applies it to the all-reduced pivot sum and size of every rank): setting = TWOSD_TRAIN_KCAP if
// set, else the context's (twosd_set_refresh_kcap); > 0 that cap, < 0 none, 0 auto =
// max(32, ceil(3 sum / n)) in integers, none before any large batch.
static int training_cap_rule(const twosd_ctx *c, int64_t sum, int64_t n) {
    const char *e = getenv("TWOSD_TRAIN_KCAP");   // A/B knob
    const int setting = e ? atoi(e) : (c ? c->train_kcap : 0);
    if (setting > 0) return setting;
    if (setting < 0 || n <= 0 || sum <= 0) return 0;
    const int64_t q = (3 * sum + n - 1) / n;
    return (int)std::max<int64_t>(32, std::min<int64_t>(q, INT32_MAX));
}
static int train_kcap(const twosd_ctx *c) { return training_cap_rule(c, c->piv_ref_sum, c->piv_ref_n); }

// The training solves of a refresh (basis keys, eta files, final heads) under the pivot cap.  The
// auto cap follows the last batch's pivots at the previous x; when x moved far from the pool's x
// (bench with warmup 4: the x_EV pool trained from the primary basis, next x SD candidate 4 --
// 58.5 pivots a scenario against a cap of 35), most training scenarios hit the cap and the
// refresh would find almost no optimal bases.  If fewer than half end optimal, the training is
// solved again without a cap (one extra launch, only on such a jump).
static int refresh_training(twosd_ctx *c, const double *x, const double *d_dv, int count, int kcap, bool retry, int *n_opt) {
    LpRun o;
    o.want_bkey = true;
    o.want_etas = true;
    o.want_head = true;
    // training scenarios beyond the pivot cap only drop out of the basis count (one launch
    // lasts as long as its slowest scenario: with one scenario per wave the cap bounds it)
    o.kcap = kcap;
    int rc;
    if ((rc = run_lp_ex(c, x, d_dv, count, o))) return rc;
    int opt = count;
    if (o.kcap > 0) {
        std::vector<int> st(count);
        HIPCHK(hipMemcpy(st.data(), c->d_status, sizeof(int) * count, hipMemcpyDeviceToHost));
        opt = (int)std::count(st.begin(), st.end(), (int)TWOSD_LP_OPTIMAL);
        if (retry && 2 * opt < count) {
            if (getenv("TWOSD_DEBUG")) fprintf(stderr, "refresh training: %d of %d optimal under cap %d, solved again uncapped\n", opt, count, o.kcap);
            o.kcap = 0;
            if ((rc = run_lp_ex(c, x, d_dv, count, o))) return rc;
        }
    }
    c->last_train_opt = opt;
    if (n_opt) *n_opt = opt;
    return TWOSD_OK;
}

extern "C" int twosd_pool_refresh(twosd_ctx *c, int epi, const double *x, int first, int count, int max_pool,
                                  int *pool_size) {
    if (!c || !c->has_basis) return fail(TWOSD_E_STATE, "pool_refresh: no primary basis");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "pool_refresh: epigraph %d does not exist", epi);
    const EpiDevice &E = c->epis[epi];
    if (first < 0 || count < 1 || first + count > E.count || max_pool < 1 || (c->n1 > 0 && !x))
        return fail(TWOSD_E_ARG, "pool_refresh: bad arguments");
    if (c->CH <= 0) return fail(TWOSD_E_UNSUPPORTED, "pool_refresh: needs the hypersparse LP kernel");
    HIPCHK(hipSetDevice(c->device));
    const auto t0 = std::chrono::steady_clock::now();
    const int m = c->L.m;
    const double *d_dv = E.d_dv + (size_t)first * c->k;
    int rc;
    // 1. training solves at x from the current pool: basis keys, eta files and heads by scenario
    if ((rc = refresh_training(c, x, d_dv, count, train_kcap(c), true, nullptr))) return rc;
    if (getenv("TWOSD_DEBUG")) {
        std::vector<int> st(count), itv(count);
        HIPCHK(hipMemcpy(st.data(), c->d_status, sizeof(int) * count, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(itv.data(), c->d_iters, sizeof(int) * count, hipMemcpyDeviceToHost));
        int h[8] = {0};
        long long itsum = 0;
        for (int s2 = 0; s2 < count; ++s2) { h[std::min(std::max(st[s2], 0), 7)]++; itsum += itv[s2]; }
        fprintf(stderr, "pool_refresh training: kcap %d (ref %.2f), pool %zu, statuses 0:%d 1:%d 2:%d 3:%d 4:%d 5+:%d, mean iters %.2f\n",
                train_kcap(c), c->piv_mean_ref, c->pool.size(), h[0], h[1], h[2], h[3], h[4], h[5] + h[6] + h[7], (double)itsum / count);
    }
    const auto t1 = std::chrono::steady_clock::now();
    // 2. distinct optimal bases, most frequent first (ties: first occurrence), primary excluded
    const int *d_list = nullptr, *d_counts = nullptr;
    int U = 0;
    if ((rc = vkey_first_occurrences(c, count, c->d_bkey, c->d_status, &d_list, &U, &d_counts))) return rc;
    std::vector<int> reps(U), cnts(U);
    if (U > 0) {
        HIPCHK(hipMemcpy(reps.data(), d_list, sizeof(int) * U, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(cnts.data(), d_counts, sizeof(int) * U, hipMemcpyDeviceToHost));
    }
    const auto t1b = std::chrono::steady_clock::now();
    std::vector<int> ord(U);
    for (int a = 0; a < U; ++a) ord[a] = a;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return cnts[a] > cnts[b]; });
    const int R = std::min(U, max_pool - 1);
    std::vector<int> sel(R);
    for (int a = 0; a < R; ++a) sel[a] = reps[ord[a]];
    std::vector<PoolBasis> fresh;
    bool device_built = false;
    c->last_refresh_ms[1] = std::chrono::duration<double, std::milli>(t1b - t1).count();
    c->last_refresh_ms[2] = c->last_refresh_ms[3] = 0.0;
    if (R > 0 && !getenv("TWOSD_REFRESH_HOST")) {
        // 3. B^{-1} of the representatives from their eta files, and the pool arrays, on the device
        if ((size_t)R > c->refresh_sel_cap) {
            if ((rc = dalloc(&c->d_refresh_sel, (size_t)R))) return rc;
            c->refresh_sel_cap = R;
        }
        HIPCHK(hipMemcpyAsync(c->d_refresh_sel, sel.data(), sizeof(int) * R, hipMemcpyHostToDevice, c->stream));
        const int dev = refresh_build_device(c, sel);
        if (dev < 0) return dev;
        device_built = dev == 0;
        c->last_refresh_ms[2] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1b).count();
    }
    if (R > 0 && !device_built) {
        // 3'. host path: compose on the host threads, then upload_pool + prepare_elements
        if ((rc = ensure_host_pool(c))) return rc;   // start bases in host form
        const int kmax = c->eo_kmax;
        std::vector<int> pb(count), K(count), off(count), etap((size_t)count * kmax), etaoff((size_t)count * (kmax + 1)),
            heads((size_t)count * m);
        int used = 0;
        HIPCHK(hipMemcpy(pb.data(), c->d_eo_pb, sizeof(int) * count, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(K.data(), c->d_eo_K, sizeof(int) * count, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(off.data(), c->d_eo_off, sizeof(int) * count, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(etap.data(), c->d_eo_etap, sizeof(int) * etap.size(), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(etaoff.data(), c->d_eo_etaoff, sizeof(int) * etaoff.size(), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(heads.data(), c->d_head_out, sizeof(int) * heads.size(), hipMemcpyDeviceToHost));
        unsigned long long used64 = 0;
        HIPCHK(hipMemcpy(&used64, c->d_eo_used, sizeof(used64), hipMemcpyDeviceToHost));
        used = (int)std::min<unsigned long long>(used64, std::min<size_t>(c->eo_cap, INT32_MAX));
        std::vector<int> ei(std::max(used, 1));
        std::vector<double> ev(std::max(used, 1));
        if (used > 0) {
            HIPCHK(hipMemcpy(ei.data(), c->d_eo_eidx, sizeof(int) * used, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(ev.data(), c->d_eo_evals, sizeof(double) * used, hipMemcpyDeviceToHost));
        }
        const auto t2 = std::chrono::steady_clock::now();
        fresh.resize(R);
        std::vector<char> ok(R, 0);
        const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nth; ++t)
            th.emplace_back([&, t]() {
                for (int a = (int)t; a < R; a += (int)nth) {
                    const int l = sel[a];   // eta-file row: the training scenario
                    if (K[l] < 0 || pb[l] < 0 || pb[l] >= (int)c->pool.size()) continue;
                    PoolBasis &B = fresh[a];
                    B.head.assign(heads.begin() + (size_t)l * m, heads.begin() + (size_t)(l + 1) * m);
                    const int *eo = etaoff.data() + (size_t)l * (kmax + 1);
                    const PoolBasis &B0 = c->pool[pb[l]];
                    compose_binv(m, B0.rptr, B0.rcol, B0.rval, K[l], etap.data() + (size_t)l * kmax, eo, ei.data() + off[l],
                                 ev.data() + off[l], B.rptr, B.rcol, B.rval);
                    ok[a] = finish_composed(c, B) == nullptr;
                }
            });
        for (auto &t : th) t.join();
        c->last_refresh_ms[2] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count();
        std::vector<PoolBasis> keep;
        keep.reserve(R + 1);
        keep.push_back(std::move(c->pool[0]));   // the primary basis stays pool[0]
        for (int a = 0; a < R; ++a)
            if (ok[a]) keep.push_back(std::move(fresh[a]));
        c->pool.swap(keep);
        // the old pool's host data is released on a helper thread (thousands of vectors)
        std::thread([old = std::move(keep)]() mutable { old.clear(); }).detach();
    }
    // R == 0 (no training scenario optimal): the current pool stays (any pool basis is a valid
    // start; dropping to the primary basis alone would cost ~90 pivots a scenario)
    const auto tb = std::chrono::steady_clock::now();
    // training box of the deltas (selection row pruning), as twosd_pool_build; cached per
    // training range
    if (c->k > 0 && !(c->box_epi == epi && c->box_first == first && c->box_count == count && c->box_n == E.count)) {
        c->box_epi = epi; c->box_first = first; c->box_count = count; c->box_n = E.count;
        std::vector<double> dv((size_t)count * c->k);
        HIPCHK(hipMemcpy(dv.data(), d_dv, sizeof(double) * dv.size(), hipMemcpyDeviceToHost));
        c->sel_lo.assign(c->k, INFINITY);
        c->sel_hi.assign(c->k, -INFINITY);
        for (int s2 = 0; s2 < count; ++s2)
            for (int e = 0; e < c->k; ++e) {
                c->sel_lo[e] = std::min(c->sel_lo[e], dv[(size_t)s2 * c->k + e]);
                c->sel_hi[e] = std::max(c->sel_hi[e], dv[(size_t)s2 * c->k + e]);
            }
    }
    const auto tu = std::chrono::steady_clock::now();
    const bool host_built = R > 0 && !device_built;   // R == 0: the pool is unchanged
    if (host_built && (rc = upload_pool(c))) return rc;
    const auto tua = std::chrono::steady_clock::now();
    if (host_built && (rc = prepare_elements(c))) return rc;
    const auto t3 = std::chrono::steady_clock::now();
    if (getenv("TWOSD_DEBUG")) {
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "pool_refresh: train %.2f, keys %.2f, build %.2f, box %.2f, upload_pool %.2f, elements %.2f ms (R=%d)\n",
                ms(t0, t1), ms(t1, t1b), ms(t1b, tb), ms(tb, tu), ms(tu, tua), ms(tua, t3), R);
    }
    c->last_refresh_ms[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    c->last_refresh_ms[3] = std::chrono::duration<double, std::milli>(t3 - tu).count();
    c->last_refresh_ms[4] = std::chrono::duration<double, std::milli>(t3 - t0).count();
    if (pool_size) *pool_size = (int)c->pool.size();
    return TWOSD_OK;
}

// ---- distributed pool refresh -------------------------------------------------------------
// The refresh of twosd_pool_refresh split over the ranks (one process per GPU, the pool
// replicated): each rank solves its slice of the training scenarios (twosd_refresh_train), the
// ranks exchange the distinct optimal bases with their counts and pick the same most frequent
// max_pool - 1 (the caller's selection, sqlp_amd/dist.py), each rank composes the B^{-1} of the
// picked bases whose first occurrence it holds (twosd_refresh_build_local -> a pack of the
// intermediate CSC, counts and heads), the packs are all-gathered, and every rank assembles the
// same pool from the gathered table (twosd_refresh_assemble).  With the training scenarios
// split contiguously the pool equals the single-rank refresh of all of them, bit for bit.

// pack: 8-byte aligned sections of n sources with nz intermediate entries
struct RtPack {
    size_t heads, cnt, tot, nztot, valid, irow, ival, bytes;
};
static inline size_t al8(size_t b) { return (b + 7) & ~(size_t)7; }
static RtPack rt_layout(long long n, long long nz, int m) {
    RtPack L{};
    size_t o = 32;   // header: n, nz, bytes, m (int64)
    L.heads = o; o = al8(o + sizeof(int) * (size_t)n * m);
    L.cnt = o; o = al8(o + sizeof(int) * 4 * (size_t)n * m);
    L.tot = o; o = al8(o + sizeof(int) * 4 * (size_t)n);
    L.nztot = o; o = al8(o + sizeof(int) * (size_t)n);
    L.valid = o; o = al8(o + sizeof(int) * (size_t)n);
    L.irow = o; o = al8(o + sizeof(int) * (size_t)nz);
    L.ival = o; o = al8(o + sizeof(double) * (size_t)nz);
    L.bytes = o;
    return L;
}

// rows src_row[j] of the training heads -> out row j
__global__ void rt_heads_kernel(int n, int m, const int *__restrict__ heads, const int *__restrict__ src_row, int *__restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)n * m; i += (size_t)gridDim.x * blockDim.x)
        out[i] = heads[(size_t)src_row[i / m] * m + i % m];
}

// batched copy: segment blockIdx.y = (src, dst, 4-byte words)
struct CopySeg { const int *src; int *dst; long long words; };
__global__ void rt_copy_kernel(const CopySeg *__restrict__ seg) {
    const CopySeg S = seg[blockIdx.y];
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < S.words; i += (long long)gridDim.x * blockDim.x)
        S.dst[i] = S.src[i];
}
static int rt_copy(twosd_ctx *c, const std::vector<CopySeg> &segs) {
    if (segs.empty()) return TWOSD_OK;
    CopySeg *h = stage_buf<CopySeg>(c, 13, segs.size());
    if (!h) return fail(TWOSD_E_DEVICE, "refresh: pinned staging allocation failed");
    std::copy(segs.begin(), segs.end(), h);
    if (!c->d_gs_seg || c->gs_seg_cap < segs.size()) {
        if (c->d_gs_seg) hipFree(c->d_gs_seg);
        c->d_gs_seg = nullptr;
        c->gs_seg_cap = 0;
        HIPCHK(hipMalloc(&c->d_gs_seg, sizeof(CopySeg) * std::max<size_t>(segs.size(), 64)));
        c->gs_seg_cap = std::max<size_t>(segs.size(), 64);
    }
    HIPCHK(hipMemcpyAsync(c->d_gs_seg, h, sizeof(CopySeg) * segs.size(), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(rt_copy_kernel, dim3(64, (unsigned)segs.size()), dim3(256), 0, c->stream, (const CopySeg *)c->d_gs_seg);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));   // the staging buffer is reused by the next call
    return TWOSD_OK;
}

// kcap: the training pivot cap (> 0; <= 0 none); retry: solve again uncapped when fewer than
// half end optimal (the single-rank rule, decided by this rank alone)
static int refresh_train_impl(twosd_ctx *c, int epi, const double *x, int first, int count, int kcap, bool retry,
                              int *n_bases, int *n_opt, double *box_lo, double *box_hi) {
    if (!c || !c->has_basis) return fail(TWOSD_E_STATE, "refresh_train: no primary basis");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "refresh_train: epigraph %d does not exist", epi);
    const EpiDevice &E = c->epis[epi];
    if (first < 0 || count < 1 || first + count > E.count || (c->n1 > 0 && !x) || !n_bases)
        return fail(TWOSD_E_ARG, "refresh_train: bad arguments");
    if (c->CH <= 0) return fail(TWOSD_E_UNSUPPORTED, "refresh_train: needs the hypersparse LP kernel");
    HIPCHK(hipSetDevice(c->device));
    const auto t0 = std::chrono::steady_clock::now();
    const double *d_dv = E.d_dv + (size_t)first * c->k;
    int rc;
    c->rt_trained = false;
    if ((rc = refresh_training(c, x, d_dv, count, kcap, retry, n_opt))) return rc;   // as twosd_pool_refresh step 1
    const auto t1 = std::chrono::steady_clock::now();
    const int *d_list = nullptr, *d_counts = nullptr;
    int U = 0;
    if ((rc = vkey_first_occurrences(c, count, c->d_bkey, c->d_status, &d_list, &U, &d_counts))) return rc;
    c->rt_reps.resize(U);
    c->rt_counts.resize(U);
    c->rt_keys.resize(U);
    std::vector<unsigned long long> bk(count);
    if (U > 0) {
        HIPCHK(hipMemcpy(c->rt_reps.data(), d_list, sizeof(int) * U, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(c->rt_counts.data(), d_counts, sizeof(int) * U, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(bk.data(), c->d_bkey, sizeof(unsigned long long) * count, hipMemcpyDeviceToHost));
        for (int a = 0; a < U; ++a) c->rt_keys[a] = bk[c->rt_reps[a]];
    }
    // training box of the slice (cached per training range, as the single-rank refresh)
    if (c->k > 0 && !(c->rt_epi == epi && c->rt_first == first && c->rt_count == count && c->rt_n == E.count)) {
        std::vector<double> dv((size_t)count * c->k);
        HIPCHK(hipMemcpy(dv.data(), d_dv, sizeof(double) * dv.size(), hipMemcpyDeviceToHost));
        c->rt_lo.assign(c->k, INFINITY);
        c->rt_hi.assign(c->k, -INFINITY);
        for (int s2 = 0; s2 < count; ++s2)
            for (int e = 0; e < c->k; ++e) {
                c->rt_lo[e] = std::min(c->rt_lo[e], dv[(size_t)s2 * c->k + e]);
                c->rt_hi[e] = std::max(c->rt_hi[e], dv[(size_t)s2 * c->k + e]);
            }
    }
    c->rt_epi = epi; c->rt_first = first; c->rt_count = count; c->rt_n = E.count;
    if (box_lo) std::copy(c->rt_lo.begin(), c->rt_lo.end(), box_lo);
    if (box_hi) std::copy(c->rt_hi.begin(), c->rt_hi.end(), box_hi);
    c->rt_nown = -1;
    c->rt_trained = true;
    c->last_refresh_ms[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    c->last_refresh_ms[1] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    *n_bases = U;
    return TWOSD_OK;
}

extern "C" int twosd_refresh_train(twosd_ctx *c, int epi, const double *x, int first, int count, int *n_bases,
                                   double *box_lo, double *box_hi) {
    if (!c) return fail(TWOSD_E_ARG, "refresh_train: NULL context");
    return refresh_train_impl(c, epi, x, first, count, train_kcap(c), true, n_bases, nullptr, box_lo, box_hi);
}

extern "C" int twosd_refresh_train_ex(twosd_ctx *c, int epi, const double *x, int first, int count, int kcap, int *n_bases,
                                      int *n_optimal, double *box_lo, double *box_hi) {
    return refresh_train_impl(c, epi, x, first, count, kcap > 0 ? kcap : 0, false, n_bases, n_optimal, box_lo, box_hi);
}

extern "C" int twosd_refresh_train_bases(twosd_ctx *c, uint64_t *keys, int *counts, int *reps) {
    if (!c || !c->rt_trained) return fail(TWOSD_E_STATE, "refresh_train_bases: no training solve (twosd_refresh_train)");
    const size_t U = c->rt_keys.size();
    if (keys) std::copy(c->rt_keys.begin(), c->rt_keys.end(), keys);
    if (counts) std::copy(c->rt_counts.begin(), c->rt_counts.end(), counts);
    if (reps) std::copy(c->rt_reps.begin(), c->rt_reps.begin() + U, reps);
    return TWOSD_OK;
}

extern "C" int twosd_refresh_build_local(twosd_ctx *c, int n_own, const int *reps, int64_t *pack_bytes) {
    if (!c || !c->rt_trained) return fail(TWOSD_E_STATE, "refresh_build_local: no training solve (twosd_refresh_train)");
    if (n_own < 0 || (n_own > 0 && !reps) || !pack_bytes) return fail(TWOSD_E_ARG, "refresh_build_local: bad arguments");
    for (int j = 0; j < n_own; ++j)
        if (reps[j] < 0 || reps[j] >= c->rt_count) return fail(TWOSD_E_ARG, "refresh_build_local: representative %d outside the slice", reps[j]);
    if (!pg_supported(c->L.m, c->L.n, c->eo_kmax))
        return fail(TWOSD_E_UNSUPPORTED, "refresh_build_local: the device pool build does not fit this template");
    HIPCHK(hipSetDevice(c->device));
    const auto t0 = std::chrono::steady_clock::now();
    const int m = c->L.m;
    int rc;
    if ((size_t)std::max(n_own, 1) > c->refresh_sel_cap) {
        if ((rc = dalloc(&c->d_refresh_sel, (size_t)std::max(n_own, 1)))) return rc;
        c->refresh_sel_cap = std::max(n_own, 1);
    }
    if (n_own) HIPCHK(hipMemcpyAsync(c->d_refresh_sel, reps, sizeof(int) * n_own, hipMemcpyHostToDevice, c->stream));
    PgArgs A;
    int *h_tot = nullptr, *h_valid = nullptr;
    long long inz = 0;
    const int nsrc = n_own + 1;
    if ((rc = pg_compute(c, nsrc, A, &h_tot, &h_valid, &inz, getenv("TWOSD_DEBUG") != nullptr))) return rc;
    const long long *h_ioff = static_cast<const long long *>(c->stage[12]);
    const long long nz0 = n_own ? h_ioff[1] : inz;
    const RtPack L = rt_layout(n_own, inz - nz0, m);
    if ((rc = dev_reserve(c, &c->d_rt_pack, L.bytes))) return rc;
    long long *hdr = stage_buf<long long>(c, 14, 4);
    if (!hdr) return fail(TWOSD_E_DEVICE, "refresh: pinned staging allocation failed");
    hdr[0] = n_own; hdr[1] = inz - nz0; hdr[2] = (long long)L.bytes; hdr[3] = m;
    HIPCHK(hipMemcpyAsync(c->d_rt_pack, hdr, 32, hipMemcpyHostToDevice, c->stream));
    char *P = c->d_rt_pack;
    if (n_own) {
        hipLaunchKernelGGL(rt_heads_kernel, dim3(std::min(1024, (n_own * m + 255) / 256)), dim3(256), 0, c->stream, n_own, m,
                           c->d_head_out, c->d_refresh_sel, reinterpret_cast<int *>(P + L.heads));
        HIPCHK(hipGetLastError());
    }
    std::vector<CopySeg> seg;
    auto add = [&](const void *src, void *dst, size_t bytes) {
        if (bytes) seg.push_back({static_cast<const int *>(src), static_cast<int *>(dst), (long long)(bytes / 4)});
    };
    const size_t nm = (size_t)n_own * m;
    for (int f = 0; f < 4; ++f)   // nzc, keptc, rowcnt, erowcnt: rows 1..n_own of each
        add(c->d_pg_cnt + (size_t)f * nsrc * m + m, P + L.cnt + sizeof(int) * f * nm, sizeof(int) * nm);
    add(c->d_pg_tot + 4, P + L.tot, sizeof(int) * 4 * n_own);
    add(c->d_pg_tot + (size_t)4 * nsrc + 1, P + L.nztot, sizeof(int) * n_own);
    add(c->d_pg_valid + 1, P + L.valid, sizeof(int) * n_own);
    add(c->d_pg_irow + nz0, P + L.irow, sizeof(int) * (inz - nz0));
    add(c->d_pg_ival + nz0, P + L.ival, sizeof(double) * (inz - nz0));
    if ((rc = rt_copy(c, seg))) return rc;
    c->rt_nz0 = nz0;
    c->rt_nsrc_local = nsrc;
    c->rt_nown = n_own;
    c->last_refresh_ms[2] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *pack_bytes = (int64_t)L.bytes;
    return TWOSD_OK;
}

extern "C" int twosd_refresh_pack(twosd_ctx *c, void *d_dst) {
    if (!c || c->rt_nown < 0 || !d_dst) return fail(TWOSD_E_STATE, "refresh_pack: no local build (twosd_refresh_build_local)");
    HIPCHK(hipSetDevice(c->device));
    const RtPack L = rt_layout(c->rt_nown, 0, c->L.m);
    long long bytes = 0;
    HIPCHK(hipMemcpy(&bytes, c->d_rt_pack + 16, sizeof(bytes), hipMemcpyDeviceToHost));
    (void)L;
    HIPCHK(hipMemcpyAsync(d_dst, c->d_rt_pack, (size_t)bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return TWOSD_OK;
}

extern "C" int twosd_refresh_assemble(twosd_ctx *c, int G, const void *d_packs, int64_t stride, int R, const int *order,
                                      const double *box_lo, const double *box_hi, int *pool_size) {
    if (!c || c->rt_nown < 0) return fail(TWOSD_E_STATE, "refresh_assemble: no local build (twosd_refresh_build_local)");
    if (G < 1 || !d_packs || stride < 32 || (stride & 7) || R < 0 || (R > 0 && !order) || (c->k > 0 && (!box_lo || !box_hi)))
        return fail(TWOSD_E_ARG, "refresh_assemble: bad arguments");
    HIPCHK(hipSetDevice(c->device));
    const auto t0 = std::chrono::steady_clock::now();
    const int m = c->L.m;
    int rc;
    const char *packs = static_cast<const char *>(d_packs);
    std::vector<long long> hdr((size_t)4 * G);
    HIPCHK(hipMemcpy2D(hdr.data(), 32, packs, (size_t)stride, 32, G, hipMemcpyDeviceToHost));
    std::vector<long long> an(G + 1, 1), zn(G + 1, c->rt_nz0);
    for (int r = 0; r < G; ++r) {
        if (hdr[4 * r] < 0 || hdr[4 * r + 3] != m || hdr[4 * r + 2] > stride)
            return fail(TWOSD_E_ARG, "refresh_assemble: pack %d is not a pack of this template", r);
        an[r + 1] = an[r] + hdr[4 * r];
        zn[r + 1] = zn[r] + hdr[4 * r + 1];
    }
    const long long nsrc = an[G], nzg = zn[G];
    if (nsrc > INT32_MAX / std::max(m, 1)) return fail(TWOSD_E_UNSUPPORTED, "refresh_assemble: too many sources");
    for (int i = 0; i < R; ++i)
        if (order[i] < 1 || order[i] >= nsrc) return fail(TWOSD_E_ARG, "refresh_assemble: source %d outside [1, %lld)", order[i], nsrc);
    if ((rc = dev_reserve(c, &c->d_gs_heads, (size_t)std::max<long long>(nsrc - 1, 1) * m)) ||
        (rc = dev_reserve(c, &c->d_gs_cnt, (size_t)4 * nsrc * m)) || (rc = dev_reserve(c, &c->d_gs_tot, (size_t)5 * nsrc)) ||
        (rc = dev_reserve(c, &c->d_gs_valid, (size_t)nsrc)) || (rc = dev_reserve(c, &c->d_gs_ioff, (size_t)nsrc)) ||
        (rc = dev_reserve(c, &c->d_gs_irow, (size_t)nzg)) || (rc = dev_reserve(c, &c->d_gs_ival, (size_t)nzg)))
        return rc;
    // the table: source 0 = this rank's primary (local compute row 0), then every rank's pack
    std::vector<CopySeg> seg;
    auto add = [&](const void *src, void *dst, size_t bytes) {
        if (bytes) seg.push_back({static_cast<const int *>(src), static_cast<int *>(dst), (long long)(bytes / 4)});
    };
    const size_t nl = (size_t)c->rt_nsrc_local;
    for (int f = 0; f < 4; ++f) add(c->d_pg_cnt + f * nl * m, c->d_gs_cnt + (size_t)f * nsrc * m, sizeof(int) * m);
    add(c->d_pg_tot, c->d_gs_tot, sizeof(int) * 4);
    add(c->d_pg_tot + 4 * nl, c->d_gs_tot + 4 * nsrc, sizeof(int));
    add(c->d_pg_valid, c->d_gs_valid, sizeof(int));
    add(c->d_pg_irow, c->d_gs_irow, sizeof(int) * c->rt_nz0);
    add(c->d_pg_ival, c->d_gs_ival, sizeof(double) * c->rt_nz0);
    for (int r = 0; r < G; ++r) {
        const long long n = hdr[4 * r], nz = hdr[4 * r + 1], a = an[r];
        const RtPack L = rt_layout(n, nz, m);
        const char *P = packs + (size_t)r * stride;
        const size_t nm = (size_t)n * m;
        add(P + L.heads, c->d_gs_heads + (size_t)(a - 1) * m, sizeof(int) * nm);
        for (int f = 0; f < 4; ++f) add(P + L.cnt + sizeof(int) * f * nm, c->d_gs_cnt + (size_t)f * nsrc * m + (size_t)a * m, sizeof(int) * nm);
        add(P + L.tot, c->d_gs_tot + 4 * a, sizeof(int) * 4 * n);
        add(P + L.nztot, c->d_gs_tot + 4 * nsrc + a, sizeof(int) * n);
        add(P + L.valid, c->d_gs_valid + a, sizeof(int) * n);
        add(P + L.irow, c->d_gs_irow + zn[r], sizeof(int) * nz);
        add(P + L.ival, c->d_gs_ival + zn[r], sizeof(double) * nz);
    }
    if ((rc = rt_copy(c, seg))) return rc;
    const auto t_copy = std::chrono::steady_clock::now();
    if (getenv("TWOSD_DEBUG"))
        fprintf(stderr, "refresh_assemble: %lld sources, %lld entries, unpack %.2f ms\n", nsrc, nzg,
                std::chrono::duration<double, std::milli>(t_copy - t0).count());
    int *h_tot = stage_buf<int>(c, 9, (size_t)6 * nsrc);
    long long *h_ioff = stage_buf<long long>(c, 12, (size_t)nsrc);
    if (!h_tot || !h_ioff) return fail(TWOSD_E_DEVICE, "refresh: pinned staging allocation failed");
    int *h_nz = h_tot + 4 * nsrc, *h_valid = h_tot + 5 * nsrc;
    HIPCHK(hipMemcpyAsync(h_tot, c->d_gs_tot, sizeof(int) * 5 * nsrc, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(h_valid, c->d_gs_valid, sizeof(int) * nsrc, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    long long z = 0;
    for (long long a = 0; a < nsrc; ++a) {
        h_ioff[a] = z;
        z += h_nz[a];
    }
    if (z != nzg) return fail(TWOSD_E_ARG, "refresh_assemble: packs inconsistent (%lld vs %lld entries)", z, nzg);
    HIPCHK(hipMemcpyAsync(c->d_gs_ioff, h_ioff, sizeof(long long) * nsrc, hipMemcpyHostToDevice, c->stream));
    // source table of the gathered build (template fields as the local compute)
    PgArgs A;
    if ((rc = pg_args(c, c->rt_nsrc_local, A))) return rc;
    A.nzc = c->d_gs_cnt; A.keptc = c->d_gs_cnt + (size_t)nsrc * m;
    A.rowcnt = c->d_gs_cnt + (size_t)2 * nsrc * m; A.erowcnt = c->d_gs_cnt + (size_t)3 * nsrc * m;
    A.tot = c->d_gs_tot; A.nztot = c->d_gs_tot + 4 * nsrc; A.valid = c->d_gs_valid;
    A.inter_off = c->d_gs_ioff; A.inter_row = c->d_gs_irow; A.inter_val = c->d_gs_ival;
    A.gheads = c->d_gs_heads;
    // R == 0 (no rank had an optimal training scenario, or max_pool <= 1): the current pool stays,
    // as in twosd_pool_refresh (falling back to the primary basis alone costs ~90 pivots a scenario)
    if (R > 0) {
        std::vector<int> ord(R + 1);
        ord[0] = 0;
        std::copy(order, order + R, ord.begin() + 1);
        if ((rc = pg_assemble(c, A, h_tot, h_valid, ord)) != 0)
            return rc < 0 ? rc : fail(TWOSD_E_STATE, "refresh_assemble: the primary basis failed the device checks");
    } else {
        c->prep_valid = false;   // the selection box below changes
    }
    // selection box: the union of the ranks' training boxes
    if (c->k > 0) {
        c->sel_lo.assign(box_lo, box_lo + c->k);
        c->sel_hi.assign(box_hi, box_hi + c->k);
        c->box_epi = -1;   // not the single-rank cache
    }
    c->rt_nown = -1;
    c->rt_trained = false;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->last_refresh_ms[3] = ms;
    c->last_refresh_ms[4] = c->last_refresh_ms[0] + c->last_refresh_ms[1] + c->last_refresh_ms[2] + ms;
    if (pool_size) *pool_size = (int)c->pool.size();
    return TWOSD_OK;
}

extern "C" int twosd_last_refresh_ms(twosd_ctx *c, double *ms5) {
    if (!c || !ms5) return fail(TWOSD_E_ARG, "last_refresh_ms: NULL");
    for (int i = 0; i < 5; ++i) ms5[i] = c->last_refresh_ms[i];
    return TWOSD_OK;
}


// Two-level selection from training scenarios [first, first + count) of epigraph epi at x:
// level 1 = pool[0, level1) (the most frequent bases); the candidates of a level-1 basis p are
// the ncand bases that the flat selection over the whole pool picks most often for training
// scenarios whose level-1 pick is p (ties: lower index).  level1 = 0 back to flat selection.
// flat and level-1 picks of training scenarios [first, first + count) of epi at x
static int candidate_picks(twosd_ctx *c, const EpiDevice &E, const double *x, int first, int count, int level1,
                           int *p1, int *pf) {
    int rc;
    if ((rc = prepare_x(c, x))) return rc;
    if ((rc = dev_reserve(c, &c->d_cpick, (size_t)count))) return rc;   // grow-only: no hipMalloc / hipFree per refresh
    int *d_p = c->d_cpick;
    const double *dv = E.d_dv + (size_t)first * c->k;
    auto picks = [&](int np, int *out) {   // selection runs on c->stream
        int r = select_pool(c, dv, count, d_p, np);
        if (!r && (hipStreamSynchronize(c->stream) != hipSuccess ||
                   hipMemcpy(out, d_p, sizeof(int) * count, hipMemcpyDeviceToHost) != hipSuccess))
            r = fail(TWOSD_E_DEVICE, "pool candidates: selection failed");
        return r;
    };
    rc = picks(level1, p1);
    if (!rc) rc = picks((int)c->pool.size(), pf);
    return rc;
}

// candidate lists from the picks of the training scenarios (any order): the ncand bases the flat
// selection picks most often among the scenarios of each level-1 pick (ties: lower index)
static int set_candidates(twosd_ctx *c, int level1, int ncand, int n, const int *p1, const int *pf) {
    // the differing (level-1 pick, flat pick) pairs bucketed by level-1 pick (counting sort), then
    // per bucket the flat picks sorted and counted by runs; the ncand most frequent kept (ties:
    // lower basis)
    std::vector<int> start(level1 + 1, 0);
    for (int s = 0; s < n; ++s)
        if (pf[s] != p1[s] && p1[s] >= 0 && p1[s] < level1) ++start[p1[s] + 1];
    for (int p = 0; p < level1; ++p) start[p + 1] += start[p];
    std::vector<int> fill(start.begin(), start.end() - 1), bucket(start[level1]);
    for (int s = 0; s < n; ++s)
        if (pf[s] != p1[s] && p1[s] >= 0 && p1[s] < level1) bucket[fill[p1[s]]++] = pf[s];
    std::vector<int> cand((size_t)level1 * ncand, -1);
    std::vector<std::pair<int, int>> v;   // (-count, basis) of one level-1 pick
    for (int p = 0; p < level1; ++p) {
        int *b0 = bucket.data() + start[p], *b1 = bucket.data() + start[p + 1];
        if (b0 == b1) continue;
        std::sort(b0, b1);
        v.clear();
        for (int *a = b0; a < b1;) {
            int *b = a;
            while (b < b1 && *b == *a) ++b;
            v.push_back({-(int)(b - a), *a});
            a = b;
        }
        const size_t nk = std::min<size_t>(v.size(), ncand);
        std::partial_sort(v.begin(), v.begin() + nk, v.end());
        for (size_t i = 0; i < nk; ++i) cand[(size_t)p * ncand + i] = v[i].second;
    }
    if (getenv("TWOSD_DEBUG")) {
        int diff = 0, filled = 0;
        for (int s = 0; s < n; ++s) diff += pf[s] != p1[s];
        for (int v : cand) filled += v >= 0;
        fprintf(stderr, "pool candidates: P=%zu level1=%d: %d of %d training picks change, %d candidate slots filled\n",
                c->pool.size(), level1, diff, n, filled);
    }
    int rc;
    int *h = stage_buf<int>(c, 15, cand.size());
    if (!h) return fail(TWOSD_E_DEVICE, "pool candidates: pinned staging allocation failed");
    std::copy(cand.begin(), cand.end(), h);
    if ((rc = dev_reserve(c, &c->d_cand, cand.size()))) return rc;
    HIPCHK(hipMemcpyAsync(c->d_cand, h, sizeof(int) * cand.size(), hipMemcpyHostToDevice, c->stream));
    c->pool_l1 = level1;
    c->pool_ncand = ncand;
    c->cand_pending = false;
    return TWOSD_OK;
}

// the lists are built by the next two-level selection (select_pool), on the host while its
// level-1 pass runs on the device: same lists, the host time off the critical path
static int defer_candidates(twosd_ctx *c, int level1, int ncand, std::vector<int> &&p1, std::vector<int> &&pf) {
    c->cand_p1 = std::move(p1);
    c->cand_pf = std::move(pf);
    c->cand_pl1 = level1;
    c->cand_pnc = ncand;
    c->cand_pending = true;
    c->pool_l1 = level1;
    c->pool_ncand = ncand;
    return TWOSD_OK;
}

extern "C" int twosd_pool_candidate_picks(twosd_ctx *c, int epi, const double *x, int first, int count, int level1, int *p1,
                                          int *pf) {
    if (!c || !c->has_basis) return fail(TWOSD_E_STATE, "pool_candidate_picks: no primary basis");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "pool_candidate_picks: epigraph %d does not exist", epi);
    const EpiDevice &E = c->epis[epi];
    const int P = (int)c->pool.size();
    if (first < 0 || count < 1 || first + count > E.count || level1 < 1 || level1 >= P || !p1 || !pf || (c->n1 > 0 && !x) ||
        c->CH <= 0)
        return fail(TWOSD_E_ARG, "pool_candidate_picks: bad arguments");
    HIPCHK(hipSetDevice(c->device));
    reset_candidates(c);   // the flat pick runs over the whole pool
    return candidate_picks(c, E, x, first, count, level1, p1, pf);
}

extern "C" int twosd_pool_set_candidates(twosd_ctx *c, int level1, int ncand, int n, const int *p1, const int *pf) {
    if (!c || !c->has_basis) return fail(TWOSD_E_STATE, "pool_set_candidates: no primary basis");
    const int P = (int)c->pool.size();
    if (level1 < 1 || level1 >= P || ncand < 1 || ncand > 1024 || n < 0 || (n > 0 && (!p1 || !pf)))
        return fail(TWOSD_E_ARG, "pool_set_candidates: bad arguments");
    for (int s = 0; s < n; ++s)
        if (p1[s] < 0 || p1[s] >= P || pf[s] < 0 || pf[s] >= P) return fail(TWOSD_E_ARG, "pool_set_candidates: pick outside the pool");
    HIPCHK(hipSetDevice(c->device));
    return defer_candidates(c, level1, ncand, std::vector<int>(p1, p1 + n), std::vector<int>(pf, pf + n));
}

extern "C" int twosd_pool_build_candidates(twosd_ctx *c, int epi, const double *x, int first, int count, int level1,
                                           int ncand) {
    if (!c || !c->has_basis) return fail(TWOSD_E_STATE, "pool_build_candidates: no primary basis");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "pool_build_candidates: epigraph %d does not exist", epi);
    const EpiDevice &E = c->epis[epi];
    const int P = (int)c->pool.size();
    if (first < 0 || count < 1 || first + count > E.count || level1 < 0 || ncand < 0 || ncand > 1024 || (c->n1 > 0 && !x))
        return fail(TWOSD_E_ARG, "pool_build_candidates: bad arguments");
    reset_candidates(c);
    if (level1 == 0 || ncand == 0 || level1 >= P || P < 2 || c->CH <= 0) return TWOSD_OK;   // flat selection
    HIPCHK(hipSetDevice(c->device));
    std::vector<int> p1(count), pf(count);
    int rc;
    if ((rc = candidate_picks(c, E, x, first, count, level1, p1.data(), pf.data()))) return rc;
    return defer_candidates(c, level1, ncand, std::move(p1), std::move(pf));
}

extern "C" int twosd_last_pool_picks(twosd_ctx *c, int N, int *picks) {
    if (!c || !picks || N < 0 || N > c->last_lp_N) return fail(TWOSD_E_ARG, "last_pool_picks: bad arguments");
    if (c->pool.size() <= 1 || !c->d_pool_pick) {
        std::fill(picks, picks + N, 0);
        return TWOSD_OK;
    }
    HIPCHK(hipMemcpy(picks, c->d_pool_pick, sizeof(int) * N, hipMemcpyDeviceToHost));
    return TWOSD_OK;
}

extern "C" int twosd_invalidate_x(twosd_ctx *c) {
    if (!c) return fail(TWOSD_E_ARG, "invalidate_x: NULL context");
    c->prep_valid = false;   // (the cut's PK rows do not depend on x: kept)
    return TWOSD_OK;
}

extern "C" int twosd_epigraph_create(twosd_ctx *c, int *epi_out) {
    if (!c || !c->has_template || !epi_out) return fail(TWOSD_E_STATE, "epigraph_create: no template");
    c->epis.emplace_back();
    *epi_out = (int)c->epis.size() - 1;
    return TWOSD_OK;
}

extern "C" int twosd_add_scenarios(twosd_ctx *c, int epi, int N, const double *values, const double *weights) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "add_scenarios: no template");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "add_scenarios: epigraph %d does not exist", epi);
    if (N < 0 || (N > 0 && c->k > 0 && !values)) return fail(TWOSD_E_ARG, "add_scenarios: bad arguments");
    if (N == 0) return TWOSD_OK;
    HIPCHK(hipSetDevice(c->device));
    EpiDevice &E = c->epis[epi];
    const int k = c->k;
    std::vector<double> dv((size_t)N * k), w(N, 1.0);
    for (int s = 0; s < N; ++s)
        for (int e = 0; e < k; ++e) dv[(size_t)s * k + e] = values[(size_t)s * k + e] - template_value(c, e);
    if (weights)
        for (int s = 0; s < N; ++s) {
            if (!(weights[s] >= 0.0) || !std::isfinite(weights[s])) return fail(TWOSD_E_ARG, "weight[%d] = %g must be finite and >= 0", s, weights[s]);
            w[s] = weights[s];
        }
    int rc;
    if ((rc = dgrow(&E.d_dv, &E.dv_cap, (size_t)(E.count + N) * k, (size_t)E.count * k, c->stream))) return rc;
    if ((rc = dgrow(&E.d_w, &E.w_cap, (size_t)(E.count + N), (size_t)E.count, c->stream))) return rc;
    if (k) HIPCHK(hipMemcpy(E.d_dv + (size_t)E.count * k, dv.data(), sizeof(double) * N * k, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(E.d_w + E.count, w.data(), sizeof(double) * N, hipMemcpyHostToDevice));
    E.w_host.insert(E.w_host.end(), w.begin(), w.end());
    for (int s = 0; s < N; ++s) E.total_weight += w[s];   // epigraph.jl:89, in insertion order
    E.count += N;
    return TWOSD_OK;
}

extern "C" int twosd_set_distributions(twosd_ctx *c, int k, const int *kind, const int *nsupport, const double *values,
                                       const double *probs, const double *param0, const double *param1) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "set_distributions: no template");
    if (k != c->k) return fail(TWOSD_E_ARG, "set_distributions: %d distributions for %d random elements", k, c->k);
    if (k > 0 && (!kind || !nsupport || !param0 || !param1)) return fail(TWOSD_E_ARG, "set_distributions: NULL argument");
    HIPCHK(hipSetDevice(c->device));
    std::vector<int> kd(std::max(k, 1), 0), off(k + 1, 0);
    std::vector<double> val, prob, p0(std::max(k, 1), 0.0), p1(std::max(k, 1), 0.0), tmpl(std::max(k, 1), 0.0);
    size_t at = 0;
    for (int e = 0; e < k; ++e) {
        kd[e] = kind[e];
        tmpl[e] = template_value(c, e);
        if (kind[e] == 0) {   // DISCRETE: DiscreteNonParametric sorts its support, values unique
            const int n = nsupport[e];
            if (n < 1 || !values || !probs) return fail(TWOSD_E_ARG, "set_distributions: element %d has an empty support", e);
            std::vector<std::pair<double, double>> sp(n);
            for (int i = 0; i < n; ++i) sp[i] = {values[at + i], probs[at + i]};
            at += n;
            std::stable_sort(sp.begin(), sp.end(), [](const std::pair<double, double> &a, const std::pair<double, double> &b) { return a.first < b.first; });
            for (int i = 0; i < n; ++i) {
                if (i && sp[i].first == sp[i - 1].first) return fail(TWOSD_E_ARG, "set_distributions: element %d support values not unique", e);
                if (!(sp[i].second >= 0.0)) return fail(TWOSD_E_ARG, "set_distributions: element %d has a negative probability", e);
                val.push_back(sp[i].first);
                prob.push_back(sp[i].second);
            }
        } else if (kind[e] == 1) {   // NORMAL(mean, variance) -> Normal(mean, sqrt(variance)), smps_sto.jl:122-125
            if (!(param1[e] >= 0.0)) return fail(TWOSD_E_ARG, "set_distributions: element %d has a negative variance", e);
            p0[e] = param0[e];
            p1[e] = std::sqrt(param1[e]);
        } else if (kind[e] == 2) {   // UNIFORM(left, right)
            p0[e] = param0[e];
            p1[e] = param1[e];
        } else {
            return fail(TWOSD_E_ARG, "set_distributions: element %d has unknown kind %d", e, kind[e]);
        }
        off[e + 1] = (int)val.size();
    }
    int rc;
    if ((rc = upload(&c->d_dist_kind, kd)) || (rc = upload(&c->d_dist_off, off)) || (rc = upload(&c->d_dist_val, val)) ||
        (rc = upload(&c->d_dist_prob, prob)) || (rc = upload(&c->d_dist_p0, p0)) || (rc = upload(&c->d_dist_p1, p1)) ||
        (rc = upload(&c->d_dist_tmpl, tmpl)))
        return rc;
    // mean absolute deviation E|V_e - E V_e| per element: the spread of the scenarios (the scale
    // of the selection key's count weight)
    c->dist_mad.assign(std::max(k, 1), 0.0);
    for (int e = 0; e < k; ++e) {
        double mad = 0.0;
        if (kd[e] == 0) {
            double ps = 0.0, mu = 0.0;
            for (int i = off[e]; i < off[e + 1]; ++i) { mu += prob[i] * val[i]; ps += prob[i]; }
            mu = ps > 0.0 ? mu / ps : 0.0;
            for (int i = off[e]; i < off[e + 1]; ++i) mad += prob[i] * fabs(val[i] - mu);
            mad = ps > 0.0 ? mad / ps : 0.0;
        } else if (kd[e] == 1) {   // Normal(mu, sigma): sigma sqrt(2 / pi)
            mad = p1[e] * std::sqrt(2.0 / M_PI);
        } else {                   // Uniform(a, b): |b - a| / 4
            mad = 0.25 * fabs(p1[e] - p0[e]);
        }
        c->dist_mad[e] = std::isfinite(mad) ? mad : 0.0;
    }
    c->has_dist = true;
    return TWOSD_OK;
}

extern "C" int twosd_add_sampled_scenarios(twosd_ctx *c, int epi, int N, uint64_t seed, uint64_t first_index,
                                           const double *weights) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "add_sampled_scenarios: no template");
    if (!c->has_dist) return fail(TWOSD_E_STATE, "add_sampled_scenarios: no distributions (twosd_set_distributions)");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "add_sampled_scenarios: epigraph %d does not exist", epi);
    if (N < 0) return fail(TWOSD_E_ARG, "add_sampled_scenarios: N < 0");
    if (N == 0) return TWOSD_OK;
    HIPCHK(hipSetDevice(c->device));
    EpiDevice &E = c->epis[epi];
    const int k = c->k;
    std::vector<double> w(N, 1.0);
    if (weights)
        for (int s = 0; s < N; ++s) {
            if (!(weights[s] >= 0.0) || !std::isfinite(weights[s])) return fail(TWOSD_E_ARG, "weight[%d] = %g must be finite and >= 0", s, weights[s]);
            w[s] = weights[s];
        }
    int rc;
    if ((rc = dgrow(&E.d_dv, &E.dv_cap, (size_t)(E.count + N) * k, (size_t)E.count * k, c->stream))) return rc;
    if ((rc = dgrow(&E.d_w, &E.w_cap, (size_t)(E.count + N), (size_t)E.count, c->stream))) return rc;
    SampleParams S{};
    S.N = N; S.k = k; S.seed = seed; S.first_index = first_index;
    S.kind = c->d_dist_kind; S.off = c->d_dist_off; S.val = c->d_dist_val; S.prob = c->d_dist_prob;
    S.p0 = c->d_dist_p0; S.p1 = c->d_dist_p1; S.tmpl = c->d_dist_tmpl; S.out = E.d_dv + (size_t)E.count * k;
    HIPCHK(launch_sample(S, c->stream));
    HIPCHK(hipMemcpyAsync(E.d_w + E.count, w.data(), sizeof(double) * N, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    E.w_host.insert(E.w_host.end(), w.begin(), w.end());
    for (int s = 0; s < N; ++s) E.total_weight += w[s];   // epigraph.jl:89, in insertion order
    E.count += N;
    return TWOSD_OK;
}

static int copy_lp_outputs(twosd_ctx *c, int N, double *obj, double *pi, double *y, int *status, const double *d_w);

// evaluate(sp1, sp2, sto, x; N) stage-2 part (smps_routines.jl:67-82) on device-drawn
// scenarios: *s2 = sum over scenarios first..first+count-1 of the stream `seed`, in index
// order, of (1/N_total) * obj (s2_cost += 1/N*obj, :79).  Chunks of <= 1M scenarios:
// sample into scratch, LP solve (objective only), objectives summed on the host in order.
extern "C" int twosd_evaluate_sampled(twosd_ctx *c, const double *x, int64_t N_total, int64_t first, int64_t count,
                                      uint64_t seed, double *s2) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "evaluate_sampled: no template");
    if (!c->has_basis) return fail(TWOSD_E_STATE, "evaluate_sampled: no warm-start basis");
    if (!c->has_dist) return fail(TWOSD_E_STATE, "evaluate_sampled: no distributions (twosd_set_distributions)");
    if (!s2 || N_total <= 0 || first < 0 || count < 0 || (c->n1 > 0 && !x)) return fail(TWOSD_E_ARG, "evaluate_sampled: bad arguments");
    HIPCHK(hipSetDevice(c->device));
    const int k = c->k;
    const int64_t chunk = 1 << 20;
    const double invN = 1.0 / (double)N_total;
    double acc = 0.0;
    std::vector<double> obj;
    for (int64_t at = 0; at < count; at += chunk) {
        const int n = (int)std::min(chunk, count - at);
        int rc;
        if ((rc = dgrow(&c->d_dvtmp, &c->dvtmp_cap, (size_t)n * std::max(k, 1), 0, c->stream))) return rc;
        SampleParams S{};
        S.N = n; S.k = k; S.seed = seed; S.first_index = (unsigned long long)(first + at);
        S.kind = c->d_dist_kind; S.off = c->d_dist_off; S.val = c->d_dist_val; S.prob = c->d_dist_prob;
        S.p0 = c->d_dist_p0; S.p1 = c->d_dist_p1; S.tmpl = c->d_dist_tmpl; S.out = c->d_dvtmp;
        HIPCHK(launch_sample(S, c->stream));
        if ((rc = run_lp(c, x, c->d_dvtmp, n, false, false))) return rc;
        obj.resize(n);
        if ((rc = copy_lp_outputs(c, n, obj.data(), nullptr, nullptr, nullptr, nullptr))) return rc;
        for (int i = 0; i < n; ++i) acc += invN * obj[i];
    }
    *s2 = acc;
    return TWOSD_OK;
}

extern "C" int twosd_get_scenarios(twosd_ctx *c, int epi, int first, int count, double *values) {
    if (!c || epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "get_scenarios: bad epigraph");
    const EpiDevice &E = c->epis[epi];
    if (first < 0 || count < 0 || first + count > E.count || (count > 0 && c->k > 0 && !values))
        return fail(TWOSD_E_ARG, "get_scenarios: range [%d,%d) outside %d scenarios", first, first + count, E.count);
    if (count == 0 || c->k == 0) return TWOSD_OK;
    HIPCHK(hipSetDevice(c->device));
    const int k = c->k;
    HIPCHK(hipMemcpy(values, E.d_dv + (size_t)first * k, sizeof(double) * count * k, hipMemcpyDeviceToHost));
    for (int s = 0; s < count; ++s)
        for (int e = 0; e < k; ++e) values[(size_t)s * k + e] += template_value(c, e);
    return TWOSD_OK;
}

extern "C" int twosd_epigraph_info(twosd_ctx *c, int epi, int *ns, double *tw) {
    if (!c || epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "epigraph_info: bad epigraph");
    if (ns) *ns = c->epis[epi].count;
    if (tw) *tw = c->epis[epi].total_weight;
    return TWOSD_OK;
}

// x-independent element data of the pool (rebuilt when the pool or the positions change):
// per basis p the rows of B_p^{-1}[:, row_e] over the random elements e (host CSR kptr/ke/
// kraw, e ascending) and the same as sliced ELL on the device (kslot pool-strided, absolute
// into kix/kv).  The kernels multiply the scenario deltas by coef_e(x) (d_kcoef) themselves.
static int prepare_elements(twosd_ctx *c) {
    const auto t_pe0 = std::chrono::steady_clock::now();
    if (int rc0 = ensure_host_pool(c)) return rc0;
    const int m = c->L.m, k = c->k, R = c->R;
    std::vector<std::vector<int>> bycol(m);   // random elements on each row
    for (int e = 0; e < k; ++e) bycol[c->pos_row[e]].push_back(e);
    const int P = (int)c->pool.size();
    std::vector<int8_t> bt(c->L.n + m);
    HIPCHK(hipMemcpy(bt.data(), c->d_btype, bt.size(), hipMemcpyDeviceToHost));
    // pass 1: per basis and row the number of element entries; CSR / ELL / record sizes
    std::vector<int> rowcnt((size_t)P * m), width((size_t)P * R);
    std::vector<size_t> kcnt(P + 1, 0), ecnt(P + 1, 0);
    std::vector<int64_t> ccnt(P + 1, 0);
    parallel_for(P, [&](int p) {
        const PoolBasis &B = c->pool[p];
        int *rc = rowcnt.data() + (size_t)p * m;
        size_t tot = 0;
        int64_t cp = 0;   // selection records: every row active; rows of fixed (E) basics twice
        for (int i = 0; i < m; ++i) {
            int n_i = 0;
            for (int q = B.rptr[i]; q < B.rptr[i + 1]; ++q) n_i += (int)bycol[B.rcol[q]].size();
            rc[i] = n_i;
            tot += n_i;
            cp += (int64_t)(1 + n_i) * (bt[B.head[i]] == BT_E ? 2 : 1);
        }
        size_t ell = 0;
        for (int t = 0; t < R; ++t) {
            int w = 0;
            for (int l = 0; l < 64 && 64 * t + l < m; ++l) w = std::max(w, rc[64 * t + l]);
            width[(size_t)p * R + t] = w;
            ell += (size_t)w * 64;
        }
        kcnt[p + 1] = tot;
        ecnt[p + 1] = ell;
        ccnt[p + 1] = cp;
    });
    for (int p = 0; p < P; ++p) { kcnt[p + 1] += kcnt[p]; ecnt[p + 1] += ecnt[p]; ccnt[p + 1] += ccnt[p]; }
    if (kcnt[P] > INT32_MAX || ecnt[P] / 64 > INT32_MAX || ccnt[P] > INT32_MAX)
        return fail(TWOSD_E_UNSUPPORTED, "basis pool element data too large (> 2^31 entries)");
    // pass 2: rows of B_p^{-1}[:, row_e] (e ascending) as CSR (selection inputs) and sliced ELL
    // by row (x_B warm start of the LP kernel), written in place
    const size_t kz = std::max<size_t>(kcnt[P], 1), ez = std::max<size_t>(ecnt[P], 1);
    std::vector<int> kp((size_t)P * (m + 1)), ks((size_t)P * (R + 1)), cap(P + 1);
    int *ke = stage_buf<int>(c, 5, kz), *ki = stage_buf<int>(c, 6, ez);
    double *kr = stage_buf<double>(c, 7, kz), *kv = stage_buf<double>(c, 8, ez);
    if (!ke || !ki || !kr || !kv) return fail(TWOSD_E_DEVICE, "pool elements: pinned staging allocation failed");
    for (int p = 0; p <= P; ++p) cap[p] = (int)ccnt[p];
    parallel_for(P, [&](int p) {
        const PoolBasis &B = c->pool[p];
        const int *rc = rowcnt.data() + (size_t)p * m;
        std::vector<std::pair<int, double>> row;
        size_t at = kcnt[p];
        const size_t e_row0 = ecnt[p] / 64;   // first ELL entry row of this basis
        size_t so = 0;                        // slot offset (entry rows) within the basis
        for (int t = 0; t <= R; ++t) {
            ks[(size_t)p * (R + 1) + t] = (int)(e_row0 + so);
            if (t < R) so += width[(size_t)p * R + t];
        }
        for (int i = 0; i < m; ++i) {
            row.clear();
            for (int q = B.rptr[i]; q < B.rptr[i + 1]; ++q)
                for (int e : bycol[B.rcol[q]]) row.push_back({e, B.rval[q]});
            std::sort(row.begin(), row.end());
            kp[(size_t)p * (m + 1) + i] = (int)at;
            for (auto &ev : row) { ke[at] = ev.first; kr[at] = ev.second; ++at; }
        }
        kp[(size_t)p * (m + 1) + m] = (int)at;
        (void)rc;
        for (int t = 0; t < R; ++t) {
            const int w = width[(size_t)p * R + t];
            const size_t r0 = (size_t)ks[(size_t)p * (R + 1) + t];
            for (int l = 0; l < 64; ++l) {
                const int i = 64 * t + l;
                const int q0 = i < m ? kp[(size_t)p * (m + 1) + i] : 0, q1 = i < m ? kp[(size_t)p * (m + 1) + i + 1] : 0;
                for (int e = 0; e < w; ++e) {
                    const bool has = q0 + e < q1;
                    ki[(r0 + e) * 64 + l] = has ? ke[q0 + e] : 0;
                    kv[(r0 + e) * 64 + l] = has ? kr[q0 + e] : 0.0;
                }
            }
        }
    });
    const auto t_pe1 = std::chrono::steady_clock::now();
    int rc;
    if (c->CH > 0 && ((rc = upload_big(c, &c->d_kslot, ks)) || (rc = upload_big(c, &c->d_kix, ki, ecnt[P])) ||
                      (rc = upload_big(c, &c->d_kv, kv, ecnt[P]))))
        return rc;
    const auto t_pe2 = std::chrono::steady_clock::now();
    if (c->CH > 0 && P > 1) {
        // device selection-stream inputs: CSR rows of every basis, and a static record capacity
        // per basis (every row active: m row starts + all its entries)
        if ((rc = upload_big(c, &c->d_kp, kp)) || (rc = upload_big(c, &c->d_ke, ke, kz)) || (rc = upload_big(c, &c->d_kraw, kr, kz)) ||
            (rc = upload_big(c, &c->d_sel_ptr, cap)) || (rc = reserve_selection(c, P, cap[P])))
            return rc;
    }
    c->k_valid = true;
    if (getenv("TWOSD_DEBUG")) {
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "prepare_elements P=%d: build %.1f ms, upload ell %.1f ms (%zu entries), selection inputs %.1f ms\n",
                P, ms(t_pe0, t_pe1), ms(t_pe1, t_pe2), ecnt[P], ms(t_pe2, std::chrono::steady_clock::now()));
    }
    return TWOSD_OK;
}

// x_B of every pool basis at b: xbase[p][i] = sum_q B_p^{-1}[i][col_q] b[col_q] over the CSR
// rows (pool-strided brptr, MP + 1 per basis; rows >= m are empty), q ascending
__global__ void pool_xbase_kernel(int P, int MP, const int *__restrict__ brptr, const int *__restrict__ brcol,
                                  const double *__restrict__ brval, const double *__restrict__ b, double *__restrict__ xbase) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)P * MP) return;
    const size_t p = t / MP, i = t - p * MP;
    const int *rp = brptr + p * (MP + 1);
    double s = 0.0;
    int q = rp[i];
    const int q1 = rp[i + 1];
    // four entries' loads in flight together; the fmas stay in column order (same bits)
    for (; q + 4 <= q1; q += 4) {
        const int c0 = brcol[q], c1 = brcol[q + 1], c2 = brcol[q + 2], c3 = brcol[q + 3];
        const double v0 = brval[q], v1 = brval[q + 1], v2 = brval[q + 2], v3 = brval[q + 3];
        const double b0 = b[c0], b1 = b[c1], b2 = b[c2], b3 = b[c3];
        s = fma(v0, b0, s);
        s = fma(v1, b1, s);
        s = fma(v2, b2, s);
        s = fma(v3, b3, s);
    }
    for (; q < q1; ++q) s = fma(brval[q], b[brcol[q]], s);
    xbase[t] = s;
}

// primal infeasibility of a basic variable at value x (h_infeas of lp_hyper.hip, tolerance 1e-9)
__device__ __forceinline__ double dev_infeas(double x, int bt) {
    const double tol = 1e-9;
    if (bt == BT_Y || bt == BT_L) return x < -tol ? x : 0.0;
    if (bt == BT_G) return x > tol ? x : 0.0;
    return fabs(x) > tol ? x : 0.0;
}

// Selection stream of one pool basis per block (prepare_x, per x; hb0 = head * 4 + bound type): the rows of basis p that can
// turn infeasible on the training box of the deltas, ordered by their worst box infeasibility
// (largest first, row index on ties), each written as a row-start record (-1 - bound type,
// x_B,i) followed by its element entries (e, B_p^{-1}[i][row_e]) at the basis's static capacity
// offset; rows without entries add their constant infeasibility to cinf[p] (fixed-order sum).
constexpr int kSelStreamThreads = 256;
// count weight of the selection key in units of the mean |coef_e| E|V_e - E V_e| (storm: 13.5;
// 1M bench: 0 -> 111.5 ms per step, 0.37 - 0.74 -> 105.5 - 105.8, 1.5 -> 112, 3 -> 115; ssn: no effect)
constexpr double kSelCountWeight = 0.5;
constexpr int kSelStreamRows = 1024;   // MP <= 1024 (R <= 16)
__global__ void __launch_bounds__(kSelStreamThreads) pool_selstream_kernel(
    int m, int MP, int k, const double *__restrict__ xbase, const int *__restrict__ hb0,
    const int *__restrict__ kp, const int *__restrict__ ke, const double *__restrict__ kraw, const double *__restrict__ xaux,
    int box, int order_rows, float cw, const int *__restrict__ scap, int2 *__restrict__ rec, int *__restrict__ send,
    float *__restrict__ cinf) {
    __shared__ double skey[kSelStreamRows];
    __shared__ int sidx[kSelStreamRows];
    __shared__ int soff[kSelStreamRows];
    __shared__ float cpart[kSelStreamThreads];
    __shared__ int tsum[kSelStreamThreads];
    const int p = blockIdx.x, tid = threadIdx.x;
    const double *coef = xaux + m, *lo_e = xaux + m + k, *hi_e = xaux + m + 2 * k;
    const int *kpp = kp + (size_t)p * (m + 1);
    float cf = 0.0f;
    for (int i = tid; i < kSelStreamRows; i += kSelStreamThreads) {
        double key = INFINITY;   // inactive rows sort last
        if (i < m) {
            const int t = (hb0[(size_t)p * MP + i] & 3);
            const double xv = xbase[(size_t)p * MP + i];
            const int q0 = kpp[i], q1 = kpp[i + 1];
            if (q0 == q1) {
                const double f = fabs(dev_infeas(xv, t));
                cf += (float)f + (f > 0.0 ? cw : 0.0f);
            } else {
                double worst = 0.0;
                bool active = true;
                if (box) {
                    double lo = xv, hi = xv, mag = fabs(xv);
                    for (int q = q0; q < q1; ++q) {
                        const int e = ke[q];
                        const double g = coef[e] * kraw[q];
                        const double a = g * lo_e[e], bb = g * hi_e[e];
                        lo += fmin(a, bb);
                        hi += fmax(a, bb);
                        mag += fmax(fabs(a), fabs(bb));
                    }
                    const double tol = 1e-9 + 1e-12 * mag;
                    const bool feasible_box = (t == BT_Y || t == BT_L) ? lo > tol : (t == BT_G) ? hi < -tol : false;
                    if (isfinite(lo) && isfinite(hi) && feasible_box) active = false;
                    worst = (t == BT_Y || t == BT_L) ? -lo : (t == BT_G) ? hi : fmax(fabs(lo), fabs(hi));
                    if (!isfinite(worst)) worst = HUGE_VAL;
                }
                if (active) key = order_rows ? -worst : 0.0;
            }
        }
        skey[i] = key;
        sidx[i] = i;
    }
    cpart[tid] = cf;
    __syncthreads();
    // bitonic sort of (key, row) ascending: (-worst, i) lexicographic = the host's stable sort
    for (int kk = 2; kk <= kSelStreamRows; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int t2 = tid; t2 < kSelStreamRows / 2; t2 += kSelStreamThreads) {
                const int a = 2 * j * (t2 / j) + (t2 % j), b2 = a + j;
                const bool up = (a & kk) == 0;
                const double ka = skey[a], kb = skey[b2];
                const int ia = sidx[a], ib = sidx[b2];
                const bool gt = ka > kb || (ka == kb && ia > ib);
                if (gt == up) {
                    skey[a] = kb; skey[b2] = ka;
                    sidx[a] = ib; sidx[b2] = ia;
                }
            }
            __syncthreads();
        }
    }
    // records per sorted position, exclusive scan (4 consecutive positions per thread)
    constexpr int PER = kSelStreamRows / kSelStreamThreads;
    int loc[PER], run = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int sp = tid * PER + u;
        const int i = sidx[sp];
        const int c = skey[sp] != INFINITY ? (1 + kpp[i + 1] - kpp[i]) * ((hb0[(size_t)p * MP + i] & 3) == BT_E ? 2 : 1) : 0;
        loc[u] = run;
        run += c;
    }
    tsum[tid] = run;
    __syncthreads();
    if (tid == 0) {   // fixed-order sums: 256 partials (records, constant-row infeasibility)
        int acc = 0;
        float cacc = 0.0f;
        for (int t = 0; t < kSelStreamThreads; ++t) {
            const int v = tsum[t];
            tsum[t] = acc;
            acc += v;
            cacc += cpart[t];
        }
        send[p] = scap[p] + acc;
        cinf[p] = cacc;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) soff[tid * PER + u] = tsum[tid] + loc[u];
    __syncthreads();
    // emit: one wave per sorted row at a time, the row's entries written by consecutive lanes
    const int lane = tid & 63, wv = tid >> 6;
    const size_t base = (size_t)scap[p];
    for (int sp = wv; sp < kSelStreamRows; sp += kSelStreamThreads / 64) {
        if (skey[sp] == INFINITY) break;   // sorted: the inactive rows are all at the end
        const int i = sidx[sp];
        const int q0 = kpp[i], q1 = kpp[i + 1];
        int2 *out = rec + base + soff[sp];
        // records are sign-folded so that the kernels' test is always "x' > tol": x' = -x for
        // Y / L basics (infeasible below 0), x for G (above 0); a fixed (E) basic is written
        // twice, with +x and -x (|x| > tol <=> one of them > tol)
        const int t = hb0[(size_t)p * MP + i] & 3;
        const int ncopy = t == BT_E ? 2 : 1;
        for (int cpy = 0; cpy < ncopy; ++cpy) {
            const float sg = (t == BT_Y || t == BT_L || cpy == 1) ? -1.0f : 1.0f;
            int2 *o = out + cpy * (1 + q1 - q0);
            // record (value bits, byte offset of the element's staged pair row e * 65 * 8; -1: row start)
            if (lane == 0) o[0] = make_int2(__float_as_int(sg * (float)xbase[(size_t)p * MP + i]), -1);
            for (int q = q0 + lane; q < q1; q += 64) o[1 + q - q0] = make_int2(__float_as_int(sg * (float)kraw[q]), ke[q] * 65 * 8);
        }
    }
}

// copy n host elements to a device array grown only when n exceeds its capacity
template <typename T>
static int upload_cap(T **d, size_t *cap, const T *h, size_t n) {
    if (!*d || n > *cap) {
        const size_t nc = std::max<size_t>(n, 1);
        int rc = dalloc(d, nc);
        if (rc) return rc;
        *cap = nc;
    }
    if (n) HIPCHK(hipMemcpy(*d, h, sizeof(T) * n, hipMemcpyHostToDevice));
    return TWOSD_OK;
}

// per-x shared data: b = r - T x; per pool basis xbase_p = B_p^{-1} b (sparse rows);
// coef_e(x); with a pool, the
// selection stream (active rows that can turn infeasible on the training box of the deltas).
// Every pool basis is independent, so the per-basis work runs on host threads.
int twosd::prepare_x(twosd_ctx *c, const double *x) {
    const int m = c->L.m, MP = c->MP, k = c->k, n1 = c->n1;
    if (c->prep_valid && c->prep_x.size() == (size_t)n1 && (n1 == 0 || std::equal(c->prep_x.begin(), c->prep_x.end(), x)))
        return TWOSD_OK;
    int rc;
    const auto t_start = std::chrono::steady_clock::now();
    if (!c->k_valid && (rc = prepare_elements(c))) return rc;
    std::vector<double> b;
    rhs_at(c, x, nullptr, b);
    const int P = (int)c->pool.size();
    std::vector<double> coef(std::max(k, 1), 1.0);
    for (int e = 0; e < k; ++e) coef[e] = c->pos_col[e] < 0 ? 1.0 : -x[c->pos_col[e]];
    if (!c->d_xbase || (size_t)P * MP > c->xbase_cap) {
        if ((rc = dalloc(&c->d_xbase, (size_t)P * MP))) return rc;
        c->xbase_cap = (size_t)P * MP;
    }
    if (c->CH > 0) {
        // everything per x on the device: one upload of [b, coef, box lo, box hi], x_B of every
        // pool basis, then the selection stream (pool_selstream_kernel)
        const bool sel = P > 1;
        const bool box = !c->sel_lo.empty();
        std::vector<double> aux((size_t)m + 3 * (size_t)k, 0.0);
        std::copy(b.begin(), b.end(), aux.begin());
        std::copy(coef.begin(), coef.begin() + k, aux.begin() + m);
        if (box) {
            std::copy(c->sel_lo.begin(), c->sel_lo.end(), aux.begin() + m + k);
            std::copy(c->sel_hi.begin(), c->sel_hi.end(), aux.begin() + m + 2 * k);
        }
        if ((rc = upload_cap(&c->d_xaux, &c->xaux_cap, aux.data(), aux.size())) ||
            (rc = upload_cap(&c->d_kcoef, &c->kcoef_cap, coef.data(), coef.size())))
            return rc;
        const size_t tot = (size_t)P * MP;
        hipLaunchKernelGGL(pool_xbase_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, P, MP, c->d_brptr,
                           c->d_brcol, c->d_brval, c->d_xaux, c->d_xbase);
        HIPCHK(hipGetLastError());
        if (sel) {
            if (MP > kSelStreamRows) return fail(TWOSD_E_UNSUPPORTED, "pool selection: m = %d rows > %d", m, kSelStreamRows);
            // count weight of the selection key: kSelCountWeight x the mean over the random elements
            // of |coef_e(x)| E|V_e - E V_e| (one infeasible row is worth about half a typical
            // scenario perturbation), 0 without distributions.  The same on every rank.
            double sc = 0.0;
            if (c->has_dist && k > 0) {
                for (int e = 0; e < k; ++e) sc += fabs(coef[e]) * c->dist_mad[e];
                sc /= k;
            }
            c->sel_cw = (float)(kSelCountWeight * sc);
            if (const char *e = getenv("TWOSD_SEL_CW")) c->sel_cw = (float)atof(e);   // selection-key experiments
            static const bool sel_order = !getenv("TWOSD_SEL_ROWORDER") || atoi(getenv("TWOSD_SEL_ROWORDER")) != 0;   // A/B knob
            hipLaunchKernelGGL(pool_selstream_kernel, dim3(P), dim3(kSelStreamThreads), 0, c->stream, m, MP, k, c->d_xbase,
                               c->d_hb0, c->d_kp, c->d_ke, c->d_kraw, c->d_xaux, box ? 1 : 0, sel_order ? 1 : 0,
                               c->sel_cw, c->d_sel_ptr, reinterpret_cast<int2 *>(c->d_sel_code), c->d_sel_end, c->d_sel_cinf);
            HIPCHK(hipGetLastError());
        }
        if (getenv("TWOSD_DEBUG") && sel) {
            HIPCHK(hipStreamSynchronize(c->stream));
            std::vector<int> beg(P + 1), end(P);
            HIPCHK(hipMemcpy(beg.data(), c->d_sel_ptr, sizeof(int) * (P + 1), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(end.data(), c->d_sel_end, sizeof(int) * P, hipMemcpyDeviceToHost));
            c->sel_nnz = 0;
            for (int p = 0; p < P; ++p) c->sel_nnz += end[p] - beg[p];
            c->sel_rows = 0;
        }
    }
    c->prep_x.assign(x, x + n1);
    c->prep_valid = true;
    if (getenv("TWOSD_DEBUG")) {
        HIPCHK(hipStreamSynchronize(c->stream));
        fprintf(stderr, "prepare_x: P=%d %.3f ms (%lld selection records)\n", P,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count(),
                (long long)(c->sel_nnz + c->sel_rows));
    }
    return TWOSD_OK;
}

// Warm-start selection for scenarios [0, N) at the prepared x: pick[s] = pool basis, and
// c->d_order = the scenarios grouped by pick (stable).  Flat: least key over the whole pool.
// Two-level (pool_l1 > 0): least key over pool[0, pool_l1), then over the candidates of that
// pick.  npool_override > 0: flat over pool[0, npool_override) (candidate training).
static int select_pool(twosd_ctx *c, const double *d_dv, int N, int *d_pick, int npool_override) {
    const int P = (int)c->pool.size();
    const bool two = npool_override <= 0 && c->pool_l1 > 0 && c->pool_l1 < P && c->pool_ncand > 0 && (c->d_cand || c->cand_pending);
    const int np1 = npool_override > 0 ? npool_override : two ? c->pool_l1 : P;
    int rc;
    size_t tb = 0, tb2 = 0;
    HIPCHK(sort_by_pool(d_pick, nullptr, N, P, nullptr, &tb, c->stream));
    HIPCHK(sort_by_pool(d_pick, nullptr, N, np1, nullptr, &tb2, c->stream));
    tb = std::max(tb, tb2);
    if ((size_t)N > c->order_cap || tb > c->sort_tmp_bytes) {
        if ((rc = dalloc(&c->d_order, (size_t)N)) || (rc = dalloc(&c->d_sort_tmp, tb))) return rc;
        c->order_cap = N;
        c->sort_tmp_bytes = tb;
    }
    if (two && (size_t)N > c->key_cap) {
        if ((rc = dalloc(&c->d_sel_key, (size_t)N))) return rc;
        c->key_cap = N;
    }
    // partials of the chunked selections (small batches: several pool chunks per scenario tile)
    const int g1 = pool_select_split(N, np1), g2 = two ? pool_refine_split(N, c->pool_ncand) : 1;
    const size_t pneed = (size_t)std::max(g1, g2) * N;
    if (std::max(g1, g2) > 1 && pneed > c->sel_pcap) {
        if ((rc = dalloc(&c->d_sel_pkey, pneed)) || (rc = dalloc(&c->d_sel_ppick, pneed))) return rc;
        c->sel_pcap = pneed;
    }
    PoolSelParams S{};
    S.N = N; S.k = c->k; S.npool = np1; S.dv = d_dv;
    S.kcoef = c->d_kcoef;
    S.cinf = c->d_sel_cinf; S.sptr = c->d_sel_ptr; S.send = c->d_sel_end; S.rec = reinterpret_cast<const int2 *>(c->d_sel_code);
    S.pick = d_pick;
    S.cw = c->sel_cw;
    S.key = two ? c->d_sel_key : nullptr;
    S.pkey = g1 > 1 ? c->d_sel_pkey : nullptr;
    S.ppick = g1 > 1 ? c->d_sel_ppick : nullptr;
    HIPCHK(launch_pool_select(S, c->stream));
    if (two && c->cand_pending &&
        (rc = set_candidates(c, c->cand_pl1, c->cand_pnc, (int)c->cand_p1.size(), c->cand_p1.data(), c->cand_pf.data())))
        return rc;
    if (two) {
        HIPCHK(sort_by_pool(d_pick, c->d_order, N, np1, c->d_sort_tmp, &tb, c->stream));
        PoolRefineParams Q{};
        Q.N = N; Q.k = c->k; Q.ncand = c->pool_ncand; Q.dv = d_dv; Q.kcoef = c->d_kcoef;
        Q.cinf = c->d_sel_cinf; Q.sptr = c->d_sel_ptr; Q.send = c->d_sel_end; Q.rec = S.rec;
        Q.order = c->d_order; Q.cand = c->d_cand; Q.pick = d_pick; Q.key = c->d_sel_key; Q.cw = c->sel_cw;
        Q.pkey = g2 > 1 ? c->d_sel_pkey : nullptr;
        Q.pci = g2 > 1 ? c->d_sel_ppick : nullptr;
        HIPCHK(launch_pool_refine(Q, c->stream));
    }
    HIPCHK(sort_by_pool(d_pick, c->d_order, N, P, c->d_sort_tmp, &tb, c->stream));
    return TWOSD_OK;
}

// Launch the LP kernel over N scenarios whose deltas start at d_dv (device); results in
// c->d_obj / d_pi / d_y / d_status / d_iters [0, N).
int twosd::run_lp(twosd_ctx *c, const double *x, const double *d_dv, int N, bool want_pi, bool want_y) {
    LpRun o;
    o.want_pi = want_pi;
    o.want_y = want_y;
    return run_lp_ex(c, x, d_dv, N, o);
}

// N = scenarios of d_dv addressed by the launch (outputs obj / status / iters / pool picks are
// indexed by scenario); list mode solves only o.d_list[0, o.nlist) from their recorded picks
// and writes pi at the list position
int twosd::run_lp_ex(twosd_ctx *c, const double *x, const double *d_dv, int N, const LpRun &o) {
    const bool want_pi = o.want_pi, want_y = o.want_y;
    const bool list = o.d_list != nullptr;
    const int NL = list ? o.nlist : N;   // scenarios this launch solves
    int rc;
    if ((rc = prepare_x(c, x))) return rc;
    if (list && c->pool.size() > 1 && (size_t)N > c->pick_cap) return fail(TWOSD_E_STATE, "LP list mode: no recorded pool picks");
    const int m = c->L.m, n = c->L.n, MP = c->MP, R = c->R;
    if (N > c->out_cap) {
        size_t cap = std::max<size_t>(N, 1024);
        if ((rc = dalloc(&c->d_obj, cap)) || (rc = dalloc(&c->d_status, cap)) || (rc = dalloc(&c->d_iters, cap)) ||
            (rc = dalloc(&c->d_ops, cap)) || (rc = dalloc(&c->d_etan, cap)))
            return rc;
        dfree(c->d_pi); dfree(c->d_y);
        c->pi_cap = c->y_cap = 0;
        c->out_cap = (int)cap;
    }
    if (want_pi && (size_t)NL > c->pi_cap) {
        if ((rc = dalloc(&c->d_pi, (size_t)c->out_cap * m))) return rc;
        c->pi_cap = c->out_cap;
    }
    if (o.want_key && (size_t)N > c->vkey_cap) {
        if ((rc = dalloc(&c->d_vkey, (size_t)c->out_cap))) return rc;
        c->vkey_cap = c->out_cap;
    }
    if (o.want_bkey && (size_t)N > c->bkey_cap) {
        if ((rc = dalloc(&c->d_bkey, (size_t)c->out_cap))) return rc;
        c->bkey_cap = c->out_cap;
    }
    if (want_y && (size_t)N > c->y_cap) {
        if ((rc = dalloc(&c->d_y, (size_t)c->out_cap * n))) return rc;
        c->y_cap = c->out_cap;
    }
    if (!c->d_queue && (rc = dalloc(&c->d_queue, (size_t)kMaxQueueGroups * kQueueStride))) return rc;
    {
        // eta capacity (pivots per scenario): 2m + 32, at least 64.  256 keeps storm's two 4-wave
        // blocks per CU within the LDS; past 256 the file grows (up to 1024, in steps of 32) as far as
        // the LDS keeps the occupancy of 256 -- a scenario that needs more pivots from its pool start
        // than the file holds is retried from the primary basis (ssn 100k: 11 in 8 steps at 256)
        const int CH = c->CH;
        int kmax = c->kmax_override > 0 ? c->kmax_override : std::min(256, std::max(64, 2 * m + 32));
        if (c->kmax_override <= 0 && 2 * m + 32 > kmax) {
            const int b0 = hyper_max_blocks_per_cu(R, CH, kmax, c->k);
            for (int k2 = std::min(1024, (2 * m + 32) & ~31); k2 > kmax; k2 -= 32)
                if (hyper_max_blocks_per_cu(R, CH, k2, c->k) >= b0) { kmax = k2; break; }
        }
        // per-wave eta arena: 32 entries per row, scaled with the file past 256 pivots
        const int ecap = (int)std::min<long long>(INT32_MAX / 2, (long long)std::max(4096, 32 * MP) * std::max(256, kmax) / 256);
        int bpc = hyper_max_blocks_per_cu(R, CH, kmax, c->k);
        if (const char *e = getenv("TWOSD_BPC")) bpc = std::min(bpc, std::max(1, atoi(e)));   // diagnostics: occupancy sweep
        if (bpc < 1) return fail(TWOSD_E_UNSUPPORTED, "LP kernel: LDS slice too large (m = %d, k = %d)", m, c->k);
        const int nblocks = std::max(1, std::min((NL + kWavesPerBlock - 1) / kWavesPerBlock, bpc * c->num_cus));
        const size_t slots = (size_t)nblocks * kWavesPerBlock;
        if (slots > c->earena_slots || ecap != c->earena_cap) {
            if ((rc = dalloc(&c->d_eidx, slots * ecap)) || (rc = dalloc(&c->d_evals, slots * ecap))) return rc;
            c->earena_slots = slots;
            c->earena_cap = ecap;
        }
        HIPCHK(hipMemsetAsync(c->d_queue, 0, sizeof(int) * kMaxQueueGroups * kQueueStride, c->stream));
        HyperParams H{};
        H.m = m; H.n = n; H.k = c->k; H.N = NL; H.kmax = kmax; H.ecap = ecap;
        H.kcap = o.kcap > 0 ? std::min(o.kcap, kmax) : kmax;
        H.retry = o.kcap > 0 ? 0 : 1;
        H.colptr = c->d_colptr; H.rowidx = c->d_rowidx; H.val = c->d_val; H.q = c->d_q; H.btype = c->d_btype;
        H.wcp = c->d_wcp; H.wcc = c->d_wcc; H.wcv = c->d_wcv;
        H.bcp = c->d_bcp; H.bci = c->d_bci; H.bcv = c->d_bcv;
        H.brptr = c->d_brptr; H.brcol = c->d_brcol; H.brval = c->d_brval;
        H.kslot = c->d_kslot; H.kix = c->d_kix; H.kv = c->d_kv; H.kcoef = c->d_kcoef;
        H.xbase = c->d_xbase; H.d0 = c->d_d0; H.hb0 = c->d_hb0;
        H.basic0 = c->d_basic0; H.fixedmask = c->d_fixedmask; H.ubmask = c->d_ubmask;
        H.dv = d_dv; H.eidx = c->d_eidx; H.evals = c->d_evals; H.queue = c->d_queue;
        H.qgroups = std::max(1, std::min(16, nblocks));   // two ranges per XCD (8 / 16 / 32 / 64: 143.6 / 142.7 / 142.8 / 146.3 ms, storm 1M)
        if (const char *e = getenv("TWOSD_QGROUPS")) H.qgroups = std::max(1, std::min({kMaxQueueGroups, nblocks, atoi(e)}));   // A/B knob
        H.obj = c->d_obj; H.pi = want_pi ? c->d_pi : nullptr; H.y = want_y ? c->d_y : nullptr;
        H.vkey = o.want_key ? c->d_vkey : nullptr;
        H.key_zero = 1e-12;   // = HPI_ZERO of the pi recovery (lp_hyper.hip)
        if (const char *e = getenv("TWOSD_KEY_ZERO")) H.key_zero = atof(e);   // A/B knob
        H.bkey = o.want_bkey ? c->d_bkey : nullptr;
        if (o.want_etas) {   // rows: list positions, or scenarios
            const size_t need = list ? (size_t)NL : (size_t)N;
            // eta-file offsets are 32-bit (eo_off, the device pool build): the arena of
            // 4096 entries per row must stay below 2^31 entries
            if (need * 4096 > (size_t)INT32_MAX)
                return fail(TWOSD_E_UNSUPPORTED, "eta files of %zu solves exceed the 2^31-entry arena (at most %d)", need,
                            INT32_MAX / 4096);
            if (need > c->eo_rows || c->eo_kmax != kmax) {
                const size_t rows = std::max<size_t>(need, 256);
                if ((rc = dalloc(&c->d_eo_pb, rows)) || (rc = dalloc(&c->d_eo_K, rows)) || (rc = dalloc(&c->d_eo_off, rows)) ||
                    (rc = dalloc(&c->d_eo_etap, rows * kmax)) || (rc = dalloc(&c->d_eo_etaoff, rows * (kmax + 1))) ||
                    (rc = dalloc(&c->d_eo_eidx, rows * 4096)) || (rc = dalloc(&c->d_eo_evals, rows * 4096)))
                    return rc;
                if (!c->d_eo_used && (rc = dalloc(&c->d_eo_used, 1))) return rc;
                c->eo_rows = rows;
                c->eo_cap = rows * 4096;
                c->eo_kmax = kmax;
            }
            HIPCHK(hipMemsetAsync(c->d_eo_used, 0, sizeof(unsigned long long), c->stream));
            H.eo_pb = c->d_eo_pb; H.eo_K = c->d_eo_K; H.eo_off = c->d_eo_off; H.eo_etap = c->d_eo_etap;
            H.eo_etaoff = c->d_eo_etaoff; H.eo_eidx = c->d_eo_eidx; H.eo_evals = c->d_eo_evals; H.eo_used = c->d_eo_used;
            H.eo_cap = (long long)std::min<size_t>(c->eo_cap, INT32_MAX);
        }
        if (o.want_head) {   // rows: list positions, or scenarios
            const size_t need = list ? (size_t)NL : (size_t)N;
            if (need > c->head_cap) {
                if ((rc = dalloc(&c->d_head_out, need * m))) return rc;
                c->head_cap = need;
            }
            H.head_out = c->d_head_out;
        }
        H.pi_by_pos = list ? 1 : 0;
        H.status = c->d_status; H.iters = c->d_iters; H.ops = c->d_ops; H.etan = c->d_etan;
        if (!c->d_lpstats && (rc = dalloc(&c->d_lpstats, 6))) return rc;
        if (!list) HIPCHK(hipMemsetAsync(c->d_lpstats + 5, 0, sizeof(unsigned long long), c->stream));
        H.retries = list ? nullptr : c->d_lpstats + 5;   // a list re-solve repeats recorded picks: no retries
        if (!c->d_stamps) {
            if ((rc = dalloc(&c->d_stamps, 16))) return rc;
            HIPCHK(hipMemset(c->d_stamps, 0, sizeof(unsigned long long) * 16));
        }
        H.stamps = c->d_stamps;
        H.npool = (int)c->pool.size();
        H.bnnz = c->d_bnnz;
        if (c->want_head && !list) {
            if ((size_t)N > c->head_cap) {
                if ((rc = dalloc(&c->d_head_out, (size_t)N * m))) return rc;
                c->head_cap = N;
            }
            H.head_out = c->d_head_out;
        }
        if (H.npool > 1) {
            if (!list && (size_t)N > c->pick_cap) {
                if ((rc = dalloc(&c->d_pool_pick, (size_t)N))) return rc;
                c->pick_cap = N;
            }
            H.pool_pick = c->d_pool_pick;
        }
        HIPCHK(hipEventRecord(c->ev[0], c->stream));
        if (list) {
            H.order = o.d_list;
        } else if (H.npool > 1) {
            if ((rc = select_pool(c, d_dv, N, c->d_pool_pick, 0))) return rc;
            H.order = c->d_order;
        }
        HIPCHK(hipEventRecord(c->ev[2], c->stream));
        HIPCHK(launch_hyper(R, CH, H, nblocks, hyper_lds_bytes(R, CH, kmax, c->k), c->stream));
        HIPCHK(hipEventRecord(c->ev[1], c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        float ms = 0, ms_sel = 0;
        hipEventElapsedTime(&ms, c->ev[2], c->ev[1]);
        hipEventElapsedTime(&ms_sel, c->ev[0], c->ev[2]);
        c->t_us[0] = 1e3 * ms;
        c->t_us[4] = 1e3 * ms_sel;
        if (list) return TWOSD_OK;
        c->last_lp_N = N;
        c->last_lp_blocks = nblocks;
        c->last_ops_width = 1;
        return TWOSD_OK;
    }
}

// batch statistics on the device (integer sums: exact, order independent): [0] pivots,
// [1] executed FMAs, [2] max pivots, [3] non-optimal scenarios
__global__ void __launch_bounds__(256) lp_stats_kernel(int N, const int *__restrict__ its, const long long *__restrict__ ops,
                                                      const int *__restrict__ st, const int *__restrict__ etan,
                                                      unsigned long long *out) {
    __shared__ unsigned long long red[4][5];
    unsigned long long a = 0, b = 0, d = 0, e = 0;
    unsigned long long mx = 0;
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < N; s += gridDim.x * blockDim.x) {
        a += (unsigned long long)its[s];
        b += (unsigned long long)ops[s];
        mx = its[s] > (int)mx ? (unsigned long long)its[s] : mx;
        d += st[s] != TWOSD_LP_OPTIMAL;
        e += (unsigned long long)etan[s];
    }
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_down(a, o);
        b += __shfl_down(b, o);
        d += __shfl_down(d, o);
        e += __shfl_down(e, o);
        const unsigned long long m2 = __shfl_down(mx, o);
        mx = m2 > mx ? m2 : mx;
    }
    // one set of atomics per block (per wave they serialised on five addresses: ~0.25 ms at 1M)
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[w][0] = a; red[w][1] = b; red[w][2] = mx; red[w][3] = d; red[w][4] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int v = 1; v < (int)(blockDim.x >> 6); ++v) {
            a += red[v][0]; b += red[v][1]; mx = red[v][2] > mx ? red[v][2] : mx; d += red[v][3]; e += red[v][4];
        }
        atomicAdd(&out[0], a);
        atomicAdd(&out[1], b);
        atomicMax(&out[2], mx);
        atomicAdd(&out[3], d);
        atomicAdd(&out[4], e);
    }
}

// incumbent objective of a batch: sum_s w_s obj_s and sum_s w_s (w = 1 without weights), each
// block over a fixed stride of scenarios, then a fixed tree in the block; the host adds the
// kObjBlocks partials in block order, so the sums do not depend on scheduling
constexpr int kObjBlocks = 256;
__global__ void __launch_bounds__(256) lp_obj_kernel(int N, const double *__restrict__ obj, const double *__restrict__ w,
                                                     double *__restrict__ part) {
    __shared__ double sa[256], sb[256];
    double a = 0.0, b = 0.0;
    for (int s = blockIdx.x * 256 + threadIdx.x; s < N; s += kObjBlocks * 256) {
        const double ws = w ? w[s] : 1.0;
        a = fma(ws, obj[s], a);
        b += ws;
    }
    sa[threadIdx.x] = a;
    sb[threadIdx.x] = b;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            sa[threadIdx.x] += sa[threadIdx.x + o];
            sb[threadIdx.x] += sb[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = sa[0];
        part[2 * blockIdx.x + 1] = sb[0];
    }
}

// d_w: the batch's scenario weights (nullable: 1.0), for the objective sum
static int copy_lp_outputs(twosd_ctx *c, int N, double *obj, double *pi, double *y, int *status, const double *d_w) {
    if (!c->d_lpstats) {
        int rc = dalloc(&c->d_lpstats, 6);
        if (rc) return rc;
    }
    if (!c->d_objpart) {
        int rc = dalloc(&c->d_objpart, (size_t)2 * kObjBlocks);
        if (rc) return rc;
    }
    HIPCHK(hipMemsetAsync(c->d_lpstats, 0, 5 * sizeof(unsigned long long), c->stream));
    hipLaunchKernelGGL(lp_stats_kernel, dim3((unsigned)std::min(256, (N + 255) / 256)), dim3(256), 0, c->stream, N,
                       c->d_iters, c->d_ops, c->d_status, c->d_etan, c->d_lpstats);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(lp_obj_kernel, dim3(kObjBlocks), dim3(256), 0, c->stream, N, c->d_obj, d_w, c->d_objpart);
    HIPCHK(hipGetLastError());
    unsigned long long stv[6];
    double part[2 * kObjBlocks];
    HIPCHK(hipMemcpyAsync(stv, c->d_lpstats, sizeof(stv), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(part, c->d_objpart, sizeof(part), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (obj) HIPCHK(hipMemcpy(obj, c->d_obj, sizeof(double) * N, hipMemcpyDeviceToHost));
    if (pi) HIPCHK(hipMemcpy(pi, c->d_pi, sizeof(double) * N * c->L.m, hipMemcpyDeviceToHost));
    if (y) HIPCHK(hipMemcpy(y, c->d_y, sizeof(double) * N * c->L.n, hipMemcpyDeviceToHost));
    if (status) HIPCHK(hipMemcpy(status, c->d_status, sizeof(int) * N, hipMemcpyDeviceToHost));
    c->last_pivots_sum = (int64_t)stv[0]; c->last_ops_sum = (int64_t)stv[1]; c->last_pivots_max = (int)stv[2];
    c->last_eta_entries = (int64_t)stv[4];
    c->last_retries = (int64_t)stv[5];
    if (N >= 4096) {
        c->piv_mean_ref = (double)stv[0] / N;
        c->piv_ref_sum = (int64_t)stv[0];
        c->piv_ref_n = N;
    }
    double ow = 0.0, wt = 0.0;
    for (int b = 0; b < kObjBlocks; ++b) {
        ow += part[2 * b];
        wt += part[2 * b + 1];
    }
    c->last_obj_wsum = ow;
    c->last_obj_w = wt;
    const long long bad = (long long)stv[3];
    if (bad) return fail(TWOSD_E_LP, "%lld of %d scenario LPs not optimal (see status[])", bad, N);
    return TWOSD_OK;
}

extern "C" int twosd_last_objective(twosd_ctx *c, double *weighted_sum, double *weight_sum) {
    if (!c) return fail(TWOSD_E_ARG, "last_objective: NULL");
    if (weighted_sum) *weighted_sum = c->last_obj_wsum;
    if (weight_sum) *weight_sum = c->last_obj_w;
    return TWOSD_OK;
}

extern "C" int twosd_training_cap(twosd_ctx *c, int64_t pivots_sum, int64_t scenarios, int *cap) {
    if (!cap) return fail(TWOSD_E_ARG, "training_cap: NULL");   // ctx NULL: setting 0 (host code only)
    if (pivots_sum < 0 || scenarios < 0) return fail(TWOSD_E_ARG, "training_cap: negative pivot sum / size");
    *cap = training_cap_rule(c, pivots_sum, scenarios);
    return TWOSD_OK;
}

extern "C" int twosd_refresh_cap_stats(twosd_ctx *c, int64_t *pivots_sum, int64_t *scenarios) {
    if (!c) return fail(TWOSD_E_ARG, "refresh_cap_stats: NULL");
    if (pivots_sum) *pivots_sum = c->piv_ref_sum;
    if (scenarios) *scenarios = c->piv_ref_n;
    return TWOSD_OK;
}

// The global basis selection of a distributed refresh (host, no context): the bases the ranks
// list (concatenated in rank order), a key seen by several ranks counting the sum of its counts
// and owned by its first occurrence; the max_pool - 1 largest totals, ties by first occurrence --
// the single-rank refresh's stable sort over all training scenarios.
extern "C" int twosd_select_refresh_bases(const uint64_t *keys, const int64_t *counts, const int64_t *reps, const int32_t *rank_of,
                                          int n, int max_pool, int64_t *owner, int64_t *rep, int *npick) {
    if (n < 0 || !npick || (n > 0 && (!keys || !counts || !reps || !rank_of))) return fail(TWOSD_E_ARG, "select_refresh_bases: bad arguments");
    *npick = 0;
    if (n == 0 || max_pool <= 1) return TWOSD_OK;
    if (!owner || !rep) return fail(TWOSD_E_ARG, "select_refresh_bases: NULL output");
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return keys[a] != keys[b] ? keys[a] < keys[b] : a < b; });
    struct G { int64_t tot; int first; };
    std::vector<G> g;
    g.reserve(n);
    for (int a = 0; a < n;) {
        int b = a;
        int64_t t = 0;
        while (b < n && keys[idx[b]] == keys[idx[a]]) t += counts[idx[b++]];
        g.push_back({t, idx[a]});   // the lowest index of the key: its first occurrence
        a = b;
    }
    const size_t k = std::min<size_t>(g.size(), (size_t)max_pool - 1);
    std::partial_sort(g.begin(), g.begin() + k, g.end(),
                      [](const G &a, const G &b) { return a.tot != b.tot ? a.tot > b.tot : a.first < b.first; });
    for (size_t i = 0; i < k; ++i) {
        owner[i] = rank_of[g[i].first];
        rep[i] = reps[g[i].first];
    }
    *npick = (int)k;
    return TWOSD_OK;
}

extern "C" int twosd_solve_batch(twosd_ctx *c, int epi, const double *x, int first, int count, double *obj,
                                 double *pi, double *y, int *status) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "solve_batch: no template");
    if (!c->has_basis) return fail(TWOSD_E_STATE, "solve_batch: no warm-start basis (twosd_compute_basis / twosd_set_basis)");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "solve_batch: epigraph %d does not exist", epi);
    const EpiDevice &E = c->epis[epi];
    if (first < 0 || count < 0 || first + count > E.count) return fail(TWOSD_E_ARG, "solve_batch: range [%d,%d) outside %d scenarios", first, first + count, E.count);
    if (!obj || !status || (c->n1 > 0 && !x)) return fail(TWOSD_E_ARG, "solve_batch: obj/status/x required");
    if (count == 0) return TWOSD_OK;
    HIPCHK(hipSetDevice(c->device));
    int rc = run_lp(c, x, E.d_dv + (size_t)first * c->k, count, pi != nullptr, y != nullptr);
    if (rc) return rc;
    return copy_lp_outputs(c, count, obj, pi, y, status, E.d_w + first);
}

extern "C" int twosd_solve_values(twosd_ctx *c, const double *x, int N, const double *values, double *obj, double *pi,
                                  double *y, int *status) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "solve_values: no template");
    if (!c->has_basis) return fail(TWOSD_E_STATE, "solve_values: no warm-start basis");
    if (N < 0 || (N > 0 && c->k > 0 && !values) || !obj || !status || (c->n1 > 0 && !x)) return fail(TWOSD_E_ARG, "solve_values: bad arguments");
    if (N == 0) return TWOSD_OK;
    HIPCHK(hipSetDevice(c->device));
    const int k = c->k;
    std::vector<double> dv((size_t)N * std::max(k, 1), 0.0);
    for (int s = 0; s < N; ++s)
        for (int e = 0; e < k; ++e) dv[(size_t)s * k + e] = values[(size_t)s * k + e] - template_value(c, e);
    int rc;
    if ((rc = dgrow(&c->d_dvtmp, &c->dvtmp_cap, (size_t)N * std::max(k, 1), 0, c->stream))) return rc;
    HIPCHK(hipMemcpy(c->d_dvtmp, dv.data(), sizeof(double) * dv.size(), hipMemcpyHostToDevice));
    if ((rc = run_lp(c, x, c->d_dvtmp, N, pi != nullptr, y != nullptr))) return rc;
    return copy_lp_outputs(c, N, obj, pi, y, status, nullptr);
}

extern "C" int twosd_last_timings(twosd_ctx *c, double *us5) {
    if (!c || !us5) return fail(TWOSD_E_ARG, "last_timings: NULL");
    for (int i = 0; i < 5; ++i) us5[i] = c->t_us[i];
    return TWOSD_OK;
}

extern "C" int twosd_last_lp_eta_entries(twosd_ctx *c, int64_t *entries, int64_t *retries) {
    if (!c || !entries) return fail(TWOSD_E_ARG, "last_lp_eta_entries: NULL");
    *entries = c->last_eta_entries;
    if (retries) *retries = c->last_retries;
    return TWOSD_OK;
}

extern "C" int twosd_last_lp_stats(twosd_ctx *c, int64_t *sum, int *mx) {
    if (!c) return fail(TWOSD_E_ARG, "last_lp_stats: NULL");
    if (sum) *sum = c->last_pivots_sum;
    if (mx) *mx = c->last_pivots_max;
    return TWOSD_OK;
}

extern "C" int twosd_set_refresh_kcap(twosd_ctx *c, int kcap) {
    if (!c) return fail(TWOSD_E_ARG, "set_refresh_kcap: NULL");
    c->train_kcap = kcap;
    return TWOSD_OK;
}

extern "C" int twosd_last_lp_iters(twosd_ctx *c, int N, int *iters, int *status) {
    if (!c || N < 0 || N > c->out_cap || !c->d_iters) return fail(TWOSD_E_ARG, "last_lp_iters: N = %d outside the last batch", N);
    HIPCHK(hipStreamSynchronize(c->stream));
    if (iters) HIPCHK(hipMemcpy(iters, c->d_iters, sizeof(int) * N, hipMemcpyDeviceToHost));
    if (status) HIPCHK(hipMemcpy(status, c->d_status, sizeof(int) * N, hipMemcpyDeviceToHost));
    return TWOSD_OK;
}

extern "C" int twosd_debug_stamps(twosd_ctx *c, uint64_t *out10, int reset) {
    if (!c || !out10) return fail(TWOSD_E_ARG, "debug_stamps: NULL");
    for (int i = 0; i < 10; ++i) out10[i] = 0;
    if (!c->d_stamps) return TWOSD_OK;
    HIPCHK(hipMemcpy(out10, c->d_stamps, sizeof(uint64_t) * 10, hipMemcpyDeviceToHost));
    if (reset) HIPCHK(hipMemset(c->d_stamps, 0, sizeof(uint64_t) * 16));
    return TWOSD_OK;
}

extern "C" int twosd_last_lp_ops(twosd_ctx *c, int64_t *row_ops, int *row_width) {
    if (!c) return fail(TWOSD_E_ARG, "last_lp_ops: NULL");
    if (row_ops) *row_ops = c->last_ops_sum;
    if (row_width) *row_width = c->last_ops_width;
    return TWOSD_OK;
}

// rows list[0..U) of pi (m doubles each) gathered in list order (the push of a full-mode solve_push)
__global__ void gather_rows_kernel(int U, int m, const int *__restrict__ list, const double *__restrict__ pi, double *__restrict__ out) {
    const size_t tot = (size_t)U * m;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
        const int u = (int)(i / m), r = (int)(i % m);
        out[i] = pi[(size_t)list[u] * m + r];
    }
}

// non-optimal statuses among the scenarios of a list-mode re-solve (status is by scenario)
__global__ void list_status_kernel(int U, const int *__restrict__ list, const int *__restrict__ st,
                                   unsigned long long *bad) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < U; i += gridDim.x * blockDim.x)
        if (st[list[i]] != TWOSD_LP_OPTIMAL) atomicAdd(bad, 1ull);
}

extern "C" int twosd_solve_push(twosd_ctx *c, int epi, const double *x, int first, int count, double *obj, int *status,
                                int *new_size) {
    if (!c || !c->has_template) return fail(TWOSD_E_STATE, "solve_push: no template");
    if (!c->has_basis) return fail(TWOSD_E_STATE, "solve_push: no warm-start basis");
    if (epi < 0 || epi >= (int)c->epis.size()) return fail(TWOSD_E_ARG, "solve_push: epigraph %d does not exist", epi);
    const EpiDevice &E = c->epis[epi];
    if (first < 0 || count < 0 || first + count > E.count) return fail(TWOSD_E_ARG, "solve_push: range outside the epigraph");
    if (c->n1 > 0 && !x) return fail(TWOSD_E_ARG, "solve_push: x is NULL");
    if (count == 0) { if (new_size) *new_size = c->dvs.size; return TWOSD_OK; }
    HIPCHK(hipSetDevice(c->device));
    const double *d_dv = E.d_dv + (size_t)first * c->k;
    // TWOSD_PUSH_ALL=1: recover and push the dual of every scenario (the pre-key path, kept for
    // the equivalence test); default: vertex keys, first occurrences, re-solve of those only
    const bool all = getenv("TWOSD_PUSH_ALL") && atoi(getenv("TWOSD_PUSH_ALL")) != 0;
    // Full mode: the main pass recovers every scenario's dual (and its key), and the representatives'
    // rows are gathered from it -- the same rows the re-solve would produce (same start, same pivots,
    // same recovery), without solving them twice.  Chosen when the last keyed push re-solved more
    // than a quarter of its scenarios (ssn: ~every scenario its own vertex; storm: < 1 %).
    // TWOSD_PUSH_MODE: 0 auto (default), 1 always re-solve, 2 always full.
    const int pmode = getenv("TWOSD_PUSH_MODE") ? atoi(getenv("TWOSD_PUSH_MODE")) : 0;
    const bool full = !all && (pmode == 2 || (pmode == 0 && c->push_rep_frac > 0.25));
    c->last_push_full = full ? 1 : 0;
    LpRun o;
    o.want_pi = all || full;
    o.want_key = !all;
    int rc = run_lp_ex(c, x, d_dv, count, o);
    if (rc) return rc;
    const double t_lp = c->t_us[0], t_sel = c->t_us[4];
    rc = copy_lp_outputs(c, count, obj, nullptr, nullptr, status, E.d_w + first);
    if (rc) return rc;   // some LP not optimal: nothing pushed
    const double obj_wsum = c->last_obj_wsum, obj_w = c->last_obj_w;
    const int64_t piv_sum = c->last_pivots_sum, ops_sum = c->last_ops_sum, eta_sum = c->last_eta_entries;
    const int64_t retries = c->last_retries;
    const int piv_max = c->last_pivots_max;
    float ms = 0, ms_key = 0;
    if (all) {
        HIPCHK(hipEventRecord(c->ev[2], c->stream));
        if ((rc = dvs_push_device(c, count, c->d_pi, nullptr))) return rc;
        HIPCHK(hipEventRecord(c->ev[3], c->stream));
        HIPCHK(hipEventSynchronize(c->ev[3]));
        hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
        c->last_push_reps = count;
    } else {
        HIPCHK(hipEventRecord(c->ev[5], c->stream));
        const int *d_list = nullptr;
        int U = 0;
        if ((rc = vkey_first_occurrences(c, count, c->d_vkey, c->d_status, &d_list, &U))) return rc;
        HIPCHK(hipEventRecord(c->ev[6], c->stream));
        HIPCHK(hipEventSynchronize(c->ev[6]));
        hipEventElapsedTime(&ms_key, c->ev[5], c->ev[6]);
        c->last_push_reps = U;
        c->push_rep_frac = (double)U / count;
        if (U > 0 && full) {
            const int m = c->L.m;
            if ((size_t)U > c->pi_rep_cap) {
                if ((rc = dalloc(&c->d_pi_rep, (size_t)U * m))) return rc;
                c->pi_rep_cap = U;
            }
            hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)std::min<size_t>(4096, ((size_t)U * m + 255) / 256)), dim3(256), 0,
                               c->stream, U, m, d_list, c->d_pi, c->d_pi_rep);
            HIPCHK(hipGetLastError());
            c->t_us[0] = t_lp;
            HIPCHK(hipEventRecord(c->ev[2], c->stream));
            if ((rc = dvs_push_device(c, U, c->d_pi_rep, nullptr))) return rc;
            HIPCHK(hipEventRecord(c->ev[3], c->stream));
            HIPCHK(hipEventSynchronize(c->ev[3]));
            hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
        } else if (U > 0) {
            LpRun r;
            r.want_pi = true;
            r.d_list = d_list;
            r.nlist = U;
            if ((rc = run_lp_ex(c, x, d_dv, count, r))) return rc;
            // the re-solve starts every representative from its recorded pick and repeats its
            // optimal solve; should one ever end otherwise, its pi row must not reach V
            HIPCHK(hipMemsetAsync(c->d_lpstats, 0, sizeof(unsigned long long), c->stream));
            hipLaunchKernelGGL(list_status_kernel, dim3((unsigned)std::min(256, (U + 255) / 256)), dim3(256), 0, c->stream, U,
                               d_list, c->d_status, c->d_lpstats);
            HIPCHK(hipGetLastError());
            unsigned long long bad = 0;
            HIPCHK(hipMemcpyAsync(&bad, c->d_lpstats, sizeof(bad), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            if (bad) return fail(TWOSD_E_LP, "solve_push: %llu of %d re-solved representatives not optimal; nothing pushed", bad, U);
            c->t_us[0] += t_lp;   // LP kernel time of the batch: main pass + representatives
            HIPCHK(hipEventRecord(c->ev[2], c->stream));
            if ((rc = dvs_push_device(c, U, c->d_pi, nullptr))) return rc;
            HIPCHK(hipEventRecord(c->ev[3], c->stream));
            HIPCHK(hipEventSynchronize(c->ev[3]));
            hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
        } else {
            c->t_us[0] = t_lp;
        }
        c->t_us[4] = t_sel;
        c->last_pivots_sum = piv_sum; c->last_ops_sum = ops_sum; c->last_pivots_max = piv_max;
        c->last_eta_entries = eta_sum;
        c->last_retries = retries;
    }
    c->last_obj_wsum = obj_wsum; c->last_obj_w = obj_w;   // of the batch, not of the representatives' re-solve
    c->t_us[1] = 1e3 * (ms + ms_key);
    if (new_size) *new_size = c->dvs.size;
    return TWOSD_OK;
}

extern "C" int twosd_last_push_mode(twosd_ctx *c, int *full) {
    if (!c || !full) return fail(TWOSD_E_ARG, "last_push_mode: NULL");
    *full = c->last_push_full;
    return TWOSD_OK;
}

extern "C" int twosd_last_push_reps(twosd_ctx *c, int *reps) {
    if (!c || !reps) return fail(TWOSD_E_ARG, "last_push_reps: NULL");
    *reps = c->last_push_reps;
    return TWOSD_OK;
}
