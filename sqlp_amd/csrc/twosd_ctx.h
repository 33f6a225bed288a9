// twosd_ctx.h -- the opaque twosd_ctx behind the C ABI (library-internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <map>
#include <vector>
#include "twosd_internal.h"

namespace twosd {

struct EpiDevice {
    double *d_dv = nullptr;       // count x k scenario deltas (value - template value)
    double *d_w = nullptr;        // count weights
    size_t dv_cap = 0, w_cap = 0;
    int count = 0;
    double total_weight = 0.0;    // epigraph.jl:89, accumulated in insertion order
    std::vector<double> w_host;
};

// one warm-start basis of the pool (pool[0] is the primary basis head0)
struct PoolBasis {
    std::vector<int> head;        // m basic columns (0-based over [y; slacks])
    std::vector<double> Binv;     // m x m row-major
    std::vector<double> pi0;      // c_B' B^{-1}
    std::vector<int> rptr, rcol;  // B^{-1} rows, CSR (|v| > 1e-14 max|B^{-1}|)
    std::vector<double> rval;
    bool dev_only = false;        // built on the device (refresh): rptr / rcol / rval / pi0 are
                                  // fetched from the pool arrays when the host needs them
    int hb_row = -1;              // >= 0: head not materialised yet; row of c->pool_hb (4 head + type)
};

}  // namespace twosd

struct twosd_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[8] = {};
    int num_cus = 256;
    int kmax_override = 0;
    int train_kcap = 0;           // pivot cap of the refresh training solves (> 0; 0: auto; < 0: none)
    double piv_mean_ref = 0.0;    // mean pivots of the last large batch solve (the auto cap's scale)
    int64_t piv_ref_sum = 0, piv_ref_n = 0;   // that batch's pivot sum and size (ranks agree on one cap)
    int last_train_opt = 0;       // optimal training scenarios of the last refresh
    double t_us[5] = {0, 0, 0, 0, 0};   // LP kernel, dedup, cut partial, cut finalize, pool select
    // template
    bool has_template = false, has_basis = false;
    twosd::HostLP L;              // W CSC, q, sense (host)
    int n1 = 0, R = 0, MP = 0, C = 0, k = 0;
    std::vector<double> r, T;     // r (m2), dense T (m2 x n1, row-major)
    std::vector<int> pos_row, pos_col;
    int *d_colptr = nullptr, *d_rowidx = nullptr;
    double *d_val = nullptr, *d_q = nullptr;
    int8_t *d_btype = nullptr;
    uint64_t *d_fixedmask = nullptr, *d_ubmask = nullptr;
    // basis
    std::vector<int> head0;
    int *d_hb0 = nullptr;
    uint64_t *d_basic0 = nullptr;
    double *d_xbase = nullptr;
    std::vector<twosd::PoolBasis> pool;   // warm-start basis pool, pool[0] = head0
    // pool selection data (per x, prepare_x): constant-row infeasibility, active rows, entries
    float *d_sel_cinf = nullptr;
    int *d_sel_ptr = nullptr, *d_sel_code = nullptr;   // code: (code, float bits) record pairs
    int *d_sel_end = nullptr;            // npool: end of each basis's records (begin = d_sel_ptr, static capacity)
    // x-independent element rows of the pool on the device (CSR, pool-strided kp: npool x (m+1)
    // absolute offsets into ke / kraw), inputs of the device selection-stream build
    int *d_kp = nullptr, *d_ke = nullptr;
    double *d_kraw = nullptr;
    double *d_xaux = nullptr;            // per x: b (m), coef (k), box lo (k), box hi (k)
    size_t xaux_cap = 0;
    int64_t sel_cap_total = 0;           // records the static capacity layout holds
    size_t sel_code_cap = 0;             // records d_sel_code has room for
    int64_t sel_nnz = 0, sel_rows = 0;
    float sel_cw = 0.0f;                 // pool selection key: sum |infeas| + sel_cw * #infeasible rows (per x)
    std::vector<double> dist_mad;        // mean absolute deviation E|V_e - E V_e| of each random element
    std::vector<double> sel_lo, sel_hi;   // training box of the deltas (empty: no row pruning)
    int *d_bnnz = nullptr;        // npool: nnz of each pool B^{-1} (FMA accounting)
    int *d_head_out = nullptr, *d_pool_pick = nullptr;   // optional LP outputs (pool building)
    size_t head_cap = 0, pick_cap = 0;
    // two-level pool selection (twosd_pool_build_candidates): level 1 over pool[0, pool_l1),
    // level 2 over the candidate bases of the level-1 pick (d_cand: pool_l1 x pool_ncand)
    int pool_l1 = 0, pool_ncand = 0;
    int *d_cand = nullptr;
    // candidate lists of the last refresh, built on the host by the next two-level selection while
    // its level-1 pass runs (select_pool); pool_l1 / pool_ncand already describe them
    std::vector<int> cand_p1, cand_pf;
    int cand_pl1 = 0, cand_pnc = 0;
    bool cand_pending = false;
    int *d_cpick = nullptr;       // candidate picks of the training scenarios (grow-only)
    float *d_sel_key = nullptr;
    float *d_sel_pkey = nullptr;          // chunked selection partials (split x N)
    int *d_sel_ppick = nullptr;
    size_t sel_pcap = 0;
    size_t key_cap = 0;
    int *d_order = nullptr;       // LP visiting order grouped by pool basis
    char *d_sort_tmp = nullptr;
    size_t order_cap = 0, sort_tmp_bytes = 0;
    bool want_head = false;
    bool prep_valid = false;
    bool k_valid = false;         // K rows / ELL of the pool (depend on the pool and the positions)
    double *d_kcoef = nullptr;    // k: coef_e(x) = 1 (RHS element) or -x[col] (T element)
    std::vector<double> prep_x;
    // capacities of the per-x device arrays (prepare_x re-uploads in place, no hipFree/hipMalloc per x)
    size_t xbase_cap = 0, kcoef_cap = 0;
    // hypersparse kernel data
    int CH = 0;                   // column slots per lane of the hypersparse kernel
    int *d_kslot = nullptr, *d_kix = nullptr;
    double *d_kv = nullptr, *d_d0 = nullptr;
    int *d_bcp = nullptr, *d_bci = nullptr;
    double *d_bcv = nullptr;
    int *d_wcp = nullptr, *d_wcc = nullptr;   // W by rows (CSR) for the segmented pricing scatter
    double *d_wcv = nullptr;
    int *d_brptr = nullptr, *d_brcol = nullptr;
    double *d_brval = nullptr;
    int *d_eidx = nullptr;
    double *d_evals = nullptr;
    size_t earena_slots = 0;
    int earena_cap = 0;
    int64_t last_iterlimit = 0;
    int64_t b0_nnz = 0;
    unsigned long long *d_stamps = nullptr;
    int last_ops_width = 1;
    // LP workspace + outputs
    int *d_queue = nullptr;
    unsigned long long *d_lpstats = nullptr;   // lp_stats_kernel output (5 words)
    double *d_obj = nullptr, *d_pi = nullptr, *d_y = nullptr;
    int *d_status = nullptr, *d_iters = nullptr;
    long long *d_ops = nullptr;
    int *d_etan = nullptr;
    int64_t last_eta_entries = 0;
    int64_t last_retries = 0;     // pool starts of the last batch retried from the primary basis
    int64_t last_ops_sum = 0;
    int out_cap = 0;
    size_t pi_cap = 0, y_cap = 0;
    double *d_dvtmp = nullptr;
    size_t dvtmp_cap = 0;
    int last_lp_N = 0, last_lp_blocks = 0;
    int64_t last_pivots_sum = 0;
    int last_pivots_max = 0;
    // weighted objective sum of the last batch (sum_s w_s obj_s, fixed-order reduction) and its weight
    double last_obj_wsum = 0.0, last_obj_w = 0.0;
    double *d_objpart = nullptr;
    // scenario distributions (on-device sampler)
    bool has_dist = false;
    int *d_dist_kind = nullptr, *d_dist_off = nullptr;
    double *d_dist_val = nullptr, *d_dist_prob = nullptr, *d_dist_p0 = nullptr, *d_dist_p1 = nullptr, *d_dist_tmpl = nullptr;
    // epigraphs
    std::vector<twosd::EpiDevice> epis;
    // dual vertex set
    twosd::DvsDevice dvs;
    void *dvs_ws = nullptr;       // dvs scratch (dvs_kernel.hip)
    // cut workspace (cut_kernel.hip)
    void *cut_ws = nullptr;
    // dual-vertex key workspace (vkey.hip) and the key output of the LP kernel
    void *vkey_ws = nullptr;
    unsigned long long *d_vkey = nullptr, *d_bkey = nullptr;
    size_t vkey_cap = 0, bkey_cap = 0;
    // eta-file output of a pool refresh (list positions x kmax / kmax + 1, shared entry arena)
    int *d_eo_pb = nullptr, *d_eo_K = nullptr, *d_eo_off = nullptr, *d_eo_etap = nullptr, *d_eo_etaoff = nullptr;
    int *d_eo_eidx = nullptr;
    unsigned long long *d_eo_used = nullptr;
    double *d_eo_evals = nullptr;
    size_t eo_rows = 0, eo_cap = 0;
    int eo_kmax = 0;
    double last_refresh_ms[5] = {0, 0, 0, 0, 0};   // train solves, re-solves, compose, upload, total
    int *d_refresh_sel = nullptr;                  // refresh: scenarios to re-solve
    size_t refresh_sel_cap = 0;
    int box_epi = -1, box_first = -1, box_count = -1, box_n = -1;   // training range of sel_lo / sel_hi
    // device pool build of a refresh (pool_gpu.hip): intermediate CSC, per-source counts and
    // checks, pool map / offsets, primary head and d0
    double *d_pg_amax = nullptr, *d_pg_d0p = nullptr, *d_pg_ival = nullptr;
    int *d_pg_irow = nullptr;
    long long *d_pg_ioff = nullptr;
    int *d_pg_cnt = nullptr, *d_pg_tot = nullptr, *d_pg_valid = nullptr, *d_pg_head0 = nullptr;
    int *d_pg_map = nullptr, *d_pg_off = nullptr, *d_pg_pos = nullptr;
    // FTRAN results of the first pass kept for the gather (pool_gpu.hip): per source sc_cap entries
    int *d_pg_scrow = nullptr, *d_pg_scoff = nullptr;
    double *d_pg_scval = nullptr;
    long long pg_sc_cap = 0;                       // entries per source of the last build (0: first build)
    // distributed refresh (twosd_refresh_*): this rank's training keys, its pack of built
    // sources, and the source table gathered from all ranks
    std::vector<unsigned long long> rt_keys;
    std::vector<int> rt_counts, rt_reps;
    std::vector<double> rt_lo, rt_hi;     // training box of this rank's slice
    int rt_epi = -1, rt_first = -1, rt_count = -1, rt_n = -1, rt_nown = -1;
    bool rt_trained = false;              // a twosd_refresh_train* ran since the last assemble
    long long rt_nz0 = 0;                 // intermediate entries of the primary (local source 0)
    int rt_nsrc_local = 0;
    char *d_rt_pack = nullptr;
    int *d_gs_heads = nullptr, *d_gs_cnt = nullptr, *d_gs_tot = nullptr, *d_gs_valid = nullptr, *d_gs_irow = nullptr;
    long long *d_gs_ioff = nullptr;
    double *d_gs_ival = nullptr;
    void *d_gs_seg = nullptr;             // copy-segment list of the gather unpack
    size_t gs_seg_cap = 0;
    // pinned host staging buffers of the pool upload, kept across uploads (no page faults,
    // no unmapping per refresh, page-locked copies)
    int *pool_hb = nullptr;       // pinned: the heads of the last device-built pool (P x MP, 4 head + type)
    size_t pool_hb_cap = 0;
    bool pool_hb_valid = false;   // pool_hb holds d_hb0 of the current pool
    void *stage[16] = {};
    size_t stage_bytes[16] = {};
    std::map<const void *, size_t> dcap;   // element capacity of grow-only device arrays (by member address)
    int last_push_reps = 0;       // representatives re-solved by the last solve_push
    double push_rep_frac = 0.0;   // representatives / scenarios of the last keyed solve_push (push mode choice)
    int last_push_full = 0;       // 1: the last solve_push recovered every dual in its main pass
    double *d_pi_rep = nullptr;   // the representatives' dual rows gathered for the push (full mode)
    size_t pi_rep_cap = 0;
};

namespace twosd {
int fail(int code, const char *fmt, ...);
int poison_byte(int family);   // TWOSD_POISON test hook (-1: off); family bit 1 dalloc, 2 dgrow, 4 cut workspace
template <typename T>
int dgrow(T **p, size_t *cap, size_t count, size_t keep, hipStream_t s);
int prepare_x(twosd_ctx *c, const double *x);
int run_lp(twosd_ctx *c, const double *x, const double *d_dv, int N, bool want_pi, bool want_y);
// options of run_lp_ex: vertex keys instead of pi (solve_push), or a list of scenarios to
// re-solve from their recorded pool picks with pi at the list position
struct LpRun {
    bool want_pi = false, want_y = false, want_key = false;
    bool want_bkey = false;       // basis keys into c->d_bkey
    bool want_etas = false;       // eta files into c->eo (pool refresh), rows by list position / scenario
    bool want_head = false;       // final heads into c->d_head_out, rows by list position / scenario
    const int *d_list = nullptr;  // list mode: scenarios (indices into d_dv) to solve, no selection
    int nlist = 0;
    int kcap = 0;                 // > 0: pivot cap below kmax, no retry from the primary basis (refresh training)
};
int run_lp_ex(twosd_ctx *c, const double *x, const double *d_dv, int N, const LpRun &o);
// vkey.hip
int vkey_first_occurrences(twosd_ctx *c, int N, const unsigned long long *d_vkey, const int *d_status, const int **d_list,
                           int *U, const int **d_counts = nullptr);
void vkey_free(twosd_ctx *c);
// dual vertex set (dvs_kernel.hip)
int dvs_init(twosd_ctx *c);
void dvs_free(twosd_ctx *c);
// d_hash / d_fp / d_nan: keys precomputed by the producer (nullable: computed here)
int dvs_push_device(twosd_ctx *c, int count, const double *d_pis, int *d_out_index, const uint64_t *d_hash = nullptr,
                    const uint64_t *d_fp = nullptr, const int *d_nan = nullptr);
// cut (cut_kernel.hip)
void cut_free(twosd_ctx *c);
void cut_invalidate_pk(twosd_ctx *c);
void cut_truncate_pk(twosd_ctx *c, int size);   // V truncated to size: PK rows past it are stale
}  // namespace twosd
