// twosd_internal.h -- shared declarations of libtwosd_hip.so (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>
#include "twosd_hip.h"

namespace twosd {

// ---- LP kernel envelope ----------------------------------------------------------
// One wavefront solves one scenario.  Row i of the basis lives in lane (i % 64),
// register slot (i / 64); R = ceil(m / 64) slots (template parameter).  Columns
// j (structural y then slacks) are strided over lanes, C = ceil((n + m) / 64) <= 64.
constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kMaxColsPerLane = 64;

// variable bound types (all nonbasic variables sit at 0)
enum : int { BT_Y = 0, BT_G = 1, BT_L = 2, BT_E = 3 };


// hypersparse kernel (lp_hyper.hip)
constexpr int kQueueStride = 32;   // queue heads one 128-B line apart
constexpr int kMaxQueueGroups = 64;
struct HyperParams {
    int m, n, k, N, kmax, ecap;
    int kcap;                                           // pivot cap (<= kmax; beyond: TWOSD_LP_ITER_LIMIT)
    int retry;                                          // a pool start ending non-optimal is retried from pool[0]
    const int *colptr, *rowidx; const double *val;      // W CSC
    const double *q; const int8_t *btype;
    const int *wcp, *wcc; const double *wcv;            // W by rows as CSR (columns ascending)
    const int *bcp, *bci; const double *bcv;            // B^{-1} CSC (MP + 1 column pointers, rows ascending)
    const int *brptr, *brcol; const double *brval;      // B^{-1} CSR (MP rows)
    // sliced ELL (entry e of slot s for lane l at [(slot_off[s] + e) * 64 + l]; padding: idx 0, val 0):
    // per pool basis p, rows i = 64t + lane of coef_e B_p^{-1}[i][row_e] as sliced ELL (R slots,
    // kslot pool-strided npool x (R+1), absolute into the concatenated kix (= e) / kv)
    const int *kslot, *kix; const double *kv;           // values B_p^{-1}[i][row_e] (x-independent)
    const double *kcoef;                                // k: coef_e(x) applied to the deltas
    const double *xbase;                                // MP
    const double *d0;                                   // 64*C reduced costs at B0 (lane-slot order j = 64c+lane)
    const int *hb0;                                     // MP
    const uint64_t *basic0, *fixedmask, *ubmask;        // 64
    const double *dv;                                   // N x k
    int *eidx; double *evals;                           // nslots x ecap sparse eta arena
    int *queue;                                         // qgroups heads, kQueueStride ints apart
    int qgroups;                                        // XCD-group work queues (>= 1)
    double *obj, *pi, *y;
    int *status, *iters;
    long long *ops;                                     // executed FMAs
    int *etan;                                          // N: eta-file entries of the final solve (nullable)
    unsigned long long *retries;                        // pool starts retried from the primary basis (nullable)
    unsigned long long *stamps;                         // [10] phase cycles (TWOSD_STAMPS builds only)
    // basis pool: xbase, hb0 (npool x MP), brptr / bcp (npool x (MP+1), absolute offsets),
    // basic0 (npool x 64), d0 (npool x 64C) are pool-strided
    int npool;
    const int *bnnz;                                    // npool: nnz of B^{-1} (ops accounting)
    int *head_out;                                      // N x m final basis (nullable)
    int *pool_pick;                                     // N pool basis per scenario (in; npool > 1)
    const int *order;                                   // N visiting order of the scenarios (nullable)
    // dual key mode (solve_push): per scenario a 64-bit key of its optimal dual (from the
    // maintained slack reduced costs, 24 significant bits); with pi == y == nullptr the vertex
    // recovery is skipped
    unsigned long long *vkey;                           // N (nullable)
    double key_zero;                                    // key components <= key_zero (1 + max) snap to 0
    int pi_by_pos;                                      // pi / head row = queue position instead of scenario
    // basis key (pool refresh): sum of mix64(j) over the basic columns of the optimal basis
    unsigned long long *bkey;                           // N (nullable)
    // eta-file output (pool refresh, list mode): per list position the start pool basis, the
    // pivot count (-1: did not fit), the pivot rows and offsets (kmax / kmax + 1 per position)
    // and the eta entries, appended at an atomically claimed offset of a shared arena
    int *eo_pb, *eo_K, *eo_off, *eo_etap, *eo_etaoff;   // nullable (eo_K == nullptr: off)
    int *eo_eidx; double *eo_evals;
    unsigned long long *eo_used; long long eo_cap;      // claim counter (64-bit); arena entries (<= INT32_MAX)
};

// ---- device pool build of a refresh (pool_gpu.hip) ---------------------------------
// Source a of a build: a = 0 the primary basis (start pool basis 0, no etas, head0), a >= 1
// the eta file and head of training scenario src_row[a - 1] of the refresh.  Every column of
// B^{-1} is the start basis's column pushed through the eta file (pg_ftran_kernel, two
// passes: max / counts, then the kept entries into an intermediate CSC), checked and counted
// (pg_count_kernel), and written into the pool-strided arrays of upload_pool /
// prepare_elements at host-computed offsets (pg_fill_kernel).
struct PgArgs {
    int m, n, MP, CH, R9, k, kmax, npool_old;
    const int *colptr, *rowidx; const double *val, *q; const int8_t *btype; const int *pos_row;
    const int *bcp0, *bci0; const double *bcv0;          // start pool: B^{-1} CSC (pool-strided)
    const int *eo_pb, *eo_K, *eo_off, *eo_etap, *eo_etaoff, *eo_eidx; const double *eo_evals;
    const int *head0, *heads;                            // primary head (m); heads (eta-file rows)
    const int *src_row;                                  // source a >= 1: eta-file / head row src_row[a - 1]
    const int *gheads;                                   // fill only (nullable): head of source a >= 1 at
                                                         //   gheads + (a - 1) m (a gathered source table)
    int a0;                                              // first source of the launch
    double *amax;                                        // nsrc (-1: source unusable)
    int *nzc, *keptc;                                    // nsrc x m: nonzeros / kept entries per column
    int *nztot;                                          // nsrc: sum of nzc
    const long long *inter_off;                          // nsrc: intermediate CSC offsets
    int *inter_row; double *inter_val;
    int *rowcnt, *erowcnt;                               // nsrc x m
    int *tot;                                            // nsrc x 4: nnz, element entries, ELL rows, records
    int *valid;                                          // nsrc
    // the first FTRAN pass keeps its nonzeros (rows ascending per column) in a scratch of sc_cap
    // entries per source, columns at sc_off (claimed in completion order); a source whose nztot
    // exceeds sc_cap is left to the second FTRAN pass (sc_cap = 0: every source)
    long long sc_cap;
    int *sc_row, *sc_off; double *sc_val;                // nsrc x sc_cap, nsrc x m, nsrc x sc_cap
};
struct PgFill {
    int P0, P;                                           // pool bases [P0, P0 + grid) of P
    const int *map;                                      // P: source of pool basis p
    const int *off;                                      // P x 4: offsets (prefix of tot over the pool)
    int sel_total;
    const double *d0_primary;                            // 64 CH: d0 of pool[0], kept as uploaded
    int *brptr, *brcol; double *brval; int *bcp, *bci; double *bcv;
    int *kp, *ke; double *kraw; int *kslot, *kix; double *kv;
    int *hb0; uint64_t *basic0; int *bnnz; double *d0; int *sel_ptr;
};
int pg_supported(int m, int n, int kmax);                // the LDS layouts fit
hipError_t pg_launch_ftran(const PgArgs &A, int pass, int nb, hipStream_t s);
hipError_t pg_launch_gather(const PgArgs &A, int nb, hipStream_t s);
hipError_t pg_launch_count(const PgArgs &A, int nb, hipStream_t s);
hipError_t pg_launch_fill(const PgArgs &A, const PgFill &F, int np, hipStream_t s);

// splitmix64 finalizer (basis keys: host and device must agree)
__host__ __device__ inline unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// warm-start selection over the basis pool (pool_select_kernel in lp_hyper.hip)
struct PoolSelParams {
    int N, k, npool;
    const double *dv;                                   // N x k
    const double *kcoef;                                // k: coef_e(x)
    const float *cinf;                                  // npool: infeasibility of the constant rows
    const int *sptr, *send;                             // npool: [sptr[p], send[p]) = records of basis p
    const int2 *rec;                                    // (float bits, code): row start (sign-folded xbase_i,
                                                        //   -1); entry (sign * B^{-1}[i][row_e], e * 65 * 8)
    int *pick;                                          // N out
    float cw;                                           // key = sum |infeas| + cw * #infeasible rows
    float *key;                                         // N out (nullable): key of the pick
    float *pkey; int *ppick;                            // split x N partials (nullable: no split)
};
// second level of the two-level pool selection: scenarios in `order` (grouped by their
// level-1 pick) try the candidate bases of their level-1 pick (cand: nl1 x ncand, -1 pad)
struct PoolRefineParams {
    int N, k, ncand;
    const double *dv, *kcoef;
    const float *cinf;
    const int *sptr, *send;
    const int2 *rec;
    const int *order, *cand;
    int *pick;                                          // N in (level 1) / out
    const float *key;                                   // N: level-1 key
    float cw;
    float *pkey; int *pci;                              // split x N partials (nullable: no split)
};
hipError_t launch_pool_refine(const PoolRefineParams &p, hipStream_t s);
size_t pool_select_lds_bytes(int k);
// chunks of the pool / candidate lists per scenario tile for a batch of N (<= 16)
int pool_select_split(int N, int npool);
int pool_refine_split(int N, int ncand);
// stable sort of scenarios [0, N) by pool pick -> order (pool_sort.hip); tmp == nullptr: size query
hipError_t sort_by_pool(const int *pick, int *order, int N, int npool, void *tmp, size_t *tmp_bytes, hipStream_t s);
hipError_t launch_pool_select(const PoolSelParams &p, hipStream_t s);
size_t hyper_lds_bytes(int R, int C, int kmax, int k);   // C = column slots (hyper_cols_per_lane(n + m))
int hyper_rows_per_lane(int m);
int hyper_cols_per_lane(int ncols);
hipError_t launch_hyper(int R, int C, const HyperParams &p, int nblocks, size_t lds, hipStream_t s);
int hyper_max_blocks_per_cu(int R, int C, int kmax, int k);


// ---- on-device scenario sampler (sampler.hip)
struct SampleParams {
    int N, k;
    unsigned long long seed, first_index;
    const int *kind;                      // k: 0 DISCRETE, 1 NORMAL, 2 UNIFORM
    const int *off;                       // k + 1: DISCRETE support ranges into val / prob
    const double *val, *prob;             // DISCRETE support (ascending) and probabilities
    const double *p0, *p1;                // NORMAL mean / sd, UNIFORM left / right
    const double *tmpl;                   // k template values
    double *out;                          // N x k deltas
};
hipError_t launch_sample(const SampleParams &S, hipStream_t st);

// ---- host-side setup (host_basis.cpp) --------------------------------------------
struct HostLP {
    int m = 0, n = 0;
    std::vector<int> colptr, rowidx;   // W CSC, 0-based
    std::vector<double> val, q;
    std::vector<char> sense;           // 'G','L','E'
};
// dense inverse (row-major m x m), partial pivoting; false if singular
bool dense_inverse(int m, const std::vector<double> &A, std::vector<double> &Ainv);
void basis_matrix(const HostLP &L, const std::vector<int> &head, std::vector<double> &B);
// setup solve from the slack basis (explicit-inverse revised dual simplex with periodic
// re-inversion); returns LP status, fills head (optimal basis) and obj
int setup_solve(const HostLP &L, const std::vector<double> &b, std::vector<int> &head, double &obj,
                int &iters, std::string &err);
// max dual infeasibility of basis head (0 = dual feasible); pi0 = c_B' B^{-1}
double basis_dual_infeasibility(const HostLP &L, const std::vector<int> &head,
                                const std::vector<double> &Binv, std::vector<double> &pi0);
// pool refresh: rows of B^{-1} = E_K..E_1 B0^{-1} (CSR, columns ascending, |v| <= 1e-14 max
// dropped) from B0^{-1}'s rows and an eta file (pivot rows etap[K], entries [etaoff[t],
// etaoff[t+1]) of (eidx, evals), the pivot row's entry being 1 / alpha_rq)
void compose_binv(int m, const std::vector<int> &rptr0, const std::vector<int> &rcol0, const std::vector<double> &rval0,
                  int K, const int *etap, const int *etaoff, const int *eidx, const double *evals, std::vector<int> &rptr,
                  std::vector<int> &rcol, std::vector<double> &rval);
// max dual infeasibility of head given pi0 = c_B' B^{-1}; max |B^{-1} a_{head[i]} - e_i| over
// `probes` positions i of the CSR rows of B^{-1}
double sparse_dual_infeasibility(const HostLP &L, const std::vector<int> &head, const std::vector<double> &pi0);
double sparse_basis_residual(const HostLP &L, const std::vector<int> &head, const std::vector<int> &rptr,
                             const std::vector<int> &rcol, const std::vector<double> &rval, int probes);

// ---- dual vertex set kernels (dvs_kernel.hip) ------------------------------------
struct DvsDevice {
    int m = 0, cap = 0, size = 0;
    double *V = nullptr;          // cap x m
    uint64_t *hash = nullptr;     // cap: reference hash (bits of round16(L1 norm))
    uint64_t *fp = nullptr;       // cap: fingerprint of (hash, rounded components)
    int *table = nullptr;         // tcap slots: vertex id or -1
    int tcap = 0;                 // power of two
};

// ---- cut kernels (cut_kernel.hip) --------------------------------------------------
}  // namespace twosd
