/*
 * twosd_hip.h -- C ABI of libtwosd_hip.so, the MI355X (gfx950) implementation of the
 * TwoSD per-iteration scenario-subproblem + cut-generation hot path.
 *
 * Reference: yhz0/SQLP (module TwoSD, pure Julia) @ 2025-02-19.  The reference has no
 * FFI/plugin API for this path (src/sd_algorithm/plugin/ holds 0-byte files); the
 * entry points below are what a Julia `ccall` shim binds to add
 * accelerated methods for the same generic functions.  Each entry cites the reference
 * function it replaces.
 *
 * Conventions
 *   - All calls are synchronous: outputs are valid on return.  Host buffers are owned by
 *     the caller; the library copies in and out.  Device memory is owned by the context.
 *   - Return value: TWOSD_OK (0) or a negative TWOSD_E_* code; twosd_last_error() gives a
 *     thread-local message.  A context is not re-entrant; distinct contexts are
 *     independent (one context per GPU / process).
 *   - Indices: `index_base` = 1 accepts Julia's 1-based SparseMatrixCSC arrays directly.
 *   - Stage-2 LP of one scenario w at first-stage x (smps_routines.jl:50-62):
 *         min q'y  s.t.  W y  (G: >=, L: <=, E: ==)  r_w - T_w x,   y >= 0
 *     duals pi follow JuMP's MIN convention (G rows >= 0, L rows <= 0, E free;
 *     pi = d obj / d rhs), so obj = pi . (r_w - T_w x).
 *   - Variables of the simplex basis ("head"): j < n2 is structural y_j; j = n2 + i is the
 *     slack of row i.
 */
#ifndef TWOSD_HIP_H
#define TWOSD_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct twosd_ctx twosd_ctx;

enum {
    TWOSD_OK = 0,
    TWOSD_E_ARG = -1,        /* bad argument (sizes, indices, NULL)          */
    TWOSD_E_DEVICE = -2,     /* HIP runtime / kernel launch failure           */
    TWOSD_E_STATE = -3,      /* call out of order (e.g. no template yet)      */
    TWOSD_E_LP = -4,         /* LP not solved to optimality (see status[])    */
    TWOSD_E_UNSUPPORTED = -5 /* template outside the kernel's envelope        */
};

/* per-scenario LP status (status[] outputs) */
enum { TWOSD_LP_OPTIMAL = 0, TWOSD_LP_INFEASIBLE = 1, TWOSD_LP_ITER_LIMIT = 2, TWOSD_LP_NUMERIC = 3 };

/* Thread-local message for the last failing call on this thread. */
const char *twosd_last_error(void);

/* Library version string. */
const char *twosd_version(void);

/* Create a context on HIP device `device` (one context per GPU / rank). */
int twosd_create(int device, twosd_ctx **out);
int twosd_destroy(twosd_ctx *ctx);

/*
 * Stage-2 template (replaces extract_coefficients, subprob.jl:15-69, and the JuMP model
 * held by spStageProblem, prob.jl:10-15).
 *   T: m2 x n1 CSC (colptr[n1+1], rowval[nnzT], nzval[nnzT]); W: m2 x n2 CSC.
 *   q[n2], r[m2], sense[m2] in {'G','L','E'}, ylb/yub[n2] (only [0, +inf) is supported:
 *   the reference warns on other bounds, subprob.jl:19-26).
 * Re-setting the template clears basis, scenarios, dual vertex set and cuts.
 */
int twosd_set_template(twosd_ctx *ctx, int m2, int n1, int n2,
                       const int64_t *T_colptr, const int64_t *T_rowval, const double *T_nzval,
                       const int64_t *W_colptr, const int64_t *W_rowval, const double *W_nzval,
                       const double *q, const double *r, const char *sense,
                       const double *ylb, const double *yub, int index_base);

/*
 * Random element positions of a scenario (spSmpsScenario entries, smps_sto.jl:135):
 * element e sits at stage-2 row row[e]; col[e] = -1 for an RHS entry, else the
 * first-stage column of a T entry (delta_coefficients, subprob.jl:104-121).
 */
int twosd_set_random_positions(twosd_ctx *ctx, int k, const int *row, const int *col, int index_base);

/*
 * Warm-start basis shared by every scenario (dual feasible for all RHS).
 * twosd_compute_basis solves the LP at x for the scenario `values` (k entries; NULL =
 * template rhs) from the slack basis once on the host and installs its optimal basis.
 * twosd_set_basis installs a caller-provided basis (m2 variable indices, 0-based).
 */
int twosd_compute_basis(twosd_ctx *ctx, const double *x, const double *values);
int twosd_set_basis(twosd_ctx *ctx, const int *head);
int twosd_get_basis(twosd_ctx *ctx, int *head);

/* Warm-start basis pool (no reference counterpart: the reference warm-starts each
 * solve from the solver's previous basis, smps_routines.jl:50-62).  With only the
 * RHS random, every optimal basis of one scenario is dual feasible for all of them;
 * the LP kernel starts each scenario from the pool basis with the least primal
 * infeasibility.  Results are the same optimal vertices (same tie rules) -- only
 * the pivot count changes.  set_basis / compute_basis reset the pool to one basis.
 *   pool_add_basis: append a (dual-feasible) basis; *added = 0 if already present.
 *   pool_build: solve training scenarios [first, first+count) of epigraph epi at x
 *     and add their optimal bases, most frequent first, up to max_pool bases. */
int twosd_pool_add_basis(twosd_ctx *ctx, const int *head, int *added);
int twosd_pool_build(twosd_ctx *ctx, int epi, const double *x, int first, int count, int max_pool,
                     int *pool_size);
/* Two-level pool selection: level 1 over pool[0, level1), level 2 over the ncand bases
 * that a flat selection over the whole pool picks most often for the training scenarios
 * [first, first+count) of epi at x sharing the level-1 pick.  Cuts the selection cost of a
 * large pool to about that of its first level1 bases.  level1 = 0: flat selection;
 * ncand <= 1024.  Reset by any change of the pool.  The lists themselves are counted on the
 * host by the next two-level selection while its level-1 pass runs (twosd_pool_set_candidates
 * likewise): an allocation failure of their upload is reported by that solve. */
int twosd_pool_build_candidates(twosd_ctx *ctx, int epi, const double *x, int first, int count, int level1,
                                int ncand);
/* Rebuild the pool at x: solve the training scenarios [first, first+count) of epi at x from
 * the current pool and replace the pool by the primary basis plus their max_pool - 1 most
 * frequent optimal bases (ties: first occurrence).  A pool's bases are optimal near the x they
 * were harvested at, so a first-stage point far from the last one (an SD candidate, the x
 * of an evaluate) gets a pool of its own.  B^{-1} of each new basis is composed from its start
 * basis and the eta file of its training solve (no refactorisation), on the device by default
 * (TWOSD_REFRESH_HOST=1: on the host, then uploaded; same pool).  Selection becomes flat
 * (candidate lists reset).  last_refresh_ms: [training solves, basis keys + selection, pool
 * build (device; host path: composition), host upload (host path only), total] of the last
 * refresh. */
int twosd_pool_refresh(twosd_ctx *ctx, int epi, const double *x, int first, int count, int max_pool,
                       int *pool_size);
int twosd_last_refresh_ms(twosd_ctx *ctx, double *ms5);

/* Distributed refresh (one rank per GPU, the pool replicated; no reference counterpart: the
 * reference is single-process).  The twosd_pool_refresh of all ranks' training scenarios, split:
 *   1. twosd_refresh_train: solve this rank's training slice [first, first+count) of epi at x;
 *      *n_bases = its distinct optimal bases; box_lo/box_hi[k] (nullable) = the slice's delta box.
 *      twosd_refresh_train_bases: their 64-bit keys, counts and first scenarios (ascending).
 *   2. the caller all-gathers (keys, counts, first scenarios) and selects, identically on every
 *      rank, the max_pool - 1 most frequent bases (ties: first occurrence in rank order), each
 *      owned by the rank of its first occurrence.
 *   3. twosd_refresh_build_local: compose B^{-1} of the n_own bases this rank owns (its first
 *      scenarios reps[], in selection order) into a pack of *pack_bytes bytes;
 *      twosd_refresh_pack copies it to a caller DEVICE buffer for the all-gather.
 *   4. twosd_refresh_assemble: from the G gathered packs (DEVICE, `stride` bytes apart, rank
 *      order), the pool = primary + the sources order[0, R) (source ids: 1 + the rank-major
 *      position of a base among all packs), with the union box_lo/box_hi[k] of the slices.
 *      R = 0 (no optimal training scenario on any rank) keeps the current pool, as
 *      twosd_pool_refresh does.
 * Selection becomes flat; twosd_pool_candidate_picks / twosd_pool_set_candidates split the
 * two-level candidate lists the same way (picks of each rank's slice, lists from all picks). */
int twosd_refresh_train(twosd_ctx *ctx, int epi, const double *x, int first, int count, int *n_bases, double *box_lo,
                        double *box_hi);
/* The training solve of step 1 under a cap the ranks agree on: kcap > 0 pivots (<= 0: none), one
 * launch, no retry; *n_optimal = training scenarios of the slice that ended optimal.  The caller
 * derives kcap from every rank's twosd_refresh_cap_stats (pivot sum and size of the last batch of
 * >= 4096 scenarios: 3 x the global mean, at least 32) and, when fewer than half of ALL ranks'
 * training scenarios ended optimal, calls it again with kcap = 0 on every rank -- the rule
 * twosd_pool_refresh applies to one rank, decided once for all of them. */
int twosd_refresh_train_ex(twosd_ctx *ctx, int epi, const double *x, int first, int count, int kcap, int *n_bases,
                           int *n_optimal, double *box_lo, double *box_hi);
int twosd_refresh_cap_stats(twosd_ctx *ctx, int64_t *pivots_sum, int64_t *scenarios);
/* The training pivot cap twosd_pool_refresh would use for a last large batch of `scenarios`
 * solves with `pivots_sum` pivots in all, under this context's setting (and TWOSD_TRAIN_KCAP):
 * > 0 the setting, < 0 none (0), auto max(32, ceil(3 sum / n)).  The distributed refresh calls it
 * with the all-reduced sums, so every rank and the single-rank refresh apply one rule.  Host code
 * only; ctx may be NULL (setting 0). */
int twosd_training_cap(twosd_ctx *ctx, int64_t pivots_sum, int64_t scenarios, int *cap);
/* Step 2 of the distributed refresh, identical on every rank (host code, no context): over the n
 * bases all ranks list (twosd_refresh_train_bases, concatenated in rank order; rank_of[i] = the
 * listing rank), a key listed by several ranks counts the sum of its counts and belongs to its
 * first occurrence; the min(distinct, max_pool - 1) largest totals, ties by first occurrence, go
 * to owner[] / rep[] (the owning rank and its first scenario), *npick of them. */
int twosd_select_refresh_bases(const uint64_t *keys, const int64_t *counts, const int64_t *reps, const int32_t *rank_of,
                               int n, int max_pool, int64_t *owner, int64_t *rep, int *npick);
int twosd_refresh_train_bases(twosd_ctx *ctx, uint64_t *keys, int *counts, int *reps);
int twosd_refresh_build_local(twosd_ctx *ctx, int n_own, const int *reps, int64_t *pack_bytes);
int twosd_refresh_pack(twosd_ctx *ctx, void *d_dst);
int twosd_refresh_assemble(twosd_ctx *ctx, int G, const void *d_packs, int64_t stride, int R, const int *order,
                           const double *box_lo, const double *box_hi, int *pool_size);
int twosd_pool_candidate_picks(twosd_ctx *ctx, int epi, const double *x, int first, int count, int level1, int *p1,
                               int *pf);
int twosd_pool_set_candidates(twosd_ctx *ctx, int level1, int ncand, int n, const int *p1, const int *pf);
int twosd_pool_size(twosd_ctx *ctx, int *size);
int twosd_pool_get(twosd_ctx *ctx, int p, int *head);
/* Pool basis each scenario of the last LP batch started from (first N of it; 0 = the
 * primary basis, also after a pool start was retried from it). */
int twosd_last_pool_picks(twosd_ctx *ctx, int N, int *picks);

/* Drop the per-x data cached from the last x (x_B of every pool basis, coef_e(x), the
 * pool-selection stream, the cut's per-x products); the next call at any x rebuilds it.
 * Results never depend on it -- benchmarks call it so each pass pays its per-x setup. */
int twosd_invalidate_x(twosd_ctx *ctx);

/* Epigraphs (sdEpigraph, epigraph.jl:17-61): per-epigraph scenario pool + weights. */
int twosd_epigraph_create(twosd_ctx *ctx, int *epi_out);
/* add_scenario!(epi, w, weight) batched (epigraph.jl:81-96): values[N*k] are the
 * scenario's element values in position order; weights[N] (NULL = all 1.0). */
int twosd_add_scenarios(twosd_ctx *ctx, int epi, int N, const double *values, const double *weights);
int twosd_epigraph_info(twosd_ctx *ctx, int epi, int *num_scenarios, double *total_weight);

/*
 * On-device scenario sampling (rand(rng, sto), smps_sto.jl:117-149).
 * set_distributions: one distribution per random element (position order): kind[e] =
 *   0 DISCRETE (nsupport[e] (value, probability) pairs, concatenated over elements in
 *   values/probs; sorted by value like DiscreteNonParametric), 1 NORMAL (param0 = mean,
 *   param1 = VARIANCE: Normal(mean, sqrt(variance)), smps_sto.jl:122-125), 2 UNIFORM
 *   (param0 = left, param1 = right).  Reset by twosd_set_random_positions.
 * add_sampled_scenarios: appends N i.i.d. scenarios to epigraph epi (weights NULL = 1.0).
 *   Element e of scenario number first_index + s is drawn from Philox4x32-10(counter =
 *   (index, e), key = seed), so a stream is reproducible under any sharding.
 * get_scenarios: element values (template + stored delta) of scenarios [first, first+count).
 */
int twosd_set_distributions(twosd_ctx *ctx, int k, const int *kind, const int *nsupport, const double *values,
                            const double *probs, const double *param0, const double *param1);
int twosd_add_sampled_scenarios(twosd_ctx *ctx, int epi, int N, uint64_t seed, uint64_t first_index,
                                const double *weights);
int twosd_get_scenarios(twosd_ctx *ctx, int epi, int first, int count, double *values);

/* evaluate(sp1, sp2, sto, x; N) (smps_routines.jl:67-82), stage-2 part, on device-drawn
 * scenarios [first, first+count) of the stream `seed` (a shard of N_total):
 * *s2 = sum in index order of (1/N_total) * obj.  The caller adds c'x (and, across ranks,
 * the shards' s2 in rank order).  TWOSD_E_LP if any LP is not optimal. */
int twosd_evaluate_sampled(twosd_ctx *ctx, const double *x, int64_t N_total, int64_t first, int64_t count,
                           uint64_t seed, double *s2);

/*
 * solve_problem! (smps_routines.jl:50-62) for scenarios [first, first+count) of epigraph
 * `epi` at first-stage x[n1].  obj[count], status[count] required; pi[count*m2] and
 * y[count*n2] nullable.  Returns TWOSD_E_LP if any status != OPTIMAL (outputs still set).
 */
int twosd_solve_batch(twosd_ctx *ctx, int epi, const double *x, int first, int count,
                      double *obj, double *pi, double *y, int *status);

/* Same for scenarios given by value (evaluate(), smps_routines.jl:67-82): values[N*k]. */
int twosd_solve_values(twosd_ctx *ctx, const double *x, int N, const double *values,
                       double *obj, double *pi, double *y, int *status);

/*
 * push!(::sdDualVertexSet, pi) batched (dual_set.jl:84-94): pis[count*m2] are pushed in
 * order; out_index[count] (nullable) receives the 0-based vertex index each one maps to;
 * *new_size the set size afterwards.  Exact reference dedup semantics: 16-significant-bit
 * L1 hash + component-wise 16-bit rounding compare, first occurrence kept.
 */
int twosd_dvs_push(twosd_ctx *ctx, int count, const double *pis, int *out_index, int *new_size);
int twosd_dvs_size(twosd_ctx *ctx, int *size);
int twosd_dvs_get(twosd_ctx *ctx, int first, int count, double *out /* count*m2 */);
int twosd_dvs_clear(twosd_ctx *ctx);
/* Truncate the set to its first `size` vertices (rollback of a speculative push). */
int twosd_dvs_truncate(twosd_ctx *ctx, int size);
/* Order-dependent 64-bit digest of the set (size and the per-vertex dedup fingerprints in
 * insertion order).  No reference counterpart: ranks compare it so that a cut all-reduce
 * over vertex indices only runs on identical ordered sets (the reference is single-process,
 * cell.jl:25 shares one set). */
int twosd_dvs_fingerprint(twosd_ctx *ctx, uint64_t *digest);

/*
 * sd_iteration! hot segment for one epigraph (algorithm.jl:45-55): solve scenarios
 * [first, first+count) at x and push their duals into the vertex set on the device
 * (no host round trip).  obj/status nullable.
 */
int twosd_solve_push(twosd_ctx *ctx, int epi, const double *x, int first, int count,
                     double *obj, int *status, int *new_size);
/* Scenarios whose dual the last twosd_solve_push recovered and pushed: the first scenario of
 * each distinct optimal dual vertex of the batch (every later scenario at a vertex pushes an
 * equal vector, a no-op of push!, dual_set.jl:84-94); `count` with TWOSD_PUSH_ALL=1. */
int twosd_last_push_reps(twosd_ctx *ctx, int *reps);
/* How the last twosd_solve_push obtained the representatives' duals: 0 = re-solved with dual
 * recovery after the keyed main pass; 1 = recovered for every scenario in the main pass and
 * gathered (chosen when the previous keyed push re-solved more than a quarter of its batch;
 * TWOSD_PUSH_MODE=1 / 2 forces one or the other).  The pushed rows are the same either way. */
int twosd_last_push_mode(twosd_ctx *ctx, int *full);

/*
 * build_sasa_cut (epigraph.jl:125-146) incl. argmax_procedure (subprob.jl:141-169) over
 * every scenario of epigraph `epi` and the current vertex set, at x:
 *   alpha, beta[n1], weight_mark (= total scenario weight); max_val[N], max_arg[N]
 *   (0-based vertex index) nullable.  Ties: lowest vertex index among scores within
 *   tie_rel*(1+|max|) of the maximum (tie_rel = 0 -> strict '>' as the reference).
 */
int twosd_build_cut(twosd_ctx *ctx, int epi, const double *x, double tie_rel,
                    double *alpha, double *beta, double *weight_mark,
                    double *max_val, int *max_arg);

/*
 * Counters of the last twosd_build_cut / twosd_cut_partial (diagnostics, synchronous read):
 * out[0] scenarios re-decided in the restatement's arithmetic (several vertices within the
 * MFMA scores' error band of the maximum), out[1] candidate vertices scored for them, out[2]
 * scenarios re-scanned over every vertex (a candidate log overflowed), out[3] vertices left out
 * of the argmax as dominated twins (a lower vertex with a bit-identical PK row and an equal base
 * at this x: never the pick under either tie rule).  out has 4 entries.
 */
int twosd_cut_stats(twosd_ctx *ctx, int64_t *out);

/*
 * The MFMA pass the last twosd_build_cut / twosd_cut_partial ran (diagnostics, synchronous read):
 * *fp32 = 1 the fp32 pass (v_mfma_f32_16x16x4f32, decisions within its wider error band), 0 the
 * fp64 pass (TWOSD_CUT_F32=0, or operands outside the fp32 envelope); *band = that pass's
 * decision band.  Either pass gives the restatement's picks (cut_fixup_kernel re-decides every
 * row with several vertices in the band).
 */
int twosd_cut_pass(twosd_ctx *ctx, int *fp32, double *band);

/*
 * Multi-GPU split of twosd_build_cut: each rank computes partial sums over its own
 * scenarios into a caller-provided DEVICE buffer (layout in twosd_cut_partial_len),
 * the caller all-reduces it (sum; e.g. torch.distributed / RCCL), then finalize.
 * The partial holds the vertex weight histogram as uint64 fixed point (exact, order
 * independent) followed by fp64 sums.  total_weight is the global total scenario weight.
 */
int twosd_cut_partial_len(twosd_ctx *ctx, int64_t *n_u64, int64_t *n_f64);
int twosd_cut_partial(twosd_ctx *ctx, int epi, const double *x, double tie_rel, double total_weight,
                      uint64_t *d_hist_u64, double *d_sums_f64, double *max_val, int *max_arg);
int twosd_cut_finalize(twosd_ctx *ctx, const double *x, const uint64_t *d_hist_u64, const double *d_sums_f64,
                       double *alpha, double *beta);

/* Timing of the last kernel phases on the context's stream (HIP events), microseconds:
 * [0] LP kernel, [1] dedup push, [2] argmax+cut partial, [3] cut finalize,
 * [4] warm-start pool selection of the last LP batch (0 without a pool). */
int twosd_last_timings(twosd_ctx *ctx, double *us5);

/* Statistics of the last LP batch: sum of simplex pivots, max pivots. */
int twosd_last_lp_stats(twosd_ctx *ctx, int64_t *pivots_sum, int *pivots_max);
/* Eta-file entries the last LP batch wrote to the per-wavefront eta arena (12 bytes each: row index
 * and value), summed over its scenarios: the algorithmic share of the LP kernel's HBM writes.
 * *retries (nullable): its scenarios whose pool start ended non-optimal (iteration cap, numerics)
 * and were solved again from the primary basis. */
int twosd_last_lp_eta_entries(twosd_ctx *ctx, int64_t *entries, int64_t *retries);

/* Incumbent objective of the last twosd_solve_batch / twosd_solve_push / twosd_solve_values
 * batch: *weighted_sum = sum_s w_s obj_s and *weight_sum = sum_s w_s over its scenarios (the
 * epigraph's add_scenario! weights; 1.0 for solve_values), reduced in a fixed order (the same
 * bits on every run).  weighted_sum / weight_sum is the sample-average recourse at x that
 * evaluate (smps_routines.jl:67-82) and the incumbent estimate of sd_iteration! form; across
 * ranks the caller adds the ranks' sums (north star: the all-reduce of the incumbent objective). */
int twosd_last_objective(twosd_ctx *ctx, double *weighted_sum, double *weight_sum);

/* Diagnostic: pivots and status of every scenario of the last LP launch (by scenario index;
 * after a pool refresh: its training solves). */
int twosd_last_lp_iters(twosd_ctx *ctx, int N, int *iters, int *status);

/* Pivot cap of the training solves of a pool refresh: > 0 explicit, 0 auto (default: 3 x the
 * mean pivots of the last batch of >= 4096 scenarios, at least 32; none before such a batch),
 * < 0 none (the kernel's kmax).  A training scenario that needs more pivots drops out of the
 * basis count instead of holding the launch: one wavefront per scenario, so a launch lasts as
 * long as its slowest scenario. */
int twosd_set_refresh_kcap(twosd_ctx *ctx, int kcap);

/* Executed fp64 row operations of the last LP batch: each is one fused multiply-add over
 * a padded basis row of *row_width (= 64 * ceil(m2/64)) doubles, i.e. 2 * row_width flops
 * (used for the counted-FLOP roofline of the LP kernel). */
int twosd_last_lp_ops(twosd_ctx *ctx, int64_t *row_ops, int *row_width);

/* Diagnostic: per-phase cycle totals of the hypersparse LP kernel, summed over waves
 * (non-zero only in the TWOSD_STAMPS build libtwosd_hip_stamps.so).  reset != 0 clears. */
int twosd_debug_stamps(twosd_ctx *ctx, uint64_t *out10, int reset);

#ifdef __cplusplus
}
#endif
#endif /* TWOSD_HIP_H */
