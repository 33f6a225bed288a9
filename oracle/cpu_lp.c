/*
 * cpu_lp.c -- CPU oracle + timed CPU baseline ("port") for the TwoSD hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): linked only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product.
 *
 * What it restates (reference yhz0/SQLP @ 2025-02-19):
 *   - solve_problem!  src/smps/smps_routines.jl:50-62: min q'y s.t. W y (G/L/E) b, y>=0,
 *     b = r_w - T x; returns obj, y and the row duals pi in JuMP's MIN convention
 *     (pi = d obj / d b).  The reference delegates to GLPK's simplex on a warm basis;
 *     this is a bounded dual simplex warm-started from a shared optimal basis B0 with
 *     product-form (eta) updates of B0^{-1}.  RHS-only randomness keeps B0 dual
 *     feasible for every scenario and every x.
 *   - argmax_procedure  src/sd_algorithm/subprob.jl:141-169 (MIN_SENSE, strict '>'
 *     first max, plus the documented near-tie rule when tie_rel > 0)
 *   - build_sasa_cut    src/sd_algorithm/epigraph.jl:125-146 (reference loop order)
 *
 * The pivot rules (dual Devex leaving row, Harris two-pass ratio test, lowest index on
 * ties, tolerances) are the same as the HIP kernel's so the two pick the same vertex on
 * degenerate LPs; optimality of every result is checked independently in tests.
 *
 * Variables: j < n structural y_j in [0, inf); j = n+i slack s_i of row i,
 *   W_i y + s_i = b_i with s_i in (-inf,0] (G), [0,inf) (L), [0,0] (E).
 * Every nonbasic variable sits at 0, so x_B = B^{-1} b.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { ST_OPTIMAL = 0, ST_INFEASIBLE = 1, ST_ITER_LIMIT = 2, ST_NUMERIC = 3 };

#define TOL_P 1e-9     /* primal feasibility (scaled by 1+|bound|)  */
#define TOL_D 1e-9     /* dual feasibility                          */
#define TOL_PIV 1e-9   /* smallest admissible |alpha_rj|            */
#define PI_ZERO 1e-12  /* |pi_i| below this * (1+max|pi|) snapped to 0 */

typedef struct {
    int m, n;
    const int *colptr, *rowidx;   /* W CSC, 0-based, n+1 / nnz            */
    const double *val;
    const double *q;              /* n                                    */
    const signed char *sense;     /* m: 'G','L','E'                       */
} lp_t;

static inline double var_lb(const lp_t *L, int j) {
    if (j < L->n) return 0.0;
    return L->sense[j - L->n] == 'G' ? -INFINITY : 0.0;
}
static inline double var_ub(const lp_t *L, int j) {
    if (j < L->n) return INFINITY;
    return L->sense[j - L->n] == 'L' ? INFINITY : 0.0;
}
static inline double var_cost(const lp_t *L, int j) { return j < L->n ? L->q[j] : 0.0; }

/* alpha = rho' a_j */
static inline double col_dot(const lp_t *L, int j, const double *rho) {
    if (j >= L->n) return rho[j - L->n];
    double s = 0.0;
    for (int p = L->colptr[j]; p < L->colptr[j + 1]; ++p) s += rho[L->rowidx[p]] * L->val[p];
    return s;
}

/* ---------- dense LU inverse (partial pivoting) ---------- */
int oracle_dense_inverse(int m, const double *A /* row-major m*m */, double *Ainv) {
    double *M = (double *)malloc(sizeof(double) * (size_t)m * m);
    int *perm = (int *)malloc(sizeof(int) * m);
    memcpy(M, A, sizeof(double) * (size_t)m * m);
    for (int i = 0; i < m; ++i) perm[i] = i;
    int rc = 0;
    for (int k = 0; k < m; ++k) {
        int p = k; double best = fabs(M[(size_t)k * m + k]);
        for (int i = k + 1; i < m; ++i) { double v = fabs(M[(size_t)i * m + k]); if (v > best) { best = v; p = i; } }
        if (best < 1e-14) { rc = -1; break; }
        if (p != k) {
            for (int j = 0; j < m; ++j) { double t = M[(size_t)k * m + j]; M[(size_t)k * m + j] = M[(size_t)p * m + j]; M[(size_t)p * m + j] = t; }
            int t = perm[k]; perm[k] = perm[p]; perm[p] = t;
        }
        double piv = M[(size_t)k * m + k];
        for (int i = k + 1; i < m; ++i) {
            double f = M[(size_t)i * m + k] / piv;
            if (f == 0.0) continue;
            M[(size_t)i * m + k] = f;
            double *ri = M + (size_t)i * m, *rk = M + (size_t)k * m;
            for (int j = k + 1; j < m; ++j) ri[j] -= f * rk[j];
        }
    }
    if (rc == 0) {
        /* solve A X = I column by column: P A = L U */
        double *col = (double *)malloc(sizeof(double) * m);
        for (int c = 0; c < m; ++c) {
            for (int i = 0; i < m; ++i) col[i] = (perm[i] == c) ? 1.0 : 0.0;
            for (int i = 0; i < m; ++i) { double s = col[i]; const double *ri = M + (size_t)i * m; for (int j = 0; j < i; ++j) s -= ri[j] * col[j]; col[i] = s; }
            for (int i = m - 1; i >= 0; --i) { double s = col[i]; const double *ri = M + (size_t)i * m; for (int j = i + 1; j < m; ++j) s -= ri[j] * col[j]; col[i] = s / ri[i]; }
            for (int i = 0; i < m; ++i) Ainv[(size_t)i * m + c] = col[i];
        }
        free(col);
    }
    free(M); free(perm);
    return rc;
}

/* basis matrix B (row-major) from head */
static void build_basis(const lp_t *L, const int *head, double *B) {
    int m = L->m;
    memset(B, 0, sizeof(double) * (size_t)m * m);
    for (int c = 0; c < m; ++c) {
        int j = head[c];
        if (j >= L->n) B[(size_t)(j - L->n) * m + c] = 1.0;
        else for (int p = L->colptr[j]; p < L->colptr[j + 1]; ++p) B[(size_t)L->rowidx[p] * m + c] = L->val[p];
    }
}

/* ---------- per-scenario workspace ---------- */
typedef struct {
    double *xB, *pi, *rho, *u, *aq, *w, *eta; int *etap; int *head; unsigned char *isbasic;
    int kmax;
} ws_t;

static void ws_alloc(ws_t *W, int m, int n, int kmax) {
    W->xB = (double *)malloc(sizeof(double) * m);
    W->pi = (double *)malloc(sizeof(double) * m);
    W->rho = (double *)malloc(sizeof(double) * m);
    W->u = (double *)malloc(sizeof(double) * m);
    W->aq = (double *)malloc(sizeof(double) * m);
    W->w = (double *)malloc(sizeof(double) * m);
    W->eta = (double *)malloc(sizeof(double) * (size_t)m * (kmax > 0 ? kmax : 1));
    W->etap = (int *)malloc(sizeof(int) * (kmax > 0 ? kmax : 1));
    W->head = (int *)malloc(sizeof(int) * m);
    W->isbasic = (unsigned char *)malloc(n + m);
    W->kmax = kmax;
}
static void ws_free(ws_t *W) {
    free(W->xB); free(W->pi); free(W->rho); free(W->u); free(W->aq); free(W->w);
    free(W->eta); free(W->etap); free(W->head); free(W->isbasic);
}

/* B^{-1} v in place: v <- E_K..E_1 (B0inv v) ; B0invT is column-major (= B0inv^T row-major) */
static void ftran_dense(int m, const double *B0inv, const ws_t *W, int K, const double *v_in, double *v_out) {
    for (int i = 0; i < m; ++i) { const double *ri = B0inv + (size_t)i * m; double s = 0; for (int j = 0; j < m; ++j) s += ri[j] * v_in[j]; v_out[i] = s; }
    for (int t = 0; t < K; ++t) {
        const double *e = W->eta + (size_t)t * m; int p = W->etap[t]; double vp = v_out[p];
        if (vp == 0.0) continue;
        for (int i = 0; i < m; ++i) v_out[i] += e[i] * vp;
        v_out[p] = e[p] * vp;
    }
}

/* FTRAN of a column a_j of [W I] */
static void ftran_col(const lp_t *L, const double *B0invT, const ws_t *W, int K, int j, double *out) {
    int m = L->m;
    if (j >= L->n) { memcpy(out, B0invT + (size_t)(j - L->n) * m, sizeof(double) * m); }
    else {
        memset(out, 0, sizeof(double) * m);
        for (int p = L->colptr[j]; p < L->colptr[j + 1]; ++p) {
            const double *c = B0invT + (size_t)L->rowidx[p] * m; double a = L->val[p];
            for (int i = 0; i < m; ++i) out[i] += a * c[i];
        }
    }
    for (int t = 0; t < K; ++t) {
        const double *e = W->eta + (size_t)t * m; int p = W->etap[t]; double vp = out[p];
        if (vp == 0.0) continue;
        for (int i = 0; i < m; ++i) out[i] += e[i] * vp;
        out[p] = e[p] * vp;
    }
}

/* row r of B^{-1}: u = e_r' E_K .. E_1 (dense u), rho = u' B0inv */
static void btran_row(int m, const double *B0inv, ws_t *W, int K, int r) {
    double *u = W->u; memset(u, 0, sizeof(double) * m); u[r] = 1.0;
    for (int t = K - 1; t >= 0; --t) {
        const double *e = W->eta + (size_t)t * m; double s = 0;
        for (int i = 0; i < m; ++i) s += u[i] * e[i];
        u[W->etap[t]] = s;
    }
    double *rho = W->rho; memset(rho, 0, sizeof(double) * m);
    for (int i = 0; i < m; ++i) {
        double ui = u[i]; if (ui == 0.0) continue;
        const double *ri = B0inv + (size_t)i * m;
        for (int j = 0; j < m; ++j) rho[j] += ui * ri[j];
    }
}

/* y' B^{-1} for a dense y (used for the final pi = c_B' B^{-1}) */
static void btran_dense(int m, const double *B0inv, ws_t *W, int K, const double *y, double *out) {
    double *u = W->u; memcpy(u, y, sizeof(double) * m);
    for (int t = K - 1; t >= 0; --t) {
        const double *e = W->eta + (size_t)t * m; double s = 0;
        for (int i = 0; i < m; ++i) s += u[i] * e[i];
        u[W->etap[t]] = s;
    }
    memset(out, 0, sizeof(double) * m);
    for (int i = 0; i < m; ++i) {
        double ui = u[i]; if (ui == 0.0) continue;
        const double *ri = B0inv + (size_t)i * m;
        for (int j = 0; j < m; ++j) out[j] += ui * ri[j];
    }
}

/*
 * One dual-simplex solve from basis (head0, B0inv) for rhs b.
 * pi0 = c_B0' B0inv.  w0 = initial dual pricing weights (NULL -> 1).
 * Outputs obj, pi[m], y[n] (nullable), iters.  Returns status.
 */
static int solve_one(const lp_t *L, const int *head0, const double *B0inv, const double *B0invT,
                     const double *pi0, const double *b, ws_t *W, int max_iter,
                     double *obj_out, double *pi_out, double *y_out, int *iters_out, int *head_out) {
    const int m = L->m, n = L->n;
    memcpy(W->head, head0, sizeof(int) * m);
    memset(W->isbasic, 0, n + m);
    for (int i = 0; i < m; ++i) W->isbasic[head0[i]] = 1;
    for (int i = 0; i < m; ++i) { const double *ri = B0inv + (size_t)i * m; double s = 0; for (int j = 0; j < m; ++j) s += ri[j] * b[j]; W->xB[i] = s; }
    memcpy(W->pi, pi0, sizeof(double) * m);
    for (int i = 0; i < m; ++i) W->w[i] = 1.0;
    int K = 0, it = 0, status = ST_OPTIMAL;
    for (;;) {
        /* 1. leaving row: max infeas^2 / w, lowest index on ties */
        int r = -1; double best = 0.0, delta = 0.0;
        for (int i = 0; i < m; ++i) {
            int j = W->head[i]; double x = W->xB[i], lb = var_lb(L, j), ub = var_ub(L, j), d = 0.0;
            if (x < lb - TOL_P * (1.0 + fabs(lb))) d = x - lb;
            else if (x > ub + TOL_P * (1.0 + fabs(ub))) d = x - ub;
            else continue;
            double sc = d * d / W->w[i];
            if (sc > best) { best = sc; r = i; delta = d; }
        }
        if (r < 0) break;
        if (it >= max_iter || K >= W->kmax) { status = ST_ITER_LIMIT; break; }
        /* 2. BTRAN */
        btran_row(m, B0inv, W, K, r);
        const double s = delta > 0 ? 1.0 : -1.0;   /* x_r above ub: decrease it */
        /* 3. Harris ratio test, pass 1 */
        double theta_max = INFINITY;
        for (int j = 0; j < n + m; ++j) {
            if (W->isbasic[j]) continue;
            if (j >= n && L->sense[j - n] == 'E') continue;   /* fixed */
            double a = s * col_dot(L, j, W->rho);
            int atlb = (j < n) || (L->sense[j - n] == 'L');
            if (atlb ? (a > TOL_PIV) : (a < -TOL_PIV)) {
                double d = var_cost(L, j) - col_dot(L, j, W->pi);
                double ratio = atlb ? (d + TOL_D) / a : (d - TOL_D) / a;
                if (ratio < theta_max) theta_max = ratio;
            }
        }
        if (theta_max == INFINITY) { status = ST_INFEASIBLE; break; }
        /* pass 2: largest |alpha| with ratio <= theta_max */
        int q = -1; double amax = 0.0, dq = 0.0, aq_s = 0.0;
        for (int j = 0; j < n + m; ++j) {
            if (W->isbasic[j]) continue;
            if (j >= n && L->sense[j - n] == 'E') continue;
            double a = s * col_dot(L, j, W->rho);
            int atlb = (j < n) || (L->sense[j - n] == 'L');
            if (atlb ? (a > TOL_PIV) : (a < -TOL_PIV)) {
                double d = var_cost(L, j) - col_dot(L, j, W->pi);
                /* d / a <= theta_max as a product (a != 0, sign known): the kernel's form */
                if ((a > 0.0 ? d <= theta_max * a : d >= theta_max * a) && fabs(a) > amax) { amax = fabs(a); q = j; dq = d; aq_s = a; }
            }
        }
        if (q < 0) { status = ST_NUMERIC; break; }
        double thetaD = dq / aq_s;
        /* 4. FTRAN entering column */
        ftran_col(L, B0invT, W, K, q, W->aq);
        double arq = W->aq[r];
        if (fabs(arq) < 1e-12) { status = ST_NUMERIC; break; }
        /* 5. updates */
        for (int i = 0; i < m; ++i) W->pi[i] += s * thetaD * W->rho[i];
        double thetaP = delta / arq;
        for (int i = 0; i < m; ++i) W->xB[i] -= thetaP * W->aq[i];
        W->xB[r] = thetaP;
        /* dual Devex weights */
        double wr = W->w[r];
        for (int i = 0; i < m; ++i) {
            if (i == r) continue;
            double ratio = W->aq[i] / arq, cand = ratio * ratio * wr;
            if (cand > W->w[i]) W->w[i] = cand;
        }
        { double t = wr / (arq * arq); W->w[r] = t > 1.0 ? t : 1.0; }
        /* eta */
        double *e = W->eta + (size_t)K * m;
        for (int i = 0; i < m; ++i) e[i] = -W->aq[i] / arq;
        e[r] = 1.0 / arq;
        W->etap[K] = r; ++K;
        W->isbasic[W->head[r]] = 0; W->isbasic[q] = 1; W->head[r] = q;
        ++it;
    }
    *iters_out = it;
    if (head_out) memcpy(head_out, W->head, sizeof(int) * m);
    if (status != ST_OPTIMAL) { *obj_out = NAN; return status; }
    /* vertex recovery: pi = c_B' B^{-1} fresh, snap tiny components */
    double *cB = W->aq;
    for (int i = 0; i < m; ++i) cB[i] = var_cost(L, W->head[i]);
    btran_dense(m, B0inv, W, K, cB, pi_out);
    double pmax = 0; for (int i = 0; i < m; ++i) if (fabs(pi_out[i]) > pmax) pmax = fabs(pi_out[i]);
    for (int i = 0; i < m; ++i) if (fabs(pi_out[i]) <= PI_ZERO * (1.0 + pmax)) pi_out[i] = 0.0;
    /* primal y from the updated x_B; obj = q'y */
    double obj = 0.0;
    if (y_out) memset(y_out, 0, sizeof(double) * n);
    for (int i = 0; i < m; ++i) {
        int j = W->head[i];
        if (j < n) { if (y_out) y_out[j] = W->xB[i]; obj += L->q[j] * W->xB[i]; }
    }
    *obj_out = obj;
    return ST_OPTIMAL;
}

/* ================= exported API (ctypes) ================= */

typedef struct {
    lp_t L;
    int *colptr, *rowidx; double *val, *q; signed char *sense;
    int *head0; double *B0inv, *B0invT, *pi0;
    /* warm-start pool (oracle_lp_set_pool): P bases with dense inverses */
    int P;
    int *pheads; double *pBinv, *pBinvT, *ppi0;
} oracle_ctx;

void *oracle_lp_create(int m, int n, const int *colptr, const int *rowidx, const double *val,
                       const double *q, const signed char *sense) {
    oracle_ctx *C = (oracle_ctx *)calloc(1, sizeof(oracle_ctx));
    int nnz = colptr[n];
    C->colptr = (int *)malloc(sizeof(int) * (n + 1)); memcpy(C->colptr, colptr, sizeof(int) * (n + 1));
    C->rowidx = (int *)malloc(sizeof(int) * (nnz ? nnz : 1)); memcpy(C->rowidx, rowidx, sizeof(int) * nnz);
    C->val = (double *)malloc(sizeof(double) * (nnz ? nnz : 1)); memcpy(C->val, val, sizeof(double) * nnz);
    C->q = (double *)malloc(sizeof(double) * n); memcpy(C->q, q, sizeof(double) * n);
    C->sense = (signed char *)malloc(m); memcpy(C->sense, sense, m);
    C->L.m = m; C->L.n = n; C->L.colptr = C->colptr; C->L.rowidx = C->rowidx; C->L.val = C->val;
    C->L.q = C->q; C->L.sense = C->sense;
    C->head0 = (int *)malloc(sizeof(int) * m);
    C->B0inv = (double *)malloc(sizeof(double) * (size_t)m * m);
    C->B0invT = (double *)malloc(sizeof(double) * (size_t)m * m);
    C->pi0 = (double *)malloc(sizeof(double) * m);
    return C;
}

void oracle_lp_destroy(void *p) {
    oracle_ctx *C = (oracle_ctx *)p; if (!C) return;
    free(C->pheads); free(C->pBinv); free(C->pBinvT); free(C->ppi0);
    free(C->colptr); free(C->rowidx); free(C->val); free(C->q); free(C->sense);
    free(C->head0); free(C->B0inv); free(C->B0invT); free(C->pi0); free(C);
}

/* install basis head0 (m var indices); computes B0inv, pi0.  returns 0 / -1 singular */
int oracle_lp_set_basis(void *p, const int *head0) {
    oracle_ctx *C = (oracle_ctx *)p; int m = C->L.m;
    memcpy(C->head0, head0, sizeof(int) * m);
    double *B = (double *)malloc(sizeof(double) * (size_t)m * m);
    build_basis(&C->L, head0, B);
    int rc = oracle_dense_inverse(m, B, C->B0inv);
    free(B);
    if (rc) return rc;
    for (int i = 0; i < m; ++i) for (int j = 0; j < m; ++j) C->B0invT[(size_t)j * m + i] = C->B0inv[(size_t)i * m + j];
    for (int j = 0; j < m; ++j) { double s = 0; for (int i = 0; i < m; ++i) s += var_cost(&C->L, head0[i]) * C->B0inv[(size_t)i * m + j]; C->pi0[j] = s; }
    return 0;
}

/* max dual infeasibility of the installed basis (>0 means not dual feasible) */
double oracle_lp_basis_dual_infeas(void *p) {
    oracle_ctx *C = (oracle_ctx *)p; const lp_t *L = &C->L; int m = L->m, n = L->n;
    unsigned char *isb = (unsigned char *)calloc(n + m, 1);
    for (int i = 0; i < m; ++i) isb[C->head0[i]] = 1;
    double worst = 0;
    for (int j = 0; j < n + m; ++j) {
        if (isb[j] || (j >= n && L->sense[j - n] == 'E')) continue;
        double d = var_cost(L, j) - col_dot(L, j, C->pi0);
        int atlb = (j < n) || (L->sense[j - n] == 'L');
        double inf = atlb ? -d : d;
        if (inf > worst) worst = inf;
    }
    free(isb);
    return worst;
}

/*
 * Solve from the slack basis with periodic refactorisation (setup / reference solve).
 * Requires q >= 0 (slack basis dual feasible).  Writes the optimal head to head_out.
 */
int oracle_lp_solve_from_slack(void *p, const double *b, int *head_out, double *obj, int *iters) {
    oracle_ctx *C = (oracle_ctx *)p; int m = C->L.m, n = C->L.n;
    int *head = (int *)malloc(sizeof(int) * m);
    for (int i = 0; i < m; ++i) head[i] = n + i;
    ws_t W; ws_alloc(&W, m, n, 100);
    double *pi = (double *)malloc(sizeof(double) * m);
    int total = 0, st = ST_ITER_LIMIT;
    for (int round = 0; round < 200; ++round) {
        if (oracle_lp_set_basis(p, head)) { st = ST_NUMERIC; break; }
        int it = 0;
        st = solve_one(&C->L, C->head0, C->B0inv, C->B0invT, C->pi0, b, &W, 100, obj, pi, NULL, &it, head);
        total += it;
        if (st != ST_ITER_LIMIT) break;
    }
    memcpy(head_out, head, sizeof(int) * m);
    *iters = total;
    free(head); free(pi); ws_free(&W);
    return st;
}

/*
 * Batched per-scenario solve (the timed CPU path): for s in [0,N):
 *   b_s = base + sum_j DR[s,j] e_{rows[j]}   (base = r - T x, RHS-only scenarios)
 * obj[N], pi[N*m] (nullable), y[N*n] (nullable), status[N], iters[N].
 * nthreads <= 0 -> OpenMP default.
 */
int oracle_lp_solve_batch(void *p, int N, int k, const int *rows, const double *base, const double *DR,
                          int kmax, double *obj, double *pi, double *y, int *status, int *iters, int nthreads) {
    oracle_ctx *C = (oracle_ctx *)p; int m = C->L.m, n = C->L.n;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
    {
        ws_t W; ws_alloc(&W, m, n, kmax);
        double *b = (double *)malloc(sizeof(double) * m);
        double *pi_l = (double *)malloc(sizeof(double) * m);
#pragma omp for schedule(dynamic, 4)
        for (int s = 0; s < N; ++s) {
            memcpy(b, base, sizeof(double) * m);
            for (int j = 0; j < k; ++j) b[rows[j]] += DR[(size_t)s * k + j];
            int it = 0;
            status[s] = solve_one(&C->L, C->head0, C->B0inv, C->B0invT, C->pi0, b, &W, 1 << 30, &obj[s],
                                  pi ? pi + (size_t)s * m : pi_l, y ? y + (size_t)s * n : NULL, &it, NULL);
            if (iters) iters[s] = it;
        }
        ws_free(&W); free(b); free(pi_l);
    }
    return 0;
}

/*
 * argmax_procedure + build_sasa_cut in reference loop order for RHS-only scenarios.
 *   base_rhs = r (m), T (m x n1 row-major), x (n1), V (nv x m row-major),
 *   scenario s: dr = DR[s,:] on rows[]; weights w[s].
 * Scores are computed as the reference does: dot(pi, r - T x) + dot(pi, dvec)
 * (subprob.jl:147-155), each dot sequential in row order with every product and sum rounded
 * on its own (built with -ffp-contract=off): base[i] = r[i] - tx[i] with tx[i] = T[i][0] x[0] + T[i][1] x[1] + ...
 * accumulated from zero in column order (`coef.rhs - coef.transfer * x`, subprob.jl:147: SparseArrays'
 * CSC mat-vec adds column by column; a zero entry adds an exact 0);
 * vb[v] = sum_i pi[i] base[i]; t = sum over the random rows in ascending order of
 * pi[row] dvec[row] (the zero rows of the dense dvec add exactly nothing).  This is the
 * arithmetic every tie decision of the build is pinned to (the GPU re-decides rows with
 * several vertices within its error band in exactly this order).  The reference's own
 * OpenBLAS ddot sums in a CPU-dependent blocked order, so its picks at rounding-level ties
 * cannot be pinned by any restatement.
 * tie_rel == 0: strict '>' (first max); > 0: lowest index within tie_rel*(1+|max|).
 */
void oracle_build_cut(int m, int n1, int nv, int N, int k, const int *rows, const double *r, const double *T,
                      const double *x, const double *V, const double *DR, const double *w, double tie_rel,
                      double *alpha, double *beta, double *max_val, int *max_arg, int nthreads) {
    double *base = (double *)malloc(sizeof(double) * m);
    for (int i = 0; i < m; ++i) { double tx = 0.0; for (int j = 0; j < n1; ++j) tx += T[(size_t)i * n1 + j] * x[j]; base[i] = r[i] - tx; }
    double *vb = (double *)malloc(sizeof(double) * (nv ? nv : 1));
    for (int v = 0; v < nv; ++v) { double s = 0; for (int i = 0; i < m; ++i) s += V[(size_t)v * m + i] * base[i]; vb[v] = s; }
    /* elements by ascending row (element order within a row): insertion sort, k is small */
    int *ord = (int *)malloc(sizeof(int) * (k ? k : 1));
    for (int j = 0; j < k; ++j) {
        int q = j;
        while (q > 0 && rows[ord[q - 1]] > rows[j]) { ord[q] = ord[q - 1]; --q; }
        ord[q] = j;
    }
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
    {
        double *sc = (double *)malloc(sizeof(double) * (nv ? nv : 1));
#pragma omp for schedule(static)
        for (int s = 0; s < N; ++s) {
            const double *d = DR + (size_t)s * k;
            double M = -INFINITY; int arg = -1;
            for (int v = 0; v < nv; ++v) {
                const double *pv = V + (size_t)v * m; double t = 0;
                for (int q = 0; q < k; ++q) { const int j = ord[q]; t += pv[rows[j]] * d[j]; }
                sc[v] = vb[v] + t;
                if (sc[v] > M) { M = sc[v]; arg = v; }
            }
            if (tie_rel > 0 && arg >= 0) {
                double tol = tie_rel * (1.0 + fabs(M));
                for (int v = 0; v < arg; ++v) if (sc[v] >= M - tol) { arg = v; break; }
            }
            max_arg[s] = arg; max_val[s] = arg >= 0 ? sc[arg] : -INFINITY;
        }
        free(sc);
    }
    /* cut accumulation in scenario order (epigraph.jl:134-143) */
    double W = 0; for (int s = 0; s < N; ++s) W += w[s];
    double a = 0; for (int j = 0; j < n1; ++j) beta[j] = 0;
    double *g = (double *)malloc(sizeof(double) * m);
    for (int s = 0; s < N; ++s) {
        if (max_arg[s] < 0) continue;
        const double *pv = V + (size_t)max_arg[s] * m; double p = w[s] / W;
        double t = 0; for (int i = 0; i < m; ++i) t += pv[i] * r[i];
        for (int j = 0; j < k; ++j) t += pv[rows[j]] * DR[(size_t)s * k + j];
        a += p * t;
        for (int j = 0; j < n1; ++j) { double c = 0; for (int i = 0; i < m; ++i) c += T[(size_t)i * n1 + j] * pv[i]; beta[j] += -p * c; }
    }
    *alpha = a;
    free(g); free(base); free(vb); free(ord);
}

/* ================= warm-start pool (CPU counterpart of the GPU basis pool) ================= */

/*
 * Install P dual-feasible bases (heads[P*m]) with their dense inverses (setup, OpenMP over
 * the bases).  Returns 0, or -1 - p for the first singular basis p.
 */
int oracle_lp_set_pool(void *p, int P, const int *heads) {
    oracle_ctx *C = (oracle_ctx *)p; const int m = C->L.m;
    free(C->pheads); free(C->pBinv); free(C->pBinvT); free(C->ppi0);
    C->P = P;
    C->pheads = (int *)malloc(sizeof(int) * (size_t)P * m);
    memcpy(C->pheads, heads, sizeof(int) * (size_t)P * m);
    C->pBinv = (double *)malloc(sizeof(double) * (size_t)P * m * m);
    C->pBinvT = (double *)malloc(sizeof(double) * (size_t)P * m * m);
    C->ppi0 = (double *)malloc(sizeof(double) * (size_t)P * m);
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 1)
    for (int q = 0; q < P; ++q) {
        const int *h = C->pheads + (size_t)q * m;
        double *B = (double *)malloc(sizeof(double) * (size_t)m * m);
        double *Bi = C->pBinv + (size_t)q * m * m, *BiT = C->pBinvT + (size_t)q * m * m;
        build_basis(&C->L, h, B);
        if (oracle_dense_inverse(m, B, Bi)) {
#pragma omp critical
            if (!bad) bad = -1 - q;
        } else {
            for (int i = 0; i < m; ++i) for (int j = 0; j < m; ++j) BiT[(size_t)j * m + i] = Bi[(size_t)i * m + j];
            for (int j = 0; j < m; ++j) {
                double sum = 0; for (int i = 0; i < m; ++i) sum += var_cost(&C->L, h[i]) * Bi[(size_t)i * m + j];
                C->ppi0[(size_t)q * m + j] = sum;
            }
        }
        free(B);
    }
    return bad;
}

/*
 * Batched solve with a per-scenario warm start from the pool: the basis with the least total
 * primal infeasibility sum_i |infeas(x_B,i)| at b_s (lowest p on ties) -- the selection key of
 * the GPU's level-1 pool selection -- then the same dual simplex as oracle_lp_solve_batch.
 * x_B of basis p at b_s = B_p^{-1} base + sum_j B_p^{-1}[:, rows_j] DR[s,j]; the second term
 * runs over the nonzeros of B_p^{-1}[:, rows] (setup per call, like the GPU's per-x data).
 * picks[N] (nullable): the chosen pool basis.
 */
int oracle_lp_solve_batch_pool(void *p, int N, int k, const int *rows, const double *base, const double *DR,
                               int kmax, double *obj, double *pi, int *status, int *iters, int *picks, int nthreads) {
    oracle_ctx *C = (oracle_ctx *)p; const int m = C->L.m, n = C->L.n, P = C->P;
    if (P <= 0) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    double *xb = (double *)malloc(sizeof(double) * (size_t)P * m);
    int *kp = (int *)malloc(sizeof(int) * ((size_t)P * m + 1));
    int *kc = NULL; double *kv = NULL; size_t cap = 0, nz = 0;
    for (int q = 0; q < P; ++q) {   /* x-dependent part and the element columns as per-row lists */
        const double *Bi = C->pBinv + (size_t)q * m * m;
        for (int i = 0; i < m; ++i) {
            double sum = 0; for (int j = 0; j < m; ++j) sum += Bi[(size_t)i * m + j] * base[j];
            xb[(size_t)q * m + i] = sum;
            kp[(size_t)q * m + i] = (int)nz;
            for (int e = 0; e < k; ++e) {
                const double v = Bi[(size_t)i * m + rows[e]];
                if (v == 0.0) continue;
                if (nz == cap) { cap = cap ? 2 * cap : 4096; kc = (int *)realloc(kc, sizeof(int) * cap); kv = (double *)realloc(kv, sizeof(double) * cap); }
                kc[nz] = e; kv[nz] = v; ++nz;
            }
        }
    }
    kp[(size_t)P * m] = (int)nz;
#pragma omp parallel
    {
        ws_t W; ws_alloc(&W, m, n, kmax);
        double *b = (double *)malloc(sizeof(double) * m);
        double *pi_l = (double *)malloc(sizeof(double) * m);
#pragma omp for schedule(dynamic, 4)
        for (int s = 0; s < N; ++s) {
            const double *dr = DR + (size_t)s * k;
            int best_p = 0; double best = INFINITY;
            for (int q = 0; q < P; ++q) {
                const int *h = C->pheads + (size_t)q * m;
                double inf = 0.0;
                for (int i = 0; i < m && inf < best; ++i) {
                    double x = xb[(size_t)q * m + i];
                    for (int t = kp[(size_t)q * m + i]; t < kp[(size_t)q * m + i + 1]; ++t) x += kv[t] * dr[kc[t]];
                    const int j = h[i]; const double lb = var_lb(&C->L, j), ub = var_ub(&C->L, j);
                    if (x < lb - TOL_P * (1.0 + fabs(lb))) inf += lb - x;
                    else if (x > ub + TOL_P * (1.0 + fabs(ub))) inf += x - ub;
                }
                if (inf < best) { best = inf; best_p = q; }
            }
            memcpy(b, base, sizeof(double) * m);
            for (int j = 0; j < k; ++j) b[rows[j]] += dr[j];
            int it = 0;
            status[s] = solve_one(&C->L, C->pheads + (size_t)best_p * m, C->pBinv + (size_t)best_p * m * m,
                                  C->pBinvT + (size_t)best_p * m * m, C->ppi0 + (size_t)best_p * m, b, &W, 1 << 30,
                                  &obj[s], pi ? pi + (size_t)s * m : pi_l, NULL, &it, NULL);
            if (iters) iters[s] = it;
            if (picks) picks[s] = best_p;
        }
        ws_free(&W); free(b); free(pi_l);
    }
    free(xb); free(kp); free(kc); free(kv);
    return 0;
}
