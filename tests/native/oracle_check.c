/* oracle_check.c -- sanitizer driver for the oracle's C restatement (oracle/cpu_lp.c,
 * oracle/sampler.c; test infrastructure): built with -fsanitize=address,undefined by
 * tests/test_native_sanitize.py and run on the same LP files as host_check.
 * Per file: solve from the slack basis, install that basis, a batch of RHS-perturbed solves
 * (primary warm start and a two-basis pool), a reference-order cut over their duals; plus the
 * Random123 Philox4x32-10 known answer. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void *oracle_lp_create(int m, int n, const int *colptr, const int *rowidx, const double *val, const double *q,
                       const signed char *sense);
void oracle_lp_destroy(void *p);
int oracle_lp_set_basis(void *p, const int *head0);
int oracle_lp_solve_from_slack(void *p, const double *b, int *head_out, double *obj, int *iters);
int oracle_lp_solve_batch(void *p, int N, int k, const int *rows, const double *base, const double *DR, int kmax,
                          double *obj, double *pi, double *y, int *status, int *iters, int nthreads);
int oracle_lp_set_pool(void *p, int P, const int *heads);
int oracle_lp_solve_batch_pool(void *p, int N, int k, const int *rows, const double *base, const double *DR, int kmax,
                               double *obj, double *pi, int *status, int *iters, int *picks, int nthreads);
void oracle_build_cut(int m, int n1, int nv, int N, int k, const int *rows, const double *r, const double *T,
                      const double *x, const double *V, const double *DR, const double *w, double tie_rel, double *alpha,
                      double *beta, double *max_val, int *max_arg, int nthreads);
void oracle_philox4x32_10(const uint32_t *ctr, const uint32_t *key, uint32_t *out);

static int check(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return 1;
    int mn[2];
    if (fread(mn, sizeof(int), 2, f) != 2) { fclose(f); return 1; }
    const int m = mn[0], n = mn[1];
    int *colptr = malloc(sizeof(int) * (n + 1));
    if (fread(colptr, sizeof(int), n + 1, f) != (size_t)n + 1) { fclose(f); return 1; }
    const int nnz = colptr[n];
    int *rowidx = malloc(sizeof(int) * (nnz ? nnz : 1));
    double *val = malloc(sizeof(double) * (nnz ? nnz : 1)), *q = malloc(sizeof(double) * n), *b = malloc(sizeof(double) * m);
    signed char *sense = malloc(m);
    double expected = 0;
    int ok = fread(rowidx, sizeof(int), nnz, f) == (size_t)nnz && fread(val, sizeof(double), nnz, f) == (size_t)nnz &&
             fread(q, sizeof(double), n, f) == (size_t)n && fread(sense, 1, m, f) == (size_t)m &&
             fread(b, sizeof(double), m, f) == (size_t)m && fread(&expected, sizeof(double), 1, f) == 1;
    fclose(f);
    int bad = !ok;
    void *lp = ok ? oracle_lp_create(m, n, colptr, rowidx, val, q, sense) : NULL;
    int *head = malloc(sizeof(int) * m);
    double obj = 0;
    int it = 0;
    if (lp && (oracle_lp_solve_from_slack(lp, b, head, &obj, &it) != 0 || fabs(obj - expected) > 1e-9 * (1 + fabs(expected)))) {
        fprintf(stderr, "%s: oracle slack solve %.17g vs %.17g\n", path, obj, expected);
        bad = 1;
    }
    if (lp && !bad && oracle_lp_set_basis(lp, head) != 0) bad = 1;
    const int N = 64, k = m < 3 ? m : 3;
    int rows[3] = {0, m / 2, m - 1};
    double *DR = calloc((size_t)N * k, sizeof(double)), *o = malloc(sizeof(double) * N), *o2 = malloc(sizeof(double) * N);
    double *pi = malloc(sizeof(double) * (size_t)N * m), *pi2 = malloc(sizeof(double) * (size_t)N * m);
    int *st = malloc(sizeof(int) * N), *st2 = malloc(sizeof(int) * N), *its = malloc(sizeof(int) * N), *picks = malloc(sizeof(int) * N);
    srand(7);
    for (int s = 0; s < N * k; ++s) DR[s] = 0.05 * ((double)rand() / RAND_MAX - 0.5) * (1 + fabs(b[rows[s % k]]));
    if (!bad) {
        oracle_lp_solve_batch(lp, N, k, rows, b, DR, 512, o, pi, NULL, st, its, 2);
        int *heads = malloc(sizeof(int) * 2 * m);
        memcpy(heads, head, sizeof(int) * m);
        memcpy(heads + m, head, sizeof(int) * m);
        if (oracle_lp_set_pool(lp, 2, heads) != 0) bad = 1;
        else oracle_lp_solve_batch_pool(lp, N, k, rows, b, DR, 512, o2, pi2, st2, its, picks, 2);
        free(heads);
        int nopt = 0;
        for (int s = 0; s < N; ++s)
            if (st[s] == 0 && st2[s] == 0) {
                ++nopt;
                if (fabs(o[s] - o2[s]) > 1e-9 * (1 + fabs(o[s]))) bad = 1;
            }
        /* cut over the first duals as V (T = 0, n1 = 1) */
        double r0 = 0, T0 = 0, x0 = 0, alpha = 0, beta = 0, *w = malloc(sizeof(double) * N), *mv = malloc(sizeof(double) * N);
        int *ma = malloc(sizeof(int) * N);
        double *rr = malloc(sizeof(double) * m), *TT = calloc(m, sizeof(double));
        for (int i = 0; i < m; ++i) rr[i] = b[i];
        for (int s = 0; s < N; ++s) w[s] = 1.0;
        int nv = 0;
        for (int s = 0; s < N && nv < 8; ++s)
            if (st[s] == 0) memmove(pi + (size_t)nv++ * m, pi + (size_t)s * m, sizeof(double) * m);
        if (nv > 0) oracle_build_cut(m, 1, nv, N, k, rows, rr, TT, &x0, pi, DR, w, 0.0, &alpha, &beta, mv, ma, 2);
        (void)r0; (void)T0;
        printf("%s: m=%d n=%d obj %.10g, %d/%d batch optimal, cut alpha %.6g over %d vertices\n", path, m, n, obj, nopt, N, alpha, nv);
        free(w); free(mv); free(ma); free(rr); free(TT);
    }
    if (lp) oracle_lp_destroy(lp);
    free(colptr); free(rowidx); free(val); free(q); free(b); free(sense); free(head); free(DR); free(o); free(o2);
    free(pi); free(pi2); free(st); free(st2); free(its); free(picks);
    return bad;
}

int main(int argc, char **argv) {
    const uint32_t ctr[4] = {0, 0, 0, 0}, key[2] = {0, 0}, want[4] = {0x6627e8d5u, 0xe169c58du, 0xbc57ac4cu, 0x9b00dbd8u};
    uint32_t out[4];
    oracle_philox4x32_10(ctr, key, out);
    int bad = memcmp(out, want, sizeof out) != 0;
    if (bad) fprintf(stderr, "philox4x32-10 known answer mismatch\n");
    for (int i = 1; i < argc; ++i) bad |= check(argv[i]);
    return bad;
}
