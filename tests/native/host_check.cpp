// host_check.cpp -- sanitizer driver for the host C++ of libtwosd_hip.so (host_basis.cpp):
// built with -fsanitize=address,undefined (Makefile target `sanitize`, host side only) and run
// by tests/test_native_sanitize.py on LP files that test writes.
//
// Per LP file: setup_solve from the slack basis (objective vs the file's expected value),
// dense_inverse + basis_dual_infeasibility of the optimal basis, then a chain of random basis
// exchanges whose eta file is replayed by compose_binv; the composed rows must equal the dense
// inverse of the final basis, and sparse_dual_infeasibility / sparse_basis_residual must agree
// with their dense counterparts.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>
#include "twosd_internal.h"

using namespace twosd;

static bool read_lp(const char *path, HostLP &L, std::vector<double> &b, double &expected) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    int mn[2];
    bool ok = fread(mn, sizeof(int), 2, f) == 2;
    L.m = mn[0]; L.n = mn[1];
    L.colptr.resize(L.n + 1);
    ok = ok && fread(L.colptr.data(), sizeof(int), L.n + 1, f) == (size_t)L.n + 1;
    const int nnz = ok ? L.colptr[L.n] : 0;
    L.rowidx.resize(nnz); L.val.resize(nnz); L.q.resize(L.n); L.sense.resize(L.m); b.resize(L.m);
    ok = ok && fread(L.rowidx.data(), sizeof(int), nnz, f) == (size_t)nnz;
    ok = ok && fread(L.val.data(), sizeof(double), nnz, f) == (size_t)nnz;
    ok = ok && fread(L.q.data(), sizeof(double), L.n, f) == (size_t)L.n;
    ok = ok && fread(L.sense.data(), 1, L.m, f) == (size_t)L.m;
    ok = ok && fread(b.data(), sizeof(double), L.m, f) == (size_t)L.m;
    ok = ok && fread(&expected, sizeof(double), 1, f) == 1;
    fclose(f);
    return ok;
}

static int check(const char *path) {
    HostLP L;
    std::vector<double> b;
    double expected = 0;
    if (!read_lp(path, L, b, expected)) { fprintf(stderr, "%s: unreadable\n", path); return 1; }
    const int m = L.m, n = L.n;
    std::vector<int> head;
    double obj = 0;
    int iters = 0;
    std::string err;
    const int st = setup_solve(L, b, head, obj, iters, err);
    if (st != TWOSD_LP_OPTIMAL || std::fabs(obj - expected) > 1e-9 * (1 + std::fabs(expected))) {
        fprintf(stderr, "%s: setup_solve status %d obj %.17g expected %.17g (%s)\n", path, st, obj, expected, err.c_str());
        return 1;
    }
    std::vector<double> B, Binv, pi0;
    basis_matrix(L, head, B);
    if (!dense_inverse(m, B, Binv)) { fprintf(stderr, "%s: singular optimal basis\n", path); return 1; }
    if (basis_dual_infeasibility(L, head, Binv, pi0) > 1e-7) { fprintf(stderr, "%s: not dual feasible\n", path); return 1; }
    if (sparse_dual_infeasibility(L, head, pi0) > 1e-7) { fprintf(stderr, "%s: sparse dual check disagrees\n", path); return 1; }
    // CSR of the start inverse
    std::vector<int> rp0(1, 0), rc0;
    std::vector<double> rv0;
    for (int i = 0; i < m; ++i) {
        for (int c = 0; c < m; ++c)
            if (Binv[(size_t)i * m + c] != 0.0) { rc0.push_back(c); rv0.push_back(Binv[(size_t)i * m + c]); }
        rp0.push_back((int)rc0.size());
    }
    // random exchanges: entering q, leaving row r = argmax |(B^{-1} a_q)_r|, eta as the GPU kernel writes it
    std::mt19937 rng(12345);
    std::vector<int> etap, etaoff(1, 0), eidx;
    std::vector<double> evals, a(m), col(m);
    std::vector<char> isb(n + m, 0);
    for (int i = 0; i < m; ++i) isb[head[i]] = 1;
    std::vector<double> Bcur = Binv;
    int K = 0;
    for (int tries = 0; tries < 200 && K < 8; ++tries) {
        const int q = (int)(rng() % (unsigned)(n + m));
        if (isb[q] || (q >= n && L.sense[q - n] == 'E')) continue;
        std::fill(a.begin(), a.end(), 0.0);
        if (q >= n) a[q - n] = 1.0;
        else
            for (int p = L.colptr[q]; p < L.colptr[q + 1]; ++p) a[L.rowidx[p]] = L.val[p];
        int r = -1;
        double best = 1e-3;
        for (int i = 0; i < m; ++i) {
            double s = 0;
            for (int c = 0; c < m; ++c) s += Bcur[(size_t)i * m + c] * a[c];
            col[i] = s;
            if (std::fabs(s) > best) { best = std::fabs(s); r = i; }
        }
        if (r < 0) continue;
        etap.push_back(r);
        for (int i = 0; i < m; ++i)
            if (col[i] != 0.0) { eidx.push_back(i); evals.push_back(i == r ? 1.0 / col[r] : -col[i] / col[r]); }
        etaoff.push_back((int)eidx.size());
        isb[head[r]] = 0; isb[q] = 1; head[r] = q;
        basis_matrix(L, head, B);
        if (!dense_inverse(m, B, Bcur)) { fprintf(stderr, "%s: exchange made a singular basis\n", path); return 1; }
        ++K;
    }
    std::vector<int> rp, rc;
    std::vector<double> rv;
    compose_binv(m, rp0, rc0, rv0, K, etap.data(), etaoff.data(), eidx.data(), evals.data(), rp, rc, rv);
    double amax = 0, worst = 0;
    std::vector<double> dense((size_t)m * m, 0.0);
    for (int i = 0; i < m; ++i)
        for (int p = rp[i]; p < rp[i + 1]; ++p) dense[(size_t)i * m + rc[p]] = rv[p];
    for (size_t t = 0; t < dense.size(); ++t) {
        amax = std::max(amax, std::fabs(Bcur[t]));
        worst = std::max(worst, std::fabs(dense[t] - Bcur[t]));
    }
    const double resid = sparse_basis_residual(L, head, rp, rc, rv, 8);
    if (worst > 1e-9 * (1 + amax) || resid > 1e-8) {
        fprintf(stderr, "%s: composed inverse off by %.3g (max %.3g), residual %.3g after %d exchanges\n", path, worst, amax,
                resid, K);
        return 1;
    }
    printf("%s: m=%d n=%d obj %.10g, %d setup pivots, %d composed exchanges, max dev %.2g\n", path, m, n, obj, iters, K, worst);
    return 0;
}

int main(int argc, char **argv) {
    int bad = 0;
    for (int i = 1; i < argc; ++i) bad |= check(argv[i]);
    return bad;
}
