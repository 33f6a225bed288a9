// host_basis.cpp -- one-time host setup of the shared warm-start basis.
//
// The per-scenario LPs of solve_problem! (smps_routines.jl:50-62) differ only in their
// right-hand side, so one optimal basis B0 (computed once, here) is dual feasible for
// every scenario and every x; the GPU kernel warm-starts every scenario from it.  This
// file is NOT on the per-scenario path: it runs once per template (like the crash
// basis a simplex code computes before its first solve).
//
// setup_solve: revised dual simplex with an explicit dense inverse updated by rank-1
// pivots and re-inverted every kRefactor pivots (O(m^2) per pivot).  Dantzig leaving
// row, Harris two-pass ratio test, from the slack basis (dual feasible when q >= 0).  With
// negative costs (baa99-20) the slack basis is not dual feasible: a dual-simplex phase on
// max(q, 0) finds a primal-feasible basis, then a primal simplex phase on q ends optimal.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include "twosd_internal.h"

namespace twosd {

static constexpr double kTolP = 1e-9, kTolD = 1e-9, kTolPiv = 1e-9;
static constexpr int kRefactor = 64;

bool dense_inverse(int m, const std::vector<double> &A, std::vector<double> &Ainv) {
    // Gauss-Jordan with partial pivoting on [A | I]
    std::vector<double> M(A);
    Ainv.assign((size_t)m * m, 0.0);
    for (int i = 0; i < m; ++i) Ainv[(size_t)i * m + i] = 1.0;
    for (int c = 0; c < m; ++c) {
        int p = c;
        double best = std::fabs(M[(size_t)c * m + c]);
        for (int i = c + 1; i < m; ++i) {
            double v = std::fabs(M[(size_t)i * m + c]);
            if (v > best) { best = v; p = i; }
        }
        if (best < 1e-13) return false;
        if (p != c) {
            for (int j = 0; j < m; ++j) {
                std::swap(M[(size_t)p * m + j], M[(size_t)c * m + j]);
                std::swap(Ainv[(size_t)p * m + j], Ainv[(size_t)c * m + j]);
            }
        }
        const double inv = 1.0 / M[(size_t)c * m + c];
        double *mc = &M[(size_t)c * m], *ic = &Ainv[(size_t)c * m];
        for (int j = 0; j < m; ++j) { mc[j] *= inv; ic[j] *= inv; }
        for (int i = 0; i < m; ++i) {
            if (i == c) continue;
            const double f = M[(size_t)i * m + c];
            if (f == 0.0) continue;
            double *mi = &M[(size_t)i * m], *ii = &Ainv[(size_t)i * m];
            for (int j = 0; j < m; ++j) { mi[j] -= f * mc[j]; ii[j] -= f * ic[j]; }
        }
    }
    return true;
}

void basis_matrix(const HostLP &L, const std::vector<int> &head, std::vector<double> &B) {
    const int m = L.m;
    B.assign((size_t)m * m, 0.0);
    for (int c = 0; c < m; ++c) {
        const int j = head[c];
        if (j >= L.n) B[(size_t)(j - L.n) * m + c] = 1.0;
        else
            for (int p = L.colptr[j]; p < L.colptr[j + 1]; ++p) B[(size_t)L.rowidx[p] * m + c] = L.val[p];
    }
}

static inline int btype_of(const HostLP &L, int j) {
    if (j < L.n) return BT_Y;
    char s = L.sense[j - L.n];
    return s == 'G' ? BT_G : (s == 'L' ? BT_L : BT_E);
}

static inline double col_dot(const HostLP &L, int j, const double *v) {
    if (j >= L.n) return v[j - L.n];
    double s = 0.0;
    for (int p = L.colptr[j]; p < L.colptr[j + 1]; ++p) s += v[L.rowidx[p]] * L.val[p];
    return s;
}

double basis_dual_infeasibility(const HostLP &L, const std::vector<int> &head,
                                const std::vector<double> &Binv, std::vector<double> &pi0) {
    const int m = L.m, n = L.n;
    pi0.assign(m, 0.0);
    for (int i = 0; i < m; ++i) {
        const int j = head[i];
        const double c = j < n ? L.q[j] : 0.0;
        if (c == 0.0) continue;
        const double *row = &Binv[(size_t)i * m];
        for (int t = 0; t < m; ++t) pi0[t] += c * row[t];
    }
    std::vector<char> isb(n + m, 0);
    for (int i = 0; i < m; ++i) isb[head[i]] = 1;
    double worst = 0.0;
    for (int j = 0; j < n + m; ++j) {
        if (isb[j]) continue;
        const int bt = btype_of(L, j);
        if (bt == BT_E) continue;
        const double d = (j < n ? L.q[j] : 0.0) - col_dot(L, j, pi0.data());
        const double inf = (bt == BT_G) ? d : -d;   // G slack sits at its upper bound
        if (inf > worst) worst = inf;
    }
    return worst;
}

// dual simplex from the dual-feasible basis `head` (the slack basis when every q_j >= 0) to an
// optimal basis of L at rhs b
static int dual_simplex(const HostLP &L, const std::vector<double> &b, std::vector<int> &head, int &iters,
                        std::string &err) {
    const int m = L.m, n = L.n;
    std::vector<char> isb(n + m, 0);
    for (int i = 0; i < m; ++i) isb[head[i]] = 1;
    std::vector<double> Binv, B, xB(m), pi(m), rho(m), col(m);
    auto reinvert = [&]() -> bool {
        basis_matrix(L, head, B);
        if (!dense_inverse(m, B, Binv)) return false;
        for (int i = 0; i < m; ++i) {
            const double *row = &Binv[(size_t)i * m];
            double s = 0.0;
            for (int t = 0; t < m; ++t) s += row[t] * b[t];
            xB[i] = s;
        }
        std::fill(pi.begin(), pi.end(), 0.0);
        for (int i = 0; i < m; ++i) {
            const int j = head[i];
            const double c = j < n ? L.q[j] : 0.0;
            if (c == 0.0) continue;
            const double *row = &Binv[(size_t)i * m];
            for (int t = 0; t < m; ++t) pi[t] += c * row[t];
        }
        return true;
    };
    if (!reinvert()) { err = "setup_solve: singular start basis"; return TWOSD_LP_NUMERIC; }
    const int max_iter = 50 * (m + n) + 1000;
    for (;;) {
        // leaving row: largest primal infeasibility (lowest index on ties)
        int r = -1;
        double best = 0.0, delta = 0.0;
        for (int i = 0; i < m; ++i) {
            const int bt = btype_of(L, head[i]);
            const double x = xB[i];
            double d = 0.0;
            if ((bt == BT_Y || bt == BT_L) && x < -kTolP) d = x;
            else if (bt == BT_G && x > kTolP) d = x;
            else if (bt == BT_E && std::fabs(x) > kTolP) d = x;
            else continue;
            if (std::fabs(d) > best) { best = std::fabs(d); r = i; delta = d; }
        }
        if (r < 0) break;
        if (iters >= max_iter) { err = "setup_solve: iteration limit"; return TWOSD_LP_ITER_LIMIT; }
        std::memcpy(rho.data(), &Binv[(size_t)r * m], sizeof(double) * m);
        const double s = delta > 0 ? 1.0 : -1.0;
        double thmax = std::numeric_limits<double>::infinity();
        // pass 1
        for (int j = 0; j < n + m; ++j) {
            if (isb[j]) continue;
            const int bt = btype_of(L, j);
            if (bt == BT_E) continue;
            const double a = s * col_dot(L, j, rho.data());
            const bool atlb = bt != BT_G;
            if (atlb ? a > kTolPiv : a < -kTolPiv) {
                const double d = (j < n ? L.q[j] : 0.0) - col_dot(L, j, pi.data());
                const double ratio = (atlb ? d + kTolD : d - kTolD) / a;
                if (ratio < thmax) thmax = ratio;
            }
        }
        if (thmax == std::numeric_limits<double>::infinity()) { err = "setup_solve: primal infeasible"; return TWOSD_LP_INFEASIBLE; }
        int q = -1;
        double amax = 0.0, dq = 0.0, aqs = 0.0;
        for (int j = 0; j < n + m; ++j) {
            if (isb[j]) continue;
            const int bt = btype_of(L, j);
            if (bt == BT_E) continue;
            const double a = s * col_dot(L, j, rho.data());
            const bool atlb = bt != BT_G;
            if (atlb ? a > kTolPiv : a < -kTolPiv) {
                const double d = (j < n ? L.q[j] : 0.0) - col_dot(L, j, pi.data());
                if (d / a <= thmax && std::fabs(a) > amax) { amax = std::fabs(a); q = j; dq = d; aqs = a; }
            }
        }
        if (q < 0) { err = "setup_solve: ratio test failed"; return TWOSD_LP_NUMERIC; }
        const double thetaD = dq / aqs;
        // entering column
        std::fill(col.begin(), col.end(), 0.0);
        if (q >= n) {
            for (int i = 0; i < m; ++i) col[i] = Binv[(size_t)i * m + (q - n)];
        } else {
            for (int p = L.colptr[q]; p < L.colptr[q + 1]; ++p) {
                const int rr = L.rowidx[p];
                const double a = L.val[p];
                for (int i = 0; i < m; ++i) col[i] += a * Binv[(size_t)i * m + rr];
            }
        }
        const double arq = col[r];
        if (std::fabs(arq) < 1e-12) { err = "setup_solve: tiny pivot"; return TWOSD_LP_NUMERIC; }
        for (int i = 0; i < m; ++i) pi[i] += s * thetaD * rho[i];
        const double thetaP = delta / arq;
        for (int i = 0; i < m; ++i) xB[i] -= thetaP * col[i];
        xB[r] = thetaP;
        // explicit inverse update
        double *rr = &Binv[(size_t)r * m];
        for (int t = 0; t < m; ++t) rr[t] /= arq;
        for (int i = 0; i < m; ++i) {
            if (i == r || col[i] == 0.0) continue;
            const double f = col[i];
            double *ri = &Binv[(size_t)i * m];
            for (int t = 0; t < m; ++t) ri[t] -= f * rr[t];
        }
        isb[head[r]] = 0;
        isb[q] = 1;
        head[r] = q;
        ++iters;
        if (iters % kRefactor == 0 && !reinvert()) { err = "setup_solve: singular basis"; return TWOSD_LP_NUMERIC; }
    }
    return TWOSD_LP_OPTIMAL;
}

// primal simplex from the primal-feasible basis `head` to an optimal basis of L at rhs b.
// Nonbasic variables sit at 0: y_j and L slacks may increase, G slacks (upper bound 0) may
// decrease, E slacks are fixed.  Dantzig pricing (lowest index on ties), Harris two-pass ratio
// test; after 50 consecutive degenerate pivots the entering variable is the lowest-index
// candidate (Bland) until a pivot makes progress.
static int primal_simplex(const HostLP &L, const std::vector<double> &b, std::vector<int> &head, int &iters,
                          std::string &err) {
    const int m = L.m, n = L.n;
    std::vector<char> isb(n + m, 0);
    for (int i = 0; i < m; ++i) isb[head[i]] = 1;
    std::vector<double> Binv, B, xB(m), pi(m), col(m);
    auto reinvert = [&]() -> bool {
        basis_matrix(L, head, B);
        if (!dense_inverse(m, B, Binv)) return false;
        for (int i = 0; i < m; ++i) {
            const double *row = &Binv[(size_t)i * m];
            double s = 0.0;
            for (int t = 0; t < m; ++t) s += row[t] * b[t];
            xB[i] = s;
        }
        return true;
    };
    auto duals = [&]() {
        std::fill(pi.begin(), pi.end(), 0.0);
        for (int i = 0; i < m; ++i) {
            const int j = head[i];
            const double c = j < n ? L.q[j] : 0.0;
            if (c == 0.0) continue;
            const double *row = &Binv[(size_t)i * m];
            for (int t = 0; t < m; ++t) pi[t] += c * row[t];
        }
    };
    if (!reinvert()) { err = "setup_solve: singular phase-1 basis"; return TWOSD_LP_NUMERIC; }
    const int max_iter = 50 * (m + n) + 1000;
    int degenerate = 0;
    for (;;) {
        duals();
        const bool bland = degenerate >= 50;
        int q = -1;
        double best = 0.0, sigma = 0.0;
        for (int j = 0; j < n + m; ++j) {
            if (isb[j]) continue;
            const int bt = btype_of(L, j);
            if (bt == BT_E) continue;
            const double d = (j < n ? L.q[j] : 0.0) - col_dot(L, j, pi.data());
            const double gain = bt == BT_G ? d : -d;        // objective decrease per unit move
            if (gain > kTolD && (q < 0 || (!bland && gain > best))) {
                q = j; best = gain; sigma = bt == BT_G ? -1.0 : 1.0;
                if (bland) break;
            }
        }
        if (q < 0) break;                                   // optimal
        if (iters >= max_iter) { err = "setup_solve: iteration limit (primal)"; return TWOSD_LP_ITER_LIMIT; }
        std::fill(col.begin(), col.end(), 0.0);
        if (q >= n) {
            for (int i = 0; i < m; ++i) col[i] = Binv[(size_t)i * m + (q - n)];
        } else {
            for (int p = L.colptr[q]; p < L.colptr[q + 1]; ++p) {
                const int rr = L.rowidx[p];
                const double a = L.val[p];
                for (int i = 0; i < m; ++i) col[i] += a * Binv[(size_t)i * m + rr];
            }
        }
        // x_B(t) = x_B - t * sigma * col, t >= 0: basic y / L slacks stay >= 0, G slacks <= 0,
        // E slacks at 0
        auto blocks = [&](int i, double a, bool relaxed, double &ratio) -> bool {
            const int bt = btype_of(L, head[i]);
            const double tol = relaxed ? kTolP : 0.0;
            if ((bt == BT_Y || bt == BT_L || bt == BT_E) && a > kTolPiv) { ratio = (xB[i] + tol) / a; return true; }
            if ((bt == BT_G || bt == BT_E) && a < -kTolPiv) { ratio = (xB[i] - tol) / a; return true; }
            return false;
        };
        double thmax = std::numeric_limits<double>::infinity();
        for (int i = 0; i < m; ++i) {
            double ratio;
            if (blocks(i, sigma * col[i], true, ratio) && ratio < thmax) thmax = ratio;
        }
        if (thmax == std::numeric_limits<double>::infinity()) { err = "setup_solve: stage-2 LP unbounded"; return TWOSD_LP_NUMERIC; }
        int r = -1;
        double amax = 0.0, theta = 0.0;
        for (int i = 0; i < m; ++i) {
            double ratio;
            const double a = sigma * col[i];
            if (blocks(i, a, false, ratio) && ratio <= thmax && std::fabs(a) > amax) {
                amax = std::fabs(a); r = i; theta = std::max(ratio, 0.0);
            }
        }
        if (r < 0) { err = "setup_solve: primal ratio test failed"; return TWOSD_LP_NUMERIC; }
        const double arq = col[r];
        for (int i = 0; i < m; ++i) xB[i] -= theta * sigma * col[i];
        xB[r] = theta * sigma;
        double *rr = &Binv[(size_t)r * m];
        for (int t = 0; t < m; ++t) rr[t] /= arq;
        for (int i = 0; i < m; ++i) {
            if (i == r || col[i] == 0.0) continue;
            const double f = col[i];
            double *ri = &Binv[(size_t)i * m];
            for (int t = 0; t < m; ++t) ri[t] -= f * rr[t];
        }
        isb[head[r]] = 0;
        isb[q] = 1;
        head[r] = q;
        ++iters;
        degenerate = theta > 1e-12 ? 0 : degenerate + 1;
        if (iters % kRefactor == 0 && !reinvert()) { err = "setup_solve: singular basis (primal)"; return TWOSD_LP_NUMERIC; }
    }
    return TWOSD_LP_OPTIMAL;
}

int setup_solve(const HostLP &L, const std::vector<double> &b, std::vector<int> &head, double &obj,
                int &iters, std::string &err) {
    const int m = L.m, n = L.n;
    head.resize(m);
    for (int i = 0; i < m; ++i) head[i] = n + i;
    iters = 0;
    bool negative = false;
    for (int j = 0; j < n; ++j) negative |= L.q[j] < 0;
    int st;
    if (!negative) {
        // q >= 0: the slack basis is dual feasible
        st = dual_simplex(L, b, head, iters, err);
    } else {
        // phase 1: the dual simplex on costs max(q, 0) (slack basis dual feasible) ends at a
        // primal-feasible basis of the same rows; phase 2: primal simplex on q from there
        HostLP L1 = L;
        for (double &c : L1.q) c = std::max(c, 0.0);
        st = dual_simplex(L1, b, head, iters, err);
        if (st == TWOSD_LP_OPTIMAL) st = primal_simplex(L, b, head, iters, err);
    }
    if (st != TWOSD_LP_OPTIMAL) return st;
    std::vector<double> B, Binv;
    basis_matrix(L, head, B);
    if (!dense_inverse(m, B, Binv)) { err = "setup_solve: singular final basis"; return TWOSD_LP_NUMERIC; }
    obj = 0.0;
    for (int i = 0; i < m; ++i) {
        if (head[i] >= n) continue;
        double xb = 0.0;
        const double *row = &Binv[(size_t)i * m];
        for (int t = 0; t < m; ++t) xb += row[t] * b[t];
        obj += L.q[head[i]] * xb;
    }
    return TWOSD_LP_OPTIMAL;
}

// ---- composed pool bases (twosd_pool_refresh) ---------------------------------------------

void compose_binv(int m, const std::vector<int> &rptr0, const std::vector<int> &rcol0, const std::vector<double> &rval0,
                  int K, const int *etap, const int *etaoff, const int *eidx, const double *evals, std::vector<int> &rptr,
                  std::vector<int> &rcol, std::vector<double> &rval) {
    // E_t = I + (eta - e_r) e_r' on the left: row r <- eta_r row r, row i <- row i + eta_i row r
    // (the old row r for every i), as sorted sparse row merges.  Only rows in the support of
    // some eta change (the pivot row is in its own eta); the others are copied from B0^{-1}.
    std::vector<int> slot(m, -1);
    std::vector<std::vector<std::pair<int, double>>> rows;
    for (int e = 0; e < (K > 0 ? etaoff[K] : 0); ++e) {
        const int i = eidx[e];
        if (slot[i] >= 0) continue;
        slot[i] = (int)rows.size();
        rows.emplace_back();
        auto &row = rows.back();
        for (int q = rptr0[i]; q < rptr0[i + 1]; ++q) row.push_back({rcol0[q], rval0[q]});
    }
    std::vector<std::pair<int, double>> rr, tmp;
    for (int t = 0; t < K; ++t) {
        const int r = etap[t];
        rr = rows[slot[r]];
        for (int e = etaoff[t]; e < etaoff[t + 1]; ++e) {
            const int i = eidx[e];
            const double v = evals[e];
            auto &a = rows[slot[i]];
            if (i == r) {
                a = rr;
                for (auto &cv : a) cv.second *= v;
                continue;
            }
            tmp.clear();
            size_t p = 0, q = 0;
            while (p < a.size() || q < rr.size()) {
                if (q == rr.size() || (p < a.size() && a[p].first < rr[q].first)) tmp.push_back(a[p++]);
                else if (p == a.size() || rr[q].first < a[p].first) { tmp.push_back({rr[q].first, v * rr[q].second}); ++q; }
                else { tmp.push_back({a[p].first, std::fma(v, rr[q].second, a[p].second)}); ++p; ++q; }
            }
            a.swap(tmp);
        }
    }
    double amax = 0.0;
    for (double v : rval0) amax = std::max(amax, std::fabs(v));
    for (auto &row : rows)
        for (auto &cv : row) amax = std::max(amax, std::fabs(cv.second));
    const double drop = 1e-14 * amax;
    rptr.assign(1, 0);
    rcol.clear();
    rval.clear();
    rcol.reserve(rcol0.size() + rcol0.size() / 4);
    rval.reserve(rcol0.size() + rcol0.size() / 4);
    for (int i = 0; i < m; ++i) {
        if (slot[i] < 0) {
            rcol.insert(rcol.end(), rcol0.begin() + rptr0[i], rcol0.begin() + rptr0[i + 1]);
            rval.insert(rval.end(), rval0.begin() + rptr0[i], rval0.begin() + rptr0[i + 1]);
        } else {
            for (auto &cv : rows[slot[i]])
                if (std::fabs(cv.second) > drop) { rcol.push_back(cv.first); rval.push_back(cv.second); }
        }
        rptr.push_back((int)rcol.size());
    }
}

double sparse_dual_infeasibility(const HostLP &L, const std::vector<int> &head, const std::vector<double> &pi0) {
    const int m = L.m, n = L.n;
    std::vector<char> isb(n + m, 0);
    for (int i = 0; i < m; ++i) isb[head[i]] = 1;
    double worst = 0.0;
    for (int j = 0; j < n + m; ++j) {
        if (isb[j]) continue;
        const int bt = btype_of(L, j);
        if (bt == BT_E) continue;
        const double d = (j < n ? L.q[j] : 0.0) - col_dot(L, j, pi0.data());
        const double inf = bt == BT_G ? d : -d;   // a G slack sits at its upper bound 0
        worst = std::max(worst, inf);
    }
    return worst;
}

double sparse_basis_residual(const HostLP &L, const std::vector<int> &head, const std::vector<int> &rptr,
                             const std::vector<int> &rcol, const std::vector<double> &rval, int probes) {
    const int m = L.m, n = L.n;
    std::vector<double> a(m);
    double worst = 0.0;
    for (int probe = 0; probe < probes; ++probe) {
        const int i0 = (int)(((long long)probe * 7919 + 13) % m);
        const int j = head[i0];
        std::fill(a.begin(), a.end(), 0.0);
        if (j >= n) a[j - n] = 1.0;
        else
            for (int q = L.colptr[j]; q < L.colptr[j + 1]; ++q) a[L.rowidx[q]] = L.val[q];
        for (int i = 0; i < m; ++i) {
            double v = 0.0;
            for (int q = rptr[i]; q < rptr[i + 1]; ++q) v += rval[q] * a[rcol[q]];
            worst = std::max(worst, std::fabs(v - (i == i0 ? 1.0 : 0.0)));
        }
    }
    return worst;
}

}  // namespace twosd
