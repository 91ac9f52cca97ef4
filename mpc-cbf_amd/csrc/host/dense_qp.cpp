// dense_qp.cpp — exact equality elimination for the generic flattened-QP path (see dense_qp.hpp).
#include "dense_qp.hpp"

#include <cmath>
#include <stdexcept>
#include <string>

namespace mpccbf {

namespace {

constexpr double kInf = 1e300;       // |bound| >= 1e300 means "absent" (numeric_limits lowest/max)
constexpr double kFeasTol = 1e-6;    // CPLEX default feasibility tolerance (CPLEX.cpp:8 default ctor)

bool finite_bound(double v) { return std::isfinite(v) && std::fabs(v) < kInf; }

void require(bool ok, const char* msg) {
    if (!ok) throw std::invalid_argument(msg);
}

}  // namespace

ReducedQP reduce_dense_qp(const mpccbf_dense_qp& qp) {
    require(qp.n >= 1, "dense QP: n must be >= 1");
    require(qp.m >= 0, "dense QP: m must be >= 0");
    require(qp.H && qp.c, "dense QP: H and c are required");
    require(qp.m == 0 || (qp.A && qp.lo && qp.hi), "dense QP: A, lo, hi are required when m > 0");
    const int n = qp.n, m = qp.m;
    ReducedQP r;
    r.n = n;
    r.c0 = qp.c0;
    r.Hs = Mat(n, n);
    r.c.assign(qp.c, qp.c + n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const double v = 0.5 * (qp.H[(size_t)i * n + j] + qp.H[(size_t)j * n + i]);
            require(std::isfinite(v), "dense QP: H has a non-finite entry");
            r.Hs(i, j) = v;
        }
    for (int i = 0; i < n; i++) require(std::isfinite(r.c[i]), "dense QP: c has a non-finite entry");

    // ---- equalities: rows with lo == hi (finite) and fixed variables
    std::vector<std::vector<double>> eq_rows;
    std::vector<double> eq_rhs;
    std::vector<int> ineq;  // remaining row indices
    for (int k = 0; k < m; k++) {
        const double lo = qp.lo[k], hi = qp.hi[k];
        require(!std::isnan(lo) && !std::isnan(hi), "dense QP: NaN row bound");
        if (finite_bound(lo) && lo == hi) {
            eq_rows.emplace_back(qp.A + (size_t)k * n, qp.A + (size_t)(k + 1) * n);
            eq_rhs.push_back(lo);
        } else if (finite_bound(lo) || finite_bound(hi)) {
            ineq.push_back(k);
        }
    }
    std::vector<int> vbound;  // variables with a (non-fixing) finite bound
    for (int i = 0; i < n; i++) {
        const double lo = qp.vlo ? qp.vlo[i] : -kInf, hi = qp.vhi ? qp.vhi[i] : kInf;
        require(!std::isnan(lo) && !std::isnan(hi), "dense QP: NaN variable bound");
        if (finite_bound(lo) && lo == hi) {
            std::vector<double> e(n, 0.0);
            e[i] = 1.0;
            eq_rows.push_back(e);
            eq_rhs.push_back(lo);
        } else if (finite_bound(lo) || finite_bound(hi)) {
            vbound.push_back(i);
        }
    }
    Mat E((int)eq_rows.size(), n);
    for (int k = 0; k < E.r; k++)
        for (int j = 0; j < n; j++) E(k, j) = eq_rows[k][j];
    Mat Xp;
    int rank = 0;
    null_space(E, 1e-12, r.Z, Xp, rank);
    r.nz = n - rank;
    r.xp.assign(n, 0.0);
    for (int i = 0; i < n; i++)
        for (int k = 0; k < E.r; k++) r.xp[i] += Xp(i, k) * eq_rhs[k];
    // inconsistent equalities -> infeasible (same absolute tolerance as every other row)
    for (int k = 0; k < E.r; k++) {
        double v = 0.0;
        for (int j = 0; j < n; j++) v += E(k, j) * r.xp[j];
        if (std::fabs(v - eq_rhs[k]) > kFeasTol) r.status = MPCCBF_INFEASIBLE, r.eq_infeasible = true;
    }

    // ---- reduced objective: x^T Hs x with x = xp + Z y  ->  1/2 y^T (2 Z^T Hs Z) y + ...
    const int nz = r.nz;
    std::vector<double> hx(n, 0.0);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) hx[i] += r.Hs(i, j) * r.xp[j];
    r.k0 = qp.c0;
    for (int i = 0; i < n; i++) r.k0 += r.xp[i] * (hx[i] + r.c[i]);
    r.P = Mat(nz, nz);
    r.q.assign(nz, 0.0);
    Mat HZ(n, nz);
    for (int i = 0; i < n; i++)
        for (int b = 0; b < nz; b++) {
            double v = 0.0;
            for (int j = 0; j < n; j++) v += r.Hs(i, j) * r.Z(j, b);
            HZ(i, b) = v;
        }
    for (int a = 0; a < nz; a++) {
        for (int b = 0; b < nz; b++) {
            double v = 0.0;
            for (int i = 0; i < n; i++) v += r.Z(i, a) * HZ(i, b);
            r.P(a, b) = 2.0 * v;
        }
        double v = 0.0;
        for (int i = 0; i < n; i++) v += r.Z(i, a) * (2.0 * hx[i] + r.c[i]);
        r.q[a] = v;
    }
    for (int a = 0; a < nz; a++)  // exact symmetry for the device Cholesky
        for (int b = a + 1; b < nz; b++) r.P(a, b) = r.P(b, a) = 0.5 * (r.P(a, b) + r.P(b, a));
    try {
        r.LP = cholesky(r.P);
        r.pd = nz > 0;
    } catch (const std::exception&) {
        r.pd = false;
    }

    // ---- inequality rows in y: g = Z^T a, bounds shifted by a^T xp
    std::vector<std::vector<double>> gs;
    auto add_row = [&](const double* a, double lo, double hi) {
        std::vector<double> g(nz, 0.0);
        double amax = 0.0, shift = 0.0, gmax = 0.0;
        for (int j = 0; j < n; j++) {
            amax = std::max(amax, std::fabs(a[j]));
            shift += a[j] * r.xp[j];
        }
        for (int b = 0; b < nz; b++) {
            double v = 0.0;
            for (int j = 0; j < n; j++) v += a[j] * r.Z(j, b);
            g[b] = v;
            gmax = std::max(gmax, std::fabs(v));
        }
        const bool hl = finite_bound(lo), hu = finite_bound(hi);
        if (gmax <= 1e-13 * std::max(1.0, amax)) {  // constant row: a feasibility check of xp
            if ((hl && shift < lo - kFeasTol) || (hu && shift > hi + kFeasTol)) r.status = MPCCBF_INFEASIBLE;
            return;
        }
        gs.push_back(g);
        r.lo.push_back(hl ? lo - shift : -kInf);
        r.hi.push_back(hu ? hi - shift : kInf);
    };
    for (int k : ineq) add_row(qp.A + (size_t)k * n, qp.lo[k], qp.hi[k]);
    std::vector<double> unit(n, 0.0);
    for (int i : vbound) {
        unit[i] = 1.0;
        add_row(unit.data(), qp.vlo ? qp.vlo[i] : -kInf, qp.vhi ? qp.vhi[i] : kInf);
        unit[i] = 0.0;
    }
    r.m = (int)gs.size();
    r.G = Mat(r.m, nz);
    for (int k = 0; k < r.m; k++)
        for (int b = 0; b < nz; b++) r.G(k, b) = gs[k][b];
    if (r.status < 0 && nz == 0) r.status = MPCCBF_OPTIMAL;  // x = xp is the only point
    return r;
}

void expand_solution(const ReducedQP& r, const double* y, double* x, double* obj) {
    const int n = r.n;
    for (int i = 0; i < n; i++) {
        double v = r.xp[i];
        for (int b = 0; b < r.nz; b++) v += r.Z(i, b) * y[b];
        x[i] = v;
    }
    double f = r.c0;
    for (int i = 0; i < n; i++) {
        double hxi = 0.0;
        for (int j = 0; j < n; j++) hxi += r.Hs(i, j) * x[j];
        f += x[i] * (hxi + r.c[i]);
    }
    *obj = f;
}

}  // namespace mpccbf
