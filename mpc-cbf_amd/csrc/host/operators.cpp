// operators.cpp — host precompute of the parameter-only MPC-CBF QP operators.
//
// What the reference assembles per call through hash maps (PiecewiseBezierMPCQPGenerator.cpp,
// BezierQPOperations.cpp, ConnectivityIMPCCBF.cpp:102-197) is, apart from a handful of
// state-dependent vectors, identical for every agent and every control step. This file builds
// those shared pieces once, eliminates the equality constraints (initial state + C^d
// continuity) by a null-space basis, and removes provably redundant shared rows, so that the
// device solves an nz-dimensional inequality QP per agent (nz = 6 for base_config.json).
#include "operators.hpp"

#include <cmath>
#include <cstdint>
#include <limits>
#include <sstream>

namespace mpccbf {

namespace {

double binom(int n, int k) {
    if (k < 0 || k > n) return 0.0;
    double r = 1.0;
    for (int i = 1; i <= k; i++) r = r * (n - k + i) / i;
    return std::round(r);
}
double falling(int j, int d) {  // j! / (j-d)!
    double r = 1.0;
    for (int i = 0; i < d; i++) r *= (j - i);
    return r;
}

// Monomial coefficients (in t) of the d-th derivative of the degree-p Bernstein basis on
// [0, T]: row i gives b_i^(d)(t) = sum_k coef(i, k) t^k  (same function as
// splines/src/detail/BezierOperations.cpp:11-50 and :54-121 compute).
Mat bernstein_derivative_monomials(int p, double T, int d) {
    Mat M(p + 1, p + 1);
    if (T == 0.0) {
        if (d == 0) M(0, 0) = 1.0;
        return M;
    }
    for (int i = 0; i <= p; i++)
        for (int j = i; j <= p; j++) {
            if (j < d) continue;
            const double sign = ((j - i) % 2 == 0) ? 1.0 : -1.0;
            const double cj = binom(p, i) * binom(p - i, j - i) * sign / std::pow(T, j);
            M(i, j - d) += cj * falling(j, d);
        }
    return M;
}

std::vector<double> eval_monomials(const Mat& M, double t) {
    std::vector<double> v(M.r, 0.0);
    for (int i = 0; i < M.r; i++) {
        double s = 0.0, tp = 1.0;
        for (int k = 0; k < M.c; k++, tp *= t) s += M(i, k) * tp;
        v[i] = s;
    }
    return v;
}

struct Curve {
    int P, C, n_piece, n;
    double T;
    std::vector<double> cum;
    explicit Curve(const mpccbf_params& p)
        : P(p.num_pieces), C(p.num_control_points), n_piece(DIM * p.num_control_points),
          n(p.num_pieces * DIM * p.num_control_points), T(p.piece_max_parameter) {
        double acc = 0.0;
        for (int i = 0; i < P; i++) cum.push_back(acc = (i == 0 ? T : acc + T));
    }
    // piece + local parameter for global t (lower_bound on cumulative parameters, local t
    // clamped: PiecewiseBezierMPCQPOperations.cpp:190-223, SingleParameterPiecewiseCurve.cpp:94-127)
    void locate(double t, int& piece, double& local) const {
        int i = 0;
        while (i < P && cum[i] < t) i++;
        if (i >= P) throw std::invalid_argument("parameter is out of range [0, max parameter]");
        piece = i;
        local = (i == 0) ? t : t - cum[i - 1];
        local = std::min(std::max(local, 0.0), T);
    }
    // full-length row (n) selecting dim `dim` of the d-th derivative at global parameter t
    std::vector<double> row_at(double t, int dim, int d) const {
        int piece;
        double local;
        locate(t, piece, local);
        return row_local(piece, local, dim, d);
    }
    std::vector<double> row_local(int piece, double local, int dim, int d) const {
        std::vector<double> r(n, 0.0);
        Mat M = bernstein_derivative_monomials(C - 1, T, d);
        std::vector<double> b = eval_monomials(M, local);
        for (int i = 0; i < C; i++) r[piece * n_piece + dim * C + i] = b[i];
        return r;
    }
};

// Eigen::VectorXd::LinSpaced(K, 0, (K-1) h): i * step except the last sample, which is exactly
// `high` (Eigen 3.4 linspaced_op_impl); the h_samples of PiecewiseBezierMPCQPOperations.cpp:33-34
// and ConnectivityIMPCCBF.cpp:43.
std::vector<double> h_samples(int K, double h) {
    std::vector<double> v(K);
    const double high = (K - 1) * h;
    if (K == 1) {
        v[0] = high;
        return v;
    }
    const double step = (high - 0.0) / double(K - 1);
    for (int i = 0; i < K; i++) v[i] = (i == K - 1) ? high : 0.0 + double(i) * step;
    return v;
}

Mat row_to_mat(const std::vector<double>& r) {
    Mat m(1, (int)r.size());
    m.a = r;
    return m;
}

double dotv(const std::vector<double>& a, const std::vector<double>& b) {
    double s = 0;
    for (size_t i = 0; i < a.size(); i++) s += a[i] * b[i];
    return s;
}

}  // namespace

std::string validate_params(const mpccbf_params& p) {
    std::ostringstream os;
    if (p.Ts > p.h) return "Control timestep Ts must be <= MPC timestep h";
    if (p.h <= 0 || p.Ts <= 0) return "Time parameters h and Ts must be positive";
    const double ratio = p.h / p.Ts;
    if (std::fabs(ratio - std::round(ratio)) > 1e-10)
        return "MPC timestep h must be an integer multiple of control timestep Ts";
    if (p.spd_f > p.k_hor) return "Speed factor spd_f must be <= prediction horizon k_hor";
    if (p.spd_f < 1) return "Speed factor spd_f must be at least 1";
    if (p.k_hor < 1) return "Prediction horizon k_hor must be at least 1";
    if (p.cbf_horizon < 1) return "CBF horizon must be at least 1";
    if (p.impc_iter < 1) return "IMPC iterations must be at least 1";
    if (p.slack_mode && p.slack_cost <= 0) return "Slack cost must be positive when slack_mode is enabled";
    if (p.slack_mode && (p.slack_decay_rate <= 0 || p.slack_decay_rate > 1))
        return "Slack decay rate must be in (0,1] when slack_mode is enabled";
    if (p.cbf_horizon > p.k_hor) return "CBF horizon must be <= MPC prediction horizon k_hor";
    if (static_cast<double>(p.k_hor - 1) * p.h > static_cast<double>(p.num_pieces) * p.piece_max_parameter)
        return "MPC sampling range exceeds Bezier curve parameter range";
    if (p.num_pieces < 1 || p.num_control_points < 1) return "num_pieces and num_control_points must be >= 1";
    if (p.continuity_upto_degree < 0) return "bezier_continuity_upto_degree must be >= 0";
    if (p.slack_mode && p.cbf_mode == 1 && p.cbf_horizon > 2)
        return "slack_mode for the FoV controller supports cbf_horizon <= 2 (8 rows per neighbour)";
    if (p.cbf_mode != 0 && p.cbf_mode != 1) return "cbf_mode must be 0 (collision) or 1 (field of view)";
    if (p.cbf_mode == 1) {
        if (!(p.fov_beta > 0 && p.fov_beta <= 2 * M_PI + 1e-9)) return "fov must be in (0, 2 pi]";
        if (!(p.fov_Ds >= 0) || !(p.fov_Rs > 0)) return "FoV safety distance must be >= 0 and range > 0";
        if (p.continuity_upto_degree < 1) return "FoV controller needs bezier_continuity_upto_degree >= 1";
    }
    return "";
}

Operators build_operators(const mpccbf_params& p, bool keep_redundant) {
    Operators op;
    Curve cv(p);
    const int n = cv.n, K = p.k_hor, R = DIM * K;
    op.n = n;
    op.K = K;
    op.spd_f = p.spd_f;
    op.cbf_h = p.cbf_horizon;
    const double h = p.h;
    const std::vector<double> hs = h_samples(K, h);

    // ---- acceleration sampling basis U (3K x n): U_basis (PiecewiseBezierMPCQPOperations.cpp:35-60)
    Mat U(R, n);
    for (int k = 0; k < K; k++)
        for (int d = 0; d < DIM; d++) {
            std::vector<double> r = cv.row_at(hs[k], d, 2);
            for (int j = 0; j < n; j++) U(k * DIM + d, j) = r[j];
        }

    // ---- prediction: XYYaw double integrator with step h (DoubleIntegratorXYYaw.cpp:9-20).
    // x_{k+1}.pos = pos + (k+1) h vel + sum_{j<=k} h^2 (k - j + 1/2) u_j   (closed form of
    // get_A0 / get_lambda, DoubleIntegrator.cpp:9-51)
    Mat A0(R, SD), Lam(R, R);
    for (int k = 0; k < K; k++)
        for (int d = 0; d < DIM; d++) {
            A0(k * DIM + d, d) = 1.0;
            A0(k * DIM + d, DIM + d) = (k + 1) * h;
            for (int j = 0; j <= k; j++) Lam(k * DIM + d, j * DIM + d) = h * h * (k - j + 0.5);
        }
    Mat Phi = Lam * U;  // 3K x n
    std::vector<double> qw(R, 0.0);
    for (int i = DIM * (K - p.spd_f); i < R; i++) qw[i] = p.w_pos_err;

    // ---- quadratic terms. qpcpp keeps one coefficient per unordered pair and accumulates
    // every (i,j) and (j,i) entry of each cost term whose magnitude exceeds 100*eps
    // (Problem.cpp:89-117, PiecewiseBezierMPCQPGenerator.cpp:283-321,350-395); CPLEX then
    // minimises sum_{i<=j} q_ij x_i x_j (CPLEX.cpp:122-147) == x^T H x with H = sym(q).
    const double drop = std::numeric_limits<double>::epsilon() * 100.0;
    Mat q(n, n);
    auto accumulate = [&](const Mat& term, int offset) {
        for (int i = 0; i < term.r; i++)
            for (int j = 0; j < term.c; j++) {
                const double v = term(i, j);
                if (std::fabs(v) <= drop) continue;
                int a = offset + i, b = offset + j;
                if (a > b) std::swap(a, b);
                q(a, b) += v;
            }
    };
    {
        Mat Hpe(n, n);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                double s = 0;
                for (int r = 0; r < R; r++) s += Phi(r, i) * qw[r] * Phi(r, j);
                Hpe(i, j) = s;
            }
        accumulate(Hpe, 0);
    }
    // integrated squared derivative cost, d = 1..continuity, per piece
    // (BezierQPOperations.cpp:207-246): lambda * int_0^T b^(d) b^(d)^T dt, by Gauss-Legendre
    {
        static const double gx[8] = {-0.9602898564975363, -0.7966664774136267, -0.5255324099163290,
                                     -0.1834346424956498, 0.1834346424956498,  0.5255324099163290,
                                     0.7966664774136267,  0.9602898564975363};
        static const double gw[8] = {0.1012285362903763, 0.2223810344533745, 0.3137066458778873,
                                     0.3626837833783620, 0.3626837833783620, 0.3137066458778873,
                                     0.2223810344533745, 0.1012285362903763};
        const int C = cv.C;
        for (int d = 1; d <= p.continuity_upto_degree; d++) {
            if (d > C - 1) continue;
            Mat M = bernstein_derivative_monomials(C - 1, cv.T, d);
            Mat S(C, C);
            for (int g = 0; g < 8; g++) {
                const double t = 0.5 * cv.T * (gx[g] + 1.0), w = 0.5 * cv.T * gw[g];
                std::vector<double> b = eval_monomials(M, t);
                for (int i = 0; i < C; i++)
                    for (int j = 0; j < C; j++) S(i, j) += w * b[i] * b[j];
            }
            Mat blk(cv.n_piece, cv.n_piece);
            for (int dim = 0; dim < DIM; dim++)
                for (int i = 0; i < C; i++)
                    for (int j = 0; j < C; j++) blk(dim * C + i, dim * C + j) = p.w_u_eff * S(i, j);
            for (int pc = 0; pc < cv.P; pc++) accumulate(blk, pc * cv.n_piece);
        }
    }
    op.H = Mat(n, n);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            if (i == j)
                op.H(i, i) = q(i, i);
            else
                op.H(i, j) = op.H(j, i) = 0.5 * q(i, j);
        }

    // ---- linear term of the position cost: c = 2 Phi^T Q (A0 s0 - ref) (:64-90)
    Mat Cx(n, SD), Ct(n, DIM), Cr(n, DIM * p.spd_f);
    for (int j = 0; j < n; j++) {
        for (int r = 0; r < R; r++) {
            if (qw[r] == 0) continue;
            const double w = 2.0 * Phi(r, j) * qw[r];
            for (int s = 0; s < SD; s++) Cx(j, s) += w * A0(r, s);
            Ct(j, r % DIM) -= w;
            Cr(j, r - DIM * (K - p.spd_f)) -= w;
        }
    }

    // ---- equality rows: initial position and velocity on piece 0 (addEvalConstraint,
    // ConnectivityIMPCCBF.cpp:123-124) then C^d continuity, d <= continuity (:126-131)
    std::vector<std::vector<double>> eq;
    for (int d = 0; d <= 1; d++)
        for (int dim = 0; dim < DIM; dim++) eq.push_back(cv.row_at(0.0, dim, d));
    // C^d continuity: d <= degree (ConnectivityIMPCCBF.cpp:126-131), d < degree for the FoV
    // controller (FovBezierIMPCCBF.cpp:107-113)
    const int dmax = p.cbf_mode == 1 ? p.continuity_upto_degree - 1 : p.continuity_upto_degree;
    for (int pc = 0; pc + 1 < cv.P; pc++)
        for (int d = 0; d <= dmax; d++)
            for (int dim = 0; dim < DIM; dim++) {
                std::vector<double> a = cv.row_local(pc, cv.T, dim, d);
                std::vector<double> b = cv.row_local(pc + 1, 0.0, dim, d);
                for (int j = 0; j < n; j++) a[j] -= b[j];
                eq.push_back(a);
            }
    op.me = (int)eq.size();
    Mat Ae(op.me, n);
    for (int e = 0; e < op.me; e++)
        for (int j = 0; j < n; j++) Ae(e, j) = eq[e][j];
    Mat Xp;
    int rank = 0;
    auto var_dim = [&](int j) { return (j % cv.n_piece) / cv.C; };  // layout [piece][dim][cp]
    // separable? every equality row and every cost entry stays within one channel
    bool sep = true;
    std::vector<int> eq_dim(op.me, -1);
    for (int e = 0; e < op.me && sep; e++)
        for (int j = 0; j < n; j++) {
            if (Ae(e, j) == 0.0) continue;
            if (eq_dim[e] < 0) eq_dim[e] = var_dim(j);
            else if (eq_dim[e] != var_dim(j)) sep = false;
        }
    for (int i = 0; i < n && sep; i++)
        for (int j = 0; j < n; j++)
            if (op.H(i, j) != 0.0 && var_dim(i) != var_dim(j)) sep = false;
    if (sep) {
        // per-channel null spaces, assembled block-diagonally (columns [x | y | yaw])
        std::vector<Mat> Zd(DIM), Xpd(DIM);
        std::vector<std::vector<int>> vars(DIM), rows_d(DIM);
        for (int j = 0; j < n; j++) vars[var_dim(j)].push_back(j);
        for (int e = 0; e < op.me; e++) rows_d[eq_dim[e] < 0 ? 0 : eq_dim[e]].push_back(e);
        int nzd = -1;
        for (int d = 0; d < DIM && sep; d++) {
            Mat Ed((int)rows_d[d].size(), (int)vars[d].size());
            for (int a = 0; a < Ed.r; a++)
                for (int b = 0; b < Ed.c; b++) Ed(a, b) = Ae(rows_d[d][a], vars[d][b]);
            int rk = 0;
            null_space(Ed, 1e-12, Zd[d], Xpd[d], rk);
            if (nzd < 0) nzd = Zd[d].c;
            if (Zd[d].c != nzd) sep = false;  // channels must share one reduced size
            rank += rk;
        }
        if (sep) {
            op.Z = Mat(n, DIM * nzd);
            Xp = Mat(n, op.me);
            for (int d = 0; d < DIM; d++) {
                for (size_t b = 0; b < vars[d].size(); b++) {
                    for (int c = 0; c < nzd; c++) op.Z(vars[d][b], d * nzd + c) = Zd[d](b, c);
                    for (size_t a = 0; a < rows_d[d].size(); a++) Xp(vars[d][b], rows_d[d][a]) = Xpd[d](b, a);
                }
            }
            op.sep = true;
            op.nzd = nzd;
        }
    }
    if (!op.sep) null_space(Ae, 1e-12, op.Z, Xp, rank);
    // consistency: the initial-state rows must be independent of the rest (always true for
    // C >= 2); otherwise b_eq could be inconsistent for some s0.
    op.Xs = Mat(n, SD);
    for (int i = 0; i < n; i++)
        for (int s = 0; s < SD; s++) op.Xs(i, s) = Xp(i, s);
    {
        Mat chk = Ae * op.Xs;  // must be [I6; 0]
        for (int e = 0; e < op.me; e++)
            for (int s = 0; s < SD; s++)
                if (std::fabs(chk(e, s) - (e == s ? 1.0 : 0.0)) > 1e-9)
                    throw std::runtime_error("initial-state equality rows are rank deficient");
    }
    op.nz = op.Z.c;
    if (op.nz < 1) throw std::runtime_error("no free decision variables after equality constraints");

    // ---- reduced objective
    Mat Zt = op.Z.t(), Xst = op.Xs.t();
    op.Pr = 2.0 * (Zt * op.H * op.Z);
    for (int i = 0; i < op.nz; i++)  // exact symmetry
        for (int j = 0; j < i; j++) op.Pr(i, j) = op.Pr(j, i) = 0.5 * (op.Pr(i, j) + op.Pr(j, i));
    op.LPr = cholesky(op.Pr);
    op.Qs = 2.0 * (Zt * op.H * op.Xs) + Zt * Cx;
    op.Qt = Zt * Ct;
    op.Qr = Zt * Cr;
    op.Ks = Xst * op.H * op.Xs + Cx.t() * op.Xs;
    op.Kt = Ct.t() * op.Xs;
    op.Kr = Cr.t() * op.Xs;

    // ---- shared inequality rows: acceleration then velocity bounds at every h_sample
    // (addEvalBoundConstraints(2, a) / (1, v), ConnectivityIMPCCBF.cpp:196-197)
    struct Row {
        std::vector<double> g, gs;  // reduced (nz) and state (6) parts
        double lo, hi;
        int kind, dim;
        bool constant;
    };
    std::vector<Row> rows;
    for (int kind = 0; kind < 2; kind++) {
        const int deriv = kind == 0 ? 2 : 1;
        const double* lb = kind == 0 ? p.a_min : p.v_min;
        const double* ub = kind == 0 ? p.a_max : p.v_max;
        for (int k = 0; k < K; k++)
            for (int dim = 0; dim < DIM; dim++) {
                std::vector<double> r = cv.row_at(hs[k], dim, deriv);
                Mat rm = row_to_mat(r);
                Mat g = rm * op.Z, gs = rm * op.Xs;
                double gmax = 0, rmax = 0;
                for (double v : g.a) gmax = std::max(gmax, std::fabs(v));
                for (double v : r) rmax = std::max(rmax, std::fabs(v));
                rows.push_back({g.a, gs.a, lb[dim], ub[dim], kind, dim, gmax <= 1e-12 * std::max(rmax, 1.0)});
            }
    }
    op.rows_total = (int)rows.size();
    // Exact redundancy: a row that is a convex combination (in the joint (s0, y) space) of two
    // KEPT rows with the same bounds is implied by them for every state. Transitive, so removing
    // such rows one at a time never changes the feasible set (e.g. the acceleration of a cubic
    // is affine in t, so only the end samples of each dimension remain).
    std::vector<bool> keep(rows.size(), true);
    if (!keep_redundant) {
        for (size_t i = 0; i < rows.size(); i++) {
            if (rows[i].constant) continue;
            bool removed = false;
            for (size_t j = 0; j < rows.size() && !removed; j++) {
                if (j == i || !keep[j] || rows[j].constant) continue;
                if (rows[j].lo != rows[i].lo || rows[j].hi != rows[i].hi) continue;
                for (size_t k = j + 1; k < rows.size() && !removed; k++) {
                    if (k == i || !keep[k] || rows[k].constant) continue;
                    if (rows[k].lo != rows[i].lo || rows[k].hi != rows[i].hi) continue;
                    // solve for lambda: r_i ~ lambda r_j + (1 - lambda) r_k
                    std::vector<double> ri, rj, rk;
                    for (auto* v : {&rows[i].g, &rows[i].gs}) ri.insert(ri.end(), v->begin(), v->end());
                    for (auto* v : {&rows[j].g, &rows[j].gs}) rj.insert(rj.end(), v->begin(), v->end());
                    for (auto* v : {&rows[k].g, &rows[k].gs}) rk.insert(rk.end(), v->begin(), v->end());
                    std::vector<double> dj(rj.size()), di(ri.size());
                    for (size_t t = 0; t < rj.size(); t++) {
                        dj[t] = rj[t] - rk[t];
                        di[t] = ri[t] - rk[t];
                    }
                    const double den = dotv(dj, dj);
                    if (den <= 0) continue;
                    const double lam = dotv(di, dj) / den;
                    if (lam < -1e-12 || lam > 1 + 1e-12) continue;
                    double res = 0, scale = 0;
                    for (size_t t = 0; t < ri.size(); t++) {
                        res = std::max(res, std::fabs(di[t] - lam * dj[t]));
                        scale = std::max(scale, std::fabs(ri[t]));
                    }
                    if (res <= 1e-12 * std::max(scale, 1.0)) {
                        keep[i] = false;
                        removed = true;
                    }
                }
            }
        }
    }
    int m = 0, mc = 0;
    for (size_t i = 0; i < rows.size(); i++) {
        if (rows[i].constant)
            mc++;
        else if (keep[i])
            m++;
    }
    op.rows_removed = op.rows_total - m - mc;
    op.G = Mat(m, op.nz);
    op.Gs = Mat(m, SD);
    op.Cs = Mat(mc, SD);
    int im = 0, ic = 0;
    for (size_t i = 0; i < rows.size(); i++) {
        const Row& r = rows[i];
        if (r.constant) {
            for (int s = 0; s < SD; s++) op.Cs(ic, s) = r.gs[s];
            op.clo.push_back(r.lo);
            op.chi.push_back(r.hi);
            ic++;
        } else if (keep[i]) {
            for (int j = 0; j < op.nz; j++) op.G(im, j) = r.g[j];
            for (int s = 0; s < SD; s++) op.Gs(im, s) = r.gs[s];
            op.lo.push_back(r.lo);
            op.hi.push_back(r.hi);
            op.row_kind.push_back(r.kind);
            op.row_dim.push_back(r.dim);
            im++;
        }
    }

    // ---- CBF operators: acceleration basis rows at sample k (U_basis rows 3k..3k+2,
    // ConnectivityMPCCBFQPOperations.cpp:200-202, :265-267)
    for (int k = 0; k < p.cbf_horizon; k++) {
        Mat Uk = U.rows(k * DIM, DIM);
        op.UZ.push_back(Uk * op.Z);
        op.US.push_back(Uk * op.Xs);
        // predicted ego state at h_samples(k) from the previous curve (ConnectivityIMPCCBF.cpp:161-168)
        Mat E(SD, n);
        for (int d = 0; d <= 1; d++)
            for (int dim = 0; dim < DIM; dim++) {
                std::vector<double> r = cv.row_at(hs[k], dim, d);
                for (int j = 0; j < n; j++) E(d * DIM + dim, j) = r[j];
            }
        op.PZ.push_back(E * op.Z);
        op.PS.push_back(E * op.Xs);
    }
    {
        // closed-loop update: the kept curve evaluated at t = h (example :188-207)
        Mat E(SD, n);
        for (int d = 0; d <= 1; d++)
            for (int dim = 0; dim < DIM; dim++) {
                std::vector<double> r = cv.row_at(std::min(h, cv.cum.back()), dim, d);
                for (int j = 0; j < n; j++) E(d * DIM + dim, j) = r[j];
            }
        op.AZ = E * op.Z;
        op.AS = E * op.Xs;
    }
    op.EB0 = bernstein_derivative_monomials(cv.C - 1, cv.T, 0);
    op.EB1 = bernstein_derivative_monomials(cv.C - 1, cv.T, 1);
    op.cum = cv.cum;
    op.eval_step = p.Ts * (double)(int)(p.h / p.Ts);  // example :188-190, last sub-step
    if (p.cbf_mode == 1) {
        for (int j = 0; j < cv.C; j++) {
            Mat E(2, n);
            for (int d = 0; d < 2; d++) E(d, 0 * cv.n_piece + d * cv.C + j) = 1.0;
            op.VZ.push_back(E * op.Z);
            op.VS.push_back(E * op.Xs);
        }
    }
    for (int d = 0; d < DIM; d++) {
        op.a_lo[d] = p.a_min[d];
        op.a_hi[d] = p.a_max[d];
    }
    return op;
}

}  // namespace mpccbf
