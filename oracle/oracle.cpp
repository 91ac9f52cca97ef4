// oracle.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h header for scope and pinning).
//
// CPU restatement of the reference MPC-CBF QP hot path. Every function cites the reference
// file:line it restates (paths relative to /root/reference/workspace/lib). Nothing here is
// shipped or called by the product; the product (mpc-cbf_amd/) has its own, independent host
// precompute and a GPU solver, and this file is the checker they are compared against.

#include "oracle.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <stdexcept>
#include <thread>
#include <vector>

namespace orc {

constexpr int DIM = 3;
constexpr double INF = std::numeric_limits<double>::max();
constexpr double LOWEST = std::numeric_limits<double>::lowest();

static inline bool is_neg_inf(double v) { return v <= -1e300; }
static inline bool is_pos_inf(double v) { return v >= 1e300; }

// ---------------------------------------------------------------- math/src/Combinatorics.cpp
uint64_t fac(uint64_t n) {  // :10-19
    if (n > 20) throw std::runtime_error("fac overflow");
    uint64_t r = 1;
    for (uint64_t i = 2; i <= n; i++) r *= i;
    return r;
}
uint64_t comb(uint64_t n, uint64_t k) {  // :21-31
    if (k > n) return 0;
    k = std::min(k, n - k);
    uint64_t top = 1, bottom = 1;
    for (uint64_t i = 0; i < k; i++) {
        bottom *= (i + 1);
        top *= (n - i);
    }
    return top / bottom;
}
uint64_t perm(uint64_t n, uint64_t k) {  // :33-40
    if (k > n) return 0;
    uint64_t r = 1;
    for (uint64_t i = n - k + 1; i <= n; ++i) r *= i;
    return r;
}
template <typename U>
double mpow(double base, U exp) {  // :42-51
    if (base == 0 && exp == 0) return 1;
    return std::pow(base, exp);
}

// -------------------------------------------------- splines/src/detail/BezierOperations.cpp
// bernsteinBasis :11-50
std::vector<double> bernsteinBasis(uint64_t deg, double maxp, double t, uint64_t d) {
    if (t < 0 || t > maxp) throw std::runtime_error("bernsteinBasis: parameter outside range");
    std::vector<double> res(deg + 1, 0.0);
    if (maxp == 0) {
        if (d == 0) res[0] = 1.0;
        return res;
    }
    const double oneOverA = 1.0 / maxp;
    for (uint64_t i = 0; i <= deg; i++) {
        double base = 0.0, mult = 1.0;
        for (uint64_t j = 0; j + d <= deg; j++, mult *= t) {
            if (j + d >= i) {
                const uint64_t cr = comb(deg - i, j + d - i);
                const uint64_t pr = perm(j + d, d);
                const double pw = mpow(oneOverA, j + d);
                base += (cr) * (pw) * (pr)*mult * ((j + d - i) % 2 == 0 ? 1 : -1);
            }
        }
        base *= comb(deg, i);
        res[i] = base;
    }
    return res;
}

// bernsteinCoefficientMatrix :54-121 (returned row-major (deg+1)x(deg+1))
std::vector<double> bernsteinCoefficientMatrix(uint64_t deg, double maxp, uint64_t d) {
    const int N = (int)deg + 1;
    std::vector<double> bm(N * N, 0.0), der(N * N, 0.0), out(N * N, 0.0);
    if (maxp == 0) {
        if (d == 0) out[0] = 1.0;
        return out;
    }
    uint64_t dcombi = 1;
    const double oneOverA = 1.0 / maxp;
    for (uint64_t i = 0; i < deg + 1; ++i) {
        uint64_t dmc = 1;
        double min1 = 1;
        double pw = mpow<uint64_t>(oneOverA, i);
        for (uint64_t j = i; j < deg + 1; ++j, min1 *= -1, pw *= oneOverA) {
            bm[i * N + j] = dcombi * dmc * min1 * pw;
            dmc *= (deg - j);
            dmc /= (j + 1 - i);
        }
        dcombi *= (deg - i);
        dcombi /= (i + 1);
    }
    uint64_t jpermk = fac(d);
    for (uint64_t j = d; j < deg + 1; ++j) {
        der[j * N + (j - d)] = (double)jpermk;
        jpermk *= (j + 1);
        jpermk /= (j + 1 - d);
    }
    for (int i = 0; i < N; i++)
        for (int k = 0; k < N; k++) {
            double s = 0;
            for (int j = 0; j < N; j++) s += bm[i * N + j] * der[j * N + k];
            out[i * N + k] = s;
        }
    return out;
}

// ------------------------------------------- model/src/DoubleIntegratorXYYaw.cpp:9-20 (A, B)
struct Model {
    double A[6][6];
    double B[6][3];
    explicit Model(double ts) {
        std::memset(A, 0, sizeof(A));
        std::memset(B, 0, sizeof(B));
        for (int i = 0; i < 6; i++) A[i][i] = 1;
        for (int i = 0; i < 3; i++) {
            A[i][i + 3] = ts;
            B[i][i] = 0.5 * std::pow(ts, 2.0);
            B[i + 3][i] = ts;
        }
    }
};

// get_A0 (model/src/DoubleIntegrator.cpp:9-27) -> pos rows (3K x 6)
std::vector<double> getA0pos(const Model& m, int K) {
    std::vector<double> out(3 * K * 6, 0.0);
    double prev[6][6], nw[6][6];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) prev[i][j] = (i == j);
    for (int k = 0; k < K; ++k) {
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) {
                double s = 0;
                for (int l = 0; l < 6; l++) s += m.A[i][l] * prev[l][j];
                nw[i][j] = s;
            }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 6; j++) out[(3 * k + i) * 6 + j] = nw[i][j];
        std::memcpy(prev, nw, sizeof(prev));
    }
    return out;
}

// get_lambda (model/src/DoubleIntegrator.cpp:30-51) -> pos rows (3K x 3K)
std::vector<double> getLambdaPos(const Model& m, int K) {
    const int C = 3 * K;
    std::vector<double> out(C * C, 0.0), prev(6 * C, 0.0), nw(6 * C, 0.0);
    for (int k = 0; k < K; ++k) {
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < C; j++) {
                double s = 0;
                for (int l = 0; l < 6; l++) s += m.A[i][l] * prev[l * C + j];
                int blk = j / 3;
                double addb = (blk == k) ? m.B[i][j % 3] : 0.0;
                nw[i * C + j] = s + addb;
            }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < C; j++) out[(3 * k + i) * C + j] = nw[i * C + j];
        prev = nw;
    }
    return out;
}

// Eigen::VectorXd::LinSpaced(size, low, high) (Eigen 3.4 linspaced_op_impl, non-integer path)
std::vector<double> linSpaced(int size, double low, double high) {
    std::vector<double> v(size);
    if (size == 1) {
        v[0] = high;
        return v;
    }
    const double step = (high - low) / double(size - 1);
    const bool flip = std::fabs(high) < std::fabs(low);
    const int size1 = size - 1;
    for (int i = 0; i < size; i++) {
        if (flip)
            v[i] = (i == 0) ? low : (high - double(size1 - i) * step);
        else
            v[i] = (i == size1) ? high : (low + double(i) * step);
    }
    return v;
}

// ---------------------------------------------------------------- problem-layout helpers
struct Layout {
    int P, C, K, cont, n_curve, n_piece;
    double T;
    std::vector<double> cum;  // cumulative max parameters (PiecewiseBezierMPCQPOperations::addPiece :159-171)
    explicit Layout(const orc_params* p) {
        P = p->num_pieces;
        C = p->num_control_points;
        K = p->k_hor;
        cont = p->continuity_upto_degree;
        T = p->piece_max_parameter;
        n_piece = DIM * C;
        n_curve = P * n_piece;
        for (int i = 0; i < P; i++) cum.push_back(i == 0 ? T : cum.back() + T);
    }
    // getPieceIndexAndParameter (mpc/src/optimization/PiecewiseBezierMPCQPOperations.cpp:190-223)
    void pieceIndexAndParameter(double t, int* idx, double* par) const {
        if (t < 0 || t > cum.back()) throw std::runtime_error("parameter out of range");
        int i = int(std::lower_bound(cum.begin(), cum.end(), t) - cum.begin());
        if (i >= P) throw std::runtime_error("piece_idx out of range");
        *idx = i;
        if (i == 0)
            *par = std::clamp(t, 0.0, T);
        else
            *par = std::clamp(t - cum[i - 1], 0.0, T);
    }
    // BezierQPOperations::evalBasisRow (splines/src/optimization/BezierQPOperations.cpp:186-204),
    // placed at the piece's variable block (PiecewiseBezierMPCQPOperations.cpp:50-56)
    void evalBasisRowFull(int piece, int dim, double t, int d, double* row) const {
        std::fill(row, row + n_curve, 0.0);
        if (C == 0) return;
        std::vector<double> b = bernsteinBasis(C - 1, T, t, d);
        for (int i = 0; i < C; i++) row[piece * n_piece + dim * C + i] = b[i];
    }
};

// PiecewiseBezierMPCQPOperations::evalSamplingBasisMatrix (:42-60) -> (3*hor) x n_curve
std::vector<double> samplingBasis(const Layout& L, const std::vector<double>& ts, int deriv) {
    const int hor = (int)ts.size();
    std::vector<double> U(DIM * hor * L.n_curve, 0.0);
    for (int k = 0; k < hor; k++) {
        int pi;
        double par;
        L.pieceIndexAndParameter(ts[k], &pi, &par);
        for (int d = 0; d < DIM; d++) L.evalBasisRowFull(pi, d, par, deriv, &U[(k * DIM + d) * L.n_curve]);
    }
    return U;
}

// --------------------------------------------------------------------- the dense QP record
struct DenseQP {
    int n = 0;
    std::vector<double> H, c;  // objective x^T H x + c^T x + c0 (H symmetric)
    double c0 = 0;
    int m = 0;
    std::vector<double> A, lo, hi;
    std::vector<double> vlo, vhi;
};

// qpcpp::CostFunction::addQuadraticTerm (qpcpp/src/Problem.cpp:89-117) stores ONE coefficient per
// unordered pair (i<=j, accumulated with +=); CPLEX then minimises sum_{i<=j} q_ij x_i x_j
// (CPLEX.cpp:125-142). We keep the canonical upper-triangular q and expand to symmetric H at the end.
struct CostAccum {
    int n;
    std::vector<double> q;    // n x n upper triangle used
    std::vector<double> lin;  // n
    double cst = 0;
    explicit CostAccum(int n_) : n(n_), q(n_ * n_, 0.0), lin(n_, 0.0) {}
    // isApproximatelyEqual(v, 0, 100*eps) drop (math/src/Helpers.cpp:74-80;
    // PiecewiseBezierMPCQPGenerator.cpp:285,307,314)
    static bool keep(double v) { return !(std::fabs(v - 0.0) <= std::numeric_limits<double>::epsilon() * 100.0); }
    void addQuad(int i, int j, double v) {
        if (i > j) std::swap(i, j);
        q[i * n + j] += v;
    }
    // addCostAdditionForPiecewise (:283-321) / ForPiece (:350-395) with a variable index map
    void addCostAddition(const std::vector<int>& vars, const double* quad, const double* linear,
                         double constant) {
        const int nv = (int)vars.size();
        if (constant != 0) cst += constant;
        for (int i = 0; i < nv; i++) {
            if (keep(linear[i])) lin[vars[i]] += linear[i];
            for (int j = 0; j < nv; j++)
                if (keep(quad[i * nv + j])) addQuad(vars[i], vars[j], quad[i * nv + j]);
        }
    }
};

// ---------------------------------------------------------------- FoV CBF rows (closed form)
// FovCBF::initSafetyCBF / initBorder1CBF / initBorder2CBF / initRangeCBF
// (cbf/src/detail/FovCBF.cpp:152-535) evaluated symbolically by hand. With d = target - p,
// rel = R(th) d = (c dx + s dy, -s dx + c dy), f = (vx, vy, w, 0, 0, 0), g = [0; I]:
//   every barrier is b(px, py, th), Ac = LgLf b = (b_px, b_py, b_th), Lf b = Ac . v,
//   Lf^2 b = v^T Hess(b) v, Bc = Lf^2 b + alpha'(b) Lf b + alpha(Lf b + alpha(b)),
//   alpha(x) = gamma x^5 (fifthAlpha, :23-29), gamma = 0.1 (:58).
// The border barriers are b = kap rel_x + sig rel_y with (kap, sig) per the fov branch of
// :211-231 (fov < pi: (tan(fov/2), +1) left, (tan(fov/2), -1) right; fov == pi: (1, 0);
// pi < fov < 2 pi: (tan((2 pi - fov)/2), -1) left, (.., +1) right — GiNaC's `py >= 0` on a symbol
// is false; fov == 2 pi: vacuous row).
struct FovRow {
    double a[3], b;
    bool present;
};

static void fov_rows(const double* st, const double* tg, double fov, double Ds, double Rs, FovRow out[4]) {
    const double gamma = 0.1;
    const double px = st[0], py = st[1], th = st[2], vx = st[3], vy = st[4], w = st[5];
    const double dx = tg[0] - px, dy = tg[1] - py;
    const double c = std::cos(th), s = std::sin(th);
    const double rx = c * dx + s * dy, ry = -s * dx + c * dy;
    auto finish = [&](FovRow& r, double bval, double lf2) {
        const double lf = r.a[0] * vx + r.a[1] * vy + r.a[2] * w;
        const double alpha_b = gamma * std::pow(bval, 5);
        const double lf_alpha = 5.0 * gamma * std::pow(bval, 4) * lf;
        r.b = lf2 + lf_alpha + gamma * std::pow(lf + alpha_b, 5);
        r.present = true;
    };
    // safety: b = |rel|^2 - Ds^2 = dx^2 + dy^2 - Ds^2 (rotation invariant)
    {
        FovRow& r = out[0];
        r.a[0] = -2 * dx;
        r.a[1] = -2 * dy;
        r.a[2] = 0.0;
        finish(r, dx * dx + dy * dy - Ds * Ds, 2 * (vx * vx + vy * vy));
    }
    // borders
    auto border = [&](FovRow& r, double kap, double sig) {
        const double bval = kap * rx + sig * ry;
        r.a[0] = -kap * c + sig * s;
        r.a[1] = -kap * s - sig * c;
        r.a[2] = kap * ry - sig * rx;
        const double lf2 = 2 * w * ((kap * s + sig * c) * vx + (-kap * c + sig * s) * vy) - w * w * bval;
        finish(r, bval, lf2);
    };
    const bool full = std::fabs(fov - 2 * M_PI) <= 1e-9 * std::max(1.0, 2 * M_PI);  // isApproximatelyEqual
    if (fov < M_PI) {
        border(out[1], std::tan(fov / 2), +1.0);
        border(out[2], std::tan(fov / 2), -1.0);
    } else if (fov == M_PI) {
        border(out[1], 1.0, 0.0);
        border(out[2], 1.0, 0.0);
    } else if (full) {
        for (int k : {1, 2}) {
            out[k].a[0] = out[k].a[1] = out[k].a[2] = 0.0;
            out[k].b = std::numeric_limits<double>::max();
            out[k].present = false;
        }
    } else {
        const double t2 = std::tan((2 * M_PI - fov) / 2);
        border(out[1], t2, -1.0);
        border(out[2], t2, +1.0);
    }
    // range: b = Rs^2 - |rel|^2
    {
        FovRow& r = out[3];
        r.a[0] = 2 * dx;
        r.a[1] = 2 * dy;
        r.a[2] = 0.0;
        finish(r, Rs * Rs - dx * dx - dy * dy, -2 * (vx * vx + vy * vy));
    }
}

// separating_hyperplanes::voronoi (separating_hyperplanes/src/Voronoi.cpp:10-29) of the planar
// positions (last dimension zeroed, FovBezierIMPCCBF.cpp:135-141), shifted by the robot box
// (math::shiftHyperplane, math/src/Helpers.cpp:20-36): n . x + off <= 0 with off the max over
// the box corners. Returns the 3-vector normal and the shifted offset.
static void voronoi_shifted(const double* self_xy, const double* other_xy, const double* bbox,
                            double n[3], double* off) {
    double d0 = other_xy[0] - self_xy[0], d1 = other_xy[1] - self_xy[1];
    const double nrm = std::sqrt(d0 * d0 + d1 * d1);
    if (nrm > 0) {  // Eigen normalize(): no-op on a zero vector
        d0 /= nrm;
        d1 /= nrm;
    }
    n[0] = d0;
    n[1] = d1;
    n[2] = 0.0;
    const double mid0 = 0.5 * (self_xy[0] + other_xy[0]), mid1 = 0.5 * (self_xy[1] + other_xy[1]);
    const double offset = -(n[0] * mid0 + n[1] * mid1);
    double best = std::numeric_limits<double>::lowest();
    for (int corner = 0; corner < 8; corner++) {
        double v = offset;
        for (int d = 0; d < 3; d++) v += n[d] * ((corner & (1 << d)) ? -bbox[d] : bbox[d]);
        best = std::max(best, v);
    }
    *off = best;
}

struct Assembler {
    const orc_params* p;
    Layout L;
    Model model;
    std::vector<double> A0pos, Lpos, hs, U, Phi;
    int nvar_total;  // curve + slack
    int nslack;

    Assembler(const orc_params* p_, int num_neighbors)
        : p(p_), L(p_), model(p_->h) {
        const int K = L.K;
        // PiecewiseBezierMPCQPOperations ctor (:9-38)
        A0pos = getA0pos(model, K);
        Lpos = getLambdaPos(model, K);
        hs = linSpaced(K, 0, (K - 1) * p->h);
        U = samplingBasis(L, hs, 2);
        // Phi = Lambda.pos * U_basis (:81)
        const int R = DIM * K, n = L.n_curve;
        Phi.assign(R * n, 0.0);
        for (int i = 0; i < R; i++)
            for (int k = 0; k < R; k++) {
                double a = Lpos[i * R + k];
                if (a == 0) continue;
                for (int j = 0; j < n; j++) Phi[i * n + j] += a * U[k * n + j];
            }
        nslack = p->slack_mode ? num_neighbors : 0;
        nvar_total = L.n_curve + nslack;
    }

    // positionErrorPenaltyCost (PiecewiseBezierMPCQPOperations.cpp:64-90)
    void positionErrorCost(const double* x0, const double* ref, std::vector<double>& quad,
                           std::vector<double>& lin) const {
        const int K = L.K, R = DIM * K, n = L.n_curve, spd = p->spd_f;
        std::vector<double> qdiag(R, 0.0);
        for (int i = DIM * (K - spd); i < R; i++) qdiag[i] = p->w_pos_err;
        quad.assign(n * n, 0.0);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                double s = 0;
                for (int r = 0; r < R; r++) s += Phi[r * n + i] * qdiag[r] * Phi[r * n + j];
                quad[i * n + j] = s;
            }
        // linear_term_coef = 2 (A0 x0)^T Q - 2 ref^T Q ; linear = (coef * Phi)^T
        std::vector<double> coef(R);
        for (int r = 0; r < R; r++) {
            double ax = 0;
            for (int j = 0; j < 6; j++) ax += A0pos[r * 6 + j] * x0[j];
            coef[r] = 2.0 * ax * qdiag[r];
            coef[r] += -2.0 * ref[r] * qdiag[r];
        }
        lin.assign(n, 0.0);
        for (int j = 0; j < n; j++) {
            double s = 0;
            for (int r = 0; r < R; r++) s += coef[r] * Phi[r * n + j];
            lin[j] = s;
        }
    }

    // BezierQPOperations::integratedSquaredDerivativeCost (BezierQPOperations.cpp:207-246)
    std::vector<double> integratedSquaredDerivativeCost(int d, double lambda) const {
        const int C = L.C, nv = L.n_piece;
        std::vector<double> quad(nv * nv, 0.0);
        if (C == 0) return quad;
        if (d <= C - 1) {
            std::vector<double> B = bernsteinCoefficientMatrix(C - 1, L.T, d);
            std::vector<double> SQI(C * C), tmp(C * C, 0.0), cost(C * C, 0.0);
            for (int i = 0; i < C; i++)
                for (int j = 0; j < C; j++) SQI[i * C + j] = mpow(L.T, (uint64_t)(i + j + 1)) / (i + j + 1);
            for (int i = 0; i < C; i++)
                for (int j = 0; j < C; j++) {
                    double s = 0;
                    for (int k = 0; k < C; k++) s += B[i * C + k] * SQI[k * C + j];
                    tmp[i * C + j] = s;
                }
            for (int i = 0; i < C; i++)
                for (int j = 0; j < C; j++) {
                    double s = 0;
                    for (int k = 0; k < C; k++) s += tmp[i * C + k] * B[j * C + k];
                    cost[i * C + j] = lambda * s;
                }
            for (int dim = 0; dim < DIM; dim++)
                for (int i = 0; i < C; i++)
                    for (int j = 0; j < C; j++) quad[(dim * C + i) * nv + dim * C + j] = cost[i * C + j];
        }
        return quad;
    }

    void addRow(DenseQP& qp, const std::vector<double>& row, double lo, double hi) const {
        qp.A.insert(qp.A.end(), row.begin(), row.end());
        qp.lo.push_back(lo);
        qp.hi.push_back(hi);
        qp.m++;
    }

    // The whole per-iteration assembly of ConnectivityIMPCCBF::optimize (ConnectivityIMPCCBF.cpp:102-197).
    DenseQP build(const double* st, const double* ref, int nb, const double* nbs,
                  const double* slack_w, int iter, const double* pred) const {
        const int n = nvar_total, nc = L.n_curve, K = L.K;
        DenseQP qp;
        qp.n = n;
        CostAccum acc(n);
        std::vector<int> curve_vars(nc), slack_vars(nslack);
        std::iota(curve_vars.begin(), curve_vars.end(), 0);
        std::iota(slack_vars.begin(), slack_vars.end(), nc);
        // addPositionErrorPenaltyCost (:108) -> PiecewiseBezierMPCQPGenerator.cpp:102-107
        {
            std::vector<double> quad, lin;
            positionErrorCost(st, ref, quad, lin);
            acc.addCostAddition(curve_vars, quad.data(), lin.data(), 0);
        }
        // addIntegratedSquaredDerivativeCost d = 1..continuity (:112-115) -> Generator :135-146
        for (int d = 1; d <= L.cont; d++) {
            std::vector<double> quad = integratedSquaredDerivativeCost(d, p->w_u_eff);
            std::vector<double> zero(L.n_piece, 0.0);
            for (int pc = 0; pc < L.P; pc++) {
                std::vector<int> vars(L.n_piece);
                for (int i = 0; i < L.n_piece; i++) vars[i] = pc * L.n_piece + i;
                acc.addCostAddition(vars, quad.data(), zero.data(), 0);
            }
        }
        // addSlackCost (MPCCBFQPGeneratorBase.cpp:121-130): plain addLinearTerm, no drop
        if (nslack > 0)
            for (int i = 0; i < nslack; i++) acc.lin[slack_vars[i]] += slack_w[i];

        std::vector<double> row(n, 0.0);
        auto zero_row = [&]() { std::fill(row.begin(), row.end(), 0.0); };
        // addEvalConstraint(0, 0, pos), (0, 1, vel) (:123-124) -> BezierQPOperations.cpp:283-301
        for (int d = 0; d <= 1; d++) {
            int pi;
            double par;
            L.pieceIndexAndParameter(0.0, &pi, &par);
            std::vector<double> b = bernsteinBasis(L.C - 1, L.T, par, d);
            for (int dim = 0; dim < DIM; dim++) {
                zero_row();
                for (int i = 0; i < L.C; i++) row[pi * L.n_piece + dim * L.C + i] = b[i];
                double target = st[d * 3 + dim];
                addRow(qp, row, target, target);
            }
        }
        // addContinuityConstraint(p, d): d <= continuity for ConnectivityIMPCCBF (:126-131),
        // d < continuity for FovBezierIMPCCBF (FovBezierIMPCCBF.cpp:107-113) -> Generator :182-226
        const int dmax = p->cbf_mode == 1 ? L.cont - 1 : L.cont;
        for (int pc = 0; pc + 1 < L.P; pc++)
            for (int d = 0; d <= dmax; d++) {
                std::vector<double> b1 = bernsteinBasis(L.C - 1, L.T, L.T, d);
                std::vector<double> b2 = bernsteinBasis(L.C - 1, L.T, 0.0, d);
                for (int dim = 0; dim < DIM; dim++) {
                    zero_row();
                    for (int i = 0; i < L.C; i++) {
                        row[pc * L.n_piece + dim * L.C + i] = b1[i];
                        row[(pc + 1) * L.n_piece + dim * L.C + i] = -b2[i];
                    }
                    addRow(qp, row, 0.0, 0.0);
                }
            }
        // CBF rows (:135-193)
        const double gamma = 5.0;
        (void)gamma;
        auto cbf_row = [&](const double* ego, const double* nbst, int k, int nbi) {
            double a[3], b;
            orc_safety_cbf(ego, nbst, p->d_min, a, &b);
            // ConnectivityMPCCBFQPOperations.cpp:192-205 (k=0) / :252-272 (pred k)
            zero_row();
            for (int j = 0; j < nc; j++) {
                double s = 0;
                for (int d = 0; d < DIM; d++) s += a[d] * U[(k * DIM + d) * nc + j];
                row[j] = -1.0 * s;
            }
            if (nslack > 0) {
                // slack mode: a row that every acceleration of the box at sample k satisfies with
                // v_i = 0 (b >= max over the box of -a^T u) holds for every v_i >= 0 too, and the
                // box rows of sample k (addEvalBoundConstraints(2, ...), below) are in every QP —
                // dropping it leaves the feasible set and the optimum unchanged (the kernel's
                // filter, impc_kernel.hip lane_cbf_rows). Kept, a distant neighbour's row has a
                // bound ~1e26 next to a slack weight down to ~1e-9, and the dense PDIP stalls on
                // its dual residual (round 3: two all-neighbour slack QPs UNKNOWN).
                double bmax = 0.0;
                for (int d = 0; d < DIM; d++) bmax += std::max(-a[d] * p->a_min[d], -a[d] * p->a_max[d]);
                if (b >= bmax) return;
                row[nc + nbi] = -1.0;  // ConnectivityMPCCBFQPGenerator.cpp:33-40
            }
            addRow(qp, row, LOWEST, b + 0.0);     // slack_value = 0 (:138, :172)
        };
        if (p->cbf_mode == 1) {
            // Voronoi rows on every control point of piece 0 (FovBezierIMPCCBF.cpp:130-147 ->
            // BezierQPOperations::hyperplaneConstraintAll :270-285, epsilon 1e-8)
            for (int i = 0; i < nb; i++) {
                double nrm[3], off;
                voronoi_shifted(st, nbs + 6 * i, p->bbox, nrm, &off);
                for (int cp = 0; cp < L.C; cp++) {
                    zero_row();
                    for (int d = 0; d < DIM; d++) row[0 * L.n_piece + d * L.C + cp] = nrm[d];
                    addRow(qp, row, LOWEST, -off - 1e-8);
                }
            }
            // FoV CBF rows: iter 0 at the current state (:150-171), later iterations at the
            // predicted states, per neighbour all k of one kind, then the next kind (:172-210)
            // slack mode: every FoV row of neighbour i carries -1 on slack variable i
            // (FovMPCCBFQPGenerator.cpp:110-207 *WithSlackVariables, slack_coefficients(i) = -1);
            // the Voronoi rows above never do
            auto fov_row = [&](const FovRow& fr, int k, int nbi) {
                zero_row();
                for (int j = 0; j < nc; j++) {
                    double sum = 0;
                    for (int d = 0; d < DIM; d++) sum += fr.a[d] * U[(k * DIM + d) * nc + j];
                    row[j] = -1.0 * sum;
                }
                if (nslack > 0) row[nc + nbi] = -1.0;
                addRow(qp, row, LOWEST, fr.b + 0.0);
            };
            for (int i = 0; i < nb; i++) {
                const double* tg = nbs + 6 * i;  // target = neighbour position (x, y)
                if (iter == 0) {
                    FovRow fr[4];
                    fov_rows(st, tg, p->fov_beta, p->fov_Ds, p->fov_Rs, fr);
                    for (int r = 0; r < 4; r++) fov_row(fr[r], 0, i);
                } else {
                    std::vector<std::array<FovRow, 4>> per_k(p->cbf_horizon);
                    for (int k = 0; k < p->cbf_horizon; k++)
                        fov_rows(pred + 6 * k, tg, p->fov_beta, p->fov_Ds, p->fov_Rs, per_k[k].data());
                    for (int r = 0; r < 4; r++)
                        for (int k = 0; k < p->cbf_horizon; k++) fov_row(per_k[k][r], k, i);
                }
            }
        } else if (iter == 0) {
            for (int i = 0; i < nb; i++) cbf_row(st, nbs + 6 * i, 0, i);
        } else {
            for (int i = 0; i < nb; i++)
                for (int k = 0; k < p->cbf_horizon; k++) cbf_row(pred + 6 * k, nbs + 6 * i, k, i);
        }
        // addEvalBoundConstraints(2, a) then (1, v) (:196-197) -> Generator :148-164
        for (int deriv : {2, 1}) {
            const double* lb = deriv == 2 ? p->a_min : p->v_min;
            const double* ub = deriv == 2 ? p->a_max : p->v_max;
            for (int k = 0; k < K; k++) {
                int pi;
                double par;
                L.pieceIndexAndParameter(hs[k], &pi, &par);
                std::vector<double> b = bernsteinBasis(L.C - 1, L.T, par, deriv);
                for (int dim = 0; dim < DIM; dim++) {
                    zero_row();
                    for (int i = 0; i < L.C; i++) row[pi * L.n_piece + dim * L.C + i] = b[i];
                    addRow(qp, row, lb[dim], ub[dim]);
                }
            }
        }
        // variable bounds: curve vars free (addVariable() defaults, Problem.h:366-367),
        // slack vars [0, max) (MPCCBFQPGeneratorBase.cpp:386-389)
        qp.vlo.assign(n, LOWEST);
        qp.vhi.assign(n, INF);
        for (int i = 0; i < nslack; i++) qp.vlo[nc + i] = 0.0;
        // expand canonical q into symmetric H: sum_{i<=j} q_ij x_i x_j = x^T H x
        qp.H.assign(n * n, 0.0);
        for (int i = 0; i < n; i++)
            for (int j = i; j < n; j++) {
                double v = acc.q[i * n + j];
                if (i == j)
                    qp.H[i * n + i] = v;
                else {
                    qp.H[i * n + j] = 0.5 * v;
                    qp.H[j * n + i] = 0.5 * v;
                }
            }
        qp.c = acc.lin;
        qp.c0 = acc.cst;
        return qp;
    }

    // SingleParameterPiecewiseCurve::eval (splines/src/curves/SingleParameterPiecewiseCurve.cpp:94-127)
    // over the curve generated by BezierQPOperations::generateCurveFromSolution (:155-178)
    void evalCurve(const double* x, double t, int d, double* out) const {
        if (t < 0 || t > L.cum.back()) throw std::runtime_error("eval: parameter out of range");
        int i = int(std::lower_bound(L.cum.begin(), L.cum.end(), t) - L.cum.begin());
        double par = (i == 0) ? t : std::min(L.T, t - L.cum[i - 1]);
        std::vector<double> b = bernsteinBasis(L.C - 1, L.T, par, d);  // Bezier::eval (Bezier.cpp:61-75)
        for (int dim = 0; dim < DIM; dim++) {
            double s = 0;
            for (int cp = 0; cp < L.C; cp++) s += x[i * L.n_piece + dim * L.C + cp] * b[cp];
            out[dim] = s;
        }
    }
};

// ================================================================= dense QP solver (CPU)
// Full-space Mehrotra primal-dual interior point on
//   min 1/2 x^T P x + c^T x   (P = 2H)
//   s.t. A_e x = b_e (rows with lo == hi), lo <= G x <= hi (other rows), vlo <= x <= vhi,
// with a dense LU KKT solve, active-set polishing, and a phase-1 LP that decides INFEASIBLE the
// way a 1e-6 feasibility tolerance (CPLEX's default) would. Independent of the GPU algorithm
// (which works in a null-space-condensed space).

struct LU {
    int n;
    std::vector<double> a;
    std::vector<int> piv;
    bool ok = true;
    void factor(std::vector<double> m, int n_) {
        n = n_;
        a = std::move(m);
        piv.resize(n);
        ok = true;
        for (int k = 0; k < n; k++) {
            int p = k;
            double best = std::fabs(a[k * n + k]);
            for (int i = k + 1; i < n; i++)
                if (std::fabs(a[i * n + k]) > best) {
                    best = std::fabs(a[i * n + k]);
                    p = i;
                }
            piv[k] = p;
            if (best < 1e-300) {
                ok = false;
                a[k * n + k] = 1e-300;
            }
            if (p != k)
                for (int j = 0; j < n; j++) std::swap(a[k * n + j], a[p * n + j]);
            const double inv = 1.0 / a[k * n + k];
            for (int i = k + 1; i < n; i++) {
                double f = a[i * n + k] * inv;
                a[i * n + k] = f;
                if (f != 0)
                    for (int j = k + 1; j < n; j++) a[i * n + j] -= f * a[k * n + j];
            }
        }
    }
    void solve(std::vector<double>& b) const {
        // rows were swapped in full during factor (PA = LU): permute b first, then forward-solve
        for (int k = 0; k < n; k++)
            if (piv[k] != k) std::swap(b[k], b[piv[k]]);
        for (int k = 0; k < n; k++)
            for (int i = k + 1; i < n; i++) b[i] -= a[i * n + k] * b[k];
        for (int k = n - 1; k >= 0; k--) {
            double s = b[k];
            for (int j = k + 1; j < n; j++) s -= a[k * n + j] * b[j];
            b[k] = s / a[k * n + k];
        }
    }
};

struct Side {  // one finite inequality side: s = sg * (g.x - b) >= 0
    int row;   // >= 0: general row index; < 0: variable bound -(var+1)
    double b;
    double sg;
};

struct Solver {
    int n;
    std::vector<double> P, c;  // P = 2H
    std::vector<double> Ae, be;
    int me = 0;
    const DenseQP* qp;
    std::vector<Side> sides;

    double gdot(const Side& s, const double* x) const {
        if (s.row < 0) return x[-s.row - 1];
        const double* g = &qp->A[(size_t)s.row * n];
        double v = 0;
        for (int j = 0; j < n; j++) v += g[j] * x[j];
        return v;
    }
    void gaxpy(const Side& s, double alpha, double* y) const {  // y += alpha * g
        if (s.row < 0) {
            y[-s.row - 1] += alpha;
            return;
        }
        const double* g = &qp->A[(size_t)s.row * n];
        for (int j = 0; j < n; j++) y[j] += alpha * g[j];
    }

    explicit Solver(const DenseQP& q) : n(q.n), qp(&q) {
        P.resize(n * n);
        for (int i = 0; i < n * n; i++) P[i] = 2.0 * q.H[i];
        c = q.c;
        for (int r = 0; r < q.m; r++) {
            double lo = q.lo[r], hi = q.hi[r];
            if (!is_neg_inf(lo) && !is_pos_inf(hi) && lo == hi) {
                Ae.insert(Ae.end(), q.A.begin() + (size_t)r * n, q.A.begin() + (size_t)(r + 1) * n);
                be.push_back(lo);
                me++;
                continue;
            }
            if (!is_neg_inf(lo)) sides.push_back({r, lo, +1.0});
            if (!is_pos_inf(hi)) sides.push_back({r, hi, -1.0});
        }
        for (int i = 0; i < n; i++) {
            if (!is_neg_inf(q.vlo[i])) sides.push_back({-(i + 1), q.vlo[i], +1.0});
            if (!is_pos_inf(q.vhi[i])) sides.push_back({-(i + 1), q.vhi[i], -1.0});
        }
    }

    // KKT solve for given diag weights D (per side) and rhs.
    bool kkt(const std::vector<double>& D, const std::vector<double>& P_, const std::vector<double>& rhs_x,
             const std::vector<double>& rhs_e, std::vector<double>& dx, std::vector<double>& dl,
             double reg) const {
        const int N = n + me;
        std::vector<double> M(N * N, 0.0);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) M[i * N + j] = P_[i * n + j];
        for (size_t k = 0; k < sides.size(); k++) {
            const Side& s = sides[k];
            if (D[k] == 0) continue;
            if (s.row < 0) {
                int v = -s.row - 1;
                M[v * N + v] += D[k];
            } else {
                const double* g = &qp->A[(size_t)s.row * n];
                for (int i = 0; i < n; i++) {
                    if (g[i] == 0) continue;
                    double gi = D[k] * g[i];
                    for (int j = 0; j < n; j++) M[i * N + j] += gi * g[j];
                }
            }
        }
        for (int e = 0; e < me; e++)
            for (int j = 0; j < n; j++) {
                M[j * N + n + e] = -Ae[e * n + j];
                M[(n + e) * N + j] = Ae[e * n + j];
            }
        // factor with a small ridge on the x block, then refine against the exact system
        std::vector<double> M0 = M;
        for (int i = 0; i < n; i++) M[i * N + i] += reg;
        LU lu;
        lu.factor(std::move(M), N);
        std::vector<double> rhs(N);
        for (int i = 0; i < n; i++) rhs[i] = rhs_x[i];
        for (int e = 0; e < me; e++) rhs[n + e] = rhs_e[e];
        std::vector<double> b = rhs;
        lu.solve(b);
        for (int pass = 0; pass < 2; pass++) {  // iterative refinement against M0 (no ridge)
            std::vector<double> r = rhs;
            for (int i = 0; i < N; i++) {
                double v = 0;
                for (int j = 0; j < N; j++) v += M0[(size_t)i * N + j] * b[j];
                r[i] -= v;
            }
            lu.solve(r);
            for (int i = 0; i < N; i++) b[i] += r[i];
        }
        dx.assign(b.begin(), b.begin() + n);
        dl.assign(b.begin() + n, b.end());
        return lu.ok;
    }

    struct Result {
        int status;
        std::vector<double> x, lam, z, s;
        int iters;
        double kkt[4];
    };

    // residual norms of (x, lam, z) w.r.t. the original problem
    void certificate(const std::vector<double>& x, const std::vector<double>& lam,
                     const std::vector<double>& z, double* out) const {
        std::vector<double> rd(n, 0.0);
        for (int i = 0; i < n; i++) {
            double s = c[i];
            for (int j = 0; j < n; j++) s += P[i * n + j] * x[j];
            rd[i] = s;
        }
        for (int e = 0; e < me; e++)
            for (int j = 0; j < n; j++) rd[j] -= Ae[e * n + j] * lam[e];
        for (size_t k = 0; k < sides.size(); k++) gaxpy(sides[k], -sides[k].sg * z[k], rd.data());
        double st = 0, pinf = 0, dinf = 0, comp = 0;
        for (int i = 0; i < n; i++) st = std::max(st, std::fabs(rd[i]));
        for (int e = 0; e < me; e++) {
            double v = -be[e];
            for (int j = 0; j < n; j++) v += Ae[e * n + j] * x[j];
            pinf = std::max(pinf, std::fabs(v));
        }
        for (size_t k = 0; k < sides.size(); k++) {
            double s = sides[k].sg * (gdot(sides[k], x.data()) - sides[k].b);
            pinf = std::max(pinf, -s);
            dinf = std::max(dinf, -z[k]);
            comp = std::max(comp, std::fabs(std::max(s, 0.0) * z[k]));
        }
        out[0] = st;
        out[1] = pinf;
        out[2] = dinf;
        out[3] = comp;
    }

    Result pdip(int maxit, double tol) const {
        const int ns = (int)sides.size();
        Result R;
        R.status = ORC_UNKNOWN;
        std::vector<double> x, lam, dx, dl;
        // start: argmin 1/2 x'(P + rho I)x + c'x s.t. A_e x = b_e
        double pscale = 1.0;
        for (double v : P) pscale = std::max(pscale, std::fabs(v));
        {
            std::vector<double> D(ns, 0.0), rx(n), re(me);
            for (int i = 0; i < n; i++) rx[i] = -c[i];
            for (int e = 0; e < me; e++) re[e] = be[e];
            kkt(D, P, rx, re, x, lam, 1e-8 * pscale);
            // variables without curvature (slack variables: linear cost only) come out of the
            // ridge-regularised start at -c / ridge; pull bounded variables into their bounds
            for (int i = 0; i < n; i++) {
                if (!is_neg_inf(qp->vlo[i])) x[i] = std::max(x[i], qp->vlo[i]);
                if (!is_pos_inf(qp->vhi[i])) x[i] = std::min(x[i], qp->vhi[i]);
            }
            // ... and a variable without curvature that relaxes upper-bounded rows (a slack
            // variable: -1 in its neighbour's CBF rows) starts at the smallest value that satisfies
            // them at the start point, max(lower bound, max_r (g_r x - hi_r) / -A_ri): its optimum
            // can be ~1e8 (a neighbour deep inside d_min), which steps limited by the ridge on a
            // zero-curvature column (dv ~ rd / ridge) never reach (round 3's UNKNOWN slack QPs)
            for (int i = 0; i < n; i++) {
                if (P[(size_t)i * n + i] != 0.0 || is_neg_inf(qp->vlo[i])) continue;
                double v = x[i];
                for (int r = 0; r < qp->m; r++) {
                    const double a = qp->A[(size_t)r * n + i];
                    if (!(a < 0.0) || is_pos_inf(qp->hi[r]) || qp->lo[r] == qp->hi[r]) continue;
                    double gx = 0.0;
                    for (int j = 0; j < n; j++)
                        if (j != i) gx += qp->A[(size_t)r * n + j] * x[j];
                    v = std::max(v, (gx - qp->hi[r]) / -a);
                }
                if (!is_pos_inf(qp->vhi[i])) v = std::min(v, qp->vhi[i]);
                x[i] = v;
            }
        }
        std::vector<double> s(ns), z(ns);
        for (int k = 0; k < ns; k++) {
            double v = sides[k].sg * (gdot(sides[k], x.data()) - sides[k].b);
            s[k] = std::max(v, 1.0);
            z[k] = 1.0 / s[k];
            // a lower bound on a variable without curvature (slack variable) carries its linear
            // cost at the optimum (w - sum_rows z = z_bound): start the dual there
            if (sides[k].row < 0 && sides[k].sg > 0) {
                const int i = -sides[k].row - 1;
                if (P[(size_t)i * n + i] == 0.0 && c[i] > 0.0) z[k] = c[i];
            }
        }
        lam.assign(me, 0.0);
        std::vector<double> rd(n), re(me), rs(ns), D(ns), rhs(n), nre(me), dsa(ns), dza(ns),
            ds(ns), dz(ns), rc(ns);
        double cinf = 0;
        for (double v : c) cinf = std::max(cinf, std::fabs(v));
        int it;
        double best_merit = 1e300;
        int best_it = 0;
        std::vector<double> bx, blam, bz, bs;
        for (it = 0; it < maxit; it++) {
            // residuals
            for (int i = 0; i < n; i++) {
                double v = c[i];
                for (int j = 0; j < n; j++) v += P[i * n + j] * x[j];
                rd[i] = v;
            }
            for (int e = 0; e < me; e++)
                for (int j = 0; j < n; j++) rd[j] -= Ae[e * n + j] * lam[e];
            for (int k = 0; k < ns; k++) gaxpy(sides[k], -sides[k].sg * z[k], rd.data());
            double rpmax = 0, rdmax = 0, mu = 0, compmax = 0;
            for (int e = 0; e < me; e++) {
                double v = -be[e];
                for (int j = 0; j < n; j++) v += Ae[e * n + j] * x[j];
                re[e] = v;
                rpmax = std::max(rpmax, std::fabs(v) / (1.0 + std::fabs(be[e])));
            }
            for (int k = 0; k < ns; k++) {
                rs[k] = sides[k].sg * (gdot(sides[k], x.data()) - sides[k].b) - s[k];
                rpmax = std::max(rpmax, std::fabs(rs[k]) / (1.0 + std::fabs(sides[k].b)));
                mu += s[k] * z[k];
                compmax = std::max(compmax, s[k] * z[k]);
            }
            for (int i = 0; i < n; i++) rdmax = std::max(rdmax, std::fabs(rd[i]));
            rdmax /= (1.0 + cinf);
            mu = ns ? mu / ns : 0.0;
            const bool finite = std::isfinite(rpmax) && std::isfinite(rdmax) && std::isfinite(mu) &&
                                std::isfinite(compmax);
            if (!finite) break;  // diverged: status stays UNKNOWN (phase 1 decides)
            if (std::getenv("ORC_TRACE")) {
                int ia = 0;
                for (int i = 0; i < n; i++)
                    if (std::fabs(rd[i]) > std::fabs(rd[ia])) ia = i;
                std::fprintf(stderr, "it %d rp %.3e rd %.3e (var %d: x %.3e c %.3e) mu %.3e comp %.3e\n", it,
                             rpmax, rdmax, ia, x[ia], c[ia], mu, compmax);
            }
            // duality gap relative to the objective (rows whose bound is astronomically far,
            // e.g. b ~ 1e25 for a distant neighbour's CBF row, must not force mu -> 0 forever)
            double objv = 0;
            for (int i = 0; i < n; i++) {
                double px = 0;
                for (int j = 0; j < n; j++) px += P[i * n + j] * x[j];
                objv += x[i] * (0.5 * px + c[i]);
            }
            const double gap = mu * ns / (1.0 + std::fabs(objv));
            const double merit = std::max(std::max(rpmax, rdmax), gap);
            if (merit < best_merit) {
                best_merit = merit;
                best_it = it;
                bx = x;
                blam = lam;
                bz = z;
                bs = s;
            }
            if (rpmax < tol && rdmax < tol && gap < tol) {
                R.status = ORC_OPTIMAL;
                break;
            }
            if (it - best_it > 40) break;  // stalled
            for (int k = 0; k < ns; k++) D[k] = z[k] / s[k];
            // affine
            auto solve_dir = [&](const std::vector<double>& rcv, std::vector<double>& dxo,
                                 std::vector<double>& dlo, std::vector<double>& dso,
                                 std::vector<double>& dzo) {
                for (int i = 0; i < n; i++) rhs[i] = -rd[i];
                for (int k = 0; k < ns; k++)
                    gaxpy(sides[k], sides[k].sg * (rcv[k] - z[k] * rs[k]) / s[k], rhs.data());
                for (int e = 0; e < me; e++) nre[e] = -re[e];
                kkt(D, P, rhs, nre, dxo, dlo, 1e-14 * pscale);
                for (int k = 0; k < ns; k++) {
                    dso[k] = sides[k].sg * gdot(sides[k], dxo.data()) + rs[k];
                    dzo[k] = (rcv[k] - z[k] * dso[k]) / s[k];
                }
            };
            for (int k = 0; k < ns; k++) rc[k] = -s[k] * z[k];
            solve_dir(rc, dx, dl, dsa, dza);
            double ap = 1, ad = 1;
            for (int k = 0; k < ns; k++) {
                if (dsa[k] < 0) ap = std::min(ap, -s[k] / dsa[k]);
                if (dza[k] < 0) ad = std::min(ad, -z[k] / dza[k]);
            }
            double mua = 0;
            for (int k = 0; k < ns; k++) mua += (s[k] + ap * dsa[k]) * (z[k] + ad * dza[k]);
            mua = ns ? mua / ns : 0;
            double sigma = (mu > 0) ? std::min(1.0, std::pow(mua / mu, 3)) : 0;
            for (int k = 0; k < ns; k++) rc[k] = sigma * mu - s[k] * z[k] - dsa[k] * dza[k];
            solve_dir(rc, dx, dl, ds, dz);
            double amax = 1.0 / 0.99;
            for (int k = 0; k < ns; k++) {
                if (ds[k] < 0) amax = std::min(amax, -s[k] / ds[k]);
                if (dz[k] < 0) amax = std::min(amax, -z[k] / dz[k]);
            }
            double alpha = std::min(1.0, 0.99 * amax);
            for (int i = 0; i < n; i++) x[i] += alpha * dx[i];
            for (int e = 0; e < me; e++) lam[e] += alpha * dl[e];
            for (int k = 0; k < ns; k++) {
                s[k] += alpha * ds[k];
                z[k] += alpha * dz[k];
                s[k] = std::max(s[k], 1e-300);
                z[k] = std::max(z[k], 1e-300);
            }
        }
        R.iters = it;
        if (R.status != ORC_OPTIMAL && !bx.empty()) {
            // numerical stall after reaching a near-optimal point (best merit < 1e-8): keep the best
            // iterate as the optimum; otherwise it is still the best start for the caller's
            // active-set finish (solve(): certified, or UNKNOWN)
            if (best_merit < 1e-8) R.status = ORC_OPTIMAL;
            x = bx;
            lam = blam;
            z = bz;
            s = bs;
        }
        R.x = x;
        R.lam = lam;
        R.z = z;
        R.s = s;
        certificate(x, lam, z, R.kkt);
        return R;
    }

    // Equality-constrained re-solve on the active set (polish, no regularisation, two steps of
    // iterative refinement). Accepted only if its KKT certificate is no worse than the IPM's.
    static double merit(const double* kk, double cinf, double zinf) {
        return std::max(std::max(kk[0] / (1.0 + cinf), kk[1]), std::max(kk[2] / (1.0 + zinf), kk[3]));
    }
    bool polish(Result& R) const {
        const int ns = (int)sides.size();
        std::vector<int> act;
        for (int k = 0; k < ns; k++)
            if (R.z[k] > R.s[k]) act.push_back(k);
        const int na = (int)act.size();
        const int N = n + me + na;
        std::vector<double> M(N * N, 0.0), b(N, 0.0);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) M[i * N + j] = P[i * n + j];
        for (int i = 0; i < n; i++) b[i] = -c[i];
        for (int e = 0; e < me; e++) {
            for (int j = 0; j < n; j++) {
                M[j * N + n + e] = -Ae[e * n + j];
                M[(n + e) * N + j] = Ae[e * n + j];
            }
            b[n + e] = be[e];
        }
        for (int a = 0; a < na; a++) {
            const Side& sd = sides[act[a]];
            std::vector<double> g(n, 0.0);
            gaxpy(sd, 1.0, g.data());
            const int r = n + me + a;
            for (int j = 0; j < n; j++) {
                M[j * N + r] = -sd.sg * g[j];
                M[r * N + j] = g[j];
            }
            b[r] = sd.b;
        }
        LU lu;
        lu.factor(M, N);
        if (!lu.ok) return false;
        std::vector<double> sol = b;
        lu.solve(sol);
        for (int ref = 0; ref < 2; ref++) {  // iterative refinement
            std::vector<double> res(N);
            for (int i = 0; i < N; i++) {
                double v = b[i];
                for (int j = 0; j < N; j++) v -= M[i * N + j] * sol[j];
                res[i] = v;
            }
            lu.solve(res);
            for (int i = 0; i < N; i++) sol[i] += res[i];
        }
        std::vector<double> x(sol.begin(), sol.begin() + n), lam(sol.begin() + n, sol.begin() + n + me),
            z(ns, 0.0);
        for (int a = 0; a < na; a++) z[act[a]] = sol[n + me + a];
        double kk[4];
        certificate(x, lam, z, kk);
        double cinf = 0, zi = 0, zp = 0;
        for (double v : c) cinf = std::max(cinf, std::fabs(v));
        for (double v : z) zp = std::max(zp, std::fabs(v));
        for (double v : R.z) zi = std::max(zi, std::fabs(v));
        if (!(merit(kk, cinf, zp) <= merit(R.kkt, cinf, zi))) return false;
        R.x = x;
        R.lam = lam;
        R.z = z;
        for (int k = 0; k < ns; k++) R.s[k] = sides[k].sg * (gdot(sides[k], x.data()) - sides[k].b);
        std::memcpy(R.kkt, kk, sizeof(kk));
        return true;
    }
};

// Phase-1: min t s.t. A_e x = b_e, sg_k (g_k x - b_k) + t >= 0, t >= 0 (tiny ridge on x).
// Returns the minimal uniform violation t*.
double phase1(const DenseQP& q) {
    DenseQP f;
    const int n = q.n + 1;
    f.n = n;
    f.H.assign(n * n, 0.0);
    for (int i = 0; i < q.n; i++) f.H[i * n + i] = 1e-10;
    f.c.assign(n, 0.0);
    f.c[q.n] = 1.0;
    f.c0 = 0;
    // rows: equalities unchanged; each finite inequality side becomes its own relaxed row
    for (int r = 0; r < q.m; r++) {
        double lo = q.lo[r], hi = q.hi[r];
        std::vector<double> row(n, 0.0);
        std::copy(q.A.begin() + (size_t)r * q.n, q.A.begin() + (size_t)(r + 1) * q.n, row.begin());
        if (!is_neg_inf(lo) && !is_pos_inf(hi) && lo == hi) {
            f.A.insert(f.A.end(), row.begin(), row.end());
            f.lo.push_back(lo);
            f.hi.push_back(hi);
            f.m++;
            continue;
        }
        if (!is_neg_inf(lo)) {  // g x + t >= lo
            row[q.n] = 1.0;
            f.A.insert(f.A.end(), row.begin(), row.end());
            f.lo.push_back(lo);
            f.hi.push_back(INF);
            f.m++;
        }
        if (!is_pos_inf(hi)) {  // g x - t <= hi
            row[q.n] = -1.0;
            f.A.insert(f.A.end(), row.begin(), row.end());
            f.lo.push_back(LOWEST);
            f.hi.push_back(hi);
            f.m++;
        }
    }
    for (int i = 0; i < q.n; i++) {
        std::vector<double> row(n, 0.0);
        row[i] = 1.0;
        if (!is_neg_inf(q.vlo[i])) {
            row[q.n] = 1.0;
            f.A.insert(f.A.end(), row.begin(), row.end());
            f.lo.push_back(q.vlo[i]);
            f.hi.push_back(INF);
            f.m++;
        }
        if (!is_pos_inf(q.vhi[i])) {
            row[q.n] = -1.0;
            f.A.insert(f.A.end(), row.begin(), row.end());
            f.lo.push_back(LOWEST);
            f.hi.push_back(q.vhi[i]);
            f.m++;
        }
    }
    f.vlo.assign(n, LOWEST);
    f.vhi.assign(n, INF);
    f.vlo[q.n] = 0.0;
    Solver s(f);
    Solver::Result r = s.pdip(200, 1e-11);
    return r.x[q.n];
}

struct Solution {
    int status;
    std::vector<double> x;
    double obj;
    int iters;
    double kkt[4];
};

// Rows whose finite bound dwarfs any attainable activity (FoV HOCBF bounds reach 1e30+ through
// alpha(x) = 0.1 x^5) wreck the interior-point scaling; dividing such a row by a positive
// constant leaves the feasible set unchanged. Rows with |bound| > 1e6 are scaled to |bound| 1e6.
static DenseQP scale_huge_rows(const DenseQP& q) {
    DenseQP r = q;
    for (int i = 0; i < r.m; i++) {
        if (r.lo[i] == r.hi[i]) continue;
        double b = 0.0;
        if (!is_neg_inf(r.lo[i])) b = std::max(b, std::fabs(r.lo[i]));
        if (!is_pos_inf(r.hi[i])) b = std::max(b, std::fabs(r.hi[i]));
        if (!(b > 1e6)) continue;
        const double f = 1e6 / b;
        for (int j = 0; j < r.n; j++) r.A[(size_t)i * r.n + j] *= f;
        if (!is_neg_inf(r.lo[i])) r.lo[i] *= f;
        if (!is_pos_inf(r.hi[i])) r.hi[i] *= f;
    }
    return r;
}

// Columns of variables without curvature that relax upper-bounded rows (slack variables, lower
// bound 0, linear cost only) scaled to the magnitude of the bounds they offset: x_i = sigma_i x'_i
// with sigma_i = max(1, max_r |hi_r / A_ri| over rows with hi_r < 0). A neighbour deep inside d_min
// has a CBF bound ~ -1e8
// (gamma (2 d.dv + gamma h^3)^3), so its slack's optimum is ~1e8 next to a weight ~1e-4; unscaled,
// the interior point reaches it only in ridge-limited steps (round 3's two UNKNOWN all-neighbour
// slack QPs). A change of variables: same optimum, sigma_i times the multiplier scale.
static DenseQP scale_slack_columns(const DenseQP& q, std::vector<double>& sigma) {
    DenseQP r = q;
    const int n = q.n;
    sigma.assign(n, 1.0);
    for (int i = 0; i < n; i++) {
        if (q.vlo[i] != 0.0 || !is_pos_inf(q.vhi[i]) || q.c[i] <= 0.0) continue;
        bool curv = false;
        for (int j = 0; j < n; j++) curv = curv || q.H[(size_t)i * n + j] != 0.0 || q.H[(size_t)j * n + i] != 0.0;
        if (curv) continue;
        double sg = 1.0;
        for (int k = 0; k < q.m; k++) {
            const double a = q.A[(size_t)k * n + i];
            // (rows whose bound is negative: they force the variable up to about -hi / -a; a row
            // with a large positive bound leaves it at 0 and says nothing about its scale)
            if (!(a < 0.0) || is_pos_inf(q.hi[k]) || q.lo[k] == q.hi[k] || !(q.hi[k] < 0.0)) continue;
            sg = std::max(sg, std::fabs(q.hi[k] / a));
        }
        sigma[i] = sg;
        r.c[i] *= sg;
        for (int k = 0; k < q.m; k++) r.A[(size_t)k * n + i] *= sg;
    }
    return r;
}

Solution solve_kept(const DenseQP& q_in);

// Exact presolve: a variable that appears in no row, has no curvature, a finite lower bound and a
// positive linear cost sits at that bound at the optimum (a slack variable whose rows the exact
// box filter removed: v_i = 0). Removed here — left in, its central-path value mu / w_i with a
// weight down to ~1e-9 keeps the interior point far from the optimum. keep: kept columns.
static DenseQP drop_idle_columns(const DenseQP& q, std::vector<int>& keep, std::vector<double>& fixed) {
    const int n = q.n;
    keep.clear();
    fixed.assign(n, 0.0);
    for (int i = 0; i < n; i++) {
        bool used = false;
        for (int k = 0; k < q.m && !used; k++) used = q.A[(size_t)k * n + i] != 0.0;
        for (int j = 0; j < n && !used; j++) used = q.H[(size_t)i * n + j] != 0.0 || q.H[(size_t)j * n + i] != 0.0;
        if (!used && !is_neg_inf(q.vlo[i]) && q.c[i] > 0.0) {
            fixed[i] = q.vlo[i];
            continue;
        }
        keep.push_back(i);
    }
    DenseQP r;
    const int nk = (int)keep.size();
    r.n = nk;
    r.m = q.m;
    r.c0 = q.c0;
    for (int i = 0; i < n; i++) r.c0 += fixed[i] * q.c[i];  // (fixed columns: no rows, no curvature)
    r.H.assign((size_t)nk * nk, 0.0);
    r.c.resize(nk);
    r.vlo.resize(nk);
    r.vhi.resize(nk);
    for (int a = 0; a < nk; a++) {
        r.c[a] = q.c[keep[a]];
        r.vlo[a] = q.vlo[keep[a]];
        r.vhi[a] = q.vhi[keep[a]];
        for (int b = 0; b < nk; b++) r.H[(size_t)a * nk + b] = q.H[(size_t)keep[a] * n + keep[b]];
    }
    r.A.resize((size_t)q.m * nk);
    for (int k = 0; k < q.m; k++)
        for (int a = 0; a < nk; a++) r.A[(size_t)k * nk + a] = q.A[(size_t)k * n + keep[a]];
    r.lo = q.lo;
    r.hi = q.hi;
    return r;
}

Solution solve(const DenseQP& q_full) {
    std::vector<int> keep;
    std::vector<double> fixed;
    const DenseQP q_in = drop_idle_columns(q_full, keep, fixed);
    Solution out = solve_kept(q_in);
    std::vector<double> x = fixed;
    for (size_t a = 0; a < keep.size(); a++) x[keep[a]] = out.x[a];
    out.x = x;
    if (out.status == ORC_OPTIMAL) {
        double obj = q_full.c0;
        const int n = q_full.n;
        for (int i = 0; i < n; i++) {
            double hx = 0;
            for (int j = 0; j < n; j++) hx += q_full.H[(size_t)i * n + j] * x[j];
            obj += x[i] * hx + q_full.c[i] * x[i];
        }
        out.obj = obj;
    }
    return out;
}

Solution solve_kept(const DenseQP& q_in) {
    Solution out;
    std::vector<double> sigma;
    const DenseQP q = scale_slack_columns(scale_huge_rows(q_in), sigma);
    Solver s(q);
    Solver::Result r = s.pdip(200, 1e-10);
    if (r.status == ORC_OPTIMAL) {
        s.polish(r);
    } else if (s.polish(r)) {
        // the interior point stalled short of the tolerance (slack QPs whose optimal slack is
        // ~1e8 next to weights ~1e-4: the dual residual floors at ~1e-7): the equality QP on its
        // active sides, accepted as the optimum only with an exact KKT certificate (stationarity,
        // primal and dual feasibility, complementarity) at 1e-9
        double cinf = 0.0, zinf = 0.0, binf = 0.0;
        for (double v : s.c) cinf = std::max(cinf, std::fabs(v));
        for (double v : r.z) zinf = std::max(zinf, std::fabs(v));
        for (const auto& sd : s.sides) binf = std::max(binf, std::fabs(sd.b));
        if (r.kkt[0] <= 1e-9 * (1.0 + cinf) && r.kkt[1] <= 1e-9 * (1.0 + binf) &&
            r.kkt[2] <= 1e-9 * (1.0 + zinf) && r.kkt[3] <= 1e-9 * (1.0 + zinf) * (1.0 + binf))
            r.status = ORC_OPTIMAL;
    }
    out.iters = r.iters;
    std::memcpy(out.kkt, r.kkt, sizeof(out.kkt));
    for (int i = 0; i < q.n; i++) r.x[i] *= sigma[i];  // back to the caller's variables
    if (r.status != ORC_OPTIMAL) {
        // CPLEX default feasibility tolerance 1e-6 decides infeasibility
        double t = phase1(q);
        out.status = (t > 1e-6) ? ORC_INFEASIBLE : ORC_UNKNOWN;
        out.x = r.x;
        out.obj = std::numeric_limits<double>::quiet_NaN();
        return out;
    }
    out.status = ORC_OPTIMAL;
    out.x = r.x;
    const int n = q.n;
    double obj = q_in.c0;
    for (int i = 0; i < n; i++) {
        double hx = 0;
        for (int j = 0; j < n; j++) hx += q_in.H[i * n + j] * r.x[j];
        obj += r.x[i] * hx + q_in.c[i] * r.x[i];
    }
    out.obj = obj;
    return out;
}

// FovBezierIMPCCBF::distanceToEllipse (mpc_cbf/src/controller/FovBezierIMPCCBF.cpp:226-280):
// signed distance from the robot to the point of the 90 % confidence ellipse (s = 4.605) of the
// target estimate at parametric angle (slope - theta), negative inside. cov = (cxx, cxy, cyy),
// the 2x2 position block (:144-145). The reference diagonalises with Eigen::EigenSolver; the
// result is invariant to the eigenpair order and eigenvector signs (a, b are swapped to
// a >= b, theta is the major axis angle, and every term is a product of two sign flips), so the
// closed-form symmetric 2x2 eigen-decomposition stands in for it.
double distance_to_ellipse(const double* robot, const double* mean, const double* cov) {
    if (std::isinf(cov[0])) return -5.0;  // (:229, :279)
    const double cxx = cov[0], cxy = cov[1], cyy = cov[2];
    const double hm = 0.5 * (cxx + cyy), hd = 0.5 * (cxx - cyy);
    const double rt = std::sqrt(hd * hd + cxy * cxy);
    const double lmax = hm + rt, lmin = hm - rt;
    const double s = 4.605;
    const double a = std::sqrt(s * lmax), b = std::sqrt(s * lmin);  // a >= b (:238-246)
    // major-axis direction: eigenvector of lmax (:248-258); any sign / pi shift is equivalent
    double theta = 0.0;
    if (rt > 0.0) theta = 0.5 * std::atan2(2.0 * cxy, cxx - cyy);
    if (theta < 0.0) theta += M_PI;
    const double slope = std::atan2(-mean[1] + robot[1], -mean[0] + robot[0]);
    const double xn = mean[0] + a * std::cos(slope - theta) * std::cos(theta) -
                      b * std::sin(slope - theta) * std::sin(theta);
    const double yn = mean[1] + a * std::cos(slope - theta) * std::sin(theta) +
                      b * std::sin(slope - theta) * std::cos(theta);
    const double dist = std::sqrt(std::pow(xn - robot[0], 2) + std::pow(yn - robot[1], 2));
    if (std::isnan(dist)) return 5.0;  // (:266-269)
    const double d = std::sqrt(std::pow(mean[0] - robot[0], 2) + std::pow(mean[1] - robot[1], 2));
    const double range = std::sqrt(std::pow(mean[0] - xn, 2) + std::pow(mean[1] - yn, 2));
    return d < range ? -dist : dist;  // (:271-277)
}

// ConnectivityIMPCCBF::optimize (mpc_cbf/src/controller/ConnectivityIMPCCBF.cpp:47-215), and
// FovBezierIMPCCBF::optimize (FovBezierIMPCCBF.cpp:48-223) when p->cbf_mode == 1.
// covs: num_states x 3 position covariances (cxx, cxy, cyy) of the neighbour estimates (FoV slack
// weights only), or nullptr = unknown (infinite: distanceToEllipse returns -5 for every one).
int impc(const orc_params* p, int N, const double* states, int self, int nb, const int* nbidx,
         const double* ref, int* status, double* obj, double* x, int* qp_iters,
         const double* covs = nullptr) {
    Assembler as(p, nb);
    const double* st = states + 6 * self;
    std::vector<double> nbs(6 * nb);
    for (int i = 0; i < nb; i++) std::memcpy(&nbs[6 * i], states + 6 * nbidx[i], 6 * sizeof(double));
    // slack weights (:73-100): sort by planar distance, w * decay^rank
    std::vector<double> sw(nb, 0.0);
    if (p->slack_mode && p->cbf_mode == 1) {
        // FovBezierIMPCCBF.cpp:58-81: sort by distanceToEllipse (compareDist, :283-288), then the
        // weight of neighbour i is w * decay^{idx[i]} — the sorted position's index, not the rank
        // of i (reference quirk, kept). Ties keep the list order (std::sort is an insertion sort
        // below 17 elements in libstdc++; the batch path allows at most 16 neighbours).
        const double inf_cov[3] = {INFINITY, 0.0, INFINITY};
        std::vector<double> de(nb);
        for (int i = 0; i < nb; i++)
            de[i] = distance_to_ellipse(st, &nbs[6 * i], covs ? covs + 3 * (size_t)nbidx[i] : inf_cov);
        std::vector<size_t> idx(nb);
        std::iota(idx.begin(), idx.end(), 0);
        std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return de[a] < de[b]; });
        for (int i = 0; i < nb; i++) sw[i] = p->slack_cost * std::pow(p->slack_decay_rate, (double)idx[i]);
    } else if (p->slack_mode) {
        std::vector<size_t> idx(nb);
        std::iota(idx.begin(), idx.end(), 0);
        std::vector<double> dist(nb);
        for (int i = 0; i < nb; i++)
            dist[i] = std::hypot(nbs[6 * i] - st[0], nbs[6 * i + 1] - st[1]);
        std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return dist[a] < dist[b]; });
        for (int i = 0; i < nb; i++) sw[idx[i]] = p->slack_cost * std::pow(p->slack_decay_rate, (double)i);
    }
    const int n = as.nvar_total;
    std::vector<double> pred(6 * std::max(1, p->cbf_horizon));
    bool success = true;
    int attempted = 0;
    std::vector<double> last_x;
    for (int it = 0; it < p->impc_iter; it++) {
        if (it > 0) {
            // pred states from the previous OPTIMAL curve at h_samples(k), k < cbf_horizon (:158-168)
            for (int k = 0; k < p->cbf_horizon; k++) {
                as.evalCurve(last_x.data(), as.hs[k], 0, &pred[6 * k]);
                as.evalCurve(last_x.data(), as.hs[k], 1, &pred[6 * k + 3]);
            }
        }
        DenseQP q = as.build(st, ref, nb, nbs.data(), sw.data(), it, pred.data());
        Solution sol = solve(q);
        if (p->slack_mode && sol.status == ORC_OPTIMAL && nb > 0) {
            // slack polish: at the optimum v_i = max(0, max over its rows of the control points'
            // excess g x - h) exactly. The dense solve stops on a dual residual relative to the
            // largest slack cost, so a slack with a tiny weight (decay^rank down to 1e-14) whose
            // rows have astronomically far bounds (h ~ 1e26, 5 h^3 of a distant neighbour) can
            // stall far above that minimum: visible in the objective, not in the curve.
            const int ncp = n - nb;
            for (int j = ncp; j < n; j++) {
                double v = 0.0;
                for (int r = 0; r < q.m; r++) {
                    const double a = q.A[(size_t)r * n + j];
                    if (!(a < 0.0) || is_pos_inf(q.hi[r])) continue;
                    double gx = 0.0;
                    for (int k = 0; k < ncp; k++) gx += q.A[(size_t)r * n + k] * sol.x[k];
                    v = std::max(v, (gx - q.hi[r]) / -a);
                }
                sol.x[j] = v;
            }
            double ob = q.c0;
            for (int i = 0; i < n; i++) {
                double hx = 0.0;
                for (int j = 0; j < n; j++) hx += q.H[(size_t)i * n + j] * sol.x[j];
                ob += sol.x[i] * hx + q.c[i] * sol.x[i];
            }
            sol.obj = ob;
        }
        attempted++;
        status[it] = sol.status;
        obj[it] = sol.obj;
        if (qp_iters) qp_iters[it] = sol.iters;
        std::memcpy(x + (size_t)it * n, sol.x.data(), n * sizeof(double));
        if (sol.status == ORC_OPTIMAL) {
            success = true;
            last_x = sol.x;
        } else {
            success = false;
            break;
        }
    }
    (void)success;
    return attempted;
}

}  // namespace orc

// ====================================================================== C ABI
extern "C" {

uint64_t orc_fac(uint64_t n) { return orc::fac(n); }
uint64_t orc_comb(uint64_t n, uint64_t k) { return orc::comb(n, k); }
uint64_t orc_perm(uint64_t n, uint64_t k) { return orc::perm(n, k); }

int orc_bernstein_basis(uint64_t degree, double maxp, double t, uint64_t d, double* out) {
    try {
        std::vector<double> b = orc::bernsteinBasis(degree, maxp, t, d);
        std::memcpy(out, b.data(), b.size() * sizeof(double));
        return 0;
    } catch (...) {
        return -1;
    }
}

int orc_bernstein_coefficient_matrix(uint64_t degree, double maxp, uint64_t d, double* out) {
    try {
        std::vector<double> b = orc::bernsteinCoefficientMatrix(degree, maxp, d);
        std::memcpy(out, b.data(), b.size() * sizeof(double));
        return 0;
    } catch (...) {
        return -1;
    }
}

// ConnectivityCBF::initSafetyCBF (cbf/src/detail/ConnectivityCBF.cpp:152-198) evaluated at
// (state, neighbor) as getSafetyConstraints/getSafetyBound (:292-304, :560-566) do through
// matrixSubs/valueSubs (cbf/include/cbf/Helpers.hpp:10-44: ego px,py,th,vx,vy,w; neighbour
// px_n,py_n,vx_n,vy_n). gamma = 5 (:62), alpha(x) = gamma x^3 (:19-21, :91).
void orc_safety_cbf(const double* st, const double* nb, double d_min, double* a3, double* b) {
    const double gamma = 5.0;
    const double dx = st[0] - nb[0], dy = st[1] - nb[1];
    const double dvx = st[3] - nb[3], dvy = st[4] - nb[4];
    const double h = dx * dx + dy * dy - std::pow(d_min, 2);
    const double Lf_h = 2 * (dx * dvx + dy * dvy);
    const double Lf2_h = 2 * (dvx * dvx + dvy * dvy);
    const double alpha_h = gamma * std::pow(h, 3);
    // grad alpha = 3 gamma h^2 * (2dx, 2dy, 0, 0, 0, 0); f = A x = (vx, vy, w, 0, 0, 0)
    const double Lf_alpha = 3 * gamma * h * h * (2 * dx) * st[3] + 3 * gamma * h * h * (2 * dy) * st[4];
    const double psi1 = Lf_h + alpha_h;
    *b = Lf2_h + Lf_alpha + gamma * std::pow(psi1, 3);
    a3[0] = 2 * dx;
    a3[1] = 2 * dy;
    a3[2] = 0.0;
}

void orc_fov_cbf(const double* st, const double* tg, double fov, double Ds, double Rs, double* a12,
                 double* b4, int32_t* present4) {
    orc::FovRow fr[4];
    orc::fov_rows(st, tg, fov, Ds, Rs, fr);
    for (int r = 0; r < 4; r++) {
        for (int d = 0; d < 3; d++) a12[3 * r + d] = fr[r].a[d];
        b4[r] = fr[r].b;
        if (present4) present4[r] = fr[r].present ? 1 : 0;
    }
}

void orc_apply_input(double ts, const double* st, const double* u, double* out) {
    orc::Model m(ts);
    for (int i = 0; i < 6; i++) {
        double v = 0;
        for (int j = 0; j < 6; j++) v += m.A[i][j] * st[j];
        for (int j = 0; j < 3; j++) v += m.B[i][j] * u[j];
        out[i] = v;
    }
}

void orc_prediction_matrices(double ts, int32_t K, double* A0pos, double* Lpos) {
    orc::Model m(ts);
    std::vector<double> a = orc::getA0pos(m, K), l = orc::getLambdaPos(m, K);
    std::memcpy(A0pos, a.data(), a.size() * sizeof(double));
    std::memcpy(Lpos, l.data(), l.size() * sizeof(double));
}

int orc_num_vars(const orc_params* p, int32_t nb) {
    return p->num_pieces * 3 * p->num_control_points + (p->slack_mode ? nb : 0);
}

int orc_assemble_qp(const orc_params* p, const double* st, const double* ref, int32_t nb,
                    const double* nbs, const double* sw, int32_t iter, const double* pred,
                    int32_t max_rows, double* H, double* c, double* c0, double* A, double* lo,
                    double* hi, double* vlo, double* vhi) {
    try {
        orc::Assembler as(p, nb);
        std::vector<double> zero_w(std::max(nb, 1), 0.0);
        orc::DenseQP q = as.build(st, ref, nb, nbs, sw ? sw : zero_w.data(), iter, pred);
        if (q.m > max_rows) return -1;
        const int n = q.n;
        std::memcpy(H, q.H.data(), n * n * sizeof(double));
        std::memcpy(c, q.c.data(), n * sizeof(double));
        *c0 = q.c0;
        std::memcpy(A, q.A.data(), (size_t)q.m * n * sizeof(double));
        std::memcpy(lo, q.lo.data(), q.m * sizeof(double));
        std::memcpy(hi, q.hi.data(), q.m * sizeof(double));
        std::memcpy(vlo, q.vlo.data(), n * sizeof(double));
        std::memcpy(vhi, q.vhi.data(), n * sizeof(double));
        return q.m;
    } catch (...) {
        return -2;
    }
}

int orc_solve_dense_qp(int32_t n, const double* H, const double* c, double c0, int32_t m,
                       const double* A, const double* lo, const double* hi, const double* vlo,
                       const double* vhi, double* x_out, double* obj_out, int32_t* iters_out,
                       double* kkt_out) {
    orc::DenseQP q;
    q.n = n;
    q.H.assign(H, H + n * n);
    q.c.assign(c, c + n);
    q.c0 = c0;
    q.m = m;
    q.A.assign(A, A + (size_t)m * n);
    q.lo.assign(lo, lo + m);
    q.hi.assign(hi, hi + m);
    q.vlo.assign(vlo, vlo + n);
    q.vhi.assign(vhi, vhi + n);
    orc::Solution s = orc::solve(q);
    std::memcpy(x_out, s.x.data(), n * sizeof(double));
    *obj_out = s.obj;
    if (iters_out) *iters_out = s.iters;
    if (kkt_out) std::memcpy(kkt_out, s.kkt, sizeof(s.kkt));
    return s.status;
}

int orc_impc_optimize(const orc_params* p, int32_t N, const double* states, int32_t self,
                      int32_t nb, const int32_t* nbidx, const double* ref, int32_t* status,
                      double* obj, double* x, int32_t* qp_iters) {
    try {
        for (int i = 0; i < p->impc_iter; i++) {
            status[i] = ORC_UNKNOWN;
            obj[i] = std::numeric_limits<double>::quiet_NaN();
        }
        return orc::impc(p, N, states, self, nb, nbidx, ref, status, obj, x, qp_iters);
    } catch (...) {
        return -1;
    }
}

int orc_impc_optimize_cov(const orc_params* p, int32_t N, const double* states, int32_t self,
                          int32_t nb, const int32_t* nbidx, const double* ref, const double* covs,
                          int32_t* status, double* obj, double* x, int32_t* qp_iters) {
    try {
        for (int i = 0; i < p->impc_iter; i++) {
            status[i] = ORC_UNKNOWN;
            obj[i] = std::numeric_limits<double>::quiet_NaN();
        }
        return orc::impc(p, N, states, self, nb, nbidx, ref, status, obj, x, qp_iters, covs);
    } catch (...) {
        return -1;
    }
}

void orc_voronoi(const double* self2, const double* other2, const double* bbox3, double* normal3,
                 double* offset) {
    orc::voronoi_shifted(self2, other2, bbox3, normal3, offset);
}

double orc_distance_to_ellipse(const double* robot2, const double* mean2, const double* cov3) {
    return orc::distance_to_ellipse(robot2, mean2, cov3);
}

int64_t orc_impc_batch(const orc_params* p, int32_t N, const double* states, const double* refs,
                       const int32_t* rp, const int32_t* col, int32_t first, int32_t count,
                       int32_t nthreads, int32_t* status, double* obj, double* x_last,
                       const double* covs) {
    std::atomic<int> next(0);
    std::atomic<int64_t> solved(0);
    const int K = p->k_hor, it_n = p->impc_iter;
    auto work = [&]() {
        for (;;) {
            int i = next.fetch_add(1);
            if (i >= count) break;
            const int a = first + i;
            const int nb = rp[a + 1] - rp[a];
            const int n = orc_num_vars(p, nb);
            std::vector<double> xs((size_t)n * it_n, 0.0);
            int att = orc::impc(p, N, states, a, nb, col + rp[a], refs + (size_t)a * 3 * K,
                                status + (size_t)i * it_n, obj + (size_t)i * it_n, xs.data(), nullptr,
                                covs);
            solved += att;
            int last_ok = -1;
            for (int t = 0; t < att; t++)
                if (status[(size_t)i * it_n + t] == ORC_OPTIMAL) last_ok = t;
            if (x_last) {
                const int nc = p->num_pieces * 3 * p->num_control_points;
                if (last_ok >= 0)
                    std::memcpy(x_last + (size_t)i * nc, xs.data() + (size_t)last_ok * n, nc * sizeof(double));
                else
                    std::fill(x_last + (size_t)i * nc, x_last + (size_t)(i + 1) * nc,
                              std::numeric_limits<double>::quiet_NaN());
            }
        }
    };
    const int T = std::max(1, (int)nthreads);
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    return solved.load();
}

int orc_fov_control_slack(double fov, double Ds, double Rs, const double* vmin3, const double* vmax3,
                          const double* umin3, const double* umax3, const double* st,
                          const double* ud, int32_t nb, const double* nb_xy, int32_t slack_mode,
                          double slack_cost, double slack_decay, const double* nb_cov,
                          double* u_out, double* obj_out) {
    try {
        orc::DenseQP q;
        // decision variables: u (3), then one slack per neighbour in slack mode
        // (CBFQPGeneratorBase.cpp:9-27: addVariable(0, max))
        const int ns = slack_mode ? nb : 0;
        const int n = 3 + ns;
        q.n = n;
        // addDesiredControlCost (CBFQPGeneratorBase.cpp:36-57): I, -2 u_des, |u_des|^2
        q.H.assign((size_t)n * n, 0.0);
        q.c.assign(n, 0.0);
        for (int d = 0; d < 3; d++) {
            q.H[d * n + d] = 1.0;
            q.c[d] = -2.0 * ud[d];
            q.c0 += ud[d] * ud[d];
        }
        if (slack_mode) {
            // FovControl.cpp:25-46: sort by distanceToEllipse (:90-148, the same restatement as
            // FovBezierIMPCCBF's), weight of neighbour i = w * decay^{idx[i]}; addSlackCost ->
            // linear terms (CBFQPGeneratorBase.cpp:59-74, 136-170)
            const double inf_cov[3] = {INFINITY, 0.0, INFINITY};
            std::vector<double> de(nb);
            for (int i = 0; i < nb; i++)
                de[i] = orc::distance_to_ellipse(st, nb_xy + 2 * i, nb_cov ? nb_cov + 3 * i : inf_cov);
            std::vector<size_t> idx(nb);
            std::iota(idx.begin(), idx.end(), 0);
            std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return de[a] < de[b]; });
            for (int i = 0; i < nb; i++) q.c[3 + i] = slack_cost * std::pow(slack_decay, (double)idx[i]);
        }
        auto add_row = [&](const double* g, double hi, int slack) {
            for (int d = 0; d < n; d++) q.A.push_back(d < 3 ? g[d] : (d - 3 == slack ? -1.0 : 0.0));
            q.lo.push_back(-std::numeric_limits<double>::max());
            q.hi.push_back(hi);
            q.m++;
        };
        for (int i = 0; i < nb; i++) {  // safety, left border, right border, range (:58-68)
            orc::FovRow fr[4];
            orc::fov_rows(st, nb_xy + 2 * i, fov, Ds, Rs, fr);
            for (int r = 0; r < 4; r++) {
                if (!fr[r].present) continue;  // 360-degree FoV: no border rows
                const double g[3] = {-fr[r].a[0], -fr[r].a[1], -fr[r].a[2]};
                add_row(g, fr[r].b, slack_mode ? i : -1);  // FovQPGenerator.cpp:24-36: -1 on slack i
            }
        }
        for (int d = 0; d < 3; d++) {  // addMinVelConstraints: -(+e_d) u <= v_d - vmin_d
            double g[3] = {0, 0, 0};
            g[d] = -1.0;
            add_row(g, st[3 + d] - vmin3[d], -1);
        }
        for (int d = 0; d < 3; d++) {  // addMaxVelConstraints: -(-e_d) u <= vmax_d - v_d
            double g[3] = {0, 0, 0};
            g[d] = 1.0;
            add_row(g, vmax3[d] - st[3 + d], -1);
        }
        q.vlo.assign(n, 0.0);
        q.vhi.assign(n, std::numeric_limits<double>::infinity());
        for (int d = 0; d < 3; d++) {
            q.vlo[d] = umin3[d];
            q.vhi[d] = umax3[d];
        }
        orc::Solution r = orc::solve(q);
        for (int d = 0; d < 3; d++) u_out[d] = (int)r.x.size() == n ? r.x[d] : 0.0;
        if (obj_out) *obj_out = r.obj;
        return r.status;
    } catch (...) {
        return ORC_ERROR;
    }
}

int orc_fov_control(double fov, double Ds, double Rs, const double* vmin3, const double* vmax3,
                    const double* umin3, const double* umax3, const double* st,
                    const double* ud, int32_t nb, const double* nb_xy, double* u_out,
                    double* obj_out) {
    return orc_fov_control_slack(fov, Ds, Rs, vmin3, vmax3, umin3, umax3, st, ud, nb, nb_xy, 0, 0.0,
                                 1.0, nullptr, u_out, obj_out);
}

int orc_eval_curve(const orc_params* p, const double* x, double t, int32_t d, double* out3) {
    try {
        orc::Assembler as(p, 0);
        as.evalCurve(x, t, d, out3);
        return 0;
    } catch (...) {
        return -1;
    }
}

}  // extern "C"

// ================================================================ ConnectivityControl (CBF-only)
// cbf/src/controller/ConnectivityControl.cpp:22-99 with the rows of
// cbf/src/detail/ConnectivityCBF.cpp (safety :152-198, CLF :200-243, velocity :250-286,
// lambda2 :375-414, connectivity gradient :430-456, connectivity CBF :458-512) and
// cbf/src/optimization/ConnectivityQPGenerator.cpp:13-150.
namespace orc {

// ConnectivityCBF::getLambda2 (:375-414): weighted Laplacian of the planar positions,
// A_ij = exp((Rs^2 - d_ij^2)^2 / sigma) - 1 within Rs = dmax, sigma = dmax^4 / ln 2 (getSigma,
// :368-370); second smallest eigenvalue and its unit eigenvector. Eigen's
// SelfAdjointEigenSolver is restated by a cyclic Jacobi sweep to machine precision (eigenvalues
// sorted ascending; the eigenvector's sign is immaterial: it enters squared differences only).
static void lambda2(int N, const double* pos2, double dmax, double* l2, double* vec) {
    const double Rs2 = dmax * dmax, sigma = std::pow(dmax, 4) / std::log(2.0);
    std::vector<double> A((size_t)N * N, 0.0), V((size_t)N * N, 0.0);
    for (int i = 0; i < N; i++) {
        double deg = 0.0;
        for (int j = 0; j < N; j++) {
            if (i == j) continue;
            const double dx = pos2[2 * i] - pos2[2 * j], dy = pos2[2 * i + 1] - pos2[2 * j + 1];
            const double d2 = dx * dx + dy * dy;
            const double wij = d2 <= Rs2 ? std::exp(std::pow(Rs2 - d2, 2) / sigma) - 1.0 : 0.0;
            A[(size_t)i * N + j] = -wij;
            deg += wij;
        }
        A[(size_t)i * N + i] = deg;
        V[(size_t)i * N + i] = 1.0;
    }
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0.0, tot = 0.0;
        for (int i = 0; i < N; i++)
            for (int j = 0; j < N; j++) {
                const double a = A[(size_t)i * N + j] * A[(size_t)i * N + j];
                tot += a;
                if (i != j) off += a;
            }
        if (off <= 1e-32 * tot || off == 0.0) break;
        for (int p = 0; p < N - 1; p++)
            for (int q = p + 1; q < N; q++) {
                const double apq = A[(size_t)p * N + q];
                if (apq == 0.0) continue;
                const double app = A[(size_t)p * N + p], aqq = A[(size_t)q * N + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < N; k++) {  // A <- J^T A J, V <- V J
                    const double akp = A[(size_t)k * N + p], akq = A[(size_t)k * N + q];
                    A[(size_t)k * N + p] = c * akp - s * akq;
                    A[(size_t)k * N + q] = s * akp + c * akq;
                }
                for (int k = 0; k < N; k++) {
                    const double apk = A[(size_t)p * N + k], aqk = A[(size_t)q * N + k];
                    A[(size_t)p * N + k] = c * apk - s * aqk;
                    A[(size_t)q * N + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < N; k++) {
                    const double vkp = V[(size_t)k * N + p], vkq = V[(size_t)k * N + q];
                    V[(size_t)k * N + p] = c * vkp - s * vkq;
                    V[(size_t)k * N + q] = s * vkp + c * vkq;
                }
            }
    }
    std::vector<int> ord(N);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(),
                     [&](int a, int b) { return A[(size_t)a * N + a] < A[(size_t)b * N + b]; });
    const int k = N > 1 ? ord[1] : ord[0];
    *l2 = A[(size_t)k * N + k];
    double nrm = 0.0;
    for (int i = 0; i < N; i++) nrm += V[(size_t)i * N + k] * V[(size_t)i * N + k];
    nrm = std::sqrt(nrm);
    for (int i = 0; i < N; i++) vec[i] = V[(size_t)i * N + k] / nrm;  // eigenvec.normalize()
}

// ConnectivityCBF::initConnCBF / getConnConstraints / getConnBound (:430-512) for robot `self`:
// h = lambda2 - 0.1; grad h over the self position (compute_full_grad_h, :430-456: every other
// robot j, in range or not), its Hessian over the self position (eigenvector entries held
// fixed, as the symbols are substituted after differentiation), Lf h = grad . v,
// Lf^2 h = v^T Hess v, and with the linear alpha (setAlpha(defaultAlpha), gamma = 5)
// Bc = Lf^2 h + alpha(Lf h) + alpha(Lf h + alpha(h)). Ac = (dh/dx, dh/dy, 0).
static void conn_row(int N, const double* states, int self, const double* ev, double l2,
                     double dmax, double* a3, double* b, double* dbg /* gx gy Hxx Hxy Hyy Lfh Lf2h */) {
    const double Rs2 = dmax * dmax, sigma = std::pow(dmax, 4) / std::log(2.0);
    const double* si = states + 6 * self;
    double gx = 0, gy = 0, hxx = 0, hxy = 0, hyy = 0;
    for (int j = 0; j < N; j++) {
        if (j == self) continue;
        const double* sj = states + 6 * j;
        const double dx = si[0] - sj[0], dy = si[1] - sj[1];
        const double diff = Rs2 - (dx * dx + dy * dy);
        const double E = std::exp(diff * diff / sigma);  // A_ij + 1
        const double c = std::pow(ev[self] - ev[j], 2);
        const double k = -4.0 * c / sigma;  // dA/dx = -4 (A + 1) diff / sigma dx
        gx += k * E * diff * dx;
        gy += k * E * diff * dy;
        // d/dx (E diff dx) = -4 E diff^2 dx^2 / sigma - 2 E dx^2 + E diff, etc.
        hxx += k * (-4.0 * E * diff * diff * dx * dx / sigma - 2.0 * E * dx * dx + E * diff);
        hxy += k * (-4.0 * E * diff * diff * dx * dy / sigma - 2.0 * E * dx * dy);
        hyy += k * (-4.0 * E * diff * diff * dy * dy / sigma - 2.0 * E * dy * dy + E * diff);
    }
    const double vx = si[3], vy = si[4];
    const double lfh = gx * vx + gy * vy;
    const double lf2h = vx * (hxx * vx + hxy * vy) + vy * (hxy * vx + hyy * vy);
    const double gamma = 5.0, h = l2 - 0.1;
    *b = lf2h + gamma * lfh + gamma * (lfh + gamma * h);
    a3[0] = gx;
    a3[1] = gy;
    a3[2] = 0.0;
    if (dbg) {
        const double d[7] = {gx, gy, hxx, hxy, hyy, lfh, lf2h};
        std::memcpy(dbg, d, sizeof d);
    }
}

// ConnectivityCBF::initCLFCBF (:200-243) at (state, neighbour): V = (|p - p_n| - 2)^2, ego
// velocity only; Ac = grad V (x, y), Bc = Lf^2 V + 5 Lf V + 2 V.
static void clf_row(const double* st, const double* nb, double* a3, double* b) {
    const double dx = st[0] - nb[0], dy = st[1] - nb[1];
    const double dist = std::sqrt(dx * dx + dy * dy), e = dist - 2.0;
    const double gx = 2.0 * e * dx / dist, gy = 2.0 * e * dy / dist;
    const double vx = st[3], vy = st[4];
    const double lfv = gx * vx + gy * vy;
    const double dv = (dx * vx + dy * vy) / dist;  // v . grad dist
    const double vv = vx * vx + vy * vy;
    const double lf2v = 2.0 * dv * dv + 2.0 * e * (vv - dv * dv) / dist;  // v^T Hess V v
    *b = lf2v + 5.0 * lfv + 2.0 * e * e;
    a3[0] = gx;
    a3[1] = gy;
    a3[2] = 0.0;
}

}  // namespace orc

extern "C" {

void orc_lambda2(int32_t N, const double* pos2, double dmax, double* l2, double* vec) {
    orc::lambda2(N, pos2, dmax, l2, vec);
}

void orc_conn_cbf(int32_t N, const double* states, int32_t self, const double* ev, double l2,
                  double dmax, double* a3, double* b, double* dbg7) {
    orc::conn_row(N, states, self, ev, l2, dmax, a3, b, dbg7);
}

void orc_clf_cbf(const double* st, const double* nb, double* a3, double* b) { orc::clf_row(st, nb, a3, b); }

int orc_connectivity_control(double dmin, double dmax, const double* vmin3, const double* vmax3,
                             int32_t slack_mode, double slack_cost, double slack_decay, int32_t N,
                             const double* states, int32_t self, const double* ud, double* u_out,
                             double* obj_out, double* l2_out) {
    try {
        orc::DenseQP q;
        const int ns = slack_mode ? N : 0;  // CBFQPGeneratorBase(num_robots, slack): N slacks
        const int n = 3 + ns;
        q.n = n;
        q.H.assign((size_t)n * n, 0.0);
        q.c.assign(n, 0.0);
        for (int d = 0; d < 3; d++) {  // addDesiredControlCost
            q.H[d * n + d] = 1.0;
            q.c[d] = -2.0 * ud[d];
            q.c0 += ud[d] * ud[d];
        }
        for (int i = 0; i < ns; i++) q.c[3 + i] = slack_cost * std::pow(slack_decay, (double)i);  // :31-38
        auto add_row = [&](const double* g, double hi, int slack) {
            for (int d = 0; d < n; d++) q.A.push_back(d < 3 ? g[d] : (d - 3 == slack ? -1.0 : 0.0));
            q.lo.push_back(-std::numeric_limits<double>::max());
            q.hi.push_back(hi);
            q.m++;
        };
        const double* st = states + 6 * self;
        // safety rows vs every other robot (:49-55), slack i
        for (int i = 0; i < N - 1; i++) {
            const double* nb = states + 6 * (i + (i >= self ? 1 : 0));
            double a[3], b;
            orc_safety_cbf(st, nb, dmin, a, &b);
            const double g[3] = {-a[0], -a[1], -a[2]};
            add_row(g, b, slack_mode ? i : -1);
        }
        // velocity CBFs (:58-59): -u_d <= v_d - vmin_d, u_d <= vmax_d - v_d; no control bounds
        // (addControlBoundConstraint is commented out, :60)
        for (int d = 0; d < 3; d++) {
            double g[3] = {0, 0, 0};
            g[d] = -1.0;
            add_row(g, st[3 + d] - vmin3[d], -1);
        }
        for (int d = 0; d < 3; d++) {
            double g[3] = {0, 0, 0};
            g[d] = 1.0;
            add_row(g, vmax3[d] - st[3 + d], -1);
        }
        std::vector<double> pos(2 * N), ev(N);
        for (int i = 0; i < N; i++) {
            pos[2 * i] = states[6 * i];
            pos[2 * i + 1] = states[6 * i + 1];
        }
        double l2 = 0.0;
        orc::lambda2(N, pos.data(), dmax, &l2, ev.data());
        if (l2_out) *l2_out = l2;
        if (l2 > 0.1) {  // addConnConstraint (:70-71; ConnectivityQPGenerator.cpp:13-44): last slack
            double a[3], b;
            orc::conn_row(N, states, self, ev.data(), l2, dmax, a, &b, nullptr);
            const double g[3] = {-a[0], -a[1], -a[2]};
            add_row(g, b, slack_mode ? N - 1 : -1);
        } else {  // CLF rows (:72-82; :47-69): +Ac u <= -Bc, slack i
            for (int i = 0; i < N - 1; i++) {
                const double* nb = states + 6 * (i + (i >= self ? 1 : 0));
                double a[3], b;
                orc::clf_row(st, nb, a, &b);
                add_row(a, -b, slack_mode ? i : -1);
            }
        }
        q.vlo.assign(n, 0.0);  // slack variables [0, max)
        q.vhi.assign(n, std::numeric_limits<double>::infinity());
        for (int d = 0; d < 3; d++) {  // control inputs: free (addVariable() defaults)
            q.vlo[d] = -std::numeric_limits<double>::infinity();
            q.vhi[d] = std::numeric_limits<double>::infinity();
        }
        orc::Solution r = orc::solve(q);
        for (int d = 0; d < 3; d++) u_out[d] = (int)r.x.size() == n ? r.x[d] : 0.0;
        double obj = r.obj;
        if (ns > 0 && r.status == ORC_OPTIMAL) {
            // slack polish: at the optimum v_i = max(0, max over its rows of g u - h) exactly.
            // The dense solve's v carries its tolerance relative to the rows' bounds, which reach
            // 1e6 here (safety Bc); with weights up to 1e5 that is visible in the objective.
            std::vector<double> v(ns, 0.0);
            for (int row = 0; row < q.m; row++)
                for (int i = 0; i < ns; i++)
                    if (q.A[(size_t)row * n + 3 + i] == -1.0) {
                        double gu = 0.0;
                        for (int d = 0; d < 3; d++) gu += q.A[(size_t)row * n + d] * u_out[d];
                        v[i] = std::max(v[i], gu - q.hi[row]);
                    }
            obj = q.c0;
            for (int d = 0; d < 3; d++) obj += u_out[d] * u_out[d] + q.c[d] * u_out[d];
            for (int i = 0; i < ns; i++) obj += q.c[3 + i] * v[i];
        }
        if (obj_out) *obj_out = obj;
        return r.status;
    } catch (...) {
        return ORC_ERROR;
    }
}

}  // extern "C"
