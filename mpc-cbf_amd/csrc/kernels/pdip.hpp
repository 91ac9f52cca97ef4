// pdip.hpp — batched FP64 Mehrotra primal-dual interior-point core for small dense QPs
//
//     minimise 1/2 y^T P y + q^T y     s.t.   lo_i <= g_i^T y <= hi_i   (i = rows)
//
// executed by a group of G lanes per QP. Row i lives in register slot r = i / G of lane
// i % G (R slots per lane), together with its slacks and duals, so one Newton step is:
//   per lane:  row residuals, rank-1 terms D_i g_i g_i^T and right-hand sides (branch-free:
//              an absent side has mask 0, slack 1 and dual 0, so it contributes nothing)
//   group:     one all-reduce of the packed normal matrix + vector (DPP butterfly)
//   uniform:   Cholesky of the NZ x NZ normal matrix (every lane of the group, same values)
// Mehrotra predictor-corrector (Nocedal & Wright, Alg. 16.4) on two-sided rows; the dual
// residual is tracked (an exact Newton step scales it by 1 - alpha) and recomputed when the
// tracked value claims convergence. This is the solver that stands in for
// CPLEXSolver::solve (qpcpp/src/solvers/CPLEX.cpp:35-177); the QP it receives is the reference
// QP condensed onto the null space of its equality constraints.
#pragma once

#include "group.hpp"

// Profiling build only (make prof): cycle stamps at the phase boundaries of Newton step 2.
#ifdef MPCCBF_PDIP_STAMPS
#define PSTAMP(k)                                                             \
    do {                                                                      \
        if (dbg && it == 2) dbg[k] = (long long)__builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define PSTAMP(k) \
    do {          \
    } while (0)
#endif

namespace mpccbf {
namespace dev {

constexpr int ST_OPTIMAL = 0, ST_INFEASIBLE = 3, ST_ERROR = 4, ST_UNKNOWN = 5;

template <int NZ>
struct Sym {
    static constexpr int P = NZ * (NZ + 1) / 2;
    __host__ __device__ static constexpr int idx(int i, int j) {  // i <= j, packed upper, row-major
        return i * NZ - (i * (i - 1)) / 2 + (j - i);
    }
};

// In-place Cholesky of packed symmetric M (upper triangle becomes L^T, diagonal stores L_jj,
// dinv the reciprocal diagonal). Returns false if a pivot is not positive.
template <int NZ>
__device__ __forceinline__ bool chol_packed(double (&M)[Sym<NZ>::P], double (&dinv)[NZ]) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NZ; j++) {
        double d = M[Sym<NZ>::idx(j, j)];
#pragma unroll
        for (int k = 0; k < j; k++) d = fma(-M[Sym<NZ>::idx(k, j)], M[Sym<NZ>::idx(k, j)], d);
        ok = ok && (d > 0.0);
        d = d > 0.0 ? d : 1e-300;
        const double r = rsqrt(d);
        dinv[j] = r;
        M[Sym<NZ>::idx(j, j)] = d * r;
#pragma unroll
        for (int i = j + 1; i < NZ; i++) {
            double v = M[Sym<NZ>::idx(j, i)];
#pragma unroll
            for (int k = 0; k < j; k++) v = fma(-M[Sym<NZ>::idx(k, i)], M[Sym<NZ>::idx(k, j)], v);
            M[Sym<NZ>::idx(j, i)] = v * r;
        }
    }
    return ok;
}

template <int NZ>
__device__ __forceinline__ void chol_solve(const double (&M)[Sym<NZ>::P], const double (&dinv)[NZ],
                                           const double (&b)[NZ], double (&x)[NZ]) {
    double w[NZ];
#pragma unroll
    for (int i = 0; i < NZ; i++) {
        double v = b[i];
#pragma unroll
        for (int k = 0; k < i; k++) v = fma(-M[Sym<NZ>::idx(k, i)], w[k], v);
        w[i] = v * dinv[i];
    }
#pragma unroll
    for (int i = NZ - 1; i >= 0; i--) {
        double v = w[i];
#pragma unroll
        for (int k = i + 1; k < NZ; k++) v = fma(-M[Sym<NZ>::idx(i, k)], x[k], v);
        x[i] = v * dinv[i];
    }
}

template <int NZ>
__device__ __forceinline__ double dotz(const double (&a)[NZ], const double (&b)[NZ]) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < NZ; j++) s = fma(a[j], b[j], s);
    return s;
}

// Row storage of one lane: R slots. ml/mu are 1.0 when the lower/upper side is finite, else 0;
// lo/hi are 0 for absent sides.
template <int NZ, int R>
struct Rows {
    double g[R][NZ];
    double lo[R], hi[R];
    double ml[R], mu[R];
};

struct PdipCfg {
    int maxit;
    double tol;
    double reg = 0.0;  // added to the Newton matrix diagonal (direction only; residuals exact)
    // divergence test of pdip_solve_sep: from Newton step early_it on, complementarity above
    // early_mu x its starting value stops the solve (0: off). A QP with no feasible point drives
    // mu up while the iterate stalls; phase 1 then decides, and a feasible QP is re-solved
    // without the test, so statuses never depend on it.
    int early_it = 0;
    double early_mu = 1.5;
    // pdip_solve_sep: Newton matrix shifted by 1e-12 of its largest diagonal entry at every step
    // (inexact Newton, exact residuals and convergence test): the last attempt after a
    // factorisation breakdown at a degenerate point (active rows' D = z/s ~1e20 against P ~1e5)
    bool robust = false;
    // pdip_solve_sep: return the unconstrained minimiser when it satisfies every row
    bool fast_start = true;
    // pdip_solve_sep: relative dual residual accepted once primal feasibility and mu are three
    // orders past their targets (SURVEY.md §8c parity rule; CPLEX's default optimality tolerance)
    double rd_relax = 1e-6;
    // pdip_solve_sep (no slack variables): when the unconstrained minimiser violates a row, the
    // dual active-set method (sep_dual_as) with at most this many steps first; 0: off
    int dual_as = 0;
    // sep_dual_as: evaluate the returned point's dual residual (PdipOut::rd; else 0) / its scaled
    // primal residual (PdipOut::rp; else 0)
    bool want_rd = true;
    bool want_rp = true;
};

struct PdipOut {
    int status;
    int iters;
    bool early = false;  // stopped by the divergence test (phase 1 decides; pdip_solve_sep)
    bool polished = false;  // finished by the active-set solve (pdip_solve_sep)
    // OPTIMAL: scaled primal residual max_i |r_i| / (1 + |bound_i|) (bounds every row's violation)
    // and relative dual residual ||P y + q + G^T z||_inf / (1 + ||q||_inf) of the returned
    // iterate (mpccbf_batch.primal_res / dual_res); NaN otherwise
    double rp = __builtin_nan("");
    double rd = __builtin_nan("");
    // stopped by the dual active set without a feasible point: a lower bound on phase 1's t*
    // from the certificate sum_i lam_i n_i = 0, lam >= 0 (t* >= -sum lam b / sum lam)
    double tlow = 0.0;
};

// step-to-boundary of s + a ds >= 0 (or z): returns the limiting a, or `big` if ds >= 0
__device__ __forceinline__ double step_bound(double s, double ds, double big) {
    return ds < 0.0 ? -s * rcp(ds) : big;
}

// P: NZ x NZ row-major, LP: lower Cholesky factor of P (row-major) or nullptr when P is only
// positive semidefinite (generic dense path); uniform per group (global).
template <int NZ, int G, int R>
__device__ PdipOut pdip_solve(const Rows<NZ, R>& rw, const double* __restrict__ P,
                              const double* __restrict__ LP, const double (&q)[NZ],
                              double (&y)[NZ], const PdipCfg cfg) {
    using S = Sym<NZ>;
    // ---- start: y0 = argmin of the unconstrained objective when P is SPD (LP given), else 0
    if (LP == nullptr) {
#pragma unroll
        for (int i = 0; i < NZ; i++) y[i] = 0.0;
    } else {
        double w[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++) {
            double v = -q[i];
#pragma unroll
            for (int k = 0; k < i; k++) v = fma(-LP[i * NZ + k], w[k], v);
            w[i] = v * rcp(LP[i * NZ + i]);
        }
#pragma unroll
        for (int i = NZ - 1; i >= 0; i--) {
            double v = w[i];
#pragma unroll
            for (int k = i + 1; k < NZ; k++) v = fma(-LP[k * NZ + i], y[k], v);
            y[i] = v * rcp(LP[i * NZ + i]);
        }
    }
    double sl[R], su[R], zl[R], zu[R], pl[R], pu[R];
    double nsides = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const double t = dotz<NZ>(rw.g[r], y);
        sl[r] = rw.ml[r] > 0.0 ? fmax(t - rw.lo[r], 1.0) : 1.0;
        su[r] = rw.mu[r] > 0.0 ? fmax(rw.hi[r] - t, 1.0) : 1.0;
        zl[r] = rw.ml[r] * rcp(sl[r]);
        zu[r] = rw.mu[r] * rcp(su[r]);
        pl[r] = rw.ml[r] * rcp(1.0 + fabs(rw.lo[r]));  // relative primal-residual scale
        pu[r] = rw.mu[r] * rcp(1.0 + fabs(rw.hi[r]));
        nsides += rw.ml[r] + rw.mu[r];
    }
    nsides = grp_sum<G>(nsides);
    double qn = 0.0;
#pragma unroll
    for (int j = 0; j < NZ; j++) qn = fmax(qn, fabs(q[j]));
    const double inv_ns = nsides > 0.0 ? rcp(nsides) : 0.0;
    const double inv_qn = rcp(1.0 + qn);

    PdipOut out{ST_UNKNOWN, 0};
    double mu0 = 1.0;
    double rd_track = 1e300;  // tracked ||r_d||_inf / (1 + ||q||_inf)
    bool rd_exact = true;     // recompute r_d exactly this iteration
    for (int it = 0;; it++) {
        // ---- residuals, normal matrix, rhs: acc = [M (packed) | G^T w | mu], accr = G^T (zu - zl)
        constexpr int NM = S::P;
        constexpr int NA = NM + NZ + 1;
        double acc[NA], accr[NZ];
#pragma unroll
        for (int k = 0; k < NA; k++) acc[k] = 0.0;
#pragma unroll
        for (int k = 0; k < NZ; k++) accr[k] = 0.0;
        double rp = 0.0;
        double rsl[R], rsu[R], Dl[R], Du[R], isl[R], isu[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double t = dotz<NZ>(rw.g[r], y);
            rsl[r] = rw.ml[r] * (t - rw.lo[r] - sl[r]);
            rsu[r] = rw.mu[r] * (rw.hi[r] - t - su[r]);
            isl[r] = rcp(sl[r]);
            isu[r] = rcp(su[r]);
            Dl[r] = zl[r] * isl[r];
            Du[r] = zu[r] * isu[r];
            const double D = Dl[r] + Du[r];
            const double wv = Du[r] * rsu[r] - Dl[r] * rsl[r];
#pragma unroll
            for (int i = 0; i < NZ; i++) {
                const double dg = D * rw.g[r][i];
#pragma unroll
                for (int j = i; j < NZ; j++) acc[S::idx(i, j)] = fma(dg, rw.g[r][j], acc[S::idx(i, j)]);
                acc[NM + i] = fma(rw.g[r][i], wv, acc[NM + i]);
            }
            acc[NM + NZ] = fma(sl[r], zl[r], fma(su[r], zu[r], acc[NM + NZ]));
            if (rd_exact) {
#pragma unroll
                for (int i = 0; i < NZ; i++) accr[i] = fma(rw.g[r][i], zu[r] - zl[r], accr[i]);
            }
            rp = fmax(rp, fmax(fabs(rsl[r]) * pl[r], fabs(rsu[r]) * pu[r]));
        }
        grp_sum_vec<G, NA>(acc);
        if (rd_exact) grp_sum_vec<G, NZ>(accr);
        rp = grp_max<G>(rp);
        const double mu = acc[NM + NZ] * inv_ns;
        double py[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++) {
            double v = q[i];
#pragma unroll
            for (int j = 0; j < NZ; j++) v = fma(P[i * NZ + j], y[j], v);
            py[i] = v;  // P y + q
        }
        if (rd_exact) {
            double rdn = 0.0;
#pragma unroll
            for (int i = 0; i < NZ; i++) rdn = fmax(rdn, fabs(py[i] + accr[i]));
            rd_track = rdn * inv_qn;
            rd_exact = false;
        }
        out.iters = it;
        // NaN-safe: fmax drops NaN operands, so test finiteness of every reduced quantity
        const bool finite = isfinite(rp) && isfinite(rd_track) && isfinite(mu) && isfinite(acc[0]);
        if (finite && rp <= cfg.tol && mu <= cfg.tol * 0.1) {
            if (rd_track <= cfg.tol) {
                // confirm with the exact dual residual before accepting
                double chk[NZ];
#pragma unroll
                for (int i = 0; i < NZ; i++) chk[i] = 0.0;
#pragma unroll
                for (int r = 0; r < R; r++)
#pragma unroll
                    for (int i = 0; i < NZ; i++) chk[i] = fma(rw.g[r][i], zu[r] - zl[r], chk[i]);
                grp_sum_vec<G, NZ>(chk);
                double rdn = 0.0;
#pragma unroll
                for (int i = 0; i < NZ; i++) rdn = fmax(rdn, fabs(py[i] + chk[i]));
                rd_track = rdn * inv_qn;
                if (rd_track <= cfg.tol) {
                    out.status = ST_OPTIMAL;
                    out.rp = rp;
                    out.rd = rd_track;
                    break;
                }
            }
        }
        if (it == 0) mu0 = mu;
        // divergence (no feasible point): complementarity grows instead of shrinking
        if (it >= cfg.maxit || !finite || mu > 1e8 * fmax(mu0, 1.0)) {
            out.status = ST_UNKNOWN;
            break;
        }
        // ---- factor M = P + G^T D G
        double M[NM], dinv[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++)
#pragma unroll
            for (int j = i; j < NZ; j++) M[S::idx(i, j)] = acc[S::idx(i, j)] + P[i * NZ + j];
#pragma unroll
        for (int i = 0; i < NZ; i++) M[S::idx(i, i)] += cfg.reg;
        if (!chol_packed<NZ>(M, dinv)) {
            out.status = ST_UNKNOWN;  // numerically singular: phase 1 decides feasibility
            break;
        }
        // ---- predictor (affine) direction
        double rhs[NZ], dya[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++) rhs[i] = acc[NM + i] - py[i];
        chol_solve<NZ>(M, dinv, rhs, dya);
        double dsla[R], dzla[R], dsua[R], dzua[R];
        double ap = 1.0, ad = 1.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double td = dotz<NZ>(rw.g[r], dya);
            dsla[r] = rw.ml[r] * (td + rsl[r]);
            dsua[r] = rw.mu[r] * (rsu[r] - td);
            dzla[r] = -zl[r] - Dl[r] * dsla[r];
            dzua[r] = -zu[r] - Du[r] * dsua[r];
            ap = fmin(ap, fmin(step_bound(sl[r], dsla[r], 1.0), step_bound(su[r], dsua[r], 1.0)));
            ad = fmin(ad, fmin(step_bound(zl[r], dzla[r], 1.0), step_bound(zu[r], dzua[r], 1.0)));
        }
        ap = grp_min<G>(ap);
        ad = grp_min<G>(ad);
        double mua = 0.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            mua = fma(sl[r] + ap * dsla[r], zl[r] + ad * dzla[r], mua);
            mua = fma(su[r] + ap * dsua[r], zu[r] + ad * dzua[r], mua);
        }
        mua = grp_sum<G>(mua) * inv_ns;
        double sig = mu > 0.0 ? mua * rcp(mu) : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        // ---- corrector: extra right-hand side from sigma*mu and the second-order term
        double vc[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++) vc[i] = 0.0;
        double cl[R], cu[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            cl[r] = rw.ml[r] * (smu - dsla[r] * dzla[r]);
            cu[r] = rw.mu[r] * (smu - dsua[r] * dzua[r]);
            const double w = cl[r] * isl[r] - cu[r] * isu[r];
#pragma unroll
            for (int i = 0; i < NZ; i++) vc[i] = fma(rw.g[r][i], w, vc[i]);
        }
        grp_sum_vec<G, NZ>(vc);
        double dyc[NZ], dy[NZ];
        chol_solve<NZ>(M, dinv, vc, dyc);
#pragma unroll
        for (int i = 0; i < NZ; i++) dy[i] = dya[i] + dyc[i];
        double dsl[R], dzl[R], dsu[R], dzu[R];
        double amax = 1e300;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double td = dotz<NZ>(rw.g[r], dy);
            dsl[r] = rw.ml[r] * (td + rsl[r]);
            dsu[r] = rw.mu[r] * (rsu[r] - td);
            // dz = (sigma mu - s z - ds_a dz_a - z ds) / s   (absent side: cl = 0, z = 0 -> 0)
            dzl[r] = (cl[r] - sl[r] * zl[r] - zl[r] * dsl[r]) * isl[r];
            dzu[r] = (cu[r] - su[r] * zu[r] - zu[r] * dsu[r]) * isu[r];
            amax = fmin(amax, fmin(step_bound(sl[r], dsl[r], 1e300), step_bound(su[r], dsu[r], 1e300)));
            amax = fmin(amax, fmin(step_bound(zl[r], rw.ml[r] * dzl[r], 1e300),
                                   step_bound(zu[r], rw.mu[r] * dzu[r], 1e300)));
        }
        amax = grp_min<G>(amax);
        const double alpha = fmin(1.0, 0.99 * amax);
#pragma unroll
        for (int i = 0; i < NZ; i++) y[i] = fma(alpha, dy[i], y[i]);
#pragma unroll
        for (int r = 0; r < R; r++) {
            sl[r] = fmax(fma(alpha, dsl[r], sl[r]), 1e-300);
            su[r] = fmax(fma(alpha, dsu[r], su[r]), 1e-300);
            zl[r] = rw.ml[r] * fmax(fma(alpha, dzl[r], zl[r]), 1e-300);
            zu[r] = rw.mu[r] * fmax(fma(alpha, dzu[r], zu[r]), 1e-300);
        }
        rd_track *= (1.0 - alpha);
        if (it % 8 == 7) rd_exact = true;  // refresh against rounding drift
    }
    return out;
}

// Phase 1 (feasibility): minimal uniform violation
//     t* = min_{y, t >= 0} t   s.t.  lo_i - t <= g_i^T y <= hi_i + t
// solved by the same Mehrotra scheme in the (y, t) space (a tiny ridge eps/2 |y|^2 keeps the
// Newton matrix definite). The QP is INFEASIBLE iff t* exceeds the feasibility tolerance --
// the decision a 1e-6 row-violation tolerance (CPLEX's default) makes, and the rule the oracle
// applies (oracle/oracle.cpp phase1). Only run for QPs whose main solve did not converge.
template <int NZ, int G, int R>
__device__ double pdip_phase1(const Rows<NZ, R>& rw, const PdipCfg cfg, int* iters_out = nullptr) {
    constexpr int NV = NZ + 1;
    using S = Sym<NV>;
    constexpr double eps = 1e-10;
    double y[NZ], t;
#pragma unroll
    for (int i = 0; i < NZ; i++) y[i] = 0.0;
    double viol = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) viol = fmax(viol, fmax(rw.ml[r] * rw.lo[r], -rw.mu[r] * rw.hi[r]));
    t = grp_max<G>(viol) + 1.0;
    // sides: lower a_l = (g, 1), s_l = g y + t - lo ; upper a_u = (-g, 1), s_u = hi - g y + t ;
    // plus t >= 0 (uniform, s_t = t exactly)
    double sl[R], su[R], zl[R], zu[R];
    double nloc = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        sl[r] = rw.ml[r] > 0.0 ? t - rw.lo[r] : 1.0;
        su[r] = rw.mu[r] > 0.0 ? rw.hi[r] + t : 1.0;
        zl[r] = rw.ml[r] * rcp(sl[r]);
        zu[r] = rw.mu[r] * rcp(su[r]);
        nloc += rw.ml[r] + rw.mu[r];
    }
    double zt = rcp(t);
    const double inv_ns = rcp(grp_sum<G>(nloc) + 1.0);
    int it = 0;
    for (; it < 2 * cfg.maxit; it++) {
        constexpr int NA = S::P + NV + 1;
        double acc[NA];
#pragma unroll
        for (int k = 0; k < NA; k++) acc[k] = 0.0;
        double rsl[R], rsu[R], Dl[R], Du[R], isl[R], isu[R];
        double rp = 0.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double gy = dotz<NZ>(rw.g[r], y);
            rsl[r] = rw.ml[r] * (gy + t - rw.lo[r] - sl[r]);
            rsu[r] = rw.mu[r] * (rw.hi[r] - gy + t - su[r]);
            isl[r] = rcp(sl[r]);
            isu[r] = rcp(su[r]);
            Dl[r] = zl[r] * isl[r];
            Du[r] = zu[r] * isu[r];
            // affine rhs term: -a D rs (the dual +a z part cancels the -r_d term)
            const double wl = -Dl[r] * rsl[r], wu = -Du[r] * rsu[r];
            const double Ds = Dl[r] + Du[r], Dd = Dl[r] - Du[r];
#pragma unroll
            for (int i = 0; i < NZ; i++) {
#pragma unroll
                for (int j = i; j < NZ; j++)
                    acc[S::idx(i, j)] = fma(Ds * rw.g[r][i], rw.g[r][j], acc[S::idx(i, j)]);
                acc[S::idx(i, NZ)] = fma(Dd, rw.g[r][i], acc[S::idx(i, NZ)]);
                acc[S::P + i] = fma(rw.g[r][i], wl - wu, acc[S::P + i]);
            }
            acc[S::idx(NZ, NZ)] += Ds;
            acc[S::P + NZ] += wl + wu;
            acc[NA - 1] = fma(sl[r], zl[r], fma(su[r], zu[r], acc[NA - 1]));
            rp = fmax(rp, fmax(fabs(rsl[r]) * rw.ml[r] * rcp(1.0 + fabs(rw.lo[r])),
                               fabs(rsu[r]) * rw.mu[r] * rcp(1.0 + fabs(rw.hi[r]))));
        }
        grp_sum_vec<G, NA>(acc);
        rp = grp_max<G>(rp);
        const double mu = (acc[NA - 1] + t * zt) * inv_ns;
        if (!isfinite(mu) || !isfinite(rp)) {
            if (iters_out) *iters_out = it;
            return 1e300;
        }
        if (rp <= cfg.tol && mu <= cfg.tol * 0.1) break;
        double M[S::P], dinv[NV], rhs[NV], dv[NV];
        const double Dt = zt * rcp(t);
#pragma unroll
        for (int k = 0; k < S::P; k++) M[k] = acc[k];
#pragma unroll
        for (int i = 0; i < NZ; i++) M[S::idx(i, i)] += eps;
        M[S::idx(NZ, NZ)] += Dt;
        if (!chol_packed<NV>(M, dinv)) break;  // degenerate vertex: the iterate's violation stands
#pragma unroll
        for (int i = 0; i < NZ; i++) rhs[i] = -eps * y[i] + acc[S::P + i];
        rhs[NZ] = -1.0 + acc[S::P + NZ];
        chol_solve<NV>(M, dinv, rhs, dv);
        double ap = 1.0, ad = 1.0, dsla[R], dzla[R], dsua[R], dzua[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            double dgy = 0.0;
#pragma unroll
            for (int i = 0; i < NZ; i++) dgy = fma(rw.g[r][i], dv[i], dgy);
            dsla[r] = rw.ml[r] * (dgy + dv[NZ] + rsl[r]);
            dsua[r] = rw.mu[r] * (-dgy + dv[NZ] + rsu[r]);
            dzla[r] = -zl[r] - Dl[r] * dsla[r];
            dzua[r] = -zu[r] - Du[r] * dsua[r];
            ap = fmin(ap, fmin(step_bound(sl[r], dsla[r], 1.0), step_bound(su[r], dsua[r], 1.0)));
            ad = fmin(ad, fmin(step_bound(zl[r], dzla[r], 1.0), step_bound(zu[r], dzua[r], 1.0)));
        }
        const double dsta = dv[NZ], dzta = -zt - Dt * dsta;
        ap = fmin(ap, step_bound(t, dsta, 1.0));
        ad = fmin(ad, step_bound(zt, dzta, 1.0));
        ap = grp_min<G>(ap);
        ad = grp_min<G>(ad);
        double mua = 0.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            mua = fma(sl[r] + ap * dsla[r], zl[r] + ad * dzla[r], mua);
            mua = fma(su[r] + ap * dsua[r], zu[r] + ad * dzua[r], mua);
        }
        mua = (grp_sum<G>(mua) + (t + ap * dsta) * (zt + ad * dzta)) * inv_ns;
        double sig = mu > 0.0 ? mua * rcp(mu) : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        double vc[NV];
#pragma unroll
        for (int i = 0; i < NV; i++) vc[i] = 0.0;
        double cl[R], cu[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            cl[r] = rw.ml[r] * (smu - dsla[r] * dzla[r]);
            cu[r] = rw.mu[r] * (smu - dsua[r] * dzua[r]);
            const double a = cl[r] * isl[r], b = cu[r] * isu[r];
#pragma unroll
            for (int i = 0; i < NZ; i++) vc[i] = fma(rw.g[r][i], a - b, vc[i]);
            vc[NZ] += a + b;
        }
        grp_sum_vec<G, NV>(vc);
        const double ct = smu - dsta * dzta;
        vc[NZ] += ct * rcp(t);
        double dvc[NV];
        chol_solve<NV>(M, dinv, vc, dvc);
#pragma unroll
        for (int i = 0; i < NV; i++) dv[i] += dvc[i];
        double amax = 1e300, dsl[R], dzl[R], dsu[R], dzu[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            double dgy = 0.0;
#pragma unroll
            for (int i = 0; i < NZ; i++) dgy = fma(rw.g[r][i], dv[i], dgy);
            dsl[r] = rw.ml[r] * (dgy + dv[NZ] + rsl[r]);
            dsu[r] = rw.mu[r] * (-dgy + dv[NZ] + rsu[r]);
            dzl[r] = (cl[r] - sl[r] * zl[r] - zl[r] * dsl[r]) * isl[r];
            dzu[r] = (cu[r] - su[r] * zu[r] - zu[r] * dsu[r]) * isu[r];
            amax = fmin(amax, fmin(step_bound(sl[r], dsl[r], 1e300), step_bound(su[r], dsu[r], 1e300)));
            amax = fmin(amax, fmin(step_bound(zl[r], rw.ml[r] * dzl[r], 1e300),
                                   step_bound(zu[r], rw.mu[r] * dzu[r], 1e300)));
        }
        const double dst = dv[NZ];
        const double dzt = (ct - t * zt - zt * dst) * rcp(t);
        amax = fmin(amax, fmin(step_bound(t, dst, 1e300), step_bound(zt, dzt, 1e300)));
        amax = grp_min<G>(amax);
        const double alpha = fmin(1.0, 0.99 * amax);
#pragma unroll
        for (int i = 0; i < NZ; i++) y[i] = fma(alpha, dv[i], y[i]);
        t = fmax(fma(alpha, dst, t), 1e-300);
        zt = fmax(fma(alpha, dzt, zt), 1e-300);
#pragma unroll
        for (int r = 0; r < R; r++) {
            sl[r] = fmax(fma(alpha, dsl[r], sl[r]), 1e-300);
            su[r] = fmax(fma(alpha, dsu[r], su[r]), 1e-300);
            zl[r] = rw.ml[r] * fmax(fma(alpha, dzl[r], zl[r]), 1e-300);
            zu[r] = rw.mu[r] * fmax(fma(alpha, dzu[r], zu[r]), 1e-300);
        }
    }
    if (iters_out) *iters_out = it;
    // t* from the iterate: the largest actual row violation at y (>= 0)
    double worst = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const double gy = dotz<NZ>(rw.g[r], y);
        worst = fmax(worst, fmax(rw.ml[r] * (rw.lo[r] - gy), rw.mu[r] * (gy - rw.hi[r])));
    }
    return grp_max<G>(worst);
}

}  // namespace dev
}  // namespace mpccbf
