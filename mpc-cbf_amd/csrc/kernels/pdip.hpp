// pdip.hpp — batched FP64 Mehrotra primal-dual interior-point core for small dense QPs
//
//     minimise 1/2 y^T P y + q^T y     s.t.   lo_i <= g_i^T y <= hi_i   (i = rows)
//
// executed by a group of G lanes per QP. Row i lives in register slot r = i / G of lane
// i % G (R slots per lane), together with its slacks and duals, so one Newton step is:
//   per lane:  row residuals, the rank-1 terms D_i g_i g_i^T, right-hand sides
//   group:     one all-reduce of the packed normal matrix + vectors
//   uniform:   Cholesky of the NZ x NZ normal matrix (every lane of the group, same values)
// Mehrotra predictor-corrector (Nocedal & Wright, Alg. 16.4 adapted to two-sided rows).
// This is the solver that stands in for CPLEXSolver::solve (qpcpp/src/solvers/CPLEX.cpp:35-177);
// the QP it receives is the reference QP condensed onto the null space of its equalities.
#pragma once

#include "group.hpp"

namespace mpccbf {
namespace dev {

constexpr int ST_OPTIMAL = 0, ST_INFEASIBLE = 3, ST_ERROR = 4, ST_UNKNOWN = 5;

template <int NZ>
struct Sym {
    static constexpr int P = NZ * (NZ + 1) / 2;
    __device__ static constexpr int idx(int i, int j) {  // i <= j, packed upper triangle row-major
        return i * NZ - (i * (i - 1)) / 2 + (j - i);
    }
};

// In-place Cholesky of packed symmetric M (upper triangle holds L^T). Returns false if a pivot
// is not positive (caller regularises).
template <int NZ>
__device__ __forceinline__ bool chol_packed(double (&M)[Sym<NZ>::P], double (&dinv)[NZ]) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NZ; j++) {
        double d = M[Sym<NZ>::idx(j, j)];
#pragma unroll
        for (int k = 0; k < j; k++) d -= M[Sym<NZ>::idx(k, j)] * M[Sym<NZ>::idx(k, j)];
        ok = ok && (d > 0.0);
        d = d > 0.0 ? d : 1e-300;
        const double r = rsqrt(d);
        const double ljj = d * r;
        dinv[j] = r;
        M[Sym<NZ>::idx(j, j)] = ljj;
#pragma unroll
        for (int i = j + 1; i < NZ; i++) {
            double v = M[Sym<NZ>::idx(j, i)];
#pragma unroll
            for (int k = 0; k < j; k++) v -= M[Sym<NZ>::idx(k, i)] * M[Sym<NZ>::idx(k, j)];
            M[Sym<NZ>::idx(j, i)] = v * r;
        }
    }
    return ok;
}

// Solve (L L^T) x = b with the factor from chol_packed.
template <int NZ>
__device__ __forceinline__ void chol_solve(const double (&M)[Sym<NZ>::P], const double (&dinv)[NZ],
                                           const double (&b)[NZ], double (&x)[NZ]) {
    double w[NZ];
#pragma unroll
    for (int i = 0; i < NZ; i++) {
        double v = b[i];
#pragma unroll
        for (int k = 0; k < i; k++) v -= M[Sym<NZ>::idx(k, i)] * w[k];
        w[i] = v * dinv[i];
    }
#pragma unroll
    for (int i = NZ - 1; i >= 0; i--) {
        double v = w[i];
#pragma unroll
        for (int k = i + 1; k < NZ; k++) v -= M[Sym<NZ>::idx(i, k)] * x[k];
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

// Row storage of one lane: R slots.
template <int NZ, int R>
struct Rows {
    double g[R][NZ];
    double lo[R], hi[R];
    bool hl[R], hu[R];  // finite lower / upper side present
};

struct PdipCfg {
    int maxit;
    double tol;
};

struct PdipOut {
    int status;
    int iters;
};

// P: NZ x NZ row-major (uniform, global), LP: its lower Cholesky factor (row-major) used for
// the unconstrained start. q: uniform. y: result (uniform).
template <int NZ, int G, int R>
__device__ PdipOut pdip_solve(const Rows<NZ, R>& rw, const double* __restrict__ P,
                              const double* __restrict__ LP, const double (&q)[NZ],
                              double (&y)[NZ], const PdipCfg cfg) {
    using S = Sym<NZ>;
    // ---- start: y0 = argmin of the unconstrained objective (P is SPD on the reduced space)
    {
        double w[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++) {
            double v = -q[i];
#pragma unroll
            for (int k = 0; k < i; k++) v -= LP[i * NZ + k] * w[k];
            w[i] = v / LP[i * NZ + i];
        }
#pragma unroll
        for (int i = NZ - 1; i >= 0; i--) {
            double v = w[i];
#pragma unroll
            for (int k = i + 1; k < NZ; k++) v -= LP[k * NZ + i] * y[k];
            y[i] = v / LP[i * NZ + i];
        }
    }
    double sl[R], su[R], zl[R], zu[R];
    double nsides = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const double t = dotz<NZ>(rw.g[r], y);
        sl[r] = rw.hl[r] ? fmax(t - rw.lo[r], 1.0) : 1.0;
        su[r] = rw.hu[r] ? fmax(rw.hi[r] - t, 1.0) : 1.0;
        zl[r] = rw.hl[r] ? 1.0 / sl[r] : 0.0;
        zu[r] = rw.hu[r] ? 1.0 / su[r] : 0.0;
        nsides += (rw.hl[r] ? 1.0 : 0.0) + (rw.hu[r] ? 1.0 : 0.0);
    }
    nsides = grp_sum<G>(nsides);
    double qn = 0.0;
#pragma unroll
    for (int j = 0; j < NZ; j++) qn = fmax(qn, fabs(q[j]));
    const double inv_ns = nsides > 0.0 ? 1.0 / nsides : 0.0;

    PdipOut out{ST_UNKNOWN, 0};
    double mu0 = 1.0;
    for (int it = 0;; it++) {
        // ---- residuals and the normal matrix
        constexpr int NV = S::P + 2 * NZ + 1;
        double acc[NV];
#pragma unroll
        for (int k = 0; k < NV; k++) acc[k] = 0.0;
        double rp = 0.0;
        double rsl[R], rsu[R], Dl[R], Du[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double t = dotz<NZ>(rw.g[r], y);
            rsl[r] = rw.hl[r] ? (t - rw.lo[r] - sl[r]) : 0.0;
            rsu[r] = rw.hu[r] ? (rw.hi[r] - t - su[r]) : 0.0;
            Dl[r] = zl[r] / sl[r];
            Du[r] = zu[r] / su[r];
            const double D = Dl[r] + Du[r];
            const double wv = Du[r] * rsu[r] - Dl[r] * rsl[r];
            const double wd = zu[r] - zl[r];
#pragma unroll
            for (int i = 0; i < NZ; i++) {
                const double dg = D * rw.g[r][i];
#pragma unroll
                for (int j = i; j < NZ; j++) acc[S::idx(i, j)] = fma(dg, rw.g[r][j], acc[S::idx(i, j)]);
                acc[S::P + i] = fma(rw.g[r][i], wd, acc[S::P + i]);
                acc[S::P + NZ + i] = fma(rw.g[r][i], wv, acc[S::P + NZ + i]);
            }
            acc[NV - 1] += sl[r] * zl[r] + su[r] * zu[r];
            if (rw.hl[r]) rp = fmax(rp, fabs(rsl[r]) / (1.0 + fabs(rw.lo[r])));
            if (rw.hu[r]) rp = fmax(rp, fabs(rsu[r]) / (1.0 + fabs(rw.hi[r])));
        }
        grp_sum_vec<G, NV>(acc);
        rp = grp_max<G>(rp);
        const double mu = acc[NV - 1] * inv_ns;
        double py[NZ];
        double rdn = 0.0;
#pragma unroll
        for (int i = 0; i < NZ; i++) {
            double v = q[i];
#pragma unroll
            for (int j = 0; j < NZ; j++) v = fma(P[i * NZ + j], y[j], v);
            py[i] = v;  // P y + q
            rdn = fmax(rdn, fabs(v + acc[S::P + i]));
        }
        rdn /= (1.0 + qn);
        out.iters = it;
        // NaN-safe: fmax drops NaN operands, so test finiteness of every reduced quantity
        const bool finite = isfinite(rp) && isfinite(rdn) && isfinite(mu) && isfinite(acc[0]);
        if (finite && rp <= cfg.tol && rdn <= cfg.tol && mu <= cfg.tol * 0.1) {
            out.status = ST_OPTIMAL;
            break;
        }
        if (it == 0) mu0 = mu;
        // divergence (no feasible point): complementarity grows instead of shrinking
        if (it >= cfg.maxit || !finite || mu > 1e8 * fmax(mu0, 1.0)) {
            out.status = ST_UNKNOWN;
            break;
        }
        // ---- factor M = P + G^T D G
        double M[S::P], dinv[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++)
#pragma unroll
            for (int j = i; j < NZ; j++) M[S::idx(i, j)] = acc[S::idx(i, j)] + P[i * NZ + j];
        if (!chol_packed<NZ>(M, dinv)) {
            out.status = ST_UNKNOWN;  // numerically singular: let phase 1 decide feasibility
            break;
        }
        // ---- predictor (affine) direction
        double rhs[NZ], dya[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++) rhs[i] = -py[i] + acc[S::P + NZ + i];
        chol_solve<NZ>(M, dinv, rhs, dya);
        double dsla[R], dzla[R], dsua[R], dzua[R];
        double ap = 1.0, ad = 1.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double td = dotz<NZ>(rw.g[r], dya);
            dsla[r] = rw.hl[r] ? td + rsl[r] : 0.0;
            dsua[r] = rw.hu[r] ? -td + rsu[r] : 0.0;
            dzla[r] = rw.hl[r] ? -zl[r] - Dl[r] * dsla[r] : 0.0;
            dzua[r] = rw.hu[r] ? -zu[r] - Du[r] * dsua[r] : 0.0;
            if (dsla[r] < 0.0) ap = fmin(ap, -sl[r] / dsla[r]);
            if (dsua[r] < 0.0) ap = fmin(ap, -su[r] / dsua[r]);
            if (dzla[r] < 0.0) ad = fmin(ad, -zl[r] / dzla[r]);
            if (dzua[r] < 0.0) ad = fmin(ad, -zu[r] / dzua[r]);
        }
        ap = grp_min<G>(ap);
        ad = grp_min<G>(ad);
        double mua = 0.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (rw.hl[r]) mua += (sl[r] + ap * dsla[r]) * (zl[r] + ad * dzla[r]);
            if (rw.hu[r]) mua += (su[r] + ap * dsua[r]) * (zu[r] + ad * dzua[r]);
        }
        mua = grp_sum<G>(mua) * inv_ns;
        double sig = mu > 0.0 ? mua / mu : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        // ---- corrector: extra right-hand side from sigma*mu and the second-order term
        double vc[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++) vc[i] = 0.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double w = (rw.hl[r] ? (smu - dsla[r] * dzla[r]) / sl[r] : 0.0) -
                             (rw.hu[r] ? (smu - dsua[r] * dzua[r]) / su[r] : 0.0);
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
            dsl[r] = rw.hl[r] ? td + rsl[r] : 0.0;
            dsu[r] = rw.hu[r] ? -td + rsu[r] : 0.0;
            dzl[r] = rw.hl[r] ? (smu - sl[r] * zl[r] - dsla[r] * dzla[r] - zl[r] * dsl[r]) / sl[r] : 0.0;
            dzu[r] = rw.hu[r] ? (smu - su[r] * zu[r] - dsua[r] * dzua[r] - zu[r] * dsu[r]) / su[r] : 0.0;
            if (dsl[r] < 0.0) amax = fmin(amax, -sl[r] / dsl[r]);
            if (dsu[r] < 0.0) amax = fmin(amax, -su[r] / dsu[r]);
            if (dzl[r] < 0.0) amax = fmin(amax, -zl[r] / dzl[r]);
            if (dzu[r] < 0.0) amax = fmin(amax, -zu[r] / dzu[r]);
        }
        amax = grp_min<G>(amax);
        const double alpha = fmin(1.0, 0.99 * amax);
#pragma unroll
        for (int i = 0; i < NZ; i++) y[i] = fma(alpha, dy[i], y[i]);
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (rw.hl[r]) {
                sl[r] = fmax(fma(alpha, dsl[r], sl[r]), 1e-300);
                zl[r] = fmax(fma(alpha, dzl[r], zl[r]), 1e-300);
            }
            if (rw.hu[r]) {
                su[r] = fmax(fma(alpha, dsu[r], su[r]), 1e-300);
                zu[r] = fmax(fma(alpha, dzu[r], zu[r]), 1e-300);
            }
        }
    }
    return out;
}


// Phase 1 (feasibility): minimal uniform violation
//     t* = min_{y, t >= 0} t   s.t.  lo_i - t <= g_i^T y <= hi_i + t
// solved by the same Mehrotra scheme in the (y, t) space (tiny ridge eps/2 |y|^2 keeps the
// Newton matrix definite). The QP is INFEASIBLE iff t* exceeds the feasibility tolerance --
// the decision a 1e-6 row-violation tolerance (CPLEX's default) makes, and the rule the oracle
// applies (oracle/oracle.cpp phase1). Only run for QPs whose main solve did not converge.
template <int NZ, int G, int R>
__device__ double pdip_phase1(const Rows<NZ, R>& rw, const PdipCfg cfg) {
    constexpr int NV = NZ + 1;
    using S = Sym<NV>;
    constexpr double eps = 1e-10;
    double v[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) v[i] = 0.0;
    // t0 = max violation at y = 0, plus one
    double viol = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        if (rw.hl[r]) viol = fmax(viol, rw.lo[r]);
        if (rw.hu[r]) viol = fmax(viol, -rw.hi[r]);
    }
    v[NZ] = grp_max<G>(viol) + 1.0;
    double sl[R], su[R], zl[R], zu[R];
    double nsides = 1.0;  // the t >= 0 side (uniform, tracked by every lane)
    double st_ = v[NZ], zt = 1.0 / st_;
    double nloc = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        sl[r] = rw.hl[r] ? v[NZ] - rw.lo[r] : 1.0;
        su[r] = rw.hu[r] ? rw.hi[r] + v[NZ] : 1.0;
        zl[r] = rw.hl[r] ? 1.0 / sl[r] : 0.0;
        zu[r] = rw.hu[r] ? 1.0 / su[r] : 0.0;
        nloc += (rw.hl[r] ? 1.0 : 0.0) + (rw.hu[r] ? 1.0 : 0.0);
    }
    nsides += grp_sum<G>(nloc);
    const double inv_ns = 1.0 / nsides;
    for (int it = 0; it < 2 * cfg.maxit; it++) {
        constexpr int NA = S::P + NV + 1;
        double acc[NA];
#pragma unroll
        for (int k = 0; k < NA; k++) acc[k] = 0.0;
        double rsl[R], rsu[R], Dl[R], Du[R];
        double rp = 0.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double t = dotz<NZ>(rw.g[r], *reinterpret_cast<const double(*)[NZ]>(v));
            rsl[r] = rw.hl[r] ? (t + v[NZ] - rw.lo[r] - sl[r]) : 0.0;
            rsu[r] = rw.hu[r] ? (rw.hi[r] - t + v[NZ] - su[r]) : 0.0;
            Dl[r] = zl[r] / sl[r];
            Du[r] = zu[r] / su[r];
            // side vectors a_l = (g, 1), a_u = (-g, 1); affine rhs term a (z + (rc - z rs)/s)
            // = -a D rs with rc = -s z (the +a z part cancels the -r_d dual term)
            const double wl = rw.hl[r] ? -Dl[r] * rsl[r] : 0.0;
            const double wu = rw.hu[r] ? -Du[r] * rsu[r] : 0.0;
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
            acc[NA - 1] += sl[r] * zl[r] + su[r] * zu[r];
            if (rw.hl[r]) rp = fmax(rp, fabs(rsl[r]) / (1.0 + fabs(rw.lo[r])));
            if (rw.hu[r]) rp = fmax(rp, fabs(rsu[r]) / (1.0 + fabs(rw.hi[r])));
        }
        grp_sum_vec<G, NA>(acc);
        rp = grp_max<G>(rp);
        // affine rhs = -(eps y, 1) - sum_j a_j D_j rs_j  (rs of the t >= 0 side is exactly 0)
        const double mu = (acc[NA - 1] + st_ * zt) * inv_ns;
        if (!isfinite(mu) || !isfinite(rp)) return 1e300;
        if (rp <= cfg.tol && mu <= cfg.tol * 0.1) break;
        double M[S::P], dinv[NV], rhs[NV], dv[NV];
        const double Dt = zt / st_;
#pragma unroll
        for (int k = 0; k < S::P; k++) M[k] = acc[k];
#pragma unroll
        for (int i = 0; i < NZ; i++) M[S::idx(i, i)] += eps;
        M[S::idx(NZ, NZ)] += Dt;
        if (!chol_packed<NV>(M, dinv)) return 1e300;
#pragma unroll
        for (int i = 0; i < NZ; i++) rhs[i] = -eps * v[i] + acc[S::P + i];
        rhs[NZ] = -1.0 + acc[S::P + NZ];
        // predictor
        chol_solve<NV>(M, dinv, rhs, dv);
        double ap = 1.0, ad = 1.0, dsla[R], dzla[R], dsua[R], dzua[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double td = dotz<NZ>(rw.g[r], *reinterpret_cast<const double(*)[NZ]>(dv));
            dsla[r] = rw.hl[r] ? td + dv[NZ] + rsl[r] : 0.0;
            dsua[r] = rw.hu[r] ? -td + dv[NZ] + rsu[r] : 0.0;
            dzla[r] = rw.hl[r] ? -zl[r] - Dl[r] * dsla[r] : 0.0;
            dzua[r] = rw.hu[r] ? -zu[r] - Du[r] * dsua[r] : 0.0;
            if (dsla[r] < 0.0) ap = fmin(ap, -sl[r] / dsla[r]);
            if (dsua[r] < 0.0) ap = fmin(ap, -su[r] / dsua[r]);
            if (dzla[r] < 0.0) ad = fmin(ad, -zl[r] / dzla[r]);
            if (dzua[r] < 0.0) ad = fmin(ad, -zu[r] / dzua[r]);
        }
        const double dsta = dv[NZ], dzta = -zt - Dt * dsta;
        if (dsta < 0.0) ap = fmin(ap, -st_ / dsta);
        if (dzta < 0.0) ad = fmin(ad, -zt / dzta);
        ap = grp_min<G>(ap);
        ad = grp_min<G>(ad);
        double mua = 0.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (rw.hl[r]) mua += (sl[r] + ap * dsla[r]) * (zl[r] + ad * dzla[r]);
            if (rw.hu[r]) mua += (su[r] + ap * dsua[r]) * (zu[r] + ad * dzua[r]);
        }
        mua = (grp_sum<G>(mua) + (st_ + ap * dsta) * (zt + ad * dzta)) * inv_ns;
        double sig = mu > 0.0 ? mua / mu : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        double vc[NV];
#pragma unroll
        for (int i = 0; i < NV; i++) vc[i] = 0.0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double cl = rw.hl[r] ? (smu - dsla[r] * dzla[r]) / sl[r] : 0.0;
            const double cu = rw.hu[r] ? (smu - dsua[r] * dzua[r]) / su[r] : 0.0;
#pragma unroll
            for (int i = 0; i < NZ; i++) vc[i] = fma(rw.g[r][i], cl - cu, vc[i]);
            vc[NZ] += cl + cu;
        }
        grp_sum_vec<G, NV>(vc);
        vc[NZ] += (smu - dsta * dzta) / st_;
        double dvc[NV];
        chol_solve<NV>(M, dinv, vc, dvc);
#pragma unroll
        for (int i = 0; i < NV; i++) dv[i] += dvc[i];
        double amax = 1e300, dsl[R], dzl[R], dsu[R], dzu[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double td = dotz<NZ>(rw.g[r], *reinterpret_cast<const double(*)[NZ]>(dv));
            dsl[r] = rw.hl[r] ? td + dv[NZ] + rsl[r] : 0.0;
            dsu[r] = rw.hu[r] ? -td + dv[NZ] + rsu[r] : 0.0;
            dzl[r] = rw.hl[r] ? (smu - sl[r] * zl[r] - dsla[r] * dzla[r] - zl[r] * dsl[r]) / sl[r] : 0.0;
            dzu[r] = rw.hu[r] ? (smu - su[r] * zu[r] - dsua[r] * dzua[r] - zu[r] * dsu[r]) / su[r] : 0.0;
            if (dsl[r] < 0.0) amax = fmin(amax, -sl[r] / dsl[r]);
            if (dsu[r] < 0.0) amax = fmin(amax, -su[r] / dsu[r]);
            if (dzl[r] < 0.0) amax = fmin(amax, -zl[r] / dzl[r]);
            if (dzu[r] < 0.0) amax = fmin(amax, -zu[r] / dzu[r]);
        }
        const double dst = dv[NZ];
        const double dzt = (smu - st_ * zt - dsta * dzta - zt * dst) / st_;
        if (dst < 0.0) amax = fmin(amax, -st_ / dst);
        if (dzt < 0.0) amax = fmin(amax, -zt / dzt);
        amax = grp_min<G>(amax);
        const double alpha = fmin(1.0, 0.99 * amax);
#pragma unroll
        for (int i = 0; i < NV; i++) v[i] = fma(alpha, dv[i], v[i]);
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (rw.hl[r]) {
                sl[r] = fmax(fma(alpha, dsl[r], sl[r]), 1e-300);
                zl[r] = fmax(fma(alpha, dzl[r], zl[r]), 1e-300);
            }
            if (rw.hu[r]) {
                su[r] = fmax(fma(alpha, dsu[r], su[r]), 1e-300);
                zu[r] = fmax(fma(alpha, dzu[r], zu[r]), 1e-300);
            }
        }
        st_ = fmax(fma(alpha, dst, st_), 1e-300);
        zt = fmax(fma(alpha, dzt, zt), 1e-300);
    }
    // t* from the iterate: the largest actual row violation at y (>= 0)
    double worst = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const double t = dotz<NZ>(rw.g[r], *reinterpret_cast<const double(*)[NZ]>(v));
        if (rw.hl[r]) worst = fmax(worst, rw.lo[r] - t);
        if (rw.hu[r]) worst = fmax(worst, t - rw.hi[r]);
    }
    return grp_max<G>(worst);
}

}  // namespace dev
}  // namespace mpccbf
