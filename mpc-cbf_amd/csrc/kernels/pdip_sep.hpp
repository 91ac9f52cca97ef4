// pdip_sep.hpp — the Mehrotra PDIP of pdip.hpp specialised to the dimension-separable MPC-CBF QP
// (base_config.json): reduced variables y = [y_x | y_y | y_yaw] with 2 per channel, objective
// block-diagonal by channel, every box row (acceleration / velocity bound at a sample) inside one
// channel and two-sided, and the collision-CBF rows one-sided and coupling x and y only
// (a = (2dx, 2dy, 0), ConnectivityCBF.cpp:152-198 — no yaw term).
//
// Lane layout (group of G = 16 lanes per agent): lane l holds box row l of each channel
// (SB slots per channel: rows l, l+16, ...) and CBF row l (CB slots). Unused slots hold inert
// rows (g = 0, -1 <= 0 <= 1 for box slots, 0 <= 1 for CBF slots), so no side masks are needed:
// such a row has constant slacks, its dual decays with mu, and it adds nothing to the Newton
// matrix or the right-hand side. Per Newton step a lane touches 3 normal-matrix entries per box
// row and 10 per CBF row, and the group all-reduces 20 values (x, y, yaw 2x2 blocks, the 2x2 x-y
// coupling, the right-hand side, the complementarity sum) — 16 when no CBF row is present —
// instead of the 28 of the dense 6x6 form. Factorisation: 4x4 (x, y) and 2x2 (yaw) Cholesky.
// Step lengths come from max(-ds/s, -dz/z) (one reciprocal per group, not one per row).
// Termination tests and statuses are those of pdip_solve.
#pragma once

#include "pdip.hpp"

namespace mpccbf {
namespace dev {

constexpr int SEP_D = 3;     // channels
constexpr int SEP_NZD = 2;   // reduced variables per channel
constexpr int SEP_NZ = SEP_D * SEP_NZD;

template <int SB, int CB>
struct SepRows {
    double bg[SEP_D][SB][SEP_NZD];  // box rows: coefficients on the own channel's columns
    double blo[SEP_D][SB], bhi[SEP_D][SB];
    double cg[CB][4];               // CBF rows: coefficients on (x0, x1, y0, y1); upper side only
    double chi[CB];
};

// accumulator layout of one Newton step
constexpr int A_MX = 0, A_MY = 3, A_MW = 6, A_MC = 9, A_RHS = 13, A_MU = 19, A_N = 20;

// 2x2 symmetric block (a00, a01, a11) += D g g^T
__device__ __forceinline__ void acc_blk2(double* a, double D, double g0, double g1) {
    const double d0 = D * g0;
    a[0] = fma(d0, g0, a[0]);
    a[1] = fma(d0, g1, a[1]);
    a[2] = fma(D * g1, g1, a[2]);
}

// Solve with the separable Newton matrix: 4x4 packed (x, y) factor + 2x2 packed yaw factor.
__device__ __forceinline__ void sep_solve(const double (&Mxy)[10], const double (&dxy)[4],
                                          const double (&Mw)[3], const double (&dw)[2],
                                          const double (&b)[6], double (&x)[6]) {
    double bx[4] = {b[0], b[1], b[2], b[3]}, xx[4];
    chol_solve<4>(Mxy, dxy, bx, xx);
    double bw[2] = {b[4], b[5]}, xw[2];
    chol_solve<2>(Mw, dw, bw, xw);
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = xx[i];
    x[4] = xw[0];
    x[5] = xw[1];
}

// P: 6x6 row-major block-diagonal reduced Hessian, LP its lower Cholesky factor (uniform).
// has_cbf: group-uniform flag (some CBF slot of the group is live); when false the CBF slots
// are skipped entirely (and do not count as sides).
template <int G, int SB, int CB>
__device__ PdipOut pdip_solve_sep(const SepRows<SB, CB>& rw, bool has_cbf, const double* __restrict__ P,
                                  const double* __restrict__ LP, const double (&q)[SEP_NZ],
                                  double (&y)[SEP_NZ], const PdipCfg cfg, long long* dbg = nullptr) {
    (void)dbg;
    // ---- start: unconstrained minimiser (block-diagonal P: per-channel 2x2 solves)
#pragma unroll
    for (int d = 0; d < SEP_D; d++) {
        const int o = 2 * d;
        const double l00 = LP[o * 6 + o], l10 = LP[(o + 1) * 6 + o], l11 = LP[(o + 1) * 6 + o + 1];
        const double w0 = -q[o] * rcp(l00);
        const double w1 = (-q[o + 1] - l10 * w0) * rcp(l11);
        y[o + 1] = w1 * rcp(l11);
        y[o] = (w0 - l10 * y[o + 1]) * rcp(l00);
    }
    // slacks (s) and duals (z): box lower / upper sides, CBF upper side
    double sl[SEP_D][SB], su[SEP_D][SB], zl[SEP_D][SB], zu[SEP_D][SB], cs[CB], cz[CB];
    double pl[SEP_D][SB], pu[SEP_D][SB], pc[CB];  // relative primal-residual scales
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const double t = rw.bg[d][k][0] * y[2 * d] + rw.bg[d][k][1] * y[2 * d + 1];
            sl[d][k] = fmax(t - rw.blo[d][k], 1.0);
            su[d][k] = fmax(rw.bhi[d][k] - t, 1.0);
            zl[d][k] = rcp(sl[d][k]);
            zu[d][k] = rcp(su[d][k]);
            pl[d][k] = rcp(1.0 + fabs(rw.blo[d][k]));
            pu[d][k] = rcp(1.0 + fabs(rw.bhi[d][k]));
        }
#pragma unroll
    for (int c = 0; c < CB; c++) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++) t = fma(rw.cg[c][j], y[j], t);
        cs[c] = fmax(rw.chi[c] - t, 1.0);
        cz[c] = rcp(cs[c]);
        pc[c] = rcp(1.0 + fabs(rw.chi[c]));
    }
    const double nsides = (double)(G * (2 * SEP_D * SB + (has_cbf ? CB : 0)));
    double qn = 0.0;
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) qn = fmax(qn, fabs(q[j]));
    const double inv_ns = 1.0 / nsides;
    const double inv_qn = rcp(1.0 + qn);

    PdipOut out{ST_UNKNOWN, 0};
    double mu0 = 1.0;
    double rd_track = 1e300;
    bool rd_exact = true;
    for (int it = 0;; it++) {
        PSTAMP(0);
        double acc[A_N], accr[SEP_NZ];
#pragma unroll
        for (int k = 0; k < A_N; k++) acc[k] = 0.0;
#pragma unroll
        for (int k = 0; k < SEP_NZ; k++) accr[k] = 0.0;
        double rp = 0.0;
        // per side: residual r, 1/s, D = z/s
        double rl[SEP_D][SB], ru[SEP_D][SB], il[SEP_D][SB], iu[SEP_D][SB];
        double cr[CB], ci[CB];
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const double g0 = rw.bg[d][k][0], g1 = rw.bg[d][k][1];
                const double t = g0 * y[2 * d] + g1 * y[2 * d + 1];
                rl[d][k] = t - rw.blo[d][k] - sl[d][k];
                ru[d][k] = rw.bhi[d][k] - t - su[d][k];
                il[d][k] = rcp(sl[d][k]);
                iu[d][k] = rcp(su[d][k]);
                const double Dl = zl[d][k] * il[d][k], Du = zu[d][k] * iu[d][k];
                const double wv = Du * ru[d][k] - Dl * rl[d][k];
                acc_blk2(acc + 3 * d, Dl + Du, g0, g1);
                acc[A_RHS + 2 * d] = fma(g0, wv, acc[A_RHS + 2 * d]);
                acc[A_RHS + 2 * d + 1] = fma(g1, wv, acc[A_RHS + 2 * d + 1]);
                acc[A_MU] = fma(sl[d][k], zl[d][k], fma(su[d][k], zu[d][k], acc[A_MU]));
                if (rd_exact) {
                    const double dz = zu[d][k] - zl[d][k];
                    accr[2 * d] = fma(g0, dz, accr[2 * d]);
                    accr[2 * d + 1] = fma(g1, dz, accr[2 * d + 1]);
                }
                rp = fmax(rp, fmax(fabs(rl[d][k]) * pl[d][k], fabs(ru[d][k]) * pu[d][k]));
            }
        if (has_cbf) {
#pragma unroll
            for (int c = 0; c < CB; c++) {
                const double* g = rw.cg[c];
                double t = 0.0;
#pragma unroll
                for (int j = 0; j < 4; j++) t = fma(g[j], y[j], t);
                cr[c] = rw.chi[c] - t - cs[c];
                ci[c] = rcp(cs[c]);
                const double D = cz[c] * ci[c];
                const double wv = D * cr[c];
                acc_blk2(acc + A_MX, D, g[0], g[1]);
                acc_blk2(acc + A_MY, D, g[2], g[3]);
                const double d0 = D * g[0], d1 = D * g[1];
                acc[A_MC + 0] = fma(d0, g[2], acc[A_MC + 0]);
                acc[A_MC + 1] = fma(d0, g[3], acc[A_MC + 1]);
                acc[A_MC + 2] = fma(d1, g[2], acc[A_MC + 2]);
                acc[A_MC + 3] = fma(d1, g[3], acc[A_MC + 3]);
#pragma unroll
                for (int j = 0; j < 4; j++) acc[A_RHS + j] = fma(g[j], wv, acc[A_RHS + j]);
                acc[A_MU] = fma(cs[c], cz[c], acc[A_MU]);
                if (rd_exact) {
#pragma unroll
                    for (int j = 0; j < 4; j++) accr[j] = fma(g[j], cz[c], accr[j]);
                }
                rp = fmax(rp, fabs(cr[c]) * pc[c]);
            }
            PSTAMP(1);
            grp_sum_vec<G, A_N>(acc);
        } else {
            // no CBF row in this group: the x-y coupling block stays zero
            double part[A_N - 4];
#pragma unroll
            for (int k = 0; k < A_MC; k++) part[k] = acc[k];
#pragma unroll
            for (int k = A_RHS; k < A_N; k++) part[k - 4] = acc[k];
            PSTAMP(1);
            grp_sum_vec<G, A_N - 4>(part);
#pragma unroll
            for (int k = 0; k < A_MC; k++) acc[k] = part[k];
#pragma unroll
            for (int k = A_RHS; k < A_N; k++) acc[k] = part[k - 4];
        }
        if (rd_exact) grp_sum_vec<G, SEP_NZ>(accr);
        PSTAMP(2);
        rp = grp_max<G>(rp);
        const double mu = acc[A_MU] * inv_ns;
        double py[SEP_NZ];
#pragma unroll
        for (int d = 0; d < SEP_D; d++) {
            const int o = 2 * d;
            py[o] = fma(P[o * 6 + o], y[o], fma(P[o * 6 + o + 1], y[o + 1], q[o]));
            py[o + 1] = fma(P[(o + 1) * 6 + o], y[o], fma(P[(o + 1) * 6 + o + 1], y[o + 1], q[o + 1]));
        }
        if (rd_exact) {
            double rdn = 0.0;
#pragma unroll
            for (int i = 0; i < SEP_NZ; i++) rdn = fmax(rdn, fabs(py[i] + accr[i]));
            rd_track = rdn * inv_qn;
            rd_exact = false;
        }
        out.iters = it;
        const bool finite = isfinite(rp) && isfinite(rd_track) && isfinite(mu) && isfinite(acc[0]);
        if (finite && rp <= cfg.tol && mu <= cfg.tol * 0.1) {
            if (rd_track <= cfg.tol) {
                double chk[SEP_NZ];
#pragma unroll
                for (int i = 0; i < SEP_NZ; i++) chk[i] = 0.0;
#pragma unroll
                for (int d = 0; d < SEP_D; d++)
#pragma unroll
                    for (int k = 0; k < SB; k++) {
                        const double dz = zu[d][k] - zl[d][k];
                        chk[2 * d] = fma(rw.bg[d][k][0], dz, chk[2 * d]);
                        chk[2 * d + 1] = fma(rw.bg[d][k][1], dz, chk[2 * d + 1]);
                    }
                if (has_cbf) {
#pragma unroll
                    for (int c = 0; c < CB; c++)
#pragma unroll
                        for (int j = 0; j < 4; j++) chk[j] = fma(rw.cg[c][j], cz[c], chk[j]);
                }
                grp_sum_vec<G, SEP_NZ>(chk);
                double rdn = 0.0;
#pragma unroll
                for (int i = 0; i < SEP_NZ; i++) rdn = fmax(rdn, fabs(py[i] + chk[i]));
                rd_track = rdn * inv_qn;
                if (rd_track <= cfg.tol) {
                    out.status = ST_OPTIMAL;
                    break;
                }
            }
        }
        if (it == 0) mu0 = mu;
        if (it >= cfg.maxit || !finite || mu > 1e8 * fmax(mu0, 1.0)) {
            out.status = ST_UNKNOWN;
            break;
        }
        PSTAMP(3);
        // ---- factor: (x, y) 4x4 with the CBF coupling, yaw 2x2
        double Mxy[10], dxy[4], Mw[3], dw[2];
        using S4 = Sym<4>;
        Mxy[S4::idx(0, 0)] = acc[A_MX + 0] + P[0 * 6 + 0];
        Mxy[S4::idx(0, 1)] = acc[A_MX + 1] + P[0 * 6 + 1];
        Mxy[S4::idx(1, 1)] = acc[A_MX + 2] + P[1 * 6 + 1];
        Mxy[S4::idx(2, 2)] = acc[A_MY + 0] + P[2 * 6 + 2];
        Mxy[S4::idx(2, 3)] = acc[A_MY + 1] + P[2 * 6 + 3];
        Mxy[S4::idx(3, 3)] = acc[A_MY + 2] + P[3 * 6 + 3];
        Mxy[S4::idx(0, 2)] = acc[A_MC + 0];
        Mxy[S4::idx(0, 3)] = acc[A_MC + 1];
        Mxy[S4::idx(1, 2)] = acc[A_MC + 2];
        Mxy[S4::idx(1, 3)] = acc[A_MC + 3];
        Mw[0] = acc[A_MW + 0] + P[4 * 6 + 4];
        Mw[1] = acc[A_MW + 1] + P[4 * 6 + 5];
        Mw[2] = acc[A_MW + 2] + P[5 * 6 + 5];
        const bool ok4 = chol_packed<4>(Mxy, dxy);
        const bool ok2 = chol_packed<2>(Mw, dw);
        if (!(ok4 && ok2)) {
            out.status = ST_UNKNOWN;
            break;
        }
        PSTAMP(4);
        // ---- predictor (affine) direction
        double rhs[SEP_NZ], dya[SEP_NZ];
#pragma unroll
        for (int i = 0; i < SEP_NZ; i++) rhs[i] = acc[A_RHS + i] - py[i];
        sep_solve(Mxy, dxy, Mw, dw, rhs, dya);
        PSTAMP(5);
        // ds = +-g dy + r,  dz = -z - D ds;  the largest -ds/s and -dz/z (= 1 + ds/s) give the
        // step to the boundary as their reciprocal
        double dsl[SEP_D][SB], dsu[SEP_D][SB], dzl[SEP_D][SB], dzu[SEP_D][SB], cds[CB], cdz[CB];
        double rs = 0.0, rz = 0.0;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const double td = rw.bg[d][k][0] * dya[2 * d] + rw.bg[d][k][1] * dya[2 * d + 1];
                dsl[d][k] = td + rl[d][k];
                dsu[d][k] = ru[d][k] - td;
                const double ql = dsl[d][k] * il[d][k], qu = dsu[d][k] * iu[d][k];
                dzl[d][k] = -zl[d][k] * (1.0 + ql);
                dzu[d][k] = -zu[d][k] * (1.0 + qu);
                rs = fmax(rs, fmax(-ql, -qu));
                rz = fmax(rz, fmax(1.0 + ql, 1.0 + qu));
            }
        if (has_cbf) {
#pragma unroll
            for (int c = 0; c < CB; c++) {
                double td = 0.0;
#pragma unroll
                for (int j = 0; j < 4; j++) td = fma(rw.cg[c][j], dya[j], td);
                cds[c] = cr[c] - td;
                const double qc = cds[c] * ci[c];
                cdz[c] = -cz[c] * (1.0 + qc);
                rs = fmax(rs, -qc);
                rz = fmax(rz, 1.0 + qc);
            }
        }
        grp_max2<G>(rs, rz);
        const double ap = rcp(fmax(1.0, rs)), ad = rcp(fmax(1.0, rz));
        PSTAMP(6);
        double mua = 0.0;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                mua = fma(sl[d][k] + ap * dsl[d][k], zl[d][k] + ad * dzl[d][k], mua);
                mua = fma(su[d][k] + ap * dsu[d][k], zu[d][k] + ad * dzu[d][k], mua);
            }
        if (has_cbf) {
#pragma unroll
            for (int c = 0; c < CB; c++) mua = fma(cs[c] + ap * cds[c], cz[c] + ad * cdz[c], mua);
        }
        mua = grp_sum<G>(mua) * inv_ns;
        double sig = mu > 0.0 ? mua * rcp(mu) : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        PSTAMP(7);
        // ---- corrector: sigma mu - ds_a dz_a per side, folded into the right-hand side
        double vc[SEP_NZ];
#pragma unroll
        for (int i = 0; i < SEP_NZ; i++) vc[i] = 0.0;
        double kl[SEP_D][SB], ku[SEP_D][SB], kc[CB];
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                kl[d][k] = smu - dsl[d][k] * dzl[d][k];
                ku[d][k] = smu - dsu[d][k] * dzu[d][k];
                const double w = kl[d][k] * il[d][k] - ku[d][k] * iu[d][k];
                vc[2 * d] = fma(rw.bg[d][k][0], w, vc[2 * d]);
                vc[2 * d + 1] = fma(rw.bg[d][k][1], w, vc[2 * d + 1]);
            }
        if (has_cbf) {
#pragma unroll
            for (int c = 0; c < CB; c++) {
                kc[c] = smu - cds[c] * cdz[c];
                const double w = -kc[c] * ci[c];
#pragma unroll
                for (int j = 0; j < 4; j++) vc[j] = fma(rw.cg[c][j], w, vc[j]);
            }
        }
        grp_sum_vec<G, SEP_NZ>(vc);
        PSTAMP(8);
        double dyc[SEP_NZ], dy[SEP_NZ];
        sep_solve(Mxy, dxy, Mw, dw, vc, dyc);
        PSTAMP(9);
#pragma unroll
        for (int i = 0; i < SEP_NZ; i++) dy[i] = dya[i] + dyc[i];
        // combined direction: ds from dy; dz = (k - s z - z ds) / s
        double rmax = 0.0;  // largest -ds/s, -dz/z over all sides
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const double td = rw.bg[d][k][0] * dy[2 * d] + rw.bg[d][k][1] * dy[2 * d + 1];
                dsl[d][k] = td + rl[d][k];
                dsu[d][k] = ru[d][k] - td;
                dzl[d][k] = (kl[d][k] - sl[d][k] * zl[d][k] - zl[d][k] * dsl[d][k]) * il[d][k];
                dzu[d][k] = (ku[d][k] - su[d][k] * zu[d][k] - zu[d][k] * dsu[d][k]) * iu[d][k];
                rmax = fmax(rmax, fmax(-dsl[d][k] * il[d][k], -dsu[d][k] * iu[d][k]));
                rmax = fmax(rmax, fmax(-dzl[d][k] * rcp_fast(zl[d][k]), -dzu[d][k] * rcp_fast(zu[d][k])));
            }
        if (has_cbf) {
#pragma unroll
            for (int c = 0; c < CB; c++) {
                double td = 0.0;
#pragma unroll
                for (int j = 0; j < 4; j++) td = fma(rw.cg[c][j], dy[j], td);
                cds[c] = cr[c] - td;
                cdz[c] = (kc[c] - cs[c] * cz[c] - cz[c] * cds[c]) * ci[c];
                rmax = fmax(rmax, fmax(-cds[c] * ci[c], -cdz[c] * rcp_fast(cz[c])));
            }
        }
        rmax = grp_max<G>(rmax);
        PSTAMP(10);
        // fraction to the boundary: alpha = min(1, 0.99 / rmax)
        const double alpha = 0.99 * rcp(fmax(0.99, rmax));
#pragma unroll
        for (int i = 0; i < SEP_NZ; i++) y[i] = fma(alpha, dy[i], y[i]);
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                sl[d][k] = fmax(fma(alpha, dsl[d][k], sl[d][k]), 1e-300);
                su[d][k] = fmax(fma(alpha, dsu[d][k], su[d][k]), 1e-300);
                zl[d][k] = fmax(fma(alpha, dzl[d][k], zl[d][k]), 1e-300);
                zu[d][k] = fmax(fma(alpha, dzu[d][k], zu[d][k]), 1e-300);
            }
        if (has_cbf) {
#pragma unroll
            for (int c = 0; c < CB; c++) {
                cs[c] = fmax(fma(alpha, cds[c], cs[c]), 1e-300);
                cz[c] = fmax(fma(alpha, cdz[c], cz[c]), 1e-300);
            }
        }
        rd_track *= (1.0 - alpha);
        if (it % 8 == 7) rd_exact = true;
        PSTAMP(11);
    }
    return out;
}

// Phase 1 on the separable rows: expand to the dense row form and reuse pdip_phase1 (only runs
// for QPs whose main solve did not converge).
template <int G, int SB, int CB>
__device__ double pdip_phase1_sep(const SepRows<SB, CB>& rw, const PdipCfg cfg) {
    constexpr int R = SEP_D * SB + CB;
    Rows<SEP_NZ, R> dr;
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const int r = d * SB + k;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) dr.g[r][j] = 0.0;
            dr.g[r][2 * d] = rw.bg[d][k][0];
            dr.g[r][2 * d + 1] = rw.bg[d][k][1];
            dr.lo[r] = rw.blo[d][k];
            dr.hi[r] = rw.bhi[d][k];
            dr.ml[r] = 1.0;
            dr.mu[r] = 1.0;
        }
#pragma unroll
    for (int c = 0; c < CB; c++) {
        const int r = SEP_D * SB + c;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) dr.g[r][j] = j < 4 ? rw.cg[c][j] : 0.0;
        dr.lo[r] = 0.0;
        dr.ml[r] = 0.0;
        dr.hi[r] = rw.chi[c];
        dr.mu[r] = 1.0;
    }
    return pdip_phase1<SEP_NZ, G, R>(dr, cfg);
}

}  // namespace dev
}  // namespace mpccbf
