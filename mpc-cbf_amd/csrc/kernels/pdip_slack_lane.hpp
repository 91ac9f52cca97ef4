// pdip_slack_lane.hpp — Mehrotra PDIP of a CBF-only QP (3 control variables) in slack mode, one
// 16-lane group per QP, one slack variable per lane.
//
// Used by the batched CBF-only controllers (cbf_control.hip): FovControl in slack mode
// (FovControl.cpp:25-62: the 4 FoV rows of neighbour i carry -v_i) and ConnectivityControl in
// slack mode (ConnectivityControl.cpp:31-83: the safety and CLF rows of neighbour i carry -v_i,
// the connectivity row the last slack). Problem per group:
//   min 1/2 u^T (2 I) u + q^T u + sum_l w_l v_l
//   s.t. g_la^T u - v_l <= h_la   (lane l, slack rows a < NSR; inert when live = 0)
//        lo_l <= o_l^T u <= hi_l  (one ordinary row per lane: velocity CBFs, control bounds;
//                                  inert rows 0 in [-1, 1]; ml / mu = 0 drop a side)
//        v_l >= 0                 (lanes with son = true)
// Lane l eliminates v_l from the Newton system lane-locally in the centred form of
// pdip_wave.hpp (WaveSlack): with D_a = z_a / s_a (live rows), T = sum D_a, Db = zb / sb,
// S = T + Db and gbar = sum D_a g_a / T,
//   sum_a D_a (g_a - gbar)(g_a - gbar)^T + (T Db / S) gbar gbar^T
// enters the 3x3 Newton matrix, and every right-hand side takes sum_a (g_a - gbar) phi_a
// + gbar (Db sum phi_a + T c) / S: positive terms only, no cancellation when a row is nearly
// active while its slack is in use. The Newton matrix, right-hand side and complementarity are
// one 10-value group reduction per step.
#pragma once

#include "group.hpp"
#include "pdip.hpp"

namespace mpccbf {
namespace dev {

// Accepted dual residual at primal convergence in slack mode: the recovered duals of strongly
// active slack rows carry the rounding of the elimination (see pdip_wave.hpp MPCCBF_SLK_RD).
constexpr double SLACK_LANE_RD_FLOOR = 1e-6;

struct SlackLaneOut {
    int status;
    int iters;
    double vcost;  // sum_l w_l v_l (group total)
};

template <int NSR, int G = 16>
__device__ SlackLaneOut pdip_slack_lane(const double (&g)[NSR][3], const double (&h)[NSR],
                                        const double (&live)[NSR], bool son, double w,
                                        const Rows<3, 1>& orw, const double (&q)[3], double (&y)[3],
                                        const PdipCfg cfg, double feas_tol) {
    constexpr int NZ = 3;
    using S3 = Sym<NZ>;
    auto dot3 = [](const double* a, const double* b) { return fma(a[0], b[0], fma(a[1], b[1], a[2] * b[2])); };
    const double og[3] = {orw.g[0][0], orw.g[0][1], orw.g[0][2]};
    const double olo = orw.lo[0], ohi = orw.hi[0], oml = orw.ml[0], omu = orw.mu[0];
    // start: the unconstrained minimiser -P^{-1} q (P = 2 I)
#pragma unroll
    for (int d = 0; d < NZ; d++) y[d] = -0.5 * q[d];
    double osl, osu, ozl, ozu;
    {
        const double t = dot3(og, y);
        osl = oml > 0.0 ? fmax(t - olo, 1.0) : 1.0;
        osu = omu > 0.0 ? fmax(ohi - t, 1.0) : 1.0;
        ozl = oml * rcp(osl);
        ozu = omu * rcp(osu);
    }
    const double opl = oml * rcp(1.0 + fabs(olo)), opu = omu * rcp(1.0 + fabs(ohi));
    // slack pair started centred (sb zb = 1), zb at the cost the bound carries when no row is active
    double zb = son ? fmax(w, 1.0) : 1.0;
    double sb = rcp(zb), v = son ? sb : 0.0;
    double cs[NSR], cz[NSR], pc[NSR];
#pragma unroll
    for (int r = 0; r < NSR; r++) {
        cs[r] = fmax(h[r] - (dot3(g[r], y) - live[r] * v), 1.0);
        cz[r] = rcp(cs[r]);
        pc[r] = rcp(1.0 + fabs(h[r]));
    }
    const double inv_ns = rcp(grp_sum<G>(oml + omu + (double)NSR + (son ? 1.0 : 0.0)));
    double qn = 0.0;
#pragma unroll
    for (int d = 0; d < NZ; d++) qn = fmax(qn, fabs(q[d]));
    const double inv_qn = rcp(1.0 + qn);
    SlackLaneOut out{ST_UNKNOWN, 0, 0.0};
    double mu0 = 1.0;
    for (int it = 0;; it++) {
        constexpr int NM = S3::P, NA = NM + NZ + 1;
        double acc[NA], accr[NZ];
#pragma unroll
        for (int k = 0; k < NA; k++) acc[k] = 0.0;
#pragma unroll
        for (int k = 0; k < NZ; k++) accr[k] = 0.0;
        // ordinary row
        const double ot = dot3(og, y);
        const double orl = oml * (ot - olo - osl), oru = omu * (ohi - ot - osu);
        const double oil = rcp(osl), oiu = rcp(osu);
        const double oDl = ozl * oil, oDu = ozu * oiu;
        {
            const double D = oDl + oDu, wv = oDu * oru - oDl * orl;
#pragma unroll
            for (int i = 0; i < NZ; i++) {
#pragma unroll
                for (int j = i; j < NZ; j++) acc[S3::idx(i, j)] = fma(D * og[i], og[j], acc[S3::idx(i, j)]);
                acc[NM + i] = fma(og[i], wv, acc[NM + i]);
                accr[i] = fma(og[i], ozu - ozl, accr[i]);
            }
            acc[NA - 1] = fma(osl, ozl, osu * ozu);
        }
        double rp = fmax(fabs(orl) * opl, fabs(oru) * opu);
        // slack rows: residual cr = h - g u + v - s, centred weights
        double cr[NSR], ci[NSR], Dl[NSR];
        double T = 0.0, SR = 0.0, gb[NZ] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < NSR; r++) {
            cr[r] = h[r] - dot3(g[r], y) + live[r] * v - cs[r];
            ci[r] = rcp(cs[r]);
            Dl[r] = live[r] * cz[r] * ci[r];
            T += Dl[r];
            SR = fma(Dl[r], cr[r], SR);
#pragma unroll
            for (int d = 0; d < NZ; d++) {
                gb[d] = fma(Dl[r], g[r][d], gb[d]);
                accr[d] = fma(g[r][d], live[r] * cz[r], accr[d]);
            }
            acc[NA - 1] = fma(cs[r], cz[r], acc[NA - 1]);
            rp = fmax(rp, fabs(cr[r]) * pc[r]);
        }
        const double iT = T > 0.0 ? rcp(T) : 0.0;
#pragma unroll
        for (int d = 0; d < NZ; d++) gb[d] *= iT;
        const double isb = rcp(sb);
        const double Db = son ? zb * isb : 0.0, rb = son ? v - sb : 0.0;
        const double iS = son ? rcp(T + Db) : 0.0;
        double c[NSR][NZ];
#pragma unroll
        for (int r = 0; r < NSR; r++) {
#pragma unroll
            for (int d = 0; d < NZ; d++) c[r][d] = g[r][d] - gb[d];
#pragma unroll
            for (int i = 0; i < NZ; i++) {
                const double dc = Dl[r] * c[r][i];
#pragma unroll
                for (int j = i; j < NZ; j++) acc[S3::idx(i, j)] = fma(dc, c[r][j], acc[S3::idx(i, j)]);
                acc[NM + i] = fma(c[r][i], Dl[r] * cr[r], acc[NM + i]);
            }
        }
        {
            const double wm = T * Db * iS;
            const double fm = (Db * SR - T * fma(Db, rb, w)) * iS;
#pragma unroll
            for (int i = 0; i < NZ; i++) {
#pragma unroll
                for (int j = i; j < NZ; j++) acc[S3::idx(i, j)] = fma(wm * gb[i], gb[j], acc[S3::idx(i, j)]);
                acc[NM + i] = fma(gb[i], fm, acc[NM + i]);
            }
        }
        if (son) {
            acc[NA - 1] = fma(sb, zb, acc[NA - 1]);
            rp = fmax(rp, fabs(rb));
        }
        grp_sum_vec<G, NA>(acc);
        grp_sum_vec<G, NZ>(accr);
        rp = grp_max<G>(rp);
        const double mu = acc[NA - 1] * inv_ns;
        double py[NZ];
#pragma unroll
        for (int d = 0; d < NZ; d++) py[d] = fma(2.0, y[d], q[d]);
        double zsum = 0.0;
#pragma unroll
        for (int r = 0; r < NSR; r++) zsum = fma(live[r], cz[r], zsum);
        const double rv = son ? fabs(w - zsum - zb) * rcp(1.0 + w) : 0.0;
        double rdn = 0.0;
#pragma unroll
        for (int d = 0; d < NZ; d++) rdn = fmax(rdn, fabs(py[d] + accr[d]));
        const double rd = fmax(rdn * inv_qn, grp_max<G>(rv));  // exact every step (cheap here)
        out.iters = it;
        const bool finite = isfinite(rp) && isfinite(rd) && isfinite(mu) && isfinite(acc[0]);
        if (finite && rp <= cfg.tol && mu <= cfg.tol * 0.1 && rd <= fmax(cfg.tol, SLACK_LANE_RD_FLOOR)) {
            out.status = ST_OPTIMAL;
            break;
        }
        if (it == 0) mu0 = mu;
        if (it >= cfg.maxit || !finite || mu > 1e8 * fmax(mu0, 1.0)) {
            out.status = ST_UNKNOWN;
            break;
        }
        double M[NM], dinv[NZ];
#pragma unroll
        for (int i = 0; i < NZ; i++)
#pragma unroll
            for (int j = i; j < NZ; j++) M[S3::idx(i, j)] = acc[S3::idx(i, j)] + (i == j ? 2.0 : 0.0);
        if (!chol_packed<NZ>(M, dinv)) {  // shifted refactorisation (see pdip_wave.hpp)
            const double tau =
                1e-12 * fmax(fmax(acc[S3::idx(0, 0)], acc[S3::idx(1, 1)]), acc[S3::idx(2, 2)]);
#pragma unroll
            for (int i = 0; i < NZ; i++)
#pragma unroll
                for (int j = i; j < NZ; j++) M[S3::idx(i, j)] = acc[S3::idx(i, j)] + (i == j ? 2.0 + tau : 0.0);
            if (!chol_packed<NZ>(M, dinv)) {
                out.status = ST_UNKNOWN;
                break;
            }
        }
        // ---- predictor
        double rhs[NZ], dya[NZ];
#pragma unroll
        for (int d = 0; d < NZ; d++) rhs[d] = acc[NM + d] - py[d];
        chol_solve<NZ>(M, dinv, rhs, dya);
        double ap = 1.0, ad = 1.0;
        const double otd = dot3(og, dya);
        const double odsl = oml * (otd + orl), odsu = omu * (oru - otd);
        const double odzl = -ozl - oDl * odsl, odzu = -ozu - oDu * odsu;
        ap = fmin(ap, fmin(step_bound(osl, odsl, 1.0), step_bound(osu, odsu, 1.0)));
        ad = fmin(ad, fmin(step_bound(ozl, odzl, 1.0), step_bound(ozu, odzu, 1.0)));
        // slack rows: dv = (sum_a D_a (g_a du - cr_a) - Db rb - w) / S, ds = cr - g du + dv
        double sd = 0.0;
#pragma unroll
        for (int r = 0; r < NSR; r++) sd = fma(Dl[r], dot3(g[r], dya) - cr[r], sd);
        const double dva = (sd - fma(Db, rb, w)) * iS;
        double dsa[NSR], dza[NSR];
#pragma unroll
        for (int r = 0; r < NSR; r++) {
            dsa[r] = cr[r] - dot3(g[r], dya) + live[r] * dva;
            dza[r] = -cz[r] * (1.0 + dsa[r] * ci[r]);
            ap = fmin(ap, step_bound(cs[r], dsa[r], 1.0));
            ad = fmin(ad, step_bound(cz[r], dza[r], 1.0));
        }
        const double dsba = son ? dva + rb : 0.0;
        const double dzba = son ? -zb * (1.0 + dsba * isb) : 0.0;
        if (son) {
            ap = fmin(ap, step_bound(sb, dsba, 1.0));
            ad = fmin(ad, step_bound(zb, dzba, 1.0));
        }
        ap = grp_min<G>(ap);
        ad = grp_min<G>(ad);
        double mua = fma(osl + ap * odsl, ozl + ad * odzl, (osu + ap * odsu) * (ozu + ad * odzu));
#pragma unroll
        for (int r = 0; r < NSR; r++) mua = fma(cs[r] + ap * dsa[r], cz[r] + ad * dza[r], mua);
        if (son) mua = fma(sb + ap * dsba, zb + ad * dzba, mua);
        mua = grp_sum<G>(mua) * inv_ns;
        double sig = mu > 0.0 ? mua * rcp(mu) : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        // ---- corrector right-hand side (slack rows: weights om = -kc / s, centred; the mean
        // row takes (Db sum om + T kb / sb) / S; the v equation keeps -sum om + kb / sb)
        const double ocl = oml * (smu - odsl * odzl), ocu = omu * (smu - odsu * odzu);
        double vc[NZ];
        {
            const double wo = ocl * oil - ocu * oiu;
#pragma unroll
            for (int d = 0; d < NZ; d++) vc[d] = og[d] * wo;
        }
        double kc[NSR], som = 0.0;
#pragma unroll
        for (int r = 0; r < NSR; r++) {
            kc[r] = smu - dsa[r] * dza[r];
            const double om = -live[r] * kc[r] * ci[r];
            som += om;
#pragma unroll
            for (int d = 0; d < NZ; d++) vc[d] = fma(c[r][d], om, vc[d]);
        }
        const double kb = son ? smu - dsba * dzba : 0.0;
        const double vcv = fma(kb, isb, -som);
        {
            const double fm = fma(Db, som, T * kb * isb) * iS;
#pragma unroll
            for (int d = 0; d < NZ; d++) vc[d] = fma(gb[d], fm, vc[d]);
        }
        grp_sum_vec<G, NZ>(vc);
        double dyc[NZ], dy[NZ];
        chol_solve<NZ>(M, dinv, vc, dyc);
#pragma unroll
        for (int d = 0; d < NZ; d++) dy[d] = dya[d] + dyc[d];
        // ---- combined direction, fraction to the boundary
        double amax = 1e300;
        const double otc = dot3(og, dy);
        const double odl = oml * (otc + orl), odu = omu * (oru - otc);
        const double ozdl = (ocl - osl * ozl - ozl * odl) * oil, ozdu = (ocu - osu * ozu - ozu * odu) * oiu;
        amax = fmin(amax, fmin(step_bound(osl, odl, 1e300), step_bound(osu, odu, 1e300)));
        amax = fmin(amax, fmin(step_bound(ozl, oml * ozdl, 1e300), step_bound(ozu, omu * ozdu, 1e300)));
        sd = 0.0;
#pragma unroll
        for (int r = 0; r < NSR; r++) sd = fma(Dl[r], dot3(g[r], dy) - cr[r], sd);
        const double dv = (sd - fma(Db, rb, w) + vcv) * iS;
        double ds[NSR], dz[NSR];
#pragma unroll
        for (int r = 0; r < NSR; r++) {
            ds[r] = cr[r] - dot3(g[r], dy) + live[r] * dv;
            dz[r] = (kc[r] - cs[r] * cz[r] - cz[r] * ds[r]) * ci[r];
            amax = fmin(amax, fmin(step_bound(cs[r], ds[r], 1e300), step_bound(cz[r], dz[r], 1e300)));
        }
        const double dsb = son ? dv + rb : 0.0;
        const double dzb = son ? (kb - sb * zb - zb * dsb) * isb : 0.0;
        if (son) amax = fmin(amax, fmin(step_bound(sb, dsb, 1e300), step_bound(zb, dzb, 1e300)));
        amax = grp_min<G>(amax);
        const double alpha = fmin(1.0, 0.99 * amax);
#pragma unroll
        for (int d = 0; d < NZ; d++) y[d] = fma(alpha, dy[d], y[d]);
        osl = fmax(fma(alpha, odl, osl), 1e-300);
        osu = fmax(fma(alpha, odu, osu), 1e-300);
        ozl = oml * fmax(fma(alpha, ozdl, ozl), 1e-300);
        ozu = omu * fmax(fma(alpha, ozdu, ozu), 1e-300);
#pragma unroll
        for (int r = 0; r < NSR; r++) {
            cs[r] = fmax(fma(alpha, ds[r], cs[r]), 1e-300);
            cz[r] = fmax(fma(alpha, dz[r], cz[r]), 1e-300);
        }
        if (son) {
            v = fma(alpha, dv, v);
            sb = fmax(fma(alpha, dsb, sb), 1e-300);
            zb = fmax(fma(alpha, dzb, zb), 1e-300);
        }
    }
    if (out.status != ST_OPTIMAL) {
        // the slack rows are always satisfiable: phase 1 certifies the ordinary rows
        const double tstar = pdip_phase1<NZ, G, 1>(orw, cfg);
        out.status = (tstar > feas_tol && tstar < 1e300) ? ST_INFEASIBLE : ST_UNKNOWN;
    }
    out.vcost = grp_sum<G>(son ? w * v : 0.0);
    return out;
}

// Stable rank order of the group's keys (ties by lane) and the reference's slack weight
// w_l = cost * decay^{idx[l]}, idx = the sorted list of lanes (FovControl.cpp:25-46,
// FovBezierIMPCCBF.cpp:58-81: the weight of neighbour l uses the index of the l-th smallest).
template <int G = 16>
__device__ double sorted_slack_weight(double key, bool on, int n, int gl, double cost, double decay) {
    int rank = 0;
#pragma unroll
    for (int j = 0; j < G; j++) {
        const double kj = __shfl(key, j, G);
        rank += (on && j < n && (kj < key || (kj == key && j < gl))) ? 1 : 0;
    }
    int idx = 0;
#pragma unroll
    for (int m = 0; m < G; m++) {
        const int rm = __shfl(rank, m, G);
        idx = (m < n && rm == gl) ? m : idx;
    }
    return on ? cost * pow(decay, (double)idx) : 0.0;
}

}  // namespace dev
}  // namespace mpccbf
