// impc_kernel.hip — one fused launch per control step: ConnectivityIMPCCBF::optimize for a
// batch of agents (mpc_cbf/src/controller/ConnectivityIMPCCBF.cpp:47-215).
//
// Mapping (gfx950, wave64): one agent per group of G lanes. Per agent:
//   1. state-dependent parts of the condensed QP: q = Qs s0 + Qt t, shared row bounds shifted by
//      Gs s0, constant-row feasibility (e.g. the k = 0 velocity bound, which the initial-state
//      equality pins);
//   2. IMPC iteration 0: closed-form safety-CBF rows at the current state
//      (ConnectivityCBF.cpp:152-198 via ConnectivityMPCCBFQPOperations.cpp:192-205), exact
//      redundancy filter, compaction into the group's LDS staging area, PDIP solve;
//   3. IMPC iteration 1 (only after OPTIMAL, :158): predicted ego states from iteration 0's curve
//      at h_samples(k), k < cbf_horizon (:161-168), CBF rows per (neighbour, k) (:252-272), solve;
//   4. outputs: per-iteration status/objective/iterations, control points of the kept curve
//      (x = Xs s0 + Z y), and the closed-loop next state (curve at t = h).
// Two solver layouts share steps 1-4:
//   impc_sep_kernel — dimension-separable operators (base_config.json): G = 16 lanes, lane l holds
//                     box row l of each channel and CBF row l; pdip_sep.hpp;
//   impc_kernel     — any operators: rows spread over G lanes x R slots, dense NZ x NZ normal
//                     matrix; pdip.hpp.
// Shared operators are read through the scalar/L1/L2 path (uniform addresses); per-agent inputs
// are a 48-byte state, a 24-byte target and the neighbour states (gathered, L2-resident).
#include <hip/hip_runtime.h>

#include <cmath>

#include "impc.hpp"
#include "impc_common.hpp"
#include "impc_wide.hpp"
#include "pdip.hpp"
#include "pdip_sep.hpp"

namespace mpccbf {
namespace dev {

// ---------------------------------------------------------------------------------------------
// Dense layout (any operators)
// ---------------------------------------------------------------------------------------------
template <int NZ, int G, int R>
__global__ void __launch_bounds__(256) impc_kernel(const DevOps op, const double* __restrict__ buf,
                                                    const ImpcArgs args) {
    constexpr int GPB = 256 / G;
    const int gl = threadIdx.x & (G - 1);
    const int gib = threadIdx.x / G;
    const int ai = blockIdx.x * GPB + gib;  // agent index within the batch
    grid_clear<256>(args);
    if (ai >= args.num_agents) return;      // whole group leaves together
    stamp(args, ai, gl, 0);

    extern __shared__ double lds_stage[];
    const int cap = R * G - op.m;  // CBF row slots per agent
    double* stage = lds_stage + (size_t)gib * cap * (NZ + 1);

    const int self = args.agent_first + ai;
    double s0[6];
#pragma unroll
    for (int i = 0; i < 6; i++) s0[i] = args.states[(size_t)self * 6 + i];
    double q[NZ], kconst;
    agent_linear_term<NZ>(op, buf, args, ai, s0, q, kconst);

    // ---- shared rows into register slots
    Rows<NZ, R> rw;
    {
        const double* Gm = opp(buf, op.o_G);
        const double* Gs = opp(buf, op.o_Gs);
        const double* lo = opp(buf, op.o_lo);
        const double* hi = opp(buf, op.o_hi);
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int slot = r * G + gl;
            const bool on = slot < op.m;
            const int si = on ? slot : 0;
            double sh = 0.0;
#pragma unroll
            for (int s = 0; s < 6; s++) sh = fma(Gs[si * 6 + s], s0[s], sh);
#pragma unroll
            for (int j = 0; j < NZ; j++) rw.g[r][j] = on ? Gm[si * NZ + j] : 0.0;
            const double l = lo[si], h = hi[si];
            const bool hl = on && l > -1e300, hu = on && h < 1e300;
            rw.ml[r] = hl ? 1.0 : 0.0;
            rw.mu[r] = hu ? 1.0 : 0.0;
            rw.lo[r] = hl ? l - sh : 0.0;
            rw.hi[r] = hu ? h - sh : 0.0;
        }
    }
    const bool infeasible = constant_rows_infeasible<G>(op, buf, s0, gl);
    stamp(args, ai, gl, 1);

    // ---- neighbours: CSR (caller-provided, e.g. all N-1 others as the reference does) or the
    // k nearest within the radius from the spatial hash (3 x 3 cells around the agent)
    const bool grid_mode = args.nb_row_ptr == nullptr;
    int nb0 = 0, nnb = 0;
    __shared__ NbScratch nb_scratch[GPB];
    if (!grid_mode) {
        nb0 = args.nb_row_ptr[ai];
        nnb = args.nb_row_ptr[ai + 1] - nb0;
    } else {
        nnb = grid_neighbors<G>(args, self, s0[0], s0[1], nb_scratch[gib], gl);
    }
    const bool nb_overflow = nnb < 0;
    if (nb_overflow) nnb = 0;
    write_nb_out(args, ai, gl, grid_mode, nb_scratch[gib], nb0, nnb);
    stamp(args, ai, gl, 2);

    double y[NZ], ykeep[NZ];
#pragma unroll
    for (int i = 0; i < NZ; i++) y[i] = ykeep[i] = 0.0;
    bool have_curve = false, success = true;
    const PdipCfg cfg{op.maxit, op.tol};

    for (int it = 0; it < op.impc_iter; it++) {
        const size_t oi = (size_t)ai * op.impc_iter + it;
        if (!success) {  // the reference breaks out of the IMPC loop (:208-211)
            write_iteration(args, oi, gl, ST_UNKNOWN, __builtin_nan(""), 0);
            continue;
        }
        bool row_infeasible = false;
        const int count = stage_cbf_rows<NZ, G>(op, buf, args, it, s0, y, grid_mode, &nb_scratch[gib],
                                                nb0, nnb, stage, cap, gl, &row_infeasible);
        if (it < 2) stamp(args, ai, gl, 3 + 2 * it);
        // ---- CBF rows into the free slots (previous iteration's CBF rows are replaced)
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int slot = r * G + gl;
            if (slot >= op.m) {
                const int ci = slot - op.m;
                const bool on = ci < count && ci < cap;
                const double* src = stage + (size_t)(on ? ci : 0) * (NZ + 1);
#pragma unroll
                for (int jz = 0; jz < NZ; jz++) rw.g[r][jz] = on ? src[jz] : 0.0;
                rw.ml[r] = 0.0;
                rw.mu[r] = on ? 1.0 : 0.0;
                rw.lo[r] = 0.0;
                rw.hi[r] = on ? src[NZ] : 0.0;
            }
        }
        int st;
        int nit = 0;
        double prs = __builtin_nan(""), drs = __builtin_nan("");
        bool nfin = false;  // non-finite data: not solved, ERROR (see impc_sep_agent)
#pragma unroll
        for (int j = 0; j < NZ; j++) nfin = nfin || !isfinite(q[j]);
#pragma unroll
        for (int r = 0; r < R; r++) {
            nfin = nfin || !isfinite(rw.lo[r]) || !isfinite(rw.hi[r]);
#pragma unroll
            for (int j = 0; j < NZ; j++) nfin = nfin || !isfinite(rw.g[r][j]);
        }
        if (count > cap || nb_overflow || grp_ballot<G>(nfin) != 0ull) {
            st = ST_ERROR;  // capacity (CBF rows beyond this instantiation's slots) / non-finite data
        } else if (infeasible || row_infeasible) {
            st = ST_INFEASIBLE;
        } else {
            const PdipOut po =
                pdip_solve<NZ, G, R>(rw, opp(buf, op.o_Pr), opp(buf, op.o_LPr), q, y, cfg);
            st = po.status;
            nit = po.iters;
            prs = po.rp;
            drs = po.rd;
            if (st != ST_OPTIMAL) {
                // certify: minimal uniform row violation above the feasibility tolerance
                const double tstar = pdip_phase1<NZ, G, R>(rw, cfg);
                if (tstar > op.feas_tol) {
                    st = ST_INFEASIBLE;
                    prs = tstar;
                }
            }
        }
        double objv = __builtin_nan("");
        if (st == ST_OPTIMAL) {
            objv = reduced_objective<NZ>(op, buf, q, y, kconst);
#pragma unroll
            for (int i = 0; i < NZ; i++) ykeep[i] = y[i];
            have_curve = true;
        } else {
            success = false;
        }
        write_iteration(args, oi, gl, st, objv, nit, prs, drs);
        if (it < 2) stamp(args, ai, gl, 4 + 2 * it);
        wave_lds_sync();  // staging is rewritten by the next iteration
    }
    write_agent_outputs<NZ, G>(op, buf, args, ai, gl, s0, ykeep, have_curve);
    stamp(args, ai, gl, 7);
}

// ---------------------------------------------------------------------------------------------
// Separable layout (x / y / yaw channels, 2 reduced variables each; pdip_sep.hpp)
// ---------------------------------------------------------------------------------------------
// Slack mode: a lane builds the CBF rows of its neighbour (list position jn, -1: none) itself
// (slot k = sample k), so all rows of one slack variable live in the lane that owns it. Filtered
// rows stay inert (ccv = 0). Returns whether some row of this lane is live.
template <int SB, int CB>
__device__ bool lane_cbf_rows(const DevOps& op, const double* buf, const ImpcArgs& args, int it,
                              const double (&s0)[6], const double (&y)[SEP_NZ], bool grid_mode,
                              const int32_t* nbl, int nb0, int jn, SepRows<SB, CB>& rw) {
    const double* UZ = opp(buf, op.o_UZ);
    const double* US = opp(buf, op.o_US);
    const int nk = (it == 0) ? 1 : op.cbf_h;
    bool live = false;
#pragma unroll
    for (int k = 0; k < CB; k++) {
#pragma unroll
        for (int j = 0; j < 4; j++) rw.cg[k][j] = 0.0;
        rw.chi[k] = 1.0;
        rw.ccv[k] = 0.0;
        if (k < nk && jn >= 0) {
            double e[6];
            cbf_ego_state<SEP_NZ>(op, buf, it, k, s0, y, e);
            const int nbi = grid_mode ? nbl[jn] : args.nb_col[nb0 + jn];
            const double* ns = args.states + (size_t)nbi * 6;
            double a[3], b;
            safety_cbf(e, ns[0], ns[1], ns[3], ns[4], op.d_min, a, b);
            double bmax = 0.0;
#pragma unroll
            for (int d = 0; d < 3; d++) bmax += fmax(-a[d] * op.a_lo[d], -a[d] * op.a_hi[d]);
            if (!(op.cbf_filter && b >= bmax)) {  // implied by the acceleration box: drop
                const double* UZk = UZ + (size_t)k * 3 * SEP_NZ;
                const double* USk = US + (size_t)k * 18;
                double us = 0.0;
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    double v = 0.0;
#pragma unroll
                    for (int s = 0; s < 6; s++) v = fma(USk[d * 6 + s], s0[s], v);
                    us = fma(a[d], v, us);
                }
#pragma unroll
                for (int j = 0; j < 4; j++)
                    rw.cg[k][j] = -(a[0] * UZk[j] + a[1] * UZk[SEP_NZ + j] + a[2] * UZk[2 * SEP_NZ + j]);
                rw.chi[k] = b + us;
                rw.ccv[k] = 1.0;
                live = true;
            }
        }
    }
    return live;
}

// Whether neighbour jn (-1: none) has a CBF row the acceleration box does not imply (the filter of
// lane_cbf_rows without the row coefficients).
__device__ bool lane_cbf_live(const DevOps& op, const double* buf, const ImpcArgs& args, int it,
                              const double (&s0)[6], const double (&y)[SEP_NZ], bool grid_mode,
                              const int32_t* nbl, int nb0, int jn) {
    if (jn < 0) return false;
    const int nk = (it == 0) ? 1 : op.cbf_h;
    const int nbi = grid_mode ? nbl[jn] : args.nb_col[nb0 + jn];
    const double* ns = args.states + (size_t)nbi * 6;
    bool live = false;
    for (int k = 0; k < nk; k++) {
        double e[6], a[3], b;
        cbf_ego_state<SEP_NZ>(op, buf, it, k, s0, y, e);
        safety_cbf(e, ns[0], ns[1], ns[3], ns[4], op.d_min, a, b);
        double bmax = 0.0;
#pragma unroll
        for (int d = 0; d < 3; d++) bmax += fmax(-a[d] * op.a_lo[d], -a[d] * op.a_hi[d]);
        live = live || !(op.cbf_filter && b >= bmax);
    }
    return live;
}

template <int G>
__device__ double lane_slack_weight(const DevOps& op, const ImpcArgs& args, const double (&s0)[6],
                                    bool grid_mode, const int32_t* nbl, int nb0, int nnb, int jn);

// Slack mode with more than G neighbours: the ones with a live row in IMPC iteration `it` are
// compacted into the lanes (lane l takes the l-th: jn, its weight); returns their count (more than
// G: capacity exceeded, jn = -1). State and kept solution from LDS.
template <int G>
__device__ int slack_compact(const DevOps& op, const double* buf, const ImpcArgs& args, int it,
                                          const double* s0k, const double* ykeep, bool grid_mode,
                                          const int32_t* nbl, int nb0, int nnb, int gl, int& jn,
                                          double& wslack) {
    double sx[6], y[SEP_NZ];
#pragma unroll
    for (int i = 0; i < 6; i++) sx[i] = s0k[i];
#pragma unroll
    for (int i = 0; i < SEP_NZ; i++) y[i] = ykeep[16 * i];
    int nlive = 0;
    jn = -1;
    for (int base = 0; base < nnb; base += G) {
        const bool lv = lane_cbf_live(op, buf, args, it, sx, y, grid_mode, nbl, nb0, base + gl < nnb ? base + gl : -1);
        const unsigned long long msk = grp_ballot<G>(lv);
        const int want = gl - nlive;
        int c = 0;
        for (int b = 0; b < G; b++) {
            if ((msk >> b) & 1ull) {
                if (c == want) jn = base + b;
                c++;
            }
        }
        nlive += c;
    }
    if (nlive > G) jn = -1;
    wslack = lane_slack_weight<G>(op, args, sx, grid_mode, nbl, nb0, nnb, jn);
    return nlive;
}

// Slack weight of the lane's neighbour (list position jn, -1: none): slack_cost * decay^rank,
// rank by planar distance among all nnb neighbours (ConnectivityIMPCCBF.cpp:73-100; ties by list
// position — the reference's std::sort leaves them unspecified). Lanes without a neighbour get
// cost 1 (their slack has no rows: v -> 0). Up to G neighbours by lane shuffles, beyond by a
// scan of the whole list.
template <int G>
__device__ double lane_slack_weight(const DevOps& op, const ImpcArgs& args, const double (&s0)[6],
                                    bool grid_mode, const int32_t* nbl, int nb0, int nnb, int jn) {
    auto dist_of = [&](int j) {
        const int nbi = grid_mode ? nbl[j] : args.nb_col[nb0 + j];
        const double dx = args.states[(size_t)nbi * 6] - s0[0], dy = args.states[(size_t)nbi * 6 + 1] - s0[1];
        return sqrt(dx * dx + dy * dy);
    };
    const double dist = jn >= 0 ? dist_of(jn) : 0.0;
    int rank = 0;
    if (nnb <= G) {  // (jn = this lane's index)
        for (int k = 0; k < nnb; k++) {
            const double dk = __shfl(dist, k, G);
            rank += (dk < dist || (dk == dist && k < jn)) ? 1 : 0;
        }
    } else {
        for (int k = 0; k < nnb; k++) {
            const double dk = dist_of(k);
            rank += (dk < dist || (dk == dist && k < jn)) ? 1 : 0;
        }
    }
    return jn >= 0 ? op.slack_cost * pow(op.slack_decay, (double)rank) : 1.0;
}

// Slack-pattern active set of the collision slack mode (ConnectivityIMPCCBF.cpp:73-119,
// MPCCBFQPGeneratorBase.cpp:28-130; the FoV kernel's run_patterns on the separable layout). Lane l
// owns neighbour l's slack v_l >= 0 (cost w) and its CBF rows g_c y - v_l <= h_c (slots c with
// ccv = 1). A pattern fixes per lane either v_l = 0 (lead = -1: its rows hard, g_c y <= h_c) or a
// leader slot l with v_l = g_l y - h_l >= 0: w g_l joins the linear term, the other rows become
// (g_c - g_l) y <= h_c - h_l and the leader's own row the bound -g_l y <= -h_l. Each pattern is a
// strictly convex QP in y alone, solved exactly by sep_dual_as; it is the slack QP's optimum when
// every lane's multipliers are consistent — v_l = 0: the rows' multipliers sum to at most w
// (stationarity in v, the bound's multiplier w - sum >= 0); led: the leader row's implied
// multiplier w - sum(others) - mu >= 0 (mu: the bound's). Otherwise a lane over its cost takes its
// largest-multiplier row as leader, a led lane with a negative leader multiplier its other active
// row; a pattern without a feasible point lets the unreachable candidate's row lead when that is a
// CBF row of a lane without a leader. lead: per lane, in (the first pattern) and out. Returns 1 with
// yo, vo (this lane's slack), the residuals and the summed steps; 0: no consistent pattern found
// (the caller's PDIP solves). mult: 16 doubles of the group's LDS (sep_dual_as's multipliers).
template <int G, int SB, int CB>
__device__ int sep_slack_patterns(const SepRows<SB, CB>& rw, double w, int& lead, const double* __restrict__ P,
                                  const double* __restrict__ Pinv, const double (&q)[SEP_NZ], double tol,
                                  int maxstep, int npat, double* pol, double* mult, double (&yo)[SEP_NZ], double& vo,
                                  double& rp_out, double& rd_out, int& steps) {
    const int gl = lane_bits_opaque<G - 1>();
    constexpr int SCBF = 2 * SEP_D * SB;  // first CBF side index (sep_stage_side)
    steps = 0;
    for (int pat = 0; pat < npat; pat++) {
        double g4[4] = {0.0, 0.0, 0.0, 0.0}, hl = 0.0;
#pragma unroll
        for (int c = 0; c < CB; c++) {
            if (c != lead) continue;
#pragma unroll
            for (int j = 0; j < 4; j++) g4[j] = rw.cg[c][j];
            hl = rw.chi[c];
        }
        SepRows<SB, CB> rp = rw;
#pragma unroll
        for (int c = 0; c < CB; c++) {
            if (lead < 0 || rw.ccv[c] == 0.0) continue;  // (inert slots stay inert)
            const double keep = c == lead ? 0.0 : 1.0;  // leader: -g_l; others: g_c - g_l
#pragma unroll
            for (int j = 0; j < 4; j++) rp.cg[c][j] = fma(keep, rw.cg[c][j], -g4[j]);
            rp.chi[c] = fma(keep, rw.chi[c], -hl);
        }
        double qa[4];
#pragma unroll
        for (int j = 0; j < 4; j++) qa[j] = lead >= 0 ? w * g4[j] : 0.0;
        grp_sum_vec<G, 4>(qa);
        double qp[SEP_NZ], yu[SEP_NZ], yg[SEP_NZ], rpg = 0.0, rdg = 0.0, tl = 0.0;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) qp[j] = j < 4 ? q[j] + qa[j] : q[j];
#pragma unroll
        for (int d = 0; d < SEP_D; d++) {
            const int o = 2 * d;
            yu[o] = -fma(Pinv[3 * d], qp[o], Pinv[3 * d + 1] * qp[o + 1]);
            yu[o + 1] = -fma(Pinv[3 * d + 1], qp[o], Pinv[3 * d + 2] * qp[o + 1]);
        }
        int st = 0;
        const int r = sep_dual_as<G, SB, CB>(rp, true, P, Pinv, qp, yu, tol, maxstep, pol, yg, rpg, rdg, st, nullptr,
                                             true, tl, nullptr, 0, nullptr, nullptr, mult);
        steps += st;
        if (r == 0) return 0;
        if (r < 0) {
            // no feasible point with this pattern: the unreachable candidate's row leads its lane
            const int id = (int)pol[POL_K * 16 + POL_ID];
            const int s = id >> 4, ln = id & 15;
            if (s < SCBF || __shfl(lead, ln, G) >= 0) return 0;
            wave_lds_sync();
            if (gl == ln) lead = s - SCBF;
            continue;
        }
        // per lane: multipliers of its rows (lam) and of its leader's bound (mu)
        const int k = (int)mult[7];
        double lam = 0.0, mu = 0.0, best = -1.0;
        int pick = -1;
        for (int a = 0; a < k; a++) {
            const int id = (int)mult[8 + a];
            const int s = id >> 4;
            if ((id & 15) != gl || s < SCBF) continue;
            const int c = s - SCBF;
            const double ua = mult[a];
            if (c == lead) {
                mu += ua;
            } else {
                lam += ua;
                if (ua > best) best = ua, pick = c;
            }
        }
        const bool bad = lead < 0 ? !(lam <= w) : !(w - lam - mu >= 0.0);
        wave_lds_sync();  // (mult is rewritten by the next pattern)
        if (grp_ballot<G>(bad) == 0ull) {
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) yo[j] = yg[j];
            double t = -hl;
#pragma unroll
            for (int j = 0; j < 4; j++) t = fma(g4[j], yg[j], t);
            vo = lead >= 0 ? fmax(t, 0.0) : 0.0;
            rp_out = rpg;
            rd_out = rdg;
            return 1;
        }
        if (grp_ballot<G>(bad && pick < 0) != 0ull) return 0;
        if (bad) lead = pick;
    }
    return 0;
}

// state row `row` of the batch (re-read where needed instead of held in registers)
__device__ __forceinline__ void load_state_lds(const double* s0k, double (&s)[6]) {
    wave_lds_sync();  // (written by lanes 0..5 of the group)
#pragma unroll
    for (int i = 0; i < 6; i++) s[i] = s0k[i];
}

// Hand agent ai to the fallback launch (lane 0 appends it to args.defer: [count, -, agents...]).
__device__ __forceinline__ void defer_agent(const ImpcArgs& args, int ai, int gl) {
    if (gl == 0) {
        const int slot = atomicAdd(&args.defer[0], 1);
        args.defer[2 + slot] = ai;
    }
}

// One agent's IMPC step on the separable layout (the body of impc_sep_kernel). stage / red / nbs:
// this group's LDS (CBF-row staging, Newton-sum all-reduce, neighbour query).
// The (non-slack) fallback launch keeps a lane's rows (SepRows, e.g. 8 CBF slots: 60 doubles) in
// LDS instead of registers: its occupancy is one wave per SIMD either way, and in registers they
// spilled (1236 -> 424 B/lane for 8 slots, 44 -> 0 for 1). Padded to an odd number of doubles per
// lane (bank spread of the per-lane struct reads). The slack fallback too since round 4 (156 -> 0
// B/lane; round 3 had kept them in registers because in LDS one all-neighbour slack QP of the
// stress line flipped to UNKNOWN in the last bits — with the slack-pattern active set the 1000-step
// stress line stays at 0 UNKNOWN either way, `profiles/r04_slack_fallback_lds.log`).
template <int SB, int CB>
struct SepRowsLds {
    SepRows<SB, CB> r;
    double pad[(sizeof(SepRows<SB, CB>) / 8) % 2 == 0 ? 1 : 2];
};

// LDS of the separable pipeline per agent (doubles): CBF-row staging / the dual active set's
// scratch, and the kept solution | warm duals | state | warm-start side ids | linear term
template <int SB, int CB, bool SLACK>
constexpr int sep_stage_doubles() {
    return SLACK ? sep_pol_doubles<SB, CB>() + 16
                 : (CB * 16 * (SEP_NZ + 1) > sep_pol_doubles<SB, CB>() ? CB * 16 * (SEP_NZ + 1)
                                                                      : sep_pol_doubles<SB, CB>());
}
template <int SB, bool SLACK, bool LEAN>
constexpr int sep_keep_doubles() {
    return 16 * (SEP_NZ + (LEAN ? 0 : 2 * SEP_D * SB)) + 8 + (SLACK ? 0 : POL_K + 1) + 10 + 6;
}

// (lds: this group's 16 entries, one per lane)
template <bool LDS, int SB, int CB>
__device__ __forceinline__ SepRows<SB, CB>& pick_rows(SepRows<SB, CB>& reg, SepRowsLds<SB, CB>* lds) {
    if constexpr (LDS) return lds[threadIdx.x & 15u].r;
    else return reg;
}

// (force-inlined: instantiated by two kernels, an out-of-line call would copy the kernel arguments
// to the stack at every launch's start)
template <int SB, int CB, bool SLACK, bool QUEUE, bool LEAN = false>
__device__ __forceinline__ void impc_sep_agent(const DevOps& op, const double* __restrict__ buf, const ImpcArgs& args,
                               const int ai, const int gl, double* stage, double* red, NbScratch& nbs,
                               double* keep, SepRowsLds<SB, CB>* rows_lds = nullptr, double* bconst = nullptr) {
    constexpr int G = 16;
    constexpr int NZ = SEP_NZ;
    constexpr int cap = CB * G;  // CBF rows per agent
    stamp(args, ai, gl, 0);

    const int self = args.agent_first + ai;
    double s0[6];
#pragma unroll
    for (int i = 0; i < 6; i++) s0[i] = args.states[(size_t)self * 6 + i];
    // the next state's noise draws, while the state is in flight (the keep area's last 6 doubles)
    double* const noise0 = keep + sep_keep_doubles<SB, SLACK, LEAN>() - 6;
    early_noise(args, ai, gl, noise0);
    // grid mode: the neighbour query's loads are staged between the setup's (gq_*)
    const bool grid_mode = args.nb_row_ptr == nullptr;
    GridQuery<G> gq;
    // (the state arrives before the branch: waited for only on one side, the join would wait for
    // every load in flight, the query's included)
    asm volatile("" ::"v"(s0[0]), "v"(s0[1]), "v"(s0[2]), "v"(s0[3]), "v"(s0[4]), "v"(s0[5]));
    if (grid_mode) gq_begin<G>(args, s0[0], s0[1], gq);
    // the linear term and constant, group-uniform: kept in LDS (qk, after the warm-start ids) and
    // read back inside each IMPC iteration, so they are not live in registers across the loop
    double* qk = keep + 16 * (SEP_NZ + (LEAN ? 0 : 2 * SEP_D * SB)) + 8 + (SLACK ? 0 : POL_K + 1);
    {
        double kc0;
        const double q0 = agent_linear_term_lanes<NZ, G>(op, buf, args, ai, s0, gl, kc0);
        if (gl < NZ) qk[gl] = q0;
        if (gl == 0) {
            qk[NZ] = kc0;
            *(int*)(qk + NZ + 1) = ai;
        }
    }
    // the agent index and the returned point's residuals, re-read from LDS where they are used
    // (held in registers across the solves they were the main launch's last spills)
#ifdef MPCCBF_V_REGAI  // (A/B variant: both in registers)
    auto agent = [&]() -> int { return ai; };
    double res[2];
#else
    auto agent = [&]() -> int { return *lds_vol((int*)(qk + NZ + 1)); };
    lds_vptr<double> res = lds_vol(qk + NZ + 2);
#endif

    // ---- box rows: channel d, slot k -> row k * G + gl of that channel (packed by the host:
    // per row [g0, g1, Gs(6), lo, hi], two-sided; unused rows inert: g = 0, Gs = 0, [-1, 1])
    if (grid_mode) gq_slots<G>(args, gq, gl);
    SepRows<SB, CB> rw_reg;  // (the fallback launch: rows in LDS)
    // (rows in LDS: the fallback launch, and two box slots per lane, where in registers they spill)
    SepRows<SB, CB>& rw = pick_rows<QUEUE || (SB > 1)>(rw_reg, rows_lds);
    {
        const double* B = opp(buf, op.o_Gsep);
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const double* r = B + ((size_t)(d * SB + k) * G + gl) * SEP_ROW;
                double sh = 0.0;
#pragma unroll
                for (int s = 0; s < 6; s++) sh = fma(r[2 + s], s0[s], sh);
                rw.bg[d][k][0] = r[0];
                rw.bg[d][k][1] = r[1];
                rw.blo[d][k] = r[8] - sh;
                rw.bhi[d][k] = r[9] - sh;
            }
    }
    if (grid_mode) gq_states<G>(args, gq, gl);
    const bool infeasible = constant_rows_infeasible<G>(op, buf, s0, gl);
    // the box rows' violation scales and candidate weights, formed once for both IMPC iterations'
    // active-set solves (bconst: [2 SEP_D SB sides][16] doubles, then [SEP_D SB rows][16] floats)
    double* bsc = nullptr;
    float* bw = nullptr;
#ifdef MPCCBF_NO_BOXC  // (A/B build: the constants formed by each solve)
    bconst = nullptr;
#endif
    if (!SLACK && bconst != nullptr) {
        bsc = bconst;
        bw = (float*)(bconst + 16 * 2 * SEP_D * SB);
        sep_box_consts<SB, CB>(rw, opp(buf, op.o_Pinv), bsc, bw);
    }
    stamp(args, ai, gl, 1);

    int nb0 = 0, nnb = 0;
    if (!grid_mode) {
        nb0 = args.nb_row_ptr[ai];
        nnb = args.nb_row_ptr[ai + 1] - nb0;
    } else {
        nnb = grid_neighbors_finish<G>(args, self, s0[0], s0[1], nbs, gl, 0.0, gq);
    }
    write_nb_out(args, ai, gl, grid_mode, nbs, nb0, nnb);
    if (SLACK && !QUEUE && nnb > G && args.defer) {  // slack mode: beyond one lane per neighbour
        defer_agent(args, agent(), gl);
        return;
    }
    const bool nb_overflow = nnb < 0 || (SLACK && !QUEUE && nnb > G);
    if (nb_overflow) nnb = 0;
    double wslack = 0.0, vslack = 0.0;
    // slack mode: one lane per neighbour; with more than G neighbours (the fallback launch), per
    // IMPC iteration the ones with a live row (a slack without rows is 0 at the optimum)
    if constexpr (SLACK)
        if (nnb <= G) wslack = lane_slack_weight<G>(op, args, s0, grid_mode, nbs.idx, nb0, nnb, gl < nnb ? gl : -1);
    stamp(args, ai, gl, 2);

    // the kept solution and the warm-start duals live in per-lane LDS slots (keep: [ykeep 6 x 16 |
    // warm 2 x 3 x SB x 16]), not registers: they are touched once per IMPC iteration
    double y[NZ];
    double* ykeep = keep + gl;  // ykeep[16 * i]
#pragma unroll
    for (int i = 0; i < NZ; i++) y[i] = ykeep[16 * i] = 0.0;
    // the agent's state, kept for the CBF rows and the outputs (group-uniform: LDS broadcast reads
    // instead of further global round trips)
    double* s0k = keep + 16 * (SEP_NZ + (LEAN ? 0 : 2 * SEP_D * SB));
    {
        double v = s0[0];
#pragma unroll
        for (int i = 1; i < 6; i++) v = gl == i ? s0[i] : v;
        if (gl < 6) s0k[gl] = v;
    }
    bool have_curve = false, success = true;
    const PdipCfg cfg{op.maxit, op.tol};
    SepWarm<SB> warm{keep + 16 * NZ};  // box duals of the previous OPTIMAL solve (iteration 1 warm start)
    const double warm_delta = SLACK ? 0.0 : op.warm_delta;
    // the dual active set's warm start: iteration 0's final active set (side ids, their count at
    // act[POL_K]) starts iteration 1's solve (same box rows and cost, sample-0 CBF rows) when
    // iteration 0 took at least op.das_warm steps. Measured on the bench swarm: after a long
    // iteration-0 solve (a transient: several sides) iteration 1 then takes 0 steps where a cold
    // start repeats them; after a 1-2 step solve (steady state: one CBF side, which iteration 1's
    // sample-1 row usually replaces) the warm set costs a step more than the cold start.
    double* act = s0k + 8;  // (no such area in slack mode: never touched there)
    if (!SLACK && gl == 0) act[POL_K] = 0.0;
    int steps0 = 0;  // iteration 0's solver steps
    auto warm_count = [&](int it) -> int {
        if (SLACK || it == 0 || op.das_warm <= 0 || steps0 < op.das_warm) return 0;
        wave_lds_sync();
        return (int)act[POL_K];
    };

    for (int it = 0; it < op.impc_iter; it++) {
        const size_t oi = (size_t)agent() * op.impc_iter + it;
        if (!success) {
            write_iteration(args, oi, gl, ST_UNKNOWN, __builtin_nan(""), 0);
            continue;
        }
        bool row_infeasible = false;
        int count = 0;
        bool live = false;
        bool slack_overflow = false;
        wave_lds_sync();
        asm volatile("" ::: "memory");  // (the reads below stay inside the iteration)
        double q[NZ];
#pragma unroll
        for (int j = 0; j < NZ; j++) q[j] = qk[j];
        if constexpr (SLACK) {
            // slack mode: rows stay in their neighbour's lane; a slack row is never infeasible
            double sx[6];  // the state again (not kept in registers across the solves)
            load_state_lds(s0k, sx);
            int jn = gl < nnb ? gl : -1;
            if (QUEUE && nnb > G) {
                const int nlive = slack_compact<G>(op, buf, args, it, s0k, ykeep, grid_mode, nbs.idx, nb0, nnb,
                                                   gl, jn, wslack);
                slack_overflow = nlive > G;
            }
            live = grp_ballot<G>(lane_cbf_rows<SB, CB>(op, buf, args, it, sx, y, grid_mode, nbs.idx, nb0, jn, rw)) != 0ull;
        } else {
            double sx[6];  // the state again (not kept in registers across the solves)
            load_state_lds(s0k, sx);
            // (the staging area's tail beyond the cap rows holds the samples' terms when it has
            // room: the dual active set's scratch is larger than 16 rows)
            constexpr int STG = CB * 16 * (SEP_NZ + 1) > sep_pol_doubles<SB, CB>() ? CB * 16 * (SEP_NZ + 1)
                                                                                   : sep_pol_doubles<SB, CB>();
            if (STG - cap * (NZ + 1) >= 27 && it > 0)
                count = stage_cbf_rows_pairs<NZ>(op, buf, args, it, sx, y, grid_mode, &nbs, nb0, nnb, stage, cap, gl,
                                                 &row_infeasible, stage + cap * (NZ + 1));
            else
                count = stage_cbf_rows<NZ, G>(op, buf, args, it, sx, y, grid_mode, &nbs,
                                              nb0, nnb, stage, cap, gl, &row_infeasible);
            live = count > 0;
#pragma unroll
            for (int c = 0; c < CB; c++) {
                const int ci = c * G + gl;
                const bool on = ci < count && ci < cap;
                const double* src = stage + (size_t)(on ? ci : 0) * (NZ + 1);
#pragma unroll
                for (int j = 0; j < 4; j++) rw.cg[c][j] = on ? src[j] : 0.0;  // yaw columns are 0
                rw.chi[c] = on ? src[NZ] : 1.0;  // unused slot: inert row 0 <= 1
                rw.ccv[c] = 0.0;
            }
        }
        if (it < 2) stamp(args, ai, gl, 3 + 2 * it);
        if (count > cap && args.defer) {  // beyond this instantiation: the fallback launch solves it
            defer_agent(args, agent(), gl);
            return;
        }
#ifdef MPCCBF_PDIP_STAMPS  // (profiling build: the solve phase's parts around the solver, slots 16 ..)
        long long* const dbgs = (args.stamps && it == 0)
                                    ? (long long*)args.stamps + (size_t)args.num_agents * NSTAMP + (size_t)ai * 32
                                    : nullptr;
#define SSTAMP(k)                                                                \
    do {                                                                         \
        if (dbgs) dbgs[k] = (long long)__builtin_amdgcn_s_memtime();             \
    } while (0)
#else
#define SSTAMP(k) \
    do {          \
    } while (0)
#endif
        SSTAMP(16);
        int st;
        int nit = 0;
        if (gl == 0) res[0] = res[1] = __builtin_nan("");
        // non-finite data (a NaN / Inf state, target or neighbour state): such a model is not
        // solved (CPLEX rejects non-finite coefficients); reported as ERROR
        bool nfin = false;
#pragma unroll
        for (int j = 0; j < NZ; j++) nfin = nfin || !isfinite(q[j]);
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) nfin = nfin || !isfinite(rw.blo[d][k]) || !isfinite(rw.bhi[d][k]);
#pragma unroll
        for (int c = 0; c < CB; c++)
            nfin = nfin || !isfinite(rw.chi[c]) || !isfinite(rw.cg[c][0]) || !isfinite(rw.cg[c][1]) ||
                   !isfinite(rw.cg[c][2]) || !isfinite(rw.cg[c][3]);
        const bool nonfinite = grp_ballot<G>(nfin) != 0ull;
        SSTAMP(17);
        if (count > cap || nb_overflow || slack_overflow || nonfinite) {
            st = ST_ERROR;
        } else if (infeasible || row_infeasible) {
            st = ST_INFEASIBLE;
        } else if constexpr (LEAN) {
            // lean main launch: the fast start and the dual active set only. A QP that needs more
            // (the active set gives up, or no feasible point without a certificate well above the
            // tolerance: phase 1) defers the whole agent to the fallback launch, which runs the
            // full pipeline (PDIP attempts, phase 1) on the same inputs — so the main kernel's
            // registers are those of the active-set path, not the interior-point solver's.
            const double* Pi = opp(buf, op.o_Pinv);
            double yu[NZ];
#pragma unroll
            for (int d = 0; d < SEP_D; d++) {
                const int o = 2 * d;
                yu[o] = -fma(Pi[3 * d], q[o], Pi[3 * d + 1] * q[o + 1]);
                yu[o + 1] = -fma(Pi[3 * d + 1], q[o], Pi[3 * d + 2] * q[o + 1]);
            }
            double tl = 0.0, prs = __builtin_nan(""), drs = __builtin_nan("");
            const int k0 = warm_count(it);
            const int r = sep_dual_as<G, SB, CB>(rw, live, opp(buf, op.o_Pr), Pi, q, yu, op.tol, op.dual_as, stage, y,
                                                 prs, drs, nit, nullptr, true, tl, nullptr, k0, act,
                                                 it == 0 ? act : nullptr, nullptr, bsc, bw);
            if (r > 0) {
                st = ST_OPTIMAL;
            } else if (r < 0 && tl > 10.0 * op.feas_tol) {
                st = ST_INFEASIBLE;
                prs = tl;
                drs = __builtin_nan("");
            } else {
                defer_agent(args, agent(), gl);
                return;
            }
            if (gl == 0) res[0] = prs, res[1] = drs;
        } else {
#ifdef MPCCBF_PDIP_STAMPS
            long long* dbg = (args.stamps && it == 0)
                                 ? (long long*)args.stamps + (size_t)args.num_agents * NSTAMP + (size_t)agent() * 32
                                 : nullptr;
#elif defined(MPCCBF_SOLVE_TRACE)  // per-step (rp, mu, alpha, rd) of the first solve + phase 1
            long long* dbg = args.stamps ? (long long*)args.stamps + (size_t)args.num_agents * NSTAMP +
                                               ((size_t)agent() * 2 + it) * 256
                                         : nullptr;
#else
            long long* dbg = nullptr;
#endif
            // Attempts (group-uniform; one call site): 0 = warm start (IMPC iteration 1) or cold,
            // with the divergence test; 1 = cold to the iteration limit; 2 = cold with the shifted
            // Newton matrix. Before any retry, phase 1 certifies feasibility (minimal uniform row
            // violation above the tolerance, from the failed solve's last iterate), so an
            // infeasible QP needs no retry and statuses never depend on the first attempt's
            // warm start or divergence test.
            // (with the dual active-set solve first, the PDIP runs cold: no warm-start duals kept)
            const bool warm_try = it > 0 && warm_delta > 0.0 && op.dual_as <= 0;
            int tr_warm = 0, tr_cold = 0, tr_p1 = 0;  // per kind (MPCCBF_SOLVE_TRACE); phase-1 steps
            int attempt = 0, total = 0;
            bool certified = false, infeas = false;
            double tstar = 0.0;
            PdipOut po{ST_UNKNOWN, 0};
            // slack mode: the slack-pattern active set first (every slack at zero, then leader
            // rows); the PDIP below only when it finds no consistent pattern
            bool pattern_done = false;
            double* pat_mult = SLACK ? stage + sep_pol_doubles<SB, CB>() : nullptr;
            if constexpr (SLACK) {
                if (op.dual_as > 0 && live) {
                    int lead = -1, pst = 0;
                    double yg[NZ], vg = 0.0, rpg = 0.0, rdg = 0.0;
                    if (sep_slack_patterns<G, SB, CB>(rw, wslack, lead, opp(buf, op.o_Pr), opp(buf, op.o_Pinv), q,
                                                      op.tol, 2 * op.dual_as, 8, stage, pat_mult, yg, vg, rpg, rdg,
                                                      pst)) {
#pragma unroll
                        for (int j = 0; j < NZ; j++) y[j] = yg[j];
                        vslack = vg;
                        po = PdipOut{ST_OPTIMAL, 0};
                        po.rp = rpg;
                        po.rd = rdg;
                        pattern_done = true;
                    }
                    total += pst;
                }
            }
            for (; !pattern_done;) {
                PdipCfg ca = cfg;
                ca.early_it = attempt == 0 ? op.early_it : 0;
                ca.fast_start = op.fast_start != 0;
                ca.robust = attempt == 2;
                ca.dual_as = attempt == 0 ? op.dual_as : 0;
                ca.want_rd = args.dual_res != nullptr;
                const int k0 = attempt == 0 ? warm_count(it) : 0;
                po = pdip_solve_sep<G, SB, CB, SLACK>(rw, live, opp(buf, op.o_Pr), opp(buf, op.o_Pinv), q, y,
                                                      ca, dbg, wslack, &vslack, red, &warm,
                                                      (attempt == 0 && warm_try) ? warm_delta : 0.0,
                                                      SLACK ? nullptr : stage, k0, SLACK ? nullptr : act,
                                                      (!SLACK && attempt == 0 && it == 0) ? act : nullptr, bsc, bw);
                total += po.iters;
                ((attempt == 0 && warm_try) ? tr_warm : tr_cold) += po.iters;
                if (po.status == ST_OPTIMAL) break;
                if (!certified && po.tlow > 10.0 * op.feas_tol) {
                    // the dual active set's infeasibility certificate bounds t* from below: no
                    // phase 1 needed (a bound within 10x of the tolerance still goes to phase 1)
                    tstar = po.tlow;
                    infeas = true;
                    certified = true;
                }
                if (!certified) {
                    SepRows<SB, CB> rp1 = rw;
                    if constexpr (SLACK) {  // slack rows are always satisfiable: certify the box rows
#pragma unroll
                        for (int c = 0; c < CB; c++) {
#pragma unroll
                            for (int j = 0; j < 4; j++) rp1.cg[c][j] = 0.0;
                            rp1.chi[c] = 1.0;
                        }
                    }
                    tstar = pdip_phase1_sep<G, SB, CB>(rp1, cfg, op.feas_tol, y, red, &tr_p1, dbg);
                    infeas = tstar > op.feas_tol && tstar < 1e300;  // 1e300: phase 1 failed
                    certified = true;
#ifdef MPCCBF_DEBUG_EXIT
                    total += tstar >= 1e300 ? 10000 : 0;
#endif
                }
                if (infeas) {
                    po.status = ST_INFEASIBLE;
                    break;
                }
                if (attempt == 0 && (warm_try || po.early)) attempt = 1;
                else if (attempt < 2) attempt = 2;
                else break;
            }
            if constexpr (SLACK) {
                // the slack PDIP's point fixes a pattern — a lane with v > 0 leads with its row of
                // largest excess g y - h — and one active-set solve of it (plus one exchange)
                // returns the exact optimum, which replaces the interior point's when consistent
                // (also a PDIP that stalled short of its tolerance: round 3's UNKNOWN all-neighbour
                // slack QPs)
                if (!pattern_done && !infeas && op.dual_as > 0 && live) {
                    int lead = -1;
                    double best = -1e300;
#pragma unroll
                    for (int c = 0; c < CB; c++) {
                        double t = -rw.chi[c];
#pragma unroll
                        for (int j = 0; j < 4; j++) t = fma(rw.cg[c][j], y[j], t);
                        if (rw.ccv[c] != 0.0 && t > best) best = t, lead = c;
                    }
                    if (!(vslack > 1e-9)) lead = -1;
                    int pst = 0;
                    double yg[NZ], vg = 0.0, rpg = 0.0, rdg = 0.0;
                    if (sep_slack_patterns<G, SB, CB>(rw, wslack, lead, opp(buf, op.o_Pr), opp(buf, op.o_Pinv), q,
                                                      op.tol, 2 * op.dual_as, 2, stage, pat_mult, yg, vg, rpg, rdg,
                                                      pst)) {
#pragma unroll
                        for (int j = 0; j < NZ; j++) y[j] = yg[j];
                        vslack = vg;
                        po.status = ST_OPTIMAL;
                        po.rp = rpg;
                        po.rd = rdg;
                    }
                    total += pst;
                }
            }
            st = po.status;
            nit = total + tr_p1;  // active-set, PDIP and phase-1 steps
            if (gl == 0) res[0] = st == ST_INFEASIBLE ? tstar : po.rp, res[1] = po.rd;
#ifdef MPCCBF_SOLVE_TRACE  // diagnostics build: warm + 100 cold + 10000 phase-1 iterations
            nit = tr_warm + 100 * tr_cold + 10000 * tr_p1;
#else
            (void)tr_warm, (void)tr_cold;
#endif
        }
        SSTAMP(18);
        double objv = __builtin_nan("");
        if (st == ST_OPTIMAL) {
            objv = sep_objective(opp(buf, op.o_Pr), q, y, qk[NZ]);
            if constexpr (SLACK) objv += grp_sum<G>(live ? wslack * vslack : 0.0);  // + w^T v
            SSTAMP(19);
#pragma unroll
            for (int i = 0; i < NZ; i++) ykeep[16 * i] = y[i];
            have_curve = true;
        } else {
            success = false;
        }
        SSTAMP(20);
        write_iteration(args, oi, gl, st, objv, nit, res[0], res[1]);
        SSTAMP(21);
        if (it == 0) steps0 = nit;
        if (it < 2) stamp(args, ai, gl, 4 + 2 * it);
        wave_lds_sync();
#undef SSTAMP
    }
    double yk[NZ], sx[6];
#pragma unroll
    for (int i = 0; i < NZ; i++) yk[i] = ykeep[16 * i];
    load_state_lds(s0k, sx);
    write_agent_outputs<NZ, G>(op, buf, args, agent(), gl, sx, yk, have_curve, noise0);
    stamp(args, ai, gl, 7);
}

// QUEUE = false: one agent per 16-lane group. QUEUE = true (fallback launch): the agents the main
// launch deferred (args.queue: [count, blocks done, agents...]), one per group (the grid covers
// every agent of the batch); the last block to finish empties the queue for the next step.
template <int SB, int CB, bool SLACK, int BS, bool QUEUE = false, bool LEAN = false>
__global__ void __launch_bounds__(BS) impc_sep_kernel(const DevOps op, const double* __restrict__ buf,
                                                       const ImpcArgs args) {
    constexpr int GPB = BS / 16;
    // CBF-row staging, reused as the dual active set's scratch (sep_pol_doubles)
    // (slack mode: the slack-pattern active set's scratch + its multipliers, sep_slack_patterns)
    __shared__ double stage_all[GPB][sep_stage_doubles<SB, CB, SLACK>()];
    __shared__ double red_all[GPB][LEAN ? 1 : 16 * (A_N + 1)];  // LDS all-reduce of the Newton sums
    __shared__ NbScratch nb_scratch[GPB];
    // kept solution | warm-start duals (not in the lean launch) | the agent's state | the dual active
    // set's warm-start side ids and their count (not in slack mode) | linear term and constant, the
    // agent index, the residuals
    __shared__ double keep_all[GPB][sep_keep_doubles<SB, SLACK, LEAN>()];
    constexpr bool rows_lds_per_lane = QUEUE || SB > 1;
    __shared__ SepRowsLds<SB, CB> rows_lds[rows_lds_per_lane ? BS : 1];
    // the box rows' constants per agent (sep_box_consts; not in slack mode)
    __shared__ double bconst_all[SLACK ? 1 : GPB][SLACK ? 1 : 16 * 2 * SEP_D * SB + 8 * SEP_D * SB];
    const int gl = threadIdx.x & 15;
    const int gib = threadIdx.x / 16;
    lds_poison();
    if constexpr (!QUEUE) {
        kclock_start(args);
        grid_clear<BS>(args);
        const int ai = xcd_block((int)blockIdx.x, (int)gridDim.x) * GPB + gib;
        if (ai >= args.num_agents) return;
        impc_sep_agent<SB, CB, SLACK, false, LEAN>(op, buf, args, ai, gl, stage_all[gib], red_all[gib],
                                                   nb_scratch[gib], keep_all[gib],
                                                   rows_lds + (rows_lds_per_lane ? gib * 16 : 0),
                                                   SLACK ? nullptr : bconst_all[SLACK ? 0 : gib]);
        kclock_end<BS>(args);
    } else {
        // one queue entry per group (no grid-stride loop: carried across iterations the agent's
        // state spills, 0 -> 372 B/lane, and a 16-block grid saved 0.2 us of the empty launch,
        // r06d); groups beyond the queue's length leave at once. The queue's header is zeroed by
        // the main launch after next (the queues alternate by step parity), so no block has to
        // find out that it is the last one
        const int k = blockIdx.x * GPB + gib;
        if (k < args.queue[0])
            impc_sep_agent<SB, CB, SLACK, true>(op, buf, args, args.queue[2 + k], gl, stage_all[gib], red_all[gib],
                                                nb_scratch[gib], keep_all[gib],
                                                rows_lds + (rows_lds_per_lane ? gib * 16 : 0),
                                                SLACK ? nullptr : bconst_all[SLACK ? 0 : gib]);
    }
}

// ---------------------------------------------------------------------------------------------
// One agent per wave (impc_wide.hpp)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void wide_defer(const ImpcArgs& args, int ai, int gl) {
    if (gl == 0) {
        const int slot = atomicAdd(&args.defer[0], 1);
        args.defer[2 + slot] = ai;
    }
}

__device__ void impc_wide_agent(const DevOps& op, const double* __restrict__ buf, const ImpcArgs& args,
                                const int ai, WideLds& L) {
    constexpr int NZ = SEP_NZ;
    const int gl = (int)(threadIdx.x & 63u);
    stamp(args, ai, gl, 0);
    const int self = args.agent_first + ai;
    double s0[6];
#pragma unroll
    for (int i = 0; i < 6; i++) s0[i] = args.states[(size_t)self * 6 + i];
    early_noise(args, ai, gl, L.noise);  // (while the state is in flight)
    const bool grid_mode = args.nb_row_ptr == nullptr;
    WideQuery gq;
    WideCells gc;
    if (grid_mode) wn_issue(args, s0[0], s0[1], gl, gq);
    // linear term: lane i < 6 forms q_i, the constant's terms summed over the first 16-lane row
    // (agent_linear_term_lanes; lanes >= 9 contribute 0, so the row total is the whole sum)
    double kconst;
    const double qlane = agent_linear_term_lanes<NZ, 16>(op, buf, args, ai, s0, gl, kconst);
    // this lane's box row: channel d = gl / 16, slot gl % 16 (host layout [channel][16][SEP_ROW])
    WRow rw;
    {
        const int lb = gl < W_BOX ? gl : 0;
        const double* r = opp(buf, op.o_Gsep) + (size_t)lb * SEP_ROW;
        double rv[SEP_ROW];
#pragma unroll
        for (int i = 0; i < SEP_ROW; i++) rv[i] = r[i];
        double sh = 0.0;
#pragma unroll
        for (int s = 0; s < 6; s++) sh = fma(rv[2 + s], s0[s], sh);
        const int d = gl >> 4;
#pragma unroll
        for (int j = 0; j < NZ; j++) rw.g[j] = 0.0;
        if (gl < W_BOX) {
#pragma unroll
            for (int dd = 0; dd < SEP_D; dd++)
                if (dd == d) {
                    rw.g[2 * dd] = rv[0];
                    rw.g[2 * dd + 1] = rv[1];
                }
        }
        rw.lo = gl < W_BOX ? rv[8] - sh : -1e300;
        rw.hi = gl < W_BOX ? rv[9] - sh : 1.0;
        const double* pd = opp(buf, op.o_Pinv) + 3 * (d < SEP_D ? d : 0);
        rw.w = wide_weight(wide_n2(pd[0], pd[1], pd[2], rv[0], rv[1]));
        rw.sl = rcp(1.0 + fabs(rw.lo));
        rw.su = rcp(1.0 + fabs(rw.hi));
    }
    wide_sample_us(op, buf, s0, L, gl);
    if (grid_mode) wn_cells(args, gq, gc);
    const bool infeasible = constant_rows_infeasible<64>(op, buf, s0, gl);
    stamp(args, ai, gl, 1);

    int nb0 = 0, nnb = 0;
    if (!grid_mode) {
        nb0 = args.nb_row_ptr[ai];
        nnb = args.nb_row_ptr[ai + 1] - nb0;
    } else {
        nnb = wn_finish(args, self, s0[0], s0[1], gc, gq, L, gl);
    }
    nnb = uni_i(nnb);
    if (args.nb_out && gl < 16)  // diagnostics: the list the rows are built from
        args.nb_out[(size_t)ai * 16 + gl] = gl < nnb ? (grid_mode ? L.nbi[gl] : args.nb_col[nb0 + gl]) : -1;
    const bool nb_overflow = nnb < 0;
    if (nb_overflow) nnb = 0;
    stamp(args, ai, gl, 2);

    double q[NZ], yu[NZ];
#pragma unroll
    for (int j = 0; j < NZ; j++) q[j] = lane_of(qlane, j);
    kconst = uni(kconst);
    const double* Pinv = opp(buf, op.o_Pinv);
#pragma unroll
    for (int d = 0; d < SEP_D; d++) {  // the unconstrained minimiser -P^-1 q (both IMPC iterations)
        const int o = 2 * d;
        yu[o] = -fma(Pinv[3 * d], q[o], Pinv[3 * d + 1] * q[o + 1]);
        yu[o + 1] = -fma(Pinv[3 * d + 1], q[o], Pinv[3 * d + 2] * q[o + 1]);
    }
    // non-finite data (a NaN / Inf state, target or neighbour state): such a model is not solved
    // (CPLEX rejects non-finite coefficients), ERROR; the linear term and the box rows are checked
    // here, the CBF rows per iteration
    bool nfin_fixed;
    {
        bool nf = gl < W_BOX && (!isfinite(rw.lo) || !isfinite(rw.hi));
#pragma unroll
        for (int j = 0; j < NZ; j++) nf = nf || !isfinite(q[j]);
        nfin_fixed = __ballot(nf) != 0ull;
    }
#ifdef MPCCBF_PDIP_STAMPS
    long long* wdbg = args.stamps ? (long long*)args.stamps + (size_t)args.num_agents * NSTAMP + (size_t)ai * 16 : nullptr;
#else
    long long* wdbg = nullptr;
#endif
    double y[NZ], yk[NZ];
#pragma unroll
    for (int j = 0; j < NZ; j++) y[j] = yk[j] = 0.0;
    bool have_curve = false, success = true;
    if (gl == 0) L.act[POL_K] = 0.0;
    int steps0 = 0;
    // per-iteration results, written together after the loop (impc_iter <= 2 here; more iterations
    // are written as they finish)
    int st_w0 = ST_UNKNOWN, st_w1 = ST_UNKNOWN, nit_w0 = 0, nit_w1 = 0;
    double obj_w0 = __builtin_nan(""), obj_w1 = __builtin_nan(""), prs_w0 = obj_w0, prs_w1 = obj_w0,
           drs_w0 = obj_w0, drs_w1 = obj_w0;
    const bool want_rp = args.primal_res != nullptr;

    for (int it = 0; it < op.impc_iter; it++) {
        const size_t oi = (size_t)ai * op.impc_iter + it;
        if (!success) {  // the reference breaks out of the IMPC loop (:208-211)
            if (it >= 2) write_iteration(args, oi, gl, ST_UNKNOWN, __builtin_nan(""), 0);
            continue;
        }
        bool row_infeasible = false;
        long long* wd = it == 0 ? wdbg : nullptr;
        const int count = uni_i(wide_cbf_rows(op, buf, args, it, s0, y, grid_mode, L, nb0, nnb, gl, row_infeasible, wd));
        bool nfin = false;
        if (gl >= W_BOX) {  // this iteration's CBF rows into the CBF lanes (unused: inert 0 <= 1)
            const int c = gl - W_BOX;
            const bool on = c < count;
            const double* src = L.stage + (on ? c : 0) * W_ROW;
#pragma unroll
            for (int j = 0; j < 4; j++) rw.g[j] = on ? src[j] : 0.0;
            rw.hi = on ? src[4] : 1.0;
            rw.w = wide_weight(wide_n2(Pinv[0], Pinv[1], Pinv[2], rw.g[0], rw.g[1]) +
                               wide_n2(Pinv[3], Pinv[4], Pinv[5], rw.g[2], rw.g[3]));
            rw.su = rcp(1.0 + fabs(rw.hi));
            nfin = !isfinite(rw.hi) || !isfinite(rw.g[0]) || !isfinite(rw.g[1]) || !isfinite(rw.g[2]) ||
                   !isfinite(rw.g[3]);
        }
        {
            long long* wdbg = wd;
            (void)wdbg;
            WST(4);
        }
        if (it < 2) stamp(args, ai, gl, 3 + 2 * it);
        if (count > W_CBF) {  // beyond the 16 CBF lanes: the fallback launch (8 slots per lane)
            if (args.defer) {
                wide_defer(args, ai, gl);
                return;
            }
        }
        const bool nonfinite = nfin_fixed || __ballot(nfin) != 0ull;
        int st, nit = 0;
        double prs = __builtin_nan(""), drs = __builtin_nan("");
        if (count > W_CBF || nb_overflow || nonfinite) {
            st = ST_ERROR;
        } else if (infeasible || row_infeasible) {
            st = ST_INFEASIBLE;
        } else {
            int k0 = 0;
            if (it > 0 && op.das_warm > 0 && steps0 >= op.das_warm) {
                wave_lds_sync();
                k0 = uni_i((int)L.act[POL_K]);
            }
            double tl = 0.0;
            const int r = wide_dual_as(rw, opp(buf, op.o_Pr), Pinv, q, yu, op.tol, op.dual_as, L.pol, y, prs, drs,
                                       nit, tl, k0, L.act, it == 0 ? L.act : nullptr, want_rp, wd);
            if (r > 0) {
                st = ST_OPTIMAL;
                if (!want_rp) prs = __builtin_nan("");
            } else if (r < 0 && tl > 10.0 * op.feas_tol) {
                st = ST_INFEASIBLE;
                prs = tl;
                drs = __builtin_nan("");
            } else {
                if (args.defer) {
                    wide_defer(args, ai, gl);
                    return;
                }
                st = ST_UNKNOWN;
            }
        }
        double objv = __builtin_nan("");
        if (st == ST_OPTIMAL) {
            // 1/2 y^T P y + q^T y + k (reduced_objective) on the first 16-lane row: lane i < 6 row i
            const double* Pr = opp(buf, op.o_Pr) + (size_t)(gl < NZ ? gl : 0) * NZ;
            double pr[NZ], pyi = 0.0, yi = y[0], qi = q[0];
#pragma unroll
            for (int j = 0; j < NZ; j++) pr[j] = Pr[j];
#pragma unroll
            for (int j = 1; j < NZ; j++) {
                yi = gl == j ? y[j] : yi;
                qi = gl == j ? q[j] : qi;
            }
#pragma unroll
            for (int j = 0; j < NZ; j++) pyi = fma(pr[j], y[j], pyi);
            objv = grp_sum<16>(gl < NZ ? yi * (0.5 * pyi + qi) : (gl == NZ ? kconst : 0.0));
#pragma unroll
            for (int i = 0; i < NZ; i++) yk[i] = y[i];
            have_curve = true;
        } else {
            success = false;
        }
        {
            long long* wdbg = wd;
            (void)wdbg;
            WST(12);
        }
        if (it == 0) {
            st_w0 = st, nit_w0 = nit, obj_w0 = objv, prs_w0 = prs, drs_w0 = drs;
        } else if (it == 1) {
            st_w1 = st, nit_w1 = nit, obj_w1 = objv, prs_w1 = prs, drs_w1 = drs;
        } else {
            write_iteration(args, oi, gl, st, objv, nit, prs, drs);
        }
        if (it == 0) steps0 = nit;
        if (it < 2) stamp(args, ai, gl, 4 + 2 * it);
    }
    write_iteration(args, (size_t)ai * op.impc_iter, gl, st_w0, obj_w0, nit_w0, prs_w0, drs_w0);
    if (op.impc_iter > 1) write_iteration(args, (size_t)ai * op.impc_iter + 1, gl, st_w1, obj_w1, nit_w1, prs_w1, drs_w1);
    write_agent_outputs<NZ, 64>(op, buf, args, ai, gl, s0, yk, have_curve, L.noise);
    stamp(args, ai, gl, 7);
}

// The operators (the buffer's hot prefix, DevOps::hot doubles) are staged into LDS once per block,
// while the agents' state loads are in flight: every operator read of the agent chain is then an
// LDS read (~100 cycles) instead of a scalar / vector memory round trip (~1,000 cycles under load).
// (MPCCBF_WIDE_WPE: diagnostics builds with N waves per SIMD, registers capped at 512 / N)
#ifdef MPCCBF_WIDE_WPE
#define WIDE_WPE_ATTR __attribute__((amdgpu_waves_per_eu(MPCCBF_WIDE_WPE, MPCCBF_WIDE_WPE)))
#else
#define WIDE_WPE_ATTR
#endif
template <int BS>
__global__ void __launch_bounds__(BS) WIDE_WPE_ATTR impc_wide_kernel(const DevOps op, const double* __restrict__ buf,
                                                                      const ImpcArgs args) {
    constexpr int WPB = BS / 64;
    constexpr int PER = WIDE_OPS / BS;
    __shared__ WideLds lds_all[WPB];
    __shared__ double ops[WIDE_OPS];
    lds_poison();
    kclock_start(args);
    {
        double v[PER];
#pragma unroll
        for (int r = 0; r < PER; r++) {
            const int i = r * BS + (int)threadIdx.x;
            v[r] = i < op.hot ? buf[i] : 0.0;
        }
#pragma unroll
        for (int r = 0; r < PER; r++) ops[r * BS + threadIdx.x] = v[r];
    }
    grid_clear<BS>(args);
    __syncthreads();
    const int wv = uni_i((int)(threadIdx.x >> 6));
    const int ai = xcd_block((int)blockIdx.x, (int)gridDim.x) * WPB + wv;
    if (ai >= args.num_agents) return;
    impc_wide_agent(op, ops, args, ai, lds_all[wv]);
    kclock_end<BS>(args);
}

}  // namespace dev

template <int NZ, int G, int R>
static hipError_t launch_impc_t(const DevOps& op, const double* buf, const ImpcArgs& a,
                                hipStream_t s) {
    constexpr int GPB = 256 / G;
    const int blocks = (a.num_agents + GPB - 1) / GPB;
    const size_t lds = (size_t)GPB * (R * G - op.m) * (NZ + 1) * sizeof(double);
    hipLaunchKernelGGL((dev::impc_kernel<NZ, G, R>), dim3(blocks), dim3(256), lds, s, op, buf, a);
    return hipGetLastError();
}

template <int SB, int CB, bool SLACK, int BS = 256, bool QUEUE = false, bool LEAN = false>
static hipError_t launch_impc_sep_t(const DevOps& op, const double* buf, const ImpcArgs& a,
                                    hipStream_t s) {
    constexpr int GPB = BS / 16;
    int blocks = (a.num_agents + GPB - 1) / GPB;
    hipLaunchKernelGGL((dev::impc_sep_kernel<SB, CB, SLACK, BS, QUEUE, LEAN>), dim3(blocks), dim3(BS), 0, s, op, buf,
                       a);
    return hipGetLastError();
}

// Whether the one-agent-per-wave kernel applies: the separable collision controller (no slack
// variables) with the dual active set on; CBF samples <= MAX_CBF_H.
static bool impc_wide_ok(const DevOps& op) {
    return op.cbf_mode == 0 && !op.slack_mode && op.sep && op.nzd == SEP_NZD_HOST && op.sep_rows_per_dim <= 16 &&
           op.dual_as > 0 && op.cbf_h <= MAX_CBF_H && op.hot > 0 && op.hot <= dev::WIDE_OPS;
}

static hipError_t launch_impc_wide(const DevOps& op, const double* buf, const ImpcArgs& a, hipStream_t s) {
    constexpr int BS = 256, WPB = BS / 64;
    const int blocks = (a.num_agents + WPB - 1) / WPB;
    hipLaunchKernelGGL((dev::impc_wide_kernel<BS>), dim3(blocks), dim3(BS), 0, s, op, buf, a);
    return hipGetLastError();
}

// Layouts of the separable collision controller (mpccbf_set_variant):
//   0 (default) — share-adaptive: up to one agent per SIMD of the device (1,024 on MI355X: config
//       4's rank share) the one-agent-per-wave kernel (its fallback as a second launch); beyond,
//       the 16-lane kernel (4 agents per wave: one wave per SIMD covers 4 x as many agents);
//   VARIANT_SEP16 — the 16-lane kernel at any count (the layout of rounds 1-4);
//   VARIANT_WIDE — the one-agent-per-wave kernel at any count.
// (Round 6, measured and dropped: a lean-then-full variant — the fast start and the dual active
// set, the full pipeline in place after the IMPC loop for the agents they do not settle — ran the
// lean part 1.6 us slower than the lean kernel alone and 0.5 us slower than the full kernel.)
constexpr int VARIANT_SEP16 = 4, VARIANT_WIDE = 5;
static bool sep_variant(int variant) { return variant == 0 || variant == VARIANT_SEP16; }
static bool use_wide(const DevOps& op, int variant, int n) {
    return impc_wide_ok(op) && (variant == VARIANT_WIDE || (variant == 0 && n <= op.wide_max));
}

// Row slots per lane and channel of the separable slack kernel (1: up to 16 box rows per channel,
// 2: up to 32, e.g. K = 16 as in the reference's instance files); 0: no slack instantiation fits
static int slack_sb(const DevOps& op) {
    if (!(op.sep && op.nzd == SEP_NZD_HOST && op.cbf_h <= 2)) return 0;
    return op.sep_rows_per_dim <= 16 ? 1 : (op.sep_rows_per_dim <= 32 ? 2 : 0);
}

// The separable layout's lean main launch (fast start + dual active set; everything else deferred)
static bool sep_lean(const DevOps& op, int variant, int n) {
    return sep_variant(variant) && !use_wide(op, variant, n) && !op.slack_mode && op.sep && op.nzd == SEP_NZD_HOST &&
           op.sep_rows_per_dim <= 16 && op.lean && op.dual_as > 0;
}

// Agents the main launch deferred are solved by this launch (the queue in a.queue):
//   slack mode, more than 16 neighbours — the slack solver, the neighbours with a live row
//   compacted into the lanes;
//   otherwise — the full separable pipeline (dual active set, PDIP attempts, phase 1): with 16 CBF
//   row slots when no agent can exceed them, else 8 slots per lane (128 rows). Agents beyond
//   that report ERROR.
hipError_t launch_impc_fallback(const DevOps& op, const double* buf, const ImpcArgs& a, bool wide,
                                hipStream_t s) {
    if (a.num_agents <= 0 || !a.queue) return hipSuccess;
    if (op.slack_mode) {
        if (slack_sb(op) == 2) return launch_impc_sep_t<2, 2, true, 64, true>(op, buf, a, s);
        return launch_impc_sep_t<1, 2, true, 64, true>(op, buf, a, s);
    }
    if (wide) return launch_impc_sep_t<1, 8, false, 64, true>(op, buf, a, s);
    return launch_impc_sep_t<1, 1, false, 64, true>(op, buf, a, s);
}

// Whether some agent can exceed the default separable kernel's 16 CBF row slots (caller lists,
// or k nearest x CBF samples > 16).
bool impc_rows_may_exceed(const DevOps& op, bool csr, int knn_k) { return csr || knn_k * op.cbf_h > 16; }

// Whether launch_impc defers agents (so launch_impc_fallback must follow): the lean main launches
// always may; the full separable kernel and the wide kernel with the inline fallback when their 16
// CBF row slots can be exceeded.
bool impc_may_defer(const DevOps& op, int variant, bool csr, int knn_k, int n) {
    // slack mode: more than 16 neighbours only from caller lists (grid mode takes knn_k <= 16,
    // impc_enqueue)
    if (op.slack_mode) return slack_sb(op) > 0 && csr;
    if (use_wide(op, variant, n) || sep_lean(op, variant, n)) return true;
    if (!(sep_variant(variant) && op.sep && op.nzd == SEP_NZD_HOST && op.sep_rows_per_dim <= 16)) return false;
    return impc_rows_may_exceed(op, csr, knn_k);
}

// Waves of the main IMPC launch for n agents that write the launch clock (ImpcArgs::kclock: the
// separable and wide collision kernels; 0 for the others)
int impc_clock_waves(const DevOps& op, int variant, int n) {
    if (n <= 0 || op.cbf_mode != 0) return 0;
    if (use_wide(op, variant, n)) return ((n + 3) / 4) * 4;  // 256-thread blocks, one agent per wave
    const bool sep = op.sep && op.nzd == SEP_NZD_HOST && op.sep_rows_per_dim <= 16;
    if (op.slack_mode && slack_sb(op) == 2) return ((n + 7) / 8) * 2;  // 128-thread blocks of 8 groups
    if (op.slack_mode ? slack_sb(op) > 0 : (sep && sep_variant(variant)))
        return ((n + 15) / 16) * 4;  // 256-thread blocks of 16 groups
    return 0;
}

// Instantiation launch_impc picks for (operators, variant, agents per launch); nullptr if none fits.
const char* impc_kernel_name(const DevOps& op, int variant, int n) {
    if (op.slack_mode) {  // slack variables: separable layout, one lane per neighbour, cbf_h <= 2
        const int sb = slack_sb(op);
        return sb == 1 ? "impc_sep_kernel<1,2,true,256>" : (sb == 2 ? "impc_sep_kernel<2,2,true,128>" : nullptr);
    }
    if (use_wide(op, variant, n)) return "impc_wide_kernel<256>";
    if (sep_lean(op, variant, n)) return "impc_sep_kernel<1,1,false,256,false,true>";
    if (sep_variant(variant) && op.sep && op.nzd == SEP_NZD_HOST && op.sep_rows_per_dim <= 16)
        return "impc_sep_kernel<1,1,false,256>";
    if (op.nz == 6) {
        if ((variant == 0 || variant == 3) && op.m < 64) return "impc_kernel<6,16,4>";
        if (variant == 1 && op.m < 64) return "impc_kernel<6,64,1>";
        if (op.m < 256) return "impc_kernel<6,64,4>";
    }
    return nullptr;
}

hipError_t launch_impc(const DevOps& op, const double* buf, const ImpcArgs& a, int variant,
                       hipStream_t s) {
    if (a.num_agents <= 0) return hipSuccess;
    if (op.slack_mode) {
        const int sb = slack_sb(op);
        if (sb == 1) return launch_impc_sep_t<1, 2, true>(op, buf, a, s);
        // (two box slots per lane: 128-thread blocks, the 256-thread block's LDS is past 160 KB)
        if (sb == 2) return launch_impc_sep_t<2, 2, true, 128>(op, buf, a, s);
        return hipErrorInvalidValue;
    }
    if (use_wide(op, variant, a.num_agents)) return launch_impc_wide(op, buf, a, s);
    if (sep_lean(op, variant, a.num_agents)) return launch_impc_sep_t<1, 1, false, 256, false, true>(op, buf, a, s);
    if (sep_variant(variant) && op.sep && op.nzd == SEP_NZD_HOST && op.sep_rows_per_dim <= 16) {
        return launch_impc_sep_t<1, 1, false>(op, buf, a, s);
    }
    if (op.nz == 6) {
        if ((variant == 0 || variant == 3) && op.m < 64) return launch_impc_t<6, 16, 4>(op, buf, a, s);
        if (variant == 1 && op.m < 64) return launch_impc_t<6, 64, 1>(op, buf, a, s);
        if (op.m < 256) return launch_impc_t<6, 64, 4>(op, buf, a, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace mpccbf
