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
#include "pdip.hpp"
#include "pdip_sep.hpp"

namespace mpccbf {
namespace dev {

__device__ __forceinline__ const double* opp(const double* buf, int off) { return buf + off; }

// Safety HOCBF row of ConnectivityCBF::initSafetyCBF (cbf/src/detail/ConnectivityCBF.cpp:152-198)
// evaluated at (ego e, neighbour nb): a = L_g L_f h = (2dx, 2dy, 0),
// b = L_f^2 h + L_f alpha(h) + alpha(L_f h + alpha(h)), alpha(x) = 5 x^3 (gamma = 5, :62, :19-21),
// where L_f alpha differentiates the ego position only (f = A x, :171-184).
__device__ __forceinline__ void safety_cbf(const double e[6], double npx, double npy, double nvx,
                                           double nvy, double dmin, double a[3], double& b) {
    constexpr double gamma = 5.0;
    const double dx = e[0] - npx, dy = e[1] - npy;
    const double dvx = e[3] - nvx, dvy = e[4] - nvy;
    const double hh = dx * dx + dy * dy - dmin * dmin;
    const double lfh = 2.0 * (dx * dvx + dy * dvy);
    const double lf2h = 2.0 * (dvx * dvx + dvy * dvy);
    const double alpha_h = gamma * hh * hh * hh;
    const double lf_alpha = 3.0 * gamma * hh * hh * (2.0 * dx * e[3] + 2.0 * dy * e[4]);
    const double psi = lfh + alpha_h;
    b = lf2h + lf_alpha + gamma * psi * psi * psi;
    a[0] = 2.0 * dx;
    a[1] = 2.0 * dy;
    a[2] = 0.0;
}

// Per-group LDS scratch of the grid neighbour query.
struct NbScratch {
    int32_t idx[NB_CAP];   // candidate / final neighbour indices
    int32_t tmp[NB_CAP];   // sorted output
    double d2[NB_CAP];     // candidate squared distances
    int32_t keep[NB_CAP];  // k-nearest flags
};

// k nearest other agents (planar distance, ties by index) within the radius, found through the
// spatial hash; the result is left in sc.idx sorted by agent index. Returns the count, or -1 if
// more than NB_CAP candidates lie within the radius. Distance-only test: agents of a colliding
// cell that share a bucket are still filtered by distance, and a bucket reached from two of the
// 9 cells is scanned once.
template <int G>
__device__ int grid_neighbors(const ImpcArgs& args, int self, double px, double py, NbScratch& sc,
                              int gl) {
    const GridArgs& gr = args.grid;
    const long long cx = (long long)floor(px * gr.inv_cell), cy = (long long)floor(py * gr.inv_cell);
    const double r2 = gr.radius * gr.radius;
    uint32_t hs[9], b0[9], b1[9];
#pragma unroll
    for (int c = 0; c < 9; c++) {
        hs[c] = cell_hash(cx + (c % 3) - 1, cy + (c / 3) - 1, gr.mask);
        b0[c] = gr.start[hs[c]];
        b1[c] = gr.start[hs[c] + 1];
    }
    int cnt = 0;
#pragma unroll
    for (int c = 0; c < 9; c++) {
        bool dup = false;
#pragma unroll
        for (int p = 0; p < c; p++) dup = dup || (hs[p] == hs[c]);
        if (dup) continue;
        for (uint32_t base = b0[c]; base < b1[c]; base += G) {
            const uint32_t e = base + gl;
            bool keep = false;
            int j = -1;
            double d2 = 0.0;
            if (e < b1[c]) {
                j = (int)gr.sorted[e];
                const double ex = args.states[(size_t)j * 6] - px;
                const double ey = args.states[(size_t)j * 6 + 1] - py;
                d2 = ex * ex + ey * ey;
                keep = (j != self) && (d2 <= r2);
            }
            const unsigned long long msk = grp_ballot<G>(keep);
            const int slot = cnt + __popcll(msk & ((1ull << gl) - 1ull));
            if (keep && slot < NB_CAP) {
                sc.idx[slot] = j;
                sc.d2[slot] = d2;
            }
            cnt += __popcll(msk);
        }
    }
    if (cnt > NB_CAP) return -1;
    wave_lds_sync();
    // rank by (d2, index): keep the k nearest
    const int k = gr.k;
    for (int i = gl; i < cnt; i += G) {
        const double di = sc.d2[i];
        const int ji = sc.idx[i];
        int rank = 0;
        for (int m = 0; m < cnt; m++) {
            const double dm = sc.d2[m];
            rank += (dm < di || (dm == di && sc.idx[m] < ji)) ? 1 : 0;
        }
        sc.keep[i] = rank < k ? 1 : 0;
    }
    const int nk = cnt < k ? cnt : k;
    wave_lds_sync();
    // order the kept set by agent index
    for (int i = gl; i < cnt; i += G) {
        if (sc.keep[i]) {
            const int ji = sc.idx[i];
            int pos = 0;
            for (int m = 0; m < cnt; m++) pos += (sc.keep[m] && sc.idx[m] < ji) ? 1 : 0;
            sc.tmp[pos] = ji;
        }
    }
    wave_lds_sync();
    for (int i = gl; i < nk; i += G) sc.idx[i] = sc.tmp[i];
    wave_lds_sync();
    return nk;
}

// ---------------------------------------------------------------------------------------------
// Steps shared by both layouts
// ---------------------------------------------------------------------------------------------

// q = Qs s0 + Qt t (or Qs s0 + Qr ref tail) and the objective constant.
template <int NZ>
__device__ __forceinline__ void agent_linear_term(const DevOps& op, const double* buf,
                                                  const ImpcArgs& args, int ai, const double (&s0)[6],
                                                  double (&q)[NZ], double& kconst) {
    const double* Qs = opp(buf, op.o_Qs);
    const double* Ks = opp(buf, op.o_Ks);
    kconst = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; i++) {
        double v = 0.0;
#pragma unroll
        for (int s = 0; s < 6; s++) v = fma(Qs[i * 6 + s], s0[s], v);
        q[i] = v;
    }
#pragma unroll
    for (int s = 0; s < 6; s++) {
        double v = 0.0;
#pragma unroll
        for (int u = 0; u < 6; u++) v = fma(Ks[s * 6 + u], s0[u], v);
        kconst = fma(s0[s], v, kconst);
    }
    if (args.targets) {
        const double* Qt = opp(buf, op.o_Qt);
        const double* Kt = opp(buf, op.o_Kt);
        double t[3];
#pragma unroll
        for (int d = 0; d < 3; d++) t[d] = args.targets[(size_t)ai * 3 + d];
#pragma unroll
        for (int i = 0; i < NZ; i++)
#pragma unroll
            for (int d = 0; d < 3; d++) q[i] = fma(Qt[i * 3 + d], t[d], q[i]);
#pragma unroll
        for (int d = 0; d < 3; d++) {
            double v = 0.0;
#pragma unroll
            for (int s = 0; s < 6; s++) v = fma(Kt[d * 6 + s], s0[s], v);
            kconst = fma(t[d], v, kconst);
        }
    } else {
        const double* Qr = opp(buf, op.o_Qr);
        const double* Kr = opp(buf, op.o_Kr);
        const int nr = 3 * op.spd_f;
        const double* rt = args.refs + (size_t)ai * 3 * op.K + 3 * (op.K - op.spd_f);
        for (int j = 0; j < nr; j++) {
            const double rv = rt[j];
#pragma unroll
            for (int i = 0; i < NZ; i++) q[i] = fma(Qr[i * nr + j], rv, q[i]);
            double v = 0.0;
#pragma unroll
            for (int s = 0; s < 6; s++) v = fma(Kr[j * 6 + s], s0[s], v);
            kconst = fma(rv, v, kconst);
        }
    }
}

// Constant rows (zero in y): pure feasibility checks on s0, group-uniform result.
template <int G>
__device__ __forceinline__ bool constant_rows_infeasible(const DevOps& op, const double* buf,
                                                         const double (&s0)[6], int gl) {
    const double* Cs = opp(buf, op.o_Cs);
    const double* clo = opp(buf, op.o_clo);
    const double* chi = opp(buf, op.o_chi);
    bool bad = false;
    for (int i = gl; i < op.mc; i += G) {
        double v = 0.0;
#pragma unroll
        for (int s = 0; s < 6; s++) v = fma(Cs[i * 6 + s], s0[s], v);
        if (v < clo[i] - op.feas_tol || v > chi[i] + op.feas_tol) bad = true;
    }
    return grp_ballot<G>(bad) != 0ull;
}

// Ego state the CBF rows are evaluated at: s0 (iteration 0) or the previous curve at
// h_samples(k) (iteration 1, ConnectivityIMPCCBF.cpp:161-168).
template <int NZ>
__device__ __forceinline__ void cbf_ego_state(const DevOps& op, const double* buf, int it, int k,
                                              const double (&s0)[6], const double (&y)[NZ], double (&e)[6]) {
    if (it == 0) {
#pragma unroll
        for (int s = 0; s < 6; s++) e[s] = s0[s];
        return;
    }
    const double* PZ = opp(buf, op.o_PZ) + (size_t)k * 6 * NZ;
    const double* PS = opp(buf, op.o_PS) + (size_t)k * 36;
#pragma unroll
    for (int s = 0; s < 6; s++) {
        double v = 0.0;
#pragma unroll
        for (int u = 0; u < 6; u++) v = fma(PS[s * 6 + u], s0[u], v);
#pragma unroll
        for (int j = 0; j < NZ; j++) v = fma(PZ[s * NZ + j], y[j], v);
        e[s] = v;
    }
}

// CBF rows of one IMPC iteration, filtered and compacted into `stage` ((NZ + 1) doubles per
// row: coefficients then upper bound). Returns the group-uniform row count; *infeasible is set
// when a single row already excludes every acceleration in the box.
template <int NZ, int G>
__device__ int stage_cbf_rows(const DevOps& op, const double* buf, const ImpcArgs& args, int it,
                              const double (&s0)[6], const double (&y)[NZ], bool grid_mode,
                              const int32_t* nbl, int nb0, int nnb, double* stage, int cap, int gl,
                              bool* infeasible) {
    const double* UZ = opp(buf, op.o_UZ);
    const double* US = opp(buf, op.o_US);
    const int nk = (it == 0) ? 1 : op.cbf_h;
    int count = 0;
    bool row_infeasible = false;
    for (int k = 0; k < nk; k++) {
        double e[6];
        cbf_ego_state<NZ>(op, buf, it, k, s0, y, e);
        // U_k s0 part of the acceleration at sample k
        const double* UZk = UZ + (size_t)k * 3 * NZ;
        const double* USk = US + (size_t)k * 18;
        double us[3];
#pragma unroll
        for (int d = 0; d < 3; d++) {
            double v = 0.0;
#pragma unroll
            for (int s = 0; s < 6; s++) v = fma(USk[d * 6 + s], s0[s], v);
            us[d] = v;
        }
        for (int base = 0; base < nnb; base += G) {
            const int j = base + gl;
            bool keep = false;
            double a[3] = {0.0, 0.0, 0.0}, b = 0.0;
            if (j < nnb) {
                const int nbi = grid_mode ? nbl[j] : args.nb_col[nb0 + j];
                const double* ns = args.states + (size_t)nbi * 6;
                safety_cbf(e, ns[0], ns[1], ns[3], ns[4], op.d_min, a, b);
                // max / min of -a^T u over the acceleration box at sample k (those box rows
                // are part of every QP): b >= max  -> the row is implied (exactly redundant);
                // b < min - tol -> no acceleration satisfies it (infeasible).
                double bmax = 0.0, bmin = 0.0;
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    const double v1 = -a[d] * op.a_lo[d], v2 = -a[d] * op.a_hi[d];
                    bmax += fmax(v1, v2);
                    bmin += fmin(v1, v2);
                }
                keep = !(op.cbf_filter && b >= bmax);
                if (b < bmin - op.feas_tol) row_infeasible = true;
            }
            const unsigned long long msk = grp_ballot<G>(keep);
            const int slot = count + __popcll(msk & ((1ull << gl) - 1ull));
            if (keep && slot < cap) {
                double* dst = stage + (size_t)slot * (NZ + 1);
                // row: -a^T (US_k s0 + UZ_k y) <= b
#pragma unroll
                for (int jz = 0; jz < NZ; jz++)
                    dst[jz] = -(a[0] * UZk[jz] + a[1] * UZk[NZ + jz] + a[2] * UZk[2 * NZ + jz]);
                dst[NZ] = b + (a[0] * us[0] + a[1] * us[1] + a[2] * us[2]);
            }
            count += __popcll(msk);
        }
    }
    *infeasible = grp_ballot<G>(row_infeasible) != 0ull;
    wave_lds_sync();
    return count;
}

// Objective value 1/2 y^T P y + q^T y + k at the solution (x^T H x + c^T x of the full QP).
template <int NZ>
__device__ __forceinline__ double reduced_objective(const DevOps& op, const double* buf,
                                                   const double (&q)[NZ], const double (&y)[NZ],
                                                   double kconst) {
    const double* Pr = opp(buf, op.o_Pr);
    double v = kconst;
#pragma unroll
    for (int i = 0; i < NZ; i++) {
        double pyi = 0.0;
#pragma unroll
        for (int j = 0; j < NZ; j++) pyi = fma(Pr[i * NZ + j], y[j], pyi);
        v = fma(y[i], 0.5 * pyi + q[i], v);
    }
    return v;
}

// Control points of the kept curve and the closed-loop next state (curve at t = h).
template <int NZ, int G>
__device__ __forceinline__ void write_agent_outputs(const DevOps& op, const double* buf,
                                                    const ImpcArgs& args, int ai, int gl,
                                                    const double (&s0)[6], const double (&yk)[NZ],
                                                    bool have_curve) {
    if (args.x) {
        const double* Z = opp(buf, op.o_Z);
        const double* Xs = opp(buf, op.o_Xs);
        for (int i = gl; i < op.n; i += G) {
            double v = 0.0;
            if (have_curve) {
#pragma unroll
                for (int s = 0; s < 6; s++) v = fma(Xs[i * 6 + s], s0[s], v);
#pragma unroll
                for (int j = 0; j < NZ; j++) v = fma(Z[i * NZ + j], yk[j], v);
            } else {
                v = __builtin_nan("");
            }
            args.x[(size_t)ai * op.n + i] = v;
        }
    }
    if (args.next_states && gl < 6) {
        double v = 0.0;
        if (have_curve) {
            const double* AZ = opp(buf, op.o_AZ);
            const double* AS = opp(buf, op.o_AS);
#pragma unroll
            for (int s = 0; s < 6; s++) v = fma(AS[gl * 6 + s], s0[s], v);
#pragma unroll
            for (int j = 0; j < NZ; j++) v = fma(AZ[gl * NZ + j], yk[j], v);
        } else {
#pragma unroll
            for (int s = 0; s < 6; s++)
                if (s == gl) v = s0[s];
        }
        args.next_states[(size_t)ai * 6 + gl] = v;
    }
}

// diagnostics: wall-clock stamp (s_memrealtime, 100 MHz, chip-wide) of phase `k` of agent ai
__device__ __forceinline__ void stamp(const ImpcArgs& args, int ai, int gl, int k) {
    if (args.stamps) {
        const long long t = (long long)__builtin_amdgcn_s_memrealtime();
        if (gl == 0) args.stamps[(size_t)ai * NSTAMP + k] = t;
    }
}

__device__ __forceinline__ void write_iteration(const ImpcArgs& args, size_t oi, int gl, int st,
                                                double obj, int iters) {
    if (gl == 0) {
        if (args.status) args.status[oi] = st;
        if (args.obj) args.obj[oi] = obj;
        if (args.iters) args.iters[oi] = iters;
    }
}

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
        const int count = stage_cbf_rows<NZ, G>(op, buf, args, it, s0, y, grid_mode, nb_scratch[gib].idx,
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
        if (count > cap || nb_overflow) {
            st = ST_ERROR;  // capacity: caller re-runs with a wider instantiation
        } else if (infeasible || row_infeasible) {
            st = ST_INFEASIBLE;
        } else {
            const PdipOut po =
                pdip_solve<NZ, G, R>(rw, opp(buf, op.o_Pr), opp(buf, op.o_LPr), q, y, cfg);
            st = po.status;
            nit = po.iters;
            if (st != ST_OPTIMAL) {
                // certify: minimal uniform row violation above the feasibility tolerance
                const double tstar = pdip_phase1<NZ, G, R>(rw, cfg);
                if (tstar > op.feas_tol) st = ST_INFEASIBLE;
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
        write_iteration(args, oi, gl, st, objv, nit);
        if (it < 2) stamp(args, ai, gl, 4 + 2 * it);
        wave_lds_sync();  // staging is rewritten by the next iteration
    }
    write_agent_outputs<NZ, G>(op, buf, args, ai, gl, s0, ykeep, have_curve);
    stamp(args, ai, gl, 7);
}

// ---------------------------------------------------------------------------------------------
// Separable layout (x / y / yaw channels, 2 reduced variables each; pdip_sep.hpp)
// ---------------------------------------------------------------------------------------------
template <int SB, int CB>
__global__ void __launch_bounds__(256) impc_sep_kernel(const DevOps op, const double* __restrict__ buf,
                                                        const ImpcArgs args) {
    constexpr int G = 16;
    constexpr int NZ = SEP_NZ;
    constexpr int GPB = 256 / G;
    constexpr int cap = CB * G;  // CBF rows per agent
    const int gl = threadIdx.x & (G - 1);
    const int gib = threadIdx.x / G;
    const int ai = blockIdx.x * GPB + gib;
    if (ai >= args.num_agents) return;
    stamp(args, ai, gl, 0);

    __shared__ double stage_all[GPB][cap * (NZ + 1)];
    double* stage = stage_all[gib];

    const int self = args.agent_first + ai;
    double s0[6];
#pragma unroll
    for (int i = 0; i < 6; i++) s0[i] = args.states[(size_t)self * 6 + i];
    double q[NZ], kconst;
    agent_linear_term<NZ>(op, buf, args, ai, s0, q, kconst);

    // ---- box rows: channel d, slot k -> row k * G + gl of that channel (packed by the host:
    // per row [g0, g1, Gs(6), lo, hi], two-sided; unused rows inert: g = 0, Gs = 0, [-1, 1])
    SepRows<SB, CB> rw;
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
    const bool infeasible = constant_rows_infeasible<G>(op, buf, s0, gl);
    stamp(args, ai, gl, 1);

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
    stamp(args, ai, gl, 2);

    double y[NZ], ykeep[NZ];
#pragma unroll
    for (int i = 0; i < NZ; i++) y[i] = ykeep[i] = 0.0;
    bool have_curve = false, success = true;
    const PdipCfg cfg{op.maxit, op.tol};

    for (int it = 0; it < op.impc_iter; it++) {
        const size_t oi = (size_t)ai * op.impc_iter + it;
        if (!success) {
            write_iteration(args, oi, gl, ST_UNKNOWN, __builtin_nan(""), 0);
            continue;
        }
        bool row_infeasible = false;
        const int count = stage_cbf_rows<NZ, G>(op, buf, args, it, s0, y, grid_mode, nb_scratch[gib].idx,
                                                nb0, nnb, stage, cap, gl, &row_infeasible);
        if (it < 2) stamp(args, ai, gl, 3 + 2 * it);
#pragma unroll
        for (int c = 0; c < CB; c++) {
            const int ci = c * G + gl;
            const bool on = ci < count && ci < cap;
            const double* src = stage + (size_t)(on ? ci : 0) * (NZ + 1);
#pragma unroll
            for (int j = 0; j < 4; j++) rw.cg[c][j] = on ? src[j] : 0.0;  // yaw columns are 0
            rw.chi[c] = on ? src[NZ] : 1.0;  // unused slot: inert row 0 <= 1
        }
        int st;
        int nit = 0;
        if (count > cap || nb_overflow) {
            st = ST_ERROR;
        } else if (infeasible || row_infeasible) {
            st = ST_INFEASIBLE;
        } else {
#ifdef MPCCBF_PDIP_STAMPS
            long long* dbg = (args.stamps && it == 0)
                                 ? (long long*)args.stamps + (size_t)args.num_agents * NSTAMP + (size_t)ai * 16
                                 : nullptr;
#else
            long long* dbg = nullptr;
#endif
            const PdipOut po = pdip_solve_sep<G, SB, CB>(rw, count > 0, opp(buf, op.o_Pr),
                                                         opp(buf, op.o_LPr), q, y, cfg, dbg);
            st = po.status;
            nit = po.iters;
            if (st != ST_OPTIMAL) {
                const double tstar = pdip_phase1_sep<G, SB, CB>(rw, cfg);
                if (tstar > op.feas_tol) st = ST_INFEASIBLE;
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
        write_iteration(args, oi, gl, st, objv, nit);
        if (it < 2) stamp(args, ai, gl, 4 + 2 * it);
        wave_lds_sync();
    }
    write_agent_outputs<NZ, G>(op, buf, args, ai, gl, s0, ykeep, have_curve);
    stamp(args, ai, gl, 7);
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

template <int SB, int CB>
static hipError_t launch_impc_sep_t(const DevOps& op, const double* buf, const ImpcArgs& a,
                                    hipStream_t s) {
    constexpr int GPB = 256 / 16;
    const int blocks = (a.num_agents + GPB - 1) / GPB;
    hipLaunchKernelGGL((dev::impc_sep_kernel<SB, CB>), dim3(blocks), dim3(256), 0, s, op, buf, a);
    return hipGetLastError();
}

// Instantiation launch_impc picks for (operators, variant); nullptr if none fits.
const char* impc_kernel_name(const DevOps& op, int variant) {
    if (variant == 0 && op.sep && op.nzd == SEP_NZD_HOST && op.sep_rows_per_dim <= 16) return "impc_sep_kernel<1,1>";
    if (op.nz == 6) {
        if ((variant == 0 || variant == 3) && op.m < 64) return "impc_kernel<6,16,4>";
        if (variant == 1 && op.m < 64) return "impc_kernel<6,64,1>";
        if (op.m < 256) return "impc_kernel<6,64,4>";
    }
    return nullptr;
}

// Returns hipErrorInvalidValue if no instantiation fits (nz, m).
//   variant 0: separable layout when the operators allow it (16 lanes, 16 box rows per channel,
//              16 CBF rows), else 16 lanes x 4 dense slots
//   variant 1: dense, 64 lanes x 1 slot;  variant 2: dense, 64 lanes x 4 slots (wide rows)
//   variant 3: dense, 16 lanes x 4 slots (the pre-separable default)
hipError_t launch_impc(const DevOps& op, const double* buf, const ImpcArgs& a, int variant,
                       hipStream_t s) {
    if (a.num_agents <= 0) return hipSuccess;
    if (variant == 0 && op.sep && op.nzd == SEP_NZD_HOST && op.sep_rows_per_dim <= 16)
        return launch_impc_sep_t<1, 1>(op, buf, a, s);
    if (op.nz == 6) {
        if ((variant == 0 || variant == 3) && op.m < 64) return launch_impc_t<6, 16, 4>(op, buf, a, s);
        if (variant == 1 && op.m < 64) return launch_impc_t<6, 64, 1>(op, buf, a, s);
        if (op.m < 256) return launch_impc_t<6, 64, 4>(op, buf, a, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace mpccbf
