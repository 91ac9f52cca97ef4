// das_wave.hpp — dual active-set solve (Goldfarb & Idnani's method, range-space form) of one QP
// per wavefront on the layouts of pdip_wave.hpp: the FoV controller's first attempt, the PDIP
// solving only the QPs it hands on.
//
// From the unconstrained minimiser y = -P^-1 q, the violated side with the largest violation per
// unit P^-1 norm is the candidate; the direction z = P^-1 (n_p - N_A r) keeps the active sides exact
// and moves y onto the candidate unless an active multiplier reaches zero first, in which case
// that side leaves and the step is retried. Every step keeps the iterate dual feasible and raises
// the objective. With K = G_A P^-1 G_A^T = L L^T (k <= 15 active rows):
//   c = G_A P^-1 n_p,  v = L^-1 c,  r = L^-T v,  zn = n_p P^-1 n_p - |v|^2 (> 0: n_p independent)
// and a joining side appends (v^T, sqrt(zn)) to L; a leaving side refactors K.
//
// Layouts (64 lanes, i = lane & 15, the four 16-lane rows replicate): vectors of the reduced
// dimension and the per-active-row quantities (c, v, r, multipliers u) on the row layout — lane i
// holds element / active row i; L row i in lane i's registers and row-major in sc.M (the
// backward substitution reads its columns); the active rows' P^-1 g, image row, side sign and
// bound in LDS (WaveAS). Rows are read from the wave's row image Gs (16 doubles per row).
#pragma once

#include "pdip_wave.hpp"

namespace mpccbf {
namespace dev {

struct WaveAS {
    double W[WNZ * WNZ];     // active row a: P^-1 g_a (16 doubles)
    double Pi[WNZ * 17];     // P^-1, rows padded to 17 doubles (lane i reads row i: spread banks)
    double P[WNZ * 17];      // P, the same layout (dual residual)
    double w[WNZ];           // the candidate's P^-1 g
    double b[WNZ], sg[WNZ];  // active rows' bound and side sign (+1 upper, -1 lower)
    double u[WNZ];           // multipliers (shift scratch; at the optimum: the active rows')
    int32_t row[WNZ];        // active rows' image row
    int32_t k;               // at the optimum: the number of active rows
    float wn[WROWS];         // candidate weights 1 / sqrt(g P^-1 g) per image row
};

// row i of a 16 x 16 LDS matrix stored with row stride 17 times a 16-vector (LDS): every load first
// (interleaved with the FMAs the compiler waited for each pair of loads in turn), then the same
// sequential FMA chain
__device__ __forceinline__ double rowdot17(const double* M, int i, const double* v, double init = 0.0) {
    double m[WNZ], x[WNZ];
#pragma unroll
    for (int j = 0; j < WNZ; j++) {
        m[j] = M[i * 17 + j];
        x[j] = v[j];
    }
    __builtin_amdgcn_sched_barrier(0);
    double a = init;
#pragma unroll
    for (int j = 0; j < WNZ; j++) a = fma(m[j], x[j], a);
    return a;
}

// dotl with every load first, then the same two FMA chains (BATCH; the FoV slack kernel keeps the
// interleaved form, where the batch costs scratch)
template <bool BATCH>
__device__ __forceinline__ double dotl_b(const double* a, const double* b) {
    if constexpr (!BATCH) return dotl(a, b);
    double x[WNZ], z[WNZ];
#pragma unroll
    for (int j = 0; j < WNZ; j++) {
        x[j] = a[j];
        z[j] = b[j];
    }
    __builtin_amdgcn_sched_barrier(0);
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < WNZ; j += 2) {
        s0 = fma(x[j], z[j], s0);
        s1 = fma(x[j + 1], z[j + 1], s1);
    }
    return s0 + s1;
}

// a row (LDS) times a vector of scalar operands
__device__ __forceinline__ double dot_rows_s(const double* a, const double (&ys)[WNZ]) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < WNZ; j += 2) {
        s0 = fma(a[j], ys[j], s0);
        s1 = fma(a[j + 1], ys[j + 1], s1);
    }
    return s0 + s1;
}

// first half of solve_rows: v = L^-1 b on the row layout, over the first kk rows (kk wave-uniform:
// rows from kk on are identity rows of L with a zero right-hand side, v_i = 0 there)
__device__ __forceinline__ double fwd_rows(const double (&L)[WNZ], double inv_i, double b, int i, int kk) {
    double res = b, wl = 0.0;
#pragma unroll
    for (int k = 0; k < WNZ; k++) {
        if (k < kk) {  // (uniform branch; a break here defeats the full unroll the DPP needs)
            const double wk = bcast16v(k, res * inv_i);
            res = fma(-L[k], wk, res);
            wl = (i == k) ? wk : wl;
        }
    }
    return wl;
}

// second half of solve_rows: x = L^-T v (L's columns from the row-major copy Lm), over the first kk
// rows (v_i = 0 from kk on, so x_i = 0 there)
__device__ __forceinline__ double bwd_rows(const double* __restrict__ Lm, double inv_i, double v, int i, int kk) {
    double res = v, xl = 0.0;
#pragma unroll
    for (int k = WNZ - 1; k >= 0; k--) {
        if (k < kk) {
            const double xk = bcast16v(k, res * inv_i);
            res = fma(-Lm[k * WNZ + i], xk, res);
            xl = (i == k) ? xk : xl;
        }
    }
    return xl;
}

// P and P^-1 (16 x 16, global) into the workspace, once per agent: every das_solve_wave call of
// the agent reads them there (a per-call copy was a global round trip on each solve's chain).
// Also zeroes ws.W: the direction reads row 0 of it while the active set is empty and multiplies
// it by 0 (the slack patterns' unbounded loops, kk = 16); never written, it holds whatever an
// earlier kernel left in this LDS — NaN / Inf included, and 0 * NaN is NaN. That was round 3's
// FoV-slack step-0 nondeterminism (profiles/r04_lds_poison_nan.log). (Zeroed here rather than a
// select in the loop: the select pushed the FoV kernels from 0 / 76 to 524 / 972 B/lane of scratch.)
// BATCH: every load first (as a loop, each element's two loads were waited for before the next's;
// off in the FoV slack kernel, where the batch costs scratch).
template <bool BATCH = true>
__device__ __forceinline__ void das_load_operators(WaveAS& ws, const double* __restrict__ P,
                                                   const double* __restrict__ Pinv, int lane) {
    if constexpr (!BATCH) {
        for (int e = lane; e < WNZ * WNZ; e += 64) {
            ws.Pi[(e >> 4) * 17 + (e & 15)] = Pinv[e];
            ws.P[(e >> 4) * 17 + (e & 15)] = P[e];
            ws.W[e] = 0.0;
        }
        wave_lds_sync();
        return;
    }
    constexpr int NE = WNZ * WNZ / 64;
    double pi[NE], pp[NE];
#pragma unroll
    for (int k = 0; k < NE; k++) {
        pi[k] = Pinv[lane + 64 * k];
        pp[k] = P[lane + 64 * k];
    }
#pragma unroll
    for (int k = 0; k < NE; k++) {
        const int e = lane + 64 * k;
        ws.Pi[(e >> 4) * 17 + (e & 15)] = pi[k];
        ws.P[(e >> 4) * 17 + (e & 15)] = pp[k];
        ws.W[e] = 0.0;
    }
    wave_lds_sync();
}

// das_load_operators' stores from operands the caller loaded (P^-1 / P entries lane + 64 k)
__device__ __forceinline__ void das_store_operators(WaveAS& ws, const double (&pi)[WNZ * WNZ / 64],
                                                    const double (&pp)[WNZ * WNZ / 64], int lane) {
#pragma unroll
    for (int k = 0; k < WNZ * WNZ / 64; k++) {
        const int e = lane + 64 * k;
        ws.Pi[(e >> 4) * 17 + (e & 15)] = pi[k];
        ws.P[(e >> 4) * 17 + (e & 15)] = pp[k];
        ws.W[e] = 0.0;
    }
    wave_lds_sync();
}

// Returns 1: optimal (sc.y, rp_out, rd_out; the active rows' multipliers in ws.u[0 .. ws.k)); -1: no
// step reaches the candidate (no feasible point; tlow = the certificate's lower bound on phase
// 1's t*; cand = the unreachable candidate's image row, the active rows in ws.row[0 .. ws.k) with
// their certificate weights in ws.u: candidate + sum_a u_a n_a = 0); 0: gave up (step limit,
// breakdown, dual residual) — the PDIP solves.
// ws.Pi / ws.P: P^-1 and P (das_load_operators); the P / Pinv arguments are not read.
template <bool BOUND = true>
__device__ __forceinline__ int das_solve_wave(const WaveRows& rw, const double* __restrict__ Gs, WaveScratch& sc,
                              WaveAS& ws, const double* __restrict__ P, const double* __restrict__ Pinv,
                              double tol, int maxstep, bool want_rd, int lane, double& rp_out,
                              double& rd_out, int& steps, double& tlow, int* cand = nullptr,
                              int nfirst = 0, int nrows = WROWS, long long* dbg = nullptr,
                              bool want_rp = true) {
    (void)dbg;
#ifdef MPCCBF_PDIP_STAMPS  // profiling build: shader-clock stamps of the solve's first steps
#define WSTAMP(kk, cond)                                                              \
    do {                                                                              \
        if (dbg && lane == 0 && (cond)) dbg[kk] = (long long)__builtin_amdgcn_s_memtime(); \
    } while (0)
    if (dbg && lane == 0) dbg[15] = 2;
#else
#define WSTAMP(kk, cond) \
    do {                 \
    } while (0)
#endif
    WSTAMP(0, true);
    const int i = lane16_opaque(lane);
    steps = 0;
    (void)Pinv;  // (ws.Pi / ws.P: loaded once per agent by das_load_operators)
    // per-slot violation scales, the factor of the empty active set (identity)
    double pl[WR], pu[WR];
#pragma unroll
    for (int s = 0; s < WR; s++) {
        pl[s] = rw.ml[s] * rcp(1.0 + fabs(rw.lo[s]));
        pu[s] = rcp(1.0 + fabs(rw.hi[s]));
    }
    double L[WNZ], inv_i = 1.0, ui = 0.0;
#pragma unroll
    for (int k = 0; k < WNZ; k++) L[k] = k == i ? 1.0 : 0.0;
    if (lane < WNZ) {
#pragma unroll
        for (int k = 0; k < WNZ; k++) sc.M[i * WNZ + k] = k == i ? 1.0 : 0.0;
    }
    wave_lds_sync();
    // y = -P^-1 q
    double yi;
    {
        const double a = rowdot17(ws.Pi, i, sc.q);
        yi = -a;
    }
    publish16(sc.y, yi, lane);
    WSTAMP(1, true);
    int k = 0;
    double m = 0.0;
    const double add_tol = 0.1 * tol;
    // candidate rule (as pdip_sep.hpp sep_dual_as): among the sides violated beyond the tolerance
    // (scaled as the primal residual), the largest violation per unit P^-1 norm, v / sqrt(g P^-1 g).
    // On the FoV bench's infeasible iteration-1 QPs the scaled rule cycled 24 steps on average (47
    // at most) before the certificate, this rule 7 (12) (tools/das_sim.py --fov --it1). The
    // weights are formed once, at the first scan that finds a violation (most QPs never get
    // there), for the image rows nfirst .. nrows-1 (rows below nfirst are constant, their weights
    // the caller's): four rows per pass (one per 16-lane row of the wave; lane i forms
    // (P^-1 g)_i from P^-1's row i in LDS), kept in LDS.
    bool have_wn = nfirst >= nrows;  // (every weight given: no lazy pass)
    auto row_weights = [&]() {
        const int grp = lane >> 4;
        for (int r0 = nfirst; r0 < nrows; r0 += 4) {
            const int r = r0 + grp;
            const double* g = Gs + (r < nrows ? r : 0) * WNZ;
            const double w = rowdot17(ws.Pi, i, g);
            const double n2 = grp_sum<16>(g[i] * w);
            if (i == 0 && r < nrows) ws.wn[r] = rsqrtf((float)fmax(n2, 1e-30));
        }
        wave_lds_sync();
    };
    // the candidate weights of this lane's row slots, in registers once they exist
    float wnr[WR];
#pragma unroll
    for (int s = 0; s < WR; s++) {
        const int r = wave_owner_row(lane, s);
        wnr[s] = have_wn ? ws.wn[r < nrows ? r : 0] : 0.0f;
    }
    for (;;) {
        // every slot's row and the iterate (broadcast reads of sc.y) first: 32 LDS reads in flight
        // together (slot by slot, each slot's reads waited for the previous slot's arithmetic; the
        // iterate as 16 scalar operands took 32 readlanes and spilled scalar registers)
        double ts[WR];
        {
            double rr[WR][WNZ], yv[WNZ];
#pragma unroll
            for (int s = 0; s < WR; s++)
#pragma unroll
                for (int j = 0; j < WNZ; j++) rr[s][j] = rw.g[s][j];
#pragma unroll
            for (int j = 0; j < WNZ; j++) yv[j] = sc.y[j];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < WR; s++) {
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int j = 0; j < WNZ; j += 2) {
                    s0 = fma(rr[s][j], yv[j], s0);
                    s1 = fma(rr[s][j + 1], yv[j + 1], s1);
                }
                ts[s] = s0 + s1;
            }
        }
        // this lane's largest scaled violation (convergence) and its candidate: the eligible side
        // with the largest normalised violation (lowest slot on ties)
        double vb = -1.0, eb = -1.0;
        int rb = 0, sdb = 1;
        double bb = 0.0;
        bool nf = false;  // a NaN row or iterate fails every comparison: give up instead
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double t = ts[s];
            const double al = rw.lo[s] - t, au = t - rw.hi[s];
            const double vl = rw.ml[s] > 0.0 ? al * pl[s] : -1.0;
            const double vu = au * pu[s];
            const int r = wave_owner_row(lane, s);
            nf = nf || vl != vl || vu != vu;
            vb = fmax(vb, fmax(vl, vu));
            const double w = (double)wnr[s];
            const double el = vl > add_tol ? al * w : -1.0;
            const double eu = vu > add_tol ? au * w : -1.0;
            const bool tl = el > eb;
            eb = tl ? el : eb;
            rb = tl ? r : rb;
            sdb = tl ? 0 : sdb;
            bb = tl ? rw.lo[s] : bb;
            const bool tu = eu > eb;
            eb = tu ? eu : eb;
            rb = tu ? r : rb;
            sdb = tu ? 1 : sdb;
            bb = tu ? rw.hi[s] : bb;
        }
        if (__ballot(nf) != 0ull) return 0;
        WSTAMP(steps == 0 ? 2 : 8, steps <= 1);
        // converged: no side violated beyond add_tol (m = the scaled primal residual, reduced once)
        if (__ballot(vb > add_tol) == 0ull) {
            if (want_rp) m = grp_max<64>(vb);  // (only for the caller's primal-residual output)
            break;
        }
        if (!have_wn) {  // first violation: form the weights and scan again
            row_weights();
            have_wn = true;
#pragma unroll
            for (int s = 0; s < WR; s++) {
                const int r = wave_owner_row(lane, s);
                wnr[s] = ws.wn[r < nrows ? r : 0];
            }
            continue;
        }
        if (steps >= maxstep) return 0;
        // the candidate: the largest normalised violation as a float bit pattern (a violated side's
        // is positive: at least 1), its lowest lane on ties
        const unsigned key = eb > 0.0 ? max(__float_as_uint((float)eb), 1u) : 0u;
        const unsigned kmax = (unsigned)__builtin_amdgcn_readfirstlane((int)wave_max_u32(key));
        const int owner = __ffsll((long long)__ballot(key == kmax)) - 1;
        if (owner < 0) return 0;
        const int rp = __builtin_amdgcn_readlane(rb, owner);
        const double sp = __builtin_amdgcn_readlane(sdb, owner) ? 1.0 : -1.0;
        const double bp = readlane_d(bb, owner);
        const double* gp = Gs + rp * WNZ;
        // the candidate's P^-1 g on the row layout, published
        const double wi = rowdot17(ws.Pi, i, gp);
        publish16(ws.w, wi, lane);
        // n_p^T P^-1 n_p from the lanes' own products (a 16-lane sum), not read back from ws.w
        const double nw = grp_sum<16>(gp[i] * wi);
        WSTAMP(3, steps == 0);
        double up = 0.0;  // the candidate's multiplier
        for (;;) {
            if (++steps > maxstep) return 0;
            // BOUND: the active count as a wave-uniform bound — the substitutions, the direction and
            // the dual residual run over the active rows only (scalar branches; typically k <= 3 of
            // 15). The slack-pattern solves keep the full loops (bounded, their kernel spills).
            const int kk = BOUND ? __builtin_amdgcn_readfirstlane(k) : WNZ;
            // c_a = n_a-side coefficient: g_a P^-1 n_p (lane a < k), v = L^-1 c, r = L^-T v
            double ci = 0.0, sgi = 0.0;
            if (kk > 0) {
                const int ra = i < k ? ws.row[i] : rp;
                ci = i < k ? sp * dotl_b<BOUND>(Gs + ra * WNZ, ws.w) : 0.0;
                sgi = i < k ? ws.sg[i] : 0.0;
            }
            const double vi = fwd_rows(L, inv_i, ci, i, kk);
            const double rhoi = bwd_rows(sc.M, inv_i, vi, i, kk);
            const double zn = nw - grp_sum<16>(vi * vi);
            const double vp = sp * (grp_sum<16>(gp[i] * yi) - bp);  // (y's lanes in registers, as nw)
            WSTAMP(4, steps == 1);
            // dual step: the first active multiplier to reach zero
            const double r_i = sgi * rhoi;
            const double ratio = (i < k && r_i > 0.0) ? ui * rcp(r_i) : 1e300;
            const double t1 = grp_min<16>(ratio);
            const int l = t1 < 1e300 ? __ffsll((long long)grp_ballot<16>(ratio == t1)) - 1 : -1;
            const bool full = zn > 1e-10 * nw;  // else n_p lies in the span of the active sides
            const double t2 = full ? vp * rcp(zn) : 1e300;
            WSTAMP(5, steps == 1);
            if (l < 0 && !full) {
                // certificate lam = (1, -r) >= 0 (every r <= 0): t* >= vp / (1 - sum r)
                tlow = vp * rcp(1.0 + grp_sum<16>((i < k && r_i < 0.0) ? -r_i : 0.0));
                if (lane < WNZ) ws.u[lane] = (i < k && r_i < 0.0) ? -r_i : 0.0;
                if (lane == 0) ws.k = k;
                if (cand) *cand = rp;
                wave_lds_sync();
                return -1;
            }
            const double t = fmin(t1, t2);
            if (full) {
                double zi = sp * wi;
#pragma unroll
                for (int a = 0; a < WNZ - 1; a++) {
                    if (a < kk) {
                        const double ra_ = bcast16v(a, rhoi);
                        // (rows a >= k: ws.W finite, zeroed by das_load_operators, times 0)
                        zi = fma(a < k ? -ra_ : 0.0, ws.W[(a < k ? a : 0) * WNZ + i], zi);
                    }
                }
                yi = fma(-t, zi, yi);
            }
            ui = i < k ? fma(-t, r_i, ui) : ui;
            up += t;
            publish16(sc.y, yi, lane);
            WSTAMP(6, steps == 1);
            if (t2 <= t1) {  // the candidate joins: L gains (v^T, sqrt(zn))
                if (k == WNZ - 1) return 0;
                const double dz = sqrt(zn), rz = rcp(dz);
                // K's new column (g-form) is c / sp: L's new row is L^-1 c / sp = sp v
                if (lane < WNZ) {
                    ws.W[k * WNZ + lane] = wi;
                    sc.M[k * WNZ + lane] = lane < k ? sp * vi : (lane == k ? dz : 0.0);
                }
                if (lane == 0) {
                    ws.row[k] = rp;
                    ws.sg[k] = sp;
                    ws.b[k] = bp;
                }
#pragma unroll
                for (int j = 0; j < WNZ; j++) {
                    const double vj = sp * bcast16v(j, vi);
                    L[j] = (i == k) ? (j < k ? vj : (j == k ? dz : 0.0)) : L[j];
                }
                inv_i = i == k ? rz : inv_i;
                ui = i == k ? up : ui;
                k++;
                wave_lds_sync();
                WSTAMP(7, steps == 1);
                break;
            }
            // side l leaves: rows above it move down (lane j: column j), K refactored
            if (lane < WNZ) ws.u[lane] = ui;
            wave_lds_sync();
            if (lane < WNZ) {
                for (int a = l; a < k - 1; a++) ws.W[a * WNZ + lane] = ws.W[(a + 1) * WNZ + lane];
            }
            if (lane == 0) {
                for (int a = l; a < k - 1; a++) {
                    ws.row[a] = ws.row[a + 1];
                    ws.sg[a] = ws.sg[a + 1];
                    ws.b[a] = ws.b[a + 1];
                }
            }
            ui = i >= l ? (i + 1 < k ? ws.u[i + 1] : 0.0) : ui;
            k--;
            wave_lds_sync();
            double Kr[WNZ];
            {
                const double* gi_ = Gs + (i < k ? ws.row[i] : 0) * WNZ;
#pragma unroll
                for (int b = 0; b < WNZ; b++)
                    Kr[b] = (i < k && b < k) ? dotl_b<BOUND>(gi_, ws.W + b * WNZ) : (i == b ? 1.0 : 0.0);
            }
            if (!chol_rows(Kr, L, inv_i, sc.M, lane)) return 0;
        }
    }
    // a non-finite iterate fails every violation test, so it would pass as converged: give up
    WSTAMP(9, true);
    if (dbg && lane == 0) dbg[14] = steps;
    if (__ballot(!isfinite(yi)) != 0ull) return 0;
    // converged: primal residual = the last scan's worst violation; dual residual of the iterate
    // P y + q + G_A^T lam (lam_a = sign_a u_a), checked whether or not the caller stores it when a
    // side is active
    // With no active side the iterate is -P^-1 q (P^-1 from the host): its dual residual is rounding,
    // so (BOUND) it is only evaluated when the caller stores it.
    double rd = 0.0;
    const int kk = BOUND ? __builtin_amdgcn_readfirstlane(k) : WNZ;
    if (kk > 0 || want_rd) {
        double r = rowdot17(ws.P, i, sc.y, sc.q[i]);
        const double lsi = ui * (i < k ? ws.sg[i < k ? i : 0] : 0.0);
        // (up to 4 active rows, the usual case: every index and entry load first, no branch per
        // row — 50.0 -> 49.7 us per FoV launch; beyond, the loop over the active rows)
        if (kk <= 4) {
            int ra[4];
            double gv[4];
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const int idx = ws.row[a];
                ra[a] = a < k ? idx : 0;
            }
#pragma unroll
            for (int a = 0; a < 4; a++) gv[a] = Gs[ra[a] * WNZ + i];
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const double la = bcast16v(a, lsi);
                r = fma(a < k ? la : 0.0, gv[a], r);
            }
        } else {
#pragma unroll
            for (int a = 0; a < WNZ - 1; a++) {
                if (a < kk) {
                    const double la = bcast16v(a, lsi);
                    r = fma(a < k ? la : 0.0, Gs[(a < k ? ws.row[a] : 0) * WNZ + i], r);
                }
            }
        }
        double qn = fabs(sc.q[i]);
        rd = grp_max<16>(fabs(r)) * rcp(1.0 + grp_max<16>(qn));
        if (!(rd <= tol)) return 0;
    }
    if (lane < WNZ) ws.u[lane] = i < k ? ui : 0.0;
    if (lane == 0) ws.k = k;
    rp_out = fmax(m, 0.0);
    rd_out = rd;
    WSTAMP(10, true);
    return 1;
}
#undef WSTAMP

}  // namespace dev
}  // namespace mpccbf
