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
    double ccv[CB];                 // slack mode: 1 if the row carries -v of this lane's neighbour
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

// Box-row duals of the last OPTIMAL solve: IMPC iteration 1 has the same box rows and cost as
// iteration 0 and differs only in its CBF rows, so it starts from iteration 0's primal-dual point.
template <int SB>
struct SepWarm {  // per-lane slots in the group's LDS ([2][SEP_D][SB][16] doubles): no registers
    double* base;
    __device__ __forceinline__ double& zl(int d, int k) const {
        return base[(d * SB + k) * 16 + (threadIdx.x & 15)];
    }
    __device__ __forceinline__ double& zu(int d, int k) const {
        return base[((SEP_D + d) * SB + k) * 16 + (threadIdx.x & 15)];
    }
};

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

// ---- Active-set solves (no slack variables)
// The equality-constrained QP on a set A of active sides,
//   min 1/2 y^T P y + q^T y  s.t.  g_i y = b_i (i in A),
// is solved exactly in the condensed space:
//   yu = -P^-1 q,   (G_A P^-1 G_A^T) lam = G_A yu - b_A,   y = yu - P^-1 G_A^T lam
// (P^-1 by 2x2 channel blocks; the k <= 6 rows staged in the group's LDS scratch `pol`, the k x k
// system factored redundantly by every lane). Its dual residual is zero up to rounding and
// complementarity exact; it is the QP's optimum when every row holds at y to the primal
// tolerance and every multiplier has its side's sign.
constexpr int POL_K = 6;
// staged row (16 doubles): g (6) | b | side sign (+1 upper, -1 lower) | P^-1 g (6) | side id | -
constexpr int POL_B = 6, POL_SGN = 7, POL_W = 8, POL_ID = 14;
// sep_dual_as scratch (doubles per group): POL_K staged rows + the candidate, then the candidate
// weights (one float per row and lane)
template <int SB, int CB>
constexpr int sep_pol_doubles() {
    return (POL_K + 1) * 16 + 8 * (3 * SB + CB);
}

// inverse of P's 2x2 channel blocks (DevOps::o_Pinv, computed on the host): pi[d] = (a, b, c)
// of [[a b] [b c]]
__device__ __forceinline__ void sep_pinv(const double* __restrict__ Pinv, double (&pi)[SEP_D][3]) {
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int e = 0; e < 3; e++) pi[d][e] = Pinv[d * 3 + e];
}

// Side s of this lane (s = 2 (d SB + kk) + upper for the box rows, 2 SEP_D SB + c for the CBF
// rows) staged as the 16-double row r; s may be a run-time value (the unrolled compares select).
template <int SB, int CB>
__device__ __forceinline__ void sep_stage_side(const SepRows<SB, CB>& rw, const double (&pi)[SEP_D][3], int s,
                                               int gl, double* __restrict__ r) {
    double g[SEP_NZ], b = 0.0, sg = 1.0;
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) g[j] = 0.0;
    int i = 0;
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int kk = 0; kk < SB; kk++)
#pragma unroll
            for (int side = 0; side < 2; side++, i++) {
                if (i != s) continue;
                g[2 * d] = rw.bg[d][kk][0];
                g[2 * d + 1] = rw.bg[d][kk][1];
                b = side ? rw.bhi[d][kk] : rw.blo[d][kk];
                sg = side ? 1.0 : -1.0;
            }
    if constexpr (CB > 2) {
        // (the wide capacity fallback: its rows live in LDS, so the slot is indexed directly — the
        // unrolled compares over 8 slots kept every slot's row in registers and spilled)
        const int c = s - i;
        if (c >= 0 && c < CB) {
#pragma unroll
            for (int j = 0; j < 4; j++) g[j] = rw.cg[c][j];
            b = rw.chi[c];
            sg = 1.0;
        }
    } else {
#pragma unroll
        for (int c = 0; c < CB; c++, i++) {
            if (i != s) continue;
#pragma unroll
            for (int j = 0; j < 4; j++) g[j] = rw.cg[c][j];
            b = rw.chi[c];
            sg = 1.0;
        }
    }
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) r[j] = g[j];
    r[POL_B] = b;
    r[POL_SGN] = sg;
#pragma unroll
    for (int d = 0; d < SEP_D; d++) {
        r[POL_W + 2 * d] = fma(pi[d][0], g[2 * d], pi[d][1] * g[2 * d + 1]);
        r[POL_W + 2 * d + 1] = fma(pi[d][1], g[2 * d], pi[d][2] * g[2 * d + 1]);
    }
    r[POL_ID] = (double)(s * 16 + gl);
}

// The EQP on the k staged rows of pol, verified: returns true (yo, scaled primal residual, relative
// dual residual ||P y + q + G_A^T lam||_inf / (1 + ||q||_inf) — RD false: 0, its value by
// construction, not re-evaluated where registers are short — and the multipliers as the next
// warm start's box duals) when every row holds at y to tol and every multiplier has its side's
// sign. sc: the sides' violation scales 1 / (1 + |bound|) (box lower, upper per slot, then CBF).
template <int G, int SB, int CB, bool RD, int NR = POL_K>
__device__ bool sep_eqp_finish(const SepRows<SB, CB>& rw, bool has_cbf, const double* __restrict__ P,
                               const double (&q)[SEP_NZ], const double (&yu)[SEP_NZ], int k,
                               const double* __restrict__ pol, const double (&sc)[2 * SEP_D * SB + CB],
                               double tol, double (&yo)[SEP_NZ], double& rp_out, double& rd_out,
                               SepWarm<SB>* warm, double* __restrict__ mult = nullptr) {
    const int gl = lane_bits_opaque<G - 1>();
    using S6 = Sym<NR>;
    double K[S6::P], rhs[NR], dk[NR], lam[NR];
#pragma unroll
    for (int i = 0; i < NR; i++) {
        const bool ai = i < k;
        const double* ri = pol + (ai ? i : 0) * 16;
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) t = fma(ri[j], yu[j], t);
        rhs[i] = ai ? t - ri[POL_B] : 0.0;
#pragma unroll
        for (int j = i; j < NR; j++) {
            const double* wj = pol + (j < k ? j : 0) * 16 + POL_W;
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < SEP_NZ; m++) v = fma(ri[m], wj[m], v);
            K[S6::idx(i, j)] = (ai && j < k) ? v : (i == j ? 1.0 : 0.0);
        }
    }
    const bool okf = chol_packed<NR>(K, dk);
    chol_solve<NR>(K, dk, rhs, lam);
    double y[SEP_NZ], lmax = 0.0;
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) y[j] = yu[j];
#pragma unroll
    for (int i = 0; i < NR; i++) {  // (lam_i = 0 beyond k: the padded rows read row 0)
        const double* wi = pol + (i < k ? i : 0) * 16 + POL_W;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) y[j] = fma(-lam[i], wi[j], y[j]);
        lmax = fmax(lmax, fabs(lam[i]));
    }
    bool bad = !okf;
#pragma unroll
    for (int i = 0; i < NR; i++)
        bad = bad || (i < k && !(pol[(i < k ? i : 0) * 16 + POL_SGN] * lam[i] >= -1e-9 * (1.0 + lmax)));
    // every row at y (scaled violation, as the PDIP's primal residual)
    double rp = 0.0;
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int kk = 0; kk < SB; kk++) {
            const double t = rw.bg[d][kk][0] * y[2 * d] + rw.bg[d][kk][1] * y[2 * d + 1];
            rp = fmax(rp, fmax((rw.blo[d][kk] - t) * sc[2 * (d * SB + kk)], (t - rw.bhi[d][kk]) * sc[2 * (d * SB + kk) + 1]));
        }
    if (has_cbf) {
#pragma unroll
        for (int c = 0; c < CB; c++) {
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < 4; j++) t = fma(rw.cg[c][j], y[j], t);
            rp = fmax(rp, (t - rw.chi[c]) * sc[2 * SEP_D * SB + c]);
        }
    }
    rp = grp_max<G>(rp);
    const bool ok = !bad && rp <= tol;
    if (ok) {
        // dual residual P y + q + G_A^T lam (group-uniform)
        double rd = 0.0, qn = 0.0;
#pragma unroll
        for (int d = 0; d < (RD ? SEP_D : 0); d++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int o = 2 * d + h;
                double v = fma(P[o * 6 + 2 * d], y[2 * d], fma(P[o * 6 + 2 * d + 1], y[2 * d + 1], q[o]));
#pragma unroll
                for (int i = 0; i < NR; i++) v = fma(lam[i], pol[(i < k ? i : 0) * 16 + o], v);
                rd = fmax(rd, fabs(v));
                qn = fmax(qn, fabs(q[o]));
            }
        }
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) yo[j] = y[j];
        rp_out = rp;
        rd_out = rd * rcp(1.0 + qn);
        if (warm != nullptr) {  // the multipliers as the next warm start's box duals
#pragma unroll
            for (int d = 0; d < SEP_D; d++)
#pragma unroll
                for (int kk = 0; kk < SB; kk++) {
                    const double il = (double)((2 * (d * SB + kk)) * 16 + gl), iu = il + 16.0;
                    double ml = 0.0, mu = 0.0;
#pragma unroll
                    for (int i = 0; i < NR; i++) {
                        const double id = i < k ? pol[(i < k ? i : 0) * 16 + POL_ID] : -1.0;
                        ml = id == il ? -lam[i] : ml;
                        mu = id == iu ? lam[i] : mu;
                    }
                    warm->zl(d, kk) = fmax(ml, 0.0);
                    warm->zu(d, kk) = fmax(mu, 0.0);
                }
        }
        if (mult != nullptr) {  // the active sides' multipliers (>= 0) and ids (sep_dual_as)
            double ui = 0.0;
#pragma unroll
            for (int i = 0; i < NR; i++) ui = gl == i ? pol[(i < k ? i : 0) * 16 + POL_SGN] * lam[i] : ui;
            if (gl < k) {
                mult[gl] = ui;
                mult[8 + gl] = pol[gl * 16 + POL_ID];
            }
            if (gl == 0) mult[7] = (double)k;
        }
    }
    wave_lds_sync();  // the scratch is reused
    return ok;
}

// Active-set finish of the PDIP: A = the iterate's active sides (slack below dual), when there
// are at most 6 of them.
template <int G, int SB, int CB>
__device__ bool sep_polish(const SepRows<SB, CB>& rw, bool has_cbf, const double* __restrict__ P,
                           const double* __restrict__ Pinv, const double (&q)[SEP_NZ], const double (&sl)[SEP_D][SB],
                           const double (&su)[SEP_D][SB], const double (&zl)[SEP_D][SB],
                           const double (&zu)[SEP_D][SB], const double (&cs)[CB], const double (&cz)[CB],
                           const double (&pl)[SEP_D][SB], const double (&pu)[SEP_D][SB],
                           const double (&pc)[CB], double tol, double* __restrict__ pol,
                           double (&yo)[SEP_NZ], double& rp_out, double& rd_out, SepWarm<SB>* warm) {
    const int gl = lane_bits_opaque<G - 1>();
    double pi[SEP_D][3], yu[SEP_NZ];
    sep_pinv(Pinv, pi);
#pragma unroll
    for (int d = 0; d < SEP_D; d++) {
        const int o = 2 * d;
        yu[o] = -fma(pi[d][0], q[o], pi[d][1] * q[o + 1]);
        yu[o + 1] = -fma(pi[d][1], q[o], pi[d][2] * q[o + 1]);
    }
    // active sides -> compact list (box lower / upper per channel and slot, then CBF rows)
    constexpr int NS = 2 * SEP_D * SB + CB;
    bool act[NS];
    int pos[NS], k = 0;
    {
        int s = 0;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int kk = 0; kk < SB; kk++) {
                act[s++] = sl[d][kk] < zl[d][kk];
                act[s++] = su[d][kk] < zu[d][kk];
            }
#pragma unroll
        for (int c = 0; c < CB; c++) act[s++] = has_cbf && cs[c] < cz[c];
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const unsigned long long m = grp_ballot<G>(act[s]);
        pos[s] = k + __popcll(m & ((1ull << gl) - 1ull));
        k += __popcll(m);
    }
    if (k == 0 || k > POL_K) return false;
#pragma unroll
    for (int s = 0; s < NS; s++)
        if (act[s]) sep_stage_side<SB, CB>(rw, pi, s, gl, pol + pos[s] * 16);
    wave_lds_sync();
    double sc[NS];
    {
        int s = 0;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int kk = 0; kk < SB; kk++) {
                sc[s++] = pl[d][kk];
                sc[s++] = pu[d][kk];
            }
#pragma unroll
        for (int c = 0; c < CB; c++) sc[s++] = pc[c];
    }
    return sep_eqp_finish<G, SB, CB, false>(rw, has_cbf, P, q, yu, k, pol, sc, tol, yo, rp_out, rd_out, warm);
}

// reduced_objective (1/2 y^T P y + q^T y + k) with P block-diagonal by channel: the same sums in
// the same order without the off-block terms, which add fma(0, y_j, s) = s — so bit-identical —
// from 12 entries of P instead of 36
__device__ __forceinline__ double sep_objective(const double* __restrict__ Pr, const double (&q)[SEP_NZ],
                                                const double (&y)[SEP_NZ], double kconst) {
    double v = kconst;
#pragma unroll
    for (int i = 0; i < SEP_NZ; i++) {
        const int o = 2 * (i / 2);
        const double pyi = fma(Pr[i * SEP_NZ + o + 1], y[o + 1], fma(Pr[i * SEP_NZ + o], y[o], 0.0));
        v = fma(y[i], 0.5 * pyi + q[i], v);
    }
    return v;
}

// The box rows' constants of one agent, the same for both IMPC iterations (the rows' bounds are
// shifted by the state, their coefficients and P^-1 fixed): per side the violation scale
// 1 / (1 + |bound|) (bsc[s * 16 + lane], s = 2 (d SB + kk) + upper) and per row the candidate weight
// 1 / sqrt(g P^-1 g) (bw[r * 16 + lane], r = d SB + kk) — sep_dual_as's own arithmetic, formed once
// per agent into the group's LDS instead of at the start of every solve.
template <int SB, int CB>
__device__ __forceinline__ void sep_box_consts(const SepRows<SB, CB>& rw, const double* __restrict__ Pinv,
                                               double* __restrict__ bsc, float* __restrict__ bw) {
    const int gl = lane_bits_opaque<15>();
    double pi[SEP_D][3];
    sep_pinv(Pinv, pi);
    int s = 0, r = 0;
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int kk = 0; kk < SB; kk++, r++) {
            bsc[s * 16 + gl] = rcp(1.0 + fabs(rw.blo[d][kk]));
            bsc[(s + 1) * 16 + gl] = rcp(1.0 + fabs(rw.bhi[d][kk]));
            s += 2;
            const double g0 = rw.bg[d][kk][0], g1 = rw.bg[d][kk][1];
            const double n2 = fma(fma(pi[d][0], g0, 2.0 * pi[d][1] * g1), g0, pi[d][2] * g1 * g1);
            bw[r * 16 + gl] = rsqrtf((float)fmax(n2, 1e-30));
        }
}

// K = G_A P^-1 G_A^T of the k staged rows of pol (packed upper, identity beyond k)
template <int NR>
__device__ __forceinline__ void sep_gram(const double* __restrict__ pol, int k, double (&K)[Sym<NR>::P]) {
#pragma unroll
    for (int i = 0; i < NR; i++) {
        const double* ri = pol + (i < k ? i : 0) * 16;
#pragma unroll
        for (int j = i; j < NR; j++) {
            const double* wj = pol + (j < k ? j : 0) * 16 + POL_W;
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < SEP_NZ; m++) v = fma(ri[m], wj[m], v);
            K[Sym<NR>::idx(i, j)] = (i < k && j < k) ? v : (i == j ? 1.0 : 0.0);
        }
    }
}

// Dual active-set solve (Goldfarb & Idnani's method, range-space form) from the unconstrained
// minimiser yu: the most violated side (scaled as the primal residual) is the candidate; the
// direction z that keeps the active sides exact moves y onto it unless an active multiplier
// reaches zero first, in which case that side leaves and the step is retried. Every step keeps
// the iterate dual feasible and raises the objective. The Cholesky factor L of
// K = G_A P^-1 G_A^T (k <= 6 active rows staged in pol, the candidate in row POL_K) stays in
// registers: a step costs one forward and one backward substitution with the candidate's column
// c = G_A P^-1 g_p, and when the candidate joins, L^-1 c is L's new row and the Schur complement
// g_p P^-1 g_p - |L^-1 c|^2 its squared diagonal; a leaving side refactors K. Converged (no side
// violated beyond tol / 10), the iterate is returned when its dual residual meets tol (the
// updates hold stationarity up to rounding), else the active set's EQP (sep_eqp_finish) re-solves
// it. Returns 1: optimal (yo, residuals, warm duals set); -1: no step reaches the candidate (its
// side is a combination of the active ones and no multiplier can leave: no feasible point, phase
// 1 decides; yo = last iterate); 0: gave up (step limit, breakdown, failed verification) — the
// PDIP solves the QP.
#ifdef MPCCBF_PDIP_STAMPS  // profiling build: shader-clock stamps of the first solve's first steps
#define GSTAMP(k, cond)                                                              \
    do {                                                                             \
        if (dbg && (cond)) dbg[k] = (long long)__builtin_amdgcn_s_memtime();         \
    } while (0)
#else
#define GSTAMP(k, cond) \
    do {                \
    } while (0)
#endif
// Warm start (k0 > 0): warm_ids[0 .. k0-1] name sides (POL_ID values) of an earlier solve with
// the same box rows and cost — IMPC iteration 0's final active set for iteration 1, whose CBF rows
// of sample 0 are iteration 0's rows (the curve at h_samples(0) = 0 is the state) in the same
// slots. Each side is staged from this QP's own rows by the lane that owns it; when the equality QP
// on them has multipliers of the right signs, that point (dual feasible, the sides exact) is the
// start instead of the unconstrained minimiser; else the solve starts cold. Any set of this QP's
// sides is a valid start, so a side whose slot now holds another row only costs steps.
// save: at convergence the final active set's side ids are written there (lane 0; their count
// at save[POL_K]).
// Active sides the dual active set's factor holds (L, multipliers, substitutions): DAS_K <= POL_K
// (the staged-row layout); a QP that needs more gives up to the PDIP. (MPCCBF_DAS_K: A/B builds)
#ifndef MPCCBF_DAS_K
#define MPCCBF_DAS_K 5
#endif
constexpr int DK = MPCCBF_DAS_K;
static_assert(DK >= 1 && DK <= POL_K, "the factor holds at most POL_K staged rows");
template <int G, int SB, int CB>
__device__ int sep_dual_as(const SepRows<SB, CB>& rw, bool has_cbf, const double* __restrict__ P,
                           const double* __restrict__ Pinv, const double (&q)[SEP_NZ], const double (&yu)[SEP_NZ], double tol, int maxstep,
                           double* __restrict__ pol, double (&yo)[SEP_NZ], double& rp_out, double& rd_out,
                           int& steps, SepWarm<SB>* warm, bool want_rd, double& tlow,
                           long long* dbg = nullptr, int k0 = 0, const double* __restrict__ warm_ids = nullptr,
                           double* __restrict__ save = nullptr, double* __restrict__ mult = nullptr,
                           const double* __restrict__ box_sc = nullptr, const float* __restrict__ box_w = nullptr,
                           bool want_rp = true) {
    static_assert(G == 16, "rows of pol are copied one column per lane");
    (void)dbg;
    GSTAMP(0, true);
#ifdef MPCCBF_PDIP_STAMPS
    if (dbg) dbg[15] = 1;
#endif
    const int gl = lane_bits_opaque<G - 1>();
    double pi[SEP_D][3];
    sep_pinv(Pinv, pi);
    constexpr int NS = 2 * SEP_D * SB + CB;
    double sc[NS];  // violation scale 1 / (1 + |bound|) per side
    {
        // the box sides' from the agent's constants (sep_box_consts: the same values, formed once
        // for both IMPC iterations) when given
        int s = 0;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int kk = 0; kk < SB; kk++) {
                if (box_sc != nullptr) {
                    sc[s] = box_sc[s * 16 + gl];
                    sc[s + 1] = box_sc[(s + 1) * 16 + gl];
                } else {
                    sc[s] = rcp(1.0 + fabs(rw.blo[d][kk]));
                    sc[s + 1] = rcp(1.0 + fabs(rw.bhi[d][kk]));
                }
                s += 2;
            }
#pragma unroll
        for (int c = 0; c < CB; c++) sc[s++] = rcp(1.0 + fabs(rw.chi[c]));
    }
    // candidate rule: among the sides violated beyond the tolerance (scaled as above), the one
    // with the largest violation per unit norm in the P^-1 metric, v / sqrt(g P^-1 g) — the side
    // whose addition alone raises the dual objective most (v^2 / 2 g P^-1 g). The plain scaled
    // rule picked sides that later left again: on the driver bench's slowest QPs 10-12 steps
    // where this rule needs 4-8 (tools/das_sim.py, the same QPs in numpy). One weight per row
    // (both sides of a box row share it), formed once per solve into the scratch after the
    // staged rows (wrow[r * 16 + lane]); inert rows (g = 0) are never violated.
    // (the box rows' weights from the agent's constants, box_w, when given)
    float* wrow = (float*)(pol + (POL_K + 1) * 16);
    const float* __restrict__ wbox = box_w != nullptr ? box_w : wrow;
    {
        int r = 0;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int kk = 0; kk < SB; kk++, r++) {
                if (box_w != nullptr) continue;
                const double g0 = rw.bg[d][kk][0], g1 = rw.bg[d][kk][1];
                const double n2 = fma(fma(pi[d][0], g0, 2.0 * pi[d][1] * g1), g0, pi[d][2] * g1 * g1);
                wrow[r * 16 + gl] = rsqrtf((float)fmax(n2, 1e-30));
            }
#pragma unroll
        for (int c = 0; c < CB; c++, r++) {
            const double* g = rw.cg[c];
            const double n2 = fma(fma(pi[0][0], g[0], 2.0 * pi[0][1] * g[1]), g[0], pi[0][2] * g[1] * g[1]) +
                              fma(fma(pi[1][0], g[2], 2.0 * pi[1][1] * g[3]), g[2], pi[1][2] * g[3] * g[3]);
            wrow[r * 16 + gl] = rsqrtf((float)fmax(n2, 1e-30));
        }
    }
    double y[SEP_NZ], u[DK];
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) y[j] = yu[j];
#pragma unroll
    for (int i = 0; i < DK; i++) u[i] = 0.0;
    int k = 0;
    steps = 0;
    const double add_tol = 0.1 * tol;
    double* cand = pol + POL_K * 16;
    using S6 = Sym<DK>;
    double L[S6::P], dl[DK];  // chol_packed layout of K's factor (identity beyond k), 1 / diagonal
#pragma unroll
    for (int i = 0; i < DK; i++) {
        dl[i] = 1.0;
#pragma unroll
        for (int j = i; j < DK; j++) L[S6::idx(i, j)] = i == j ? 1.0 : 0.0;
    }
    if (k0 > 0) {
        // the EQP on the given sides: lam = K^-1 (G_A yu - b_A), y = yu - P^-1 G_A^T lam; start
        // there when every multiplier u_i = sign_i lam_i >= 0 (group-uniform: LDS rows)
        double rhs[DK], lam[DK];
        for (int i = 0; i < k0; i++) {
            const int id = (int)warm_ids[i];
            if ((id & 15) == gl) sep_stage_side<SB, CB>(rw, pi, id >> 4, gl, pol + i * 16);
        }
        wave_lds_sync();
        sep_gram<DK>(pol, k0, L);
#pragma unroll
        for (int i = 0; i < DK; i++) {
            const double* ri = pol + (i < k0 ? i : 0) * 16;
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) t = fma(ri[j], yu[j], t);
            rhs[i] = i < k0 ? t - ri[POL_B] : 0.0;
        }
        bool ok = chol_packed<DK>(L, dl);
        chol_solve<DK>(L, dl, rhs, lam);
#pragma unroll
        for (int i = 0; i < DK; i++) {
            const double* ri = pol + (i < k0 ? i : 0) * 16;
            u[i] = i < k0 ? ri[POL_SGN] * lam[i] : 0.0;
            ok = ok && (i >= k0 || (u[i] >= 0.0 && isfinite(u[i])));
        }
        if (ok) {
#pragma unroll
            for (int i = 0; i < DK; i++) {
                const double* wi = pol + (i < k0 ? i : 0) * 16 + POL_W;
#pragma unroll
                for (int j = 0; j < SEP_NZ; j++) y[j] = fma(i < k0 ? -lam[i] : 0.0, wi[j], y[j]);
            }
            k = k0;
        } else {  // cold: empty active set, identity factor
#pragma unroll
            for (int i = 0; i < DK; i++) {
                u[i] = 0.0;
                dl[i] = 1.0;
#pragma unroll
                for (int j = i; j < DK; j++) L[S6::idx(i, j)] = i == j ? 1.0 : 0.0;
            }
        }
    }
    double m = 0.0;
    GSTAMP(1, true);
    for (int outer = 0;; outer++) {
        (void)outer;
        // the group's largest scaled violation (convergence) and the candidate (lowest lane on
        // ties): the side violated beyond the tolerance with the largest normalised violation. A
        // NaN row or iterate (a NaN state, target or neighbour state) shows as a NaN violation on
        // the first scan: give up, the caller's finiteness checks decide.
#ifndef MPCCBF_SCAN_F64
        // keys: a violated side's normalised violation as a float bit pattern (at least 1: a score
        // that rounds to 0 in float still counts as violated), 0 for the others — the wide
        // kernel's rule (impc_wide.hpp): the group max is one u32 DPP reduction, the lane's best
        // side the first of its largest key; the scaled violation vb is reduced only when the
        // caller stores the primal residual
        unsigned kb = 0u;
        double vb = -1.0;
        int sb = 0;
        bool nanv = false;
        {
            int s = 0, r = 0;
#pragma unroll
            for (int d = 0; d < SEP_D; d++)
#pragma unroll
                for (int kk = 0; kk < SB; kk++, r++) {
                    const double t = rw.bg[d][kk][0] * y[2 * d] + rw.bg[d][kk][1] * y[2 * d + 1];
                    const double w = (double)wbox[r * 16 + gl];
                    const double al = rw.blo[d][kk] - t, vl = al * sc[s];
                    const unsigned kl = vl > add_tol ? max(__float_as_uint((float)(al * w)), 1u) : 0u;
                    if (kl > kb) kb = kl, sb = s;
                    s++;
                    const double au = t - rw.bhi[d][kk], vu = au * sc[s];
                    const unsigned ku = vu > add_tol ? max(__float_as_uint((float)(au * w)), 1u) : 0u;
                    if (ku > kb) kb = ku, sb = s;
                    s++;
                    nanv = nanv || vl != vl || vu != vu;
                    vb = fmax(vb, fmax(vl, vu));
                }
            if (has_cbf) {
#pragma unroll
                for (int c = 0; c < CB; c++, s++, r++) {
                    double t = 0.0;
#pragma unroll
                    for (int j = 0; j < 4; j++) t = fma(rw.cg[c][j], y[j], t);
                    const double ac = t - rw.chi[c], vc = ac * sc[s];
                    const unsigned kc =
                        vc > add_tol ? max(__float_as_uint((float)(ac * (double)wrow[r * 16 + gl])), 1u) : 0u;
                    if (kc > kb) kb = kc, sb = s;
                    nanv = nanv || vc != vc;
                    vb = fmax(vb, vc);
                }
            }
        }
        if (outer == 0 && grp_ballot<G>(nanv) != 0ull) return 0;
        const unsigned kmax = row_max_u32(kb);
        GSTAMP(2 + 6 * outer, outer < 2);
        if (kmax == 0u) {
            m = want_rp ? grp_max<G>(vb) : 0.0;
            break;
        }
        if (steps >= maxstep) return 0;
        if (kmax == 1u) return 0;  // the best score is 0 or denormal in float: no usable rule (PDIP)
        const int owner = __ffsll((long long)grp_ballot<G>(kb == kmax)) - 1;
#else  // (A/B build: double scores, two interleaved max reductions)
        double vb = -1.0, eb = -1.0;
        int sb = 0;
        bool nanv = false;
        {
            int s = 0, r = 0;
#pragma unroll
            for (int d = 0; d < SEP_D; d++)
#pragma unroll
                for (int kk = 0; kk < SB; kk++, r++) {
                    const double t = rw.bg[d][kk][0] * y[2 * d] + rw.bg[d][kk][1] * y[2 * d + 1];
                    const double w = (double)wbox[r * 16 + gl];
                    const double al = rw.blo[d][kk] - t, vl = al * sc[s];
                    const double el = vl > add_tol ? al * w : -1.0;
                    if (el > eb) eb = el, sb = s;
                    s++;
                    const double au = t - rw.bhi[d][kk], vu = au * sc[s];
                    const double eu = vu > add_tol ? au * w : -1.0;
                    if (eu > eb) eb = eu, sb = s;
                    s++;
                    nanv = nanv || vl != vl || vu != vu;
                    vb = fmax(vb, fmax(vl, vu));
                }
            if (has_cbf) {
#pragma unroll
                for (int c = 0; c < CB; c++, s++, r++) {
                    double t = 0.0;
#pragma unroll
                    for (int j = 0; j < 4; j++) t = fma(rw.cg[c][j], y[j], t);
                    const double ac = t - rw.chi[c], vc = ac * sc[s];
                    const double ec = vc > add_tol ? ac * (double)wrow[r * 16 + gl] : -1.0;
                    if (ec > eb) eb = ec, sb = s;
                    nanv = nanv || vc != vc;
                    vb = fmax(vb, vc);
                }
            }
        }
        if (outer == 0 && grp_ballot<G>(nanv) != 0ull) return 0;
        m = vb;
        double em = eb;
        grp_max2<G>(m, em);
        GSTAMP(2 + 6 * outer, outer < 2);
        if (!(m > add_tol)) break;
        if (steps >= maxstep) return 0;
        const int owner = __ffsll((long long)grp_ballot<G>(eb == em)) - 1;
#endif
        if (gl == owner) sep_stage_side<SB, CB>(rw, pi, sb, gl, cand);
        wave_lds_sync();
        GSTAMP(3, outer == 0);
        GSTAMP(7, outer == 1);  // (the second step's: stamps 7, 4, 11, 5, 14)
        if (k == 0) {
            // first side of an empty active set: z = P^-1 n_p, the step reaches it (no factor yet),
            // and L = (sqrt(g_p P^-1 g_p))
            ++steps;
            const double sp = cand[POL_SGN];
            double nw = 0.0, gy = 0.0;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) {
                nw = fma(cand[j], cand[POL_W + j], nw);
                gy = fma(cand[j], y[j], gy);
            }
            if (!(nw > 0.0)) return 0;
            const double t = sp * (gy - cand[POL_B]) * rcp(nw);
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) y[j] = fma(-t * sp, cand[POL_W + j], y[j]);
            wave_lds_sync();
            pol[gl] = cand[gl];
            const double rz = rsqrt(nw);
            L[S6::idx(0, 0)] = nw * rz;
            dl[0] = rz;
            u[0] = t;
            k = 1;
            wave_lds_sync();
            GSTAMP(6, outer == 0);
            continue;
        }
        double up = 0.0;  // the candidate's multiplier
        for (;;) {
            if (++steps > maxstep) return 0;
            double gp[SEP_NZ];
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) gp[j] = cand[j];
            const double sp = cand[POL_SGN];
            // rows at or beyond the wave's largest active count kw are identity rows of L with zero
            // right-hand side (v = rho = 0 there): skipped by scalar branches (kw is wave-uniform)
#ifndef MPCCBF_NO_KW
            int kw = 0;
#pragma unroll
            for (int i = 1; i <= DK; i++) kw += __ballot(k >= i) != 0ull ? 1 : 0;
#else  // comparison build: every row
            constexpr int kw = DK;
#endif
            // v = L^-1 (sp c), c_i = g_i P^-1 g_p: the forward substitution fused with the dots
            double v[DK], sgn[DK];
#pragma unroll
            for (int i = 0; i < DK; i++) {
                v[i] = 0.0;
                sgn[i] = 0.0;
                if (i < kw) {
                    const double* ri = pol + (i < k ? i : 0) * 16;
                    double t = 0.0;
#pragma unroll
                    for (int j = 0; j < SEP_NZ; j++) t = fma(ri[POL_W + j], gp[j], t);
                    sgn[i] = ri[POL_SGN];
                    double s = i < k ? sp * t : 0.0;
#pragma unroll
                    for (int mm = 0; mm < i; mm++) s = fma(-L[S6::idx(mm, i)], v[mm], s);
                    v[i] = s * dl[i];
                }
            }
            // rho = L^-T v = K^-1 G_A P^-1 n_p: the active multipliers' change per unit step
            double rho[DK];
#pragma unroll
            for (int i = DK - 1; i >= 0; i--) {
                rho[i] = 0.0;
                if (i < kw) {
                    double s = v[i];
#pragma unroll
                    for (int mm = i + 1; mm < DK; mm++) s = fma(-L[S6::idx(i, mm)], rho[mm], s);
                    rho[i] = s * dl[i];
                }
            }
            GSTAMP(4, steps == 2);
            double nw = 0.0, vv = 0.0, vp = 0.0;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) {
                nw = fma(gp[j], cand[POL_W + j], nw);
                vp = fma(gp[j], y[j], vp);
            }
#pragma unroll
            for (int i = 0; i < DK; i++) vv = fma(v[i], v[i], vv);
            const double zn = nw - vv;  // n_p z: the Schur complement of K in [K c; c^T nw]
            vp = sp * (vp - cand[POL_B]);
            // dual step: the first active multiplier to reach zero (smallest u_i / r_i, compared
            // by cross products: one reciprocal)
            double un = 1.0, rn = 0.0;  // (un / rn = +inf until a blocking multiplier is found)
            int l = -1;
#pragma unroll
            for (int i = 0; i < DK; i++) {
                const double r = sgn[i] * rho[i];
                const bool better = i < k && r > 0.0 && u[i] * rn < un * r;
                un = better ? u[i] : un;
                rn = better ? r : rn;
                l = better ? i : l;
            }
            const double t1 = l >= 0 ? un * rcp(rn) : 1e300;
            const bool full = zn > 1e-10 * nw;  // else n_p lies in the span of the active sides
            const double t2 = full ? vp * rcp(zn) : 1e300;
            if (l < 0 && !full) {
                // n_p = N_A r with every r <= 0: lam = (1, -r) >= 0 combines the sides to zero, and
                // t* >= -sum lam b / sum lam = (n_p y - b_p) / (1 - sum r) (active sides exact at y)
                double lsum = 1.0;
#pragma unroll
                for (int i = 0; i < DK; i++) {
                    const double r = sgn[i] * rho[i];
                    lsum += (i < k && r < 0.0) ? -r : 0.0;
                }
                tlow = vp * rcp(lsum);
#pragma unroll
                for (int j = 0; j < SEP_NZ; j++) yo[j] = y[j];
                wave_lds_sync();
                return -1;
            }
            const double t = fmin(t1, t2);
            GSTAMP(11, steps == 2);
            if (full) {
                // primal direction z = P^-1 (n_p - N_A r), n = sign * g (rows re-read: the
                // compiler barrier keeps them from staying live across the substitutions)
                // (loads never under a condition: inactive rows read row 0 and weigh 0)
                asm volatile("" ::: "memory");
                double z[SEP_NZ];
#pragma unroll
                for (int j = 0; j < SEP_NZ; j++) z[j] = sp * cand[POL_W + j];
#pragma unroll
                for (int i = 0; i < DK; i++) {
                    if (i < kw) {
                        const double* wi = pol + (i < k ? i : 0) * 16 + POL_W;
                        const double ri = i < k ? rho[i] : 0.0;
#pragma unroll
                        for (int j = 0; j < SEP_NZ; j++) z[j] = fma(-ri, wi[j], z[j]);
                    }
                }
#pragma unroll
                for (int j = 0; j < SEP_NZ; j++) y[j] = fma(-t, z[j], y[j]);
            }
#pragma unroll
            for (int i = 0; i < DK; i++)
                u[i] = i < k ? fma(-t, sgn[i] * rho[i], u[i]) : u[i];
            up += t;
            wave_lds_sync();  // every lane has read the rows it is about to move
            GSTAMP(5, steps == 2);
            if (t2 <= t1) {  // the candidate joins: L gains the row L^-1 c, diagonal sqrt(zn)
                if (k == DK) return 0;
                pol[k * 16 + gl] = cand[gl];
                const double rz = rsqrt(zn);
#pragma unroll
                for (int i = 0; i < DK; i++) {
                    u[i] = i == k ? up : u[i];
                    dl[i] = i == k ? rz : dl[i];
#pragma unroll
                    for (int j = i; j < DK; j++)
                        if (j == k) L[S6::idx(i, j)] = i < k ? sp * v[i] : (i == k ? zn * rz : L[S6::idx(i, j)]);
                }
                k++;
                wave_lds_sync();
                GSTAMP(14, steps == 2);
                break;
            }
            // side l leaves: the rows above it move down (one column per lane); K refactored
#pragma unroll
            for (int i = 0; i < DK - 1; i++)
                if (i >= l && i < k - 1) pol[i * 16 + gl] = pol[(i + 1) * 16 + gl];
#pragma unroll
            for (int i = 0; i < DK; i++) u[i] = i >= l ? (i + 1 < DK ? u[i + 1] : 0.0) : u[i];
            k--;
            wave_lds_sync();
            sep_gram<DK>(pol, k, L);
            if (!chol_packed<DK>(L, dl)) return 0;
        }
    }
    // converged: primal residual = the last scan's worst violation; the iterate's dual residual
    // P y + q + G_A^T lam (lam = sign * u), checked whether or not the caller stores it (the
    // updates hold stationarity by construction, so the check only guards against rounding); a
    // non-finite iterate gives up
    // An empty active set returns the unconstrained minimiser -P^-1 q itself (finite: q and the
    // rows were checked finite; P^-1 from the host), whose residual is that 2 x 2 solve's
    // rounding: evaluated only when the caller stores it
    if (k > 0) {
        bool nf = false;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) nf = nf || !isfinite(y[j]);
        if (grp_ballot<G>(nf) != 0ull) return 0;
    }
    // P's 2x2 channel blocks (uniform), loaded here where the dual residual uses them: loaded at
    // the solve's start, their 24 scalar registers stayed live across every step (round 6: with
    // the branch-free row reads below, 29.3 -> 28.7 us per config-3 launch)
    double pb[SEP_NZ][2];
#pragma unroll
    for (int o = 0; o < SEP_NZ; o++) {
        pb[o][0] = P[o * 6 + 2 * (o / 2)];
        pb[o][1] = P[o * 6 + 2 * (o / 2) + 1];
    }
    double rd = 0.0, qn = 0.0;
    if (k == 0 && !want_rd) {
        // (rd = 0: not stored, and below the tolerance by construction)
    } else if (k == 0) {  // (group-uniform) the unconstrained minimiser, most QPs: P y + q alone
#pragma unroll
        for (int o = 0; o < SEP_NZ; o++) {
            const int d = o / 2;
            rd = fmax(rd, fabs(fma(pb[o][0], y[2 * d], fma(pb[o][1], y[2 * d + 1], q[o]))));
            qn = fmax(qn, fabs(q[o]));
        }
    } else {
        double r[SEP_NZ];
#pragma unroll
        for (int o = 0; o < SEP_NZ; o++) {
            const int d = o / 2;
            r[o] = fma(pb[o][0], y[2 * d], fma(pb[o][1], y[2 * d + 1], q[o]));
        }
        // G_A^T lam: every staged row's entries loaded first, no per-row branch (rows past k read
        // row 0 and weigh 0: the same sums as over the active rows alone)
        {
            double g[DK][SEP_NZ + 1];
#pragma unroll
            for (int i = 0; i < DK; i++) {
                const double* ri = pol + (i < k ? i : 0) * 16;  // (rows past k: row 0, weight 0)
#pragma unroll
                for (int o = 0; o < SEP_NZ; o++) g[i][o] = ri[o];
                g[i][SEP_NZ] = ri[POL_SGN];
            }
#pragma unroll
            for (int i = 0; i < DK; i++) {
                const double li = i < k ? g[i][SEP_NZ] * u[i] : 0.0;
#pragma unroll
                for (int o = 0; o < SEP_NZ; o++) r[o] = fma(li, g[i][o], r[o]);
            }
        }
#pragma unroll
        for (int o = 0; o < SEP_NZ; o++) {
            rd = fmax(rd, fabs(r[o]));
            qn = fmax(qn, fabs(q[o]));
        }
    }
    rd *= rcp(1.0 + qn);
    GSTAMP(9, true);
    auto save_sides = [&]() {  // the final active set's side ids, for a later warm start
        if (save == nullptr) return;
        if (gl < k) save[gl] = pol[gl * 16 + POL_ID];
        if (gl == 0) save[POL_K] = (double)k;
    };
    if (!(rd <= tol)) {
        // rounding accumulated over the steps: the active set's equality QP, re-solved exactly
        const bool ok = sep_eqp_finish<G, SB, CB, true, DK>(rw, has_cbf, P, q, yu, k, pol, sc, tol, yo, rp_out, rd_out, warm,
                                                        mult);
        if (ok) save_sides();
        wave_lds_sync();
        return ok ? 1 : 0;
    }
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) yo[j] = y[j];
    rp_out = fmax(m, 0.0);
    rd_out = rd;
    if (warm != nullptr) {  // the multipliers as the next warm start's box duals
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int kk = 0; kk < SB; kk++) {
                const double il = (double)((2 * (d * SB + kk)) * 16 + gl), iu = il + 16.0;
                double ml = 0.0, mu = 0.0;
#pragma unroll
                for (int i = 0; i < DK; i++) {
                    const double id = i < k ? pol[(i < k ? i : 0) * 16 + POL_ID] : -1.0;
                    ml = id == il ? u[i] : ml;
                    mu = id == iu ? u[i] : mu;
                }
                warm->zl(d, kk) = ml;
                warm->zu(d, kk) = mu;
            }
    }
    save_sides();
    if (mult != nullptr) {  // mult[0 .. k): the active sides' multipliers (>= 0), mult[7] = k,
                            // mult[8 .. 8 + k): their side ids (POL_ID)
        double ui = 0.0;
#pragma unroll
        for (int i = 0; i < DK; i++) ui = gl == i ? u[i] : ui;
        if (gl < k) {
            mult[gl] = ui;
            mult[8 + gl] = pol[gl * 16 + POL_ID];
        }
        if (gl == 0) mult[7] = (double)k;
    }
    wave_lds_sync();  // the scratch is reused
    GSTAMP(10, true);
    return 1;
}

// P: 6x6 row-major block-diagonal reduced Hessian, Pinv its per-channel inverse blocks (uniform).
// has_cbf: group-uniform flag (some CBF slot of the group is live); when false the CBF slots
// are skipped entirely (and do not count as sides).
//
// SLACK (slack_mode, MPCCBFQPGeneratorBase.cpp:28-130): lane l owns the slack variable v >= 0 of
// neighbour l, with linear cost wv; its CBF rows read g^T y - v <= chi (ccv = 1). v couples
// only to the (x, y) block and to its own rows, so it is eliminated per lane (Schur complement
// of the scalar v-block d): the group still reduces the same 20 values, with
//   M_xy -= u u^T / d,  rhs_xy -= u rhs_v / d,   u = -sum_rows D g,  d = sum_rows D + D_bound,
// and dv = (rhs_v - u^T dy) / d is recovered lane-locally after each solve.
template <int G, int SB, int CB, bool SLACK>
__device__ PdipOut pdip_solve_sep_ip(const SepRows<SB, CB>& rw, bool has_cbf, const double* __restrict__ P,
                                     const double* __restrict__ Pinv, const double (&q)[SEP_NZ],
                                     double (&y)[SEP_NZ], const PdipCfg cfg, long long* dbg, double wv_cost,
                                     double* v_out, double* red, SepWarm<SB>* warm, double warm_delta, double* pol,
                                     int as_steps);
// (pdip_solve_sep_ip stays inline: as an out-of-line call — operands by reference or by value —
// the caller kept its rows and loop state in scratch around it, 392-784 B/lane across the hot path)
template <int G, int SB, int CB, bool SLACK = false>
__device__ PdipOut pdip_solve_sep(const SepRows<SB, CB>& rw, bool has_cbf, const double* __restrict__ P,
                                  const double* __restrict__ Pinv, const double (&q)[SEP_NZ],
                                  double (&y)[SEP_NZ], const PdipCfg cfg, long long* dbg = nullptr,
                                  double wv_cost = 0.0, double* v_out = nullptr, double* red = nullptr,
                                  SepWarm<SB>* warm = nullptr, double warm_delta = 0.0,
                                  double* pol = nullptr, int das_k0 = 0, const double* das_ids = nullptr,
                                  double* das_save = nullptr, const double* box_sc = nullptr,
                                  const float* box_w = nullptr) {
    (void)dbg;
    GSTAMP(12, true);
    // warm start (group-uniform): y holds the previous solution (pdip_solve_sep_ip)
    const bool use_warm = warm != nullptr && warm_delta > 0.0;
    int as_steps = 0;  // dual active-set steps before the PDIP (counted in iters)
    // ---- start: unconstrained minimiser (block-diagonal P: per-channel 2x2 solves). When it
    // satisfies every row it is the optimum (convex QP, all multipliers zero; slack mode: v = 0
    // since its cost is positive): no Newton step needed.
    {
        double yu[SEP_NZ];
#pragma unroll
        for (int d = 0; d < SEP_D; d++) {
            const int o = 2 * d;
            const double a = Pinv[3 * d], b = Pinv[3 * d + 1], c = Pinv[3 * d + 2];
            yu[o] = -fma(a, q[o], b * q[o + 1]);
            yu[o + 1] = -fma(b, q[o], c * q[o + 1]);
        }
        // with the dual active-set solve on, its first scan is the fast-start test (an empty
        // active set it returns unchanged): no separate row check
        const bool das = !SLACK && cfg.dual_as > 0 && pol != nullptr;
        bool bad = das;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const double t = rw.bg[d][k][0] * yu[2 * d] + rw.bg[d][k][1] * yu[2 * d + 1];
                bad = bad || !(t >= rw.blo[d][k] && t <= rw.bhi[d][k]);  // NaN-safe
            }
        if (has_cbf && !das) {
#pragma unroll
            for (int c = 0; c < CB; c++) {
                double t = 0.0;
#pragma unroll
                for (int j = 0; j < 4; j++) t = fma(rw.cg[c][j], yu[j], t);
                bad = bad || !(t <= rw.chi[c]);
            }
        }
        if (cfg.fast_start && !das && grp_ballot<G>(bad) == 0ull) {
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) y[j] = yu[j];
            if (v_out) *v_out = 0.0;
            if (warm != nullptr) {
#pragma unroll
                for (int d = 0; d < SEP_D; d++)
#pragma unroll
                    for (int k = 0; k < SB; k++) warm->zl(d, k) = warm->zu(d, k) = 0.0;
            }
            // residuals of the returned point: rows satisfied exactly, multipliers zero
            double rdn = 0.0, qn0 = 0.0;
#pragma unroll
            for (int d = 0; d < SEP_D; d++) {
                const int o = 2 * d;
                rdn = fmax(rdn, fabs(fma(P[o * 6 + o], yu[o], fma(P[o * 6 + o + 1], yu[o + 1], q[o]))));
                rdn = fmax(rdn, fabs(fma(P[(o + 1) * 6 + o], yu[o], fma(P[(o + 1) * 6 + o + 1], yu[o + 1], q[o + 1]))));
                qn0 = fmax(qn0, fmax(fabs(q[o]), fabs(q[o + 1])));
            }
            PdipOut fo{ST_OPTIMAL, 0};
            fo.rp = 0.0;
            fo.rd = rdn / (1.0 + qn0);
            return fo;
        }
        // dual active-set solve (PdipCfg::dual_as): the PDIP below runs only when it gives up
        // (no warm-start duals: the caller's PDIP attempts run cold when it is on)
        GSTAMP(13, true);
        if constexpr (!SLACK) {
            if (das) {
                double yg[SEP_NZ], rpg = 0.0, rdg = 0.0, tlg = 0.0;
                const int r = sep_dual_as<G, SB, CB>(rw, has_cbf, P, Pinv, q, yu, cfg.tol, cfg.dual_as, pol, yg, rpg,
                                                     rdg, as_steps, nullptr, cfg.want_rd, tlg, dbg, das_k0, das_ids,
                                                     das_save, nullptr, box_sc, box_w, cfg.want_rp);
                if (r != 0) {
                    PdipOut fo{r > 0 ? ST_OPTIMAL : ST_UNKNOWN, as_steps};
#pragma unroll
                    for (int j = 0; j < SEP_NZ; j++) y[j] = yg[j];
                    if (r > 0) {
                        fo.rp = rpg;
                        fo.rd = rdg;
                        fo.polished = true;
                    } else {
                        fo.early = true;  // no feasible point in sight: phase 1 decides
                        fo.tlow = tlg;
                    }
                    return fo;
                }
                wave_lds_sync();  // the scratch is reused by the polish
            }
        }
        if (!use_warm) {
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) y[j] = yu[j];
        }
    }
    return pdip_solve_sep_ip<G, SB, CB, SLACK>(rw, has_cbf, P, Pinv, q, y, cfg, dbg, wv_cost, v_out, red, warm,
                                               warm_delta, pol, as_steps);
}

// The Mehrotra PDIP of pdip_solve_sep from its start point (y: the unconstrained minimiser or the
// warm start); as_steps: the dual active set's steps before it (counted in the iterations).
template <int G, int SB, int CB, bool SLACK>
__device__ __forceinline__ PdipOut pdip_solve_sep_ip(const SepRows<SB, CB>& rw, bool has_cbf,
                                                     const double* __restrict__ P, const double* __restrict__ Pinv,
                                                     const double (&q)[SEP_NZ], double (&y)[SEP_NZ],
                                                     const PdipCfg cfg, long long* dbg, double wv_cost, double* v_out,
                                                     double* red, SepWarm<SB>* warm, double warm_delta, double* pol,
                                                     int as_steps) {
    (void)dbg;
    const bool slk = SLACK && has_cbf;  // group-uniform
    // slack variable, its bound's slack and dual; the dual starts at the linear cost it carries at
    // the optimum (w = sum_rows z + z_bound with inactive rows)
    double v = 1.0, sb = 1.0, zb = SLACK ? fmax(wv_cost, 1.0) : 1.0;
    // warm start (group-uniform): y holds the previous solution; slacks from it and the stored
    // duals, both floored at delta (complementarity >= delta^2), CBF rows centred at delta^2
    const bool use_warm = warm != nullptr && warm_delta > 0.0;
    const double wd = warm_delta, wd2 = warm_delta * warm_delta;
    // slacks (s) and duals (z): box lower / upper sides, CBF upper side
    double sl[SEP_D][SB], su[SEP_D][SB], zl[SEP_D][SB], zu[SEP_D][SB], cs[CB], cz[CB];
    double pl[SEP_D][SB], pu[SEP_D][SB], pc[CB];  // relative primal-residual scales
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const double t = rw.bg[d][k][0] * y[2 * d] + rw.bg[d][k][1] * y[2 * d + 1];
            if (use_warm) {
                sl[d][k] = fmax(t - rw.blo[d][k], wd);
                su[d][k] = fmax(rw.bhi[d][k] - t, wd);
                zl[d][k] = fmax(warm->zl(d, k), wd);
                zu[d][k] = fmax(warm->zu(d, k), wd);
            } else {
                sl[d][k] = fmax(t - rw.blo[d][k], 1.0);
                su[d][k] = fmax(rw.bhi[d][k] - t, 1.0);
                zl[d][k] = rcp(sl[d][k]);
                zu[d][k] = rcp(su[d][k]);
            }
            pl[d][k] = rcp(1.0 + fabs(rw.blo[d][k]));
            pu[d][k] = rcp(1.0 + fabs(rw.bhi[d][k]));
        }
#pragma unroll
    for (int c = 0; c < CB; c++) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++) t = fma(rw.cg[c][j], y[j], t);
        if (slk) t -= rw.ccv[c] * v;
        cs[c] = fmax(rw.chi[c] - t, use_warm ? wd : 1.0);
        cz[c] = use_warm ? wd2 * rcp(cs[c]) : rcp(cs[c]);
        pc[c] = rcp(1.0 + fabs(rw.chi[c]));
    }
    const double nsides = (double)(G * (2 * SEP_D * SB + (has_cbf ? CB : 0) + (slk ? 1 : 0)));
    double qn = 0.0;
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) qn = fmax(qn, fabs(q[j]));
    const double inv_ns = 1.0 / nsides;
    const double inv_qn = rcp(1.0 + qn);

    PdipOut out{ST_UNKNOWN, 0};
    double mu0 = 1.0;
    double rd_track = 1e300;
    bool rd_exact = true;
    // endgame (primal feasible, mu at target, dual residual not yet): the iterate with the
    // smallest exact dual residual — lane j < 6 keeps its component j — in case the dual
    // residual stalls (see below)
    double ybest_l = 0.0, best_rd = 1e300, best_rp = 0.0;
    int endgame = 0;
    double polish_mu = 0.0;
    const int gl_s = threadIdx.x & (G - 1);
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
        double rb = 0.0, ib = 0.0, dS = 0.0;
        double DcA[CB];  // slack mode: D of the live rows
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
                if (slk) t -= rw.ccv[c] * v;
                cr[c] = rw.chi[c] - t - cs[c];
                ci[c] = rcp(cs[c]);
                double D = cz[c] * ci[c];
                DcA[c] = 0.0;
                if (slk) {  // live slack rows enter through the stable Schur form below
                    DcA[c] = D * rw.ccv[c];
                    D -= DcA[c];
                }
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
            if (slk) {
                // bound v >= 0 (lower side, own slack sb). Eliminating v leaves, for the live rows
                // a, b of this lane, W = diag(D) - D D^T / S (S = sum D + D_b) between their g's,
                // accumulated in the Laplacian form
                //   sum_{a<b} (D_a D_b / S) (g_a - g_b)(g_a - g_b)^T + sum_a (D_a D_b' / S) g_a g_a^T
                // (D_b': the bound's weight): positive terms only, so nearly active rows (huge D)
                // on nearly parallel g (samples k = 0, 1 of one neighbour) do not cancel.
                rb = v - sb;
                ib = rcp(sb);
                const double Db = zb * ib;
                dS = Db;
#pragma unroll
                for (int a = 0; a < CB; a++) dS += DcA[a];
                const double iS = rcp(dS);
#pragma unroll
                for (int a = 0; a < CB; a++) {
                    const double* g = rw.cg[a];
                    const double wa = DcA[a] * Db * iS;
                    acc_blk2(acc + A_MX, wa, g[0], g[1]);
                    acc_blk2(acc + A_MY, wa, g[2], g[3]);
                    acc[A_MC + 0] = fma(wa * g[0], g[2], acc[A_MC + 0]);
                    acc[A_MC + 1] = fma(wa * g[0], g[3], acc[A_MC + 1]);
                    acc[A_MC + 2] = fma(wa * g[1], g[2], acc[A_MC + 2]);
                    acc[A_MC + 3] = fma(wa * g[1], g[3], acc[A_MC + 3]);
                    const double f = DcA[a] * fma(Db, cr[a] - rb, -wv_cost) * iS;
#pragma unroll
                    for (int j = 0; j < 4; j++) acc[A_RHS + j] = fma(g[j], f, acc[A_RHS + j]);
#pragma unroll
                    for (int b = a + 1; b < CB; b++) {
                        double e[4];
#pragma unroll
                        for (int j = 0; j < 4; j++) e[j] = g[j] - rw.cg[b][j];
                        const double wab = DcA[a] * DcA[b] * iS;
                        acc_blk2(acc + A_MX, wab, e[0], e[1]);
                        acc_blk2(acc + A_MY, wab, e[2], e[3]);
                        acc[A_MC + 0] = fma(wab * e[0], e[2], acc[A_MC + 0]);
                        acc[A_MC + 1] = fma(wab * e[0], e[3], acc[A_MC + 1]);
                        acc[A_MC + 2] = fma(wab * e[1], e[2], acc[A_MC + 2]);
                        acc[A_MC + 3] = fma(wab * e[1], e[3], acc[A_MC + 3]);
                        const double fab = wab * (cr[a] - cr[b]);
#pragma unroll
                        for (int j = 0; j < 4; j++) acc[A_RHS + j] = fma(e[j], fab, acc[A_RHS + j]);
                    }
                }
                acc[A_MU] = fma(sb, zb, acc[A_MU]);
                rp = fmax(rp, fabs(rb));
            }
            PSTAMP(1);
            if (red) grp_sum_vec_lds<A_N>(acc, red, threadIdx.x & (G - 1));
            else grp_sum_vec<G, A_N>(acc);
#ifdef MPCCBF_DEBUG_EXIT
            if (dbg) {  // is the reduced accumulator group-uniform?
                double dvg = 0.0;
#pragma unroll
                for (int k = 0; k < A_N; k++) dvg = fmax(dvg, fabs(acc[k] - __shfl(acc[k], 0, G)));
                dvg = grp_max<G>(dvg);
                double* dd = (double*)dbg;
                if (dvg > 0.0 && dd[13] == 0.0) {
                    dd[12] = dvg;
                    dd[13] = (double)(it + 1);
                }
            }
#endif
        } else {
            // no CBF row in this group: the x-y coupling block stays zero
            double part[A_N - 4];
#pragma unroll
            for (int k = 0; k < A_MC; k++) part[k] = acc[k];
#pragma unroll
            for (int k = A_RHS; k < A_N; k++) part[k - 4] = acc[k];
            PSTAMP(1);
            if (red) grp_sum_vec_lds<A_N - 4>(part, red, threadIdx.x & (G - 1));
            else grp_sum_vec<G, A_N - 4>(part);
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
            if (slk) {  // v: w - sum_rows cz - zb (relative to the slack cost scale)
                double rv = wv_cost - zb;
#pragma unroll
                for (int c = 0; c < CB; c++) rv = fma(-rw.ccv[c], cz[c], rv);
                rdn = fmax(rdn, grp_max<G>(fabs(rv) * rcp(1.0 + fabs(wv_cost))) * (1.0 + qn));  // per-lane scale, then the group max
            }
            rd_track = rdn * inv_qn;
            rd_exact = false;
        }
        out.iters = as_steps + it;
        const bool finite = isfinite(rp) && isfinite(rd_track) && isfinite(mu) && isfinite(acc[0]);
        // exact dual residual (relative), group-uniform
        auto exact_rd = [&]() {
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
            if (slk) {
                double rv = wv_cost - zb;
#pragma unroll
                for (int c = 0; c < CB; c++) rv = fma(-rw.ccv[c], cz[c], rv);
                rdn = fmax(rdn, grp_max<G>(fabs(rv) * rcp(1.0 + fabs(wv_cost))) * (1.0 + qn));  // per-lane scale, then the group max
            }
            return rdn * inv_qn;
        };
        // At a degenerate optimum (active rows' D = z/s ~1e20) the Newton step's dz carries
        // rounding of order eps D |ds|, so once mu is at its target the dual residual can stall
        // above the tolerance (and grow if the iteration goes on). The endgame keeps the iterate
        // with the smallest exact dual residual; after 3 endgame steps without convergence (or
        // any other stop) it is accepted if that residual meets the dual tolerance of the parity
        // rule / CPLEX (PdipCfg::rd_relax).
        bool stop_best = false;
        if (finite && rp <= cfg.tol && mu <= cfg.tol * 0.1) {
            rd_track = exact_rd();
            if (rd_track <= cfg.tol) {
                out.status = ST_OPTIMAL;
                out.rp = rp;
                out.rd = rd_track;
                break;
            }
            if (rd_track < best_rd) {
                best_rd = rd_track;
                best_rp = rp;
                double yl = y[0];
#pragma unroll
                for (int j = 1; j < SEP_NZ; j++) yl = gl_s == j ? y[j] : yl;
                ybest_l = yl;
            }
            stop_best = ++endgame >= 3;
        }
        if (it == 0) {
            mu0 = mu;
            polish_mu = 1e-3 * mu;
        }
        // active-set finish (sep_polish) once mu has fallen 1000x, then after every further 100x
        if constexpr (!SLACK) {
            if (pol != nullptr && finite && it > 0 && mu <= polish_mu) {
                double rpp = 0.0, rdp = 0.0;
                if (sep_polish<G, SB, CB>(rw, has_cbf, P, Pinv, q, sl, su, zl, zu, cs, cz, pl, pu, pc, cfg.tol, pol, y,
                                          rpp, rdp, warm)) {
                    out.status = ST_OPTIMAL;
                    out.rp = rpp;
                    out.rd = rdp;
                    out.polished = true;
                    break;
                }
                polish_mu = 1e-2 * mu;
            }
        }
        auto take_best = [&]() {  // the endgame's best iterate, if it meets the relaxed tolerance
            if (slk || !(best_rd <= cfg.rd_relax)) return false;  // slack mode: v is not kept
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) y[j] = __shfl(ybest_l, j, G);
            out.status = ST_OPTIMAL;
            out.rp = best_rp;
            out.rd = best_rd;
            return true;
        };
        if (stop_best) {
            if (!take_best()) out.status = ST_UNKNOWN;
            break;
        }
        if (cfg.early_it > 0 && it >= cfg.early_it && mu > cfg.early_mu * mu0) {
            out.status = ST_UNKNOWN;  // diverging: phase 1 decides (see PdipCfg::early_it)
            out.early = true;
            break;
        }
        if (it >= cfg.maxit || !finite || mu > 1e8 * fmax(mu0, 1.0)) {
            if (take_best()) break;
            out.status = ST_UNKNOWN;
#ifdef MPCCBF_DEBUG_EXIT  // diagnostics build: exit reason in the iteration count
            out.iters = it + 1000 * (it >= cfg.maxit ? 1 : !finite ? 2 : 3);
#endif
            break;
        }
        PSTAMP(3);
        // ---- factor: (x, y) 4x4 with the CBF coupling, yaw 2x2
        double Mxy[10], dxy[4], Mw[3], dw[2];
        using S4 = Sym<4>;
        auto form = [&](double tau) {  // Newton matrix from the reduced accumulators (+ tau I)
            Mxy[S4::idx(0, 0)] = acc[A_MX + 0] + P[0 * 6 + 0] + tau;
            Mxy[S4::idx(0, 1)] = acc[A_MX + 1] + P[0 * 6 + 1];
            Mxy[S4::idx(1, 1)] = acc[A_MX + 2] + P[1 * 6 + 1] + tau;
            Mxy[S4::idx(2, 2)] = acc[A_MY + 0] + P[2 * 6 + 2] + tau;
            Mxy[S4::idx(2, 3)] = acc[A_MY + 1] + P[2 * 6 + 3];
            Mxy[S4::idx(3, 3)] = acc[A_MY + 2] + P[3 * 6 + 3] + tau;
            Mxy[S4::idx(0, 2)] = acc[A_MC + 0];
            Mxy[S4::idx(0, 3)] = acc[A_MC + 1];
            Mxy[S4::idx(1, 2)] = acc[A_MC + 2];
            Mxy[S4::idx(1, 3)] = acc[A_MC + 3];
            Mw[0] = acc[A_MW + 0] + P[4 * 6 + 4] + tau;
            Mw[1] = acc[A_MW + 1] + P[4 * 6 + 5];
            Mw[2] = acc[A_MW + 2] + P[5 * 6 + 5] + tau;
        };
        double tau0 = 0.0;
        if (cfg.robust)
            tau0 = 1e-12 * fmax(fmax(fmax(acc[A_MX + 0] + P[0], acc[A_MX + 2] + P[7]),
                                     fmax(acc[A_MY + 0] + P[14], acc[A_MY + 2] + P[21])),
                                fmax(acc[A_MW + 0] + P[28], acc[A_MW + 2] + P[35]));
        form(tau0);
        bool ok4 = chol_packed<4>(Mxy, dxy);
        bool ok2 = chol_packed<2>(Mw, dw);
        if (!(ok4 && ok2)) {
            // breakdown at a degenerate near-optimal point (D = z/s of the active rows ~1e20
            // swamps P in the normal matrix): the endgame's best iterate, as the oracle keeps
            // its best iterate (oracle.cpp pdip); else the caller certifies and retries
            if (take_best()) break;
            out.status = ST_UNKNOWN;
#ifdef MPCCBF_DEBUG_EXIT
            out.iters = it + 4000;
            if (dbg) {  // the matrices that failed (as bits), for tools/dbg_slack.py
                using S4b = Sym<4>;
                double* dd = (double*)dbg;
                dd[0] = acc[A_MX + 0] + P[0];
                dd[1] = acc[A_MX + 2] + P[7];
                dd[2] = acc[A_MY + 0] + P[14];
                dd[3] = acc[A_MY + 2] + P[21];
                dd[4] = acc[A_MC + 0];
                dd[5] = acc[A_MC + 3];
                dd[6] = Mw[0];
                dd[7] = Mw[2];
                dd[8] = ok4 ? 1.0 : 0.0;
                dd[9] = ok2 ? 1.0 : 0.0;
                dd[10] = mu;
                dd[11] = slk ? dS : 0.0;

                (void)S4b::idx(0, 0);
            }
#endif
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
        double dv = 0.0, dsb = 0.0, dzb = 0.0;
        if (slk) {  // dv = (rhs_v - u^T dy) / S = sum_a D_a (g_a dy - cr_a) / S - (D_b r_b + w) / S
            dv = -(zb * ib) * rb - wv_cost;
#pragma unroll
            for (int a = 0; a < CB; a++) {
                double gd = -cr[a];
#pragma unroll
                for (int j = 0; j < 4; j++) gd = fma(rw.cg[a][j], dya[j], gd);
                dv = fma(DcA[a], gd, dv);
            }
            dv *= rcp(dS);
            dsb = dv + rb;
            const double qb = dsb * ib;
            dzb = -zb * (1.0 + qb);
            rs = fmax(rs, -qb);
            rz = fmax(rz, 1.0 + qb);
        }
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
                if (slk) td -= rw.ccv[c] * dv;
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
            if (slk) mua = fma(sb + ap * dsb, zb + ad * dzb, mua);
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
        double kb = 0.0, vcv = 0.0;
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
                if (slk) vcv = fma(-rw.ccv[c], w, vcv);
                const double wstd = slk ? w * (1.0 - rw.ccv[c]) : w;
#pragma unroll
                for (int j = 0; j < 4; j++) vc[j] = fma(rw.cg[c][j], wstd, vc[j]);
            }
            if (slk) {
                // live rows: sum_a (w_a + D_a vcv / S) g_a in the same pairwise form:
                //   sum_{a<b} (w_a D_b - D_a w_b)/S (g_a - g_b) + sum_a (w_a D_b' + D_a kb/sb)/S g_a
                kb = smu - dsb * dzb;
                vcv = fma(kb, ib, vcv);
                const double iS = rcp(dS), Db = zb * ib;
                double wl[CB];
#pragma unroll
                for (int a = 0; a < CB; a++) wl[a] = -kc[a] * ci[a] * rw.ccv[a];
#pragma unroll
                for (int a = 0; a < CB; a++) {
                    const double f = fma(wl[a], Db, DcA[a] * kb * ib) * iS;
#pragma unroll
                    for (int j = 0; j < 4; j++) vc[j] = fma(rw.cg[a][j], f, vc[j]);
#pragma unroll
                    for (int b = a + 1; b < CB; b++) {
                        const double fab = fma(wl[a], DcA[b], -DcA[a] * wl[b]) * iS;
#pragma unroll
                        for (int j = 0; j < 4; j++) vc[j] = fma(rw.cg[a][j] - rw.cg[b][j], fab, vc[j]);
                    }
                }
            }
        }
        grp_sum_vec<G, SEP_NZ>(vc);  // (6 values: the DPP butterfly beats the LDS round trip)
        PSTAMP(8);
        double dyc[SEP_NZ], dy[SEP_NZ];
        sep_solve(Mxy, dxy, Mw, dw, vc, dyc);
        PSTAMP(9);
#pragma unroll
        for (int i = 0; i < SEP_NZ; i++) dy[i] = dya[i] + dyc[i];
        // combined direction: ds from dy; dz = (k - s z - z ds) / s
        double rmax = 0.0;  // largest -ds/s, -dz/z over all sides
        if (slk) {
            dv = vcv - (zb * ib) * rb - wv_cost;
#pragma unroll
            for (int a = 0; a < CB; a++) {
                double gd = -cr[a];
#pragma unroll
                for (int j = 0; j < 4; j++) gd = fma(rw.cg[a][j], dy[j], gd);
                dv = fma(DcA[a], gd, dv);
            }
            dv *= rcp(dS);
            dsb = dv + rb;
            dzb = (kb - sb * zb - zb * dsb) * ib;
            rmax = fmax(rmax, fmax(-dsb * ib, -dzb * rcp_fast(zb)));
        }
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
                if (slk) td -= rw.ccv[c] * dv;
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
            if (slk) {
                v = fma(alpha, dv, v);
                sb = fmax(fma(alpha, dsb, sb), 1e-300);
                zb = fmax(fma(alpha, dzb, zb), 1e-300);
            }
        }
        rd_track *= (1.0 - alpha);
        if (it % 8 == 7) rd_exact = true;
        PSTAMP(11);
#ifdef MPCCBF_SOLVE_TRACE
        if (dbg && it < 32 && (threadIdx.x & (G - 1)) == 0) {
            double* dd = (double*)dbg;
            dd[it * 4 + 0] = rp;
            dd[it * 4 + 1] = mu;
            dd[it * 4 + 2] = alpha;
            dd[it * 4 + 3] = rd_track;
        }
#endif
#ifdef MPCCBF_DEBUG_EXIT
        if (dbg) {  // lane divergence of the iterate (must stay 0: y is group-uniform)
            double dvg = 0.0;
#pragma unroll
            for (int i = 0; i < SEP_NZ; i++) dvg = fmax(dvg, fabs(y[i] - __shfl(y[i], 0, G)));
            dvg = grp_max<G>(dvg);
            double* dd = (double*)dbg;
            if (dvg > 0.0 && dd[15] == 0.0) {
                dd[14] = dvg;
                dd[15] = (double)(it + 1);
            }
        }
#endif
    }
    if (v_out) *v_out = slk ? v : 0.0;
    if (warm != nullptr && out.status == ST_OPTIMAL && !out.polished) {
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                warm->zl(d, k) = zl[d][k];
                warm->zu(d, k) = zu[d][k];
            }
    }
#ifdef MPCCBF_DEBUG_EXIT
    if (dbg) {  // per-lane exit iteration (all lanes of a group must agree)
        const int gl = lane_bits_opaque<G - 1>();
        dbg[16 * 64 + gl] = out.iters;  // caller's buffer: + num_agents * 16 slots (see dbg_slack.py)
    }
#endif
    return out;
}

// Phase 1 on the separable rows (only runs for QPs whose main solve did not converge):
//     t* = min t   s.t.  lo - t <= g y <= hi + t  (box rows),  cg y - t <= chi  (CBF rows),  t >= 0
// with the ridge eps/2 |y|^2 of pdip_phase1. The Newton matrix keeps the separable structure,
// M = [[A, b], [b^T, c]] with A the (x, y) 4x4 + yaw 2x2 blocks of pdip_solve_sep and (b, c) the
// t column; it is solved through the Schur complement on t (u = A^-1 b once per step, then
// dt = (r_t - b^T A^-1 r_y) / (c - b^T u), dy = A^-1 r_y - u dt), so a step costs about one main
// Newton step instead of a dense 7x7 one. Returns the largest row violation at the final y (an
// upper bound of t*, equal to it at convergence; the QP is INFEASIBLE iff it exceeds feas_tol).
// It stops as soon as that decision is settled:
//   * the row violation at the iterate is <= feas_tol (a point feasible within the tolerance);
//   * the iterate is primal feasible for the phase-1 LP (relative residual <= tol), t >= 1e-4
//     and the duality gap is <= 1e-3 t, so t* >= t - gap > 0.999e-4 >> feas_tol;
// otherwise it converges fully (residual and mu at the main tolerance), as pdip_phase1 does.
template <int G, int SB, int CB>
__device__ double pdip_phase1_sep(const SepRows<SB, CB>& rw, const PdipCfg cfg, double feas_tol,
                                  const double (&ystart)[SEP_NZ], double* red = nullptr,
                                  int* iters_out = nullptr, long long* dbg = nullptr) {
    (void)dbg;
    constexpr double eps = 1e-10;
    constexpr int P_MX = 0, P_MY = 3, P_MW = 6, P_MC = 9, P_B = 13, P_C = 19, P_R = 20, P_RT = 26,
                  P_MU = 27, P_N = 28;
    // start at ystart (the main solve's last iterate: close to the least violating point; the
    // origin if it is not finite), t = its largest violation + 1, so every slack is >= 1
    double y[SEP_NZ];
    bool fin = true;
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) fin = fin && isfinite(ystart[j]);
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) y[j] = fin ? ystart[j] : 0.0;
    double viol = 0.0;
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const double ty = rw.bg[d][k][0] * y[2 * d] + rw.bg[d][k][1] * y[2 * d + 1];
            viol = fmax(viol, fmax(rw.blo[d][k] - ty, ty - rw.bhi[d][k]));
        }
#pragma unroll
    for (int c = 0; c < CB; c++) {
        double tc = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++) tc = fma(rw.cg[c][j], y[j], tc);
        viol = fmax(viol, tc - rw.chi[c]);
    }
    double t = grp_max<G>(viol) + 1.0;
    double sl[SEP_D][SB], su[SEP_D][SB], zl[SEP_D][SB], zu[SEP_D][SB], pl[SEP_D][SB], pu[SEP_D][SB];
    double cs[CB], cz[CB], pc[CB];
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const double ty = rw.bg[d][k][0] * y[2 * d] + rw.bg[d][k][1] * y[2 * d + 1];
            sl[d][k] = ty + t - rw.blo[d][k];
            su[d][k] = rw.bhi[d][k] - ty + t;
            zl[d][k] = rcp(sl[d][k]);
            zu[d][k] = rcp(su[d][k]);
            pl[d][k] = rcp(1.0 + fabs(rw.blo[d][k]));
            pu[d][k] = rcp(1.0 + fabs(rw.bhi[d][k]));
        }
#pragma unroll
    for (int c = 0; c < CB; c++) {
        double tc = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++) tc = fma(rw.cg[c][j], y[j], tc);
        cs[c] = rw.chi[c] - tc + t;
        cz[c] = rcp(cs[c]);
        pc[c] = rcp(1.0 + fabs(rw.chi[c]));
    }
    double zt = rcp(t);
    const double inv_ns = 1.0 / (double)(G * (2 * SEP_D * SB + CB) + 1);
    const int gl = lane_bits_opaque<G - 1>();
    int it = 0;
    for (; it < 2 * cfg.maxit; it++) {
        double acc[P_N];
#pragma unroll
        for (int k = 0; k < P_N; k++) acc[k] = 0.0;
        double rl[SEP_D][SB], ru[SEP_D][SB], il[SEP_D][SB], iu[SEP_D][SB], cr[CB], ci[CB], Dc[CB];
        double rp = 0.0, worst = 0.0;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const double g0 = rw.bg[d][k][0], g1 = rw.bg[d][k][1];
                const double ty = g0 * y[2 * d] + g1 * y[2 * d + 1];
                rl[d][k] = ty + t - rw.blo[d][k] - sl[d][k];
                ru[d][k] = rw.bhi[d][k] - ty + t - su[d][k];
                il[d][k] = rcp(sl[d][k]);
                iu[d][k] = rcp(su[d][k]);
                const double Dl = zl[d][k] * il[d][k], Du = zu[d][k] * iu[d][k];
                const double wl = -Dl * rl[d][k], wu = -Du * ru[d][k];
                acc_blk2(acc + P_MX + 3 * d, Dl + Du, g0, g1);
                acc[P_B + 2 * d] = fma(Dl - Du, g0, acc[P_B + 2 * d]);
                acc[P_B + 2 * d + 1] = fma(Dl - Du, g1, acc[P_B + 2 * d + 1]);
                acc[P_C] += Dl + Du;
                acc[P_R + 2 * d] = fma(g0, wl - wu, acc[P_R + 2 * d]);
                acc[P_R + 2 * d + 1] = fma(g1, wl - wu, acc[P_R + 2 * d + 1]);
                acc[P_RT] += wl + wu;
                acc[P_MU] = fma(sl[d][k], zl[d][k], fma(su[d][k], zu[d][k], acc[P_MU]));
                rp = fmax(rp, fmax(fabs(rl[d][k]) * pl[d][k], fabs(ru[d][k]) * pu[d][k]));
                worst = fmax(worst, fmax(rw.blo[d][k] - ty, ty - rw.bhi[d][k]));
            }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            const double* g = rw.cg[c];
            double tc = 0.0;
#pragma unroll
            for (int j = 0; j < 4; j++) tc = fma(g[j], y[j], tc);
            cr[c] = rw.chi[c] - tc + t - cs[c];
            ci[c] = rcp(cs[c]);
            Dc[c] = cz[c] * ci[c];
            const double D = Dc[c], w = -D * cr[c];
            acc_blk2(acc + P_MX, D, g[0], g[1]);
            acc_blk2(acc + P_MY, D, g[2], g[3]);
            acc[P_MC + 0] = fma(D * g[0], g[2], acc[P_MC + 0]);
            acc[P_MC + 1] = fma(D * g[0], g[3], acc[P_MC + 1]);
            acc[P_MC + 2] = fma(D * g[1], g[2], acc[P_MC + 2]);
            acc[P_MC + 3] = fma(D * g[1], g[3], acc[P_MC + 3]);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                acc[P_B + j] = fma(-D, g[j], acc[P_B + j]);
                acc[P_R + j] = fma(-g[j], w, acc[P_R + j]);
            }
            acc[P_C] += D;
            acc[P_RT] += w;
            acc[P_MU] = fma(cs[c], cz[c], acc[P_MU]);
            rp = fmax(rp, fabs(cr[c]) * pc[c]);
            worst = fmax(worst, tc - rw.chi[c]);
        }
        if (red) {  // two LDS passes through the 16 x 21 table of the main solver
            double h0[14], h1[14];
#pragma unroll
            for (int k = 0; k < 14; k++) {
                h0[k] = acc[k];
                h1[k] = acc[14 + k];
            }
            grp_sum_vec_lds<14>(h0, red, gl);
            grp_sum_vec_lds<14>(h1, red, gl);
#pragma unroll
            for (int k = 0; k < 14; k++) {
                acc[k] = h0[k];
                acc[14 + k] = h1[k];
            }
        } else {
            grp_sum_vec<G, P_N>(acc);
        }
        grp_max2<G>(rp, worst);
        const double gap = acc[P_MU] + t * zt;
        const double mu = gap * inv_ns;
        if (!isfinite(mu) || !isfinite(rp) || !isfinite(t)) {
            if (iters_out) *iters_out = it;
            return 1e300;
        }
#ifdef MPCCBF_SOLVE_TRACE
        if (dbg && it < 32 && gl == 0) {
            double* dd = (double*)dbg + 128;
            dd[it * 4 + 0] = rp;
            dd[it * 4 + 1] = mu;
            dd[it * 4 + 2] = t;
            dd[it * 4 + 3] = worst;
        }
#endif
        if (worst <= feas_tol) break;  // feasible within the tolerance
        if (rp <= cfg.tol && (mu <= cfg.tol * 0.1 || (t >= 1e-4 && gap <= 1e-3 * t))) break;
        // ---- Newton matrix: A (4x4 + 2x2, ridge eps), t column b, corner c
        using S4 = Sym<4>;
        double Mxy[10], dxy[4], Mw[3], dw[2];
        Mxy[S4::idx(0, 0)] = acc[P_MX + 0] + eps;
        Mxy[S4::idx(0, 1)] = acc[P_MX + 1];
        Mxy[S4::idx(1, 1)] = acc[P_MX + 2] + eps;
        Mxy[S4::idx(2, 2)] = acc[P_MY + 0] + eps;
        Mxy[S4::idx(2, 3)] = acc[P_MY + 1];
        Mxy[S4::idx(3, 3)] = acc[P_MY + 2] + eps;
        Mxy[S4::idx(0, 2)] = acc[P_MC + 0];
        Mxy[S4::idx(0, 3)] = acc[P_MC + 1];
        Mxy[S4::idx(1, 2)] = acc[P_MC + 2];
        Mxy[S4::idx(1, 3)] = acc[P_MC + 3];
        Mw[0] = acc[P_MW + 0] + eps;
        Mw[1] = acc[P_MW + 1];
        Mw[2] = acc[P_MW + 2] + eps;
        if (!(chol_packed<4>(Mxy, dxy) && chol_packed<2>(Mw, dw))) break;  // the iterate stands
        const double Dt = zt * rcp(t);
        double bv[SEP_NZ], u[SEP_NZ];
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) bv[j] = acc[P_B + j];
        sep_solve(Mxy, dxy, Mw, dw, bv, u);
        double sch = acc[P_C] + Dt;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) sch = fma(-bv[j], u[j], sch);
        if (!(sch > 0.0)) break;
        const double isch = rcp(sch);
        // solve [A b; b^T c] [dy; dt] = [ry; rt]
        auto solve7 = [&](const double (&ry)[SEP_NZ], double rt, double (&dy)[SEP_NZ], double& dt) {
            double w[SEP_NZ];
            sep_solve(Mxy, dxy, Mw, dw, ry, w);
            double v = rt;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) v = fma(-bv[j], w[j], v);
            dt = v * isch;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) dy[j] = fma(-u[j], dt, w[j]);
        };
        // ---- predictor
        double ry[SEP_NZ], dya[SEP_NZ], dta;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) ry[j] = fma(-eps, y[j], acc[P_R + j]);
        solve7(ry, acc[P_RT] - 1.0, dya, dta);
        double dsl[SEP_D][SB], dsu[SEP_D][SB], dzl[SEP_D][SB], dzu[SEP_D][SB], cds[CB], cdz[CB];
        double rs = fmax(0.0, -dta * rcp(t)), rz = 1.0 + dta * rcp(t);  // t >= 0 side: s_t = t
        const double dzta = -zt - Dt * dta;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const double td = rw.bg[d][k][0] * dya[2 * d] + rw.bg[d][k][1] * dya[2 * d + 1];
                dsl[d][k] = td + dta + rl[d][k];
                dsu[d][k] = -td + dta + ru[d][k];
                const double ql = dsl[d][k] * il[d][k], qu = dsu[d][k] * iu[d][k];
                dzl[d][k] = -zl[d][k] * (1.0 + ql);
                dzu[d][k] = -zu[d][k] * (1.0 + qu);
                rs = fmax(rs, fmax(-ql, -qu));
                rz = fmax(rz, fmax(1.0 + ql, 1.0 + qu));
            }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            double td = 0.0;
#pragma unroll
            for (int j = 0; j < 4; j++) td = fma(rw.cg[c][j], dya[j], td);
            cds[c] = -td + dta + cr[c];
            const double qc = cds[c] * ci[c];
            cdz[c] = -cz[c] * (1.0 + qc);
            rs = fmax(rs, -qc);
            rz = fmax(rz, 1.0 + qc);
        }
        grp_max2<G>(rs, rz);
        const double ap = rcp(fmax(1.0, rs)), ad = rcp(fmax(1.0, rz));
        double mua = 0.0;
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                mua = fma(sl[d][k] + ap * dsl[d][k], zl[d][k] + ad * dzl[d][k], mua);
                mua = fma(su[d][k] + ap * dsu[d][k], zu[d][k] + ad * dzu[d][k], mua);
            }
#pragma unroll
        for (int c = 0; c < CB; c++) mua = fma(cs[c] + ap * cds[c], cz[c] + ad * cdz[c], mua);
        mua = (grp_sum<G>(mua) + (t + ap * dta) * (zt + ad * dzta)) * inv_ns;
        double sig = mu > 0.0 ? mua * rcp(mu) : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        // ---- corrector right-hand side
        double vc[SEP_NZ + 1];
#pragma unroll
        for (int j = 0; j <= SEP_NZ; j++) vc[j] = 0.0;
        double kl[SEP_D][SB], ku[SEP_D][SB], kc[CB];
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                kl[d][k] = smu - dsl[d][k] * dzl[d][k];
                ku[d][k] = smu - dsu[d][k] * dzu[d][k];
                const double a = kl[d][k] * il[d][k], b = ku[d][k] * iu[d][k];
                vc[2 * d] = fma(rw.bg[d][k][0], a - b, vc[2 * d]);
                vc[2 * d + 1] = fma(rw.bg[d][k][1], a - b, vc[2 * d + 1]);
                vc[SEP_NZ] += a + b;
            }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            kc[c] = smu - cds[c] * cdz[c];
            const double a = kc[c] * ci[c];
#pragma unroll
            for (int j = 0; j < 4; j++) vc[j] = fma(-rw.cg[c][j], a, vc[j]);
            vc[SEP_NZ] += a;
        }
        grp_sum_vec<G, SEP_NZ + 1>(vc);
        const double kt = smu - dta * dzta;
        double vy[SEP_NZ], dyc[SEP_NZ], dtc;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) vy[j] = vc[j];
        solve7(vy, vc[SEP_NZ] + kt * rcp(t), dyc, dtc);
        double dy[SEP_NZ];
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) dy[j] = dya[j] + dyc[j];
        const double dt = dta + dtc;
        // ---- combined direction, step to the boundary
        const double dzt = (kt - t * zt - zt * dt) * rcp(t);
        double rmax = fmax(-dt * rcp(t), -dzt * rcp_fast(zt));
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const double td = rw.bg[d][k][0] * dy[2 * d] + rw.bg[d][k][1] * dy[2 * d + 1];
                dsl[d][k] = td + dt + rl[d][k];
                dsu[d][k] = -td + dt + ru[d][k];
                dzl[d][k] = (kl[d][k] - sl[d][k] * zl[d][k] - zl[d][k] * dsl[d][k]) * il[d][k];
                dzu[d][k] = (ku[d][k] - su[d][k] * zu[d][k] - zu[d][k] * dsu[d][k]) * iu[d][k];
                rmax = fmax(rmax, fmax(-dsl[d][k] * il[d][k], -dsu[d][k] * iu[d][k]));
                rmax = fmax(rmax, fmax(-dzl[d][k] * rcp_fast(zl[d][k]), -dzu[d][k] * rcp_fast(zu[d][k])));
            }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            double td = 0.0;
#pragma unroll
            for (int j = 0; j < 4; j++) td = fma(rw.cg[c][j], dy[j], td);
            cds[c] = -td + dt + cr[c];
            cdz[c] = (kc[c] - cs[c] * cz[c] - cz[c] * cds[c]) * ci[c];
            rmax = fmax(rmax, fmax(-cds[c] * ci[c], -cdz[c] * rcp_fast(cz[c])));
        }
        rmax = grp_max<G>(rmax);
        const double alpha = 0.99 * rcp(fmax(0.99, rmax));
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) y[j] = fma(alpha, dy[j], y[j]);
        t = fmax(fma(alpha, dt, t), 1e-300);
        zt = fmax(fma(alpha, dzt, zt), 1e-300);
#pragma unroll
        for (int d = 0; d < SEP_D; d++)
#pragma unroll
            for (int k = 0; k < SB; k++) {
                sl[d][k] = fmax(fma(alpha, dsl[d][k], sl[d][k]), 1e-300);
                su[d][k] = fmax(fma(alpha, dsu[d][k], su[d][k]), 1e-300);
                zl[d][k] = fmax(fma(alpha, dzl[d][k], zl[d][k]), 1e-300);
                zu[d][k] = fmax(fma(alpha, dzu[d][k], zu[d][k]), 1e-300);
            }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            cs[c] = fmax(fma(alpha, cds[c], cs[c]), 1e-300);
            cz[c] = fmax(fma(alpha, cdz[c], cz[c]), 1e-300);
        }
    }
    if (iters_out) *iters_out = it;
    // t* from the iterate: the largest actual row violation at y (>= 0)
    double worst = 0.0;
#pragma unroll
    for (int d = 0; d < SEP_D; d++)
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const double ty = rw.bg[d][k][0] * y[2 * d] + rw.bg[d][k][1] * y[2 * d + 1];
            worst = fmax(worst, fmax(rw.blo[d][k] - ty, ty - rw.bhi[d][k]));
        }
#pragma unroll
    for (int c = 0; c < CB; c++) {
        double tc = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++) tc = fma(rw.cg[c][j], y[j], tc);
        worst = fmax(worst, tc - rw.chi[c]);
    }
    return grp_max<G>(worst);
}

}  // namespace dev
}  // namespace mpccbf
