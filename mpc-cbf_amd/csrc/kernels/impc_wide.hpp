// impc_wide.hpp — ConnectivityIMPCCBF::optimize (mpc_cbf/src/controller/ConnectivityIMPCCBF.cpp:47-215)
// with ONE AGENT PER WAVE64 and one QP row per lane: the layout for small agent counts per GPU
// (config 4's 1,024-agent rank share) and, because its lanes hold a row each instead of four, the
// default separable collision kernel.
//
// Lane layout (64 lanes = one agent):
//   lanes  0..47  box row l % 16 of channel l / 16 (x, y, yaw): two-sided, coefficients on the
//                 channel's 2 reduced variables (inert slots: g = 0, -1 <= 0 <= 1);
//   lanes 48..63  CBF row c = l - 48 of the current IMPC iteration (the kept rows compacted in
//                 (sample, neighbour) order, ConnectivityIMPCCBF.cpp:135-141 / :170-178); one-sided.
// Everything per agent that is not a row (linear term, the active set's k <= 6 rows and their
// Cholesky factor, the iterate) is wave-uniform: every lane holds the same values, so the
// dependent chain of an active-set step is one row scan (one evaluation per lane), a 64-lane
// max reduction (DPP in the 16-lane rows, then permlane16/32 swaps across them) and k x k
// substitutions, with no per-lane loop over row slots.
//
// Solver: the same pipeline as the 16-lane kernel's first attempt — fast start (the unconstrained
// minimiser; the dual active set's first scan), then the dual active set (Goldfarb-Idnani, range
// space; the normalised candidate rule v / sqrt(g P^-1 g); IMPC iteration 1 warm-started from
// iteration 0's final active set after >= das_warm steps). What that solve does not settle — the
// step limit, a breakdown, a dual residual the updates lost to rounding, no feasible point without
// a certificate well above the tolerance — defers the whole agent to the fallback launch
// (impc_sep_kernel<.., QUEUE>: the full pipeline with the PDIP and phase 1), exactly as the lean
// 16-lane launch did. So every status this kernel returns is either the active set's exact optimum,
// a certified infeasibility, or the 16-lane pipeline's own result.
// (Device code, included by impc_kernel.hip, which instantiates the kernels: the inline-fallback
// form calls that file's 16-lane agent pipeline, impc_sep_agent.)
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#include "impc.hpp"
#include "impc_common.hpp"
#include "pdip.hpp"
#include "pdip_sep.hpp"

namespace mpccbf {
namespace dev {

constexpr int W_BOX = 48;   // box lanes (3 channels x 16 slots)
constexpr int W_CBF = 16;   // CBF lanes
constexpr int W_ROW = 5;    // staged CBF row: 4 coefficients (x0, x1, y0, y1) + upper bound
// active sides the wide solver holds (the 16-lane pipeline's POL_K = 6: a QP that needs more is
// deferred to it; k <= 2 at steady state)
constexpr int WK = 4;
// operator doubles the wide kernel stages in LDS (DevOps::hot must fit: ~1,700 at K = 15)
constexpr int WIDE_OPS = 2048;

// ---- wave-uniform helpers -------------------------------------------------------------------
__device__ __forceinline__ double uni(double v) {  // lane 0's value, as a scalar (uniform) operand
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double lane_of(double v, int l) {  // lane l's value (l uniform)
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// profiling build (make prof): shader-clock stamps of iteration 0's sub-phases, 16 per agent after
// the phase stamps (tools/wide_stamps.py): WST(k) writes stamp k of this agent (lane 0)
#ifdef MPCCBF_PDIP_STAMPS
#define WST(k)                                                                                         \
    do {                                                                                               \
        if (wdbg) {                                                                                    \
            const long long t_ = (long long)__builtin_amdgcn_s_memtime();                              \
            if ((threadIdx.x & 63u) == 0) wdbg[k] = t_;                                                \
        }                                                                                              \
    } while (0)
#else
#define WST(k) \
    do {       \
    } while (0)
#endif

template <int N>
__device__ __forceinline__ void uni_arr(double (&a)[N]) {
#pragma unroll
    for (int i = 0; i < N; i++) a[i] = uni(a[i]);
}
__device__ __forceinline__ int uni_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ bool uni_b(bool v) { return __builtin_amdgcn_readfirstlane((int)v) != 0; }

// two 64-lane max all-reductions, stage-interleaved (every lane ends with both maxima)
__device__ __forceinline__ void wave_max2(double& a, double& b) {
    grp_max2<16>(a, b);
    double a0, a1, b0, b1;
    row_pair<false>(a, a0, a1);
    row_pair<false>(b, b0, b1);
    a = fmax(a0, a1);
    b = fmax(b0, b1);
    row_pair<true>(a, a0, a1);
    row_pair<true>(b, b0, b1);
    a = fmax(a0, a1);
    b = fmax(b0, b1);
}

__device__ __forceinline__ double wave_max_f64(double a) {
    a = grp_max<16>(a);
    double a0, a1;
    row_pair<false>(a, a0, a1);
    a = fmax(a0, a1);
    row_pair<true>(a, a0, a1);
    return fmax(a0, a1);
}

// ---- this lane's row -----------------------------------------------------------------------
struct WRow {
    double g[SEP_NZ];  // coefficients on y (box: the channel's pair, CBF: x and y pairs)
    double lo, hi;     // CBF lanes: lo = -1e300 (no lower side)
    double w;          // candidate weight 1 / sqrt(g P^-1 g), float-rounded (the 16-lane wrow)
    double sl, su;     // violation scales 1 / (1 + |lo|), 1 / (1 + |hi|)
};

// the candidate weight of a row with coefficients (g0, g1) on one channel whose P^-1 block is
// (p0, p1; p1, p2): the arithmetic of sep_dual_as's wrow
__device__ __forceinline__ double wide_n2(double p0, double p1, double p2, double g0, double g1) {
    return fma(fma(p0, g0, 2.0 * p1 * g1), g0, p2 * g1 * g1);
}
__device__ __forceinline__ double wide_weight(double n2) { return (double)rsqrtf((float)fmax(n2, 1e-30)); }

// side `side` (0 lower, 1 upper) of this lane's row as a 16-double record (pdip_sep.hpp POL_*
// layout: g | b | sign | P^-1 g | id); the same arithmetic as sep_stage_side
__device__ __forceinline__ void wide_stage(const WRow& rw, const double (&pi)[SEP_D][3], int side, int gl,
                                           double* __restrict__ r) {
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) r[j] = rw.g[j];
    r[POL_B] = side ? rw.hi : rw.lo;
    r[POL_SGN] = side ? 1.0 : -1.0;
#pragma unroll
    for (int d = 0; d < SEP_D; d++) {
        r[POL_W + 2 * d] = fma(pi[d][0], rw.g[2 * d], pi[d][1] * rw.g[2 * d + 1]);
        r[POL_W + 2 * d + 1] = fma(pi[d][1], rw.g[2 * d], pi[d][2] * rw.g[2 * d + 1]);
    }
    r[POL_ID] = (double)(gl * 2 + side);
}

__device__ __forceinline__ double dot6(const double (&g)[SEP_NZ], const double (&y)[SEP_NZ]) {
    double t = 0.0;
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) t = fma(g[j], y[j], t);
    return t;
}

// Dual active-set solve (sep_dual_as on the one-row-per-lane layout; same candidate rule, step,
// factor updates and convergence test). pol: this wave's LDS rows ((POL_K + 1) x 16 doubles, the
// candidate in row POL_K). Returns 1: optimal (yo, residuals); -1: no step reaches the candidate
// (tlow: the certificate's lower bound on phase 1's t*); 0: gave up — the caller defers the agent.
// k0 > 0: warm start from the side ids warm_ids[0 .. k0); save: the final active set's ids.
__device__ int wide_dual_as(const WRow& rw, const double* __restrict__ P, const double* __restrict__ Pinv,
                            const double (&q)[SEP_NZ], const double (&yu)[SEP_NZ], double tol, int maxstep,
                            double* __restrict__ pol, double (&yo)[SEP_NZ], double& rp_out, double& rd_out,
                            int& steps, double& tlow, int k0, const double* __restrict__ warm_ids,
                            double* __restrict__ save, bool want_rp, long long* wdbg = nullptr) {
    (void)wdbg;
    WST(5);
    const int gl = lane_bits_opaque<63>();
    double pi[SEP_D][3];
    sep_pinv(Pinv, pi);
    // violation scales 1 / (1 + |bound|) and the candidate weight 1 / sqrt(g P^-1 g): the row's
    // (formed where the row is)
    const double sl = rw.sl, su = rw.su;
    const double w = rw.w;
    double y[SEP_NZ], u[WK];
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) y[j] = yu[j];
#pragma unroll
    for (int i = 0; i < WK; i++) u[i] = 0.0;
    int k = 0;
    steps = 0;
    const double add_tol = 0.1 * tol;
    double* cand = pol + POL_K * 16;
    using S6 = Sym<WK>;
    double L[S6::P], dl[WK];
#pragma unroll
    for (int i = 0; i < WK; i++) {
        dl[i] = 1.0;
#pragma unroll
        for (int j = i; j < WK; j++) L[S6::idx(i, j)] = i == j ? 1.0 : 0.0;
    }
    if (k0 > 0) {
        // the equality QP on the given sides; start there when every multiplier has its sign
        double rhs[WK], lam[WK];
        for (int i = 0; i < k0; i++) {
            const int id = (int)warm_ids[i];
            if ((id >> 1) == gl) wide_stage(rw, pi, id & 1, gl, pol + i * 16);
        }
        wave_lds_sync();
        sep_gram<WK>(pol, k0, L);
#pragma unroll
        for (int i = 0; i < WK; i++) {
            const double* ri = pol + (i < k0 ? i : 0) * 16;
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) t = fma(ri[j], yu[j], t);
            rhs[i] = i < k0 ? t - ri[POL_B] : 0.0;
        }
        bool ok = chol_packed<WK>(L, dl);
        chol_solve<WK>(L, dl, rhs, lam);
#pragma unroll
        for (int i = 0; i < WK; i++) {
            const double* ri = pol + (i < k0 ? i : 0) * 16;
            u[i] = i < k0 ? ri[POL_SGN] * lam[i] : 0.0;
            ok = ok && (i >= k0 || (u[i] >= 0.0 && isfinite(u[i])));
        }
        if (uni_b(ok)) {
#pragma unroll
            for (int i = 0; i < WK; i++) {
                const double* wi = pol + (i < k0 ? i : 0) * 16 + POL_W;
#pragma unroll
                for (int j = 0; j < SEP_NZ; j++) y[j] = fma(i < k0 ? -lam[i] : 0.0, wi[j], y[j]);
            }
            k = k0;
        } else {
#pragma unroll
            for (int i = 0; i < WK; i++) {
                u[i] = 0.0;
                dl[i] = 1.0;
#pragma unroll
                for (int j = i; j < WK; j++) L[S6::idx(i, j)] = i == j ? 1.0 : 0.0;
            }
        }
    }
    double m = 0.0;
    WST(6);
    for (int outer = 0;; outer++) {
        // this lane's sides: scaled violation (convergence) and normalised violation (candidate)
        double vb, eb;
        int sb;
        bool nanv;
        {
            const double t = dot6(rw.g, y);
            const double al = rw.lo - t, vl = al * sl;
            const double au = t - rw.hi, vu = au * su;
            const double el = vl > add_tol ? al * w : -1.0;
            const double eu = vu > add_tol ? au * w : -1.0;
            eb = -1.0;
            sb = 0;
            if (el > eb) eb = el, sb = 0;
            if (eu > eb) eb = eu, sb = 1;
            nanv = vl != vl || vu != vu;
            vb = fmax(-1.0, fmax(vl, vu));
        }
        if (outer == 0) WST(7);
        if (outer == 0 && __ballot(nanv) != 0ull) return 0;
        // the candidate: the largest normalised violation (as a float bit pattern), its lowest lane
        // on ties. A side violated beyond add_tol keys at least 1 — also when its score rounds to 0
        // in float (a weight w = 0 from a row norm beyond the float range) — so the solve is
        // converged exactly when every key is 0 (das_wave's rule)
        const bool viol = vb > add_tol;
        const unsigned key = viol ? max(__float_as_uint((float)fmax(eb, 0.0)), 1u) : 0u;
        const unsigned kmax = (unsigned)uni_i((int)wave_max_u32(key));
        if (outer == 0) WST(8);
        if (kmax == 0u) {
            if (want_rp) m = uni(wave_max_f64(vb));  // the scaled primal residual of the returned point
            break;
        }
        if (steps >= maxstep) return 0;
        // the best candidate's score is 0 or denormal in float: no usable rule (the 16-lane
        // pipeline solves it, deferred)
        if (kmax == 1u) return 0;
        const int owner = __ffsll((long long)__ballot(key == kmax)) - 1;
        if (owner < 0) return 0;
        if (gl == owner) wide_stage(rw, pi, sb, gl, cand);
        wave_lds_sync();
        if (k == 0) {
            // first side of an empty active set: the step reaches it, L = (sqrt(g P^-1 g))
            ++steps;
            const double sp = cand[POL_SGN];
            double nw = 0.0, gy = 0.0;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) {
                nw = fma(cand[j], cand[POL_W + j], nw);
                gy = fma(cand[j], y[j], gy);
            }
            if (!uni_b(nw > 0.0)) return 0;
            const double t = sp * (gy - cand[POL_B]) * rcp(nw);
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) y[j] = fma(-t * sp, cand[POL_W + j], y[j]);
            wave_lds_sync();
            if (gl < 16) pol[gl] = cand[gl];
            const double rz = rsqrt(nw);
            L[S6::idx(0, 0)] = nw * rz;
            dl[0] = rz;
            u[0] = t;
            k = 1;
            wave_lds_sync();
            continue;
        }
        double up = 0.0;
        for (;;) {
            if (++steps > maxstep) return 0;
            double gp[SEP_NZ];
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) gp[j] = cand[j];
            const double sp = cand[POL_SGN];
            // v = L^-1 (sp c), c_i = g_i P^-1 g_p
            double v[WK], sgn[WK];
#pragma unroll
            for (int i = 0; i < WK; i++) {
                v[i] = 0.0;
                sgn[i] = 0.0;
                if (i < k) {
                    const double* ri = pol + i * 16;
                    double t = 0.0;
#pragma unroll
                    for (int j = 0; j < SEP_NZ; j++) t = fma(ri[POL_W + j], gp[j], t);
                    sgn[i] = ri[POL_SGN];
                    double s = sp * t;
#pragma unroll
                    for (int mm = 0; mm < i; mm++) s = fma(-L[S6::idx(mm, i)], v[mm], s);
                    v[i] = s * dl[i];
                }
            }
            // rho = L^-T v
            double rho[WK];
#pragma unroll
            for (int i = WK - 1; i >= 0; i--) {
                rho[i] = 0.0;
                if (i < k) {
                    double s = v[i];
#pragma unroll
                    for (int mm = i + 1; mm < WK; mm++) s = fma(-L[S6::idx(i, mm)], rho[mm], s);
                    rho[i] = s * dl[i];
                }
            }
            double nw = 0.0, vv = 0.0, vp = 0.0;
#pragma unroll
            for (int j = 0; j < SEP_NZ; j++) {
                nw = fma(gp[j], cand[POL_W + j], nw);
                vp = fma(gp[j], y[j], vp);
            }
#pragma unroll
            for (int i = 0; i < WK; i++) vv = fma(v[i], v[i], vv);
            const double zn = nw - vv;
            vp = sp * (vp - cand[POL_B]);
            double un = 1.0, rn = 0.0;
            int l = -1;
#pragma unroll
            for (int i = 0; i < WK; i++) {
                const double r = sgn[i] * rho[i];
                const bool better = i < k && r > 0.0 && u[i] * rn < un * r;
                un = better ? u[i] : un;
                rn = better ? r : rn;
                l = better ? i : l;
            }
            l = uni_i(l);
            const double t1 = l >= 0 ? un * rcp(rn) : 1e300;
            const bool full = uni_b(zn > 1e-10 * nw);
            const double t2 = full ? vp * rcp(zn) : 1e300;
            if (l < 0 && !full) {
                double lsum = 1.0;
#pragma unroll
                for (int i = 0; i < WK; i++) {
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
            if (full) {
                asm volatile("" ::: "memory");
                double z[SEP_NZ];
#pragma unroll
                for (int j = 0; j < SEP_NZ; j++) z[j] = sp * cand[POL_W + j];
#pragma unroll
                for (int i = 0; i < WK; i++) {
                    if (i < k) {
                        const double* wi = pol + i * 16 + POL_W;
#pragma unroll
                        for (int j = 0; j < SEP_NZ; j++) z[j] = fma(-rho[i], wi[j], z[j]);
                    }
                }
#pragma unroll
                for (int j = 0; j < SEP_NZ; j++) y[j] = fma(-t, z[j], y[j]);
            }
#pragma unroll
            for (int i = 0; i < WK; i++) u[i] = i < k ? fma(-t, sgn[i] * rho[i], u[i]) : u[i];
            up += t;
            wave_lds_sync();
            if (uni_b(t2 <= t1)) {  // the candidate joins
                if (k == WK) return 0;
                if (gl < 16) pol[k * 16 + gl] = cand[gl];
                const double rz = rsqrt(zn);
#pragma unroll
                for (int i = 0; i < WK; i++) {
                    u[i] = i == k ? up : u[i];
                    dl[i] = i == k ? rz : dl[i];
#pragma unroll
                    for (int j = i; j < WK; j++)
                        if (j == k) L[S6::idx(i, j)] = i < k ? sp * v[i] : (i == k ? zn * rz : L[S6::idx(i, j)]);
                }
                k++;
                wave_lds_sync();
                break;
            }
            // side l leaves: the rows above it move down; K refactored
#pragma unroll
            for (int i = 0; i < WK - 1; i++)
                if (i >= l && i < k - 1 && gl < 16) pol[i * 16 + gl] = pol[(i + 1) * 16 + gl];
#pragma unroll
            for (int i = 0; i < WK; i++) u[i] = i >= l ? (i + 1 < WK ? u[i + 1] : 0.0) : u[i];
            k--;
            wave_lds_sync();
            sep_gram<WK>(pol, k, L);
            if (!uni_b(chol_packed<WK>(L, dl))) return 0;
        }
    }
    // converged: the iterate's dual residual P y + q + G_A^T lam must meet the tolerance (else the
    // 16-lane pipeline re-solves the active set's equality QP: deferred)
    WST(9);
    {
        bool nf = false;
#pragma unroll
        for (int j = 0; j < SEP_NZ; j++) nf = nf || !isfinite(y[j]);
        if (__ballot(nf) != 0ull) return 0;
    }
    // P's blocks loaded here, where they are used (not live across the steps), and the active rows
    // read without a branch per row (as sep_dual_as)
    double pb[SEP_NZ][2];
#pragma unroll
    for (int o = 0; o < SEP_NZ; o++) {
        pb[o][0] = P[o * 6 + 2 * (o / 2)];
        pb[o][1] = P[o * 6 + 2 * (o / 2) + 1];
    }
    double rd = 0.0, qn = 0.0;
    if (k == 0) {
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
        double g[WK][SEP_NZ + 1];
#pragma unroll
        for (int i = 0; i < WK; i++) {
            const double* ri = pol + (i < k ? i : 0) * 16;  // (rows past k: row 0, weight 0)
#pragma unroll
            for (int o = 0; o < SEP_NZ; o++) g[i][o] = ri[o];
            g[i][SEP_NZ] = ri[POL_SGN];
        }
#pragma unroll
        for (int i = 0; i < WK; i++) {
            const double li = i < k ? g[i][SEP_NZ] * u[i] : 0.0;
#pragma unroll
            for (int o = 0; o < SEP_NZ; o++) r[o] = fma(li, g[i][o], r[o]);
        }
#pragma unroll
        for (int o = 0; o < SEP_NZ; o++) {
            rd = fmax(rd, fabs(r[o]));
            qn = fmax(qn, fabs(q[o]));
        }
    }
    rd *= rcp(1.0 + qn);
    if (!uni_b(rd <= tol)) return 0;
    WST(10);
#pragma unroll
    for (int j = 0; j < SEP_NZ; j++) yo[j] = y[j];
    rp_out = fmax(m, 0.0);
    rd_out = rd;
    if (save != nullptr) {
        if (gl < k) save[gl] = pol[gl * 16 + POL_ID];
        if (gl == 0) save[POL_K] = (double)k;
    }
    wave_lds_sync();
    WST(11);
    return 1;
}

// ---- per-wave LDS ---------------------------------------------------------------------------
struct WideLds {
    double nbx[4][NB_MAX];              // the neighbours' (px, py, vx, vy), in agent-index order
    int32_t nbi[NB_MAX];                // their agent indices
    double kd[NB_MAX], kx[4][NB_MAX];   // k-nearest merge scratch
    int32_t kj[NB_MAX];
    double pol[(POL_K + 1) * 16];       // active rows + candidate (wide_dual_as)
    double stage[W_CBF * W_ROW];        // this iteration's kept CBF rows, compacted
    double smp[MAX_CBF_H * 9];          // per CBF sample k: ego state (6) | U_k s0 (3)
    double act[POL_K + 1];              // iteration 0's final active set: side ids | count
    double noise[8];                    // the next state's noise draws (early_noise)
};

// ---- neighbour query on the wave (grid mode) -------------------------------------------------
// The spatial hash of impc.hpp (GridArgs) in ONE dependent round trip after the agent's state:
// lane t < 63 takes slot t % 7 of cell t / 7 of the 3 x 3 cells around the agent and loads, at
// addresses that depend on the position alone, the cell's bucket count, the slot's row and the
// row's (px, py, vx, vy) from the table's slot-state plane (GridArgs::sst, GRID_SST = 7 slots) —
// wn_issue, staged by the caller between the setup's loads; wn_finish keeps the k nearest (planar
// distance, ties by agent index: the 16-lane query's order) and leaves them in L.nbx / L.nbi sorted
// by agent index. A bucket with more than 7 rows: its further slots (row, then state) in chunks of
// 64 merged into the running set; a bucket past its capacity: the whole state table (same result).
struct WideQuery {
    uint32_t h, n;   // this lane's cell's bucket and count
    int j;           // this lane's slot row
    double st[4];    // its (px, py, vx, vy)
};

__device__ __forceinline__ void wn_issue(const ImpcArgs& args, double px, double py, int gl, WideQuery& q) {
    const GridArgs& gr = args.grid;
    const long long cx = (long long)floor(px * gr.inv_cell), cy = (long long)floor(py * gr.inv_cell);
    const int t = gl < 9 * GRID_SST ? gl : 0;
    const int c = t / GRID_SST, js = t - c * GRID_SST;
    q.h = cell_hash(cx + (c % 3) - 1, cy + (c / 3) - 1, gr.mask);
    q.n = gr.cnt[q.h];
    q.j = (int)gr.slots[grid_slot_at(q.h, (uint32_t)js)];
    const double4 v = reinterpret_cast<const double4*>(gr.sst)[grid_sst_at(q.h, (uint32_t)js)];
    q.st[0] = v.x;
    q.st[1] = v.y;
    q.st[2] = v.z;
    q.st[3] = v.w;
}

// the cells as uniform values: bucket, count (0 for a repeated bucket) and first index among the
// rows past the 7 inline slots; total such rows; full = some bucket past its capacity
struct WideCells {
    uint32_t hs[9], nc[9], off[9], total;
    bool full;
};

__device__ __forceinline__ void wn_cells(const ImpcArgs& args, const WideQuery& q, WideCells& c) {
    uint32_t tot = 0;
    bool full = false;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        c.hs[k] = (uint32_t)__builtin_amdgcn_readlane((int)q.h, k * GRID_SST);
        uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)q.n, k * GRID_SST);
        full = full || n > (uint32_t)GRID_CAP;
        bool dup = false;
#pragma unroll
        for (int p = 0; p < k; p++) dup = dup || c.hs[p] == c.hs[k];
        n = dup ? 0u : n;
        c.nc[k] = n;
        c.off[k] = tot;
        tot += n > (uint32_t)GRID_SST ? n - GRID_SST : 0u;
    }
    c.full = full;
    c.total = full ? (uint32_t)args.num_states : tot;
}

// row index of candidate t among the rows past the inline slots (-1: none)
__device__ __forceinline__ int wn_more(const GridArgs& gr, const WideCells& c, uint32_t t) {
    if (t >= c.total) return -1;
    if (c.full) return (int)t;
    uint32_t e = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        const uint32_t u = t - c.off[k];
        const uint32_t extra = c.nc[k] > (uint32_t)GRID_SST ? c.nc[k] - GRID_SST : 0u;
        e = ((c.off[k] <= t) & (u < extra)) ? grid_slot_at(c.hs[k], u + GRID_SST) : e;
    }
    return (int)gr.slots[e];
}

__device__ __forceinline__ bool wn_before(double da, int ja, double db, int jb) {
    return da < db || (da == db && ja < jb);
}

__device__ __forceinline__ int wn_finish(const ImpcArgs& args, int self, double px, double py, const WideCells& c,
                                         const WideQuery& q, WideLds& L, int gl) {
    const GridArgs& gr = args.grid;
    const double r2 = gr.radius * gr.radius;
    const int kk = gr.k < NB_MAX ? gr.k : NB_MAX;
    // the running set: lane l < nk holds the l-th nearest so far
    double kd = 1e300, kx0 = 0.0, kx1 = 0.0, kx2 = 0.0, kx3 = 0.0;
    int kj = 0x7fffffff, nk = 0;
    // chunk 0: the inline slots (lane t: slot t % 7 of cell t / 7); then the rows past them
    for (int ch = 0;; ch++) {
        const uint32_t t0 = ch == 0 ? 0u : (uint32_t)(ch - 1) * 64u;
        if (ch > 0 && t0 >= c.total) break;
        int j;
        double st[4];
        bool valid;
        if (ch == 0) {
            const int cc = gl / GRID_SST, js = gl - cc * GRID_SST;
            uint32_t ncell = 0;
#pragma unroll
            for (int k = 0; k < 9; k++) ncell = cc == k ? c.nc[k] : ncell;
            valid = !c.full && gl < 9 * GRID_SST && (uint32_t)js < ncell;
            j = q.j;
#pragma unroll
            for (int i = 0; i < 4; i++) st[i] = q.st[i];
        } else {
            j = wn_more(gr, c, t0 + (uint32_t)gl);
            valid = j >= 0;
            const size_t r = (size_t)(j >= 0 ? j : 0) * 6;
            st[0] = args.states[r];
            st[1] = args.states[r + 1];
            st[2] = args.states[r + 3];
            st[3] = args.states[r + 4];
        }
        const double ex = st[0] - px, ey = st[1] - py;
        const double d2 = ex * ex + ey * ey;
        const bool keep = valid && j != self && d2 <= r2;
        const unsigned long long msk = __ballot(keep);
        if (msk == 0ull) continue;
        const double dn = keep ? d2 : 1e300;
        const int jn = keep ? j : 0x7fffffff;
        // ranks in (running set) U (this chunk's kept candidates); the running set is sorted
        int r_new = 0, r_old = gl;
        for (unsigned long long mm = msk; mm != 0ull; mm &= mm - 1ull) {
            const int m = __builtin_ctzll(mm);
            const double dm = lane_of(dn, m);
            const int jm = __builtin_amdgcn_readlane(jn, m);
            r_new += wn_before(dm, jm, dn, jn) ? 1 : 0;
            r_old += wn_before(dm, jm, kd, kj) ? 1 : 0;
        }
        for (int l = 0; l < nk; l++) {
            const double dl = lane_of(kd, l);
            const int jl = __builtin_amdgcn_readlane(kj, l);
            r_new += wn_before(dl, jl, dn, jn) ? 1 : 0;
        }
        wave_lds_sync();
        if (gl < nk && r_old < kk) {
            L.kd[r_old] = kd;
            L.kj[r_old] = kj;
            L.kx[0][r_old] = kx0;
            L.kx[1][r_old] = kx1;
            L.kx[2][r_old] = kx2;
            L.kx[3][r_old] = kx3;
        }
        if (keep && r_new < kk) {
            L.kd[r_new] = dn;
            L.kj[r_new] = jn;
            L.kx[0][r_new] = st[0];
            L.kx[1][r_new] = st[1];
            L.kx[2][r_new] = st[2];
            L.kx[3][r_new] = st[3];
        }
        nk += __popcll(msk);
        nk = nk < kk ? nk : kk;
        wave_lds_sync();
        if (gl < nk) {
            kd = L.kd[gl];
            kj = L.kj[gl];
            kx0 = L.kx[0][gl];
            kx1 = L.kx[1][gl];
            kx2 = L.kx[2][gl];
            kx3 = L.kx[3][gl];
        }
    }
    // the kept set ordered by agent index
    int pos = 0;
    for (int l = 0; l < nk; l++) pos += __builtin_amdgcn_readlane(kj, l) < kj ? 1 : 0;
    wave_lds_sync();
    if (gl < nk) {
        L.nbi[pos] = kj;
        L.nbx[0][pos] = kx0;
        L.nbx[1][pos] = kx1;
        L.nbx[2][pos] = kx2;
        L.nbx[3][pos] = kx3;
    }
    wave_lds_sync();
    return nk;
}

// U_k s0 (the state's part of the acceleration at CBF sample k; stage_cbf_rows' us), one component
// per lane into the per-sample table: the same for both IMPC iterations, formed once at setup
__device__ __forceinline__ void wide_sample_us(const DevOps& op, const double* __restrict__ buf, const double (&s0)[6],
                                               WideLds& L, int gl) {
    for (int t = gl; t < 3 * op.cbf_h; t += 64) {
        const int k = t / 3, d = t - 3 * k;
        const double* USk = opp(buf, op.o_US) + (size_t)k * 18 + d * 6;
        double us[6], v = 0.0;
#pragma unroll
        for (int s = 0; s < 6; s++) us[s] = USk[s];
#pragma unroll
        for (int s = 0; s < 6; s++) v = fma(us[s], s0[s], v);
        L.smp[k * 9 + 6 + d] = v;
    }
}

// The CBF rows of IMPC iteration `it` (stage_cbf_rows on the wave: one (sample, neighbour) row per
// lane, filtered and compacted into L.stage in (sample, neighbour) order). Returns the row count
// (wave-uniform); row_infeasible: a row no acceleration in the box satisfies.
__device__ int wide_cbf_rows(const DevOps& op, const double* __restrict__ buf, const ImpcArgs& args, int it,
                             const double (&s0)[6], const double (&y)[SEP_NZ], bool grid_mode, WideLds& L,
                             int nb0, int nnb, int gl, bool& row_infeasible, long long* wdbg = nullptr) {
    (void)wdbg;
    constexpr int NZ = SEP_NZ;
    WST(0);
    const int nk = (it == 0) ? 1 : op.cbf_h;
    // iteration 1: the ego state at sample k (the previous curve at h_samples(k), :161-168;
    // cbf_ego_state), one component per lane into the per-sample table (U_k s0 is there since the
    // setup, wide_sample_us); iteration 0: the state itself, from registers
    if (it > 0) {
        for (int t = gl; t < 6 * nk; t += 64) {
            const int k = t / 6, s = t - 6 * k;
            const double* PZ = opp(buf, op.o_PZ) + (size_t)k * 6 * NZ + s * NZ;
            const double* PS = opp(buf, op.o_PS) + (size_t)k * 36 + s * 6;
            double ps[6], pz[NZ], v = 0.0;
#pragma unroll
            for (int u = 0; u < 6; u++) ps[u] = PS[u];
#pragma unroll
            for (int j = 0; j < NZ; j++) pz[j] = PZ[j];
#pragma unroll
            for (int u = 0; u < 6; u++) v = fma(ps[u], s0[u], v);
#pragma unroll
            for (int j = 0; j < NZ; j++) v = fma(pz[j], y[j], v);
            L.smp[k * 9 + s] = v;
        }
    }
    wave_lds_sync();
    WST(1);
    const double* UZ = opp(buf, op.o_UZ);
    const int ntot = nnb * nk;
    int count = 0;
    bool rinf = false;
    for (int base = 0; base < ntot; base += 64) {
        const int t = base + gl;
        bool keep = false;
        double cg[4] = {0.0, 0.0, 0.0, 0.0}, chi = 0.0;
        if (t < ntot) {
            const int k = t / nnb, j = t - k * nnb;
            const double* UZk = UZ + (size_t)k * 3 * NZ;
            double uz[12];
#pragma unroll
            for (int d = 0; d < 3; d++)
#pragma unroll
                for (int jz = 0; jz < 4; jz++) uz[d * 4 + jz] = UZk[d * NZ + jz];
            double npx, npy, nvx, nvy;
            if (grid_mode) {
                npx = L.nbx[0][j];
                npy = L.nbx[1][j];
                nvx = L.nbx[2][j];
                nvy = L.nbx[3][j];
            } else {
                const double* ns = args.states + (size_t)args.nb_col[nb0 + j] * 6;
                npx = ns[0];
                npy = ns[1];
                nvx = ns[3];
                nvy = ns[4];
                // (keeps the two reads apart: merged after the branch they became one flat load)
                asm volatile("" : "+v"(npx), "+v"(npy), "+v"(nvx), "+v"(nvy));
            }
            double e[6];
#pragma unroll
            for (int s = 0; s < 6; s++) e[s] = it == 0 ? s0[s] : L.smp[k * 9 + s];
            double a[3], b;
            safety_cbf(e, npx, npy, nvx, nvy, op.d_min, a, b);
            double bmax = 0.0, bmin = 0.0;
#pragma unroll
            for (int d = 0; d < 3; d++) {
                const double v1 = -a[d] * op.a_lo[d], v2 = -a[d] * op.a_hi[d];
                bmax += fmax(v1, v2);
                bmin += fmin(v1, v2);
            }
            keep = !(op.cbf_filter && b >= bmax);
            if (b < bmin - op.feas_tol) rinf = true;
#pragma unroll
            for (int jz = 0; jz < 4; jz++) cg[jz] = -(a[0] * uz[jz] + a[1] * uz[4 + jz] + a[2] * uz[8 + jz]);
            chi = b + (a[0] * L.smp[k * 9 + 6] + a[1] * L.smp[k * 9 + 7] + a[2] * L.smp[k * 9 + 8]);
        }
        if (base == 0) WST(2);
        const unsigned long long msk = __ballot(keep);
        const int slot = count + __popcll(msk & ((1ull << gl) - 1ull));
        if (keep && slot < W_CBF) {
            double* dst = L.stage + slot * W_ROW;
#pragma unroll
            for (int jz = 0; jz < 4; jz++) dst[jz] = cg[jz];
            dst[4] = chi;
        }
        count += __popcll(msk);
    }
    row_infeasible = __ballot(rinf) != 0ull;
    wave_lds_sync();
    WST(3);
    return count;
}

}  // namespace dev

}  // namespace mpccbf
