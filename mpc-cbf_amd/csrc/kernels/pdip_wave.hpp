// pdip_wave.hpp — one QP per wavefront: the Mehrotra PDIP of pdip.hpp for reduced dimensions up
// to 16 and up to 192 rows, with the Newton matrix assembled on the matrix cores.
//
// Used by the FoV controller (nz = 15: 5 per channel over 4 Bezier pieces, rows coupling all
// channels), where a per-lane packed normal matrix (120 entries) would not fit the registers.
//
// Layouts (64 lanes, lane = 16 q + p):
//   rows    row r lives in slot s = r / 64 of lane 16 (r % 4) + (r / 4) % 16 ("owner"); the owner
//           keeps the row's bounds, slacks and duals in registers and reads its 16 coefficients
//           from the wave's LDS row image (G, 16 doubles per row, padded column 15 = 0).
//   vectors of the reduced dimension (iterate, directions, right-hand sides) live on the row
//           layout: lane i (of every 16-lane row) holds element i — one register per vector.
//           Where a row needs a whole vector (row activities g.y) it is published to LDS and
//           read back as a wave-uniform broadcast.
//   G^T v   lane (q, p) accumulates G[4c + q][p] v[4c + q] over the chunks c, then two
//           permlane swaps sum the four q-groups: the product arrives on the row layout.
//   Gram    chunk c (rows 4c .. 4c+3) feeds one v_mfma_f64_16x16x4f64 with A = G_chunk^T
//           (lane: G[4c + q][p]) and B = diag(D) G_chunk (lane: D_{4c+q} G[4c + q][p]); column
//           15 of B carries the right-hand side weights instead (G[.][15] = 0), so one MFMA chain
//           yields M = G^T D G and G^T w. Per-row weights reach the chunk lanes through LDS.
//   rows-of-M  the 16x16 result is transposed through LDS so that lane i holds row i of M;
//           Cholesky (left-looking, DPP broadcasts of row j) and both triangular solves run on
//           that layout (L's columns for the backward solve are read from LDS).
// Phase 1 (feasibility) reuses the machinery with the padded variable as the violation t.
#pragma once

#include "group.hpp"
#include "pdip.hpp"

namespace mpccbf {
namespace dev {

constexpr int WNZ = 16;   // padded reduced dimension
constexpr int WR = 3;     // row slots per lane
constexpr int WROWS = 64 * WR;
constexpr int WCH = WROWS / 4;  // MFMA chunks

typedef double wd4 __attribute__((ext_vector_type(4)));

// lane of row r / row of (lane, slot)
__host__ __device__ constexpr int wave_row_owner(int r) { return 16 * (r & 3) + ((r >> 2) & 15); }
__host__ __device__ constexpr int wave_owner_row(int lane, int slot) { return 64 * slot + 4 * (lane & 15) + (lane >> 4); }

// ---- 64-lane collectives -------------------------------------------------------------------
// ---- 64-lane collectives -------------------------------------------------------------------
template <int SRC>
__device__ __forceinline__ double bcast16(double v) {  // row_newbcast:SRC (inside each 16-lane row)
    return __longlong_as_double(__builtin_amdgcn_mov_dpp(__double_as_longlong(v), 0x150 + SRC, 0xF, 0xF, true));
}

// bcast16 with a source index known only after loop unrolling (folds to one DPP move)
__device__ __forceinline__ double bcast16v(int src, double v) {
    switch (src & 15) {
        case 0: return bcast16<0>(v);
        case 1: return bcast16<1>(v);
        case 2: return bcast16<2>(v);
        case 3: return bcast16<3>(v);
        case 4: return bcast16<4>(v);
        case 5: return bcast16<5>(v);
        case 6: return bcast16<6>(v);
        case 7: return bcast16<7>(v);
        case 8: return bcast16<8>(v);
        case 9: return bcast16<9>(v);
        case 10: return bcast16<10>(v);
        case 11: return bcast16<11>(v);
        case 12: return bcast16<12>(v);
        case 13: return bcast16<13>(v);
        case 14: return bcast16<14>(v);
        default: return bcast16<15>(v);
    }
}

// value of lane l ^ 16 and of lane l ^ 32 combined with the own value (v_permlane*_swap)
template <Op OP>
__device__ __forceinline__ double xrow16(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)(b & 0xffffffffll), hi = (unsigned)(b >> 32);
    auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto c = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const double x0 = __longlong_as_double(((long long)c[0] << 32) | a[0]);
    const double x1 = __longlong_as_double(((long long)c[1] << 32) | a[1]);
    return combine<OP>(x0, x1);
}
template <Op OP>
__device__ __forceinline__ double xrow32(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)(b & 0xffffffffll), hi = (unsigned)(b >> 32);
    auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto c = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const double x0 = __longlong_as_double(((long long)c[0] << 32) | a[0]);
    const double x1 = __longlong_as_double(((long long)c[1] << 32) | a[1]);
    return combine<OP>(x0, x1);
}

template <Op OP>
__device__ __forceinline__ double wave_reduce(double v) {
    v = grp_reduce<16, OP>(v);
    v = xrow16<OP>(v);
    return xrow32<OP>(v);
}


// two independent all-reductions, stage-interleaved
template <Op OA, Op OB>
__device__ __forceinline__ void wave_reduce2(double& a, double& b) {
    a = combine<OA>(a, dpp_mov<DPP_XOR1>(a));
    b = combine<OB>(b, dpp_mov<DPP_XOR1>(b));
    a = combine<OA>(a, dpp_mov<DPP_XOR2>(a));
    b = combine<OB>(b, dpp_mov<DPP_XOR2>(b));
    a = combine<OA>(a, dpp_mov<DPP_HALF_MIRROR>(a));
    b = combine<OB>(b, dpp_mov<DPP_HALF_MIRROR>(b));
    a = combine<OA>(a, dpp_mov<DPP_MIRROR>(a));
    b = combine<OB>(b, dpp_mov<DPP_MIRROR>(b));
    a = xrow16<OA>(a);
    b = xrow16<OB>(b);
    a = xrow32<OA>(a);
    b = xrow32<OB>(b);
}

// ---- LDS workspace -------------------------------------------------------------------------
struct WaveScratch {      // per-wave LDS besides the row image
    double M[WNZ * WNZ];  // Gram transpose, then L (row-major) for the backward solves
    double Dv[WROWS];     // per-row Newton weight
    double wv[WROWS];     // per-row right-hand side weight (Gram column 15)
    double cv[WROWS];     // per-row weights of a G^T v product
    double y[WNZ];        // iterate, wave-uniform copy (caller: result of pdip_solve_wave)
    double d[WNZ];        // current direction, wave-uniform copy
    double q[WNZ];        // linear term (caller fills; q[15] = 0)
};

// Row storage of one lane (owner layout). Every row has an upper side; ml = 1 adds the lower.
// Unused slots hold inert rows (g = 0, -1 <= 0 <= 1). g[s] points at the slot's row in the LDS
// image (an all-zero row for unused slots).
struct WaveRows {
    const double* g[WR];
    double lo[WR], hi[WR], ml[WR];
};

#ifndef MPCCBF_SLK_RD  // slack mode: accepted dual-residual floor at primal convergence
#define MPCCBF_SLK_RD 1e-6
#endif
#ifndef MPCCBF_SLK_INIT  // slack start: 1 = balanced (v = sb = 1/zb), 0 = v = sb = 1
#define MPCCBF_SLK_INIT 1
#endif
// ---- slack mode (FovBezierIMPCCBF slack_mode, FovMPCCBFQPGenerator.cpp:110-207) --------------
// Neighbour i (< 8) owns a slack variable v_i >= 0 with linear cost w_i that relaxes all of its
// FoV rows  g_a^T y - v_i <= h_a  (up to 8: 4 kinds x cbf_horizon <= 2). Lane l holds row a = l & 7
// of neighbour i = l >> 3 (inert when filtered: g = 0, 0 <= 1), so per-neighbour sums are 8-lane
// DPP reductions and v_i, its bound slack sb_i and dual zb_i are replicated in the 8 lanes.
// v_i is eliminated from the Newton system per neighbour. With D_a = z_a / s_a, T = sum D_a,
// S = T + zb/sb and the D-weighted mean row gbar = sum D_a g_a / T, the Schur complement is
//   sum_a D_a g_a g_a^T - (sum_a D_a g_a)(..)^T / S = sum_a D_a (g_a - gbar)(g_a - gbar)^T
//                                                   + (T zb / (sb S)) gbar gbar^T,
// a sum of positive terms: no cancellation when a row is nearly active (D ~ 1e20) while its slack
// is in use (the textbook downdate would subtract two 1e20-sized terms). The same split applies
// to every right-hand side: sum_a g_a phi_a + u c / S = sum_a (g_a - gbar) phi_a
// + gbar (Db sum phi_a + T c) / S. So the matrix cores see the centred rows and one mean row per
// neighbour as ordinary weighted rows of a second image (Gc).
constexpr int WSL_NB = 8;                 // neighbours with a slack variable (one 8-lane segment each)
constexpr int WSL_ROWS = 8 * WSL_NB;      // slack rows (lane = row)
constexpr int WSL_CROWS = 80;             // centred rows + mean rows, padded to 16

struct WaveSlack {
    const double* Go;  // WSL_ROWS x 16 original slack rows (LDS; rows >= 8 nnb zero up to the 16-row pad)
    // The centred rows (8 i + a) and mean rows (8 nnb + i) sit in the main row image right after
    // the ordinary rows, at image row coff (a multiple of 16), so one MFMA Gram chain and one
    // G^T v cover both; Dvs / wvs / cvs alias the WaveScratch weight arrays at coff.
    int coff;
    double* Gc;
    double* Dvs;
    double* wvs;
    double* cvs;
    double* zvs;       // z of the Go rows (dual residual)
    double* Tn;        // per neighbour: sum of the live rows' D
    int nnb;           // neighbours (<= WSL_NB)
    int nchunk_c;      // chunks of Gc in use (multiple of 4)
    int nchunk_o;      // chunks of Go in use (multiple of 4)
    double h, live;    // this lane's row: bound, 1 if live (0: inert)
    double w;          // slack cost of this lane's neighbour
    double* st;        // WSL_NST x 64 per-lane solver state in LDS (keeps the registers for the
                       // Newton matrix, factor and solves; the slack state is touched a few times
                       // per step)
};
constexpr int WSL_NST = 24;

// sum over the 8-lane segment (row_half_mirror pairs the two quads of each half-row)
__device__ __forceinline__ double seg8_sum(double v) {
    v += dpp_mov<DPP_XOR1>(v);
    v += dpp_mov<DPP_XOR2>(v);
    return v + dpp_mov<DPP_HALF_MIRROR>(v);
}

// Rebuild the centred image from the current weights: lane (q, p) handles column p of
// neighbours q and q + 4.
__device__ __forceinline__ void wave_slack_center(const WaveSlack& sk, int lane) {
    const int q = lane >> 4, p = lane & 15;
#pragma unroll
    for (int u = 0; u < WSL_NB / 4; u++) {
        const int i = q + 4 * u;
        if (i < sk.nnb) {
            double g[8], acc = 0.0;
#pragma unroll
            for (int a = 0; a < 8; a++) {
                g[a] = sk.Go[(8 * i + a) * WNZ + p];
                acc = fma(sk.Dvs[8 * i + a], g[a], acc);
            }
            const double T = sk.Tn[i];
            const double gb = T > 0.0 ? acc * rcp(T) : 0.0;
#pragma unroll
            for (int a = 0; a < 8; a++) sk.Gc[(8 * i + a) * WNZ + p] = g[a] - gb;
            sk.Gc[(8 * sk.nnb + i) * WNZ + p] = gb;
        }
    }
    wave_lds_sync();
}

// a . b over 16 entries, both in LDS (b wave-uniform: broadcast reads)
__device__ __forceinline__ double dotl(const double* a, const double* b) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < WNZ; j += 2) {
        s0 = fma(a[j], b[j], s0);
        s1 = fma(a[j + 1], b[j + 1], s1);
    }
    return s0 + s1;
}

__device__ __forceinline__ double dotr(const double (&a)[WNZ], const double* b) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < WNZ; j += 2) {
        s0 = fma(a[j], b[j], s0);
        s1 = fma(a[j + 1], b[j + 1], s1);
    }
    return s0 + s1;
}

// (G^T v)_i on the row layout; v: one weight per image row (LDS). nchunk is a multiple of 4
// (the caller zeroes the image rows that complete the last group of chunks). Fully unrolled
// over the 12 groups with wave-uniform guards: a runtime loop would carry the accumulators
// through copies.
__device__ __forceinline__ double wave_gt(const double* __restrict__ Gs, const double* __restrict__ v,
                                          int nchunk, int lane) {
    const int q = lane >> 4, p = lane & 15;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < WCH; c += 4) {
        if (c < nchunk) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int r = 4 * (c + u) + q;
                a[u] = fma(Gs[r * WNZ + p], v[r], a[u]);
            }
        }
    }
    return xrow32<Op::Sum>(xrow16<Op::Sum>((a[0] + a[1]) + (a[2] + a[3])));
}

// acc = G^T diag(D) G with column 15 replaced by G^T w. nchunk: a multiple of 4.
__device__ __forceinline__ wd4 wave_gram(const double* __restrict__ Gs, const double* __restrict__ Dv,
                                         const double* __restrict__ wv, int nchunk, int lane) {
    const int q = lane >> 4, p = lane & 15;
    const double rhs_col = (p == WNZ - 1) ? 1.0 : 0.0;  // G[.][15] = 0: column 15 takes w only
    wd4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; u++) acc[u] = wd4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < WCH; c += 4) {
        if (c < nchunk) {
            double g[4], b[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int r = 4 * (c + u) + q;
                g[u] = Gs[r * WNZ + p];
                b[u] = fma(rhs_col, wv[r], Dv[r] * g[u]);  // branch-free
            }
#pragma unroll
            for (int u = 0; u < 4; u++) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(g[u], b[u], acc[u], 0, 0, 0);
        }
    }
    return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// Transpose the MFMA result (lane (q, p): M[q + 4i][p]) into rows: lane -> row (lane & 15).
__device__ __forceinline__ void gram_rows(const wd4 acc, double* __restrict__ Mbuf, int lane,
                                          double (&row)[WNZ]) {
    const int q = lane >> 4, p = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; i++) Mbuf[(q + 4 * i) * WNZ + p] = acc[i];
    wave_lds_sync();
    const int r = lane & 15;
#pragma unroll
    for (int k = 0; k < WNZ; k++) row[k] = Mbuf[r * WNZ + k];
    wave_lds_sync();
}

// lane & 15 as a value the compiler cannot see through: the lane masks derived from it (i == k
// for every k) are then formed inside each solve instead of hoisted out of the caller's loops,
// where 16 of them stay live across everything and spill
__device__ __forceinline__ int lane16_opaque(int lane) {
    int i;
    asm volatile("v_and_b32 %0, 15, %1" : "=v"(i) : "v"(lane));
    return i;
}

// Left-looking Cholesky on the row layout: lane i holds row i of M (k <= i used) and gets row i
// of L and inv_i = 1 / L_ii; L's rows are then stored to Mbuf (row-major) for the backward
// solves. Returns false if a pivot is not positive.
__device__ __forceinline__ bool chol_rows(const double (&M)[WNZ], double (&L)[WNZ], double& inv_i,
                                          double* __restrict__ Mbuf, int lane) {
    const int i = lane16_opaque(lane);
    bool ok = true;
    inv_i = 0.0;
#pragma unroll
    for (int j = 0; j < WNZ; j++) {
        double part[4] = {M[j], 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < j; k++) part[k & 3] = fma(-L[k], bcast16v(j, L[k]), part[k & 3]);
        const double v = (part[0] + part[1]) + (part[2] + part[3]);
        const double d = bcast16v(j, v);
        ok = ok && (d > 0.0);
        const double r = rsqrt(d > 0.0 ? d : 1e-300);
        inv_i = (i == j) ? r : inv_i;
        L[j] = (i >= j) ? v * r : 0.0;
    }
    if (lane < WNZ) {
#pragma unroll
        for (int k = 0; k < WNZ; k++) Mbuf[i * WNZ + k] = L[k];
    }
    wave_lds_sync();
    return ok;
}

// Solve L L^T x = b on the row layout (lane i: b_i in, x_i out). L: row i of L (registers),
// Lm: L row-major (LDS, or global for the start factor), inv_i = 1 / L_ii.
__device__ __forceinline__ double solve_rows(const double (&L)[WNZ], const double* __restrict__ Lm,
                                             double inv_i, double b, int i) {
    double res = b, wl = 0.0;
#pragma unroll
    for (int k = 0; k < WNZ; k++) {
        const double wk = bcast16v(k, res * inv_i);
        res = fma(-L[k], wk, res);
        wl = (i == k) ? wk : wl;
    }
    res = wl;
    double xl = 0.0;
#pragma unroll
    for (int k = WNZ - 1; k >= 0; k--) {
        const double xk = bcast16v(k, res * inv_i);
        res = fma(-Lm[k * WNZ + i], xk, res);
        xl = (i == k) ? xk : xl;
    }
    return xl;
}

// a load the compiler may not hoist out of the enclosing loop (keeps a loop-invariant row out of
// the registers: the "memory" clobber orders it after every earlier store)
__device__ __forceinline__ double ldg_nohoist(const double* p) {
    asm volatile("" ::: "memory");
    return *p;
}

// publish a row-layout vector as a wave-uniform LDS copy
__device__ __forceinline__ void publish16(double* __restrict__ dst, double v, int lane) {
    if (lane < WNZ) dst[lane] = v;
    wave_lds_sync();
}

// Main solve. P, LP: 16x16 row-major, padded with the identity (uniform, global). sc.q: linear
// term; on return sc.y holds the iterate. nchunk: row chunks in use.
// SLK: slack mode — skp holds the slack rows (see WaveSlack); v_obj gets sum_i w_i v_i.
template <bool SLK = false>
__device__ __forceinline__ PdipOut pdip_solve_wave(const WaveRows& rw, const double* __restrict__ Gs, int nchunk,
                                   WaveScratch& sc, const double* __restrict__ P,
                                   const double* __restrict__ LP, const PdipCfg cfg, int lane,
                                   long long* dbg = nullptr, const WaveSlack* skp = nullptr,
                                   double* v_obj = nullptr) {
    (void)dbg;
    (void)skp;
    (void)v_obj;
    const int i = lane16_opaque(lane);
    const double qi = sc.q[i];
    double L[WNZ], inv_i;
    // ---- start: y0 = -P^{-1} q with the factor of P
    {
#pragma unroll
        for (int k = 0; k < WNZ; k++) L[k] = (k <= i) ? LP[i * WNZ + k] : 0.0;
        inv_i = rcp(LP[i * WNZ + i]);
    }
    double yi = solve_rows(L, LP, inv_i, -qi, i);
    publish16(sc.y, yi, lane);
    double sl[WR], su[WR], zl[WR], zu[WR], pl[WR], pu[WR];
    double nloc = 0.0;
#pragma unroll
    for (int s = 0; s < WR; s++) {
        const double t = dotl(rw.g[s], sc.y);
        sl[s] = rw.ml[s] > 0.0 ? fmax(t - rw.lo[s], 1.0) : 1.0;
        su[s] = fmax(rw.hi[s] - t, 1.0);
        zl[s] = rw.ml[s] * rcp(sl[s]);
        zu[s] = rcp(su[s]);
        pl[s] = rw.ml[s] * rcp(1.0 + fabs(rw.lo[s]));
        pu[s] = rcp(1.0 + fabs(rw.hi[s]));
        nloc += rw.ml[s] + 1.0;
    }
    // slack rows: this lane holds row (lane & 7) of neighbour (lane >> 3); lanes of neighbours
    // >= nnb hold inert rows and no slack variable. Start: zb = max(w, 1) (the dual the bound
    // carries when no row is active), v = sb = 1 / zb (a centred pair: sb zb = 1 like the rows'
    // s z; with sb = 1 the pair sat 1e3 off the central path and some crowded QPs broke down
    // near the optimum), row slacks from the residual.
    const bool son = SLK && (lane >> 3) < (SLK ? skp->nnb : 0);
    const bool lead = son && (lane & 7) == 0;  // counts the neighbour's bound once in sums
    double lst_dummy[WSL_NST];  // (non-slack instantiation: never touched)
    double* const lst = SLK ? skp->st + lane : lst_dummy;
    constexpr int lsd = SLK ? 64 : 1;
    double &v = lst[0 * lsd], &sb = lst[1 * lsd], &zb = lst[2 * lsd], &cs = lst[3 * lsd],
           &cz = lst[4 * lsd], &pc = lst[5 * lsd], &slh = lst[6 * lsd], &sliv = lst[7 * lsd],
           &slw = lst[8 * lsd];
    if constexpr (SLK) {
        const WaveSlack& sk = *skp;
        slh = son ? sk.h : 1.0;
        sliv = son ? sk.live : 0.0;
        slw = son ? sk.w : 0.0;
        zb = fmax(slw, 1.0);
#if MPCCBF_SLK_INIT == 1
        sb = rcp(zb);  // balanced start: sb zb = 1
        v = sb;
#endif
        const double t = son ? dotl(sk.Go + lane * WNZ, sc.y) : 0.0;
        cs = fmax(slh - (t - sliv * v), 1.0);
        cz = rcp(cs);
        pc = rcp(1.0 + fabs(slh));
        nloc += lead ? 2.0 : 1.0;
    }
    const double inv_ns = rcp(wave_reduce<Op::Sum>(nloc));
    const double inv_qn = rcp(1.0 + grp_max<16>(fabs(qi)));
    // row i of P is re-read where it is used (L2-resident, 2 KB for the whole launch) instead of
    // held in 32 registers across the Newton loop
    const double* __restrict__ Prow = P + i * WNZ;

    PdipOut out{ST_UNKNOWN, 0};
    double mu0 = 1.0, rd_track = 1e300;
    bool rd_exact = true;
    for (int it = 0;; it++) {
        PSTAMP(0);
        double rl[WR], ru[WR], il[WR], iu[WR];
        double mloc = 0.0, rp = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double t = dotl(rw.g[s], sc.y);
            rl[s] = rw.ml[s] * (t - rw.lo[s] - sl[s]);
            ru[s] = rw.hi[s] - t - su[s];
            il[s] = rcp(sl[s]);
            iu[s] = rcp(su[s]);
            const double Dl = zl[s] * il[s], Du = zu[s] * iu[s];
            const int r = wave_owner_row(lane, s);
            if (!SLK || r < skp->coff) {  // (slack mode: rows past coff are the slack image's)
                sc.Dv[r] = Dl + Du;
                sc.wv[r] = Du * ru[s] - Dl * rl[s];
                sc.cv[r] = zu[s] - zl[s];
            }
            mloc = fma(sl[s], zl[s], fma(su[s], zu[s], mloc));
            rp = fmax(rp, fmax(fabs(rl[s]) * pl[s], fabs(ru[s]) * pu[s]));
        }
        // slack rows: residual cr = h - g y + v - s, D = z / s; per neighbour T = sum D (live),
        // S = T + Db; weights of the centred rows and of the mean row (predictor right-hand side
        // phi = D cr, v-equation term -(Db rb + w))
        double &scr = lst[9 * lsd], &sci = lst[10 * lsd], &sD = lst[11 * lsd], &sT = lst[12 * lsd],
               &siS = lst[13 * lsd], &sDb = lst[14 * lsd], &srb = lst[15 * lsd];
        if constexpr (SLK) {
            const WaveSlack& sk = *skp;
            const double t = son ? dotl(sk.Go + lane * WNZ, sc.y) : 0.0;
            scr = slh - t + sliv * v - cs;
            sci = rcp(cs);
            sD = cz * sci;
            const double Dl = sliv * sD;
            sT = seg8_sum(Dl);
            const double SR = seg8_sum(Dl * scr);
            sDb = zb * rcp(sb);
            srb = v - sb;
            siS = rcp(sT + sDb);
            mloc = fma(cs, cz, mloc);
            if (lead) mloc = fma(sb, zb, mloc);
            rp = fmax(rp, fabs(scr) * pc);
            if (son) {
                rp = fmax(rp, fabs(srb));
                sk.Dvs[lane] = Dl;
                sk.wvs[lane] = Dl * scr;
                sk.zvs[lane] = sliv * cz;
            }
            if (lead) {
                const int nb = lane >> 3;
                sk.Tn[nb] = sT;
                sk.Dvs[8 * sk.nnb + nb] = sT * sDb * siS;
                sk.wvs[8 * sk.nnb + nb] = (sDb * SR - sT * fma(sDb, srb, slw)) * siS;
            }
            wave_lds_sync();
            wave_slack_center(sk, lane);
        }
        PSTAMP(1);
        wave_lds_sync();
        const wd4 acc = wave_gram(Gs, sc.Dv, sc.wv, nchunk + (SLK ? skp->nchunk_c : 0), lane);
        double Mr[WNZ];
        gram_rows(acc, sc.M, lane, Mr);
        const double rhs_i = Mr[WNZ - 1];  // G^T w (column 15)
        PSTAMP(2);
#pragma unroll
        for (int k = 0; k < WNZ; k++) Mr[k] = (k == WNZ - 1 && i != WNZ - 1 ? 0.0 : Mr[k]) + ldg_nohoist(Prow + k);
        wave_reduce2<Op::Sum, Op::Max>(mloc, rp);
        const double mu = mloc * inv_ns;
        double py_i = qi;  // (P y + q)_i
#pragma unroll
        for (int k = 0; k < WNZ; k++) py_i = fma(ldg_nohoist(Prow + k), sc.y[k], py_i);
        // exact relative dual residual; slack mode adds the slack rows (original g, weights z) and
        // the v equations w - sum_a z_a - zb (relative to 1 + w)
        auto dual_res = [&]() {
            double gt = wave_gt(Gs, sc.cv, nchunk, lane);
            if constexpr (SLK) gt += wave_gt(skp->Go, skp->zvs, skp->nchunk_o, lane);
            double r = grp_max<16>(fabs(py_i + gt)) * inv_qn;
            if constexpr (SLK) {
                const double zs = seg8_sum(sliv * cz);
                const double rv = son ? fabs(slw - zs - zb) * rcp(1.0 + slw) : 0.0;
                r = fmax(r, wave_reduce<Op::Max>(rv));
            }
            return r;
        };
        bool rd_fresh = false;
        if (rd_exact) {
            rd_track = dual_res();
            rd_exact = false;
            rd_fresh = true;
        }
        out.iters = it;
        const bool finite = isfinite(rp) && isfinite(rd_track) && isfinite(mu) && isfinite(Mr[0]);
        if (finite && rp <= cfg.tol && mu <= cfg.tol * 0.1 && rd_track <= cfg.tol) {
            if (!rd_fresh)  // the tracked dual residual is a prediction: confirm it exactly
                rd_track = dual_res();
            // slack mode: the recovered slack-row duals carry the rounding of the per-neighbour
            // elimination (errors ~ eps D |dy| in dz of strongly active rows), which floors the
            // exact dual residual near 1e-8 .. 1e-7 once D ~ 1e13 while the primal iterate is
            // converged; with primal feasibility and complementarity at tolerance, a dual residual
            // below MPCCBF_SLK_RD is accepted
            if (rd_track <= cfg.tol || (SLK && rd_track <= MPCCBF_SLK_RD)) {
                out.status = ST_OPTIMAL;
                out.rp = rp;
                out.rd = rd_track;
                break;
            }
        }
        if (it == 0) mu0 = mu;
        if (it >= cfg.maxit || !finite || mu > 1e8 * fmax(mu0, 1.0)) {
            out.status = ST_UNKNOWN;
#ifdef MPCCBF_DEBUG_EXIT  // diagnostics build: exit reason in the iteration count
            out.iters = it + 1000 * (it >= cfg.maxit ? 1 : !finite ? 2 : 3);
#endif
            break;
        }
        PSTAMP(3);
        // ---- factor
        bool fok = chol_rows(Mr, L, inv_i, sc.M, lane);
#ifdef MPCCBF_DEBUG_TRACE
        const bool fok0 = fok;
#endif
        if constexpr (SLK) {
            if (!fok) {
                // a pivot lost to cancellation (active rows' D ~ 1e20 against P ~ 1e5, more
                // frequent with the slack rows' coupled pairs): refactor with a diagonal shift of
                // 1e-12 of the largest diagonal entry (inexact Newton step; residuals stay exact)
                double dg = 0.0;
#pragma unroll
                for (int k = 0; k < WNZ; k++) dg = (k == i) ? Mr[k] : dg;
                const double tau = 1e-12 * grp_max<16>(fabs(dg));
#pragma unroll
                for (int k = 0; k < WNZ; k++) Mr[k] += (k == i) ? tau : 0.0;
                fok = chol_rows(Mr, L, inv_i, sc.M, lane);
            }
        }
        if (!fok) {
            out.status = ST_UNKNOWN;
#ifdef MPCCBF_DEBUG_EXIT
            out.iters = it + 4000;
#endif
            break;
        }
        PSTAMP(4);
        // ---- predictor
        const double dya_i = solve_rows(L, sc.M, inv_i, rhs_i - py_i, i);
        publish16(sc.d, dya_i, lane);
        PSTAMP(5);
        double dsl[WR], dsu[WR], dzl[WR], dzu[WR];
        double rs = 0.0, rz = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double td = dotl(rw.g[s], sc.d);
            dsl[s] = rw.ml[s] * (td + rl[s]);
            dsu[s] = ru[s] - td;
            const double ql = dsl[s] * il[s], qu = dsu[s] * iu[s];
            dzl[s] = -zl[s] * (1.0 + ql);
            dzu[s] = -zu[s] * (1.0 + qu);
            rs = fmax(rs, fmax(-ql, -qu));
            rz = fmax(rz, fmax(rw.ml[s] * (1.0 + ql), 1.0 + qu));
        }
        // slack rows: dv = (sum_a D_a (g_a dy - cr_a) - Db rb - w) / S, ds = cr - g dy + dv
        double &sds = lst[16 * lsd], &sdz = lst[17 * lsd], &sdv = lst[18 * lsd], &sdsb = lst[19 * lsd],
               &sdzb = lst[20 * lsd];
        if constexpr (SLK) sdsb = sdzb = 0.0;
        if constexpr (SLK) {
            const double td = son ? dotl(skp->Go + lane * WNZ, sc.d) : 0.0;
            const double sd = seg8_sum(sliv * sD * (td - scr));
            sdv = (sd - fma(sDb, srb, slw)) * siS;
            sds = scr - td + sliv * sdv;
            const double qs = sds * sci;
            sdz = -cz * (1.0 + qs);
            rs = fmax(rs, -qs);
            rz = fmax(rz, 1.0 + qs);
            if (son) {
                sdsb = sdv + srb;
                const double qb = sdsb * rcp(sb);
                sdzb = -zb * (1.0 + qb);
                rs = fmax(rs, -qb);
                rz = fmax(rz, 1.0 + qb);
            }
        }
        wave_reduce2<Op::Max, Op::Max>(rs, rz);
        const double ap = rcp(fmax(1.0, rs)), ad = rcp(fmax(1.0, rz));
        double mua = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            mua = fma(sl[s] + ap * dsl[s], zl[s] + ad * dzl[s], mua);
            mua = fma(su[s] + ap * dsu[s], zu[s] + ad * dzu[s], mua);
        }
        if constexpr (SLK) {
            mua = fma(cs + ap * sds, cz + ad * sdz, mua);
            if (lead) mua = fma(sb + ap * sdsb, zb + ad * sdzb, mua);
        }
        mua = wave_reduce<Op::Sum>(mua) * inv_ns;
        double sig = mu > 0.0 ? mua * rcp(mu) : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        PSTAMP(6);
        // ---- corrector right-hand side G^T (kl/sl - ku/su)
        double kl[WR], ku[WR];
#pragma unroll
        for (int s = 0; s < WR; s++) {
            kl[s] = rw.ml[s] * (smu - dsl[s] * dzl[s]);
            ku[s] = smu - dsu[s] * dzu[s];
            const int r = wave_owner_row(lane, s);
            if (!SLK || r < skp->coff) sc.cv[r] = kl[s] * il[s] - ku[s] * iu[s];
        }
        // slack rows: row weights om = -kc / s on the centred rows; the mean row takes
        // (Db sum om + T kb / sb) / S; the v equation keeps vcv = -sum om + kb / sb
        double &skc = lst[21 * lsd], &skb = lst[22 * lsd], &svcv = lst[23 * lsd];
        if constexpr (SLK) {
            const WaveSlack& sk = *skp;
            skc = smu - sds * sdz;
            const double om = -skc * sci;
            const double som = seg8_sum(sliv * om);
            skb = smu - sdsb * sdzb;
            const double isb = rcp(sb);
            svcv = fma(skb, isb, -som);
            if (son) sk.cvs[lane] = sliv * om;
            if (lead) sk.cvs[8 * sk.nnb + (lane >> 3)] = fma(sDb, som, sT * skb * isb) * siS;
        }
        wave_lds_sync();
        const double vc_i = wave_gt(Gs, sc.cv, nchunk + (SLK ? skp->nchunk_c : 0), lane);
        PSTAMP(7);
        const double dy_i = dya_i + solve_rows(L, sc.M, inv_i, vc_i, i);
        publish16(sc.d, dy_i, lane);
        PSTAMP(8);
        double rmax = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double td = dotl(rw.g[s], sc.d);
            dsl[s] = rw.ml[s] * (td + rl[s]);
            dsu[s] = ru[s] - td;
            dzl[s] = (kl[s] - sl[s] * zl[s] - zl[s] * dsl[s]) * il[s];
            dzu[s] = (ku[s] - su[s] * zu[s] - zu[s] * dsu[s]) * iu[s];
            const double izl = rcp_fast(zl[s] + (1.0 - rw.ml[s]));
            rmax = fmax(rmax, fmax(-dsl[s] * il[s], -dsu[s] * iu[s]));
            rmax = fmax(rmax, fmax(-rw.ml[s] * dzl[s] * izl, -dzu[s] * rcp_fast(zu[s])));
        }
        // slack rows, combined direction: dv adds the corrector's v-equation term vcv
        if constexpr (SLK) {
            const double td = son ? dotl(skp->Go + lane * WNZ, sc.d) : 0.0;
            const double sd = seg8_sum(sliv * sD * (td - scr));
            sdv = (sd - fma(sDb, srb, slw) + svcv) * siS;
            sds = scr - td + sliv * sdv;
            sdz = (skc - cs * cz - cz * sds) * sci;
            rmax = fmax(rmax, fmax(-sds * sci, -sdz * rcp_fast(cz)));
            if (son) {
                sdsb = sdv + srb;
                const double isb = rcp(sb);
                sdzb = (skb - sb * zb - zb * sdsb) * isb;
                rmax = fmax(rmax, fmax(-sdsb * isb, -sdzb * rcp_fast(zb)));
            }
        }
        rmax = wave_reduce<Op::Max>(rmax);
        const double alpha = 0.99 * rcp(fmax(0.99, rmax));
#ifdef MPCCBF_DEBUG_TRACE
        if (dbg && lane == 0 && it < 64) {  // mu, rp, rd, alpha, sigma, ap, ad, first-try factor ok
            double* tr = (double*)dbg + 8 * it;
            tr[0] = mu; tr[1] = rp; tr[2] = rd_track; tr[3] = alpha; tr[4] = sig; tr[5] = ap;
            tr[6] = ad; tr[7] = fok0 ? 1.0 : 0.0;
        }
#endif
        PSTAMP(9);
        yi = fma(alpha, dy_i, yi);
        publish16(sc.y, yi, lane);
#pragma unroll
        for (int s = 0; s < WR; s++) {
            sl[s] = fmax(fma(alpha, dsl[s], sl[s]), 1e-300);
            su[s] = fmax(fma(alpha, dsu[s], su[s]), 1e-300);
            zl[s] = rw.ml[s] * fmax(fma(alpha, dzl[s], zl[s]), 1e-300);
            zu[s] = fmax(fma(alpha, dzu[s], zu[s]), 1e-300);
        }
        if constexpr (SLK) {
            cs = fmax(fma(alpha, sds, cs), 1e-300);
            cz = fmax(fma(alpha, sdz, cz), 1e-300);
            if (son) {
                v = fma(alpha, sdv, v);
                sb = fmax(fma(alpha, sdsb, sb), 1e-300);
                zb = fmax(fma(alpha, sdzb, zb), 1e-300);
            }
        }
        PSTAMP(10);
        rd_track *= (1.0 - alpha);
        PSTAMP(11);
        if (it % 8 == 7) rd_exact = true;
    }
    if constexpr (SLK) *v_obj = wave_reduce<Op::Sum>(lead ? slw * v : 0.0);
    return out;
}

// Phase 1: t* = min t s.t. lo - t <= g y <= hi + t, y in R^nz (nz <= 15), with a ridge eps/2 |y|^2;
// t is carried as the padded 16th variable. Every side becomes one one-sided row
// (lower: (-g, -1) v <= -lo; upper: (g, -1) v <= hi), so the Newton matrix is
//   [G^T (Dl + Du) G + eps I , G^T (Dl - Du) ; . , sum (Dl + Du) + Dt]
// — the first block on the matrix cores (column 15 = G^T (Dl - Du)), the corner by a reduction.
// The t >= 0 bound is one more side. Uses sc.y / sc.d / sc.M. Returns t* (>= 0), 1e300 on
// numerical failure.
__device__ __forceinline__ double pdip_phase1_wave(const WaveRows& rw, const double* __restrict__ Gs, int nchunk,
                                   WaveScratch& sc, int nz, const PdipCfg cfg, int lane) {
    constexpr double eps = 1e-10;
    const int i = lane16_opaque(lane);
    double vi = 0.0;  // y_i (i < 15) on the row layout
    publish16(sc.y, 0.0, lane);
    double viol = 0.0, nloc = 0.0;
#pragma unroll
    for (int s = 0; s < WR; s++) {
        viol = fmax(viol, fmax(rw.ml[s] * rw.lo[s], -rw.hi[s]));
        nloc += rw.ml[s] + 1.0;
    }
    double t = wave_reduce<Op::Max>(viol) + 1.0;
    const double inv_ns = rcp(wave_reduce<Op::Sum>(nloc) + 1.0);
    double sl[WR], su[WR], zl[WR], zu[WR];
#pragma unroll
    for (int s = 0; s < WR; s++) {
        sl[s] = rw.ml[s] > 0.0 ? t - rw.lo[s] : 1.0;
        su[s] = rw.hi[s] + t;
        zl[s] = rw.ml[s] * rcp(sl[s]);
        zu[s] = rcp(su[s]);
    }
    double zt = rcp(t);
    for (int it = 0; it < 2 * cfg.maxit; it++) {
        double rsl[WR], rsu[WR], il[WR], iu[WR], Dl[WR], Du[WR];
        double rp = 0.0, mloc = 0.0, dsum = 0.0, tcorner = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double gy = dotl(rw.g[s], sc.y);
            rsl[s] = rw.ml[s] * (gy + t - rw.lo[s] - sl[s]);
            rsu[s] = rw.hi[s] - gy + t - su[s];
            il[s] = rcp(sl[s]);
            iu[s] = rcp(su[s]);
            Dl[s] = zl[s] * il[s];
            Du[s] = zu[s] * iu[s];
            const double wl = -Dl[s] * rsl[s], wu = -Du[s] * rsu[s];
            const int r = wave_owner_row(lane, s);
            sc.Dv[r] = Dl[s] + Du[s];
            sc.wv[r] = Dl[s] - Du[s];
            sc.cv[r] = wl - wu;
            tcorner += wl + wu;
            dsum += Dl[s] + Du[s];
            mloc = fma(sl[s], zl[s], fma(su[s], zu[s], mloc));
            rp = fmax(rp, fmax(fabs(rsl[s]) * rw.ml[s] * rcp(1.0 + fabs(rw.lo[s])),
                               fabs(rsu[s]) * rcp(1.0 + fabs(rw.hi[s]))));
        }
        wave_lds_sync();
        const wd4 acc = wave_gram(Gs, sc.Dv, sc.wv, nchunk, lane);
        double Mr[WNZ];
        gram_rows(acc, sc.M, lane, Mr);  // column 15 = G^T (Dl - Du)
        const double rhs_i = wave_gt(Gs, sc.cv, nchunk, lane);
        tcorner = wave_reduce<Op::Sum>(tcorner);
        dsum = wave_reduce<Op::Sum>(dsum);
        rp = wave_reduce<Op::Max>(rp);
        const double mu = (wave_reduce<Op::Sum>(mloc) + t * zt) * inv_ns;
        if (!isfinite(mu) || !isfinite(rp)) return 1e300;
        if (rp <= cfg.tol && mu <= cfg.tol * 0.1) break;
        const double Dt = zt * rcp(t);
        // assemble the 16x16 phase-1 matrix on the row layout: rows/cols >= nz (but < 15) are
        // padding (identity); column/row 15 is t
        const double c15 = Mr[WNZ - 1];  // (G^T (Dl - Du))_i
        double row[WNZ];
#pragma unroll
        for (int k = 0; k < WNZ - 1; k++) row[k] = (i < WNZ - 1) ? Mr[k] + (i == k ? eps : 0.0) : 0.0;
        row[WNZ - 1] = (i < WNZ - 1) ? c15 : dsum + Dt;
#pragma unroll
        for (int k = 0; k < WNZ - 1; k++) {  // the t-row (lane 15) takes column 15 of the others
            const double ck = bcast16v(k, c15);
            row[k] = (i == WNZ - 1) ? ck : row[k];
        }
#pragma unroll
        for (int k = 0; k < WNZ - 1; k++)  // padding variables: identity rows / columns
            if (k >= nz) row[k] = (i == k) ? 1.0 : 0.0;
        if (i >= nz && i < WNZ - 1) {
#pragma unroll
            for (int k = 0; k < WNZ; k++) row[k] = (k == i) ? 1.0 : 0.0;
        }
        double L[WNZ], inv_i;
        if (!chol_rows(row, L, inv_i, sc.M, lane)) break;  // degenerate vertex: the iterate's violation stands
        // rhs: y part -eps y + G^T(wl - wu); t part -1 + sum(wl + wu)
        double b_i = (i < WNZ - 1) ? fma(-eps, vi, rhs_i) : -1.0 + tcorner;
        if (i >= nz && i < WNZ - 1) b_i = 0.0;
        double dv_i = solve_rows(L, sc.M, inv_i, b_i, i);
        publish16(sc.d, dv_i, lane);
        const double dsta = sc.d[WNZ - 1];
        double ap = 1.0, ad = 1.0, dsla[WR], dzla[WR], dsua[WR], dzua[WR];
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double dgy = dotl(rw.g[s], sc.d);  // g[15] = 0: the y part only
            dsla[s] = rw.ml[s] * (dgy + dsta + rsl[s]);
            dsua[s] = -dgy + dsta + rsu[s];
            dzla[s] = -zl[s] - Dl[s] * dsla[s];
            dzua[s] = -zu[s] - Du[s] * dsua[s];
            ap = fmin(ap, fmin(step_bound(sl[s], dsla[s], 1.0), step_bound(su[s], dsua[s], 1.0)));
            ad = fmin(ad, fmin(step_bound(zl[s], dzla[s], 1.0), step_bound(zu[s], dzua[s], 1.0)));
        }
        const double dzta = -zt - Dt * dsta;
        ap = fmin(wave_reduce<Op::Min>(ap), step_bound(t, dsta, 1.0));
        ad = fmin(wave_reduce<Op::Min>(ad), step_bound(zt, dzta, 1.0));
        double mua = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            mua = fma(sl[s] + ap * dsla[s], zl[s] + ad * dzla[s], mua);
            mua = fma(su[s] + ap * dsua[s], zu[s] + ad * dzua[s], mua);
        }
        mua = (wave_reduce<Op::Sum>(mua) + (t + ap * dsta) * (zt + ad * dzta)) * inv_ns;
        double sig = mu > 0.0 ? mua * rcp(mu) : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        double vct = 0.0, cl[WR], cu[WR];
#pragma unroll
        for (int s = 0; s < WR; s++) {
            cl[s] = rw.ml[s] * (smu - dsla[s] * dzla[s]);
            cu[s] = smu - dsua[s] * dzua[s];
            const double a = cl[s] * il[s], b = cu[s] * iu[s];
            sc.cv[wave_owner_row(lane, s)] = a - b;
            vct += a + b;
        }
        wave_lds_sync();
        const double vc_i = wave_gt(Gs, sc.cv, nchunk, lane);
        const double ct = smu - dsta * dzta;
        vct = wave_reduce<Op::Sum>(vct) + ct * rcp(t);
        double bc_i = (i < WNZ - 1) ? vc_i : vct;
        if (i >= nz && i < WNZ - 1) bc_i = 0.0;
        dv_i += solve_rows(L, sc.M, inv_i, bc_i, i);
        publish16(sc.d, dv_i, lane);
        const double dst = sc.d[WNZ - 1];
        double amax = 1e300, dsl[WR], dzl[WR], dsu[WR], dzu[WR];
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double dgy = dotl(rw.g[s], sc.d);
            dsl[s] = rw.ml[s] * (dgy + dst + rsl[s]);
            dsu[s] = -dgy + dst + rsu[s];
            dzl[s] = (cl[s] - sl[s] * zl[s] - zl[s] * dsl[s]) * il[s];
            dzu[s] = (cu[s] - su[s] * zu[s] - zu[s] * dsu[s]) * iu[s];
            amax = fmin(amax, fmin(step_bound(sl[s], dsl[s], 1e300), step_bound(su[s], dsu[s], 1e300)));
            amax = fmin(amax, fmin(step_bound(zl[s], rw.ml[s] * dzl[s], 1e300), step_bound(zu[s], dzu[s], 1e300)));
        }
        const double dzt = (ct - t * zt - zt * dst) * rcp(t);
        amax = fmin(wave_reduce<Op::Min>(amax), fmin(step_bound(t, dst, 1e300), step_bound(zt, dzt, 1e300)));
        const double alpha = fmin(1.0, 0.99 * amax);
        if (i < WNZ - 1) vi = fma(alpha, dv_i, vi);
        publish16(sc.y, vi, lane);
        t = fmax(fma(alpha, dst, t), 1e-300);
        zt = fmax(fma(alpha, dzt, zt), 1e-300);
#pragma unroll
        for (int s = 0; s < WR; s++) {
            sl[s] = fmax(fma(alpha, dsl[s], sl[s]), 1e-300);
            su[s] = fmax(fma(alpha, dsu[s], su[s]), 1e-300);
            zl[s] = rw.ml[s] * fmax(fma(alpha, dzl[s], zl[s]), 1e-300);
            zu[s] = fmax(fma(alpha, dzu[s], zu[s]), 1e-300);
        }
    }
    double worst = 0.0;
#pragma unroll
    for (int s = 0; s < WR; s++) {
        const double gy = dotl(rw.g[s], sc.y);
        worst = fmax(worst, fmax(rw.ml[s] * (rw.lo[s] - gy), gy - rw.hi[s]));
    }
    return wave_reduce<Op::Max>(worst);
}

}  // namespace dev
}  // namespace mpccbf
