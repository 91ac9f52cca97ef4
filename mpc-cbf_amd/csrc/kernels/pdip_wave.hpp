// pdip_wave.hpp — one QP per wavefront: the Mehrotra PDIP of pdip.hpp for reduced dimensions up
// to 16 and up to 192 rows, with the Newton matrix assembled on the matrix cores.
//
// Used by the FoV controller (nz = 15: 5 per channel over 4 Bezier pieces, rows coupling all
// channels), where a per-lane packed normal matrix (120 entries) would not fit the registers.
//
// Layouts (64 lanes, lane = 16 q + p):
//   rows   row r lives in slot s = r / 64 of lane 16 (r % 4) + (r / 4) % 16 ("owner"); the owner
//          keeps the row's 16 coefficients, bounds, slacks and duals in registers.
//   G      all rows, 16 doubles each, in the wave's LDS image; chunk c (rows 4c .. 4c+3) feeds one
//          v_mfma_f64_16x16x4f64 with A = G_chunk^T (lane: G[4c + q][p]) and
//          B = diag(D) G_chunk (lane: D_{4c+q} G[4c + q][p]); D_{4c+q} reaches lane (q, p) from
//          its owner (q, c % 16) by a DPP row broadcast. Column 15 of B carries the right-hand
//          side weights instead (the padded 16th variable has G[.][15] = 0), so one MFMA chain
//          yields M = G^T D G and G^T w.
//   rows-of-M  the 16x16 result is transposed through LDS so that lane i (of every 16-lane
//          row) holds row i of M; Cholesky (left-looking, DPP broadcasts of row j) and both
//          triangular solves run on that layout, and every solve ends with the solution in
//          every lane.
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

// all-reduce (sum) of a 16-vector over the wave, stage-major
__device__ __forceinline__ void wave_sum16(double (&v)[WNZ]) {
    grp_sum_vec<16, WNZ>(v);
#pragma unroll
    for (int i = 0; i < WNZ; i++) v[i] = xrow16<Op::Sum>(v[i]);
#pragma unroll
    for (int i = 0; i < WNZ; i++) v[i] = xrow32<Op::Sum>(v[i]);
}

// element (lane & 15) of a wave-uniform 16-vector
__device__ __forceinline__ double lane_pick16(const double (&u)[WNZ], int i) {
    double v = u[0];
#pragma unroll
    for (int k = 1; k < WNZ; k++) v = (i == k) ? u[k] : v;
    return v;
}

// ---- Gram matrix on the matrix cores -------------------------------------------------------
// acc = G^T diag(D) G with column 15 replaced by G^T w (rows beyond nchunk*4 skipped).
// Gs: the wave's LDS row image (WROWS x 16); D, w: per owned slot.
__device__ __forceinline__ wd4 wave_gram(const double* __restrict__ Gs, int nchunk, const double (&D)[WR],
                                         const double (&w)[WR], int lane) {
    const int q = lane >> 4, p = lane & 15;
    wd4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < WCH; c++) {
        if (c < nchunk) {  // wave-uniform
            const double g = Gs[(4 * c + q) * WNZ + p];
            const double Dq = bcast16v(c, D[c >> 4]);
            const double wq = bcast16v(c, w[c >> 4]);
            const double b = (p == WNZ - 1) ? wq : Dq * g;
            if (c & 1)
                acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(g, b, acc1, 0, 0, 0);
            else
                acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(g, b, acc0, 0, 0, 0);
        }
    }
    return acc0 + acc1;
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

// Left-looking Cholesky on the row layout: lane i holds row i of M (k <= i used) and gets row i
// of L; inv[j] = 1 / L_jj (wave-uniform). Returns false if a pivot is not positive.
__device__ __forceinline__ bool chol_rows(const double (&M)[WNZ], double (&L)[WNZ], double (&inv)[WNZ], int i) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < WNZ; j++) {
        double v = M[j];
#pragma unroll
        for (int k = 0; k < j; k++) v = fma(-L[k], bcast16v(j, L[k]), v);
        const double d = bcast16v(j, v);
        ok = ok && (d > 0.0);
        const double r = rsqrt(d > 0.0 ? d : 1e-300);
        inv[j] = r;
        L[j] = (i >= j) ? v * r : 0.0;
    }
    return ok;
}

// Column layout of L through LDS: lane i gets Lc[k] = L[k][i].
__device__ __forceinline__ void chol_cols(const double (&L)[WNZ], double* __restrict__ Mbuf, int lane,
                                          double (&Lc)[WNZ]) {
    const int i = lane & 15;
    if (lane < 16) {
#pragma unroll
        for (int k = 0; k < WNZ; k++) Mbuf[i * WNZ + k] = L[k];
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < WNZ; k++) Lc[k] = Mbuf[k * WNZ + i];
    wave_lds_sync();
}

// Solve L L^T x = b, b given on the row layout (lane i: b_i); x returned wave-uniform.
__device__ __forceinline__ void solve_rows(const double (&L)[WNZ], const double (&Lc)[WNZ],
                                           const double (&inv)[WNZ], double b, int i, double (&x)[WNZ]) {
    double res = b, wl = 0.0;
#pragma unroll
    for (int k = 0; k < WNZ; k++) {
        const double wk = bcast16v(k, res) * inv[k];
        res = fma(-L[k], wk, res);
        wl = (i == k) ? wk : wl;
    }
    res = wl;
#pragma unroll
    for (int k = WNZ - 1; k >= 0; k--) {
        const double xk = bcast16v(k, res) * inv[k];
        res = fma(-Lc[k], xk, res);
        x[k] = xk;
    }
}

// Row storage of one lane (owner layout). Every row has an upper side; ml = 1 adds the lower.
// Unused slots hold inert rows (g = 0, -1 <= 0 <= 1).
struct WaveRows {
    double g[WR][WNZ];
    double lo[WR], hi[WR], ml[WR];
};

__device__ __forceinline__ double dot16(const double (&a)[WNZ], const double (&b)[WNZ]) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < WNZ; j++) s = fma(a[j], b[j], s);
    return s;
}

struct WaveScratch {     // per-wave LDS besides the row image
    double M[WNZ * WNZ];
};

// Main solve. P, LP: 16x16 row-major, padded with the identity (uniform, global). q, y uniform.
// nz: true reduced dimension (<= 15; the 16th variable is padding). nchunk: row chunks in use.
__device__ PdipOut pdip_solve_wave(const WaveRows& rw, const double* __restrict__ Gs, int nchunk,
                                   WaveScratch& sc, const double* __restrict__ P,
                                   const double* __restrict__ LP, const double (&q)[WNZ],
                                   double (&y)[WNZ], const PdipCfg cfg, int lane) {
    const int i = lane & 15;
    // ---- start: y0 = -P^{-1} q (uniform triangular solves with LP)
    {
        double w[WNZ];
#pragma unroll
        for (int r = 0; r < WNZ; r++) {
            double v = -q[r];
#pragma unroll
            for (int k = 0; k < r; k++) v = fma(-LP[r * WNZ + k], w[k], v);
            w[r] = v * rcp(LP[r * WNZ + r]);
        }
#pragma unroll
        for (int r = WNZ - 1; r >= 0; r--) {
            double v = w[r];
#pragma unroll
            for (int k = r + 1; k < WNZ; k++) v = fma(-LP[k * WNZ + r], y[k], v);
            y[r] = v * rcp(LP[r * WNZ + r]);
        }
    }
    double sl[WR], su[WR], zl[WR], zu[WR], pl[WR], pu[WR];
    double nloc = 0.0;
#pragma unroll
    for (int s = 0; s < WR; s++) {
        const double t = dot16(rw.g[s], y);
        sl[s] = rw.ml[s] > 0.0 ? fmax(t - rw.lo[s], 1.0) : 1.0;
        su[s] = fmax(rw.hi[s] - t, 1.0);
        zl[s] = rw.ml[s] * rcp(sl[s]);
        zu[s] = rcp(su[s]);
        pl[s] = rw.ml[s] * rcp(1.0 + fabs(rw.lo[s]));
        pu[s] = rcp(1.0 + fabs(rw.hi[s]));
        nloc += rw.ml[s] + 1.0;
    }
    const double inv_ns = rcp(wave_reduce<Op::Sum>(nloc));
    double qn = 0.0;
#pragma unroll
    for (int j = 0; j < WNZ; j++) qn = fmax(qn, fabs(q[j]));
    const double inv_qn = rcp(1.0 + qn);
    // P row i (row layout) for P y
    double Prow[WNZ];
#pragma unroll
    for (int k = 0; k < WNZ; k++) Prow[k] = P[i * WNZ + k];
    const double qi = lane_pick16(q, i);

    PdipOut out{ST_UNKNOWN, 0};
    double mu0 = 1.0, rd_track = 1e300;
    bool rd_exact = true;
    for (int it = 0;; it++) {
        double rl[WR], ru[WR], il[WR], iu[WR], D[WR], wv[WR];
        double mloc = 0.0, rp = 0.0;
        double dz[WNZ];
#pragma unroll
        for (int j = 0; j < WNZ; j++) dz[j] = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double t = dot16(rw.g[s], y);
            rl[s] = rw.ml[s] * (t - rw.lo[s] - sl[s]);
            ru[s] = rw.hi[s] - t - su[s];
            il[s] = rcp(sl[s]);
            iu[s] = rcp(su[s]);
            const double Dl = zl[s] * il[s], Du = zu[s] * iu[s];
            D[s] = Dl + Du;
            wv[s] = Du * ru[s] - Dl * rl[s];
            mloc = fma(sl[s], zl[s], fma(su[s], zu[s], mloc));
            rp = fmax(rp, fmax(fabs(rl[s]) * pl[s], fabs(ru[s]) * pu[s]));
            if (rd_exact) {
#pragma unroll
                for (int j = 0; j < WNZ; j++) dz[j] = fma(rw.g[s][j], zu[s] - zl[s], dz[j]);
            }
        }
        const wd4 acc = wave_gram(Gs, nchunk, D, wv, lane);
        double Mr[WNZ];
        gram_rows(acc, sc.M, lane, Mr);
        const double rhs_i = Mr[WNZ - 1];  // G^T w (column 15)
#pragma unroll
        for (int k = 0; k < WNZ; k++) Mr[k] = (k == WNZ - 1 && i != WNZ - 1 ? 0.0 : Mr[k]) + Prow[k];
        const double mu = wave_reduce<Op::Sum>(mloc) * inv_ns;
        rp = wave_reduce<Op::Max>(rp);
        const double py_i = dot16(Prow, y) + qi;  // (P y + q)_i
        if (rd_exact) {
            wave_sum16(dz);
            rd_track = grp_max<16>(fabs(py_i + lane_pick16(dz, i))) * inv_qn;
            rd_exact = false;
        }
        out.iters = it;
        const bool finite = isfinite(rp) && isfinite(rd_track) && isfinite(mu) && isfinite(Mr[0]);
        if (finite && rp <= cfg.tol && mu <= cfg.tol * 0.1) {
            if (rd_track <= cfg.tol) {
                double chk[WNZ];
#pragma unroll
                for (int j = 0; j < WNZ; j++) chk[j] = 0.0;
#pragma unroll
                for (int s = 0; s < WR; s++)
#pragma unroll
                    for (int j = 0; j < WNZ; j++) chk[j] = fma(rw.g[s][j], zu[s] - zl[s], chk[j]);
                wave_sum16(chk);
                rd_track = grp_max<16>(fabs(py_i + lane_pick16(chk, i))) * inv_qn;
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
        // ---- factor
        double L[WNZ], Lc[WNZ], inv[WNZ];
        if (!chol_rows(Mr, L, inv, i)) {
            out.status = ST_UNKNOWN;
            break;
        }
        chol_cols(L, sc.M, lane, Lc);
        // ---- predictor
        double dya[WNZ];
        solve_rows(L, Lc, inv, rhs_i - py_i, i, dya);
        double dsl[WR], dsu[WR], dzl[WR], dzu[WR];
        double rs = 0.0, rz = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double td = dot16(rw.g[s], dya);
            dsl[s] = rw.ml[s] * (td + rl[s]);
            dsu[s] = ru[s] - td;
            const double ql = dsl[s] * il[s], qu = dsu[s] * iu[s];
            dzl[s] = -zl[s] * (1.0 + ql);
            dzu[s] = -zu[s] * (1.0 + qu);
            rs = fmax(rs, fmax(-ql, -qu));
            rz = fmax(rz, fmax(rw.ml[s] * (1.0 + ql), 1.0 + qu));
        }
        rs = wave_reduce<Op::Max>(rs);
        rz = wave_reduce<Op::Max>(rz);
        const double ap = rcp(fmax(1.0, rs)), ad = rcp(fmax(1.0, rz));
        double mua = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            mua = fma(sl[s] + ap * dsl[s], zl[s] + ad * dzl[s], mua);
            mua = fma(su[s] + ap * dsu[s], zu[s] + ad * dzu[s], mua);
        }
        mua = wave_reduce<Op::Sum>(mua) * inv_ns;
        double sig = mu > 0.0 ? mua * rcp(mu) : 0.0;
        sig = fmin(sig * sig * sig, 1.0);
        const double smu = sig * mu;
        // ---- corrector right-hand side G^T (kl/sl - ku/su)
        double kl[WR], ku[WR], vc[WNZ];
#pragma unroll
        for (int j = 0; j < WNZ; j++) vc[j] = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            kl[s] = rw.ml[s] * (smu - dsl[s] * dzl[s]);
            ku[s] = smu - dsu[s] * dzu[s];
            const double wgt = kl[s] * il[s] - ku[s] * iu[s];
#pragma unroll
            for (int j = 0; j < WNZ; j++) vc[j] = fma(rw.g[s][j], wgt, vc[j]);
        }
        wave_sum16(vc);
        double dyc[WNZ], dy[WNZ];
        solve_rows(L, Lc, inv, lane_pick16(vc, i), i, dyc);
#pragma unroll
        for (int j = 0; j < WNZ; j++) dy[j] = dya[j] + dyc[j];
        double rmax = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double td = dot16(rw.g[s], dy);
            dsl[s] = rw.ml[s] * (td + rl[s]);
            dsu[s] = ru[s] - td;
            dzl[s] = (kl[s] - sl[s] * zl[s] - zl[s] * dsl[s]) * il[s];
            dzu[s] = (ku[s] - su[s] * zu[s] - zu[s] * dsu[s]) * iu[s];
            const double izl = rcp_fast(zl[s] + (1.0 - rw.ml[s]));
            rmax = fmax(rmax, fmax(-dsl[s] * il[s], -dsu[s] * iu[s]));
            rmax = fmax(rmax, fmax(-rw.ml[s] * dzl[s] * izl, -dzu[s] * rcp_fast(zu[s])));
        }
        rmax = wave_reduce<Op::Max>(rmax);
        const double alpha = 0.99 * rcp(fmax(0.99, rmax));
#pragma unroll
        for (int j = 0; j < WNZ; j++) y[j] = fma(alpha, dy[j], y[j]);
#pragma unroll
        for (int s = 0; s < WR; s++) {
            sl[s] = fmax(fma(alpha, dsl[s], sl[s]), 1e-300);
            su[s] = fmax(fma(alpha, dsu[s], su[s]), 1e-300);
            zl[s] = rw.ml[s] * fmax(fma(alpha, dzl[s], zl[s]), 1e-300);
            zu[s] = fmax(fma(alpha, dzu[s], zu[s]), 1e-300);
        }
        rd_track *= (1.0 - alpha);
        if (it % 8 == 7) rd_exact = true;
    }
    return out;
}

// Phase 1: t* = min t s.t. lo - t <= g y <= hi + t, y in R^nz (nz <= 15), with a ridge eps/2 |y|^2;
// t is carried as the padded 16th variable. Every side becomes one one-sided row
// (lower: (-g, -1) v <= -lo; upper: (g, -1) v <= hi), so the Newton matrix is
//   [G^T (Dl + Du) G + eps I , G^T (Dl - Du) ; . , sum (Dl + Du) + Dt]
// — the first block on the matrix cores (column 15 = G^T (Dl - Du)), the corner by a reduction.
// The t >= 0 bound is one more side. Returns t* (>= 0), 1e300 on numerical failure.
__device__ double pdip_phase1_wave(const WaveRows& rw, const double* __restrict__ Gs, int nchunk,
                                   WaveScratch& sc, int nz, const PdipCfg cfg, int lane) {
    constexpr double eps = 1e-10;
    const int i = lane & 15;
    double y[WNZ];
#pragma unroll
    for (int j = 0; j < WNZ; j++) y[j] = 0.0;
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
        double rsl[WR], rsu[WR], il[WR], iu[WR], Dl[WR], Du[WR], Ds[WR], Dd[WR];
        double rp = 0.0, mloc = 0.0, dsum = 0.0, tcorner = 0.0;
        double rhs[WNZ];
#pragma unroll
        for (int j = 0; j < WNZ; j++) rhs[j] = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            const double gy = dot16(rw.g[s], y);
            rsl[s] = rw.ml[s] * (gy + t - rw.lo[s] - sl[s]);
            rsu[s] = rw.hi[s] - gy + t - su[s];
            il[s] = rcp(sl[s]);
            iu[s] = rcp(su[s]);
            Dl[s] = zl[s] * il[s];
            Du[s] = zu[s] * iu[s];
            Ds[s] = Dl[s] + Du[s];
            Dd[s] = Dl[s] - Du[s];
            const double wl = -Dl[s] * rsl[s], wu = -Du[s] * rsu[s];
#pragma unroll
            for (int j = 0; j < WNZ; j++) rhs[j] = fma(rw.g[s][j], wl - wu, rhs[j]);
            tcorner += wl + wu;
            dsum += Ds[s];
            mloc = fma(sl[s], zl[s], fma(su[s], zu[s], mloc));
            rp = fmax(rp, fmax(fabs(rsl[s]) * rw.ml[s] * rcp(1.0 + fabs(rw.lo[s])),
                               fabs(rsu[s]) * rcp(1.0 + fabs(rw.hi[s]))));
        }
        const wd4 acc = wave_gram(Gs, nchunk, Ds, Dd, lane);
        double Mr[WNZ];
        gram_rows(acc, sc.M, lane, Mr);  // column 15 = G^T (Dl - Du)
        wave_sum16(rhs);
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
        // the t-row (lane 15) needs the column 15 entries of the other rows: gather them
        double col15[WNZ];
#pragma unroll
        for (int k = 0; k < WNZ; k++) col15[k] = bcast16v(k, c15);
        if (i == WNZ - 1) {
#pragma unroll
            for (int k = 0; k < WNZ - 1; k++) row[k] = col15[k];
        }
#pragma unroll
        for (int k = 0; k < WNZ - 1; k++)  // padding variables: identity rows / columns
            if (k >= nz) row[k] = (i == k) ? 1.0 : 0.0;
        if (i >= nz && i < WNZ - 1) {
#pragma unroll
            for (int k = 0; k < WNZ; k++) row[k] = (k == i) ? 1.0 : 0.0;
        }
        double L[WNZ], Lc[WNZ], inv[WNZ];
        if (!chol_rows(row, L, inv, i)) return 1e300;
        chol_cols(L, sc.M, lane, Lc);
        // rhs: y part -eps y + G^T(wl - wu); t part -1 + sum(wl + wu)
        double b_i = (i < WNZ - 1) ? fma(-eps, lane_pick16(y, i), lane_pick16(rhs, i)) : -1.0 + tcorner;
        if (i >= nz && i < WNZ - 1) b_i = 0.0;
        double dv[WNZ];
        solve_rows(L, Lc, inv, b_i, i, dv);
        double ap = 1.0, ad = 1.0, dsla[WR], dzla[WR], dsua[WR], dzua[WR];
#pragma unroll
        for (int s = 0; s < WR; s++) {
            double dgy = 0.0;
#pragma unroll
            for (int j = 0; j < WNZ - 1; j++) dgy = fma(rw.g[s][j], dv[j], dgy);
            dsla[s] = rw.ml[s] * (dgy + dv[WNZ - 1] + rsl[s]);
            dsua[s] = -dgy + dv[WNZ - 1] + rsu[s];
            dzla[s] = -zl[s] - Dl[s] * dsla[s];
            dzua[s] = -zu[s] - Du[s] * dsua[s];
            ap = fmin(ap, fmin(step_bound(sl[s], dsla[s], 1.0), step_bound(su[s], dsua[s], 1.0)));
            ad = fmin(ad, fmin(step_bound(zl[s], dzla[s], 1.0), step_bound(zu[s], dzua[s], 1.0)));
        }
        const double dsta = dv[WNZ - 1], dzta = -zt - Dt * dsta;
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
        double vc[WNZ], vct = 0.0, cl[WR], cu[WR];
#pragma unroll
        for (int j = 0; j < WNZ; j++) vc[j] = 0.0;
#pragma unroll
        for (int s = 0; s < WR; s++) {
            cl[s] = rw.ml[s] * (smu - dsla[s] * dzla[s]);
            cu[s] = smu - dsua[s] * dzua[s];
            const double a = cl[s] * il[s], b = cu[s] * iu[s];
#pragma unroll
            for (int j = 0; j < WNZ; j++) vc[j] = fma(rw.g[s][j], a - b, vc[j]);
            vct += a + b;
        }
        wave_sum16(vc);
        const double ct = smu - dsta * dzta;
        vct = wave_reduce<Op::Sum>(vct) + ct * rcp(t);
        double bc_i = (i < WNZ - 1) ? lane_pick16(vc, i) : vct;
        if (i >= nz && i < WNZ - 1) bc_i = 0.0;
        double dvc[WNZ];
        solve_rows(L, Lc, inv, bc_i, i, dvc);
#pragma unroll
        for (int j = 0; j < WNZ; j++) dv[j] += dvc[j];
        double amax = 1e300, dsl[WR], dzl[WR], dsu[WR], dzu[WR];
#pragma unroll
        for (int s = 0; s < WR; s++) {
            double dgy = 0.0;
#pragma unroll
            for (int j = 0; j < WNZ - 1; j++) dgy = fma(rw.g[s][j], dv[j], dgy);
            dsl[s] = rw.ml[s] * (dgy + dv[WNZ - 1] + rsl[s]);
            dsu[s] = -dgy + dv[WNZ - 1] + rsu[s];
            dzl[s] = (cl[s] - sl[s] * zl[s] - zl[s] * dsl[s]) * il[s];
            dzu[s] = (cu[s] - su[s] * zu[s] - zu[s] * dsu[s]) * iu[s];
            amax = fmin(amax, fmin(step_bound(sl[s], dsl[s], 1e300), step_bound(su[s], dsu[s], 1e300)));
            amax = fmin(amax, fmin(step_bound(zl[s], rw.ml[s] * dzl[s], 1e300), step_bound(zu[s], dzu[s], 1e300)));
        }
        const double dst = dv[WNZ - 1];
        const double dzt = (ct - t * zt - zt * dst) * rcp(t);
        amax = fmin(wave_reduce<Op::Min>(amax), fmin(step_bound(t, dst, 1e300), step_bound(zt, dzt, 1e300)));
        const double alpha = fmin(1.0, 0.99 * amax);
#pragma unroll
        for (int j = 0; j < WNZ - 1; j++) y[j] = fma(alpha, dv[j], y[j]);
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
        const double gy = dot16(rw.g[s], y);
        worst = fmax(worst, fmax(rw.ml[s] * (rw.lo[s] - gy), gy - rw.hi[s]));
    }
    return wave_reduce<Op::Max>(worst);
}

}  // namespace dev
}  // namespace mpccbf
