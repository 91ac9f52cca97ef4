// impc_fov.hip — FovBezierIMPCCBF::optimize (mpc_cbf/src/controller/FovBezierIMPCCBF.cpp:44-223)
// for a batch of agents, one agent per wavefront (BASELINE config 5).
//
// Per agent and IMPC iteration the QP has 15 free variables (4 Bezier pieces, C^0..C^2
// continuity eliminated), the shared box rows (two-sided), and per observed neighbour
//   * 4 Voronoi rows on the piece-0 control points (separating_hyperplanes::voronoi shifted by
//     the robot box, hyperplaneConstraintAll, epsilon 1e-8), in both iterations, and
//   * 4 FoV HOCBF rows (safety, left / right FoV border, range; FovCBF.cpp:152-535) at the
//     current state (iteration 0) or at each predicted state (iteration 1), with the exact
//     acceleration-box redundancy filter of the collision path.
// Rows are staged as a dense 16-wide image in LDS and solved by pdip_wave.hpp (MFMA Gram).
#include <hip/hip_runtime.h>

#include <cmath>

#include "impc.hpp"
#include "impc_common.hpp"
#include "fov_cbf.hpp"
#include "das_wave.hpp"

namespace mpccbf {
namespace dev {

constexpr int FOV_NB_CAP = 16;  // observed neighbours per agent

// Diagnostics build (make setupst): stamps 2 .. 6 mark points inside the setup (after the operator
// loads' issue, the linear term, the box rows, the neighbour states, the constant rows) instead of
// the later phases (tools/setup_stamps.py)
#ifdef MPCCBF_SETUP_STAMPS
#define SSTAMP(k) stamp(args, ai, lane, k)
#define PHSTAMP(k) \
    do {          \
    } while (0)
#else
#define SSTAMP(k) \
    do {          \
    } while (0)
#define PHSTAMP(k) stamp(args, ai, lane, k)
#endif

// LDS of the slack rows (slack mode only)
struct FovSlackLds {
    double Go[WSL_ROWS * WNZ];
    double zvs[WSL_ROWS];
    double st[WSL_NST * 64];  // per-lane slack solver state (WaveSlack::st)
    double h[WSL_ROWS], live[WSL_ROWS];
    double Tn[WSL_NB], w[WSL_NB], dist[WSL_NB];
    int32_t order[WSL_NB];
    int32_t rowl[WSL_ROWS];  // FoV row compacted after the ordinary image -> its slack-image row
    int32_t lead[WSL_NB];    // per neighbour: its leader row (slack-image row), -1 = v_i at 0
};

// Position of observed neighbour i: from the neighbour query's LDS copy in grid mode, else the
// state table.
__device__ __forceinline__ void nb_position(const ImpcArgs& args, const NbScratch& sc, bool grid_mode, int nb0,
                                            int i, double& px, double& py) {
    if (grid_mode) {
        const int c = sc.src[i];
        px = sc.cst[0][c];
        py = sc.cst[1][c];
    } else {
        const int nbi = args.nb_col[nb0 + i];
        px = args.states[(size_t)nbi * 6];
        py = args.states[(size_t)nbi * 6 + 1];
        // (keeps the two branches' reads apart: merged, the LDS and global reads became one flat
        // load through a selected pointer)
        asm volatile("" : "+v"(px), "+v"(py));
    }
}

template <bool SLACK>
__global__ void __launch_bounds__(64) impc_fov_kernel(const DevOps op, const double* __restrict__ buf,
                                                       const ImpcArgs args) {
    constexpr int NZ = 15;
    const int lane = threadIdx.x;
    const int ai = xcd_block((int)blockIdx.x, (int)gridDim.x);
    lds_poison();
    grid_clear<64>(args);
    if (ai >= args.num_agents) return;
    stamp(args, ai, lane, 0);
    const double* zero_row = nullptr;
    FovSlackLds* slk = nullptr;
    if constexpr (SLACK) {
        __shared__ FovSlackLds slk_mem;
        slk = &slk_mem;
    }
    __shared__ double Gimg[(WROWS + 1) * WNZ];  // + one all-zero row for unused slots
    __shared__ double rlo[WROWS], rhi[WROWS], rml[WROWS];
    __shared__ WaveScratch sc;
    __shared__ NbScratch nb_scratch;
    __shared__ WaveAS was;  // dual active-set workspace

    const int self = args.agent_first + ai;
    double s0[6];
#pragma unroll
    for (int k = 0; k < 6; k++) s0[k] = args.states[(size_t)self * 6 + k];
    // grid mode: the neighbour query's loads are staged between the setup's (gq_*; the state
    // arrives before the branch, else the join waits for every load in flight)
    const bool grid_mode = args.nb_row_ptr == nullptr;
    GridQuery<64> gq;
    asm volatile("" ::"v"(s0[0]), "v"(s0[1]), "v"(s0[2]), "v"(s0[3]), "v"(s0[4]), "v"(s0[5]));
    if (grid_mode) gq_begin<64>(args, s0[0], s0[1], gq);
    __shared__ double ykeep_s[WNZ], q_s[WNZ];  // wave-uniform vectors kept out of the registers
    __shared__ double ypd[WNZ];                // slack mode: the slack PDIP's point during its polish
    __shared__ double kconst_s;                // the objective's constant (read once per IMPC iteration)
    __shared__ double ego_s[2][8];             // IMPC iteration >= 1: the ego state at each CBF sample
    // the FoV rows' per-sample operators (acceleration rows U_k: Z and s0 parts; the P^-1 Grams of
    // the rows' weights), copied once per agent: read by every row task of both IMPC iterations
    __shared__ double uz_s[MAX_CBF_H * 3 * 15], us_s[MAX_CBF_H * 18], mf_s[MAX_CBF_H * 6];
    // non-finite QP data (a NaN / Inf state, target or neighbour position), checked where the rows
    // are formed (v * 0 is NaN for a non-finite v): the rows that persist across the IMPC
    // iterations (q, box-row bounds, Voronoi rows) and each iteration's FoV rows
    bool nfin_fixed = false;
    // The setup's state-independent operator loads — the box rows' shift coefficients, bounds,
    // weights and the first BOXB image entries per lane, P and P^-1, the FoV rows' per-sample
    // operators, the first pass of constant rows — are issued in one batch with the linear term's,
    // so the whole batch is one round trip; issued block by block, each waited for the one before
    // (six round trips ahead of the first solve).
    constexpr int BOXB = 18;
    constexpr int NE = WNZ * WNZ / 64;
    constexpr int NL = (MAX_CBF_H * (3 * 15 + 18 + 6) + 63) / 64;
    const int mb = op.m;
    const int ng = mb * WNZ;
    const double* W = opp(buf, op.o_Wbox);
    const double* wb = opp(buf, op.o_wbox);
    const int n1 = op.cbf_h * 3 * NZ, n2 = op.cbf_h * 18, n3 = op.cbf_h * 6;
    const double* s1 = opp(buf, op.o_UZ);
    const double* s2 = opp(buf, op.o_US);
    const double* s3 = opp(buf, op.o_wfov);
    const bool has_c = op.mc > 0;
    const double* Cs = has_c ? opp(buf, op.o_Cs) : buf;
    const double* clo = has_c ? opp(buf, op.o_clo) : buf;
    const double* chi = has_c ? opp(buf, op.o_chi) : buf;
    double bt[WR][8], bw[WR], bv[BOXB], pi[NE], pp[NE], fo[NL], cr[8];
    {
#pragma unroll
        for (int sl = 0; sl < WR; sl++) {
            const int r = lane + 64 * sl;
            const double* src = W + (size_t)(r < mb ? r : 0) * WBOX_ROW + WNZ;
#pragma unroll
            for (int k = 0; k < 8; k++) bt[sl][k] = src[k];
            bw[sl] = wb[r < mb ? r : 0];
        }
#pragma unroll
        for (int b = 0; b < BOXB; b++) {
            const int f = 64 * b + lane;
            const int fc = f < ng ? f : 0;
            bv[b] = W[(size_t)(fc / WNZ) * WBOX_ROW + fc % WNZ];
        }
        const double* P16 = opp(buf, op.o_P16);
        const double* Pi16 = opp(buf, op.o_Pinv16);
#pragma unroll
        for (int k = 0; k < NE; k++) {
            pi[k] = Pi16[lane + 64 * k];
            pp[k] = P16[lane + 64 * k];
        }
#pragma unroll
        for (int b = 0; b < NL; b++) {
            const int f = lane + 64 * b;
            const double* src = f < n1 ? s1 + f : (f < n1 + n2 ? s2 + (f - n1) : s3 + (f < n1 + n2 + n3 ? f - n1 - n2 : 0));
            fo[b] = *src;
        }
        const int ci = lane < op.mc ? lane : 0;
#pragma unroll
        for (int k = 0; k < 6; k++) cr[k] = Cs[ci * 6 + k];
        cr[6] = clo[ci];
        cr[7] = chi[ci];
    }
    SSTAMP(2);
    {
        double kconst0;
        const double q = agent_linear_term_lanes<NZ, 64>(op, buf, args, ai, s0, lane, kconst0);
        nfin_fixed = !(fma(q, 0.0, kconst0 * 0.0) == 0.0);  // (per lane; the solve ballots it)
        if (lane < WNZ) {
            q_s[lane] = q;  // (0 for the padding entry)
            ykeep_s[lane] = 0.0;
        }
        if (lane == 0) kconst_s = kconst0;
    }

    SSTAMP(3);
    // ---- shared box rows into the image (rows 0 .. mb-1), bounds shifted by Gs s0
    if (grid_mode) gq_slots<64>(args, gq, lane);
    {
#pragma unroll
        for (int b = 0; b < BOXB; b++) {
            const int f = 64 * b + lane;
            if (f < ng) Gimg[f] = bv[b];
        }
        // (more than 64 BOXB entries: the rest as before, BOXB per lane at a time, indices clamped)
        for (int f0 = 64 * BOXB; f0 < ng; f0 += 64 * BOXB) {
            double v[BOXB];
#pragma unroll
            for (int b = 0; b < BOXB; b++) {
                const int f = f0 + 64 * b + lane;
                const int fc = f < ng ? f : 0;
                v[b] = W[(size_t)(fc / WNZ) * WBOX_ROW + fc % WNZ];
            }
#pragma unroll
            for (int b = 0; b < BOXB; b++) {
                const int f = f0 + 64 * b + lane;
                if (f < ng) Gimg[f] = v[b];
            }
        }
#pragma unroll
        for (int sl = 0; sl < WR; sl++) {
            const int r = lane + 64 * sl;
            if (r < mb) {
                double sh = 0.0;
#pragma unroll
                for (int k = 0; k < 6; k++) sh = fma(bt[sl][k], s0[k], sh);
                rlo[r] = bt[sl][6] - sh;
                rhi[r] = bt[sl][7] - sh;
                nfin_fixed = nfin_fixed || !(sh * 0.0 == 0.0);  // (the rows themselves: host constants)
                rml[r] = 1.0;
                was.wn[r] = (float)bw[sl];  // (constant rows: the host's weights)
            }
        }
    }
    SSTAMP(4);
    if (grid_mode) gq_states<64>(args, gq, lane);
    if (lane < WNZ) Gimg[WROWS * WNZ + lane] = 0.0;
    zero_row = &Gimg[WROWS * WNZ];
    SSTAMP(5);
    // constant rows (constant_rows_infeasible; the first 64 from the batch)
    bool infeasible;
    {
        bool bad = false;
        if (lane < op.mc) {
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < 6; k++) v = fma(cr[k], s0[k], v);
            bad = (v < cr[6] - op.feas_tol) | (v > cr[7] + op.feas_tol);
        }
        for (int i = lane + 64; i < op.mc; i += 64) {
            const double lo = clo[i], hi = chi[i];
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < 6; k++) v = fma(Cs[i * 6 + k], s0[k], v);
            bad = bad | (v < lo - op.feas_tol) | (v > hi + op.feas_tol);
        }
        infeasible = __ballot(bad) != 0ull;
    }
    SSTAMP(6);
    das_store_operators(was, pi, pp, lane);
#pragma unroll
    for (int b = 0; b < NL; b++) {
        const int f = lane + 64 * b;
        if (f < n1) uz_s[f] = fo[b];
        else if (f < n1 + n2) us_s[f - n1] = fo[b];
        else if (f < n1 + n2 + n3) mf_s[f - n1 - n2] = fo[b];
    }
    stamp(args, ai, lane, 1);

    int nb0 = 0, nnb = 0;
    if (!grid_mode) {
        nb0 = args.nb_row_ptr[ai];
        nnb = args.nb_row_ptr[ai + 1] - nb0;
    } else {
        nnb = grid_neighbors_finish<64>(args, self, s0[0], s0[1], nb_scratch, lane, s0[2], gq);
    }
    const bool nb_overflow = nnb < 0 || nnb > (SLACK ? WSL_NB : FOV_NB_CAP);
    if (nb_overflow) nnb = 0;
    if constexpr (SLACK) {
        // slack weights (FovBezierIMPCCBF.cpp:58-81): sort the neighbours by distanceToEllipse
        // (ties keep the list order, as libstdc++'s insertion sort below 17 elements does); the
        // weight of neighbour i is slack_cost * decay^{idx[i]}, idx = the sorted list of indices
        // (the reference's indexing, kept). Unknown covariances (args.cov == NULL) are infinite.
        if (lane < nnb) {
            int nbi;
            if (grid_mode) {
                nbi = nb_scratch.idx[lane];
            } else {
                nbi = args.nb_col[nb0 + lane];
                asm volatile("" : "+v"(nbi));  // (the two reads kept apart: merged, one flat load)
            }
            const double* cv = args.cov ? args.cov + (size_t)nbi * 3 : nullptr;
            slk->dist[lane] = cv ? distance_to_ellipse(s0[0], s0[1], args.states[(size_t)nbi * 6],
                                                       args.states[(size_t)nbi * 6 + 1], cv[0], cv[1], cv[2])
                                 : -5.0;
        }
        wave_lds_sync();
        if (lane < nnb) {
            const double di = slk->dist[lane];
            int rank = 0;
            for (int j = 0; j < nnb; j++) {
                const double dj = slk->dist[j];
                rank += (dj < di || (dj == di && j < lane)) ? 1 : 0;
            }
            slk->order[rank] = lane;
        }
        wave_lds_sync();
        if (lane < nnb) slk->w[lane] = op.slack_cost * pow(op.slack_decay, (double)slk->order[lane]);
        wave_lds_sync();
    }
    PHSTAMP(2);

    bool have_curve = false, success = true;
    const PdipCfg cfg{op.maxit, op.tol};
    const int C = op.C;
    const FovBorder fborder{op.fov_kap, op.fov_sig, op.fov_none != 0};  // (fov_border, host)

    for (int it = 0; it < op.impc_iter; it++) {
        // (keeps the operator tables' loads inside the iteration: hoisted out of it they stay live
        // across the solves and spill)
        asm volatile("" ::: "memory");
        const size_t oi = (size_t)ai * op.impc_iter + it;
        if (!success) {
            write_iteration(args, oi, lane, ST_UNKNOWN, __builtin_nan(""), 0);
            continue;
        }
        // ---- Voronoi rows: rows mb .. mb + nnb*C - 1, the same in every iteration: formed in
        // iteration 0 and kept in the image (the solves never write rows below the FoV rows)
        const int nvor = nnb * C;
        for (int v = lane; v < nvor && it == 0; v += 64) {
            const int i = v / C, j = v % C;
            // control point j's operator rows first (they do not depend on the neighbour; behind
            // its position and the row's arithmetic they were three dependent round trips)
            const double* VZ = opp(buf, op.o_VZ) + (size_t)j * 2 * NZ;
            const double* VS = opp(buf, op.o_VS) + (size_t)j * 12;
            const double* M = opp(buf, op.o_wvor) + 3 * j;  // g P^-1 g = (nx, ny) M (nx, ny)^T
            double vz[2 * NZ], vs[12], mw[3];
#pragma unroll
            for (int k = 0; k < 2 * NZ; k++) vz[k] = VZ[k];
#pragma unroll
            for (int k = 0; k < 12; k++) vs[k] = VS[k];
#pragma unroll
            for (int k = 0; k < 3; k++) mw[k] = M[k];
            __builtin_amdgcn_sched_barrier(0);
            double ox, oy, nx, ny, off;
            nb_position(args, nb_scratch, grid_mode, nb0, i, ox, oy);
            voronoi_row(s0[0], s0[1], ox, oy, op.bbox[0], op.bbox[1], nx, ny, off);
            const int r = mb + v;
            double sh = 0.0;
#pragma unroll
            for (int k = 0; k < 6; k++) sh = fma(nx * vs[k] + ny * vs[6 + k], s0[k], sh);
#pragma unroll
            for (int jz = 0; jz < NZ; jz++) Gimg[r * WNZ + jz] = nx * vz[jz] + ny * vz[NZ + jz];
            Gimg[r * WNZ + NZ] = 0.0;
            rlo[r] = 0.0;
            rml[r] = 0.0;
            rhi[r] = -off - 1e-8 - sh;
            nfin_fixed = nfin_fixed || !(fma(nx, 0.0, ny * 0.0) + (off + sh) * 0.0 == 0.0);
            was.wn[r] = rsqrtf((float)fmax(fma(nx, fma(mw[0], nx, 2.0 * mw[1] * ny), mw[2] * ny * ny), 1e-30));
        }
        // ---- FoV CBF rows, compacted after the Voronoi rows
        const int nk = (it == 0) ? 1 : op.cbf_h;
        const int base = mb + nvor;
        int count = 0;
        bool row_infeasible = false;
        const double* UZ = uz_s;
        const double* US = us_s;
        const int ntask = nnb * 4 * nk;
        if (it > 0) {
            // the ego state at each CBF sample (the previous curve at h_samples(k)), once per sample:
            // lane 6 k + s forms component s of sample k (ConnectivityIMPCCBF.cpp:161-168)
            if (lane < 6 * nk && nk <= 2) {
                const int k = lane / 6, c = lane - 6 * k;
                const double* PZ = opp(buf, op.o_PZ) + (size_t)k * 6 * NZ + c * NZ;
                const double* PS = opp(buf, op.o_PS) + (size_t)k * 36 + c * 6;
                double ps[6], pz[NZ];  // (loaded together, then the sums)
#pragma unroll
                for (int u = 0; u < 6; u++) ps[u] = PS[u];
#pragma unroll
                for (int j = 0; j < NZ; j++) pz[j] = PZ[j];
                __builtin_amdgcn_sched_barrier(0);
                double v = 0.0;
#pragma unroll
                for (int u = 0; u < 6; u++) v = fma(ps[u], s0[u], v);
#pragma unroll
                for (int j = 0; j < NZ; j++) v = fma(pz[j], ykeep_s[j], v);
                ego_s[k][c] = v;
            }
            wave_lds_sync();
        }
        bool nfin_it = false;
        if constexpr (SLACK) {
            // slack mode: neighbour i's rows go to lanes 8 i .. 8 i + 7 of the slack images
            // (WaveSlack), uncompacted; every row starts inert, pads stay zero
            for (int e = lane; e < WSL_ROWS * WNZ; e += 64) slk->Go[e] = 0.0;
            slk->zvs[lane] = 0.0;
            slk->h[lane] = 1.0;
            slk->live[lane] = 0.0;
            wave_lds_sync();
        }
        for (int t0 = 0; t0 < ntask; t0 += 64) {
            const int task = t0 + lane;
            bool keep = false;
            double a[3] = {0.0, 0.0, 0.0}, bb = 0.0, us[3] = {0.0, 0.0, 0.0};
            int k = 0, i = 0, kind = 0;
            if (task < ntask) {
                // order of FovBezierIMPCCBF.cpp:150-210: per neighbour, per kind, per k
                i = task / (4 * nk);
                kind = (task / nk) % 4;
                k = task % nk;
                double e[6], npx, npy;
                nb_position(args, nb_scratch, grid_mode, nb0, i, npx, npy);
                if (it == 0 || nk > 2) {
                    double yk[NZ];
#pragma unroll
                    for (int j = 0; j < NZ; j++) yk[j] = ykeep_s[j];
                    cbf_ego_state<NZ>(op, buf, it, k, s0, yk, e);
                } else {
#pragma unroll
                    for (int c = 0; c < 6; c++) e[c] = ego_s[k][c];
                }
                bool present;
                fov_cbf_row(kind, e, npx, npy, fborder, op.fov_Ds, op.fov_Rs, a, bb, present);
                double bmax = 0.0, bmin = 0.0;
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    const double v1 = -a[d] * op.a_lo[d], v2 = -a[d] * op.a_hi[d];
                    bmax += fmax(v1, v2);
                    bmin += fmin(v1, v2);
                }
                keep = present && !(op.cbf_filter && bb >= bmax);  // (exact: v >= 0 only relaxes)
                if (!SLACK && present && bb < bmin - op.feas_tol) row_infeasible = true;
                const double* USk = US + (size_t)k * 18;
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    double v = 0.0;
#pragma unroll
                    for (int s = 0; s < 6; s++) v = fma(USk[d * 6 + s], s0[s], v);
                    us[d] = v;
                }
            }
            if constexpr (SLACK) {
                if (keep) {
                    const int r = 8 * i + kind * nk + k;
                    const double* UZk = UZ + (size_t)k * 3 * NZ;
#pragma unroll
                    for (int jz = 0; jz < NZ; jz++)
                        slk->Go[r * WNZ + jz] = -(a[0] * UZk[jz] + a[1] * UZk[NZ + jz] + a[2] * UZk[2 * NZ + jz]);
                    slk->h[r] = bb + a[0] * us[0] + a[1] * us[1] + a[2] * us[2];
                    slk->live[r] = 1.0;
                }
                continue;
            }
            const unsigned long long msk = __ballot(keep);
            const int slot = count + __popcll(msk & ((1ull << lane) - 1ull));
            if (keep && base + slot < WROWS) {
                const int r = base + slot;
                const double* UZk = UZ + (size_t)k * 3 * NZ;
#pragma unroll
                for (int jz = 0; jz < NZ; jz++)
                    Gimg[r * WNZ + jz] = -(a[0] * UZk[jz] + a[1] * UZk[NZ + jz] + a[2] * UZk[2 * NZ + jz]);
                Gimg[r * WNZ + NZ] = 0.0;
                rlo[r] = 0.0;
                rml[r] = 0.0;
                const double hr = bb + a[0] * us[0] + a[1] * us[1] + a[2] * us[2];
                rhi[r] = hr;
                nfin_it = nfin_it || !(fma(a[0], 0.0, fma(a[1], 0.0, a[2] * 0.0)) + hr * 0.0 == 0.0);
                const double* M = mf_s + 6 * k;  // g P^-1 g = a^T M_k a
                const double n2 = a[0] * (M[0] * a[0] + 2.0 * (M[1] * a[1] + M[2] * a[2])) +
                                  a[1] * (M[3] * a[1] + 2.0 * M[4] * a[2]) + a[2] * M[5] * a[2];
                was.wn[r] = rsqrtf((float)fmax(n2, 1e-30));
            }
            count += __popcll(msk);
        }
        row_infeasible = __ballot(row_infeasible) != 0ull;
        const int mtot = base + count;
        const int nchunk = ((mtot + 15) / 16) * 4;  // whole groups of 4 chunks (WCH = 48 is one)
        // zero the image rows that complete the last chunk; slack mode: also the slack image
        // (centred + mean rows, WSL_CROWS from row 4 nchunk) and its weights
        const int zend = SLACK ? 4 * nchunk + WSL_CROWS : 4 * nchunk;
        for (int r = mtot + lane; r < zend && r < WROWS; r += 64) {
#pragma unroll
            for (int j = 0; j < WNZ; j++) Gimg[r * WNZ + j] = 0.0;
            if (SLACK && r >= 4 * nchunk) {
                sc.Dv[r] = 0.0;
                sc.wv[r] = 0.0;
                sc.cv[r] = 0.0;
            }
        }
        if (lane < WNZ) sc.q[lane] = q_s[lane];
        wave_lds_sync();
        if (it < 2) PHSTAMP(3 + 2 * it);
        int st;
        int nit = 0;
        double prs = __builtin_nan(""), drs = __builtin_nan("");
        double vobj = 0.0;  // slack mode: sum_i w_i v_i (addSlackCost, MPCCBFQPGeneratorBase.cpp:121-130)
        // non-finite data (a NaN / Inf state, target or neighbour position): not solved, ERROR
        bool nfin = nfin_fixed || nfin_it;
        if constexpr (SLACK) {  // the slack rows (lane = row) and the neighbours' slack weights
            if (slk->live[lane] != 0.0) {
                nfin = nfin || !isfinite(slk->h[lane]);
                for (int j = 0; j < WNZ; j++) nfin = nfin || !isfinite(slk->Go[lane * WNZ + j]);
            }
            nfin = nfin || ((lane >> 3) < nnb && !isfinite(slk->w[lane >> 3]));
        }
        if (mtot > WROWS || nb_overflow || (SLACK && 4 * nchunk + WSL_CROWS > WROWS) || __ballot(nfin) != 0ull) {
            st = ST_ERROR;  // capacity (rows per agent / observed neighbours) / non-finite data
        } else if (infeasible || row_infeasible) {
            st = ST_INFEASIBLE;
        } else {
            // the row slots of the first mr image rows
            // (re-read at every use: the compiler would otherwise keep the slots live across solves)
            auto image_rows = [&](int mr) {
                asm volatile("" ::: "memory");
                WaveRows rw;
#pragma unroll
                for (int s = 0; s < WR; s++) {
                    const int r = wave_owner_row(lane, s);
                    const bool on = r < mr;
                    rw.g[s] = on ? &Gimg[r * WNZ] : zero_row;
                    rw.lo[s] = on ? rlo[r] : -1.0;
                    rw.hi[s] = on ? rhi[r] : 1.0;
                    rw.ml[s] = on ? rml[r] : 1.0;
                }
                return rw;
            };
#ifdef MPCCBF_PDIP_STAMPS
            long long* dbg = (args.stamps && it == 0)
                                 ? (long long*)args.stamps + (size_t)args.num_agents * NSTAMP + (size_t)ai * 16
                                 : nullptr;
#elif defined(MPCCBF_DEBUG_TRACE)  // per-iteration trace of the last IMPC iteration's solve
            long long* dbg = (args.stamps && it == op.impc_iter - 1)
                                 ? (long long*)args.stamps + (size_t)args.num_agents * NSTAMP + (size_t)ai * 512
                                 : nullptr;
#else
            long long* dbg = nullptr;
#endif
            // first attempt: the dual active-set solve; a QP it finds without a feasible point goes
            // to phase 1 directly, one it gives up on to the PDIP
            int das = 0, dsteps = 0;
            double drp = 0.0, drd = 0.0, dtlow = 0.0;
            // slack mode: the dual active set on a hard-row QP per slack pattern. Neighbour i is
            // either at v_i = 0 (its FoV rows hard: g_a y <= h_a) or, with a leader row l, at
            // v_i = g_l y - h_l >= 0: w_i g_l joins the linear term, its other rows become
            // (g_a - g_l) y <= h_a - h_l and row l the bound g_l y >= h_l. A solve is the slack
            // QP's optimum when every neighbour's multipliers are consistent (stationarity in
            // v_i: at v_i = 0 the FoV multipliers sum to at most w_i; with a leader, its own
            // multiplier w_i - sum(others) - mu_i is >= 0). All start at v = 0; a neighbour
            // over its cost takes its largest-multiplier row as leader, one with a negative
            // leader multiplier the next-largest. A pattern without a feasible point relaxes a
            // FoV row of its infeasibility certificate: the unreachable candidate when it is a
            // slack row (it leads its neighbour), else the certificate's active slack row of
            // largest weight whose neighbour has no leader. After SLK_PATTERNS patterns, or
            // when no rule applies, the slack PDIP solves.
#ifndef MPCCBF_SLK_PATTERNS
#define MPCCBF_SLK_PATTERNS 8
#endif
            constexpr int SLK_PATTERNS = MPCCBF_SLK_PATTERNS;
            bool lv = false, pattern_ok = false;
            int ncbf = 0, c_me = 0;
            if constexpr (SLACK) {
                lv = slk->live[lane] != 0.0;
                const unsigned long long lm = __ballot(lv);
                ncbf = __popcll(lm);
                c_me = __popcll(lm & ((1ull << lane) - 1ull));
                if (lane < WSL_NB) slk->lead[lane] = -1;
                pattern_ok = op.dual_as > 0 && mtot + ncbf <= WROWS;
            }
            auto run_patterns = [&](int npat) -> int {
                if constexpr (!SLACK) {
                    (void)npat;
                    return 0;
                } else {
                int res = 0, tot_steps = 0;
                for (int pat = 0; pat < npat; pat++) {
                    wave_lds_sync();
                    const int ld = slk->lead[lane >> 3];
                    if (lv) {
                        const int r = mtot + c_me;
                        const double* go = slk->Go + lane * WNZ;
                        const double* gl_ = slk->Go + (ld < 0 ? lane : ld) * WNZ;
                        const bool diff = ld >= 0 && ld != lane;
#pragma unroll
                        for (int j = 0; j < WNZ; j++) Gimg[r * WNZ + j] = diff ? go[j] - gl_[j] : go[j];
                        const bool lead_row = ld == lane;
                        rlo[r] = lead_row ? slk->h[lane] : 0.0;
                        rml[r] = lead_row ? 1.0 : 0.0;
                        rhi[r] = lead_row ? 1e300 : (diff ? slk->h[lane] - slk->h[ld] : slk->h[lane]);
                    }
                    if (lane < WNZ) {  // q + sum over led neighbours of w_i g_l
                        double qv = q_s[lane];
                        for (int g = 0; g < nnb; g++) {
                            const int l = slk->lead[g];
                            if (l >= 0) qv = fma(slk->w[g], slk->Go[l * WNZ + lane], qv);
                        }
                        sc.q[lane] = qv;
                    }
                    wave_lds_sync();
                    int st_ = 0, cand = -1;
                    const int d = das_solve_wave<false>(image_rows(mtot + ncbf), Gimg, sc, was, opp(buf, op.o_P16),
                                                 opp(buf, op.o_Pinv16), op.tol, 2 * op.dual_as,
                                                 args.dual_res != nullptr, lane, drp, drd, st_, dtlow, &cand,
                                                 mtot, mtot + ncbf);
                    tot_steps += st_;
                    if (d < 0) {
                        // no feasible point with this pattern: a FoV row of the certificate
                        // takes the slack (wave-uniform choice, every lane scans the same LDS)
                        int pick = -1;
                        if (cand >= mtot) {
                            const int sl = slk->rowl[cand - mtot];
                            if (slk->lead[sl >> 3] != sl) pick = sl;  // (not the leader's own bound)
                        } else {
                            double best = 0.0;
                            for (int a = 0; a < was.k; a++) {
                                const int r = was.row[a];
                                if (r < mtot || was.sg[a] < 0.0) continue;
                                const int sl = slk->rowl[r - mtot];
                                if (slk->lead[sl >> 3] < 0 && was.u[a] > best) best = was.u[a], pick = sl;
                            }
                        }
                        if (pick < 0) break;
                        wave_lds_sync();
                        if (lane == 0) slk->lead[pick >> 3] = pick;
                        continue;
                    }
                    if (d != 1) break;
                    wave_lds_sync();
                    // per neighbour (lane g < nnb): multipliers of its upper sides, of its leader's
                    // bound, and its largest-multiplier active rows other than the leader
                    bool bad = false;
                    int pick = -1;
                    if (lane < nnb) {
                        const int l = slk->lead[lane];
                        double lam = 0.0, mu = 0.0, best = -1.0;
                        for (int a = 0; a < was.k; a++) {
                            const int r = was.row[a];
                            if (r < mtot) continue;
                            const int sl = slk->rowl[r - mtot];
                            if ((sl >> 3) != lane) continue;
                            const double ua = was.u[a];
                            if (was.sg[a] < 0.0) {
                                mu += ua;  // the leader's bound v_i >= 0
                            } else {
                                lam += ua;
                                if (sl != l && ua > best) best = ua, pick = sl;
                            }
                        }
                        bad = l < 0 ? !(lam <= slk->w[lane]) : !(slk->w[lane] - lam - mu >= 0.0);
                    }
                    const unsigned long long badm = __ballot(bad);
                    if (badm == 0ull) {
                        // consistent: v_i = g_l y - h_l for led neighbours, the cost into the objective
                        double vw = 0.0;
                        if (lane < nnb) {
                            const int l = slk->lead[lane];
                            if (l >= 0) vw = slk->w[lane] * (dotl(slk->Go + l * WNZ, sc.y) - slk->h[l]);
                        }
                        vobj = wave_reduce<Op::Sum>(vw);
                        res = 1;
                        break;
                    }
                    if (__ballot(bad && pick < 0) != 0ull) break;  // no row to lead: the PDIP
                    wave_lds_sync();
                    if (bad) slk->lead[lane] = pick;
                }
                dsteps += tot_steps;
                if (res != 1) {
                    vobj = 0.0;
                    for (int e = lane; e < ncbf * WNZ; e += 64) Gimg[mtot * WNZ + e] = 0.0;
                    if (lane < WNZ) sc.q[lane] = q_s[lane];
                    wave_lds_sync();
                }
                return res;
            }
            };
            auto polish = [&]() -> bool {
                if constexpr (!SLACK) {
                    return false;
                } else {
                // the slack PDIP's solution fixes the pattern — neighbour i with v_i > 0 leads with
                // its row of largest excess g_r y - h_r — and one active-set solve of that pattern
                // (plus one exchange) returns its exact optimum, which replaces the interior
                // point's when consistent (the PDIP's tolerance, priced at slack-cost-sized
                // multipliers, otherwise shows in the objective)
                if (!pattern_ok) return false;
                wave_lds_sync();
                const double vi = slk->st[lane];  // (WaveSlack::st row 0: this lane's neighbour's v)
                const double ex = lv ? dotl(slk->Go + lane * WNZ, sc.y) - slk->h[lane] : -1e300;
                // segment argmax of the excess (8 lanes per neighbour)
                double m = ex;
                m = fmax(m, dpp_mov<DPP_XOR1>(m));
                m = fmax(m, dpp_mov<DPP_XOR2>(m));
                m = fmax(m, dpp_mov<DPP_HALF_MIRROR>(m));
                const unsigned long long hit = __ballot(lv && ex == m);
                const unsigned long long seg = 0xFFull << (lane & ~7);
                const int lead = __ffsll((long long)(hit & seg)) - 1;
                if (lane < WNZ) ypd[lane] = sc.y[lane];
                wave_lds_sync();
                if ((lane & 7) == 0 && (lane >> 3) < nnb)
                    slk->lead[lane >> 3] = (vi > 1e-9 && lead >= 0) ? lead : -1;
                const int r = run_patterns(2);
                if (r != 1 && lane < WNZ) sc.y[lane] = ypd[lane];  // keep the interior point's
                wave_lds_sync();
                return r == 1;
            }
            };
            if constexpr (!SLACK) {
                if (op.dual_as > 0)
                    das = das_solve_wave(image_rows(mtot), Gimg, sc, was, opp(buf, op.o_P16), opp(buf, op.o_Pinv16),
                                         op.tol, 2 * op.dual_as, args.dual_res != nullptr, lane, drp, drd, dsteps,
                                         dtlow, nullptr, mtot, mtot, dbg, args.primal_res != nullptr);
            } else if (pattern_ok) {
                if (lv) slk->rowl[c_me] = lane;
                das = run_patterns(SLK_PATTERNS);
            }
            WaveSlack sk{};
            if constexpr (SLACK) {
                wave_lds_sync();  // the slack rows written above
                sk.Go = slk->Go;
                sk.coff = 4 * nchunk;
                sk.Gc = Gimg + (size_t)sk.coff * WNZ;
                sk.Dvs = sc.Dv + sk.coff;
                sk.wvs = sc.wv + sk.coff;
                sk.cvs = sc.cv + sk.coff;
                sk.zvs = slk->zvs;
                sk.Tn = slk->Tn;
                sk.st = slk->st;
                sk.nnb = nnb;
                sk.nchunk_c = ((9 * nnb + 15) / 16) * 4;
                sk.nchunk_o = ((8 * nnb + 15) / 16) * 4;
                sk.h = slk->h[lane];
                sk.live = slk->live[lane];
                sk.w = (lane >> 3) < nnb ? slk->w[lane >> 3] : 0.0;
            }
            bool settled = false;
            if (das == 1) {
                st = ST_OPTIMAL;
                nit = dsteps;
                prs = drp;
                drs = drd;
                settled = true;
            } else if (das < 0 && dtlow > 10.0 * op.feas_tol) {
                // the active set's infeasibility certificate bounds t* from below: no phase 1
                st = ST_INFEASIBLE;
                nit = dsteps;
                prs = dtlow;
                settled = true;
            } else if (das < 0) {
                const double tstar = pdip_phase1_wave(image_rows(mtot), Gimg, nchunk, sc, NZ, cfg, lane);
                if (tstar > op.feas_tol && tstar < 1e300) {  // (1e300: phase 1 failed, the PDIP decides)
                    st = ST_INFEASIBLE;
                    nit = dsteps;
                    prs = tstar;
                    settled = true;
                }
            }
            if (!settled) {
                const PdipOut po = pdip_solve_wave<SLACK>(image_rows(mtot), Gimg, nchunk, sc, opp(buf, op.o_P16),
                                                          opp(buf, op.o_LP16), cfg, lane, dbg, &sk, &vobj);
                st = po.status;
                nit = dsteps + po.iters;
                prs = po.rp;
                drs = po.rd;
                if (SLACK && st == ST_OPTIMAL) {
                    double vkeep = vobj;
                    if (polish()) {  // the pattern's exact optimum (sc.y, drp / drd, vobj)
                        prs = drp;
                        drs = drd;
                    } else {
                        vobj = vkeep;
                    }
                }
                // slack mode: the slack rows are always satisfiable, phase 1 certifies the box and
                // Voronoi rows (the ordinary image)
                if (st != ST_OPTIMAL) {
                    const double tstar = pdip_phase1_wave(image_rows(mtot), Gimg, nchunk, sc, NZ, cfg, lane);
                    if (tstar > op.feas_tol) {
                        st = ST_INFEASIBLE;
                        prs = tstar;
                    }
                }
            }
        }
        double objv = __builtin_nan("");
        if (st == ST_OPTIMAL) {
            // 1/2 y^T P y + q^T y + k on the row layout: (P y)_i from P's row in LDS (lane i)
            const int i16 = lane & 15;
            double pyi = 0.0;
#pragma unroll
            for (int j = 0; j < WNZ; j++) pyi = fma(was.P[i16 * 17 + j], sc.y[j], pyi);
            const double term = i16 < NZ ? sc.y[i16] * fma(0.5, pyi, q_s[i16]) : 0.0;
            objv = grp_sum<16>(term) + kconst_s + vobj;
            wave_lds_sync();
            if (lane < NZ) ykeep_s[lane] = sc.y[lane];
            have_curve = true;
        } else {
            success = false;
        }
        write_iteration(args, oi, lane, st, objv, nit, prs, drs);
        if (it < 2) PHSTAMP(4 + 2 * it);
        wave_lds_sync();
    }
    {
        double yk[NZ];
#pragma unroll
        for (int j = 0; j < NZ; j++) yk[j] = ykeep_s[j];
        write_agent_outputs<NZ, 64, !SLACK, false>(op, buf, args, ai, lane, s0, yk, have_curve);
    }
    // (diagnostics; here, not after the query: there it pushed the kernel into scratch)
    write_nb_out(args, ai, lane, grid_mode, nb_scratch, nb0, nnb);
    stamp(args, ai, lane, 7);
}

// The FoV controller's per-neighbour rows for `count` (ego, neighbour) pairs, evaluated by the same
// device functions the IMPC kernel uses (mpccbf_fov_rows_eval): Voronoi (nx, ny, 0, off) and the
// four FoV HOCBF rows (a0, a1, a2, b; safety, left, right, range; b = DBL_MAX when absent).
__global__ void __launch_bounds__(64) fov_rows_eval_kernel(int count, const double* __restrict__ ego,
                                                           const double* __restrict__ nb, double fov, double Ds,
                                                           double Rs, double bbx, double bby,
                                                           double* __restrict__ vor, double* __restrict__ rows) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= count) return;
    double e[6];
#pragma unroll
    for (int k = 0; k < 6; k++) e[k] = ego[(size_t)i * 6 + k];
    const double ox = nb[(size_t)i * 2], oy = nb[(size_t)i * 2 + 1];
    if (vor) {
        double nx, ny, off;
        voronoi_row(e[0], e[1], ox, oy, bbx, bby, nx, ny, off);
        vor[(size_t)i * 4 + 0] = nx;
        vor[(size_t)i * 4 + 1] = ny;
        vor[(size_t)i * 4 + 2] = 0.0;
        vor[(size_t)i * 4 + 3] = off;
    }
    if (rows) {
        for (int kind = 0; kind < 4; kind++) {
            double a[3], b;
            bool present;
            fov_cbf_row(kind, e, ox, oy, fov, Ds, Rs, a, b, present);
            double* r = rows + ((size_t)i * 4 + kind) * 4;
            r[0] = a[0];
            r[1] = a[1];
            r[2] = a[2];
            r[3] = b;
        }
    }
}

}  // namespace dev

hipError_t launch_fov_rows_eval(int count, const double* ego, const double* nb, double fov, double Ds, double Rs,
                                double bbx, double bby, double* vor, double* rows, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(dev::fov_rows_eval_kernel, dim3((count + 63) / 64), dim3(64), 0, s, count, ego, nb, fov, Ds,
                       Rs, bbx, bby, vor, rows);
    return hipGetLastError();
}

hipError_t launch_impc_fov(const DevOps& op, const double* buf, const ImpcArgs& a, hipStream_t s) {
    if (a.num_agents <= 0) return hipSuccess;
    if (op.nz != 15 || op.m > dev::WROWS) return hipErrorInvalidValue;
    if (op.slack_mode) {
        if (op.cbf_h > 2) return hipErrorInvalidValue;  // 4 kinds x cbf_h rows per 8-lane segment
        hipLaunchKernelGGL(dev::impc_fov_kernel<true>, dim3(a.num_agents), dim3(64), 0, s, op, buf, a);
    } else {
        hipLaunchKernelGGL(dev::impc_fov_kernel<false>, dim3(a.num_agents), dim3(64), 0, s, op, buf, a);
    }
    return hipGetLastError();
}

}  // namespace mpccbf
