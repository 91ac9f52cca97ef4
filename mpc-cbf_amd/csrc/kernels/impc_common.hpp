// impc_common.hpp — device steps shared by the IMPC kernels (impc_kernel.hip, impc_fov.hip):
// the collision HOCBF row, the in-kernel neighbour query, the state-dependent linear term, the
// constant-row check, CBF-row staging, objective and output writes, diagnostics stamps.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#include "group.hpp"
#include "impc.hpp"

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
    int32_t src[NB_CAP];   // final neighbour i -> its candidate slot
    double cst[4][NB_CAP];  // candidates' (px, py, vx, vy), read once by the query for the CBF rows
};

// Broadcast of lane K's 32-bit value within a 16-lane DPP row (row_newbcast).
template <int K>
__device__ __forceinline__ int row_bcast_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xF, 0xF, true);
}

// (d_a, j_a) before (d_b, j_b): nearer first, ties by agent index
__device__ __forceinline__ bool nb_before(double da, int ja, double db, int jb) {
    return da < db || (da == db && ja < jb);
}

// The query of grid_neighbors when more than NB_CAP candidates lie within the radius (crowds, the
// reference's all-(N-1) semantics at short range): no cap — the candidate list (hs, nc, off,
// total, full as grid_neighbors built them) is streamed 16 entries at a time through a running
// k-nearest set: lane l of each 16-lane row holds the l-th nearest so far; a chunk's candidates
// within the radius and the kept set are ranked against each other by DPP row broadcasts and the
// first k go back to the lanes by rank (through sc's first NB_MAX entries). Leaves the k nearest
// in sc.idx / sc.cst[.] positions 0 .. nk-1 sorted by agent index (sc.src[p] = p); returns nk.
// G = 64: the four rows of the wave run the same query redundantly.
template <int G>
__device__ __forceinline__ int grid_neighbors_stream(const ImpcArgs& args, int self, double px, double py,
                                                  NbScratch& sc, int gl, double yaw, const uint32_t (&hs)[9],
                                                  const uint32_t (&nc)[9], const uint32_t (&off)[9], uint32_t total,
                                                  bool full) {
    static_assert(G == 16 || G == 64, "16-lane rows");
    const int l = gl & 15;
    const GridArgs& gr = args.grid;
    const double r2 = gr.radius * gr.radius;
    const int k = gr.k < NB_MAX ? gr.k : NB_MAX;
    // the kept set (lane l: the l-th nearest so far; unused: (1e300, INT_MAX))
    double kd = 1e300, kx = 0.0, ky = 0.0, kvx = 0.0, kvy = 0.0;
    int kj = 0x7fffffff, nk = 0;
    for (uint32_t t0 = 0; t0 < total; t0 += 16) {
        const uint32_t t = t0 + l;
        bool keep = false;
        int j = 0x7fffffff;
        double d2 = 1e300, nx = 0.0, ny = 0.0, nvx = 0.0, nvy = 0.0;
        if (t < total) {
            if (full) {
                j = (int)t;
            } else {
                uint32_t e = 0;
#pragma unroll
                for (int c = 0; c < 9; c++)  // the cell whose range holds t
                    if (off[c] <= t && t - off[c] < nc[c]) e = grid_slot_at(hs[c], t - off[c]);
                j = (int)gr.slots[e];
            }
            nx = args.states[(size_t)j * 6];
            ny = args.states[(size_t)j * 6 + 1];
            nvx = args.states[(size_t)j * 6 + 3];
            nvy = args.states[(size_t)j * 6 + 4];
            const double ex = nx - px;
            const double ey = ny - py;
            const double dd = ex * ex + ey * ey;
            keep = (j != self) && (dd <= r2);
            if (keep && gr.cone > 0.0) {  // inside the field of view (strict)
                double offa = atan2(ey, ex) - yaw;
                offa -= 6.283185307179586 * rint(offa * 0.15915494309189535);
                keep = fabs(offa) < gr.cone;
            }
            d2 = dd;
        }
        const unsigned long long msk = grp_ballot<16>(keep);
        if (msk == 0ull) continue;
        const double dn = keep ? d2 : 1e300;
        const int jn = keep ? j : 0x7fffffff;
        // ranks in (kept set) U (this chunk's candidates); the kept set is sorted, so a kept entry
        // is preceded by the l kept entries before it and by the candidates nearer than it
        int r_old = l, r_new = 0;
        auto rank_step = [&](double dm, int jm, double dk, int jk) {
            r_old += nb_before(dm, jm, kd, kj) ? 1 : 0;
            r_new += (nb_before(dm, jm, dn, jn) ? 1 : 0) + (nb_before(dk, jk, dn, jn) ? 1 : 0);
        };
#define MPCCBF_NB_RANK(K) \
    rank_step(row_bcast_k<K>(dn), row_bcast_i<K>(jn), row_bcast_k<K>(kd), row_bcast_i<K>(kj));
        // (scheduling barriers every four broadcasts: hoisted together, the 64 broadcast values
        // would stay live at once)
        MPCCBF_NB_RANK(0) MPCCBF_NB_RANK(1) MPCCBF_NB_RANK(2) MPCCBF_NB_RANK(3)
        __builtin_amdgcn_sched_barrier(0);
        MPCCBF_NB_RANK(4) MPCCBF_NB_RANK(5) MPCCBF_NB_RANK(6) MPCCBF_NB_RANK(7)
        __builtin_amdgcn_sched_barrier(0);
        MPCCBF_NB_RANK(8) MPCCBF_NB_RANK(9) MPCCBF_NB_RANK(10) MPCCBF_NB_RANK(11)
        __builtin_amdgcn_sched_barrier(0);
        MPCCBF_NB_RANK(12) MPCCBF_NB_RANK(13) MPCCBF_NB_RANK(14) MPCCBF_NB_RANK(15)
#undef MPCCBF_NB_RANK
        wave_lds_sync();  // the previous chunk's reads of the buffer are done
        auto put = [&](int s, int jj, double dd, double x, double y, double vx, double vy) {
            sc.idx[s] = jj;
            sc.d2[s] = dd;
            sc.cst[0][s] = x;
            sc.cst[1][s] = y;
            sc.cst[2][s] = vx;
            sc.cst[3][s] = vy;
        };
        if (l < nk && r_old < k) put(r_old, kj, kd, kx, ky, kvx, kvy);
        if (keep && r_new < k) put(r_new, jn, dn, nx, ny, nvx, nvy);
        nk += __popcll(msk);
        nk = nk < k ? nk : k;
        wave_lds_sync();
        if (l < nk) {
            kj = sc.idx[l];
            kd = sc.d2[l];
            kx = sc.cst[0][l];
            ky = sc.cst[1][l];
            kvx = sc.cst[2][l];
            kvy = sc.cst[3][l];
        }
    }
    // the kept set ordered by agent index: position = kept entries with a smaller index
    int pos = 0;
#define MPCCBF_NB_POS(K) pos += row_bcast_i<K>(kj) < kj ? 1 : 0;
    MPCCBF_NB_POS(0) MPCCBF_NB_POS(1) MPCCBF_NB_POS(2) MPCCBF_NB_POS(3)
    MPCCBF_NB_POS(4) MPCCBF_NB_POS(5) MPCCBF_NB_POS(6) MPCCBF_NB_POS(7)
    MPCCBF_NB_POS(8) MPCCBF_NB_POS(9) MPCCBF_NB_POS(10) MPCCBF_NB_POS(11)
    MPCCBF_NB_POS(12) MPCCBF_NB_POS(13) MPCCBF_NB_POS(14) MPCCBF_NB_POS(15)
#undef MPCCBF_NB_POS
    wave_lds_sync();
    if (l < nk) {
        sc.idx[pos] = kj;
        sc.src[pos] = pos;
        sc.d2[pos] = kd;
        sc.cst[0][pos] = kx;
        sc.cst[1][pos] = ky;
        sc.cst[2][pos] = kvx;
        sc.cst[3][pos] = kvy;
    }
    wave_lds_sync();
    return nk;
}

// The neighbour query in stages, so that its dependent global round trips (the 9 cells' bucket
// counts, then the first pass's bucket slots, then those candidates' states) can be issued between
// the setup's own loads instead of after them: gq_begin (counts), gq_slots (the candidate list and
// the first pass's slots), gq_states (the first pass's states), then grid_neighbors_finish.
// The first pass covers candidates gl and G + gl (G = 16) or gl (G = 64).
template <int G>
struct GridQuery {
    static constexpr int NP = G == 16 ? 2 : 1;
    uint32_t hs[9], nc[9], off[9], total;
    bool full;
    int j[NP];           // first pass: raw slot entry (gq_slots), then the candidate agent (-1: none)
    double st[NP][4];    // its (px, py, vx, vy)
};

template <int G>
__device__ __forceinline__ void gq_begin(const ImpcArgs& args, double px, double py, GridQuery<G>& q) {
    const GridArgs& gr = args.grid;
    const long long cx = (long long)floor(px * gr.inv_cell), cy = (long long)floor(py * gr.inv_cell);
#pragma unroll
    for (int c = 0; c < 9; c++) {
        q.hs[c] = cell_hash(cx + (c % 3) - 1, cy + (c / 3) - 1, gr.mask);
        q.nc[c] = gr.cnt[q.hs[c]];
    }
}

// candidate t's entry in the slot table (entry 0 when unused: the slot loads are unconditional —
// behind a branch, the join waited for them)
template <int G>
__device__ __forceinline__ uint32_t gq_entry(const GridArgs& gr, const GridQuery<G>& q, uint32_t t) {
    uint32_t e = 0;
#pragma unroll
    for (int c = 0; c < 9; c++) {  // the cell whose range holds t
        const uint32_t u = t - q.off[c];
        e = ((q.off[c] <= t) & (u < q.nc[c])) ? grid_slot_at(q.hs[c], u) : e;
    }
    return (t < q.total && !q.full) ? e : 0u;
}

// candidate t's agent from its raw slot entry: the entry, or t itself when scanning the whole
// table (-1: none)
template <int G>
__device__ __forceinline__ int gq_agent(const GridQuery<G>& q, uint32_t t, int raw) {
    return t >= q.total ? -1 : (q.full ? (int)t : raw);
}

template <int G>
__device__ __forceinline__ void gq_slots(const ImpcArgs& args, GridQuery<G>& q, int gl) {
    // a bucket that overflowed its slots: scan the whole state table instead (same result); a
    // bucket reached from two of the 9 cells is scanned once
    bool full = false;
    uint32_t total = 0;
#pragma unroll
    for (int c = 0; c < 9; c++) {
        full = full || q.nc[c] > (uint32_t)GRID_CAP;
        bool dup = false;
#pragma unroll
        for (int p = 0; p < c; p++) dup = dup || (q.hs[p] == q.hs[c]);
        if (dup) q.nc[c] = 0;
        q.off[c] = total;
        total += q.nc[c];
    }
    q.full = full;
    q.total = full ? (uint32_t)args.num_states : total;
    // every pass's entry first, then the loads (their results stay in flight until gq_states)
    uint32_t e[GridQuery<G>::NP];
#pragma unroll
    for (int p = 0; p < GridQuery<G>::NP; p++) e[p] = gq_entry<G>(args.grid, q, (uint32_t)(p * G + gl));
#pragma unroll
    for (int p = 0; p < GridQuery<G>::NP; p++) q.j[p] = (int)args.grid.slots[e[p]];
}

template <int G>
__device__ __forceinline__ void gq_states(const ImpcArgs& args, GridQuery<G>& q, int gl) {
#pragma unroll
    for (int p = 0; p < GridQuery<G>::NP; p++) {
        q.j[p] = gq_agent<G>(q, (uint32_t)(p * G + gl), q.j[p]);
        const size_t r = (size_t)(q.j[p] >= 0 ? q.j[p] : 0) * 6;
        q.st[p][0] = args.states[r];
        q.st[p][1] = args.states[r + 1];
        q.st[p][2] = args.states[r + 3];
        q.st[p][3] = args.states[r + 4];
    }
}

// k nearest other agents (planar distance, ties by index) within the radius, found through the
// spatial hash (q: the staged query's first pass, gq_*); the result is left in sc.idx sorted by
// agent index (sc.src: each one's slot in sc.cst). Returns the count. Up to NB_CAP candidates
// within the radius are gathered and ranked at once; beyond, grid_neighbors_stream re-runs the
// query without a cap. Distance-only test: agents of a colliding cell that share a bucket are
// still filtered by distance.
template <int G>
__device__ int grid_neighbors_finish(const ImpcArgs& args, int self, double px, double py, NbScratch& sc,
                                     int gl, double yaw, GridQuery<G>& q) {
    const GridArgs& gr = args.grid;
    const double r2 = gr.radius * gr.radius;
    const uint32_t total = q.total;
    int cnt = 0;
    // whether candidate j at (nx, ny) is a neighbour (within the radius and, for the FoV
    // controller, the cone); d2: its squared distance
    auto is_nb = [&](int j, double nx, double ny, double& d2) -> bool {
        const double ex = nx - px;
        const double ey = ny - py;
        d2 = ex * ex + ey * ey;
        bool keep = j >= 0 && (j != self) && (d2 <= r2);
        if (keep && gr.cone > 0.0) {  // inside the field of view (strict)
            double offa = atan2(ey, ex) - yaw;
            offa -= 6.283185307179586 * rint(offa * 0.15915494309189535);
            keep = fabs(offa) < gr.cone;
        }
        return keep;
    };
    // compaction of one chunk of G candidates into sc (in candidate order)
    auto put_chunk = [&](bool keep, int j, double d2, double nx, double ny, double nvx, double nvy) {
        const unsigned long long msk = grp_ballot<G>(keep);
        const int slot = cnt + __popcll(msk & ((1ull << gl) - 1ull));
        if (keep && slot < NB_CAP) {
            sc.idx[slot] = j;
            sc.d2[slot] = d2;
            sc.cst[0][slot] = nx;
            sc.cst[1][slot] = ny;
            sc.cst[2][slot] = nvx;
            sc.cst[3][slot] = nvy;
        }
        cnt += __popcll(msk);
    };
    constexpr int NP = GridQuery<G>::NP;
    // the first pass from the staged loads
#pragma unroll
    for (int p = 0; p < NP; p++) {
        double d2;
        const bool keep = is_nb(q.j[p], q.st[p][0], q.st[p][1], d2);
        put_chunk(keep, q.j[p], d2, q.st[p][0], q.st[p][1], q.st[p][2], q.st[p][3]);
    }
    // the rest, NP chunks per pass: the chunks' dependent loads (bucket slot, then the agent's
    // state) are in flight together
    for (uint32_t t0 = NP * G; t0 < total; t0 += NP * G) {
        int j[NP];
        double st[NP][4];
#pragma unroll
        for (int p = 0; p < NP; p++) j[p] = (int)gq_entry<G>(gr, q, t0 + p * G + gl);
#pragma unroll
        for (int p = 0; p < NP; p++) j[p] = (int)gr.slots[(uint32_t)j[p]];
#pragma unroll
        for (int p = 0; p < NP; p++) j[p] = gq_agent<G>(q, t0 + p * G + gl, j[p]);
#pragma unroll
        for (int p = 0; p < NP; p++) {
            const size_t r = (size_t)(j[p] >= 0 ? j[p] : 0) * 6;
            st[p][0] = args.states[r];
            st[p][1] = args.states[r + 1];
            st[p][2] = args.states[r + 3];
            st[p][3] = args.states[r + 4];
        }
#pragma unroll
        for (int p = 0; p < NP; p++) {
            double d2;
            const bool keep = is_nb(j[p], st[p][0], st[p][1], d2);
            put_chunk(keep, j[p], d2, st[p][0], st[p][1], st[p][2], st[p][3]);
        }
    }
    if (cnt > NB_CAP)
        return grid_neighbors_stream<G>(args, self, px, py, sc, gl, yaw, q.hs, q.nc, q.off, total, q.full);
    wave_lds_sync();
    // rank by (d2, index): keep the k nearest
    const int k = gr.k;
    const int nk = cnt < k ? cnt : k;
    if constexpr (G == 16) {
        if (cnt <= 2 * G) {
            // two candidates per lane (slots gl, gl + 16) compared against all by DPP row
            // broadcasts, in registers; then ordered by agent index the same way
            const bool v0 = gl < cnt, v1 = gl + G < cnt;
            const double d0 = v0 ? sc.d2[gl] : 1e300, d1 = v1 ? sc.d2[gl + G] : 1e300;
            const int j0 = v0 ? sc.idx[gl] : 0x7fffffff, j1 = v1 ? sc.idx[gl + G] : 0x7fffffff;
            int r0 = 0, r1 = 0;
            auto rank_step = [&](double dm, int jm) {
                r0 += nb_before(dm, jm, d0, j0) ? 1 : 0;
                r1 += nb_before(dm, jm, d1, j1) ? 1 : 0;
            };
#define MPCCBF_NB_RANK(K)                                           \
    rank_step(row_bcast_k<K>(d0), row_bcast_i<K>(j0));              \
    rank_step(row_bcast_k<K>(d1), row_bcast_i<K>(j1));
            MPCCBF_NB_RANK(0) MPCCBF_NB_RANK(1) MPCCBF_NB_RANK(2) MPCCBF_NB_RANK(3)
            MPCCBF_NB_RANK(4) MPCCBF_NB_RANK(5) MPCCBF_NB_RANK(6) MPCCBF_NB_RANK(7)
            MPCCBF_NB_RANK(8) MPCCBF_NB_RANK(9) MPCCBF_NB_RANK(10) MPCCBF_NB_RANK(11)
            MPCCBF_NB_RANK(12) MPCCBF_NB_RANK(13) MPCCBF_NB_RANK(14) MPCCBF_NB_RANK(15)
#undef MPCCBF_NB_RANK
            const bool k0 = v0 && r0 < k, k1 = v1 && r1 < k;
            // order the kept set by agent index: position = kept candidates with a smaller index
            const int jk0 = k0 ? j0 : 0x7fffffff, jk1 = k1 ? j1 : 0x7fffffff;
            int p0 = 0, p1 = 0;
            auto pos_step = [&](int jm) {
                p0 += jm < j0 ? 1 : 0;
                p1 += jm < j1 ? 1 : 0;
            };
#define MPCCBF_NB_POS(K) pos_step(row_bcast_i<K>(jk0)); pos_step(row_bcast_i<K>(jk1));
            MPCCBF_NB_POS(0) MPCCBF_NB_POS(1) MPCCBF_NB_POS(2) MPCCBF_NB_POS(3)
            MPCCBF_NB_POS(4) MPCCBF_NB_POS(5) MPCCBF_NB_POS(6) MPCCBF_NB_POS(7)
            MPCCBF_NB_POS(8) MPCCBF_NB_POS(9) MPCCBF_NB_POS(10) MPCCBF_NB_POS(11)
            MPCCBF_NB_POS(12) MPCCBF_NB_POS(13) MPCCBF_NB_POS(14) MPCCBF_NB_POS(15)
#undef MPCCBF_NB_POS
            wave_lds_sync();  // every lane has read its candidates
            if (k0) {
                sc.idx[p0] = j0;
                sc.src[p0] = gl;
            }
            if (k1) {
                sc.idx[p1] = j1;
                sc.src[p1] = gl + G;
            }
            wave_lds_sync();
            return nk;
        }
    }
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
    wave_lds_sync();
    // order the kept set by agent index
    for (int i = gl; i < cnt; i += G) {
        if (sc.keep[i]) {
            const int ji = sc.idx[i];
            int pos = 0;
            for (int m = 0; m < cnt; m++) pos += (sc.keep[m] && sc.idx[m] < ji) ? 1 : 0;
            sc.tmp[pos] = ji;
            sc.src[pos] = i;
        }
    }
    wave_lds_sync();
    for (int i = gl; i < nk; i += G) sc.idx[i] = sc.tmp[i];
    wave_lds_sync();
    return nk;
}

// the whole query in one call (no setup loads to overlap)
template <int G>
__device__ __forceinline__ int grid_neighbors(const ImpcArgs& args, int self, double px, double py, NbScratch& sc,
                                              int gl, double yaw = 0.0) {
    GridQuery<G> q;
    gq_begin<G>(args, px, py, q);
    gq_slots<G>(args, q, gl);
    gq_states<G>(args, q, gl);
    return grid_neighbors_finish<G>(args, self, px, py, sc, gl, yaw, q);
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

// agent_linear_term spread over the group's lanes: lane i < NZ forms q_i (the same sums in the
// same order as agent_linear_term), lanes 0 .. 5 and 6 .. 8 (targets) or 6 .. G-1 (reference
// tail) the objective constant's terms, summed over the group. Every operator entry is a vector
// load issued at once (the one-lane form serialised ~12 scalar-cache round trips). Returns this
// lane's q_i (0 beyond NZ) and the constant (every lane).
template <int NZ, int G>
__device__ __forceinline__ double agent_linear_term_lanes(const DevOps& op, const double* buf,
                                                          const ImpcArgs& args, int ai, const double (&s0)[6],
                                                          int gl, double& kconst) {
    static_assert(NZ <= G && G >= 9, "one lane per linear-term entry");
    const int i = gl < NZ ? gl : 0;
    // constant: s0^T Ks s0 + t^T Kt s0 — lane s < 6: s0_s (Ks s0)_s; lane 6 + d: t_d (Kt s0)_d
    const int sr = gl < 6 ? gl : 0;
    const int dr = (gl >= 6 && gl < 9) ? gl - 6 : 0;
    double s0s = s0[0];
#pragma unroll
    for (int k = 1; k < 6; k++) s0s = sr == k ? s0[k] : s0s;
    if (args.targets) {
        // every load first (a scheduling barrier keeps them ahead of the arithmetic: interleaved,
        // each group of loads waited for the previous one)
        double qs[6], qt[3], t[3], kr[6];
        const double* Qs = opp(buf, op.o_Qs) + (size_t)i * 6;
        const double* Qt = opp(buf, op.o_Qt) + (size_t)i * 3;
        const double* Kr = gl < 6 ? opp(buf, op.o_Ks) + (size_t)sr * 6 : opp(buf, op.o_Kt) + (size_t)dr * 6;
#pragma unroll
        for (int s = 0; s < 6; s++) qs[s] = Qs[s];
#pragma unroll
        for (int d = 0; d < 3; d++) qt[d] = Qt[d];
#pragma unroll
        for (int d = 0; d < 3; d++) t[d] = args.targets[(size_t)ai * 3 + d];
#pragma unroll
        for (int u = 0; u < 6; u++) kr[u] = Kr[u];
        __builtin_amdgcn_sched_barrier(0);
        double q = 0.0;
#pragma unroll
        for (int s = 0; s < 6; s++) q = fma(qs[s], s0[s], q);
#pragma unroll
        for (int d = 0; d < 3; d++) q = fma(qt[d], t[d], q);
        double v = 0.0;
#pragma unroll
        for (int u = 0; u < 6; u++) v = fma(kr[u], s0[u], v);
        const double td = dr == 0 ? t[0] : (dr == 1 ? t[1] : t[2]);
        const double kc = gl < 6 ? s0s * v : (gl < 9 ? td * v : 0.0);
        kconst = grp_sum<G>(kc);
        return gl < NZ ? q : 0.0;
    }
    // reference-tail form (refs): + Qr r, + r^T Kr s0 (lanes 6 .. G-1: entries j = gl - 6,
    // gl - 6 + (G - 6), ...)
    const double* Qs = opp(buf, op.o_Qs) + (size_t)i * 6;
    double q = 0.0;
#pragma unroll
    for (int s = 0; s < 6; s++) q = fma(Qs[s], s0[s], q);
    double kc = 0.0;
    {
        const double* Ks = opp(buf, op.o_Ks) + (size_t)sr * 6;
        double v = 0.0;
#pragma unroll
        for (int u = 0; u < 6; u++) v = fma(Ks[u], s0[u], v);
        kc = gl < 6 ? s0s * v : 0.0;
    }
    const double* Qr = opp(buf, op.o_Qr);
    const double* Kr = opp(buf, op.o_Kr);
    const int nr = 3 * op.spd_f;
    const double* rt = args.refs + (size_t)ai * 3 * op.K + 3 * (op.K - op.spd_f);
    // (8 entries' loads at a time, indices clamped: as a plain loop each entry's two loads were
    // waited for before the next entry's issued)
    for (int j0 = 0; j0 < nr; j0 += 8) {
        double qa[8], ra[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int j = j0 + u < nr ? j0 + u : nr - 1;
            qa[u] = Qr[(size_t)i * nr + j];
            ra[u] = rt[j];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) q = j0 + u < nr ? fma(qa[u], ra[u], q) : q;
    }
    for (int j = gl - 6; gl >= 6 && j < nr; j += G - 6) {
        double v = 0.0;
#pragma unroll
        for (int s = 0; s < 6; s++) v = fma(Kr[j * 6 + s], s0[s], v);
        kc = fma(rt[j], v, kc);
    }
    kconst = grp_sum<G>(kc);
    return gl < NZ ? q : 0.0;
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
        // (bounds loaded with the row: the short-circuit test loaded chi after clo, after Cs)
        const double lo = clo[i], hi = chi[i];
        double v = 0.0;
#pragma unroll
        for (int s = 0; s < 6; s++) v = fma(Cs[i * 6 + s], s0[s], v);
        bad = bad | (v < lo - op.feas_tol) | (v > hi + op.feas_tol);
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
                              const NbScratch* nbs, int nb0, int nnb, double* stage, int cap, int gl,
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
                double npx, npy, nvx, nvy;
                if (grid_mode) {  // read by the neighbour query (LDS)
                    const int c = nbs->src[j];
                    npx = nbs->cst[0][c];
                    npy = nbs->cst[1][c];
                    nvx = nbs->cst[2][c];
                    nvy = nbs->cst[3][c];
                } else {
                    const double* ns = args.states + (size_t)args.nb_col[nb0 + j] * 6;
                    npx = ns[0];
                    npy = ns[1];
                    nvx = ns[3];
                    nvy = ns[4];
                    // (keeps the two branches' reads apart: merged, the LDS and global reads
                    // became one flat load through a selected pointer)
                    asm volatile("" : "+v"(npx), "+v"(npy), "+v"(nvx), "+v"(nvy));
                }
                safety_cbf(e, npx, npy, nvx, nvy, op.d_min, a, b);
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

// The same rows in one pass over the (sample, neighbour) pairs (16-lane groups, the separable
// kernel): lane p of a pass takes sample k0 + p / nnb and neighbour p % nnb, so iteration 1's two
// samples fill one pass where stage_cbf_rows makes one per sample with half the lanes idle. The
// samples' ego states and U_k s0 terms are formed once per group into smp (up to 3 samples at a
// time: lane 6 k + s the state, lane 18 + 3 k + d the U_k s0 term, 27 doubles) with the same
// arithmetic as cbf_ego_state, and the pairs go in the same sample-major order: the staged rows
// are bit-identical to stage_cbf_rows'.
template <int NZ>
__device__ int stage_cbf_rows_pairs(const DevOps& op, const double* buf, const ImpcArgs& args, int it,
                                    const double (&s0)[6], const double (&y)[NZ], bool grid_mode,
                                    const NbScratch* nbs, int nb0, int nnb, double* stage, int cap, int gl,
                                    bool* infeasible, double* smp) {
    constexpr int G = 16, KC = 3;
    const double* UZ = opp(buf, op.o_UZ);
    const double* US = opp(buf, op.o_US);
    const int nk = (it == 0) ? 1 : op.cbf_h;
    int count = 0;
    bool row_infeasible = false;
    for (int k0 = 0; k0 < nk; k0 += KC) {
        const int kn = nk - k0 < KC ? nk - k0 : KC;
        wave_lds_sync();  // (the previous chunk's reads of smp are done)
        for (int t = gl; t < 27; t += G) {
            const bool st = t < 18;
            const int kk = st ? t / 6 : (t - 18) / 3;
            if (kk >= kn) continue;
            const int k = k0 + kk;
            double v = 0.0;
            if (st) {
                const int sr = t - 6 * kk;
                if (it == 0) {
#pragma unroll
                    for (int u = 0; u < 6; u++) v = u == sr ? s0[u] : v;
                } else {
                    const double* PS = opp(buf, op.o_PS) + (size_t)k * 36 + (size_t)sr * 6;
                    const double* PZ = opp(buf, op.o_PZ) + (size_t)k * 6 * NZ + (size_t)sr * NZ;
#pragma unroll
                    for (int u = 0; u < 6; u++) v = fma(PS[u], s0[u], v);
#pragma unroll
                    for (int jz = 0; jz < NZ; jz++) v = fma(PZ[jz], y[jz], v);
                }
            } else {
                const int d = t - 18 - 3 * kk;
                const double* USkd = US + (size_t)k * 18 + (size_t)d * 6;
#pragma unroll
                for (int u = 0; u < 6; u++) v = fma(USkd[u], s0[u], v);
            }
            smp[t] = v;
        }
        wave_lds_sync();
        const int np = kn * nnb;
        for (int base = 0; base < np; base += G) {
            const int p = base + gl;
            int kk = 0;
            for (int c = 1; c < KC; c++) kk += p >= c * nnb ? 1 : 0;
            const int j = p - kk * nnb;
            bool keep = false;
            double a[3] = {0.0, 0.0, 0.0}, b = 0.0;
            if (p < np) {
                double e[6];
#pragma unroll
                for (int sr = 0; sr < 6; sr++) e[sr] = smp[6 * kk + sr];
                double npx, npy, nvx, nvy;
                if (grid_mode) {
                    const int c = nbs->src[j];
                    npx = nbs->cst[0][c];
                    npy = nbs->cst[1][c];
                    nvx = nbs->cst[2][c];
                    nvy = nbs->cst[3][c];
                } else {
                    const double* ns = args.states + (size_t)args.nb_col[nb0 + j] * 6;
                    npx = ns[0];
                    npy = ns[1];
                    nvx = ns[3];
                    nvy = ns[4];
                    // (keeps the two branches' reads apart: merged, the LDS and global reads
                    // became one flat load through a selected pointer)
                    asm volatile("" : "+v"(npx), "+v"(npy), "+v"(nvx), "+v"(nvy));
                }
                safety_cbf(e, npx, npy, nvx, nvy, op.d_min, a, b);
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
                const double* UZk = UZ + (size_t)(k0 + kk) * 3 * NZ;  // (this lane's sample)
#pragma unroll
                for (int jz = 0; jz < NZ; jz++)
                    dst[jz] = -(a[0] * UZk[jz] + a[1] * UZk[NZ + jz] + a[2] * UZk[2 * NZ + jz]);
                dst[NZ] = b + (a[0] * smp[18 + 3 * kk] + a[1] * smp[18 + 3 * kk + 1] + a[2] * smp[18 + 3 * kk + 2]);
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

// Counter-based normal samples for the closed-loop noise (math::addRandomNoise draws from a
// std::mt19937 seeded by std::random_device, i.e. irreproducibly; here every sample is a pure
// function of (seed, step, agent, component) so runs repeat): splitmix64 + Box-Muller.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// sub: control sub-step counted back from the last one (0 = the last draw of the step)
__device__ __forceinline__ double normal_sample(uint64_t seed, int64_t step, int64_t agent, int comp,
                                                int sub = 0) {
    uint64_t k = mix64(seed);
    k = mix64(k ^ (uint64_t)step);
    k = mix64(k ^ ((uint64_t)agent * 8u + (uint64_t)comp));
    if (sub > 0) k = mix64(k ^ ((uint64_t)sub << 40));
    const double u1 = (double)((k >> 11) + 1) * 0x1.0p-53;  // (0, 1]
    const double u2 = (double)(mix64(k) >> 11) * 0x1.0p-53;
    return sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
}

// The closed-loop noise draws of the kept curve's next state (normal_sample(..., comp, 0), comp =
// lane < 6), formed at the start of the agent (they depend on the seed, step and agent alone: the
// transcendental chain overlaps the setup's loads instead of closing the agent) into noise0[0..6)
__device__ __forceinline__ void early_noise(const ImpcArgs& args, int ai, int gl, double* noise0) {
    if (args.traj_t == nullptr || gl >= 6) return;
    const double sd = gl < 3 ? args.pos_std : args.vel_std;
    if (sd > 0.0) noise0[gl] = normal_sample(args.noise_seed, args.step_index, args.agent_first + ai, gl);
}

// Component comp (0..2 position x/y/yaw, 3..5 velocity) at parameter t of a piecewise Bezier
// curve (SingleParameterPiecewiseCurve::eval, SingleParameterPiecewiseCurve.cpp:94-127:
// lower_bound piece lookup, local parameter min(T, t - cum[i-1]); Bezier::eval with the
// monomial Bernstein basis). The control points come from xrow (stored curve) or, when xrow is
// null, from x = Xs s0 + Z y of this step's solution.
// CC > 0: the control points per piece as a compile-time constant (op.C == CC; every loop unrolls,
// so the piece's operator rows are loaded together instead of one dependent round trip per
// control point); CC = 0: op.C at run time. The piece index counts the cumulative parameters below
// t (branch-free over at most 8 pieces, else the loop).
template <int NZ, int CC = 0>
__device__ double curve_component(const DevOps& op, const double* buf, const double* xrow,
                                  const double (&s0)[6], const double (&yk)[NZ], double t, int comp) {
    const double* cum = opp(buf, op.o_cum);
    int piece = 0;
    if (op.P <= 8) {
#pragma unroll
        for (int p = 0; p < 7; p++) {
            const double c = cum[p < op.P - 1 ? p : 0];
            piece += (p < op.P - 1 && c < t) ? 1 : 0;
        }
    } else {
        while (piece < op.P - 1 && cum[piece] < t) piece++;
    }
    const double par = piece == 0 ? t : fmin(cum[0], t - cum[piece - 1]);
    const int d = comp % 3;
    const double* EB = opp(buf, comp < 3 ? op.o_EB0 : op.o_EB1);
    const double* Z = opp(buf, op.o_Z);
    const double* Xs = opp(buf, op.o_Xs);
    const int C = CC > 0 ? CC : op.C;
    double v = 0.0;
    for (int cp = 0; cp < C; cp++) {  // (constant trip count when CC > 0: unrolled)
        const int idx = piece * 3 * C + d * C + cp;
        double xv;
        if (xrow) {
            xv = xrow[idx];
        } else {
            xv = 0.0;
#pragma unroll
            for (int s = 0; s < 6; s++) xv = fma(Xs[idx * 6 + s], s0[s], xv);
#pragma unroll
            for (int j = 0; j < NZ; j++) xv = fma(Z[idx * NZ + j], yk[j], xv);
        }
        double b = 0.0, tp = 1.0;
        for (int j = 0; j < C; j++, tp *= par) b = fma(EB[cp * C + j], tp, b);
        v = fma(xv, b, v);
    }
    return v;
}

template <int NZ, bool FIXED = true>
__device__ __forceinline__ double curve_component_any(const DevOps& op, const double* buf, const double* xrow,
                                                      const double (&s0)[6], const double (&yk)[NZ], double t,
                                                      int comp) {
    if constexpr (FIXED)
        if (op.C == 4) return curve_component<NZ, 4>(op, buf, xrow, s0, yk, t, comp);
    return curve_component<NZ, 0>(op, buf, xrow, s0, yk, t, comp);
}

// Control points of the kept curve and the closed-loop next state.
//   default: x = this step's curve (NaN if none), next state = that curve at t = h, or the
//            current state when optimize() produced no curve;
//   args.traj_t set (closed-loop simulator, MPCCBFFormationControl_example.cpp:150-221): x is
//            the persistent last successful curve, next state = it at the advanced time.
// FIXED: the curve evaluation's compile-time control-point count (C = 4) when it applies (off for the
// FoV slack kernel, whose registers it pushes into scratch); AZE: a fresh curve's next state from the
// AZ / AS rows when DevOps::az_at_eval (off in the FoV kernels, where it costs scratch)
template <int NZ, int G, bool FIXED = true, bool AZE = true>
__device__ __forceinline__ void write_agent_outputs(const DevOps& op, const double* buf,
                                                    const ImpcArgs& args, int ai, int gl,
                                                    const double (&s0)[6], const double (&yk)[NZ],
                                                    bool have_curve, const double* noise0 = nullptr) {
    const bool sim = args.traj_t != nullptr;
    const double t_stored = sim ? args.traj_t[ai] : 0.0;  // (loaded here: in flight during the x rows)
    // this step's control points x = Xs s0 + Z y to args.x, XU rows per lane at a time (their loads
    // in flight together; one row at a time, each row's loads waited for the previous row's)
    // (staging them in LDS for the curve evaluation below, with its piece lookup from the kernel
    // arguments, measured slower: 0.15 us per agent)
    const bool want_x = args.x && (have_curve || !sim);
    if (want_x && !have_curve) {
        for (int i = gl; i < op.n; i += G) args.x[(size_t)ai * op.n + i] = __builtin_nan("");
    } else if (want_x) {
        const double* Z = opp(buf, op.o_Z);
        const double* Xs = opp(buf, op.o_Xs);
        constexpr int XU = (64 + G - 1) / G;
        for (int i0 = 0; i0 < op.n; i0 += XU * G) {
            double v[XU];
#pragma unroll
            for (int u = 0; u < XU; u++) {
                const int i = i0 + u * G + gl;
                const int ic = i < op.n ? i : 0;
                double a = 0.0;
#pragma unroll
                for (int s = 0; s < 6; s++) a = fma(Xs[ic * 6 + s], s0[s], a);
#pragma unroll
                for (int j = 0; j < NZ; j++) a = fma(Z[ic * NZ + j], yk[j], a);
                v[u] = a;
            }
#pragma unroll
            for (int u = 0; u < XU; u++) {
                const int i = i0 + u * G + gl;
                if (i < op.n) args.x[(size_t)ai * op.n + i] = v[u];
            }
        }
    }
    if (gl >= 6) return;
    double v = 0.0;
    const double sd = gl < 3 ? args.pos_std : args.vel_std;
    const int64_t agent = args.agent_first + ai;
    if (sim) {
        const double t_prev = have_curve ? 0.0 : t_stored;
        double t_new = t_prev;
        const double tmax = opp(buf, op.o_cum)[op.P - 1];
        if (have_curve || t_prev >= 0.0) {
            t_new = fmin(t_prev + op.eval_step, tmax);  // example :190-193
            const double* xr = have_curve ? nullptr : args.x + (size_t)ai * op.n;
            if (AZE && have_curve && op.az_at_eval) {
                // a fresh curve at min(eval_step, T_end) = min(h, T_end): the AZ / AS rows
                const double* AZ = opp(buf, op.o_AZ);
                const double* AS = opp(buf, op.o_AS);
#pragma unroll
                for (int s = 0; s < 6; s++) v = fma(AS[gl * 6 + s], s0[s], v);
#pragma unroll
                for (int j = 0; j < NZ; j++) v = fma(AZ[gl * NZ + j], yk[j], v);
            } else {
                v = curve_component_any<NZ, FIXED>(op, buf, xr, s0, yk, t_new, gl);
            }
            if (args.substeps) {  // sub-steps 1 .. nsub - 1: the curve at t_prev + Ts k, own draws
                for (int k = 1; k < op.nsub; k++) {
                    double u = curve_component_any<NZ, FIXED>(op, buf, xr, s0, yk, fmin(t_prev + op.Ts * k, tmax), gl);
                    if (sd > 0.0) u = fma(sd, normal_sample(args.noise_seed, args.step_index, agent, gl, op.nsub - k), u);
                    args.substeps[((size_t)ai * op.nsub + k - 1) * 6 + gl] = u;
                }
            }
            if (sd > 0.0)
                v = fma(sd, noise0 != nullptr ? noise0[gl] : normal_sample(args.noise_seed, args.step_index, agent, gl), v);
        } else {
            // no trajectory yet: hold the position at zero velocity, with each sub-step's noise
            // added to the previous sub-step's state (example :210-216): the position draws
            // accumulate, the velocity keeps the last one
            double p = 0.0;
#pragma unroll
            for (int s = 0; s < 3; s++)
                if (s == gl) p = s0[s];
            for (int k = 1; k <= op.nsub; k++) {
                const double n = sd > 0.0 ? sd * normal_sample(args.noise_seed, args.step_index, agent, gl, op.nsub - k) : 0.0;
                p = gl < 3 ? p + n : n;
                if (args.substeps && k < op.nsub) args.substeps[((size_t)ai * op.nsub + k - 1) * 6 + gl] = p;
            }
            v = p;
        }
        if (gl == 0) args.traj_t[ai] = t_new;  // every lane read t_prev above (same wave)
    } else {
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
        if (sd > 0.0) v = fma(sd, normal_sample(args.noise_seed, args.step_index, agent, gl), v);
    }
    if (args.substeps) args.substeps[((size_t)ai * op.nsub + op.nsub - 1) * 6 + gl] = v;
    if (args.next_states) args.next_states[(size_t)ai * 6 + gl] = v;
    if (args.grid.ins_cnt) {  // the next step's neighbour table gets this row (lanes 0, 1, 3, 4)
        const int base = (int)(threadIdx.x & 63u) & ~(G - 1);
        const double y = __shfl(v, base + 1, 64), vx = __shfl(v, base + 3, 64), vy = __shfl(v, base + 4, 64);
        if (gl == 0) grid_insert(args.grid, v, y, vx, vy, (uint32_t)(args.agent_first + ai));
    }
}

// XCD-aware block order: workgroups are dispatched round-robin over the 8 XCDs (block b runs on
// XCD b % 8), each with its own L2. Block b takes logical block xcd_block(b) so that every XCD
// gets one contiguous range of the batch: consecutive agents are spatial neighbours (the swarms are
// laid out in lattice / heading order and the hash table by cell), so an XCD's neighbour-state and
// bucket reads stay mostly inside its own range instead of every XCD's L2 fetching the whole state
// table each step. A bijection of [0, gridDim.x).
__host__ __device__ __forceinline__ int xcd_block(int b, int nb) {
    const int q = nb >> 3, r = nb & 7;
    const int x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

// the bucket counts of the table two steps ahead are zeroed by the launch's threads, and the other
// step parity's defer-queue header by block 0 (called by every thread before any early exit).
// NT: the launch's block size as a constant — blockDim.x is a 16-bit field of the dispatch packet,
// fetched with a vector load whose wait put one memory round trip at the head of every launch.
template <int NT>
__device__ __forceinline__ void grid_clear(const ImpcArgs& args) {
    if (args.defer_clear && blockIdx.x == 0 && threadIdx.x == 0) args.defer_clear[0] = 0;
    if (!args.grid.clr_cnt) return;
    const uint32_t T = args.grid.mask + 1u;
    const uint32_t nthr = gridDim.x * (uint32_t)NT;
    for (uint32_t e = blockIdx.x * (uint32_t)NT + threadIdx.x; e < T; e += nthr) args.grid.clr_cnt[e] = 0u;
}

// launch clock (ImpcArgs::kclock): every wave of the launch writes its start and end time
// (s_memrealtime, 100 MHz, chip-wide) into its own pair kclock[2 w, 2 w + 1] (w = the hardware
// block x waves per block + the wave in the block) with one 16-byte store at its end; the start
// waits in an LDS word (one per wave of the block). Plain stores to distinct words: one atomic per
// wave on a shared counter serialised ~2,000 atomics and delayed the waves' first loads. Collision
// kernels only: in the FoV kernels any clock code at the start moved the register allocation into
// 36-108 B/lane of scratch
__device__ __forceinline__ lds_vptr<unsigned long long> kclock_lds() {
    __shared__ unsigned long long t0[16];  // one per wave of a block (<= 1024 threads)
    return lds_vol(t0);
}
__device__ __forceinline__ void kclock_start(const ImpcArgs& args) {
    (void)args;
    if ((threadIdx.x & 63u) == 0) kclock_lds()[threadIdx.x >> 6] = __builtin_amdgcn_s_memrealtime();
}
template <int NT>  // the block size (as grid_clear)
__device__ __forceinline__ void kclock_end(const ImpcArgs& args) {
    if (!args.kclock || (threadIdx.x & 63u) != 0) return;
    const unsigned w = blockIdx.x * (unsigned)(NT >> 6) + (threadIdx.x >> 6);
    ulonglong2 v;
    v.x = kclock_lds()[threadIdx.x >> 6];
    // the end once the wave's own stores (outputs, table inserts) are acknowledged: the launch is
    // not over before they are
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    v.y = __builtin_amdgcn_s_memrealtime();
    reinterpret_cast<ulonglong2*>(args.kclock)[w] = v;
}

// diagnostics: wall-clock stamp (s_memrealtime, 100 MHz, chip-wide) of phase `k` of agent ai —
// compiled in the diagnostics builds only (make stamps / prof: MPCCBF_STAMPS); in the release
// kernels the stamp code kept the agent index live across the kernel and cost a 4-byte spill
__device__ __forceinline__ void stamp(const ImpcArgs& args, int ai, int gl, int k) {
#if defined(MPCCBF_STAMPS) || defined(MPCCBF_PDIP_STAMPS)
    if (args.stamps) {
        const long long t = (long long)__builtin_amdgcn_s_memrealtime();
        if (gl == 0) args.stamps[(size_t)ai * NSTAMP + k] = t;
    }
#else
    (void)args, (void)ai, (void)gl, (void)k;
#endif
}

// diagnostics (args.nb_out): the first 16 entries of the agent's neighbour list as the kernel built
// its rows from (grid mode: the query's result in LDS, sorted by index; CSR: the caller's list)
__device__ __forceinline__ void write_nb_out(const ImpcArgs& args, int ai, int gl, bool grid_mode,
                                             const NbScratch& nbs, int nb0, int nnb) {
    if (!args.nb_out || gl >= 16) return;
    int v = -1;
    if (gl < nnb) {
        if (grid_mode) {
            v = nbs.idx[gl];
        } else {
            v = args.nb_col[nb0 + gl];
            asm volatile("" : "+v"(v));  // (the two reads kept apart: merged, one flat load)
        }
    }
    args.nb_out[(size_t)ai * 16 + gl] = v;
}

__device__ __forceinline__ void write_iteration(const ImpcArgs& args, size_t oi, int gl, int st,
                                                double obj, int iters,
                                                double prs = __builtin_nan(""), double drs = __builtin_nan("")) {
    if (gl == 0) {
        if (args.status) args.status[oi] = st;
        if (args.obj) args.obj[oi] = obj;
        if (args.iters) args.iters[oi] = iters;
        if (args.primal_res) args.primal_res[oi] = prs;
        if (args.dual_res) args.dual_res[oi] = drs;
    }
}

}  // namespace dev
}  // namespace mpccbf
