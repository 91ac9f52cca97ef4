// impc.hpp — device-side layout of the condensed MPC-CBF operators and kernel arguments.
#pragma once

#include <stdint.h>

namespace mpccbf {

constexpr int MAX_CBF_H = 8;

// Offsets (in doubles) of each operator inside one device buffer (see operators.hpp).
struct DevOps {
    int32_t n, nz, m, mc, K, spd_f, cbf_h, impc_iter;
    int32_t o_Z, o_Xs, o_Pr, o_LPr, o_Qs, o_Qt, o_Qr, o_Ks, o_Kt, o_Kr;
    int32_t o_G, o_Gs, o_lo, o_hi, o_Cs, o_clo, o_chi;
    int32_t o_UZ, o_US, o_PZ, o_PS, o_AZ, o_AS;
    double a_lo[3], a_hi[3];
    double d_min;
    int32_t cbf_filter;
    int32_t maxit;
    double tol;
    double feas_tol;  // absolute row-violation tolerance for constant rows / single-row checks
    // separable layout (impc_sep_kernel): per channel d, slot k < sep_sb and lane l, row k * 16 + l
    // of channel d as [g0, g1, Gs(6), lo, hi] (SEP_ROW doubles) at ((d * sep_sb + k) * 16 + l);
    // 16 * sep_sb rows per channel (unused: inert g = 0, [-1, 1]); sep_sb = 1 up to 16 rows per
    // channel (K <= 15 at base_config.json), 2 up to 32 (K = 16 .. 31)
    int32_t sep, nzd, sep_rows_per_dim, sep_sb;
    int32_t o_Gsep;
    int32_t o_Pinv;  // separable layout: per-channel inverse 2x2 blocks of Pr, (a, b, c) x 3
    // FoV controller (cbf_mode 1, impc_fov_kernel): Voronoi operators VZ (C x 2 x nz), VS (C x 2 x 6),
    // box rows as dense 16-wide rows [g(16) | Gs(6) | lo | hi] (WBOX_ROW doubles), P and its
    // Cholesky factor padded to 16 x 16 with the identity
    int32_t cbf_mode, C;
    double fov_beta, fov_Ds, fov_Rs, bbox[3];
    double fov_kap, fov_sig;  // fov_border(fov_beta), formed on the host (a device tan per agent
    int32_t fov_none;         // was ~0.4 us on the FoV kernel's chain)
    int32_t o_VZ, o_VS, o_Wbox, o_P16, o_LP16;
    int32_t o_Pinv16;  // FoV: P^-1 padded to 16 x 16 (dual active-set solve)
    int32_t o_wbox;    // FoV: box rows' candidate weights 1 / sqrt(g P^-1 g) (dual active-set solve)
    // FoV: the P^-1 Grams of the Voronoi rows' two parts per control point (C x [xx xy yy]) and
    // of the FoV rows' three acceleration rows per CBF sample (cbf_h x [00 01 02 11 12 22]): a
    // row's weight from its few coefficients
    int32_t o_wvor, o_wfov;
    // closed-loop simulator: stored-curve evaluation (EB0 / EB1: C x C Bernstein monomials of
    // value / first derivative, cum: P cumulative piece parameters)
    int32_t P, o_EB0, o_EB1, o_cum;
    double eval_step;
    double Ts;        // control period: the driver integrates nsub = int(h / Ts) sub-steps per step
    int32_t nsub;
    // slack mode: one slack variable per neighbour; collision controller: cost
    // slack_cost * slack_decay^rank (ConnectivityIMPCCBF.cpp:73-100); FoV controller: by
    // distanceToEllipse with the reference's idx[i] indexing (FovBezierIMPCCBF.cpp:58-81)
    int32_t slack_mode;
    double slack_cost, slack_decay;
    // IMPC iteration 1 warm start (impc_sep_kernel, no slack mode): the PDIP starts from
    // iteration 0's solution with slacks and duals floored at warm_delta (0: cold start)
    double warm_delta;
    // divergence test of the first solve (PdipCfg::early_it; 0 = off)
    int32_t early_it;
    int32_t fast_start;  // PdipCfg::fast_start
    int32_t dual_as;     // PdipCfg::dual_as (first attempt)
    // separable layout: the main launch runs the fast start and the dual active set only and
    // defers agents that need the PDIP or phase 1 to the fallback launch (0: one full launch)
    int32_t lean;
    // dual active set: IMPC iteration 1 starts from iteration 0's final active set when iteration 0
    // took at least this many steps (0: always cold)
    int32_t das_warm;
    // closed-loop simulator: 1 when AZ / AS (the curve at t = min(h, T_end)) are also the curve at
    // a fresh curve's evaluation time min(eval_step, T_end), so the next state of an agent with a new
    // curve is one operator product (no piece lookup and Bernstein evaluation on the device)
    int32_t az_at_eval;
    // the operator buffer's prefix [0, hot) holds every operator of the separable collision kernels
    // (staged in LDS by impc_wide_kernel)
    int32_t hot;
    // share-adaptive layout: agents per launch up to which the one-agent-per-wave kernel is the
    // default (one wave per SIMD: 4 x the device's CUs, set per context at mpccbf_create)
    int32_t wide_max;
};

constexpr int WBOX_ROW = 16 + 6 + 2;

constexpr int SEP_ROW = 10;
constexpr int SEP_NZD_HOST = 2;  // reduced variables per channel the separable kernel handles

// Spatial hash of agent positions (uniform cells of edge `radius`) with fixed-capacity buckets:
// bucket h holds the state rows slots[h * GRID_CAP + j], j < cnt[h], in insertion order
// (bucket-major, round 6: a query touches one line of a cell's entries and two of its slot states;
// slot-major, the one-agent-per-wave query's unconditional loads of the 3 x 3 cells' 7 inline
// slots touched 63 entry lines and 63 state lines in 7 planes)
// (cnt[h] > GRID_CAP: overflow, an agent reading that bucket scans the whole state table
// instead, so the neighbour sets never depend on the capacity). Filled by atomics, so no
// scan: mpccbf_run_steps rotates three tables (read this step | filled with this step's next
// states by the IMPC kernel itself | zeroed by the IMPC kernel for the step after next).
constexpr int GRID_CAP = 64;
// The first GRID_SST slots of every bucket also carry their row's planar state (px, py, vx, vy):
// a query reads the 3 x 3 cells' counts, entries and states in one round trip (impc_wide.hpp)
constexpr int GRID_SST = 7;
constexpr int GRID_SSTR = 8;  // slot states per bucket in the state plane (GRID_SST, padded to 256 B)
// bucket h's slot j in the entry table and in the state plane (double4 index)
__host__ __device__ inline uint32_t grid_slot_at(uint32_t h, uint32_t j) { return h * (uint32_t)GRID_CAP + j; }
__host__ __device__ inline uint32_t grid_sst_at(uint32_t h, uint32_t j) { return h * (uint32_t)GRID_SSTR + j; }

struct GridArgs {
    const uint32_t* cnt;   // T bucket counts of the table read this step
    const uint32_t* slots; // T x GRID_CAP state rows (bucket-major, grid_slot_at)
    const double* sst;     // T x GRID_SSTR x 4: slot j < GRID_SST's (px, py, vx, vy) (grid_sst_at)
    uint32_t* ins_cnt;     // table of the next step (NULL: none): next_states rows are inserted
    uint32_t* ins_slots;
    double* ins_sst;
    uint32_t* clr_cnt;     // bucket counts zeroed by this launch (NULL: none)
    uint32_t mask;
    double inv_cell;
    double radius;
    int32_t k;     // keep the k nearest within radius
    double cone;   // > 0: keep only agents whose bearing is within +-cone of the ego yaw (FoV)
};

constexpr int NB_CAP = 64;  // grid mode: candidates ranked at once (more: the streaming query)
constexpr int NB_MAX = 16;  // grid mode: at most this many nearest neighbours per agent (knn_k)

// bucket of uniform cell (cx, cy) in a power-of-two hash table (mask = size - 1)
__host__ __device__ inline uint32_t cell_hash(long long cx, long long cy, uint32_t mask) {
    const uint64_t h = (uint64_t)(cx * 73856093LL) ^ (uint64_t)(cy * 19349663LL);
    return (uint32_t)(h ^ (h >> 29)) & mask;
}

// insert state row `row` at planar position (x, y), velocity (vx, vy) into the table (ins_cnt,
// ins_slots, ins_sst)
__device__ inline void grid_insert(const GridArgs& g, double x, double y, double vx, double vy, uint32_t row) {
    const uint32_t h = cell_hash((long long)floor(x * g.inv_cell), (long long)floor(y * g.inv_cell), g.mask);
    const uint32_t j = atomicAdd(&g.ins_cnt[h], 1u);
    if (j < (uint32_t)GRID_CAP) g.ins_slots[grid_slot_at(h, j)] = row;
    if (j < (uint32_t)GRID_SST) {
        double4* d = reinterpret_cast<double4*>(g.ins_sst) + grid_sst_at(h, j);
        *d = make_double4(x, y, vx, vy);
    }
}

// hash table size for n agents: power of two >= n (>= 1024)
inline uint32_t grid_table_size(int n) {
    uint32_t T = 1024;
    while (T < (uint32_t)n) T <<= 1;
    return T;
}

struct ImpcArgs {
    int32_t num_states;
    const double* states;
    int32_t agent_first;
    int32_t num_agents;
    const double* targets;
    const double* refs;  // full 3K per agent (tail used)
    const int32_t* nb_row_ptr;  // CSR mode (NULL: grid mode)
    const int32_t* nb_col;
    GridArgs grid;
    double* x;
    int32_t* status;
    double* obj;
    int32_t* iters;
    double* next_states;
    int64_t* stamps;  // diagnostics: num_agents x NSTAMP shader-clock stamps, or nullptr
    // closed-loop simulator semantics (traj_t != nullptr): x keeps the last successful curve,
    // traj_t its evaluation time (-1: none yet); Gaussian noise on the next state
    double* traj_t;
    double pos_std, vel_std;
    uint64_t noise_seed;
    int64_t step_index;
    // FoV slack weights: num_states x 3 position covariances (cxx, cxy, cyy) of the neighbour
    // estimates, or nullptr (unknown)
    const double* cov;
    // per-iteration residuals of the returned solution (PdipOut::rp / rd; INFEASIBLE: phase 1's
    // minimal violation t* and NaN), num_agents x impc_iter, or nullptr
    double* primal_res;
    double* dual_res;
    // capacity fallback (impc_sep_kernel / impc_wide_kernel): the main launch appends agents it does
    // not finish to defer ([count, -, agent...], device) and leaves their outputs to the fallback
    // launch, which solves exactly the agents in queue (the same buffer) with the full pipeline
    int32_t* defer;
    int32_t* queue;
    // the other step parity's queue header, zeroed by the main launch (block 0): the queues are
    // double-buffered by step parity, so the fallback launch never has to reset its own
    int32_t* defer_clear;
    // closed-loop simulator: the state after every control sub-step (num_agents x nsub x 6), the
    // records the example writes to states.json, or nullptr
    double* substeps;
    // diagnostics: num_agents x 16 neighbour ids as the kernel uses them (-1 padded), or nullptr
    int32_t* nb_out;
    // launch clock (mpccbf_run::kernel_clock): per wave of the launch its (start, end)
    // s_memrealtime pair (100 MHz; impc_common.hpp kclock_*), or nullptr
    unsigned long long* kclock;
};

constexpr int NSTAMP = 8;

}  // namespace mpccbf
