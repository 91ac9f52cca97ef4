/*
 * mpccbf.h — C ABI of the MI355X-native batched MPC-CBF QP solver (libmpccbf.so).
 *
 * This is the drop-in boundary that replaces the CPLEX call of the reference hot path:
 *
 *   qpcpp::Solver<double>::solve(Problem&)          workspace/lib/qpcpp/include/qpcpp/solvers/Solver.h:27-37
 *   qpcpp::CPLEXSolver<double>::solve(Problem&)     workspace/lib/qpcpp/src/solvers/CPLEX.cpp:35-177
 *   called from ConnectivityIMPCCBF::optimize        workspace/lib/mpc_cbf/src/controller/ConnectivityIMPCCBF.cpp:199-211
 *
 * Two entry families:
 *   (1) mpccbf_qp_solve_dense*: one generic dense QP in the flattened CPLEX form (what
 *       CPLEXSolver::solve builds from a qpcpp::Problem, CPLEX.cpp:52-147). The C++ adapter
 *       qpcpp::HIPSolver<double> (mpc-cbf_amd/csrc/qpcpp/) flattens a Problem into this.
 *   (2) mpccbf_create / mpccbf_impc_solve: the structured, batched path. The parameter-only
 *       operators of the MPC-CBF QP (PiecewiseBezierMPCQPOperations ctor, :9-38) are built once
 *       per context; each call runs ConnectivityIMPCCBF::optimize (ConnectivityIMPCCBF.cpp:47-215)
 *       for a whole batch of agents on the GPU: both IMPC iterations, the closed-form safety-CBF
 *       rows (ConnectivityCBF.cpp:152-198, in place of GiNaC substitution), and the QP solves.
 *
 * Conventions
 *   - All numbers are FP64 (the reference instantiates <double, 3U>).
 *   - A state is 6 doubles [px, py, yaw, vx, vy, vyaw] (model::State, DIM = 3).
 *   - Infinite bounds: any value <= -1e300 / >= 1e300 (numeric_limits<double>::lowest()/max()
 *     as used by qpcpp::Problem, Problem.h:366-372).
 *   - Solve statuses are qpcpp::SolveStatus indices (Solver.h:13-21): MPCCBF_OPTIMAL == 0 ...
 *   - Functions return MPCCBF_OK (0) or a negative error code; they never throw. The last
 *     error message of the calling thread is available from mpccbf_last_error().
 *   - Pointers in mpccbf_batch are DEVICE pointers; work is enqueued on the given hipStream_t
 *     (passed as void*; NULL = default stream) and is asynchronous. The dense-QP functions take
 *     HOST pointers and are synchronous.
 *   - One context per host thread/stream (contexts hold device buffers; not thread-safe).
 */
#ifndef MPCCBF_H
#define MPCCBF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCCBF_ABI_VERSION 12

/* qpcpp::SolveStatus (Solver.h:13-21) */
enum {
    MPCCBF_OPTIMAL = 0,
    MPCCBF_FEASIBLE = 1,
    MPCCBF_UNBOUNDED = 2,
    MPCCBF_INFEASIBLE = 3,
    MPCCBF_ERROR = 4,
    MPCCBF_UNKNOWN = 5, /* also: IMPC iteration not attempted (reference `break`, :208-211) */
    MPCCBF_INFEASIBLEORUNBOUNDED = 6
};

/* API return codes */
enum {
    MPCCBF_OK = 0,
    MPCCBF_ERR_INVALID_ARGUMENT = -1, /* std::invalid_argument / runtime_error in the reference */
    MPCCBF_ERR_HIP = -2,
    MPCCBF_ERR_CAPACITY = -3,
    MPCCBF_ERR_NO_DEVICE = -4,
    MPCCBF_ERR_INTERNAL = -5
};

/* Parameters: the JSON keys of experiments/config/base_config.json as parsed and validated by
 * common/include/common/parsing.hpp:20-214 (mpc_params, physical_limits, cbf_params, bezier_params). */
typedef struct mpccbf_params {
    double h, Ts;
    int32_t k_hor;
    double w_pos_err, w_u_eff;
    int32_t spd_f;
    double v_min[3], v_max[3], a_min[3], a_max[3];
    double d_min;
    int32_t cbf_horizon, impc_iter, slack_mode;
    double slack_cost, slack_decay_rate;
    int32_t num_pieces, num_control_points;
    double piece_max_parameter;
    int32_t continuity_upto_degree;
    /* controller family: 0 = ConnectivityIMPCCBF (collision CBF against neighbour states,
     * continuity d <= degree), 1 = FovBezierIMPCCBF (FoV CBFs against neighbour positions +
     * Voronoi rows on piece 0, continuity d < degree; FovBezierIMPCCBF.cpp:44-223) */
    int32_t cbf_mode;
    double fov_beta;  /* field of view (rad); FovCBF(fov, Ds, Rs, ...) (FovCBF.cpp:41-52) */
    double fov_Ds;    /* safety distance (the FoV example passes aligned_box[0]) */
    double fov_Rs;    /* sensing range (fov_cbf_params.Rs) */
    double bbox[3];   /* robot aligned-box half extents (Voronoi shift, math/src/Helpers.cpp:20-36) */
} mpccbf_params;

typedef struct mpccbf_ctx mpccbf_ctx;

/* Context options (all optional; zero-initialise for defaults). */
typedef struct mpccbf_options {
    int32_t device;            /* HIP device ordinal (default 0) */
    int32_t keep_redundant;    /* 1: keep every box row (no exact host-side redundancy removal) */
    int32_t no_cbf_filter;     /* 1: keep every CBF row (no exact in-kernel redundancy filter) */
    int32_t max_pdip_iters;    /* default 60 */
    double tolerance;          /* PDIP relative tolerance, default 1e-9 */
    /* Interior-point warm start of IMPC iteration 1 — used only when the dual active-set solve
     * is off (dual_as_steps < 0; by default the active set solves first and the PDIP runs cold):
     * iteration 0's primal-dual point, slacks and duals floored at warm_delta: 0 = default
     * (0.3), < 0 = cold start. A warm start that does not converge is certified by phase 1 and,
     * when the QP is feasible, re-solved cold, so statuses do not depend on it. */
    double warm_delta;
    /* Solver pipeline (ABI 10). Zero selects the default; these are the only inputs that change
     * the solver's path (no environment variable does, except in the diagnostics build). */
    int32_t dual_as_steps;     /* dual active-set step limit per QP: 0 = 24, < 0 = off (the PDIP alone) */
    int32_t no_fast_start;     /* 1: no unconstrained-minimiser fast start in the PDIP path */
    int32_t early_it;          /* PDIP divergence test from this iteration on: 0 = 10, < 0 = off */
    int32_t das_warm_steps;    /* IMPC iteration 1 starts the active set from iteration 0's when that
                                  took at least this many steps: 0 = 3, < 0 = never */
    int32_t lean;              /* 1: lean main launch (fast start + active set; the rest deferred to
                                  the fallback launch). Collision controller only */
} mpccbf_options;

/* Validates p like parsing.hpp:37-135,182-214, builds the parameter-only operators on the host
 * and uploads them. Returns MPCCBF_ERR_INVALID_ARGUMENT with the reference's message on bad
 * parameters. */
int mpccbf_create(const mpccbf_params* p, const mpccbf_options* opt, mpccbf_ctx** out);
void mpccbf_destroy(mpccbf_ctx* ctx);

/* Sizes: n = num_pieces * 3 * num_control_points decision variables (curve control points,
 * layout [piece][dim][control point], BezierQPOperations.cpp:180-204); nz = free dimension
 * after the equality constraints; rows = shared inequality rows kept after exact reduction. */
int mpccbf_num_vars(const mpccbf_ctx* ctx);
int mpccbf_reduced_dim(const mpccbf_ctx* ctx);
int mpccbf_num_shared_rows(const mpccbf_ctx* ctx);

/* One IMPC control step for a batch of agents (ConnectivityIMPCCBF::optimize per agent).
 * Inputs (device):
 *   states      num_states x 6, every agent visible to this batch (local + gathered)
 *   agent_first the batch solves agents [agent_first, agent_first + num_agents) of `states`
 *   targets     num_agents x 3: reference position replicated over the horizon
 *               (MPCCBFFormationControl_example.cpp:143-144); or NULL and give `refs`
 *   refs        num_agents x 3*k_hor full reference trajectory (ref_positions); or NULL
 *   nb_row_ptr  num_agents + 1 CSR offsets (nb_row_ptr[0] may be nonzero)
 *   nb_col      neighbour indices into `states` (the reference uses all N-1 others, :59-67)
 *   knn_k, knn_radius   used when nb_row_ptr is NULL: the neighbours of each agent are its
 *               knn_k nearest others (planar) within knn_radius, found on the device in the same
 *               launch sequence (spatial hash of `states` + in-kernel 3x3-cell query; in
 *               mpccbf_run_steps the IMPC kernel itself fills the next step's hash table);
 *               knn_k <= 16; any number of agents within the radius (beyond 64 candidates the
 *               query streams them through a running k-nearest set)
 *               Capacity: the default separable kernel keeps up to 16 live (unfiltered) CBF rows
 *               per IMPC iteration and agent (slack mode: 16 neighbours); an agent beyond it is
 *               re-solved in the same call by the fallback launch of the same separable solver
 *               with 8 CBF row slots per lane (128 rows; slack mode: the neighbours with a live
 *               row compacted into the 16 lanes); beyond that its QPs report ERROR. A QP whose
 *               data is not finite (NaN / Inf state, target or neighbour state) reports ERROR
 * Outputs (device, any may be NULL):
 *   x           num_agents x n: control points of the last OPTIMAL iteration (the curve the
 *               driver keeps, example :160-164); NaN if no iteration was OPTIMAL
 *   status      num_agents x impc_iter SolveStatus per IMPC iteration (UNKNOWN = not attempted)
 *   obj         num_agents x impc_iter optimal objective x^T H x + c^T x (CPLEX.cpp:144-146)
 *   iters       num_agents x impc_iter solver steps of that QP: dual active-set steps plus the
 *               interior-point Newton steps of every PDIP attempt (when the active-set solve
 *               gives up, or in slack mode); 0 when the unconstrained minimiser satisfies every
 *               row; phase-1 steps not included
 *   primal_res, dual_res  num_agents x impc_iter: OPTIMAL — scaled primal residual
 *               max_i |r_i| / (1 + |bound_i|) over the condensed QP's rows (bounds every row's
 *               violation) and relative dual residual ||P y + q + G^T z||_inf / (1 + ||q||_inf)
 *               of the returned point; INFEASIBLE certified by phase 1 — the minimal uniform row
 *               violation t* (absolute, > 1e-6) and NaN; otherwise NaN
 *   next_states num_agents x 6: position/velocity of the kept curve at t = h (Jacobi update of
 *               the closed-loop driver, example :188-207, without noise); unchanged input if no
 *               curve was found.
 *   stamps      diagnostics, normally NULL: num_agents x 8 int64 wall-clock stamps (s_memrealtime)
 *               at the kernel's phase boundaries (start, setup, neighbours, CBF rows 0, solve 0,
 *               CBF rows 1, solve 1, end) — written by the diagnostics builds only (make stamps /
 *               prof); the release library compiles the stamp code out and ignores the pointer.
 *   nb_out      diagnostics, normally NULL (ABI 10): num_agents x 16 int32, the neighbour list each
 *               agent's QPs were built from, in the kernel's order (grid mode: the in-kernel query's
 *               k nearest, sorted by index; CSR: the given list), -1 after the last; lists longer
 *               than 16 are truncated here (not in the solve). */
typedef struct mpccbf_batch {
    int32_t num_states;
    const double* states;
    int32_t agent_first;
    int32_t num_agents;
    const double* targets;
    const double* refs;
    const int32_t* nb_row_ptr;
    const int32_t* nb_col;
    double* x;
    int32_t* status;
    double* obj;
    int32_t* iters;
    double* next_states;
    int32_t knn_k;
    double knn_radius;
    int64_t* stamps;
    /* Closed-loop simulator semantics (MPCCBFFormationControl_example.cpp:150-221), optional.
     * traj_t != NULL (device, num_agents): x is the persistent trajectory store — an agent whose
     * optimize() yields a curve (trajs non-empty) gets it written to x and traj_t = 0; one
     * without keeps its previous x; the next state is that curve (position, velocity) at
     * t = min(traj_t + Ts * int(h / Ts), max parameter), which becomes the new traj_t. With no
     * curve yet (traj_t < 0; initialise to -1) the agent holds its position at zero velocity.
     * traj_t == NULL: next state = this step's curve at t = h, or the current state if none. */
    double* traj_t;
    double pos_std, vel_std;  /* Gaussian noise added to the next state's position / velocity
                                 (math::addRandomNoise, Random.cpp:7-28) at each of the int(h / Ts)
                                 control sub-steps: with a curve only the last draw remains (each
                                 sub-step re-evaluates the curve); holding position (no curve yet)
                                 the position draws accumulate; 0 = off */
    uint64_t noise_seed;      /* counter-based: noise(seed, step_index, agent, component) */
    int64_t step_index;       /* mpccbf_run_steps adds the step number */
    /* FoV controller in slack mode (FovBezierIMPCCBF::optimize's other_robot_covs,
     * FovBezierIMPCCBF.cpp:48-81): device, num_states x 3 = (cxx, cxy, cyy), the position block
     * of each agent's estimate covariance as its observers hold it; orders the neighbours by
     * distanceToEllipse for the slack weights. NULL = unknown (infinite: every distance is -5,
     * weights follow the neighbour list order). Ignored otherwise. */
    const double* cov;
    double* primal_res;       /* out, num_agents x impc_iter, or NULL (see above) */
    double* dual_res;
    /* Closed-loop records (needs traj_t): device, num_agents x int(h / Ts) x 6, the state after
     * each control sub-step of this step as the example appends them to states.json
     * (MPCCBFFormationControl_example.cpp:188-221): the kept curve at traj_t + Ts k (clamped) plus
     * noise, or, with no curve yet, the held position with the noise accumulated over the
     * sub-steps and a zero velocity plus noise. The last record is the next state. NULL: none. */
    double* substeps;
    int32_t* nb_out;          /* out, num_agents x 16, or NULL (see above) */
} mpccbf_batch;

int mpccbf_impc_solve(mpccbf_ctx* ctx, const mpccbf_batch* batch, void* hip_stream);

/* ---- Closed-loop stepping (the MPCCBFFormationControl_example.cpp:131-231 loop: every agent
 * re-plans from the states the previous step produced — a Jacobi sweep, where the reference
 * updates robots one after another — with the batch's fallback / noise semantics) ------------
 *
 * mpccbf_run_steps enqueues num_steps control steps back to back on the stream. Step s reads
 * table T_s (T_0 = batch->states, then alternating with run->states_alt; both num_states x 6,
 * device) and writes the next states of agents [agent_first, agent_first + num_agents) into
 * T_{s+1}. Rows of other agents are carried over (copy), or, with a communicator, filled by one
 * in-place RCCL all-gather of every rank's block (ranks own equal contiguous blocks:
 * agent_first = rank * num_agents, num_states = nranks * num_agents). batch->next_states is
 * ignored; batch->status / iters receive the last step unless per-step logs are given.
 * When step_ms or solve_ms is given the call waits for the GPU and fills them (host arrays,
 * num_steps entries: device time of each step, and of its IMPC kernel alone). */
typedef struct mpccbf_comm mpccbf_comm;
#define MPCCBF_COMM_ID_BYTES 128
int mpccbf_comm_unique_id(char id_out[MPCCBF_COMM_ID_BYTES]);  /* on one rank; share the bytes */
int mpccbf_comm_create(const char id[MPCCBF_COMM_ID_BYTES], int32_t nranks, int32_t rank,
                       int32_t device, mpccbf_comm** out);     /* collective over the nranks */
void mpccbf_comm_destroy(mpccbf_comm* comm);
/* In-process group of nranks communicators (comms_out[r] for rank r) on one device: the ranks are
 * host threads of this process, each running mpccbf_run_steps on its own stream with its own
 * context and state tables; the per-step all-gather becomes device copies between those tables
 * (one event per rank and step, a host barrier per step). The multi-GPU data flow on one GPU —
 * for testing and for running several shards on one device. */
int mpccbf_comm_create_local(int32_t nranks, int32_t device, mpccbf_comm** comms_out);

typedef struct mpccbf_run {
    int32_t num_steps;
    double* states_alt;     /* second state table (device) */
    int32_t* status_log;    /* num_steps x num_agents x impc_iter (device), or NULL */
    int32_t* iters_log;     /* likewise, or NULL */
    float* step_ms;         /* host, num_steps, or NULL */
    float* solve_ms;        /* host, num_steps, or NULL */
    mpccbf_comm* comm;      /* NULL: single process */
    int32_t reserve_steps;  /* keep timing events for this many steps (avoids creating them later) */
    int32_t solve_stride;   /* time the IMPC kernel on every solve_stride-th step only (<= 1: all);
                               solve_ms of untimed steps is set to -1 */
    int32_t final_table;    /* out: 0 = batch->states holds the final states, 1 = states_alt */
    /* ABI 11: device clock of every step's IMPC launch, or NULL: num_steps x kernel_clock_waves x 2
     * uint64 (device, zero-filled by the call). Wave w of step s's launch writes the pair [s][w] =
     * (the s_memrealtime counter, 100 MHz, when the wave started, when it finished) with plain
     * stores; waves without an agent write nothing. The launch's own duration is the largest end
     * minus the smallest start over the nonzero pairs, without the dispatch gaps that events around
     * it include. kernel_clock_waves >= mpccbf_impc_launch_waves(ctx, num_agents); the collision
     * kernels only (the FoV kernels write nothing). */
    uint64_t* kernel_clock;
    int32_t kernel_clock_waves;
    /* ABI 12: 1 = this call continues the context's previous mpccbf_run_steps call: batch->states
     * is that call's final table, unchanged since, with the same agent range and neighbour
     * query (knn_k, knn_radius). Its first step then reads the neighbour table the previous call's
     * last step filled, instead of rebuilding table 0 (two memsets and an insert launch per call).
     * The library checks pointer, range and query against the previous call and rebuilds when any
     * differs (or when an mpccbf_impc_solve in grid mode came between); 0: always rebuild. */
    int32_t continue_tables;
} mpccbf_run;

int mpccbf_run_steps(mpccbf_ctx* ctx, const mpccbf_batch* batch, mpccbf_run* run, void* hip_stream);

/* Tuning knob: kernel layout for mpccbf_impc_solve. 0 (default): share-adaptive — the separable
 * collision controller runs one agent per wave64 (impc_wide_kernel) up to one agent per SIMD of the
 * device (1,024 on MI355X) and 16 lanes per agent (impc_sep_kernel, 4 agents per wave) beyond;
 * 4: the 16-lane kernel at any count; 5: the one-agent-per-wave kernel at any count; 1 / 3: the
 * dense 6 x 6 layouts (64 / 16 lanes per agent). */
int mpccbf_set_variant(mpccbf_ctx* ctx, int variant);
/* Name of the IMPC kernel instantiation the current variant launches (diagnostics). */
const char* mpccbf_kernel_name(const mpccbf_ctx* ctx);

/* ABI 11: waves of the IMPC launch mpccbf_impc_solve / mpccbf_run_steps makes for num_agents
 * agents with the context's variant that write mpccbf_run::kernel_clock (0: that kernel has no
 * clock). */
int32_t mpccbf_impc_launch_waves(const mpccbf_ctx* ctx, int32_t num_agents);

/* Neighbour lists on the device: for each agent of [agent_first, agent_first+num_agents) the
 * (at most) k nearest other agents of `states` (planar distance) within `radius`, sorted by
 * index; k <= 0 means all N-1 others (reference semantics, radius ignored). row_ptr gets
 * num_agents + 1 entries, col capacity num_agents * (k > 0 ? k : num_states - 1). */
int mpccbf_build_neighbors(mpccbf_ctx* ctx, const double* states, int32_t num_states,
                           int32_t agent_first, int32_t num_agents, int32_t k, double radius,
                           int32_t* row_ptr, int32_t* col, void* hip_stream);

/* The FoV controller's per-neighbour rows on the device, by the same device functions the IMPC
 * kernel evaluates (for parity checks of the rows themselves): for count (ego, neighbour) pairs
 * (ego: count x 6, nb_xy: count x 2, device) the box-shifted Voronoi hyperplane
 * (separating_hyperplanes::voronoi, Voronoi.cpp:10-29, math::shiftHyperplane, Helpers.cpp:20-36;
 * bbox: host, 3 half extents, NULL = 0) as voronoi[i] = (nx, ny, 0, offset), n . p + offset = 0,
 * and the four FoV HOCBF rows (FovCBF::get{Safety,LB,RB,Range}{Constraints,Bound},
 * FovCBF.cpp:622-810) as fov_rows[i][kind] = (a0, a1, a2, b), kind = safety, left, right, range
 * (b = DBL_MAX for the border rows of a 360-degree field of view). Either output may be NULL. */
int mpccbf_fov_rows_eval(int32_t count, const double* ego, const double* nb_xy, double fov, double Ds,
                         double Rs, const double* bbox, double* voronoi, double* fov_rows, void* hip_stream);

/* ---- Batched CBF-only controller (FovControl::optimize, cbf/src/controller/FovControl.cpp:17-86)
 * Per agent: min ||u - u_des||^2 over the control input u (3) subject to the 4 FoV HOCBF rows of
 * every observed neighbour (FovQPGenerator.cpp:12-115), the velocity CBF rows
 * u_d <= vmax_d - v_d and -u_d <= v_d - vmin_d (FovCBF.cpp:112-146, linear alpha) and
 * u_min <= u <= u_max. slack_mode: one slack variable >= 0 per observed neighbour relaxes its FoV
 * rows (FovControl.cpp:25-62). No context needed; all pointers are device pointers, asynchronous
 * on the stream. */
typedef struct mpccbf_fov_control_params {
    double fov, Ds, Rs;       /* FovCBF(fov, safety_dist, max_dist, ...) */
    double v_min[3], v_max[3];
    double u_min[3], u_max[3];
    int32_t slack_mode;
    double slack_cost, slack_decay_rate;
    int32_t max_pdip_iters;   /* default 60 */
    double tolerance;         /* default 1e-9 */
} mpccbf_fov_control_params;

typedef struct mpccbf_fov_control_batch {
    int32_t num_agents;
    const double* states;      /* num_agents x 6: ego (x, y, yaw, vx, vy, w) */
    const double* desired_u;   /* num_agents x 3 */
    const int32_t* nb_row_ptr; /* num_agents + 1: observed neighbours of agent i are */
    const double* nb_xy;       /* rows nb_row_ptr[i] .. nb_row_ptr[i+1]-1 of nb_xy (x, y) */
    double* u;                 /* out, num_agents x 3 (NaN when not OPTIMAL) */
    int32_t* status;           /* out, num_agents (qpcpp::SolveStatus), or NULL */
    double* obj;               /* out, ||u - u_des||^2, or NULL */
    int32_t* iters;            /* out, PDIP iterations, or NULL */
    const double* nb_cov;      /* slack mode: per observed neighbour (cxx, cxy, cyy), the estimate's
                                  position covariance ordering the slack weights by
                                  distanceToEllipse (FovControl.cpp:25-46); NULL = unknown */
} mpccbf_fov_control_batch;

/* Capacity: 4 * neighbours + 9 <= 64 rows per agent (13 observed neighbours) without slack;
 * 16 observed neighbours in slack mode (one slack variable each, cost slack_cost *
 * decay^{idx[i]}, included in obj); beyond it the agent's status is MPCCBF_ERROR. */
int mpccbf_fov_control_solve(const mpccbf_fov_control_params* p, const mpccbf_fov_control_batch* b,
                             int32_t device, void* hip_stream);

/* ---- Batched CBF-only connectivity controller (ConnectivityControl::optimize,
 * cbf/src/controller/ConnectivityControl.cpp:22-99) for teams of robots ----------------------
 * Per robot of a team (<= 16 robots; robots of team t are rows team_ptr[t] .. team_ptr[t+1]-1):
 * min ||u - u_des||^2 over u (3) subject to the safety CBF rows against every other team member
 * (ConnectivityCBF.cpp:152-198, d_min, cubic alpha), the velocity CBF rows (:250-286) and, when the
 * team's algebraic connectivity lambda2 (weighted Laplacian, :375-414, d_max) exceeds 0.1, the
 * connectivity CBF row (:430-512), else one CLF row per other member (:200-243). u is unbounded
 * (the reference's addControlBoundConstraint is commented out, :60). slack_mode: num_robots slack
 * variables, weights slack_cost * decay^i (:31-38); neighbour i's safety / CLF rows take slack i,
 * the connectivity row the last one. All pointers are device pointers; asynchronous. */
typedef struct mpccbf_connectivity_control_params {
    double d_min, d_max;
    double v_min[3], v_max[3];
    int32_t slack_mode;
    double slack_cost, slack_decay_rate;
    int32_t max_pdip_iters;   /* default 60 */
    double tolerance;         /* default 1e-9 */
} mpccbf_connectivity_control_params;

typedef struct mpccbf_connectivity_control_batch {
    int32_t num_teams;
    const int32_t* team_ptr;   /* num_teams + 1 offsets into the robot rows */
    const double* states;      /* robots x 6 (x, y, yaw, vx, vy, w) */
    const double* desired_u;   /* robots x 3 */
    double* u;                 /* out, robots x 3 (NaN when not OPTIMAL) */
    int32_t* status;           /* out, robots (qpcpp::SolveStatus), or NULL */
    double* obj;               /* out, ||u - u_des||^2 (+ slack cost), or NULL */
    int32_t* iters;            /* out, PDIP iterations, or NULL */
    double* lambda2;           /* out, num_teams, or NULL */
} mpccbf_connectivity_control_batch;

/* A team with more than 16 robots gets status MPCCBF_ERROR for all its robots. */
int mpccbf_connectivity_control_solve(const mpccbf_connectivity_control_params* p,
                                      const mpccbf_connectivity_control_batch* b, int32_t device,
                                      void* hip_stream);

/* Generic dense QP in the flattened CPLEX form (host pointers; synchronous):
 *   minimise  x^T H x + c^T x + c0        (H symmetric: sum_{i<=j} q_ij x_i x_j, CPLEX.cpp:122-147)
 *   s.t.      lo_r <= A_r x <= hi_r       (rows; lo == hi is an equality)
 *             vlo_i <= x_i <= vhi_i
 * The host validates and packs the nonzeros; the device eliminates the equalities (Householder QR
 * with column pivoting: null space + minimum-norm particular solution) and solves the reduced
 * problem with the interior-point kernel. A QP with more than 64 variables or 64 equality rows
 * (fixed variables count as equalities) is reduced on the host the same way and solved by the same
 * device kernel. Inconsistent equalities are INFEASIBLE whatever the sizes; otherwise reduced
 * dimension <= 8 and 256 reduced rows (MPCCBF_ERR_CAPACITY beyond). x_out is written only if
 * *status_out is OPTIMAL (Solver.h:33-35). */
typedef struct mpccbf_dense_qp {
    int32_t n, m;
    const double* H;  /* n x n row-major */
    const double* c;  /* n */
    double c0;
    const double* A;  /* m x n row-major */
    const double* lo;
    const double* hi;
    const double* vlo; /* n, or NULL = free */
    const double* vhi;
} mpccbf_dense_qp;

int mpccbf_qp_solve_dense(const mpccbf_dense_qp* qp, double* x_out, double* obj_out,
                          int32_t* status_out);
/* Batched form: count independent QPs solved in one launch. */
int mpccbf_qp_solve_dense_batch(int32_t count, const mpccbf_dense_qp* qps, double* const* x_out,
                                double* obj_out, int32_t* status_out);

/* Host-only inspection of the condensed operators (no device needed; used by the CPU tests).
 * Call once with capacity_ok = 0 to get the sizes, then again with every pointer sized:
 *   H n*n, Z n*nz, Xs n*6, Pr nz*nz, Qs nz*6, Qt nz*3, Ks 6*6, Kt 3*6,
 *   G m*nz, Gs m*6, lo/hi m, Cs mc*6, clo/chi mc, UZ0 3*nz, US0 3*6 (any pointer may be NULL).
 * Objective of the condensed QP: 1/2 y^T Pr y + (Qs s0 + Qt t)^T y + s0^T Ks s0 + t^T Kt s0,
 * full decision vector x = Xs s0 + Z y. */
typedef struct mpccbf_host_ops {
    int32_t n, nz, m, mc, rows_total, rows_removed;
    int32_t capacity_ok;
    double *H, *Z, *Xs, *Pr, *Qs, *Qt, *Ks, *Kt, *G, *Gs, *lo, *hi, *Cs, *clo, *chi, *UZ0, *US0;
} mpccbf_host_ops;
int mpccbf_host_operators(const mpccbf_params* p, int32_t keep_redundant, mpccbf_host_ops* out);
const char* mpccbf_host_last_error(void);

/* Diagnostics */
const char* mpccbf_last_error(void);
const char* mpccbf_status_string(int32_t status); /* SolveStatusToStr, Solver.cpp:4-28 */
int mpccbf_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MPCCBF_H */
