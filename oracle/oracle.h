/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference (ywang760/mpc-cbf @ 2025-08-29) hot path:
 * assembly of the per-agent MPC-CBF QP (workspace/lib/{model,splines,mpc,cbf,mpc_cbf})
 * and an independent full-space dense QP solver standing in for CPLEXSolver::solve
 * (workspace/lib/qpcpp/src/solvers/CPLEX.cpp:35-177), which cannot run here (CPLEX 22.1.1 is
 * proprietary and absent, as are Eigen3 and GiNaC; see DESIGN.md "Oracle").
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the CPU baseline. The product (mpc-cbf_amd/) never links it.
 *
 * Pinning: the restatement is checked against every known-answer test the reference holds for
 * this path (tests/golden/reference_kats.json: TestInitSafetyCBF.cpp:50-143, CPLEXTest.cpp:28-56,
 * DoubleIntegratorXYYawTest.cpp:19-47, CombinatoricsTest.cpp) and, for whole QPs (which no
 * reference test pins), by KKT certificates plus an independent numpy restatement
 * (tests/golden/make_golden.py).
 */
#ifndef MPCCBF_ORACLE_H
#define MPCCBF_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Parameters: same meaning as experiments/config/base_config.json parsed by
 * common/include/common/parsing.hpp:20-135. DIM is fixed to 3 (x, y, yaw) as in
 * mpc_cbf (only <double, 3U> is instantiated, MPCCBFQPOperationsBase.cpp:35). */
typedef struct orc_params {
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
    /* controller family: 0 = ConnectivityIMPCCBF (collision CBF vs neighbour states),
     * 1 = FovBezierIMPCCBF (FoV CBFs vs neighbour positions + Voronoi rows on piece 0,
     *     continuity d < degree; mpc_cbf/src/controller/FovBezierIMPCCBF.cpp:44-223) */
    int32_t cbf_mode;
    double fov_beta;   /* field of view (rad), FovCBF ctor fov (cbf/src/detail/FovCBF.cpp:41) */
    double fov_Ds;     /* safety distance Ds (= aligned_box[0] in the FoV example) */
    double fov_Rs;     /* sensing range Rs (fov_cbf_params.Rs) */
    double bbox[3];    /* robot aligned-box half extents (collision_shape.aligned_box) */
} orc_params;

/* Status codes: index of qpcpp::SolveStatus (qpcpp/include/qpcpp/solvers/Solver.h:13-21). */
enum { ORC_OPTIMAL = 0, ORC_FEASIBLE = 1, ORC_UNBOUNDED = 2, ORC_INFEASIBLE = 3, ORC_ERROR = 4,
       ORC_UNKNOWN = 5, ORC_INFEASIBLEORUNBOUNDED = 6 };

/* --- known-answer surface (for pinning against the reference's own tests) --- */
uint64_t orc_fac(uint64_t n);
uint64_t orc_comb(uint64_t n, uint64_t k);
uint64_t orc_perm(uint64_t n, uint64_t k);
/* bernsteinBasis (splines/src/detail/BezierOperations.cpp:11-50); returns 0 ok, -1 out of range */
int orc_bernstein_basis(uint64_t degree, double max_parameter, double parameter, uint64_t deriv,
                        double* out /* degree+1 */);
int orc_bernstein_coefficient_matrix(uint64_t degree, double max_parameter, uint64_t deriv,
                                     double* out /* (degree+1)^2 row-major */);
/* ConnectivityCBF safety row, closed form of ConnectivityCBF.cpp:152-198 (gamma 5, cubic alpha) */
void orc_safety_cbf(const double* state6, const double* neighbor6, double d_min, double* a3,
                    double* b);
/* FovCBF rows (cbf/src/detail/FovCBF.cpp:152-535, gamma 0.1, alpha(x) = gamma x^5) at ego state
 * state6 = (px, py, th, vx, vy, w) against a static target other2 = (x, y): rows 0..3 = safety,
 * left border, right border, range; a12 = 4 x (Ac over (ux, uy, uw)), b4 = Bc; present4[r] = 0
 * for a vacuous row (fov = 2 pi: Ac = 0, Bc = max). */
void orc_fov_cbf(const double* state6, const double* other2, double fov, double Ds, double Rs,
                 double* a12, double* b4, int32_t* present4);
/* DoubleIntegratorXYYaw(ts).applyInput (model/src/DoubleIntegrator.cpp:54-63) */
void orc_apply_input(double ts, const double* state6, const double* u3, double* out6);
/* get_A0(K).pos_ (3K x 6) and get_lambda(K).pos_ (3K x 3K) (DoubleIntegrator.cpp:9-51) */
void orc_prediction_matrices(double ts, int32_t K, double* A0pos, double* Lpos);

/* --- QP sizes for a parameter set --- */
int orc_num_vars(const orc_params* p, int32_t num_neighbors); /* curve vars (+ slack vars) */

/* --- assembly of one QP (one IMPC iteration) into the dense "flattened CPLEX" form ---
 * objective  x^T H x + c^T x + c0  (CPLEX.cpp:122-147: sum_{i<=j} q_ij x_i x_j, H symmetric)
 * rows       lo_r <= A_r x <= hi_r  (+-1e308 mean +-inf: numeric_limits lowest()/max())
 * var bounds vlo_i <= x_i <= vhi_i
 * iter == 0: CBF rows at the current ego state; iter > 0: CBF rows at pred_states (cbf_horizon x 6)
 * Returns number of rows, or -1 if capacity (max_rows) is too small. */
int orc_assemble_qp(const orc_params* p, const double* state6, const double* ref /* 3K */,
                    int32_t num_neighbors, const double* neighbors /* nb x 6 */,
                    const double* slack_weights /* nb, or NULL */, int32_t iter,
                    const double* pred_states /* cbf_horizon x 6 */, int32_t max_rows,
                    double* H /* n x n */, double* c /* n */, double* c0, double* A /* rows x n */,
                    double* lo, double* hi, double* vlo, double* vhi);

/* --- dense QP solve (stands in for CPLEXSolver<double>::solve) ---
 * kkt_out[0..3] = stationarity, primal infeasibility, dual infeasibility, complementarity
 * (all inf-norms; dual infeasibility = max(-z)). Returns status. */
int orc_solve_dense_qp(int32_t n, const double* H, const double* c, double c0, int32_t m,
                       const double* A, const double* lo, const double* hi, const double* vlo,
                       const double* vhi, double* x_out, double* obj_out, int32_t* iters_out,
                       double* kkt_out);

/* --- one agent's ConnectivityIMPCCBF::optimize (mpc_cbf/src/controller/ConnectivityIMPCCBF.cpp:47-215)
 * states: all agents (N x 6); neighbors of self are given explicitly (indices into states)
 * (the reference passes all N-1 others; pass them all for reference semantics).
 * ref: 3K reference positions of this agent.
 * Outputs per IMPC iteration it (< impc_iter): status[it], obj[it], x[it*n ..] (n = orc_num_vars).
 * Returns number of iterations attempted; success = (status[last attempted] == OPTIMAL). */
int orc_impc_optimize(const orc_params* p, int32_t num_agents, const double* states,
                      int32_t self_idx, int32_t num_neighbors, const int32_t* neighbor_idx,
                      const double* ref, int32_t* status, double* obj, double* x,
                      int32_t* qp_iters);

/* orc_impc_optimize with the neighbour covariances of FovBezierIMPCCBF::optimize
 * (FovBezierIMPCCBF.cpp:48-81; used for the slack weights only): covs = num_agents x 3
 * (cxx, cxy, cyy) indexed like states, or NULL (unknown: every distance is -5). */
int orc_impc_optimize_cov(const orc_params* p, int32_t num_agents, const double* states,
                          int32_t self_idx, int32_t num_neighbors, const int32_t* neighbor_idx,
                          const double* ref, const double* covs, int32_t* status, double* obj,
                          double* x, int32_t* qp_iters);
/* FovBezierIMPCCBF::distanceToEllipse (FovBezierIMPCCBF.cpp:226-280); cov3 = (cxx, cxy, cyy) */
double orc_distance_to_ellipse(const double* robot2, const double* mean2, const double* cov3);
/* separating_hyperplanes::voronoi (Voronoi.cpp:10-29) of two planar points, shifted by the robot
 * box bbox3 (math::shiftHyperplane, Helpers.cpp:20-36; bbox3 = 0: the plain Voronoi hyperplane):
 * normal3 . x + *offset = 0, as the FoV controller uses it (FovBezierIMPCCBF.cpp:130-147) */
void orc_voronoi(const double* self2, const double* other2, const double* bbox3, double* normal3,
                 double* offset);

/* Batched CPU baseline: agents [first, first+count) with neighbor CSR (row_ptr, col).
 * nthreads worker threads, one agent per task (CPLEX Threads=1 per solve, CPLEX.cpp:158).
 * x_last: n per agent (solution of the last OPTIMAL iteration). Returns total QPs solved. */
int64_t orc_impc_batch(const orc_params* p, int32_t num_agents, const double* states,
                       const double* refs /* N x 3K */, const int32_t* nb_row_ptr,
                       const int32_t* nb_col, int32_t first, int32_t count, int32_t nthreads,
                       int32_t* status /* count x impc_iter */, double* obj /* count x impc_iter */,
                       double* x_last /* count x n_curve */,
                       const double* covs /* N x 3 (FoV slack weights), or NULL */);

/* Curve evaluation of a solution vector (SingleParameterPiecewiseCurve::eval,
 * splines/src/curves/SingleParameterPiecewiseCurve.cpp:94-127): out3 = d-th derivative at t. */
/* FovControl::optimize (cbf/src/controller/FovControl.cpp:17-86), non-slack: the CBF-only QP
 * min ||u - u_des||^2 over u (3) s.t. per observed neighbour the 4 FoV rows -a^T u <= b
 * (FovQPGenerator.cpp:12-115), the velocity CBF rows u_i <= vmax_i - v_i and
 * -u_i <= v_i - vmin_i (FovCBF.cpp:112-146, 543-574, linear alpha), and the variable bounds
 * u_min <= u <= u_max (CBFQPGeneratorBase.cpp:75-91). Returns the qpcpp status; u_out gets the
 * solution (or the solver's last iterate), obj_out the objective with its constant. */
int orc_fov_control(double fov, double Ds, double Rs, const double* vmin3, const double* vmax3,
                    const double* umin3, const double* umax3, const double* state6,
                    const double* desired_u3, int32_t num_neighbors, const double* nb_xy,
                    double* u_out3, double* obj_out);
/* orc_fov_control with slack_mode (FovControl.cpp:25-46, FovQPGenerator.cpp:12-115): one slack
 * variable >= 0 per observed neighbour relaxes its 4 FoV rows (-1 coefficient), linear cost
 * slack_cost * decay^{idx[i]} with idx the neighbours sorted by distanceToEllipse (nb_cov:
 * nb x 3 = (cxx, cxy, cyy) per neighbour, or NULL = unknown). obj_out includes the slack cost. */
int orc_fov_control_slack(double fov, double Ds, double Rs, const double* vmin3, const double* vmax3,
                          const double* umin3, const double* umax3, const double* state6,
                          const double* desired_u3, int32_t num_neighbors, const double* nb_xy,
                          int32_t slack_mode, double slack_cost, double slack_decay,
                          const double* nb_cov, double* u_out3, double* obj_out);
/* ---- ConnectivityControl (cbf/src/controller/ConnectivityControl.cpp:22-99) ----
 * orc_lambda2: ConnectivityCBF::getLambda2 (:375-414): lambda2 and the unit Fiedler vector of
 * the weighted Laplacian of N planar positions (pos2: N x 2). orc_conn_cbf: the connectivity
 * HOCBF row of robot self (Ac over (ux, uy, uw) and Bc, :430-512; dbg7 = grad x, grad y, Hxx,
 * Hxy, Hyy, Lf h, Lf^2 h, or NULL). orc_clf_cbf: the connectivity CLF row (:200-243).
 * orc_connectivity_control: the whole CBF-only QP of robot self (states: N x 6), solved densely;
 * u free (the control bounds are commented out in the reference), N slack variables in slack
 * mode with weights slack_cost * decay^i. Returns the status; l2_out gets lambda2. */
void orc_lambda2(int32_t N, const double* pos2, double dmax, double* l2, double* vec);
void orc_conn_cbf(int32_t N, const double* states, int32_t self, const double* eigvec,
                  double lambda2, double dmax, double* a3, double* b, double* dbg7);
void orc_clf_cbf(const double* state6, const double* neighbor6, double* a3, double* b);
int orc_connectivity_control(double dmin, double dmax, const double* vmin3, const double* vmax3,
                             int32_t slack_mode, double slack_cost, double slack_decay, int32_t N,
                             const double* states, int32_t self, const double* desired_u3,
                             double* u_out3, double* obj_out, double* l2_out);
int orc_eval_curve(const orc_params* p, const double* x, double t, int32_t deriv, double* out3);

#ifdef __cplusplus
}
#endif
#endif
