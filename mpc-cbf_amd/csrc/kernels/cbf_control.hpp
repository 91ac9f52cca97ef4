// cbf_control.hpp — arguments of the batched CBF-only controller kernel (cbf_control.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mpccbf {

struct FovControlArgs {
    int32_t num_agents;
    const double* states;       // num_agents x 6
    const double* desired_u;    // num_agents x 3
    const int32_t* nb_row_ptr;  // num_agents + 1
    const double* nb_xy;        // observed neighbour positions, nb_row_ptr[num_agents] x 2
    double* u;                  // num_agents x 3 (NaN rows: not OPTIMAL)
    int32_t* status;
    double* obj;
    int32_t* iters;
    double fov, Ds, Rs;
    double vmin[3], vmax[3], umin[3], umax[3];
    int32_t maxit;
    double tol, feas_tol;
    double P[9], LP[9];  // 2 I and its Cholesky factor (objective 1/2 u^T P u + q^T u)
    // slack mode (FovControl.cpp:25-62): one slack per observed neighbour (<= 16)
    int32_t slack_mode;
    double slack_cost, slack_decay;
    const double* nb_cov;  // per observed neighbour (cxx, cxy, cyy), or nullptr (unknown)
};

// ConnectivityControl::optimize for a batch of teams (connectivity_control.hip)
struct ConnControlArgs {
    int32_t num_teams;
    const int32_t* team_ptr;    // num_teams + 1
    const double* states;       // robots x 6
    const double* desired_u;    // robots x 3
    double* u;                  // robots x 3 (NaN rows: not OPTIMAL)
    int32_t* status;
    double* obj;
    int32_t* iters;
    double* lambda2;            // num_teams, or nullptr
    double dmin, dmax;
    double vmin[3], vmax[3];
    int32_t maxit;
    double tol, feas_tol;
    int32_t slack_mode;
    double slack_cost, slack_decay;
};

hipError_t launch_connectivity_control(const ConnControlArgs& a, hipStream_t s);

constexpr int FOV_CONTROL_ROW_CAP = 4 * 16;  // rows per agent (R = 4 slots x 16 lanes)

hipError_t launch_fov_control(const FovControlArgs& a, hipStream_t s);

}  // namespace mpccbf
