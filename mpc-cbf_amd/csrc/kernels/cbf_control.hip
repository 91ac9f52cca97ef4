// cbf_control.hip — FovControl::optimize (cbf/src/controller/FovControl.cpp:17-86) for a batch of
// agents: the CBF-only QP over each agent's control input u (3 variables),
//   min ||u - u_des||^2  s.t.  -a_r^T u <= b_r  (4 FoV HOCBF rows per observed neighbour,
//                                                FovQPGenerator.cpp:12-115)
//                              u_d <= vmax_d - v_d,  -u_d <= v_d - vmin_d  (velocity CBFs with
//                                                linear alpha, FovCBF.cpp:112-146, 543-574)
//                              u_min <= u <= u_max  (CBFQPGeneratorBase.cpp:75-91)
// One 16-lane group per agent; lane l builds rows l, l + 16, ... on the device and the group PDIP
// of pdip.hpp solves them (the 3x3 Newton matrix is a 6-value group reduction). Slack mode has a
// kernel of its own (fov_control_slack_kernel: one neighbour and its slack per lane).
#include <hip/hip_runtime.h>

#include "cbf_control.hpp"
#include "fov_cbf.hpp"
#include "pdip.hpp"
#include "pdip_slack_lane.hpp"

namespace mpccbf {
namespace dev {

template <int R>
__global__ void __launch_bounds__(256) fov_control_kernel(const FovControlArgs a) {
    constexpr int G = 16, NZ = 3, GPB = 256 / G;
    const int gl = threadIdx.x & (G - 1);
    const int ai = blockIdx.x * GPB + threadIdx.x / G;
    if (ai >= a.num_agents) return;
    double st[6];
#pragma unroll
    for (int k = 0; k < 6; k++) st[k] = a.states[(size_t)ai * 6 + k];
    const int nb0 = a.nb_row_ptr[ai], nnb = a.nb_row_ptr[ai + 1] - nb0;
    const int nfov = 4 * nnb;
    const int total = nfov + 9;
    Rows<NZ, R> rw;
#pragma unroll
    for (int s = 0; s < R; s++) {
        const int t = s * G + gl;
        // inert row: 0 in [-1, 1]
#pragma unroll
        for (int d = 0; d < NZ; d++) rw.g[s][d] = 0.0;
        rw.lo[s] = -1.0;
        rw.hi[s] = 1.0;
        rw.ml[s] = 1.0;
        rw.mu[s] = 1.0;
        if (t < nfov) {  // safety, left border, right border, range of neighbour t / 4
            const double* o = a.nb_xy + (size_t)(nb0 + t / 4) * 2;
            double av[3], b;
            bool present;
            fov_cbf_row(t % 4, st, o[0], o[1], a.fov, a.Ds, a.Rs, av, b, present);
            if (present) {
#pragma unroll
                for (int d = 0; d < NZ; d++) rw.g[s][d] = -av[d];
                rw.lo[s] = 0.0;
                rw.ml[s] = 0.0;
                rw.hi[s] = b;
            }
        } else if (t < nfov + 3) {  // addMinVelConstraints: -u_d <= v_d - vmin_d
            const int d = t - nfov;
#pragma unroll
            for (int k = 0; k < NZ; k++) rw.g[s][k] = (k == d) ? -1.0 : 0.0;
            rw.lo[s] = 0.0;
            rw.ml[s] = 0.0;
            rw.hi[s] = st[3 + d] - a.vmin[d];
        } else if (t < nfov + 6) {  // addMaxVelConstraints: u_d <= vmax_d - v_d
            const int d = t - nfov - 3;
#pragma unroll
            for (int k = 0; k < NZ; k++) rw.g[s][k] = (k == d) ? 1.0 : 0.0;
            rw.lo[s] = 0.0;
            rw.ml[s] = 0.0;
            rw.hi[s] = a.vmax[d] - st[3 + d];
        } else if (t < total) {  // control bounds (variable bounds in the reference)
            const int d = t - nfov - 6;
#pragma unroll
            for (int k = 0; k < NZ; k++) rw.g[s][k] = (k == d) ? 1.0 : 0.0;
            rw.lo[s] = a.umin[d];
            rw.hi[s] = a.umax[d];
        }
    }
    int st_out = ST_ERROR, nit = 0;
    double y[NZ] = {0.0, 0.0, 0.0};
    bool ok = false;
    if (total <= R * G && nnb >= 0) {
        double q[NZ];
#pragma unroll
        for (int d = 0; d < NZ; d++) q[d] = -2.0 * a.desired_u[(size_t)ai * 3 + d];
        const PdipCfg cfg{a.maxit, a.tol};
        const PdipOut po = pdip_solve<NZ, G, R>(rw, a.P, a.LP, q, y, cfg);
        st_out = po.status;
        nit = po.iters;
        if (st_out != ST_OPTIMAL) {
            const double tstar = pdip_phase1<NZ, G, R>(rw, cfg);
            if (tstar > a.feas_tol && tstar < 1e300) st_out = ST_INFEASIBLE;
        }
        ok = st_out == ST_OPTIMAL;
    }
    if (gl < NZ) {
        double v = __builtin_nan("");
#pragma unroll
        for (int d = 0; d < NZ; d++)
            if (d == gl && ok) v = y[d];
        a.u[(size_t)ai * 3 + gl] = v;
    }
    if (gl == 0) {
        if (a.status) a.status[ai] = st_out;
        if (a.iters) a.iters[ai] = nit;
        if (a.obj) {
            double o = 0.0;
#pragma unroll
            for (int d = 0; d < NZ; d++) {
                const double e = y[d] - a.desired_u[(size_t)ai * 3 + d];
                o = fma(e, e, o);
            }
            a.obj[ai] = ok ? o : __builtin_nan("");
        }
    }
}


// Slack mode (FovControl.cpp:25-62; FovQPGenerator.cpp:12-115 with use_slack): lane l owns
// observed neighbour l — its 4 FoV rows and slack v_l — and the 9 ordinary rows (velocity CBFs,
// control bounds) take lanes 0 .. 8; pdip_slack_lane.hpp eliminates each slack lane-locally.
__global__ void __launch_bounds__(256) fov_control_slack_kernel(const FovControlArgs a) {
    constexpr int G = 16, NZ = 3, GPB = 256 / G;
    const int gl = threadIdx.x & (G - 1);
    const int ai = blockIdx.x * GPB + threadIdx.x / G;
    if (ai >= a.num_agents) return;  // uniform per group
    double st[6];
#pragma unroll
    for (int k = 0; k < 6; k++) st[k] = a.states[(size_t)ai * 6 + k];
    const int nb0 = a.nb_row_ptr[ai], nnb = a.nb_row_ptr[ai + 1] - nb0;
    const bool cap_ok = nnb >= 0 && nnb <= G;
    const bool son = cap_ok && gl < nnb;
    // slack weight: neighbours sorted by distanceToEllipse (FovControl.cpp:25-46, :90-148)
    double de = 0.0;
    if (son) {
        const double* o = a.nb_xy + (size_t)(nb0 + gl) * 2;
        const double* cv = a.nb_cov ? a.nb_cov + (size_t)(nb0 + gl) * 3 : nullptr;
        de = cv ? distance_to_ellipse(st[0], st[1], o[0], o[1], cv[0], cv[1], cv[2]) : -5.0;
    }
    const double w = sorted_slack_weight<G>(de, son, cap_ok ? nnb : 0, gl, a.slack_cost, a.slack_decay);
    double g[4][NZ], h[4], live[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int d = 0; d < NZ; d++) g[r][d] = 0.0;
        h[r] = 1.0;
        live[r] = 0.0;
        if (son) {  // safety, left border, right border, range (FovControl.cpp:54-61)
            const double* o = a.nb_xy + (size_t)(nb0 + gl) * 2;
            double av[3], b;
            bool present;
            fov_cbf_row(r, st, o[0], o[1], a.fov, a.Ds, a.Rs, av, b, present);
            if (present) {
#pragma unroll
                for (int d = 0; d < NZ; d++) g[r][d] = -av[d];
                h[r] = b;
                live[r] = 1.0;
            }
        }
    }
    Rows<NZ, 1> orw;
#pragma unroll
    for (int d = 0; d < NZ; d++) orw.g[0][d] = 0.0;
    orw.lo[0] = -1.0;
    orw.hi[0] = 1.0;
    orw.ml[0] = 1.0;
    orw.mu[0] = 1.0;
    if (gl < 3) {  // addMinVelConstraints: -u_d <= v_d - vmin_d
        orw.g[0][gl] = -1.0;
        orw.lo[0] = 0.0;
        orw.ml[0] = 0.0;
        orw.hi[0] = st[3 + gl] - a.vmin[gl];
    } else if (gl < 6) {  // addMaxVelConstraints: u_d <= vmax_d - v_d
        orw.g[0][gl - 3] = 1.0;
        orw.lo[0] = 0.0;
        orw.ml[0] = 0.0;
        orw.hi[0] = a.vmax[gl - 3] - st[gl];
    } else if (gl < 9) {  // control bounds (addControlBoundConstraint, variable bounds)
        orw.g[0][gl - 6] = 1.0;
        orw.lo[0] = a.umin[gl - 6];
        orw.hi[0] = a.umax[gl - 6];
    }
    double q[NZ], y[NZ] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int d = 0; d < NZ; d++) q[d] = -2.0 * a.desired_u[(size_t)ai * 3 + d];
    SlackLaneOut so{ST_ERROR, 0, 0.0};
    if (cap_ok) so = pdip_slack_lane<4, G>(g, h, live, son, w, orw, q, y, PdipCfg{a.maxit, a.tol}, a.feas_tol);
    const bool ok = so.status == ST_OPTIMAL;
    if (gl < NZ) {
        double uv = __builtin_nan("");
#pragma unroll
        for (int d = 0; d < NZ; d++)
            if (d == gl && ok) uv = y[d];
        a.u[(size_t)ai * 3 + gl] = uv;
    }
    if (gl == 0) {
        if (a.status) a.status[ai] = so.status;
        if (a.iters) a.iters[ai] = so.iters;
        if (a.obj) {
            double o = 0.0;
#pragma unroll
            for (int d = 0; d < NZ; d++) {
                const double e = y[d] - a.desired_u[(size_t)ai * 3 + d];
                o = fma(e, e, o);
            }
            a.obj[ai] = ok ? o + so.vcost : __builtin_nan("");
        }
    }
}

}  // namespace dev

hipError_t launch_fov_control(const FovControlArgs& a, hipStream_t s) {
    if (a.num_agents <= 0) return hipSuccess;
    constexpr int GPB = 256 / 16;
    const int blocks = (a.num_agents + GPB - 1) / GPB;
    if (a.slack_mode)
        hipLaunchKernelGGL(dev::fov_control_slack_kernel, dim3(blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(dev::fov_control_kernel<4>, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace mpccbf
