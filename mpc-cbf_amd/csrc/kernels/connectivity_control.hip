// connectivity_control.hip — ConnectivityControl::optimize (cbf/src/controller/ConnectivityControl.cpp:22-99)
// for a batch of robot teams: one wavefront per team (<= 16 robots).
//
// Phase 1 (per team, all 64 lanes): the weighted Laplacian of the team's planar positions
// (ConnectivityCBF::getLambda2, ConnectivityCBF.cpp:375-414: A_ij = exp((Rs^2 - d^2)^2 / sigma) - 1
// within Rs = d_max, sigma = d_max^4 / ln 2) in LDS, diagonalised by a parallel cyclic Jacobi
// sweep (round-robin pairing: the N/2 rotations of a round touch disjoint rows / columns, so a
// round is two passes over (pair, column) tasks) to machine precision; lambda2 and the unit
// Fiedler vector are what every robot's connectivity row needs.
// Phase 2 (per robot, one 16-lane group each, 4 robots at a time): the CBF-only QP over u (3):
//   min ||u - u_des||^2  s.t.  safety rows vs every other robot (:49-55, cubic alpha, gamma 5),
//   velocity CBFs (:58-59), and either the lambda2 connectivity row (lambda2 > 0.1, :70-71,
//   ConnectivityQPGenerator.cpp:13-44) or the per-neighbour CLF rows (:72-82; :47-69); u is free
//   (addControlBoundConstraint is commented out, :60). Lane l holds neighbour l's safety row and
//   CLF row; the connectivity row's gradient and Hessian terms are summed over the lanes.
//   Slack mode: lane l's slack relaxes its safety and CLF rows, lane N-1's the connectivity
//   row, weights slack_cost * decay^l (:31-38) — solved by pdip_slack_lane.hpp; without slack
//   by the group PDIP of pdip.hpp.
#include <hip/hip_runtime.h>

#include <cmath>

#include "cbf_control.hpp"
#include "impc_common.hpp"
#include "pdip.hpp"
#include "pdip_slack_lane.hpp"

namespace mpccbf {
namespace dev {

constexpr int CC_MAX = 16;  // robots per team

struct ConnLds {
    double A[CC_MAX * CC_MAX];  // Laplacian, diagonalised in place
    double V[CC_MAX * CC_MAX];  // eigenvectors (columns)
    double rot[CC_MAX][2];      // (c, s) of the round's rotations
    double pos[CC_MAX][2];
    double l2, ev[CC_MAX];
    int32_t pairs[CC_MAX / 2][2];
};

// lambda2 and the unit Fiedler vector of the team (n <= 16) into L.l2 / L.ev (all lanes).
__device__ void team_lambda2(ConnLds& L, int n, double dmax, int lane) {
    const double Rs2 = dmax * dmax, sigma = dmax * dmax * dmax * dmax / 0.69314718055994530942;
    for (int e = lane; e < CC_MAX * CC_MAX; e += 64) {
        const int i = e / CC_MAX, j = e % CC_MAX;
        double a = 0.0;
        if (i < n && j < n && i != j) {
            const double dx = L.pos[i][0] - L.pos[j][0], dy = L.pos[i][1] - L.pos[j][1];
            const double d2 = dx * dx + dy * dy;
            a = d2 <= Rs2 ? -(exp((Rs2 - d2) * (Rs2 - d2) / sigma) - 1.0) : 0.0;
        }
        L.A[e] = a;
        L.V[e] = (i == j && i < n) ? 1.0 : 0.0;
    }
    wave_lds_sync();
    if (lane < n) {  // degrees on the diagonal
        double dg = 0.0;
        for (int j = 0; j < n; j++) dg -= L.A[lane * CC_MAX + j];
        L.A[lane * CC_MAX + lane] = dg;
    }
    wave_lds_sync();
    const int m = n + (n & 1);  // round-robin over m slots (slot n is a dummy when n is odd)
    const int np = m / 2;
    for (int sweep = 0; sweep < 30; sweep++) {
        // convergence: off-diagonal mass against the total
        double off = 0.0, tot = 0.0;
        for (int e = lane; e < CC_MAX * CC_MAX; e += 64) {
            const double a = L.A[e] * L.A[e];
            tot += a;
            off += (e / CC_MAX != e % CC_MAX) ? a : 0.0;
        }
        off = grp_sum<64>(off);
        tot = grp_sum<64>(tot);
        if (off <= 1e-32 * tot || off == 0.0) break;
        for (int round = 0; round < m - 1; round++) {
            // pairing of this round (circle method: slot 0 fixed, the others rotate)
            if (lane < np) {
                const int k = lane;
                int p = (k == 0) ? 0 : 1 + (round + k - 1) % (m - 1);
                int q = 1 + (round + m - 2 - k) % (m - 1);
                if (p > q) { const int t = p; p = q; q = t; }
                L.pairs[k][0] = p;
                L.pairs[k][1] = q;
                double c = 1.0, s = 0.0;
                if (q < n) {
                    const double apq = L.A[p * CC_MAX + q];
                    if (apq != 0.0) {
                        const double theta = (L.A[q * CC_MAX + q] - L.A[p * CC_MAX + p]) / (2.0 * apq);
                        const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                        c = 1.0 / sqrt(t * t + 1.0);
                        s = t * c;
                    }
                }
                L.rot[k][0] = c;
                L.rot[k][1] = s;
            }
            wave_lds_sync();
            // A <- A J (columns p, q) and V <- V J
            for (int task = lane; task < np * CC_MAX; task += 64) {
                const int k = task / CC_MAX, r = task % CC_MAX;
                const int p = L.pairs[k][0], q = L.pairs[k][1];
                if (q < n && r < n) {
                    const double c = L.rot[k][0], s = L.rot[k][1];
                    const double ap = L.A[r * CC_MAX + p], aq = L.A[r * CC_MAX + q];
                    L.A[r * CC_MAX + p] = c * ap - s * aq;
                    L.A[r * CC_MAX + q] = s * ap + c * aq;
                    const double vp = L.V[r * CC_MAX + p], vq = L.V[r * CC_MAX + q];
                    L.V[r * CC_MAX + p] = c * vp - s * vq;
                    L.V[r * CC_MAX + q] = s * vp + c * vq;
                }
            }
            wave_lds_sync();
            // A <- J^T A (rows p, q)
            for (int task = lane; task < np * CC_MAX; task += 64) {
                const int k = task / CC_MAX, r = task % CC_MAX;
                const int p = L.pairs[k][0], q = L.pairs[k][1];
                if (q < n && r < n) {
                    const double c = L.rot[k][0], s = L.rot[k][1];
                    const double ap = L.A[p * CC_MAX + r], aq = L.A[q * CC_MAX + r];
                    L.A[p * CC_MAX + r] = c * ap - s * aq;
                    L.A[q * CC_MAX + r] = s * ap + c * aq;
                }
            }
            wave_lds_sync();
        }
    }
    // second smallest eigenvalue (ties: lower index), its unit eigenvector (eigenvec.normalize())
    if (lane == 0) {
        int k0 = 0;
        for (int i = 1; i < n; i++)
            if (L.A[i * CC_MAX + i] < L.A[k0 * CC_MAX + k0]) k0 = i;
        int k1 = -1;
        for (int i = 0; i < n; i++) {
            if (i == k0) continue;
            if (k1 < 0 || L.A[i * CC_MAX + i] < L.A[k1 * CC_MAX + k1]) k1 = i;
        }
        if (k1 < 0) k1 = k0;
        L.l2 = L.A[k1 * CC_MAX + k1];
        double nrm = 0.0;
        for (int i = 0; i < n; i++) nrm += L.V[i * CC_MAX + k1] * L.V[i * CC_MAX + k1];
        nrm = sqrt(nrm);
        for (int i = 0; i < n; i++) L.ev[i] = L.V[i * CC_MAX + k1] / nrm;
    }
    wave_lds_sync();
}

template <bool SLACK>
__global__ void __launch_bounds__(64) connectivity_control_kernel(const ConnControlArgs a) {
    constexpr int G = 16, NZ = 3;
    const int lane = threadIdx.x;
    const int team = blockIdx.x;
    if (team >= a.num_teams) return;
    __shared__ ConnLds L;
    const int r0 = a.team_ptr[team], n = a.team_ptr[team + 1] - r0;
    const bool cap_ok = n >= 1 && n <= CC_MAX;
    if (lane < CC_MAX) {
        L.pos[lane][0] = (cap_ok && lane < n) ? a.states[(size_t)(r0 + lane) * 6] : 0.0;
        L.pos[lane][1] = (cap_ok && lane < n) ? a.states[(size_t)(r0 + lane) * 6 + 1] : 0.0;
    }
    wave_lds_sync();
    if (cap_ok) team_lambda2(L, n, a.dmax, lane);
    const double l2 = cap_ok ? L.l2 : 0.0;
    if (lane == 0 && a.lambda2) a.lambda2[team] = cap_ok ? l2 : __builtin_nan("");
    const bool conn = l2 > 0.1;  // ConnectivityControl.cpp:69 (threshold 0.1)
    const int gi = lane / G, gl = lane & (G - 1);
    const double Rs2 = a.dmax * a.dmax, sigma = Rs2 * Rs2 / 0.69314718055994530942;
    for (int pass = 0; pass < CC_MAX / 4; pass++) {
        const int self = gi + 4 * pass;
        if (!cap_ok || self >= n) continue;  // group-uniform
        const size_t ri = (size_t)(r0 + self);
        double st[6];
#pragma unroll
        for (int k = 0; k < 6; k++) st[k] = a.states[ri * 6 + k];
        // neighbour l of this lane (the reference's order: other robots by index, :49-55)
        const bool has_nb = gl < n - 1;
        const int j = gl + (gl >= self ? 1 : 0);
        double nb[6] = {0, 0, 0, 0, 0, 0};
        if (has_nb) {
#pragma unroll
            for (int k = 0; k < 6; k++) nb[k] = a.states[(size_t)(r0 + j) * 6 + k];
        }
        // safety row: -Ac u <= Bc
        double sa[3] = {0, 0, 0}, sb = 1.0;
        if (has_nb) {
            double ac[3], bc;
            safety_cbf(st, nb[0], nb[1], nb[3], nb[4], a.dmin, ac, bc);
            sa[0] = -ac[0];
            sa[1] = -ac[1];
            sa[2] = -ac[2];
            sb = bc;
        }
        // connectivity row (grad / Hessian of lambda2 over the self position, summed over the
        // lanes: lane gl takes robot j, ConnectivityCBF.cpp:430-512) or this lane's CLF row
        double ca[3] = {0, 0, 0}, cb = 1.0;
        bool clive = false;
        if (conn) {
            double t[5] = {0, 0, 0, 0, 0};
            if (has_nb) {
                const double dx = st[0] - nb[0], dy = st[1] - nb[1];
                const double diff = Rs2 - (dx * dx + dy * dy);
                const double E = exp(diff * diff / sigma);
                const double dev = L.ev[self] - L.ev[j];
                const double k = -4.0 * dev * dev / sigma;
                t[0] = k * E * diff * dx;
                t[1] = k * E * diff * dy;
                t[2] = k * (-4.0 * E * diff * diff * dx * dx / sigma - 2.0 * E * dx * dx + E * diff);
                t[3] = k * (-4.0 * E * diff * diff * dx * dy / sigma - 2.0 * E * dx * dy);
                t[4] = k * (-4.0 * E * diff * diff * dy * dy / sigma - 2.0 * E * dy * dy + E * diff);
            }
            grp_sum_vec<G, 5>(t);
            const double vx = st[3], vy = st[4];
            const double lfh = t[0] * vx + t[1] * vy;
            const double lf2h = vx * (t[2] * vx + t[3] * vy) + vy * (t[3] * vx + t[4] * vy);
            const double hh = l2 - 0.1;
            const int owner = SLACK ? n - 1 : 0;  // slack mode: the last slack variable
            if (gl == owner) {
                ca[0] = -t[0];
                ca[1] = -t[1];
                cb = lf2h + 5.0 * lfh + 5.0 * (lfh + 5.0 * hh);
                clive = true;
            }
        } else if (has_nb) {  // CLF: +Ac u <= -Bc
            const double dx = st[0] - nb[0], dy = st[1] - nb[1];
            const double dist = sqrt(dx * dx + dy * dy), e = dist - 2.0;
            const double gx = 2.0 * e * dx / dist, gy = 2.0 * e * dy / dist;
            const double vx = st[3], vy = st[4];
            const double lfv = gx * vx + gy * vy, dv = (dx * vx + dy * vy) / dist;
            const double lf2v = 2.0 * dv * dv + 2.0 * e * (vx * vx + vy * vy - dv * dv) / dist;
            ca[0] = gx;
            ca[1] = gy;
            cb = -(lf2v + 5.0 * lfv + 2.0 * e * e);
            clive = true;
        }
        // velocity CBF row of lanes 0..5: -u_d <= v_d - vmin_d, u_d <= vmax_d - v_d
        double og[3] = {0, 0, 0}, ohi = 1.0, olo = -1.0, oml = 1.0;
        if (gl < 3) {
            og[gl] = -1.0;
            ohi = st[3 + gl] - a.vmin[gl];
            olo = 0.0;
            oml = 0.0;
        } else if (gl < 6) {
            og[gl - 3] = 1.0;
            ohi = a.vmax[gl - 3] - st[gl];
            olo = 0.0;
            oml = 0.0;
        }
        double q[NZ], y[NZ] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int d = 0; d < NZ; d++) q[d] = -2.0 * a.desired_u[ri * 3 + d];
        const PdipCfg cfg{a.maxit, a.tol};
        int status;
        int iters;
        double vcost = 0.0;
        if constexpr (SLACK) {
            double g[2][3], h[2], live[2];
#pragma unroll
            for (int d = 0; d < 3; d++) {
                g[0][d] = sa[d];
                g[1][d] = ca[d];
            }
            h[0] = sb;
            h[1] = cb;
            live[0] = has_nb ? 1.0 : 0.0;
            live[1] = clive ? 1.0 : 0.0;
            if (!clive) {
                g[1][0] = g[1][1] = g[1][2] = 0.0;
                h[1] = 1.0;
            }
            const bool son = gl < n;  // N slack variables (CBFQPGeneratorBase.cpp:20-27)
            const double w = son ? a.slack_cost * pow(a.slack_decay, (double)gl) : 0.0;
            Rows<NZ, 1> orw;
#pragma unroll
            for (int d = 0; d < 3; d++) orw.g[0][d] = og[d];
            orw.lo[0] = olo;
            orw.hi[0] = ohi;
            orw.ml[0] = oml;
            orw.mu[0] = 1.0;
            const SlackLaneOut so = pdip_slack_lane<2, G>(g, h, live, son, w, orw, q, y, cfg, a.feas_tol);
            status = so.status;
            iters = so.iters;
            vcost = so.vcost;
        } else {
            Rows<NZ, 3> rw;
#pragma unroll
            for (int d = 0; d < 3; d++) {
                rw.g[0][d] = has_nb ? sa[d] : 0.0;
                rw.g[1][d] = clive ? ca[d] : 0.0;
                rw.g[2][d] = og[d];
            }
            rw.lo[0] = has_nb ? 0.0 : -1.0;
            rw.hi[0] = has_nb ? sb : 1.0;
            rw.ml[0] = has_nb ? 0.0 : 1.0;
            rw.mu[0] = 1.0;
            rw.lo[1] = clive ? 0.0 : -1.0;
            rw.hi[1] = clive ? cb : 1.0;
            rw.ml[1] = clive ? 0.0 : 1.0;
            rw.mu[1] = 1.0;
            rw.lo[2] = olo;
            rw.hi[2] = ohi;
            rw.ml[2] = oml;
            rw.mu[2] = 1.0;
            const double LP[9] = {1.4142135623730951, 0, 0, 0, 1.4142135623730951, 0, 0, 0, 1.4142135623730951};
            const double P[9] = {2, 0, 0, 0, 2, 0, 0, 0, 2};
            const PdipOut po = pdip_solve<NZ, G, 3>(rw, P, LP, q, y, cfg);
            status = po.status;
            iters = po.iters;
            if (status != ST_OPTIMAL) {
                const double tstar = pdip_phase1<NZ, G, 3>(rw, cfg);
                status = (tstar > a.feas_tol && tstar < 1e300) ? ST_INFEASIBLE : ST_UNKNOWN;
            }
        }
        const bool ok = status == ST_OPTIMAL;
        if (gl < NZ) {
            double uv = __builtin_nan("");
#pragma unroll
            for (int d = 0; d < NZ; d++)
                if (d == gl && ok) uv = y[d];
            a.u[ri * 3 + gl] = uv;
        }
        if (gl == 0) {
            if (a.status) a.status[ri] = status;
            if (a.iters) a.iters[ri] = iters;
            if (a.obj) {
                double o = 0.0;
#pragma unroll
                for (int d = 0; d < NZ; d++) {
                    const double e = y[d] - a.desired_u[ri * 3 + d];
                    o = fma(e, e, o);
                }
                a.obj[ri] = ok ? o + vcost : __builtin_nan("");
            }
        }
    }
    if (!cap_ok) {  // team size out of range: every robot of it ERROR
        for (int i = lane; i < n; i += 64) {
            const size_t ri = (size_t)(r0 + i);
            if (a.status) a.status[ri] = ST_ERROR;
            if (a.iters) a.iters[ri] = 0;
            if (a.obj) a.obj[ri] = __builtin_nan("");
            for (int d = 0; d < NZ; d++) a.u[ri * 3 + d] = __builtin_nan("");
        }
    }
}

}  // namespace dev

hipError_t launch_connectivity_control(const ConnControlArgs& a, hipStream_t s) {
    if (a.num_teams <= 0) return hipSuccess;
    if (a.slack_mode)
        hipLaunchKernelGGL(dev::connectivity_control_kernel<true>, dim3(a.num_teams), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL(dev::connectivity_control_kernel<false>, dim3(a.num_teams), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace mpccbf
