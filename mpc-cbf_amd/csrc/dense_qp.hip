// dense_qp.hip — generic flattened-QP entry points (mpccbf_qp_solve_dense / _batch).
//
// This is the path a qpcpp::Solver<double> subclass uses (csrc/qpcpp/HIPSolver.h): it replaces
// one CPLEXSolver<double>::solve(Problem&) call (qpcpp/src/solvers/CPLEX.cpp:35-177) for any
// Problem, not only the MPC-CBF one. Host: exact equality elimination (host/dense_qp.cpp).
// Device: one 64-lane wavefront per QP running the same Mehrotra PDIP + phase-1 certificate
// as the structured IMPC kernel (kernels/pdip.hpp), reduced dimension padded to 8.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mpccbf.h"
#include "host/dense_qp.hpp"
#include "host/errors.hpp"
#include "kernels/pdip.hpp"

namespace mpccbf {

constexpr int DQ_R = DENSE_ROWS / 64;               // row slots per lane
constexpr int DQ_HDR = 2 * DENSE_NZ * DENSE_NZ + DENSE_NZ + 2;  // P, LP, q, reg, pad
constexpr int DQ_ROW = DENSE_NZ + 2;                // g, lo, hi

struct DenseArgs {
    const double* buf;     // per QP: [P | LP | q | reg, 0 | rows (g, lo, hi) x m]
    const int32_t* off;    // offset of each QP in buf (doubles)
    const int32_t* m;      // rows per QP
    const int32_t* pd;     // 1: LP holds the Cholesky factor of P
    int32_t count;
    int32_t maxit;
    double tol;
    double feas_tol;
    double* y;             // count x DENSE_NZ
    int32_t* status;
    int32_t* iters;
};

namespace dev {

template <int NZ, int R>
__global__ void __launch_bounds__(64) dense_qp_kernel(const DenseArgs a) {
    const int qi = blockIdx.x;
    const int gl = threadIdx.x;
    if (qi >= a.count) return;
    const double* base = a.buf + a.off[qi];
    const double* P = base;
    const double* LP = base + NZ * NZ;
    const double* qv = base + 2 * NZ * NZ;
    const double reg = qv[NZ];
    const double* rows = base + DQ_HDR;
    const int m = a.m[qi];
    const bool pd = a.pd[qi] != 0;

    Rows<NZ, R> rw;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int slot = r * 64 + gl;
        const bool on = slot < m;
        const double* src = rows + (size_t)(on ? slot : 0) * DQ_ROW;
#pragma unroll
        for (int j = 0; j < NZ; j++) rw.g[r][j] = on ? src[j] : 0.0;
        const double l = on ? src[NZ] : -1e300, h = on ? src[NZ + 1] : 1e300;
        const bool hl = on && l > -1e300, hu = on && h < 1e300;
        rw.ml[r] = hl ? 1.0 : 0.0;
        rw.mu[r] = hu ? 1.0 : 0.0;
        rw.lo[r] = hl ? l : 0.0;
        rw.hi[r] = hu ? h : 0.0;
    }
    double q[NZ], y[NZ];
#pragma unroll
    for (int i = 0; i < NZ; i++) q[i] = qv[i];
    PdipCfg cfg{a.maxit, a.tol};
    cfg.reg = reg;
    const PdipOut po = pdip_solve<NZ, 64, R>(rw, P, pd ? LP : nullptr, q, y, cfg);
    int st = po.status;
    if (st != ST_OPTIMAL) {
        const double tstar = pdip_phase1<NZ, 64, R>(rw, cfg);
        // feasible but no convergence: with P positive definite a feasible QP has an optimum,
        // so this is a numerical failure (UNKNOWN); otherwise the objective is unbounded below
        // along a recession direction (CPLEX: UNBOUNDED).
        st = tstar > a.feas_tol ? ST_INFEASIBLE : (pd ? ST_UNKNOWN : MPCCBF_UNBOUNDED);
    }
    if (gl == 0) {
        a.status[qi] = st;
        a.iters[qi] = po.iters;
#pragma unroll
        for (int i = 0; i < NZ; i++) a.y[(size_t)qi * NZ + i] = y[i];
    }
}

}  // namespace dev

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int device = -1;  // no destructor: freeing after the HIP runtime's own teardown is unsafe
    hipError_t reserve(size_t need, int dev) {
        if (p && bytes >= need && device == dev) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, need);
        if (e == hipSuccess) {
            bytes = need;
            device = dev;
        }
        return e;
    }
};
thread_local DevBuf g_dense_buf;

size_t align8(size_t v) { return (v + 7) & ~size_t(7); }

}  // namespace
}  // namespace mpccbf

using namespace mpccbf;

extern "C" {

int mpccbf_qp_solve_dense_batch(int32_t count, const mpccbf_dense_qp* qps, double* const* x_out,
                                double* obj_out, int32_t* status_out) {
    if (count < 0 || (count > 0 && (!qps || !status_out)))
        return set_error(MPCCBF_ERR_INVALID_ARGUMENT, "dense QP batch: null argument");
    // exact equality elimination on the host, QPs split over up to 16 threads (independent)
    std::vector<ReducedQP> red(count);
    std::vector<std::string> err(count);
    auto reduce_range = [&](int k0, int k1) {
        for (int k = k0; k < k1; k++) {
            try {
                red[k] = reduce_dense_qp(qps[k]);
            } catch (const std::exception& e) {
                err[k] = e.what();
            }
        }
    };
    const int nthr = count >= 64 ? (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency())) : 1;
    if (nthr > 1) {
        std::vector<std::thread> pool;
        const int chunk = (count + nthr - 1) / nthr;
        for (int t = 0; t < nthr; t++) {
            const int k0 = t * chunk, k1 = std::min(count, k0 + chunk);
            if (k0 < k1) pool.emplace_back(reduce_range, k0, k1);
        }
        for (auto& th : pool) th.join();
    } else {
        reduce_range(0, count);
    }
    for (int k = 0; k < count; k++) {  // the first bad QP's error, as a serial pass would report
        if (!err[k].empty()) return set_error(MPCCBF_ERR_INVALID_ARGUMENT, "QP " + std::to_string(k) + ": " + err[k]);
        if (red[k].status < 0 && (red[k].nz > DENSE_NZ || red[k].m > DENSE_ROWS))
            return set_error(MPCCBF_ERR_CAPACITY,
                             "QP " + std::to_string(k) + ": reduced dimension " + std::to_string(red[k].nz) +
                                 " / rows " + std::to_string(red[k].m) + " exceed the dense kernel (8 / 256)");
    }
    // pack the QPs that need a device solve
    std::vector<int> dev_idx;
    std::vector<double> buf;
    std::vector<int32_t> off, mrows, pd;
    for (int k = 0; k < count; k++) {
        const ReducedQP& r = red[k];
        if (r.status >= 0) continue;
        dev_idx.push_back(k);
        off.push_back((int32_t)buf.size());
        mrows.push_back(r.m);
        pd.push_back(r.pd ? 1 : 0);
        const size_t o = buf.size();
        buf.resize(o + DQ_HDR + (size_t)r.m * DQ_ROW, 0.0);
        double* P = &buf[o];
        double* LP = P + DENSE_NZ * DENSE_NZ;
        double* q = LP + DENSE_NZ * DENSE_NZ;
        double pmax = 0.0;
        for (int a = 0; a < DENSE_NZ; a++)
            for (int b = 0; b < DENSE_NZ; b++) {
                const bool in = a < r.nz && b < r.nz;
                P[a * DENSE_NZ + b] = in ? r.P(a, b) : (a == b ? 1.0 : 0.0);  // padding: identity
                LP[a * DENSE_NZ + b] = (in && r.pd) ? r.LP(a, b) : (a == b ? 1.0 : 0.0);
                if (in) pmax = std::max(pmax, std::fabs(r.P(a, b)));
            }
        for (int a = 0; a < r.nz; a++) q[a] = r.q[a];
        q[DENSE_NZ] = r.pd ? 0.0 : 1e-10 * std::max(1.0, pmax);  // Newton-matrix ridge if P is PSD
        double* rows = P + DQ_HDR;
        for (int i = 0; i < r.m; i++) {
            for (int b = 0; b < r.nz; b++) rows[i * DQ_ROW + b] = r.G(i, b);
            rows[i * DQ_ROW + DENSE_NZ] = r.lo[i];
            rows[i * DQ_ROW + DENSE_NZ + 1] = r.hi[i];
        }
    }
    const int nd = (int)dev_idx.size();
    std::vector<double> y((size_t)nd * DENSE_NZ);
    std::vector<int32_t> st(nd), its(nd);
    if (nd > 0) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            return set_error(MPCCBF_ERR_NO_DEVICE, "no HIP device visible");
        int device = 0;
        hipError_t e = hipGetDevice(&device);
        const size_t b_buf = align8(buf.size() * sizeof(double));
        const size_t b_int = align8((size_t)nd * sizeof(int32_t));
        const size_t b_y = (size_t)nd * DENSE_NZ * sizeof(double);
        const size_t need = b_buf + 6 * b_int + b_y;
        if (e == hipSuccess) e = g_dense_buf.reserve(need, device);
        if (e != hipSuccess) return set_error(MPCCBF_ERR_HIP, std::string("dense QP buffers: ") + hipGetErrorString(e));
        char* base = (char*)g_dense_buf.p;
        double* d_buf = (double*)base;
        int32_t* d_off = (int32_t*)(base + b_buf);
        int32_t* d_m = (int32_t*)(base + b_buf + b_int);
        int32_t* d_pd = (int32_t*)(base + b_buf + 2 * b_int);
        int32_t* d_st = (int32_t*)(base + b_buf + 3 * b_int);
        int32_t* d_it = (int32_t*)(base + b_buf + 4 * b_int);
        double* d_y = (double*)(base + b_buf + 6 * b_int);
        e = hipMemcpy(d_buf, buf.data(), buf.size() * sizeof(double), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(d_off, off.data(), nd * sizeof(int32_t), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(d_m, mrows.data(), nd * sizeof(int32_t), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(d_pd, pd.data(), nd * sizeof(int32_t), hipMemcpyHostToDevice);
        DenseArgs a;
        a.buf = d_buf;
        a.off = d_off;
        a.m = d_m;
        a.pd = d_pd;
        a.count = nd;
        a.maxit = 100;
        a.tol = 1e-9;
        a.feas_tol = 1e-6;
        a.y = d_y;
        a.status = d_st;
        a.iters = d_it;
        if (e == hipSuccess) {
            hipLaunchKernelGGL((dev::dense_qp_kernel<DENSE_NZ, DQ_R>), dim3(nd), dim3(64), 0, 0, a);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpy(st.data(), d_st, nd * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(its.data(), d_it, nd * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(y.data(), d_y, b_y, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return set_error(MPCCBF_ERR_HIP, std::string("dense QP solve: ") + hipGetErrorString(e));
    }
    // outputs: x only for OPTIMAL (Solver.h:33-35)
    std::vector<double> xtmp;
    for (int k = 0; k < count; k++) {
        const ReducedQP& r = red[k];
        status_out[k] = r.status;
        if (obj_out) obj_out[k] = __builtin_nan("");
    }
    const std::vector<double> zero(DENSE_NZ, 0.0);
    for (int k = 0; k < count; k++) {
        const ReducedQP& r = red[k];
        const double* yk = zero.data();
        if (r.status < 0) {
            const int j = (int)(std::lower_bound(dev_idx.begin(), dev_idx.end(), k) - dev_idx.begin());
            status_out[k] = st[j];
            yk = &y[(size_t)j * DENSE_NZ];
        }
        if (status_out[k] == MPCCBF_OPTIMAL) {
            xtmp.assign(r.n, 0.0);
            double f = 0.0;
            expand_solution(r, yk, xtmp.data(), &f);
            if (obj_out) obj_out[k] = f;
            if (x_out && x_out[k]) std::memcpy(x_out[k], xtmp.data(), r.n * sizeof(double));
        }
    }
    return MPCCBF_OK;
}

int mpccbf_qp_solve_dense(const mpccbf_dense_qp* qp, double* x_out, double* obj_out,
                          int32_t* status_out) {
    if (!qp || !status_out) return set_error(MPCCBF_ERR_INVALID_ARGUMENT, "dense QP: null argument");
    double* xs[1] = {x_out};
    return mpccbf_qp_solve_dense_batch(1, qp, xs, obj_out, status_out);
}

}  // extern "C"
