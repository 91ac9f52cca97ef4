// dense_qp.hip — generic flattened-QP entry points (mpccbf_qp_solve_dense / _batch).
//
// This is the path a qpcpp::Solver<double> subclass uses (csrc/qpcpp/HIPSolver.h): it replaces
// one CPLEXSolver<double>::solve(Problem&) call (qpcpp/src/solvers/CPLEX.cpp:35-177) for any
// Problem, not only the MPC-CBF one.
//
// Host: validation (the reference's invalid_argument cases) and a streaming sparse pack of each
// QP — nonzeros of H, c, c0, and the rows classified as equalities (lo == hi, fixed variables)
// or inequalities (a finite side; variable bounds as unit rows) in CSR — into pinned host memory
// that the kernels read over the bus (no copy), in slices: the device reduces one slice while the
// host packs the next.
// Device, one 64-lane wavefront per QP, three launches:
//   dense_reduce_kernel  exact equality elimination: Householder QR with column pivoting of E^T
//                        (lane = equality row; rank by |R_tt| <= 1e-12 |R_00|), x = xp + Z y with
//                        xp the minimum-norm solution and Z the orthonormal null-space basis
//                        (reflections applied to unit vectors), inconsistent equalities ->
//                        INFEASIBLE; reduced objective 1/2 y^T (2 Z^T Hs Z) y + ..., Cholesky of P;
//                        inequality rows g = Z^T a with bounds shifted by a^T xp (constant rows
//                        decided here), compacted;
//   dense_qp_kernel      the Mehrotra PDIP + phase-1 certificate of the structured kernel
//                        (kernels/pdip.hpp), reduced dimension padded to 8;
//   dense_expand_kernel  x = xp + Z y and the objective k0 + q^T y + 1/2 y^T P y (= the full-space
//                        x^T Hs x + c^T x + c0 at that x), written to pinned host memory.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/mpccbf.h"
#include "host/dense_pack.hpp"
#include "host/dense_qp.hpp"
#include "host/errors.hpp"
#include "kernels/group.hpp"
#include "kernels/das_wave.hpp"
#include "kernels/pdip.hpp"

namespace mpccbf {

constexpr int DENSE_NZ = 8;        // reduced dimension (padded)
constexpr int DENSE_ROWS = 256;    // reduced inequality rows: 64 lanes x 4 slots
constexpr int DENSE_NMAX = 64;     // variables per QP (lane = variable)
constexpr int DENSE_EMAX = 64;     // equalities per QP (lane = equality)
constexpr int DQ_R = DENSE_ROWS / 64;
constexpr int DQ_HDR = 2 * DENSE_NZ * DENSE_NZ + DENSE_NZ + 2;  // P, LP, q, reg, pad
constexpr int DQ_ROW = DENSE_NZ + 2;                            // g, lo, hi
constexpr double kInf = 1e300;     // |bound| >= 1e300 means "absent" (numeric_limits lowest/max)
constexpr double kFeasTol = 1e-6;  // CPLEX default feasibility tolerance (CPLEX.cpp:8 default ctor)
// reduce-kernel statuses beyond qpcpp::SolveStatus: -1 = the PDIP solves it; capacity errors
constexpr int RS_SOLVE = -1, RS_CAP_NZ = -2, RS_CAP_ROWS = -3;

// Packed QP (host -> device; dense_pack.hpp pack_qp). Int words: [n, me, mi, nh | in row ptr
// (mi + 1, int32) | eq row ptr (me + 1, u16) | Hs index (i << 6 | j, i <= j; nh, u16) | eq cols
// (u8) | in cols (u8)]. Doubles: [c (n) | c0 | Hs values (nh) | eq rhs (me) | eq values | in lo (mi)
// | in hi (mi) | in values]. Row pointers are relative to the QP; Hs = (H + H^T) / 2.
struct DenseBatch {
    const double* dbl;
    const int32_t* ints;
    const int64_t* off_d;  // per QP, + the total at [count]
    const int64_t* off_i;
    int32_t count;
    double* red;      // reduced QPs (the PDIP's input), QP k at red + red_off[k]: header + its rows
    const int64_t* red_off;  // per QP, sized by its inequality-row count (<= DENSE_ROWS rows)
    double* zx;       // count x (DENSE_NMAX x DENSE_NZ + DENSE_NMAX): Z row-major, then xp
    int32_t* status;  // count: decided status or RS_*
    int32_t* m;       // count: reduced rows
    int32_t* pd;      // count: 1 if P is positive definite (LP its factor)
    double* y;        // count x DENSE_NZ
    int32_t* iters;
    double* x;        // count x DENSE_NMAX (host, pinned: written by dense_expand_kernel)
    double* obj;      // count (host, pinned)
    int32_t* status_out;  // count (host, pinned): the final statuses
    int32_t maxit;
    double tol;
    double feas_tol;
    // count flags: 1 = reduced on the host (beyond the device elimination's 64 variables / 64
    // equalities; host/dense_qp.cpp), its reduced QP, status, m and pd uploaded, x expanded on the host
    const int32_t* hostred;  // (NULL: none)
    const int32_t* psize;    // count x 2: the packed form's doubles and ints (its slot, off_d / off_i, is a bound)
    int32_t lds_rows, lds_stride;  // the reduce kernel's E^T image (reduce_stride)
    // the packed input (dbl, ints, off_*, red_off, hostred) lives in pinned host memory and is read
    // by the kernels over the bus (no copy); the reduce kernel first stages its QP's packed words
    // into LDS with one batch of loads: stage_d / stage_i words (the batch's largest QP; 0: direct)
    int32_t stage_d, stage_i;
    int32_t first;  // dense_reduce_kernel: the slice's first QP (block b reduces QP first + b)
    int32_t das_steps;  // dense_qp_kernel: dual active-set steps before the PDIP (0: the PDIP alone)
    long long* dstamps;  // profiling build: QP 0's reduction phase stamps (24 words), else NULL
};

namespace dev {

// zero rows after the E^T image: the QR's row loops run in unguarded chunks of ET_PAD rows (16
// took the kernel to 141 registers, three waves per SIMD, for no gain in the QR)
constexpr int ET_PAD = 8;

// E^T / H image in dynamic LDS, sized per batch: rows = the batch's largest n, row stride S = the
// larger of its largest n and equality count, made odd (spread banks); at most 64 x 65 doubles
__host__ __device__ inline int reduce_stride(int nmax, int emax) {
    const int s = nmax > emax ? nmax : emax;
    return s | 1;
}

struct ReduceLds {
    double z[DENSE_NMAX * DENSE_NZ]; // Z row-major
    double xp[DENSE_NMAX];
    double hz[DENSE_NMAX * DENSE_NZ];
    double hx[DENSE_NMAX];
    double rdiag[DENSE_EMAX], beta[DENSE_EMAX], bp[DENSE_EMAX];
    double P[DENSE_NZ * DENSE_NZ];
    double Ps[DENSE_NZ * DENSE_NZ];  // symmetrised P (padding: identity), the Cholesky's input
    int32_t perm[DENSE_EMAX];
};

__device__ __forceinline__ bool fin_bound(double v) { return isfinite(v) && fabs(v) < kInf; }

// sum over rows i = t .. n-1 of the image's columns ca and cb (row stride S) in row order, in
// unguarded chunks of ET_PAD rows (the rows past n are zero: the image's own zero rows and its
// ET_PAD pad rows; their +0 terms leave the sum as the plain loop forms it), every chunk's loads first
__device__ __forceinline__ double col_dot_pad(const double* __restrict__ et, int S, int t, int n, int ca, int cb,
                                              int step = ET_PAD) {
    double acc = 0.0;
    for (int i0 = t; i0 < n; i0 += step) {
        const double* r0 = et + i0 * S;
        double x[ET_PAD], y[ET_PAD];
#pragma unroll
        for (int u = 0; u < ET_PAD; u++) {
            x[u] = r0[u * S + ca];
            y[u] = r0[u * S + cb];
        }
#pragma unroll
        for (int u = 0; u < ET_PAD; u++) acc = fma(x[u], y[u], acc);
    }
    return acc;
}


__global__ void __launch_bounds__(64) dense_reduce_kernel(const DenseBatch a) {
    const int qi = a.first + (int)blockIdx.x;
    const int l = threadIdx.x;
    if (qi >= a.count || (a.hostred && a.hostred[qi])) return;  // (reduced on the host)
    // profiling build (make prof): shader-clock stamps of the first QP's phases (dense_stamps)
#ifdef MPCCBF_PDIP_STAMPS
#define DSTAMP(k)                                                                                 \
    do {                                                                                          \
        if (a.dstamps && qi == 0 && l == 0) a.dstamps[k] = (long long)__builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define DSTAMP(k) \
    do {          \
    } while (0)
#endif
    DSTAMP(0);
    __shared__ ReduceLds s;
    extern __shared__ double et[];  // E^T: row i = variable, column c = equality (lane c)
    const int LDS_S = a.lds_stride, NROWS = a.lds_rows;
    const int32_t* ib = a.ints + a.off_i[qi];
    const double* db = a.dbl + a.off_d[qi];
    DSTAMP(1);
    if (a.stage_d > 0) {
        // the QP's packed words into LDS (after the E^T image): every load issued before any store,
        // 8 per lane in flight, so the bus latency is paid a few times instead of once per read
        double* sd = et + (size_t)(NROWS + ET_PAD) * LDS_S;
        int32_t* si = (int32_t*)(sd + a.stage_d);
        const int nd = a.psize[2 * qi], ni = a.psize[2 * qi + 1];  // (the packed sizes: the slot is a bound)
        // (doubles and ints in the same pass, 512 of each: 16 loads per lane in flight — two bus
        // round trips for a typical QP where separate passes took three)
        for (int e0 = 0; e0 < nd || e0 < ni; e0 += 8 * 64) {
            double v[8];
            int32_t w[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int e = e0 + u * 64 + l;
                v[u] = db[e < nd ? e : 0];
                w[u] = ib[e < ni ? e : 0];
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int e = e0 + u * 64 + l;
                if (e < nd) sd[e] = v[u];
                if (e < ni) si[e] = w[u];
            }
        }
        __syncthreads();
        db = sd;
        ib = si;
    }
    const int n = ib[0], me = ib[1], mi = ib[2], nh = ib[3];
    const int32_t* iptr = ib + 4;
    const uint16_t* eptr = (const uint16_t*)(iptr + mi + 1);
    const uint16_t* hidx = eptr + me + 1;
    const uint8_t* ecol = (const uint8_t*)(hidx + nh);
    const uint8_t* icol = ecol + eptr[me];
    const double* c = db;
    const double* hval = db + n + 1;
    const double* erhs = hval + nh;
    const double* eval = erhs + me;
    const double* ilo = eval + eptr[me];
    const double* ihi = ilo + mi;
    const double* ival = ihi + mi;
    double* red = a.red + a.red_off[qi];
    // inconsistent equalities (decided whatever the reduced dimension) / a constant row violated
    // (decided only within capacity: beyond it the rows' reduced coefficients are not all formed)
    bool infeasible = false, eq_infeasible = false;

    DSTAMP(2);
    // ---- E^T into LDS (lane c: equality c's row as column c), zero elsewhere
    for (int e = l; e < (NROWS + ET_PAD) * LDS_S; e += 64) et[e] = 0.0;
    __syncthreads();
    if (l < me) {
        for (int k = eptr[l]; k < eptr[l + 1]; k++) et[ecol[k] * LDS_S + l] = eval[k];
        s.perm[l] = l;
    }
    __syncthreads();
    DSTAMP(3);
    // ---- Householder QR with column pivoting: E^T Pi = Q R (reflection t stored in column t,
    // rows t .. n-1; R's diagonal in rdiag)
    const int tmax = n < me ? n : me;
    int rank = 0;
    double r00 = 0.0;
    // column norms over rows t .. n-1: reflection t's update forms the next step's in its row loop
    // from the values it stores (the same sum in the same row order: the separate loop over LDS
    // was a fifth of a reflection)
    double nrm_next = 0.0;
    // up to 32 equalities: two lanes per column (lanes 2c, 2c+1: alternate ET_PAD-row chunks, the
    // partial sums joined by one DPP move), halving every row loop's chain and loads
    const bool pair = me <= 32;
    const int cq = pair ? (l >> 1) : l;     // this lane's column
    const int h0 = pair ? (l & 1) * ET_PAD : 0;  // its first chunk's row offset
    const int cstep = pair ? 2 * ET_PAD : ET_PAD;
    auto join = [&](double v) { return pair ? v + dpp_mov<DPP_XOR1>(v) : v; };
    for (int t = 0; t < tmax; t++) {
        if (t == 10) DSTAMP(16);
        double nrm = -1.0;
        if (cq >= t && cq < me) nrm = t == 0 ? join(col_dot_pad(et, LDS_S, t + h0, n, cq, cq, cstep)) : nrm_next;
        if (t == 10) DSTAMP(11);
        const double best = grp_max<64>(nrm);
        const int pl = __ffsll((long long)__ballot(nrm == best && cq >= t && cq < me)) - 1;
        const int p = pl < 0 ? -1 : (pair ? pl >> 1 : pl);
        const double sig = sqrt(best);
        if (t == 0) r00 = sig;
        if (!(sig > 1e-12 * r00) || p < 0) break;  // the remaining columns are dependent
        if (t == 10) DSTAMP(12);
        // swap columns t and p (lane i: row i)
        if (p != t && l < n) {
            const double v = et[l * LDS_S + t];
            et[l * LDS_S + t] = et[l * LDS_S + p];
            et[l * LDS_S + p] = v;
        }
        if (p != t && l == 0) {
            const int q = s.perm[t];
            s.perm[t] = s.perm[p];
            s.perm[p] = q;
        }
        __syncthreads();
        if (t == 10) DSTAMP(13);
        const double xt = et[t * LDS_S + t];
        const double alpha = xt >= 0.0 ? -sig : sig;
        const double vt = xt - alpha;
        const double vn2 = best - xt * xt + vt * vt;  // |v|^2
        const double bt = vn2 > 0.0 ? 2.0 / vn2 : 0.0;
        __syncthreads();
        if (l == 0) {
            et[t * LDS_S + t] = vt;  // v = (vt, x_{t+1}, ...)
            s.rdiag[t] = alpha;
            s.beta[t] = bt;
        }
        __syncthreads();
        if (t == 10) DSTAMP(14);
        // apply to columns t+1 .. me-1 (lane c)
        if (cq > t && cq < me) {
            double w = join(col_dot_pad(et, LDS_S, t + h0, n, t, cq, cstep));
            w *= bt;
#ifdef MPCCBF_PDIP_STAMPS
            if (t == 10 && l == (pair ? 2 * (t + 1) : t + 1) && a.dstamps && qi == 0)
                a.dstamps[17] = (long long)__builtin_amdgcn_s_memtime();
#endif
            // (ET_PAD rows' loads before their stores, the pad rows' zeros included: as a plain loop each
            // row's store could alias the next row's loads for all the compiler knows, and every
            // row waited for its own LDS round trip — two thirds of a reflection's time)
            double acc = 0.0;
            for (int i0 = t + h0; i0 < n; i0 += cstep) {
                double* r0 = et + i0 * LDS_S;
                double x[ET_PAD], y[ET_PAD];
#pragma unroll
                for (int u = 0; u < ET_PAD; u++) {
                    x[u] = r0[u * LDS_S + t];
                    y[u] = r0[u * LDS_S + cq];
                }
#pragma unroll
                for (int u = 0; u < ET_PAD; u++) {
                    const double v = fma(-w, x[u], y[u]);
                    r0[u * LDS_S + cq] = v;
                    acc = fma(i0 + u > t ? v : 0.0, v, acc);  // (rows t+1 .. : the next norm)
                }
            }
            nrm_next = join(acc);
        }
        __syncthreads();
        if (t == 10) DSTAMP(15);
        rank = t + 1;
    }
    const int nz = n - rank;
    DSTAMP(4);
    // ---- particular solution: R11^T u = (Pi^T b)_{1..r}, xp = Q [u; 0]  (minimum norm)
    // (column-oriented: lane j holds b_j and takes R[t][j] u_t off it once u_t is known, u_t from
    // lane t by readlane — no reduction and no barrier per step)
    if (l < me) s.bp[l] = erhs[s.perm[l]];
    __syncthreads();
    double ul = 0.0;
    {
        double bl = l < rank ? s.bp[l] : 0.0;
        const double rdl = l < rank ? s.rdiag[l] : 1.0;
        for (int t = 0; t < rank; t++) {
            const double rt = l < rank ? et[t * LDS_S + l] : 0.0;  // R[t][l] (row t of R, lanes l > t)
            const double ut = readlane_d(bl / rdl, t);
            ul = l == t ? ut : ul;
            bl = l > t ? fma(-rt, ut, bl) : bl;
        }
    }
    DSTAMP(5);
    // reflections applied to the vectors [u; 0] and e_{r+j} (lane i: component i)
    double w = (l < rank) ? ul : 0.0;
    double zc[DENSE_NZ];
#pragma unroll
    for (int j = 0; j < DENSE_NZ; j++) zc[j] = (l == rank + j && j < nz) ? 1.0 : 0.0;
    for (int t = rank - 1; t >= 0; t--) {
        const double vi = (l >= t && l < n) ? et[l * LDS_S + t] : 0.0;
        const double bt = s.beta[t];
        // the nine reflection coefficients reduced together, stage-major (each value's reduction
        // tree is grp_sum's: bit-identical; one after the other, each waited for its DPP chain)
        double d[DENSE_NZ + 1];
        d[0] = vi * w;
#pragma unroll
        for (int j = 0; j < DENSE_NZ; j++) d[1 + j] = vi * zc[j];
        grp_sum_vec<64, DENSE_NZ + 1>(d);
        w = fma(-bt * d[0], vi, w);
#pragma unroll
        for (int j = 0; j < DENSE_NZ; j++) zc[j] = fma(-bt * d[1 + j], vi, zc[j]);
    }
    if (l < DENSE_NMAX) {
        s.xp[l] = l < n ? w : 0.0;
#pragma unroll
        for (int j = 0; j < DENSE_NZ; j++) s.z[l * DENSE_NZ + j] = (l < n && j < nz) ? zc[j] : 0.0;
        s.hx[l] = 0.0;
#pragma unroll
        for (int j = 0; j < DENSE_NZ; j++) s.hz[l * DENSE_NZ + j] = 0.0;
    }
    __syncthreads();
    // inconsistent equalities (redundant rows with a different right-hand side)
    if (l < me) {
        double v = 0.0;
        for (int k = eptr[l]; k < eptr[l + 1]; k++) v = fma(eval[k], s.xp[ecol[k]], v);
        if (fabs(v - erhs[l]) > kFeasTol) eq_infeasible = true;
    }
    DSTAMP(6);
    // ---- Hs Z and Hs xp, Hs = (H + H^T) / 2: the packed upper triangle's nonzeros scattered into
    // a dense n x n image in LDS (E^T's space, free from here; both triangles, each entry written
    // by one lane, so no atomics), then lane l forms row l over j = 0 .. n-1 — a fixed
    // summation order (no dependence on how the hardware orders LDS atomics), and no lane walks the
    // whole nonzero list (that serial scan of global loads and divisions cost ~1.7 ms per 4096-QP
    // call)
    for (int e = l; e < n * LDS_S; e += 64) et[e] = 0.0;
    __syncthreads();
    for (int e = l; e < nh; e += 64) {
        const int k = hidx[e], i = k >> 6, j = k & 63;
        const double v = hval[e];
        et[i * LDS_S + j] = v;  // (both triangles: row l of the image is then read along j,
        et[j * LDS_S + i] = v;  // consecutive lanes on consecutive words)
    }
    __syncthreads();
    if (l < n) {
        double hxl = 0.0, hzl[DENSE_NZ];
#pragma unroll
        for (int b = 0; b < DENSE_NZ; b++) hzl[b] = 0.0;
        for (int j = 0; j < n; j++) {
            const double hv = et[j * LDS_S + l];
            hxl = fma(hv, s.xp[j], hxl);
#pragma unroll
            for (int b = 0; b < DENSE_NZ; b++) hzl[b] = fma(hv, s.z[j * DENSE_NZ + b], hzl[b]);
        }
        s.hx[l] = hxl;
#pragma unroll
        for (int b = 0; b < DENSE_NZ; b++) s.hz[l * DENSE_NZ + b] = hzl[b];
    }
    __syncthreads();
    // P = 2 Z^T Hs Z (lane a * 8 + b), q = Z^T (2 Hs xp + c), k0 (objective constant: unused,
    // the expansion evaluates the full-space objective)
    if (nz <= DENSE_NZ) {
        const int pa = l >> 3, pb = l & 7;
        double v = 0.0;
        for (int i = 0; i < n; i++) v = fma(s.z[i * DENSE_NZ + pa], s.hz[i * DENSE_NZ + pb], v);
        s.P[pa * DENSE_NZ + pb] = 2.0 * v;
    }
    __syncthreads();
    double pmax = 0.0;
    if (l < DENSE_NZ * DENSE_NZ && nz <= DENSE_NZ) {
        const int pa = l >> 3, pb = l & 7;
        const bool in = pa < nz && pb < nz;
        const double v = in ? 0.5 * (s.P[pa * DENSE_NZ + pb] + s.P[pb * DENSE_NZ + pa]) : (pa == pb ? 1.0 : 0.0);
        red[l] = v;  // P (padding: identity)
        s.Ps[l] = v;  // (the Cholesky's copy)
        pmax = in ? fabs(v) : 0.0;
    }
    pmax = grp_max<64>(pmax);
    __syncthreads();
    if (l < DENSE_NZ && nz <= DENSE_NZ) {
        double v = 0.0;
        if (l < nz)
            for (int i = 0; i < n; i++) v = fma(s.z[i * DENSE_NZ + l], 2.0 * s.hx[i] + c[i], v);
        red[2 * DENSE_NZ * DENSE_NZ + l] = v;  // q
    }
    // the objective's constant at y = 0: c0 + xp^T (Hs xp + c) (the expansion evaluates
    // k0 + q^T y + 1/2 y^T P y: the full-space objective at x = xp + Z y)
    const double k0 = db[n] + grp_sum<64>(l < n ? s.xp[l] * (s.hx[l] + c[l]) : 0.0);
    // Cholesky of P (lane 0, in LDS; nz <= 8): the PDIP's start factor when P is positive definite
    DSTAMP(7);
    int pd = 0;
    if (l == 0 && nz <= DENSE_NZ) {
        // in registers (unrolled over the padded 8 x 8, guarded by nz) from the LDS copy of P: the
        // loop over LDS read P back from global memory and kept L in LDS, one round trip per entry
        double Pm[DENSE_NZ * DENSE_NZ], L[DENSE_NZ * DENSE_NZ];
#pragma unroll
        for (int j = 0; j < DENSE_NZ * DENSE_NZ; j++) {
            Pm[j] = s.Ps[j];
            L[j] = 0.0;
        }
        bool ok = nz > 0;
#pragma unroll
        for (int j = 0; j < DENSE_NZ; j++) {
            if (j < nz && ok) {
                double d = Pm[j * DENSE_NZ + j];
#pragma unroll
                for (int k = 0; k < j; k++) d -= L[j * DENSE_NZ + k] * L[j * DENSE_NZ + k];
                if (!(d > 0.0)) {
                    ok = false;
                } else {
                    const double ljj = sqrt(d);
                    L[j * DENSE_NZ + j] = ljj;
#pragma unroll
                    for (int i = j + 1; i < DENSE_NZ; i++) {
                        if (i < nz) {
                            double v = Pm[i * DENSE_NZ + j];
#pragma unroll
                            for (int k = 0; k < j; k++) v -= L[i * DENSE_NZ + k] * L[j * DENSE_NZ + k];
                            L[i * DENSE_NZ + j] = v / ljj;
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < DENSE_NZ * DENSE_NZ; j++) {
            const int r = j / DENSE_NZ, cc = j % DENSE_NZ;
            red[DENSE_NZ * DENSE_NZ + j] = (ok && r < nz) ? L[j] : (r == cc ? 1.0 : 0.0);  // padding: identity
        }
        red[2 * DENSE_NZ * DENSE_NZ + DENSE_NZ] = ok ? 0.0 : 1e-10 * fmax(1.0, pmax);  // Newton ridge if PSD
        red[2 * DENSE_NZ * DENSE_NZ + DENSE_NZ + 1] = k0;
        pd = ok ? 1 : 0;
    }
    DSTAMP(8);
    // ---- inequality rows in y: g = Z^T a, bounds shifted by a^T xp; constant rows decided here
    int cnt = 0;
    double* rows = red + DQ_HDR;
    for (int r0 = 0; r0 < mi; r0 += 64) {
        const int r = r0 + l;
        bool keep = false;
        double g[DENSE_NZ], lo = 0.0, hi = 0.0;
#pragma unroll
        for (int b = 0; b < DENSE_NZ; b++) g[b] = 0.0;
        if (r < mi && nz <= DENSE_NZ) {
            double amax = 0.0, shift = 0.0, gmax = 0.0;
            for (int k = iptr[r]; k < iptr[r + 1]; k++) {
                const double av = ival[k];
                const int j = icol[k];
                amax = fmax(amax, fabs(av));
                shift = fma(av, s.xp[j], shift);
#pragma unroll
                for (int b = 0; b < DENSE_NZ; b++) g[b] = fma(av, s.z[j * DENSE_NZ + b], g[b]);
            }
#pragma unroll
            for (int b = 0; b < DENSE_NZ; b++) gmax = fmax(gmax, fabs(g[b]));
            const double rl = ilo[r], rh = ihi[r];
            const bool hl = fin_bound(rl), hu = fin_bound(rh);
            if (gmax <= 1e-13 * fmax(1.0, amax)) {  // constant row: a feasibility check of xp
                if ((hl && shift < rl - kFeasTol) || (hu && shift > rh + kFeasTol)) infeasible = true;
            } else {
                keep = true;
                lo = hl ? rl - shift : -kInf;
                hi = hu ? rh - shift : kInf;
            }
        }
        const unsigned long long msk = __ballot(keep);
        const int slot = cnt + __popcll(msk & ((1ull << l) - 1ull));
        if (keep && slot < DENSE_ROWS) {
            double* dst = rows + (size_t)slot * DQ_ROW;
#pragma unroll
            for (int b = 0; b < DENSE_NZ; b++) dst[b] = g[b];
            dst[DENSE_NZ] = lo;
            dst[DENSE_NZ + 1] = hi;
        }
        cnt += __popcll(msk);
    }
    infeasible = __ballot(infeasible) != 0ull;
    eq_infeasible = __ballot(eq_infeasible) != 0ull;
    DSTAMP(9);
    // ---- expansion data and the decision
    double* zx = a.zx + (size_t)qi * (DENSE_NMAX * DENSE_NZ + DENSE_NMAX);
    for (int e = l; e < DENSE_NMAX * DENSE_NZ; e += 64) zx[e] = s.z[e];
    zx[DENSE_NMAX * DENSE_NZ + l] = s.xp[l];
    if (l < DENSE_NZ) a.y[(size_t)qi * DENSE_NZ + l] = 0.0;  // (the PDIP overwrites it when it solves)
    if (l == 0) {
        int st = RS_SOLVE;
        if (eq_infeasible) st = ST_INFEASIBLE;  // (before the capacity checks: as the host path did)
        else if (nz > DENSE_NZ) st = RS_CAP_NZ;
        else if (cnt > DENSE_ROWS) st = RS_CAP_ROWS;
        else if (infeasible) st = ST_INFEASIBLE;
        else if (nz == 0) st = ST_OPTIMAL;  // x = xp is the only point
        a.status[qi] = st;
        a.m[qi] = cnt < DENSE_ROWS ? cnt : DENSE_ROWS;
        a.pd[qi] = pd;
    }
    DSTAMP(10);
}
#undef DSTAMP

// x = xp + Z y and the objective of OPTIMAL QP qi (y: the reduced solution, global or LDS), its
// final status into the pinned output (one wave)
__device__ __forceinline__ void dense_expand_qp(const DenseBatch& a, int qi, int st, const double* yq, int l) {
    if (l == 0) a.status_out[qi] = st;
    if (st != ST_OPTIMAL || (a.hostred && a.hostred[qi])) return;  // (host-reduced: host expands)
    // x = xp + Z y; the objective from the reduced QP, k0 + q^T y + 1/2 y^T P y (P, q, k0 in the
    // device block the reduction wrote: nothing read from the host input)
    const double* zx = a.zx + (size_t)qi * (DENSE_NMAX * DENSE_NZ + DENSE_NMAX);
    const double* red = a.red + a.red_off[qi];
    double xv = zx[DENSE_NMAX * DENSE_NZ + l];
#pragma unroll
    for (int b = 0; b < DENSE_NZ; b++) xv = fma(zx[l * DENSE_NZ + b], yq[b], xv);
    const int pa = l >> 3, pb = l & 7;  // lane (a, b): 1/2 P_ab y_a y_b; lanes 0..7 also q_l y_l
    double f = 0.5 * red[l] * yq[pa] * yq[pb];
    if (l < DENSE_NZ) f = fma(red[2 * DENSE_NZ * DENSE_NZ + l], yq[l], f);
    f = grp_sum<64>(f);
    a.x[(size_t)qi * DENSE_NMAX + l] = xv;  // (beyond n: 0; the host copies n)
    if (l == 0) a.obj[qi] = f + red[2 * DENSE_NZ * DENSE_NZ + DENSE_NZ + 1];
}

// The dual active set (das_wave.hpp, the FoV controller's) on the reduced QP's row image, before
// the PDIP: a QP with P positive definite whose rows fit the image. An optimum it returns is the
// QP's exact optimum (primal and dual residuals checked): status OPTIMAL, y, its steps. Anything
// else (no feasible point in sight, the step limit, a breakdown) stays RS_SOLVE for
// dense_qp_kernel's PDIP and phase 1, as before. (Its own launch: inlined into the PDIP kernel
// its state pushed that kernel into scratch.)
template <int NZ>
__global__ void __launch_bounds__(64) dense_das_kernel(const DenseBatch a) {
    const int qi = blockIdx.x;
    const int gl = threadIdx.x;
    if (qi >= a.count) return;
    {
        const int st0 = a.status[qi];
        if (st0 != RS_SOLVE) {  // decided by the reduction: its final status (and x) now
            dense_expand_qp(a, qi, st0, a.y + (size_t)qi * NZ, gl);
            return;
        }
    }
    const double* base = a.red + a.red_off[qi];
    const double* P = base;
    const double* LP = base + NZ * NZ;
    const double* qv = base + 2 * NZ * NZ;
    const double* rows = base + DQ_HDR;
    const int m = a.m[qi];
    const bool pd = a.pd[qi] != 0;
    if (gl == 0) a.status_out[qi] = RS_SOLVE;  // (unsettled so far: the host's check, small batches)
    double q[NZ];
#pragma unroll
    for (int i = 0; i < NZ; i++) q[i] = qv[i];
    // first: the dual active set (das_wave.hpp, the FoV controller's) on the row image, when P is
    // positive definite and the rows fit its image; an optimum it returns is the QP's exact
    // optimum (primal and dual residuals checked); anything else (no feasible point found, a
    // step limit, a breakdown) goes to the PDIP below as before
    if (pd && m <= WROWS && __builtin_amdgcn_readfirstlane(a.das_steps) > 0) {
        static_assert(NZ <= WNZ, "the reduced dimension fits the 16-wide image");
        __shared__ double Gimg[(WROWS + 1) * WNZ];  // (rows 0 .. m - 1, then row m all zero)
        __shared__ double Pi8[NZ * NZ];             // P^-1 (from its Cholesky factor LP)
        __shared__ WaveScratch sc;
        __shared__ WaveAS ws;
        // image rows: g (NZ) then zeros to WNZ; row m all zero (the unused slots' row)
        for (int e = gl; e < (m + 1) * WNZ; e += 64) {
            const int r = e / WNZ, j = e - r * WNZ;
            Gimg[e] = (r < m && j < NZ) ? rows[(size_t)r * DQ_ROW + j] : 0.0;
        }
        // P^-1 column j = LP^-T LP^-1 e_j (lane j < NZ; LP lower triangular, row-major)
        if (gl < NZ) {
            double z[NZ];
#pragma unroll
            for (int i = 0; i < NZ; i++) {
                double v = i == gl ? 1.0 : 0.0;
#pragma unroll
                for (int k = 0; k < i; k++) v = fma(-LP[i * NZ + k], z[k], v);
                z[i] = v / LP[i * NZ + i];
            }
#pragma unroll
            for (int i = NZ - 1; i >= 0; i--) {
                double v = z[i];
#pragma unroll
                for (int k = i + 1; k < NZ; k++) v = fma(-LP[k * NZ + i], z[k], v);
                z[i] = v / LP[i * NZ + i];
            }
#pragma unroll
            for (int i = 0; i < NZ; i++) Pi8[i * NZ + gl] = z[i];
        }
        if (gl < WNZ) sc.q[gl] = gl < NZ ? q[gl < NZ ? gl : 0] : 0.0;
        wave_lds_sync();
        {
            // the operators padded to 16 x 16 with the identity (das_store_operators' entries)
            constexpr int NE = WNZ * WNZ / 64;
            double pi[NE], pp[NE];
#pragma unroll
            for (int k = 0; k < NE; k++) {
                const int e = gl + 64 * k, i = e >> 4, j = e & 15;
                const bool in = i < NZ && j < NZ;
                pi[k] = in ? Pi8[(in ? i : 0) * NZ + (in ? j : 0)] : (i == j ? 1.0 : 0.0);
                pp[k] = in ? P[(in ? i : 0) * NZ + (in ? j : 0)] : (i == j ? 1.0 : 0.0);
            }
            das_store_operators(ws, pi, pp, gl);
        }
        WaveRows wr;
#pragma unroll
        for (int sl = 0; sl < WR; sl++) {
            const int r = wave_owner_row(gl, sl);
            const bool on = r < m;
            const double* src = rows + (size_t)(on ? r : 0) * DQ_ROW;
            const double l = on ? src[NZ] : -1e300, h = on ? src[NZ + 1] : 1e300;
            wr.g[sl] = &Gimg[(on ? r : m) * WNZ];  // (row m: the zeroed row after the image)
            // (every row has an upper side: a row without one gets an unreachable bound)
            wr.hi[sl] = on ? (h < 1e300 ? h : 1e300) : 1.0;
            wr.lo[sl] = on ? (l > -1e300 ? l : 0.0) : -1.0;
            wr.ml[sl] = on ? (l > -1e300 ? 1.0 : 0.0) : 1.0;
        }
        double drp = 0.0, drd = 0.0, tlow = 0.0;
        int dsteps = 0;
        const int r = das_solve_wave(wr, Gimg, sc, ws, nullptr, nullptr, a.tol, a.das_steps, false, gl, drp, drd,
                                     dsteps, tlow, nullptr, 0, m, nullptr, false);
        if (r == 1) {
            if (gl == 0) {
                a.status[qi] = ST_OPTIMAL;
                a.iters[qi] = dsteps;
#pragma unroll
                for (int i = 0; i < NZ; i++) a.y[(size_t)qi * NZ + i] = sc.y[i];
            }
            dense_expand_qp(a, qi, ST_OPTIMAL, sc.y, gl);  // (x, objective, the final status)
            return;
        }
    }
}

template <int NZ, int R>
__global__ void __launch_bounds__(64) dense_qp_kernel(const DenseBatch a) {
    const int qi = blockIdx.x;
    const int gl = threadIdx.x;
    if (qi >= a.count || a.status[qi] != RS_SOLVE) return;  // decided by the reduction
    const double* base = a.red + a.red_off[qi];
    const double* P = base;
    const double* LP = base + NZ * NZ;
    const double* qv = base + 2 * NZ * NZ;
    const double reg = qv[NZ];
    const double* rows = base + DQ_HDR;
    const int m = a.m[qi];
    const bool pd = a.pd[qi] != 0;

    double q[NZ], y[NZ];
#pragma unroll
    for (int i = 0; i < NZ; i++) q[i] = qv[i];
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

// x = xp + Z y (y = 0 when the equalities decided x) and the objective for OPTIMAL QPs; every
// QP's final status into the pinned output.
__global__ void __launch_bounds__(64) dense_expand_kernel(const DenseBatch a) {
    const int qi = blockIdx.x;
    const int l = threadIdx.x;
    if (qi >= a.count) return;
    dense_expand_qp(a, qi, a.status[qi], a.y + (size_t)qi * DENSE_NZ, l);
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
struct HostBuf {  // pinned (page-locked, device-mapped) host memory the kernels read / write
    void* p = nullptr;
    void* dp = nullptr;  // the device's pointer to it
    size_t bytes = 0;
    hipError_t reserve(size_t need) {
        if (p && bytes >= need) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = dp = nullptr;
        bytes = 0;
        need += need / 4;  // (headroom: a slightly larger batch does not pin again)
        hipError_t e = hipHostMalloc(&p, need, hipHostMallocMapped);
        if (e == hipSuccess) e = hipHostGetDevicePointer(&dp, p, 0);
        if (e == hipSuccess) bytes = need;
        return e;
    }
    // device address of a host address inside the buffer
    template <typename T>
    T* dev(const void* h) const { return (T*)((char*)dp + ((const char*)h - (const char*)p)); }
};
thread_local DevBuf g_dense_buf;
thread_local HostBuf g_dense_host;
thread_local HostBuf g_dense_out;  // pinned x | obj | status of the last call

size_t align16(size_t v) { return (v + 15) & ~size_t(15); }

static_assert(dense_pack::DENSE_NMAX == DENSE_NMAX && dense_pack::DENSE_EMAX == DENSE_EMAX &&
              dense_pack::kInf == kInf, "dense_pack.hpp and dense_qp.hip agree");
using dense_pack::finite_bound;
using dense_pack::PackPlan;
using dense_pack::plan_qp;

// Host worker pool for the per-QP validation and packing: created on first use (up to 15 workers
// beside the calling thread), kept for the process (a thread spawn per call cost more than the
// packing of a small batch). One batch at a time uses it (a second concurrent caller packs on its
// own thread).
class PackPool {
  public:
    static PackPool& get() {
        static PackPool* p = new PackPool();  // never destroyed: workers block on the condition at exit
        return *p;
    }
    int width() const { return (int)workers_.size() + 1; }
    // f(k0, k1) over [0, count) in width() chunks; the caller runs chunk 0
    void run(int count, const std::function<void(int, int)>& f) {
        std::unique_lock<std::mutex> busy(busy_, std::try_to_lock);
        const int w = width();
        if (!busy.owns_lock() || w == 1 || count < 64) {
            f(0, count);
            return;
        }
        const int chunk = (count + w - 1) / w;
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &f;
            count_ = count;
            chunk_ = chunk;
            pending_ = (int)workers_.size();
            gen_++;
        }
        cv_.notify_all();
        f(0, std::min(count, chunk));
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    PackPool() {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const int nw = (int)std::min(15u, hw - 1);
        for (int t = 0; t < nw; t++) {
            workers_.emplace_back([this, t] { loop(t + 1); });
            workers_.back().detach();
        }
    }
    void loop(int idx) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int, int)>* f;
            int k0, k1;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                f = job_;
                k0 = std::min(count_, idx * chunk_);
                k1 = std::min(count_, k0 + chunk_);
            }
            if (k0 < k1) (*f)(k0, k1);
            std::lock_guard<std::mutex> lk(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex busy_, m_;
    std::condition_variable cv_, done_;
    const std::function<void(int, int)>* job_ = nullptr;
    int count_ = 0, chunk_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
};

template <typename F>
void parallel_for(int count, F f) {
    const std::function<void(int, int)> fn(f);
    PackPool::get().run(count, fn);
}

}  // namespace
}  // namespace mpccbf

using namespace mpccbf;

extern "C" {

int mpccbf_qp_solve_dense_batch(int32_t count, const mpccbf_dense_qp* qps, double* const* x_out,
                                double* obj_out, int32_t* status_out) {
    if (count < 0 || (count > 0 && (!qps || !status_out)))
        return set_error(MPCCBF_ERR_INVALID_ARGUMENT, "dense QP batch: null argument");
    if (count == 0) return MPCCBF_OK;
    // ---- host, one pass per QP (worker pool, slice by slice ahead of each slice's reduction):
    // validation, row classification and the packed form written straight into the pinned input,
    // at an offset sized beforehand from n and m alone (an upper bound of the packed size: no
    // separate sizing pass over H and A). The kernels read it there over the bus: no copy
    std::vector<int64_t> off_d(count + 1), off_i(count + 1), red_off(count);
    size_t nd = 0, ni = 0, nred = 0;
    for (int k = 0; k < count; k++) {
        off_d[k] = (int64_t)nd;
        off_i[k] = (int64_t)ni;
        red_off[k] = (int64_t)nred;
        const int64_t n = qps[k].n, m = qps[k].m;
        const bool packable = n >= 1 && n <= DENSE_NMAX && m >= 0;
        if (packable) {  // (the sizes of pack_qp with nh <= n (n + 1) / 2, me + mi <= m + n, enz + inz <= m n + n)
            const int64_t hmax = n * (n + 1) / 2, rows = m + n, nzmax = m * n + n;
            nd += (size_t)(n + 1 + hmax + 2 * rows + nzmax) + 1;  // (+1: the spare word of pack_qp's compaction)
            ni += (size_t)(4 + (rows + 1) + (2 * (rows + 1) + 2 * hmax + nzmax + 3) / 4) + 1;
        }
        // reduced-QP block: its reduced rows are a subset of the inequality rows (<= m + n); a QP
        // with more than DENSE_ROWS is a capacity error before its rows are read
        const int64_t rows_k = (n >= 1 && m >= 0) ? std::min<int64_t>(m + n, DENSE_ROWS) : 1;
        nred += (size_t)DQ_HDR + (size_t)std::max<int64_t>(rows_k, 1) * DQ_ROW;  // (>= 1 row: the kernel reads row 0)
    }
    off_d[count] = (int64_t)nd;
    off_i[count] = (int64_t)ni;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        // (no device: the QPs' own argument errors still take precedence, as a host-side check)
        for (int k = 0; k < count; k++) {
            const PackPlan pl = plan_qp(qps[k]);
            if (!pl.err.empty()) return set_error(MPCCBF_ERR_INVALID_ARGUMENT, "QP " + std::to_string(k) + ": " + pl.err);
        }
        return set_error(MPCCBF_ERR_NO_DEVICE, "no HIP device visible");
    }
    int device = 0;
    hipError_t e = hipGetDevice(&device);
    // ---- pinned input: packed doubles | packed ints | off_d | off_i | red_off | host-reduced
    // flags | packed sizes (2 per QP); pinned output: x | obj | status
    const size_t b_d = align16(nd * sizeof(double)), b_i = align16(ni * sizeof(int32_t));
    const size_t b_off = align16((size_t)(count + 1) * sizeof(int64_t));
    const size_t b_int = align16((size_t)count * sizeof(int32_t));
    const size_t b_ps = align16((size_t)count * 2 * sizeof(int32_t));
    const size_t in_bytes = b_d + b_i + 3 * b_off + b_int + b_ps;
    const size_t b_x = align16((size_t)count * DENSE_NMAX * sizeof(double));
    const size_t b_obj = align16((size_t)count * sizeof(double));
    if (e == hipSuccess) e = g_dense_host.reserve(in_bytes);
    if (e == hipSuccess) e = g_dense_out.reserve(b_x + b_obj + b_int);
    if (e != hipSuccess) return set_error(MPCCBF_ERR_HIP, std::string("dense QP staging: ") + hipGetErrorString(e));
    char* hb = (char*)g_dense_host.p;
    double* h_d = (double*)hb;
    int32_t* h_i = (int32_t*)(hb + b_d);
    int64_t* h_offd = (int64_t*)(hb + b_d + b_i);
    int64_t* h_offi = (int64_t*)(hb + b_d + b_i + b_off);
    int64_t* h_redoff = (int64_t*)(hb + b_d + b_i + 2 * b_off);
    int32_t* h_hr = (int32_t*)(hb + b_d + b_i + 3 * b_off);
    int32_t* h_ps = (int32_t*)(hb + b_d + b_i + 3 * b_off + b_int);
    std::memcpy(h_offd, off_d.data(), (count + 1) * sizeof(int64_t));
    std::memcpy(h_offi, off_i.data(), (count + 1) * sizeof(int64_t));
    std::memcpy(h_redoff, red_off.data(), count * sizeof(int64_t));
    // ---- device buffers: reduced QPs | Z, xp | y | status | m | pd | iters
    const size_t b_red = align16(nred * sizeof(double));
    const size_t b_zx = align16((size_t)count * (DENSE_NMAX * DENSE_NZ + DENSE_NMAX) * sizeof(double));
    const size_t b_y = align16((size_t)count * DENSE_NZ * sizeof(double));
    e = g_dense_buf.reserve(b_red + b_zx + b_y + 4 * b_int, device);
    if (e != hipSuccess) return set_error(MPCCBF_ERR_HIP, std::string("dense QP buffers: ") + hipGetErrorString(e));
    char* p = (char*)g_dense_buf.p;
    DenseBatch a;
    a.dbl = g_dense_host.dev<const double>(h_d);
    a.ints = g_dense_host.dev<const int32_t>(h_i);
    a.off_d = g_dense_host.dev<const int64_t>(h_offd);
    a.off_i = g_dense_host.dev<const int64_t>(h_offi);
    a.red_off = g_dense_host.dev<const int64_t>(h_redoff);
    a.hostred = g_dense_host.dev<const int32_t>(h_hr);
    a.psize = g_dense_host.dev<const int32_t>(h_ps);
    a.count = count;
    a.red = (double*)p;
    p += b_red;
    a.zx = (double*)p;
    p += b_zx;
    a.y = (double*)p;
    p += b_y;
    a.status = (int32_t*)p;
    a.m = (int32_t*)(p + b_int);
    a.pd = (int32_t*)(p + 2 * b_int);
    a.iters = (int32_t*)(p + 3 * b_int);
    char* ho = (char*)g_dense_out.p;
    a.x = g_dense_out.dev<double>(ho);
    a.obj = g_dense_out.dev<double>(ho + b_x);
    a.status_out = g_dense_out.dev<int32_t>(ho + b_x + b_obj);
    a.maxit = 100;
    a.das_steps = 48;
    a.tol = 1e-9;
    a.feas_tol = 1e-6;
    a.dstamps = nullptr;
#ifdef MPCCBF_PDIP_STAMPS
    // profiling build: QP 0's reduction phases, printed to stderr with MPCCBF_DENSE_STAMPS=1
    static long long* d_stamps = nullptr;
    const bool want_stamps = std::getenv("MPCCBF_DENSE_STAMPS") != nullptr;
    if (want_stamps && !d_stamps && hipMalloc(&d_stamps, 24 * sizeof(long long)) != hipSuccess) d_stamps = nullptr;
    if (want_stamps && d_stamps) {
        (void)hipMemset(d_stamps, 0, 24 * sizeof(long long));
        a.dstamps = d_stamps;
    }
#endif
    hipStream_t s = nullptr;
    std::vector<PackPlan> plan(count);
    // QPs beyond the device elimination (more than 64 variables or 64 equality rows): the equality
    // elimination on the host (host/dense_qp.cpp, after the slices), the reduced QP solved on the
    // device like the rest
    std::vector<int> big;
    int rows_max = 1;
    // validate + pack a slice (worker pool), launch its reduction (sized by the slice's own
    // largest QP), pack the next meanwhile; the first bad QP's error as a serial pass would report
    // it (the slices before it are finished first: the pinned input stays theirs until then)
    const int nslice = count >= 1024 ? 4 : 1;
    const int slice = (count + nslice - 1) / nslice;
    for (int q0 = 0; q0 < count && e == hipSuccess; q0 += slice) {
        const int q1 = std::min(count, q0 + slice);
        parallel_for(q1 - q0, [&](int k0, int k1) {
            thread_local dense_pack::PackScratch scratch;
            for (int k = q0 + k0; k < q0 + k1; k++) {
                plan[k] = dense_pack::pack_qp_once(qps[k], h_d + off_d[k], h_i + off_i[k], scratch);
                const PackPlan& pl = plan[k];
                const bool packed = pl.err.empty() && !pl.cap;
                h_hr[k] = pl.cap ? 1 : 0;
                h_ps[2 * k] = packed ? (int32_t)pl.nd + 1 : 0;  // (+1: the spare word, staged as before)
                h_ps[2 * k + 1] = packed ? (int32_t)pl.ni + 1 : 0;
            }
        });
        int nmax = 1, emax = 1, sd_max = 0, si_max = 0;
        for (int k = q0; k < q1; k++) {
            if (!plan[k].err.empty()) {
                (void)hipStreamSynchronize(s);
                return set_error(MPCCBF_ERR_INVALID_ARGUMENT, "QP " + std::to_string(k) + ": " + plan[k].err);
            }
            if (plan[k].cap) {
                big.push_back(k);
                continue;
            }
            rows_max = std::max(rows_max, std::min(plan[k].mi, DENSE_ROWS));
            nmax = std::max(nmax, plan[k].n);
            emax = std::max(emax, plan[k].me);
            sd_max = std::max(sd_max, (int)plan[k].nd + 1);
            si_max = std::max(si_max, (int)plan[k].ni + 1);
        }
        a.lds_rows = nmax;
        a.lds_stride = dev::reduce_stride(nmax, emax);
        size_t lds = (size_t)(a.lds_rows + dev::ET_PAD) * a.lds_stride * sizeof(double);
        const size_t stage = (size_t)sd_max * sizeof(double) + (size_t)si_max * sizeof(int32_t);
        a.stage_d = a.stage_i = 0;
        if (lds + stage <= 48 * 1024) {  // (beyond: the kernel reads its QP over the bus where it uses it)
            a.stage_d = sd_max;
            a.stage_i = si_max;
            lds += stage;
        }
        a.first = q0;
        hipLaunchKernelGGL(dev::dense_reduce_kernel, dim3(q1 - q0), dim3(64), lds, s, a);
        e = hipGetLastError();
    }
    std::vector<ReducedQP> hred(big.size());
    for (size_t b = 0; b < big.size() && e == hipSuccess; b++) {
        try {
            hred[b] = reduce_dense_qp(qps[big[b]]);
        } catch (const std::exception& ex) {
            (void)hipStreamSynchronize(s);
            return set_error(MPCCBF_ERR_INVALID_ARGUMENT, "QP " + std::to_string(big[b]) + ": " + ex.what());
        }
        rows_max = std::max(rows_max, std::min(hred[b].m, DENSE_ROWS));
    }
    a.first = 0;
    // host-reduced QPs: their reduced form in the device layout (P, LP padded with the identity, q,
    // the Newton ridge when P is only semidefinite, rows [g | lo | hi]) and the decision
    std::vector<std::vector<double>> hblk(big.size());
    std::vector<int32_t> hst(big.size()), hm(big.size()), hpd(big.size());
    for (size_t b = 0; b < big.size() && e == hipSuccess; b++) {
        const ReducedQP& r = hred[b];
        int st_b = RS_SOLVE;
        // the device kernel's order (dense_reduce_kernel): inconsistent equalities, then capacity,
        // then a violated constant row
        if (r.eq_infeasible) st_b = MPCCBF_INFEASIBLE;
        else if (r.nz > DENSE_NZ) st_b = RS_CAP_NZ;
        else if (r.m > DENSE_ROWS) st_b = RS_CAP_ROWS;
        else if (r.status >= 0) st_b = r.status;  // (a violated constant row; nz = 0: x = xp)
        std::vector<double>& blk = hblk[b];
        blk.assign((size_t)DQ_HDR + (size_t)std::min(r.m, DENSE_ROWS) * DQ_ROW, 0.0);
        double pmax = 0.0;
        if (st_b == RS_SOLVE) {
            for (int i = 0; i < DENSE_NZ; i++)
                for (int j = 0; j < DENSE_NZ; j++) {
                    const bool in = i < r.nz && j < r.nz;
                    blk[i * DENSE_NZ + j] = in ? r.P(i, j) : (i == j ? 1.0 : 0.0);
                    blk[DENSE_NZ * DENSE_NZ + i * DENSE_NZ + j] =
                        (in && r.pd) ? (j <= i ? r.LP(i, j) : 0.0) : (i == j ? 1.0 : 0.0);
                    if (in) pmax = std::max(pmax, std::fabs(r.P(i, j)));
                }
            for (int i = 0; i < r.nz; i++) blk[2 * DENSE_NZ * DENSE_NZ + i] = r.q[i];
            blk[2 * DENSE_NZ * DENSE_NZ + DENSE_NZ] = r.pd ? 0.0 : 1e-10 * std::max(1.0, pmax);
            for (int k = 0; k < r.m && k < DENSE_ROWS; k++) {
                double* row = &blk[DQ_HDR + (size_t)k * DQ_ROW];
                for (int j = 0; j < r.nz; j++) row[j] = r.G(k, j);
                row[DENSE_NZ] = r.lo[k];
                row[DENSE_NZ + 1] = r.hi[k];
            }
        }
        hst[b] = st_b;
        hm[b] = std::min(r.m, DENSE_ROWS);
        hpd[b] = r.pd ? 1 : 0;
        const int k = big[b];
        e = hipMemcpyAsync(a.red + red_off[k], blk.data(), blk.size() * sizeof(double), hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(a.status + k, &hst[b], sizeof(int32_t), hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(a.m + k, &hm[b], sizeof(int32_t), hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(a.pd + k, &hpd[b], sizeof(int32_t), hipMemcpyHostToDevice, s);
    }
    // the active-set launch settles most QPs and writes their final outputs (and those of the QPs
    // the reduction decided); a small batch whose QPs it all settled needs no PDIP and no
    // expansion launch (the host checks the pinned statuses after one synchronisation)
    bool settled = false;
    if (e == hipSuccess && a.das_steps > 0 && rows_max <= dev::WROWS) {
        hipLaunchKernelGGL((dev::dense_das_kernel<DENSE_NZ>), dim3(count), dim3(64), 0, s, a);
        e = hipGetLastError();
        if (e == hipSuccess && count <= 64 && big.empty()) {
            e = hipStreamSynchronize(s);
            const int32_t* so = (const int32_t*)(ho + b_x + b_obj);
            settled = e == hipSuccess;
            for (int k = 0; k < count && settled; k++) settled = so[k] != RS_SOLVE;
        }
    }
    if (e == hipSuccess && !settled) {
        if (rows_max <= 64) hipLaunchKernelGGL((dev::dense_qp_kernel<DENSE_NZ, 1>), dim3(count), dim3(64), 0, s, a);
        else if (rows_max <= 128) hipLaunchKernelGGL((dev::dense_qp_kernel<DENSE_NZ, 2>), dim3(count), dim3(64), 0, s, a);
        else hipLaunchKernelGGL((dev::dense_qp_kernel<DENSE_NZ, DQ_R>), dim3(count), dim3(64), 0, s, a);
        e = hipGetLastError();
    }
    if (e == hipSuccess && !settled) {
        hipLaunchKernelGGL(dev::dense_expand_kernel, dim3(count), dim3(64), 0, s, a);
        e = hipGetLastError();
    }
    std::vector<double> yb(big.size() * DENSE_NZ);
    for (size_t b = 0; b < big.size() && e == hipSuccess; b++)
        e = hipMemcpyAsync(&yb[b * DENSE_NZ], a.y + (size_t)big[b] * DENSE_NZ, DENSE_NZ * sizeof(double),
                           hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
#ifdef MPCCBF_PDIP_STAMPS
    if (a.dstamps && e == hipSuccess) {
        long long h[24];
        if (hipMemcpy(h, a.dstamps, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
            std::fprintf(stderr, "dense_stamps");
            for (int k = 1; k <= 10; k++) std::fprintf(stderr, " %lld", h[k] - h[k - 1]);
            std::fprintf(stderr, " | t10: %lld", h[11] - h[16]);
            std::fprintf(stderr, " (w loop %lld)", h[17] - h[14]);
            for (int k = 12; k <= 15; k++) std::fprintf(stderr, " %lld", h[k] - h[k - 1]);
            std::fprintf(stderr, "\n");
        }
    }
#endif
    if (e != hipSuccess) return set_error(MPCCBF_ERR_HIP, std::string("dense QP solve: ") + hipGetErrorString(e));
    const double* x = (const double*)ho;
    double* obj = (double*)(ho + b_x);
    const int32_t* st = (const int32_t*)(ho + b_x + b_obj);
    // host-reduced QPs: x = xp + Z y and the full-space objective
    std::vector<std::vector<double>> xbig(big.size());
    for (size_t b = 0; b < big.size(); b++) {
        const int k = big[b];
        if (st[k] != MPCCBF_OPTIMAL) continue;
        xbig[b].resize(qps[k].n);
        expand_solution(hred[b], &yb[b * DENSE_NZ], xbig[b].data(), &obj[k]);
    }
    for (int k = 0; k < count; k++)
        if (st[k] == RS_CAP_NZ || st[k] == RS_CAP_ROWS)
            return set_error(MPCCBF_ERR_CAPACITY, "QP " + std::to_string(k) +
                                                      (st[k] == RS_CAP_NZ ? ": reduced dimension exceeds 8"
                                                                          : ": reduced rows exceed 256"));
    // outputs: x only for OPTIMAL (Solver.h:33-35)
    size_t bi = 0;
    for (int k = 0; k < count; k++) {
        status_out[k] = st[k];
        if (obj_out) obj_out[k] = st[k] == MPCCBF_OPTIMAL ? obj[k] : __builtin_nan("");
        const double* xs = &x[(size_t)k * DENSE_NMAX];
        if (plan[k].cap) xs = xbig[bi++].data();
        if (st[k] == MPCCBF_OPTIMAL && x_out && x_out[k]) std::memcpy(x_out[k], xs, (size_t)qps[k].n * sizeof(double));
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
