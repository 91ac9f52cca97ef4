// dense_qp.hpp — host equality elimination of the generic flattened-QP path (mpccbf_qp_solve_dense*)
// for the QPs beyond the device elimination's capacity (more than 64 variables or 64 equality
// rows, dense_qp.hip dense_reduce_kernel): the same reduction on the host, the reduced QP solved
// by the same device interior-point kernel.
//
// The QP arrives in the form CPLEXSolver::solve hands to CPLEX (qpcpp/src/solvers/CPLEX.cpp:52-147):
//     minimise  x^T H x + c^T x + c0      s.t.  lo <= A x <= hi,   vlo <= x <= vhi
// Equality rows (lo == hi) and fixed variables are eliminated exactly (x = xp + Z y, Z an
// orthonormal null-space basis); what remains is the reduced problem
//     minimise  1/2 y^T P y + q^T y + k0   s.t.  lo' <= g^T y <= hi'
// Rows whose reduced coefficients vanish are decided here (they only test the feasibility of xp).
#pragma once

#include <vector>

#include "../../../include/mpccbf.h"
#include "dense.hpp"

namespace mpccbf {

struct ReducedQP {
    int n = 0, nz = 0, m = 0;
    int status = -1;            // >= 0: decided on the host (no device solve needed)
    bool eq_infeasible = false; // inconsistent equalities (INFEASIBLE whatever the sizes; a violated
                                // constant row is INFEASIBLE only within the device capacity)
    bool pd = false;            // P positive definite (Cholesky start available)
    Mat Z;                      // n x nz
    std::vector<double> xp;     // n
    Mat P, LP;                  // nz x nz
    std::vector<double> q;      // nz
    double k0 = 0.0;
    Mat G;                      // m x nz
    std::vector<double> lo, hi; // m (+-1e300 = absent side)
    Mat Hs;                     // symmetrised H (objective evaluation)
    std::vector<double> c;
    double c0 = 0.0;
};

// Throws std::invalid_argument on malformed input (NULL pointers, n < 1, m < 0, NaN data).
ReducedQP reduce_dense_qp(const mpccbf_dense_qp& qp);

// x = xp + Z y; full-space objective x^T Hs x + c^T x + c0.
void expand_solution(const ReducedQP& r, const double* y, double* x, double* obj);

}  // namespace mpccbf
