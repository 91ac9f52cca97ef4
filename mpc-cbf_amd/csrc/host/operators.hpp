// operators.hpp — parameter-only operators of the MPC-CBF QP, condensed onto the null space
// of its equality constraints. Built once per controller on the host and uploaded.
#pragma once

#include <string>
#include <vector>

#include "../../../include/mpccbf.h"
#include "dense.hpp"

namespace mpccbf {

constexpr int DIM = 3;
constexpr int SD = 2 * DIM;  // state dimension

// Validation of common/include/common/parsing.hpp (:37-135 per group, :182-214 cross-group).
// Returns "" when valid, else the reference's error message.
std::string validate_params(const mpccbf_params& p);

// Everything the kernel needs, as plain host matrices (see DESIGN.md "Data layout").
//   x = Xs * s0 + Z * y          (full decision vector from state s0 and reduced y)
//   objective(y) = 1/2 y^T Pr y + q^T y + k,    q = Qs s0 + Qt t  (or Qs s0 + Qr ref_tail)
//   shared rows:  lo_i - Gs_i s0 <= G_i y <= hi_i - Gs_i s0
//   constant rows (zero in y):  lo_i <= Cs_i s0 <= hi_i   (pure feasibility checks)
struct Operators {
    int n = 0, nz = 0, me = 0, K = 0, spd_f = 0, cbf_h = 0;
    Mat H;          // n x n symmetric: objective x^T H x (canonicalised, drop rule applied)
    Mat Z, Xs;      // n x nz, n x 6
    Mat Pr, LPr;    // nz x nz reduced Hessian (of 1/2 y^T Pr y) and its Cholesky factor
    Mat Qs, Qt, Qr; // nz x 6, nz x 3, nz x 3*spd_f
    Mat Ks, Kt, Kr; // objective constant: s0^T Ks s0 + t^T Kt s0 (Ks 6x6, Kt 3x6); ref: r^T Kr s0
    Mat G, Gs;      // m x nz, m x 6 shared inequality rows (kept after exact reduction)
    std::vector<double> lo, hi;
    std::vector<int> row_kind;  // 0 accel, 1 vel (for diagnostics)
    std::vector<int> row_dim;   // spatial dimension a kept shared row constrains (-1: several)
    // Dimension-separable structure (base_config.json): equalities and cost never couple the
    // x / y / yaw channels, so Z is block-diagonal with nzd columns per channel, ordered
    // [x | y | yaw]; every shared row then touches one channel's nzd columns only.
    bool sep = false;
    int nzd = 0;
    Mat Cs;                     // mc x 6 constant rows
    std::vector<double> clo, chi;
    int rows_total = 0, rows_removed = 0;
    // CBF: acceleration basis at sample k (U_basis rows 3k..3k+2), condensed
    std::vector<Mat> UZ, US;  // cbf_h of (3 x nz), (3 x 6)
    // predicted states at h_samples(k), k < cbf_h: pos/vel rows, condensed
    std::vector<Mat> PZ, PS;  // cbf_h of (6 x nz), (6 x 6): rows 0..2 pos, 3..5 vel
    Mat AZ, AS;               // (6 x nz), (6 x 6): state at t = h (closed-loop update)
    // closed-loop simulator (example :150-221): evaluate a stored curve at any t
    Mat EB0, EB1;             // C x C monomial coefficients of the Bernstein basis / derivative
    std::vector<double> cum;  // cumulative piece parameters (SingleParameterPiecewiseCurve)
    double eval_step = 0.0;   // Ts * int(h / Ts): eval-time advance per control step
    // FoV controller (cbf_mode 1): Voronoi rows act on the piece-0 control points
    // (BezierQPOperations::hyperplaneConstraintAll, :270-285): control point j of dims x, y
    std::vector<Mat> VZ, VS;  // C of (2 x nz), (2 x 6)
    double a_lo[3], a_hi[3];
};

Operators build_operators(const mpccbf_params& p, bool keep_redundant);

}  // namespace mpccbf
