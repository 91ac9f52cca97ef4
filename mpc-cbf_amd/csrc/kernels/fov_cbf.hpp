// fov_cbf.hpp — closed form of the FoV HOCBF rows (FovCBF::init*CBF, FovCBF.cpp:152-535), shared by
// the FoV MPC kernel (impc_fov.hip) and the batched CBF-only controller (cbf_control.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

namespace mpccbf {
namespace dev {

// The FoV border rows' constants (FovCBF.cpp initLeftCBF / initRightCBF): kap = tan of the half
// angle of the cone (fov < pi) or of its complement (fov > pi), the left border's sign (the right
// border's is its negative); none: a 360-degree field of view has no border rows.
struct FovBorder {
    double kap, sig_left;
    bool none;
};

__host__ __device__ inline FovBorder fov_border(double fov) {
    if (fov < M_PI) return FovBorder{tan(0.5 * fov), 1.0, false};
    if (fov == M_PI) return FovBorder{1.0, 0.0, false};
    if (fabs(fov - 2.0 * M_PI) <= 1e-9 * 2.0 * M_PI) return FovBorder{0.0, 0.0, true};
    return FovBorder{tan(0.5 * (2.0 * M_PI - fov)), -1.0, false};
}

// FoV HOCBF rows at ego e against target (tx, ty): closed form of FovCBF::init*CBF with
// alpha(x) = 0.1 x^5 (see oracle/oracle.cpp fov_rows for the derivation). present = false for
// the vacuous border rows of a 360-degree field of view. fb: fov_border(fov), formed once per
// agent by callers that evaluate many rows.
__device__ __forceinline__ void fov_cbf_row(int kind, const double e[6], double tx, double ty, const FovBorder& fb,
                                            double Ds, double Rs, double a[3], double& b, bool& present) {
    constexpr double gamma = 0.1;
    const double vx = e[3], vy = e[4], w = e[5];
    const double dx = tx - e[0], dy = ty - e[1];
    double sn, cs;
    sincos(e[2], &sn, &cs);
    const double rx = cs * dx + sn * dy, ry = -sn * dx + cs * dy;
    double bval, lf2;
    present = true;
    if (kind == 0 || kind == 3) {
        const double sgn = kind == 0 ? 1.0 : -1.0;  // safety: |d|^2 - Ds^2, range: Rs^2 - |d|^2
        a[0] = -2.0 * sgn * dx;
        a[1] = -2.0 * sgn * dy;
        a[2] = 0.0;
        bval = kind == 0 ? dx * dx + dy * dy - Ds * Ds : Rs * Rs - dx * dx - dy * dy;
        lf2 = 2.0 * sgn * (vx * vx + vy * vy);
    } else {
        if (fb.none) {
            a[0] = a[1] = a[2] = 0.0;
            b = 1.7976931348623157e308;
            present = false;
            return;
        }
        const double kap = fb.kap, sig = kind == 1 ? fb.sig_left : -fb.sig_left;
        bval = kap * rx + sig * ry;
        a[0] = -kap * cs + sig * sn;
        a[1] = -kap * sn - sig * cs;
        a[2] = kap * ry - sig * rx;
        lf2 = 2.0 * w * ((kap * sn + sig * cs) * vx + (-kap * cs + sig * sn) * vy) - w * w * bval;
    }
    const double lf = a[0] * vx + a[1] * vy + a[2] * w;
    const double b2 = bval * bval, b4 = b2 * b2;
    const double psi = lf + gamma * b4 * bval;
    const double p2 = psi * psi;
    b = lf2 + 5.0 * gamma * b4 * lf + gamma * p2 * p2 * psi;
}

__device__ __forceinline__ void fov_cbf_row(int kind, const double e[6], double tx, double ty, double fov, double Ds,
                                            double Rs, double a[3], double& b, bool& present) {
    fov_cbf_row(kind, e, tx, ty, fov_border(fov), Ds, Rs, a, b, present);
}

// Voronoi row of the FoV controller: separating_hyperplanes::voronoi of the planar positions
// (Voronoi.cpp:10-29: unit normal from self to other, the plane through the midpoint; Eigen's
// normalize() leaves a zero vector unchanged), shifted by the robot box (math::shiftHyperplane,
// Helpers.cpp:20-36: the offset's maximum over the box corners; the yaw component of the normal is
// zeroed, FovBezierIMPCCBF.cpp:135-141): n . p + off = 0, (nx, ny, 0).
__host__ __device__ inline void voronoi_row(double sx, double sy, double ox, double oy, double bbx,
                                            double bby, double& nx, double& ny, double& off) {
    nx = ox - sx;
    ny = oy - sy;
    const double nrm = sqrt(nx * nx + ny * ny);
    if (nrm > 0.0) {
        nx /= nrm;
        ny /= nrm;
    }
    off = -(nx * 0.5 * (sx + ox) + ny * 0.5 * (sy + oy)) + bbx * fabs(nx) + bby * fabs(ny);
}

// FovBezierIMPCCBF::distanceToEllipse (FovBezierIMPCCBF.cpp:226-280; FovControl.cpp:90-148 is the
// same function): signed distance from the
// robot to the point of the target's 90 % confidence ellipse (s = 4.605) at parametric angle
// slope - theta (negative inside); cov = (cxx, cxy, cyy). The closed-form symmetric 2x2
// eigen-decomposition replaces Eigen::EigenSolver (the result does not depend on the eigenpair
// order or the eigenvector signs).
__device__ inline double distance_to_ellipse(double rx, double ry, double mx, double my, double cxx,
                                      double cxy, double cyy) {
    if (isinf(cxx)) return -5.0;
    const double hm = 0.5 * (cxx + cyy), hd = 0.5 * (cxx - cyy);
    const double rt = sqrt(hd * hd + cxy * cxy);
    const double a = sqrt(4.605 * (hm + rt)), b = sqrt(4.605 * (hm - rt));
    double th = rt > 0.0 ? 0.5 * atan2(2.0 * cxy, cxx - cyy) : 0.0;
    if (th < 0.0) th += M_PI;
    const double sl = atan2(ry - my, rx - mx);
    const double c1 = cos(sl - th), s1 = sin(sl - th), ct = cos(th), st = sin(th);
    const double xn = mx + a * c1 * ct - b * s1 * st;
    const double yn = my + a * c1 * st + b * s1 * ct;
    const double dist = sqrt((xn - rx) * (xn - rx) + (yn - ry) * (yn - ry));
    if (isnan(dist)) return 5.0;
    const double d = sqrt((mx - rx) * (mx - rx) + (my - ry) * (my - ry));
    const double range = sqrt((mx - xn) * (mx - xn) + (my - yn) * (my - yn));
    return d < range ? -dist : dist;
}

}  // namespace dev
}  // namespace mpccbf
