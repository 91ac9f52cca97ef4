// dense.hpp — small dense FP64 linear algebra for the host-side, parameter-only precompute.
// (Eigen is not part of this image; these matrices are at most ~100 x 100 and built once per
// controller, so clarity wins over speed here.)
#pragma once

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

namespace mpccbf {

struct Mat {
    int r = 0, c = 0;
    std::vector<double> a;
    Mat() = default;
    Mat(int r_, int c_, double v = 0.0) : r(r_), c(c_), a((size_t)r_ * c_, v) {}
    double& operator()(int i, int j) { return a[(size_t)i * c + j]; }
    double operator()(int i, int j) const { return a[(size_t)i * c + j]; }
    static Mat eye(int n) {
        Mat m(n, n);
        for (int i = 0; i < n; i++) m(i, i) = 1.0;
        return m;
    }
    Mat t() const {
        Mat m(c, r);
        for (int i = 0; i < r; i++)
            for (int j = 0; j < c; j++) m(j, i) = (*this)(i, j);
        return m;
    }
    Mat rows(int i0, int n) const {
        Mat m(n, c);
        std::copy(a.begin() + (size_t)i0 * c, a.begin() + (size_t)(i0 + n) * c, m.a.begin());
        return m;
    }
    double maxabs() const {
        double v = 0;
        for (double x : a) v = std::max(v, std::fabs(x));
        return v;
    }
};

inline Mat operator*(const Mat& A, const Mat& B) {
    if (A.c != B.r) throw std::runtime_error("matmul: shape mismatch");
    Mat C(A.r, B.c);
    for (int i = 0; i < A.r; i++)
        for (int k = 0; k < A.c; k++) {
            const double v = A(i, k);
            if (v == 0.0) continue;
            for (int j = 0; j < B.c; j++) C(i, j) += v * B(k, j);
        }
    return C;
}
inline Mat operator+(const Mat& A, const Mat& B) {
    Mat C = A;
    for (size_t i = 0; i < C.a.size(); i++) C.a[i] += B.a[i];
    return C;
}
inline Mat operator*(double s, const Mat& A) {
    Mat C = A;
    for (double& v : C.a) v *= s;
    return C;
}

// One-sided Jacobi SVD of B (m x k, m >= k): B = U diag(s) V^T with U m x k (orthonormal
// columns for nonzero s), V k x k orthogonal.
inline void jacobi_svd(const Mat& B, Mat& U, std::vector<double>& s, Mat& V) {
    const int m = B.r, k = B.c;
    U = B;
    V = Mat::eye(k);
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0.0;
        for (int p = 0; p < k - 1; p++)
            for (int q = p + 1; q < k; q++) {
                double alpha = 0, beta = 0, gamma = 0;
                for (int i = 0; i < m; i++) {
                    alpha += U(i, p) * U(i, p);
                    beta += U(i, q) * U(i, q);
                    gamma += U(i, p) * U(i, q);
                }
                if (gamma == 0.0) continue;
                const double rel = std::fabs(gamma) / std::sqrt(alpha * beta);
                off = std::max(off, rel);
                if (rel < 1e-15) continue;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double cs = 1.0 / std::sqrt(1.0 + t * t), sn = cs * t;
                for (int i = 0; i < m; i++) {
                    const double up = U(i, p), uq = U(i, q);
                    U(i, p) = cs * up - sn * uq;
                    U(i, q) = sn * up + cs * uq;
                }
                for (int i = 0; i < k; i++) {
                    const double vp = V(i, p), vq = V(i, q);
                    V(i, p) = cs * vp - sn * vq;
                    V(i, q) = sn * vp + cs * vq;
                }
            }
        if (off < 1e-15) break;
    }
    s.assign(k, 0.0);
    for (int j = 0; j < k; j++) {
        double nrm = 0;
        for (int i = 0; i < m; i++) nrm += U(i, j) * U(i, j);
        nrm = std::sqrt(nrm);
        s[j] = nrm;
        if (nrm > 0)
            for (int i = 0; i < m; i++) U(i, j) /= nrm;
    }
}

// For A (me x n): orthonormal null-space basis Z (n x (n - rank)) and the minimum-norm right
// inverse Xp = A^+ (n x me), so that A (Xp b + Z y) = b for every consistent b.
inline void null_space(const Mat& A, double rtol, Mat& Z, Mat& Xp, int& rank) {
    const int me = A.r, n = A.c;
    if (me == 0) {
        Z = Mat::eye(n);
        Xp = Mat(n, 0);
        rank = 0;
        return;
    }
    Mat U, V;
    std::vector<double> s;
    jacobi_svd(A.t(), U, s, V);  // A^T = U S V^T  ->  A = V S U^T,  A^+ = U S^-1 V^T
    double smax = 0;
    for (double v : s) smax = std::max(smax, v);
    std::vector<int> keep;
    for (int j = 0; j < me; j++)
        if (s[j] > rtol * smax) keep.push_back(j);
    rank = (int)keep.size();
    Xp = Mat(n, me);
    for (int j : keep)
        for (int i = 0; i < n; i++)
            for (int e = 0; e < me; e++) Xp(i, e) += U(i, j) * (1.0 / s[j]) * V(e, j);
    // complete range(A^T) to an orthonormal basis of R^n: the complement spans null(A)
    std::vector<std::vector<double>> basis;
    for (int j : keep) {
        std::vector<double> u(n);
        for (int i = 0; i < n; i++) u[i] = U(i, j);
        basis.push_back(u);
    }
    // greedy: repeatedly take the unit vector with the largest component outside the current
    // span, orthogonalise it (two Gram-Schmidt passes) and normalise
    std::vector<std::vector<double>> nulls;
    auto project_out = [&](std::vector<double>& v) {
        for (int pass = 0; pass < 2; pass++)
            for (const auto* set : {&basis, &nulls})
                for (const auto& b : *set) {
                    double d = 0;
                    for (int i = 0; i < n; i++) d += b[i] * v[i];
                    for (int i = 0; i < n; i++) v[i] -= d * b[i];
                }
    };
    while ((int)nulls.size() < n - rank) {
        double best = -1.0;
        std::vector<double> bestv;
        for (int e = 0; e < n; e++) {
            std::vector<double> v(n, 0.0);
            v[e] = 1.0;
            project_out(v);
            double nrm = 0;
            for (double x : v) nrm += x * x;
            if (nrm > best) {
                best = nrm;
                bestv = v;
            }
        }
        if (best < 1e-20) break;
        const double nrm = std::sqrt(best);
        for (double& x : bestv) x /= nrm;
        project_out(bestv);
        double n2 = 0;
        for (double x : bestv) n2 += x * x;
        for (double& x : bestv) x /= std::sqrt(n2);
        nulls.push_back(bestv);
    }
    if ((int)nulls.size() != n - rank) throw std::runtime_error("null_space: basis completion failed");
    Z = Mat(n, n - rank);
    for (int j = 0; j < n - rank; j++)
        for (int i = 0; i < n; i++) Z(i, j) = nulls[j][i];
}

// Lower Cholesky factor of an SPD matrix; throws if not SPD.
inline Mat cholesky(const Mat& A) {
    const int n = A.r;
    Mat L(n, n);
    for (int j = 0; j < n; j++) {
        double d = A(j, j);
        for (int k = 0; k < j; k++) d -= L(j, k) * L(j, k);
        if (!(d > 0)) throw std::runtime_error("cholesky: matrix not positive definite");
        L(j, j) = std::sqrt(d);
        for (int i = j + 1; i < n; i++) {
            double v = A(i, j);
            for (int k = 0; k < j; k++) v -= L(i, k) * L(j, k);
            L(i, j) = v / L(j, j);
        }
    }
    return L;
}

}  // namespace mpccbf
