// The generic dense path's one-scan packer (dense_pack.hpp pack_qp_once) against the two-pass form
// (plan_qp, then pack_qp): the same plan, the same first error and the same packed words, on
// seeded random QPs with the cases the packer branches on — zero entries of H and A, an asymmetric
// H, equality rows, free rows, one-sided rows, fixed / bounded / free variables, m = 0, n = 64,
// more than 64 equalities (host-reduced), non-finite H or c, NaN row or variable bounds.
//   g++ -O2 -std=c++17 -I<repo> tests/cpp/dense_pack_check.cpp -o dense_pack_check && ./dense_pack_check
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "mpc-cbf_amd/csrc/host/dense_pack.hpp"

using namespace mpccbf::dense_pack;

int main() {
    std::mt19937_64 rng(20251018);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::uniform_int_distribution<int> pick(0, 99);
    PackScratch w;
    int checked = 0, errors = 0, caps = 0;
    for (int t = 0; t < 3000; t++) {
        const int n = t % 97 == 0 ? 64 : 1 + (int)(rng() % 40);
        const int m = t % 13 == 0 ? 0 : (t % 211 == 0 ? 70 + (int)(rng() % 10) : (int)(rng() % 60));
        std::vector<double> H((size_t)n * n), c(n), A((size_t)m * n), lo(m), hi(m), vlo(n), vhi(n);
        for (auto& v : H) v = pick(rng) < 60 ? 0.0 : U(rng);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < i; j++)
                if (pick(rng) < 70) H[(size_t)i * n + j] = H[(size_t)j * n + i];  // mostly symmetric
        for (auto& v : c) v = U(rng);
        for (auto& v : A) v = pick(rng) < 50 ? 0.0 : U(rng);
        for (int k = 0; k < m; k++) {
            const int r = pick(rng);
            const double a = U(rng), b = a + std::fabs(U(rng));
            if (t % 211 == 0 || r < 20) lo[k] = hi[k] = a;          // equality
            else if (r < 30) lo[k] = -1e300, hi[k] = 1e300;          // free
            else if (r < 50) lo[k] = -INFINITY, hi[k] = b;           // one-sided
            else if (r < 60) lo[k] = a, hi[k] = 1.7e308;             // one-sided
            else lo[k] = a, hi[k] = b;
        }
        for (int i = 0; i < n; i++) {
            const int r = pick(rng);
            const double a = U(rng);
            if (r < 10) vlo[i] = vhi[i] = a;
            else if (r < 40) vlo[i] = a, vhi[i] = a + 1.0;
            else if (r < 60) vlo[i] = -1e300, vhi[i] = a + 1.0;
            else vlo[i] = -1e300, vhi[i] = 1e300;
        }
        const int bad = pick(rng);
        if (bad == 0) H[rng() % H.size()] = NAN;
        if (bad == 1) c[rng() % n] = INFINITY;
        if (bad == 2 && m > 0) lo[rng() % m] = NAN;
        if (bad == 3) vhi[rng() % n] = NAN;
        const bool nov = bad == 4;  // no variable bounds at all
        mpccbf_dense_qp q{n, m, H.data(), c.data(), 0.5 * U(rng), m ? A.data() : nullptr, m ? lo.data() : nullptr,
                          m ? hi.data() : nullptr, nov ? nullptr : vlo.data(), nov ? nullptr : vhi.data()};
        const PackPlan p2 = plan_qp(q);
        const size_t room = (size_t)(n + 1) * (n + 1) + (size_t)(m + n + 2) * (n + 4) + 64;
        std::vector<double> d2(room, -7.0), d1(room, -7.0);
        std::vector<int32_t> i2(room, -7), i1(room, -7);
        if (p2.err.empty() && !p2.cap) pack_qp(q, p2, d2.data(), i2.data());
        const PackPlan p1 = pack_qp_once(q, d1.data(), i1.data(), w);
        if (p1.err != p2.err || p1.cap != p2.cap) {
            std::printf("QP %d: error / capacity differ: '%s' %d vs '%s' %d\n", t, p1.err.c_str(), p1.cap,
                        p2.err.c_str(), p2.cap);
            return 1;
        }
        if (!p2.err.empty()) {
            errors++;
            continue;
        }
        if (p2.cap) {
            caps++;
            continue;
        }
        if (p1.n != p2.n || p1.me != p2.me || p1.mi != p2.mi || p1.nh != p2.nh || p1.enz != p2.enz ||
            p1.inz != p2.inz || p1.nd != p2.nd || p1.ni != p2.ni) {
            std::printf("QP %d: plans differ\n", t);
            return 1;
        }
        // (the int words up to the last u8 column entry: the rest of the last word is padding, where
        // pack_qp's branch-free compaction leaves a stray column byte and pack_qp_once nothing)
        const size_t ibytes = 4 * (4 + (size_t)p2.mi + 1) + 2 * ((size_t)p2.me + 1 + p2.nh) + p2.enz + p2.inz;
        if (std::memcmp(d1.data(), d2.data(), p2.nd * sizeof(double)) != 0 ||
            std::memcmp(i1.data(), i2.data(), ibytes) != 0) {
            size_t fd = 0, fi = 0;
            while (fd < p2.nd && d1[fd] == d2[fd]) fd++;
            while (fi < p2.ni && i1[fi] == i2[fi]) fi++;  // (word level)
            std::printf("QP %d: packed words differ (double %zu of %zu, int %zu of %zu: %08x vs %08x)\n", t, fd,
                        p2.nd, fi, p2.ni, fi < p2.ni ? i1[fi] : 0, fi < p2.ni ? i2[fi] : 0);
            return 1;
        }
        checked++;
    }
    std::printf("dense_pack_check: %d packed QPs identical, %d errors and %d host-reduced QPs agree\n", checked,
                errors, caps);
    return checked > 1000 && errors > 0 && caps > 0 ? 0 : 1;
}
