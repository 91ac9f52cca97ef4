// Host cost of the generic dense path's validation + packing (csrc/host/dense_pack.hpp) per QP,
// one thread, on the golden MPC-CBF QPs replicated (tools/dense_pack_bench.py writes them):
//   g++ -O3 -std=c++17 -I. tools/dense_pack_bench.cpp -o /tmp/dpb && /tmp/dpb /tmp/golden.bin [once]
// (plan_qp + pack_qp, the two-pass form; with a second argument pack_qp_once, the product's)
#include <chrono>
#include <cstdio>
#include <vector>

#include "mpc-cbf_amd/csrc/host/dense_pack.hpp"

using namespace mpccbf::dense_pack;

int main(int argc, char** argv) {
    FILE* f = std::fopen(argc > 1 ? argv[1] : "/tmp/golden.bin", "rb");
    if (!f) return 1;
    int32_t count = 0;
    if (std::fread(&count, 4, 1, f) != 1) return 1;
    std::vector<std::vector<double>> store;
    std::vector<mpccbf_dense_qp> qps(count);
    for (int k = 0; k < count; k++) {
        int32_t nm[2];
        if (std::fread(nm, 4, 2, f) != 2) return 1;
        const int n = nm[0], m = nm[1];
        std::vector<double> v((size_t)n * n + n + (size_t)m * n + 2 * m);
        if (std::fread(v.data(), 8, v.size(), f) != v.size()) return 1;
        store.push_back(std::move(v));
        const double* p = store.back().data();
        qps[k] = mpccbf_dense_qp{n, m, p, p + n * n, 0.25, p + n * n + n, p + n * n + n + (size_t)m * n,
                                 p + n * n + n + (size_t)m * n + m, nullptr, nullptr};
    }
    std::fclose(f);
    const int reps = 4096;
    const bool once = argc > 2;  // (second argument: pack_qp_once)
    PackScratch w;
    std::vector<double> d;
    std::vector<int32_t> ii;
    double best = 1e30;
    for (int trial = 0; trial < 5; trial++) {
        d.clear();
        ii.clear();
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; r++) {
            const mpccbf_dense_qp& q = qps[r % count];
            const size_t od = d.size(), oi = ii.size();
            if (once) {  // one scan into a slot sized from n and m (dense_qp.hip)
                const size_t n = q.n, m = q.m, hmax = n * (n + 1) / 2, rows = m + n, nz = m * n + n;
                d.resize(od + n + 1 + hmax + 2 * rows + nz + 1);
                ii.resize(oi + 4 + (rows + 1) + (2 * (rows + 1) + 2 * hmax + nz + 3) / 4 + 1);
                const PackPlan pl = pack_qp_once(q, d.data() + od, ii.data() + oi, w);
                d.resize(od + pl.nd);
                ii.resize(oi + pl.ni);
            } else {
                const PackPlan pl = plan_qp(q);
                d.resize(od + pl.nd + 1);
                ii.resize(oi + pl.ni + 1);
                pack_qp(q, pl, d.data() + od, ii.data() + oi);
                d.pop_back();
                ii.pop_back();
            }
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        best = us < best ? us : best;
    }
    std::printf("%d QPs: %.1f us, %.3f us per QP; packed %.1f KB per QP\n", reps, best, best / reps,
                (d.size() * 8.0 + ii.size() * 4.0) / reps / 1024.0);
    return 0;
}
