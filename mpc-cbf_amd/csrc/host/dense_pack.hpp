// dense_pack.hpp — host half of the generic dense QP path (dense_qp.hip): validation of one
// mpccbf_dense_qp (the reference's invalid_argument cases) and its packed form for the device
// (layout: dense_qp.hip DenseBatch). Header-only so tools/dense_pack_bench.cpp times the same code.
#pragma once

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/mpccbf.h"

namespace mpccbf {
namespace dense_pack {

constexpr double kInf = 1e300;  // |bound| >= 1e300 means "absent" (numeric_limits lowest/max)
constexpr int DENSE_NMAX = 64;  // variables per QP on the device elimination (lane = variable)
constexpr int DENSE_EMAX = 64;  // equalities per QP on the device elimination

inline bool finite_bound(double v) { return std::isfinite(v) && std::fabs(v) < kInf; }

// Hs = (H + H^T) / 2, the only part of H the objective sees: entry (i, j), formed as the device
// formed it from the full H before the packed form carried one triangle (bit-identical: the sum
// commutes)
inline double hs_entry(const double* H, int n, int i, int j) {
    return 0.5 * (H[(size_t)i * n + j] + H[(size_t)j * n + i]);
}

// Host half: validation (the reference's invalid_argument cases: NULL pointers, n < 1, m < 0,
// non-finite H / c, NaN bounds) and the row classification; sizes of the packed form.
struct PackPlan {
    int n = 0, me = 0, mi = 0, nh = 0, enz = 0, inz = 0;
    size_t nd = 0, ni = 0;  // doubles / ints of the packed QP
    std::string err;
    bool cap = false;
};

inline PackPlan plan_qp(const mpccbf_dense_qp& qp) {
    PackPlan pl;
    auto fail = [&](const char* m) {
        pl.err = m;
        return pl;
    };
    if (qp.n < 1) return fail("dense QP: n must be >= 1");
    if (qp.m < 0) return fail("dense QP: m must be >= 0");
    if (!qp.H || !qp.c) return fail("dense QP: H and c are required");
    if (qp.m > 0 && !(qp.A && qp.lo && qp.hi)) return fail("dense QP: A, lo, hi are required when m > 0");
    const int n = qp.n, m = qp.m;
    pl.n = n;
    // branch-free scans (vectorised): a flag for a non-finite entry, the nonzero counts
    bool nonfin = false;
    for (size_t k = 0; k < (size_t)n * n; k++) nonfin |= !(std::fabs(qp.H[k]) <= DBL_MAX);
    if (nonfin) return fail("dense QP: H has a non-finite entry");
    int nh = 0;  // nonzeros of Hs = (H + H^T) / 2 on and above the diagonal (the packed half)
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) nh += hs_entry(qp.H, n, i, j) != 0.0;
    pl.nh = nh;
    for (int i = 0; i < n; i++) nonfin |= !(std::fabs(qp.c[i]) <= DBL_MAX);
    if (nonfin) return fail("dense QP: c has a non-finite entry");
    for (int k = 0; k < m; k++) {
        const double lo = qp.lo[k], hi = qp.hi[k];
        if (std::isnan(lo) || std::isnan(hi)) return fail("dense QP: NaN row bound");
        const bool eq = finite_bound(lo) && lo == hi, in = !eq && (finite_bound(lo) || finite_bound(hi));
        if (!eq && !in) continue;  // a free row: not read
        const double* a = qp.A + (size_t)k * n;
        int nnz = 0;
        for (int j = 0; j < n; j++) nnz += a[j] != 0.0;
        if (eq) {
            pl.me++;
            pl.enz += nnz;
        } else {
            pl.mi++;
            pl.inz += nnz;
        }
    }
    for (int i = 0; i < n; i++) {
        const double lo = qp.vlo ? qp.vlo[i] : -kInf, hi = qp.vhi ? qp.vhi[i] : kInf;
        if (std::isnan(lo) || std::isnan(hi)) return fail("dense QP: NaN variable bound");
        if (finite_bound(lo) && lo == hi) {
            pl.me++;
            pl.enz++;
        } else if (finite_bound(lo) || finite_bound(hi)) {
            pl.mi++;
            pl.inz++;
        }
    }
    pl.cap = n > DENSE_NMAX || pl.me > DENSE_EMAX;
    if (pl.cap) return pl;  // (reduced on the host: not packed)
    // int32 words: header, inequality row pointers, then the u16 / u8 arrays (pack_qp)
    pl.ni = 4 + (size_t)(pl.mi + 1) + (2 * (size_t)(pl.me + 1) + 2 * (size_t)pl.nh + pl.enz + pl.inz + 3) / 4;
    pl.nd = (size_t)n + 1 + pl.nh + pl.me + pl.enz + 2 * (size_t)pl.mi + pl.inz;
    return pl;
}

// Writes one QP's packed form (within capacity: n, me <= 64). Layout, int words: [n, me, mi, nh |
// in row ptr (mi + 1, int32) | eq row ptr (me + 1, u16) | Hs index (i << 6 | j, i <= j; nh, u16)
// | eq cols (u8) | in cols (u8)]; doubles: [c (n) | c0 | Hs values (nh) | eq rhs (me) | eq values |
// in lo (mi) | in hi (mi) | in values]. Branch-free compaction (each entry written, the cursor
// advanced by its nonzero flag): a section's cursor may write one entry past its end, into a later
// section, so the sections are packed in memory order (Hs, equality rows, inequality rows) and the
// caller leaves one spare double and int after the QP.
inline void pack_qp(const mpccbf_dense_qp& qp, const PackPlan& pl, double* db, int32_t* ib) {
    const int n = qp.n;
    int32_t* iptr = ib + 4;
    uint16_t* eptr = (uint16_t*)(iptr + pl.mi + 1);
    uint16_t* hidx = eptr + pl.me + 1;
    uint8_t* ecol = (uint8_t*)(hidx + pl.nh);
    uint8_t* icol = ecol + pl.enz;
    double* c = db;
    double* hval = db + n + 1;
    double* erhs = hval + pl.nh;
    double* evalv = erhs + pl.me;
    double* ilo = evalv + pl.enz;
    double* ihi = ilo + pl.mi;
    double* ivalv = ihi + pl.mi;
    int h = 0;
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            const double v = hs_entry(qp.H, n, i, j);
            hidx[h] = (uint16_t)(i << 6 | j);
            hval[h] = v;
            h += v != 0.0;
        }
    ib[0] = n;
    ib[1] = pl.me;
    ib[2] = pl.mi;
    ib[3] = pl.nh;
    std::memcpy(c, qp.c, (size_t)n * sizeof(double));
    db[n] = qp.c0;
    auto row = [&](const double* a, uint8_t* col, double* val, int z) {
        for (int j = 0; j < n; j++) {
            const double v = a[j];
            col[z] = (uint8_t)j;
            val[z] = v;
            z += v != 0.0;
        }
        return z;
    };
    // equality rows (rows with lo == hi, then fixed variables)
    eptr[0] = 0;
    int e = 0, ez = 0;
    for (int k = 0; k < qp.m; k++) {
        const double lo = qp.lo[k], hi = qp.hi[k];
        if (!(finite_bound(lo) && lo == hi)) continue;
        ez = row(qp.A + (size_t)k * n, ecol, evalv, ez);
        erhs[e] = lo;
        eptr[++e] = (uint16_t)ez;
    }
    for (int i = 0; i < n; i++) {
        const double lo = qp.vlo ? qp.vlo[i] : -kInf, hi = qp.vhi ? qp.vhi[i] : kInf;
        if (!(finite_bound(lo) && lo == hi)) continue;
        ecol[ez] = (uint8_t)i;
        evalv[ez++] = 1.0;
        erhs[e] = lo;
        eptr[++e] = (uint16_t)ez;
    }
    // inequality rows (a finite side, then variable bounds as unit rows)
    iptr[0] = 0;
    int r = 0, rz = 0;
    for (int k = 0; k < qp.m; k++) {
        const double lo = qp.lo[k], hi = qp.hi[k];
        if ((finite_bound(lo) && lo == hi) || !(finite_bound(lo) || finite_bound(hi))) continue;
        rz = row(qp.A + (size_t)k * n, icol, ivalv, rz);
        ilo[r] = lo;
        ihi[r] = hi;
        iptr[++r] = rz;
    }
    for (int i = 0; i < n; i++) {
        const double lo = qp.vlo ? qp.vlo[i] : -kInf, hi = qp.vhi ? qp.vhi[i] : kInf;
        if ((finite_bound(lo) && lo == hi) || !(finite_bound(lo) || finite_bound(hi))) continue;
        icol[rz] = (uint8_t)i;
        ivalv[rz++] = 1.0;
        ilo[r] = lo;
        ihi[r] = hi;
        iptr[++r] = rz;
    }
}

// Per-thread scratch of pack_qp_once (grown on demand, kept across QPs)
struct PackScratch {
    std::vector<double> hval, evalv, ivalv, erhs, ilo, ihi;
    std::vector<uint16_t> hidx, eptr;
    std::vector<uint8_t> ecol, icol;
    std::vector<int32_t> iptr;
};

// plan_qp and pack_qp in one scan of H and A: the same validation (the same first error), the same
// plan and the same packed words (sections are compacted into the scratch, then copied into place
// once their sizes are known). Returns the plan; packs only a QP without error within capacity.
inline PackPlan pack_qp_once(const mpccbf_dense_qp& qp, double* db, int32_t* ib, PackScratch& w) {
    if (qp.n < 1 || qp.n > DENSE_NMAX || qp.m < 0 || !qp.H || !qp.c || (qp.m > 0 && !(qp.A && qp.lo && qp.hi)))
        return plan_qp(qp);  // (argument errors and the host-reduced sizes: the two-pass form)
    PackPlan pl;
    const int n = qp.n, m = qp.m;
    pl.n = n;
    // Hs's upper triangle (compacted) with H's finiteness: every entry of H is one of a pair
    const size_t hcap = (size_t)n * (n + 1) / 2 + 1;
    if (w.hval.size() < hcap) {
        w.hval.resize(hcap);
        w.hidx.resize(hcap);
    }
    bool nonfin = false;
    int h = 0;
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            const double a = qp.H[(size_t)i * n + j], b = qp.H[(size_t)j * n + i];
            nonfin |= !(std::fabs(a) <= DBL_MAX) | !(std::fabs(b) <= DBL_MAX);
            const double v = 0.5 * (a + b);  // (hs_entry)
            w.hidx[h] = (uint16_t)(i << 6 | j);
            w.hval[h] = v;
            h += v != 0.0;
        }
    if (nonfin) {
        pl.err = "dense QP: H has a non-finite entry";
        return pl;
    }
    pl.nh = h;
    for (int i = 0; i < n; i++) nonfin |= !(std::fabs(qp.c[i]) <= DBL_MAX);
    if (nonfin) {
        pl.err = "dense QP: c has a non-finite entry";
        return pl;
    }
    // rows: equality rows (lo == hi) and inequality rows (a finite side) compacted in row order
    const size_t rcap = (size_t)m + n + 2, zcap = (size_t)(m + 1) * n + 1;
    if (w.erhs.size() < rcap) {
        w.erhs.resize(rcap);
        w.ilo.resize(rcap);
        w.ihi.resize(rcap);
        w.eptr.resize(rcap);
        w.iptr.resize(rcap);
    }
    if (w.evalv.size() < zcap) {
        w.evalv.resize(zcap);
        w.ivalv.resize(zcap);
        w.ecol.resize(zcap);
        w.icol.resize(zcap);
    }
    auto row = [&](const double* a, uint8_t* col, double* val, int z) {
        for (int j = 0; j < n; j++) {
            const double v = a[j];
            col[z] = (uint8_t)j;
            val[z] = v;
            z += v != 0.0;
        }
        return z;
    };
    int e = 0, ez = 0, r = 0, rz = 0;
    w.eptr[0] = 0;
    w.iptr[0] = 0;
    for (int k = 0; k < m; k++) {
        const double lo = qp.lo[k], hi = qp.hi[k];
        if (std::isnan(lo) || std::isnan(hi)) {
            pl.err = "dense QP: NaN row bound";
            return pl;
        }
        const bool eq = finite_bound(lo) && lo == hi, in = !eq && (finite_bound(lo) || finite_bound(hi));
        if (eq) {
            ez = row(qp.A + (size_t)k * n, w.ecol.data(), w.evalv.data(), ez);
            w.erhs[e] = lo;
            w.eptr[++e] = (uint16_t)ez;
        } else if (in) {
            rz = row(qp.A + (size_t)k * n, w.icol.data(), w.ivalv.data(), rz);
            w.ilo[r] = lo;
            w.ihi[r] = hi;
            w.iptr[++r] = rz;
        }
    }
    // variable bounds: fixed variables as equality unit rows, bounded ones as inequality unit rows
    // (after the rows of A in both lists, as pack_qp orders them)
    for (int i = 0; i < n; i++) {
        const double lo = qp.vlo ? qp.vlo[i] : -kInf, hi = qp.vhi ? qp.vhi[i] : kInf;
        if (std::isnan(lo) || std::isnan(hi)) {
            pl.err = "dense QP: NaN variable bound";
            return pl;
        }
        if (finite_bound(lo) && lo == hi) {
            w.ecol[ez] = (uint8_t)i;
            w.evalv[ez++] = 1.0;
            w.erhs[e] = lo;
            w.eptr[++e] = (uint16_t)ez;
        } else if (finite_bound(lo) || finite_bound(hi)) {
            w.icol[rz] = (uint8_t)i;
            w.ivalv[rz++] = 1.0;
            w.ilo[r] = lo;
            w.ihi[r] = hi;
            w.iptr[++r] = rz;
        }
    }
    pl.me = e;
    pl.mi = r;
    pl.enz = ez;
    pl.inz = rz;
    pl.cap = pl.me > DENSE_EMAX;
    if (pl.cap) return pl;  // (reduced on the host: not packed)
    pl.ni = 4 + (size_t)(pl.mi + 1) + (2 * (size_t)(pl.me + 1) + 2 * (size_t)pl.nh + pl.enz + pl.inz + 3) / 4;
    pl.nd = (size_t)n + 1 + pl.nh + pl.me + pl.enz + 2 * (size_t)pl.mi + pl.inz;
    // the sections into place (pack_qp's layout)
    ib[0] = n;
    ib[1] = pl.me;
    ib[2] = pl.mi;
    ib[3] = pl.nh;
    int32_t* iptr = ib + 4;
    uint16_t* eptr = (uint16_t*)(iptr + pl.mi + 1);
    uint16_t* hidx = eptr + pl.me + 1;
    uint8_t* ecol = (uint8_t*)(hidx + pl.nh);
    uint8_t* icol = ecol + pl.enz;
    std::memcpy(iptr, w.iptr.data(), (size_t)(pl.mi + 1) * sizeof(int32_t));
    std::memcpy(eptr, w.eptr.data(), (size_t)(pl.me + 1) * sizeof(uint16_t));
    std::memcpy(hidx, w.hidx.data(), (size_t)pl.nh * sizeof(uint16_t));
    std::memcpy(ecol, w.ecol.data(), (size_t)pl.enz);
    std::memcpy(icol, w.icol.data(), (size_t)pl.inz);
    double* c = db;
    double* hval = db + n + 1;
    double* erhs = hval + pl.nh;
    double* evalv = erhs + pl.me;
    double* ilo = evalv + pl.enz;
    double* ihi = ilo + pl.mi;
    double* ivalv = ihi + pl.mi;
    std::memcpy(c, qp.c, (size_t)n * sizeof(double));
    db[n] = qp.c0;
    std::memcpy(hval, w.hval.data(), (size_t)pl.nh * sizeof(double));
    std::memcpy(erhs, w.erhs.data(), (size_t)pl.me * sizeof(double));
    std::memcpy(evalv, w.evalv.data(), (size_t)pl.enz * sizeof(double));
    std::memcpy(ilo, w.ilo.data(), (size_t)pl.mi * sizeof(double));
    std::memcpy(ihi, w.ihi.data(), (size_t)pl.mi * sizeof(double));
    std::memcpy(ivalv, w.ivalv.data(), (size_t)pl.inz * sizeof(double));
    return pl;
}

}  // namespace dense_pack
}  // namespace mpccbf
