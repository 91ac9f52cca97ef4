// diag.cpp — host-only inspection of the condensed operators (no GPU needed). Used by the CPU
// test suite to check the precompute against the oracle's full-space assembly.
#include <cstring>
#include <exception>
#include <string>

#include "../../../include/mpccbf.h"
#include "operators.hpp"

using namespace mpccbf;

namespace {
thread_local std::string g_diag_err;

void put(const Mat& m, double* dst) {
    if (dst) std::memcpy(dst, m.a.data(), m.a.size() * sizeof(double));
}
void put(const std::vector<double>& m, double* dst) {
    if (dst) std::memcpy(dst, m.data(), m.size() * sizeof(double));
}
}  // namespace

extern "C" {

const char* mpccbf_host_last_error(void) { return g_diag_err.c_str(); }

int mpccbf_host_operators(const mpccbf_params* p, int32_t keep_redundant, mpccbf_host_ops* out) {
    if (!p || !out) return MPCCBF_ERR_INVALID_ARGUMENT;
    const std::string verr = validate_params(*p);
    if (!verr.empty()) {
        g_diag_err = verr;
        return MPCCBF_ERR_INVALID_ARGUMENT;
    }
    try {
        Operators o = build_operators(*p, keep_redundant != 0);
        out->n = o.n;
        out->nz = o.nz;
        out->m = o.G.r;
        out->mc = o.Cs.r;
        out->rows_total = o.rows_total;
        out->rows_removed = o.rows_removed;
        if (out->capacity_ok == 0) return MPCCBF_OK;  // sizes only
        put(o.H, out->H);
        put(o.Z, out->Z);
        put(o.Xs, out->Xs);
        put(o.Pr, out->Pr);
        put(o.Qs, out->Qs);
        put(o.Qt, out->Qt);
        put(o.Ks, out->Ks);
        put(o.Kt, out->Kt);
        put(o.G, out->G);
        put(o.Gs, out->Gs);
        put(o.lo, out->lo);
        put(o.hi, out->hi);
        put(o.Cs, out->Cs);
        put(o.clo, out->clo);
        put(o.chi, out->chi);
        if (out->UZ0) put(o.UZ[0], out->UZ0);
        if (out->US0) put(o.US[0], out->US0);
        return MPCCBF_OK;
    } catch (const std::exception& e) {
        g_diag_err = e.what();
        return MPCCBF_ERR_INVALID_ARGUMENT;
    }
}

}  // extern "C"
