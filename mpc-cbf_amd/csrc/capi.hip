// capi.hip — the C ABI of include/mpccbf.h: context lifetime, operator upload, launches.
// No exception crosses this boundary (the reference's std::invalid_argument / runtime_error
// become MPCCBF_ERR_INVALID_ARGUMENT plus a thread-local message).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/mpccbf.h"
#include "host/errors.hpp"
#include "host/operators.hpp"
#include "kernels/impc.hpp"
#include "kernels/cbf_control.hpp"
#include "kernels/fov_cbf.hpp"

namespace mpccbf {

hipError_t launch_impc(const DevOps& op, const double* buf, const ImpcArgs& a, int variant,
                       hipStream_t s);
const char* impc_kernel_name(const DevOps& op, int variant, int n);
int impc_clock_waves(const DevOps& op, int variant, int n);
hipError_t launch_impc_fov(const DevOps& op, const double* buf, const ImpcArgs& a, hipStream_t s);
hipError_t launch_fov_rows_eval(int count, const double* ego, const double* nb, double fov, double Ds, double Rs,
                                double bbx, double bby, double* vor, double* rows, hipStream_t s);
hipError_t launch_impc_fallback(const DevOps& op, const double* buf, const ImpcArgs& a, bool wide,
                                hipStream_t s);
bool impc_may_defer(const DevOps& op, int variant, bool csr, int knn_k, int n);
bool impc_rows_may_exceed(const DevOps& op, bool csr, int knn_k);
int launch_neighbors(const double* states, int num_states, int first, int num_agents, int k,
                     double radius, int32_t* row_ptr, int32_t* col, void* scratch,
                     size_t scratch_bytes, hipStream_t s);
size_t neighbors_scratch_bytes(int num_states, int num_agents, int k);
size_t grid_table_bytes(int num_states);
void grid_table_carve(void* base, int num_states, uint32_t** cnt, uint32_t** slots, double** sst);
hipError_t launch_grid_insert(const double* states, int n, int skip0, int skip1, double radius,
                              uint32_t* cnt, uint32_t* slots, double* sst, hipStream_t s);

static thread_local std::string g_err;

int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

static int fail(int code, const std::string& msg) { return set_error(code, msg); }

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return fail(MPCCBF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

}  // namespace mpccbf

struct mpccbf_ctx {
    std::vector<hipEvent_t> events;  // timing events of mpccbf_run_steps (grown on demand)
    mpccbf_params p;
    mpccbf_options opt;
    mpccbf::Operators ops;
    mpccbf::DevOps dev;
    int device = 0;
    double* dbuf = nullptr;
    size_t dbuf_elems = 0;
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    void* grid_scratch = nullptr;  // three neighbour tables (see GridArgs)
    size_t grid_bytes = 0;
    // fallback queues [count, -, agents...], two (alternating by enqueue parity: the main launch
    // zeroes the other one's header), zero-initialised
    int32_t* defer = nullptr;
    int defer_cap = 0;
    int defer_parity = 0;
    int variant = 0;
    int last_n = 0;  // agents of the last IMPC launch (the kernel name depends on it: share-adaptive)
    // grid mode: where the previous mpccbf_run_steps call left the table rotation (ABI 12,
    // mpccbf_run::continue_tables): its final state table, shape, query and the next step's table
    struct {
        bool valid = false;
        const double* states = nullptr;
        int ns = 0, first = 0, count = 0, k = 0, next = 0;
        double radius = 0.0;
    } gcont;
};

using namespace mpccbf;

static void pack(std::vector<double>& v, int32_t& off, const Mat& m) {
    off = (int32_t)v.size();
    v.insert(v.end(), m.a.begin(), m.a.end());
}
static void pack(std::vector<double>& v, int32_t& off, const std::vector<double>& m) {
    off = (int32_t)v.size();
    v.insert(v.end(), m.begin(), m.end());
}
static void pack(std::vector<double>& v, int32_t& off, const std::vector<Mat>& ms) {
    off = (int32_t)v.size();
    for (const Mat& m : ms) v.insert(v.end(), m.a.begin(), m.a.end());
}

// The three neighbour tables of grid mode in ctx scratch (grown on demand).
static int grid_tables(mpccbf_ctx* c, int num_states, uint32_t* (&cnt)[3], uint32_t* (&slots)[3],
                       double* (&sst)[3]) {
    const size_t tb = grid_table_bytes(num_states);
    if (3 * tb > c->grid_bytes) {
        c->gcont.valid = false;
        if (c->grid_scratch) (void)hipFree(c->grid_scratch);
        c->grid_scratch = nullptr;
        c->grid_bytes = 0;
        HIP_TRY(hipMalloc(&c->grid_scratch, 3 * tb));
        c->grid_bytes = 3 * tb;
    }
    for (int t = 0; t < 3; t++)
        grid_table_carve((char*)c->grid_scratch + t * tb, num_states, &cnt[t], &slots[t], &sst[t]);
    return MPCCBF_OK;
}

// One IMPC step for a batch, enqueued on `stream`; ev0 / ev1 (optional) are recorded around the
// IMPC kernel alone. Grid mode: gstep < 0 builds table 0 from b->states first (memset + insert
// kernel); gstep >= 0 (mpccbf_run_steps) reads table gstep % 3, which the previous step filled,
// has the kernel insert its next states into table (gstep + 1) % 3 and zero table (gstep + 2) % 3.
int impc_enqueue(mpccbf_ctx* c, const mpccbf_batch* b, hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1,
                 int gstep = -1, unsigned long long* kclock = nullptr) {
    if (!c || !b) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "null argument");
    if (b->num_agents < 0 || b->agent_first < 0 || b->agent_first + b->num_agents > b->num_states)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "agent range outside states");
    if (b->num_agents == 0) return MPCCBF_OK;
    const bool grid = b->nb_row_ptr == nullptr;
    if (!b->states || (!grid && !b->nb_col && b->num_states > 1))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "states / neighbour CSR missing");
    if (grid && (b->knn_k < 1 || !(b->knn_radius > 0)))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "grid neighbours need knn_k >= 1 and knn_radius > 0");
    if (grid && b->knn_k > NB_MAX)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "grid neighbours: knn_k > 16 not supported (give CSR lists)");
    if (!b->targets && !b->refs) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "targets or refs required");
    if (b->traj_t && !b->x)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "traj_t (closed-loop fallback) needs the persistent x buffer");
    if (!(b->pos_std >= 0.0) || !(b->vel_std >= 0.0))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "noise standard deviations must be >= 0");
    ImpcArgs a;
    std::memset(&a, 0, sizeof(a));
    HIP_TRY(hipSetDevice(c->device));
    if (grid) {
        uint32_t *cnt[3], *slots[3];
        double* sst[3];
        const int rc = grid_tables(c, b->num_states, cnt, slots, sst);
        if (rc != MPCCBF_OK) return rc;
        const uint32_t T = grid_table_size(b->num_states);
        int rd = 0;
        if (gstep < 0) {
            c->gcont.valid = false;  // (table 0 rebuilt: a run_steps continuation must rebuild too)
            HIP_TRY(hipMemsetAsync(cnt[0], 0, (size_t)T * 4, stream));
            HIP_TRY(launch_grid_insert(b->states, b->num_states, 0, 0, b->knn_radius, cnt[0], slots[0], sst[0],
                                       stream));
        } else {
            rd = gstep % 3;
            a.grid.ins_cnt = cnt[(gstep + 1) % 3];
            a.grid.ins_slots = slots[(gstep + 1) % 3];
            a.grid.ins_sst = sst[(gstep + 1) % 3];
            a.grid.clr_cnt = cnt[(gstep + 2) % 3];
        }
        a.grid.cnt = cnt[rd];
        a.grid.slots = slots[rd];
        a.grid.sst = sst[rd];
        a.grid.mask = T - 1;
        a.grid.inv_cell = 1.0 / b->knn_radius;
        a.grid.radius = b->knn_radius;
        a.grid.k = b->knn_k;
        // FoV controller: only agents inside the field of view are observed neighbours
        a.grid.cone = (c->dev.cbf_mode == 1 && c->dev.fov_beta < 2.0 * M_PI - 1e-9) ? 0.5 * c->dev.fov_beta : 0.0;
    }
    a.num_states = b->num_states;
    a.states = b->states;
    a.agent_first = b->agent_first;
    a.num_agents = b->num_agents;
    a.targets = b->targets;
    a.refs = b->targets ? nullptr : b->refs;
    a.nb_row_ptr = b->nb_row_ptr;
    a.nb_col = b->nb_col;
    a.x = b->x;
    a.status = b->status;
    a.obj = b->obj;
    a.iters = b->iters;
    a.next_states = b->next_states;
    a.stamps = b->stamps;
    a.traj_t = b->traj_t;
    a.pos_std = b->pos_std;
    a.vel_std = b->vel_std;
    a.noise_seed = b->noise_seed;
    a.step_index = b->step_index;
    a.cov = b->cov;
    a.primal_res = b->primal_res;
    a.dual_res = b->dual_res;
    a.substeps = b->substeps;
    a.nb_out = b->nb_out;
    a.kclock = kclock;
    if (b->substeps && !b->traj_t)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "substeps (closed-loop records) needs traj_t");
    // fallback launch: agents the main launch defers (the lean launch: QPs that need the PDIP or
    // phase 1; beyond the separable kernel's 16 CBF row slots) are solved by a second launch of
    // the full separable pipeline (128 slots when the 16 can be exceeded)
    const bool fb = c->dev.cbf_mode != 1 && impc_may_defer(c->dev, c->variant, !grid, b->knn_k, b->num_agents);
    c->last_n = b->num_agents;
    if (fb && c->defer_cap < b->num_agents) {
        if (c->defer) (void)hipFree(c->defer);
        c->defer = nullptr;
        c->defer_cap = 0;
        HIP_TRY(hipMalloc(&c->defer, 2 * (size_t)(b->num_agents + 2) * sizeof(int32_t)));
        HIP_TRY(hipMemsetAsync(c->defer, 0, 2 * (size_t)(b->num_agents + 2) * sizeof(int32_t), stream));
        c->defer_cap = b->num_agents;
        c->defer_parity = 0;
    }
    int32_t* q_this = nullptr;
    if (fb) {
        q_this = c->defer + (size_t)c->defer_parity * (c->defer_cap + 2);
        a.defer_clear = c->defer + (size_t)(c->defer_parity ^ 1) * (c->defer_cap + 2);
    }
    a.defer = q_this;
    if (ev0) HIP_TRY(hipEventRecord(ev0, stream));
    hipError_t e = c->dev.cbf_mode == 1 ? launch_impc_fov(c->dev, c->dbuf, a, stream)
                                        : launch_impc(c->dev, c->dbuf, a, c->variant, stream);
    // the queues alternate only once the main launch is enqueued: a launch that failed zeroed no
    // header, so the next call must append to this step's queue again (zeroed by the launch before)
    if (e == hipSuccess && fb) c->defer_parity ^= 1;
    if (e == hipSuccess && fb) {
        ImpcArgs f = a;
        f.defer = nullptr;
        f.defer_clear = nullptr;
        f.kclock = nullptr;  // (the clock is the main launch's)
        f.queue = q_this;
        e = launch_impc_fallback(c->dev, c->dbuf, f, impc_rows_may_exceed(c->dev, !grid, b->knn_k), stream);
        // (a queue the fallback never read is zeroed by the main launch after next)
    }
    if (e == hipSuccess && ev1) e = hipEventRecord(ev1, stream);
    if (e == hipErrorInvalidValue)
        return fail(MPCCBF_ERR_CAPACITY, "no kernel instantiation for this reduced dimension / row count");
    HIP_TRY(e);
    return MPCCBF_OK;
}


extern "C" {

int mpccbf_abi_version(void) { return MPCCBF_ABI_VERSION; }

const char* mpccbf_last_error(void) { return g_err.c_str(); }

const char* mpccbf_status_string(int32_t s) {
    switch (s) {
        case MPCCBF_OPTIMAL: return "OPTIMAL";
        case MPCCBF_FEASIBLE: return "FEASIBLE";
        case MPCCBF_UNBOUNDED: return "UNBOUNDED";
        case MPCCBF_INFEASIBLE: return "INFEASIBLE";
        case MPCCBF_ERROR: return "ERROR";
        case MPCCBF_UNKNOWN: return "UNKNOWN";
        case MPCCBF_INFEASIBLEORUNBOUNDED: return "INFEASIBLEORUNBOUNDED";
        default: return "";
    }
}

int mpccbf_create(const mpccbf_params* p, const mpccbf_options* opt, mpccbf_ctx** out) {
    if (!p || !out) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    const std::string verr = validate_params(*p);
    if (!verr.empty()) return fail(MPCCBF_ERR_INVALID_ARGUMENT, verr);
    if (p->cbf_horizon > MAX_CBF_H) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "cbf_horizon > 8 not supported");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(MPCCBF_ERR_NO_DEVICE, "no HIP device visible");
    mpccbf_ctx* c = new mpccbf_ctx();
    c->p = *p;
    if (opt) c->opt = *opt; else std::memset(&c->opt, 0, sizeof(c->opt));
    c->device = c->opt.device;
    try {
        c->ops = build_operators(*p, c->opt.keep_redundant != 0);
    } catch (const std::exception& e) {
        delete c;
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, e.what());
    }
    const Operators& o = c->ops;
    DevOps& d = c->dev;
    std::memset(&d, 0, sizeof(d));
    d.n = o.n;
    d.nz = o.nz;
    d.m = o.G.r;
    d.mc = o.Cs.r;
    d.K = o.K;
    d.spd_f = o.spd_f;
    d.cbf_h = o.cbf_h;
    d.impc_iter = p->impc_iter;
    std::vector<double> v;
    // operator buffer: the operators of the separable kernels first (the "hot" prefix the
    // one-agent-per-wave kernel stages in LDS, DevOps::hot), then the rest
    // separable layout: box rows regrouped by channel, 16 per channel (lanes of a group)
    d.sep = 0;
    d.o_Gsep = 0;
    if (o.sep && o.nzd == SEP_NZD_HOST) {
        int per[DIM] = {0, 0, 0};
        bool ok = true;
        for (int i = 0; i < o.G.r; i++) {
            if (o.row_dim[i] < 0 || o.row_dim[i] >= DIM) ok = false;
            else per[o.row_dim[i]]++;
            if (!(o.lo[i] > -1e300 && o.hi[i] < 1e300)) ok = false;  // the layout is two-sided only
        }
        const int rpd = std::max(per[0], std::max(per[1], per[2]));
        const int sb = (rpd + 15) / 16;  // row slots per lane and channel
        if (ok && sb <= 2) {
            std::vector<double> B((size_t)DIM * sb * 16 * SEP_ROW, 0.0);
            for (size_t r = 0; r < (size_t)DIM * sb * 16; r++) {
                B[r * SEP_ROW + 8] = -1.0;  // inert row: 0 in [-1, 1]
                B[r * SEP_ROW + 9] = 1.0;
            }
            int fill[DIM] = {0, 0, 0};
            for (int i = 0; i < o.G.r; i++) {
                const int dd = o.row_dim[i], f = fill[dd]++;
                // slot f / 16, lane f % 16 (sb = 1: row f of the channel in lane f)
                double* r = &B[((size_t)(dd * sb + f / 16) * 16 + f % 16) * SEP_ROW];
                r[0] = o.G(i, dd * o.nzd);
                r[1] = o.G(i, dd * o.nzd + 1);
                for (int s = 0; s < SD; s++) r[2 + s] = o.Gs(i, s);
                r[8] = o.lo[i];
                r[9] = o.hi[i];
            }
            pack(v, d.o_Gsep, B);
            std::vector<double> Pi((size_t)DIM * 3, 0.0);  // [[a b] [b c]]^-1 per channel
            for (int dd = 0; dd < DIM; dd++) {
                const int r0 = dd * o.nzd;
                const double a = o.Pr(r0, r0), b = o.Pr(r0, r0 + 1), cc = o.Pr(r0 + 1, r0 + 1);
                const double det = a * cc - b * b;
                Pi[dd * 3 + 0] = cc / det;
                Pi[dd * 3 + 1] = -b / det;
                Pi[dd * 3 + 2] = a / det;
            }
            pack(v, d.o_Pinv, Pi);
            d.sep = 1;
            d.nzd = o.nzd;
            d.sep_rows_per_dim = rpd;
            d.sep_sb = sb;
        }
    }
    pack(v, d.o_Z, o.Z);
    pack(v, d.o_Xs, o.Xs);
    pack(v, d.o_Pr, o.Pr);
    pack(v, d.o_Qs, o.Qs);
    pack(v, d.o_Qt, o.Qt);
    pack(v, d.o_Qr, o.Qr);
    pack(v, d.o_Ks, o.Ks);
    pack(v, d.o_Kt, o.Kt);
    pack(v, d.o_Kr, o.Kr);
    pack(v, d.o_Cs, o.Cs);
    pack(v, d.o_clo, o.clo);
    pack(v, d.o_chi, o.chi);
    pack(v, d.o_UZ, o.UZ);
    pack(v, d.o_US, o.US);
    pack(v, d.o_PZ, o.PZ);
    pack(v, d.o_PS, o.PS);
    pack(v, d.o_AZ, o.AZ);
    pack(v, d.o_AS, o.AS);
    d.P = p->num_pieces;
    d.slack_mode = p->slack_mode ? 1 : 0;
    d.slack_cost = p->slack_cost;
    d.slack_decay = p->slack_decay_rate;
    pack(v, d.o_EB0, o.EB0);
    pack(v, d.o_EB1, o.EB1);
    pack(v, d.o_cum, o.cum);
    d.hot = (int32_t)v.size();
    pack(v, d.o_LPr, o.LPr);
    pack(v, d.o_G, o.G);
    pack(v, d.o_Gs, o.Gs);
    pack(v, d.o_lo, o.lo);
    pack(v, d.o_hi, o.hi);
    d.eval_step = o.eval_step;
    {
        const double tend = o.cum.empty() ? 0.0 : o.cum.back();
        d.az_at_eval = (!o.cum.empty() && std::min(o.eval_step, tend) == std::min(p->h, tend)) ? 1 : 0;
    }
    d.Ts = p->Ts;
    d.nsub = (int)(p->h / p->Ts);
    // FoV controller: Voronoi operators, dense 16-wide box rows, P / LP padded to 16 x 16
    d.cbf_mode = p->cbf_mode;
    d.C = p->num_control_points;
    d.fov_beta = p->fov_beta;
    {
        const dev::FovBorder fb = dev::fov_border(p->fov_beta);
        d.fov_kap = fb.kap;
        d.fov_sig = fb.sig_left;
        d.fov_none = fb.none ? 1 : 0;
    }
    d.fov_Ds = p->fov_Ds;
    d.fov_Rs = p->fov_Rs;
    for (int k = 0; k < 3; k++) d.bbox[k] = p->bbox[k];
    if (p->cbf_mode == 1 && o.nz <= 15) {
        pack(v, d.o_VZ, o.VZ);
        pack(v, d.o_VS, o.VS);
        std::vector<double> W((size_t)o.G.r * WBOX_ROW, 0.0);
        for (int i = 0; i < o.G.r; i++) {
            double* r = &W[(size_t)i * WBOX_ROW];
            for (int j = 0; j < o.nz; j++) r[j] = o.G(i, j);
            for (int s2 = 0; s2 < SD; s2++) r[16 + s2] = o.Gs(i, s2);
            r[22] = o.lo[i];
            r[23] = o.hi[i];
        }
        pack(v, d.o_Wbox, W);
        std::vector<double> P16(256, 0.0), L16(256, 0.0);
        for (int a = 0; a < 16; a++)
            for (int b = 0; b < 16; b++) {
                const bool in = a < o.nz && b < o.nz;
                P16[a * 16 + b] = in ? o.Pr(a, b) : (a == b ? 1.0 : 0.0);
                L16[a * 16 + b] = in ? o.LPr(a, b) : (a == b ? 1.0 : 0.0);
            }
        pack(v, d.o_P16, P16);
        pack(v, d.o_LP16, L16);
        // P^-1 (padded with the identity) for the dual active-set solve: columns of
        // L^-T L^-1 e_b by forward / backward substitution with the factor L = LPr
        std::vector<double> Pi16(256, 0.0);
        for (int b = 0; b < 16; b++) {
            if (b >= o.nz) {
                Pi16[b * 16 + b] = 1.0;
                continue;
            }
            std::vector<double> x(o.nz, 0.0);
            for (int a = 0; a < o.nz; a++) {  // L x = e_b
                double s = a == b ? 1.0 : 0.0;
                for (int k = 0; k < a; k++) s -= o.LPr(a, k) * x[k];
                x[a] = s / o.LPr(a, a);
            }
            for (int a = o.nz - 1; a >= 0; a--) {  // L^T x = x
                double s = x[a];
                for (int k = a + 1; k < o.nz; k++) s -= o.LPr(k, a) * x[k];
                x[a] = s / o.LPr(a, a);
            }
            for (int a = 0; a < o.nz; a++) Pi16[a * 16 + b] = x[a];
        }
        pack(v, d.o_Pinv16, Pi16);
        std::vector<double> wb(o.G.r, 0.0);  // the box rows' weights in the active-set candidate rule
        for (int i = 0; i < o.G.r; i++) {
            double n2 = 0.0;
            for (int a = 0; a < o.nz; a++)
                for (int b = 0; b < o.nz; b++) n2 += o.G(i, a) * Pi16[a * 16 + b] * o.G(i, b);
            wb[i] = 1.0 / std::sqrt(std::max(n2, 1e-30));
        }
        pack(v, d.o_wbox, wb);
        auto pgram = [&](const Mat& A, int i, int j) {  // A_i P^-1 A_j^T
            double g = 0.0;
            for (int a = 0; a < o.nz; a++)
                for (int b = 0; b < o.nz; b++) g += A(i, a) * Pi16[a * 16 + b] * A(j, b);
            return g;
        };
        std::vector<double> wv, wf;
        for (const Mat& V : o.VZ) {
            wv.push_back(pgram(V, 0, 0));
            wv.push_back(pgram(V, 0, 1));
            wv.push_back(pgram(V, 1, 1));
        }
        for (const Mat& U : o.UZ)
            for (int i = 0; i < 3; i++)
                for (int j = i; j < 3; j++) wf.push_back(pgram(U, i, j));
        pack(v, d.o_wvor, wv);
        pack(v, d.o_wfov, wf);
    }
    v.push_back(0.0);  // keep every offset addressable even for empty operators
    for (int i = 0; i < 3; i++) {
        d.a_lo[i] = o.a_lo[i];
        d.a_hi[i] = o.a_hi[i];
    }
    d.d_min = p->d_min;
    d.cbf_filter = c->opt.no_cbf_filter ? 0 : 1;
    d.maxit = c->opt.max_pdip_iters > 0 ? c->opt.max_pdip_iters : 60;
    d.tol = c->opt.tolerance > 0 ? c->opt.tolerance : 1e-9;
    // solver pipeline: from mpccbf_options only (zero = default)
    const mpccbf_options& so = c->opt;
    d.warm_delta = so.warm_delta == 0.0 ? 0.3 : (so.warm_delta > 0.0 ? so.warm_delta : 0.0);
    d.feas_tol = 1e-6;  // CPLEX default feasibility tolerance
    d.early_it = so.early_it == 0 ? 10 : (so.early_it > 0 ? so.early_it : 0);
    d.fast_start = so.no_fast_start ? 0 : 1;
    d.dual_as = so.dual_as_steps == 0 ? 24 : (so.dual_as_steps > 0 ? so.dual_as_steps : 0);
    d.lean = so.lean ? 1 : 0;  // measured no faster at occupancy 1
    d.das_warm = so.das_warm_steps == 0 ? 3 : (so.das_warm_steps > 0 ? so.das_warm_steps : 0);
#ifdef MPCCBF_DIAG_ENV
    {  // diagnostics build only (make diag): tuning overrides from the environment
        const char* e = getenv("MPCCBF_EARLY_IT");
        if (e) d.early_it = atoi(e);
        const char* f = getenv("MPCCBF_FAST_START");
        if (f) d.fast_start = atoi(f);
        const char* g = getenv("MPCCBF_DUAL_AS");
        if (g) d.dual_as = atoi(g);
        const char* l = getenv("MPCCBF_LEAN");
        if (l) d.lean = atoi(l);
        const char* w = getenv("MPCCBF_DAS_WARM");
        if (w) d.das_warm = atoi(w);
        const char* wd = getenv("MPCCBF_WARM_DELTA");
        if (wd) d.warm_delta = std::max(0.0, std::strtod(wd, nullptr));
    }
#endif
    c->variant = 0;
    hipError_t e = hipSetDevice(c->device);
    d.wide_max = 1024;
    if (e == hipSuccess) {
        // share-adaptive layout: one agent per wave up to one agent per SIMD (4 per CU) of this
        // context's device (kept in the context: no process-wide state shared by contexts)
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, c->device) == hipSuccess && prop.multiProcessorCount > 0)
            d.wide_max = 4 * prop.multiProcessorCount;
    }
    if (e == hipSuccess) e = hipMalloc(&c->dbuf, v.size() * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(c->dbuf, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (c->dbuf) (void)hipFree(c->dbuf);
        delete c;
        return fail(MPCCBF_ERR_HIP, std::string("operator upload: ") + hipGetErrorString(e));
    }
    c->dbuf_elems = v.size();
    *out = c;
    return MPCCBF_OK;
}

void mpccbf_destroy(mpccbf_ctx* c) {
    if (!c) return;
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    if (c->dbuf) (void)hipFree(c->dbuf);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->grid_scratch) (void)hipFree(c->grid_scratch);
    if (c->defer) (void)hipFree(c->defer);
    delete c;
}

int mpccbf_num_vars(const mpccbf_ctx* c) { return c ? c->ops.n : -1; }
int mpccbf_reduced_dim(const mpccbf_ctx* c) { return c ? c->ops.nz : -1; }
int mpccbf_num_shared_rows(const mpccbf_ctx* c) { return c ? c->ops.G.r : -1; }

int mpccbf_impc_solve(mpccbf_ctx* c, const mpccbf_batch* b, void* stream) {
    return impc_enqueue(c, b, (hipStream_t)stream, nullptr, nullptr);
}

int32_t mpccbf_impc_launch_waves(const mpccbf_ctx* c, int32_t num_agents) {
    return c ? impc_clock_waves(c->dev, c->variant, num_agents) : 0;
}

const char* mpccbf_kernel_name(const mpccbf_ctx* c) {
    if (!c) return "";
    if (c->dev.cbf_mode == 1) return c->dev.slack_mode ? "impc_fov_kernel<true>" : "impc_fov_kernel<false>";
    const char* n = impc_kernel_name(c->dev, c->variant, c->last_n);
    return n ? n : "";
}

int mpccbf_set_variant(mpccbf_ctx* c, int variant) {
    if (!c) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "null argument");
    c->variant = variant;
    return MPCCBF_OK;
}

int mpccbf_build_neighbors(mpccbf_ctx* c, const double* states, int32_t num_states,
                           int32_t first, int32_t num_agents, int32_t k, double radius,
                           int32_t* row_ptr, int32_t* col, void* stream) {
    if (!c || !states || !row_ptr) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "null argument");
    if (first < 0 || num_agents < 0 || first + num_agents > num_states)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "agent range outside states");
    if (k > 16) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "k > 16 not supported (use k <= 0 for all)");
    if (k > 0 && !(radius > 0)) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "radius must be positive");
    HIP_TRY(hipSetDevice(c->device));
    const size_t need = neighbors_scratch_bytes(num_states, num_agents, k);
    if (need > c->scratch_bytes) {
        if (c->scratch) (void)hipFree(c->scratch);
        c->scratch = nullptr;
        c->scratch_bytes = 0;
        HIP_TRY(hipMalloc(&c->scratch, need));
        c->scratch_bytes = need;
    }
    const int rc = launch_neighbors(states, num_states, first, num_agents, k, radius, row_ptr, col,
                                    c->scratch, c->scratch_bytes, (hipStream_t)stream);
    if (rc != 0) return fail(MPCCBF_ERR_HIP, std::string("neighbour kernels: ") + hipGetErrorString((hipError_t)rc));
    return MPCCBF_OK;
}

}  // extern "C"


// ---------------------------------------------------------------------------------------------
// Closed-loop stepping + RCCL exchange
// ---------------------------------------------------------------------------------------------
// In-process communicator group (mpccbf_comm_create_local): the ranks are host threads of one
// process on one device; the per-step all-gather becomes device copies between their state
// tables, ordered by one event per rank and step and a host barrier, so mpccbf_run_steps runs its
// N-rank data flow (own block written by the IMPC kernel, exchange, the other blocks inserted
// into the next neighbour table) on a single GPU.
struct LocalGroup {
    int nranks = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    long long gen = 0;
    std::vector<double*> table[2];     // [step & 1][rank]: the table that rank wrote this step
    std::vector<hipEvent_t> ev[2];     // [step & 1][rank]: that rank's IMPC kernel of the step done
    // (double-buffered by step parity: a rank rewrites slot s & 1 only after the barrier of step
    // s + 1, which every peer reaches after enqueueing its step-s copies)
    std::vector<int> nsteps;           // [rank]: num_steps of the current mpccbf_run_steps call
    bool aborted = false;              // a rank left early: every barrier fails from then on
    // false: a rank aborted (the group cannot be used again; destroy and recreate it)
    bool barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) return false;
        const long long g = gen;
        if (++arrived == nranks) {
            arrived = 0;
            gen++;
            cv.notify_all();
            return true;
        }
        cv.wait(lk, [&] { return gen != g || aborted; });
        return gen != g;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m);
        aborted = true;
        cv.notify_all();
    }
};

// Aborts the rank's in-process group when mpccbf_run_steps leaves before its last barrier, so the
// peers' barriers return an error instead of waiting forever.
struct GroupAbortGuard {
    LocalGroup* g = nullptr;
    ~GroupAbortGuard() {
        if (g) g->abort();
    }
};

struct mpccbf_comm {
    ncclComm_t nccl = nullptr;
    int nranks = 1, rank = 0, device = 0;
    std::shared_ptr<LocalGroup> local;  // set: in-process group (no RCCL)
};

extern "C" {

int mpccbf_comm_unique_id(char id_out[MPCCBF_COMM_ID_BYTES]) {
    if (!id_out) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "null argument");
    static_assert(sizeof(ncclUniqueId) == MPCCBF_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(MPCCBF_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(id_out, &id, sizeof(id));
    return MPCCBF_OK;
}

int mpccbf_comm_create(const char id[MPCCBF_COMM_ID_BYTES], int32_t nranks, int32_t rank, int32_t device,
                       mpccbf_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "bad communicator arguments");
    *out = nullptr;
    HIP_TRY(hipSetDevice(device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    mpccbf_comm* cm = new mpccbf_comm();
    cm->nranks = nranks;
    cm->rank = rank;
    cm->device = device;
    const ncclResult_t r = ncclCommInitRank(&cm->nccl, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete cm;
        return fail(MPCCBF_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    *out = cm;
    return MPCCBF_OK;
}

int mpccbf_comm_create_local(int32_t nranks, int32_t device, mpccbf_comm** out) {
    if (!out || nranks < 1) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "bad communicator arguments");
    HIP_TRY(hipSetDevice(device));
    auto g = std::make_shared<LocalGroup>();
    g->nranks = nranks;
    for (int p = 0; p < 2; p++) {
        g->table[p].assign(nranks, nullptr);
        g->ev[p].assign(nranks, nullptr);
        for (int r = 0; r < nranks; r++) HIP_TRY(hipEventCreateWithFlags(&g->ev[p][r], hipEventDisableTiming));
    }
    g->nsteps.assign(nranks, 0);
    for (int r = 0; r < nranks; r++) {
        out[r] = new mpccbf_comm();
        out[r]->nranks = nranks;
        out[r]->rank = r;
        out[r]->device = device;
        out[r]->local = g;
    }
    return MPCCBF_OK;
}

void mpccbf_comm_destroy(mpccbf_comm* cm) {
    if (!cm) return;
    if (cm->nccl) (void)ncclCommDestroy(cm->nccl);
    if (cm->local && cm->local.use_count() == 1)
        for (int p = 0; p < 2; p++)
            for (hipEvent_t e : cm->local->ev[p]) (void)hipEventDestroy(e);
    delete cm;
}

int mpccbf_run_steps(mpccbf_ctx* c, const mpccbf_batch* b, mpccbf_run* r, void* stream_) {
    if (!c || !b || !r) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "null argument");
    // in-process group: any return before the last step's barrier aborts the group (the peers
    // get an error), and every rank must run the same number of steps
    LocalGroup* lg = (r->comm && r->comm->nranks > 1 && r->comm->local) ? r->comm->local.get() : nullptr;
    GroupAbortGuard guard{lg};
    if (lg) {
        {
            std::lock_guard<std::mutex> lk(lg->m);
            lg->nsteps[r->comm->rank] = r->num_steps;
        }
        if (!lg->barrier()) return fail(MPCCBF_ERR_HIP, "run: a rank of the in-process group aborted");
        bool same = true;
        {
            std::lock_guard<std::mutex> lk(lg->m);
            for (int v : lg->nsteps) same = same && v == r->num_steps;
        }
        // (every rank reads the counts before any rank can overwrite them at its next call's
        // entry: that write follows this call's step barriers, or the abort below)
        if (!same) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "run: ranks of the in-process group differ in num_steps");
        if (r->num_steps == 0) {
            if (!lg->barrier()) return fail(MPCCBF_ERR_HIP, "run: a rank of the in-process group aborted");
            guard.g = nullptr;
            return MPCCBF_OK;
        }
    }
    if (r->num_steps < 0 || !r->states_alt || !b->states)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "run: num_steps < 0 or missing state tables");
    const int first = b->agent_first, count = b->num_agents, ns = b->num_states;
    if (first < 0 || count < 0 || first + count > ns) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "agent range outside states");
    if (r->comm && (ns != r->comm->nranks * count || first != r->comm->rank * count))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "run: ranks must own equal contiguous agent blocks");
    hipStream_t stream = (hipStream_t)stream_;
    HIP_TRY(hipSetDevice(c->device));
    const bool timing = r->step_ms || r->solve_ms;
    const int kcw = impc_clock_waves(c->dev, c->variant, count);  // (pairs per step)
    if (r->kernel_clock && r->kernel_clock_waves < kcw)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "run: kernel_clock_waves < mpccbf_impc_launch_waves (" +
                                                     std::to_string(kcw) + ")");
    if (r->kernel_clock && r->num_steps > 0)
        HIP_TRY(hipMemsetAsync(r->kernel_clock, 0,
                               2 * sizeof(uint64_t) * (size_t)r->kernel_clock_waves * (size_t)r->num_steps, stream));
    const int need = 3 * std::max(r->num_steps, r->reserve_steps) + 1;
    while ((int)c->events.size() < need) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        c->events.push_back(e);
    }
    double* tables[2] = {const_cast<double*>(b->states), r->states_alt};
    const size_t per_log = (size_t)count * c->p.impc_iter;
    mpccbf_batch sb = *b;
    hipEvent_t* ev = c->events.data();
    if (timing) HIP_TRY(hipEventRecord(ev[0], stream));
    // grid mode: neighbour table 0 from the initial states, table 1 zeroed for step 0's inserts
    // (each IMPC launch zeroes the table two steps ahead, see impc_enqueue)
    const bool gtab = b->nb_row_ptr == nullptr && count > 0 && r->num_steps > 0;
    uint32_t *gcnt[3] = {}, *gslots[3] = {};
    double* gsst[3] = {};
    int gbase = 0;  // the first step's table index (gstep = gbase + s)
    if (gtab) {
        if (b->knn_k < 1 || !(b->knn_radius > 0))
            return fail(MPCCBF_ERR_INVALID_ARGUMENT, "grid neighbours need knn_k >= 1 and knn_radius > 0");
        const int rc = grid_tables(c, ns, gcnt, gslots, gsst);
        if (rc != MPCCBF_OK) return rc;
        const auto& g = c->gcont;
        const bool cont = r->continue_tables && g.valid && g.states == b->states && g.ns == ns && g.first == first &&
                          g.count == count && g.k == b->knn_k && g.radius == b->knn_radius;
        if (cont) {
            // the previous call's last step filled table g.next with these states and zeroed the
            // one after it: this call's first step reads the former and fills the latter
            gbase = g.next;
        } else {
            const size_t cb = (size_t)grid_table_size(ns) * 4;
            HIP_TRY(hipMemsetAsync(gcnt[0], 0, cb, stream));
            HIP_TRY(hipMemsetAsync(gcnt[1], 0, cb, stream));
            HIP_TRY(launch_grid_insert(b->states, ns, 0, 0, b->knn_radius, gcnt[0], gslots[0], gsst[0], stream));
        }
        c->gcont.valid = false;  // (set again once every step is enqueued)
    }
    for (int s = 0; s < r->num_steps; s++) {
        double* cur = tables[s & 1];
        double* nxt = tables[(s & 1) ^ 1];
        sb.states = cur;
        sb.next_states = nxt + (size_t)first * 6;
        sb.step_index = b->step_index + s;
        if (r->status_log) sb.status = r->status_log + (size_t)s * per_log;
        if (r->iters_log) sb.iters = r->iters_log + (size_t)s * per_log;
        if (!r->comm) {  // rows this batch does not solve (static agents) carry over
            if (first > 0)
                HIP_TRY(hipMemcpyAsync(nxt, cur, (size_t)first * 6 * sizeof(double), hipMemcpyDeviceToDevice, stream));
            const int tail = ns - first - count;
            if (tail > 0)
                HIP_TRY(hipMemcpyAsync(nxt + (size_t)(first + count) * 6, cur + (size_t)(first + count) * 6,
                                       (size_t)tail * 6 * sizeof(double), hipMemcpyDeviceToDevice, stream));
        }
        const bool tk = r->solve_ms && (r->solve_stride <= 1 || s % r->solve_stride == 0);
        const int rc = impc_enqueue(c, &sb, stream, tk ? ev[3 * s + 1] : nullptr, tk ? ev[3 * s + 2] : nullptr,
                                    gtab ? gbase + s : -1,
                                    r->kernel_clock ? (unsigned long long*)r->kernel_clock +
                                                          2 * (size_t)r->kernel_clock_waves * s
                                                    : nullptr);
        if (rc != MPCCBF_OK) return rc;
        if (r->comm && r->comm->nranks > 1 && r->comm->local) {
            // in-process group: every rank's block of this step copied into this rank's table
            LocalGroup& g = *r->comm->local;
            const int me = r->comm->rank;
            g.table[s & 1][me] = nxt;
            HIP_TRY(hipEventRecord(g.ev[s & 1][me], stream));
            if (!g.barrier()) return fail(MPCCBF_ERR_HIP, "run: a rank of the in-process group aborted");
            for (int p = 0; p < g.nranks; p++) {
                if (p == me) continue;
                HIP_TRY(hipStreamWaitEvent(stream, g.ev[s & 1][p], 0));
                HIP_TRY(hipMemcpyAsync(nxt + (size_t)p * count * 6, g.table[s & 1][p] + (size_t)p * count * 6,
                                       (size_t)count * 6 * sizeof(double), hipMemcpyDeviceToDevice, stream));
            }
        } else if (r->comm && r->comm->nranks > 1) {
            const ncclResult_t nr = ncclAllGather(nxt + (size_t)first * 6, nxt, (size_t)count * 6, ncclDouble,
                                                  r->comm->nccl, stream);
            if (nr != ncclSuccess) return fail(MPCCBF_ERR_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(nr));
        }
        // the rows the kernel did not insert (static rows / the other ranks' rows) join the table
        // of the next step
        if (gtab && count < ns) {
            const int t = (gbase + s + 1) % 3;
            HIP_TRY(launch_grid_insert(nxt, ns, first, first + count, b->knn_radius, gcnt[t], gslots[t], gsst[t],
                                       stream));
        }
        if (r->step_ms || (timing && s == r->num_steps - 1)) HIP_TRY(hipEventRecord(ev[3 * s + 3], stream));
    }
    guard.g = nullptr;  // every barrier of the call passed: the peers no longer wait on this rank
    r->final_table = r->num_steps & 1;
    if (gtab) {  // where a continuing call picks the rotation up (mpccbf_run::continue_tables)
        auto& g = c->gcont;
        g.valid = true;
        g.states = tables[r->num_steps & 1];
        g.ns = ns;
        g.first = first;
        g.count = count;
        g.k = b->knn_k;
        g.radius = b->knn_radius;
        g.next = (gbase + r->num_steps) % 3;
    }
    if (timing && r->num_steps > 0) {
        HIP_TRY(hipEventSynchronize(ev[3 * (r->num_steps - 1) + 3]));
        for (int s = 0; s < r->num_steps; s++) {
            float ms = 0.f;
            if (r->step_ms) {
                HIP_TRY(hipEventElapsedTime(&ms, ev[s == 0 ? 0 : 3 * (s - 1) + 3], ev[3 * s + 3]));
                r->step_ms[s] = ms;
            }
            if (r->solve_ms) {
                if (r->solve_stride <= 1 || s % r->solve_stride == 0) {
                    HIP_TRY(hipEventElapsedTime(&ms, ev[3 * s + 1], ev[3 * s + 2]));
                    r->solve_ms[s] = ms;
                } else {
                    r->solve_ms[s] = -1.f;
                }
            }
        }
    }
    return MPCCBF_OK;
}

}  // extern "C"

extern "C" {

int mpccbf_connectivity_control_solve(const mpccbf_connectivity_control_params* p,
                                      const mpccbf_connectivity_control_batch* b, int32_t device,
                                      void* stream) {
    if (!p || !b) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "null argument");
    if (!(p->d_min > 0.0) || !(p->d_max > 0.0))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "d_min and d_max must be positive");
    for (int d = 0; d < 3; d++)
        if (!(p->v_min[d] <= p->v_max[d])) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "v_min must not exceed v_max");
    if (p->slack_mode && !(p->slack_cost > 0.0))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "Slack cost must be positive when slack_mode is enabled");
    if (p->slack_mode && !(p->slack_decay_rate > 0.0 && p->slack_decay_rate <= 1.0))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "Slack decay rate must be in (0,1] when slack_mode is enabled");
    if (b->num_teams < 0) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "num_teams < 0");
    if (b->num_teams == 0) return MPCCBF_OK;
    if (!b->team_ptr || !b->states || !b->desired_u || !b->u)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "team_ptr, states, desired_u and u are required");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(MPCCBF_ERR_NO_DEVICE, "no HIP device visible");
    HIP_TRY(hipSetDevice(device));
    ConnControlArgs a;
    std::memset(&a, 0, sizeof(a));
    a.num_teams = b->num_teams;
    a.team_ptr = b->team_ptr;
    a.states = b->states;
    a.desired_u = b->desired_u;
    a.u = b->u;
    a.status = b->status;
    a.obj = b->obj;
    a.iters = b->iters;
    a.lambda2 = b->lambda2;
    a.dmin = p->d_min;
    a.dmax = p->d_max;
    for (int d = 0; d < 3; d++) {
        a.vmin[d] = p->v_min[d];
        a.vmax[d] = p->v_max[d];
    }
    a.maxit = p->max_pdip_iters > 0 ? p->max_pdip_iters : 60;
    a.tol = p->tolerance > 0.0 ? p->tolerance : 1e-9;
    a.feas_tol = 1e-6;
    a.slack_mode = p->slack_mode ? 1 : 0;
    a.slack_cost = p->slack_cost;
    a.slack_decay = p->slack_decay_rate;
    HIP_TRY(launch_connectivity_control(a, (hipStream_t)stream));
    return MPCCBF_OK;
}

int mpccbf_fov_rows_eval(int32_t count, const double* ego, const double* nb_xy, double fov, double Ds,
                         double Rs, const double* bbox, double* voronoi, double* fov_rows, void* stream) {
    if (count < 0 || (count > 0 && (!ego || !nb_xy))) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "bad arguments");
    if (count == 0) return MPCCBF_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(MPCCBF_ERR_NO_DEVICE, "no HIP device visible");
    const double bbx = bbox ? bbox[0] : 0.0, bby = bbox ? bbox[1] : 0.0;
    HIP_TRY(launch_fov_rows_eval(count, ego, nb_xy, fov, Ds, Rs, bbx, bby, voronoi, fov_rows, (hipStream_t)stream));
    return MPCCBF_OK;
}

int mpccbf_fov_control_solve(const mpccbf_fov_control_params* p, const mpccbf_fov_control_batch* b,
                             int32_t device, void* stream) {
    if (!p || !b) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "null argument");
    if (p->slack_mode && !(p->slack_cost > 0.0))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "Slack cost must be positive when slack_mode is enabled");
    if (p->slack_mode && !(p->slack_decay_rate > 0.0 && p->slack_decay_rate <= 1.0))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "Slack decay rate must be in (0,1] when slack_mode is enabled");
    if (!(p->fov > 0.0) || !(p->Rs > 0.0))
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "fov and Rs must be positive");
    for (int d = 0; d < 3; d++)
        if (!(p->u_min[d] <= p->u_max[d]) || !(p->v_min[d] <= p->v_max[d]))
            return fail(MPCCBF_ERR_INVALID_ARGUMENT, "bounds: min must not exceed max");
    if (b->num_agents < 0) return fail(MPCCBF_ERR_INVALID_ARGUMENT, "num_agents < 0");
    if (b->num_agents == 0) return MPCCBF_OK;
    if (!b->states || !b->desired_u || !b->nb_row_ptr || !b->u)
        return fail(MPCCBF_ERR_INVALID_ARGUMENT, "states, desired_u, nb_row_ptr and u are required");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(MPCCBF_ERR_NO_DEVICE, "no HIP device visible");
    HIP_TRY(hipSetDevice(device));
    FovControlArgs a;
    std::memset(&a, 0, sizeof(a));
    a.num_agents = b->num_agents;
    a.states = b->states;
    a.desired_u = b->desired_u;
    a.nb_row_ptr = b->nb_row_ptr;
    a.nb_xy = b->nb_xy;
    a.u = b->u;
    a.status = b->status;
    a.obj = b->obj;
    a.iters = b->iters;
    a.fov = p->fov;
    a.Ds = p->Ds;
    a.Rs = p->Rs;
    for (int d = 0; d < 3; d++) {
        a.vmin[d] = p->v_min[d];
        a.vmax[d] = p->v_max[d];
        a.umin[d] = p->u_min[d];
        a.umax[d] = p->u_max[d];
    }
    a.maxit = p->max_pdip_iters > 0 ? p->max_pdip_iters : 60;
    a.tol = p->tolerance > 0.0 ? p->tolerance : 1e-9;
    a.feas_tol = 1e-6;  // CPLEX's default feasibility tolerance
    for (int i = 0; i < 9; i++) {
        a.P[i] = (i % 4 == 0) ? 2.0 : 0.0;  // ||u - u_des||^2 = 1/2 u^T (2 I) u - 2 u_des^T u + c
        a.LP[i] = (i % 4 == 0) ? std::sqrt(2.0) : 0.0;
    }
    a.slack_mode = p->slack_mode ? 1 : 0;
    a.slack_cost = p->slack_cost;
    a.slack_decay = p->slack_decay_rate;
    a.nb_cov = b->nb_cov;
    HIP_TRY(launch_fov_control(a, (hipStream_t)stream));
    return MPCCBF_OK;
}

}  // extern "C"
