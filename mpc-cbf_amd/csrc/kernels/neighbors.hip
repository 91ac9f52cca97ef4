// neighbors.hip — neighbour lists for the batched IMPC step.
//
// The reference hands every other robot to the controller (ConnectivityIMPCCBF.cpp:59-67);
// `all` mode reproduces that. `knn` mode keeps the k nearest (planar) within a radius using a
// spatial hash of uniform cells (cell edge = radius): count -> scan -> scatter -> 3x3-cell
// query. Output rows are sorted by neighbour index so results do not depend on hash order.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "impc.hpp"

namespace mpccbf {
namespace dev {

constexpr int KNN_MAX = 16;


__device__ __forceinline__ void cell_of(double px, double py, double inv, long long& cx, long long& cy) {
    cx = (long long)floor(px * inv);
    cy = (long long)floor(py * inv);
}

__global__ void all_rows_kernel(int num_states, int first, int num_agents, int32_t* row_ptr,
                                int32_t* col) {
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long per = num_states - 1;
    if (tid <= num_agents) row_ptr[tid] = (int32_t)(tid * per);
    const long long total = (long long)num_agents * per;
    for (long long e = tid; e < total; e += (long long)gridDim.x * blockDim.x) {
        const long long a = e / per, j = e % per;
        const long long self = first + a;
        col[e] = (int32_t)(j < self ? j : j + 1);
    }
}

__global__ void hash_count_kernel(const double* __restrict__ st, int n, double inv, uint32_t mask,
                                  uint32_t* cnt, uint32_t* slot) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    long long cx, cy;
    cell_of(st[(size_t)i * 6], st[(size_t)i * 6 + 1], inv, cx, cy);
    const uint32_t h = cell_hash(cx, cy, mask);
    const uint32_t off = atomicAdd(&cnt[h], 1u);
    slot[i] = (h << 0);
    slot[n + i] = off;
}

// exclusive scan of cnt[0..T) into start[0..T]; one block of 1024 threads.
__global__ void scan_kernel(const uint32_t* __restrict__ cnt, uint32_t* start, int T) {
    __shared__ uint32_t part[1024];
    const int t = threadIdx.x;
    const int per = (T + 1023) / 1024;
    const int b = t * per, e = min(b + per, T);
    uint32_t s = 0;
    for (int i = b; i < e; i++) s += cnt[i];
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = t > 0 ? part[t - 1] : 0u;
    for (int i = b; i < e; i++) {
        start[i] = run;
        run += cnt[i];
    }
    if (t == 1023) start[T] = part[1023];
}

__global__ void scatter_kernel(int n, const uint32_t* __restrict__ slot,
                               const uint32_t* __restrict__ start, uint32_t* sorted) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sorted[start[slot[i]] + slot[n + i]] = (uint32_t)i;
}

__global__ void knn_query_kernel(const double* __restrict__ st, int n, int first, int num_agents,
                                 int k, double radius, double inv, uint32_t mask,
                                 const uint32_t* __restrict__ start,
                                 const uint32_t* __restrict__ sorted, int32_t* row_ptr,
                                 int32_t* col) {
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= num_agents) return;
    const int self = first + a;
    const double px = st[(size_t)self * 6], py = st[(size_t)self * 6 + 1];
    long long cx, cy;
    cell_of(px, py, inv, cx, cy);
    const double r2 = radius * radius;
    double bd[KNN_MAX];
    int bi[KNN_MAX];
#pragma unroll
    for (int i = 0; i < KNN_MAX; i++) {
        bd[i] = 1e308;
        bi[i] = 0x7fffffff;
    }
    for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
            const long long qx = cx + dx, qy = cy + dy;
            const uint32_t h = cell_hash(qx, qy, mask);
            // skip a bucket already visited by an earlier cell of this 3x3 block
            bool dup = false;
            for (int p = 0; p < (dy + 1) * 3 + (dx + 1); p++) {
                const long long px2 = cx + (p % 3) - 1, py2 = cy + (p / 3) - 1;
                if (cell_hash(px2, py2, mask) == h) dup = true;
            }
            if (dup) continue;
            for (uint32_t e = start[h]; e < start[h + 1]; e++) {
                const int j = (int)sorted[e];
                if (j == self) continue;
                const double ex = st[(size_t)j * 6] - px, ey = st[(size_t)j * 6 + 1] - py;
                double d2 = ex * ex + ey * ey;
                if (!(d2 <= r2)) continue;
                int jj = j;
                // insert (d2, jj) into the sorted list (branchless bubble over a fixed length)
#pragma unroll
                for (int i = 0; i < KNN_MAX; i++) {
                    const bool less = (d2 < bd[i]) || (d2 == bd[i] && jj < bi[i]);
                    const double td = less ? bd[i] : d2;
                    const int ti = less ? bi[i] : jj;
                    bd[i] = less ? d2 : bd[i];
                    bi[i] = less ? jj : bi[i];
                    d2 = td;
                    jj = ti;
                }
            }
        }
    // keep the k best, sorted by index
    int cntk = 0;
#pragma unroll
    for (int i = 0; i < KNN_MAX; i++)
        if (i < k && bi[i] != 0x7fffffff) cntk++;
#pragma unroll
    for (int i = 0; i < KNN_MAX; i++) {
        if (i >= cntk) bi[i] = 0x7fffffff;
    }
#pragma unroll
    for (int i = 0; i < KNN_MAX; i++)
#pragma unroll
        for (int j = 0; j < KNN_MAX - 1 - i; j++) {
            const int lo = min(bi[j], bi[j + 1]), hi = max(bi[j], bi[j + 1]);
            bi[j] = lo;
            bi[j + 1] = hi;
        }
    row_ptr[a + 1] = cntk;  // counts; converted to offsets by the fixed-stride layout below
#pragma unroll
    for (int i = 0; i < KNN_MAX; i++)
        if (i < cntk) col[(size_t)a * k + i] = bi[i];
}

// counts (row_ptr[1..]) -> offsets in place, compacting col from stride-k rows.
__global__ void knn_compact_kernel(int num_agents, int k, int32_t* row_ptr, int32_t* col,
                                   int32_t* col_tmp) {
    // single block: prefix over counts, then move rows
    __shared__ int32_t part[1024];
    const int t = threadIdx.x;
    const int per = (num_agents + 1023) / 1024;
    const int b = t * per, e = min(b + per, num_agents);
    int32_t s = 0;
    for (int i = b; i < e; i++) s += row_ptr[i + 1];
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int32_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int32_t run = t > 0 ? part[t - 1] : 0;
    if (t == 0) row_ptr[0] = 0;
    __syncthreads();
    for (int i = b; i < e; i++) {
        const int32_t c = row_ptr[i + 1];
        for (int j = 0; j < c; j++) col_tmp[run + j] = col[(size_t)i * k + j];
        run += c;
        row_ptr[i + 1] = run;
    }
}

}  // namespace dev
}  // namespace mpccbf

namespace mpccbf {

static inline uint32_t hash_table_size(int n) {
    uint32_t T = 1024;
    while (T < 2u * (uint32_t)n) T <<= 1;
    return T;
}

static inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

size_t neighbors_scratch_bytes(int num_states, int num_agents, int k) {
    if (k <= 0) return 256;
    const uint32_t T = hash_table_size(num_states);
    return align256((size_t)T * 4) + align256((size_t)(T + 1) * 4) + align256((size_t)num_states * 8) +
           align256((size_t)num_states * 4) + align256((size_t)num_agents * k * 4) + 256;
}

int launch_neighbors(const double* states, int num_states, int first, int num_agents, int k,
                     double radius, int32_t* row_ptr, int32_t* col, void* scratch,
                     size_t scratch_bytes, hipStream_t s) {
    if (num_agents <= 0) return 0;
    if (k <= 0) {
        const long long total = (long long)num_agents * (num_states - 1) + num_agents + 1;
        const int blocks = (int)std::min<long long>((total + 255) / 256, 65535);
        hipLaunchKernelGGL(dev::all_rows_kernel, dim3(blocks), dim3(256), 0, s, num_states, first,
                           num_agents, row_ptr, col);
        return (int)hipGetLastError();
    }
    const uint32_t T = hash_table_size(num_states);
    char* p = (char*)scratch;
    uint32_t* cnt = (uint32_t*)p;
    p += align256((size_t)T * 4);
    uint32_t* start = (uint32_t*)p;
    p += align256((size_t)(T + 1) * 4);
    uint32_t* slot = (uint32_t*)p;
    p += align256((size_t)num_states * 8);
    uint32_t* sorted = (uint32_t*)p;
    p += align256((size_t)num_states * 4);
    int32_t* wide = (int32_t*)p;
    (void)scratch_bytes;
    const double inv = 1.0 / radius;
    hipError_t e = hipMemsetAsync(cnt, 0, (size_t)T * 4, s);
    if (e != hipSuccess) return (int)e;
    const int nb = (num_states + 255) / 256;
    hipLaunchKernelGGL(dev::hash_count_kernel, dim3(nb), dim3(256), 0, s, states, num_states, inv,
                       T - 1, cnt, slot);
    hipLaunchKernelGGL(dev::scan_kernel, dim3(1), dim3(1024), 0, s, cnt, start, (int)T);
    hipLaunchKernelGGL(dev::scatter_kernel, dim3(nb), dim3(256), 0, s, num_states, slot, start, sorted);
    const int qb = (num_agents + 255) / 256;
    hipLaunchKernelGGL(dev::knn_query_kernel, dim3(qb), dim3(256), 0, s, states, num_states, first,
                       num_agents, k, radius, inv, T - 1, start, sorted, row_ptr, wide);
    hipLaunchKernelGGL(dev::knn_compact_kernel, dim3(1), dim3(1024), 0, s, num_agents, k, row_ptr,
                       wide, col);
    return (int)hipGetLastError();
}

}  // namespace mpccbf

namespace mpccbf {
namespace dev {

// Insert state rows [0, n) except [skip0, skip1) into a zeroed fixed-capacity bucket table, one
// thread per row (global atomics on the bucket counts; slot order inside a bucket follows atomic
// order, and the consumer orders neighbours by (distance, index), so results do not depend on it).
// Used for a whole table (standalone solve) and, in mpccbf_run_steps, for the rows the IMPC
// kernel did not write itself (static rows, or the other ranks' rows after the all-gather).
__global__ void __launch_bounds__(256) grid_insert_kernel(const double* __restrict__ st, int n, int skip0,
                                                          int skip1, GridArgs g) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int gap = skip1 - skip0;
    if (i >= n - gap) return;
    const int r = i < skip0 ? i : i + gap;
    const double* s = st + (size_t)r * 6;
    grid_insert(g, s[0], s[1], s[3], s[4], (uint32_t)r);
}

}  // namespace dev

static size_t al256(size_t b) { return (b + 255) / 256 * 256; }

// one table: bucket counts (T) | slots (T x GRID_CAP, bucket-major) | slot states (T x GRID_SSTR x 4)
size_t grid_table_bytes(int num_states) {
    const uint32_t T = grid_table_size(num_states);
    return al256((size_t)T * 4) + al256((size_t)T * GRID_CAP * 4) + (size_t)T * GRID_SSTR * 32;
}

void grid_table_carve(void* base, int num_states, uint32_t** cnt, uint32_t** slots, double** sst) {
    const uint32_t T = grid_table_size(num_states);
    *cnt = (uint32_t*)base;
    *slots = (uint32_t*)((char*)base + al256((size_t)T * 4));
    *sst = (double*)((char*)base + al256((size_t)T * 4) + al256((size_t)T * GRID_CAP * 4));
}

hipError_t launch_grid_insert(const double* states, int n, int skip0, int skip1, double radius,
                              uint32_t* cnt, uint32_t* slots, double* sst, hipStream_t s) {
    const int m = n - (skip1 - skip0);
    if (m <= 0) return hipSuccess;
    GridArgs g;
    memset(&g, 0, sizeof(g));
    g.ins_cnt = cnt;
    g.ins_slots = slots;
    g.ins_sst = sst;
    g.mask = grid_table_size(n) - 1u;
    g.inv_cell = 1.0 / radius;
    hipLaunchKernelGGL(dev::grid_insert_kernel, dim3((m + 255) / 256), dim3(256), 0, s, states, n, skip0, skip1, g);
    return hipGetLastError();
}

}  // namespace mpccbf
