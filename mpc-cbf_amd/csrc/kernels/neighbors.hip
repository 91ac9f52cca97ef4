// neighbors.hip — neighbour lists for the batched IMPC step.
//
// The reference hands every other robot to the controller (ConnectivityIMPCCBF.cpp:59-67);
// `all` mode reproduces that. `knn` mode keeps the k nearest (planar) within a radius using a
// spatial hash of uniform cells (cell edge = radius): count -> scan -> scatter -> 3x3-cell
// query. Output rows are sorted by neighbour index so results do not depend on hash order.
#include <hip/hip_runtime.h>

#include <cstdint>

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

// Spatial hash of all agents in ONE workgroup (n <= 32768): LDS histogram -> block scan ->
// scatter. One launch instead of count/scan/scatter; bucket order inside a cell follows LDS
// atomic order (the consumer orders neighbours by index, so results do not depend on it).
// Each thread keeps the bucket and in-bucket offset of its (up to GB_PER) agents in registers
// between the passes; the bucket scan is a per-thread serial sum, a wave-level DPP/shuffle scan
// and one scan of the 16 wave totals (3 barriers instead of a 1024-wide Hillis-Steele).
constexpr int GB_THREADS = 1024;
constexpr int GB_PER = 32;  // agents per thread: n <= 32768

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

__global__ void __launch_bounds__(GB_THREADS) grid_build_kernel(const double* __restrict__ st, int n,
                                                                double inv, uint32_t T, uint32_t* start,
                                                                uint32_t* sorted) {
    extern __shared__ uint32_t cnt[];  // T buckets
    __shared__ uint32_t wsum[GB_THREADS / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (uint32_t i = tid; i < T; i += GB_THREADS) cnt[i] = 0u;
    __syncthreads();
    uint32_t h[GB_PER], off[GB_PER];
#pragma unroll
    for (int k = 0; k < GB_PER; k++) {
        const int i = tid + k * GB_THREADS;
        if (i < n) {
            const long long cx = (long long)floor(st[(size_t)i * 6] * inv);
            const long long cy = (long long)floor(st[(size_t)i * 6 + 1] * inv);
            h[k] = cell_hash(cx, cy, T - 1);
            off[k] = atomicAdd(&cnt[h[k]], 1u);
        }
    }
    __syncthreads();
    // exclusive scan of cnt: thread t owns buckets [t*per, (t+1)*per)
    const uint32_t per = T / GB_THREADS, b = tid * per;
    uint32_t s = 0;
    for (uint32_t i = 0; i < per; i++) s += cnt[b + i];
    const uint32_t incl = wave_incl_scan(s, lane);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    if (wid == 0) {
        const uint32_t w = lane < GB_THREADS / 64 ? wsum[lane] : 0u;
        const uint32_t wi = wave_incl_scan(w, lane);
        if (lane < GB_THREADS / 64) wsum[lane] = wi - w;  // exclusive wave offsets
        if (lane == GB_THREADS / 64 - 1) start[T] = wi;
    }
    __syncthreads();
    uint32_t run = wsum[wid] + incl - s;
    for (uint32_t i = 0; i < per; i++) {
        const uint32_t c = cnt[b + i];
        cnt[b + i] = run;
        start[b + i] = run;
        run += c;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GB_PER; k++) {
        const int i = tid + k * GB_THREADS;
        if (i < n) sorted[cnt[h[k]] + off[k]] = (uint32_t)i;
    }
}

// Large tables (the multi-GPU bench gathers 8 x 4096 = 32768 states per rank: the single
// workgroup above needs ~68 us there): count (global atomics, one thread per agent, the bucket
// and in-bucket offset kept in scratch) -> one-workgroup scan of the T bucket counts -> scatter.
constexpr int GB_MULTI_MIN = 8192;  // n above which the three-kernel build is used

__global__ void __launch_bounds__(256) grid_count_kernel(const double* __restrict__ st, int n, double inv,
                                                         uint32_t T, uint32_t* __restrict__ gcnt,
                                                         uint32_t* __restrict__ hb, uint32_t* __restrict__ ob) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const long long cx = (long long)floor(st[(size_t)i * 6] * inv);
    const long long cy = (long long)floor(st[(size_t)i * 6 + 1] * inv);
    const uint32_t h = cell_hash(cx, cy, T - 1);
    hb[i] = h;
    ob[i] = atomicAdd(&gcnt[h], 1u);
}

// Exclusive scan of the T bucket counts in one workgroup: a coalesced copy into LDS (padded by
// one word per 32 so that thread t's contiguous run of T/1024 buckets is bank-conflict free), a
// per-thread serial sum, wave / block scans of the 1024 partial sums, a per-thread serial
// rewrite in LDS and a coalesced copy out.
__device__ __forceinline__ uint32_t pad32(uint32_t j) { return j + (j >> 5); }

__global__ void __launch_bounds__(GB_THREADS) grid_scan_kernel(uint32_t* __restrict__ gcnt, uint32_t T,
                                                                uint32_t* __restrict__ start) {
    extern __shared__ uint32_t lc[];  // pad32(T) words
    __shared__ uint32_t wsum[GB_THREADS / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (uint32_t j = tid; j < T; j += GB_THREADS) {
        lc[pad32(j)] = gcnt[j];
        gcnt[j] = 0u;  // ready for the next build with the same layout (no memset then)
    }
    __syncthreads();
    const uint32_t per = T / GB_THREADS, b = tid * per;  // T: power of two >= 1024
    uint32_t s = 0;
    for (uint32_t i = 0; i < per; i++) s += lc[pad32(b + i)];
    const uint32_t incl = wave_incl_scan(s, lane);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    if (wid == 0) {
        const uint32_t w = lane < GB_THREADS / 64 ? wsum[lane] : 0u;
        const uint32_t wi = wave_incl_scan(w, lane);
        if (lane < GB_THREADS / 64) wsum[lane] = wi - w;
        if (lane == GB_THREADS / 64 - 1) start[T] = wi;
    }
    __syncthreads();
    uint32_t run = wsum[wid] + incl - s;
    for (uint32_t i = 0; i < per; i++) {
        const uint32_t c = lc[pad32(b + i)];
        lc[pad32(b + i)] = run;
        run += c;
    }
    __syncthreads();
    for (uint32_t j = tid; j < T; j += GB_THREADS) start[j] = lc[pad32(j)];
}

__global__ void __launch_bounds__(256) grid_scatter_kernel(int n, const uint32_t* __restrict__ start,
                                                           const uint32_t* __restrict__ hb,
                                                           const uint32_t* __restrict__ ob,
                                                           uint32_t* __restrict__ sorted) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    sorted[start[hb[i]] + ob[i]] = (uint32_t)i;
}

}  // namespace dev

static size_t al256(size_t b) { return (b + 255) / 256 * 256; }

size_t grid_scratch_bytes(int num_states) {
    const uint32_t T = grid_table_size(num_states);
    // start (T+1) | sorted (n) [| counts (T) | bucket (n) | offset (n) for the multi-kernel build]
    size_t b = al256((size_t)(T + 1) * 4) + al256((size_t)num_states * 4);
    if (num_states > dev::GB_MULTI_MIN) b += al256((size_t)T * 4) + 2 * al256((size_t)num_states * 4);
    return b;
}

// start (T+1) | sorted (n) | slot_off (n) carved from scratch; returns T or 0 on error
uint32_t launch_grid_build(const double* states, int n, double radius, void* scratch,
                           uint32_t** start, uint32_t** sorted, hipStream_t s, bool clear_counts) {
    const uint32_t T = grid_table_size(n);
    if (T > 32768 || n > dev::GB_THREADS * dev::GB_PER) return 0;  // single-workgroup limits
    char* p = (char*)scratch;
    *start = (uint32_t*)p;
    p += al256((size_t)(T + 1) * 4);
    *sorted = (uint32_t*)p;
    p += al256((size_t)n * 4);
    if (n > dev::GB_MULTI_MIN) {
        uint32_t* gcnt = (uint32_t*)p;
        p += al256((size_t)T * 4);
        uint32_t* hb = (uint32_t*)p;
        p += al256((size_t)n * 4);
        uint32_t* ob = (uint32_t*)p;
        // the scan kernel leaves the counts zeroed: the caller asks for a clear only when this
        // scratch was not used with the same n by the previous build
        if (clear_counts && hipMemsetAsync(gcnt, 0, (size_t)T * 4, s) != hipSuccess) return 0;
        const int blocks = (n + 255) / 256;
        hipLaunchKernelGGL(dev::grid_count_kernel, dim3(blocks), dim3(256), 0, s, states, n, 1.0 / radius, T,
                           gcnt, hb, ob);
        static bool scan_attr = false;  // > 64 KiB of dynamic LDS needs an opt-in
        if (!scan_attr) {
            if (hipFuncSetAttribute((const void*)dev::grid_scan_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (32768 + 1024) * 4) != hipSuccess)
                return 0;
            scan_attr = true;
        }
        hipLaunchKernelGGL(dev::grid_scan_kernel, dim3(1), dim3(dev::GB_THREADS), (size_t)(T + T / 32) * 4, s,
                           gcnt, T, *start);
        hipLaunchKernelGGL(dev::grid_scatter_kernel, dim3(blocks), dim3(256), 0, s, n, *start, hb, ob, *sorted);
        return hipGetLastError() == hipSuccess ? T : 0;
    }
    static bool attr_set = false;  // > 64 KiB of dynamic LDS needs an opt-in (gfx950: 160 KiB/CU)
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)dev::grid_build_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 32768 * 4) != hipSuccess)
            return 0;
        attr_set = true;
    }
    hipLaunchKernelGGL(dev::grid_build_kernel, dim3(1), dim3(dev::GB_THREADS), (size_t)T * 4, s, states,
                       n, 1.0 / radius, T, *start, *sorted);
    return hipGetLastError() == hipSuccess ? T : 0;
}

}  // namespace mpccbf
