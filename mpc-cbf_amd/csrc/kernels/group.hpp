// group.hpp — lane-group collectives for gfx950 (wave64).
//
// One QP is owned by a group of G lanes (G in {16, 32, 64}; G divides the 64-lane wavefront,
// so a group never straddles waves). Rows of the QP are spread over the group's lanes; the
// reductions below combine per-lane partials across the group with butterfly exchanges.
#pragma once

#include <hip/hip_runtime.h>

namespace mpccbf {
namespace dev {

template <int G>
__device__ __forceinline__ double grp_sum(double v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, G);
    return v;
}

template <int G>
__device__ __forceinline__ double grp_max(double v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, G));
    return v;
}

template <int G>
__device__ __forceinline__ double grp_min(double v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, G));
    return v;
}

// In-place all-reduce (sum) of N values: every lane of the group ends with the totals.
// Independent exchanges are issued back to back so their latencies overlap.
template <int G, int N>
__device__ __forceinline__ void grp_sum_vec(double (&v)[N]) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
#pragma unroll
        for (int i = 0; i < N; i++) v[i] += __shfl_xor(v[i], o, G);
    }
}

// Group-local ballot: bit l set if lane l of this group has pred true.
template <int G>
__device__ __forceinline__ unsigned long long grp_ballot(bool pred) {
    const unsigned long long all = __ballot(pred);
    const int base = (threadIdx.x & 63) & ~(G - 1);
    if constexpr (G == 64)
        return all;
    else
        return (all >> base) & ((1ull << G) - 1ull);
}

template <int G>
__device__ __forceinline__ int grp_lane() {
    return threadIdx.x & (G - 1);
}

// Make this wave's LDS writes visible to its other lanes before they read them.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace dev
}  // namespace mpccbf
