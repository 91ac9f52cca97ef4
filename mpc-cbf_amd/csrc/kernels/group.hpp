// group.hpp — lane-group collectives for gfx950 (wave64).
//
// One QP is owned by a group of G lanes (G in {16, 32, 64}; G divides the 64-lane wavefront,
// so a group never straddles waves). Rows of the QP are spread over the group's lanes; the
// reductions below combine per-lane partials across the group.
//
// Within a 16-lane DPP row the butterfly uses DPP lane moves (no LDS traffic):
//   quad_perm [1,0,3,2]  (xor 1)      quad_perm [2,3,0,1]  (xor 2)
//   row_half_mirror      (i <-> 7-i)  row_mirror           (i <-> 15-i)
// after the two quad stages every lane of a quad holds the quad total, so the mirrors pair each
// lane with a lane of the other quad / other half-row, which is all an all-reduce needs.
// Stages across 16-lane rows (G = 32, 64) use v_permlane16_swap / v_permlane32_swap (VALU lane
// swaps, no LDS round trip; bit-identical to the lane-xor exchange since the combines commute).
#pragma once

#include <hip/hip_runtime.h>

namespace mpccbf {
namespace dev {

// threadIdx.x & M as a value the compiler cannot see through: lane masks derived from it are
// formed inside each solve instead of hoisted out of the callers' loops, where they stay live
// across everything and spill
template <int M>
__device__ __forceinline__ int lane_bits_opaque() {
    int r;
    asm volatile("v_and_b32 %0, %1, %2" : "=v"(r) : "i"(M), "v"((int)threadIdx.x));
    return r;
}

// A pointer into this block's LDS (a __shared__ array reached through a generic pointer) as a
// volatile LDS-address-space pointer: reads and writes through it are ds_read / ds_write, never
// re-used from registers. (A volatile generic pointer compiles to flat accesses with the
// system-coherence bits, whose waits also wait for every global load in flight.)
template <class T>
using lds_vptr = volatile __attribute__((address_space(3))) T*;
template <class T>
__device__ __forceinline__ lds_vptr<T> lds_vol(T* p) {
    return (lds_vptr<T>)p;
}

constexpr int DPP_XOR1 = 0xB1;         // quad_perm(1,0,3,2)
constexpr int DPP_XOR2 = 0x4E;         // quad_perm(2,3,0,1)
constexpr int DPP_HALF_MIRROR = 0x141; // row_half_mirror
constexpr int DPP_MIRROR = 0x140;      // row_mirror

// Every control used here reads a lane of the same 16-lane row that always exists, so the
// "old" operand is never observed: mov_dpp (old = undef, bound_ctrl) lets the compiler skip
// materialising a zero register per move.
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    const long long b = __double_as_longlong(v);
    return __longlong_as_double(__builtin_amdgcn_mov_dpp(b, CTRL, 0xF, 0xF, true));
}

__device__ __forceinline__ double mk_double(unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// the other 16-lane row's value of v (S32 false: rows 0<->1, 2<->3; true: rows 0,1 <-> 2,3) as
// the pair {own, partner} in lane-dependent order (the ops applied to it are commutative)
template <bool S32>
__device__ __forceinline__ void row_pair(double v, double& a, double& b) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    if constexpr (S32) {
        const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        a = mk_double(l[0], h[0]);
        b = mk_double(l[1], h[1]);
    } else {
        const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        a = mk_double(l[0], h[0]);
        b = mk_double(l[1], h[1]);
    }
}

// 64-lane max of a 32-bit unsigned key (every lane ends with it): DPP row stages folded into
// v_max_u32, then the permlane16 / permlane32 swaps across the 16-lane rows. The candidate rule's
// normalised violations are non-negative and reduced as float bit patterns (a violated side has a
// positive score; the key is 0 when no side is violated), a third of the instructions of the f64
// max (no NaN canonicalisation, one register instead of two).
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
// max over a 16-lane row (every lane ends with it): DPP moves fused into v_max_u32
__device__ __forceinline__ unsigned row_max_u32(unsigned v) {
    v = max(v, dpp_u32<DPP_XOR1>(v));
    v = max(v, dpp_u32<DPP_XOR2>(v));
    v = max(v, dpp_u32<DPP_HALF_MIRROR>(v));
    v = max(v, dpp_u32<DPP_MIRROR>(v));
    return v;
}

__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
    v = max(v, dpp_u32<DPP_XOR1>(v));
    v = max(v, dpp_u32<DPP_XOR2>(v));
    v = max(v, dpp_u32<DPP_HALF_MIRROR>(v));
    v = max(v, dpp_u32<DPP_MIRROR>(v));
    {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = max(r[0], r[1]);
    }
    {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        v = max(r[0], r[1]);
    }
    return v;
}

// lane l's double as a wave-uniform (scalar) value
__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)lo);
}

enum class Op { Sum, Max, Min };

template <Op OP>
__device__ __forceinline__ double combine(double a, double b) {
    if constexpr (OP == Op::Sum) return a + b;
    else if constexpr (OP == Op::Max) return fmax(a, b);
    else return fmin(a, b);
}

template <int G, Op OP>
__device__ __forceinline__ double grp_reduce(double v) {
    static_assert(G == 16 || G == 32 || G == 64, "group size");
    v = combine<OP>(v, dpp_mov<DPP_XOR1>(v));
    v = combine<OP>(v, dpp_mov<DPP_XOR2>(v));
    v = combine<OP>(v, dpp_mov<DPP_HALF_MIRROR>(v));
    v = combine<OP>(v, dpp_mov<DPP_MIRROR>(v));
    double a, b;
    if constexpr (G >= 32) {
        row_pair<false>(v, a, b);
        v = combine<OP>(a, b);
    }
    if constexpr (G >= 64) {
        row_pair<true>(v, a, b);
        v = combine<OP>(a, b);
    }
    return v;
}

template <int G> __device__ __forceinline__ double grp_sum(double v) { return grp_reduce<G, Op::Sum>(v); }
template <int G> __device__ __forceinline__ double grp_max(double v) { return grp_reduce<G, Op::Max>(v); }
template <int G> __device__ __forceinline__ double grp_min(double v) { return grp_reduce<G, Op::Min>(v); }

// In-place all-reduce (sum) of N values: every lane of the group ends with the totals.
// Stage-major so the N independent exchanges of a stage overlap.
template <int G, int N>
__device__ __forceinline__ void grp_sum_vec(double (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += dpp_mov<DPP_XOR1>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += dpp_mov<DPP_XOR2>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += dpp_mov<DPP_HALF_MIRROR>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += dpp_mov<DPP_MIRROR>(v[i]);
    double a, b;
    if constexpr (G >= 32) {
#pragma unroll
        for (int i = 0; i < N; i++) {
            row_pair<false>(v[i], a, b);
            v[i] = a + b;
        }
    }
    if constexpr (G >= 64) {
#pragma unroll
        for (int i = 0; i < N; i++) {
            row_pair<true>(v[i], a, b);
            v[i] = a + b;
        }
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

// Fast FP64 reciprocal: v_rcp_f64 refined by two Newton steps (full precision for the normal
// range; the PDIP never divides by zero: slacks are clamped >= 1e-300).
__device__ __forceinline__ double rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    r = fma(fma(-x, r, 1.0), r, r);
    return r;
}

// Raw v_rcp_f64 (unrefined hardware estimate): only for step-length ratios, where the
// fraction-to-boundary factor 0.99 absorbs its error.
__device__ __forceinline__ double rcp_fast(double x) { return __builtin_amdgcn_rcp(x); }

// Two independent group max-reductions, stage-interleaved.
template <int G>
__device__ __forceinline__ void grp_max2(double& a, double& b) {
    static_assert(G == 16, "grp_max2: 16-lane groups");
    a = fmax(a, dpp_mov<DPP_XOR1>(a));
    b = fmax(b, dpp_mov<DPP_XOR1>(b));
    a = fmax(a, dpp_mov<DPP_XOR2>(a));
    b = fmax(b, dpp_mov<DPP_XOR2>(b));
    a = fmax(a, dpp_mov<DPP_HALF_MIRROR>(a));
    b = fmax(b, dpp_mov<DPP_HALF_MIRROR>(b));
    a = fmax(a, dpp_mov<DPP_MIRROR>(a));
    b = fmax(b, dpp_mov<DPP_MIRROR>(b));
}

// Make this wave's LDS writes visible to its other lanes before they read them.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Diagnostics build (make poison): every kernel that calls this fills its block's static LDS with
// MPCCBF_LDS_POISON (NaN with MPCCBF_LDS_POISON_NAN) before any other work, so builds with
// different fill values give
// bit-identical results unless something reads LDS it never wrote (tools/lds_poison_check.py).
__device__ __forceinline__ void lds_poison() {
#ifdef MPCCBF_LDS_POISON
    const unsigned n = __builtin_amdgcn_groupstaticsize() / 8;
#ifdef MPCCBF_LDS_POISON_NAN  // a quiet NaN: also exposes unwritten LDS that is multiplied by 0
    const double v = __builtin_nan("");
#else
    const double v = MPCCBF_LDS_POISON;
#endif
    for (unsigned e = threadIdx.x; e < n; e += blockDim.x) {
        const unsigned addr = e * 8;
        asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
#endif
}

// Value of lane k (0..15) of this lane's 16-lane row (DPP row_newbcast; k folds to a constant
// after unrolling).
template <int K>
__device__ __forceinline__ double row_bcast_k(double v) {
    return dpp_mov<0x150 + K>(v);
}
__device__ __forceinline__ double row_bcast(int k, double v) {
    switch (k & 15) {
        case 0: return row_bcast_k<0>(v);
        case 1: return row_bcast_k<1>(v);
        case 2: return row_bcast_k<2>(v);
        case 3: return row_bcast_k<3>(v);
        case 4: return row_bcast_k<4>(v);
        case 5: return row_bcast_k<5>(v);
        case 6: return row_bcast_k<6>(v);
        case 7: return row_bcast_k<7>(v);
        case 8: return row_bcast_k<8>(v);
        case 9: return row_bcast_k<9>(v);
        case 10: return row_bcast_k<10>(v);
        case 11: return row_bcast_k<11>(v);
        case 12: return row_bcast_k<12>(v);
        case 13: return row_bcast_k<13>(v);
        case 14: return row_bcast_k<14>(v);
        default: return row_bcast_k<15>(v);
    }
}

// The same all-reduce through LDS (16-lane groups of one wave, G = 16): every lane writes its N
// values as one row of a padded 16 x (N + 1) table (odd row stride: the column reads hit distinct
// banks), lane c sums column c (and c + 16), and the totals return by DPP row broadcasts. One LDS
// round trip plus N broadcasts against the 4N DPP moves and adds of grp_sum_vec.
// red: per-group scratch of 16 * (N + 1) doubles, private to the group.
template <int N>
__device__ __forceinline__ void grp_sum_vec_lds(double (&v)[N], double* __restrict__ red, int gl) {
    static_assert(N <= 32, "two columns per lane at most");
    constexpr int S = N + 1;
#pragma unroll
    for (int k = 0; k < N; k++) red[gl * S + k] = v[k];
    wave_lds_sync();
    double col[2] = {0.0, 0.0};
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int c = 16 * h + gl;
        if (16 * h < N && c < N) {
            double p[16];
#pragma unroll
            for (int l = 0; l < 16; l++) p[l] = red[l * S + c];
#pragma unroll
            for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
                for (int l = 0; l < w; l++) p[l] += p[l + w];
            col[h] = p[0];
        }
    }
#pragma unroll
    for (int k = 0; k < N; k++) v[k] = row_bcast(k, col[k >> 4]);
    wave_lds_sync();  // the table is reused by the next reduction
}

}  // namespace dev
}  // namespace mpccbf
