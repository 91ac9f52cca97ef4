// Launch-overhead microbenchmark (diagnostic, not part of the library): back-to-back launches of
// near-empty kernels shaped like the IMPC kernel (256 blocks x 256 threads) with different LDS
// and register footprints, timed with HIP events over many launches. Tells how much of the IMPC
// launch (~37 us, agent span ~26 us) is dispatch / drain rather than the agents' own work.
//   hipcc --offload-arch=gfx950 -O3 tools/launch_overhead.hip -o build/launch_overhead
#include <hip/hip_runtime.h>

#include <cstdio>

template <int LDS_DOUBLES>
__global__ void __launch_bounds__(256) k_lds(double* out, int n) {
    __shared__ double s[LDS_DOUBLES > 0 ? LDS_DOUBLES : 1];
    const int t = threadIdx.x;
    if (LDS_DOUBLES > 0) s[t % (LDS_DOUBLES > 0 ? LDS_DOUBLES : 1)] = t;
    __syncthreads();
    if (blockIdx.x * 256 + t == n) out[0] = LDS_DOUBLES > 0 ? s[0] : 0.0;  // never true: keeps s
}

// many live VGPRs / AGPRs (forces a high allocation) — values kept opaque through asm
template <int NV>
__global__ void __launch_bounds__(256) k_regs(double* out, int n) {
    double v[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) {
        v[i] = (double)(threadIdx.x + i);
        asm volatile("" : "+v"(v[i]));
    }
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NV; i++) acc += v[i];
    if (blockIdx.x * 256 + threadIdx.x == n) out[0] = acc;
}

template <typename F>
float time_launches(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 20; i++) launch();
    hipEventRecord(a, nullptr);
    for (int i = 0; i < reps; i++) launch();
    hipEventRecord(b, nullptr);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return 1e3f * ms / reps;
}

int main() {
    double* out;
    if (hipMalloc(&out, 8) != hipSuccess) return 1;
    const int reps = 2000, n = -1;
    const dim3 g(256), b(256);
    printf("empty, no LDS:          %.2f us\n", time_launches([&] { hipLaunchKernelGGL(k_lds<0>, g, b, 0, nullptr, out, n); }, reps));
    printf("LDS 32 KB:              %.2f us\n", time_launches([&] { hipLaunchKernelGGL(k_lds<4096>, g, b, 0, nullptr, out, n); }, reps));
    printf("LDS 80 KB:              %.2f us\n", time_launches([&] { hipLaunchKernelGGL(k_lds<10240>, g, b, 0, nullptr, out, n); }, reps));
    printf("LDS 140 KB:             %.2f us\n", time_launches([&] { hipLaunchKernelGGL(k_lds<17920>, g, b, 0, nullptr, out, n); }, reps));
    printf("~128 VGPR:              %.2f us\n", time_launches([&] { hipLaunchKernelGGL(k_regs<60>, g, b, 0, nullptr, out, n); }, reps));
    printf("~256 VGPR:              %.2f us\n", time_launches([&] { hipLaunchKernelGGL(k_regs<124>, g, b, 0, nullptr, out, n); }, reps));
    printf("~512 VGPR+AGPR:         %.2f us\n", time_launches([&] { hipLaunchKernelGGL(k_regs<250>, g, b, 0, nullptr, out, n); }, reps));
    printf("1024 blocks x 64, none: %.2f us\n", time_launches([&] { hipLaunchKernelGGL(k_lds<0>, dim3(1024), dim3(64), 0, nullptr, out, n); }, reps));
    hipFree(out);
    return 0;
}
