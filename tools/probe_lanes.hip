// probe_lanes.hip — checks, on the GPU, the cross-lane primitives the FoV kernel relies on:
//   v_permlane16_swap / v_permlane32_swap pair sums, DPP row_newbcast on 64-bit values, and the
//   lane layout of v_mfma_f64_16x16x4_f64 (A[l&15][l>>4], B[l>>4][l&15],
//   D[row (l>>4) + 4 i][col l&15]) with exact integer data.
// Build: hipcc -O2 --offload-arch=gfx950 tools/probe_lanes.hip -o mpc-cbf_amd/build/probe_lanes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void probe(const double* in, double* out_sw16, double* out_sw32, double* out_bc, double* out_mfma) {
    const int l = threadIdx.x;
    const double v = in[l];
    const unsigned lo = (unsigned)(__double_as_longlong(v) & 0xffffffffull);
    const unsigned hi = (unsigned)(__double_as_longlong(v) >> 32);
    {
        auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        const double x0 = __longlong_as_double(((long long)b[0] << 32) | a[0]);
        const double x1 = __longlong_as_double(((long long)b[1] << 32) | a[1]);
        out_sw16[l] = x0 + x1;
    }
    {
        auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        const double x0 = __longlong_as_double(((long long)b[0] << 32) | a[0]);
        const double x1 = __longlong_as_double(((long long)b[1] << 32) | a[1]);
        out_sw32[l] = x0 + x1;
    }
    {
        const long long bits = __double_as_longlong(v);
        out_bc[l] = __longlong_as_double(__builtin_amdgcn_mov_dpp(bits, 0x150 + 5, 0xF, 0xF, true));  // row_newbcast:5
    }
    {
        // A[i][k] = i + 16 k + 1, B[k][j] = 3 k - j + 2
        const double a = (double)((l & 15) + 16 * (l >> 4) + 1);
        const double b = (double)(3 * (l >> 4) - (l & 15) + 2);
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        for (int i = 0; i < 4; i++) out_mfma[l * 4 + i] = acc[i];
    }
}

int main() {
    double h_in[64], h16[64], h32[64], hbc[64], hm[256];
    for (int i = 0; i < 64; i++) h_in[i] = (double)(i * i + 1);
    double *d_in, *d16, *d32, *dbc, *dm;
    (void)hipMalloc(&d_in, sizeof(h_in));
    (void)hipMalloc(&d16, sizeof(h16));
    (void)hipMalloc(&d32, sizeof(h32));
    (void)hipMalloc(&dbc, sizeof(hbc));
    (void)hipMalloc(&dm, sizeof(hm));
    (void)hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_in, d16, d32, dbc, dm);
    (void)hipMemcpy(h16, d16, sizeof(h16), hipMemcpyDeviceToHost);
    (void)hipMemcpy(h32, d32, sizeof(h32), hipMemcpyDeviceToHost);
    (void)hipMemcpy(hbc, dbc, sizeof(hbc), hipMemcpyDeviceToHost);
    (void)hipMemcpy(hm, dm, sizeof(hm), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++) {
        const int r = l >> 4, p = l & 15;
        const double e16 = h_in[((r ^ 1) << 4) | p] + h_in[l];
        const double e32 = h_in[l ^ 32] + h_in[l];
        const double ebc = h_in[(r << 4) | 5];
        if (h16[l] != e16) { bad++; printf("sw16 lane %d got %g want %g\n", l, h16[l], e16); }
        if (h32[l] != e32) { bad++; printf("sw32 lane %d got %g want %g\n", l, h32[l], e32); }
        if (hbc[l] != ebc) { bad++; printf("bcast lane %d got %g want %g\n", l, hbc[l], ebc); }
        for (int i = 0; i < 4; i++) {
            const int row = r + 4 * i, col = p;
            double e = 0;
            for (int k = 0; k < 4; k++) e += (double)(row + 16 * k + 1) * (double)(3 * k - col + 2);
            if (hm[l * 4 + i] != e) { bad++; printf("mfma lane %d i %d got %g want %g\n", l, i, hm[l * 4 + i], e); }
        }
    }
    printf("probe_lanes: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    return bad ? 1 : 0;
}
