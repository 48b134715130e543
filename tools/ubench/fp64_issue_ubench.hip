// Microbenchmark: issue cost of v_mfma_f64_16x16x4_f64 and of FP64 VALU FMA on gfx950,
// alone and interleaved across waves (does the matrix core run beside the VALU?).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/fp64_issue_ubench tools/ubench/fp64_issue_ubench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4v __attribute__((ext_vector_type(4)));

template <int MODE>   // 0: MFMA only, 1: VALU only, 2: even waves MFMA, odd waves VALU,
                      // 3: v_mfma_f64_4x4x4 (4 blocks) only
__global__ __launch_bounds__(256) void kern(double* out, int iters) {
    const int wave = threadIdx.x >> 6;
    d4v acc[4] = {};
    double v[8];
    for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * 1e-3 + i;
    const double a = 1.0000001, b = threadIdx.x * 1e-7;
    double acc4[8] = {};
    const bool do_mfma = MODE == 0 || (MODE == 2 && !(wave & 1));
    const bool do_valu = MODE == 1 || (MODE == 2 && (wave & 1));
    for (int it = 0; it < iters; ++it) {
        if (do_mfma) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u], 0, 0, 0);
        }
        if (MODE == 3) {
#pragma unroll
            for (int u = 0; u < 8; ++u) acc4[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc4[u], 0, 0, 0);
        }
        if (do_valu) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = fma(v[i], a, b);
        }
    }
    double s = 0;
    for (int u = 0; u < 4; ++u) s += acc[u][0] + acc[u][1] + acc[u][2] + acc[u][3];
    for (int i = 0; i < 8; ++i) s += v[i] + acc4[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 4, threads = 256, iters = 4000;
    double* d;
    hipMalloc(&d, sizeof(double) * blocks * threads);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[4] = {"mfma only (4 MFMA/iter/wave)", "valu only (128 FMA/iter/wave)",
                            "half waves each", "mfma 4x4x4 only (8/iter/wave)"};
    for (int m = 0; m < 4; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (m == 0) kern<0><<<blocks, threads>>>(d, iters);
            if (m == 1) kern<1><<<blocks, threads>>>(d, iters);
            if (m == 2) kern<2><<<blocks, threads>>>(d, iters);
            if (m == 3) kern<3><<<blocks, threads>>>(d, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double waves = (double)blocks * threads / 64;
            // per SIMD: waves/1024 waves, each iters iterations
            const double per_simd_iters = waves / 1024.0 * iters;
            if (rep) printf("%-32s %8.3f ms  %8.1f ns per SIMD-iteration\n", names[m], ms,
                            ms * 1e6 / per_simd_iters);
        }
    }
    hipFree(d);
    return 0;
}
