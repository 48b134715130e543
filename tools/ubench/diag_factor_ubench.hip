// Microbenchmark (diagnostic, not part of the product): cycles per call of the MFMA
// Cholesky's 16x16 diagonal-block factorisation, one wave, no other work on the CU.
#include <cstdio>
#include "../../semi-blind-channel-estimation-for-mimo-ris-communication-system-using-em-algo_amd/csrc/chol.hip"

namespace sbce {
__global__ void ubench_kernel(cd* Rg, unsigned long long* out, int reps, int mode,
                              unsigned long long* clk) {
    __shared__ cd A[256], Di[256];
    __shared__ int flag;
    __shared__ double dinv[16];
    const int lane = threadIdx.x;
    unsigned long long acc = 0;
    for (int it = 0; it < reps; ++it) {
        for (int e = lane; e < 256; e += 64) {
            const int r = e / 16, c = e % 16;
            A[e] = (r == c) ? cmk(20.0 + r, 0.0) : cmk(0.1 * (r + 1) / (c + 2), 0.05 * (r - c));
        }
        wave_sync();
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        if (mode == 0) factor_diag_lds(A, 16, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        if (mode == 2) factor_diag_lds(A, 16, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16, clk);
        wave_sync();
        acc += __builtin_amdgcn_s_memtime() - t0;
    }
    if (lane == 0) out[0] = acc / reps;
}
}  // namespace sbce

int main() {
    sbce::cd* R;
    unsigned long long* o;
    hipMalloc(&R, 256 * sizeof(sbce::cd));
    hipMalloc(&o, 8);
    unsigned long long* clk;
    hipMalloc(&clk, 32 * 8);
    hipMemset(clk, 0, 32 * 8);
    for (int mode = 0; mode < 3; ++mode) {
        hipLaunchKernelGGL(sbce::ubench_kernel, dim3(1), dim3(64), 0, 0, R, o, 50, mode, clk);
        unsigned long long h = 0;
        hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost);
        printf("mode %d: %llu cycles per call\n", mode, h);
    }
    unsigned long long hc[32];
    hipMemcpy(hc, clk, sizeof(hc), hipMemcpyDeviceToHost);
    printf("per call: column loop %llu (reads+pivot %llu, writes %llu), inverse %llu, R writes %llu\n",
           hc[0] / 50, hc[9] / 50, hc[10] / 50, hc[1] / 50, hc[8] / 50);
    return 0;
}
