// Microbenchmark (diagnostic, not part of the product): cycles per call of the MFMA
// Cholesky's 16x16 diagonal-block factorisation, one wave, no other work on the CU.
#include <cstdio>
#include "../../semi-blind-channel-estimation-for-mimo-ris-communication-system-using-em-algo_amd/csrc/chol.hip"

namespace sbce {
__global__ void ubench_kernel(cd* Rg, unsigned long long* out, int reps, int mode,
                              unsigned long long* clk, cd* Dout, cd* Aout) {
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
        if (mode == 0) factor_diag_lds<false>(A, 16, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        if (mode == 2) factor_diag_lds<false>(A, 16, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16, clk);
        if (mode == 3) factor_diag_lds<true, false>(A, 16, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        if (mode == 6) factor_diag_lds<true, true>(A, 16, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        if (mode == 7) factor_diag_lds<true, true>(A, 13, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        if (mode == 8) factor_diag_lds<true, true, true>(A, 16, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        if (mode == 9) factor_diag_lds<true, true, true>(A, 13, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        if (mode == 4) factor_diag_lds<false>(A, 13, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        if (mode == 5) factor_diag_lds<true, false>(A, 13, lane, 1e-14, 0, Di, dinv, &flag, Rg, 16);
        wave_sync();
        acc += __builtin_amdgcn_s_memtime() - t0;
    }
    if (lane == 0) out[0] = acc / reps;
    for (int e = lane; e < 256; e += 64) { Dout[e] = Di[e]; Aout[e] = A[e]; }
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
    sbce::cd *Dd, *Ad;
    hipMalloc(&Dd, 256 * sizeof(sbce::cd));
    hipMalloc(&Ad, 256 * sizeof(sbce::cd));
    sbce::cd Dh[10][256], Ah[10][256];
    for (int mode = 0; mode < 10; ++mode) {
        hipLaunchKernelGGL(sbce::ubench_kernel, dim3(1), dim3(64), 0, 0, R, o, 50, mode, clk, Dd, Ad);
        unsigned long long h = 0;
        hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost);
        hipMemcpy(Dh[mode], Dd, sizeof(Dh[mode]), hipMemcpyDeviceToHost);
        hipMemcpy(Ah[mode], Ad, sizeof(Ah[mode]), hipMemcpyDeviceToHost);
        printf("mode %d: %llu cycles per call\n", mode, h);
    }
    // the recursive-doubling inverse (modes 3, 5) against the row recurrence (0, 4): max |diff|
    for (int pr = 0; pr < 6; ++pr) {
        const int m1s[6] = {3, 5, 6, 7, 8, 9};
        const int m0 = (pr & 1) ? 4 : 0, m1 = m1s[pr];
        double mx = 0, mag = 0;
        for (int e = 0; e < 256; ++e) {
            const double dx = Dh[m0][e].x - Dh[m1][e].x, dy = Dh[m0][e].y - Dh[m1][e].y;
            mx = fmax(mx, fabs(dx) + fabs(dy));
            mag = fmax(mag, fabs(Dh[m0][e].x) + fabs(Dh[m0][e].y));
        }
        double ma = 0;
        for (int e = 0; e < 256; ++e)
            if ((e & 15) <= (e >> 4) && (e >> 4) < ((pr & 1) ? 13 : 16))     // L's rows < w
                ma = fmax(ma, fabs(Ah[m0][e].x - Ah[m1][e].x) + fabs(Ah[m0][e].y - Ah[m1][e].y));
        printf("modes %d vs %d (w=%d): max |Di diff| = %.3g (max |Di| %.3g), max |L diff| = %.3g\n", m0, m1,
               (pr & 1) ? 13 : 16, mx, mag, ma);
    }
    unsigned long long hc[32];
    hipMemcpy(hc, clk, sizeof(hc), hipMemcpyDeviceToHost);
    printf("per call: column loop %llu (reads+pivot %llu, writes %llu), inverse %llu, R writes %llu\n",
           hc[0] / 50, hc[9] / 50, hc[10] / 50, hc[1] / 50, hc[8] / 50);
    return 0;
}
