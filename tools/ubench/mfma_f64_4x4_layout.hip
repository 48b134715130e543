// Microbenchmark + layout probe for v_mfma_f64_4x4x4_4b_f64 on gfx950:
//   1. one instruction on random operands; the host finds the lane <-> (block, row, k/col)
//      maps by checking every assignment of the lane's bit pairs;
//   2. throughput with operands that change every iteration (no constant-data power bias),
//      against v_mfma_f64_16x16x4 under the same loop.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/mfma_f64_4x4_layout tools/ubench/mfma_f64_4x4_layout.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>

typedef double d4v __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void probe(const double* a, const double* b, double* d) {
    const int l = threadIdx.x;
    d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 0, 0, 0);
}

// A-block broadcast (CBSZ = 2, ABID = q): four instructions against the 16x16x4 product.
__global__ void probe_bcast(const double* a, const double* b, double* d4, double* d16) {
    const int l = threadIdx.x;
    d4[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, 0, 0);
    d4[64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, 1, 0);
    d4[128 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, 2, 0);
    d4[192 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, 3, 0);
    d4v z = {0, 0, 0, 0};
    d4v r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[l], b[l], z, 0, 0, 0);
    for (int q = 0; q < 4; ++q) d16[64 * q + l] = r[q];
}

// rotate a double by 4 lanes inside each 16-lane row (DPP row_ror:4 on both halves)
__device__ __forceinline__ double ror4(double v) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)u, 0x124, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0x124, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// 16x16x4 product from four 4x4x4_4b instructions, B rotated by one 4-lane block per step
__global__ void probe_rot(const double* a, const double* b, double* d4) {
    const int l = threadIdx.x;
    double bb = b[l];
    for (int m = 0; m < 4; ++m) {
        d4[64 * m + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], bb, 0.0, 0, 0, 0);
        bb = ror4(bb);
    }
}

// throughput: two 16x16x4-equivalents (A = a and a2) per iteration, B rotated by DPP
__global__ __launch_bounds__(256) void tput_rot(const double* in, double* out, int iters) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double a = in[t & 1023], b = in[(t + 511) & 1023], a2 = in[(t + 77) & 1023];
    double acc[8] = {};
    for (int it = 0; it < iters; ++it) {
        const double b1 = ror4(b), b2 = ror4(b1), b3 = ror4(b2);
        acc[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a2, b, acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b1, acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f64_4x4x4f64(a2, b1, acc[3], 0, 0, 0);
        acc[4] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b2, acc[4], 0, 0, 0);
        acc[5] = __builtin_amdgcn_mfma_f64_4x4x4f64(a2, b2, acc[5], 0, 0, 0);
        acc[6] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b3, acc[6], 0, 0, 0);
        acc[7] = __builtin_amdgcn_mfma_f64_4x4x4f64(a2, b3, acc[7], 0, 0, 0);
        a = fma(a, 0.999999, b);
        a2 = fma(a2, 0.999999, b);
        b = fma(b, 1.000001, -a * 1e-3);
    }
    double s = 0;
    for (int u = 0; u < 8; ++u) s += acc[u];
    out[t] = s;
}

template <int KIND>   // 3: 4 x 4x4x4 broadcast (one 16x16x4 equivalent) x 2 accumulator sets
__global__ __launch_bounds__(256) void tput_bc(const double* in, double* out, int iters) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double a = in[t & 1023], b = in[(t + 511) & 1023];
    double acc[8] = {};
    for (int it = 0; it < iters; ++it) {
        acc[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[0], 2, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[1], 2, 1, 0);
        acc[2] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[2], 2, 2, 0);
        acc[3] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[3], 2, 3, 0);
        acc[4] = __builtin_amdgcn_mfma_f64_4x4x4f64(b, a, acc[4], 2, 0, 0);
        acc[5] = __builtin_amdgcn_mfma_f64_4x4x4f64(b, a, acc[5], 2, 1, 0);
        acc[6] = __builtin_amdgcn_mfma_f64_4x4x4f64(b, a, acc[6], 2, 2, 0);
        acc[7] = __builtin_amdgcn_mfma_f64_4x4x4f64(b, a, acc[7], 2, 3, 0);
        a = fma(a, 0.999999, b);
        b = fma(b, 1.000001, -a * 1e-3);
    }
    double s = 0;
    for (int u = 0; u < 8; ++u) s += acc[u];
    out[t] = s;
}

template <int KIND>   // 0: 4x4x4 (8 chains), 1: 16x16x4 (4 chains), 2: 16x16x4 (8 chains)
__global__ __launch_bounds__(256) void tput(const double* in, double* out, int iters) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double a = in[t & 1023], b = in[(t + 511) & 1023];
    double acc[8] = {};
    d4v acc4[8] = {};
    for (int it = 0; it < iters; ++it) {
        if (KIND == 0) {
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[u], 0, 0, 0);
        } else {
#pragma unroll
            for (int u = 0; u < (KIND == 1 ? 4 : 8); ++u)
                acc4[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc4[u], 0, 0, 0);
        }
        a = fma(a, 0.999999, b);      // operands move every iteration
        b = fma(b, 1.000001, -a * 1e-3);
    }
    double s = 0;
    for (int u = 0; u < 8; ++u) s += acc[u];
    for (int u = 0; u < 8; ++u) s += acc4[u][0] + acc4[u][1] + acc4[u][2] + acc4[u][3];
    out[t] = s;
}

static int field(int l, int which, const int* perm) {   // bit pair perm[which] of lane l
    return (l >> (2 * perm[which])) & 3;
}

int main() {
    double ha[64], hb[64], hd[64];
    srand(1);
    for (int i = 0; i < 64; ++i) { ha[i] = rand() / (double)RAND_MAX - 0.5; hb[i] = rand() / (double)RAND_MAX - 0.5; }
    double *da, *db, *dd;
    CK(hipMalloc(&da, 512)); CK(hipMalloc(&db, 512)); CK(hipMalloc(&dd, 512));
    CK(hipMemcpy(da, ha, 512, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb, 512, hipMemcpyHostToDevice));
    probe<<<1, 64>>>(da, db, dd);
    CK(hipMemcpy(hd, dd, 512, hipMemcpyDeviceToHost));
    // fields: A lane -> (blk, row, k); B lane -> (blk, k, col); D lane -> (blk, row, col).
    const int perms[6][3] = {{0,1,2},{0,2,1},{1,0,2},{1,2,0},{2,0,1},{2,1,0}};
    int found = 0;
    for (int pa = 0; pa < 6; ++pa) for (int pb = 0; pb < 6; ++pb) for (int pd = 0; pd < 6; ++pd) {
        double A[4][4][4], B[4][4][4];
        for (int l = 0; l < 64; ++l) {
            A[field(l, 0, perms[pa])][field(l, 1, perms[pa])][field(l, 2, perms[pa])] = ha[l];
            B[field(l, 0, perms[pb])][field(l, 1, perms[pb])][field(l, 2, perms[pb])] = hb[l];
        }
        double err = 0;
        for (int l = 0; l < 64; ++l) {
            int bl = field(l, 0, perms[pd]), i = field(l, 1, perms[pd]), j = field(l, 2, perms[pd]);
            double s = 0;
            for (int k = 0; k < 4; ++k) s += A[bl][i][k] * B[bl][k][j];
            err = fmax(err, fabs(s - hd[l]));
        }
        if (err < 1e-12) {
            printf("match: A (blk,row,k) at lane bit-pairs (%d,%d,%d); B (blk,k,col) at (%d,%d,%d); "
                   "D (blk,row,col) at (%d,%d,%d)\n", perms[pa][0], perms[pa][1], perms[pa][2],
                   perms[pb][0], perms[pb][1], perms[pb][2], perms[pd][0], perms[pd][1], perms[pd][2]);
            ++found;
        }
    }
    if (!found) printf("no layout matched\n");
    {
        double *d4, *d16, h4[256], h16[256];
        CK(hipMalloc(&d4, 2048)); CK(hipMalloc(&d16, 2048));
        probe_bcast<<<1, 64>>>(da, db, d4, d16);
        CK(hipMemcpy(h4, d4, 2048, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h16, d16, 2048, hipMemcpyDeviceToHost));
        double err = 0, mx = 0;
        for (int i = 0; i < 256; ++i) { err = fmax(err, fabs(h4[i] - h16[i])); mx = fmax(mx, fabs(h16[i])); }
        printf("broadcast 4 x 4x4x4 (CBSZ=2, ABID=q) vs 16x16x4 component q: max|diff| %.3e (max %.3e)\n", err, mx);
        double hr[256];
        probe_rot<<<1, 64>>>(da, db, d4);
        CK(hipMemcpy(hr, d4, 2048, hipMemcpyDeviceToHost));
        for (int dir = 0; dir < 2; ++dir) {
            double er = 0;
            for (int m = 0; m < 4; ++m)
                for (int l = 0; l < 64; ++l) {
                    const int blk = (l >> 2) & 3, row = (l >> 4) & 3, col = l & 3;
                    const int bblk = dir ? (blk + m) & 3 : (blk - m) & 3;
                    double c = 0;
                    for (int k = 0; k < 4; ++k) c += ha[row + 4 * blk + 16 * k] * hb[col + 4 * bblk + 16 * k];
                    er = fmax(er, fabs(hr[64 * m + l] - c));
                }
            printf("rotated-B 4x4x4, B block = blk %s m: max err %.3e\n", dir ? "+" : "-", er);
        }
        FILE* f = fopen("gpurun_out/mfma44_dump.txt", "w");
        if (f) {
            for (int i = 0; i < 64; ++i) fprintf(f, "%.17g %.17g\n", ha[i], hb[i]);
            for (int i = 0; i < 256; ++i) fprintf(f, "%.17g %.17g\n", h4[i], h16[i]);
            fclose(f);
        }
        // what does ABID = q compute?  A[blk][row][k] = ha[row + 4 blk + 16 k], B[blk][k][col] = hb[col + 4 blk + 16 k]
        for (int q = 0; q < 4; ++q) {
            double e[3] = {0, 0, 0};
            for (int l = 0; l < 64; ++l) {
                const int blk = (l >> 2) & 3, row = (l >> 4) & 3, col = l & 3;
                double c0 = 0, c1 = 0, c2 = 0;
                for (int k = 0; k < 4; ++k) {
                    c0 += ha[row + 4 * blk + 16 * k] * hb[col + 4 * blk + 16 * k];
                    c1 += ha[row + 4 * q + 16 * k] * hb[col + 4 * blk + 16 * k];
                    c2 += ha[row + 4 * blk + 16 * k] * hb[col + 4 * q + 16 * k];
                }
                e[0] = fmax(e[0], fabs(h4[64 * q + l] - c0));
                e[1] = fmax(e[1], fabs(h4[64 * q + l] - c1));
                e[2] = fmax(e[2], fabs(h4[64 * q + l] - c2));
            }
            printf("ABID=%d: |d - no-bcast| %.2e  |d - A-block q| %.2e  |d - B-block q| %.2e\n", q, e[0], e[1], e[2]);
        }
    }
    double* in; double* out;
    const int blocks = 1024, threads = 256, iters = 4000;
    CK(hipMalloc(&in, 1024 * 8)); CK(hipMalloc(&out, (size_t)blocks * threads * 8));
    double hin[1024];
    for (int i = 0; i < 1024; ++i) hin[i] = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(in, hin, 8192, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int kind = 0; kind < 5; ++kind)
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            if (kind == 0) tput<0><<<blocks, threads>>>(in, out, iters);
            else if (kind == 1) tput<1><<<blocks, threads>>>(in, out, iters);
            else if (kind == 2) tput<2><<<blocks, threads>>>(in, out, iters);
            else if (kind == 3) tput_bc<3><<<blocks, threads>>>(in, out, iters);
            else tput_rot<<<blocks, threads>>>(in, out, iters);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double flops = (double)blocks * threads / 64 * iters * (kind == 0 || kind >= 3 ? 8 * 512.0 : kind == 1 ? 4 * 2048.0 : 8 * 2048.0);
            if (rep) printf("%s: %.3f ms  %.1f TF/s\n", kind == 0 ? "4x4x4_4b x8" : kind == 1 ? "16x16x4 x4" : kind == 2 ? "16x16x4 x8" : kind == 3 ? "4x4x4 bcast x8" : "4x4x4 rotB x8", ms,
                            flops / (ms * 1e-3) / 1e12);
        }
    return 0;
}
