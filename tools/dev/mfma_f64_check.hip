// Dev check (not product code): operand / result layout of v_mfma_f64_16x16x4_f64 on gfx950.
// Measured on MI355X (ROCm 7.2): A[16x4]: lane l holds A[l%16][l/16]; B[4x16]: lane l holds
// B[l/16][l%16]; D[16x16]: register r (0..3) of lane l holds D[l/16 + 4r][l%16] (row-interleaved).
// The check prints, for lanes 0/1 of each 16-lane group, which D entry each register holds.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* D) {
    int l = threadIdx.x;
    double a = A[(l % 16) * 4 + l / 16];
    double b = B[(l / 16) * 16 + l % 16];
    d4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];   // raw: lane-major
}
int main() {
    double hA[64], hB[64], hD[256], ref[256];
    for (int i = 0; i < 64; ++i) { hA[i] = sin(1.0 + i) ; hB[i] = cos(2.0 + 3 * i); }
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { double s = 0; for (int q = 0; q < 4; ++q) s += hA[i * 4 + q] * hB[q * 16 + j]; ref[i * 16 + j] = s; }
    double *dA, *dB, *dD;
    hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 2048);
    hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
    // find, for every raw (lane, r), the (i, j) of ref it equals
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
        int hit = -1; for (int q = 0; q < 256; ++q) if (fabs(hD[l * 4 + r] - ref[q]) < 1e-12) hit = q;
        if (l % 16 == 0 || l % 16 == 1 || hit < 0) printf("lane %d r %d -> i %d j %d\n", l, r, hit / 16, hit % 16);
        if (hit < 0) bad = 1;
    }
    double e = bad;
    printf("mfma_f64_16x16x4 layout check: max err %.3e %s\n", e, e < 1e-12 ? "OK" : "MISMATCH");
    return e < 1e-12 ? 0 : 1;
}
