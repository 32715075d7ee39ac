// Dev probe: issue rate and dependent latency of v_mfma_f64_16x16x4_f64 on gfx950 (one wave per
// SIMD, operands in registers). Prints cycles per MFMA for 1, 2, 3 and 6 independent accumulators.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NA>
__global__ void __launch_bounds__(256) k(double* out, long long* cyc, int n) {
    d4 acc[NA];
    for (int j = 0; j < NA; ++j) acc[j] = d4{0.0, 0.0, 0.0, 0.0};
    double a = 1.0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-3;
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int j = 0; j < NA; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    }
    const long long t1 = clock64();
    double s = 0.0;
    for (int j = 0; j < NA; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int NA>
void run(double* out, long long* cyc, int n) {
    hipLaunchKernelGGL(k<NA>, dim3(256), dim3(256), 0, 0, out, cyc, n);
    hipDeviceSynchronize();
    long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += h[i];
    m /= 256;
    printf("accumulators %d: %.1f cycles per MFMA (per wave)\n", NA, m / (double)(n * NA));
}
int main() {
    double* out; long long* cyc;
    hipMalloc(&out, sizeof(double) * 65536);
    hipMalloc(&cyc, sizeof(long long) * 256);
    const int n = 4096;
    run<1>(out, cyc, n); run<1>(out, cyc, n);
    run<2>(out, cyc, n);
    run<3>(out, cyc, n);
    run<6>(out, cyc, n);
    return 0;
}
