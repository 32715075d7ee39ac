// f64_peak.hip — measured f64 vector FMA peak of the part (the denominator of the bench line's
// compute_utilization; MI355X_MICROARCH.md lists only fp32 / bf16 peaks).
// Every lane runs 8 independent v_fma_f64 chains (no dependency stalls), 8 waves per SIMD
// (4 x 256-thread workgroups per CU), 64 x 256 CUs x 4 workgroups; FLOP = 2 per FMA per lane.
// Build: hipcc -O3 --offload-arch=gfx950 tools/dev/f64_peak.hip -o tools/dev/f64_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int CHAINS = 8;

__global__ void __launch_bounds__(256) fma_f64(double* out, int iters, double a, double b) {
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-9 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = fma(x[c], a, b);
    }
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.678) out[blockIdx.x * blockDim.x + threadIdx.x] = s;   // keep the chains live
}

__global__ void __launch_bounds__(256) fma_f32(float* out, int iters, float a, float b) {
    float x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-6f + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = fmaf(x[c], a, b);
    }
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.678f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8, threads = 256, iters = 1 << 16;
    double* d;
    hipMalloc(&d, sizeof(double) * blocks * threads);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(fma_f64, dim3(blocks), dim3(threads), 0, 0, d, iters, 0.999999, 1e-7);
        hipEventRecord(e0);
        hipLaunchKernelGGL(fma_f64, dim3(blocks), dim3(threads), 0, 0, d, iters, 0.999999, 1e-7);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = 2.0 * CHAINS * (double)iters * blocks * threads;
        printf("f64 fma: %.3f ms, %.2f TFLOP/s (%d CUs)\n", ms, flops / (ms * 1e-3) / 1e12, cus);
        hipLaunchKernelGGL(fma_f32, dim3(blocks), dim3(threads), 0, 0, (float*)d, iters, 0.999999f, 1e-7f);
        hipEventRecord(e0);
        hipLaunchKernelGGL(fma_f32, dim3(blocks), dim3(threads), 0, 0, (float*)d, iters, 0.999999f, 1e-7f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("f32 fma: %.3f ms, %.2f TFLOP/s\n", ms, flops / (ms * 1e-3) / 1e12);
    }
    hipFree(d);
    return 0;
}
