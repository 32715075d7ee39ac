// rcp_check.hip — accuracy of v_rcp_f64 and of one / two Newton steps on it against the correctly
// rounded 1 / x (the division sequence), in ulps, over 2^22 inputs spread over [2^-20, 2^20].
// Build: hipcc -O3 --offload-arch=gfx950 tools/dev/rcp_check.hip -o tools/dev/rcp_check
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <math.h>

__global__ void k(unsigned long long* out) {   // out[0..2]: max ulp error of raw, 1 NR, 2 NR
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long h = (i + 1) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
    const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);   // [0, 1)
    const double x = exp2(40.0 * u - 20.0);
    const double ref = 1.0 / x;
    double r = __builtin_amdgcn_rcp(x);
    double r1 = fma(r, fma(-x, r, 1.0), r);
    double r2 = fma(r1, fma(-x, r1, 1.0), r1);
    const double v[3] = {r, r1, r2};
    for (int k = 0; k < 3; ++k) {
        const long long d = __builtin_bit_cast(long long, v[k]) - __builtin_bit_cast(long long, ref);
        atomicMax(&out[k], (unsigned long long)(d < 0 ? -d : d));
    }
}

int main() {
    unsigned long long* d;
    (void)hipMalloc(&d, 3 * sizeof(unsigned long long));
    (void)hipMemset(d, 0, 3 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k, dim3(1 << 14), dim3(256), 0, 0, d);
    unsigned long long h[3];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("v_rcp_f64 max ulp error: raw %llu, one Newton step %llu, two Newton steps %llu\n", h[0], h[1], h[2]);
    (void)hipFree(d);
    return 0;
}
