// Dev check (run on the GPU box): semantics of v_permlane32_swap / v_permlane16_swap and the
// DPP mirror moves used by the solver's wave reductions. Prints per-op lane maps.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
    const int l = threadIdx.x;
    const int a = l, b = 100 + l;
    auto p32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    auto p16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[0 * 64 + l] = p32[0];
    out[1 * 64 + l] = p32[1];
    out[2 * 64 + l] = p16[0];
    out[3 * 64 + l] = p16[1];
    out[4 * 64 + l] = __builtin_amdgcn_update_dpp(0, a, 0x140, 0xf, 0xf, false);   // row_mirror
    out[5 * 64 + l] = __builtin_amdgcn_update_dpp(0, a, 0x141, 0xf, 0xf, false);   // row_half_mirror
    out[6 * 64 + l] = __builtin_amdgcn_update_dpp(0, a, 0x4e, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
    out[7 * 64 + l] = __builtin_amdgcn_update_dpp(0, a, 0xb1, 0xf, 0xf, false);    // quad_perm [1,0,3,2]
}

int main() {
    int* d;
    int h[8 * 64];
    hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[8] = {"p32.vdst", "p32.src0", "p16.vdst", "p16.src0", "row_mirror", "row_half_mirror",
                            "quad[2,3,0,1]", "quad[1,0,3,2]"};
    for (int k = 0; k < 8; ++k) {
        printf("%-16s", names[k]);
        for (int l = 0; l < 64; ++l) printf(" %d", h[k * 64 + l]);
        printf("\n");
    }
    hipFree(d);
    return 0;
}
