// kmpc_npexp.h — the reference's gross returns R = np.exp(yhat) on a float32 array (mpc.py:55),
// bit for bit as numpy computes them.
//
// The reference hands cvxpy R = np.exp(predicted_log_returns) where predicted_log_returns is the
// float32 [H, N] array of backtest.py:121; cvxpy then promotes R to float64. numpy (2.2, x86-64 with
// AVX2 or AVX512F — every host the reference's uv.lock targets in practice) evaluates float32 exp
// with its own SIMD routine, not libm: Cody-Waite range reduction with k = rint(x·log2 e), a
// [5/2] rational minimax approximation on the reduced argument (all steps float32 FMAs, one
// float32 division), and a 2^k scaling; saturation to +inf at x >= 88.7228…, to 0 at
// x <= -103.972…, NaN through. It is up to ~2 ulp from the correctly rounded exp, so
// (float)exp((double)x) disagrees with numpy on ~40% of log-return-sized inputs. This restatement
// reproduces it exactly (pinned against np.exp on every finite float32 with |x| < 100 in the build
// container, and on the device by tests/test_solver_gpu.py::test_gross_returns_bit_exact).
//
// The solve kernels then use m = (double)R - 1 (exact: R has 24 significant bits) and R·w = (1 + m)·w
// — the same float64 numbers cvxpy builds its problem from.
#pragma once
#include <hip/hip_runtime.h>

namespace kmpc {

__device__ __forceinline__ float np_expf(float x) {
#pragma clang fp contract(off)
    if (!(x == x)) return x;                                   // NaN in, NaN out
    if (x >= 88.72283935546875f) return __builtin_inff();      // overflow
    if (x <= -103.97208404541015625f) return 0.0f;             // underflow
    // k = rint(x log2 e) by the 1.5·2^23 magic-number round (two float32 roundings, no FMA). The
    // empty asm statements pin each rounded intermediate: __fmul_rn / __fadd_rn are plain operators
    // in a header outside this function's contract(off) scope, and the backend fused x·log2e + magic
    // into one FMA there (k off by one on rare inputs, 1-2 ulp from numpy past x ~ 72, measured).
    const float magic = 0x1.8p+23f;
    float q = x * 1.442695040888963407359924681001892137f;
    asm volatile("" : "+v"(q));
    q = q + magic;
    asm volatile("" : "+v"(q));
    q = q - magic;
    // Cody-Waite reduction: r = x - k ln2 with ln2 split high / low (float32 FMAs)
    float r = __builtin_fmaf(q, -6.93145752e-1f, x);
    r = __builtin_fmaf(q, -1.42860677e-6f, r);
    r = __builtin_fmaf(q, 0.0f, r);
    // exp(r) ~ P(r) / Q(r), Horner in float32 FMAs
    float p = __builtin_fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
    p = __builtin_fmaf(p, r, 5.114512081637298353406e-02f);
    p = __builtin_fmaf(p, r, 2.473615434895520810817e-01f);
    p = __builtin_fmaf(p, r, 7.257664613233124478488e-01f);
    p = __builtin_fmaf(p, r, 9.999999999980870924916e-01f);
    float d = __builtin_fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
    d = __builtin_fmaf(d, r, 1.0f);
    // correctly rounded float32 quotient: the float64 quotient rounded once more is correctly
    // rounded for division (53 >= 2·24 + 2), independent of the compiler's f32 division lowering
    const float e = (float)((double)p / (double)d);
    return ldexpf(e, (int)q);
}

// m = R - 1 in float64 (exact), R = np.exp(y) in float32
__device__ __forceinline__ double np_expm1_d(float y) { return (double)np_expf(y) - 1.0; }

}  // namespace kmpc
