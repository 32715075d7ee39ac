// kmpc_rollout.hip — batched Koopman rollout on gfx950 (replaces backtest.py:99-121).
//
//   z  = encode(obs)                       GenericKM: MLPCoder (model.py:108-117) + norm_fn
//                                          LISTAKM:   LISTA (model.py:190-209)
//   for k in 0..H-1:
//     z = z @ K  (+ norm_fn)               model.py:311-321 / 787-797 (row-vector convention)
//     yhat[:, k, :] = decode(z)[:, :N] * std + mean      model.py:768-777 / 839-850,
//                                          data_finance.py:729 (slice), :740-742 (de-standardize)
//
// Every dense contraction is one fp32 GEMM — the arithmetic type of the reference's torch fp32
// path — on the bf16 MFMA with each fp32 operand split exactly into three bf16 planes
// (gemm_nt_x3_kernel; desc->dtype = KMPC_DTYPE_F32, the default) or on the f32-input MFMA
// (v_mfma_f32_32x32x2_f32, KMPC_DTYPE_F32_F32MFMA); or, with KMPC_DTYPE_BF16, a bf16 MFMA GEMM
// (operands rounded to bf16, fp32 accumulation; BASELINE configs[4]) — with a fused epilogue
// (bias + activation, LISTA shrink, de-standardize-and-scatter). Only the first N decoder rows are
// evaluated. Weights in the reference's nn.Linear [out, in] layout are consumed as-is ("NT");
// K and S (right-multiplied, [in, out]) are transposed once per call into the workspace.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kmpc_internal.h"

namespace kmpc {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

enum Epi : int {
    EPI_NONE = 0,        // out = acc (+ bias)
    EPI_ACT = 1,         // out = act(acc + bias)
    EPI_SHRINK = 2,      // out = shrink(acc + R, thr)            (LISTA, model.py:30-40,205-207)
    EPI_DESTD = 3,       // out = acc * std[n] + mean[n]          (data_finance.py:740-742)
};

struct GemmArgs {
    int M, N, K;
    const float* A; int lda;      // [M, K]
    const float* B; int ldb;      // [N, K]  (nn.Linear weight layout)
    const float* bias;            // [N] or null
    float* C; int ldc;            // [M, N] (row stride ldc)
    int epi, act;
    const float* R; int ldr;      // EPI_SHRINK addend [M, N]
    float thr;
    const float* mean; const float* stdv;   // EPI_DESTD [N]
    int bf16;                     // 1: operands rounded to bf16, v_mfma_f32_32x32x16_bf16 (fp32 accumulate);
                                  // 2: fp32 operands as three bf16 planes (gemm_nt_x3_kernel)
    int ksplit;                   // > 1: blockIdx.z takes a K slice, raw partials to part[z][M][N]
    float* part;                  //      (splitk_epilogue_kernel sums them in slice order, then the epilogue)
};

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

__device__ __forceinline__ float apply_act(float x, int act) {
    if (act == KMPC_ACT_RELU) return fmaxf(x, 0.0f);
    if (act == KMPC_ACT_TANH) return tanhf(x);
    return gelu_erf(x);
}

// Tile: GM x GN waves per block, each a (32 WM) x (32 WN) block of 32 x 32 accumulator tiles, BK = 32.
// 128 x 128 as 4 x 2 waves of 32 x 64 (512 threads) for GEMMs with 512 or more such tiles, as 4 x 4
// waves of 32 x 32 (1024 threads) below that (one workgroup per CU); split K for the narrow last
// encoder layer of small batches (configs[1]).
constexpr int BM = 128, BN = 128, BK = 32, LDS_STRIDE = BK + 4;

// C = epi(A . B^T). Each lane of an MFMA consumes 16 contiguous k (k = 16h + s, h = lane >> 5),
// so operand fragments are two ds_read_b128 per row; the k permutation is the same for A and B.
// y * std + mean with two float32 roundings, as the reference's torch mul then add
// (data_finance.py:742): FMA contraction off here so yhat matches it bit for bit.
__device__ __forceinline__ float destandardize(float y, float sd, float mu) {
#pragma clang fp contract(off)
    const float p = y * sd;
    return p + mu;
}

// the epilogue of one output element
__device__ __forceinline__ float epi_value(const GemmArgs& g, int m, int n, float acc) {
    float v = acc + (g.bias ? g.bias[n] : 0.0f);
    if (g.epi == EPI_ACT) {
        v = apply_act(v, g.act);
    } else if (g.epi == EPI_SHRINK) {
        v += g.R[(size_t)m * g.ldr + n];
        const float av = fabsf(v) - g.thr;
        v = (av > 0.0f) ? copysignf(av, v) : 0.0f * v;
    } else if (g.epi == EPI_DESTD) {
        v = destandardize(v, g.stdv[n], g.mean[n]);
    }
    return v;
}

// fused epilogue of a WM x WN block of 32 x 32 accumulator tiles (either MFMA dtype: the C/D
// layout is dtype-independent on gfx950)
template <int WM, int WN>
__device__ __forceinline__ void epilogue(const GemmArgs& g, f32x16 (&acc)[WM][WN], int m0, int n0, int wm, int wn,
                                         int lane) {
    // epilogue: C/D layout col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b) {
            const int n = n0 + wn + b * 32 + (lane & 31);
            if (n >= g.N) continue;
            const float bias = g.bias ? g.bias[n] : 0.0f;
            float mu = 0.0f, sd = 1.0f;
            if (g.epi == EPI_DESTD) { mu = g.mean[n]; sd = g.stdv[n]; }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (m >= g.M) continue;
                float v = acc[a][b][r] + bias;
                if (g.epi == EPI_ACT) {
                    v = apply_act(v, g.act);
                } else if (g.epi == EPI_SHRINK) {
                    v += g.R[(size_t)m * g.ldr + n];
                    const float av = fabsf(v) - g.thr;
                    v = (av > 0.0f) ? copysignf(av, v) : 0.0f * v;
                } else if (g.epi == EPI_DESTD) {
                    v = destandardize(v, sd, mu);
                }
                g.C[(size_t)m * g.ldc + n] = v;
            }
        }
}

// XCD-aware tile order: the dispatcher deals workgroups round-robin over the 8 XCDs by linear id,
// so neighbouring tiles of one row panel of A would land in 8 different L2s. Renumber so that each
// XCD gets a contiguous run of tiles (same A row panels): id -> (id % 8) * (total / 8) + id / 8.
__device__ __forceinline__ void xcd_tile(int& m0, int& n0, int tm = BM, int tn = BN) {
    const int gx = gridDim.x, total = gridDim.x * gridDim.y;
    int id = blockIdx.y * gx + blockIdx.x;
    if ((total & 7) == 0) id = (id & 7) * (total >> 3) + (id >> 3);
    m0 = (id / gx) * tm;
    n0 = (id % gx) * tn;
}

// k-tile depth of the 64 x 64 tile (small window batches): 32, or 64 (one barrier pair per 32 MFMAs
// per wave instead of per 16; dev A/B: tools/ab_c2.sh)
#ifndef KMPC_GEMM_BK1
#define KMPC_GEMM_BK1 32
#endif
// Workgroup tile (64 WM) x (64 WN): 4 waves as 2 x 2, each a (32 WM) x (32 WN) block of 32 x 32
// accumulator tiles. (1, 1) / (2, 2): the 64- / 128-square tiles; (2, 1): 128 x 64, half the
// workgroups of the 64-square tile with each B fragment feeding two MFMAs.
// GM x GN waves per workgroup (2 x 2: 256 threads; 4 x 2: 512 threads, two waves per SIMD for the
// one-workgroup-per-CU grids)
template <int WM, int WN, int BKT = ((WM == 1 && WN == 1) ? KMPC_GEMM_BK1 : BK), int GM = 2, int GN = 2>
__global__ void __launch_bounds__(64 * GM * GN) gemm_nt_kernel(GemmArgs g) {
    constexpr int NT = 64 * GM * GN;
    constexpr int TM = 32 * GM * WM, TN = 32 * GN * WN;
    constexpr int LS = BKT + 4;   // LDS row stride (floats): conflict-free ds_read_b128 fragments
    __shared__ float As[TM * LS];
    __shared__ float Bs[TN * LS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int m0, n0;
    xcd_tile(m0, n0, TM, TN);
    const int wm = (wv / GN) * 32 * WM, wn = (wv % GN) * 32 * WN;
    f32x16 acc[WM][WN];
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

    const bool vec_ok = ((g.lda & 3) == 0) && ((g.ldb & 3) == 0) &&
                        ((((uintptr_t)g.A) & 15) == 0) && ((((uintptr_t)g.B) & 15) == 0);
    // split K: slice blockIdx.z of ksplit (whole BK tiles)
    int kbeg = 0, kend = g.K;
    if (g.ksplit > 1) {
        const int kc = ((g.K + g.ksplit * BKT - 1) / (g.ksplit * BKT)) * BKT;
        kbeg = blockIdx.z * kc;
        kend = min(g.K, kbeg + kc);
    }
    // A tile: TM rows x BKT k = TM BKT / 4 float4, TM BKT / 1024 per thread (B: TN rows). The next
    // k-tile's global loads are issued into registers before this tile's MFMAs (register double
    // buffering: one LDS buffer, the HBM / L2 latency under the math).
    constexpr int QA = TM * BKT / (4 * NT), QB = TN * BKT / (4 * NT);
    static_assert(QA * 4 * NT == TM * BKT && QB * 4 * NT == TN * BKT, "tile loads per thread");
    constexpr int RQ = BKT / 4;                     // float4 per row
    f32x4 va[QA], vb[QB];
    auto fetch_row = [&](const float* P, int ld, int rows, int r0, int row, int kk, f32x4& v) {
        v = f32x4{0.f, 0.f, 0.f, 0.f};
        const int rr = r0 + row;
        if (rr >= rows) return;
        if (vec_ok && kk + 3 < kend) {
            v = *(const f32x4*)(P + (size_t)rr * ld + kk);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (kk + e < kend) v[e] = P[(size_t)rr * ld + kk + e];
        }
    };
    auto fetch = [&](int k0) {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int idx = tid + q * NT;           // 0 .. TM RQ - 1
            fetch_row(g.A, g.lda, g.M, m0, idx / RQ, k0 + (idx % RQ) * 4, va[q]);
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) {
            const int idx = tid + q * NT;
            fetch_row(g.B, g.ldb, g.N, n0, idx / RQ, k0 + (idx % RQ) * 4, vb[q]);
        }
    };
    auto stage = [&]() {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int idx = tid + q * NT;
            *(f32x4*)(As + (idx / RQ) * LS + (idx % RQ) * 4) = va[q];
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) {
            const int idx = tid + q * NT;
            *(f32x4*)(Bs + (idx / RQ) * LS + (idx % RQ) * 4) = vb[q];
        }
    };
    auto compute = [&]() {
        const int r = lane & 31, h = lane >> 5;
#pragma unroll
        for (int kb = 0; kb < BKT; kb += 32) {   // 32-k sub-steps: lane (r, h) takes k = kb + 16 h + s
            float af[WM][16], bf[WN][16];
#pragma unroll
            for (int a = 0; a < WM; ++a) {
                const float* pa = As + (wm + a * 32 + r) * LS + kb + 16 * h;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 x = *(const f32x4*)(pa + 4 * q);
#pragma unroll
                    for (int e = 0; e < 4; ++e) af[a][4 * q + e] = x[e];
                }
            }
#pragma unroll
            for (int b = 0; b < WN; ++b) {
                const float* pb = Bs + (wn + b * 32 + r) * LS + kb + 16 * h;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 y = *(const f32x4*)(pb + 4 * q);
#pragma unroll
                    for (int e = 0; e < 4; ++e) bf[b][4 * q + e] = y[e];
                }
            }
#pragma unroll
            for (int s = 0; s < 16; ++s)
#pragma unroll
                for (int a = 0; a < WM; ++a)
#pragma unroll
                    for (int b = 0; b < WN; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
        }
    };
    fetch(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += BKT) {
        stage();
        __syncthreads();
        if (k0 + BKT < kend) fetch(k0 + BKT);
        compute();
        __syncthreads();
    }
    if (g.ksplit > 1) {   // raw partial of this K slice
        float* P = g.part + (size_t)blockIdx.z * g.M * g.N;
#pragma unroll
        for (int a = 0; a < WM; ++a)
#pragma unroll
            for (int b = 0; b < WN; ++b) {
                const int n = n0 + wn + b * 32 + (lane & 31);
                if (n >= g.N) continue;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (m < g.M) P[(size_t)m * g.N + n] = acc[a][b][r];
                }
            }
        return;
    }
    epilogue<WM, WN>(g, acc, m0, n0, wm, wn, lane);
}

// split-K: C = epi(sum of the ksplit partials, in slice order)
__global__ void __launch_bounds__(256) splitk_epilogue_kernel(GemmArgs g) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)g.M * g.N) return;
    const int m = (int)(i / g.N), n = (int)(i % g.N);
    float v = g.part[i];
    for (int z = 1; z < g.ksplit; ++z) v += g.part[(size_t)z * g.M * g.N + i];
    g.C[(size_t)m * g.ldc + n] = epi_value(g, m, n, v);
}

// bf16 variant (BASELINE configs[4]: "bf16 MFMA rollout"): the same 128 x 128 tile and epilogues;
// A and B are rounded to bf16 (RNE, v_cvt_pk_bf16_f32) while being staged into LDS, the products
// run on v_mfma_f32_32x32x16_bf16 with fp32 accumulation. Lane (r, h) of a 32x32x16 step holds
// A[row r][k = 8h + j] and B[col r][k = 8h + j], j = 0..7: one ds_read_b128 per operand per step.
constexpr int LDS_STRIDE_H = BK + 8;   // bf16 elements per LDS row (80 B: 16-B aligned fragments)

// WT = 2: 128 x 128 tile (4 waves of 64 x 64); WT = 1: 64 x 64 (4 waves of 32 x 32), for grids with
// fewer 128-tiles than CUs and a short K (configs[4]'s LISTA and latent-step layers)
template <int WT>
__global__ void __launch_bounds__(256) gemm_nt_bf16_kernel(GemmArgs g) {
    constexpr int TM = 64 * WT;
    __shared__ __bf16 As[TM * LDS_STRIDE_H];
    __shared__ __bf16 Bs[TM * LDS_STRIDE_H];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int m0, n0;
    xcd_tile(m0, n0, TM, TM);
    const int wm = (wv >> 1) * 32 * WT, wn = (wv & 1) * 32 * WT;
    f32x16 acc[WT][WT];
#pragma unroll
    for (int a = 0; a < WT; ++a)
#pragma unroll
        for (int b = 0; b < WT; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

    const bool vec_ok = ((g.lda & 3) == 0) && ((g.ldb & 3) == 0) &&
                        ((((uintptr_t)g.A) & 15) == 0) && ((((uintptr_t)g.B) & 15) == 0);
    // split K: slice blockIdx.z of ksplit (whole BK tiles), raw partials as gemm_nt_kernel
    int kbeg = 0, kend = g.K;
    if (g.ksplit > 1) {
        const int kc = ((g.K + g.ksplit * BK - 1) / (g.ksplit * BK)) * BK;
        kbeg = blockIdx.z * kc;
        kend = min(g.K, kbeg + kc);
    }
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
#pragma unroll
        for (int q = 0; q < 2 * WT; ++q) {
            const int idx = tid + q * 256;          // TM rows x 8 groups of 4 k
            const int row = idx >> 3, c4 = (idx & 7) * 4;
            const int kk = k0 + c4;
            f32x4 va = {0.f, 0.f, 0.f, 0.f}, vb = {0.f, 0.f, 0.f, 0.f};
            const int ma = m0 + row, nb = n0 + row;
            if (vec_ok && kk + 3 < kend) {
                if (ma < g.M) va = *(const f32x4*)(g.A + (size_t)ma * g.lda + kk);
                if (nb < g.N) vb = *(const f32x4*)(g.B + (size_t)nb * g.ldb + kk);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (kk + e < kend) {
                        if (ma < g.M) va[e] = g.A[(size_t)ma * g.lda + kk + e];
                        if (nb < g.N) vb[e] = g.B[(size_t)nb * g.ldb + kk + e];
                    }
                }
            }
            bf16x4 ha, hb;
#pragma unroll
            for (int e = 0; e < 4; ++e) { ha[e] = (__bf16)va[e]; hb[e] = (__bf16)vb[e]; }
            *(bf16x4*)(As + row * LDS_STRIDE_H + c4) = ha;
            *(bf16x4*)(Bs + row * LDS_STRIDE_H + c4) = hb;
        }
        __syncthreads();
        const int r = lane & 31, h = lane >> 5;
#pragma unroll
        for (int st = 0; st < BK / 16; ++st) {
            bf16x8 af[WT], bfr[WT];
#pragma unroll
            for (int a = 0; a < WT; ++a) {
                af[a] = *(const bf16x8*)(As + (wm + a * 32 + r) * LDS_STRIDE_H + 16 * st + 8 * h);
                bfr[a] = *(const bf16x8*)(Bs + (wn + a * 32 + r) * LDS_STRIDE_H + 16 * st + 8 * h);
            }
#pragma unroll
            for (int a = 0; a < WT; ++a)
#pragma unroll
                for (int b = 0; b < WT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
    if (g.ksplit > 1) {   // raw partial of this K slice
        float* P = g.part + (size_t)blockIdx.z * g.M * g.N;
#pragma unroll
        for (int a = 0; a < WT; ++a)
#pragma unroll
            for (int b = 0; b < WT; ++b) {
                const int n = n0 + wn + b * 32 + (lane & 31);
                if (n >= g.N) continue;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (m < g.M) P[(size_t)m * g.N + n] = acc[a][b][r];
                }
            }
        return;
    }
    epilogue<WT, WT>(g, acc, m0, n0, wm, wn, lane);
}

// fp32 GEMM as three bf16 planes (round 5): every fp32 operand x is split exactly into
// x = hi + mid + lo, three bf16 numbers (8 significant bits each, 24 in all: hi = bf16(x),
// mid = bf16(x - hi), lo = x - hi - mid, every subtraction exact in fp32), and
//   a . b = sum over the six plane pairs of order <= 2^-16:  hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid
// on v_mfma_f32_32x32x16_bf16 (bf16 x bf16 products are exact in fp32, fp32 accumulation). The
// dropped pairs (mid.lo, lo.mid, lo.lo) are below 2^-24 of |a b|: the same order as the one fp32
// rounding of an fp32 product, so the result is an fp32 GEMM in accuracy (measured against an fp64
// reference beside the native f32-input MFMA: tests/test_rollout_gpu.py) at 12 MFMA cycles per k
// instead of 32 (v_mfma_f32_32x32x2_f32: 64 cycles for k = 2; the bf16 form: 32 cycles for k = 16).
// Same tiles, k loop (register double buffering), split-K and epilogues as gemm_nt_kernel; the
// planes are formed while staging into LDS.
#ifndef KMPC_F32_GEMM   // the GEMM form of KMPC_DTYPE_F32: 2 three bf16 planes, 0 f32-input MFMA (dev A/B)
#define KMPC_F32_GEMM 2
#endif
#ifndef KMPC_X3_TIMING   // dev timing bounds only (wrong results): 1 no split, 2 half the products
#define KMPC_X3_TIMING 0
#endif
__device__ __forceinline__ void split3(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
    hi = (__bf16)x;
    if (KMPC_X3_TIMING == 1) { mid = hi; lo = hi; return; }
    const float r1 = x - (float)hi;
    mid = (__bf16)r1;
    lo = (__bf16)(r1 - (float)mid);
}

#ifndef KMPC_X3_DB   // 1: two LDS buffers, the next k-tile split between this tile's MFMA steps
#define KMPC_X3_DB 1
#endif
template <int WM, int WN, int GM = 2, int GN = 2, int BKT = BK>
__global__ void __launch_bounds__(64 * GM * GN) gemm_nt_x3_kernel(GemmArgs g) {
    constexpr int NT = 64 * GM * GN;
    constexpr int TM = 32 * GM * WM, TN = 32 * GN * WN;
    constexpr int NS = BKT / 16;               // 16-k MFMA steps per k-tile (BKT = 32: two)
    static_assert(NS * 16 == BKT && NS >= 1, "k-tile of whole 16-k steps");
    constexpr int LS = BKT + 8;                // bf16 elements per LDS row (80 B: aligned ds_read_b128)
    // two buffers when they fit and the workgroup alone holds four waves per SIMD (a smaller one
    // keeps the single buffer: two workgroups per CU share the LDS; dev A/B tools/ab_x3.sh)
    constexpr bool DB = KMPC_X3_DB && 2 * 3 * (TM + TN) * LS * 2 <= 160 * 1024 && GM * GN >= 16;
    constexpr int NB = DB ? 2 : 1;
    __shared__ __bf16 As[NB][3][TM * LS];
    __shared__ __bf16 Bs[NB][3][TN * LS];
    static_assert(sizeof(As) + sizeof(Bs) <= 160 * 1024, "LDS");
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int m0, n0;
    xcd_tile(m0, n0, TM, TN);
    const int wm = (wv / GN) * 32 * WM, wn = (wv % GN) * 32 * WN;
    f32x16 acc[WM][WN];
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

    const bool vec_ok = ((g.lda & 3) == 0) && ((g.ldb & 3) == 0) &&
                        ((((uintptr_t)g.A) & 15) == 0) && ((((uintptr_t)g.B) & 15) == 0);
    int kbeg = 0, kend = g.K;
    if (g.ksplit > 1) {
        const int kc = ((g.K + g.ksplit * BKT - 1) / (g.ksplit * BKT)) * BKT;
        kbeg = blockIdx.z * kc;
        kend = min(g.K, kbeg + kc);
    }
    constexpr int QA = TM * BKT / (4 * NT), QB = TN * BKT / (4 * NT);
    static_assert(QA * 4 * NT == TM * BKT && QB * 4 * NT == TN * BKT, "tile loads per thread");
    constexpr int RQ = BKT / 4;
    f32x4 va[QA], vb[QB];
    auto fetch_row = [&](const float* P, int ld, int rows, int r0, int row, int kk, f32x4& v) {
        v = f32x4{0.f, 0.f, 0.f, 0.f};
        const int rr = r0 + row;
        if (rr >= rows) return;
        if (vec_ok && kk + 3 < kend) {
            v = *(const f32x4*)(P + (size_t)rr * ld + kk);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (kk + e < kend) v[e] = P[(size_t)rr * ld + kk + e];
        }
    };
    auto fetch = [&](int k0) {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int idx = tid + q * NT;
            fetch_row(g.A, g.lda, g.M, m0, idx / RQ, k0 + (idx % RQ) * 4, va[q]);
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) {
            const int idx = tid + q * NT;
            fetch_row(g.B, g.ldb, g.N, n0, idx / RQ, k0 + (idx % RQ) * 4, vb[q]);
        }
    };
    auto put = [&](__bf16* S0, __bf16* S1, __bf16* S2, int idx, const f32x4& v) {
        bf16x4 h, m, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            __bf16 x0, x1, x2;
            split3(v[e], x0, x1, x2);
            h[e] = x0; m[e] = x1; l[e] = x2;
        }
        const int o = (idx / RQ) * LS + (idx % RQ) * 4;
        *(bf16x4*)(S0 + o) = h;
        *(bf16x4*)(S1 + o) = m;
        *(bf16x4*)(S2 + o) = l;
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int q = 0; q < QA; ++q) put(As[buf][0], As[buf][1], As[buf][2], tid + q * NT, va[q]);
#pragma unroll
        for (int q = 0; q < QB; ++q) put(Bs[buf][0], Bs[buf][1], Bs[buf][2], tid + q * NT, vb[q]);
    };
    auto substep = [&](int buf, int st) {   // lane (r, h): k = 16 st + 8 h + j
        const int r = lane & 31, h = lane >> 5;
        {
            bf16x8 af[3][WM], bf[3][WN];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
#pragma unroll
                for (int a = 0; a < WM; ++a)
                    af[p][a] = *(const bf16x8*)(As[buf][p] + (wm + a * 32 + r) * LS + 16 * st + 8 * h);
#pragma unroll
                for (int b = 0; b < WN; ++b)
                    bf[p][b] = *(const bf16x8*)(Bs[buf][p] + (wn + b * 32 + r) * LS + 16 * st + 8 * h);
            }
#pragma unroll
            for (int a = 0; a < WM; ++a)
#pragma unroll
                for (int b = 0; b < WN; ++b) {
                    // the small pairs first, hi.hi last (fixed order: deterministic)
                    f32x16 c = acc[a][b];
                    if (KMPC_X3_TIMING == 2) {
                        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[1][b], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][a], bf[2][b], c, 0, 0, 0);
                        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[0][b], c, 0, 0, 0);
                        continue;
                    }
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[1][b], c, 0, 0, 0);   // mid.mid
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][a], bf[0][b], c, 0, 0, 0);   // lo.hi
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[2][b], c, 0, 0, 0);   // hi.lo
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[0][b], c, 0, 0, 0);   // mid.hi
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[1][b], c, 0, 0, 0);   // hi.mid
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[0][b], c, 0, 0, 0);   // hi.hi
                    acc[a][b] = c;
                }
        }
    };
    if constexpr (DB) {
        // one barrier per k-tile: tile k's MFMA steps read buffer k & 1 while tile k + 1 (fetched
        // into registers one iteration earlier) is split into the other buffer between them
        fetch(kbeg);
        stage(0);
        if (kbeg + BKT < kend) fetch(kbeg + BKT);
        __syncthreads();
        int buf = 0;
        for (int k0 = kbeg; k0 < kend; k0 += BKT) {
            substep(buf, 0);
            if (k0 + BKT < kend) {
                stage(buf ^ 1);
                if (k0 + 2 * BKT < kend) fetch(k0 + 2 * BKT);
            }
#pragma unroll
            for (int st = 1; st < NS; ++st) substep(buf, st);
            __syncthreads();
            buf ^= 1;
        }
    } else {
        fetch(kbeg);
        for (int k0 = kbeg; k0 < kend; k0 += BKT) {
            stage(0);
            __syncthreads();
            if (k0 + BKT < kend) fetch(k0 + BKT);
#pragma unroll
            for (int st = 0; st < NS; ++st) substep(0, st);
            __syncthreads();
        }
    }
    if (g.ksplit > 1) {   // raw partial of this K slice
        float* P = g.part + (size_t)blockIdx.z * g.M * g.N;
#pragma unroll
        for (int a = 0; a < WM; ++a)
#pragma unroll
            for (int b = 0; b < WN; ++b) {
                const int n = n0 + wn + b * 32 + (lane & 31);
                if (n >= g.N) continue;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (m < g.M) P[(size_t)m * g.N + n] = acc[a][b][r];
                }
            }
        return;
    }
    epilogue<WM, WN>(g, acc, m0, n0, wm, wn, lane);
}

// shrink in place (LISTA initial z = shrink(c, thr), model.py:203)
__global__ void shrink_kernel(const float* x, float* y, size_t n, float thr) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float v = x[i];
        const float av = fabsf(v) - thr;
        y[i] = (av > 0.0f) ? copysignf(av, v) : 0.0f * v;
    }
}

// x / ||x||_2 per row (norm_fn 'ball', model.py:750-751); one wave per row
__global__ void ball_norm_kernel(float* x, int M, int L) {
    const int row = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, lane = threadIdx.x & 63;
    if (row >= M) return;
    float* p = x + (size_t)row * L;
    float s = 0.0f;
    for (int j = lane; j < L; j += 64) s += p[j] * p[j];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    const float nrm = sqrtf(s);
    for (int j = lane; j < L; j += 64) p[j] = p[j] / nrm;
}

// out[j][i] = in[i][j]  (L x L)
__global__ void transpose_kernel(const float* in, float* out, int R, int Cc) {
    __shared__ float tile[32][33];
    const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 8 rows per pass
    for (int r = ty; r < 32; r += 8) {
        const int i = by + r, j = bx + tx;
        if (i < R && j < Cc) tile[r][tx] = in[(size_t)i * Cc + j];
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int j = bx + r, i = by + tx;
        if (i < R && j < Cc) out[(size_t)j * R + i] = tile[tx][r];
    }
}

// Fused latent steps (fp32, single-layer decoder): the whole H-step loop of backtest.py:101-119
// in one launch. A block owns 32 windows; their z rows stay in LDS for all H steps (ping-pong
// tiles), each step computes z <- z K on v_mfma_f32_32x32x2_f32 (K^T rows streamed from L2, the
// next 32-k chunk prefetched under the current one), the ball norm if any (model.py:750-751),
// then decode rows 0..N-1 with bias + de-standardize straight into yhat[:, k, :]
// (model.py:768-777, data_finance.py:729-742). Same k order per MFMA lane as gemm_nt_kernel (lane
// (r, h) consumes k = k0 + 16 h + s); the chunks alternate between two accumulators, so the
// fp32 sums are regrouped (not bit-identical to the unfused launches; within the rollout tests'
// 1e-4 of the reference). Replaces 2H small GEMM launches that are latency-bound at small batch.
struct LatentArgs {
    int B, L, N, H;
    const float* z0;     // [B, L]
    // z0 as the raw split-K partials of the last encoder layer (nparts > 0): z0 = sum of the parts in
    // slice order + zbias, as splitk_epilogue_kernel would have formed it (bit-identical)
    const float* zparts; int nparts; const float* zbias;
    const float* Kt;     // [L, L]: row j = column j of K (32-row kernel)
    const float* K;      // [L, L] row-major, z <- z K (16-row kernel: read in place, no transpose launch)
    const float* D;      // decoder rows 0..N-1, [N, L]
    const float* bias;   // [N] or null
    const float* mean; const float* stdv;
    float* yhat;         // [B, H, N]
    int ball;
};
constexpr int LAT_ROWS = 32;

__device__ __forceinline__ float latent_z0(const LatentArgs& a, int m, int col) {
    const size_t i = (size_t)m * a.L + col;
    if (a.nparts == 0) return a.z0[i];
    float v = a.zparts[i];
    for (int z = 1; z < a.nparts; ++z) v += a.zparts[(size_t)z * a.B * a.L + i];
    return v + (a.zbias ? a.zbias[col] : 0.0f);
}

// acc (+)= A[32 rows of As, stride lda] . B[32 rows of Bg, stride L]^T over k in [0, L)
__device__ __forceinline__ void tile_dot(const float* As, int lda, const float* Bg, int L, bool brow_ok,
                                         int lane, f32x16& acc) {
    const int r = lane & 31, h = lane >> 5;
    f32x16 acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc1[i] = 0.0f;
    const float* pa = As + r * lda + 16 * h;
    const float* pb = Bg + (size_t)r * L + 16 * h;
    f32x4 bn[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bn[q] = brow_ok ? *(const f32x4*)(pb + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < L; k0 += 32) {
        float af[16], bf[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 x = *(const f32x4*)(pa + k0 + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) { af[4 * q + e] = x[e]; bf[4 * q + e] = bn[q][e]; }
        }
        if (k0 + 32 < L) {   // next chunk of B under this chunk's MFMAs
#pragma unroll
            for (int q = 0; q < 4; ++q) bn[q] = brow_ok ? *(const f32x4*)(pb + k0 + 32 + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if ((k0 >> 5) & 1) {
#pragma unroll
            for (int s = 0; s < 16; ++s) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc1, 0, 0, 0);
        } else {
#pragma unroll
            for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] += acc1[i];
}

#ifndef KMPC_LAT_WAVES   // waves per block of latent_steps_kernel
#define KMPC_LAT_WAVES 4
#endif
template <int NWV>
__global__ void __launch_bounds__(64 * NWV) latent_steps_kernel(LatentArgs a) {
    extern __shared__ float zs[];   // [2][32][L + 4]
    const int L = a.L, LS = L + 4, N = a.N;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5;
    const int m0 = blockIdx.x * LAT_ROWS;
    float* zc = zs;
    float* zn = zs + LAT_ROWS * LS;
    for (int idx = tid; idx < LAT_ROWS * L; idx += 64 * NWV) {
        const int row = idx / L, col = idx - row * L;
        zc[row * LS + col] = (m0 + row < a.B) ? latent_z0(a, m0 + row, col) : 0.0f;
    }
    __syncthreads();
    const int nct = L / 32, ndt = (N + 31) / 32;
    for (int k = 0; k < a.H; ++k) {
        // z <- z K: output column tiles ct = wv, wv + NWV, ...
        for (int ct = wv; ct < nct; ct += NWV) {
            f32x16 acc;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
            tile_dot(zc, LS, a.Kt + (size_t)ct * 32 * L, L, true, lane, acc);
#pragma unroll
            for (int i = 0; i < 16; ++i)
                zn[((i & 3) + 8 * (i >> 2) + 4 * h) * LS + ct * 32 + (lane & 31)] = acc[i];
        }
        __syncthreads();
        if (a.ball) {   // x / ||x||_2 per row: 8 threads per row (the first 256 threads)
            if (tid < 8 * LAT_ROWS) {
                const int row = tid >> 3, part = tid & 7;
                float sq = 0.0f;
                for (int j = part; j < L; j += 8) sq += zn[row * LS + j] * zn[row * LS + j];
                sq += __shfl_xor(sq, 1, 64);
                sq += __shfl_xor(sq, 2, 64);
                sq += __shfl_xor(sq, 4, 64);
                const float nrm = sqrtf(sq);
                for (int j = part; j < L; j += 8) zn[row * LS + j] = zn[row * LS + j] / nrm;
            }
            __syncthreads();
        }
        // decode rows 0..N-1 (+ bias), de-standardize into yhat[:, k, :]
        for (int ct = wv; ct < ndt; ct += NWV) {
            f32x16 acc;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
            const int nrow = ct * 32 + (lane & 31);
            tile_dot(zn, LS, a.D + (size_t)ct * 32 * L, L, nrow < N, lane, acc);
            if (nrow < N) {
                const float bias = a.bias ? a.bias[nrow] : 0.0f, mu = a.mean[nrow], sd = a.stdv[nrow];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int m = m0 + (i & 3) + 8 * (i >> 2) + 4 * h;
                    if (m < a.B) a.yhat[((size_t)m * a.H + k) * N + nrow] = destandardize(acc[i] + bias, sd, mu);
                }
            }
        }
        float* t = zc; zc = zn; zn = t;
        __syncthreads();
    }
}

// Small window batches (fewer than 8,192 windows: 32-row blocks would leave CUs idle, BASELINE
// configs[1] has 4,096 -> 128 blocks): the same H-step loop with 16 windows per block on
// v_mfma_f32_16x16x4_f32 (A[l&15][k], B[k][l&15], k = 4 (l>>4) + e over a 16-k chunk; C/D
// col = l&15, row = 4 (l>>4) + i). z <- z K: L / 16 column tiles over the 4 waves; decode: the
// ceil(N / 16) decoder row tiles. One accumulator per tile (exact fp32, the k order of a chunk is
// the same for both operands).
constexpr int LAT16 = 16;
__device__ __forceinline__ void tile_dot16(const float* As, int lda, const float* Bg, int L, bool brow_ok, int lane,
                                           f32x4& acc) {
    const int r = lane & 15, kq = lane >> 4;
    const float* pa = As + r * lda + 4 * kq;
    const float* pb = Bg + (size_t)r * L + 4 * kq;
    f32x4 bn = brow_ok ? *(const f32x4*)pb : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < L; k0 += 16) {
        const f32x4 av = *(const f32x4*)(pa + k0);
        const f32x4 bv = bn;
        if (k0 + 16 < L) bn = brow_ok ? *(const f32x4*)(pb + k0 + 16) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], bv[e], acc, 0, 0, 0);
    }
}

// tile_dot16 with B = columns col0.. col0 + 15 of the row-major K read in place: lane (r, kq) loads
// K[k0 + 4 kq + e][col0 + r], e = 0..3 (16 lanes cover 64 contiguous bytes of a K row; K is L2
// resident). Same values and k order as tile_dot16 on K^T, so the sums are bit-identical.
__device__ __forceinline__ void tile_dot16_k(const float* As, int lda, const float* K, int col0, int L, int lane,
                                             f32x4& acc) {
    const int r = lane & 15, kq = lane >> 4;
    const float* pa = As + r * lda + 4 * kq;
    const float* pb = K + (size_t)(4 * kq) * L + col0 + r;
    f32x4 bn = {pb[0], pb[L], pb[2 * L], pb[3 * L]};
    for (int k0 = 0; k0 < L; k0 += 16) {
        const f32x4 av = *(const f32x4*)(pa + k0);
        const f32x4 bv = bn;
        if (k0 + 16 < L) {
            const float* q = pb + (size_t)(k0 + 16) * L;
            bn = f32x4{q[0], q[L], q[2 * L], q[3 * L]};
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], bv[e], acc, 0, 0, 0);
    }
}

// NWV waves per block: the L / 16 column tiles of z K spread over them (8 waves: one tile each at
// L = 128, two waves per SIMD at configs[1]'s 256 blocks)
#ifndef KMPC_LAT16_MAXB   // batches below this run the 16-row kernel
#define KMPC_LAT16_MAXB (256 * 32)
#endif
#ifndef KMPC_LAT16_WAVES
#define KMPC_LAT16_WAVES 8
#endif
template <int NWV, bool KDIR>
__global__ void __launch_bounds__(64 * NWV) latent_steps16_kernel(LatentArgs a) {
    extern __shared__ float zs[];   // [2][16][L + 4]
    const int L = a.L, LS = L + 4, N = a.N;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int m0 = blockIdx.x * LAT16;
    float* zc = zs;
    float* zn = zs + LAT16 * LS;
    for (int idx = tid; idx < LAT16 * L; idx += 64 * NWV) {
        const int row = idx / L, col = idx - row * L;
        zc[row * LS + col] = (m0 + row < a.B) ? latent_z0(a, m0 + row, col) : 0.0f;
    }
    __syncthreads();
    const int nct = L / 16, ndt = (N + 15) / 16;
    const int c = lane & 15, rq = 4 * (lane >> 4);
    for (int k = 0; k < a.H; ++k) {
        for (int ct = wv; ct < nct; ct += NWV) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            if (KDIR) tile_dot16_k(zc, LS, a.K, ct * 16, L, lane, acc);
            else tile_dot16(zc, LS, a.Kt + (size_t)ct * 16 * L, L, true, lane, acc);
#pragma unroll
            for (int i = 0; i < 4; ++i) zn[(rq + i) * LS + ct * 16 + c] = acc[i];
        }
        __syncthreads();
        if (a.ball) {   // x / ||x||_2 per row: 16 threads per row (the first 256 threads)
            if (tid < 16 * LAT16) {
                const int row = tid >> 4, part = tid & 15;
                float sq = 0.0f;
                for (int j = part; j < L; j += 16) sq += zn[row * LS + j] * zn[row * LS + j];
                sq += __shfl_xor(sq, 1, 64);
                sq += __shfl_xor(sq, 2, 64);
                sq += __shfl_xor(sq, 4, 64);
                sq += __shfl_xor(sq, 8, 64);
                const float nrm = sqrtf(sq);
                for (int j = part; j < L; j += 16) zn[row * LS + j] = zn[row * LS + j] / nrm;
            }
            __syncthreads();
        }
        for (int ct = wv; ct < ndt; ct += NWV) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            const int nrow = ct * 16 + c;
            tile_dot16(zn, LS, a.D + (size_t)ct * 16 * L, L, nrow < N, lane, acc);
            if (nrow < N) {
                const float bias = a.bias ? a.bias[nrow] : 0.0f, mu = a.mean[nrow], sd = a.stdv[nrow];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m = m0 + rq + i;
                    if (m < a.B) a.yhat[((size_t)m * a.H + k) * N + nrow] = destandardize(acc[i] + bias, sd, mu);
                }
            }
        }
        float* t = zc; zc = zn; zn = t;
        __syncthreads();
    }
}

// The H-step loop with the fp32 products on the bf16 MFMA in three exact planes (dtype
// KMPC_DTYPE_F32 at L = 256 — the C3 latent — identity norm; other shapes keep the f32-input
// kernels). 64 windows per block: z lives in LDS as its three bf16 planes (hi + mid + lo = z
// exactly; [3][64][L + 8], 101 KB, one block of 8 waves per CU), K^T and the decoder rows are split
// into planes once per call (split_planes_kernel, [3][rows][L] in the workspace, L2 resident) and
// read straight into the B fragments with 16-byte loads, two 16-k steps ahead; each B fragment
// feeds both 32-row tiles (half the L2 stream of 32-row blocks: a 32-row version of this kernel
// measured 1.54 ms against the f32-input kernel's 1.46 ms at C3, bound by that stream). Per 16-k
// step and tile six v_mfma_f32_32x32x16_bf16 (192 cycles) against eight v_mfma_f32_32x32x2_f32
// (512). One z buffer: each wave keeps its z K tiles in accumulators, a barrier, then the tiles are
// split into the buffer.
__global__ void __launch_bounds__(256) split_planes_kernel(const float* src, int R, int Rp, int L, int ld,
                                                           __bf16* dst) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t n = (size_t)Rp * L;
    if (i >= n) return;
    const int row = (int)(i / L), col = (int)(i % L);
    const float x = row < R ? src[(size_t)row * ld + col] : 0.0f;
    __bf16 h, m, l;
    split3(x, h, m, l);
    dst[i] = h;
    dst[n + i] = m;
    dst[2 * n + i] = l;
}

constexpr int LATX3_ROWS = 64;
// acc0 / acc1 += rows 0..31 / 32..63 of the z planes . B[32 plane rows at Bp, row stride L, plane
// stride PS]^T over k in [0, L); the six plane products per 16-k step, small pairs first
template <int L, int LSP, int PL>
__device__ __forceinline__ void tile_x3_2(const __bf16* zp, const __bf16* Bp, size_t PS, int lane, f32x16& acc0,
                                         f32x16& acc1) {
    const int r = lane & 31, h = lane >> 5;
    const __bf16* pa = zp + r * LSP + 8 * h;
    const __bf16* pb = Bp + (size_t)r * L + 8 * h;
    bf16x8 b0[3], b1[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        b0[p] = *(const bf16x8*)(pb + p * PS);
        b1[p] = *(const bf16x8*)(pb + p * PS + 16);
    }
#pragma unroll 2
    for (int k0 = 0; k0 < L; k0 += 16) {
        bf16x8 bf[3], a0[3], a1[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            bf[p] = b0[p];
            b0[p] = b1[p];
            if (k0 + 32 < L) b1[p] = *(const bf16x8*)(pb + p * PS + k0 + 32);
            a0[p] = *(const bf16x8*)(pa + p * PL + k0);
            a1[p] = *(const bf16x8*)(pa + 32 * LSP + p * PL + k0);
        }
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[1], bf[1], acc0, 0, 0, 0);   // mid.mid
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[1], bf[1], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[2], bf[0], acc0, 0, 0, 0);   // lo.hi
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[2], bf[0], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[0], bf[2], acc0, 0, 0, 0);   // hi.lo
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[0], bf[2], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[1], bf[0], acc0, 0, 0, 0);   // mid.hi
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[1], bf[0], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[0], bf[1], acc0, 0, 0, 0);   // hi.mid
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[0], bf[1], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[0], bf[0], acc0, 0, 0, 0);   // hi.hi
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[0], bf[0], acc1, 0, 0, 0);
    }
}

#ifndef KMPC_LATX3
#define KMPC_LATX3 1
#endif
template <int NWV, int L>
__global__ void __launch_bounds__(64 * NWV) latent_steps_x3_kernel(LatentArgs a, const __bf16* Kp,
                                                                   const __bf16* Dp, int Dpad) {
    extern __shared__ __bf16 zp[];   // [3][64][L + 8]
    // L a compile-time constant: the tile write-back's LDS offsets are instruction immediates
    constexpr int LSP = L + 8, PL = LATX3_ROWS * LSP, NCT = L / 32;
    static_assert(NCT <= NWV, "one z K column tile per wave");
    const int N = a.N;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * LATX3_ROWS;
    for (int idx = tid; idx < LATX3_ROWS * L; idx += 64 * NWV) {
        const int row = idx / L, col = idx - row * L;
        const float x = (m0 + row < a.B) ? latent_z0(a, m0 + row, col) : 0.0f;
        __bf16 p0, p1, p2;
        split3(x, p0, p1, p2);
        zp[row * LSP + col] = p0;
        zp[PL + row * LSP + col] = p1;
        zp[2 * PL + row * LSP + col] = p2;
    }
    __syncthreads();
    const int ndt = (N + 31) / 32;
    const size_t KPS = (size_t)L * L, DPS = (size_t)Dpad * L;
    float* yhat = a.yhat;
    for (int k = 0; k < a.H; ++k) {
        // per-step launder of the base pointers: the addresses derived from them are recomputed
        // each step (scalar work) instead of being hoisted into VGPRs for all H steps
        asm volatile("" : "+s"(Kp), "+s"(Dp), "+s"(yhat));
        // z <- z K: column tile wv of both row tiles, held in registers until every wave has read z
        f32x16 acc0, acc1;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.0f;
        if (wv < NCT) tile_x3_2<L, LSP, PL>(zp, Kp + (size_t)wv * 32 * L, KPS, lane, acc0, acc1);
        __syncthreads();
        if (wv < NCT) {
            __bf16* zt = zp + 4 * h * LSP + wv * 32 + r;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int o = ((i & 3) + 8 * (i >> 2)) * LSP;
                __bf16 p0, p1, p2;
                split3(acc0[i], p0, p1, p2);
                zt[o] = p0;
                zt[PL + o] = p1;
                zt[2 * PL + o] = p2;
                split3(acc1[i], p0, p1, p2);
                zt[32 * LSP + o] = p0;
                zt[PL + 32 * LSP + o] = p1;
                zt[2 * PL + 32 * LSP + o] = p2;
            }
        }
        __syncthreads();
        // decode rows 0..N-1 (+ bias), de-standardize into yhat[:, k, :]
        for (int ct = wv; ct < ndt; ct += NWV) {
            f32x16 d0, d1;
#pragma unroll
            for (int i = 0; i < 16; ++i) d0[i] = d1[i] = 0.0f;
            tile_x3_2<L, LSP, PL>(zp, Dp + (size_t)ct * 32 * L, DPS, lane, d0, d1);
            const int nrow = ct * 32 + r;
            if (nrow < N) {
                const float bias = a.bias ? a.bias[nrow] : 0.0f, mu = a.mean[nrow], sd = a.stdv[nrow];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int m = m0 + (i & 3) + 8 * (i >> 2) + 4 * h;
                    if (m < a.B) yhat[((size_t)m * a.H + k) * N + nrow] = destandardize(d0[i] + bias, sd, mu);
                    if (m + 32 < a.B)
                        yhat[((size_t)(m + 32) * a.H + k) * N + nrow] = destandardize(d1[i] + bias, sd, mu);
                }
            }
        }
        // (the next step's z K only reads the planes; its writes follow the barrier after it)
    }
}

// Latent powers (round 5): for a linear latent step (z_t = z_{t-1} K, identity norm) and a one-layer
// decoder, y_t = z_t D_N^T + b = z_0 (D_N (K^T)^t)^T + b, so the whole H-step loop is ONE GEMM of
// z_0 against W = [W_1; ...; W_H], W_t = D_N (K^T)^t = W_{t-1} K^T ([H N, L], latent_powers_kernel
// per call, float64 chains rounded once per W_t): L H N multiply-adds per window instead of
// H (L^2 + L N) — 3.6x fewer at C3 (L = 256, N = 100, H = 10). The same fp32 GEMM arithmetic,
// with the K products taken on the weights instead of the activations (checked against float64:
// tests/test_rollout_gpu.py). From KMPC_LATPOW_MINB windows.
#ifndef KMPC_LATPOW
#define KMPC_LATPOW 1
#endif
#ifndef KMPC_LATPOW_MINB   // (at configs[1]'s 4,096 windows the fused 16-row loop is faster: 0.152 vs 0.159 ms per step)
#define KMPC_LATPOW_MINB 8192
#endif
// W_t rows: one workgroup per decoder row i (rows are independent: W_t[i] = W_{t-1}[i] K^T), one
// thread per column j, the row chain carried in float64 in LDS and each W_t rounded once to fp32;
// Kt = K^T read coalesced (thread j reads Kt[k][j]). ~10 us where H GEMM launches took ~160 us.
__global__ void latent_powers_kernel(const float* __restrict__ D, const float* __restrict__ Kt, int L, int N, int H,
                                     float* __restrict__ W) {
    extern __shared__ double prow[];   // [L]
    const int i = blockIdx.x, j = threadIdx.x;
    if (j < L) prow[j] = (double)D[(size_t)i * L + j];
    __syncthreads();
    for (int t = 0; t < H; ++t) {
        double acc = 0.0;
        if (j < L) {
            // eight independent partial sums, sixteen loads in flight (L % 32 == 0: latent_fusable)
            double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
            for (int k0 = 0; k0 < L; k0 += 16) {
                float kv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) kv[u] = Kt[(size_t)(k0 + u) * L + j];
#pragma unroll
                for (int u = 0; u < 16; ++u) a[u & 7] = fma(prow[k0 + u], (double)kv[u], a[u & 7]);
            }
            acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
        }
        __syncthreads();
        if (j < L) {
            prow[j] = acc;
            W[((size_t)t * N + i) * L + j] = (float)acc;
        }
        __syncthreads();
    }
}

__global__ void tile_epilogue_kernel(int H, int N, const float* bias, const float* mean, const float* stdv,
                                     float* tb, float* tm, float* ts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= H * N) return;
    const int n = i % N;
    tb[i] = bias ? bias[n] : 0.0f;
    tm[i] = mean[n];
    ts[i] = stdv[n];
}

// the fused H-step kernel: fp32, one decoder layer, L % 32 == 0 and <= 512 (2 x 32 rows of z in
// LDS: 132 KB at L = 512), decoder rows read with 16-byte loads (16-byte aligned base); the
// descriptor's latent_unfused = KMPC_LATENT_UNFUSED forces the per-step launches, KMPC_LATENT_SEQUENTIAL
// the fused step-by-step loop even where the latent powers would run (A/B and the GPU tests)
static bool latent_fusable(const kmpc_rollout_desc* d) {
    return d->latent_unfused != KMPC_LATENT_UNFUSED && d->dtype != KMPC_DTYPE_BF16 && d->decoder.n_layers == 1 && d->L % 32 == 0 &&
           d->L <= 512 && ((uintptr_t)d->decoder.weight[0] & 15) == 0 &&
           !(d->model_kind == KMPC_MODEL_GENERIC && d->norm_fn != KMPC_NORM_ID && d->norm_fn != KMPC_NORM_BALL);
}

// split-K partial buffer: SPLITK slices of at most SPLITK_ELEMS outputs (split only when the
// 64 x 64 tiles number fewer than 256, i.e. M N <= 256 * 64 * 64)
#ifndef KMPC_F32_SPLITK   // K slices of the fp32 split-K GEMM (<= SPLITK_BUF)
#define KMPC_F32_SPLITK 4
#endif
constexpr int SPLITK = KMPC_F32_SPLITK;
constexpr int SPLITK_BUF = 8;   // slices the partial buffer holds (the bf16 long-K split uses all 8)
constexpr size_t SPLITK_ELEMS = (size_t)256 * 64 * 64;

// tile of the mid-size GEMMs (fewer than 512 128-square tiles): 11 = 64 x 64, 21 = 128 x 64,
// 12 = 64 x 128, 22 = 128 x 128 (4 waves), 42 = 128 x 128 as 4 x 2 waves of 32 x 64 (512 threads:
// two waves per SIMD at one workgroup per CU), 44 = 128 x 128 as 4 x 4 waves of 32 x 32 (1024
// threads, four per SIMD) — 44 measured best here, 42 for the large GEMMs (dev A/B:
// tools/ab_c2.sh)
#ifndef KMPC_GEMM_MID
#define KMPC_GEMM_MID 44
#endif
#ifndef KMPC_BF16_SPLITK
#define KMPC_BF16_SPLITK 1
#endif
#ifndef KMPC_Z0_FUSE   // the last encoder layer's split-K sum folded into the fused latent loop
#define KMPC_Z0_FUSE 1
#endif
#ifndef KMPC_BF16_SPLIT_MINK   // bf16 split-K only for long K (the LISTA encoder's obs = 10,000)
#define KMPC_BF16_SPLIT_MINK 2048
#endif
#ifndef KMPC_BF16_SMALL
#define KMPC_BF16_SMALL 1
#endif
#ifndef KMPC_GEMM_BIG   // tile of the large GEMMs: 22 = 128 x 128 (4 waves), 42 (8 waves), 82 = 256 x 128 (16 waves)
#define KMPC_GEMM_BIG 42
#endif
// nparts (optional): a split-K layer with no epilogue (EPI_NONE) leaves its raw partials in part and
// reports the slice count instead of launching splitk_epilogue_kernel (the latent kernels sum them)
// an fp32 GEMM launch: the f32-input MFMA kernel, or (g.bf16 == 2) the same tile on three bf16 planes
template <int WM, int WN, int GM = 2, int GN = 2>
static void launch_f32(dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (g.bf16 == 2)
        hipLaunchKernelGGL((gemm_nt_x3_kernel<WM, WN, GM, GN>), grid, dim3(64 * GM * GN), 0, s, g);
    else
        hipLaunchKernelGGL((gemm_nt_kernel<WM, WN, BK, GM, GN>), grid, dim3(64 * GM * GN), 0, s, g);
}

static int gemm(GemmArgs g, hipStream_t s, float* part = nullptr, int* nparts = nullptr) {
    if (nparts) *nparts = 0;
    if (g.M <= 0 || g.N <= 0) return KMPC_OK;
    g.ksplit = 1;
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM);
    if (g.bf16 == 1) {
        // fewer 128 x 128 tiles than CUs (BASELINE configs[4]: 1,024 windows x 512 -> 32 tiles) with a
        // long K: SPLITK slices, summed in slice order by the epilogue kernel (deterministic)
        const bool few = (size_t)grid.x * grid.y < 256;
        if (KMPC_BF16_SPLITK && few && part && g.K >= KMPC_BF16_SPLIT_MINK && (size_t)g.M * g.N <= SPLITK_ELEMS) {
            g.ksplit = SPLITK_BUF;
            g.part = part;
            hipLaunchKernelGGL(gemm_nt_bf16_kernel<2>, dim3(grid.x, grid.y, SPLITK_BUF), dim3(256), 0, s, g);
            const size_t n = (size_t)g.M * g.N;
            hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
            return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
        }
        if (few && KMPC_BF16_SMALL)   // short K: 64 x 64 tiles (4x the workgroups), no partials
            hipLaunchKernelGGL(gemm_nt_bf16_kernel<1>, dim3((g.N + 63) / 64, (g.M + 63) / 64), dim3(256), 0, s, g);
        else
            hipLaunchKernelGGL(gemm_nt_bf16_kernel<2>, grid, dim3(256), 0, s, g);
    } else if ((size_t)grid.x * grid.y < 512) {
        dim3 grid64((g.N + 63) / 64, (g.M + 63) / 64);
        // fewer 64 x 64 tiles than CUs (e.g. the 128-wide last encoder layer of BASELINE configs[1]:
        // 4,096 x 128 -> 128 tiles) with a long K: split K in SPLITK slices (4 x the workgroups), the
        // partials summed in slice order by the epilogue kernel (deterministic)
        static_assert(SPLITK >= 2 && SPLITK <= SPLITK_BUF, "split-K slices");
        if (part && (size_t)grid64.x * grid64.y < 256 && g.K >= 128 * SPLITK) {
            g.ksplit = SPLITK;
            g.part = part;
            launch_f32<1, 1>(dim3(grid64.x, grid64.y, SPLITK), s, g);
            if (nparts && g.epi == EPI_NONE) {
                *nparts = SPLITK;
                return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
            }
            const size_t n = (size_t)g.M * g.N;
            hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
            return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
        }
        if (KMPC_GEMM_MID == 21)
            launch_f32<2, 1>(dim3((g.N + 63) / 64, (g.M + 127) / 128), s, g);
        else if (KMPC_GEMM_MID == 12)
            launch_f32<1, 2>(dim3((g.N + 127) / 128, (g.M + 63) / 64), s, g);
        else if (KMPC_GEMM_MID == 22)
            launch_f32<2, 2>(grid, s, g);
        else if (KMPC_GEMM_MID == 42)   // 128 x 128, 8 waves of 32 x 64
            launch_f32<1, 2, 4, 2>(grid, s, g);
        else if (KMPC_GEMM_MID == 44)   // 128 x 128, 16 waves of 32 x 32
            launch_f32<1, 1, 4, 4>(grid, s, g);
        else
            launch_f32<1, 1>(grid64, s, g);
    } else if (KMPC_GEMM_BIG == 42) {   // 128 x 128, 8 waves of 32 x 64
        launch_f32<1, 2, 4, 2>(grid, s, g);
    } else if (KMPC_GEMM_BIG == 44) {   // 128 x 128, 16 waves of 32 x 32
        launch_f32<1, 1, 4, 4>(grid, s, g);
    } else if (KMPC_GEMM_BIG == 82) {   // 256 x 128, 16 waves of 32 x 64
        launch_f32<1, 2, 8, 2>(dim3((g.N + 127) / 128, (g.M + 255) / 256), s, g);
    } else {
        launch_f32<2, 2>(grid, s, g);
    }
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

static GemmArgs linear(int M, int N, int K, const float* A, int lda, const float* W, const float* bias,
                       float* C, int ldc) {
    GemmArgs g = {};
    g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.B = W; g.ldb = K; g.bias = bias;
    g.C = C; g.ldc = ldc; g.epi = EPI_NONE;
    return g;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static int max_width(const kmpc_mlp& m) {
    int w = 0;
    for (int l = 0; l <= m.n_layers; ++l) w = m.dims[l] > w ? m.dims[l] : w;
    return w;
}

size_t rollout_workspace_bytes(const kmpc_rollout_desc* d) {
    if (!d) return 0;
    const size_t B = (size_t)d->B;
    int wmax = d->L;
    const int we = max_width(d->encoder), wd = max_width(d->decoder);
    if (we > wmax) wmax = we;
    if (wd > wmax) wmax = wd;
    size_t bytes = 0;
    bytes += align256(sizeof(float) * (size_t)d->L * d->L);        // K^T
    bytes += align256(sizeof(float) * (size_t)d->L * d->L);        // S^T (LISTA)
    bytes += 2 * align256(sizeof(float) * B * wmax);               // ping-pong activations
    bytes += 2 * align256(sizeof(float) * B * d->L);               // z, c (LISTA) / z next
    const size_t part = B * (size_t)wmax < SPLITK_ELEMS ? B * (size_t)wmax : SPLITK_ELEMS;
    bytes += align256(sizeof(float) * SPLITK_BUF * part);          // split-K partials (small batches)
    bytes += align256((size_t)6 * d->L * (d->L + 32 * (size_t)((d->N + 31) / 32)));   // K^T, D bf16 planes
    bytes += align256(sizeof(float) * (size_t)d->H * d->N * (d->L + 3));   // latent powers W_t, tiled epilogue
    return bytes;
}

// run an MLP on X [B, dims[0]] -> out [B, dims[n]] (only the first `last_cols` outputs of the last
// layer, written with row stride ldo); ping/pong are [B, wmax] scratch buffers.
static int run_mlp(const kmpc_mlp& m, int Bn, const float* X, int ldx, float* out, int ldo,
                   int last_cols, int last_epi, const float* mean, const float* stdv, float* ping,
                   float* pong, int wmax, int bf16, hipStream_t s, float* part, int* last_nparts = nullptr) {
    const float* cur = X;
    int ldc = ldx;
    for (int l = 0; l < m.n_layers; ++l) {
        const bool last = (l == m.n_layers - 1);
        const int nout = last ? last_cols : m.dims[l + 1];
        float* dst = last ? out : ((l & 1) ? pong : ping);
        GemmArgs g = linear(Bn, nout, m.dims[l], cur, ldc, m.weight[l], m.bias[l], dst,
                            last ? ldo : wmax);
        g.bf16 = bf16;
        if (!last) { g.epi = EPI_ACT; g.act = m.act; }
        else if (last_epi == EPI_DESTD) { g.epi = EPI_DESTD; g.mean = mean; g.stdv = stdv; }
        else if (m.last_relu) { g.epi = EPI_ACT; g.act = KMPC_ACT_RELU; }
        int rc = gemm(g, s, part, last ? last_nparts : nullptr);
        if (rc) return rc;
        cur = dst;
        ldc = wmax;
    }
    return KMPC_OK;
}

int rollout_launch(const kmpc_rollout_desc* d, const float* obs, float* yhat, void* ws,
                   size_t ws_bytes, hipStream_t s) {
    if (!d || !obs || !yhat || !d->kmat || !d->mean || !d->std) return KMPC_ERR_INVALID;
    if (d->B < 0 || d->N < 1 || d->H < 1 || d->L < 1 || d->obs < d->N) return KMPC_ERR_INVALID;
    if (d->encoder.n_layers < 1 || d->encoder.n_layers > KMPC_MAX_LAYERS) return KMPC_ERR_INVALID;
    if (d->decoder.n_layers < 1 || d->decoder.n_layers > KMPC_MAX_LAYERS) return KMPC_ERR_INVALID;
    if (d->encoder.dims[0] != d->obs || d->encoder.dims[d->encoder.n_layers] != d->L) return KMPC_ERR_INVALID;
    if (d->decoder.dims[0] != d->L || d->decoder.dims[d->decoder.n_layers] < d->N) return KMPC_ERR_INVALID;
    if (d->model_kind == KMPC_MODEL_LISTA && !d->lista_S) return KMPC_ERR_INVALID;
    if (ws_bytes < rollout_workspace_bytes(d) || (!ws && ws_bytes)) return KMPC_ERR_WORKSPACE;
    if (d->obs_ld < 0 || (d->obs_ld > 0 && d->obs_ld < d->N)) return KMPC_ERR_INVALID;
    if (d->dtype != KMPC_DTYPE_F32 && d->dtype != KMPC_DTYPE_BF16 && d->dtype != KMPC_DTYPE_F32_F32MFMA)
        return KMPC_ERR_INVALID;
    if (d->latent_unfused < KMPC_LATENT_AUTO || d->latent_unfused > KMPC_LATENT_SEQUENTIAL) return KMPC_ERR_INVALID;
    // GemmArgs::bf16: 2 = three bf16 planes (fp32 arithmetic), 1 = bf16 operands, 0 = f32-input MFMA
    const int bf = d->dtype == KMPC_DTYPE_F32 ? KMPC_F32_GEMM : d->dtype == KMPC_DTYPE_BF16 ? 1 : 0;
    if (d->B == 0) return KMPC_OK;
    const int Bn = d->B, L = d->L, N = d->N, H = d->H;
    const int obs_ld = d->obs_ld > 0 ? d->obs_ld : d->obs;
    int wmax = L;
    {
        const int we = max_width(d->encoder), wd = max_width(d->decoder);
        if (we > wmax) wmax = we;
        if (wd > wmax) wmax = wd;
    }
    char* p = (char*)ws;
    float* Kt = (float*)p;   p += align256(sizeof(float) * (size_t)L * L);
    float* St = (float*)p;   p += align256(sizeof(float) * (size_t)L * L);
    float* ping = (float*)p; p += align256(sizeof(float) * (size_t)Bn * wmax);
    float* pong = (float*)p; p += align256(sizeof(float) * (size_t)Bn * wmax);
    float* z0 = (float*)p;   p += align256(sizeof(float) * (size_t)Bn * L);
    float* z1 = (float*)p;   p += align256(sizeof(float) * (size_t)Bn * L);
    float* part = (float*)p;   // split-K partials (gemm(): only M N <= SPLITK_ELEMS outputs are split)
    {
        const size_t pe = (size_t)Bn * wmax < SPLITK_ELEMS ? (size_t)Bn * wmax : SPLITK_ELEMS;
        p += align256(sizeof(float) * SPLITK_BUF * pe);
    }
    __bf16* planes = (__bf16*)p;   // K^T and decoder-row bf16 planes (latent_steps_x3_kernel)
    p += align256((size_t)6 * L * (L + 32 * (size_t)((N + 31) / 32)));
    float* Wpow = (float*)p;      // latent powers [H N, L], then the tiled bias / mean / std [3][H N]
    int rc;
    const bool latpow = KMPC_LATPOW && d->latent_unfused == KMPC_LATENT_AUTO && latent_fusable(d) && Bn >= KMPC_LATPOW_MINB &&
                        !(d->model_kind == KMPC_MODEL_GENERIC && d->norm_fn == KMPC_NORM_BALL);
    // Small batches (the fused 16-row latent loop below KMPC_LAT16_MAXB windows) read K in place and
    // skip the transpose launch (configs[1]: 0.194 -> 0.190 ms per step); at 65,536 windows the
    // in-place read costs the latent loop more than the launch, so K^T stays (A/B).
    const bool lat16 = latent_fusable(d) && (Bn < KMPC_LAT16_MAXB || L <= 16 * KMPC_LAT16_WAVES);
    const bool kdir = lat16 && Bn < KMPC_LAT16_MAXB && !latpow;   // (the powers kernel reads K^T)
    dim3 tg((L + 31) / 32, (L + 31) / 32);
    if (!kdir) hipLaunchKernelGGL(transpose_kernel, tg, dim3(256), 0, s, d->kmat, Kt, L, L);
    if (d->model_kind == KMPC_MODEL_LISTA)
        hipLaunchKernelGGL(transpose_kernel, tg, dim3(256), 0, s, d->lista_S, St, L, L);
    if (hipGetLastError() != hipSuccess) return KMPC_ERR_LAUNCH;

    // ---- encode ----
    int znparts = 0;   // > 0: z0 left as split-K partials for the fused latent loop to sum
    const bool zfuse = KMPC_Z0_FUSE && d->model_kind == KMPC_MODEL_GENERIC && latent_fusable(d) &&
                       d->norm_fn != KMPC_NORM_BALL && !latpow;
    if (d->model_kind == KMPC_MODEL_GENERIC) {
        rc = run_mlp(d->encoder, Bn, obs, obs_ld, z0, L, L, EPI_NONE, nullptr, nullptr, ping, pong, wmax, bf, s, part,
                     zfuse ? &znparts : nullptr);
        if (rc) return rc;
        if (d->norm_fn == KMPC_NORM_BALL)
            hipLaunchKernelGGL(ball_norm_kernel, dim3((Bn + 3) / 4), dim3(256), 0, s, z0, Bn, L);
    } else {
        // c = We(x) (z1 holds c), z = shrink(c); loops: z = shrink(z S + c)   (model.py:200-209)
        rc = run_mlp(d->encoder, Bn, obs, obs_ld, z1, L, L, EPI_NONE, nullptr, nullptr, ping, pong, wmax, bf, s, part);
        if (rc) return rc;
        const size_t n = (size_t)Bn * L;
        hipLaunchKernelGGL(shrink_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, z1, z0, n,
                           d->lista_thresh);
        float* zc = z0;
        float* zn = ping;   // ping is [B, wmax] >= [B, L]
        for (int it = 0; it < d->lista_loops; ++it) {
            GemmArgs g = linear(Bn, L, L, zc, L, St, nullptr, zn, L);
            g.epi = EPI_SHRINK; g.R = z1; g.ldr = L; g.thr = d->lista_thresh; g.bf16 = bf;
            if ((rc = gemm(g, s, part))) return rc;
            float* t = zc; zc = zn; zn = t;
        }
        if (zc != z0 && hipMemcpyAsync(z0, zc, sizeof(float) * n, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return KMPC_ERR_LAUNCH;
    }
    if (hipGetLastError() != hipSuccess) return KMPC_ERR_LAUNCH;
    // znparts > 0: the last encoder layer left z0 UNWRITTEN — its raw split-K partials sit in
    // `part`, and the fused latent loop below rebuilds z0 from them (same slice order and bias).
    // Nothing may be launched between here and that loop that reuses `part` or reads z0
    // (tests/test_rollout_gpu.py::test_fused_z0_is_never_read fills the workspace with NaN).
    if (znparts > 0 && !latent_fusable(d)) return KMPC_ERR_INVALID;   // (zfuse implies fusable)

    // ---- H x (step_latent, decode[:N], destandardize) ----
    if (latpow) {
        const int HN = H * N;
        float* tb = Wpow + (size_t)HN * L;
        float* tm = tb + HN;
        float* ts = tm + HN;
        // W_1 = D_N K^T, W_t = W_{t-1} K^T (float64 chains per row, fp32 W_t)
        hipLaunchKernelGGL(latent_powers_kernel, dim3(N), dim3(64 * ((L + 63) / 64)), sizeof(double) * L, s,
                           d->decoder.weight[0], Kt, L, N, H, Wpow);
        hipLaunchKernelGGL(tile_epilogue_kernel, dim3((HN + 255) / 256), dim3(256), 0, s, H, N, d->decoder.bias[0],
                           d->mean, d->std, tb, tm, ts);
        GemmArgs g = linear(Bn, HN, L, z0, L, Wpow, tb, yhat, HN);   // yhat [B, H, N] = [B, H N]
        g.epi = EPI_DESTD; g.mean = tm; g.stdv = ts; g.bf16 = bf;
        if ((rc = gemm(g, s, part))) return rc;
        return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
    }
    if (latent_fusable(d)) {
        LatentArgs la;
        la.B = Bn; la.L = L; la.N = N; la.H = H; la.z0 = z0; la.Kt = Kt; la.K = d->kmat; la.D = d->decoder.weight[0];
        la.zparts = part; la.nparts = znparts;
        la.zbias = d->encoder.bias[d->encoder.n_layers - 1];
        la.bias = d->decoder.bias[0]; la.mean = d->mean; la.stdv = d->std; la.yhat = yhat;
        la.ball = d->model_kind == KMPC_MODEL_GENERIC && d->norm_fn == KMPC_NORM_BALL;
        // 16 windows per block: twice the blocks of the 32-row kernel for small batches, and one z K
        // column tile per wave at L <= 128 (65,536 windows, L = 128: 263 -> 184 us; at L = 256 the
        // 32-row kernel stays ahead: 1,346 vs 1,575 us)
        if (lat16) {
            const size_t lds = sizeof(float) * 2 * LAT16 * (L + 4);
            if (kdir)
                hipLaunchKernelGGL((latent_steps16_kernel<KMPC_LAT16_WAVES, true>), dim3((Bn + LAT16 - 1) / LAT16),
                                   dim3(64 * KMPC_LAT16_WAVES), lds, s, la);
            else
                hipLaunchKernelGGL((latent_steps16_kernel<KMPC_LAT16_WAVES, false>), dim3((Bn + LAT16 - 1) / LAT16),
                                   dim3(64 * KMPC_LAT16_WAVES), lds, s, la);
            return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
        }
        if (KMPC_LATX3 && bf == 2 && !la.ball && L == 256) {
            const int Dpad = 32 * ((N + 31) / 32);
            __bf16* Kp = planes;
            __bf16* Dp = planes + (size_t)3 * L * L;
            const size_t nk = (size_t)L * L, nd = (size_t)Dpad * L;
            hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, s, Kt, L, L, L, L, Kp);
            hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, s, la.D, N, Dpad, L,
                               L, Dp);
            const size_t lds = sizeof(__bf16) * 3 * LATX3_ROWS * (L + 8);
            hipLaunchKernelGGL((latent_steps_x3_kernel<8, 256>), dim3((Bn + LATX3_ROWS - 1) / LATX3_ROWS), dim3(512), lds,
                               s, la, (const __bf16*)Kp, (const __bf16*)Dp, Dpad);
            return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
        }
        const size_t lds = sizeof(float) * 2 * LAT_ROWS * (L + 4);
        hipLaunchKernelGGL(latent_steps_kernel<KMPC_LAT_WAVES>, dim3((Bn + LAT_ROWS - 1) / LAT_ROWS),
                           dim3(64 * KMPC_LAT_WAVES), lds, s, la);
        return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
    }
    float* zc = z0;
    float* zn = z1;
    for (int k = 0; k < H; ++k) {
        GemmArgs g = linear(Bn, L, L, zc, L, Kt, nullptr, zn, L);
        g.bf16 = bf;
        if ((rc = gemm(g, s, part))) return rc;
        if (d->model_kind == KMPC_MODEL_GENERIC && d->norm_fn == KMPC_NORM_BALL)
            hipLaunchKernelGGL(ball_norm_kernel, dim3((Bn + 3) / 4), dim3(256), 0, s, zn, Bn, L);
        // decoder: hidden layers full width, last layer first-N rows + destandardize into yhat[:, k, :]
        rc = run_mlp(d->decoder, Bn, zn, L, yhat + (size_t)k * N, H * N, N, EPI_DESTD, d->mean, d->std,
                     ping, pong, wmax, bf, s, part);
        if (rc) return rc;
        float* t = zc; zc = zn; zn = t;
    }
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

// z = f32((y - mean) / std): float64 arithmetic, one rounding to float32 (data_finance.py:243-260, 331)
__global__ void standardize_kernel(int T, int N, const double* y, const double* mean, const double* stdv,
                                   float* z) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)T * N) return;
    const int n = (int)(i % N);
    z[i] = (float)((y[i] - mean[n]) / stdv[n]);
}

int standardize_launch(int T, int N, const double* y, const double* mean, const double* stdv, float* z,
                       hipStream_t s) {
    const size_t n = (size_t)T * N;
    if (n == 0) return KMPC_OK;
    hipLaunchKernelGGL(standardize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, T, N, y, mean,
                       stdv, z);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

}  // namespace kmpc
