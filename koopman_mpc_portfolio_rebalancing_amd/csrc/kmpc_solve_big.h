#pragma once
// kmpc_solve_big.h — batched MPC solve for large windows (replaces solve_mpc_log_utility,
// mpc.py:27-117, for N > 256 assets or H > 10 periods): the same program and the same Mehrotra
// predictor-corrector interior point as ipm_kernel / oracle/kmpc_oracle.c (same reductions,
// refinement rule, step rule, status and fallback), laid out for windows whose state does not fit
// one CU.
//
// Why a second kernel: a window's IPM state is ~17 arrays of H x N doubles (1.4 MB at N = 500,
// H = 20, BASELINE configs[4]); ipm_kernel keeps it in registers (one asset per lane, every period
// in VGPRs) and past 128 assets or 10 periods spills it to scratch. Here the state lives in a
// per-window slab of the caller's workspace, [array][t][i] with the assets contiguous, so every
// access is one coalesced wave load; each phase streams only the arrays it needs. The slack
// reciprocals are recomputed from the state where they are used; the s-elimination coefficients
// (P, bma P) are written once per iteration by the factor pass and read by the Newton passes.
// The solve is bound by that HBM / Infinity-Cache stream.
//
// Layout: one workgroup per window, one asset per thread (blockDim = 64 ceil(N / 64) <= 1024), a
// persistent grid of slots_for(B, N) <= 768 workgroups walks the windows (workspace = slots x slab).
// Period loops are runtime loops with scalar carries (no per-period register arrays: small code,
// bounded registers); per-period block sums are wave butterflies (permlane / DPP) per period into
// LDS slots, then one pass over the waves. Per-period scalars, the Schur matrix and the reduction
// slots sit in LDS (~60 KB).
//
// Schur (Woodbury) matrix on the matrix cores. G = I' + sum_i Z_i^T Q_i^{-1} Z_i with Q_i the
// per-asset tridiagonal (in t) and Z_i = [v_t | a_t | 1_t] columns (index j = 3t + type, types
// v, a, 1). The inverse of a tridiagonal is semiseparable: Q^{-1}[r][c] = dq_c prod_{r<k<=c} Lr_k =
// g_r beta_c (r <= c) with g = 1 / pi, beta = dq pi, pi_t = prod_{k<=t} Lr_k. So for j <= l (index
// order) every entry of an asset's contribution is a product Lgen_i[j] * Rgen_i[l], and the sum over
// assets is the GEMM Lgen^T Rgen: v_mfma_f64_16x16x4_f64 with the assets as the K dimension (exact
// f64 products, no cross-lane reduction). The one entry whose product form cancels
// catastrophically, (v_t, v_t), is summed directly. Lr is clamped at 1e-14 (pi stays in the normal
// range over 21 periods) and pi is centred (pi * 2^(-e/2), pi_H ~ 2^e); the clamp changes Q^{-1}
// entries only where they are already below 1e-14 of the diagonal, i.e. at f64 rounding level.
#include "kmpc_solve_kernel.h"

namespace kmpc {
namespace big {

constexpr int KP = 64;             // padded Schur width (3 HM <= 63)
constexpr int NWX = 16;            // max waves per window (1024 threads)
// G / L in LDS: packed lower triangle (row r at r (r + 1) / 2; every access is on or below the
// diagonal), 16.3 KB instead of the 33.3 KB of a full row-stride-65 square — with the reduction
// slots sized to the block's waves, a 512-thread window's LDS drops from 56.4 to 39.8 KB, room for
// four windows per CU (KMPC_BIG_TRI 0: the square, dev A/B). Same speed at two
// per CU (C5: 64.8 vs 64.4 ms). More windows per CU do not pay: the registers are the limit, not
// the LDS — three per CU (<= 80 VGPRs) took C5 from 64.8 to 117.6 ms, four (64 VGPRs, 524 B of
// scratch per lane) to 151.7 ms, with spill reloads inside the load-latency-bound sweeps; one per
// CU 79.1 ms (r05, tools/ab_c5.sh)
#ifndef KMPC_BIG_TRI
#define KMPC_BIG_TRI 1
#endif
constexpr int LDG = 65;            // (square layout) row stride: conflict-free row and column reads
constexpr int G_DOUBLES = KMPC_BIG_TRI ? KP * (KP + 1) / 2 : KP * LDG;
__device__ __forceinline__ int gi(int r, int k) { return KMPC_BIG_TRI ? ((r * (r + 1)) >> 1) + k : r * LDG + k; }
// windows in flight = workspace slabs: two workgroups per CU for the >= 512-thread blocks (the
// slab stream is HBM-bound there: 768 slots measured -9% at N = 300, H = 15, equal at N = 500),
// three (the LDS limit) for windows of <= 256 assets, which are latency-bound (N = 100, H = 20:
// 512 -> 768 slots +17%, measured r02)
#ifndef KMPC_BIG_MAX_SLOTS
#define KMPC_BIG_MAX_SLOTS 512
#endif
#ifndef KMPC_BIG_MAX_SLOTS_SMALL
#define KMPC_BIG_MAX_SLOTS_SMALL 768
#endif
// 512-thread windows (256 < N <= 512): two per CU (see KMPC_BIG_TRI; dev A/B with KMPC_BIG_WPE)
#ifndef KMPC_BIG_MAX_SLOTS_MID
#define KMPC_BIG_MAX_SLOTS_MID 512
#endif
constexpr int MAX_SLOTS = KMPC_BIG_MAX_SLOTS;
constexpr int MAX_SLOTS_SMALL = KMPC_BIG_MAX_SLOTS_SMALL;
constexpr int MAX_SLOTS_MID = KMPC_BIG_MAX_SLOTS_MID;
__host__ __device__ inline int slots_for(int B, int N) {
    const int cap = N <= 256 ? MAX_SLOTS_SMALL : (N <= 512 ? MAX_SLOTS_MID : MAX_SLOTS);
    return B < cap ? B : cap;
}
constexpr double LR_FLOOR = 1e-14;
// the Gram generator and Newton back-substitution / Zq sweeps: loads two periods ahead (1) or one
// (0) — C5 64.7 -> 61.5 ms, N = 500 / H = 10 57.7 -> 55.7, N = 300 / H = 15 55.7 -> 53.6 (r05,
// tools/ab_c5.sh, tools/ab_big.sh; same iterates)
#ifndef KMPC_BIG_PF2S
#define KMPC_BIG_PF2S 1
#endif
#ifndef KMPC_BIG_PF3S   // ... three periods ahead (dev A/B: C5 61.8 -> 64.9 ms, every shape slower; r05)
#define KMPC_BIG_PF3S 0
#endif
#ifndef KMPC_BIG_WPE   // waves per SIMD of the >= 512-thread kernels: 2 workgroups per CU
#define KMPC_BIG_WPE 4
#endif

typedef double d4 __attribute__((ext_vector_type(4)));

// per-(t, i) arrays of a window's slab (assets contiguous)
// (P and BP = bma P are this iteration's s-elimination coefficients, written by the factor pass
// so that the Newton passes read 1-2 arrays instead of recomputing them from the whole state;
// DS holds P bs, the s right-hand side already scaled by P; RC* hold the corrector's targets
// without the centring term -smu, which every reader subtracts)
enum : int { A_W, A_S, A_L1, A_L2, A_L3, A_M, A_LR, A_IDD, A_RC1, A_RC2, A_RC3, A_DW, A_DS,
             A_BW, A_BS, A_X, A_Y, A_R0, A_R1, A_P, A_BP, N_ARR };

__host__ __device__ inline size_t slab_doubles(int HM, int NP) {
    return (size_t)N_ARR * HM * NP + 2 * (size_t)KP * NP;
}

struct BigArgs {
    SolveArgs s;
    double* ws;      // slots x slab doubles
    size_t slab;     // doubles per slab
    int NP;          // padded asset count (blockDim)
};

// LDS of the fused solves: the raw Gram's v-columns, c_t = sqrt(rho_t) px_t, per-wave px partials
template <int HM, int NW = NWX>
constexpr int fx_doubles() { return KP * HM + HM + NW * HM; }

// (allocated as LDS of bs_bytes<HM>(waves): red is the last member and only the block's waves'
// rows of it exist)
template <int HM>
struct BigShared {
    double G[G_DOUBLES];         // Schur matrix (lower triangle), then L (unit lower, strictly below)
    double gid[KP];              // 1 / D of G = L D L^T
    double q[KP];                // Schur solution (period-major index 3t + type)
    double tot[KP];              // block-reduction totals (slots < 3 HM <= 63)
    double sc[2][NWX][2];        // per-wave partials of scalar reductions (alternating)
    double den[HM], iden[HM], rp[HM], rg4[HM], z4[HM], iz4[HM], l4[HM], nu[HM], rho[HM], sr[HM];
    double rc4[HM], b5[HM], b6[HM], lb5[HM], lb6[HM], dnu[HM], dz4[HM], dl4[HM];
    double rw[HM], best_rw[HM], best_l1[HM], px[HM], adw[HM], sds[HM], sdw[HM];
    double isp1[HM];   // 1 / (1 + gamma SP), SP = sum_i P (rho = gamma isp1)
    double pxa[HM];    // the direction's px summed over its solves: ds = P (DS - rho pxa), sum_i ds = pxa isp1
    double lsc[HM];    // log S_t of a period run on R / S_t (tiny gross returns), else 0
    int flag;
    double red[NWX][KP];         // per-wave partial slots of a period reduction (rows < waves)
};
// LDS doubles of a BigShared whose blocks have nw waves (the red rows past nw cut off)
template <int HM>
constexpr int bs_doubles(int nw) { return (int)((sizeof(BigShared<HM>) - sizeof(double) * (NWX - nw) * KP + 7) / 8); }

// state of one (t, i) with its slack-derived quantities (recomputed, never stored)
struct St {
    double w, s, d, l1, l2, l3, m;
    double iw, iz2, iz3, P, bma;
};

// 1 / x to ~1 ulp: v_rcp_f64 and two Newton steps (no division sequence)
__device__ __forceinline__ double rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    r = fma(r, fma(-x, r, 1.0), r);
    return r;
}

// One slab element of this thread's asset, read and written through the window's buffer
// descriptor: the lane's byte offset (one VGPR, shared by every array) plus a wave-uniform byte
// offset per (array, period) — instead of a 64-bit VGPR address per array, which the compiler
// keeps live across the whole iteration (register pressure that spilled at 2 workgroups per CU).
struct Ref {
    __amdgpu_buffer_rsrc_t rs;
    unsigned vo, so;
    __device__ __forceinline__ operator double() const {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0));
    }
    __device__ __forceinline__ const Ref& operator=(double v) const {
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0)), v), rs, vo, so, 0);
        return *this;
    }
    __device__ __forceinline__ const Ref& operator+=(double v) const { return *this = (double)*this + v; }
};

// A float32-stored slab element (the first half of its array's rows, like the M array's R): the
// factor-only arrays under KMPC_BIG_F32FAC (dev A/B: half the bytes of the arrays the Newton
// sweeps read most; the float64 refinement against the unreduced system restores the direction)
struct Ref32 {
    __amdgpu_buffer_rsrc_t rs;
    unsigned vo, so;
    __device__ __forceinline__ operator double() const {
        return (double)__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0));
    }
    __device__ __forceinline__ const Ref32& operator=(double v) const {
        __builtin_amdgcn_raw_buffer_store_b32(
            __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0)), (float)v), rs, vo, so, 0);
        return *this;
    }
};
#ifndef KMPC_BIG_F32FAC
#define KMPC_BIG_F32FAC 0
#endif

template <int HM, int FL>
struct Win {
    const SolveArgs& a;
    BigShared<HM>& sh;
    double* g;       // this window's slab
    int N, H, NP, nw, i;
    bool act;        // this thread's asset exists
    Case<FL> cs;
    double tau, isig, irsig, cs_c, wpi;
    int sbuf;
    __amdgpu_buffer_rsrc_t rs;   // the slab (wave-uniform base and size)
    unsigned vo;                 // i * 8
    // fused solves (>= 512-thread blocks): LDS block [Gv: KP x HM][cv: HM][pxr: NWX x HM] (fx_doubles);
    // nullptr: the unfused right-hand-side sweep with its own px reduction
    double* fx;
    __device__ __forceinline__ double* gv() const { return fx; }
    __device__ __forceinline__ double* cv() const { return fx + KP * HM; }
    __device__ __forceinline__ double* pxr() const { return fx + KP * HM + HM; }


    __device__ __forceinline__ void bind(size_t slab_doubles) {
        rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, (int)(slab_doubles * sizeof(double)), 0x00020000);
        vo = (unsigned)i * 8u;
    }

    __device__ __forceinline__ bool hw() const { return cs.hw; }
    __device__ __forceinline__ bool hs() const { return cs.hs; }
    __device__ __forceinline__ bool ht() const { return cs.ht; }
    __device__ __forceinline__ Ref at(int arr, int t) const { return Ref{rs, vo, (unsigned)((arr * HM + t) * NP) * 8u}; }
    // the factor-only arrays (Lr, 1/Dd, P, BP): float32 under KMPC_BIG_F32FAC
#if KMPC_BIG_F32FAC
    __device__ __forceinline__ Ref32 fat(int arr, int t) const {
        return Ref32{rs, vo >> 1, (unsigned)(arr * HM * NP) * 8u + (unsigned)(t * NP) * 4u};
    }
#else
    __device__ __forceinline__ Ref fat(int arr, int t) const { return at(arr, t); }
#endif
    // m = R - 1 of (t, i): the slab keeps the float32 R (exact: (double)R - 1 is the kernels' m) in
    // the first half of the M array's rows — half the bytes of the most-read input array
    __device__ __forceinline__ double mload(int t) const {
        const unsigned so = (unsigned)(A_M * HM * NP) * 8u + (unsigned)(t * NP) * 4u;
        return (double)__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo >> 1, so, 0)) - 1.0;
    }
    __device__ __forceinline__ double rload(int t) const {   // the stored float32 R itself
        const unsigned so = (unsigned)(A_M * HM * NP) * 8u + (unsigned)(t * NP) * 4u;
        return (double)__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo >> 1, so, 0));
    }
    __device__ __forceinline__ void mstore(int t, float r) const {
        const unsigned so = (unsigned)(A_M * HM * NP) * 8u + (unsigned)(t * NP) * 4u;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b32(rs, 0u, 0u, 0)), r),
                                              rs, vo >> 1, so, 0);
    }
    __device__ __forceinline__ double* lg(int j) const { return g + (size_t)N_ARR * HM * NP + (size_t)j * NP; }
    __device__ __forceinline__ double* rg(int j) const { return g + (size_t)N_ARR * HM * NP + (size_t)(KP + j) * NP; }
    __device__ __forceinline__ double wprev(int t) const { return t ? at(A_W, t - 1) : wpi; }

    // the stored state of (t, i) and the direction / targets the step, update and corrector
    // sweeps read with it: loaded one period ahead of its use, so that a wave keeps the next
    // period's loads in flight while it computes this one (the sweeps are load-latency bound)
    struct Pre {
        double w, s, l1, l2, l3, m, dw, ds, rc1, rc2, rc3, r0, r1;
    };
    // dir: + DW, DS; rc: + RC1..RC3; rr: + R0, R1 (a refinement pass's right-hand side)
    __device__ __forceinline__ Pre pre(int t, bool dir = true, bool rc = true, bool rr = false) const {
        Pre p{};
        p.w = at(A_W, t);
        p.s = at(A_S, t);
        p.l1 = at(A_L1, t);
        p.l2 = at(A_L2, t);
        p.l3 = at(A_L3, t);
        p.m = mload(t);
        if (dir) { p.dw = at(A_DW, t); p.ds = at(A_DS, t); }
        if (rc) { p.rc1 = at(A_RC1, t); p.rc2 = at(A_RC2, t); p.rc3 = at(A_RC3, t); }
        if (rr) { p.r0 = at(A_R0, t); p.r1 = at(A_R1, t); }
        return p;
    }
    __device__ __forceinline__ St st(const Pre& p, double wp) const {
        St e;
        e.w = p.w;
        e.s = p.s;
        e.l1 = p.l1;
        e.l2 = p.l2;
        e.l3 = p.l3;
        e.m = p.m;
        return derive(e, wp);
    }
    __device__ __forceinline__ St st(int t, double wp) const {
        St e;
        e.w = at(A_W, t);
        e.s = at(A_S, t);
        e.l1 = at(A_L1, t);
        e.l2 = at(A_L2, t);
        e.l3 = at(A_L3, t);
        e.m = mload(t);
        return derive(e, wp);
    }
    __device__ __forceinline__ St derive(St e, double wp) const {
        e.d = e.w - wp;
        e.iw = hw() ? rcp(e.w) : 0.0;
        if (hs()) {
            e.iz2 = rcp(e.s - e.d);
            e.iz3 = rcp(e.s + e.d);
            const double al = e.l2 * e.iz2, be = e.l3 * e.iz3;
            e.P = rcp(al + be);
            e.bma = be - al;
        } else {
            e.iz2 = e.iz3 = e.P = e.bma = 0.0;
        }
        return e;
    }
    // dual residual rows (1)-(2) at period t (ipm_kernel dual_residual); l2n / l3n of period t + 1
    __device__ __forceinline__ void dres(int t, const St& e, double l2n, double l3n, double& rdw, double& rds) const {
        rdw = -e.m * sh.iden[t] * isig - (e.l1 + (e.l3 - e.l2) - (l3n - l2n)) + sh.nu[t];
        rds = hs() ? cs_c - (e.l2 + e.l3 - sh.l4[t]) : 0.0;
    }
    // multipliers of a direction (complementarity rows with targets rc)
    __device__ __forceinline__ void ddirs(const St& e, double rc1, double rc2, double rc3, double dw, double ds,
                                          double dd, double& dl1, double& dl2, double& dl3) const {
        dl1 = hw() ? (-rc1 - e.l1 * dw) * e.iw : 0.0;
        dl2 = hs() ? (-rc2 - e.l2 * (ds - dd)) * e.iz2 : 0.0;
        dl3 = hs() ? (-rc3 - e.l3 * (ds + dd)) * e.iz3 : 0.0;
    }
    // ds of (t, i) from the stored DS (P times the back-substituted s right-hand sides, summed over
    // the direction's solves): ds = DS - P rho pxa — the s elimination's last step, never stored
    __device__ __forceinline__ double dsv(int t, const St& e, double DSp) const {
        return hs() ? DSp - e.P * (sh.rho[t] * sh.pxa[t]) : 0.0;
    }
    __device__ __forceinline__ double alpha(int t, double m) const { return m * sh.iden[t] * irsig; }
    __device__ __forceinline__ double eps(int t, const St& e) const { return ht() ? sh.sr[t] * e.bma * e.P : 0.0; }
    __device__ __forceinline__ double epsa(int t) const { return ht() ? sh.sr[t] * fat(A_BP, t) : 0.0; }

    // ---- reductions ----
    // wave total of v into this wave's partial slot j (every lane of the wave must call)
    __device__ __forceinline__ void slot(int j, double v) const {
        v = wave_sum(v);
        if ((threadIdx.x & (WAVE - 1)) == 0) sh.red[threadIdx.x / WAVE][j] = v;
    }
    // block totals of slots 0..n-1 -> sh.tot
    __device__ __forceinline__ void finish(int n) const {
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            double s = sh.red[0][j];
            for (int q = 1; q < nw; ++q) s += sh.red[q][j];
            sh.tot[j] = s;
        }
        __syncthreads();
    }
    // block sum of s and block max of mx (one barrier)
    __device__ __forceinline__ void sum_max(double& s, double& mx) {
        s = wave_sum(s);
        mx = wave_max(mx);
        const int wv = threadIdx.x / WAVE;
        if ((threadIdx.x & (WAVE - 1)) == 0) { sh.sc[sbuf][wv][0] = s; sh.sc[sbuf][wv][1] = mx; }
        __syncthreads();
        double S = sh.sc[sbuf][0][0], MX = sh.sc[sbuf][0][1];
        for (int q = 1; q < nw; ++q) { S += sh.sc[sbuf][q][0]; MX = fmax(MX, sh.sc[sbuf][q][1]); }
        s = S;
        mx = MX;
        sbuf ^= 1;
    }
    // block max of a and of b (one barrier)
    __device__ __forceinline__ void max_max(double& a, double& b) {
        a = wave_max(a);
        b = wave_max(b);
        const int wv = threadIdx.x / WAVE;
        if ((threadIdx.x & (WAVE - 1)) == 0) { sh.sc[sbuf][wv][0] = a; sh.sc[sbuf][wv][1] = b; }
        __syncthreads();
        double A = sh.sc[sbuf][0][0], B = sh.sc[sbuf][0][1];
        for (int q = 1; q < nw; ++q) { A = fmax(A, sh.sc[sbuf][q][0]); B = fmax(B, sh.sc[sbuf][q][1]); }
        a = A;
        b = B;
        sbuf ^= 1;
    }
    // the predictor's complementarity targets rc = x l of (t, i), from the state (never stored:
    // three arrays less to write and to read back in the predictor's sweeps)
    __device__ __forceinline__ void xl(const St& e, double& r1, double& r2, double& r3) const {
        r1 = hw() ? e.w * e.l1 : 0.0;
        r2 = hs() ? (e.s - e.d) * e.l2 : 0.0;
        r3 = hs() ? (e.s + e.d) * e.l3 : 0.0;
    }
    // corrector targets of (t, i) from the affine direction: b = x l + dx dl_aff written to RC*,
    // b - smu returned (ipm_kernel's corrector rows)
    __device__ __forceinline__ void cbase(const St& e, double dw, double ds, double dd, double& b1, double& b2,
                                          double& b3, double& dl1, double& dl2, double& dl3) const {
        double rc1, rc2, rc3;
        xl(e, rc1, rc2, rc3);
        ddirs(e, rc1, rc2, rc3, dw, ds, dd, dl1, dl2, dl3);
        b1 = hw() ? rc1 + dw * dl1 : 0.0;
        b2 = hs() ? rc2 + (ds - dd) * dl2 : 0.0;
        b3 = hs() ? rc3 + (ds + dd) * dl3 : 0.0;
    }
    __device__ __forceinline__ void corr_rc(int t, const St& e, const Pre& p, double dd, double smu,
                                            double& r1, double& r2, double& r3) const {
        double b1, b2, b3, dl1, dl2, dl3;
        cbase(e, p.dw, dsv(t, e, p.ds), dd, b1, b2, b3, dl1, dl2, dl3);
        if (hw()) at(A_RC1, t) = b1;
        if (hs()) { at(A_RC2, t) = b2; at(A_RC3, t) = b3; }
        r1 = hw() ? b1 - smu : 0.0;
        r2 = hs() ? b2 - smu : 0.0;
        r3 = hs() ? b3 - smu : 0.0;
    }
};

// period owners: den, iden, rp, rg4, rc4, iz4, rw from the slot totals of (R - 1).w, 1'w, 1's
template <int HM, int FL>
__device__ __forceinline__ void sums_owner(Win<HM, FL>& W) {
    auto& sh = W.sh;
    if (threadIdx.x < HM) {
        const int t = threadIdx.x;
        const bool on = t < W.H;
        const double mw = on ? sh.tot[3 * t] : 0.0, sw = on ? sh.tot[3 * t + 1] : 0.0, ss = on ? sh.tot[3 * t + 2] : 0.0;
        sh.rw[t] = sw + mw;   // sum_i exp(yhat) w = sum w + sum expm1(yhat) w
        sh.den[t] = 1.0 + mw;
        sh.iden[t] = 1.0 / (1.0 + mw);
        sh.rp[t] = on ? sw - 1.0 : 0.0;
        sh.rg4[t] = (W.ht() && on) ? W.tau - ss - sh.z4[t] : 0.0;
        sh.rc4[t] = (W.ht() && on) ? sh.z4[t] * sh.l4[t] : 0.0;
        sh.iz4[t] = 1.0 / sh.z4[t];
        if (t == 0) sh.flag = 0;
    }
    __syncthreads();
}

// (1) period sums R.w, 1'w, 1's -> den, iden, rp, rg4, rc4, iz4, rw (period owners)
template <int HM, int FL>
__device__ __forceinline__ void ph_sums(Win<HM, FL>& W) {
    for (int t = 0; t < W.H; ++t) {
        double mw = 0.0, w = 0.0, s = 0.0;
        if (W.act) {
            w = W.at(A_W, t);
            mw = W.mload(t) * w;
            s = W.at(A_S, t);
        }
        W.slot(3 * t, mw);
        W.slot(3 * t + 1, w);
        W.slot(3 * t + 2, s);
    }
    W.finish(3 * W.H);
    sums_owner(W);
}

// (2) dual residual and complementarity sums, per-asset LDL^T of Q (LR, IDD), targets rc (RC*),
// sum_i P per period -> rho, sr (owners). Returns mu (unscaled block sum) and rd (block max).
template <int HM, int FL>
__device__ __forceinline__ void ph_factor(Win<HM, FL>& W, double& mu_l, double& rd) {
    auto& sh = W.sh;
    const bool hw = W.hw(), hs = W.hs(), ht = W.ht();
    const int H = W.H;
    mu_l = 0.0;
    rd = 0.0;
    bool ok = true;
    St cur{};
    double W1c = 0.0, Ec = 0.0, pi = 0.0, lr = 0.0;
    double pm = 1.0;   // prod_{1<=k<=t} max(Lr_k, LR_FLOOR) = pm 2^pe (renormalised: no underflow)
    int pe = 0;
    typename Win<HM, FL>::Pre pn{};   // the state of period t + 1, loaded at step t - 1
    if (W.act) {
        cur = W.st(0, W.wpi);
        if (H > 1) pn = W.pre(1, false, false);
        W1c = cur.l1 * cur.iw;
        Ec = hs ? 4.0 * (cur.l2 * cur.iz2) * (cur.l3 * cur.iz3) * cur.P : 0.0;
        pi = W1c + Ec;
    }
    for (int t = 0; t < H; ++t) {
        double P = 0.0;
        if (W.act) {
            const bool nx = t + 1 < H;
            St nxt = cur;
            double W1n = 0.0, En = 0.0;
            if (nx) {
                nxt = W.st(pn, cur.w);
                if (t + 2 < H) pn = W.pre(t + 2, false, false);
                W1n = nxt.l1 * nxt.iw;
                En = hs ? 4.0 * (nxt.l2 * nxt.iz2) * (nxt.l3 * nxt.iz3) * nxt.P : 0.0;
            }
            double rdw, rds;
            W.dres(t, cur, nx ? nxt.l2 : 0.0, nx ? nxt.l3 : 0.0, rdw, rds);
            const double r1 = hw ? cur.w * cur.l1 : 0.0;
            const double r2 = hs ? (cur.s - cur.d) * cur.l2 : 0.0;
            const double r3 = hs ? (cur.s + cur.d) * cur.l3 : 0.0;
            mu_l += r1 + r2 + r3;
            rd = fmax(rd, fmax(fabs(rdw), fabs(rds)));
            P = cur.P;
            W.fat(A_P, t) = cur.P;
            W.fat(A_BP, t) = cur.bma * cur.P;
            // LDL^T of Q = diag(W1) + D^T E D, cancellation-free pivots
            const double Dd = pi + (nx ? En : 0.0);
            ok = ok && (Dd > 0.0) && (Dd < 1e300);
            const double iDd = rcp(Dd);
            W.fat(A_IDD, t) = iDd;
            W.fat(A_LR, t) = lr;
            if (t) {
                int ex;
                pm = frexp(pm * fmax(lr, LR_FLOOR), &ex);
                pe += ex;
            }
            if (nx) {
                lr = En * iDd;
                pi = W1n + lr * pi;
            }
            cur = nxt;
        }
        W.slot(t, P);
    }
    if (W.act) {
        // the Schur generators' centred pi_{H-1} (ph_gram runs its pi recursion backward from it):
        // pi_{H-1} = m 2^e, m in [0.5, 1) -> pi_{H-1} 2^-(e/2); X is free until the Newton solves
        int e2;
        const double m = frexp(pm, &e2);
        const int e = pe + e2;
        W.at(A_X, 0) = ldexp(m, e - e / 2);
    }
    W.finish(H);
    if (threadIdx.x < HM) {
        const int t = threadIdx.x;
        const double st = t < H ? sh.tot[t] : 0.0;
        const double ga = (ht && t < H) ? sh.l4[t] / sh.z4[t] : 0.0;
        const double i1 = 1.0 / (1.0 + ga * st);
        sh.rho[t] = (ht && t < H) ? ga * i1 : 0.0;
        sh.sr[t] = sqrt(sh.rho[t]);
        sh.isp1[t] = i1;
    }
    if (!ok) sh.flag = 1;
    W.sum_max(mu_l, rd);   // (its barrier publishes rho, sr and flag)
}

// W (t < tw) of the current iterate to the output, and the per-period ||w_t - w_{t-1}||_1 and R.w
// of this iterate (its objective is evaluated after the loop). (Folding this sweep into the update
// or factor sweeps — w double-buffered in the slab, or W written by the update that replaces the
// best iterate, the norm as an extra reduction slot — measured slower on C5: 61.7 -> 64.2 / 62.4 ms,
// 60 -> 74 / 63 spilled VGPRs in the load-latency-bound sweeps; r06, commit 518ee52)
template <int HM, int FL>
__device__ __forceinline__ void ph_record(Win<HM, FL>& W, double* wout, int tw) {
    auto& sh = W.sh;
    double wprev = W.wpi, wn = 0.0;
    if (W.act) wn = W.at(A_W, 0);
    for (int t = 0; t < W.H; ++t) {
        double v = 0.0;
        if (W.act) {
            const double w = wn;
            if (t + 1 < W.H) wn = W.at(A_W, t + 1);
            if (t < tw) wout[t * W.N + W.i] = w;
            v = fabs(w - wprev);
            wprev = w;
        }
        W.slot(t, v);
    }
    W.finish(W.H);
    if (threadIdx.x < HM) {
        sh.best_rw[threadIdx.x] = sh.rw[threadIdx.x];
        sh.best_l1[threadIdx.x] = (int)threadIdx.x < W.H ? sh.tot[threadIdx.x] : 0.0;
    }
}

// (3) Schur matrix: generators (slab) and the direct (v_t, v_t) sums, MFMA tiles of Lgen^T Rgen
template <int HM, int FL>
__device__ __forceinline__ void ph_gram(Win<HM, FL>& W) {
    auto& sh = W.sh;
    const int H = W.H, K3 = 3 * H, N4 = (W.N + 3) & ~3;
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    // One backward sweep: dq_t = 1/Dd_t + Lr_{t+1}^2 dq_{t+1} (diagonal of Q^{-1}), the centred
    // pi_t = pi_{t+1} / max(Lr_{t+1}, floor) from ph_factor's pi_{H-1} (X[0]), g = 1 / pi,
    // beta = dq pi. The v-type generators need period t-1's g / beta: period t's are written at
    // step t-1 (and period 0's after the loop), as is the direct (v_t, v_t) sum.
    {
        struct Gv { double idd, lr, m, bp; };
        auto ldG = [&](int t) {
            Gv v;
            v.idd = W.fat(A_IDD, t);
            v.lr = W.fat(A_LR, t);
            v.m = W.mload(t);
            v.bp = W.ht() ? (double)W.fat(A_BP, t) : 0.0;
            return v;
        };
        Gv gnx{}, gnx2{}, gnx3{};
        double pi = 1.0;
        if (W.act) {
            pi = W.at(A_X, 0);
            gnx = ldG(H - 1);
            if (KMPC_BIG_PF2S && H > 1) gnx2 = ldG(H - 2);
            if (KMPC_BIG_PF3S && H > 2) gnx3 = ldG(H - 3);
        }
        double dqn = 0.0, lrn = 0.0, gn = 0.0, bn = 0.0, epn = 0.0;
        for (int t = H - 1; t >= 0; --t) {
            double vvn = 0.0;
            if (W.act) {
                const Gv c = gnx;
                if (KMPC_BIG_PF3S) {
                    gnx = gnx2;
                    gnx2 = gnx3;
                    if (t > 2) gnx3 = ldG(t - 3);
                } else if (KMPC_BIG_PF2S) {
                    gnx = gnx2;
                    if (t > 1) gnx2 = ldG(t - 2);
                } else if (t > 0) {
                    gnx = ldG(t - 1);
                }
                const double idd = c.idd, lr = c.lr;
                const double dq = idd + lrn * lrn * dqn;
                if (t + 1 < H) pi *= rcp(fmax(lrn, LR_FLOOR));
                const double al = W.alpha(t, c.m), ep = W.ht() ? sh.sr[t] * c.bp : 0.0;
                const double gt = rcp(pi), bt = dq * pi;
                W.lg(3 * t + 1)[W.i] = al * gt;
                W.lg(3 * t + 2)[W.i] = gt;
                W.rg(3 * t + 1)[W.i] = al * bt;
                W.rg(3 * t + 2)[W.i] = bt;
                if (t + 1 < H) {
                    W.lg(3 * t + 3)[W.i] = epn * (gn - gt);
                    W.rg(3 * t + 3)[W.i] = epn * (bn - bt);
                    // (v_{t+1}, v_{t+1}) = eps^2 (Qi[t+1][t+1] - 2 Qi[t][t+1] + Qi[t][t]), Qi[t][t+1] = Lr_{t+1} dq_{t+1}
                    vvn = epn * epn * (dqn - 2.0 * lrn * dqn + dq);
                }
                if (t == 0) {
                    W.lg(0)[W.i] = ep * gt;
                    W.rg(0)[W.i] = ep * bt;
                }
                dqn = dq;
                lrn = lr;
                gn = gt;
                bn = bt;
                epn = ep;
            } else if (W.i < N4) {
                // padding assets of the last K group of the MFMA loop contribute zeros
                for (int ty = 0; ty < 3; ++ty) { W.lg(3 * t + ty)[W.i] = 0.0; W.rg(3 * t + ty)[W.i] = 0.0; }
            }
            if (t + 1 < H) W.slot(t + 1, vvn);
        }
        W.slot(0, W.act ? epn * epn * dqn : 0.0);   // (v_0, v_0) = eps_0^2 dq_0
    }
    W.finish(H);   // (its barriers also publish the generators to the workgroup)
    if ((int)threadIdx.x < H) sh.G[gi(3 * threadIdx.x, 3 * threadIdx.x)] = sh.tot[threadIdx.x];
#ifndef KMPC_BIG_GRAM_SUPER
#define KMPC_BIG_GRAM_SUPER 1
#endif
    const int NB = (K3 + 15) / 16;
    auto store_tile = [&](int I, int J, const d4& acc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = 16 * I + (lane >> 4) + 4 * r, l = 16 * J + (lane & 15);
            if (j < K3 && l < K3) {
                const int tj = j / 3, tyj = j - 3 * tj, tl = l / 3, tyl = l - 3 * tl;
                const bool use = tj < tl || (tj == tl && tyj <= tyl && !(tyj == 0 && tyl == 0));
                if (use) sh.G[gi(l, j)] = acc[r];
            }
        }
    };
    if (KMPC_BIG_GRAM_SUPER) {
        // 32-row super-blocks: one wave per super tile (I2 <= J2) computes its 2 x 2 tiles (three on
        // the diagonal) from two L and two R generator rows per k-step — each generator row is read
        // by half as many waves as with one tile per wave (the generator stream is HBM traffic)
        const int SB = (NB + 1) / 2, nst = SB * (SB + 1) / 2;
        for (int q = wv; q < nst; q += W.nw) {
            int I2 = 0, J2 = 0, rem = q;
            for (int bi = 0; bi < SB; ++bi) {
                const int n = SB - bi;
                if (rem < n) { I2 = bi; J2 = bi + rem; break; }
                rem -= n;
            }
            const bool i1 = 2 * I2 + 1 < NB, j1 = 2 * J2 + 1 < NB;   // second blocks in range
            const bool t01 = j1, t10 = i1 && I2 != J2, t11 = i1 && j1;
            const double* pa0 = W.lg(32 * I2 + (lane & 15)) + (lane >> 4);
            const double* pa1 = W.lg(32 * I2 + 16 * i1 + (lane & 15)) + (lane >> 4);
            const double* pb0 = W.rg(32 * J2 + (lane & 15)) + (lane >> 4);
            const double* pb1 = W.rg(32 * J2 + 16 * j1 + (lane & 15)) + (lane >> 4);
            d4 a00 = {0.0, 0.0, 0.0, 0.0}, a01 = a00, a10 = a00, a11 = a00;
            for (int k0 = 0; k0 < N4; k0 += 4) {
                const double x0 = pa0[k0], x1 = pa1[k0], y0 = pb0[k0], y1 = pb1[k0];
                a00 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, y0, a00, 0, 0, 0);
                if (t01) a01 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, y1, a01, 0, 0, 0);
                if (t10) a10 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, y0, a10, 0, 0, 0);
                if (t11) a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, y1, a11, 0, 0, 0);
            }
            store_tile(2 * I2, 2 * J2, a00);
            if (t01) store_tile(2 * I2, 2 * J2 + 1, a01);
            if (t10) store_tile(2 * I2 + 1, 2 * J2, a10);
            if (t11) store_tile(2 * I2 + 1, 2 * J2 + 1, a11);
        }
    } else {
        // tiles (I, J), I <= J, of the 16-blocks in use, one wave per tile
        const int ntile = NB * (NB + 1) / 2;
        for (int q = wv; q < ntile; q += W.nw) {
            int I = 0, J = 0, rem = q;
            for (int bi = 0; bi < NB; ++bi) {
                const int n = NB - bi;
                if (rem < n) { I = bi; J = bi + rem; break; }
                rem -= n;
            }
            const double* pa = W.lg(16 * I + (lane & 15)) + (lane >> 4);
            const double* pb = W.rg(16 * J + (lane & 15)) + (lane >> 4);
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            for (int k0 = 0; k0 < N4; k0 += 4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[k0], pb[k0], acc, 0, 0, 0);
            store_tile(I, J, acc);
        }
    }
    __syncthreads();
}

// Wave 0: G + I' = L D L^T in LDS (lane r owns row r; unused rows become identity). Right-looking:
// step j scales column j and updates the trailing rows, one LDS read-modify-write per entry.
template <int HM>
__device__ __forceinline__ void schur_factor(BigShared<HM>& sh, int H, bool ht, double* gv = nullptr) {
    if (threadIdx.x < WAVE) {
        const int K3 = 3 * H;
        const int r = threadIdx.x;
        const int ty = r % 3;
        const bool rused = r < K3 && (ty != 0 || ht);
        // fused solves: the v-columns of Z^T Q^-1 Z (before I' and the factorization) for the s
        // elimination's rank-one term, Gv[p][tau] = G[p][3 tau] (lower-triangle storage)
        if (gv && ht && r < K3) {
            for (int tau = 0; tau < H; ++tau) {
                const int p = 3 * tau;
                gv[r * HM + tau] = p <= r ? sh.G[gi(r, p)] : sh.G[gi(p, r)];
            }
        }
        __builtin_amdgcn_wave_barrier();
        // assemble row r (lower triangle) with I' and identity rows
        if (r < K3) {
            for (int k = 0; k <= r; ++k) {
                const int tyk = k % 3;
                const bool kused = tyk != 0 || ht;
                double v = (rused && kused) ? sh.G[gi(r, k)] : 0.0;
                if (k == r) v += (ty != 2 || !rused) ? 1.0 : 0.0;
                sh.G[gi(r, k)] = v;
            }
        }
        __builtin_amdgcn_wave_barrier();
        bool bad = false;
        for (int j = 0; j < K3; ++j) {
            const double d = sh.G[gi(j, j)];
            bad = bad || !(d > 0.0) || !(d < 1e300);
            const double id = rcp(fmax(d, 1e-300));
            if (r == j) sh.gid[j] = id;
            const bool below = r > j && r < K3;
            const double l = below ? sh.G[gi(r, j)] * id : 0.0;
            __builtin_amdgcn_wave_barrier();
            if (below)
                for (int k = j + 1; k <= r; ++k) sh.G[gi(r, k)] = fma(-l, sh.G[gi(k, j)], sh.G[gi(r, k)]);
            __builtin_amdgcn_wave_barrier();
            if (below) sh.G[gi(r, j)] = l;
            __builtin_amdgcn_wave_barrier();
        }
        if (bad && r == 0) sh.flag = 1;
    }
    __syncthreads();
}

// Wave 0: q = G^{-1} rhs, rhs[3t + type] from sh.tot (type-major slots tot[type * H + t]),
// budget rows minus lb6 -> sh.q
// fx (fused solves, cap active): rhs += Gv c (the s elimination's rank-one term folded into the
// Schur system), and the v components of q are returned as q - c
template <int HM>
__device__ __forceinline__ void schur_solve(BigShared<HM>& sh, int H, const double* gv = nullptr,
                                            const double* cv = nullptr) {
    if (threadIdx.x < WAVE) {
        const int K3 = 3 * H;
        const int lane = threadIdx.x;
        double x = 0.0;
        if (lane < K3) {
            const int t = lane / 3, ty = lane - 3 * t;
            x = sh.tot[ty * H + t];
            if (ty == 2) x -= sh.lb6[t];
            if (gv)
                for (int tau = 0; tau < H; ++tau) x = fma(gv[lane * HM + tau], cv[tau], x);
        }
        // forward: L y = rhs (lane r reads row r of L), then D^{-1}
        const int lr = lane < K3 ? lane : 0;
        for (int j = 0; j + 1 < K3; ++j) {
            const double yj = bcast(x, j);
            if (lane > j) x = fma(-sh.G[gi(lr, j)], yj, x);
        }
        x *= sh.gid[lr];
        // backward: L^T q = y (lane r reads column r of L)
        for (int j = K3 - 1; j > 0; --j) {
            const double qj = bcast(x, j);
            if (lane < j) x = fma(-sh.G[gi(j, lr)], qj, x);
        }
        if (gv && lane < K3 && lane % 3 == 0) x -= cv[lane / 3];
        if (lane < K3) sh.q[lane] = x;
    }
    __syncthreads();
}

// Newton solve for rhs rows (first: -rdw, -rds with the complementarity targets rc; refinement:
// the residual arrays R0 / R1, no targets), oracle/kmpc_oracle.c:lsolve. The solution is assigned
// (first) or added to DW, DS and sh.dnu.
// corr: the first solve of the corrector — its targets rc + dx_aff dl_aff - smu are formed here
// from the affine direction (DW, DS) and written back to RC* without -smu (no sweep of their own).
template <int HM, int FL>
__device__ __forceinline__ void ph_lsolve(Win<HM, FL>& W, bool first, bool corr = false, double smu = 0.0) {
    auto& sh = W.sh;
    const bool hw = W.hw(), hs = W.hs(), ht = W.ht();
    const int H = W.H;
    // Fused (W.fx, cap active): the right-hand sides and the forward sweep of Q^-1 in ONE pass over
    // the state. The s elimination's rank-one term needs px = sum_i P bs, a block sum; instead of a
    // sweep of its own it is folded into the Schur system: with c_t = sqrt(rho_t) px_t,
    //   x = Q^-1 (rhs_w - D(BP bs)) + Q^-1 Z_v c  (the v-columns of Z: eps_t (e_t - e_{t-1}), eps = sqrt(rho) BP)
    // so Z^T x = Z^T x' + Gv c (Gv: the raw Gram's v-columns, kept by schur_factor) and
    // dw = x' - Q^-1 Z (q - E_v c). px is summed in the same block reduction as Z^T x'.
    const bool fused = W.fx != nullptr && ht;
    if (fused && !first) {
        // refinement pass: the right-hand sides are the residual arrays (no targets), so the sweep
        // needs no state — bs = R1 - lb5 / z4, rhs_w = R0 - BP bs_t + BP bs_{t+1}, px = sum_i P bs
        struct Rv { double r0, lr, P, r1n, bpn; };   // r1n / bpn: R1 / BP of period t + 1
        auto ldR = [&](int t) {
            Rv v;
            v.r0 = W.at(A_R0, t);
            v.lr = W.fat(A_LR, t);
            v.P = W.fat(A_P, t);
            v.r1n = t + 1 < H ? (double)W.at(A_R1, t + 1) : 0.0;
            v.bpn = t + 1 < H ? (double)W.fat(A_BP, t + 1) : 0.0;
            return v;
        };
        Rv rn{};
        double y = 0.0, bsc = 0.0, gpc = 0.0;
        if (W.act) {
            rn = ldR(0);
            bsc = (double)W.at(A_R1, 0) - sh.lb5[0] * sh.iz4[0];
            gpc = W.fat(A_BP, 0) * bsc;
        }
        for (int t = 0; t < H; ++t) {
            double pxv = 0.0;
            if (W.act) {
                const Rv c = rn;
                if (t + 1 < H) rn = ldR(t + 1);
                double bsn = 0.0, gpn = 0.0;
                if (t + 1 < H) {
                    bsn = c.r1n - sh.lb5[t + 1] * sh.iz4[t + 1];
                    gpn = c.bpn * bsn;
                }
                y = (c.r0 - gpc + gpn) + c.lr * y;
                W.at(A_Y, t) = y;
                W.at(A_BS, t) = bsc;
                pxv = c.P * bsc;
                bsc = bsn;
                gpc = gpn;
            }
            pxv = wave_sum(pxv);   // (every lane of the wave: outside the divergent branch)
            if ((threadIdx.x & (WAVE - 1)) == 0) W.pxr()[(threadIdx.x / WAVE) * HM + t] = pxv;
        }
    } else if (fused) {
        // the first solve of a direction (refinement passes take the branch above)
        double y = 0.0;
        St cur{};
        double rc1c = 0.0, rc2c = 0.0, rc3c = 0.0, dwc = 0.0;
        // bs of period t from its state and targets
        auto bsv = [&](int t, const St& e, double rc2, double rc3) -> double {
            const double b1 = -(W.cs_c - (e.l2 + e.l3 - sh.l4[t]));
            const double p23 = -rc2 * e.iz2 - rc3 * e.iz3;
            return b1 + p23 - sh.lb5[t] * sh.iz4[t];
        };
        typename Win<HM, FL>::Pre pq{};   // period t + 1's state (+ the affine direction), loaded at step t - 1
        double bsc = 0.0, gpc = 0.0, lrc = 0.0;
        if (W.act) {
            const auto p = W.pre(0, corr, false);
            if (H > 1) pq = W.pre(1, corr, false);
            lrc = W.fat(A_LR, 0);
            cur = W.st(p, W.wpi);
            if (corr) {
                dwc = p.dw;
                W.corr_rc(0, cur, p, dwc, smu, rc1c, rc2c, rc3c);
            } else {
                W.xl(cur, rc1c, rc2c, rc3c);
            }
            bsc = bsv(0, cur, rc2c, rc3c);
            gpc = cur.bma * cur.P * bsc;
        }
        for (int t = 0; t < H; ++t) {
            double pxv = 0.0;
            if (W.act) {
                const bool nx = t + 1 < H;
                St nxt = cur;
                double rc1n = 0.0, rc2n = 0.0, rc3n = 0.0, dwn = 0.0, lrn = 0.0;
                if (nx) {
                    const auto p = pq;
                    if (t + 2 < H) pq = W.pre(t + 2, corr, false);
                    lrn = W.fat(A_LR, t + 1);
                    nxt = W.st(p, cur.w);
                    if (corr) {
                        dwn = p.dw;
                        W.corr_rc(t + 1, nxt, p, dwn - dwc, smu, rc1n, rc2n, rc3n);
                    } else {
                        W.xl(nxt, rc1n, rc2n, rc3n);
                    }
                }
                double rdw, rds;
                W.dres(t, cur, nx ? nxt.l2 : 0.0, nx ? nxt.l3 : 0.0, rdw, rds);
                const double b0 = -rdw;
                const double p1 = hw ? -rc1c * cur.iw : 0.0;
                const double p2 = -rc2c * cur.iz2;
                const double p3 = -rc3c * cur.iz3;
                const double pn = nx ? -rc3n * nxt.iz3 + rc2n * nxt.iz2 : 0.0;
                const double bw = b0 + p1 + (p3 - p2) - pn;
                const double bsn = nx ? bsv(t + 1, nxt, rc2n, rc3n) : 0.0;
                const double gpn = nx ? nxt.bma * nxt.P * bsn : 0.0;
                y = (bw - gpc + gpn) + lrc * y;   // forward sweep of Q^-1 (Y)
                W.at(A_Y, t) = y;
                W.at(A_BS, t) = bsc;
                pxv = cur.P * bsc;
                cur = nxt;
                rc1c = rc1n; rc2c = rc2n; rc3c = rc3n;
                dwc = dwn;
                bsc = bsn;
                gpc = gpn;
                lrc = lrn;
            }
            pxv = wave_sum(pxv);   // (every lane of the wave: outside the divergent branch)
            if ((threadIdx.x & (WAVE - 1)) == 0) W.pxr()[(threadIdx.x / WAVE) * HM + t] = pxv;
        }
    }
    // ---- A: right-hand sides (BW, BS) and px = sum_i P bs ----
    if (!fused) {
        // per period: the raw state, the affine direction (corr), the targets (first) or the
        // refinement residual (!first)
        St cur{};
        double rc1c = 0.0, rc2c = 0.0, rc3c = 0.0, dwc = 0.0, r0c = 0.0, r1c = 0.0;
        if (W.act) {
            const auto p = W.pre(0, corr, false, !first);
            cur = W.st(p, W.wpi);
            if (corr) {
                dwc = p.dw;
                W.corr_rc(0, cur, p, dwc, smu, rc1c, rc2c, rc3c);
            } else if (first) {
                W.xl(cur, rc1c, rc2c, rc3c);
            }
            r0c = p.r0;
            r1c = p.r1;
        }
        for (int t = 0; t < H; ++t) {
            double px = 0.0;
            if (W.act) {
                const bool nx = t + 1 < H;
                St nxt = cur;
                double rc1n = 0.0, rc2n = 0.0, rc3n = 0.0, dwn = 0.0, r0n = 0.0, r1n = 0.0;
                if (nx) {
                    const auto p = W.pre(t + 1, corr, false, !first);
                    nxt = W.st(p, cur.w);
                    if (corr) {
                        dwn = p.dw;
                        W.corr_rc(t + 1, nxt, p, dwn - dwc, smu, rc1n, rc2n, rc3n);
                    } else if (first) {
                        W.xl(nxt, rc1n, rc2n, rc3n);
                    }
                    r0n = p.r0;
                    r1n = p.r1;
                }
                double b0, b1, p1 = 0.0, p2 = 0.0, p3 = 0.0, pn = 0.0;
                if (first) {
                    double rdw, rds;
                    W.dres(t, cur, nx ? nxt.l2 : 0.0, nx ? nxt.l3 : 0.0, rdw, rds);
                    b0 = -rdw;
                    b1 = -rds;
                    p1 = hw ? -rc1c * cur.iw : 0.0;
                    if (hs) {
                        p2 = -rc2c * cur.iz2;
                        p3 = -rc3c * cur.iz3;
                        if (nx) pn = -rc3n * nxt.iz3 + rc2n * nxt.iz2;
                    }
                } else {
                    b0 = r0c;
                    b1 = r1c;
                }
                const double bw = b0 + p1 + (p3 - p2) - pn;
                const double bs = hs ? b1 + p2 + p3 - (ht ? sh.lb5[t] * sh.iz4[t] : 0.0) : 0.0;
                W.at(A_BW, t) = bw;
                W.at(A_BS, t) = bs;
                px = cur.P * bs;
                cur = nxt;
                rc1c = rc1n;
                rc2c = rc2n;
                rc3c = rc3n;
                dwc = dwn;
                r0c = r0n;
                r1c = r1n;
            }
            W.slot(t, px);
        }
        W.finish(H);
        if (threadIdx.x < HM) sh.px[threadIdx.x] = (int)threadIdx.x < H ? sh.tot[threadIdx.x] : 0.0;
        __syncthreads();
    }
    // ---- B: s elimination, x = Q^{-1} rhs_w (X), Schur rhs Z^T x, q = G^{-1} (...) ----
    {
        if (W.act && !fused) {
            // rhs_w -= g_t - g_{t+1}, g = bma P (bs - rho px); forward sweep y_t = x_t + Lr_t y_{t-1} (Y)
            double y = 0.0;
            double gc = hs ? W.fat(A_BP, 0) * (W.at(A_BS, 0) - sh.rho[0] * sh.px[0]) : 0.0;
            for (int t = 0; t < H; ++t) {
                double gn = 0.0;
                if (hs && t + 1 < H) gn = W.fat(A_BP, t + 1) * (W.at(A_BS, t + 1) - sh.rho[t + 1] * sh.px[t + 1]);
                const double x = W.at(A_BW, t) - gc + gn;
                y = x + W.fat(A_LR, t) * y;
                W.at(A_Y, t) = y;
                gc = gn;
            }
        }
        // backward sweep x_t = y_t / Dd_t + Lr_{t+1} x_{t+1} (X), with the Z^T x slots: at step t,
        // v-slot t+1 = eps_{t+1} (x_{t+1} - x_t), a-slot t = alpha_t x_t, 1-slot t = x_t.
        // Every sweep below loads period t -+ 1 before it computes period t (two periods of loads
        // in flight per wave: the slab stream is bound by loads in flight, not by the arithmetic).
        struct Bv { double y, idd, bp, m, lr; };
        auto ldB = [&](int t) {
            Bv v;
            v.y = W.at(A_Y, t);
            v.idd = W.fat(A_IDD, t);
            v.bp = ht ? (double)W.fat(A_BP, t) : 0.0;
            v.m = W.mload(t);
            v.lr = W.fat(A_LR, t);
            return v;
        };
        Bv bn{}, bn2{}, bn3{};
        if (W.act) {
            bn = ldB(H - 1);
            if (KMPC_BIG_PF2S && H > 1) bn2 = ldB(H - 2);
            if (KMPC_BIG_PF3S && H > 2) bn3 = ldB(H - 3);
        }
        double xn = 0.0, lrn = 0.0, epn = 0.0;
        for (int t = H - 1; t >= 0; --t) {
            double x = 0.0, va = 0.0, vv1 = 0.0, ep = 0.0;
            if (W.act) {
                const Bv c = bn;
                if (KMPC_BIG_PF3S) {
                    bn = bn2;
                    bn2 = bn3;
                    if (t > 2) bn3 = ldB(t - 3);
                } else if (KMPC_BIG_PF2S) {
                    bn = bn2;
                    if (t > 1) bn2 = ldB(t - 2);
                } else if (t > 0) {
                    bn = ldB(t - 1);
                }
                x = c.y * c.idd + lrn * xn;
                W.at(A_X, t) = x;
                ep = ht ? sh.sr[t] * c.bp : 0.0;
                va = W.alpha(t, c.m) * x;
                vv1 = (t + 1 < H) ? epn * (xn - x) : 0.0;
                lrn = c.lr;
            }
            if (t + 1 < H) W.slot(t + 1, vv1);
            W.slot(H + t, va);
            W.slot(2 * H + t, x);
            if (t == 0) W.slot(0, W.act ? ep * x : 0.0);
            xn = x;
            epn = ep;
        }
        W.finish(3 * H);
        if (fused) {
            // px of this solve (the per-wave partials of the fused sweep, published by finish's
            // barrier) and c = sqrt(rho) px, on wave 0 (schur_solve's wave: no barrier between)
            if (threadIdx.x < HM) {
                const int t = threadIdx.x;
                double px = 0.0;
                if (t < H)
                    for (int q = 0; q < W.nw; ++q) px += W.pxr()[q * HM + t];
                sh.px[t] = px;
                W.cv()[t] = sh.sr[t] * px;
            }
            schur_solve(sh, H, W.gv(), W.cv());
        } else {
            schur_solve(sh, H);
        }
    }
    // ---- C: dw = x - Q^{-1} (Z q) (DW), P bs = P BS - BP dd (DS), px = sum_i P bs ----
    {
        if (W.act) {
            // Z q per period: alpha_t q_a + q_1 + eps_t q_v(t) - eps_{t+1} q_v(t+1); forward sweep (Y)
            struct Fv { double m, bpn, lr; };   // bpn: BP of period t + 1
            auto ldF = [&](int t) {
                Fv v;
                v.m = W.mload(t);
                v.bpn = (ht && t + 1 < H) ? (double)W.fat(A_BP, t + 1) : 0.0;
                v.lr = W.fat(A_LR, t);
                return v;
            };
            Fv fn = ldF(0), fn2{}, fn3{};
            if (KMPC_BIG_PF2S && H > 1) fn2 = ldF(1);
            if (KMPC_BIG_PF3S && H > 2) fn3 = ldF(2);
            double y = 0.0;
            double epc = W.epsa(0);
            for (int t = 0; t < H; ++t) {
                const Fv c = fn;
                if (KMPC_BIG_PF3S) {
                    fn = fn2;
                    fn2 = fn3;
                    if (t + 3 < H) fn3 = ldF(t + 3);
                } else if (KMPC_BIG_PF2S) {
                    fn = fn2;
                    if (t + 2 < H) fn2 = ldF(t + 2);
                } else if (t + 1 < H) {
                    fn = ldF(t + 1);
                }
                const double epn = (t + 1 < H) ? sh.sr[t + 1] * c.bpn : 0.0;
                const double zq = W.alpha(t, c.m) * sh.q[3 * t + 1] + sh.q[3 * t + 2] + epc * sh.q[3 * t] -
                                  ((t + 1 < H) ? epn * sh.q[3 * t + 3] : 0.0);
                y = zq + c.lr * y;
                W.at(A_Y, t) = y;
                epc = epn;
            }
        }
        // backward sweep; dw_t = x_t - (Q^{-1} Z q)_t; at step t: P bs_{t+1} = P BS_{t+1} - BP_{t+1} (dw_{t+1} - dw_t)
        // (refinement passes add to DW / DS: their old values are loaded with the period)
        struct Cv { double y, idd, lr, x, bp, P, bs1, dwo, ds1; };   // bs1 / ds1: BS / DS of period t + 1
        auto ldC = [&](int t) {
            Cv v;
            v.y = W.at(A_Y, t);
            v.idd = W.fat(A_IDD, t);
            v.lr = W.fat(A_LR, t);
            v.x = W.at(A_X, t);
            v.bp = hs ? (double)W.fat(A_BP, t) : 0.0;
            v.P = hs ? (double)W.fat(A_P, t) : 0.0;
            v.bs1 = (hs && t + 1 < H) ? (double)W.at(A_BS, t + 1) : 0.0;
            v.dwo = first ? 0.0 : (double)W.at(A_DW, t);
            v.ds1 = (!first && hs && t + 1 < H) ? (double)W.at(A_DS, t + 1) : 0.0;
            return v;
        };
        Cv cn{}, cn2{}, cn3{};
        if (W.act) {
            cn = ldC(H - 1);
            if (KMPC_BIG_PF2S && H > 1) cn2 = ldC(H - 2);
            if (KMPC_BIG_PF3S && H > 2) cn3 = ldC(H - 3);
        }
        double tn = 0.0, lrn = 0.0, dwn = 0.0, bpn = 0.0, Pn = 0.0;
        for (int t = H - 1; t >= 0; --t) {
            double pxn = 0.0, px0 = 0.0;
            if (W.act) {
                const Cv c = cn;
                if (KMPC_BIG_PF3S) {
                    cn = cn2;
                    cn2 = cn3;
                    if (t > 2) cn3 = ldC(t - 3);
                } else if (KMPC_BIG_PF2S) {
                    cn = cn2;
                    if (t > 1) cn2 = ldC(t - 2);
                } else if (t > 0) {
                    cn = ldC(t - 1);
                }
                const double tq = c.y * c.idd + lrn * tn;
                tn = tq;
                lrn = c.lr;
                const double dw = c.x - tq;
                W.at(A_DW, t) = first ? dw : c.dwo + dw;
                // P times the back-substituted s right-hand side goes to DS (summed over the
                // solves); ds = DS - P rho pxa is formed where it is read (Win::dsv)
                if (hs && t + 1 < H) {
                    const double pbs = Pn * c.bs1 - bpn * (dwn - dw);
                    W.at(A_DS, t + 1) = first ? pbs : c.ds1 + pbs;
                    pxn = pbs;
                }
                if (hs && t == 0) {
                    const double pbs = c.P * W.at(A_BS, 0) - c.bp * dw;
                    if (first) W.at(A_DS, 0) = pbs; else W.at(A_DS, 0) += pbs;
                    px0 = pbs;
                }
                dwn = dw;
                bpn = c.bp;
                Pn = c.P;
            }
            if (t + 1 < H) W.slot(t + 1, pxn);
            if (t == 0) W.slot(0, px0);
        }
        W.finish(H);
    }
    // ---- D: px summed over the solves (ds = P (DS - rho pxa)); budget multipliers ----
    {
        if (threadIdx.x < HM) {
            const int t = threadIdx.x;
            const double dn = t < H ? sh.q[3 * t + 2] : 0.0;
            sh.dnu[t] = first ? dn : sh.dnu[t] + dn;
            const double px = (hs && t < H) ? sh.tot[t] : 0.0;
            sh.pxa[t] = first ? px : sh.pxa[t] + px;
        }
        __syncthreads();
    }
}

// Newton direction for the current rc targets, adaptive refinement (ipm_kernel newton).
// On exit: DW, DS, sh.dnu, sh.dz4, sh.dl4.
// corr: this is the corrector — its targets (rc += dx_aff dl_aff - smu) are formed by the owners
// (rc4) here and by the first solve's right-hand-side sweep (rc1..rc3).
template <int HM, int FL>
__device__ __forceinline__ void ph_newton(Win<HM, FL>& W, int n_refine, bool corr = false, double smu = 0.0) {
    auto& sh = W.sh;
    const bool hs = W.hs(), ht = W.ht();
    const int H = W.H;
    if (threadIdx.x < HM) {
        const int t = threadIdx.x;
        if (corr && ht && t < H) sh.rc4[t] += sh.dz4[t] * sh.dl4[t] - smu;
        sh.b5[t] = (ht && t < H) ? -sh.rc4[t] - sh.l4[t] * sh.rg4[t] : 0.0;
        sh.b6[t] = (t < H) ? -sh.rp[t] : 0.0;
        sh.lb5[t] = sh.b5[t];
        sh.lb6[t] = sh.b6[t];
    }
    __syncthreads();
    // ||b||_inf of the unreduced system: this thread's rows in the first residual pass, the owner
    // rows here; reduced with the first residual norm
    double bn = 0.0;
    if (n_refine > 0 && threadIdx.x == 0)
        for (int t = 0; t < H; ++t) bn = fmax(bn, fmax(fabs(sh.b5[t]), fabs(sh.b6[t])));
    for (int r = 0;; ++r) {
        ph_lsolve(W, r == 0, corr && r == 0, smu);
        if (r >= n_refine) break;
        // residual of rows (1), (2), (7) of the direction; rows (3)-(6) hold by construction
        for (int t = 0; t < H; ++t) {
            double va = 0.0, vw = 0.0;
            if (W.act) {
                vw = W.at(A_DW, t);
                va = W.alpha(t, W.mload(t)) * vw;
            }
            W.slot(t, va);
            W.slot(H + t, vw);
        }
        W.finish(2 * H);
        if (threadIdx.x < HM) {
            const int t = threadIdx.x;
            const bool on = t < H;
            sh.adw[t] = on ? sh.tot[t] : 0.0;
            sh.sds[t] = (on && hs) ? sh.pxa[t] * sh.isp1[t] : 0.0;   // sum_i ds (no sweep)
            sh.sdw[t] = on ? sh.tot[H + t] : 0.0;
        }
        __syncthreads();
        double rn = 0.0;
        if (W.act) {
            double nl2 = 0.0, nl3 = 0.0, l2n = 0.0, l3n = 0.0;   // dl2 / dl3 / l2 / l3 of period t + 1
            for (int t = H - 1; t >= 0; --t) {
                const St e = W.st(t, W.wprev(t));
                const double dw = W.at(A_DW, t), ds = W.dsv(t, e, W.at(A_DS, t));
                const double dd = dw - (t ? W.at(A_DW, t - 1) : 0.0);
                // the targets: the corrector's (stored without -smu), or the predictor's x l
                double rc1, rc2, rc3;
                if (corr) {
                    rc1 = W.hw() ? W.at(A_RC1, t) - smu : 0.0;
                    rc2 = hs ? W.at(A_RC2, t) - smu : 0.0;
                    rc3 = hs ? W.at(A_RC3, t) - smu : 0.0;
                } else {
                    W.xl(e, rc1, rc2, rc3);
                }
                double dl1, dl2, dl3;
                W.ddirs(e, rc1, rc2, rc3, dw, ds, dd, dl1, dl2, dl3);
                double rdw, rds;
                W.dres(t, e, l2n, l3n, rdw, rds);
                if (r == 0)
                    bn = fmax(bn, fmax(fmax(fabs(rdw), fabs(rds)), fmax(fabs(rc1), fmax(fabs(rc2), fabs(rc3)))));
                const double dl4 = ht ? (sh.b5[t] + sh.l4[t] * sh.sds[t]) * sh.iz4[t] : 0.0;
                const double r0 = -rdw - (W.alpha(t, e.m) * sh.adw[t] - (dl1 + (dl3 - dl2) - (nl3 - nl2)) + sh.dnu[t]);
                const double r1 = hs ? -rds + (dl2 + dl3 - dl4) : 0.0;
                W.at(A_R0, t) = r0;
                W.at(A_R1, t) = r1;
                rn = fmax(rn, fmax(fabs(r0), fabs(r1)));
                nl2 = dl2;
                nl3 = dl3;
                l2n = e.l2;
                l3n = e.l3;
            }
        }
        if (threadIdx.x == 0)
            for (int t = 0; t < H; ++t) rn = fmax(rn, fabs(sh.b6[t] - sh.sdw[t]));
        W.max_max(rn, bn);   // (bn: block value after the first pass, unchanged by later ones)
        if (rn <= REFINE_RTOL * bn) break;
        if (threadIdx.x < HM) {
            const int t = threadIdx.x;
            sh.lb5[t] = 0.0;                                   // row (6) residual is identically 0
            sh.lb6[t] = (t < H) ? sh.b6[t] - sh.sdw[t] : 0.0;
        }
        __syncthreads();
    }
    // dz4 / dl4 of the final direction: sum_i ds = pxa / (1 + gamma SP) (no sweep)
    if (threadIdx.x < HM) {
        const int t = threadIdx.x;
        const bool on = ht && t < H;
        const double st = (hs && t < H) ? sh.pxa[t] * sh.isp1[t] : 0.0;
        sh.dz4[t] = on ? -st + sh.rg4[t] : 0.0;
        sh.dl4[t] = on ? (sh.b5[t] + sh.l4[t] * st) * sh.iz4[t] : 0.0;
    }
    __syncthreads();
}

// Largest step for the current direction (before the fraction-to-boundary), and the coefficients
// c1, c2 of the asset complementarity along it, sum (x + a dx)(l + a dl) = c0 + a c1 + a^2 c2
// (c0: ph_factor's mu sum) — the Mehrotra centring then needs no sweep of its own (ipm_kernel
// max_step does the same).
// pred: the predictor's direction, whose targets are x l (from the state, not stored)
template <int HM, int FL>
__device__ __forceinline__ double ph_step(Win<HM, FL>& W, double& c1, double& c2, bool pred, double smu = 0.0) {
    auto& sh = W.sh;
    const bool hw = W.hw(), hs = W.hs(), ht = W.ht();
    const int H = W.H;
    double a = 1e300, wprev = W.wpi, dwp = 0.0;
    c1 = c2 = 0.0;
#ifndef KMPC_BIG_PF2   // step length and update sweeps: loads two periods ahead (1) or one (0)
#define KMPC_BIG_PF2 1
#endif
    typename Win<HM, FL>::Pre pn{}, pn2{};
    if (W.act) {
        pn = W.pre(0, true, !pred);
        if (KMPC_BIG_PF2 && H > 1) pn2 = W.pre(1, true, !pred);
    }
    for (int t = 0; t < H; ++t) {
        double mdw = 0.0;
        if (W.act) {
            const auto p = pn;
            if (KMPC_BIG_PF2) {
                pn = pn2;
                if (t + 2 < H) pn2 = W.pre(t + 2, true, !pred);
            } else if (t + 1 < H) {
                pn = W.pre(t + 1, true, !pred);
            }
            const St e = W.st(p, wprev);
            wprev = e.w;
            const double dw = p.dw, ds = W.dsv(t, e, p.ds), dd = dw - dwp;
            dwp = dw;
            double r1 = p.rc1 - smu, r2 = p.rc2 - smu, r3 = p.rc3 - smu;   // (RC* without -smu)
            if (pred) W.xl(e, r1, r2, r3);
            double dl1, dl2, dl3;
            W.ddirs(e, r1, r2, r3, dw, ds, dd, dl1, dl2, dl3);
            if (hw) {
                a = to_bound(e.w, dw, a); a = to_bound(e.l1, dl1, a);
                c1 += e.w * dl1 + e.l1 * dw;
                c2 += dw * dl1;
            }
            if (hs) {
                const double x2 = e.s - e.d, dx2 = ds - dd, x3 = e.s + e.d, dx3 = ds + dd;
                a = to_bound(x2, dx2, a);
                a = to_bound(x3, dx3, a);
                a = to_bound(e.l2, dl2, a);
                a = to_bound(e.l3, dl3, a);
                c1 += x2 * dl2 + e.l2 * dx2 + x3 * dl3 + e.l3 * dx3;
                c2 += dx2 * dl2 + dx3 * dl3;
            }
            mdw = e.m * dw;
        }
        W.slot(t, mdw);
    }
    W.slot(H, c1);
    W.slot(H + 1, c2);
    {
        double z = 0.0, na = -a;
        W.sum_max(z, na);
        a = -na;
    }
    W.finish(H + 2);
    c1 = sh.tot[H];
    c2 = sh.tot[H + 1];
    for (int t = 0; t < H; ++t) {
        a = to_bound(sh.den[t], sh.tot[t], a);
        if (ht) { a = to_bound(sh.z4[t], sh.dz4[t], a); a = to_bound(sh.l4[t], sh.dl4[t], a); }
    }
    return a;
}

// iterate update (the multiplier directions need the old state: w_{t-1} is carried), fused with
// the next iteration's period sums (ph_sums) over the updated w, s
template <int HM, int FL>
__device__ __forceinline__ void ph_update(Win<HM, FL>& W, double step, double smu) {
    auto& sh = W.sh;
    const int H = W.H;
    double wprev = W.wpi, dwp = 0.0;
    typename Win<HM, FL>::Pre pn{}, pn2{};
    if (W.act) {
        pn = W.pre(0);
        if (KMPC_BIG_PF2 && H > 1) pn2 = W.pre(1);
    }
    for (int t = 0; t < H; ++t) {
        double mw = 0.0, wn = 0.0, sn = 0.0;
        if (W.act) {
            const auto p = pn;
            if (KMPC_BIG_PF2) {
                pn = pn2;
                if (t + 2 < H) pn2 = W.pre(t + 2);
            } else if (t + 1 < H) {
                pn = W.pre(t + 1);
            }
            const St e = W.st(p, wprev);
            wprev = e.w;
            const double dw = p.dw, ds = W.dsv(t, e, p.ds), dd = dw - dwp;
            dwp = dw;
            double dl1, dl2, dl3;
            W.ddirs(e, p.rc1 - smu, p.rc2 - smu, p.rc3 - smu, dw, ds, dd, dl1, dl2, dl3);   // (RC* without -smu)
            W.at(A_L1, t) = e.l1 + step * dl1;
            W.at(A_L2, t) = e.l2 + step * dl2;
            W.at(A_L3, t) = e.l3 + step * dl3;
            wn = e.w + step * dw;
            sn = e.s + step * ds;
            W.at(A_W, t) = wn;
            W.at(A_S, t) = sn;
            mw = e.m * wn;
        }
        W.slot(3 * t, mw);
        W.slot(3 * t + 1, wn);
        W.slot(3 * t + 2, sn);
    }
    W.finish(3 * H);   // (its first barrier: every ratio test has read z4 / l4 before the owners update them)
    if (threadIdx.x < HM && (int)threadIdx.x < H) {
        const int t = threadIdx.x;
        sh.z4[t] += step * sh.dz4[t];
        sh.l4[t] += step * sh.dl4[t];
        sh.nu[t] += step * sh.dnu[t];
    }
    sums_owner(W);
}

template <int HM, int FL>
__device__ __forceinline__ int ipm_iterate(Win<HM, FL>& W, double* wout, int tw, double inv_ncon, double& best,
                                        double& min_pr, int b) {
    auto& sh = W.sh;
    const SolveArgs& a = W.a;
    const int H = W.H;
    int it;
    ph_sums(W);   // later iterations: ph_update's fused sums
    for (it = 0; it < a.max_iter; ++it) {
        double mu_l, rd;
        ph_factor(W, mu_l, rd);
        double mu = mu_l, pr = 0.0;
        bool domain_ok = true;
        for (int t = 0; t < H; ++t) {
            mu += sh.rc4[t];
            pr = fmax(pr, fmax(fabs(sh.rp[t]), fabs(sh.rg4[t])));
            domain_ok = domain_ok && sh.den[t] > 0.0;
        }
        mu *= inv_ncon;
        const double merit = fmax(mu, fmax(rd, pr));
        min_pr = fmin(min_pr, pr);
        if (a.trace && b == 0 && threadIdx.x == 0) {
            a.trace[4 * it + 0] = mu; a.trace[4 * it + 1] = rd; a.trace[4 * it + 2] = pr;
        }
        if (!domain_ok || !isfinite(merit)) break;
        if (merit < best) {
            best = merit;
            ph_record(W, wout, tw);
        } else if (best < 1e-6 && merit > 1e4 * best) {
            break;   // numerical breakdown after convergence: keep the best iterate
        }
        if (mu < a.tol && rd < 10.0 * a.tol && pr < 10.0 * a.tol) break;
        if (sh.flag) break;   // Q not positive definite
        ph_gram(W);
        schur_factor(sh, H, W.ht(), W.fx ? W.gv() : nullptr);
        if (sh.flag) break;
        double step = 0.0, smu = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            ph_newton(W, (pass == 0 || mu > (W.hw() ? REFINE_MU : REFINE_MU_SHORT)) ? 0 : a.n_refine, pass == 1, smu);
            double cc1, cc2;
            const double amax = ph_step(W, cc1, cc2, pass == 0, smu);
            if (pass == 1) { step = fmin(1.0, (W.hw() ? KMPC_STEP_NOSHORT : 0.99) * amax); break; }
            const double ap = fmin(1.0, amax);
            double comp = mu_l + ap * (cc1 + ap * cc2);
            if (W.ht())
                for (int t = 0; t < H; ++t) comp += (sh.z4[t] + ap * sh.dz4[t]) * (sh.l4[t] + ap * sh.dl4[t]);
            double sg = comp * inv_ncon / mu;
            sg = sg * sg * sg;
            if (W.hw() && W.ht()) sg = fmin(sg, KMPC_SIGMA_CAP);
            smu = sg * mu;   // the corrector's targets are formed inside its first solve
        }
        if (a.trace && b == 0 && threadIdx.x == 0) a.trace[4 * it + 3] = step;
        ph_update(W, step, smu);
    }
    return it;
}

template <int HM, int MAXT, int FL>
__global__ void __launch_bounds__(MAXT) __attribute__((amdgpu_waves_per_eu(MAXT >= 512 ? KMPC_BIG_WPE : 1))) ipm_big(BigArgs A) {
    static_assert(3 * HM <= KP - 1, "Schur system must fit one wave");
    constexpr int NWB = MAXT / WAVE;
    __shared__ double shraw[bs_doubles<HM>(NWB)];
    BigShared<HM>& sh = *reinterpret_cast<BigShared<HM>*>(shraw);
    const SolveArgs& a = A.s;
    Win<HM, FL> W{a, sh, A.ws + (size_t)blockIdx.x * A.slab, a.N, a.H, A.NP, (int)(blockDim.x / WAVE),
                  (int)threadIdx.x, (int)threadIdx.x < a.N};
    W.bind(A.slab);
    W.sbuf = 0;
#ifndef KMPC_BIG_FUSE
#define KMPC_BIG_FUSE 1
#endif
    // fused solves on the >= 512-thread blocks (two per CU: the extra 13.6 KB fits; the 256-thread
    // blocks run three per CU at the LDS limit and keep the unfused sweeps)
    __shared__ double fxs[(KMPC_BIG_FUSE && MAXT >= 512) ? fx_doubles<HM, NWB>() : 1];
    W.fx = (KMPC_BIG_FUSE && MAXT >= 512) ? fxs : nullptr;
    W.cs.set_case(!a.allow_short, (a.c > 0.0) || (a.tau > 0.0), a.tau > 0.0);
    const bool hw = W.hw(), hs = W.hs(), ht = W.ht();
    const int N = a.N, H = a.H, i = threadIdx.x;

    for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
        const double* wp = a.wp + (size_t)b * N;
        const float* yh = a.yhat + (size_t)b * H * N;
        double* wout = a.wout + (size_t)b * (a.return_full ? H * N : N);
        const int tw = a.return_full ? H : 1;
        W.wpi = W.act ? wp[i] : 0.0;

        // ---- inputs: m = R - 1, R = np.exp(yhat) in float32 (mpc.py:55; slab), objective scale,
        //      finiteness (non-finite yhat or overflowing R -> solver_error) ----
        double mx = 0.0, nf = 0.0;
        if (W.act) {
            if (!isfinite(W.wpi)) nf = 1.0;
            for (int t = 0; t < H; ++t) {
                const float r = np_expf(yh[t * N + i]);
                if (!isfinite((double)r - 1.0)) nf = 1.0;
                W.mstore(t, r);
            }
        }
        {
            double z = 0.0;
            W.sum_max(z, nf);
        }
        // per period S_t = sum_i R: 0 -> the reference's exp cone is infeasible; below TINY_PERIOD the
        // period runs on R / S_t (stored back as float32) and the objective adds log S_t (as
        // ipm_kernel and the oracle)
        bool r_zero = false;
        if (nf == 0.0) {
            for (int t = 0; t < H; ++t) W.slot(t, W.act ? W.rload(t) : 0.0);
            W.finish(H);
            for (int t = 0; t < H; ++t) {
                const double S = sh.tot[t];
                r_zero = r_zero || S == 0.0;
                if (S > 0.0 && S < TINY_PERIOD && W.act) W.mstore(t, (float)(W.rload(t) / S));
                if (W.act) mx = fmax(mx, fabs(W.mload(t)));
            }
            if (threadIdx.x < HM) {
                const int t = threadIdx.x;
                const double S = t < H ? sh.tot[t] : 1.0;
                sh.lsc[t] = (S > 0.0 && S < TINY_PERIOD) ? log(S) : 0.0;
            }
        }
        {
            double z = 0.0;
            W.sum_max(z, mx);
        }
        double sig = fmax(mx, a.c);
        if (!(sig > 0.0)) sig = 1.0;
        W.isig = 1.0 / sig;
        W.irsig = 1.0 / sqrt(sig);
        W.cs_c = a.c / sig;
        W.tau = a.tau;

        int status = KMPC_STATUS_SOLVER_ERROR, it = 0;
        double best_obj = __builtin_nan("");

        if (nf == 0.0 && isfinite(a.c) && isfinite(a.tau)) {
            if (r_zero) {
                status = KMPC_STATUS_INFEASIBLE;
            } else if (a.allow_short && !hs) {
                // no bounds and no turnover terms: unbounded unless every period is flat
                for (int t = 0; t < H; ++t) W.slot(t, W.act ? W.mload(t) : 0.0);
                W.finish(H);
                double spread = 0.0, swp = W.wpi;
                if (W.act)
                    for (int t = 0; t < H; ++t) spread = fmax(spread, fabs(W.mload(t) - sh.tot[t] / N));
                W.sum_max(swp, spread);
                if (spread == 0.0) {
                    const double w = swp != 0.0 ? W.wpi / swp : 1.0 / N;
                    for (int t = 0; t < H; ++t) {
                        if (W.act && t < tw) wout[t * N + i] = w;
                        W.slot(t, W.act ? (1.0 + W.mload(t)) * w : 0.0);
                    }
                    W.finish(H);
                    double f = 0.0;
                    for (int t = 0; t < H; ++t) f += log(sh.tot[t]) + sh.lsc[t];
                    best_obj = f;
                    status = KMPC_STATUS_OPTIMAL;
                } else {
                    status = KMPC_STATUS_UNBOUNDED;
                }
            } else {
                // ---- initial point (as ipm_kernel / the oracle) ----
                const double b0 = hw ? fmax(W.wpi, 0.0) : W.wpi;
                const double w0 = 0.5 * b0 + 0.5 / N;
                for (int t = 0; t < H; ++t) {
                    double s = 0.0;
                    if (W.act) {
                        const double d = w0 - (t ? w0 : W.wpi);
                        s = hs ? fabs(d) + 1.0 / N : 0.0;
                        W.at(A_W, t) = w0;
                        W.at(A_S, t) = s;
                        W.at(A_L1, t) = hw ? KMPC_INIT_MULT : 0.0;
                        W.at(A_L2, t) = hs ? KMPC_INIT_MULT : 0.0;
                        W.at(A_L3, t) = hs ? KMPC_INIT_MULT : 0.0;
                    }
                    W.slot(t, s);
                }
                W.finish(H);
                if (threadIdx.x < HM) {
                    const int t = threadIdx.x;
                    sh.z4[t] = (ht && t < H) ? fmax(a.tau - sh.tot[t], 0.5 * a.tau) : 1.0;
                    sh.l4[t] = (ht && t < H) ? KMPC_INIT_MULT : 0.0;
                    sh.nu[t] = 0.0;
                }
                __syncthreads();
                const int ncon = (hw ? H * N : 0) + (hs ? 2 * H * N : 0) + (ht ? H : 0);
                const double inv_ncon = 1.0 / (ncon > 0 ? ncon : 1);
                double best = 1e300, min_pr = 1e300;
                it = ipm_iterate(W, wout, tw, inv_ncon, best, min_pr, b);
                __syncthreads();   // sh.best_* of the best iterate visible
                if (best < 1e300) {
                    double f = 0.0;
                    for (int t = 0; t < H; ++t) f += log(sh.best_rw[t]) + sh.lsc[t] - a.c * sh.best_l1[t];
                    best_obj = f;
                }
                if (best <= 1e-7) status = KMPC_STATUS_OPTIMAL;
                else if (best <= 1e-4) status = KMPC_STATUS_OPTIMAL_INACCURATE;
                else if (min_pr > 1e-6) status = KMPC_STATUS_INFEASIBLE;   // primal residual never closed
                else status = KMPC_STATUS_SOLVER_ERROR;
            }
        }
        __syncthreads();
        // ---- outputs: W was written by ph_record; fallback (mpc.py:113-115) otherwise ----
        const bool ok = status == KMPC_STATUS_OPTIMAL || status == KMPC_STATUS_OPTIMAL_INACCURATE;
        if (!ok && W.act)
            for (int t = 0; t < tw; ++t) wout[t * N + i] = W.wpi;
        if (threadIdx.x == 0) {
            a.obj[b] = ok ? best_obj : __builtin_nan("");
            a.status[b] = status;
            if (a.iters) a.iters[b] = it;
        }
        __syncthreads();
    }
}

// workspace bytes of the large-window launch
template <int HM>
size_t ws_bytes(const SolveArgs& a) {
    const int NP = WAVE * ((a.N + WAVE - 1) / WAVE);
    return sizeof(double) * slab_doubles(HM, NP) * (size_t)slots_for(a.B, a.N);
}

template <int HM, int MAXT>
int launch_t(const BigArgs& A, int slots, hipStream_t stream, int fl) {
    if (fl == 7) hipLaunchKernelGGL((ipm_big<HM, MAXT, 7>), dim3(slots), dim3(A.NP), 0, stream, A);
    else hipLaunchKernelGGL((ipm_big<HM, MAXT, -1>), dim3(slots), dim3(A.NP), 0, stream, A);
    return hipGetLastError() == hipSuccess ? KMPC_OK : KMPC_ERR_LAUNCH;
}

template <int HM>
int launch(const SolveArgs& a, void* ws, size_t ws_size, hipStream_t stream) {
    if (a.N > NWX * WAVE || a.H > HM) return KMPC_ERR_UNSUPPORTED;
    if (!ws || ws_size < ws_bytes<HM>(a)) return KMPC_ERR_WORKSPACE;
    BigArgs A;
    A.s = a;
    A.NP = WAVE * ((a.N + WAVE - 1) / WAVE);
    A.slab = slab_doubles(HM, A.NP);
    A.ws = (double*)ws;
    const int slots = slots_for(a.B, a.N);
    const int fl = case_of(!a.allow_short, a.c > 0.0 || a.tau > 0.0, a.tau > 0.0);
    if (A.NP <= 256) return launch_t<HM, 256>(A, slots, stream, fl);
    if (A.NP <= 512) return launch_t<HM, 512>(A, slots, stream, fl);
    return launch_t<HM, 1024>(A, slots, stream, fl);
}

}  // namespace big
}  // namespace kmpc
