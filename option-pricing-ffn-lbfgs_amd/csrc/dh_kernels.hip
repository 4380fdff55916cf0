// dh_kernels.hip -- gfx950 kernels and C-ABI of the COS pricing / calibration-objective hot path.
//
// Two kernels per request (DESIGN.md "Kernels"), each with its own small register footprint:
//
//   cos_table_kernel<TPT>  one table per (param set p, maturity group g):  for k < N
//     (blocks = resident capacity, each a contiguous range of tables; prologues of up to 64
//     tables computed lane-parallel by one wave)
//       w_k = Re(phi(u_k) e^{-i u_k a}) 2/(b-a)            (double_heston.py:48-97,163-168,187)
//     (8 bytes per term) plus per-(p, g) constants c0/c1 (call), c5 (put), w0 (k = 0 weight),
//     a, b, e^b, e^a reduced in a fixed order.  CF-bound; the table lands in an L2/MALL-resident
//     workspace.
//
//   cos_option_kernel<TPT> one task per (p, tile), a tile = <= 256 options of one maturity:
//     stage the (p, g) table into LDS, expanded to the strike-independent parts of chi_k/psi_k
//     (k >= 1, double_heston.py:141-158):  u_k = k pi/(b-a),  T2_k = w_k S0/(1+u_k^2),
//     T6_k = -T2_k/u_k;  per option one angle sum remains
//       S = sum_k T2_k cos(k th) + T6_k sin(k th),   th = pi (log(K/S0) - a)/(b - a),
//       price = e^{-rT} (const + w0 V_0 - e^{xK} S)
//     (the chi and psi parts at the log-strike, -e^{xK}(T2 cos + T2 u sin) + K (w/u) sin, with
//     K = S0 e^{xK}), computed by G lanes per group of kR options (lane j: k = 1 + j, 1 + j + G,
//     ...), cos/sin(k th) advanced by the Chebyshev recurrence x_{k+G} = 2 cos(G th) x_k -
//     x_{k-G} with an exact sincos re-anchor every kAnchor steps, then DPP butterflies.
//
//   Options whose [a, b] is widened by the log-strike clamp (double_heston.py:135-137) are
//   found and priced by the TABLE kernel (it already carries the CF code): per (p, group) it
//   writes a 64-bit mask word per 64 options and the clamped options' prices (per-term path on
//   the option's own range).  The option kernel only reads them, so it carries no CF code and
//   runs at ~100 VGPRs (4-5 waves per SIMD) instead of ~200.
//     Loss mode: fixed-order per-task partial of sum rel^2 and #invalid; the last task of p to
//     finish (agent-scope counter, sc1 hand-off) sums the partials in tile order.  No float
//     atomics: bitwise reproducible, independent of how many param sets share the launch.
//
//   Validation ("exact") mode runs cos_exact_kernel instead: per-term CF + sincos in the
//   reference's operation order, one wave per option.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <array>
#include <rccl/rccl.h>   // types only: librccl is resolved at run time (dlopen)
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <type_traits>
#include <string>
#include <type_traits>
#include <vector>

#include "dh_device.h"
#include "dh_lbfgs.h"
#include "dhcos.h"

using dh::cplx;
using dh::Params;

namespace {

constexpr int kBlock = 256;
constexpr int kTileMax = 256;
constexpr int kAnchor = 64;       // exact sincos re-anchor period of the angle recurrence
constexpr int kR = 4;             // options carried per lane in the option kernel
constexpr int kConsts = 8;        // c0, c1, c5, w0, a, b, e^b, e^a per table
constexpr size_t kTableBudget = size_t(256) << 20;   // table workspace per chunk (MALL-sized)
constexpr int kLdsMax = 160 * 1024;
constexpr int kLdsDyn = kLdsMax - 8192;   // dynamic LDS cap: the kernels keep <= 8 KB static

// Arrival counters of the loss hand-off, one per 128-byte line: every tile of a param set bumps
// its set's counter with an agent-scope atomic, and packed counters put all the sets of a
// request on one line, serialising every block's atomic (C2: 3.7k cycles per ticket).
constexpr int kCounterStride = 32;

struct PriceArgs {
    const double* prm;      // [P][16]
    int64_t P;              // param sets of the whole request
    int64_t p0, np;         // this launch covers param sets p0 .. p0 + np - 1
    const double* K;        // [M] sorted by T (absolute strike or K_relative)
    const double* T;        // [M]
    const int8_t* call;     // [M]
    const double* mkt;      // [M] or null
    const int* perm;        // [M] sorted -> caller index
    const int2* tiles;      // [n_tiles] (opt0, nopt)
    const int2* groups;     // [n_groups] (opt0, nopt) of each maturity group (null if paired)
    int max_group;          // largest group (clamp price slots per table)
    const int* tile_group;  // [n_tiles] maturity group of each tile
    const double* group_T;  // [n_groups]
    int n_tiles, n_groups;
    int opt_cap;            // >= largest tile (LDS option arrays)
    int paired;             // option i under param set i, one option per task
    int strike_mode;
    int exact;              // validation mode (host routes to cos_exact_kernel)
    int partials_only;      // 1: loss requests of the device L-BFGS-B: every task stores its partial
                            // (invalid flag in the sign bit) and ends (no hand-off); the step
                            // kernel forms the sums.  2: multi-round fused requests: every task
                            // stores its (partial, invalid count) pair and ends; loss_partials_kernel
                            // then forms the sums as the hand-off's last task would.  3: the same
                            // pairs as epoch-tagged granules (gran), summed by the grid's last
                            // P blocks in the same launch (tail_sums)
    int M;                  // options in the (sorted) option arrays
    int N;
    double L;
    double* out;            // prices [P*out_stride] or null
    int64_t out_stride;     // M (surface) or 0 (paired)
    double* part_sse;       // loss mode: [P*n_tiles] partials, else null
    int* part_bad;          // [P*n_tiles]
    unsigned* counter;      // [P * kCounterStride] arrival counters (zero between launches)
    double* sse;            // [P] final sums (loss mode)
    int* n_bad;             // [P]
    double* table;          // workspace: w_k, [np*tabs_per_p][N], or tiled (table_tiled) as
                            // [np*tabs_per_p / kTabTile][N][kTabTile]
    int table_tiled;        // set when cos_option_small_kernel reads the tables (table_w)
    double* consts;         // workspace: [np*tabs_per_p][kConsts]
    unsigned long long* cl_mask;   // workspace: [np*tabs_per_p][cl_words] clamp bits per option
    double* cl_price;       // workspace: [np*tabs_per_p][max_group] prices of clamped options
    unsigned long long* stamps;   // diagnostic builds (DH_STAMPS) only: [blocks][kStamps]
    const int* live_count;  // device-resident calibration: the launch is a no-op once every start
                            // has finished (*live_count == 0), else null
    const double* pre;      // fused kernel on large grids: [tables][kTabC] prologue constants
                            // formed by table_prologue_kernel ahead of it, else null
    double tail;            // tail_delta's scale: kTailScale, or -1 (dh_ctx_set_tail_cut(0): every
                            // term summed); set by launch_price
    // prologues ahead (fused kernel, requests of more than one round of resident blocks): block
    // q < ahead_stride (dispatch index) forms the truncation ranges and K_cf of the blocks
    // q + j ahead_stride (j = 1 .. kAheadMax) into ahead[.][kAheadRec] and then sets ahead_flag[.]
    // = ahead_epoch << 32 | K_cf; a later block whose flag holds this launch's epoch re-forms its
    // constants from the record instead of running the cumulant chain and the CF-cut test
    double* ahead;
    unsigned long long* ahead_flag;   // epoch << 32 | K_cf of the table's record
    int ahead_stride;       // 0: off
    unsigned ahead_epoch;
    // partials_only == 3: [P * n_tiles][2] granules (epoch-tagged halves of each task's pair)
    unsigned long long* gran;
    int remap;              // fused kernel: dispatch index -> table by XCD (xcd_table), else 0
    int host_out;           // sse / n_bad in mapped host memory (the host API's zero-copy
                            // requests): written by system-scope stores, drained (loss_out)
};

// w_k of table q sits at table_w(A, q)[k * table_step(A)].  The small-tile option kernel has one
// lane per table, so a row-major table puts every lane of a load on its own line (64 lines per
// wave-load, ~30% VALU issue in round 2); tiled, kTabTile consecutive tables share each line and
// a wave-load touches 4 lines.  The table kernel's writes then scatter over kTabTile-table lines
// that its 64-table batches fill within L2.
constexpr int kTabTile = 16;
__device__ __forceinline__ int table_step(const PriceArgs& A) { return A.table_tiled ? kTabTile : 1; }
__device__ __forceinline__ double* table_w(const PriceArgs& A, int64_t q) {
    return A.table_tiled ? A.table + (q / kTabTile) * kTabTile * (int64_t)A.N + (q % kTabTile)
                         : A.table + q * (int64_t)A.N;
}

// A launch enqueued ahead by dh_calibrate_lbfgs after its starts have all finished returns at
// once.  The count only changes between launches (the step kernel writes it), so every block of
// a launch takes the same branch and the loss hand-off counters stay consistent.
__device__ __forceinline__ bool halted(const PriceArgs& A) {
    return A.live_count && __builtin_amdgcn_readfirstlane(*A.live_count) <= 0;
}

// In-kernel phase stamps, compiled only into the diagnostic build (make stamps): lane 0 of each
// block of the option kernel writes s_memtime at its phase boundaries.
constexpr int kStamps = 32;     // [24, 28): HW_ID of waves 0..3 (SIMD placement)
#ifdef DH_STAMPS
#define DH_STAMP_T(A, i, thr)                                                              \
    do {                                                                                   \
        if ((A).stamps && threadIdx.x == (thr)) {                                          \
            unsigned long long _t;                                                         \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
            (A).stamps[(size_t)blockIdx.x * kStamps + (i)] = _t;                          \
        }                                                                                  \
    } while (0)
// the block's residency in the chip-wide 100 MHz clock (s_memrealtime): slot 23 = start << 32 |
// end, low 32 bits of each (tools/stamps.py --timeline)
#define DH_RT_BEGIN(A)                                                                     \
    unsigned long long _rt0 = 0;                                                           \
    if ((A).stamps && threadIdx.x == 0)                                                    \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_rt0)::"memory");    \
    if ((A).stamps && (threadIdx.x & 63) == 0 && threadIdx.x < 256) {                      \
        unsigned _hw;                                                                      \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(_hw));                  \
        (A).stamps[(size_t)blockIdx.x * kStamps + 24 + (threadIdx.x >> 6)] = _hw;          \
    }
#define DH_RT_END(A)                                                                       \
    do {                                                                                   \
        if ((A).stamps && threadIdx.x == 0) {                                              \
            unsigned long long _rt1;                                                       \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_rt1)::"memory"); \
            (A).stamps[(size_t)blockIdx.x * kStamps + 23] = (_rt0 << 32) | (_rt1 & 0xffffffffull); \
        }                                                                                  \
    } while (0)
#else
#define DH_STAMP_T(A, i, thr) do {} while (0)
#define DH_RT_BEGIN(A) do {} while (0)
#define DH_RT_END(A) do {} while (0)
#endif
#define DH_STAMP(A, i) DH_STAMP_T(A, i, 0)

__host__ __device__ inline int tabs_per_p(const PriceArgs& A) { return A.paired ? 1 : A.n_groups; }
__host__ __device__ inline int cl_words(const PriceArgs& A) { return (A.max_group + 63) / 64; }

// log(K / S0) and K / S0 (= e^{xK} to an ulp) of sorted option m under spot S0
__device__ __forceinline__ double option_logk(double K, double S0, double& ratio) {
    ratio = K / S0;
    return dh::dlog(ratio);                                          // double_heston.py:162
}

__device__ __forceinline__ double option_strike(const PriceArgs& A, int m, double S0) {
    const double Kin = A.K[m];
    return (A.strike_mode == DH_STRIKE_PCT_SPOT) ? Kin * S0 / 100.0 : Kin;
}

// ----------------------------------------------------------------------------------------------
// table kernel
// ----------------------------------------------------------------------------------------------
// Per-term path for a clamp-widened option: own range [a, b], own u grid, CF per term (fast
// exponent form) and the generic chi/psi (double_heston.py:141-158,160-192).  Lane share of
// the sum' over k = k_first, k_first + k_step, ...
__device__ __forceinline__ double clamped_term_sum(const Params& P, double T, double K, double xK,
                                                   double a, double b, bool is_call, int k_first,
                                                   int k_step, int N, const double2* sct) {
    const dh::CfConsts CC = dh::cf_consts(P, T);
    const double ba = b - a;
    const double scale = 2.0 / ba;
    double acc = 0.0;
    for (int k = k_first; k < N; k += k_step) {
        const double u = k * dh::kPi / ba;
        const double w = dh::cf_phase_re(CC, u, T, a, sct) * scale;
        double chi, psi;
        if (is_call) dh::cos_coeffs(k, xK, b, a, b, chi, psi);
        else dh::cos_coeffs(k, a, xK, a, b, chi, psi);
        const double V = is_call ? (P.S0 * chi - K * psi) : (K * psi - P.S0 * chi);
        acc += (k == 0 ? 0.5 : 1.0) * w * V;
    }
    return acc;
}

constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;
template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, Ctrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), Ctrl, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// the value of lane ^ 16 (or lane ^ 32): v_permlane16_swap / v_permlane32_swap of v with itself
// swap the odd rows (upper half) of the first copy with the even rows (lower half) of the second,
// so the second copy holds the partner's value in the even rows (lower half) and the first in the
// odd rows (upper half)
template <bool k32>
__device__ __forceinline__ double xor_partner(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    const bool upper = (__lane_id() & (k32 ? 32 : 16)) != 0;
    unsigned plo, phi;
    if constexpr (k32) {
        const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        plo = upper ? l[0] : l[1];
        phi = upper ? h[0] : h[1];
    } else {
        const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        plo = upper ? l[0] : l[1];
        phi = upper ? h[0] : h[1];
    }
    return __longlong_as_double(((long long)phi << 32) | plo);
}

// s summed over its aligned group of `width` lanes (a power of two <= 64) exactly as the xor
// butterfly s += __shfl_xor(s, off), off = 1, 2, 4, ... < width, sums it, without an LDS round
// trip per level: levels 1 and 2 are DPP quad permutes, levels 4 and 8 DPP half-row / row mirrors
// (after the lower levels every lane of a quad (half-row) holds the same value, so the mirror
// partner's operand is the xor partner's and every sum is the same bits), levels 16 and 32
// v_permlane16/32_swap.  Every lane of the wave must be active.
__device__ __forceinline__ double xor_sum(double s, int width) {
    if (width > 1) s += dpp_f64<kDppXor1>(s);
    if (width > 2) s += dpp_f64<kDppXor2>(s);
    if (width > 4) s += dpp_f64<kDppHalfMirror>(s);
    if (width > 8) s += dpp_f64<kDppMirror>(s);
    if (width > 16) s += xor_partner<false>(s);
    if (width > 32) s += xor_partner<true>(s);
    return s;
}

// Adaptive tail of the angle sums.  A table's terms k >= n_eff are not summed, n_eff - 1 being
// the last k >= 1 with |T2_k| > tail_delta.  Past it |T6_k| = |T2_k| / u_k <= |T2_k| (b - a)/pi,
// so the dropped part of S is at most (1 + (b - a)/pi) N delta = 2^-72 S0/(b - a), and a price
// moves by at most e^{-rT} e^{xK} 2^-72 S0/(b - a) = e^{-rT} 2^-72 K/(b - a): below 2^-64 of its
// own k = 0 term e^{-rT} w0 V0 (w0 = 1/(b - a); V0 >= 0.0048 K because the log-strike lies at
// least 0.1 inside [a, b] -- clamp-widened options take the per-term path), i.e. far inside the
// price's rounding.  The characteristic function decays like exp(-c u): at N = 512 (C3) a table
// keeps ~26% of its terms, at N = 256 ~46%, at N = 128 ~97%.  Every path forms n_eff from the
// same T2_k values with the same expressions, so fused and split keep their identical bits.
// NaN / inf entries (and a NaN delta) always count as kept: a NaN still reaches the price.
constexpr double kTailScale = 0x1.0p-72;
__device__ __forceinline__ double tail_delta(double scale, double S0, double ba, int N) {
    return scale * S0 / (ba * (1.0 + ba * (1.0 / dh::kPi)) * (double)N);
}
__device__ __forceinline__ int tail_keep(int k, double T2, double delta) {
    return fabs(T2) <= delta ? 0 : k + 1;
}
__device__ __forceinline__ int xor_max_i(int v, int width) {
    for (int off = 1; off < width; off <<= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

// Certified end of a table's CF entries.  For one Heston factor, conditioning on its variance
// path leaves a Gaussian part with variance (1 - rho^2) I (I = the integrated variance), so
// |phi_factor(u)| <= E[exp(-s I)] with s = u^2 (1 - rho^2) / 2: the CIR Laplace transform
// exp(A(s) - B(s) v0), which decreases in u; the jump factor's modulus is <= 1 (lambda >= 0) and
// the drift's is 1.  So |T2_k| <= 2 S0 M(u_k) / ((b - a)(1 + u_k^2)) =: bound(k), decreasing in
// k, and from the first k with bound(k) <= delta / 2 (tail_delta) on every entry would be dropped
// by the tail cut anyway: the CF is not evaluated there (K_cf, prologue slot 30).  The bound
// follows |phi| closely: at N = 512 (C3) K_cf is ~7 terms past n_eff, ~28% of N
// (tests/test_cf_cut_bound.py checks the bound against the oracle's CF).
// The test runs in fp32 at the native rate (v_exp / v_log / v_sqrt / v_rcp, ~1 ulp each; the
// errors, ~1e-6 relative on log values of magnitude < 1e3 near the threshold, sit far inside the
// 0.01 log-margin it keeps) on the
// candidates k_j = (j + 1) ceil(N / 64), j < 64: K_cf is the first that passes (else N).  The
// one-lane scan (table_prologue) and the wave's ballot (table_prologue_wave) test the same
// candidates with the same bits, so they pick the same one.  Series of N < 256 terms are not
// cut: at N = 128 (C1, C5) almost every term lies inside the bound.  At N = 256 (C2, C4) the cut
// costs C2 nothing now that the test runs on its own wave at the native fp32 rate, and C4 gains
// 2.5% (with the first, libm-rate test on wave 0 it had cost C2 12.1 -> 12.9 us).  Parameters
// outside the model's domain (kappa, sigma, T <= 0, theta, v0, lambda < 0, |rho| > 1, NaN) and a
// disabled tail cut (delta < 0) are not cut either.
constexpr int kCfCutMinN = 256;

// fp32 at the native rate: v_sqrt_f32, v_exp_f32 / v_log_f32 (base 2, ~1 ulp) and v_rcp_f32
__device__ __forceinline__ float f_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504f); }
__device__ __forceinline__ float f_log(float x) { return __builtin_amdgcn_logf(x) * 0.693147181f; }
__device__ __forceinline__ float f_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }

// log E[exp(-s I)] of one CIR factor, A(s) - B(s) v0, in a cancellation-free form.  The textbook
// A = (2 kappa theta / sigma^2) [log(2g) + (kappa - g) tau / 2 - log(den)] takes a difference of
// O(1) logs and scales it by 2 kappa theta / sigma^2: at small sigma the fp32 rounding of the logs
// is amplified past the test's margin.  With x = g tau, om = 1 - e^-x,
// h(x) = x - om >= 0, g - kappa = 2 sigma^2 s / (g + kappa) and den = 2g - (g - kappa) om:
//   A = -(2 kappa theta s / (g + kappa)) (h - om (R - 1)) / g,
//   R = -log(1 - y) / y,  y = sigma^2 s om / ((g + kappa) g) <= 1/2,
// where h and om come from one series for x < 1 (no 1 - e^-x cancellation) and R - 1 from its
// series for small y.  Each piece is within a few fp32 ulps, h - om (R - 1) cancels by at most a
// factor of 2 (om (R - 1) <= h / 2), and A, -B v0 are both <= 0: the log-bound is within ~1e-5
// relative of the exact one for every sigma > 0 (tests/test_cf_cut_bound.py, sigma down to 1e-6,
// kappa theta / sigma^2 up to 1e9).
__device__ __forceinline__ float cir_log_laplace(float s, float tau, float v0, float kap,
                                                 float th, float sig) {
#pragma clang fp contract(off)
    const float s2 = sig * sig;
    const float g = __builtin_amdgcn_sqrtf(kap * kap + 2.0f * s2 * s);
    const float gk = g + kap;
    const float x = g * tau;
    float h, om, e;
    if (x < 1.0f) {          // h = x^2/2 - x^3/6 + ... (Horner through x^11 / 11!: < 1e-8 rel.)
        float p = 1.0f / 39916800.0f;
        p = p * -x + 1.0f / 3628800.0f;
        p = p * -x + 1.0f / 362880.0f;
        p = p * -x + 1.0f / 40320.0f;
        p = p * -x + 1.0f / 5040.0f;
        p = p * -x + 1.0f / 720.0f;
        p = p * -x + 1.0f / 120.0f;
        p = p * -x + 1.0f / 24.0f;
        p = p * -x + 1.0f / 6.0f;
        p = p * -x + 0.5f;
        h = p * (x * x);
        om = x - h;
        e = 1.0f - om;
    } else {
        e = f_exp(-x);
        om = 1.0f - e;
        h = x - om;
    }
    const float y = f_div(s2 * s * om, gk * g);
    float rm1;               // R - 1 = y/2 + y^2/3 + y^3/4 + ...
    if (y < 0.125f) {
        float q = 1.0f / 9.0f;
        q = q * y + 1.0f / 8.0f;
        q = q * y + 1.0f / 7.0f;
        q = q * y + 1.0f / 6.0f;
        q = q * y + 1.0f / 5.0f;
        q = q * y + 0.25f;
        q = q * y + 1.0f / 3.0f;
        q = q * y + 0.5f;
        rm1 = q * y;
    } else {
        rm1 = f_div(-f_log(1.0f - y) - y, y);
    }
    const float D = f_div(h - om * rm1, g);
    const float A = -f_div(2.0f * kap * th * s, gk) * D;
    const float den = gk * om + 2.0f * g * e;
    const float B = f_div(2.0f * s * om, den);
    return A - B * v0;
}

__device__ __forceinline__ bool cf_cut_domain(const dh::Params& P, double T, double delta, int N) {
    return N >= kCfCutMinN && delta > 0.0 &&
           P.k1 > 0.0 && P.t1 >= 0.0 && P.s1 > 0.0 && P.v01 >= 0.0 && fabs(P.r1) <= 1.0 &&
           P.k2 > 0.0 && P.t2 >= 0.0 && P.s2 > 0.0 && P.v02 >= 0.0 && fabs(P.r2) <= 1.0 &&
           P.lam >= 0.0 && T > 0.0 && P.S0 > 0.0;
}

// log(delta / 2) less the margin: the candidates' threshold (fp32, native rate; delta > 0 and
// far above fp32's normal range: ~2^-80 S0)
__device__ __forceinline__ float cf_cut_threshold(double delta) {
    return f_log(0.5f * (float)delta) - 0.01f;
}

// bound(k) <= delta / 2 with the margin, in logs, fp32
__device__ __forceinline__ bool cf_cut_passes(const dh::Params& P, float T, float ba, float thr,
                                              int k) {
#pragma clang fp contract(off)
    const float u = (float)k * f_div(3.14159265f, ba);
    const float u2 = u * u;
    const float lm =
        cir_log_laplace(0.5f * u2 * (1.0f - (float)P.r1 * (float)P.r1), T, (float)P.v01,
                        (float)P.k1, (float)P.t1, (float)P.s1) +
        cir_log_laplace(0.5f * u2 * (1.0f - (float)P.r2 * (float)P.r2), T, (float)P.v02,
                        (float)P.k2, (float)P.t2, (float)P.s2);
    return f_log(f_div(2.0f * (float)P.S0, ba * (1.0f + u2))) + lm <= thr;
}

__host__ __device__ constexpr int cf_cut_step(int N) { return (N + 63) / 64; }

__device__ __forceinline__ int cf_cut_scan(const dh::Params& P, double T, double a, double b,
                                           double delta, int N) {
    if (!cf_cut_domain(P, T, delta, N)) return N;
    const float thr = cf_cut_threshold(delta), ba = (float)(b - a);
    const int st = cf_cut_step(N);
    for (int j = 0; j < 64; ++j) {
        const int k = (j + 1) * st;
        if (k >= N) break;
        if (cf_cut_passes(P, (float)T, ba, thr, k)) return k;
    }
    return N;
}

__device__ __forceinline__ int cf_cut_wave(const dh::Params& P, double T, double a, double b,
                                           double delta, int N, int lane) {
    if (!cf_cut_domain(P, T, delta, N)) return N;           // uniform
    const int st = cf_cut_step(N);
    const int k = (lane + 1) * st;
    const bool ok = k < N && cf_cut_passes(P, (float)T, (float)(b - a), cf_cut_threshold(delta), k);
    const unsigned long long m = __ballot(ok);
    return m ? (__ffsll((long long)m)) * st : N;      // lowest passing lane j: (j + 1) st
}

// per-table values staged in LDS by the prologue lane of the table:
//   [0..5] a, b, e^b, e^a, 2/(b-a), pi/(b-a) | [6..21] CfConsts | [22] S0, [23] r, [24] T,
//   [25] K/S0 below which the clamp test must be evaluated, [26] above which (prefilter),
//   [27] group's first option, [28] group size (as doubles), [29] the discount e^{-rT},
//   [30] K_cf: the CF entries k < K_cf are evaluated (cf_cut_scan), as a double
constexpr int kTabC = 31;
constexpr double kClampMargin = 1e-9;   // relative safety margin of the K-space prefilter
static_assert(sizeof(dh::CfConsts) == 16 * sizeof(double), "CfConsts layout");

// Prologue of table q = (p, g) of a launch: truncation range, CF constants and the staged values
// above, written to c[0 .. kTabC).
__device__ __forceinline__ void table_prologue(const PriceArgs& A, int64_t q, double* c,
                                               bool with_cut = true) {
#pragma clang fp contract(off)   // table_prologue and table_prologue_wave: same bits
    const int tpp = tabs_per_p(A);
    const int64_t p = A.p0 + q / tpp;
    const int g = (int)(q % tpp);
    const Params P = dh::load_params(A.prm + p * DH_PARAM_STRIDE);
    const double T = A.paired ? A.T[p] : A.group_T[g];
    int2 gr = make_int2((int)p, 1);
    if (!A.paired) gr = A.groups[g];
    double a, b;
    dh::trunc_unclamped(P, T, A.L, a, b);            // double_heston.py:100-132
    const dh::CfConsts CC = dh::cf_consts(P, T);
    c[0] = a;
    c[1] = b;
    c[2] = exp(b);
    c[3] = exp(a);
    c[4] = 2.0 / (b - a);
    c[5] = dh::kPi / (b - a);
    const double* cc = (const double*)&CC;
    for (int i = 0; i < 16; ++i) c[6 + i] = cc[i];
    c[22] = P.S0;
    c[23] = P.r;
    c[24] = T;
    // unclamped iff a + 0.1 <= log(K/S0) <= b - 0.1: strikes whose K/S0 is inside these
    // bounds by a 1e-9 relative margin cannot be clamped (exp/log errors are ~1e-16)
    c[25] = exp(a + 0.1) * (1.0 + kClampMargin);
    c[26] = exp(b - 0.1) * (1.0 - kClampMargin);
    c[27] = gr.x;
    c[28] = gr.y;
    c[29] = exp(-P.r * T);
    if (with_cut) c[30] = cf_cut_scan(P, T, a, b, tail_delta(A.tail, P.S0, b - a, A.N), A.N);
}

// table_prologue run by one wave in lockstep (the fused kernel's wave 0): the two variance
// factors' cumulants and CF constants on alternate lanes, the five exponentials (e^b, e^a, the
// clamp bounds' e^(a+0.1) and e^(b-0.1), and the jump compensator's e^(mu + sj^2/2)) one per lane,
// broadcast with readlane.  Every value is the same expression on the same inputs as in
// table_prologue and cf_consts, so the staged constants are the same bits.
__device__ __forceinline__ double lane_bcast(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// The fused kernel's leading arguments: what its prologue reads first.  As plain scalar kernel
// arguments ahead of PriceArgs they are preloaded into SGPRs at wave launch (gfx950 kernarg
// preloading, -mllvm -amdgpu-kernarg-preload-count, Makefile), so the parameter, maturity and
// group loads issue at once instead of behind a kernel-argument load (one memory round trip
// less on the request's critical path).  The fused launch has p0 = 0.
struct FusedHead {
    const double* prm;      // PriceArgs::prm
    const double* tsrc;     // PriceArgs::T (paired) or ::group_T
    const int2* groups;     // PriceArgs::groups
    const int* live;        // PriceArgs::live_count, or kLiveOne when null
    const double* pre;      // PriceArgs::pre
    int tpp;                // tabs_per_p
    int paired;
};

// A by-value kernel argument read in place: its fields load from the kernel-argument segment at
// their uses.  (Every use of a by-value argument is lowered to a load in the kernel's entry block;
// with the SGPR file full the compiler then spills them to VGPR lanes at once, which waits for the
// whole load before the prologue's first memory access can issue.)  off = the argument's byte
// offset in the segment: the preceding arguments at their natural alignment.
template <typename T, int off>
__device__ __forceinline__ const T& karg_ref() {
    typedef const __attribute__((address_space(4))) char* KargPtr;
    const KargPtr k = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
    return *(const T*)(const char*)(k + off);
}
// FusedHead's arguments: 5 pointers and 2 ints, so PriceArgs starts at byte 48 (kernel arguments
// are laid out in declaration order at their natural alignment, as the members of this struct)
constexpr int kFusedArgsKernargOff = 48;
struct FusedKargs {         // cos_fused_kernel's argument list as a struct (its kernarg layout)
    const double* prm;
    const double* tsrc;
    const int2* groups;
    const int* live;
    const double* pre;
    int tpp, paired;
    PriceArgs A;
};
static_assert(offsetof(FusedKargs, A) == kFusedArgsKernargOff, "PriceArgs kernarg offset");

// Small requests' param records in the kernel arguments (cos_fused_kernel<..., KP = true>): the
// host driver's function+gradient requests of one start (14 records) travel in the
// launch's kernel-argument segment, which the runtime writes to device memory ahead of the
// dispatch, instead of being read by the blocks from mapped host memory across PCIe at the start
// of the request's critical path (C1: 11.9 -> 10.1 us per kernel with the records in HBM).  One
// start's 14 records: 1,792 bytes, 2,416 with the rest of the arguments and 2,672 with the
// runtime's hidden ones (28 records would pass the 4 KiB segment).
constexpr int kKargSets = 14;
// and, for surfaces of at most kKargGroups maturity groups (C1's 3, C2's 32), the groups' maturities
// and option ranges: the prologue's first dependent load (the table's T) then comes from the
// kernel-argument segment too instead of device memory (C2 prologue chain: one memory round trip)
constexpr int kKargGroups = 32;
struct KargParams {
    double v[kKargSets * DH_PARAM_STRIDE];
    double T[kKargGroups];
    int2 groups[kKargGroups];
};
struct NoKargParams {
    int unused;
};
struct FusedKargsKP {       // cos_fused_kernel<..., true>'s argument list
    FusedKargs head;
    int tpt2;
    KargParams pb;
};
constexpr int kFusedParamsKernargOff = 384;
static_assert(offsetof(FusedKargsKP, pb) == kFusedParamsKernargOff, "param block kernarg offset");
static_assert(sizeof(FusedKargsKP) + 256 <= 4096, "kernel arguments over 4 KiB");

#ifndef DH_PRE_GROUP8
#define DH_PRE_GROUP8 1
#endif
#ifndef DH_KARG_PREFETCH
#define DH_KARG_PREFETCH 1
#endif
// The kernel-argument lines the fused kernel reads PriceArgs from (in place, karg_ref; the step
// kernel's LbArgs lie in the same byte range), pulled
// into the scalar cache in ONE round trip at entry: one s_load_dword per 64-byte line brings the
// whole line, and the wave waits once.  Without it the prologue's path met each line as its own
// dependent round trip (xcd_table's switch, the ahead stride, the tail-cut and table fields: five
// serial ~550-cycle misses before the table record could be loaded, tools/ubench/kernarg_latency).
// The lines are 64 bytes apart from byte 0x30 through 0x1b0 (PriceArgs and the arguments after
// it), so every line is touched whatever the segment's alignment.
__device__ __forceinline__ void karg_prefetch_lines() {
#if DH_KARG_PREFETCH
    const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    unsigned d0, d1, d2, d3, d4, d5, d6;
    asm volatile(
        "s_load_dword %0, %7, 0x30\n\t"
        "s_load_dword %1, %7, 0x70\n\t"
        "s_load_dword %2, %7, 0xb0\n\t"
        "s_load_dword %3, %7, 0xf0\n\t"
        "s_load_dword %4, %7, 0x130\n\t"
        "s_load_dword %5, %7, 0x170\n\t"
        "s_load_dword %6, %7, 0x1b0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(d0), "=s"(d1), "=s"(d2), "=s"(d3), "=s"(d4), "=s"(d5), "=s"(d6)
        : "s"(ka)
        : "memory");
#endif
}

// the live count read by launches without one (FusedHead::live): the halt test is then a load
// like any other, with no branch on the pointer (a branch made the compiler wait for it at the
// kernel's entry)
__device__ const int kLiveOne = 1;

// The table (p * tpp + g) the fused grid's block of dispatch index b prices.  With A.remap the
// blocks that share an XCD (b and b + 8: MI355X_MICROARCH.md, round-robin dispatch, observed, for
// speed only) take, in dispatch order, one contiguous run of the tables in maturity-major order
// (g * P + p): each XCD's L2 then holds ~1/8 of the option arrays, and the blocks running together
// on an XCD stage the same maturity group's options.  A bijection onto the grid's tables for any
// grid size, so any placement gives the same bits.
__device__ __forceinline__ int64_t xcd_table(const PriceArgs& A, int tpp, int64_t b) {
    if (!A.remap) return b;
    const unsigned nb = gridDim.x;
    const unsigned x = (unsigned)b & 7u, pos = (unsigned)b >> 3;
    const unsigned per = nb >> 3, extra = nb & 7u;
    const unsigned t = x * per + min(x, extra) + pos;        // maturity-major rank
    const unsigned np = nb / (unsigned)tpp;
    const unsigned g = t / np, p = t - g * np;
    return (int64_t)p * tpp + g;
}

// The truncation range of table q (trunc_unclamped's bits) with the two variance factors'
// cumulants on alternate lanes: table_prologue_wave's first step, and the whole of what
// prologue_cut_wave needs.
__device__ __forceinline__ void prologue_range_wave(const PriceArgs& A, const FusedHead& H,
                                                    int64_t q, int lane, Params& P, double& T,
                                                    double& a, double& b) {
#pragma clang fp contract(off)   // table_prologue and table_prologue_wave: same bits
    const int64_t p = (int64_t)((unsigned)q / (unsigned)H.tpp);
    const int g = (int)((unsigned)q % (unsigned)H.tpp);
    P = dh::load_params(H.prm + p * DH_PARAM_STRIDE);
    T = H.tsrc[H.paired ? p : g];
#ifdef DH_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the record and T (scalar loads) are in
#endif
    DH_STAMP_T(A, 31, 0);
    const bool two = lane & 1;                     // factor 2 on odd lanes
    const double v0 = two ? P.v02 : P.v01, k = two ? P.k2 : P.k1, th = two ? P.t2 : P.t1;
    const double sg = two ? P.s2 : P.s1, rh = two ? P.r2 : P.r1;
    double c1j, c2j;
    dh::factor_cumulants(T, P.r, v0, k, th, sg, rh, c1j, c2j);   // double_heston.py:101-118
    const double c1 = lane_bcast(c1j, 0) + lane_bcast(c1j, 1) + P.lam * T * P.muj;
    const double c2 = lane_bcast(c2j, 0) + lane_bcast(c2j, 1) +
                      P.lam * T * (P.sj * P.sj + P.muj * P.muj);
    const double h = A.L * sqrt(fabs(c2));
    a = c1 - h;                                    // trunc_unclamped (double_heston.py:120-132)
    b = c1 + h;
}

// K_cf of table q by one wave (cf_cut_wave on prologue_range_wave's range): in the fused kernel
// a wave other than the prologue's runs it, so the bound's fp32 chain overlaps the prologue's
// instead of following it.
__device__ __forceinline__ int prologue_cut_wave(const PriceArgs& A, const FusedHead& H,
                                                 int64_t q, int lane) {
    Params P;
    double T, a, b;
    prologue_range_wave(A, H, q, lane, P, T, a, b);
    return cf_cut_wave(P, T, a, b, tail_delta(A.tail, P.S0, b - a, A.N), A.N, lane);
}

// with_cut: also K_cf (slot 30); else the caller's other wave stores it
__device__ __forceinline__ void table_prologue_wave(const PriceArgs& A, const FusedHead& H,
                                                    int64_t q, double* c, int lane,
                                                    bool with_cut) {
#pragma clang fp contract(off)   // table_prologue and table_prologue_wave: same bits
    Params P;
    double T, a, b;
    prologue_range_wave(A, H, q, lane, P, T, a, b);
    DH_STAMP_T(A, 28, 0);
    const int64_t p = (int64_t)((unsigned)q / (unsigned)H.tpp);
    const int g = (int)((unsigned)q % (unsigned)H.tpp);
    int2 gr = make_int2((int)p, 1);
    if (!H.paired) gr = H.groups[g];
    const bool two = lane & 1;                     // factor 2 on odd lanes
    const double v0 = two ? P.v02 : P.v01, k = two ? P.k2 : P.k1, th = two ? P.t2 : P.t1;
    const double sg = two ? P.s2 : P.s1, rh = two ? P.r2 : P.r1;
    const dh::FactorC Fj = dh::factor_consts(v0, k, th, sg, rh);
    const int e_lane = lane < 6 ? lane : 0;
    const double arg = e_lane == 0 ? b : e_lane == 1 ? a : e_lane == 2 ? a + 0.1
                     : e_lane == 3 ? b - 0.1 : e_lane == 4 ? P.muj + 0.5 * (P.sj * P.sj)
                     : -P.r * T;
    const double e = exp(arg);
    dh::CfConsts CC;
    double* f1 = (double*)&CC.f1;
    double* f2 = (double*)&CC.f2;
    const double* fj = (const double*)&Fj;
    for (int i = 0; i < (int)(sizeof(dh::FactorC) / 8); ++i) {
        f1[i] = lane_bcast(fj[i], 0);
        f2[i] = lane_bcast(fj[i], 1);
    }
    const double comp = lane_bcast(e, 4) - 1.0;    // cf_consts
    CC.drift = (P.r - P.q - P.lam * comp) * T;
    CC.half_sj2 = 0.5 * (P.sj * P.sj);
    CC.muj = P.muj;
    CC.lt = P.lam * T;
    DH_STAMP_T(A, 30, 0);
    const int kcf =
        with_cut ? cf_cut_wave(P, T, a, b, tail_delta(A.tail, P.S0, b - a, A.N), A.N, lane) : 0;
    if (lane == 0) {
        c[0] = a;
        c[1] = b;
        c[2] = e;
        c[3] = lane_bcast(e, 1);
        c[4] = 2.0 / (b - a);
        c[5] = dh::kPi / (b - a);
        const double* cc = (const double*)&CC;
        for (int i = 0; i < 16; ++i) c[6 + i] = cc[i];
        c[22] = P.S0;
        c[23] = P.r;
        c[24] = T;
        c[25] = lane_bcast(e, 2) * (1.0 + kClampMargin);
        c[26] = lane_bcast(e, 3) * (1.0 - kClampMargin);
        c[27] = gr.x;
        c[28] = gr.y;
        c[29] = lane_bcast(e, 5);
        if (with_cut) c[30] = kcf;
    }
}

// cf_cut_scan by a group of 8 lanes (sub = 0..7; the group's lanes are active together): the
// candidates in chunks of 8 in increasing j, each chunk's first passing lane from the wave's
// ballot, so the same first passing candidate -- the same K_cf -- as the one-lane scan.
constexpr int kPreLanes = 8;
__device__ __forceinline__ int cf_cut_group8(const dh::Params& P, double T, double a, double b,
                                             double delta, int N, int sub) {
    if (!cf_cut_domain(P, T, delta, N)) return N;              // uniform in the group
    const float thr = cf_cut_threshold(delta), ba = (float)(b - a);
    const int st = cf_cut_step(N);
    const int sh = (int)(__lane_id() & ~(kPreLanes - 1));      // the group's bits in the ballot
    for (int j0 = 0; j0 < 64; j0 += kPreLanes) {
        if ((j0 + 1) * st >= N) break;                         // every candidate left is >= N
        const int k = (j0 + sub + 1) * st;
        const bool ok = k < N && cf_cut_passes(P, (float)T, ba, thr, k);
        const unsigned m = (unsigned)(__ballot(ok) >> sh) & ((1u << kPreLanes) - 1u);
        if (m) return (j0 + __ffs((int)m)) * st;               // j = j0 + ffs - 1, k = (j + 1) st
    }
    return N;
}

// ----------------------------------------------------------------------------------------------
// Prologues ahead (round 5).  A fused request of more than one round of resident blocks (C3:
// 4,200 tables on 1,024 slots) spends ~18% of every block's chain, and ~1,000 wave-instructions
// per table, on the serial prologue (table_prologue_wave + the CF-cut test).  Its first-round
// blocks form the later-round tables' prologues on the cut wave during the CF loop, which leaves
// that wave idle on C3's tables: 8 lanes per table (the two variance factors on sub-lanes 0 and 1,
// the six exponentials on sub-lanes 0 .. 5: table_prologue_wave's expressions on the same
// operands, uncontracted, so the same bits), the CF-cut candidates 8 at a time (cf_cut_group8:
// the same first passing candidate as the wave's ballot).  The constants go out with agent-scope
// stores; once drained (s_waitcnt vmcnt(0)), after the block's CF barrier a flag per table takes
// the launch's epoch -- MI355X_MICROARCH.md's "valid forms" row 1, as the loss hand-off.  A later
// block reads its flag: set, it loads the record (wave 0) and K_cf (the cut wave); not set (its
// writer has not got there: never seen, dispatch runs in block order and a later block starts only
// after a whole block lifetime), it forms them itself.  Either way the same values, so the same
// bits.
// ----------------------------------------------------------------------------------------------
constexpr int kAheadMax = 8;       // later tables per first-round block: 8-lane groups of a wave
// What travels per later table: the prologue's values that cost a transcendental or a cumulant
// chain -- a, b, e^b, e^a, the clamp bounds' slots 25 and 26, e^{-rT} and the CF drift -- at
// ahead[q * kAheadRec + i] (one 64-byte record per table, the writer group's 8 lanes storing it in
// one coalesced store), and K_cf in the low half of the table's 64-bit flag (its high half the
// launch's epoch); the reader re-forms the cheap slots (2/(b - a), pi/(b - a), the factors'
// constants, S0, r, T, the group) from the parameters by the same expressions.  (Round 5 sent K_cf
// in the record, one 128-byte line per table: 541 KB written per C3 request.  Sending (a, b) alone
// and re-forming the six exponentials in the reader halved the writes again but cost C3 1.3 us.)
constexpr int kAheadRec = 8;
// v of lane (lane & ~7) | l: the 8-lane group's broadcast
__device__ __forceinline__ double grp8_bcast(double v, int l) {
    const int src = ((int)__lane_id() & ~7) | l;
    const long long b = __double_as_longlong(v);
    const int lo = __shfl((int)b, src, 64);
    const int hi = __shfl((int)(b >> 32), src, 64);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ void agent_store(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double agent_load(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The later table of 8-lane group lane / 8 of first-round block q0: q0 + (j + 1) R (act: it
// exists; an inactive group runs in step on q0's own table and stores nothing).  Dispatch indices:
// the table each one prices is xcd_table's
__device__ __forceinline__ int64_t ahead_table(const PriceArgs& A, int64_t q0, int64_t nblocks,
                                               int lane, bool& act) {
    const int64_t qa = q0 + (int64_t)((lane >> 3) + 1) * A.ahead_stride;
    act = qa < nblocks;
    return act ? qa : q0;
}
// The writer (a first-round block's cut wave, during the CF loop, which leaves it idle on C3's
// tables): for the tables of dispatch indices q0 + (j + 1) R, j = lane / 8, the record's 8 values
// into ahead[], then its stores drained (the flags, which carry K_cf -- returned on sub-lane 0 --
// follow the block's CF barrier)
__device__ __forceinline__ int ahead_write(const PriceArgs& A, const FusedHead& H, int64_t q0,
                                           int64_t nblocks, int lane) {
#pragma clang fp contract(off)   // table_prologue and table_prologue_wave: same bits
    const int sub = lane & 7;
    bool act;
    const int64_t qa = ahead_table(A, q0, nblocks, lane, act);
    const int64_t q = xcd_table(A, H.tpp, qa);
    const int64_t p = (int64_t)((unsigned)q / (unsigned)H.tpp);
    const int g = (int)((unsigned)q % (unsigned)H.tpp);
    const Params P = dh::load_params(H.prm + p * DH_PARAM_STRIDE);
    const double T = H.tsrc[H.paired ? p : g];
    const bool two = sub & 1;                      // factor 2 on odd sub-lanes
    const double v0 = two ? P.v02 : P.v01, k = two ? P.k2 : P.k1, th = two ? P.t2 : P.t1;
    const double sg = two ? P.s2 : P.s1, rh = two ? P.r2 : P.r1;
    double c1j, c2j;
    dh::factor_cumulants(T, P.r, v0, k, th, sg, rh, c1j, c2j);   // double_heston.py:101-118
    const double c1 = grp8_bcast(c1j, 0) + grp8_bcast(c1j, 1) + P.lam * T * P.muj;
    const double c2 = grp8_bcast(c2j, 0) + grp8_bcast(c2j, 1) +
                      P.lam * T * (P.sj * P.sj + P.muj * P.muj);
    const double h = A.L * sqrt(fabs(c2));
    const double a = c1 - h;                       // trunc_unclamped (double_heston.py:120-132)
    const double b = c1 + h;
    const int e_lane = sub < 6 ? sub : 0;
    const double arg = e_lane == 0 ? b : e_lane == 1 ? a : e_lane == 2 ? a + 0.1
                     : e_lane == 3 ? b - 0.1 : e_lane == 4 ? P.muj + 0.5 * (P.sj * P.sj)
                     : -P.r * T;
    const double e = exp(arg);
    const double comp = grp8_bcast(e, 4) - 1.0;    // cf_consts
    const double drift = (P.r - P.q - P.lam * comp) * T;
    // record value sub of the group's table: a, b, e^b, e^a, slot 25, slot 26, e^{-rT}, drift.
    // The shuffles run on every lane, outside the selection: a lane shuffle inside a branch would
    // read the branch's inactive lanes (sub-lanes 0 and 1 hold e^b and e^a)
    const double e2 = grp8_bcast(e, 2), e3 = grp8_bcast(e, 3);
    const double es = grp8_bcast(e, sub == 2 ? 0 : sub == 3 ? 1 : 5);
    double v = sub == 0 ? a : sub == 1 ? b : es;
    v = sub == 4 ? e2 * (1.0 + kClampMargin) : v;
    v = sub == 5 ? e3 * (1.0 - kClampMargin) : v;
    v = sub == 7 ? drift : v;
    if (act) agent_store(A.ahead + qa * kAheadRec + sub, v);
    // K_cf of the group's table by cf_cut_group8 on the same operands (the same first passing
    // candidate as the wave's ballot), then every store of the wave drained
    const int kcf = A.N < kCfCutMinN
                        ? A.N
                        : cf_cut_group8(P, T, a, b, tail_delta(A.tail, P.S0, b - a, A.N), A.N, sub);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return kcf;
}

// The reader (wave 0 of a later block whose flag holds this launch's epoch): the record of dispatch
// index q and table qt's cheap slots re-formed from the parameters, into c[0 .. 30) --
// table_prologue_wave's expressions on the same operands, uncontracted, so the same bits
__device__ __forceinline__ void ahead_read(const PriceArgs& A, const FusedHead& H, int64_t q,
                                           int64_t qt, double* c, int lane) {
#pragma clang fp contract(off)   // table_prologue and table_prologue_wave: same bits
    const double v = agent_load(A.ahead + q * kAheadRec + (lane & 7));
    const int64_t p = (int64_t)((unsigned)qt / (unsigned)H.tpp);
    const int g = (int)((unsigned)qt % (unsigned)H.tpp);
    const Params P = dh::load_params(H.prm + p * DH_PARAM_STRIDE);
    const double T = H.tsrc[H.paired ? p : g];
    int2 gr = make_int2((int)p, 1);
    if (!H.paired) gr = H.groups[g];
    const double a = lane_bcast(v, 0), b = lane_bcast(v, 1);
    const bool two = lane & 1;                     // factor 2 on odd lanes (table_prologue_wave)
    const dh::FactorC Fj = two ? dh::factor_consts(P.v02, P.k2, P.t2, P.s2, P.r2)
                               : dh::factor_consts(P.v01, P.k1, P.t1, P.s1, P.r1);
    const double* fj = (const double*)&Fj;
    double f1[6], f2[6];
    for (int i = 0; i < 6; ++i) {
        f1[i] = lane_bcast(fj[i], 0);
        f2[i] = lane_bcast(fj[i], 1);
    }
    if (lane == 0) {
        c[0] = a;
        c[1] = b;
        c[2] = lane_bcast(v, 2);
        c[3] = lane_bcast(v, 3);
        c[4] = 2.0 / (b - a);
        c[5] = dh::kPi / (b - a);
        for (int i = 0; i < 6; ++i) {
            c[6 + i] = f1[i];
            c[12 + i] = f2[i];
        }
        c[18] = lane_bcast(v, 7);                  // drift
        c[19] = 0.5 * (P.sj * P.sj);               // half_sj2
        c[20] = P.muj;
        c[21] = P.lam * T;                         // lt
        c[22] = P.S0;
        c[23] = P.r;
        c[24] = T;
        c[25] = lane_bcast(v, 4);
        c[26] = lane_bcast(v, 5);
        c[27] = gr.x;
        c[28] = gr.y;
        c[29] = lane_bcast(v, 6);
    }
}

// The flags, after the writer's stores drained and a barrier (every lane of a wave calls this;
// kcf: ahead_write's value, read on sub-lane 0)
__device__ __forceinline__ void ahead_publish(const PriceArgs& A, int64_t q0, int64_t nblocks,
                                              int lane, int kcf) {
    bool act;
    const int64_t qa = ahead_table(A, q0, nblocks, lane, act);
    if ((lane & 7) == 0 && act)
        __hip_atomic_store(&A.ahead_flag[qa],
                           ((unsigned long long)A.ahead_epoch << 32) | (unsigned)kcf,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The reader: this launch's record of dispatch index q is in ahead[] (a wave-uniform answer), with
// its K_cf
__device__ __forceinline__ bool ahead_ready(const PriceArgs& A, int64_t q, int& kcf) {
    const unsigned long long f = __hip_atomic_load(&A.ahead_flag[q], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(f >> 32));
    kcf = (int)__builtin_amdgcn_readfirstlane((unsigned)f);
    return hi == A.ahead_epoch;
}


// Every table's prologue of a large fused request ahead of the fused launch (launch_fused): the
// fused blocks then load their constants instead of running the one-wave prologue chain while
// their other waves wait at the barrier.  A group of kPreLanes lanes per table: each runs
// table_prologue's chain (the bits of every other path), then the CF-cut candidates are tested
// 8 at a time (cf_cut_group8) instead of one after another (C4 at N = 256: ~30 candidates).
__global__ __launch_bounds__(kBlock) void table_prologue_kernel(PriceArgs A, int64_t n_q,
                                                                double* out) {
    if (halted(A)) return;
    const int64_t gid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t q = gid / kPreLanes;
    const int sub = (int)(gid % kPreLanes);
    if (q >= n_q) return;                                      // whole groups (kBlock % 8 == 0)
#if DH_PRE_GROUP8
    // the chain spread over the group as in ahead_write: the two factors' cumulants on sub-lanes 0
    // and 1, the six exponentials one per sub-lane, shuffled to the group -- table_prologue's
    // expressions on the same operands, uncontracted, so the same bits
  {
#pragma clang fp contract(off)
    const int tpp = tabs_per_p(A);
    const int64_t p = A.p0 + q / tpp;
    const int g = (int)(q % tpp);
    const Params P = dh::load_params(A.prm + p * DH_PARAM_STRIDE);
    const double T = A.paired ? A.T[p] : A.group_T[g];
    int2 gr = make_int2((int)p, 1);
    if (!A.paired) gr = A.groups[g];
    const bool two = sub & 1;
    const double v0 = two ? P.v02 : P.v01, k = two ? P.k2 : P.k1, th = two ? P.t2 : P.t1;
    const double sg = two ? P.s2 : P.s1, rh = two ? P.r2 : P.r1;
    double c1j, c2j;
    dh::factor_cumulants(T, P.r, v0, k, th, sg, rh, c1j, c2j);   // double_heston.py:101-118
    const double c1 = grp8_bcast(c1j, 0) + grp8_bcast(c1j, 1) + P.lam * T * P.muj;
    const double c2 = grp8_bcast(c2j, 0) + grp8_bcast(c2j, 1) +
                      P.lam * T * (P.sj * P.sj + P.muj * P.muj);
    const double h = A.L * sqrt(fabs(c2));
    const double a = c1 - h;                       // trunc_unclamped (double_heston.py:120-132)
    const double b = c1 + h;
    const int e_lane = sub < 6 ? sub : 0;
    const double arg = e_lane == 0 ? b : e_lane == 1 ? a : e_lane == 2 ? a + 0.1
                     : e_lane == 3 ? b - 0.1 : e_lane == 4 ? P.muj + 0.5 * (P.sj * P.sj)
                     : -P.r * T;
    const double e = exp(arg);
    const double eb = grp8_bcast(e, 0), ea = grp8_bcast(e, 1), e2 = grp8_bcast(e, 2);
    const double e3 = grp8_bcast(e, 3), e4 = grp8_bcast(e, 4), e5 = grp8_bcast(e, 5);
    const int kcf = cf_cut_group8(P, T, a, b, tail_delta(A.tail, P.S0, b - a, A.N), A.N, sub);
    if (sub == 0) {
        const dh::FactorC F1 = dh::factor_consts(P.v01, P.k1, P.t1, P.s1, P.r1);
        const dh::FactorC F2 = dh::factor_consts(P.v02, P.k2, P.t2, P.s2, P.r2);
        const double comp = e4 - 1.0;              // cf_consts
        double* o = out + q * kTabC;
        o[0] = a;
        o[1] = b;
        o[2] = eb;
        o[3] = ea;
        o[4] = 2.0 / (b - a);
        o[5] = dh::kPi / (b - a);
        const double* f1 = (const double*)&F1;
        const double* f2 = (const double*)&F2;
        for (int i = 0; i < 6; ++i) {
            o[6 + i] = f1[i];
            o[12 + i] = f2[i];
        }
        o[18] = (P.r - P.q - P.lam * comp) * T;    // drift
        o[19] = 0.5 * (P.sj * P.sj);               // half_sj2
        o[20] = P.muj;
        o[21] = P.lam * T;                         // lt
        o[22] = P.S0;
        o[23] = P.r;
        o[24] = T;
        o[25] = e2 * (1.0 + kClampMargin);
        o[26] = e3 * (1.0 - kClampMargin);
        o[27] = gr.x;
        o[28] = gr.y;
        o[29] = e5;
        o[30] = kcf;
    }
  }
#else
    double c[kTabC];
    table_prologue(A, q, c, false);
    const int tpp = tabs_per_p(A);
    const int64_t p = A.p0 + q / tpp;
    const Params P = dh::load_params(A.prm + p * DH_PARAM_STRIDE);
    c[30] = cf_cut_group8(P, c[24], c[0], c[1], tail_delta(A.tail, c[22], c[1] - c[0], A.N), A.N,
                          sub);
    if (sub == 0) {
        double* o = out + q * kTabC;
        for (int i = 0; i < kTabC; ++i) o[i] = c[i];
    }
#endif
}

#ifndef DH_TABLE_WAVES
#define DH_TABLE_WAVES 3    // min waves per SIMD: caps VGPR+AGPR at 168 (3 waves per SIMD)
#endif
#ifndef DH_OPTION_WAVES
#define DH_OPTION_WAVES 1
#endif
#ifndef DH_FUSED_WAVES
#define DH_FUSED_WAVES 4    // caps VGPR+AGPR at 128 (4 waves per SIMD)
#endif
#ifndef DH_FUSED_WAVES_WIDE
#define DH_FUSED_WAVES_WIDE 5   // the one-option-per-lane-group variant for large grids (<= 96 VGPRs)
#endif
#ifndef DH_PRIO
#define DH_PRIO 1
#endif
// Wave priority on a block's serial phases (the prologue, the k-sums, the loss hand-off): the
// waves the rest of the block waits for at a barrier issue ahead of the other resident blocks'
// waves on their SIMD, whose CF and option sums fill the slots they leave.  Scheduling only:
// the same instructions, so the same bits.
__device__ __forceinline__ void serial_prio(bool on) {
    if constexpr (DH_PRIO > 0) {
        if (on) __builtin_amdgcn_s_setprio(DH_PRIO);
        else __builtin_amdgcn_s_setprio(0);
    }
}


// CF entries of one table slot (thread t of TPT): k = t, t + TPT, ..., emitted in increasing k
// (the k-sums' order) as emit(k, u_k, w_k).
template <int TPT, typename F>
__device__ __forceinline__ void table_entries(const dh::CfConsts& CC, int t, int N, double piba,
                                              double T, double a, double scale,
                                              const double2* sct, F&& emit) {
    for (int k = t; k < N; k += TPT) {
        const double u = k * piba;                                   // k pi / (b - a)
        emit(k, u, dh::cf_phase_re(CC, u, T, a, sct) * scale);
    }
}

// Grid: a fixed number of blocks (resident capacity), each owning a contiguous range of tables.
// Tables are taken in batches of up to kBatch: lane i of wave 0 computes the truncation range and
// CF constants of table i of the batch (one prologue latency for up to 64 tables), then every
// table slot (TPT threads) runs the CF loops of its tables back to back; per-table sums are
// finished in a fixed order at the end of the batch (bitwise independent of the grid).
constexpr int kBatch = 64;

// Slots of TPT = 64 form the per-table k-sums in registers, in the canonical order (lane l of the
// slot accumulates k = l, l + 64, ... then an xor butterfly); wider slots (fewer, fatter work
// units when a request has few tables per slot) store T2_k in LDS and let the slot's first wave
// re-form the same sums in the same order, so every slot width gives the same bits.
template <int TPT>
__global__ __launch_bounds__(kBlock, DH_TABLE_WAVES) void cos_table_kernel(PriceArgs A_) {
    const PriceArgs& A = karg_ref<PriceArgs, 0>();   // read in place (karg_ref)
    if (halted(A)) return;
    constexpr int kTabs = kBlock / TPT;      // table slots per block
    extern __shared__ __attribute__((aligned(16))) double t2s[];   // TPT > 64: [kTabs][N] T2_k
    __shared__ double shc[kBatch][kTabC];
    __shared__ double red[kBatch][4];
    __shared__ double w0s[kTabs];
    __shared__ double2 sct[dh::kMathTab];
    dh::load_sincos_table(sct);           // synchronised by the first batch's barrier
    const int slot = __builtin_amdgcn_readfirstlane(threadIdx.x / TPT);
    const int t = threadIdx.x % TPT;
    const int lane = threadIdx.x & 63;
    const int wv = t >> 6;
    const int N = A.N;
    const int tpp = tabs_per_p(A);
    const int64_t n_q = A.np * tpp;
    const int64_t q_begin = n_q * blockIdx.x / gridDim.x;
    const int64_t q_end = n_q * (blockIdx.x + 1) / gridDim.x;
    DH_STAMP(A, 4);

    for (int64_t b0 = q_begin; b0 < q_end; b0 += kBatch) {
        const int nb = (int)min<int64_t>(kBatch, q_end - b0);
        // ---- prologue, one lane per table: truncation range and CF constants ----
        if (threadIdx.x < nb) table_prologue(A, b0 + threadIdx.x, shc[threadIdx.x]);
        __syncthreads();
        if (b0 == q_begin) DH_STAMP(A, 5);

        for (int i0 = 0; i0 < nb; i0 += kTabs) {        // every thread runs every pass (barriers)
            const int i = i0 + slot;
            const bool has = i < nb;
            const int64_t q = b0 + i;
            const double* c = shc[has ? i : 0];
            const double a = c[0], b = c[1], eb = c[2], ea = c[3], scale = c[4], piba = c[5];
            const double S0 = c[22], T = c[24], lo = c[25], hi = c[26];
            const int g0 = (int)c[27], gn = has ? (int)c[28] : 0;
            const int kcf = (int)c[30];                  // CF entries k < K_cf (cf_cut_scan)
            double* t2 = t2s + (TPT > 64 ? slot * N : 0);
            double c0 = 0.0, c5 = 0.0, w0 = 0.0;
            const double delta = tail_delta(A.tail, S0, b - a, N);
            int ne = 0;
            if (has) {
                dh::CfConsts CC;
                {
                    double* cc = (double*)&CC;
                    for (int j = 0; j < 16; ++j) cc[j] = c[6 + j];
                }
                double* tw = table_w(A, q);
                const int ts = table_step(A);
                table_entries<TPT>(CC, t, kcf, piba, T, a, scale, sct, [&](int k, double u, double w) {
                    tw[k * ts] = w;
                    if (k == 0) {
                        w0 = 0.5 * w;
                        return;
                    }
                    // chi_k / psi_k at d = b: u (b - a) = k pi, so cos = (-1)^k and sin = 0
                    // exactly (the reference evaluates them with ~1e-16 rounding noise; c1 =
                    // sum T4 sin(.) is therefore 0 and kept only for the consts layout)
                    const double cb = (k & 1) ? -1.0 : 1.0;
                    const double T2 = w * S0 * dh::drcp(1.0 + u * u);
                    if (TPT == 64) {
                        c0 += T2 * eb * cb;
                        c5 += T2 * ea;
                        ne = max(ne, tail_keep(k, T2, delta));
                    } else {
                        t2[k] = T2;
                    }
                });
            }
            if (TPT > 64) {
                if (has && t == 0) w0s[slot] = w0;
                __syncthreads();
                if (has && wv == 0) {                          // the canonical 64-lane order
                    w0 = lane == 0 ? w0s[slot] : 0.0;
                    for (int k = lane; k < kcf; k += 64) {
                        if (k == 0) continue;
                        const double T2 = t2[k];
                        const double cb = (k & 1) ? -1.0 : 1.0;
                        c0 += T2 * eb * cb;
                        c5 += T2 * ea;
                        ne = max(ne, tail_keep(k, T2, delta));
                    }
                }
            }
            if (has && wv == 0) {
                // w0 has one nonzero term (lane 0's): its butterfly would change no bit.  The
                // consts' second slot (c1, a sum of zeros) carries n_eff
                c0 = xor_sum(c0, 64);
                c5 = xor_sum(c5, 64);
                ne = xor_max_i(ne, 64);
                if (lane == 0) {
                    red[i][0] = c0;
                    red[i][1] = (double)ne;
                    red[i][2] = c5;
                    red[i][3] = w0;
                }
            }

            // ---- clamp-widened options of this table's group (double_heston.py:135-137) ----
            // 64 options per wave step: a ballot of the clamp test, then the wave prices each
            // clamped option on its own range [min(a, xK - 0.1), max(b, xK + 0.1)] (lanes over
            // k).  Mask words are written for every option, prices only for clamped ones; the
            // option kernel trusts these bits, so the two kernels never disagree on a decision.
            const int64_t slot0 = q * (int64_t)A.max_group;
            for (int base = wv * 64; base < gn; base += TPT) {
                const int o = base + lane;
                bool cl = false;
                double xK = 0.0, K = 0.0;
                if (o < gn) {
                    K = option_strike(A, g0 + o, S0);
                    const double rq = K / S0;
                    if (!(rq >= lo && rq <= hi)) {                   // near or past an edge
                        double ratio;
                        xK = option_logk(K, S0, ratio);
                        cl = xK - 0.1 < a || xK + 0.1 > b;
                    }
                }
                unsigned long long mask = __ballot(cl);
                if (lane == 0) A.cl_mask[q * cl_words(A) + base / 64] = mask;
                if (mask == 0) continue;
                const int64_t p = A.p0 + q / tpp;
                const Params P = dh::load_params(A.prm + p * DH_PARAM_STRIDE);
                const double disc = exp(-P.r * T);
                while (mask) {
                    const int l = __ffsll((long long)mask) - 1;
                    mask &= mask - 1;
                    const double x = __shfl(xK, l, 64);
                    const double Kl = __shfl(K, l, 64);
                    const int m = g0 + base + l;
                    const double ac = (x - 0.1 < a) ? x - 0.1 : a;      // Python min/max
                    const double bc = (x + 0.1 > b) ? x + 0.1 : b;
                    double v = clamped_term_sum(P, T, Kl, x, ac, bc, A.call[m] != 0, lane, 64, N,
                                                sct);
                    v = xor_sum(v, 64);
                    if (lane == 0) A.cl_price[slot0 + base + l] = disc * v;
                }
            }
            if (TPT > 64) __syncthreads();                     // t2s / w0s are reused
        }
        __syncthreads();
        if (b0 == q_begin) DH_STAMP(A, 6);
        // ---- fixed-order per-table sums of the batch ----
        if (threadIdx.x < nb) {
            const int i = threadIdx.x;
            double sm[4] = {0.0, 0.0, 0.0, 0.0};
            for (int j = 0; j < 4; ++j) sm[j] += red[i][j];
            const double* c = shc[i];
            double* cs = A.consts + (b0 + i) * kConsts;
            cs[0] = sm[0];
            cs[1] = sm[1];
            cs[2] = sm[2];
            cs[3] = sm[3];
            cs[4] = c[0];
            cs[5] = c[1];
            cs[6] = c[2];
            cs[7] = c[3];
        }
        __syncthreads();
    }
    DH_STAMP(A, 7);
}

// ----------------------------------------------------------------------------------------------
// option kernel helpers
// ----------------------------------------------------------------------------------------------
struct Consts {
    double c0, ne, c5, w0, a, b, eb, ea;   // ne: the table's n_eff (tail_keep), as a double
};


// sum' of one option from the table constants and its angle sum (k = 0 term:
// chi_0 = e^d - e^c, psi_0 = d - c, double_heston.py:142-143,154-155).
__device__ __forceinline__ double option_sum(const Consts& C, bool is_call, double S0, double K,
                                             double xK, double exK, double sum) {
    const double v0 = is_call ? (S0 * (C.eb - exK) - K * (C.b - xK))
                              : (K * (xK - C.a) - S0 * (exK - C.ea));
    const double cst = is_call ? C.c0 : C.c5;      // (the call's - K c1 term: c1 == 0 exactly)
    return cst + C.w0 * v0 - exK * sum;
}

// Angle sums of up to kR options on lanes k = k1, k1 + G, ...:
//   s_j = sum_k T2_k cos(k th_j) + T6_k sin(k th_j)
// cos/sin(k th_j) follow the Chebyshev recurrence x_{k+G} = 2 cos(G th_j) x_k - x_{k-G} (two FMAs
// per option-term; cg, sg = cos/sin(G th_j) staged once per option), re-anchored by an exact sincos
// every kAnchor steps: a rounding error introduced n steps before an anchor is amplified by at
// most n, so every cos/sin is within ~kAnchor^2 eps / 2 ~ 2e-13 of exact.  One (T2, T6)
// ds_read_b128 serves all kR options.
// Table reads run ahead of the arithmetic through a per-lane pointer and are not clamped to the
// table: an entry read past the end is never used, and an LDS read cannot fault (past the
// workgroup's allocation it returns 0), so each read is one ds_read_b128 at an immediate or
// uniform offset with no index arithmetic.
//
// One option per lane group (tile_r == 1): a lane's steps carry only this option's FMAs, so the
// cos and sin halves accumulate apart (two independent chains, summed at the end) and the table
// entries are read four steps ahead: each step's chain is one FMA deep and no LDS latency sits
// between steps.
__device__ __forceinline__ double angle_sum_1(int k1, int G, int N, double dx, double cg,
                                              double sg, double piba, const double2* t26,
                                              const double2* sct) {
    double sc = 0.0, ss = 0.0;
    const double c2 = 2.0 * cg;
    for (int k0 = k1; k0 < N; k0 += kAnchor * G) {
        double cx, sx;
        dh::dsincos_t(k0 * piba * dx, sct, &sx, &cx);          // u_k0 as the table's u
        double cp = cx * cg + sx * sg;                  // cos((k - G) th)
        double sp = sx * cg - cx * sg;                  // sin((k - G) th)
        const int kend = min(N, k0 + kAnchor * G);
        int k = k0;
        const double2* tq = t26 + k;
        double2 t0 = tq[0], t1 = tq[G], t2 = tq[2 * G], t3 = tq[3 * G];
        for (; k + 3 * G < kend; k += 4 * G) {
            tq += 4 * G;
            const double2 n0 = tq[0], n1 = tq[G], n2 = tq[2 * G], n3 = tq[3 * G];
            sc = fma(t0.x, cx, sc);                     // step k: x_{k+G} into (cp, sp)
            ss = fma(t0.y, sx, ss);
            cp = fma(c2, cx, -cp);
            sp = fma(c2, sx, -sp);
            sc = fma(t1.x, cp, sc);                     // step k + G: x_{k+2G} into (cx, sx)
            ss = fma(t1.y, sp, ss);
            cx = fma(c2, cp, -cx);
            sx = fma(c2, sp, -sx);
            sc = fma(t2.x, cx, sc);                     // step k + 2G
            ss = fma(t2.y, sx, ss);
            cp = fma(c2, cx, -cp);
            sp = fma(c2, sx, -sp);
            sc = fma(t3.x, cp, sc);                     // step k + 3G
            ss = fma(t3.y, sp, ss);
            cx = fma(c2, cp, -cx);
            sx = fma(c2, sp, -sx);
            t0 = n0;
            t1 = n1;
            t2 = n2;
            t3 = n3;
        }
        for (; k < kend; k += G) {                      // the last < 4 steps
            sc = fma(t0.x, cx, sc);
            ss = fma(t0.y, sx, ss);
            const double nc = fma(c2, cx, -cp), ns = fma(c2, sx, -sp);
            cp = cx;
            sp = sx;
            cx = nc;
            sx = ns;
            t0 = t1;
            t1 = t2;
            t2 = t3;
        }
    }
    return sc + ss;
}

template <int RR>
__device__ __forceinline__ void angle_sums_r(int k1, int G, int N, const double (&dx)[RR],
                                             const double (&cg)[RR], const double (&sg)[RR],
                                             double piba, const double2* t26,
                                             const double2* sct, double (&sum)[RR]) {
    if constexpr (RR == 1) {
        sum[0] = angle_sum_1(k1, G, N, dx[0], cg[0], sg[0], piba, t26, sct);
        return;
    }
#pragma unroll
    for (int j = 0; j < RR; ++j) sum[j] = 0.0;
    double c2[RR];
#pragma unroll
    for (int j = 0; j < RR; ++j) c2[j] = 2.0 * cg[j];
    // segments of kAnchor steps, each opened by an exact (k, k - G) pair; inside a segment four
    // steps per iteration (then at most one pair and one single step), so x_k and x_{k-G} swap
    // registers instead of being copied, with the table entries read ahead of the arithmetic
    for (int k0 = k1; k0 < N; k0 += kAnchor * G) {
        double cx[RR], sx[RR], cp[RR], sp[RR];
        const double uk = k0 * piba;                 // u_k0, the table's expression
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            dh::dsincos_t(uk * dx[j], sct, &sx[j], &cx[j]);
            cp[j] = cx[j] * cg[j] + sx[j] * sg[j];              // cos((k - G) th)
            sp[j] = sx[j] * cg[j] - cx[j] * sg[j];              // sin((k - G) th)
        }
        const int kend = min(N, k0 + kAnchor * G);
        int k = k0;
        const double2* tq = t26 + k;
        double2 ta = tq[0], tb = tq[G];
        auto step = [&](const double2& t, double (&x)[RR], double (&y)[RR], double (&xp)[RR],
                        double (&yp)[RR]) {         // x_{k+G} into (xp, yp)
#pragma unroll
            for (int j = 0; j < RR; ++j) {
                sum[j] = fma(t.x, x[j], sum[j]);
                sum[j] = fma(t.y, y[j], sum[j]);
                xp[j] = fma(c2[j], x[j], -xp[j]);
                yp[j] = fma(c2[j], y[j], -yp[j]);
            }
        };
        for (; k + 3 * G < kend; k += 4 * G) {
            const double2 tc = tq[2 * G], td = tq[3 * G];
            tq += 4 * G;
            step(ta, cx, sx, cp, sp);
            step(tb, cp, sp, cx, sx);
            ta = tq[0];
            tb = tq[G];
            step(tc, cx, sx, cp, sp);
            step(td, cp, sp, cx, sx);
        }
        if (k + G < kend) {
            step(ta, cx, sx, cp, sp);
            step(tb, cp, sp, cx, sx);
            k += 2 * G;
            ta = tq[2 * G];
        }
        if (k < kend) {
#pragma unroll
            for (int j = 0; j < RR; ++j) {
                sum[j] = fma(ta.x, cx[j], sum[j]);
                sum[j] = fma(ta.y, sx[j], sum[j]);
            }
        }
    }
}

__device__ __forceinline__ void record_price(const PriceArgs& A, int64_t p, int col, double mk,
                                             int oi, double price, double* lsse, double* lbad) {
    if (A.out) A.out[p * A.out_stride + col] = price;
    if (A.part_sse) {
        const double rel = (price - mk) / mk;
        lsse[oi] = rel * rel;
        // lbfgs_calibrator.py:152: NaN, inf or <= 0 is invalid
        lbad[oi] = (isnan(price) || isinf(price) || price <= 0.0) ? 1.0 : 0.0;
    }
}

// Loss pairs handed over inside a fused launch (partials_only == 3): the guide's data-tagged
// granule form (cdna_hip_programming.md, Guideline 16 R2; MI355X_MICROARCH.md "valid forms"):
// every byte of a granule goes out in one aligned write-through (sc1) store that carries the
// launch's epoch, and every read of it is an sc1 load, re-read until the tag matches -- no flag,
// no fence, no drain.  Granule 0 of a task: epoch << 32 | low word of the
// partial; granule 1: (epoch << 9 | invalid count) << 32 | high word.  The epoch is never 0 and
// the buffer is zeroed when allocated, so a granule from another launch never matches.
constexpr int kGranCountBits = 9;           // invalid count of a tile: <= kTileMax = 256
__device__ __forceinline__ unsigned long long gran_load(const unsigned long long* g) {
    return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A task's two granules in ONE 16-byte write-through store (buffer_store_dwordx4 with sc1: aux 16,
// cdna_hip_programming.md Guideline 16 R1's store form), one fabric write instead of two; each
// 8-byte half still carries its own tag, so a torn pair is seen as not yet written.  g: uniform.
typedef unsigned int dh_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void gran_store2(unsigned long long* g, unsigned long long v0,
                                            unsigned long long v1) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(g, 0, 16, 0x00020000);
    const dh_u32x4 d = {(unsigned)v0, (unsigned)(v0 >> 32), (unsigned)v1, (unsigned)(v1 >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(d, rsrc, 0, 0, 16);
}

// The final sse / n_bad of param set p (lane 0 of the summing wave).  Into mapped host memory
// (host_out) they go as system-scope stores and the wave waits for their acknowledgement before it
// ends, so they are complete before the kernel's end-of-dispatch signal, whichever release scope
// the runtime gives that signal (the slot's event may be the launch's own stop event,
// hipExtLaunchKernel, whose release scope HIP does not document).
#ifndef DH_HOST_OUT_DRAIN
#define DH_HOST_OUT_DRAIN 1
#endif
__device__ __forceinline__ void loss_out(const PriceArgs& A, int64_t p, double sse, int nb) {
    if (DH_HOST_OUT_DRAIN && A.host_out) {
        __hip_atomic_store(&A.sse[p], sse, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&A.n_bad[p], nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        A.sse[p] = sse;
        A.n_bad[p] = nb;
    }
}

// The loss sums of param set pc by one wave of one of the grid's last P blocks (dispatch order),
// after its own task's granules went out: every lane sweeps its tiles' granules until all carry
// this launch's epoch (the producers are earlier-dispatched blocks, or blocks of the last round
// running beside it; at most P waiting blocks of a grid larger than one round of resident ones,
// so every producer still gets a slot), then the partials are summed in loss_partials_kernel's
// order and butterfly (same bits as the hand-off's last task).  The sweep is bounded: a timeout
// (never seen; some 10^8 cycles) leaves n_bad[pc] = -1.
__device__ __forceinline__ void tail_sums(const PriceArgs& A, int64_t pc, int t) {
    const int64_t base = pc * A.n_tiles;
    const unsigned ep = A.ahead_epoch;
    const unsigned ep_hi = ep << kGranCountBits;
    const unsigned cmask = (1u << kGranCountBits) - 1u;
    double acc = 0.0, bad = 0.0;
    bool timed_out = false;
    for (int j0 = 0; j0 < A.n_tiles; j0 += 64) {
        const int j = j0 + t;
        unsigned long long g0 = 0, g1 = 0;
        bool ok = j >= A.n_tiles;
        for (unsigned spins = 0;; ++spins) {
            if (!ok) {
                g0 = gran_load(A.gran + 2 * (base + j));
                g1 = gran_load(A.gran + 2 * (base + j) + 1);
                ok = (unsigned)(g0 >> 32) == ep && ((unsigned)(g1 >> 32) & ~cmask) == (ep_hi & ~cmask);
            }
            if (__all(ok)) break;
            if (spins > (1u << 20)) {
                timed_out = true;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (j < A.n_tiles) {
            acc += __longlong_as_double((long long)((g1 << 32) | (g0 & 0xffffffffull)));
            bad += (double)((unsigned)(g1 >> 32) & cmask);
        }
    }
    acc = xor_sum(acc, 64);
    bad = xor_sum(bad, 64);
    if (t == 0) loss_out(A, pc, acc, timed_out ? -1 : (int)bad);
}

// Fixed-order loss partial of one task (wave 0 of the task).  Hand-off to the last task of param
// set p without fences (MI355X_MICROARCH.md, "Valid forms", first table row): one lane writes
// the partial with agent-scope (sc1, write-through) stores, drains them with s_waitcnt vmcnt(0),
// then adds to p's counter; in the wave whose add returns n_tiles - 1 every lane reads partials
// of p with sc1 loads, the wave sums them in a fixed order and resets the counter.
__device__ __forceinline__ void task_loss(const PriceArgs& A, int64_t p, int64_t task, int nopt,
                                          int t, const double* lsse, const double* lbad) {
    DH_STAMP(A, 13);
    double s = 0.0;
    int nb = 0;                     // invalid prices: a count (0/1 flags), so a ballot suffices
    for (int i0 = 0; i0 < nopt; i0 += 64) {
        const int i = i0 + t;
        if (i < nopt) s += lsse[i];
        nb += __popcll(__ballot(i < nopt && lbad[i] != 0.0));
    }
    // lanes >= nopt hold +0.0 and only lane 0's sum is used, so levels with off >= nopt would add
    // +0.0 to it (an exact no-op on a sum of squares): skip them (C2's 32 options: 5 levels)
    const int lvl = nopt < 64 ? nopt : 64;
    int width = 1;
    while (width < lvl) width <<= 1;
    s = xor_sum(s, width);
    const double f = nb;
    DH_STAMP(A, 14);
    const int64_t base_i = p * A.n_tiles;
    if (A.partials_only == 3) {     // the pair as two epoch-tagged 8-byte granules, write-through
        // (agent-scope) stores with no drain: each granule is its own flag (tail_sums)
        if (t == 0) {
            const unsigned long long sb = (unsigned long long)__double_as_longlong(s);
            const unsigned ep = A.ahead_epoch;
            const unsigned long long g0 = ((unsigned long long)ep << 32) | (unsigned)sb;
            const unsigned long long g1 =
                ((unsigned long long)((ep << kGranCountBits) | (unsigned)nb) << 32) | (unsigned)(sb >> 32);
            gran_store2(A.gran + 2 * task, g0, g1);
        }
        return;
    }
    if (A.partials_only == 2) {     // one plain 16-byte store (one line write per block):
        // loss_partials_kernel reads the (partial, invalid count) pairs next
        if (t == 0) reinterpret_cast<double2*>(A.part_sse)[task] = make_double2(s, f);
        return;
    }
    if (A.partials_only) {          // plain stores: the next launch (the step kernel) reads them;
        // the tile's invalid flag rides in the sign bit (a valid partial is a sum of squares: +0,
        // positive, +inf or NaN, canonicalised to + here), so the step kernel reads one array
        if (t == 0) A.part_sse[task] = f > 0.0 ? -fabs(s) : fabs(s);
        return;
    }
    unsigned old = 0;
    if (t == 0) {
        __hip_atomic_store(&A.part_sse[task], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&A.part_bad[task], (int)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        DH_STAMP(A, 15);
        old = __hip_atomic_fetch_add(&A.counter[p * kCounterStride], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    old = __builtin_amdgcn_readlane(old, 0);       // lane 0's ticket (no LDS round trip)
    DH_STAMP(A, 12);
    if (old != (unsigned)A.n_tiles - 1u) return;
    double acc = 0.0, bad = 0.0;
    for (int j = t; j < A.n_tiles; j += 64) {
        acc += __hip_atomic_load(&A.part_sse[base_i + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad += __hip_atomic_load(&A.part_bad[base_i + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    acc = xor_sum(acc, 64);
    bad = xor_sum(bad, 64);
    if (t == 0) {
        loss_out(A, p, acc, (int)bad);
        __hip_atomic_store(&A.counter[p * kCounterStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The hand-off's last task, as its own launch after a partials_only == 2 request (one 64-lane
// block per param set): the same reads in the same order and the same butterfly, so the same bits
// as task_loss.  A multi-round fused grid's blocks then end with plain stores instead of the
// agent-scope store drain and the ticket atomic (~1.8k cycles of every block's chain).
__global__ __launch_bounds__(64) void loss_partials_kernel(const double2* __restrict__ part,
                                                           int n_tiles, double* sse, int* n_bad) {
    const int64_t p = blockIdx.x;
    const int t = threadIdx.x;
    const int64_t base_i = p * n_tiles;
    double acc = 0.0, bad = 0.0;
    for (int j = t; j < n_tiles; j += 64) {
        const double2 v = part[base_i + j];
        acc += v.x;
        bad += v.y;
    }
    acc = xor_sum(acc, 64);
    bad = xor_sum(bad, 64);
    if (t == 0) {
        sse[p] = acc;
        n_bad[p] = (int)bad;
    }
}

__host__ __device__ constexpr int option_lds_doubles(int N, int opt_cap) {
    // (T2,T6)[N] | K, mkt, sse, bad, xK, e^xK, cos/sin step [opt_cap] | call, perm [opt_cap]
    // ints, rounded to whole 16-byte pairs (u_k = k pi/(b - a) is re-formed where needed)
    return 2 * N + 8 * opt_cap + ((2 * opt_cap + 3) / 4) * 2;
}

// LDS view of one staged tile: the expanded (p, g) table and the per-option arrays
struct TileLds {
    double2* t26;     // (T2_k, T6_k)
    double* K;
    double* mkt;
    double* sse;
    double* bad;
    double* xK;       // log(K / S0)
    double* exK;      // e^{log(K / S0)}
    double* cs;       // cos / sin of the G-step rotation (sin = NaN marks a clamped option)
    double* ss;
    int* call;
    int* perm;
};

__device__ __forceinline__ TileLds tile_lds(double* base, int N, int cap) {
    TileLds L;
    L.t26 = (double2*)base;
    L.K = base + 2 * N;
    L.mkt = L.K + cap;
    L.sse = L.mkt + cap;
    L.bad = L.sse + cap;
    L.xK = L.bad + cap;
    L.exK = L.xK + cap;
    L.cs = L.exK + cap;
    L.ss = L.cs + cap;
    L.call = (int*)(L.ss + cap);
    L.perm = L.call + cap;
    return L;
}

// Options per lane group of a launch whose largest tile has max_nopt options priced by tpt
// threads: kR (one table read serves kR options) unless that tile leaves >= 8 lanes per option,
// where one option per group gives each lane one anchor sincos instead of kR and a butterfly over
// one sum instead of kR (the latency path of small calibration tiles: C2's 32-option tiles, C1's
// 5).  A property of the surface and N, never of the batch: every path and batch composition
// prices a tile with the same lanes.  The request kernels are instantiated per value.
inline int tile_r(int max_nopt, int tpt) { return tpt >= 8 * std::max(max_nopt, 1) ? 1 : kR; }

// lanes per group of RT options for a tile of nopt options priced by tpt threads
// A block-wide tile (tpt == kBlock) with kR options per group takes any G (its partials are
// reduced through LDS, e.g. G = 10 for 100-option tiles: 250 of 256 lanes busy instead of 200 with
// G = 8); other tiles keep a power of two <= 64 for the in-wave butterfly.
template <int RT>
__device__ __forceinline__ int group_lanes(int nopt, int N, int tpt) {
    const int R = min(RT, max(nopt, 1));
    const int ngroups = (nopt + R - 1) / R;
#ifndef DH_GMAX
#define DH_GMAX 1024
#endif
    if (tpt == kBlock && RT == kR) return max(1, min(min(tpt / ngroups, DH_GMAX), N - 1));
    int G = 1;
    while (G * 2 <= tpt / max(ngroups, 1) && G < 64) G *= 2;
    while (G > 1 && G / 2 >= N - 1) G /= 2;                 // no more lanes than terms k >= 1
    return G;
}

// Angle sums, finalisation and price / loss-term recording of one staged tile (thread t of the
// tile's tpt).  Shared by cos_option_kernel and cos_fused_kernel, so both give the same bits.
// A block-wide tile (tpt == kBlock; every thread of the block must call this) whose G is not a
// power of two <= 64 reduces each group's G lane partials through LDS (red: kR x kBlock doubles)
// in lane order; otherwise xor butterflies inside the wave.
template <int RT>
__device__ __forceinline__ void tile_sums_r(const PriceArgs& A, int64_t p, const Consts& C,
                                            double S0, double disc, int nopt, int G, int tpt,
                                            int t, bool active, const TileLds& L, double* red,
                                            const double2* sct) {
    const int Ne = (int)C.ne;                     // the table's kept terms: k < n_eff
    const int R = min(RT, max(nopt, 1));
    const int ngroups = (nopt + R - 1) / R;
    const int groups_per_pass = max(1, tpt / G);
    const bool lds_red = tpt == kBlock && (G > 64 || (G & (G - 1)) != 0);   // else butterflies
    for (int pass = 0; pass < ngroups; pass += groups_per_pass) {
        const int gi = pass + t / G;
        const int gl = t % G;
        const bool gvalid = active && t < groups_per_pass * G && gi < ngroups;
        double dx[RT], cs[RT], ss[RT];
        bool use[RT];
#pragma unroll
        for (int j = 0; j < RT; ++j) {
            const int oi = gi * R + j;
            const bool in = gvalid && j < R && oi < nopt;
            const double sj = in ? L.ss[oi] : 0.0;
            use[j] = in && !isnan(sj);                               // clamped: recorded
            dx[j] = use[j] ? L.xK[oi] - C.a : 0.0;
            cs[j] = use[j] ? L.cs[oi] : 1.0;
            ss[j] = use[j] ? sj : 0.0;
        }
        double sm[RT];
        if (pass == 0) DH_STAMP(A, 9);
        angle_sums_r<RT>(1 + gl, G, Ne, dx, cs, ss, dh::kPi / (C.b - C.a), L.t26, sct, sm);
        if (pass == 0) DH_STAMP(A, 10);
        if (lds_red) {
            if (gvalid) {
                // the slot address formed here, not kept across the angle loop (held there, it was
                // the C3 build's one hot-path register spill: a scratch store and a reload per
                // thread, ~1.3 MB of scratch written back per request)
                int tr = t;
                asm volatile("" : "+v"(tr));
#pragma unroll
                for (int j = 0; j < RT; ++j) red[j * kBlock + tr] = sm[j];
            }
            __syncthreads();
            if (pass == 0) DH_STAMP(A, 11);
            // thread t finalises option pass R + t of the pass (one option per thread: the
            // pass's options on its first lanes, not on lanes gl < R of every group, so fewer
            // waves issue the finalisation): its group's G lane partials in lane order
            const int o_end = min(nopt, min(pass + groups_per_pass, ngroups) * R);
            for (int oi = pass * R + t; active && oi < o_end; oi += tpt) {
                if (!isnan(L.ss[oi])) {
                    const int j = oi % R;
                    const double* rj = red + j * kBlock + (oi / R - pass) * G;
                    double sum = 0.0;
                    for (int l = 0; l < G; ++l) sum += rj[l];
                    const double v = option_sum(C, L.call[oi] != 0, S0, L.K[oi], L.xK[oi],
                                                L.exK[oi], sum);
                    record_price(A, p, L.perm[oi], L.mkt[oi], oi, disc * v, L.sse, L.bad);
                }
            }
            __syncthreads();
            continue;
        }
#pragma unroll
        for (int j = 0; j < RT; ++j) sm[j] = xor_sum(sm[j], G);
        if (pass == 0) DH_STAMP(A, 11);
        // every lane of the group holds the (bitwise identical) sums: lane j finalises option j
        if (G >= R) {
            double m = sm[0];
            bool mu = use[0];
#pragma unroll
            for (int j = 1; j < RT; ++j) {
                m = gl == j ? sm[j] : m;
                mu = gl == j ? use[j] : mu;
            }
            if (gl < R && mu) {
                const int oi = gi * R + gl;
                const double sum = option_sum(C, L.call[oi] != 0, S0, L.K[oi], L.xK[oi],
                                              L.exK[oi], m);
                record_price(A, p, L.perm[oi], L.mkt[oi], oi, disc * sum, L.sse, L.bad);
            }
        } else if (gl == 0) {
#pragma unroll
            for (int j = 0; j < RT; ++j) {
                if (!use[j]) continue;
                const int oi = gi * R + j;
                const double sum = option_sum(C, L.call[oi] != 0, S0, L.K[oi], L.xK[oi],
                                              L.exK[oi], sm[j]);
                record_price(A, p, L.perm[oi], L.mkt[oi], oi, disc * sum, L.sse, L.bad);
            }
        }
    }
}

// LDS doubles of the lane partials of a block-wide tile (tile_sums' red)
constexpr int kRedDoubles = kR * kBlock;

// ----------------------------------------------------------------------------------------------
// option kernel
// ----------------------------------------------------------------------------------------------
template <int TPT, int RT>
__global__ __launch_bounds__(kBlock, DH_OPTION_WAVES) void cos_option_kernel(PriceArgs A_) {
    const PriceArgs& A = karg_ref<PriceArgs, 0>();   // read in place (karg_ref)
    if (halted(A)) return;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int kTasks = kBlock / TPT;
    const int slot = threadIdx.x / TPT;
    const int t = threadIdx.x % TPT;
    const int N = A.N;
    const int64_t n_tasks = A.paired ? A.np : A.np * (int64_t)A.n_tiles;
    // the task index is wave-uniform: make that visible so per-task values live in SGPRs
    const int64_t task_l = (int64_t)blockIdx.x * kTasks + __builtin_amdgcn_readfirstlane(slot);
    const bool active = task_l < n_tasks;
    const int64_t p = A.p0 + (active ? (A.paired ? task_l : task_l / A.n_tiles) : 0);
    const int tile = (active && !A.paired) ? (int)(task_l % A.n_tiles) : 0;
    const int64_t task = A.paired ? p : p * A.n_tiles + tile;       // global task id
    DH_STAMP(A, 0);

    const int cap = A.opt_cap;
    const TileLds L = tile_lds(smem + (size_t)slot * option_lds_doubles(N, cap), N, cap);
    double* red = smem + (size_t)kTasks * option_lds_doubles(N, cap);   // TPT == kBlock only
    __shared__ double2 sct[dh::kMathTab];
    dh::load_sincos_table(sct);                                // synchronised by the staging barrier
    double2* t26 = L.t26;
    double* lK = L.K;
    double* lmkt = L.mkt;
    double* lsse = L.sse;
    double* lbad = L.bad;
    double* lxK = L.xK;
    double* lexK = L.exK;
    double* lcs = L.cs;
    double* lss = L.ss;
    int* lcall = L.call;
    int* lperm = L.perm;

    int opt0 = 0, nopt = 0, g = 0;
    if (active) {
        if (A.paired) {
            opt0 = (int)p;
            nopt = 1;
        } else {
            const int2 tl = A.tiles[tile];
            opt0 = tl.x;
            nopt = tl.y;
            g = A.tile_group[tile];
        }
    }
    // lanes: groups of kR options on G lanes each
    const int G = group_lanes<RT>(nopt, N, TPT);

    const int64_t q = (p - A.p0) * tabs_per_p(A) + g;
    const Params P = dh::load_params(A.prm + p * DH_PARAM_STRIDE);
    Consts C{0.0, 0.0, 0.0, 0.0, 0.0, 1.0, 1.0, 1.0};
    if (active) {
        const double* cs = A.consts + q * kConsts;
        C = Consts{cs[0], cs[1], cs[2], cs[3], cs[4], cs[5], cs[6], cs[7]};
    }
    const double ba = C.b - C.a;
    const double T = active ? A.T[opt0] : 1.0;
    const double disc = exp(-P.r * T);
    // stage the (p, g) table, expanded to u, (T2, T6) (same expressions as the table
    // kernel's k-sums), and per-option data: log(K/S0), e^{xK} and the G-step rotation of each
    // option; clamp-widened options (bit set by the table kernel) are recorded right here
    if (active) {
        const double* tw = A.table + q * (int64_t)N;     // row-major (never tiled here)
        const double piba = dh::kPi / ba;
        const int ne = (int)C.ne;                        // terms past n_eff are never read
        for (int k = t; k < ne; k += TPT) {
            const double w = tw[k];
            const double u = k * piba;
            const double T2 = k == 0 ? 0.0 : w * P.S0 * dh::drcp(1.0 + u * u);
            t26[k] = make_double2(T2, k == 0 ? 0.0 : -(T2 * dh::drcp(u)));
        }
        const double ustep = G * dh::kPi / ba;
        const int g0 = A.paired ? (int)p : A.groups[g].x;
        const unsigned long long* msk = A.cl_mask + q * cl_words(A);
        const double* clp = A.cl_price + q * (int64_t)A.max_group;
        for (int i = t; i < nopt; i += TPT) {
            const double K = option_strike(A, opt0 + i, P.S0);
            double ratio;
            const double xK = option_logk(K, P.S0, ratio);
            lK[i] = K;
            lmkt[i] = A.mkt ? A.mkt[opt0 + i] : 0.0;
            lcall[i] = A.call[opt0 + i];
            lperm[i] = A.perm[opt0 + i];
            lxK[i] = xK;
            lexK[i] = ratio;                                         // e^{xK} to an ulp
            const int gpos = opt0 + i - g0;
            const bool cl = (msk[gpos >> 6] >> (gpos & 63)) & 1ull;
            double ss, cs;
            dh::dsincos(ustep * (cl ? 0.0 : xK - C.a), &ss, &cs);
            lcs[i] = cs;
            // NaN marks clamped; a NaN sine of an unclamped option (NaN params, strike or
            // range) is stored as 0: its NaN cosine and offset still make the price NaN
            lss[i] = cl ? NAN : (ss == ss ? ss : 0.0);
            if (cl) record_price(A, p, lperm[i], lmkt[i], i, clp[gpos], lsse, lbad);
        }
    }
    __syncthreads();
    DH_STAMP(A, 1);

    tile_sums_r<RT>(A, p, C, P.S0, disc, nopt, G, TPT, t, active, L, red, sct);
    DH_STAMP(A, 2);

    // ---- loss: fixed-order per-task partial, last arriver finalises the param set ----
    if (A.part_sse) {
        __syncthreads();
        if (active && t < 64) task_loss(A, p, task, nopt, t, lsse, lbad);
    }
    DH_STAMP(A, 3);
}

// ----------------------------------------------------------------------------------------------
// option kernel, small tiles (<= kSmallTile options per tile): one lane carries RS options of a
// tile through every term k = 1 .. N-1.  Its step rotation e^{i th} is also its start angle, the
// 8-byte table w_k is read straight from L2/MALL and expanded to (T2, T6) on the fly
// (amortised over RS options), and a task's partial is reduced over its L lanes (L = lanes per
// task, a power of two <= 4) before the same fence-free hand-off.  Per lane this is ~9 VALU
// instructions per option-term with no LDS, no per-lane anchors and no butterflies -- the
// large-tile kernel's fixed costs dominate when a tile has 5-16 options (generator grids).
// ----------------------------------------------------------------------------------------------
constexpr int kSmallTile = 16;
// options per lane: 4, or 8 for tiles of more than 4 options (C5's 8-option tiles: one lane per
// tile, so the per-term expansion of w_k is not repeated on a second lane: -24% VALU per tile-term)
constexpr int small_rs(int max_nopt) { return max_nopt > 4 ? 8 : 4; }
// ...and only when a call has enough tasks to fill the chip with one lane group per task
// (below this the large-tile kernel's many lanes per option win on latency).  Calibration
// launches (14 x starts param sets) stay far below it, so lockstep == sequential bit for bit.
constexpr int64_t kSmallMinTasks = 65536;

template <int RS>
__global__ __launch_bounds__(kBlock) void cos_option_small_kernel(PriceArgs A_, int L) {
    const PriceArgs& A = karg_ref<PriceArgs, 0>();   // read in place (karg_ref)
    if (halted(A)) return;
    const int64_t gid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t n_tasks = A.paired ? A.np : A.np * (int64_t)A.n_tiles;
    const int64_t task_l = gid / L;
    const int sub = (int)(gid % L);
    const bool active = task_l < n_tasks;
    const int64_t p = A.p0 + (active ? (A.paired ? task_l : task_l / A.n_tiles) : 0);
    const int tile = (active && !A.paired) ? (int)(task_l % A.n_tiles) : 0;
    const int64_t task = A.paired ? p : p * A.n_tiles + tile;
    int opt0 = 0, nopt = 0, g = 0;
    if (active) {
        if (A.paired) {
            opt0 = (int)p;
            nopt = 1;
        } else {
            const int2 tl = A.tiles[tile];
            opt0 = tl.x;
            nopt = tl.y;
            g = A.tile_group[tile];
        }
    }
    const int64_t q = (p - A.p0) * tabs_per_p(A) + g;
    const double* prm = A.prm + p * DH_PARAM_STRIDE;
    const double S0 = prm[13], r = prm[14];
    Consts C{0.0, 0.0, 0.0, 0.0, 0.0, 1.0, 1.0, 1.0};
    if (active) {
        const double* cs = A.consts + q * kConsts;
        C = Consts{cs[0], cs[1], cs[2], cs[3], cs[4], cs[5], cs[6], cs[7]};
    }
    const double ba = C.b - C.a;
    const double piba = dh::kPi / ba;
    const double T = active ? A.T[opt0] : 1.0;
    const double disc = exp(-r * T);
    const int g0 = A.paired ? (int)p : (active ? A.groups[g].x : 0);
    const unsigned long long* msk = A.cl_mask + q * cl_words(A);
    const double* clp = A.cl_price + q * (int64_t)A.max_group;

    // per option: log-strike, clamp bit; cos/sin(k th) by the Chebyshev recurrence from
    // (k = 0, k = 1) = (1 + 0i, e^{i th})
    double dx[RS], c[RS], sn[RS], cp[RS], sp[RS], cs[RS], ss[RS], sm[RS];
    bool use[RS];
    double lsum = 0.0, lbad = 0.0;
#pragma unroll
    for (int j = 0; j < RS; ++j) {
        const int oi = sub * RS + j;
        const bool in = active && oi < nopt;
        bool cl = false;
        double xK = 0.0;
        if (in) {
            const int m = opt0 + oi;
            const double K = option_strike(A, m, S0);
            double ratio;
            xK = option_logk(K, S0, ratio);
            const int gpos = m - g0;
            cl = (msk[gpos >> 6] >> (gpos & 63)) & 1ull;
            if (cl) {                      // priced by the table kernel
                const double price = clp[gpos];
                if (A.out) A.out[p * A.out_stride + A.perm[m]] = price;
                if (A.part_sse) {
                    const double mk = A.mkt[m];
                    const double rel = (price - mk) / mk;
                    lsum += rel * rel;
                    lbad += (isnan(price) || isinf(price) || price <= 0.0) ? 1.0 : 0.0;
                }
            }
        }
        use[j] = in && !cl;
        dx[j] = use[j] ? xK - C.a : 0.0;
        double s1, c1;
        dh::dsincos(piba * dx[j], &s1, &c1);
        cs[j] = c1;
        ss[j] = s1;
        c[j] = c1;
        sn[j] = s1;
        cp[j] = 1.0;
        sp[j] = 0.0;
        sm[j] = 0.0;
    }
    // the host always tiles the tables this kernel reads: entry k at tw[k * kTabTile]
    const double* tw = A.table + (q / kTabTile) * kTabTile * (int64_t)A.N + (q % kTabTile);
    double c2[RS];
#pragma unroll
    for (int j = 0; j < RS; ++j) c2[j] = 2.0 * cs[j];
    // segments of kAnchor terms (the first starts exact at k = 1; later ones re-anchor on an
    // exact (k, k - 1) pair), two terms per iteration with x_k / x_{k-1} swapping registers
    const int N = A.N;
    const int ne = (int)C.ne;                        // the table's kept terms: k < n_eff
    for (int k0 = 1; k0 < ne; k0 += kAnchor) {
        if (k0 > 1) {
            const double uk = k0 * piba;
#pragma unroll
            for (int j = 0; j < RS; ++j) {
                dh::dsincos(uk * dx[j], &sn[j], &c[j]);
                cp[j] = c[j] * cs[j] + sn[j] * ss[j];
                sp[j] = sn[j] * cs[j] - c[j] * ss[j];
            }
        }
        const int kend = min(ne, k0 + kAnchor);
        int k = k0;
        double wa = active ? tw[k * kTabTile] : 0.0;
        for (; k + 1 < kend; k += 2) {
            const double wb = active ? tw[(k + 1) * kTabTile] : 0.0;
            const double ua = k * piba, ub = (k + 1) * piba;
            const double T2a = wa * S0 * dh::drcp(1.0 + ua * ua);
            const double T6a = -(T2a * dh::drcp(ua));
            const double T2b = wb * S0 * dh::drcp(1.0 + ub * ub);
            const double T6b = -(T2b * dh::drcp(ub));
            wa = active ? tw[min(k + 2, N - 1) * kTabTile] : 0.0;
#pragma unroll
            for (int j = 0; j < RS; ++j) {
                sm[j] = fma(T2a, c[j], sm[j]);
                sm[j] = fma(T6a, sn[j], sm[j]);
                cp[j] = fma(c2[j], c[j], -cp[j]);               // x_{k+1}
                sp[j] = fma(c2[j], sn[j], -sp[j]);
                sm[j] = fma(T2b, cp[j], sm[j]);
                sm[j] = fma(T6b, sp[j], sm[j]);
                c[j] = fma(c2[j], cp[j], -c[j]);                // x_{k+2}
                sn[j] = fma(c2[j], sp[j], -sn[j]);
            }
        }
        if (k < kend) {
            const double u = k * piba;
            const double T2 = wa * S0 * dh::drcp(1.0 + u * u);
            const double T6 = -(T2 * dh::drcp(u));
#pragma unroll
            for (int j = 0; j < RS; ++j) {
                sm[j] = fma(T2, c[j], sm[j]);
                sm[j] = fma(T6, sn[j], sm[j]);
            }
        }
    }
    // finalise this lane's options, then the task partial over its L lanes (fixed tree)
#pragma unroll
    for (int j = 0; j < RS; ++j) {
        if (!use[j]) continue;
        const int m = opt0 + sub * RS + j;
        const double K = option_strike(A, m, S0);
        double ratio;
        const double xK = option_logk(K, S0, ratio);
        const double sum = option_sum(C, A.call[m] != 0, S0, K, xK, ratio, sm[j]);
        const double price = disc * sum;
        if (A.out) A.out[p * A.out_stride + A.perm[m]] = price;
        if (A.part_sse) {
            const double mk = A.mkt[m];
            const double rel = (price - mk) / mk;
            lsum += rel * rel;
            lbad += (isnan(price) || isinf(price) || price <= 0.0) ? 1.0 : 0.0;
        }
    }
    if (!A.part_sse) return;
    lsum = xor_sum(lsum, L);
    lbad = xor_sum(lbad, L);
    if (!active || sub != 0) return;
    // fence-free hand-off (as task_loss): sc1 stores, drain, agent-scope ticket
    __hip_atomic_store(&A.part_sse[task], lsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&A.part_bad[task], (int)lbad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old =
        __hip_atomic_fetch_add(&A.counter[p * kCounterStride], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old != (unsigned)A.n_tiles - 1u) return;
    const int64_t base_i = p * A.n_tiles;
    double acc = 0.0;
    int bad = 0;
    for (int j = 0; j < A.n_tiles; ++j) {           // tile order
        acc += __hip_atomic_load(&A.part_sse[base_i + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad += __hip_atomic_load(&A.part_bad[base_i + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    loss_out(A, p, acc, bad);
    __hip_atomic_store(&A.counter[p * kCounterStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ----------------------------------------------------------------------------------------------
// fused small-tile kernel (generator grids: every maturity group one tile of <= kSmallTile
// options, >= kSmallMinTasks tasks): a persistent block takes TB tables at a time, forms their
// expanded tables (T2_k, T6_k) in LDS -- no table round trip through L2/MALL and no second
// launch -- then prices their options on lanes (table, option, k-block):
//   * prologue: one lane per table (table_prologue, the split path's constants);
//   * CF: TPT = 256 / TB threads per table, entries k = t, t + TPT, ... (cf_phase_re), each
//     stored as (T2, T6) with the table kernel's expressions; c0 / c5 / w0 summed per thread in
//     increasing k, then a TPT-lane butterfly;
//   * options: OP (a power of two >= the largest tile) option slots per table x S = TPT / OP
//     k-blocks per option: lane j of an option sums k in [1 + j L, 1 + (j + 1) L), L = ceil((N - 1)
//     / S), cos/sin(k th) by the step-th Chebyshev recurrence re-anchored by an exact sincos every
//     kAnchor terms, then an S-lane butterfly; clamp-widened options (double_heston.py:135-137)
//     are priced afterwards by the whole wave (clamped_term_sum, lanes over k);
//   * loss: per table the options' rel^2 / invalid flags summed in option order, then the
//     fence-free hand-off of the other request kernels (one task = one (p, tile)).
// Prices agree with the split / fused paths to ~1e-15 relative (another summation order), as the
// lane-per-option-group small-tile kernel's did.
// ----------------------------------------------------------------------------------------------
template <int TB>
__global__ __launch_bounds__(kBlock, 3) void cos_gen_kernel(PriceArgs A_, int OP) {
    const PriceArgs& A = karg_ref<PriceArgs, 0>();   // read in place (karg_ref)
    if (halted(A)) return;
    constexpr int TPT = kBlock / TB;                 // threads per table (CF), <= 64
    static_assert(TPT <= 64 && TPT >= kSmallTile, "one table's lanes inside one wave");
    extern __shared__ __attribute__((aligned(16))) double2 gtab[];   // [TB][N] (T2, T6)
    __shared__ double shc[TB][kTabC];
    __shared__ double ks[TB][3];                     // c0, c5, w0
    __shared__ int kne[TB];                          // n_eff (tail_keep)
    __shared__ double osse[TB][kSmallTile], obad[TB][kSmallTile];
    __shared__ double2 sct[dh::kMathTab];
    dh::load_math_tables(sct, 0);                    // synchronised by the first barrier
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int N = A.N;
    const int tpp = tabs_per_p(A);
    const int64_t n_q = A.np * tpp;
    const int S = TPT / OP;                          // k-blocks per option
    const int it = t / TPT, sub = t % TPT;           // CF phase: table slot, thread in table
    const int io = t / TPT, oo = (t % TPT) / S, jj = t % S;   // option phase: table, option, k-block
    for (int64_t b0 = (int64_t)blockIdx.x * TB; b0 < n_q; b0 += (int64_t)gridDim.x * TB) {
        const int nb = (int)min<int64_t>(TB, n_q - b0);
        if (t < 64) serial_prio(true);               // the prologue lanes' wave
        if (t < nb) table_prologue(A, b0 + t, shc[t]);
        __syncthreads();
        serial_prio(false);
        // ---- CF entries of table slot `it` into LDS ----
        if (it < nb) {
            const double* c = shc[it];
            const double a = c[0], eb = c[2], ea = c[3], scale = c[4], piba = c[5];
            const double S0 = c[22], T = c[24];
            const int kcf = (int)c[30];                  // CF entries k < K_cf (cf_cut_scan)
            dh::CfConsts CC;
            {
                double* cc = (double*)&CC;
                for (int j = 0; j < 16; ++j) cc[j] = c[6 + j];
            }
            double2* tb = gtab + (size_t)it * N;
            const double delta = tail_delta(A.tail, S0, c[1] - a, N);
            double c0 = 0.0, c5 = 0.0, w0 = 0.0;
            int ne = 0;
            table_entries<TPT>(CC, sub, kcf, piba, T, a, scale, sct, [&](int k, double u, double w) {
                if (k == 0) {
                    w0 = 0.5 * w;
                    tb[0] = make_double2(0.0, 0.0);
                    return;
                }
                const double T2 = w * S0 * dh::drcp(1.0 + u * u);
                tb[k] = make_double2(T2, -(T2 * dh::drcp(u)));
                const double cb = (k & 1) ? -1.0 : 1.0;
                c0 += T2 * eb * cb;
                c5 += T2 * ea;
                ne = max(ne, tail_keep(k, T2, delta));
            });
            c0 = xor_sum(c0, TPT);
            c5 = xor_sum(c5, TPT);
            w0 = xor_sum(w0, TPT);                   // one nonzero term (thread 0's)
            ne = xor_max_i(ne, TPT);
            if (sub == 0) {
                ks[it][0] = c0;
                ks[it][1] = c5;
                ks[it][2] = w0;
                kne[it] = ne;
            }
        }
        __syncthreads();
        // ---- options of table slot `io`: option oo, k-block jj ----
        const int64_t q = b0 + io;
        const bool tab_ok = io < nb;
        const double* c = shc[tab_ok ? io : 0];
        const double a = c[0], b = c[1], piba = c[5], S0 = c[22];
        const int g0 = (int)c[27], gn = tab_ok ? (int)c[28] : 0;
        const bool in = tab_ok && oo < gn;
        const int m = g0 + (in ? oo : 0);
        double K = 0.0, xK = 0.0, ratio = 1.0;
        if (in) {
            K = option_strike(A, m, S0);
            xK = option_logk(K, S0, ratio);
        }
        const bool cl = in && (xK - 0.1 < a || xK + 0.1 > b);
        const bool use = in && !cl;
        double sum = 0.0;
        {
            const double th = use ? piba * (xK - a) : 0.0;
            double st, ct;
            dh::dsincos_t(th, sct, &st, &ct);
            const double c2 = 2.0 * ct;
            const double2* tb = gtab + (size_t)(tab_ok ? io : 0) * N;
            // the kept terms k < n_eff in S k-blocks of Lk
            const int ne = tab_ok ? kne[io] : 0;
            const int Lk = (max(ne, 1) - 1 + S - 1) / S;
            const int k_lo = 1 + jj * Lk, k_hi = min(ne, k_lo + Lk);
            double sc = 0.0, ss = 0.0;
            for (int k0 = k_lo; k0 < k_hi; k0 += kAnchor) {
                double cx, sx;                                     // cos / sin (k0 th)
                if (k0 == 1) {
                    cx = ct;
                    sx = st;
                } else {
                    dh::dsincos_t((double)k0 * piba * (xK - a), sct, &sx, &cx);
                }
                double cp = cx * ct + sx * st;                     // cos / sin ((k0 - 1) th)
                double sp = sx * ct - cx * st;
                // four steps per iteration with the entries read four ahead (immediate LDS
                // offsets), x_k / x_{k-1} swapping registers (angle_sum_1 with G = 1)
                const int kend = min(k_hi, k0 + kAnchor);
                int k = k0;
                const double2* tq = tb + k;
                double2 t0 = tq[0], t1 = tq[1], t2 = tq[2], t3 = tq[3];
                for (; k + 3 < kend; k += 4) {
                    tq += 4;
                    const double2 n0 = tq[0], n1 = tq[1], n2 = tq[2], n3 = tq[3];
                    sc = fma(t0.x, cx, sc);
                    ss = fma(t0.y, sx, ss);
                    cp = fma(c2, cx, -cp);                         // x_{k+1} into (cp, sp)
                    sp = fma(c2, sx, -sp);
                    sc = fma(t1.x, cp, sc);
                    ss = fma(t1.y, sp, ss);
                    cx = fma(c2, cp, -cx);                         // x_{k+2} into (cx, sx)
                    sx = fma(c2, sp, -sx);
                    sc = fma(t2.x, cx, sc);
                    ss = fma(t2.y, sx, ss);
                    cp = fma(c2, cx, -cp);
                    sp = fma(c2, sx, -sp);
                    sc = fma(t3.x, cp, sc);
                    ss = fma(t3.y, sp, ss);
                    cx = fma(c2, cp, -cx);
                    sx = fma(c2, sp, -sx);
                    t0 = n0;
                    t1 = n1;
                    t2 = n2;
                    t3 = n3;
                }
                for (; k < kend; ++k) {                            // the last < 4 steps
                    sc = fma(t0.x, cx, sc);
                    ss = fma(t0.y, sx, ss);
                    const double nc = fma(c2, cx, -cp), ns = fma(c2, sx, -sp);
                    cp = cx;
                    sp = sx;
                    cx = nc;
                    sx = ns;
                    t0 = t1;
                    t1 = t2;
                    t2 = t3;
                }
            }
            sum = use ? sc + ss : 0.0;
        }
        sum = xor_sum(sum, S);
        const int64_t p = A.p0 + (tab_ok ? q / tpp : 0);
        if (use && jj == 0) {
            const Consts C{ks[io][0], 0.0, ks[io][1], ks[io][2], a, b, c[2], c[3]};   // ne unused
            const double price = c[29] * option_sum(C, A.call[m] != 0, S0, K, xK, ratio, sum);
            if (A.out) A.out[p * A.out_stride + A.perm[m]] = price;
            if (A.part_sse) {
                const double mk = A.mkt[m];
                const double rel = (price - mk) / mk;
                osse[io][oo] = rel * rel;
                obad[io][oo] = (isnan(price) || isinf(price) || price <= 0.0) ? 1.0 : 0.0;
            }
        }
        // ---- clamp-widened options: the whole wave prices each (lanes over k) ----
        unsigned long long mask = __ballot(cl && jj == 0);
        while (mask) {
            const int l = __ffsll((long long)mask) - 1;
            mask &= mask - 1;
            const int src = (t & ~63) + l;                         // the clamped option's lane
            const int li = src / TPT, lo_ = (src % TPT) / S;
            const double* cl_c = shc[li];
            const double x = __shfl(xK, l, 64), Kl = __shfl(K, l, 64);
            const int ml = (int)cl_c[27] + lo_;
            const int64_t pl = A.p0 + (b0 + li) / tpp;
            const Params P = dh::load_params(A.prm + pl * DH_PARAM_STRIDE);
            const double ac = (x - 0.1 < cl_c[0]) ? x - 0.1 : cl_c[0];      // Python min/max
            const double bc = (x + 0.1 > cl_c[1]) ? x + 0.1 : cl_c[1];
            double v = clamped_term_sum(P, cl_c[24], Kl, x, ac, bc, A.call[ml] != 0, lane, 64, N,
                                        sct);
            v = xor_sum(v, 64);
            if (lane == 0) {
                const double price = cl_c[29] * v;
                if (A.out) A.out[pl * A.out_stride + A.perm[ml]] = price;
                if (A.part_sse) {
                    const double mk = A.mkt[ml];
                    const double rel = (price - mk) / mk;
                    osse[li][lo_] = rel * rel;
                    obad[li][lo_] = (isnan(price) || isinf(price) || price <= 0.0) ? 1.0 : 0.0;
                }
            }
        }
        if (A.part_sse) {
            __syncthreads();
            // one lane per table: the options' terms in option order, then the hand-off
            if (t < 64) serial_prio(true);
            if (t < nb) {
                const double* cc = shc[t];
                const int ng = (int)cc[28];
                double acc = 0.0;
                int nbad = 0;
                for (int o = 0; o < ng; ++o) {
                    acc += osse[t][o];
                    nbad += obad[t][o] != 0.0 ? 1 : 0;
                }
                const int64_t qq = b0 + t;
                const int64_t pp = A.p0 + qq / tpp;
                const int tile = A.paired ? 0 : (int)(qq % tpp);
                const int64_t task = A.paired ? pp : pp * A.n_tiles + tile;
                __hip_atomic_store(&A.part_sse[task], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&A.part_bad[task], nbad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const unsigned old = __hip_atomic_fetch_add(&A.counter[pp * kCounterStride], 1u,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int ntask = A.paired ? 1 : A.n_tiles;
                if (old == (unsigned)ntask - 1u) {
                    const int64_t base_i = A.paired ? pp : pp * A.n_tiles;
                    double s2 = 0.0;
                    int bad = 0;
                    for (int j = 0; j < ntask; ++j) {                // tile order
                        s2 += __hip_atomic_load(&A.part_sse[base_i + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        bad += __hip_atomic_load(&A.part_bad[base_i + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    loss_out(A, pp, s2, bad);
                    __hip_atomic_store(&A.counter[pp * kCounterStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        __syncthreads();                                 // gtab / shc / osse reused
    }
}

// ----------------------------------------------------------------------------------------------
// fused request kernel: one block per table (p, g) whose maturity group is one tile.
//   prologue (thread 0) || option staging (other waves first) -> CF loop writing the expanded
//   table straight into LDS + k-sums -> clamp scan -> fixed-order constants || rotations ->
//   tile sums -> fence-free loss hand-off.
// One launch and no table round trip through L2/MALL: the latency path of small requests
// (calibration function+gradient requests).  Every value is computed by the same expression, in
// the same order and with the same lane partition as cos_table_kernel<TPT1> followed by
// cos_option_kernel<tpt2>, so the two paths give the same bits.
// ----------------------------------------------------------------------------------------------
template <int TPT1, int RT, int WV = DH_FUSED_WAVES, bool KP = false>
__global__ __launch_bounds__(kBlock, WV) void cos_fused_kernel(
    const double* __restrict__ h_prm, const double* __restrict__ h_tsrc,
    const int2* __restrict__ h_groups, const int* __restrict__ h_live,
    const double* __restrict__ h_pre, int h_tpp, int h_paired, PriceArgs A_, int tpt2,
    typename std::conditional<KP, KargParams, NoKargParams>::type pb_) {
    // KP: the records are the param block at the end of the kernel arguments (read in place)
    const double* prm0 = KP ? karg_ref<KargParams, kFusedParamsKernargOff>().v : h_prm;
    const double* tsrc0 = KP ? karg_ref<KargParams, kFusedParamsKernargOff>().T : h_tsrc;
    const int2* groups0 = KP ? karg_ref<KargParams, kFusedParamsKernargOff>().groups : h_groups;
    const FusedHead H{prm0, tsrc0, groups0, h_live ? h_live : &kLiveOne, h_pre, h_tpp, h_paired};
    const PriceArgs& A = karg_ref<PriceArgs, kFusedArgsKernargOff>();
    // the halt test's load is issued here (a global load: a flat one would also hold up every
    // scalar load's wait) and its value used after the staging barrier, so it overlaps the
    // prologue instead of delaying it (a halted launch wastes the prologue only)
    const int live_v = *(const __attribute__((address_space(1))) int*)H.live;
    karg_prefetch_lines();
    extern __shared__ __attribute__((aligned(16))) double smem[];
    __shared__ double shc[kTabC];
    __shared__ double red[4][1];
    __shared__ double2 sct[dh::kMathTab];
    __shared__ unsigned long long cmask[kTileMax / 64];
    const int nthr = blockDim.x;
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wv = t >> 6;
    const int64_t q = blockIdx.x;                       // dispatch index
    const int64_t qt = xcd_table(A, H.tpp, q);          // the table it prices
    const int64_t p = (int64_t)((unsigned)qt / (unsigned)H.tpp);   // 32-bit: grids < 2^31 blocks
    const int g = (int)((unsigned)qt % (unsigned)H.tpp);
    DH_RT_BEGIN(A);
    DH_STAMP(A, 0);

    // ---- prologue (wave 0, lane-parallel) || per-option staging (wave 0 takes the last
    //      indices).  The prologue comes first in program order and reads the preloaded
    //      arguments only, so its loads issue before any kernel-argument wait ----
    // K_cf on the block's last wave (its CF-cut test overlaps wave 0's prologue; the staging loop
    // below gives that wave option indices nthr - 128 .. nthr - 65, none on C3's 100-option tiles)
    // (the <= 96-VGPR wide build runs it on wave 0 after the prologue: one range computation
    // less, and the build's register allocation gains: C4 -2.6%)
    const int wcut = (nthr > 64 && WV <= DH_FUSED_WAVES) ? nthr / 64 - 1 : 0;
    // prologues ahead (4-wave build, >= 3 waves): the first-round block's writer wave, and
    // whether this block's constants may have been formed ahead
    const int64_t R = (WV <= DH_FUSED_WAVES && nthr >= 192) ? A.ahead_stride : 0;
    const bool ahead_w = R > 0 && q < R;
    const bool ahead_r = R > 0 && q >= R && q < (kAheadMax + 1) * R;
    const int64_t nblocks = gridDim.x;
    if (!H.pre && (wv == 0 || wv == wcut)) serial_prio(true);
    if (H.pre) {
        if (t < kTabC) shc[t] = H.pre[qt * kTabC + t];
    } else if (wv == 0) {
        // (each of the two waves decides on its own flag load and fills its own slots: loaded or
        // formed, the same values, so a flag set between the two loads changes nothing)
        int kcf_f = 0;
        if (ahead_r && ahead_ready(A, q, kcf_f)) {
            ahead_read(A, H, q, qt, shc, lane);
            if (wcut == 0 && lane == 0) shc[30] = kcf_f;
        } else {
            table_prologue_wave(A, H, qt, shc, lane, wcut == 0);
        }
    } else if (wv == wcut) {
        int kcf_f = 0;
        if (ahead_r && ahead_ready(A, q, kcf_f)) {
            if (lane == 0) shc[30] = kcf_f;
        } else {
            const int kcf = A.N < kCfCutMinN ? A.N : prologue_cut_wave(A, H, qt, lane);
            if (lane == 0) shc[30] = kcf;
        }
    }
    DH_STAMP(A, 8);
    const int N = A.N;
    const int cap = A.opt_cap;
    const TileLds L = tile_lds(smem, N, cap);
    double* lclp = smem + option_lds_doubles(N, cap);     // prices of clamp-widened options
    int g0, gn;
    if (H.paired) {
        g0 = (int)p;
        gn = 1;
    } else {
        const int2 gr = H.groups[g];
        g0 = gr.x;
        gn = gr.y;
    }
    const double* prm = H.prm + p * DH_PARAM_STRIDE;
    const double S0 = prm[13];
    dh::load_math_tables(sct, nthr > 64 ? 64 : 0);      // the waves after the prologue's
    // staging order: waves 1, 2, .., then 0 (its prologue first)
    for (int i = (t + nthr - 64) % nthr; i < gn; i += nthr) {
        const int m = g0 + i;
        const double K = option_strike(A, m, S0);
        double ratio;
        const double xK = option_logk(K, S0, ratio);
        L.K[i] = K;
        L.mkt[i] = A.mkt ? A.mkt[m] : 0.0;
        L.call[i] = A.call[m];
        if (A.out) L.perm[i] = A.perm[m];                 // loss requests: no price columns
        L.xK[i] = xK;
        L.exK[i] = ratio;
    }
    __syncthreads();
    serial_prio(false);
    if (__builtin_amdgcn_readfirstlane(live_v) <= 0) return;   // every block reads the same count
    DH_STAMP(A, 1);

    const double a = shc[0], b = shc[1], eb = shc[2], ea = shc[3], scale = shc[4], piba = shc[5];
    const double T = shc[24];
    const int kcf = (int)shc[30];                    // CF entries k < K_cf (cf_cut_wave)
    // ---- clamp-widened options (double_heston.py:135-137), decided and priced per wave: the
    //      masks first (a short loop), the pricing loop only where a mask is set (rare: its
    //      register traffic stays off the common path).  The masks and prices are read after the
    //      CF barrier, so the scan may run before or after the CF loop with the same bits: before
    //      it in the 4-wave build (after it, the scan's LDS reads queue behind the table's stores
    //      on the request's critical path: C2 -1.7%), after it in the 5-wave build (before it,
    //      the register allocation of the <= 96-VGPR build costs C4 3%) ----
    auto clamp_scan = [&](int first, int step) {
        bool any_cl = false;
        for (int base = first; base < gn; base += step) {
            const int o = base + lane;
            bool cl = false;
            if (o < gn) {
                const double xK = L.xK[o];
                cl = xK - 0.1 < a || xK + 0.1 > b;
            }
            const unsigned long long mask = __ballot(cl);
            if (lane == 0) cmask[base / 64] = mask;
            any_cl = any_cl || mask != 0;
        }
        if (__builtin_expect(any_cl, 0))
        for (int base = first; base < gn; base += step) {
            const int o = base + lane;
            bool cl = false;
            if (o < gn) {
                const double xK = L.xK[o];
                cl = xK - 0.1 < a || xK + 0.1 > b;
            }
            unsigned long long mask = __ballot(cl);
            if (mask == 0) continue;
            const Params P = dh::load_params(prm);
            const double disc = exp(-P.r * T);
            while (mask) {
                const int l = __ffsll((long long)mask) - 1;
                mask &= mask - 1;
                const double x = L.xK[base + l];
                const double ac = (x - 0.1 < a) ? x - 0.1 : a;      // Python min/max
                const double bc = (x + 0.1 > b) ? x + 0.1 : b;
                double v = clamped_term_sum(P, T, L.K[base + l], x, ac, bc, L.call[base + l] != 0,
                                            lane, 64, N, sct);
                v = xor_sum(v, 64);
                if (lane == 0) lclp[base + l] = disc * v;
            }
        }
    };
    // (measured and not kept: the scan after the CF loop in multi-round requests, C3 +0.8 us)
    constexpr bool kEarlyClamp = WV <= DH_FUSED_WAVES;
    // (measured and not kept: the scan by the block's last wave when the CF loop leaves it idle,
    // so that the CF waves start their entries at once: C2 -0.1 us, C3 +0.2 us)
    if constexpr (kEarlyClamp) clamp_scan(wv * 64, nthr);
    DH_STAMP(A, 29);
    // ---- CF loop (threads < TPT1, one entry each up to N = 256): expanded table into LDS.
    //      (A lane pair per entry, one Heston factor each, cut C1 by 5% but cost C2 2%: the CF
    //      phase of a C2 request is issue-bound on the CUs that host two blocks.) ----
    __shared__ double w0s;
    if (t < TPT1) {
        dh::CfConsts CC;
        {
            double* cc = (double*)&CC;
            for (int j = 0; j < 16; ++j) cc[j] = shc[6 + j];
        }
        DH_STAMP(A, 6);
        DH_STAMP_T(A, 19, 64);
        DH_STAMP_T(A, 20, 192);
        table_entries<TPT1>(CC, t, kcf, piba, T, a, scale, sct, [&](int k, double u, double w) {
            if (k == 0) {
                w0s = 0.5 * w;
                L.t26[0] = make_double2(0.0, 0.0);
                return;
            }
            const double T2 = w * S0 * dh::drcp(1.0 + u * u);
            L.t26[k] = make_double2(T2, -(T2 * dh::drcp(u)));
        });
        DH_STAMP(A, 7);
        DH_STAMP_T(A, 16, 64);
        DH_STAMP_T(A, 17, 128);
        DH_STAMP_T(A, 18, 192);
    }
    // prologues ahead: the later tables' K_cf on the cut wave; both writer waves' stores drained
    // before the barrier, the flags after it
    int kcf_ahead = 0;
    if (ahead_w && wv == wcut) kcf_ahead = ahead_write(A, H, q, nblocks, lane);
    if constexpr (!kEarlyClamp) clamp_scan(wv * 64, nthr);
    DH_STAMP(A, 21);
    DH_STAMP_T(A, 22, 64);
    __syncthreads();
    DH_STAMP(A, 2);
    if (ahead_w && wv == wcut) ahead_publish(A, q, nblocks, lane, kcf_ahead);

    // ---- k-sums in the canonical order of a 64-thread table slot (from the LDS table; the same
    //      bits as cos_table_kernel).  c1 is a sum of zeros (+0.0) and w0 has one nonzero term
    //      (lane 0's), so their butterflies change no bit and are skipped || per-option
    //      rotations ----
    // c0 on wave 0 and c5 on the block's last wave (wave 1 stages the rotations): each wave runs
    // one sum's chain, in the same lane order and butterfly, so the same bits (4-wave build; the
    // 5-wave build keeps both on wave 0: its register allocation cost C4 2%)
    const int w5 = (WV <= DH_FUSED_WAVES && nthr >= 192) ? nthr / 64 - 1 : 0;
    if (wv == 0 || wv == w5) {
        serial_prio(true);
        const bool f0 = wv == 0, f5 = wv == w5;
        const double delta = tail_delta(A.tail, S0, b - a, N);
        double c0 = 0.0, c5 = 0.0;
        int ne = 0;                                  // n_eff (tail_keep), on wave 0 with c0
        for (int k = lane; k < kcf; k += 64) {
            if (k == 0) continue;
            const double T2 = L.t26[k].x;
            const double cb = (k & 1) ? -1.0 : 1.0;
            if (f0) {
                c0 += T2 * eb * cb;
                ne = max(ne, tail_keep(k, T2, delta));
            }
            if (f5) c5 += T2 * ea;
        }
        if (f0) {
            c0 = xor_sum(c0, 64);
            ne = xor_max_i(ne, 64);
        }
        if (f5) c5 = xor_sum(c5, 64);
        if (lane == 0) {
            if (f0) {
                red[0][0] = c0;
                red[1][0] = (double)ne;
                red[3][0] = w0s;
            }
            if (f5) red[2][0] = c5;
        }
    }
    const double disc = shc[29];                    // e^{-rT}, staged by the prologue
    const int G = group_lanes<RT>(gn, N, tpt2);
    {
        const double ustep = G * dh::kPi / (b - a);
        for (int i = (t + nthr - 64) % nthr; i < gn; i += nthr) {          // wave 0 does the sums
            const bool cl = (cmask[i >> 6] >> (i & 63)) & 1ull;
            double ss, cs;
            dh::dsincos(ustep * (cl ? 0.0 : L.xK[i] - a), &ss, &cs);
            L.cs[i] = cs;
            L.ss[i] = cl ? NAN : (ss == ss ? ss : 0.0);   // as cos_option_kernel
            if (cl) record_price(A, p, L.perm[i], L.mkt[i], i, lclp[i], L.sse, L.bad);
        }
    }
    __syncthreads();
    serial_prio(false);
    DH_STAMP(A, 3);

    const Consts C{0.0 + red[0][0], 0.0 + red[1][0], 0.0 + red[2][0], 0.0 + red[3][0], a, b, eb, ea};
    if (t < tpt2) tile_sums_r<RT>(A, p, C, S0, disc, gn, G, tpt2, t, true, L, lclp + cap, sct);
    DH_STAMP(A, 4);
    // (a block-wide tile reduced through LDS has just passed tile_sums' closing barrier, after
    // its last loss terms were written, so a second one is not needed; measured, dropping it was
    // slower on C3: 57.8 vs 57.45 us per request)
#ifndef DH_SKIP_HANDOFF_BARRIER
#define DH_SKIP_HANDOFF_BARRIER 0
#endif
    const bool lds_red = DH_SKIP_HANDOFF_BARRIER && tpt2 == kBlock && nthr == kBlock &&
                         (G > 64 || (G & (G - 1)) != 0);
    if (A.part_sse) {
        if (!lds_red) __syncthreads();
        if (t < 64) {
            serial_prio(true);
            task_loss(A, p, A.paired ? p : p * A.n_tiles + g, gn, t, L.sse, L.bad);
            // the grid's last P blocks (dispatch order) then sum one param set each
            if (A.partials_only == 3 && q >= nblocks - A.P) tail_sums(A, q - (nblocks - A.P), t);
        }
    }
    DH_STAMP(A, 5);
    DH_RT_END(A);
}

// ----------------------------------------------------------------------------------------------
// validation path: reference operation order (double_heston.py:160-192), one wave per option
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ double exact_term_sum(const Params& P, double T, double K, double xK,
                                                 double a, double b, bool is_call, int k_first,
                                                 int k_step, int N) {
    const double ba = b - a;
    const double scale = 2.0 / ba;
    double acc = 0.0;
    for (int k = k_first; k < N; k += k_step) {
        const double u = k * dh::kPi / ba;
        const cplx phi = dh::cf_eval(P, u, T);
        double sa, ca;
        dh::dsincos(u * a, &sa, &ca);
        const double re = phi.re * ca + phi.im * sa;       // Re(phi exp(-i u a))
        double chi, psi;
        if (is_call) dh::cos_coeffs(k, xK, b, a, b, chi, psi);
        else dh::cos_coeffs(k, a, xK, a, b, chi, psi);
        const double V = is_call ? scale * (P.S0 * chi - K * psi) : scale * (K * psi - P.S0 * chi);
        double term = re * V;
        if (k == 0) term *= 0.5;
        acc += term;
    }
    return acc;
}

__global__ __launch_bounds__(kBlock) void cos_exact_kernel(PriceArgs A, double* prices) {
    const int64_t item = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int M = A.M;
    const int64_t n_items = A.paired ? A.P : A.P * (int64_t)M;
    if (item >= n_items) return;                       // whole wave exits together
    const int64_t p = A.paired ? item : item / M;
    const int m = A.paired ? (int)p : (int)(item % M);
    const Params P = dh::load_params(A.prm + p * DH_PARAM_STRIDE);
    const double T = A.T[m];
    const double K = option_strike(A, m, P.S0);
    const bool is_call = A.call[m] != 0;
    const double xK = log(K / P.S0);
    double a0, b0;
    dh::trunc_unclamped(P, T, A.L, a0, b0);
    const double a = (xK - 0.1 < a0) ? xK - 0.1 : a0;   // Python min/max semantics (:136-137)
    const double b = (xK + 0.1 > b0) ? xK + 0.1 : b0;
    double acc = exact_term_sum(P, T, K, xK, a, b, is_call, lane, 64, A.N);
    acc = xor_sum(acc, 64);
    if (lane == 0) {
        const double price = exp(-P.r * T) * acc;
        if (A.out) A.out[p * A.out_stride + A.perm[m]] = price;
        if (prices) prices[A.paired ? p : p * M + m] = price;
    }
}

// Loss sums from a [P][M] price buffer (validation mode): one wave per param set, fixed order.
// The generator's param records from its sampler's columns (dh_surface_price_cols): rec[i][c] =
// params[i][c] (c < 13), spots[i], r, 0 -- one thread per record field, coalesced stores.
__global__ void gen_records_kernel(const double* __restrict__ params,
                                   const double* __restrict__ spots, double r, int64_t P,
                                   double* __restrict__ rec) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P * DH_PARAM_STRIDE) return;
    const int64_t row = i / DH_PARAM_STRIDE;
    const int c = (int)(i % DH_PARAM_STRIDE);
    rec[i] = c < 13 ? params[row * 13 + c] : (c == 13 ? spots[row] : (c == 14 ? r : 0.0));
}

__global__ void loss_from_prices_kernel(const double* __restrict__ prices,
                                        const double* __restrict__ mkt, int M, int64_t S,
                                        double* __restrict__ sse, int* __restrict__ n_bad) {
    const int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (s >= S) return;
    double acc = 0.0, bad = 0.0;
    for (int m = lane; m < M; m += 64) {
        const double pr = prices[s * M + m];
        const double rel = (pr - mkt[m]) / mkt[m];
        acc += rel * rel;
        bad += (isnan(pr) || isinf(pr) || pr <= 0.0) ? 1.0 : 0.0;
    }
    acc = xor_sum(acc, 64);
    bad = xor_sum(bad, 64);
    if (lane == 0) {
        sse[s] = acc;
        n_bad[s] = (int)bad;
    }
}

// ----------------------------------------------------------------------------------------------
// building blocks behind the reference's public methods
// ----------------------------------------------------------------------------------------------
__global__ void cf_kernel(const double* __restrict__ prm, const double* __restrict__ u, int n,
                          double tau, double* __restrict__ re, double* __restrict__ im) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Params P = dh::load_params(prm);
    const cplx c = dh::cf_eval(P, u[i], tau);
    re[i] = c.re;
    im[i] = c.im;
}

__global__ void cf_kernel_z(const double* __restrict__ prm, const double* __restrict__ ure,
                            const double* __restrict__ uim, int n, double tau,
                            double* __restrict__ re, double* __restrict__ im) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Params P = dh::load_params(prm);
    const cplx c = dh::cf_eval_z(P, {ure[i], uim[i]}, tau);
    re[i] = c.re;
    im[i] = c.im;
}

__global__ void trunc_kernel(const double* __restrict__ prm, const double* __restrict__ K,
                             const double* __restrict__ T, int64_t P, double L,
                             double* __restrict__ a, double* __restrict__ b) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const Params Q = dh::load_params(prm + i * DH_PARAM_STRIDE);
    double a0, b0;
    dh::trunc_unclamped(Q, T[i], L, a0, b0);
    const double xK = log(K[i] / Q.S0);
    a[i] = (xK - 0.1 < a0) ? xK - 0.1 : a0;
    b[i] = (xK + 0.1 > b0) ? xK + 0.1 : b0;
}

__global__ void coeff_kernel(const int32_t* __restrict__ k, int n, double c, double d, double a,
                             double b, double* __restrict__ chi, double* __restrict__ psi) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x, y;
    dh::cos_coeffs(k[i], c, d, a, b, x, y);
    chi[i] = x;
    psi[i] = y;
}

// ----------------------------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------------------------
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return fail(DH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
    } while (0)

struct DevBuf {
    void* ptr = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipMalloc(&ptr, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
};

// Pinned, device-mapped host memory (grow-only): small request inputs and outputs the kernels
// read and write directly over PCIe, so a host-API request is one launch and one sync.
struct HostBuf {
    void* ptr = nullptr;       // host address
    void* dptr = nullptr;      // device address of the same bytes
    size_t cap = 0;
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        release();
        const size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipHostMalloc(&ptr, want, hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) {
            ptr = nullptr;
            return e;
        }
        e = hipHostGetDevicePointer(&dptr, ptr, 0);
        if (e != hipSuccess) {
            release();
            return e;
        }
        cap = want;
        return hipSuccess;
    }
    void release() {
        if (ptr) (void)hipHostFree(ptr);
        ptr = dptr = nullptr;
        cap = 0;
    }
};

// Threads per table.  The fused kernel takes one entry per thread up to N = 256 (latency).  The
// split path's table kernel takes the slot width (64, 128 or 256 threads; 64 = one wave per table
// defines the canonical order of the k-sums, which the others re-form from LDS) that minimises
// rounds of resident slots x entries per thread; 64 unless a wider slot saves >= 10% (requests
// with few tables per slot, e.g. C3: 4,200 tables on 3,072 one-wave slots).
struct dh_ctx_view {
    int resident[3] = {0, 0, 0};
    int resident_gen[3] = {0, 0, 0};   // cos_gen_kernel<16 / 8 / 4> at its N's LDS
};

int fused_tpt(int N) { return N <= 64 ? 64 : (N <= 128 ? 128 : 256); }

// cos_gen_kernel<TB>: TB tables' (T2, T6) in LDS, <= 32 KB per block (three blocks per CU)
constexpr int gen_max_n(int TB) { return 2048 / TB; }
int gen_tb(int N) { return N <= gen_max_n(16) ? 16 : (N <= gen_max_n(8) ? 8 : (N <= gen_max_n(4) ? 4 : 0)); }

int table_tpt(const dh_ctx_view& v, int64_t n_q, int N) {
    auto cost = [&](int i) {
        const int tpt = 64 << i;
        const int64_t slots = (int64_t)std::max(1, v.resident[i]) * (kBlock / tpt);
        return (double)((n_q + slots - 1) / slots) * (double)((N + tpt - 1) / tpt);
    };
    const double c64 = cost(0);
    int best = 0;
    double bc = c64;
    for (int i = 1; i < 3; ++i) {
        if ((64 << i) > N) break;
        const double c = cost(i);
        if (c < bc && c <= 0.9 * c64) {
            best = i;
            bc = c;
        }
    }
    return 64 << best;
}

// option-kernel threads per task: enough lanes for ceil(nopt/kR) groups, LDS permitting
#ifndef DH_BIG_TILE_TPT
#define DH_BIG_TILE_TPT 256   // option threads of tiles of more than 64 options (128: G <= 4 lanes
#endif                        // per 4-option group on C3's 100-option tiles)
int option_tpt(int max_nopt, int N, int cap) {
    int tpt = max_nopt <= kR ? 64 : (max_nopt <= 4 * kR ? 128 : (max_nopt > 64 ? DH_BIG_TILE_TPT : 256));
    while (tpt < kBlock &&
           ((size_t)(kBlock / tpt) * option_lds_doubles(N, cap) + (tpt == kBlock ? kRedDoubles : 0)) *
                   sizeof(double) > (size_t)kLdsDyn)
        tpt *= 2;
    return tpt;
}

}  // namespace

struct GenBufs;                         // dh_gen_device.h
void gen_bufs_release(dh_ctx* ctx);

struct dh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf params, out, sse, bad, part_sse, part_bad, counter, exact_prices, table, consts, cl_mask,
        cl_price, aux0, aux1, aux2, aux3, pre;
    HostBuf h_params, h_loss;  // zero-copy inputs / outputs of small host-API loss requests
    HostBuf h_pairs;           // zero-copy inputs / outputs of small dh_price_pairs calls
    DevBuf lb_state, lb_rec, lb_sse, lb_bad, lb_live, lb_done, lb_x0;   // dh_calibrate_lbfgs
    HostBuf h_lb;              // finished flags / live list of dh_calibrate_lbfgs
    // the two in-flight slots of dh_surface_fg_begin / _end: zero-copy records in, sse / n_bad
    // out, the host-side Feller terms and FD steps, and the request's completion event
    // largest (param sets x tasks) of any dh_surface_fg_begin request on (fg_surf, fg_N): the
    // scratch reservations are a function of the surface, N and the param-set count only
    size_t fg_max_units = 0;
    const dh_surface* fg_surf = nullptr;
    int fg_N = 0;
    struct FgSlot {
        HostBuf h_params, h_loss;
        std::vector<double> pen, dx;
        int S = 0, M = 0;
        const dh_surface* surf = nullptr;   // the surface the request was enqueued on
        bool pending = false;
        hipEvent_t done = nullptr;
    } fg[DH_FG_SLOTS];
    DevBuf lb_trace, lb_trace_n;   // diagnostic request trace of dh_calibrate_lbfgs
    hipEvent_t lb_ev[2] = {nullptr, nullptr};   // chunk-completion events of dh_calibrate_lbfgs
    int64_t lb_trace_cap = 0;
    bool attr_set = false;
    dh_ctx_view view;          // resident cos_table_kernel<64/128/256> blocks, whole chip
    int exact = 0;          // validation mode: every option through the per-term exact path
    int tail_cut = 1;       // adaptive tail of the angle sums (tail_delta; dh_ctx_set_tail_cut)
    int path = DH_PATH_AUTO;   // fused / split request kernels (dh_ctx_set_path)
    int last_path = 0;         // kernels of the last fast-path request (dh_ctx_last_path)
    int stamps_on = 0;      // diagnostic builds: record per-block phase stamps
    DevBuf stamps;
    int64_t stamps_n = 0;
    // prologues ahead (launch_fused): constants and flags of the later-round tables, the launch
    // epoch, $DHCOS_AHEAD (-1: not read yet; 0 turns it off) and the resident-block counts of the
    // fused kernel builds it applies to, by (t1, r1, LDS bytes)
    DevBuf ahead, ahead_flag;
    size_t ahead_flag_cap = 0;
    DevBuf gran;               // tail_sums' granules (partials_only == 3), zeroed on allocation
    size_t gran_cap = 0;
    int remap_on = -1;         // $DHCOS_XCD_REMAP: one-round fused grids map blocks to tables by XCD
                               // (xcd_table; 0 off, 2 multi-round grids too)
    unsigned ahead_epoch = 0;
    int ahead_on = -1;
    // the host copy of the next fused launch's param records (dh_surface_fg_begin sets it
    // around its launch): fused launches of <= kKargSets records pass them in their kernel
    // arguments; $DHCOS_KARG_PARAMS=0 turns that off (kp_on: -1 not read yet)
    const double* kp_src = nullptr;
    const dh_surface* kp_surf = nullptr;   // and its surface (host copies of the groups)
    int64_t kp_n = 0;
    int kp_on = -1;
    // and its completion event: recorded by the launch itself (hipExtLaunchKernel's stop event)
    // when the fused kernel is the request's last launch; kp_done_set tells the caller
    // ($DHCOS_EXT_EVENT=0: a separate hipEventRecord; ext_on: -1 not read yet)
    hipEvent_t kp_done = nullptr;
    bool kp_done_set = false;
    int ext_on = -1;
    int defer_on = -1;         // $DHCOS_DEFER: multi-round fused loss requests sum their partials
                               // in the launch's tail (2), in loss_partials_kernel (1) or through
                               // the ticket hand-off (0); -1: not read yet
    std::vector<std::pair<std::array<int64_t, 3>, int>> resident_fused;
    GenBufs* gen = nullptr;    // the generator's device draw (dh_gen_device)
};

struct dh_surface {
    dh_ctx* ctx = nullptr;
    int M = 0;
    int n_tiles = 0;
    int n_groups = 0;       // distinct maturities
    int max_nopt = 0;       // largest tile
    int max_group = 0;      // largest maturity group
    int strike_mode = 0;
    bool has_mkt = false;
    double* K = nullptr;
    double* T = nullptr;
    double* mkt = nullptr;
    int8_t* call = nullptr;
    int* perm = nullptr;
    int2* tiles = nullptr;
    int* tile_group = nullptr;
    double* group_T = nullptr;
    int2* groups = nullptr;
    void* block = nullptr;  // the one device allocation every array above points into
    std::vector<double> h_group_T;   // host copies of group_T / groups (the fused launch's
    std::vector<int2> h_groups;      // kernel arguments, KargParams)
};

namespace {

// Requests run the per-term path (cos_exact_kernel) in validation mode, and for series longer
// than the fast path's LDS-resident table holds (N > DH_MAX_N).
bool per_term(const dh_ctx* ctx, int N) { return ctx->exact || N > DH_MAX_N; }

// A negative invalid count is tail_sums' timeout marker (a loss hand-off that never completed):
// an error, not a loss
int check_loss_counts(const int32_t* n_bad, int64_t S) {
    for (int64_t i = 0; i < S; ++i)
        if (n_bad[i] < 0)
            return fail(DH_E_HIP, "loss hand-off timed out in the fused kernel (param set " +
                                      std::to_string(i) + ")");
    return DH_OK;
}

// Busy-wait for a short request (a calibration iteration waits on it): polling hipStreamQuery
// returns as soon as the stream drains, where hipStreamSynchronize may yield the thread.
int spin_sync(hipStream_t st) {
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return DH_OK;
        if (e != hipErrorNotReady)
            return fail(DH_E_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(e));
    }
}

}  // namespace

// Makes the context's device current for one C-ABI call and restores the caller's device on
// return.  The HIP runtime is shared with torch (one libamdhip64 per process), so leaving another
// device current would move torch's current device under the caller (a rank's RCCL tensors would
// land on the wrong GPU).
struct DeviceScope {
    int prev = -1;
    int rc = DH_OK;
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev == device) return;
        const hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) {
            rc = fail(DH_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
            prev = -1;
        }
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

namespace {

int ensure_attrs(dh_ctx* ctx) {
    if (ctx->attr_set) return DH_OK;
    for (const void* f :
         {(const void*)cos_option_kernel<64, 1>, (const void*)cos_option_kernel<128, 1>,
          (const void*)cos_option_kernel<256, 1>, (const void*)cos_option_kernel<64, kR>,
          (const void*)cos_option_kernel<128, kR>, (const void*)cos_option_kernel<256, kR>,
          (const void*)cos_fused_kernel<64, 1>, (const void*)cos_fused_kernel<128, 1>,
          (const void*)cos_fused_kernel<256, 1>, (const void*)cos_fused_kernel<64, kR>,
          (const void*)cos_fused_kernel<128, kR>, (const void*)cos_fused_kernel<256, kR>,
          (const void*)cos_fused_kernel<64, 1, DH_FUSED_WAVES_WIDE>,
          (const void*)cos_fused_kernel<128, 1, DH_FUSED_WAVES_WIDE>,
          (const void*)cos_fused_kernel<256, 1, DH_FUSED_WAVES_WIDE>,
          (const void*)cos_fused_kernel<64, 1, DH_FUSED_WAVES, true>,
          (const void*)cos_fused_kernel<128, 1, DH_FUSED_WAVES, true>,
          (const void*)cos_fused_kernel<256, 1, DH_FUSED_WAVES, true>})
        HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsDyn));
    // table-kernel grid = resident capacity (each block then owns a contiguous table range)
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    const void* fns[3] = {(const void*)cos_table_kernel<64>, (const void*)cos_table_kernel<128>,
                          (const void*)cos_table_kernel<256>};
    for (int i = 0; i < 3; ++i) {
        // dynamic LDS at DH_MAX_N (T2 of each wider slot) so the count never overstates
        const size_t lds = i == 0 ? 0 : (size_t)(kBlock / (64 << i)) * DH_MAX_N * sizeof(double);
        int per_cu = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fns[i], kBlock, lds));
        ctx->view.resident[i] = std::max(1, per_cu) * std::max(1, cus);
    }
    const void* gens[3] = {(const void*)cos_gen_kernel<16>, (const void*)cos_gen_kernel<8>,
                           (const void*)cos_gen_kernel<4>};
    for (int i = 0; i < 3; ++i) {               // LDS of the largest N each build takes
        const size_t lds = (size_t)gen_max_n(16 >> i) * (16 >> i) * sizeof(double2);
        int per_cu = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gens[i], kBlock, lds));
        ctx->view.resident_gen[i] = std::max(1, per_cu) * std::max(1, cus);
    }
    ctx->attr_set = true;
    return DH_OK;
}

int check_N(int N) {
    if (N < 1 || N > DH_MAX_N_PER_TERM)
        return fail(DH_E_ARG, "N must be in [1, " + std::to_string(DH_MAX_N_PER_TERM) + "], got " +
                                  std::to_string(N));
    return DH_OK;
}

int launch_exact(dh_ctx* ctx, const PriceArgs& A, hipStream_t st) {
    const int64_t n_items = A.paired ? A.P : A.P * (int64_t)A.M;
    double* prices = nullptr;
    if (A.part_sse) {
        HIP_TRY(ctx->exact_prices.reserve((size_t)n_items * 8));
        prices = (double*)ctx->exact_prices.ptr;
    }
    const int64_t blocks = (n_items * 64 + kBlock - 1) / kBlock;
    if (blocks > 0x7fffffffLL) return fail(DH_E_ARG, "too many items for one launch");
    hipLaunchKernelGGL(cos_exact_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, A, prices);
    HIP_TRY(hipGetLastError());
    if (A.part_sse) {
        const int64_t S = A.P;
        hipLaunchKernelGGL(loss_from_prices_kernel, dim3((unsigned)((S * 64 + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, st, (const double*)prices, A.mkt, A.M, S, A.sse,
                           A.n_bad);
        HIP_TRY(hipGetLastError());
    }
    return DH_OK;
}

constexpr int kZeroCopyMaxSets = 1024;       // host-API loss requests up to this many param sets
                                             // read / write through mapped host memory

size_t fused_lds_bytes(int N, int cap) {
    return ((size_t)option_lds_doubles(N, cap) + (size_t)cap + kRedDoubles) * sizeof(double);
}

#ifndef DH_FUSED_WIDE_MIN_BLOCKS
#define DH_FUSED_WIDE_MIN_BLOCKS 4096
#endif
constexpr int64_t kFusedWideMinBlocks = DH_FUSED_WIDE_MIN_BLOCKS;
// fused grids from this size take their prologue constants from table_prologue_kernel (C4's
// 28,672 blocks: 297 -> 285 us; C3's 4,200 lose 3% to the extra launch, C2's 448 its latency)
#ifndef DH_PROLOGUE_KERNEL_MIN_BLOCKS
#define DH_PROLOGUE_KERNEL_MIN_BLOCKS 8192
#endif
constexpr int64_t kPrologueKernelMinBlocks = DH_PROLOGUE_KERNEL_MIN_BLOCKS;

// One fused launch for the whole request (every group is one tile).
int launch_fused(dh_ctx* ctx, const PriceArgs& A0, hipStream_t st) {
    const int N = A0.N;
    const int tpp = A0.paired ? 1 : A0.n_groups;
    const int t1 = fused_tpt(N);
    const int max_nopt = A0.paired ? 1 : A0.opt_cap;
    const int t2 = option_tpt(max_nopt, N, A0.opt_cap);
    const size_t lds = fused_lds_bytes(N, A0.opt_cap);
    const int64_t blocks = A0.P * tpp;
    if (blocks > 0x7fffffffLL) return fail(DH_E_ARG, "launch too large");
    PriceArgs A = A0;
    A.p0 = 0;
    A.np = A0.P;
    if (ctx->stamps_on) {
        HIP_TRY(ctx->stamps.reserve((size_t)blocks * kStamps * 8));
        HIP_TRY(hipMemsetAsync(ctx->stamps.ptr, 0, (size_t)blocks * kStamps * 8, st));
        ctx->stamps_n = blocks * kStamps;
        A.stamps = (unsigned long long*)ctx->stamps.ptr;
    }
    const dim3 grid((unsigned)blocks), block((unsigned)std::max(t1, t2));
    const double* tsrc = A.paired ? A.T : A.group_T;       // FusedHead: preloaded arguments
    const bool r1 = tile_r(max_nopt, t2) == 1;
    A.ahead = nullptr;
    A.ahead_flag = nullptr;
    A.ahead_stride = 0;
    A.gran = nullptr;
    if (ctx->remap_on < 0) {
        const char* e = std::getenv("DHCOS_XCD_REMAP");
        ctx->remap_on = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 1;
    }
    // by XCD: one-round grids of more than one maturity group (below); multi-round grids (C3)
    // measured slower with it (57.7 vs 56.5 us per request), one-round C2 0.15 us faster
    A.remap = 0;
    bool remap_ok = ctx->remap_on && !A.paired && tpp > 1;
    if (ctx->ahead_on < 0) {
        const char* e = std::getenv("DHCOS_AHEAD");
        ctx->ahead_on = (e && e[0] == '0') ? 0 : 1;
    }
    // prologues ahead: the 4-wave build of >= 3-wave blocks, more blocks than one round of
    // resident ones, in-block prologues (no prologue kernel)
    const bool wide = r1 && blocks >= kFusedWideMinBlocks;
    if (ctx->ahead_on && !wide && block.x >= 192 && blocks < kPrologueKernelMinBlocks) {
        const std::array<int64_t, 3> key{t1, r1 ? 1 : 0, (int64_t)lds};
        int res = -1;
        for (const auto& kv : ctx->resident_fused)
            if (kv.first == key) res = kv.second;
        if (res < 0) {
            const void* f = nullptr;
            switch (t1 * (r1 ? 1 : -1)) {
                case 64: f = (const void*)cos_fused_kernel<64, 1>; break;
                case 128: f = (const void*)cos_fused_kernel<128, 1>; break;
                case 256: f = (const void*)cos_fused_kernel<256, 1>; break;
                case -64: f = (const void*)cos_fused_kernel<64, kR>; break;
                case -128: f = (const void*)cos_fused_kernel<128, kR>; break;
                default: f = (const void*)cos_fused_kernel<256, kR>; break;
            }
            int per_cu = 0, cus = 0;
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, (int)block.x, lds));
            HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
            res = std::max(1, per_cu) * std::max(1, cus);
            ctx->resident_fused.push_back({key, res});
        }
        if (ctx->defer_on < 0) {
            const char* e = std::getenv("DHCOS_DEFER");
            ctx->defer_on = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 2;
        }
        const int defer = ctx->defer_on;
        if (blocks > res) {
            const size_t slots = (size_t)blocks;
            HIP_TRY(ctx->ahead.reserve(slots * kAheadRec * sizeof(double)));
            if (slots > ctx->ahead_flag_cap) {
                HIP_TRY(ctx->ahead_flag.reserve(slots * sizeof(unsigned long long)));
                HIP_TRY(hipMemsetAsync(ctx->ahead_flag.ptr, 0, ctx->ahead_flag.cap, st));
                ctx->ahead_flag_cap = ctx->ahead_flag.cap / sizeof(unsigned long long);
            }
            if (++ctx->ahead_epoch == 0) ++ctx->ahead_epoch;     // 0: the cleared flags' value
            A.ahead = (double*)ctx->ahead.ptr;
            A.ahead_flag = (unsigned long long*)ctx->ahead_flag.ptr;
            A.ahead_stride = res;
            A.ahead_epoch = ctx->ahead_epoch;
            if (ctx->remap_on == 2 && remap_ok) A.remap = 1;   // C3 +1.1 us: off by default
            // and the loss sums deferred (below), or in loss_partials_kernel ($DHCOS_DEFER=1)
            if (defer == 1 && A.part_sse && !A.partials_only && !A.paired) {
                // (partial, invalid count) pairs: 16 bytes per task
                HIP_TRY(ctx->part_sse.reserve((size_t)A.P * A.n_tiles * 2 * sizeof(double)));
                A.part_sse = (double*)ctx->part_sse.ptr;
                A.partials_only = 2;
            }
        } else if (remap_ok) {
            A.remap = 1;                         // one round of resident blocks
        }
        // loss sums in the launch's tail ($DHCOS_DEFER=2, the default; 0: the hand-off's ticket in
        // every block): C3 -1.1 us against loss_partials_kernel, C2 (one round) -0.5 us against
        // the ticket.  At most a quarter of the resident blocks wait (tail_sums)
        if (defer == 2 && A.part_sse && !A.partials_only && !A.paired && A.P <= res / 4 &&
            A.max_group < (1 << kGranCountBits)) {
            if (A.ahead_stride == 0 && ++ctx->ahead_epoch == 0) ++ctx->ahead_epoch;
            A.ahead_epoch = ctx->ahead_epoch;
            const int64_t tasks = A.P * A.n_tiles;
            if ((size_t)tasks > ctx->gran_cap) {    // two granules per task, zeroed (no epoch is 0)
                HIP_TRY(ctx->gran.reserve((size_t)tasks * 2 * sizeof(unsigned long long)));
                HIP_TRY(hipMemsetAsync(ctx->gran.ptr, 0, ctx->gran.cap, st));
                ctx->gran_cap = ctx->gran.cap / (2 * sizeof(unsigned long long));
            }
            A.gran = (unsigned long long*)ctx->gran.ptr;
            A.partials_only = 3;
        }
    }
    if (blocks >= kPrologueKernelMinBlocks && !ctx->stamps_on) {
        HIP_TRY(ctx->pre.reserve((size_t)blocks * kTabC * sizeof(double)));
        A.pre = (const double*)ctx->pre.ptr;
        hipLaunchKernelGGL(table_prologue_kernel,
                           dim3((unsigned)((blocks * kPreLanes + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, st, A, blocks, (double*)ctx->pre.ptr);
        HIP_TRY(hipGetLastError());
    }
    // small requests whose records were handed over from the host (dh_surface_fg_begin): the
    // records in the kernel arguments (in-block-prologue launches of the 4-wave build)
    if (ctx->kp_on < 0) {
        const char* e = std::getenv("DHCOS_KARG_PARAMS");
        ctx->kp_on = (e && e[0] == '0') ? 0 : 1;
    }
    if (ctx->kp_on && ctx->kp_src && ctx->kp_surf && !A.paired &&
        (int)ctx->kp_surf->h_group_T.size() == tpp && tpp <= kKargGroups &&
        A.P == ctx->kp_n && A.P <= kKargSets && r1 && !wide &&
        blocks < kPrologueKernelMinBlocks && !ctx->stamps_on && !A.exact) {
        KargParams pb{};
        std::memcpy(pb.v, ctx->kp_src, (size_t)A.P * DH_PARAM_STRIDE * sizeof(double));
        std::memcpy(pb.T, ctx->kp_surf->h_group_T.data(), (size_t)tpp * sizeof(double));
        std::memcpy(pb.groups, ctx->kp_surf->h_groups.data(), (size_t)tpp * sizeof(int2));
        if (ctx->ext_on < 0) {
            const char* e = std::getenv("DHCOS_EXT_EVENT");
            ctx->ext_on = (e && e[0] == '0') ? 0 : 1;
        }
        hipEvent_t stop = (ctx->ext_on && A.partials_only != 2) ? ctx->kp_done : nullptr;
        switch (t1) {
            case 64: hipExtLaunchKernelGGL((cos_fused_kernel<64, 1, DH_FUSED_WAVES, true>), grid, block, lds, st, nullptr, stop, 0, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, pb); break;
            case 128: hipExtLaunchKernelGGL((cos_fused_kernel<128, 1, DH_FUSED_WAVES, true>), grid, block, lds, st, nullptr, stop, 0, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, pb); break;
            default: hipExtLaunchKernelGGL((cos_fused_kernel<256, 1, DH_FUSED_WAVES, true>), grid, block, lds, st, nullptr, stop, 0, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, pb); break;
        }
        HIP_TRY(hipGetLastError());
        ctx->kp_done_set = stop != nullptr;
        if (A.partials_only == 2) {
            hipLaunchKernelGGL(loss_partials_kernel, dim3((unsigned)A.P), dim3(64), 0, st,
                               (const double2*)A.part_sse, A.n_tiles, A.sse, A.n_bad);
            HIP_TRY(hipGetLastError());
        }
        return DH_OK;
    }
    // grids of many small blocks (C4: 28,672) gain from a fifth wave per SIMD to overlap the
    // blocks' latency-bound phases; small grids keep the 4-wave build, whose blocks are shorter
    // (same arithmetic: only the register allocation differs, so the same bits)
    if (r1 && blocks >= kFusedWideMinBlocks) {
        switch (t1) {
            case 64: hipLaunchKernelGGL((cos_fused_kernel<64, 1, DH_FUSED_WAVES_WIDE>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
            case 128: hipLaunchKernelGGL((cos_fused_kernel<128, 1, DH_FUSED_WAVES_WIDE>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
            default: hipLaunchKernelGGL((cos_fused_kernel<256, 1, DH_FUSED_WAVES_WIDE>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
        }
        HIP_TRY(hipGetLastError());
        return DH_OK;
    }
    switch (t1 * (r1 ? 1 : -1)) {
        case 64: hipLaunchKernelGGL((cos_fused_kernel<64, 1>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
        case 128: hipLaunchKernelGGL((cos_fused_kernel<128, 1>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
        case 256: hipLaunchKernelGGL((cos_fused_kernel<256, 1>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
        case -64: hipLaunchKernelGGL((cos_fused_kernel<64, kR>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
        case -128: hipLaunchKernelGGL((cos_fused_kernel<128, kR>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
        default: hipLaunchKernelGGL((cos_fused_kernel<256, kR>), grid, block, lds, st, A.prm, tsrc, A.groups, A.live_count, A.pre, tpp, A.paired, A, t2, NoKargParams{}); break;
    }
    HIP_TRY(hipGetLastError());
    if (A.partials_only == 2) {
        hipLaunchKernelGGL(loss_partials_kernel, dim3((unsigned)A.P), dim3(64), 0, st,
                           (const double2*)A.part_sse, A.n_tiles, A.sse, A.n_bad);
        HIP_TRY(hipGetLastError());
    }
    return DH_OK;
}

// The generator batch path: every maturity group one tile of <= kSmallTile options, a large call
// (DESIGN.md 3.3): one persistent cos_gen_kernel launch for the whole request.
int launch_gen(dh_ctx* ctx, const PriceArgs& A0, hipStream_t st, int TB) {
    const int tpp = A0.paired ? 1 : A0.n_groups;
    const int max_nopt = A0.paired ? 1 : A0.opt_cap;
    int OP = 1;
    while (OP < max_nopt) OP *= 2;
    PriceArgs A = A0;
    A.p0 = 0;
    A.np = A0.P;
    A.partials_only = 0;
    const int64_t n_q = A.np * tpp;
    const int gi = TB == 16 ? 0 : (TB == 8 ? 1 : 2);
    const int64_t blocks = std::min<int64_t>((n_q + TB - 1) / TB, ctx->view.resident_gen[gi]);
    const size_t lds = (size_t)TB * A.N * sizeof(double2);
    if (blocks <= 0 || OP > kBlock / TB) return fail(DH_E_ARG, "generator kernel shape");
    switch (TB) {
        case 16: hipLaunchKernelGGL((cos_gen_kernel<16>), dim3((unsigned)blocks), dim3(kBlock), lds, st, A, OP); break;
        case 8: hipLaunchKernelGGL((cos_gen_kernel<8>), dim3((unsigned)blocks), dim3(kBlock), lds, st, A, OP); break;
        default: hipLaunchKernelGGL((cos_gen_kernel<4>), dim3((unsigned)blocks), dim3(kBlock), lds, st, A, OP); break;
    }
    HIP_TRY(hipGetLastError());
    return DH_OK;
}

// Table kernel then option kernel per chunk of param sets; the chunk keeps the table workspace
// within kTableBudget (L2/MALL-resident between the two launches).  Requests whose maturity
// groups are single tiles may instead run as one fused launch (ctx->path).
int launch_price(dh_ctx* ctx, const PriceArgs& A_in, hipStream_t st) {
    PriceArgs A0 = A_in;
    A0.tail = ctx->tail_cut ? kTailScale : -1.0;
    const int64_t tasks_per_p = A0.paired ? 1 : A0.n_tiles;
    if (A0.P * tasks_per_p == 0) return DH_OK;
    if (A0.exact) return launch_exact(ctx, A0, st);
    int rc = ensure_attrs(ctx);
    if (rc) return rc;
    const int N = A0.N;
    {
        const int max_nopt = A0.paired ? 1 : A0.opt_cap;
        const bool small_call = max_nopt <= kSmallTile && A0.P * tasks_per_p >= kSmallMinTasks;
        const bool fusable = (A0.paired || A0.max_group <= kTileMax) &&
                             fused_lds_bytes(N, A0.opt_cap) <= (size_t)kLdsDyn;
        // auto: fused wherever it applies except small tiles in large calls (generator grids,
        // whose lane-per-option-group kernel is 1.7x faster); measured on the current kernels:
        // C3 113 vs 133 us, C4 393 vs 407 us per request
        const bool fused = fusable && (ctx->path == DH_PATH_FUSED ||
                                       (ctx->path == DH_PATH_AUTO && !small_call));
        ctx->last_path = fused ? DH_PATH_FUSED : DH_PATH_SPLIT;
        if (fused) return launch_fused(ctx, A0, st);
        // generator grids: one fused small-tile launch (PATH_SPLIT keeps the table + option
        // kernels, for A/B)
        const int tb = gen_tb(N);
        if (small_call && ctx->path == DH_PATH_AUTO && tb &&
            (A0.paired || A0.n_tiles == A0.n_groups)) {
            ctx->last_path = DH_PATH_GEN;
            return launch_gen(ctx, A0, st, tb);
        }
    }
    const int tpp = A0.paired ? 1 : A0.n_groups;
    const int words = cl_words(A0);
    const size_t per_p =
        (size_t)tpp * ((size_t)N + kConsts + words + (size_t)A0.max_group) * sizeof(double);
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(A0.P, kTableBudget / per_p));
    // rounded up to whole kTabTile-table tiles (the small-tile kernel's layout)
    HIP_TRY(ctx->table.reserve((size_t)((chunk * tpp + kTabTile - 1) / kTabTile) * kTabTile * N *
                               sizeof(double)));
    HIP_TRY(ctx->consts.reserve((size_t)chunk * tpp * kConsts * sizeof(double)));
    HIP_TRY(ctx->cl_mask.reserve((size_t)chunk * tpp * words * 8));
    HIP_TRY(ctx->cl_price.reserve((size_t)chunk * tpp * A0.max_group * sizeof(double)));
    // Few tables per resident slot (< 2, e.g. C3's 4,200 tables on 3,072 one-wave slots): one
    // block per kTabs tables, not persistent, so the dispatcher backfills CUs as blocks finish
    // instead of fixing each block's share up front (a 5-vs-6-table tail cost C3 ~30% of the
    // table kernel).  Otherwise a resident grid of persistent blocks and the slot width of
    // table_tpt.
    const int64_t nq_max = std::min<int64_t>(A0.P, chunk) * tpp;
    const bool backfill = nq_max < 2 * (int64_t)ctx->view.resident[0] * (kBlock / 64);
    const int t1 = backfill ? 64 : table_tpt(ctx->view, nq_max, N);
    const size_t lds1 = t1 == 64 ? 0 : (size_t)(kBlock / t1) * N * sizeof(double);
    const int max_nopt = A0.paired ? 1 : A0.opt_cap;
    // small tiles in a large call take the lane-per-option-group kernel (decided once per call,
    // so every chunk of it runs the same arithmetic)
    const bool small = max_nopt <= kSmallTile && A0.P * tasks_per_p >= kSmallMinTasks;
    const int rs = small_rs(max_nopt);
    int L = 1;
    while (L * rs < max_nopt) L *= 2;
    const int t2 = small ? kBlock : option_tpt(max_nopt, N, A0.opt_cap);
    const size_t lds2 =
        small ? 0 : ((size_t)(kBlock / t2) * option_lds_doubles(N, A0.opt_cap) +
                     (t2 == kBlock ? kRedDoubles : 0)) * sizeof(double);
    if (lds2 > (size_t)kLdsDyn) return fail(DH_E_ARG, "COS table does not fit in LDS");
    if (ctx->stamps_on) {
        const int64_t nb = std::max((chunk * tasks_per_p + kBlock / t2 - 1) / (kBlock / t2),
                                    (chunk * tpp + kBlock / t1 - 1) / (kBlock / t1));
        HIP_TRY(ctx->stamps.reserve((size_t)nb * kStamps * 8));
        HIP_TRY(hipMemsetAsync(ctx->stamps.ptr, 0, (size_t)nb * kStamps * 8, st));
        ctx->stamps_n = nb * kStamps;
    }
    for (int64_t p0 = 0; p0 < A0.P; p0 += chunk) {
        PriceArgs A = A0;
        A.partials_only = 0;        // the split kernels always finish the loss hand-off
        A.p0 = p0;
        A.np = std::min<int64_t>(chunk, A0.P - p0);
        A.table = (double*)ctx->table.ptr;
        A.table_tiled = small ? 1 : 0;
        A.consts = (double*)ctx->consts.ptr;
        A.cl_mask = (unsigned long long*)ctx->cl_mask.ptr;
        A.cl_price = (double*)ctx->cl_price.ptr;
        A.stamps = ctx->stamps_on ? (unsigned long long*)ctx->stamps.ptr : nullptr;
        const int64_t n_q = A.np * tpp;
        const int res = ctx->view.resident[t1 == 64 ? 0 : (t1 == 128 ? 1 : 2)];
        const int64_t b1 = backfill ? (n_q + kBlock / t1 - 1) / (kBlock / t1)
                                    : std::min<int64_t>((n_q + kBlock / t1 - 1) / (kBlock / t1), res);
        const int64_t n_t = A.np * tasks_per_p;
        const int64_t b2 = small ? (n_t * L + kBlock - 1) / kBlock
                                 : (n_t + kBlock / t2 - 1) / (kBlock / t2);
        if (b1 > 0x7fffffffLL || b2 > 0x7fffffffLL) return fail(DH_E_ARG, "launch too large");
        switch (t1) {
            case 64: hipLaunchKernelGGL(cos_table_kernel<64>, dim3((unsigned)b1), dim3(kBlock), 0, st, A); break;
            case 128: hipLaunchKernelGGL(cos_table_kernel<128>, dim3((unsigned)b1), dim3(kBlock), lds1, st, A); break;
            default: hipLaunchKernelGGL(cos_table_kernel<256>, dim3((unsigned)b1), dim3(kBlock), lds1, st, A); break;
        }
        HIP_TRY(hipGetLastError());
        if (small) {
            if (rs == 8)
                hipLaunchKernelGGL((cos_option_small_kernel<8>), dim3((unsigned)b2), dim3(kBlock), 0, st, A, L);
            else
                hipLaunchKernelGGL((cos_option_small_kernel<4>), dim3((unsigned)b2), dim3(kBlock), 0, st, A, L);
        } else {
            const dim3 g2((unsigned)b2), bk(kBlock);
            switch (t2 * (tile_r(max_nopt, t2) == 1 ? 1 : -1)) {
                case 64: hipLaunchKernelGGL((cos_option_kernel<64, 1>), g2, bk, lds2, st, A); break;
                case 128: hipLaunchKernelGGL((cos_option_kernel<128, 1>), g2, bk, lds2, st, A); break;
                case 256: hipLaunchKernelGGL((cos_option_kernel<256, 1>), g2, bk, lds2, st, A); break;
                case -64: hipLaunchKernelGGL((cos_option_kernel<64, kR>), g2, bk, lds2, st, A); break;
                case -128: hipLaunchKernelGGL((cos_option_kernel<128, kR>), g2, bk, lds2, st, A); break;
                default: hipLaunchKernelGGL((cos_option_kernel<256, kR>), g2, bk, lds2, st, A); break;
            }
        }
        HIP_TRY(hipGetLastError());
    }
    return DH_OK;
}

}  // namespace

extern "C" {

int dh_version(void) { return 1; }

const char* dh_last_error(void) { return g_err.c_str(); }

int dh_device_count(int* count) {
    if (!count) return fail(DH_E_ARG, "count is null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(DH_E_NODEV, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *count = n;
    return DH_OK;
}

int dh_ctx_create(int device, dh_ctx** out) {
    if (!out) return fail(DH_E_ARG, "out is null");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(DH_E_NODEV, std::string("no HIP device: ") + hipGetErrorString(e));
    if (device < 0 || device >= n) return fail(DH_E_ARG, "device index out of range");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(DH_E_NODEV, std::string("libdhcos is built for gfx950, device is ") +
                                    prop.gcnArchName);
    dh_ctx* c = new (std::nothrow) dh_ctx();
    if (!c) return fail(DH_E_ALLOC, "ctx alloc");
    c->device = device;
    DeviceScope dev_scope(device);
    if (dev_scope.rc) {
        delete c;
        return dev_scope.rc;
    }
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(DH_E_HIP, std::string("stream create: ") + hipGetErrorString(e));
    }
    *out = c;
    return DH_OK;
}

int dh_ctx_destroy(dh_ctx* ctx) {
    if (!ctx) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (DevBuf* b : {&ctx->params, &ctx->out, &ctx->sse, &ctx->bad, &ctx->part_sse,
                      &ctx->part_bad, &ctx->counter, &ctx->exact_prices, &ctx->stamps, &ctx->table,
                      &ctx->consts, &ctx->cl_mask, &ctx->cl_price, &ctx->aux0,
                      &ctx->aux1, &ctx->aux2, &ctx->aux3, &ctx->pre, &ctx->lb_state, &ctx->lb_rec,
                      &ctx->lb_sse, &ctx->lb_bad, &ctx->lb_live, &ctx->lb_done, &ctx->lb_x0,
                      &ctx->lb_trace, &ctx->lb_trace_n})
        b->release();
    ctx->h_params.release();
    ctx->h_loss.release();
    ctx->h_lb.release();
    ctx->h_pairs.release();
    for (hipEvent_t e : ctx->lb_ev)
        if (e) (void)hipEventDestroy(e);
    gen_bufs_release(ctx);
    for (auto& F : ctx->fg) {
        F.h_params.release();
        F.h_loss.release();
        if (F.done) (void)hipEventDestroy(F.done);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return DH_OK;
}

int dh_ctx_synchronize(dh_ctx* ctx) {
    if (!ctx) return fail(DH_E_ARG, "ctx is null");
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return DH_OK;
}

void* dh_ctx_stream(dh_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int dh_ctx_debug_stamps(dh_ctx* ctx, int on) {
    if (!ctx) return fail(DH_E_ARG, "ctx is null");
#ifdef DH_STAMPS
    ctx->stamps_on = on ? 1 : 0;
    return DH_OK;
#else
    (void)on;
    return fail(DH_E_ARG, "library built without DH_STAMPS (use `make stamps`)");
#endif
}

int dh_ctx_read_stamps(dh_ctx* ctx, unsigned long long* out, int64_t cap, int64_t* n) {
    if (!ctx || !n) return fail(DH_E_ARG, "null argument");
    *n = ctx->stamps_n;
    if (!out || ctx->stamps_n == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, ctx->stamps.ptr, (size_t)std::min<int64_t>(cap, ctx->stamps_n) * 8,
                      hipMemcpyDeviceToHost));
    return DH_OK;
}

int dh_ctx_set_path(dh_ctx* ctx, int path) {
    if (!ctx) return fail(DH_E_ARG, "ctx is null");
    if (path != DH_PATH_AUTO && path != DH_PATH_SPLIT && path != DH_PATH_FUSED)
        return fail(DH_E_ARG, "bad path");
    ctx->path = path;
    return DH_OK;
}

int dh_ctx_last_path(dh_ctx* ctx) { return ctx ? ctx->last_path : DH_E_ARG; }

int dh_ctx_set_exact(dh_ctx* ctx, int on) {
    if (!ctx) return fail(DH_E_ARG, "ctx is null");
    ctx->exact = on ? 1 : 0;
    return DH_OK;
}

int dh_ctx_set_tail_cut(dh_ctx* ctx, int on) {
    if (!ctx) return fail(DH_E_ARG, "ctx is null");
    ctx->tail_cut = on ? 1 : 0;
    return DH_OK;
}

int dh_surface_create(dh_ctx* ctx, const double* K, const double* T, const int8_t* is_call,
                      const double* mkt, int M, int strike_mode, dh_surface** out) {
    if (!ctx || !out) return fail(DH_E_ARG, "ctx/out is null");
    *out = nullptr;
    if (M < 0) return fail(DH_E_ARG, "M < 0");
    if (M > 0 && (!K || !T || !is_call)) return fail(DH_E_ARG, "K/T/is_call is null");
    if (strike_mode != DH_STRIKE_ABSOLUTE && strike_mode != DH_STRIKE_PCT_SPOT)
        return fail(DH_E_ARG, "bad strike_mode");
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    // group by exact maturity (stable), cut groups into tiles of <= kTileMax options
    std::vector<int> perm(M);
    std::iota(perm.begin(), perm.end(), 0);
    std::stable_sort(perm.begin(), perm.end(), [&](int i, int j) { return T[i] < T[j]; });
    std::vector<double> sK(M), sT(M), sm(M, 0.0);
    std::vector<int8_t> sc(M);
    for (int i = 0; i < M; ++i) {
        sK[i] = K[perm[i]];
        sT[i] = T[perm[i]];
        sc[i] = is_call[perm[i]] ? 1 : 0;
        if (mkt) sm[i] = mkt[perm[i]];
    }
    std::vector<int2> tiles;
    std::vector<int> tile_group;
    std::vector<double> group_T;
    std::vector<int2> groups;
    int max_nopt = 0, max_group = 0;
    for (int i = 0; i < M;) {
        int j = i;
        while (j < M && sT[j] == sT[i]) ++j;
        groups.push_back(make_int2(i, j - i));
        max_group = std::max(max_group, j - i);
        for (int s = i; s < j; s += kTileMax) {
            tiles.push_back(make_int2(s, std::min(kTileMax, j - s)));
            tile_group.push_back((int)group_T.size());
            max_nopt = std::max(max_nopt, std::min(kTileMax, j - s));
        }
        group_T.push_back(sT[i]);
        i = j;
    }
    dh_surface* s = new (std::nothrow) dh_surface();
    if (!s) return fail(DH_E_ALLOC, "surface alloc");
    s->ctx = ctx;
    s->M = M;
    s->n_tiles = (int)tiles.size();
    s->n_groups = (int)group_T.size();
    s->max_nopt = max_nopt;
    s->max_group = max_group;
    s->strike_mode = strike_mode;
    s->has_mkt = mkt != nullptr;
    s->h_group_T = group_T;
    s->h_groups = groups;
    // every array in one device allocation, staged on the host and uploaded by one copy (one
    // hipMalloc and one synchronous copy instead of nine of each: ~0.5 ms of a C3 calibration)
    struct Part {
        void** dst;
        const void* src;
        size_t bytes;
    };
    const size_t m = (size_t)M;
    const Part parts[] = {{(void**)&s->K, sK.data(), m * 8},
                          {(void**)&s->T, sT.data(), m * 8},
                          {(void**)&s->mkt, sm.data(), m * 8},
                          {(void**)&s->call, sc.data(), m},
                          {(void**)&s->perm, perm.data(), m * 4},
                          {(void**)&s->tiles, tiles.data(), tiles.size() * sizeof(int2)},
                          {(void**)&s->tile_group, tile_group.data(), tile_group.size() * sizeof(int)},
                          {(void**)&s->group_T, group_T.data(), group_T.size() * sizeof(double)},
                          {(void**)&s->groups, groups.data(), groups.size() * sizeof(int2)}};
    size_t off[9], total = 0;
    for (int i = 0; i < 9; ++i) {          // 256-byte aligned, >= 16 bytes each (empty surfaces)
        off[i] = total;
        total += (std::max<size_t>(parts[i].bytes, 16) + 255) & ~(size_t)255;
    }
    hipError_t e = hipMalloc(&s->block, total);
    if (e == hipSuccess) {
        for (int i = 0; i < 9; ++i) *parts[i].dst = (char*)s->block + off[i];
        if (M > 0) {
            std::vector<char> stage(total, 0);
            for (int i = 0; i < 9; ++i)
                if (parts[i].bytes) std::memcpy(stage.data() + off[i], parts[i].src, parts[i].bytes);
            e = hipMemcpy(s->block, stage.data(), total, hipMemcpyHostToDevice);
        }
    }
    if (e != hipSuccess) {
        dh_surface_destroy(s);
        return fail(DH_E_HIP, std::string("surface upload: ") + hipGetErrorString(e));
    }
    *out = s;
    return DH_OK;
}

int dh_surface_destroy(dh_surface* s) {
    if (!s) return DH_OK;
    DeviceScope dev_scope(s->ctx ? s->ctx->device : 0);
    if (s->block) (void)hipFree(s->block);
    delete s;
    return DH_OK;
}

int dh_surface_size(const dh_surface* s, int* M, int* n_tiles) {
    if (!s) return fail(DH_E_ARG, "surface is null");
    if (M) *M = s->M;
    if (n_tiles) *n_tiles = s->n_tiles;
    return DH_OK;
}

static PriceArgs surface_args(const dh_surface* s, const double* d_params, int64_t P, int N,
                              double L) {
    PriceArgs A{};
    A.prm = d_params;
    A.P = P;
    A.K = s->K;
    A.T = s->T;
    A.call = s->call;
    A.mkt = s->mkt;
    A.perm = s->perm;
    A.tiles = s->tiles;
    A.tile_group = s->tile_group;
    A.group_T = s->group_T;
    A.groups = s->groups;
    A.max_group = s->max_group;
    A.n_tiles = s->n_tiles;
    A.n_groups = s->n_groups;
    A.opt_cap = ((s->max_nopt + 1) / 2) * 2;
    A.M = s->M;
    A.paired = 0;
    A.strike_mode = s->strike_mode;
    A.N = N;
    A.L = L;
    A.out_stride = s->M;
    return A;
}

int dh_surface_price_dev(dh_ctx* ctx, const dh_surface* s, const double* d_params, int64_t P,
                         int N, double L, double* d_out, void* stream) {
    if (!ctx || !s || (P > 0 && (!d_params || !d_out))) return fail(DH_E_ARG, "null argument");
    int rc = check_N(N);
    if (rc) return rc;
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    if (P == 0 || s->M == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    PriceArgs A = surface_args(s, d_params, P, N, L);
    A.exact = per_term(ctx, N);
    A.out = d_out;
    return launch_price(ctx, A, stream ? (hipStream_t)stream : ctx->stream);
}

}  // extern "C"

static int surface_loss_launch(dh_ctx* ctx, const dh_surface* s, const double* d_params, int S,
                               int N, double L, double* d_sse, int32_t* d_n_bad,
                               double* d_prices, void* stream, const int* live_count,
                               bool partials_only = false) {
    if (!ctx || !s || (S > 0 && (!d_params || !d_sse || !d_n_bad)))
        return fail(DH_E_ARG, "null argument");
    if (!s->has_mkt) return fail(DH_E_ARG, "surface has no market prices");
    int rc = check_N(N);
    if (rc) return rc;
    if (S < 0) return fail(DH_E_ARG, "S < 0");
    if (S == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    if (s->M == 0) {
        HIP_TRY(hipMemsetAsync(d_sse, 0, (size_t)S * 8, st));
        HIP_TRY(hipMemsetAsync(d_n_bad, 0, (size_t)S * 4, st));
        return DH_OK;
    }
    const size_t nparts = (size_t)S * s->n_tiles;
    HIP_TRY(ctx->part_sse.reserve(nparts * 8));
    HIP_TRY(ctx->part_bad.reserve(nparts * 4));
    const size_t cap0 = ctx->counter.cap;
    HIP_TRY(ctx->counter.reserve((size_t)S * kCounterStride * 4));
    if (ctx->counter.cap != cap0) {       // fresh counters start at zero; kernels self-reset
        HIP_TRY(hipMemsetAsync(ctx->counter.ptr, 0, ctx->counter.cap, st));
    }
    PriceArgs A = surface_args(s, d_params, S, N, L);
    A.exact = per_term(ctx, N);
    A.out = d_prices;
    A.part_sse = (double*)ctx->part_sse.ptr;
    A.part_bad = (int*)ctx->part_bad.ptr;
    A.counter = (unsigned*)ctx->counter.ptr;
    A.sse = d_sse;
    A.n_bad = (int*)d_n_bad;
    A.live_count = live_count;
    A.partials_only = partials_only && !A.exact ? 1 : 0;
    A.host_out = ctx->kp_src != nullptr;     // the host API's zero-copy requests (kp_src set)
    return launch_price(ctx, A, st);
}

extern "C" {

int dh_surface_loss_dev(dh_ctx* ctx, const dh_surface* s, const double* d_params, int S, int N,
                        double L, double* d_sse, int32_t* d_n_bad, double* d_prices,
                        void* stream) {
    return surface_loss_launch(ctx, s, d_params, S, N, L, d_sse, d_n_bad, d_prices, stream,
                               nullptr);
}

int dh_surface_price(dh_ctx* ctx, const dh_surface* s, const double* params, int64_t P, int N,
                     double L, double* out) {
    if (!ctx || !s || (P > 0 && (!params || !out))) return fail(DH_E_ARG, "null argument");
    int rc = check_N(N);
    if (rc) return rc;
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    if (P == 0 || s->M == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t pb = (size_t)P * DH_PARAM_STRIDE * 8, ob = (size_t)P * s->M * 8;
    HIP_TRY(ctx->params.reserve(pb));
    HIP_TRY(ctx->out.reserve(ob));
    HIP_TRY(hipMemcpyAsync(ctx->params.ptr, params, pb, hipMemcpyHostToDevice, ctx->stream));
    rc = dh_surface_price_dev(ctx, s, (const double*)ctx->params.ptr, P, N, L,
                              (double*)ctx->out.ptr, ctx->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, ctx->out.ptr, ob, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return DH_OK;
}

int dh_surface_price_cols(dh_ctx* ctx, const dh_surface* s, const double* params,
                          const double* spots, double r, int64_t P, int N, double L, double* out) {
    if (!ctx || !s || (P > 0 && (!params || !spots || !out))) return fail(DH_E_ARG, "null argument");
    int rc = check_N(N);
    if (rc) return rc;
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    if (P == 0 || s->M == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    hipStream_t st = ctx->stream;
    const size_t ob = (size_t)P * s->M * 8;
    HIP_TRY(ctx->params.reserve((size_t)P * DH_PARAM_STRIDE * 8));
    HIP_TRY(ctx->aux0.reserve((size_t)P * 13 * 8));
    HIP_TRY(ctx->aux1.reserve((size_t)P * 8));
    HIP_TRY(ctx->out.reserve(ob));
    HIP_TRY(hipMemcpyAsync(ctx->aux0.ptr, params, (size_t)P * 13 * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux1.ptr, spots, (size_t)P * 8, hipMemcpyHostToDevice, st));
    const int64_t n_el = P * DH_PARAM_STRIDE;
    const int64_t nb = (n_el + 255) / 256;
    if (nb > 0x7fffffffLL) return fail(DH_E_ARG, "launch too large");
    hipLaunchKernelGGL(gen_records_kernel, dim3((unsigned)nb), dim3(256), 0, st,
                       (const double*)ctx->aux0.ptr, (const double*)ctx->aux1.ptr, r, P,
                       (double*)ctx->params.ptr);
    HIP_TRY(hipGetLastError());
    rc = dh_surface_price_dev(ctx, s, (const double*)ctx->params.ptr, P, N, L,
                              (double*)ctx->out.ptr, st);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, ctx->out.ptr, ob, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

// A failed (un)registration is reported here and nowhere else: HIP's per-thread last error is
// read back (cleared), so the next call's hipGetLastError check after a launch does not report it
// (a caller that leaves an array pageable after a failed registration, _native.pinned, goes on)
int dh_host_register(void* ptr, size_t bytes) {
    if (!ptr || !bytes) return fail(DH_E_ARG, "null or empty range");
    const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(DH_E_HIP, std::string("hipHostRegister: ") + hipGetErrorString(e));
    }
    return DH_OK;
}

int dh_host_unregister(void* ptr) {
    if (!ptr) return fail(DH_E_ARG, "null argument");
    const hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(DH_E_HIP, std::string("hipHostUnregister: ") + hipGetErrorString(e));
    }
    return DH_OK;
}

int dh_surface_loss(dh_ctx* ctx, const dh_surface* s, const double* params, int S, int N,
                    double L, double* sse, int32_t* n_bad, double* prices) {
    if (!ctx || !s || (S > 0 && (!params || !sse || !n_bad))) return fail(DH_E_ARG, "null argument");
    int rc = check_N(N);
    if (rc) return rc;
    if (S < 0) return fail(DH_E_ARG, "S < 0");
    if (S == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t pb = (size_t)S * DH_PARAM_STRIDE * 8;
    double* d_prices = nullptr;
    const size_t ob = (size_t)S * s->M * 8;
    if (prices) {
        HIP_TRY(ctx->out.reserve(ob));
        d_prices = (double*)ctx->out.ptr;
    }
    if (S <= kZeroCopyMaxSets) {
        // calibration-sized request: the kernels read the params and write sse / n_bad through
        // pinned, mapped host memory -- one launch and one sync, no staging copies
        HIP_TRY(ctx->h_params.reserve(pb));
        HIP_TRY(ctx->h_loss.reserve((size_t)S * 12));
        std::memcpy(ctx->h_params.ptr, params, pb);
        double* h_sse = (double*)ctx->h_loss.ptr;
        int32_t* h_bad = (int32_t*)(h_sse + S);
        ctx->kp_src = (const double*)ctx->h_params.ptr;     // <= 14 records: in the arguments
        ctx->kp_surf = s;
        ctx->kp_n = S;
        rc = dh_surface_loss_dev(ctx, s, (const double*)ctx->h_params.dptr, S, N, L,
                                 (double*)ctx->h_loss.dptr, (int32_t*)((double*)ctx->h_loss.dptr + S),
                                 d_prices, ctx->stream);
        ctx->kp_src = nullptr;
        ctx->kp_surf = nullptr;
        ctx->kp_n = 0;
        if (rc) return rc;
        if (prices && s->M > 0)
            HIP_TRY(hipMemcpyAsync(prices, d_prices, ob, hipMemcpyDeviceToHost, ctx->stream));
        rc = spin_sync(ctx->stream);
        if (rc) return rc;
        std::memcpy(sse, h_sse, (size_t)S * 8);
        std::memcpy(n_bad, h_bad, (size_t)S * 4);
        return check_loss_counts(n_bad, S);
    }
    HIP_TRY(ctx->params.reserve(pb));
    HIP_TRY(ctx->sse.reserve((size_t)S * 8));
    HIP_TRY(ctx->bad.reserve((size_t)S * 4));
    HIP_TRY(hipMemcpyAsync(ctx->params.ptr, params, pb, hipMemcpyHostToDevice, ctx->stream));
    rc = dh_surface_loss_dev(ctx, s, (const double*)ctx->params.ptr, S, N, L,
                             (double*)ctx->sse.ptr, (int32_t*)ctx->bad.ptr, d_prices, ctx->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(sse, ctx->sse.ptr, (size_t)S * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(n_bad, ctx->bad.ptr, (size_t)S * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (prices && s->M > 0)
        HIP_TRY(hipMemcpyAsync(prices, d_prices, ob, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return check_loss_counts(n_bad, S);
}

int dh_price_pairs(dh_ctx* ctx, const double* params, const double* K, const double* T,
                   const int8_t* is_call, int64_t P, int N, double L, double* out) {
    if (!ctx || (P > 0 && (!params || !K || !T || !is_call || !out)))
        return fail(DH_E_ARG, "null argument");
    int rc = check_N(N);
    if (rc) return rc;
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    if (P == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t pb = (size_t)P * DH_PARAM_STRIDE * 8, vb = (size_t)P * 8;
    hipStream_t st = ctx->stream;
    PriceArgs A{};
    A.P = P;
    double* d_out = nullptr;
    const bool zc = P <= kZeroCopyMaxSets;
    if (zc) {
        // single options and small batches (DoubleHeston.pricing() calls): the kernel reads the
        // inputs and writes the prices through pinned, mapped host memory -- one launch and one
        // spin-wait instead of five staging copies, a read-back and a stream sync
        const size_t need = pb + 3 * vb + (size_t)P * 4 + (size_t)P;
        HIP_TRY(ctx->h_pairs.reserve(need));
        char* h = (char*)ctx->h_pairs.ptr;
        char* d = (char*)ctx->h_pairs.dptr;
        std::memcpy(h, params, pb);
        std::memcpy(h + pb, K, vb);
        std::memcpy(h + pb + vb, T, vb);
        int* perm = (int*)(h + pb + 3 * vb);
        for (int64_t i = 0; i < P; ++i) perm[i] = (int)i;
        std::memcpy(h + pb + 3 * vb + (size_t)P * 4, is_call, (size_t)P);
        A.prm = (const double*)d;
        A.K = (const double*)(d + pb);
        A.T = (const double*)(d + pb + vb);
        d_out = (double*)(d + pb + 2 * vb);
        A.perm = (const int*)(d + pb + 3 * vb);
        A.call = (const int8_t*)(d + pb + 3 * vb + (size_t)P * 4);
    } else {
        HIP_TRY(ctx->params.reserve(pb));
        HIP_TRY(ctx->out.reserve(vb));
        HIP_TRY(ctx->aux0.reserve(vb));
        HIP_TRY(ctx->aux1.reserve(vb));
        HIP_TRY(ctx->aux2.reserve((size_t)P));
        HIP_TRY(ctx->aux3.reserve((size_t)P * 4));
        std::vector<int> ident((size_t)P);
        std::iota(ident.begin(), ident.end(), 0);
        HIP_TRY(hipMemcpyAsync(ctx->params.ptr, params, pb, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(ctx->aux0.ptr, K, vb, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(ctx->aux1.ptr, T, vb, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(ctx->aux2.ptr, is_call, (size_t)P, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(ctx->aux3.ptr, ident.data(), (size_t)P * 4, hipMemcpyHostToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));        // `ident` is pageable and leaves scope
        A.prm = (const double*)ctx->params.ptr;
        A.K = (const double*)ctx->aux0.ptr;
        A.T = (const double*)ctx->aux1.ptr;
        A.call = (const int8_t*)ctx->aux2.ptr;
        A.perm = (const int*)ctx->aux3.ptr;
        d_out = (double*)ctx->out.ptr;
    }
    A.paired = 1;
    A.opt_cap = 2;
    A.max_group = 1;
    A.M = (int)P;
    A.exact = per_term(ctx, N);
    A.strike_mode = DH_STRIKE_ABSOLUTE;
    A.N = N;
    A.L = L;
    A.out = d_out;
    A.out_stride = 0;
    rc = launch_price(ctx, A, st);
    if (rc) return rc;
    if (zc) {
        rc = spin_sync(st);
        if (rc) return rc;
        std::memcpy(out, (char*)ctx->h_pairs.ptr + pb + 2 * vb, vb);
        return DH_OK;
    }
    HIP_TRY(hipMemcpyAsync(out, ctx->out.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

int dh_cf(dh_ctx* ctx, const double* params, const double* u, int n, double tau, double* re,
          double* im) {
    if (!ctx || !params || (n > 0 && (!u || !re || !im))) return fail(DH_E_ARG, "null argument");
    if (n < 0) return fail(DH_E_ARG, "n < 0");
    if (n == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t vb = (size_t)n * 8;
    HIP_TRY(ctx->params.reserve(DH_PARAM_STRIDE * 8));
    HIP_TRY(ctx->aux0.reserve(vb));
    HIP_TRY(ctx->aux1.reserve(vb));
    HIP_TRY(ctx->aux2.reserve(vb));
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->params.ptr, params, DH_PARAM_STRIDE * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux0.ptr, u, vb, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(cf_kernel, dim3((n + 255) / 256), dim3(256), 0, st,
                       (const double*)ctx->params.ptr, (const double*)ctx->aux0.ptr, n, tau,
                       (double*)ctx->aux1.ptr, (double*)ctx->aux2.ptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(re, ctx->aux1.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(im, ctx->aux2.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

int dh_cf_complex(dh_ctx* ctx, const double* params, const double* u_re, const double* u_im,
                  int n, double tau, double* re, double* im) {
    if (!ctx || !params || (n > 0 && (!u_re || !u_im || !re || !im)))
        return fail(DH_E_ARG, "null argument");
    if (n < 0) return fail(DH_E_ARG, "n < 0");
    if (n == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t vb = (size_t)n * 8;
    HIP_TRY(ctx->params.reserve(DH_PARAM_STRIDE * 8));
    HIP_TRY(ctx->aux0.reserve(vb));
    HIP_TRY(ctx->aux1.reserve(vb));
    HIP_TRY(ctx->aux2.reserve(vb));
    HIP_TRY(ctx->aux3.reserve(vb));
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->params.ptr, params, DH_PARAM_STRIDE * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux0.ptr, u_re, vb, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux1.ptr, u_im, vb, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(cf_kernel_z, dim3((n + 255) / 256), dim3(256), 0, st,
                       (const double*)ctx->params.ptr, (const double*)ctx->aux0.ptr,
                       (const double*)ctx->aux1.ptr, n, tau, (double*)ctx->aux2.ptr,
                       (double*)ctx->aux3.ptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(re, ctx->aux2.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(im, ctx->aux3.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

int dh_trunc_range(dh_ctx* ctx, const double* params, const double* K, const double* T,
                   int64_t P, double L, double* a, double* b) {
    if (!ctx || (P > 0 && (!params || !K || !T || !a || !b))) return fail(DH_E_ARG, "null argument");
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    if (P == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t pb = (size_t)P * DH_PARAM_STRIDE * 8, vb = (size_t)P * 8;
    HIP_TRY(ctx->params.reserve(pb));
    HIP_TRY(ctx->aux0.reserve(vb));
    HIP_TRY(ctx->aux1.reserve(vb));
    HIP_TRY(ctx->aux2.reserve(vb));
    HIP_TRY(ctx->aux3.reserve(vb));
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->params.ptr, params, pb, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux0.ptr, K, vb, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux1.ptr, T, vb, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(trunc_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st,
                       (const double*)ctx->params.ptr, (const double*)ctx->aux0.ptr,
                       (const double*)ctx->aux1.ptr, P, L, (double*)ctx->aux2.ptr,
                       (double*)ctx->aux3.ptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(a, ctx->aux2.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(b, ctx->aux3.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

int dh_cos_coeffs(dh_ctx* ctx, const int32_t* k, int n, double c, double d, double a, double b,
                  double* chi, double* psi) {
    if (!ctx || (n > 0 && (!k || !chi || !psi))) return fail(DH_E_ARG, "null argument");
    if (n < 0) return fail(DH_E_ARG, "n < 0");
    if (n == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t vb = (size_t)n * 8;
    HIP_TRY(ctx->aux0.reserve((size_t)n * 4));
    HIP_TRY(ctx->aux1.reserve(vb));
    HIP_TRY(ctx->aux2.reserve(vb));
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->aux0.ptr, k, (size_t)n * 4, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(coeff_kernel, dim3((n + 255) / 256), dim3(256), 0, st,
                       (const int32_t*)ctx->aux0.ptr, n, c, d, a, b, (double*)ctx->aux1.ptr,
                       (double*)ctx->aux2.ptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(chi, ctx->aux1.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(psi, ctx->aux2.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

}  // extern "C"

// ----------------------------------------------------------------------------------------------
// device-resident multi-start L-BFGS-B (dh_calibrate_lbfgs)
// ----------------------------------------------------------------------------------------------
// Nothing below is contracted into FMAs: the step kernel must compute the bits of the CPU build
// of dh_lbfgs.h (tests/native/lb_host.cpp).
#pragma clang fp contract(off)

namespace {

constexpr double kInvalidLoss = 1e10;                 // lbfgs_calibrator.py:152-158,176-177
constexpr double kFdStep = 1e-8;                      // SciPy L-BFGS-B eps
constexpr double kSqrtEps = 1.4901161193847656e-08;   // sqrt(DBL_EPSILON), _numdiff fallback

// A 13-vector held one component per lane of each 16-lane row (lane l holds component l & 15;
// components 13..15 are 0): the four rows are copies, so every lane computes the same scalars
// and the state machine's branches are uniform across the wave.  Reductions are DPP
// butterflies inside each 16-lane row -- quad_perm [1,0,3,2], quad_perm [2,3,0,1],
// row_half_mirror, row_mirror -- in which both partners add the same two operands, so every lane
// of the row ends with the same bits: the pairwise tree ((p0+p1)+(p2+p3)) + ... that
// tests/native/lb_host.cpp reproduces.
struct WaveVec {
    double v;
};
__device__ __forceinline__ WaveVec operator+(WaveVec a, WaveVec b) { return {a.v + b.v}; }
__device__ __forceinline__ WaveVec operator-(WaveVec a, WaveVec b) { return {a.v - b.v}; }
__device__ __forceinline__ WaveVec operator-(WaveVec a) { return {-a.v}; }
__device__ __forceinline__ WaveVec operator*(double s, WaveVec a) { return {s * a.v}; }


__device__ __forceinline__ double row_sum(double p) {
    p = p + dpp_f64<kDppXor1>(p);
    p = p + dpp_f64<kDppXor2>(p);
    p = p + dpp_f64<kDppHalfMirror>(p);
    return p + dpp_f64<kDppMirror>(p);
}
__device__ __forceinline__ double row_max(double m) {
    m = fmax(m, dpp_f64<kDppXor1>(m));
    m = fmax(m, dpp_f64<kDppXor2>(m));
    m = fmax(m, dpp_f64<kDppHalfMirror>(m));
    return fmax(m, dpp_f64<kDppMirror>(m));
}
__device__ __forceinline__ double row_min(double m) {
    m = fmin(m, dpp_f64<kDppXor1>(m));
    m = fmin(m, dpp_f64<kDppXor2>(m));
    m = fmin(m, dpp_f64<kDppHalfMirror>(m));
    return fmin(m, dpp_f64<kDppMirror>(m));
}
__device__ __forceinline__ double dot(WaveVec a, WaveVec b) { return row_sum(a.v * b.v); }
// max |a_i|; a NaN component makes it NaN (SciPy's projected-gradient norm: any NaN gradient
// component fails the pgtol test)
__device__ __forceinline__ double amax(WaveVec a) {
    const double m = fmax(0.0, row_max(fabs(a.v)));
    return __any(a.v != a.v) ? __builtin_nan("") : m;
}
__device__ __forceinline__ bool equal(WaveVec a, WaveVec b) { return __all(a.v == b.v); }

// The pair memory in LDS: s_j, y_j as 16-double rows (lane i reads column i), rho_j and the
// two-loop's alpha_j.  Every lane computes the same scalars, so the scalar writes are uniform.
struct WaveRing {
    double* rs;                // [kM][16]
    double* ry;                // [kM][16]
    double* rdr;               // [kM] rho_j = 1 / dr_j
    double* ra;                // [kM]
    int lane;
    __device__ WaveVec s(int j) const { return {rs[j * dhlb::kLanes + (lane & 15)]}; }
    __device__ WaveVec y(int j) const { return {ry[j * dhlb::kLanes + (lane & 15)]}; }
    __device__ double rho(int j) const { return rdr[j]; }
    __device__ double& a(int j) { return ra[j]; }
    __device__ void put(int j, WaveVec sj, WaveVec yj, double d) {
        if (lane < dhlb::kLanes) {
            rs[j * dhlb::kLanes + lane] = sj.v;
            ry[j * dhlb::kLanes + lane] = yj.v;
        }
        rdr[j] = d;
    }
    __device__ void shift() {
        for (int j = 0; j + 1 < dhlb::kM; ++j) {
            if (lane < dhlb::kLanes) {
                rs[j * dhlb::kLanes + lane] = rs[(j + 1) * dhlb::kLanes + lane];
                ry[j * dhlb::kLanes + lane] = ry[(j + 1) * dhlb::kLanes + lane];
            }
            rdr[j] = rdr[j + 1];
        }
    }
};

using WaveCore = dhlb::LbCore<WaveVec, WaveRing>;

// diagnostic trace record of one consumed request: start, request number, f, x[13], g[13], 3 spare,
// then (DH_STAMPS build only) s_memtime at the step kernel's phase boundaries: start, state
// loaded, request consumed, state machine done, request emitted, end
constexpr int kLbTrace = 40;
[[maybe_unused]] constexpr int kLbStamp0 = 32;

__device__ __forceinline__ unsigned long long lb_clock() {
#ifdef DH_STAMPS
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
#else
    return 0;
#endif
}

// Global state of one start: the vectors as 16-double rows (lane i holds column i), the pair
// memory (staged in LDS by the step kernel), then the scalars.
constexpr int kLbVecs = 10;                           // x g z d t r xe ge dx pen
constexpr int kLbRing = 2 * dhlb::kM * dhlb::kLanes + dhlb::kM;   // s rows, y rows, rho
struct LbSlot {
    double vec[kLbVecs][dhlb::kLanes];
    double ring[kLbRing];
    dhlb::LbScalars s;
};

constexpr int kLbInline = 64;   // live lists up to this size travel in the kernel arguments

struct LbArgs {
    LbSlot* states;            // [S]
    const int* live;           // [n_live] start index of each slot
    const double* x0;          // [S][13] (mode 0)
    const double* sse;         // [n_live * 14] loss partial sums of the last request, slot-major
    const int* bad;            // [n_live * 14]
    double* rec;               // [n_live * 14][16] param records of the next request
    int* done;                 // [S] finished flags (pinned host memory, read between chunks)
    int* live_count;           // starts not finished yet (the loss launches halt at 0)
    double* trace;             // diagnostic: [trace_cap][kLbTrace] consumed requests, or null
    unsigned long long* trace_n;
    int64_t trace_cap;
    dhlb::LbConfig cfg;
    double S0, r;
    int M;
    int mode;                  // 0 begin at x0, 1 consume the request and advance, 2 re-emit
    int part_mode;             // 1: the request ran fused with partials_only -- sum its tile
                               // partials here (the hand-off's order); 0: read sse / bad
    const double* part_sse;    // [n_live * 14][n_tiles] (part_mode 1; sign bit: invalid price)
    int n_tiles;
    int n_inline;              // live list passed by value below (saves a dependent load), or 0
    int live_inline[kLbInline];
};
static_assert(std::is_standard_layout<LbArgs>::value, "lb_live_inline reads LbArgs by offset");

// The step kernel's leading arguments (LbHead), ahead of LbArgs: plain scalars, preloaded into
// SGPRs at wave launch (Makefile PRELOAD), so the state and partial loads of the load phase issue
// at once instead of behind a kernel-argument load.  With at most kLbPre live starts their slots'
// start indices travel here as well (lb_step_kernel<true>).
constexpr int kLbPre = 4;
// byte offset of LbArgs in the kernel-argument segment: the leading arguments in declaration order
// at their natural alignment (2 pointers, 3 + kLbPre ints = 44 bytes), then LbArgs 8-aligned
constexpr int kLbArgsKernargOff = 48;
struct LbKargs {            // lb_step_kernel's argument list as a struct (its kernarg layout)
    void* states;
    const double* part;
    int ntiles, mode, part_mode, l[kLbPre];
    LbArgs A;
};
static_assert(offsetof(LbKargs, A) == kLbArgsKernargOff, "LbArgs kernarg offset");
// karg_prefetch_lines reads up to byte 0x1b4: inside the explicit arguments and the 256 bytes of
// implicit ones every HIP kernel's segment carries after them
static_assert(sizeof(LbKargs) + 256 >= 0x1b4, "kernel-argument prefetch past the segment");
static_assert(sizeof(FusedKargs) + 256 >= 0x1b4, "kernel-argument prefetch past the segment");

// live_inline[slot] as a scalar load straight from the kernel-argument segment; indexing the
// by-value argument compiled to a flat load
__device__ __forceinline__ int lb_live_inline(int slot) {
    typedef const __attribute__((address_space(4))) char* KargPtr;
    const KargPtr k = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
    return ((const __attribute__((address_space(4))) int*)(k + kLbArgsKernargOff +
                                                            offsetof(LbArgs, live_inline)))
        [slot < kLbInline ? slot : 0];
}

__device__ __forceinline__ WaveVec lb_ld(const LbSlot* g, int v, int lane) {
    return {g->vec[v][lane & 15]};
}

__device__ __forceinline__ void lb_st(LbSlot* g, int v, int lane, WaveVec x) {
    if (lane < dhlb::kLanes) g->vec[v][lane] = x.v;
}

// model parameter i from unconstrained x_i (lbfgs_calibrator.py:62-87): tanh for the two
// correlations, identity for mu_j, exp otherwise
__device__ __forceinline__ double lb_transform(int i, double x) {
    if (i == 4 || i == 9) return tanh(x);
    if (i == 11) return x;
    return exp(x);
}

// Emit the pending request at xe.  Lanes i and 16 + i (i < 13) form x_i + h_i (SciPy's step rule,
// scipy/optimize/_numdiff.py:498-511); lane i maps x_i and lane 16 + i maps x_i + h_i to a model
// param (one transform per lane), lane i keeps dx_i = (x_i + h_i) - x_i; lane t < 14 assembles
// point t (x, or x + h_{t-1} e_{t-1}), writes its record and keeps its Feller penalty
// (lbfgs_calibrator.py:113-116) in pen.
__device__ void lb_emit(const WaveCore& c, WaveVec& dx, WaveVec& pen, double* pb, double* pp,
                        const LbArgs& A, int slot, int lane) {
    const int i = lane & 15;
    const double xi = c.xe.v;                       // every row holds xe
    double h = kFdStep;
    if ((xi + h) - xi == 0.0) h = kSqrtEps * (xi >= 0.0 ? 1.0 : -1.0) * fmax(1.0, fabs(xi));
    const double xh = xi + h;
    dx.v = i < dhlb::kN ? xh - xi : 0.0;
    if (lane < 32 && i < dhlb::kN) {
        const double v = lb_transform(i, lane < 16 ? xi : xh);
        if (lane < 16) pb[i] = v;
        else pp[i] = v;
    }
    __syncthreads();
    pen.v = 0.0;
    if (lane < dhlb::kPts) {
        double p[dhlb::kN];
#pragma unroll
        for (int i = 0; i < dhlb::kN; ++i) p[i] = (i == lane - 1) ? pp[i] : pb[i];
        const double v1 = p[3] * p[3] - 2.0 * p[1] * p[2];
        const double v2 = p[8] * p[8] - 2.0 * p[6] * p[7];
        pen.v = 1000.0 * ((v1 > 0.0 ? v1 : 0.0) + (v2 > 0.0 ? v2 : 0.0));
        double* out = A.rec + ((size_t)slot * dhlb::kPts + lane) * DH_PARAM_STRIDE;
#pragma unroll
        for (int i = 0; i < dhlb::kN; ++i) out[i] = p[i];
        out[13] = A.S0;
        out[14] = A.r;
        out[15] = 0.0;
    }
}

// The loss hand-off's sum of one param set's nt tile partials (task_loss: lane l adds tiles l,
// l + 64, ... in order, then an xor butterfly), formed by one lane: leaf l as that lane's sum,
// then the butterfly's tree (level w adds leaves w apart).  Leaves past nt are +0.0 and adding
// +0.0 to a partial (a sum of squares) changes no bit, so W = 16 or 32 leaves give the 64-leaf
// tree's bits.  Loads are clamped in-bounds and issued before any add.  A tile with an invalid
// price stored its partial with the sign bit set (task_loss), so the magnitudes give the sum --
// a NaN sum (a NaN or infinite market price) stays the NaN loss the reference gives -- and any
// sign bit gives 1e10 whatever the sum.
template <int W>
__device__ __forceinline__ void lb_tile_tree(const double* ps, int nt, double& sse, int& bad) {
    double x[W];
    unsigned hi = 0;        // OR of the high words: loads past nt repeat tile nt - 1 (clamped), so
                            // the OR over all of them is the OR of the first nt sign bits (a
                            // short-circuit || compiled to an exec-mask branch per tile)
#pragma unroll
    for (int u = 0; u < W; ++u) {
        const double v = ps[min(u, nt - 1)];
        x[u] = 0.0 + (u < nt ? fabs(v) : 0.0);
        hi |= (unsigned)__double2hiint(v);
    }
    for (int j0 = W; j0 < nt; j0 += W) {          // W = 64 only
#pragma unroll
        for (int u = 0; u < W; ++u) {
            const double v = ps[min(j0 + u, nt - 1)];
            x[u] += j0 + u < nt ? fabs(v) : 0.0;
            hi |= (unsigned)__double2hiint(v);
        }
    }
#pragma unroll
    for (int w = 1; w < W; w <<= 1) {
#pragma unroll
        for (int u = 0; u < W; u += 2 * w) x[u] = x[u] + x[u + w];
    }
    sse = x[0];
    bad = (int)(hi >> 31);
}

// One wave per live start: load the state (vectors into registers, lane i = component i; the
// pair memory into LDS), consume the finished request (lane t forms loss t, lane i gradient
// component i), run the L-BFGS-B state machine until it needs a new point, emit that request,
// store the state.
template <bool kPre>
__global__ __launch_bounds__(64) void lb_step_kernel(
    LbSlot* __restrict__ h_states, const double* __restrict__ h_part, int h_ntiles, int h_mode,
    int h_part_mode, int h_l0, int h_l1, int h_l2, int h_l3, LbArgs A_) {
    const LbArgs& A = karg_ref<LbArgs, kLbArgsKernargOff>();   // read in place (karg_ref)
    karg_prefetch_lines();                             // LbArgs spans the same lines
    __shared__ double ring[kLbRing + dhlb::kM];
    __shared__ double fl[dhlb::kLanes];
    __shared__ double pb[dhlb::kLanes], pp[dhlb::kLanes];
    [[maybe_unused]] const unsigned long long t_start = lb_clock();
    const int slot = blockIdx.x;
    const int lane = threadIdx.x;
    int sidx;
    if constexpr (kPre)                                // slot < kLbPre (the host's choice)
        sidx = slot == 0 ? h_l0 : (slot == 1 ? h_l1 : (slot == 2 ? h_l2 : h_l3));
    else
        sidx = A.n_inline ? lb_live_inline(slot) : A.live[slot];
    LbSlot* G = h_states + sidx;
    WaveCore c;
    [[maybe_unused]] unsigned long long t_load = 0, t_req = 0, t_sm = 0;
    c.pairs = WaveRing{ring, ring + dhlb::kM * dhlb::kLanes, ring + 2 * dhlb::kM * dhlb::kLanes,
                       ring + kLbRing, lane};
    WaveVec dx, pen;
    double req_sse = 0.0;
    int req_bad = 0;
    if (h_mode == 0) {
        c.s = dhlb::LbScalars{};
        const WaveVec z{0.0};
        c.x = c.g = c.z = c.d = c.t = c.r = c.ge = z;
        for (int i = lane; i < kLbRing + dhlb::kM; i += 64) ring[i] = 0.0;
        const int li = lane & 15;
        const WaveVec x0{li < dhlb::kN ? A.x0[(size_t)sidx * dhlb::kN + li] : 0.0};
        dhlb::lb_begin(c, x0);
        c.s.best_loss = __builtin_huge_val();
        c.s.n_calls = 0;
    } else {
        // every load is issued before any is used (one memory round trip): the finished request's
        // loss terms, the pair memory, the vectors and the scalars
        if (h_mode == 1 && h_part_mode) {
            // the loss hand-off's sum (task_loss), formed by lane t of every row for point t
            // (lb_tile_tree: the same additions, so the same bits).  Measured alternatives, all
            // slower: staging the request's contiguous partials through LDS with coalesced loads
            // (C2 step load phase 4.4k -> 5.5k cycles); issuing these loads together with the
            // state's (5.6k)
            const int li = lane & 15;
            if (li < dhlb::kPts) {
                const int nt = h_ntiles;
                const double* ps = h_part + ((size_t)slot * dhlb::kPts + li) * nt;
                if (nt <= 16) lb_tile_tree<16>(ps, nt, req_sse, req_bad);
                else if (nt <= 32) lb_tile_tree<32>(ps, nt, req_sse, req_bad);
                else lb_tile_tree<64>(ps, nt, req_sse, req_bad);
            }
        } else if (h_mode == 1 && (lane & 15) < dhlb::kPts) {
            const size_t i = (size_t)slot * dhlb::kPts + (lane & 15);
            req_sse = A.sse[i];
            req_bad = A.bad[i];
        }
        double rg[(kLbRing + 63) / 64];
#pragma unroll
        for (int j = 0; j < (kLbRing + 63) / 64; ++j) {
            const int i = lane + 64 * j;
            rg[j] = i < kLbRing ? G->ring[i] : 0.0;
        }
        c.s = G->s;
#pragma unroll
        for (int j = 0; j < (kLbRing + 63) / 64; ++j) {
            const int i = lane + 64 * j;
            if (i < kLbRing) ring[i] = rg[j];
        }
        c.x = lb_ld(G, 0, lane);
        c.g = lb_ld(G, 1, lane);
        c.z = lb_ld(G, 2, lane);
        c.d = lb_ld(G, 3, lane);
        c.t = lb_ld(G, 4, lane);
        c.r = lb_ld(G, 5, lane);
        c.xe = lb_ld(G, 6, lane);
        c.ge = lb_ld(G, 7, lane);
        dx = lb_ld(G, 8, lane);
        pen = lb_ld(G, 9, lane);
        if (c.s.done) return;                          // uniform across the wave
    }
    int need = 1;
    double* tr = nullptr;                              // this request's trace record, if any
    if (h_mode == 1) {
        t_load = lb_clock();
        double f = __builtin_huge_val();
        if ((lane & 15) < dhlb::kPts) f = req_bad > 0 ? kInvalidLoss : req_sse / (double)A.M + pen.v;
        if (lane < dhlb::kLanes) fl[lane] = f;
        __syncthreads();
        const double lo = row_min((f == f && f != kInvalidLoss) ? f : __builtin_huge_val());
        c.s.n_calls += dhlb::kPts;
        if (lo < c.s.best_loss) c.s.best_loss = lo;
        c.s.fe = fl[0];
        c.ge.v = (lane & 15) < dhlb::kN ? (fl[(lane & 15) + 1] - fl[0]) / dx.v : 0.0;
        if (A.trace) {
            unsigned long long k = 0;
            if (lane == 0) k = atomicAdd(A.trace_n, 1ull);
            k = __shfl(k, 0, 64);
            if ((int64_t)k < A.trace_cap) {
                tr = A.trace + k * kLbTrace;
                if (lane == 0) {
                    tr[0] = sidx;
                    tr[1] = c.s.n_calls / dhlb::kPts - 1;
                    tr[2] = c.s.fe;
                }
                if (lane < dhlb::kN) {
                    tr[3 + lane] = c.xe.v;
                    tr[3 + dhlb::kN + lane] = c.ge.v;
                }
            }
        }
    }
    __syncthreads();
    if (h_mode == 1) {
        t_req = lb_clock();
        need = dhlb::lb_resume(c, A.cfg);
        t_sm = lb_clock();
        if (!need && lane == 0) {
            __hip_atomic_store(&A.done[sidx], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            atomicSub(A.live_count, 1);
        }
    }
    if (need) lb_emit(c, dx, pen, pb, pp, A, slot, lane);
    __syncthreads();
    [[maybe_unused]] const unsigned long long t_emit = lb_clock();
    {   // every LDS read before the first store (one LDS round trip, not one per store)
        double rg[(kLbRing + 63) / 64];
#pragma unroll
        for (int j = 0; j < (kLbRing + 63) / 64; ++j) rg[j] = ring[min(lane + 64 * j, kLbRing - 1)];
#pragma unroll
        for (int j = 0; j < (kLbRing + 63) / 64; ++j)
            if (lane + 64 * j < kLbRing) G->ring[lane + 64 * j] = rg[j];
    }
    lb_st(G, 0, lane, c.x);
    lb_st(G, 1, lane, c.g);
    lb_st(G, 2, lane, c.z);
    lb_st(G, 3, lane, c.d);
    lb_st(G, 4, lane, c.t);
    lb_st(G, 5, lane, c.r);
    lb_st(G, 6, lane, c.xe);
    lb_st(G, 7, lane, c.ge);
    lb_st(G, 8, lane, dx);
    lb_st(G, 9, lane, pen);
    if (lane == 0) G->s = c.s;
#ifdef DH_STAMPS
    if (tr && lane == 0) {
        const unsigned long long t_end = lb_clock();
        const unsigned long long ts[6] = {t_start, t_load, t_req, t_sm, t_emit, t_end};
        for (int i = 0; i < 6; ++i) tr[kLbStamp0 + i] = (double)ts[i];
    }
#endif
}

int launch_lb_step(hipStream_t st, const LbArgs& A, int n_live) {
    if (A.n_inline && n_live <= kLbPre) {
        int l[kLbPre] = {0, 0, 0, 0};
        for (int i = 0; i < n_live; ++i) l[i] = A.live_inline[i];
        hipLaunchKernelGGL(lb_step_kernel<true>, dim3((unsigned)n_live), dim3(64), 0, st, A.states,
                           A.part_sse, A.n_tiles, A.mode, A.part_mode, l[0], l[1], l[2], l[3], A);
    } else {
        hipLaunchKernelGGL(lb_step_kernel<false>, dim3((unsigned)n_live), dim3(64), 0, st,
                           A.states, A.part_sse, A.n_tiles, A.mode, A.part_mode, 0, 0, 0, 0, A);
    }
    HIP_TRY(hipGetLastError());
    return DH_OK;
}

}  // namespace

extern "C" int dh_calibrate_lbfgs(dh_ctx* ctx, const dh_surface* s, const double* x0, int S,
                                  double S0, double r, int N, double L, const dh_lb_options* opt,
                                  dh_lb_result* out, int32_t* n_launches) {
    if (!ctx || !s || !opt || (S > 0 && (!x0 || !out))) return fail(DH_E_ARG, "null argument");
    if (!s->has_mkt) return fail(DH_E_ARG, "surface has no market prices");
    if (s->M == 0) return fail(DH_E_ARG, "empty market (the loss is NaN; no optimisation)");
    int rc = check_N(N);
    if (rc) return rc;
    if (S < 0) return fail(DH_E_ARG, "S < 0");
    if (opt->maxiter < 0 || opt->maxfun < 0 || opt->maxls < 1)   // SciPy: maxls must be > 0
        return fail(DH_E_ARG, "maxiter and maxfun must be >= 0, maxls >= 1");
    if (n_launches) *n_launches = 0;
    if (S == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t st = ctx->stream;
    const size_t npts = (size_t)S * dhlb::kPts;
    HIP_TRY(ctx->lb_state.reserve((size_t)S * sizeof(LbSlot)));
    HIP_TRY(ctx->lb_rec.reserve(npts * DH_PARAM_STRIDE * 8));
    HIP_TRY(ctx->lb_sse.reserve(npts * 8));
    HIP_TRY(ctx->lb_bad.reserve(npts * 4));
    HIP_TRY(ctx->lb_live.reserve((size_t)S * 4));
    HIP_TRY(ctx->lb_done.reserve(4));                  // live-start count (halts launches at 0)
    HIP_TRY(ctx->lb_x0.reserve((size_t)S * dhlb::kN * 8));
    // pinned, device-mapped: finished flags (written by the step kernel) | 2 live-list buffers
    HIP_TRY(ctx->h_lb.reserve((size_t)S * 3 * 4));
    int* h_done = (int*)ctx->h_lb.ptr;
    int* h_live[2] = {h_done + S, h_done + 2 * S};
    std::memset(h_done, 0, (size_t)S * 4);
    std::vector<int> live(S);
    for (int i = 0; i < S; ++i) live[i] = h_live[0][i] = i;
    HIP_TRY(hipMemcpyAsync(ctx->lb_x0.ptr, x0, (size_t)S * dhlb::kN * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->lb_live.ptr, h_live[0], (size_t)S * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)ctx->lb_done.ptr, S, 1, st));
    if (!ctx->lb_ev[0]) {
        for (hipEvent_t& e : ctx->lb_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }

    LbArgs A;
    A.states = (LbSlot*)ctx->lb_state.ptr;
    A.live = (const int*)ctx->lb_live.ptr;
    A.x0 = (const double*)ctx->lb_x0.ptr;
    A.sse = (const double*)ctx->lb_sse.ptr;
    A.bad = (const int*)ctx->lb_bad.ptr;
    A.rec = (double*)ctx->lb_rec.ptr;
    A.done = (int*)ctx->h_lb.dptr;
    A.live_count = (int*)ctx->lb_done.ptr;
    A.trace = nullptr;
    A.trace_n = nullptr;
    A.trace_cap = 0;
    if (ctx->lb_trace_cap > 0) {
        HIP_TRY(ctx->lb_trace.reserve((size_t)ctx->lb_trace_cap * kLbTrace * 8));
        HIP_TRY(ctx->lb_trace_n.reserve(8));
        HIP_TRY(hipMemsetAsync(ctx->lb_trace_n.ptr, 0, 8, st));
        A.trace = (double*)ctx->lb_trace.ptr;
        A.trace_n = (unsigned long long*)ctx->lb_trace_n.ptr;
        A.trace_cap = ctx->lb_trace_cap;
    }
    A.cfg.maxiter = opt->maxiter;
    A.cfg.maxfun = opt->maxfun;
    A.cfg.maxls = opt->maxls;
    A.cfg.pad = 0;
    A.cfg.factr_epsmch = (opt->ftol / dhlb::kEpsMch) * dhlb::kEpsMch;   // factr * epsmch
    A.cfg.pgtol = opt->gtol;
    A.S0 = S0;
    A.r = r;
    A.M = s->M;
    A.mode = 0;
    A.part_mode = 0;
    A.part_sse = nullptr;
    A.n_tiles = s->n_tiles;
    auto set_inline = [&](const int* lst, int n) {
        A.n_inline = n <= kLbInline ? 1 : 0;
        for (int i = 0; i < kLbInline; ++i) A.live_inline[i] = i < n && A.n_inline ? lst[i] : 0;
    };
    set_inline(h_live[0], S);
    rc = launch_lb_step(st, A, S);
    if (rc) return rc;

    // Chunks of `chunk` iterations (loss launch(es) + step launch) are enqueued two ahead of the
    // host: while the GPU runs chunk k + 1, the host reads the finished flags as of the end of
    // chunk k, compacts the live starts (their requests are re-emitted at the new slots, in
    // stream order after chunk k + 1) and enqueues chunk k + 2.  Launches enqueued after the
    // last start finished return at once (live count 0).
    struct DrainOnError {      // an early error return leaves no launch writing our buffers
        hipStream_t st;
        bool armed = true;
        ~DrainOnError() {
            if (armed) (void)hipStreamSynchronize(st);
        }
    } drain{st};
    const int chunk = opt->chunk > 0 ? opt->chunk : 8;
    const int64_t max_iters = (int64_t)opt->maxfun + 2LL * opt->maxls + 8;   // nfev bound per start
    std::vector<double> t_done(S, 0.0);
    int n_live = S;
    int64_t iters = 0, launches = 0;
    auto enqueue_chunk = [&](int k) -> int {
        A.mode = 1;
        for (int c = 0; c < chunk; ++c) {
            int e = surface_loss_launch(ctx, s, A.rec, n_live * dhlb::kPts, N, L, (double*)A.sse,
                                        (int32_t*)A.bad, nullptr, st, A.live_count, true);
            if (e) return e;
            // a fused request stored its tile partials only (no hand-off): the step sums them
            A.part_mode = !per_term(ctx, N) && ctx->last_path == DH_PATH_FUSED ? 1 : 0;
            A.part_sse = (const double*)ctx->part_sse.ptr;
            e = launch_lb_step(st, A, n_live);
            if (e) return e;
            ++launches;
        }
        iters += chunk;
        HIP_TRY(hipEventRecord(ctx->lb_ev[k & 1], st));
        return DH_OK;
    };
    rc = enqueue_chunk(0);
    if (rc) return rc;
    rc = enqueue_chunk(1);
    if (rc) return rc;
    for (int k = 0;; ++k) {
        for (;;) {                                     // spin: a chunk is ~0.1-1 ms
            const hipError_t e = hipEventQuery(ctx->lb_ev[k & 1]);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady)
                return fail(DH_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(e));
        }
        const double now =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::vector<int> next;
        next.reserve(live.size());
        for (int sidx : live) {
            if (__atomic_load_n(&h_done[sidx], __ATOMIC_ACQUIRE)) {
                if (t_done[sidx] == 0.0) t_done[sidx] = now;
            } else {
                next.push_back(sidx);
            }
        }
        if (next.empty()) break;
        if (iters > max_iters) {
            (void)hipStreamSynchronize(st);
            return fail(DH_E_ARG, "L-BFGS-B starts did not terminate");
        }
        if (next.size() != live.size()) {              // compact; re-emit their requests
            live.swap(next);
            n_live = (int)live.size();
            set_inline(live.data(), n_live);
            if (!A.n_inline) {
                int* hl = h_live[(k + 1) & 1];         // the other buffer's upload has run
                std::memcpy(hl, live.data(), (size_t)n_live * 4);
                HIP_TRY(hipMemcpyAsync(ctx->lb_live.ptr, hl, (size_t)n_live * 4,
                                       hipMemcpyHostToDevice, st));
            }
            A.mode = 2;
            rc = launch_lb_step(st, A, n_live);
            if (rc) return rc;
        }
        rc = enqueue_chunk(k + 2);
        if (rc) return rc;
    }
    std::vector<LbSlot> hs(S);
    HIP_TRY(hipMemcpyAsync(hs.data(), ctx->lb_state.ptr, (size_t)S * sizeof(LbSlot),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    drain.armed = false;
    for (int i = 0; i < S; ++i) {
        const LbSlot& q = hs[i];
        dh_lb_result& o = out[i];
        for (int j = 0; j < dhlb::kN; ++j) o.x[j] = q.vec[0][j];   // row 0 = x
        o.fun = q.s.fe;
        o.best_loss = q.s.best_loss;
        o.t_done = t_done[i];
        o.nit = q.s.nit;
        o.nfev = q.s.nfev;
        o.task = q.s.task;
        o.warnflag = q.s.warnflag;
        o.n_calls = q.s.n_calls;
        o.pad = 0;
    }
    if (n_launches) *n_launches = (int32_t)launches;
    return DH_OK;
}

extern "C" int dh_ctx_set_lb_trace(dh_ctx* ctx, int64_t cap) {
    if (!ctx) return fail(DH_E_ARG, "null argument");
    if (cap < 0) return fail(DH_E_ARG, "cap < 0");
    ctx->lb_trace_cap = cap;
    return DH_OK;
}

extern "C" int dh_ctx_read_lb_trace(dh_ctx* ctx, double* out, int64_t cap, int64_t* n) {
    if (!ctx || !n || (cap > 0 && !out)) return fail(DH_E_ARG, "null argument");
    *n = 0;
    if (ctx->lb_trace_cap == 0 || !ctx->lb_trace_n.ptr) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    unsigned long long cnt = 0;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipMemcpy(&cnt, ctx->lb_trace_n.ptr, 8, hipMemcpyDeviceToHost));
    const int64_t m = std::min<int64_t>({(int64_t)cnt, ctx->lb_trace_cap, cap});
    if (m > 0) HIP_TRY(hipMemcpy(out, ctx->lb_trace.ptr, (size_t)m * kLbTrace * 8, hipMemcpyDeviceToHost));
    *n = (int64_t)cnt;
    return DH_OK;
}

// ----------------------------------------------------------------------------------------------
// one-shot entry points in the shape SURVEY.md 8(b) proposes (a surface per call)
// ----------------------------------------------------------------------------------------------
namespace {

// unconstrained x [S][13] -> param records (exp / tanh / identity, lbfgs_calibrator.py:62-87)
// and Feller penalties (:113-116); one thread per set, the expressions of lb_emit
__global__ void x_records_kernel(const double* __restrict__ x, int S, double S0, double r,
                                 double* __restrict__ rec, double* __restrict__ pen) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    double p[dhlb::kN];
#pragma unroll
    for (int i = 0; i < dhlb::kN; ++i) p[i] = lb_transform(i, x[(size_t)s * dhlb::kN + i]);
    const double v1 = p[3] * p[3] - 2.0 * p[1] * p[2];
    const double v2 = p[8] * p[8] - 2.0 * p[6] * p[7];
    pen[s] = 1000.0 * ((v1 > 0.0 ? v1 : 0.0) + (v2 > 0.0 ? v2 : 0.0));
    double* out = rec + (size_t)s * DH_PARAM_STRIDE;
#pragma unroll
    for (int i = 0; i < dhlb::kN; ++i) out[i] = p[i];
    out[13] = S0;
    out[14] = r;
    out[15] = 0.0;
}

// loss = n_bad ? 1e10 : sse / M + penalty (lbfgs_calibrator.py:152-166)
__global__ void loss_finalize_kernel(const double* __restrict__ sse, const int* __restrict__ bad,
                                     const double* __restrict__ pen, int S, int M,
                                     double* __restrict__ loss) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    loss[s] = bad[s] > 0 ? kInvalidLoss : sse[s] / (double)M + pen[s];
}

}  // namespace

extern "C" int dh_price_batch(dh_ctx* ctx, const double* params, int64_t P, const double* K,
                              const double* T, const int8_t* is_call, int M, int N, double L,
                              double* out) {
    if (!ctx || (P > 0 && M > 0 && (!params || !out))) return fail(DH_E_ARG, "null argument");
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    dh_surface* s = nullptr;
    int rc = dh_surface_create(ctx, K, T, is_call, nullptr, M, DH_STRIKE_ABSOLUTE, &s);
    if (rc) return rc;
    rc = dh_surface_price(ctx, s, params, P, N, L, out);
    dh_surface_destroy(s);
    return rc;
}

extern "C" int dh_loss_batch(dh_ctx* ctx, const double* x, int S, const double* K, const double* T,
                             const int8_t* is_call, const double* mkt, int M, double S0, double r,
                             int N, double L, double* loss, int32_t* n_invalid) {
    if (!ctx || (S > 0 && (!x || !loss || !n_invalid))) return fail(DH_E_ARG, "null argument");
    if (S < 0) return fail(DH_E_ARG, "S < 0");
    if (M > 0 && !mkt) return fail(DH_E_ARG, "mkt is null");
    int rc = check_N(N);
    if (rc) return rc;
    if (S == 0) return DH_OK;
    if (M == 0) {                                   // np.mean([]) -> nan (lbfgs_calibrator.py:163)
        for (int i = 0; i < S; ++i) {
            loss[i] = __builtin_nan("");
            n_invalid[i] = 0;
        }
        return DH_OK;
    }
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    dh_surface* s = nullptr;
    rc = dh_surface_create(ctx, K, T, is_call, mkt, M, DH_STRIKE_ABSOLUTE, &s);
    if (rc) return rc;
    hipStream_t st = ctx->stream;
    const size_t xb = (size_t)S * dhlb::kN * 8;
    auto run = [&]() -> int {
        HIP_TRY(ctx->aux0.reserve(xb));
        HIP_TRY(ctx->aux1.reserve((size_t)S * DH_PARAM_STRIDE * 8));
        HIP_TRY(ctx->aux2.reserve((size_t)S * 8 * 3));     // pen | sse | loss
        HIP_TRY(ctx->aux3.reserve((size_t)S * 4));
        double* d_x = (double*)ctx->aux0.ptr;
        double* d_rec = (double*)ctx->aux1.ptr;
        double* d_pen = (double*)ctx->aux2.ptr;
        double* d_sse = d_pen + S;
        double* d_loss = d_sse + S;
        int* d_bad = (int*)ctx->aux3.ptr;
        HIP_TRY(hipMemcpyAsync(d_x, x, xb, hipMemcpyHostToDevice, st));
        const unsigned b = (unsigned)((S + 255) / 256);
        hipLaunchKernelGGL(x_records_kernel, dim3(b), dim3(256), 0, st, d_x, S, S0, r, d_rec, d_pen);
        HIP_TRY(hipGetLastError());
        int e = surface_loss_launch(ctx, s, d_rec, S, N, L, d_sse, (int32_t*)d_bad, nullptr, st,
                                    nullptr);
        if (e) return e;
        hipLaunchKernelGGL(loss_finalize_kernel, dim3(b), dim3(256), 0, st, d_sse, d_bad, d_pen, S,
                           s->M, d_loss);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(loss, d_loss, (size_t)S * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(n_invalid, d_bad, (size_t)S * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        return DH_OK;
    };
    rc = run();
    dh_surface_destroy(s);
    return rc;
}

// ----------------------------------------------------------------------------------------------
// function + FD-gradient requests for the host (SciPy) driver
// ----------------------------------------------------------------------------------------------
namespace {

// The request's points (scipy/optimize/_numdiff.py:498-511: x0, then x0 + h_i e_i with h = 1e-8,
// or sqrt(eps) sign(x) max(1, |x|) where the absolute step vanishes), their model params (exp /
// tanh / identity, lbfgs_calibrator.py:62-87) and Feller penalties (:113-116): rec [S * 14][16],
// pen [S * 14], dx [S][13].  The caller passes the model params of x0 and x0 + h (model:
// [2][S][13]) when they must be the bits of its own exp / tanh (NumPy's, as the reference's
// transform_params); otherwise they come from libm here.
void fg_points(const double* x0, const double* model, int S, double S0, double r, double* rec,
               double* pen, double* dx) {
    constexpr int kP = dhlb::kPts, kN = dhlb::kN;
    for (int st = 0; st < S; ++st) {
        const double* x = x0 + (size_t)st * kN;
        double pb[kN], pp[kN];
        for (int i = 0; i < kN; ++i) {
            double h = kFdStep;
            if ((x[i] + h) - x[i] == 0.0)
                h = kSqrtEps * (x[i] >= 0.0 ? 1.0 : -1.0) * std::max(1.0, std::fabs(x[i]));
            const double xh = x[i] + h;
            dx[(size_t)st * kN + i] = xh - x[i];
            if (model) {
                pb[i] = model[(size_t)st * kN + i];
                pp[i] = model[((size_t)S + st) * kN + i];
            } else {
                const bool th = i == 4 || i == 9, id = i == 11;
                pb[i] = th ? std::tanh(x[i]) : (id ? x[i] : std::exp(x[i]));
                pp[i] = th ? std::tanh(xh) : (id ? xh : std::exp(xh));
            }
        }
        for (int t = 0; t < kP; ++t) {
            double* o = rec + ((size_t)st * kP + t) * DH_PARAM_STRIDE;
            for (int i = 0; i < kN; ++i) o[i] = (i == t - 1) ? pp[i] : pb[i];
            const double v1 = o[3] * o[3] - 2.0 * o[1] * o[2];
            const double v2 = o[8] * o[8] - 2.0 * o[6] * o[7];
            pen[(size_t)st * kP + t] = 1000.0 * ((v1 > 0.0 ? v1 : 0.0) + (v2 > 0.0 ? v2 : 0.0));
            o[13] = S0;
            o[14] = r;
            o[15] = 0.0;
        }
    }
}

// loss = n_bad ? 1e10 : sse / M + Feller (lbfgs_calibrator.py:152-166); f, the FD gradient
// (f_i - f_0) / dx_i as SciPy forms it, and the smallest valid loss of the request
void fg_finish(int S, int M, const double* sse, const int32_t* bad, const double* pen,
               const double* dx, double* f, double* g, double* low) {
    constexpr int kP = dhlb::kPts, kN = dhlb::kN;
    for (int st = 0; st < S; ++st) {
        double lo = __builtin_huge_val(), fl[kP];
        for (int t = 0; t < kP; ++t) {
            const size_t i = (size_t)st * kP + t;
            fl[t] = bad[i] > 0 ? kInvalidLoss : sse[i] / (double)M + pen[i];
            if (fl[t] == fl[t] && fl[t] != kInvalidLoss && fl[t] < lo) lo = fl[t];
        }
        f[st] = fl[0];
        low[st] = lo;
        for (int i = 0; i < kN; ++i)
            g[(size_t)st * kN + i] = (fl[i + 1] - fl[0]) / dx[(size_t)st * kN + i];
    }
}

int fg_check(dh_ctx* ctx, const dh_surface* s, int S) {
    if (!s->has_mkt) return fail(DH_E_ARG, "surface has no market prices");
    if (s->M == 0) return fail(DH_E_ARG, "empty market (the loss is NaN)");
    if (S < 0) return fail(DH_E_ARG, "S < 0");
    (void)ctx;
    return DH_OK;
}

}  // namespace

extern "C" int dh_surface_fg(dh_ctx* ctx, const dh_surface* s, const double* x0,
                             const double* model, int S, double S0, double r, int N, double L,
                             double* f, double* g, double* low) {
    if (!ctx || !s || (S > 0 && (!x0 || !f || !g || !low))) return fail(DH_E_ARG, "null argument");
    int rc = fg_check(ctx, s, S);
    if (rc) return rc;
    if (S == 0) return DH_OK;
    const size_t P = (size_t)S * dhlb::kPts;
    std::vector<double> rec(P * DH_PARAM_STRIDE), pen(P), dx((size_t)S * dhlb::kN), sse(P);
    std::vector<int32_t> bad(P);
    fg_points(x0, model, S, S0, r, rec.data(), pen.data(), dx.data());
    rc = dh_surface_loss(ctx, s, rec.data(), (int)P, N, L, sse.data(), bad.data(), nullptr);
    if (rc) return rc;
    fg_finish(S, s->M, sse.data(), bad.data(), pen.data(), dx.data(), f, g, low);
    return DH_OK;
}

extern "C" int dh_surface_fg_begin(dh_ctx* ctx, const dh_surface* s, const double* x0,
                                   const double* model, int S, double S0, double r, int N,
                                   double L, int slot) {
    if (!ctx || !s || (S > 0 && !x0)) return fail(DH_E_ARG, "null argument");
    if (slot < 0 || slot >= DH_FG_SLOTS) return fail(DH_E_ARG, "slot out of range");
    int rc = fg_check(ctx, s, S);
    if (rc) return rc;
    rc = check_N(N);
    if (rc) return rc;
    if (s->ctx && s->ctx->device != ctx->device)
        return fail(DH_E_ARG, "surface and context are on different devices");
    auto& F = ctx->fg[slot];
    if (F.pending) return fail(DH_E_ARG, "slot has a request in flight (call dh_surface_fg_end)");
    const size_t P = (size_t)S * dhlb::kPts;
    if (P > (size_t)kZeroCopyMaxSets)
        return fail(DH_E_ARG, "too many starts for one asynchronous request (use dh_surface_fg)");
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    // The loss launch may grow the context's device scratch (partials, counters, the prologue
    // buffer, table / clamp workspaces), whose sizes follow from the surface, N and the param-set
    // count only.  A grow frees buffers the other slot's enqueued launch still reads.  hipFree
    // happens to synchronise the device first, but nothing here relies on that: wait for the
    // other slots (their requests share the stream) whenever this request is not covered by an
    // earlier one on the same surface and N (the pipelined SciPy driver's requests always are,
    // after its first round).
    const size_t units = P * (size_t)std::max(s->n_tiles, s->n_groups);
    const bool covered = s == ctx->fg_surf && N == ctx->fg_N && units <= ctx->fg_max_units;
    bool others = false;
    for (int o = 0; o < DH_FG_SLOTS; ++o) others = others || (o != slot && ctx->fg[o].pending);
    if (others && !covered) HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (s != ctx->fg_surf || N != ctx->fg_N) {
        ctx->fg_surf = s;
        ctx->fg_N = N;
        ctx->fg_max_units = 0;
    }
    ctx->fg_max_units = std::max(ctx->fg_max_units, units);
    HIP_TRY(F.h_params.reserve(P * DH_PARAM_STRIDE * 8));
    HIP_TRY(F.h_loss.reserve(P * 12));
    F.pen.resize(P);
    F.dx.resize((size_t)S * dhlb::kN);
    if (!F.done) HIP_TRY(hipEventCreateWithFlags(&F.done, hipEventDisableTiming));
    F.S = S;
    F.M = s->M;
    F.surf = s;
    if (S == 0) {
        HIP_TRY(hipEventRecord(F.done, ctx->stream));
        F.pending = true;
        return DH_OK;
    }
    fg_points(x0, model, S, S0, r, (double*)F.h_params.ptr, F.pen.data(), F.dx.data());
    // the records also travel in the fused launch's kernel arguments when they fit (KargParams)
    ctx->kp_src = (const double*)F.h_params.ptr;
    ctx->kp_surf = s;
    ctx->kp_n = (int64_t)P;
    ctx->kp_done = F.done;
    ctx->kp_done_set = false;
    rc = dh_surface_loss_dev(ctx, s, (const double*)F.h_params.dptr, (int)P, N, L,
                             (double*)F.h_loss.dptr, (int32_t*)((double*)F.h_loss.dptr + P),
                             nullptr, ctx->stream);
    ctx->kp_src = nullptr;
    ctx->kp_surf = nullptr;
    ctx->kp_n = 0;
    ctx->kp_done = nullptr;
    if (rc) return rc;
    if (!ctx->kp_done_set) HIP_TRY(hipEventRecord(F.done, ctx->stream));
    ctx->kp_done_set = false;
    F.pending = true;
    return DH_OK;
}

extern "C" int dh_surface_fg_end(dh_ctx* ctx, const dh_surface* s, int slot, int S, double* f,
                                 double* g, double* low) {
    if (!ctx || !s) return fail(DH_E_ARG, "null argument");
    if (slot < 0 || slot >= DH_FG_SLOTS) return fail(DH_E_ARG, "slot out of range");
    auto& F = ctx->fg[slot];
    if (!F.pending) return fail(DH_E_ARG, "no request in flight in this slot");
    // the slot belongs to the context: the caller must name the request it enqueued (its surface
    // and start count, which size f / g / low), else its buffers may be smaller than F.S rows
    if (s != F.surf) return fail(DH_E_ARG, "slot's request was enqueued on another surface");
    if (S != F.S)
        return fail(DH_E_ARG, "slot's request has " + std::to_string(F.S) + " starts, caller passed " +
                                  std::to_string(S));
    if (F.S > 0 && (!f || !g || !low)) return fail(DH_E_ARG, "null argument");
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t P = (size_t)F.S * dhlb::kPts;
    for (;;) {                          // busy-wait: an optimizer iteration waits on it
        const hipError_t e = hipEventQuery(F.done);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) {
            F.pending = false;
            return fail(DH_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(e));
        }
    }
    F.pending = false;
    const int32_t* nb = (const int32_t*)((double*)F.h_loss.ptr + P);
    const int crc = check_loss_counts(nb, (int64_t)P);
    if (crc) return crc;
    fg_finish(F.S, F.M, (const double*)F.h_loss.ptr, nb, F.pen.data(), F.dx.data(), f, g, low);
    return DH_OK;
}

extern "C" int dh_surface_fg_cancel(dh_ctx* ctx, int slot) {
    if (!ctx) return fail(DH_E_ARG, "null argument");
    if (slot < 0 || slot >= DH_FG_SLOTS) return fail(DH_E_ARG, "slot out of range");
    auto& F = ctx->fg[slot];
    if (!F.pending) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    F.pending = false;                  // cleared even if the wait fails: the slot is usable again
    HIP_TRY(hipEventSynchronize(F.done));
    return DH_OK;
}

// ----------------------------------------------------------------------------------------------
// multi-GPU: an RCCL communicator for callers without torch.distributed (SURVEY 8(b)'s
// dh_allgather_best, 8(e) multi-start sharding).  librccl.so.1 is resolved at run time: with
// torch imported that is torch's own copy (the same soname), otherwise ROCm's, so a process holds
// one RCCL either way and the library does not link it.
// ----------------------------------------------------------------------------------------------
namespace {

struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

const RcclApi& rccl() {
    static const RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            a.err = std::string("librccl not found: ") + (e ? e : "");
            return a;
        }
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn && a.err.empty()) a.err = std::string("librccl lacks ") + name;
        };
        sym(a.get_unique_id, "ncclGetUniqueId");
        sym(a.comm_init_rank, "ncclCommInitRank");
        sym(a.all_gather, "ncclAllGather");
        sym(a.broadcast, "ncclBroadcast");
        sym(a.comm_destroy, "ncclCommDestroy");
        sym(a.error_string, "ncclGetErrorString");
        a.ok = a.err.empty();
        return a;
    }();
    return api;
}

int nccl_fail(const char* what, ncclResult_t r) {
    return fail(DH_E_COMM, std::string(what) + ": " + rccl().error_string(r));
}

#define NCCL_TRY(expr)                                       \
    do {                                                     \
        const ncclResult_t _r = (expr);                      \
        if (_r != ncclSuccess) return nccl_fail(#expr, _r);  \
    } while (0)

}  // namespace

struct dh_comm {
    dh_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    int world = 0, rank = 0;
    DevBuf send, recv;
};

extern "C" int dh_comm_id(unsigned char* id) {
    if (!id) return fail(DH_E_ARG, "id is null");
    const RcclApi& R = rccl();
    if (!R.ok) return fail(DH_E_COMM, R.err);
    ncclUniqueId u;
    NCCL_TRY(R.get_unique_id(&u));
    static_assert(sizeof(u) == DH_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof(u));
    return DH_OK;
}

extern "C" int dh_comm_create(dh_ctx* ctx, const unsigned char* id, int world, int rank,
                              dh_comm** out) {
    if (!ctx || !id || !out) return fail(DH_E_ARG, "null argument");
    *out = nullptr;
    if (world < 1 || rank < 0 || rank >= world) return fail(DH_E_ARG, "rank / world out of range");
    const RcclApi& R = rccl();
    if (!R.ok) return fail(DH_E_COMM, R.err);
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    dh_comm* c = new (std::nothrow) dh_comm();
    if (!c) return fail(DH_E_ALLOC, "comm alloc");
    const ncclResult_t r = R.comm_init_rank(&c->comm, world, u, rank);   // joins every rank
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail("ncclCommInitRank", r);
    }
    c->ctx = ctx;
    c->world = world;
    c->rank = rank;
    *out = c;
    return DH_OK;
}

extern "C" int dh_comm_destroy(dh_comm* c) {
    if (!c) return DH_OK;
    int rc = DH_OK;
    {
        DeviceScope dev_scope(c->ctx->device);
        if (c->comm) {
            const ncclResult_t r = rccl().comm_destroy(c->comm);
            if (r != ncclSuccess) rc = nccl_fail("ncclCommDestroy", r);
        }
        c->send.release();
        c->recv.release();
    }
    delete c;
    return rc;
}

extern "C" int dh_comm_broadcast(dh_comm* c, double* buf, int64_t n, int root) {
    if (!c || (n > 0 && !buf)) return fail(DH_E_ARG, "null argument");
    if (root < 0 || root >= c->world) return fail(DH_E_ARG, "root out of range");
    if (n <= 0) return DH_OK;
    DeviceScope dev_scope(c->ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    const size_t bytes = (size_t)n * sizeof(double);
    hipStream_t st = c->ctx->stream;
    HIP_TRY(c->send.reserve(bytes));
    if (c->rank == root) HIP_TRY(hipMemcpyAsync(c->send.ptr, buf, bytes, hipMemcpyHostToDevice, st));
    NCCL_TRY(rccl().broadcast(c->send.ptr, c->send.ptr, (size_t)n, ncclFloat64, root, c->comm, st));
    HIP_TRY(hipMemcpyAsync(buf, c->send.ptr, bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

extern "C" int dh_comm_allgather(dh_comm* c, const double* send, int64_t n, double* recv) {
    if (!c || (n > 0 && (!send || !recv))) return fail(DH_E_ARG, "null argument");
    if (n < 0) return fail(DH_E_ARG, "n < 0");
    if (n == 0) return DH_OK;
    DeviceScope dev_scope(c->ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    hipStream_t st = c->ctx->stream;
    const size_t bytes = (size_t)n * sizeof(double);
    HIP_TRY(c->send.reserve(bytes));
    HIP_TRY(c->recv.reserve(bytes * c->world));
    HIP_TRY(hipMemcpyAsync(c->send.ptr, send, bytes, hipMemcpyHostToDevice, st));
    NCCL_TRY(rccl().all_gather(c->send.ptr, c->recv.ptr, (size_t)n, ncclFloat64, c->comm, st));
    HIP_TRY(hipMemcpyAsync(recv, c->recv.ptr, bytes * c->world, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

extern "C" int dh_best_start(const double* all, int64_t rows, int width, int col_start,
                             int col_fun, int* best) {
    if (!best || (rows > 0 && !all)) return fail(DH_E_ARG, "null argument");
    if (width < 1 || col_start < 0 || col_start >= width || col_fun < 0 || col_fun >= width)
        return fail(DH_E_ARG, "column out of range");
    // lbfgs_calibrator.py:271-275: starts in order, best_loss = inf, strict < (NaN never wins);
    // rows with a negative start index are padding
    std::vector<std::pair<double, double>> by_start;           // (start, fun)
    by_start.reserve((size_t)std::max<int64_t>(rows, 0));
    for (int64_t i = 0; i < rows; ++i) {
        const double s = all[i * width + col_start];
        if (s >= 0.0) by_start.emplace_back(s, all[i * width + col_fun]);
    }
    std::stable_sort(by_start.begin(), by_start.end(),
                     [](const auto& a, const auto& b) { return a.first < b.first; });
    double best_loss = __builtin_huge_val();
    *best = -1;
    for (const auto& e : by_start)
        if (e.second < best_loss) {
            best_loss = e.second;
            *best = (int)e.first;
        }
    return DH_OK;
}

extern "C" int dh_allgather_best(dh_comm* c, const double* rec, int rows, int width,
                                 int col_start, int col_fun, double* all, int* best) {
    if (!c || !all || !best || (rows > 0 && !rec)) return fail(DH_E_ARG, "null argument");
    if (rows < 0 || width < 1) return fail(DH_E_ARG, "rows / width out of range");
    const int rc = dh_comm_allgather(c, rec, (int64_t)rows * width, all);
    if (rc) return rc;
    return dh_best_start(all, (int64_t)rows * c->world, width, col_start, col_fun, best);
}

#include "dh_gen_device.h"
