// dh_kernels.hip -- gfx950 kernels of the COS pricing / calibration-objective hot path.
//
// Work decomposition (DESIGN.md "Kernels"):
//   task  = (param set p, tile); a tile is <= 256 options sharing one maturity T.
//   block = 256 threads = 256/TPT tasks of TPT threads (TPT in {64,128,256}, chosen from N).
//   phase 1  (CF table, once per (p, T)): the task's threads evaluate phi(u_k) for k < N and
//            fold it with the k-only parts of the payoff coefficients (double_heston.py:141-158,
//            176-190) into three LDS columns T2/T3/T4 plus three k-sums (call / put constants).
//   phase 2  (per option): the COS sum splits into option-independent constants and two
//            angle sums  S2 = sum_k T2_k cos(k th) + T3_k sin(k th),  S4 = sum_k T4_k sin(k th),
//            th = pi (log(K/S0) - a) / (b - a).  A G-lane subgroup walks k interleaved (lane j:
//            k = 1 + j, 1 + j + G, ...), advancing the angle by a complex rotation e^{i G th}
//            with an exact sincos re-anchor every 64 steps, then reduces with DPP butterflies.
//            Options whose [a, b] is widened by the log-strike clamp (double_heston.py:135-137)
//            are queued and priced after a rebuild of the table on their own range (same code,
//            block-uniform trip count).  Validation ("exact") mode instead runs cos_exact_kernel:
//            per-term CF + sincos in the reference's operation order, one wave per option.
//   phase 3  (loss mode): per-task fixed-order partial of sum rel^2 and #invalid; the last task
//            of a param set to finish (agent-scope counter, release/acquire) sums the partials
//            in tile order.  One launch per request, no float atomics, bitwise reproducible and
//            independent of how many param sets share the launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "dh_device.h"
#include "dhcos.h"

using dh::cplx;
using dh::Params;

namespace {

constexpr int kBlock = 256;
constexpr int kTileMax = 256;
constexpr int kAnchor = 64;       // exact sincos re-anchor period of the angle recurrence

struct PriceArgs {
    const double* prm;      // [P][16]
    int64_t P;
    const double* K;        // [M] sorted by T (absolute strike or K_relative)
    const double* T;        // [M]
    const int8_t* call;     // [M]
    const double* mkt;      // [M] or null
    const int* perm;        // [M] sorted -> caller index
    const int2* tiles;      // [n_tiles] (opt0, nopt)
    int n_tiles;
    int paired;             // option i under param set i, one option per task
    int strike_mode;
    int exact;              // validation mode (host routes to cos_exact_kernel)
    int M;                  // options in the (sorted) option arrays
    int N;
    double L;
    double* out;            // prices [P*out_stride] or null
    int64_t out_stride;     // M (surface) or 0 (paired)
    double* part_sse;       // loss mode: [P*n_tiles] partials, else null
    int* part_bad;          // [P*n_tiles]
    unsigned* counter;      // [P] arrival counters (zero between launches)
    double* sse;            // [P] final sums (loss mode)
    int* n_bad;             // [P]
    unsigned long long* stamps;   // diagnostic builds (DH_STAMPS) only: [blocks][kStamps]
};

// In-kernel phase stamps, compiled only into the diagnostic build (make stamps): lane 0 of each
// block writes s_memtime at the phase boundaries and s_memrealtime at start/end.
constexpr int kStamps = 8;
#ifdef DH_STAMPS
#define DH_STAMP(A, i)                                                                     \
    do {                                                                                   \
        if ((A).stamps && threadIdx.x == 0) {                                              \
            unsigned long long _t;                                                         \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
            (A).stamps[(size_t)blockIdx.x * kStamps + (i)] = _t;                          \
        }                                                                                  \
    } while (0)
#define DH_RSTAMP(A, i)                                                                    \
    do {                                                                                   \
        if ((A).stamps && threadIdx.x == 0)                                                \
            (A).stamps[(size_t)blockIdx.x * kStamps + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define DH_STAMP(A, i) do {} while (0)
#define DH_RSTAMP(A, i) do {} while (0)
#endif

__host__ __device__ constexpr int task_lds_doubles(int N, int tpt) {
    // (T2,T3)[N] u[N] T4[N] | reduction [4][waves] | K, mkt, sse, bad [kTileMax] |
    // call, perm, clamp list [kTileMax] ints + count (rounded to whole 16-B pairs)
    return 4 * N + 4 * (tpt / 64) + 4 * kTileMax + ((3 * kTileMax + 4) / 2 + 1) / 2 * 2;
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

// Fixed-order loss partial of one task (wave 0 of the task).  Hand-off to the last task of param
// set p without fences (MI355X_MICROARCH.md, "Valid forms", first table row): the storing lane
// writes its partial with agent-scope (sc1, write-through) stores, drains them with
// s_waitcnt vmcnt(0), then adds to p's counter; the lane whose add returns n_tiles - 1 reads every
// partial of p with sc1 loads, sums them in tile order and resets the counter for the next launch.
__device__ __forceinline__ void task_loss(const PriceArgs& A, int64_t p, int64_t task, int nopt,
                                          int t, const double* lsse, const double* lbad) {
    double s = 0.0, f = 0.0;
    for (int i = t; i < nopt; i += 64) {
        s += lsse[i];
        f += lbad[i];
    }
    for (int off = 1; off < 64; off <<= 1) {
        s += __shfl_xor(s, off, 64);
        f += __shfl_xor(f, off, 64);
    }
    const int64_t base_i = p * A.n_tiles;
    unsigned old = 0;
    if (t == 0) {
        __hip_atomic_store(&A.part_sse[task], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&A.part_bad[task], (int)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        old = __hip_atomic_fetch_add(&A.counter[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    old = __shfl(old, 0, 64);
    if (old != (unsigned)A.n_tiles - 1u) return;
    // last arriver: the whole wave reads the partials of p (lane-strided, sc1), fixed order
    double acc = 0.0, bad = 0.0;
    for (int j = t; j < A.n_tiles; j += 64) {
        acc += __hip_atomic_load(&A.part_sse[base_i + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad += __hip_atomic_load(&A.part_bad[base_i + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int off = 1; off < 64; off <<= 1) {
        acc += __shfl_xor(acc, off, 64);
        bad += __shfl_xor(bad, off, 64);
    }
    if (t == 0) {
        A.sse[p] = acc;
        A.n_bad[p] = (int)bad;
        __hip_atomic_store(&A.counter[p], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ----------------------------------------------------------------------------------------------
// exact per-term path (validation mode): own truncation range, own u grid, CF per term, the
// reference's operation order (double_heston.py:160-192).  Lane share of sum_k' Re(phi e^{-iua}) V_k.
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

__device__ __forceinline__ double option_strike(const PriceArgs& A, int m, double S0) {
    const double Kin = A.K[m];
    return (A.strike_mode == DH_STRIKE_PCT_SPOT) ? Kin * S0 / 100.0 : Kin;
}

// Validation kernel: one wave per (param set, option); prices only (loss via loss_from_prices).
__global__ __launch_bounds__(kBlock) void cos_exact_kernel(PriceArgs A, int M, double* prices) {
    const int64_t item = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t n_items = A.paired ? A.P : A.P * (int64_t)M;
    if (item >= n_items) return;                       // whole wave exits together
    const int64_t p = A.paired ? item : item / M;
    const int m = A.paired ? (int)item : (int)(item % M);
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
    for (int off = 1; off < 64; off <<= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
        const double price = exp(-P.r * T) * acc;
        if (A.out) A.out[p * A.out_stride + A.perm[m]] = price;
        if (prices) prices[p * M + m] = price;
    }
}

// Loss sums from a [P][M] price buffer (validation mode): one wave per param set, fixed order.
__global__ void loss_from_prices_kernel(const double* __restrict__ prices,
                                        const double* __restrict__ mkt, int M, int S,
                                        double* __restrict__ sse, int* __restrict__ n_bad) {
    const int s = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (s >= S) return;
    double acc = 0.0, bad = 0.0;
    for (int m = lane; m < M; m += 64) {
        const double pr = prices[(int64_t)s * M + m];
        const double rel = (pr - mkt[m]) / mkt[m];
        acc += rel * rel;
        bad += (isnan(pr) || isinf(pr) || pr <= 0.0) ? 1.0 : 0.0;
    }
    for (int off = 1; off < 64; off <<= 1) {
        acc += __shfl_xor(acc, off, 64);
        bad += __shfl_xor(bad, off, 64);
    }
    if (lane == 0) {
        sse[s] = acc;
        n_bad[s] = (int)bad;
    }
}

// ----------------------------------------------------------------------------------------------
// table build: COS table of (p, T, [a, b]) into LDS + the four k-sums, reduced in fixed order.
// w_k = Re(phi(u_k) e^{-i u_k a}) 2/(b-a);  T2 = w S0/(1+u^2), T3 = T2 u, T4 = w/u   (k >= 1)
// c0 = sum T2 e^b (cos(u(b-a)) + u sin(u(b-a)))   (call constant)
// c1 = sum T4 sin(u(b-a))                          (call constant, times K)
// c5 = sum T2 e^a                                  (put constant)
// w0 = w_0 / 2                                     (k = 0 term weight)
// Must be reached by every thread of the block (contains a barrier).
// ----------------------------------------------------------------------------------------------
struct Consts {
    double c0, c1, c5, w0, eb, ea;
};

template <int TPT>
__device__ __forceinline__ Consts build_table(const Params& P, double T, double a, double b,
                                              bool work, int N, int t, double* tu, double2* t23,
                                              double* t4, double* red) {
    constexpr int kWaves = TPT / 64;
    const int lane = threadIdx.x & 63;
    const int wv = t >> 6;
    const double ba = b - a;
    const double scale = 2.0 / ba;
    const double eb = exp(b), ea = exp(a);
    const dh::CfConsts CC = dh::cf_consts(P, T);
    double c0 = 0.0, c1 = 0.0, c5 = 0.0, w0 = 0.0;
    if (work) {
        for (int k = t; k < N; k += TPT) {
            const double u = k * dh::kPi / ba;
            const double w = dh::cf_phase_re(CC, u, T, a) * scale;
            if (k == 0) {
                w0 = 0.5 * w;
                continue;
            }
            double sb, cb;
            dh::dsincos(u * ba, &sb, &cb);
            const double i1 = 1.0 / (1.0 + u * u);
            const double T2 = w * P.S0 * i1;
            const double T4 = w * (1.0 / u);
            tu[k] = u;
            t23[k] = make_double2(T2, T2 * u);
            t4[k] = T4;
            c0 += T2 * eb * (cb + u * sb);
            c1 += T4 * sb;
            c5 += T2 * ea;
        }
    }
    for (int off = 1; off < 64; off <<= 1) {
        c0 += __shfl_xor(c0, off, 64);
        c1 += __shfl_xor(c1, off, 64);
        c5 += __shfl_xor(c5, off, 64);
        w0 += __shfl_xor(w0, off, 64);
    }
    if (lane == 0) {
        red[0 * kWaves + wv] = c0;
        red[1 * kWaves + wv] = c1;
        red[2 * kWaves + wv] = c5;
        red[3 * kWaves + wv] = w0;
    }
    __syncthreads();
    Consts C{0.0, 0.0, 0.0, 0.0, eb, ea};
    for (int i = 0; i < kWaves; ++i) {
        C.c0 += red[0 * kWaves + i];
        C.c1 += red[1 * kWaves + i];
        C.c5 += red[2 * kWaves + i];
        C.w0 += red[3 * kWaves + i];
    }
    return C;
}

// sum' of one option from the table constants and its angle sums (k = 0 term:
// chi_0 = e^d - e^c, psi_0 = d - c, double_heston.py:142-143,154-155).
__device__ __forceinline__ double option_sum(const Consts& C, bool is_call, double S0, double K,
                                             double xK, double exK, double a, double b,
                                             double s2, double s4) {
    const double v0 = is_call ? (S0 * (C.eb - exK) - K * (b - xK))
                              : (K * (xK - a) - S0 * (exK - C.ea));
    const double cst = is_call ? (C.c0 - K * C.c1) : C.c5;
    return cst + C.w0 * v0 - exK * s2 + K * s4;
}

constexpr int kR = 4;   // options carried per lane in phase 2 (independent rotation chains)

// Angle sums of up to kR options on lanes k = k1, k1 + G, ...:
//   s2_j = sum_k T2_k cos(k th_j) + T3_k sin(k th_j),  s4_j = sum_k T4_k sin(k th_j)
// the angle u_k (xK_j - a) advances by an e^{i G th_j} rotation, exact re-anchor every kAnchor
// steps; one (T2, T3) ds_read_b128 + one T4 read serve all kR options.
__device__ __forceinline__ void angle_sums_r(int k1, int G, int N, const double (&dx)[kR],
                                             double ba, const double* tu, const double2* t23,
                                             const double* t4, double (&s2)[kR],
                                             double (&s4)[kR]) {
#pragma unroll
    for (int j = 0; j < kR; ++j) {
        s2[j] = 0.0;
        s4[j] = 0.0;
    }
    if (k1 >= N) return;
    double cx[kR], sx[kR], cs[kR], ss[kR];
    const double ustep = G * dh::kPi / ba;
    const double u1 = tu[k1];
#pragma unroll
    for (int j = 0; j < kR; ++j) {
        dh::dsincos(u1 * dx[j], &sx[j], &cx[j]);
        dh::dsincos(ustep * dx[j], &ss[j], &cs[j]);
    }
    int n = 0;
    for (int k = k1; k < N; k += G, ++n) {
        if (n == kAnchor) {
            const double uk = tu[k];
#pragma unroll
            for (int j = 0; j < kR; ++j) dh::dsincos(uk * dx[j], &sx[j], &cx[j]);
            n = 0;
        }
        const double2 a23 = t23[k];
        const double a4 = t4[k];
#pragma unroll
        for (int j = 0; j < kR; ++j) {
            s2[j] = fma(a23.x, cx[j], s2[j]);
            s2[j] = fma(a23.y, sx[j], s2[j]);
            s4[j] = fma(a4, sx[j], s4[j]);
            const double cn = cx[j] * cs[j] - sx[j] * ss[j];
            sx[j] = sx[j] * cs[j] + cx[j] * ss[j];
            cx[j] = cn;
        }
    }
}

#ifndef DH_MIN_WAVES
#define DH_MIN_WAVES 1     // occupancy hint (waves per SIMD) for the register allocator
#endif

template <int TPT>
__global__ __launch_bounds__(kBlock, DH_MIN_WAVES) void cos_price_kernel(PriceArgs A) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int kTasks = kBlock / TPT;
    const int slot = threadIdx.x / TPT;
    const int t = threadIdx.x % TPT;
    const int N = A.N;
    const int64_t n_tasks = A.paired ? A.P : A.P * (int64_t)A.n_tiles;
    // the task index is wave-uniform: make that visible so params live in SGPRs
    const int64_t task = (int64_t)blockIdx.x * kTasks + __builtin_amdgcn_readfirstlane(slot);
    const bool active = task < n_tasks;
    const int64_t p = active ? (A.paired ? task : task / A.n_tiles) : 0;
    const int tile = active ? (A.paired ? 0 : (int)(task % A.n_tiles)) : 0;
    DH_RSTAMP(A, 0);
    DH_STAMP(A, 1);

    // LDS per task: (T2,T3)[N] | u[N] | T4[N] | reduction | option data | loss | clamp list
    double* base = smem + (size_t)slot * task_lds_doubles(N, TPT);
    double2* t23 = (double2*)base;
    double* tu = base + 2 * N;
    double* t4 = base + 3 * N;
    double* red = base + 4 * N;
    double* lK = red + 4 * (TPT / 64);                 // [kTileMax] strikes
    double* lmkt = lK + kTileMax;                      // [kTileMax] market prices
    double* lsse = lmkt + kTileMax;                    // [kTileMax]
    double* lbad = lsse + kTileMax;                    // [kTileMax]
    int* lcall = (int*)(lbad + kTileMax);              // [kTileMax]
    int* lperm = lcall + kTileMax;                     // [kTileMax]
    int* lclamp = lperm + kTileMax;                    // [kTileMax] clamped option indices
    int* ncl = lclamp + kTileMax;                      // [1]
    int* nclmax = (int*)(smem + (size_t)kTasks * task_lds_doubles(N, TPT));   // [1] block max

    const Params P = dh::load_params(A.prm + p * DH_PARAM_STRIDE);
    int opt0 = 0, nopt = 0;
    if (active) {
        if (A.paired) {
            opt0 = (int)p;
            nopt = 1;
        } else {
            const int2 tl = A.tiles[tile];
            opt0 = tl.x;
            nopt = tl.y;
        }
    }
    // prefetch this tile's option data (first chunk in registers across the truncation math)
    const bool pf = active && t < nopt;
    const double pK = pf ? A.K[opt0 + t] : 0.0;
    const double pM = (pf && A.mkt) ? A.mkt[opt0 + t] : 0.0;
    const int pC = pf ? A.call[opt0 + t] : 0;
    const int pP = pf ? A.perm[opt0 + t] : 0;
    if (t == 0) *ncl = 0;
    if (threadIdx.x == 0) *nclmax = 0;
    const double T = active ? A.T[opt0] : 1.0;
    double a0, b0;
    dh::trunc_unclamped(P, T, A.L, a0, b0);
    const double ba0 = b0 - a0;
    const double disc = exp(-P.r * T);
    const bool pct = A.strike_mode == DH_STRIKE_PCT_SPOT;
    if (pf) {
        lK[t] = pct ? pK * P.S0 / 100.0 : pK;
        lmkt[t] = pM;
        lcall[t] = pC;
        lperm[t] = pP;
    }
    for (int i = t + TPT; active && i < nopt; i += TPT) {
        const double Kin = A.K[opt0 + i];
        lK[i] = pct ? Kin * P.S0 / 100.0 : Kin;
        lmkt[i] = A.mkt ? A.mkt[opt0 + i] : 0.0;
        lcall[i] = A.call[opt0 + i];
        lperm[i] = A.perm[opt0 + i];
    }
    DH_STAMP(A, 2);

    // One table-build site for both passes (a second inlined copy of the CF costs ~80 VGPRs):
    //   it = 0   table of (p, T) on the un-clamped range, then every option of the tile;
    //   it >= 1  table rebuilt on the widened range of the (it-1)-th clamped option
    //            (double_heston.py:135-137), then that option alone.
    // The trip count is block-uniform (max over the block's tasks) because of the barriers.
    int n_iter = 1;
    for (int it = 0; it < n_iter; ++it) {
        bool work = active;
        int oi1 = 0;
        double a = a0, b = b0, K1 = P.S0, xK1 = 0.0;
        if (it > 0) {
            work = active && it - 1 < *ncl;
            oi1 = work ? lclamp[it - 1] : 0;
            K1 = work ? lK[oi1] : P.S0;
            xK1 = log(K1 / P.S0);
            a = (xK1 - 0.1 < a0) ? xK1 - 0.1 : a0;          // Python min/max (:136-137)
            b = (xK1 + 0.1 > b0) ? xK1 + 0.1 : b0;
            __syncthreads();                                  // previous table readers are done
        }
        // table build (its barrier also publishes the prefetched option data on it = 0)
        const Consts C = build_table<TPT>(P, T, a, b, work, N, t, tu, t23, t4, red);
        if (it == 0) {
            DH_STAMP(A, 3);
            // ---- phase 2: option groups of kR options on G lanes each ----
            const int R = min(kR, max(nopt, 1));
            const int ngroups = (nopt + R - 1) / R;
            int G = 1;
            while (G * 2 <= TPT / max(ngroups, 1) && G < 64) G *= 2;
            while (G > 1 && G / 2 >= N - 1) G /= 2;           // no more lanes than terms k >= 1
            const int groups_per_pass = TPT / G;
            for (int pass = 0; pass < ngroups; pass += groups_per_pass) {
                const int gi = pass + t / G;
                const int gl = t % G;
                const bool gvalid = active && gi < ngroups;
                double dx[kR], xK[kR];
                bool use[kR];
#pragma unroll
                for (int j = 0; j < kR; ++j) {
                    const int oi = gi * R + j;
                    use[j] = gvalid && j < R && oi < nopt;
                    const double K = use[j] ? lK[oi] : P.S0;
                    xK[j] = log(K / P.S0);
                    if (use[j] && (xK[j] - 0.1 < a0 || xK[j] + 0.1 > b0)) {   // widened range
                        if (gl == 0) lclamp[atomicAdd(ncl, 1)] = oi;
                        use[j] = false;
                    }
                    dx[j] = use[j] ? xK[j] - a0 : 0.0;
                }
                double s2[kR], s4[kR];
                angle_sums_r(1 + gl, G, N, dx, ba0, tu, t23, t4, s2, s4);
                for (int off = 1; off < G; off <<= 1) {
#pragma unroll
                    for (int j = 0; j < kR; ++j) {
                        s2[j] += __shfl_xor(s2[j], off, 64);
                        s4[j] += __shfl_xor(s4[j], off, 64);
                    }
                }
                if (gl == 0) {
#pragma unroll
                    for (int j = 0; j < kR; ++j) {
                        if (!use[j]) continue;
                        const int oi = gi * R + j;
                        const double sum = option_sum(C, lcall[oi] != 0, P.S0, lK[oi], xK[j],
                                                      exp(xK[j]), a0, b0, s2[j], s4[j]);
                        record_price(A, p, lperm[oi], lmkt[oi], oi, disc * sum, lsse, lbad);
                    }
                }
            }
            __syncthreads();
            DH_STAMP(A, 4);
            if (t == 0 && active) atomicMax(nclmax, *ncl);
            __syncthreads();
            n_iter = 1 + *nclmax;
        } else {
            double dx[kR] = {work ? xK1 - a : 0.0, 0.0, 0.0, 0.0};
            double s2[kR], s4[kR];
            if (work && t < 64) {
                angle_sums_r(1 + t, 64, N, dx, b - a, tu, t23, t4, s2, s4);
            } else {
                s2[0] = 0.0;
                s4[0] = 0.0;
            }
            for (int off = 1; off < 64; off <<= 1) {
                s2[0] += __shfl_xor(s2[0], off, 64);
                s4[0] += __shfl_xor(s4[0], off, 64);
            }
            if (work && t == 0) {
                const double sum = option_sum(C, lcall[oi1] != 0, P.S0, K1, xK1, exp(xK1), a, b,
                                              s2[0], s4[0]);
                record_price(A, p, lperm[oi1], lmkt[oi1], oi1, disc * sum, lsse, lbad);
            }
        }
    }

    // ---- phase 3: fixed-order per-task loss partial, last arriver finalises the param set ----
    DH_STAMP(A, 5);
    if (A.part_sse) {
        __syncthreads();
        if (active && t < 64) task_loss(A, p, task, nopt, t, lsse, lbad);
    }
    DH_STAMP(A, 6);
    DH_RSTAMP(A, 7);
}

__global__ void cf_kernel(const double* __restrict__ prm, const double* __restrict__ u, int n,
                          double tau, double* __restrict__ re, double* __restrict__ im) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Params P = dh::load_params(prm);
    const cplx c = dh::cf_eval(P, u[i], tau);
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

size_t lds_bytes(int N, int tpt) {
    const int tasks = kBlock / tpt;
    return ((size_t)tasks * task_lds_doubles(N, tpt) + 2) * sizeof(double);
}

int pick_tpt(int N) { return N >= 256 ? 256 : (N >= 128 ? 128 : 64); }

}  // namespace

struct dh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf params, out, sse, bad, part_sse, part_bad, counter, exact_prices, aux0, aux1, aux2,
        aux3;
    bool attr_set = false;
    int exact = 0;          // validation mode: every option through the per-term exact path
    int stamps_on = 0;      // diagnostic builds: record per-block phase stamps
    DevBuf stamps;
    int64_t stamps_n = 0;
};

struct dh_surface {
    dh_ctx* ctx = nullptr;
    int M = 0;
    int n_tiles = 0;
    int strike_mode = 0;
    bool has_mkt = false;
    double* K = nullptr;
    double* T = nullptr;
    double* mkt = nullptr;
    int8_t* call = nullptr;
    int* perm = nullptr;
    int2* tiles = nullptr;
};

namespace {

int set_device(dh_ctx* ctx) {
    HIP_TRY(hipSetDevice(ctx->device));
    return DH_OK;
}

int ensure_attrs(dh_ctx* ctx) {
    if (ctx->attr_set) return DH_OK;
    const int lim = 160 * 1024;
    HIP_TRY(hipFuncSetAttribute((const void*)cos_price_kernel<64>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    HIP_TRY(hipFuncSetAttribute((const void*)cos_price_kernel<128>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    HIP_TRY(hipFuncSetAttribute((const void*)cos_price_kernel<256>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ctx->attr_set = true;
    return DH_OK;
}

int check_N(int N) {
    if (N < 1 || N > DH_MAX_N)
        return fail(DH_E_ARG, "N must be in [1, " + std::to_string(DH_MAX_N) + "], got " +
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
    hipLaunchKernelGGL(cos_exact_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, A, A.M,
                       prices);
    HIP_TRY(hipGetLastError());
    if (A.part_sse) {
        const int S = (int)A.P;
        hipLaunchKernelGGL(loss_from_prices_kernel, dim3((S * 64 + kBlock - 1) / kBlock),
                           dim3(kBlock), 0, st, (const double*)prices, A.mkt, A.M, S, A.sse,
                           A.n_bad);
        HIP_TRY(hipGetLastError());
    }
    return DH_OK;
}

int launch_price(dh_ctx* ctx, const PriceArgs& A, hipStream_t st) {
    const int64_t n_tasks = A.paired ? A.P : A.P * (int64_t)A.n_tiles;
    if (n_tasks == 0) return DH_OK;
    if (A.exact) return launch_exact(ctx, A, st);
    PriceArgs B = A;
    if (ctx->stamps_on) {
        const int tpb = kBlock / pick_tpt(A.N);
        const int64_t nb = (n_tasks + tpb - 1) / tpb;
        HIP_TRY(ctx->stamps.reserve((size_t)nb * kStamps * 8));
        HIP_TRY(hipMemsetAsync(ctx->stamps.ptr, 0, (size_t)nb * kStamps * 8, st));
        B.stamps = (unsigned long long*)ctx->stamps.ptr;
        ctx->stamps_n = nb * kStamps;
    }
    int rc = ensure_attrs(ctx);
    if (rc) return rc;
    const int tpt = pick_tpt(A.N);
    const int tasks_per_block = kBlock / tpt;
    const int64_t blocks = (n_tasks + tasks_per_block - 1) / tasks_per_block;
    if (blocks > 0x7fffffffLL) return fail(DH_E_ARG, "too many tasks for one launch");
    const size_t lds = lds_bytes(A.N, tpt);
    if (lds > 160 * 1024) return fail(DH_E_ARG, "COS table does not fit in LDS");
    dim3 grid((unsigned)blocks), block(kBlock);
    switch (tpt) {
        case 64: hipLaunchKernelGGL(cos_price_kernel<64>, grid, block, lds, st, B); break;
        case 128: hipLaunchKernelGGL(cos_price_kernel<128>, grid, block, lds, st, B); break;
        default: hipLaunchKernelGGL(cos_price_kernel<256>, grid, block, lds, st, B); break;
    }
    HIP_TRY(hipGetLastError());
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
    e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(DH_E_HIP, std::string("stream create: ") + hipGetErrorString(e));
    }
    *out = c;
    return DH_OK;
}

int dh_ctx_destroy(dh_ctx* ctx) {
    if (!ctx) return DH_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (DevBuf* b : {&ctx->params, &ctx->out, &ctx->sse, &ctx->bad, &ctx->part_sse,
                      &ctx->part_bad, &ctx->counter, &ctx->exact_prices, &ctx->stamps, &ctx->aux0,
                      &ctx->aux1, &ctx->aux2, &ctx->aux3})
        b->release();
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return DH_OK;
}

int dh_ctx_synchronize(dh_ctx* ctx) {
    if (!ctx) return fail(DH_E_ARG, "ctx is null");
    HIP_TRY(hipSetDevice(ctx->device));
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
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, ctx->stamps.ptr, (size_t)std::min<int64_t>(cap, ctx->stamps_n) * 8,
                      hipMemcpyDeviceToHost));
    return DH_OK;
}

int dh_ctx_set_exact(dh_ctx* ctx, int on) {
    if (!ctx) return fail(DH_E_ARG, "ctx is null");
    ctx->exact = on ? 1 : 0;
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
    int rc = set_device(ctx);
    if (rc) return rc;
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
    for (int i = 0; i < M;) {
        int j = i;
        while (j < M && sT[j] == sT[i]) ++j;
        for (int s = i; s < j; s += kTileMax) tiles.push_back(make_int2(s, std::min(kTileMax, j - s)));
        i = j;
    }
    dh_surface* s = new (std::nothrow) dh_surface();
    if (!s) return fail(DH_E_ALLOC, "surface alloc");
    s->ctx = ctx;
    s->M = M;
    s->n_tiles = (int)tiles.size();
    s->strike_mode = strike_mode;
    s->has_mkt = mkt != nullptr;
    const size_t m8 = std::max<size_t>(1, (size_t)M) * 8;
    hipError_t e = hipSuccess;
    auto alloc = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, std::max<size_t>(bytes, 16));
    };
    alloc((void**)&s->K, m8);
    alloc((void**)&s->T, m8);
    alloc((void**)&s->mkt, m8);
    alloc((void**)&s->call, std::max(1, M));
    alloc((void**)&s->perm, std::max<size_t>(1, (size_t)M) * 4);
    alloc((void**)&s->tiles, std::max<size_t>(1, tiles.size()) * sizeof(int2));
    if (e == hipSuccess && M > 0) {
        e = hipMemcpy(s->K, sK.data(), (size_t)M * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(s->T, sT.data(), (size_t)M * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(s->mkt, sm.data(), (size_t)M * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(s->call, sc.data(), (size_t)M, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(s->perm, perm.data(), (size_t)M * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(s->tiles, tiles.data(), tiles.size() * sizeof(int2), hipMemcpyHostToDevice);
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
    if (s->ctx) (void)hipSetDevice(s->ctx->device);
    for (void* p : {(void*)s->K, (void*)s->T, (void*)s->mkt, (void*)s->call, (void*)s->perm,
                    (void*)s->tiles})
        if (p) (void)hipFree(p);
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
    A.n_tiles = s->n_tiles;
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
    rc = set_device(ctx);
    if (rc) return rc;
    PriceArgs A = surface_args(s, d_params, P, N, L);
    A.exact = ctx->exact;
    A.out = d_out;
    return launch_price(ctx, A, stream ? (hipStream_t)stream : ctx->stream);
}

int dh_surface_loss_dev(dh_ctx* ctx, const dh_surface* s, const double* d_params, int S, int N,
                        double L, double* d_sse, int32_t* d_n_bad, double* d_prices,
                        void* stream) {
    if (!ctx || !s || (S > 0 && (!d_params || !d_sse || !d_n_bad)))
        return fail(DH_E_ARG, "null argument");
    if (!s->has_mkt) return fail(DH_E_ARG, "surface has no market prices");
    int rc = check_N(N);
    if (rc) return rc;
    if (S < 0) return fail(DH_E_ARG, "S < 0");
    if (S == 0) return DH_OK;
    rc = set_device(ctx);
    if (rc) return rc;
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
    HIP_TRY(ctx->counter.reserve((size_t)S * 4));
    if (ctx->counter.cap != cap0) {       // fresh counters start at zero; kernels self-reset
        HIP_TRY(hipMemsetAsync(ctx->counter.ptr, 0, ctx->counter.cap, st));
    }
    PriceArgs A = surface_args(s, d_params, S, N, L);
    A.exact = ctx->exact;
    A.out = d_prices;
    A.part_sse = (double*)ctx->part_sse.ptr;
    A.part_bad = (int*)ctx->part_bad.ptr;
    A.counter = (unsigned*)ctx->counter.ptr;
    A.sse = d_sse;
    A.n_bad = (int*)d_n_bad;
    return launch_price(ctx, A, st);
}

int dh_surface_price(dh_ctx* ctx, const dh_surface* s, const double* params, int64_t P, int N,
                     double L, double* out) {
    if (!ctx || !s || (P > 0 && (!params || !out))) return fail(DH_E_ARG, "null argument");
    int rc = check_N(N);
    if (rc) return rc;
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    if (P == 0 || s->M == 0) return DH_OK;
    rc = set_device(ctx);
    if (rc) return rc;
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

int dh_surface_loss(dh_ctx* ctx, const dh_surface* s, const double* params, int S, int N,
                    double L, double* sse, int32_t* n_bad, double* prices) {
    if (!ctx || !s || (S > 0 && (!params || !sse || !n_bad))) return fail(DH_E_ARG, "null argument");
    int rc = check_N(N);
    if (rc) return rc;
    if (S < 0) return fail(DH_E_ARG, "S < 0");
    if (S == 0) return DH_OK;
    rc = set_device(ctx);
    if (rc) return rc;
    const size_t pb = (size_t)S * DH_PARAM_STRIDE * 8;
    HIP_TRY(ctx->params.reserve(pb));
    HIP_TRY(ctx->sse.reserve((size_t)S * 8));
    HIP_TRY(ctx->bad.reserve((size_t)S * 4));
    double* d_prices = nullptr;
    const size_t ob = (size_t)S * s->M * 8;
    if (prices) {
        HIP_TRY(ctx->out.reserve(ob));
        d_prices = (double*)ctx->out.ptr;
    }
    HIP_TRY(hipMemcpyAsync(ctx->params.ptr, params, pb, hipMemcpyHostToDevice, ctx->stream));
    rc = dh_surface_loss_dev(ctx, s, (const double*)ctx->params.ptr, S, N, L,
                             (double*)ctx->sse.ptr, (int32_t*)ctx->bad.ptr, d_prices, ctx->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(sse, ctx->sse.ptr, (size_t)S * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(n_bad, ctx->bad.ptr, (size_t)S * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (prices && s->M > 0)
        HIP_TRY(hipMemcpyAsync(prices, d_prices, ob, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return DH_OK;
}

int dh_price_pairs(dh_ctx* ctx, const double* params, const double* K, const double* T,
                   const int8_t* is_call, int64_t P, int N, double L, double* out) {
    if (!ctx || (P > 0 && (!params || !K || !T || !is_call || !out)))
        return fail(DH_E_ARG, "null argument");
    int rc = check_N(N);
    if (rc) return rc;
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    if (P == 0) return DH_OK;
    rc = set_device(ctx);
    if (rc) return rc;
    const size_t pb = (size_t)P * DH_PARAM_STRIDE * 8, vb = (size_t)P * 8;
    HIP_TRY(ctx->params.reserve(pb));
    HIP_TRY(ctx->out.reserve(vb));
    HIP_TRY(ctx->aux0.reserve(vb));
    HIP_TRY(ctx->aux1.reserve(vb));
    HIP_TRY(ctx->aux2.reserve((size_t)P));
    HIP_TRY(ctx->aux3.reserve((size_t)P * 4));
    std::vector<int> ident((size_t)P);
    std::iota(ident.begin(), ident.end(), 0);
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->params.ptr, params, pb, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux0.ptr, K, vb, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux1.ptr, T, vb, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux2.ptr, is_call, (size_t)P, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->aux3.ptr, ident.data(), (size_t)P * 4, hipMemcpyHostToDevice, st));
    PriceArgs A{};
    A.prm = (const double*)ctx->params.ptr;
    A.P = P;
    A.K = (const double*)ctx->aux0.ptr;
    A.T = (const double*)ctx->aux1.ptr;
    A.call = (const int8_t*)ctx->aux2.ptr;
    A.perm = (const int*)ctx->aux3.ptr;
    A.paired = 1;
    A.M = (int)P;
    A.exact = ctx->exact;
    A.strike_mode = DH_STRIKE_ABSOLUTE;
    A.N = N;
    A.L = L;
    A.out = (double*)ctx->out.ptr;
    A.out_stride = 0;
    rc = launch_price(ctx, A, st);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, ctx->out.ptr, vb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
}

int dh_cf(dh_ctx* ctx, const double* params, const double* u, int n, double tau, double* re,
          double* im) {
    if (!ctx || !params || (n > 0 && (!u || !re || !im))) return fail(DH_E_ARG, "null argument");
    if (n < 0) return fail(DH_E_ARG, "n < 0");
    if (n == 0) return DH_OK;
    int rc = set_device(ctx);
    if (rc) return rc;
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

int dh_trunc_range(dh_ctx* ctx, const double* params, const double* K, const double* T,
                   int64_t P, double L, double* a, double* b) {
    if (!ctx || (P > 0 && (!params || !K || !T || !a || !b))) return fail(DH_E_ARG, "null argument");
    if (P < 0) return fail(DH_E_ARG, "P < 0");
    if (P == 0) return DH_OK;
    int rc = set_device(ctx);
    if (rc) return rc;
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
    int rc = set_device(ctx);
    if (rc) return rc;
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
