// dh_kernels.hip -- gfx950 kernels of the COS pricing / calibration-objective hot path.
//
// Work decomposition (see DESIGN.md "Kernels"):
//   task  = (param set p, tile) where a tile is <= 256 options sharing one maturity T.
//   block = 256 threads = 256/TPT tasks of TPT threads each (TPT in {64,128,256}).
//   phase 1: the task's threads build the per-(p, T) COS table in LDS for k = 0..N-1:
//            u_k, w_k = Re(phi(u_k) e^{-i u_k a}) * 2/(b-a) (k=0 halved), cos/sin(u_k (b-a)),
//            1/(1+u_k^2), 1/u_k                    (double_heston.py:163-168,187-188)
//   phase 2: each option is reduced by a G-lane subgroup (G = power of two, G*options ~ TPT);
//            lane j owns a contiguous k-range, evaluates the payoff coefficients chi/psi
//            (double_heston.py:141-158,176-185) against the shared table, and the subgroup is
//            reduced with DPP butterflies (__shfl_xor).  Options whose truncation range is widened
//            by the log-strike clamp (double_heston.py:135-137) evaluate their own CF per term.
//   phase 3: (loss mode) the task's relative squared errors and invalid-price count are reduced
//            in a fixed order into one partial per task; dh_loss_finalize sums the partials of each
//            param set in tile order.  No atomics: results are bitwise reproducible and do not
//            depend on how many param sets share a launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
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
constexpr int kTabFields = 6;  // u, w, cos(u(b-a)), sin(u(b-a)), 1/(1+u^2), 1/u

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
    int N;
    double L;
    double* out;            // prices or null
    int64_t out_stride;     // M (surface) or 0 (paired)
    double* part_sse;       // [P*n_tiles] or null
    int* part_bad;          // [P*n_tiles]
};

// ----------------------------------------------------------------------------------------------
// one COS term for k >= 1:  w_k * V_k where V_k is the payoff coefficient of the option.
// call: c = xK, d = b;  put: c = a, d = xK.  sx/cx = sin/cos(u (xK - a)); sb/cb = sin/cos(u(b-a)).
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ double payoff_coeff(bool is_call, double u, double i1, double iu,
                                               double cb, double sb, double cx, double sx,
                                               double eb, double ea, double exK, double S0,
                                               double K) {
    double chi, psi;
    if (is_call) {  // d = b, c = xK   (double_heston.py:176-179)
        chi = i1 * (cb * eb - cx * exK + u * sb * eb - u * sx * exK);
        psi = iu * (sb - sx);
        return S0 * chi - K * psi;
    }
    // put: d = xK, c = a: cos(u*0) = 1, sin(u*0) = 0 (double_heston.py:182-185)
    // (the reference's "- u*sin(0)*e^a" and "- sin(0)" terms are exact zeros and are dropped)
    chi = i1 * (cx * exK - ea + u * sx * exK);
    psi = iu * sx;
    return K * psi - S0 * chi;
}

template <int TPT>
__global__ __launch_bounds__(kBlock) void cos_price_kernel(PriceArgs A) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int kTasks = kBlock / TPT;
    const int slot = threadIdx.x / TPT;
    const int t = threadIdx.x % TPT;
    const int N = A.N;
    const int64_t n_tasks = A.paired ? A.P : A.P * (int64_t)A.n_tiles;
    const int64_t task = (int64_t)blockIdx.x * kTasks + slot;
    const bool active = task < n_tasks;
    const int64_t p = active ? (A.paired ? task : task / A.n_tiles) : 0;
    const int tile = active ? (A.paired ? 0 : (int)(task % A.n_tiles)) : 0;

    double* tab = smem + (size_t)slot * (kTabFields * N + 2 * kTileMax);
    double* tu = tab;
    double* tw = tab + N;
    double* tcb = tab + 2 * N;
    double* tsb = tab + 3 * N;
    double* ti1 = tab + 4 * N;
    double* tiu = tab + 5 * N;
    double* tprice = tab + kTabFields * N;       // [kTileMax] prices of this task (loss mode)
    double* tflag = tprice + kTileMax;           // [kTileMax] 1.0 if invalid

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
    const double T = active ? A.T[opt0] : 1.0;
    double a0, b0;
    dh::trunc_unclamped(P, T, A.L, a0, b0);
    const double ba0 = b0 - a0;
    const double scale0 = 2.0 / ba0;

    // ---- phase 1: COS table of this (p, T) ----
    if (active) {
        for (int k = t; k < N; k += TPT) {
            const double u = k * dh::kPi / ba0;
            const cplx phi = dh::cf_eval(P, u, T);
            double sa, ca;
            sincos(u * a0, &sa, &ca);
            // Re(phi * exp(-i u a)) (double_heston.py:187); 2/(b-a) of V_k folded in; k=0 halved
            double w = (phi.re * ca + phi.im * sa) * scale0;
            double sb, cb;
            sincos(u * ba0, &sb, &cb);
            tu[k] = u;
            tw[k] = (k == 0) ? 0.5 * w : w;
            tcb[k] = cb;
            tsb[k] = sb;
            ti1[k] = 1.0 / (1.0 + u * u);
            tiu[k] = 1.0 / u;
        }
    }
    __syncthreads();

    // ---- phase 2: per-option reductions ----
    int G = 64;
    if (active) {
        const int want = TPT / max(nopt, 1);
        G = 1;
        while (G * 2 <= want && G < 64) G *= 2;
        while (G > 1 && G / 2 >= N) G /= 2;  // no more lanes than terms
    }
    const double disc = exp(-P.r * T);
    const int opts_per_pass = TPT / G;
    for (int base = 0; base < nopt; base += opts_per_pass) {
        const int oi = base + t / G;
        const int gl = t % G;
        const bool valid = active && oi < nopt;
        double acc = 0.0;
        if (valid) {
            const int m = opt0 + oi;
            const double Kin = A.K[m];
            const double K = (A.strike_mode == DH_STRIKE_PCT_SPOT) ? Kin * P.S0 / 100.0 : Kin;
            const bool is_call = A.call[m] != 0;
            const double xK = log(K / P.S0);
            // Python min/max semantics (a NaN a0 stays NaN), double_heston.py:136-137
            const double a = (xK - 0.1 < a0) ? xK - 0.1 : a0;
            const double b = (xK + 0.1 > b0) ? xK + 0.1 : b0;
            const double exK = exp(xK);
            const double eb = exp(b), ea = exp(a);
            const int per = (N + G - 1) / G;
            const int k_lo = gl * per;
            const int k_hi = min(N, k_lo + per);
            if (a == a0 && b == b0) {
                for (int k = k_lo; k < k_hi; ++k) {
                    double v;
                    if (k == 0) {
                        // chi_0 = e^d - e^c, psi_0 = d - c
                        v = is_call ? (P.S0 * (eb - exK) - K * (b - xK))
                                    : (K * (xK - a) - P.S0 * (exK - ea));
                    } else {
                        const double u = tu[k];
                        double sx, cx;
                        sincos(u * (xK - a), &sx, &cx);
                        v = payoff_coeff(is_call, u, ti1[k], tiu[k], tcb[k], tsb[k], cx, sx, eb,
                                         ea, exK, P.S0, K);
                    }
                    acc += tw[k] * v;
                }
            } else {
                // clamp-widened range: this option needs its own u grid and CF values
                const double ba = b - a;
                const double scale = 2.0 / ba;
                for (int k = k_lo; k < k_hi; ++k) {
                    const double u = k * dh::kPi / ba;
                    const cplx phi = dh::cf_eval(P, u, T);
                    double sa, ca;
                    sincos(u * a, &sa, &ca);
                    double w = (phi.re * ca + phi.im * sa) * scale;
                    double v;
                    if (k == 0) {
                        w *= 0.5;
                        v = is_call ? (P.S0 * (eb - exK) - K * (b - xK))
                                    : (K * (xK - a) - P.S0 * (exK - ea));
                    } else {
                        double sb, cb, sx, cx;
                        sincos(u * ba, &sb, &cb);
                        sincos(u * (xK - a), &sx, &cx);
                        v = payoff_coeff(is_call, u, 1.0 / (1.0 + u * u), 1.0 / u, cb, sb, cx, sx,
                                         eb, ea, exK, P.S0, K);
                    }
                    acc += w * v;
                }
            }
        }
        // subgroup butterfly (G lanes, aligned inside one wave; all lanes of the wave take part)
        for (int off = 1; off < G; off <<= 1) acc += __shfl_xor(acc, off, 64);
        if (valid && gl == 0) {
            const double price = disc * acc;  // e^{-rT} sum' (double_heston.py:190)
            const int m = opt0 + oi;
            if (A.out) A.out[p * A.out_stride + A.perm[m]] = price;
            if (A.part_sse) {
                const double mk = A.mkt[m];
                const double rel = (price - mk) / mk;
                tprice[oi] = rel * rel;
                // lbfgs_calibrator.py:152: NaN, inf or <= 0 is invalid
                tflag[oi] = (isnan(price) || isinf(price) || price <= 0.0) ? 1.0 : 0.0;
            }
        }
    }

    // ---- phase 3: fixed-order per-task loss partial ----
    if (A.part_sse) {
        __syncthreads();
        if (active && t < 64) {
            double s = 0.0, f = 0.0;
            for (int i = t; i < nopt; i += 64) {
                s += tprice[i];
                f += tflag[i];
            }
            for (int off = 1; off < 64; off <<= 1) {
                s += __shfl_xor(s, off, 64);
                f += __shfl_xor(f, off, 64);
            }
            if (t == 0) {
                A.part_sse[task] = s;
                A.part_bad[task] = (int)f;
            }
        }
    }
}

__global__ void loss_finalize_kernel(const double* __restrict__ part_sse,
                                     const int* __restrict__ part_bad, int n_tiles, int S,
                                     double* __restrict__ sse, int32_t* __restrict__ n_bad) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    double acc = 0.0;
    int bad = 0;
    for (int j = 0; j < n_tiles; ++j) {
        acc += part_sse[(int64_t)s * n_tiles + j];
        bad += part_bad[(int64_t)s * n_tiles + j];
    }
    sse[s] = acc;
    n_bad[s] = bad;
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
    return (size_t)tasks * (kTabFields * (size_t)N + 2 * kTileMax) * sizeof(double);
}

int pick_tpt(int N) { return N >= 256 ? 256 : (N >= 128 ? 128 : 64); }

}  // namespace

struct dh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf params, out, sse, bad, part_sse, part_bad, aux0, aux1, aux2, aux3;
    bool attr_set = false;
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

int launch_price(dh_ctx* ctx, const PriceArgs& A, hipStream_t st) {
    int rc = ensure_attrs(ctx);
    if (rc) return rc;
    const int tpt = pick_tpt(A.N);
    const int64_t n_tasks = A.paired ? A.P : A.P * (int64_t)A.n_tiles;
    if (n_tasks == 0) return DH_OK;
    const int tasks_per_block = kBlock / tpt;
    const int64_t blocks = (n_tasks + tasks_per_block - 1) / tasks_per_block;
    if (blocks > 0x7fffffffLL) return fail(DH_E_ARG, "too many tasks for one launch");
    const size_t lds = lds_bytes(A.N, tpt);
    if (lds > 160 * 1024) return fail(DH_E_ARG, "COS table does not fit in LDS");
    dim3 grid((unsigned)blocks), block(kBlock);
    switch (tpt) {
        case 64: hipLaunchKernelGGL(cos_price_kernel<64>, grid, block, lds, st, A); break;
        case 128: hipLaunchKernelGGL(cos_price_kernel<128>, grid, block, lds, st, A); break;
        default: hipLaunchKernelGGL(cos_price_kernel<256>, grid, block, lds, st, A); break;
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
                      &ctx->part_bad, &ctx->aux0, &ctx->aux1, &ctx->aux2, &ctx->aux3})
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
    PriceArgs A = surface_args(s, d_params, S, N, L);
    A.out = d_prices;
    A.part_sse = (double*)ctx->part_sse.ptr;
    A.part_bad = (int*)ctx->part_bad.ptr;
    rc = launch_price(ctx, A, st);
    if (rc) return rc;
    hipLaunchKernelGGL(loss_finalize_kernel, dim3((S + 63) / 64), dim3(64), 0, st, A.part_sse,
                       A.part_bad, s->n_tiles, S, d_sse, d_n_bad);
    HIP_TRY(hipGetLastError());
    return DH_OK;
}

int dh_surface_partials_dev(dh_ctx* ctx, const dh_surface* s, const double* d_params, int S,
                            int N, double L, double* d_part_sse, int32_t* d_part_bad,
                            void* stream) {
    if (!ctx || !s || (S > 0 && (!d_params || !d_part_sse || !d_part_bad)))
        return fail(DH_E_ARG, "null argument");
    if (!s->has_mkt) return fail(DH_E_ARG, "surface has no market prices");
    int rc = check_N(N);
    if (rc) return rc;
    if (S < 0) return fail(DH_E_ARG, "S < 0");
    if (S == 0 || s->M == 0) return DH_OK;
    rc = set_device(ctx);
    if (rc) return rc;
    PriceArgs A = surface_args(s, d_params, S, N, L);
    A.part_sse = d_part_sse;
    A.part_bad = (int*)d_part_bad;
    return launch_price(ctx, A, stream ? (hipStream_t)stream : ctx->stream);
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
