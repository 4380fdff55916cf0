// dh_gen_device.h -- the generator's batch path on the device, included at
// the end of dh_kernels.hip (it uses dh_ctx / dh_surface and the pricing launch).
//
// Reference: src/data/synthetic_generator.py:98-157.  Per sample: 13 np.random.uniform draws in
// dict order (:101-102), the AR(1) blend p = 0.9 prev + (1 - 0.9) draw (:105-109), for i > 0 the
// spot walk spot *= 1 + np.random.normal(0.0003, 0.01) (:112-116), 15 calls priced at N = 128
// (:123-138), market = price + np.random.normal(0, 0.02) * price (:141-142), the relative-MSE
// loss (:154-157).  Bit for bit the reference's values: the only host work left is the serial
// part of NumPy's legacy stream (dh_gen_rng.h: the MT19937 twister and the walk over the polar
// acceptances, which give every sample its first double); per 65,536-sample chunk the device
//   gen_words_kernel   re-creates the stream's tempered words from the twister's block keys
//                      (one workgroup per 64 generations, the twist in LDS in three phases),
//   gen_draw_kernel    one thread per sample: its uniforms, its accepted polar pairs and their
//                      gauss values (glibc's log restated, dh_legacy_gauss.h), the spot return
//                      and the noise draws, in the reference's call order,
//   gen_ar1_kernel     the AR(1) blend in parallel segments: each (segment, parameter) thread
//                      starts kAr1Warm samples early from an arbitrary value -- the map is a 0.9
//                      contraction, so its fp64 iterates meet the true chain's bit for bit well
//                      within the warm-up (<= 418 steps measured) -- and records the value at
//                      its segment's start; block 0 runs the spot walk (not contracting) serially,
//   gen_fix_kernel     checks every segment's recorded value against its predecessor's last
//                      value (both final by induction) and re-runs a segment serially from the
//                      true value where they differ, so the result is the sequential chain's
//                      whatever the warm-up did,
//   pricing            the grid's surface (cos_gen_kernel / fused, exactly the host API's
//                      chunks, so the same launches and bits as dh_surface_price_cols),
//   gen_assemble_kernel  market, loss (np.mean's pairwise order), absolute strikes,
// and three streams overlap the chunk's draw, its pricing and the copies of its rows to the
// caller's (page-locked, dh_host_alloc) arrays with the host walk of the next chunk.
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <thread>

#include "dh_gen_rng.h"
#include "dh_legacy_gauss.h"

namespace {

constexpr int64_t kGenChunk = 1 << 16;      // samples per device chunk (= the host API's chunks)
constexpr int kAr1Seg = 256;                // samples per AR(1) segment
constexpr int kAr1Warm = 1024;              // warm-up samples of a segment's chain
constexpr int kGenMaxOpt = 128;             // options per sample the assembly kernel takes

struct GenDrawArgs {
    double lo[13], range[13];
    double ret_mu, ret_sigma, noise_sigma, entry_gauss;
    int n_opt;
};

// MT19937's twist of the key in LDS by one wave (LegacyRng::twist's recurrence): i < 227 reads
// old words only; 227 <= i < 454 reads words the first phase wrote; 454 <= i < 623 and i = 623
// read words of the second phase (and, for 623, the first).  Per phase every lane reads all its
// operands, then writes: a wave's LDS operations complete in order, and the compiler barriers
// (wave_sync) keep it from moving a read of another lane's word across a write.
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

__device__ __forceinline__ void wave_sync() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// element i of the twist: k[i] = k[i + 397 mod 624] ^ mix(k[i], k[i + 1 mod 624]) -- the same
// formula for i = 623 (k[396], k[0])
__device__ __forceinline__ uint32_t mt_elem(const uint32_t* k, int i) {
    const int src = i < 227 ? i + 397 : i - 227;
    const int nxt = i == 623 ? 0 : i + 1;
    return k[src] ^ mt_mix(k[i], k[nxt]);
}

// one phase of the twist over elements [lo, lo + len): every lane reads all its operands first
// (indices clamped into the phase, so the reads are branch-free), then writes its own elements
template <int Q>
__device__ __forceinline__ void mt_phase(uint32_t* k, int lane, int lo, int len) {
    uint32_t v[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int e = lane + 64 * q;
        v[q] = mt_elem(k, lo + (e < len ? e : len - 1));
    }
    wave_sync();
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int e = lane + 64 * q;
        if (q < Q - 1 || e < len) k[lo + e] = v[q];
    }
    wave_sync();
}

// MT19937's twist in LDS by one wave: [0, 227) reads old words only, [227, 454) the first phase's
// words, [454, 624) the second phase's (and, for 623, the first's)
__device__ __forceinline__ void mt_twist_wave(uint32_t* k, int lane) {
    mt_phase<4>(k, lane, 0, 227);
    mt_phase<4>(k, lane, 227, 227);
    mt_phase<3>(k, lane, 454, 170);
}

// The stream's tempered words of blocks [b0, b0 + gridDim.x), one wave per block: word w of the
// stream is key word (pos0 + w) % 624 of generation (pos0 + w) / 624 (dh_gen_rng.h); words >=
// n_words are not kept.
__global__ __launch_bounds__(64) void gen_words_kernel(const uint32_t* __restrict__ keys,
                                                       int64_t b0, int pos0, int64_t n_words,
                                                       uint32_t* __restrict__ W) {
    __shared__ uint32_t k[dhgen::kMtWords];
    const int lane = threadIdx.x;
    const int64_t b = b0 + blockIdx.x;
    const uint32_t* src = keys + b * dhgen::kMtWords;
    for (int j = lane; j < dhgen::kMtWords; j += 64) k[j] = src[j];
    wave_sync();
    for (int gi = 0; gi < dhgen::kGensPerBlock; ++gi) {
        const int64_t base = (b * dhgen::kGensPerBlock + gi) * dhgen::kMtWords - pos0;
        if (base >= n_words) break;
        if (gi > 0) mt_twist_wave(k, lane);
        if (base >= 0 && base + dhgen::kMtWords <= n_words) {
#pragma unroll
            for (int q = 0; q < 10; ++q) {
                const int j = lane + 64 * q;
                if (q < 9 || j < dhgen::kMtWords) W[base + j] = dhlog::mt_temper(k[j]);
            }
        } else {
            for (int j = lane; j < dhgen::kMtWords; j += 64) {
                const int64_t w = base + j;
                if (w >= 0 && w < n_words) W[w] = dhlog::mt_temper(k[j]);
            }
        }
    }
}

// One thread per sample i in [i0, i1): the draws of synthetic_generator.py:100-102, :112-116,
// :141 in their order, from the sample's first double T[i] (the host walk's record) and the
// source of the gauss value cached at its start (CS[i]: a pair's first double, -1 the entry's
// value, -2 none).  praw [n][13] raw uniforms; mret [n] 1 + the spot return (i > 0); noise
// [n][n_opt] = 0.0 + 0.02 g.  bad[0] is set if a sample's accepted pairs do not end at T[i + 1]
// (the walk's record; never expected).
__global__ __launch_bounds__(256) void gen_draw_kernel(const uint32_t* __restrict__ W,
                                                       const int64_t* __restrict__ T,
                                                       const int64_t* __restrict__ CS, int64_t i0,
                                                       int64_t i1, GenDrawArgs a,
                                                       double* __restrict__ praw,
                                                       double* __restrict__ mret,
                                                       double* __restrict__ noise,
                                                       int* __restrict__ bad) {
#pragma clang fp contract(off)
    const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= i1) return;
    auto D = [&](int64_t t) { return dhlog::mt_double(W[2 * t], W[2 * t + 1]); };
    int64_t tc = T[i];
    const int64_t tend = T[i + 1];
    double* p = praw + i * 13;
    for (int j = 0; j < 13; ++j) p[j] = a.lo[j] + a.range[j] * D(tc + j);       // :100-102
    tc += 13;
    const int64_t cs = CS[i];
    int hg = cs != -2;
    double cached = 0.0;
    if (cs == -1) {
        cached = a.entry_gauss;
    } else if (cs >= 0) {
        double x1, x2, r2, gn;
        dhlog::polar_pair(D(cs), D(cs + 1), x1, x2, r2);
        dhlog::gauss_values(x1, x2, r2, gn, cached);
    }
    const int c00 = i > 0 ? 1 : 0;
    const int calls = a.n_opt + c00;
    double* z = noise + i * a.n_opt;
    bool ok = true;
    for (int c = 0; c < calls; ++c) {
        double g;
        if (hg) {
            g = cached;
            hg = 0;
        } else {
            double x1 = 0.0, x2 = 0.0, r2 = 0.5;
            bool acc = false;
            while (tc + 2 <= tend) {
                acc = dhlog::polar_pair(D(tc), D(tc + 1), x1, x2, r2);
                tc += 2;
                if (acc) break;
            }
            ok = ok && acc;
            dhlog::gauss_values(x1, x2, r2, g, cached);
            hg = 1;
        }
        if (c < c00)
            mret[i] = 1.0 + (a.ret_mu + a.ret_sigma * g);                   // :112-116
        else
            z[c - c00] = 0.0 + a.noise_sigma * g;                            // :141
    }
    if (i == 0) mret[0] = 1.0;
    if (!ok || tc != tend) atomicOr(bad, 1);
}

// The AR(1) blend in segments of kAr1Seg samples (thread = (segment, parameter), segments
// numbered from sample 0).  A segment starting at s0
// runs the blend from s0 - kAr1Warm (from an arbitrary start: the raw draw before it) and records
// its value at s0 - 1 in chk[seg][j]; gen_fix_kernel checks it.  Loads run kPre steps ahead of
// the chain (a ring of registers), so the chain waits on the fp64 latency, not on memory.
constexpr int kPre = 32;

__device__ __forceinline__ double ld_or(const double* p, int64_t i, int64_t stride, int64_t off,
                                        int64_t end) {
    return i < end ? p[i * stride + off] : 0.0;
}

// v <- alpha v + beta x_i over i in [a, b), x_i = praw[i * 13 + j]; out (if set) gets every value
__device__ double ar1_run(const double* __restrict__ praw, int j, int64_t a, int64_t b, double v,
                          double alpha, double beta, double* __restrict__ params,
                          double* __restrict__ rec) {
#pragma clang fp contract(off)
    double buf[kPre];
#pragma unroll
    for (int q = 0; q < kPre; ++q) buf[q] = ld_or(praw, a + q, 13, j, b);
    for (int64_t i = a; i < b; i += kPre) {
#pragma unroll
        for (int q = 0; q < kPre; ++q) {
            const double x = buf[q];
            buf[q] = ld_or(praw, i + kPre + q, 13, j, b);
            if (i + q < b) {
                v = alpha * v + beta * x;                            // :105-109
                if (params) {
                    params[(i + q) * 13 + j] = v;
                    rec[(i + q) * DH_PARAM_STRIDE + j] = v;
                }
            }
        }
    }
    return v;
}

// The spot walk (:112-116) spot_i = spot_{i-1} (1 + ret_i) over [i0, i1), serial: lane 0 of one
// wave runs the chain, one dependent v_mul_f64 per sample, on the batch's 64 multipliers staged in
// LDS, and leaves each value in LDS; the wave then stores the batch with one coalesced store.  The
// multipliers are loaded by the whole wave kSpotAhead batches ahead (a register ring), so the
// chain never waits on memory.  The multiplier of sample 0 is 1.0 (gen_draw_kernel), which keeps
// spot0; loads past i1 are clamped (their products are not stored).
constexpr int kSpotAhead = 8;

__global__ __launch_bounds__(64) void gen_spot_kernel(const double* __restrict__ mret, int64_t i0,
                                                      int64_t i1, double spot0, double r,
                                                      double* __restrict__ carry_spot,
                                                      double* __restrict__ spots,
                                                      double* __restrict__ rec) {
#pragma clang fp contract(off)
    __shared__ double mv[64];
    __shared__ double sv[64];
    // the chain shares its SIMD with the pricing kernel's waves of the chunk before: top issue
    // priority, so that its one dependent multiply per sample issues as soon as it is ready
    __builtin_amdgcn_s_setprio(3);
    const int lane = threadIdx.x;
    const int64_t last = i1 - 1;
    double s = i0 == 0 ? spot0 : carry_spot[0];
    double ring[kSpotAhead];
#pragma unroll
    for (int k = 0; k < kSpotAhead; ++k) {
        const int64_t i = i0 + 64 * k + lane;
        ring[k] = mret[i < last ? i : last];
    }
    for (int64_t base = i0; base < i1; base += 64 * kSpotAhead) {
#pragma unroll
        for (int k = 0; k < kSpotAhead; ++k) {
            const int64_t b = base + 64 * k;
            const double m = ring[k];
            const int64_t ia = b + 64 * kSpotAhead + lane;
            ring[k] = mret[ia < last ? ia : last];
            if (b < i1) {
                const int nb = i1 - b < 64 ? (int)(i1 - b) : 64;
                mv[lane] = m;
                wave_sync();
                if (lane == 0) {
                    double ml[64];                    // all 64 reads issued ahead of the chain
#pragma unroll
                    for (int l = 0; l < 64; ++l) ml[l] = mv[l];
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    double v = s, out[64];        // the chain alone, then the 64 stores
#pragma unroll
                    for (int l = 0; l < 64; ++l) {
                        v = v * ml[l];
                        out[l] = v;
                    }
#pragma unroll
                    for (int l = 0; l < 64; ++l) sv[l] = out[l];
                }
                wave_sync();
                const double out = sv[lane];
                s = sv[nb - 1];
                if (lane < nb) {
                    const int64_t i = b + lane;
                    spots[i] = out;
                    rec[i * DH_PARAM_STRIDE + 13] = out;
                    rec[i * DH_PARAM_STRIDE + 14] = r;
                    rec[i * DH_PARAM_STRIDE + 15] = 0.0;
                }
                wave_sync();
            }
        }
    }
    if (lane == 0) carry_spot[0] = s;
}

__global__ __launch_bounds__(64) void gen_ar1_kernel(const double* __restrict__ praw,
                                                     int64_t i0, int64_t i1, double alpha,
                                                     double beta, double* __restrict__ params,
                                                     double* __restrict__ rec,
                                                     double* __restrict__ chk) {
#pragma clang fp contract(off)
    const int64_t u = (int64_t)blockIdx.x * 64 + threadIdx.x;
    const int64_t seg0 = i0 / kAr1Seg;
    const int64_t seg = seg0 + u / 13;
    const int j = (int)(u % 13);
    const int64_t s0 = seg * kAr1Seg > i0 ? seg * kAr1Seg : i0;
    const int64_t s1 = (seg + 1) * kAr1Seg < i1 ? (seg + 1) * kAr1Seg : i1;
    if (s0 >= s1) return;
    const int64_t w0 = s0 - kAr1Warm;
    double v;
    if (w0 <= 0) {                         // the true chain from sample 0 (nothing to check)
        v = ar1_run(praw, j, 1, s0, praw[j], alpha, beta, nullptr, nullptr);
        chk[(seg - seg0) * 13 + j] = NAN;
        if (s0 == 0) {                     // sample 0: the draw itself (:105 applies for i > 0)
            params[j] = v;
            rec[j] = v;
            ar1_run(praw, j, 1, s1, v, alpha, beta, params, rec);
            return;
        }
    } else {
        // an arbitrary start (the raw draw before the warm-up): the contraction forgets it
        v = ar1_run(praw, j, w0, s0, praw[(w0 - 1) * 13 + j], alpha, beta, nullptr, nullptr);
        chk[(seg - seg0) * 13 + j] = v;     // the warm chain's value at s0 - 1
    }
    ar1_run(praw, j, s0, s1, v, alpha, beta, params, rec);
}

// One block: every (segment, parameter) of [i0, i1) compares its warm chain's value at its
// start with the final value of the sample before it (both final by induction, the previous
// chunk's included); if any differs, lane j re-runs parameter j serially from the first segment
// that differs to the chunk's end (never seen; bad[1] counts the differing segments).
__global__ __launch_bounds__(256) void gen_fix_kernel(const double* __restrict__ praw,
                                                      int64_t i0, int64_t i1, double alpha,
                                                      double beta, const double* __restrict__ chk,
                                                      double* __restrict__ params,
                                                      double* __restrict__ rec,
                                                      int* __restrict__ bad) {
#pragma clang fp contract(off)
    __shared__ int first_bad[13];
    const int tid = threadIdx.x;
    if (tid < 13) first_bad[tid] = 0x7fffffff;
    __syncthreads();
    const int64_t seg0 = i0 / kAr1Seg;
    const int64_t n_seg = (i1 - 1) / kAr1Seg - seg0 + 1;
    for (int64_t u = tid; u < n_seg * 13; u += 256) {
        const int64_t seg = seg0 + u / 13;
        const int j = (int)(u % 13);
        const int64_t s0 = seg * kAr1Seg > i0 ? seg * kAr1Seg : i0;
        if (s0 == 0) continue;
        const double got = chk[(seg - seg0) * 13 + j];
        if (isnan(got) || got == params[(s0 - 1) * 13 + j]) continue;
        atomicAdd(bad + 1, 1);
        atomicMin(first_bad + j, (int)(seg - seg0));
    }
    __syncthreads();
    if (tid >= 13 || first_bad[tid] == 0x7fffffff) return;
    const int j = tid;
    const int64_t seg = seg0 + first_bad[j];
    const int64_t s0 = seg * kAr1Seg > i0 ? seg * kAr1Seg : i0;
    ar1_run(praw, j, s0, i1, params[(s0 - 1) * 13 + j], alpha, beta, params, rec);
}

// Per sample: market = model + noise * model (:141-142), loss = mean(((model - market) /
// market)^2) as np.mean forms it (NumPy 2's pairwise add.reduce: plain below 8 terms, eight
// accumulators up to 128, then one division), strikes = (K_rel * spot) / 100.
__global__ __launch_bounds__(256) void gen_assemble_kernel(const double* __restrict__ model,
                                                           const double* __restrict__ noise,
                                                           const double* __restrict__ spots,
                                                           const double* __restrict__ k_rel,
                                                           int n_opt, int64_t i0, int64_t i1,
                                                           double* __restrict__ market,
                                                           double* __restrict__ loss,
                                                           double* __restrict__ strikes) {
#pragma clang fp contract(off)
    const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= i1) return;
    const double* md = model + i * n_opt;
    const double* nz = noise + i * n_opt;
    double* mk = market + i * n_opt;
    double* st = strikes + i * n_opt;
    const double spot = spots[i];
    auto sq = [&](int j) {
        const double m = md[j];
        const double v = m + nz[j] * m;
        mk[j] = v;
        st[j] = (k_rel[j] * spot) / 100.0;
        const double rr = (m - v) / v;
        return rr * rr;
    };
    double res;
    if (n_opt < 8) {
        res = 0.0;
        for (int j = 0; j < n_opt; ++j) res += sq(j);
    } else {
        double acc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = sq(q);
        int j = 8;
        const int n8 = n_opt - n_opt % 8;
        for (; j < n8; j += 8) {
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] += sq(j + q);
        }
        res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
        for (; j < n_opt; ++j) res += sq(j);
    }
    loss[i] = res / (double)n_opt;
}

// The trading dates (synthetic_generator.py:59-67): weekdays from first_day (a Monday), as the
// 10 UCS-4 code points of 'YYYY-MM-DD' per sample (dh_gen_dates' arithmetic)
__global__ __launch_bounds__(256) void gen_dates_kernel(int64_t first_day, int64_t i0, int64_t i1,
                                                        uint32_t* __restrict__ out) {
    const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= i1) return;
    int64_t z = first_day + 7 * (i / 5) + i % 5 + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    const int d = (int)(doy - (153 * mp + 2) / 5 + 1);
    const int m = (int)(mp < 10 ? mp + 3 : mp - 9);
    const int64_t y = yoe + era * 400 + (m <= 2);
    uint32_t* c = out + i * 10;
    c[0] = '0' + (uint32_t)(y / 1000);
    c[1] = '0' + (uint32_t)(y / 100 % 10);
    c[2] = '0' + (uint32_t)(y / 10 % 10);
    c[3] = '0' + (uint32_t)(y % 10);
    c[4] = '-';
    c[5] = '0' + (uint32_t)(m / 10);
    c[6] = '0' + (uint32_t)(m % 10);
    c[7] = '-';
    c[8] = '0' + (uint32_t)(d / 10);
    c[9] = '0' + (uint32_t)(d % 10);
}

// glibc's log over an array (the restatement's GPU test, dh_gen_log)
__global__ __launch_bounds__(256) void glibc_log_kernel(const double* __restrict__ x, int64_t n,
                                                        double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = dhlog::glibc_log(x[i]);
}

}  // namespace

// Device and page-locked buffers of the device draw, kept on the context between calls
// (grow-only)
struct GenBufs {
    HostBuf h_t, h_cs, h_keys;              // the host walk's records and the twister's keys
    DevBuf W, t, cs, keys, praw, mret, noise, params, spots, rec, model, market, loss, strikes,
        dates, chk, carry, bad;
    hipStream_t s_price = nullptr, s_copy = nullptr, s_spot = nullptr;
    std::vector<hipEvent_t> ev;             // 2 per chunk in flight
    void release() {
        for (HostBuf* b : {&h_t, &h_cs, &h_keys}) b->release();
        for (DevBuf* b : {&W, &t, &cs, &keys, &praw, &mret, &noise, &params, &spots, &rec, &model,
                          &market, &loss, &strikes, &dates, &chk, &carry, &bad})
            b->release();
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        ev.clear();
        for (hipStream_t st : {s_price, s_copy, s_spot})
            if (st) (void)hipStreamDestroy(st);
        s_price = s_copy = s_spot = nullptr;
    }
};

void gen_bufs_release(dh_ctx* ctx) {
    if (ctx && ctx->gen) {
        ctx->gen->release();
        delete ctx->gen;
        ctx->gen = nullptr;
    }
}

namespace {

// A page-locked host allocator with a cache (dh_host_alloc / dh_host_free): the generator's
// outputs are ~480 B per sample, and fresh pageable arrays cost their first touch (~1 us per 4 KB
// page) on top of staged copies; cached page-locked blocks take the device's copies by DMA and are
// reused by the next call of the same size.
struct HostCache {
    std::mutex mu;
    std::multimap<size_t, void*> free_blocks;       // size -> block
    std::map<void*, size_t> size_of;                 // every live or cached block
};
HostCache& host_cache() {
    static HostCache* c = new HostCache();           // never destroyed (arrays may outlive exit)
    return *c;
}

int wait_located(dhgen::Located& L, int64_t need) {
    for (;;) {
        if (L.located.load(std::memory_order_acquire) >= need) return 1;
        const int st = L.state.load(std::memory_order_acquire);
        if (st < 0) return 0;
        if (st > 0 && L.located.load(std::memory_order_acquire) < need) return 0;
        std::this_thread::yield();
    }
}

}  // namespace

extern "C" {

int dh_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(DH_E_ARG, "out is null");
    *out = nullptr;
    if (bytes == 0) return fail(DH_E_ARG, "zero bytes");
    HostCache& c = host_cache();
    {
        std::lock_guard<std::mutex> l(c.mu);
        auto it = c.free_blocks.lower_bound(bytes);
        if (it != c.free_blocks.end() && it->first <= bytes + bytes / 4) {
            *out = it->second;
            c.free_blocks.erase(it);
            return DH_OK;
        }
    }
    const size_t want = (bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        // drop the cache and try once more
        {
            std::lock_guard<std::mutex> l(c.mu);
            for (auto& kv : c.free_blocks) {
                (void)hipHostFree(kv.second);
                c.size_of.erase(kv.second);
            }
            c.free_blocks.clear();
        }
        e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return fail(DH_E_ALLOC, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        }
    }
    std::lock_guard<std::mutex> l(c.mu);
    c.size_of[p] = want;
    *out = p;
    return DH_OK;
}

int dh_host_free(void* p) {
    if (!p) return DH_OK;
    HostCache& c = host_cache();
    std::lock_guard<std::mutex> l(c.mu);
    auto it = c.size_of.find(p);
    if (it == c.size_of.end()) return fail(DH_E_ARG, "not a dh_host_alloc block");
    c.free_blocks.emplace(it->second, p);
    return DH_OK;
}

int dh_host_cache_trim(void) {
    HostCache& c = host_cache();
    std::lock_guard<std::mutex> l(c.mu);
    for (auto& kv : c.free_blocks) {
        (void)hipHostFree(kv.second);
        c.size_of.erase(kv.second);
    }
    c.free_blocks.clear();
    return DH_OK;
}

int dh_gen_log(dh_ctx* ctx, const double* x, int64_t n, double* out) {
    if (!ctx || n < 0 || (n > 0 && (!x || !out))) return fail(DH_E_ARG, "null argument");
    if (n == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    HIP_TRY(ctx->aux0.reserve((size_t)n * 8));
    HIP_TRY(ctx->aux1.reserve((size_t)n * 8));
    HIP_TRY(hipMemcpyAsync(ctx->aux0.ptr, x, (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(glibc_log_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ctx->stream, (const double*)ctx->aux0.ptr, n, (double*)ctx->aux1.ptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->aux1.ptr, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return DH_OK;
}

int dh_gen_device(dh_ctx* ctx, const dh_surface* grid, uint32_t* mt_key, int32_t* mt_pos,
                  int32_t* has_gauss, double* cached_gauss, int64_t n_samples, const double* lo,
                  const double* hi, double alpha, double spot0, double ret_mu, double ret_sigma,
                  double noise_sigma, double r, int N, double L, const double* k_rel,
                  int64_t first_day, double* params, double* spots, double* market,
                  double* model, double* loss, double* strikes, uint32_t* dates, double* stats) {
    const double t_start = std::chrono::duration<double>(
        std::chrono::steady_clock::now().time_since_epoch()).count();
    auto now = [&] {
        return std::chrono::duration<double>(
                   std::chrono::steady_clock::now().time_since_epoch()).count() - t_start;
    };
    if (!ctx || !grid || !mt_key || !mt_pos || !has_gauss || !cached_gauss || !lo || !hi ||
        !k_rel)
        return fail(DH_E_ARG, "null argument");
    if (n_samples < 0) return fail(DH_E_ARG, "n_samples < 0");
    if (*mt_pos < 0 || *mt_pos > dhgen::kMtWords) return fail(DH_E_ARG, "bad MT19937 position");
    const int n_opt = grid->M;
    if (n_opt < 1 || n_opt > kGenMaxOpt)
        return fail(DH_E_ARG, "dh_gen_device: the grid must have 1 .. 128 options");
    if (grid->strike_mode != DH_STRIKE_PCT_SPOT)
        return fail(DH_E_ARG, "dh_gen_device: the grid's strikes must be percentages of the spot");
    int rc = check_N(N);
    if (rc) return rc;
    if (n_samples > 0 &&
        (!params || !spots || !market || !model || !loss || !strikes))
        return fail(DH_E_ARG, "null output");
    if (n_samples == 0) return DH_OK;
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.rc) return dev_scope.rc;
    if (!ctx->gen) ctx->gen = new GenBufs();
    GenBufs& G = *ctx->gen;
    if (!G.s_price) HIP_TRY(hipStreamCreateWithFlags(&G.s_price, hipStreamNonBlocking));
    if (!G.s_copy) HIP_TRY(hipStreamCreateWithFlags(&G.s_copy, hipStreamNonBlocking));
    if (!G.s_spot) {
        // the spot walk is the pipeline's serial chain: a high-priority stream, which also puts it
        // on a hardware queue of its own (not behind the copies of the stream sharing a queue)
        int lo_prio = 0, hi_prio = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
        HIP_TRY(hipStreamCreateWithPriority(&G.s_spot, hipStreamNonBlocking, hi_prio));
    }

    // the host part: twister, bit workers, walk (on their own threads from here on)
    std::unique_ptr<dhgen::Located> Lp(new dhgen::Located());
    dhgen::Located& Lc = *Lp;
    std::memcpy(Lc.key, mt_key, sizeof(Lc.key));
    Lc.pos = *mt_pos;
    Lc.has_gauss = *has_gauss ? 1 : 0;
    Lc.gauss = *cached_gauss;
    Lc.n = n_samples;
    Lc.n_opt = n_opt;
    dhgen::locate_geometry(Lc);
    const int64_t n = n_samples, M = n_opt;
    const int64_t n_words = 2 * Lc.max_t + 2;
    const int64_t n_seg_chunk = kGenChunk / kAr1Seg + 1;
    HIP_TRY(G.h_t.reserve((size_t)(n + 1) * 8));
    HIP_TRY(G.h_cs.reserve((size_t)n * 8));
    HIP_TRY(G.h_keys.reserve((size_t)Lc.max_blocks * dhgen::kMtWords * 4));
    HIP_TRY(G.W.reserve((size_t)n_words * 4));
    HIP_TRY(G.t.reserve((size_t)(n + 1) * 8));
    HIP_TRY(G.cs.reserve((size_t)n * 8));
    HIP_TRY(G.keys.reserve((size_t)Lc.max_blocks * dhgen::kMtWords * 4));
    HIP_TRY(G.praw.reserve((size_t)n * 13 * 8));
    HIP_TRY(G.params.reserve((size_t)n * 13 * 8));
    HIP_TRY(G.mret.reserve((size_t)(n + 64) * 8));     // gen_spot_kernel reads 64 past the end
    HIP_TRY(G.spots.reserve((size_t)n * 8));
    HIP_TRY(G.noise.reserve((size_t)n * M * 8));
    HIP_TRY(G.rec.reserve((size_t)n * DH_PARAM_STRIDE * 8));
    HIP_TRY(G.model.reserve((size_t)n * M * 8));
    HIP_TRY(G.market.reserve((size_t)n * M * 8));
    HIP_TRY(G.strikes.reserve((size_t)n * M * 8));
    HIP_TRY(G.loss.reserve((size_t)n * 8));
    if (dates) HIP_TRY(G.dates.reserve((size_t)n * 10 * 4));
    HIP_TRY(G.chk.reserve((size_t)n_seg_chunk * 13 * 8 * 2));
    HIP_TRY(G.carry.reserve(64));
    HIP_TRY(G.bad.reserve(64));
    const double* d_krel = nullptr;
    HIP_TRY(ctx->aux3.reserve((size_t)M * 8));
    d_krel = (const double*)ctx->aux3.ptr;
    hipStream_t s_draw = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->aux3.ptr, k_rel, (size_t)M * 8, hipMemcpyHostToDevice, s_draw));
    HIP_TRY(hipMemsetAsync(G.bad.ptr, 0, 64, s_draw));
    const int64_t n_chunks = (n + kGenChunk - 1) / kGenChunk;
    while ((int64_t)G.ev.size() < 8) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        G.ev.push_back(e);
    }
    Lc.t = (int64_t*)G.h_t.ptr;
    Lc.cs = (int64_t*)G.h_cs.ptr;
    Lc.keys = (uint32_t*)G.h_keys.ptr;

    GenDrawArgs ga{};
    for (int j = 0; j < 13; ++j) {
        ga.lo[j] = lo[j];
        ga.range[j] = hi[j] - lo[j];
    }
    ga.ret_mu = ret_mu;
    ga.ret_sigma = ret_sigma;
    ga.noise_sigma = noise_sigma;
    ga.entry_gauss = *cached_gauss;
    ga.n_opt = n_opt;
    const double beta = 1.0 - alpha;                         // (1 - alpha), :108

    std::thread walker([&Lc] { dhgen::locate_run(Lc); });
    bool joined = false;
    auto join = [&] {
        if (!joined) {
            walker.join();
            joined = true;
        }
    };
    int err = DH_OK;
    std::string err_msg;
    int64_t blocks_sent = 0;
    double t_first = -1.0, t_walk_end = -1.0;
    uint32_t* d_keys = (uint32_t*)G.keys.ptr;
    int64_t* d_t = (int64_t*)G.t.ptr;
    int64_t* d_cs = (int64_t*)G.cs.ptr;
    double* d_chk = (double*)G.chk.ptr;
    int* d_bad = (int*)G.bad.ptr;
    auto bail = [&](int code, const std::string& m) {
        if (err == DH_OK) {
            err = code;
            err_msg = m;
        }
    };
#define GEN_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) {                                                                \
            bail(DH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));                \
            break;                                                                             \
        }                                                                                      \
    } while (0)
    for (int64_t c = 0; c < n_chunks && err == DH_OK; ++c) {
        const int64_t c0 = c * kGenChunk, c1 = std::min(n, c0 + kGenChunk), nc = c1 - c0;
        if (!wait_located(Lc, c1 + 1)) {
            bail(DH_E_ARG, "dh_gen_device: the walk passed its stream bound");
            break;
        }
        if (t_first < 0) t_first = now();
        const int64_t* h_t = (const int64_t*)G.h_t.ptr;
        // blocks whose words the chunk reads: up to the word before double T[c1]
        const int64_t last_word = Lc.pos0 + 2 * h_t[c1];
        const int64_t need = std::min(Lc.max_blocks, last_word / ((int64_t)dhgen::kGensPerBlock *
                                                                  dhgen::kMtWords) + 1);
        for (;;) {
            if (Lc.keys_ready.load(std::memory_order_acquire) >= need) break;
            if (Lc.state.load(std::memory_order_acquire) != 0) {
                join();
                dhgen::locate_extend_keys(Lc, need);
                break;
            }
            std::this_thread::yield();
        }
        hipEvent_t ev_drawn = G.ev[(4 * c) % 8], ev_priced = G.ev[(4 * c + 1) % 8];
        hipEvent_t ev_raw = G.ev[(4 * c + 2) % 8], ev_spot = G.ev[(4 * c + 3) % 8];
        if (need > blocks_sent) {
            GEN_TRY(hipMemcpyAsync(d_keys + blocks_sent * dhgen::kMtWords,
                                   (const uint32_t*)G.h_keys.ptr + blocks_sent * dhgen::kMtWords,
                                   (size_t)(need - blocks_sent) * dhgen::kMtWords * 4,
                                   hipMemcpyHostToDevice, s_draw));
            hipLaunchKernelGGL(gen_words_kernel, dim3((unsigned)(need - blocks_sent)), dim3(64),
                               0, s_draw, (const uint32_t*)d_keys, blocks_sent, Lc.pos0, n_words,
                               (uint32_t*)G.W.ptr);
            GEN_TRY(hipGetLastError());
            blocks_sent = need;
        }
        if (err) break;
        GEN_TRY(hipMemcpyAsync(d_t + c0, h_t + c0, (size_t)(nc + 1) * 8, hipMemcpyHostToDevice,
                               s_draw));
        GEN_TRY(hipMemcpyAsync(d_cs + c0, (const int64_t*)G.h_cs.ptr + c0, (size_t)nc * 8,
                               hipMemcpyHostToDevice, s_draw));
        if (err) break;
        const unsigned nb = (unsigned)((nc + 255) / 256);
        hipLaunchKernelGGL(gen_draw_kernel, dim3(nb), dim3(256), 0, s_draw, (const uint32_t*)G.W.ptr,
                           (const int64_t*)d_t, (const int64_t*)d_cs, c0, c1, ga,
                           (double*)G.praw.ptr, (double*)G.mret.ptr, (double*)G.noise.ptr, d_bad);
        GEN_TRY(hipGetLastError());
        const int64_t segs = (c1 - 1) / kAr1Seg - c0 / kAr1Seg + 1;
        double* chk = d_chk + (c & 1) * n_seg_chunk * 13;
        // the spot walk on its own stream (one wave, serial), beside the AR(1) segments
        GEN_TRY(hipEventRecord(ev_raw, s_draw));
        GEN_TRY(hipStreamWaitEvent(G.s_spot, ev_raw, 0));
        hipLaunchKernelGGL(gen_spot_kernel, dim3(1), dim3(64), 0, G.s_spot,
                           (const double*)G.mret.ptr, c0, c1, spot0, r, (double*)G.carry.ptr,
                           (double*)G.spots.ptr, (double*)G.rec.ptr);
        GEN_TRY(hipGetLastError());
        GEN_TRY(hipEventRecord(ev_spot, G.s_spot));
        hipLaunchKernelGGL(gen_ar1_kernel, dim3((unsigned)((segs * 13 + 63) / 64)), dim3(64), 0,
                           s_draw, (const double*)G.praw.ptr, c0, c1, alpha, beta,
                           (double*)G.params.ptr, (double*)G.rec.ptr, chk);
        GEN_TRY(hipGetLastError());
        hipLaunchKernelGGL(gen_fix_kernel, dim3(1), dim3(256), 0, s_draw, (const double*)G.praw.ptr,
                           c0, c1, alpha, beta, (const double*)chk, (double*)G.params.ptr,
                           (double*)G.rec.ptr, d_bad);
        GEN_TRY(hipGetLastError());
        if (dates) {
            hipLaunchKernelGGL(gen_dates_kernel, dim3(nb), dim3(256), 0, s_draw, first_day, c0, c1,
                               (uint32_t*)G.dates.ptr);
            GEN_TRY(hipGetLastError());
        }
        GEN_TRY(hipEventRecord(ev_drawn, s_draw));
        GEN_TRY(hipStreamWaitEvent(G.s_price, ev_drawn, 0));
        GEN_TRY(hipStreamWaitEvent(G.s_price, ev_spot, 0));
        if (err) break;
        const int prc = dh_surface_price_dev(ctx, grid,
                                             (const double*)G.rec.ptr + c0 * DH_PARAM_STRIDE, nc,
                                             N, L, (double*)G.model.ptr + c0 * M, G.s_price);
        if (prc) {
            bail(prc, g_err);
            break;
        }
        hipLaunchKernelGGL(gen_assemble_kernel, dim3(nb), dim3(256), 0, G.s_price,
                           (const double*)G.model.ptr, (const double*)G.noise.ptr,
                           (const double*)G.spots.ptr, d_krel, n_opt, c0, c1,
                           (double*)G.market.ptr, (double*)G.loss.ptr, (double*)G.strikes.ptr);
        GEN_TRY(hipGetLastError());
        GEN_TRY(hipEventRecord(ev_priced, G.s_price));
        GEN_TRY(hipStreamWaitEvent(G.s_copy, ev_priced, 0));
        if (err) break;
        struct Cp {
            void* dst;
            const void* src;
            size_t bytes;
        };
        const Cp cps[] = {
            {params + c0 * 13, (const double*)G.params.ptr + c0 * 13, (size_t)nc * 13 * 8},
            {spots + c0, (const double*)G.spots.ptr + c0, (size_t)nc * 8},
            {model + c0 * M, (const double*)G.model.ptr + c0 * M, (size_t)nc * M * 8},
            {market + c0 * M, (const double*)G.market.ptr + c0 * M, (size_t)nc * M * 8},
            {strikes + c0 * M, (const double*)G.strikes.ptr + c0 * M, (size_t)nc * M * 8},
            {loss + c0, (const double*)G.loss.ptr + c0, (size_t)nc * 8},
            {dates ? (void*)(dates + c0 * 10) : nullptr, (const uint32_t*)G.dates.ptr + c0 * 10,
             (size_t)nc * 40}};
        for (const Cp& cp : cps)
            if (cp.dst)
                GEN_TRY(hipMemcpyAsync(cp.dst, cp.src, cp.bytes, hipMemcpyDeviceToHost, G.s_copy));
        // two chunks in flight: the events of chunk c are reused by chunk c + 2
        if (c >= 1) GEN_TRY(hipEventSynchronize(G.ev[(4 * (c - 1) + 1) % 8]));
    }
#undef GEN_TRY
    join();
    t_walk_end = Lc.s_walk;
    if (err == DH_OK && Lc.state.load() != 1) bail(DH_E_ARG, "dh_gen_device: the walk failed");
    hipError_t e1 = hipStreamSynchronize(s_draw), e2 = hipStreamSynchronize(G.s_price),
               e3 = hipStreamSynchronize(G.s_copy), e4 = hipStreamSynchronize(G.s_spot);
    if (err != DH_OK) return fail(err, err_msg);
    HIP_TRY(e1);
    HIP_TRY(e2);
    HIP_TRY(e3);
    HIP_TRY(e4);
    int h_bad[2] = {0, 0};
    HIP_TRY(hipMemcpy(h_bad, G.bad.ptr, sizeof(h_bad), hipMemcpyDeviceToHost));
    if (h_bad[0]) return fail(DH_E_ARG, "dh_gen_device: a sample's pairs disagree with the walk");
    std::memcpy(mt_key, Lc.key_end, sizeof(Lc.key_end));
    *mt_pos = Lc.pos_end;
    *has_gauss = Lc.has_gauss_end;
    *cached_gauss = Lc.gauss_end;
    if (stats) {
        stats[0] = Lc.s_twister;     // seconds from the call's start (within a few us)
        stats[1] = t_walk_end;
        stats[2] = t_first;
        stats[3] = now();
        stats[4] = (double)h_bad[1];   // AR(1) segments re-run serially
        stats[5] = (double)Lc.max_blocks;
        stats[6] = (double)blocks_sent;
        stats[7] = (double)n_chunks;
    }
    return DH_OK;
}

}  // extern "C"
