// dh_gen_rng.cpp -- host side of the generator batch path (dh_gen_draw, include/dhcos.h).
//
// The reference draws every random number of generate_synthetic_calibrations from NumPy's legacy
// global RandomState, one scalar call at a time (src/data/synthetic_generator.py:98-141):
//   per sample i: 13 x np.random.uniform(lo, hi) in dict order (:100-102), the AR(1) blend with
//   the previous sample (alpha = 0.9, :105-109), for i > 0 one np.random.normal(0.0003, 0.01)
//   spot return (:112-116), then one np.random.normal(0, 0.02) per option (:141).
// Pricing consumes no randomness, so the whole draw runs here, natively, and the GPU prices the
// samples afterwards.  To give the reference's numbers bit for bit this restates the generator
// NumPy's RandomState is built on (numpy/random/src/mt19937, legacy-distributions.c):
//   * MT19937 (Matsumoto & Nishimura): 624-word state, twist at pos == 624, tempering;
//   * legacy double: ((a >> 5) * 67108864 + (b >> 6)) / 2^53 from two 32-bit outputs;
//   * uniform(lo, hi) = lo + (hi - lo) * double;
//   * legacy gauss: polar Box-Muller, x = 2 d - 1 pairs until 0 < r2 < 1, f = sqrt(-2 log(r2) / r2),
//     returns f x2 and caches f x1 for the next call (has_gauss / gauss carry across calls);
//   * normal(loc, scale) = loc + scale * gauss.
// The caller passes NumPy's state (np.random.get_state()) in and sets the advanced state back,
// so the global stream continues exactly where the reference's loop would leave it.  No FMA
// contraction (the Makefile builds this file with -ffp-contract=off), libm log / sqrt as NumPy.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "dhcos.h"
#include "dh_gen_rng.h"

namespace {

constexpr int kMtN = 624;
constexpr int kMtM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7fffffffu;

struct LegacyRng {
    uint32_t key[kMtN];
    int pos;
    int has_gauss;
    double gauss;

    void twist() {
        int i = 0;
        uint32_t y;
        for (; i < kMtN - kMtM; ++i) {
            y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + kMtM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        }
        for (; i < kMtN - 1; ++i) {
            y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + (kMtM - kMtN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        }
        y = (key[kMtN - 1] & kUpper) | (key[0] & kLower);
        key[kMtN - 1] = key[kMtM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        pos = 0;
    }
    uint32_t next32() {
        if (pos == kMtN) twist();
        uint32_t y = key[pos++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    double next_double() {
        const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }
    double next_gauss() {
        if (has_gauss) {
            const double t = gauss;
            has_gauss = 0;
            gauss = 0.0;
            return t;
        }
        double f, x1, x2, r2;
        do {
            x1 = 2.0 * next_double() - 1.0;
            x2 = 2.0 * next_double() - 1.0;
            r2 = x1 * x1 + x2 * x2;
        } while (r2 >= 1.0 || r2 == 0.0);
        f = std::sqrt(-2.0 * std::log(r2) / r2);
        gauss = f * x1;
        has_gauss = 1;
        return f * x2;
    }
    double normal(double loc, double scale) { return loc + scale * next_gauss(); }

};

// The legacy doubles of an MT19937 stream a generation (624 words) at a time: the twist, the
// tempering and the (a >> 5, b >> 6) conversion run as straight loops over the generation (the
// compiler vectorises them) instead of a pos check per word.  While it runs, g.pos counts the
// words READ; sync() sets it to the words a word-at-a-time consumer of the same doubles would
// have taken, so the state handed back is the sequential loop's.
struct DoubleStream {
    LegacyRng& g;
    uint32_t w[kMtN + 1];
    double d[kMtN / 2 + 1];
    int n = 0, i = 0;                // doubles in d, the next one
    int s = 0, carry_in = 0;         // generation word d[] started at; d[0] took a carried word
    int has_cw = 0;                  // a tempered word read but not yet paired
    uint32_t cw = 0;
    bool filled = false;
    explicit DoubleStream(LegacyRng& g_) : g(g_) {}
    double next() {
        if (i == n) refill();
        return d[i++];
    }
    void refill() {
        do {
            if (g.pos == kMtN) g.twist();
            s = g.pos;
            carry_in = has_cw;
            int m = 0;
            if (has_cw) w[m++] = cw;
            const uint32_t* k = g.key + s;
            const int len = kMtN - s;
            for (int j = 0; j < len; ++j) {
                uint32_t y = k[j];
                y ^= (y >> 11);
                y ^= (y << 7) & 0x9d2c5680u;
                y ^= (y << 15) & 0xefc60000u;
                y ^= (y >> 18);
                w[m + j] = y;
            }
            m += len;
            g.pos = kMtN;
            n = m / 2;
            for (int j = 0; j < n; ++j) {
                const int32_t a = (int32_t)(w[2 * j] >> 5), b = (int32_t)(w[2 * j + 1] >> 6);
                d[j] = (a * 67108864.0 + b) / 9007199254740992.0;
            }
            has_cw = m & 1;
            if (has_cw) cw = w[m - 1];
            i = 0;
            filled = true;
        } while (n == 0);
    }
    void sync() {
        if (filled) g.pos = s + 2 * i - carry_in;
    }
    // The next k accepted polar pairs (next_gauss's do-while: x = 2 d - 1, rejected while
    // r2 >= 1 or r2 == 0) into x1 / x2 / r2.  The candidates of up to 16 buffered pairs are
    // tested together and the accepted ones taken by bit scan: no branch per rejection.
    void pairs(int k, double* x1, double* x2, double* r2) {
        int got = 0;
        while (got < k) {
            if (n - i < 2) {                        // a pair straddling a refill
                const double a = 2.0 * next() - 1.0, b = 2.0 * next() - 1.0;
                const double r = a * a + b * b;
                if (r < 1.0 && r != 0.0) {
                    x1[got] = a;
                    x2[got] = b;
                    r2[got] = r;
                    ++got;
                }
                continue;
            }
            const int m = std::min((n - i) / 2, 16);
            const double* q = d + i;
            uint32_t mask = 0;
            double ca[16], cb[16], cr[16];
            for (int j = 0; j < m; ++j) {
                ca[j] = 2.0 * q[2 * j] - 1.0;
                cb[j] = 2.0 * q[2 * j + 1] - 1.0;
                cr[j] = ca[j] * ca[j] + cb[j] * cb[j];
                mask |= (uint32_t)(cr[j] < 1.0 && cr[j] != 0.0) << j;
            }
            int used = m;
            while (mask) {
                const int j = __builtin_ctz(mask);
                mask &= mask - 1;
                x1[got] = ca[j];
                x2[got] = cb[j];
                r2[got] = cr[j];
                if (++got == k) {
                    used = j + 1;
                    break;
                }
            }
            i += 2 * used;
        }
    }
};

// next_gauss's arithmetic after the pair: (f x2, f x1), f = sqrt(-2 log(r2) / r2)
inline void pair_values(double x1, double x2, double r2, double& g_new, double& g_cached) {
    const double f = std::sqrt(-2.0 * std::log(r2) / r2);
    g_cached = f * x1;
    g_new = f * x2;
}

// A fixed team of worker threads for one dh_gen_draw call: run(f) calls f(0..n-1) once each,
// f(0) on the caller, and returns when all are done.
class Team {
  public:
    explicit Team(int n) : n_(n) {
        for (int w = 1; w < n_; ++w) th_.emplace_back([this, w] { loop(w); });
    }
    ~Team() {
        {
            std::lock_guard<std::mutex> l(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return n_; }
    void run(const std::function<void(int)>& f) {
        {
            std::lock_guard<std::mutex> l(mu_);
            task_ = &f;
            left_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> l(mu_);
        done_.wait(l, [this] { return left_ == 0; });
    }

  private:
    void loop(int w) {
        int seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> l(mu_);
            cv_.wait(l, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const std::function<void(int)>* f = task_;
            l.unlock();
            (*f)(w);
            l.lock();
            if (--left_ == 0) done_.notify_one();
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* task_ = nullptr;
    int gen_ = 0, left_ = 0;
    bool stop_ = false;
};

// Worker threads of a draw / assembly call: $DHCOS_GEN_THREADS, else min(16, hardware threads)
// (16: the GPU box's CPU share per GPU)
int team_size() {
    if (const char* e = std::getenv("DHCOS_GEN_THREADS")) {
        const int v = std::atoi(e);
        if (v > 0) return std::min(v, 256);
    }
    return (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Samples per chunk of the split draw (bounds its buffers), and below this many samples the
// plain sequential loop
constexpr int64_t kChunk = 1 << 16;
constexpr int64_t kSplitMin = 4096;

// samples drawn (uniforms, gauss calls, noise) by this process's draw calls (dh_gen_drawn_samples)
std::atomic<int64_t> g_drawn_total{0};

}  // namespace

namespace {

// ---------------------------------------------------------------------------------------------
// Parallel draw (round 4).  The stream positions of the samples are data dependent only through
// the polar method's acceptances: a sample takes 13 doubles (its uniforms) and then candidate
// pairs until its fresh gauss calls are served, each accepted pair serving two calls.  So:
//   1. a twister thread runs the MT19937 recurrence alone (the only inherently serial arithmetic)
//      and publishes the key at every 64th generation (a "block");
//   2. bit workers re-create each block's 64 generations from its key and mark, for every double
//      t of the stream, whether the candidate pair (D[t], D[t + 1]) is accepted (two bitmaps, by
//      the parity of t: a sample's pairs start at t, t + 2, ... of one parity);
//   3. the walker steps through the samples on those bits (13 doubles, then the k-th accepted
//      candidate by popcount), recording each 64k-sample chunk's start (double index, has_gauss);
//   4. chunk workers re-create the generator at their chunk's start and draw the chunk exactly as
//      the sequential loop would (uniforms, accepted pairs, log / sqrt, noise), leaving the
//      values that carry across samples -- the AR(1) blend, the spot walk and a gauss value cached
//      across the chunk boundary -- to
//   5. the sweep (the walker's thread, in chunk order), which also publishes the finished rows.
// Every value comes from the same words by the same operations in the same order as in the
// sequential draw, so the bits and the final RNG state are the same (tests/test_generator_rng.py).
// ---------------------------------------------------------------------------------------------
inline uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// the MT19937 recurrence on a key (LegacyRng::twist's arithmetic), built for AVX2 and baseline
// x86-64 (integer only: the same words either way), chosen at run time
#define DH_TWIST_BODY                                                                             \
    int i = 0;                                                                                    \
    uint32_t y;                                                                                   \
    for (; i < kMtN - kMtM; ++i) {                                                                \
        y = (key[i] & kUpper) | (key[i + 1] & kLower);                                            \
        key[i] = key[i + kMtM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);                               \
    }                                                                                             \
    for (; i < kMtN - 1; ++i) {                                                                   \
        y = (key[i] & kUpper) | (key[i + 1] & kLower);                                            \
        key[i] = key[i + (kMtM - kMtN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);                      \
    }                                                                                             \
    y = (key[kMtN - 1] & kUpper) | (key[0] & kLower);                                             \
    key[kMtN - 1] = key[kMtM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
__attribute__((target("avx2"))) void mt_twist_avx2(uint32_t* __restrict key) { DH_TWIST_BODY }
void mt_twist_base(uint32_t* __restrict key) { DH_TWIST_BODY }
#undef DH_TWIST_BODY
inline void mt_twist(uint32_t* key) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) mt_twist_avx2(key);
    else mt_twist_base(key);
}

inline double mt_double(uint32_t w0, uint32_t w1) {
    const int32_t a = (int32_t)(w0 >> 5), b = (int32_t)(w1 >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

inline bool polar_accept(double d0, double d1) {
    const double x1 = 2.0 * d0 - 1.0, x2 = 2.0 * d1 - 1.0;
    const double r2 = x1 * x1 + x2 * x2;
    return r2 < 1.0 && r2 != 0.0;
}

constexpr int kGensPerBlock = 64;
constexpr int64_t kBlockWords = (int64_t)kGensPerBlock * kMtN;

inline void spin_pause() { std::this_thread::yield(); }

// how far (blocks, ~600 samples each) the twister and the bit workers may run ahead of the
// walker: far enough that the walker never waits on them, not so far that the draw's end wastes
// the work of many blocks past the last sample
constexpr int64_t kLookahead = 64;
// samples per chunk of the parallel draw (its last chunk is the draw's tail)
constexpr int64_t kParChunk = 1 << 14;

// index of the (k+1)-th set bit of w (w has more than k set bits)
inline int select_bit(uint64_t w, int k) {
    for (int j = 0; j < k; ++j) w &= w - 1;
    return __builtin_ctzll(w);
}

struct ParDraw {
    // geometry: word n >= 0 of the stream is key word (pos0 + n) % 624 of generation
    // (pos0 + n) / 624; generation 0 is the entry key (after a pending twist)
    int pos0 = 0;
    uint32_t key0[kMtN];
    int64_t n = 0, n_opt = 0, n_chunks = 0, max_t = 0, max_blocks = 0;
    // chunk c covers samples [starts[c], starts[c + 1]) (starts[n_chunks] = n)
    std::vector<int64_t> starts;
    // published by the twister: keys of generations 64 b (in `snaps`, or in a caller's buffer:
    // snap points at the one in use), and mirrored to keys_ready_ext if set
    std::vector<uint32_t> snaps;
    uint32_t* snap = nullptr;
    std::atomic<int64_t> snaps_ready{0};
    std::atomic<int64_t>* keys_ready_ext = nullptr;
    // per-sample walk records for the device draw (dhgen::Located), if set: sample i's first
    // double and the source of its cached gauss value, published in located_ext
    int64_t* t_out = nullptr;
    int64_t* cs_out = nullptr;
    std::atomic<int64_t>* located_ext = nullptr;
    // acceptance bits of the candidate pair at double t, by parity: bit (t >> 1) of bits[t & 1]
    std::vector<std::atomic<uint64_t>> bits[2];
    std::vector<std::atomic<uint8_t>> block_done;
    std::atomic<int64_t> next_block{0};
    std::atomic<int64_t> walker_block{0};
    // the walk's chunk starts: double index, has_gauss, and the last accepted pair before it
    // (its first double's index; -1: none since the entry)
    std::vector<int64_t> chunk_t;
    std::vector<int32_t> chunk_hg;
    std::vector<int64_t> chunk_lp;
    std::atomic<int64_t> chunks_located{0};
    std::atomic<int64_t> next_chunk{0};
    std::vector<std::atomic<uint8_t>> chunk_done;
    std::vector<double> chunk_last_gc;      // the chunk's last pair's f x1 (NaN: no pair)
    // the chunk's gauss call served by the value cached before the chunk (at most one: after it
    // has_gauss is 0, so the next call draws a pair): sample, and -1 (spot return) or the option
    std::vector<int64_t> chunk_fb_i;
    std::vector<int32_t> chunk_fb_j;
    std::atomic<bool> walk_done{false}, failed{false};
    int64_t t_end = 0, lp_end = -1;
    int hg_end = 0;

    // the first double of the block's range, and the block of double t
    int64_t block_t0(int64_t b) const {
        const int64_t w = std::max<int64_t>(0, b * kBlockWords - pos0);
        return (w + 1) / 2;
    }
    int64_t block_of(int64_t t) const { return (pos0 + 2 * t) / kBlockWords; }

    // key of generation g into k (from the block's snapshot, twisted forward)
    void gen_key(int64_t g, uint32_t* k) const {
        std::memcpy(k, snap + (g / kGensPerBlock) * kMtN, sizeof(uint32_t) * kMtN);
        LegacyRng r;
        std::memcpy(r.key, k, sizeof(r.key));
        for (int64_t i = 0; i < g % kGensPerBlock; ++i) mt_twist(r.key);
        std::memcpy(k, r.key, sizeof(r.key));
    }
    // gen_key for any generation once the team has stopped: a block the twister never reached
    // (a walk that needed no acceptance bits there) is twisted forward from the last published
    // key, or from the entry key
    void key_any(int64_t g, uint32_t* k) const {
        const int64_t ready = snaps_ready.load(std::memory_order_acquire);
        if (g / kGensPerBlock < ready) {
            gen_key(g, k);
            return;
        }
        const int64_t g0 = ready > 0 ? (ready - 1) * kGensPerBlock : 0;
        std::memcpy(k, ready > 0 ? snap + (ready - 1) * kMtN : key0,
                    sizeof(uint32_t) * kMtN);
        for (int64_t i = g0; i < g; ++i) mt_twist(k);
    }
    // the generator positioned at double t of the stream (word pos0 + 2 t)
    void rng_at(int64_t t, LegacyRng& r) const {
        const int64_t w = pos0 + 2 * t;
        key_any(w / kMtN, r.key);
        r.pos = (int)(w % kMtN);
        r.has_gauss = 0;
        r.gauss = 0.0;
    }
    // the value next_gauss caches from the accepted pair at double t: f x1 (pair_values)
    double pair_cached(int64_t t) const {
        LegacyRng r;
        rng_at(t, r);
        const double x1 = 2.0 * r.next_double() - 1.0;
        const double x2 = 2.0 * r.next_double() - 1.0;
        const double r2 = x1 * x1 + x2 * x2;
        double gn, gc;
        pair_values(x1, x2, r2, gn, gc);
        return gc;
    }
};

void par_twister(ParDraw& P) {
    LegacyRng r;
    std::memcpy(r.key, P.key0, sizeof(r.key));
    for (int64_t b = 0; b < P.max_blocks; ++b) {
        // stay a bounded distance ahead of the walker
        while (b > P.walker_block.load(std::memory_order_acquire) + kLookahead) {
            if (P.walk_done.load(std::memory_order_acquire) || P.failed.load()) return;
            spin_pause();
        }
        if (P.walk_done.load(std::memory_order_acquire) || P.failed.load()) return;
        if (b > 0)
            for (int i = 0; i < kGensPerBlock; ++i) mt_twist(r.key);
        std::memcpy(P.snap + b * kMtN, r.key, sizeof(r.key));
        P.snaps_ready.store(b + 1, std::memory_order_release);
        if (P.keys_ready_ext) P.keys_ready_ext->store(b + 1, std::memory_order_release);
    }
}

// A block's arithmetic as straight loops the compiler vectorises: the tempering, the doubles of
// the block's range, and per parity the acceptance of each candidate pair packed 64 to a word.
// Built twice (AVX2 and baseline x86-64, chosen at run time): integer and exactly rounded fp64
// operations only, so both give the same bits.
#define DH_PAR_BITS_BODY                                                                          \
    for (int64_t j = 0; j < nw; ++j) w[j] = mt_temper(w[j]);                                     \
    for (int64_t j = 0; j < nd; ++j) d[j] = mt_double(w[q0 + 2 * j], w[q0 + 2 * j + 1]);         \
    for (int p = 0; p < 2; ++p) {                                                                 \
        /* candidates t = 2 i + p in [t0, t1): doubles d[t - t0], d[t - t0 + 1] */                \
        const int64_t i0 = (t0 - p + 1) >> 1, i1 = (t1 - p + 1) >> 1;                             \
        for (int64_t i = i0; i < i1;) {                                                           \
            const int64_t wend = std::min(i1, ((i >> 6) + 1) << 6);                              \
            const int64_t cnt = wend - i;                                                         \
            const double* dd = d + (2 * i + p - t0);                                              \
            for (int64_t j = 0; j < cnt; ++j) {                                                   \
                const double x1 = 2.0 * dd[2 * j] - 1.0, x2 = 2.0 * dd[2 * j + 1] - 1.0;          \
                const double r2 = x1 * x1 + x2 * x2;                                              \
                ok[j] = (uint8_t)((r2 < 1.0) & (r2 != 0.0));                                      \
            }                                                                                     \
            uint64_t m = 0;                                                                       \
            for (int64_t j = 0; j < cnt; ++j) m |= (uint64_t)ok[j] << j;                         \
            m <<= (i & 63);                                                                       \
            if (m) bits[p][i >> 6].fetch_or(m, std::memory_order_relaxed);                        \
            i = wend;                                                                             \
        }                                                                                         \
    }

__attribute__((target("avx2"))) void par_bits_avx2(uint32_t* w, int64_t nw, double* d,
                                                   int64_t nd, int64_t q0, int64_t t0,
                                                   int64_t t1, uint8_t* ok,
                                                   std::vector<std::atomic<uint64_t>>* bits) {
    DH_PAR_BITS_BODY
}

void par_bits_base(uint32_t* w, int64_t nw, double* d, int64_t nd, int64_t q0, int64_t t0,
                   int64_t t1, uint8_t* ok, std::vector<std::atomic<uint64_t>>* bits) {
    DH_PAR_BITS_BODY
}
#undef DH_PAR_BITS_BODY

struct BitsScratch {
    std::vector<uint32_t> w;
    std::vector<double> d;
    uint8_t ok[64];
};

void par_bits(ParDraw& P, int64_t b, BitsScratch& S) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    const int64_t t0 = P.block_t0(b), t1 = std::min(P.block_t0(b + 1), P.max_t);
    if (t1 <= t0) {             // a block past the stream bound (the last of max_blocks): no pairs
        P.block_done[b].store(1, std::memory_order_release);
        return;
    }
    // raw key words of generations 64 b .. 64 b + 64 (the next block's first words close the
    // block's last pairs), tempered in place by the body
    LegacyRng r;
    std::memcpy(r.key, P.snap + b * kMtN, sizeof(r.key));
    const int64_t nw = kBlockWords + kMtN;
    S.w.resize(nw);
    for (int gi = 0; gi <= kGensPerBlock; ++gi) {
        if (gi > 0) mt_twist(r.key);
        std::memcpy(S.w.data() + (int64_t)gi * kMtN, r.key, sizeof(r.key));
    }
    const int64_t base = b * kBlockWords - P.pos0;          // word n at w[n - base]
    const int64_t nd = t1 - t0 + 1;                          // doubles t0 .. t1
    S.d.resize(nd);
    const int64_t q0 = 2 * t0 - base;
    if (avx2)
        par_bits_avx2(S.w.data(), nw, S.d.data(), nd, q0, t0, t1, S.ok, P.bits);
    else
        par_bits_base(S.w.data(), nw, S.d.data(), nd, q0, t0, t1, S.ok, P.bits);
    P.block_done[b].store(1, std::memory_order_release);
}

// The k-th accepted candidate pair at t, t + 2, ... (k >= 1) -> the double after it; *ok false
// when the stream bound is reached (the caller falls back to the sequential draw)
int64_t par_select(ParDraw& P, int64_t t, int k, int64_t& ready_t, int64_t& next_b,
                   int64_t& last_pair, bool& ok) {
    const int p = (int)(t & 1);
    int64_t idx = t >> 1;
    for (;;) {
        const int64_t wend = ((idx >> 6) + 1) << 6;          // the word's bits are final once
        const int64_t need_t = 2 * wend + 2;                  // its last double's pair is set
        while (ready_t < std::min(need_t, P.max_t)) {
            if (next_b >= P.max_blocks) break;
            if (P.block_done[next_b].load(std::memory_order_acquire)) {
                ++next_b;
                ready_t = P.block_t0(next_b);
                P.walker_block.store(next_b, std::memory_order_release);
            } else {
                spin_pause();
            }
        }
        if (2 * wend + 1 >= P.max_t) {
            ok = false;
            return t;
        }
        const uint64_t w = P.bits[p][idx >> 6].load(std::memory_order_relaxed) >> (idx & 63);
        const int c = __builtin_popcountll(w);
        if (c >= k) {
            const int64_t j = idx + select_bit(w, k - 1);
            last_pair = 2 * j + p;
            return last_pair + 2;
        }
        k -= c;
        idx = wend;
    }
}

void par_walk(ParDraw& P, int hg0) {
    int64_t t = 0, ready_t = 0, next_b = 0, last_pair = -1;
    int hg = hg0;
    bool ok = true;
    int64_t c = 0;
    for (int64_t i = 0; i < P.n && ok; ++i) {
        if (P.t_out) {                                    // the device draw's per-sample records
            P.t_out[i] = t;
            P.cs_out[i] = hg ? last_pair : -2;            // (last_pair -1: the entry's value)
            if ((i & 1023) == 1023) P.located_ext->store(i + 1, std::memory_order_release);
        }
        while (c < P.n_chunks && P.starts[c] == i) {     // (equal starts: empty chunks)
            P.chunk_t[c] = t;
            P.chunk_hg[c] = hg;
            P.chunk_lp[c] = last_pair;
            P.chunks_located.store(c + 1, std::memory_order_release);
            ++c;
        }
        t += 13;                                              // :100-102
        const int calls = (int)P.n_opt + (i > 0 ? 1 : 0);     // :112-116, :141
        const int fresh = calls - hg;
        if (fresh > 0) {
            t = par_select(P, t, (fresh + 1) / 2, ready_t, next_b, last_pair, ok);
            hg = fresh & 1;
        } else {
            hg -= calls;
        }
    }
    if (!ok || t >= P.max_t) {
        P.failed.store(true);
    }
    for (; c < P.n_chunks; ++c) {                          // chunks starting at n (empty)
        P.chunk_t[c] = t;
        P.chunk_hg[c] = hg;
        P.chunk_lp[c] = last_pair;
    }
    P.chunks_located.store(P.n_chunks, std::memory_order_release);
    P.t_end = t;
    P.lp_end = last_pair;
    P.hg_end = hg;
    if (P.t_out && ok && t < P.max_t) {
        P.t_out[P.n] = t;
        P.located_ext->store(P.n + 1, std::memory_order_release);
    }
    P.walk_done.store(true, std::memory_order_release);
}

struct ChunkOut {
    std::vector<double> px1, px2, pr2, gn, gc;
};

// one chunk of the draw from its located start: raw uniforms into params (the blend is the
// sweep's), noise, and the spot return's normal (ret_mu + ret_sigma g) into spots; a first gauss
// call served from the value cached before the chunk is left to the sweep
void par_chunk(ParDraw& P, int64_t c, const double* lo, const double* range,
               double ret_mu, double ret_sigma, double noise_sigma, double* params,
               double* spots, double* noise, ChunkOut& o) {
    const int64_t c0 = P.starts[c], c1 = P.starts[c + 1];
    g_drawn_total.fetch_add(c1 - c0, std::memory_order_relaxed);
    const int64_t word = P.pos0 + 2 * P.chunk_t[c];
    LegacyRng g;
    // the block's key may not be published yet (chunk 0 is located before the twister's first
    // store)
    while (P.snaps_ready.load(std::memory_order_acquire) <= (word / kMtN) / kGensPerBlock)
        spin_pause();
    P.gen_key(word / kMtN, g.key);
    g.pos = (int)(word % kMtN);
    g.has_gauss = 0;
    g.gauss = 0.0;
    const int64_t n_opt = P.n_opt;
    const int64_t per = n_opt + 1;
    const int64_t cap = (c1 - c0) * per;
    o.px1.resize(cap);
    o.px2.resize(cap);
    o.pr2.resize(cap);
    o.gn.resize(cap);
    o.gc.resize(cap);
    DoubleStream ds(g);
    int hg = P.chunk_hg[c];
    int32_t np = 0;
    for (int64_t i = c0; i < c1; ++i) {
        double* p = params + i * 13;
        for (int j = 0; j < 13; ++j) p[j] = lo[j] + range[j] * ds.next();   // :100-102
        const int calls = (int)n_opt + (i > 0 ? 1 : 0);
        const int fresh = calls - hg;
        const int first = np;
        const int cached = hg;
        const int k = fresh > 0 ? (fresh + 1) / 2 : 0;
        ds.pairs(k, o.px1.data() + np, o.px2.data() + np, o.pr2.data() + np);
        for (int q = first; q < first + k; ++q)
            pair_values(o.px1[q], o.px2[q], o.pr2[q], o.gn[q], o.gc[q]);
        np += k;
        hg = fresh > 0 ? (fresh & 1) : hg - calls;
        // gauss call cc of this sample: cached first (value before the sample), then new pairs
        // each serving f x2 then f x1
        auto value = [&](int cc, bool& from_before) {
            from_before = false;
            if (cached) {
                if (cc == 0) {
                    if (first == 0) {                        // cached across the chunk start
                        from_before = true;
                        return 0.0;
                    }
                    return o.gc[first - 1];
                }
                --cc;
            }
            return (cc & 1) ? o.gc[first + cc / 2] : o.gn[first + cc / 2];
        };
        bool fb;
        const int c00 = i > 0 ? 1 : 0;
        if (i > 0) {
            const double v = value(0, fb);
            spots[i] = fb ? 0.0 : ret_mu + ret_sigma * v;
            if (fb) P.chunk_fb_i[c] = i, P.chunk_fb_j[c] = -1;
        }
        double* z = noise + i * n_opt;
        for (int j = 0; j < n_opt; ++j) {
            const double v = value(c00 + j, fb);
            z[j] = fb ? 0.0 : 0.0 + noise_sigma * v;
            if (fb) P.chunk_fb_i[c] = i, P.chunk_fb_j[c] = j;
        }
    }
    P.chunk_last_gc[c] = np > 0 ? o.gc[np - 1] : NAN;
    P.chunk_done[c].store(1, std::memory_order_release);
}

// stream bound: twice the expected doubles (acceptance pi/4) plus slack; a walk past it (never
// seen: ~thousands of standard deviations) falls back to the sequential draw
void stream_bounds(int pos0, int64_t n_samples, int n_opt, int64_t& max_t, int64_t& max_blocks) {
    const double per_sample = 13.0 + 2.0 * ((n_opt + 2) / 2) / 0.7853981633974483;
    max_t = (int64_t)(2.0 * per_sample * (double)n_samples) + (1 << 20);
    max_blocks = (pos0 + 2 * max_t) / kBlockWords + 2;
}

// The stream geometry and buffers of a parallel pass over n_samples from g's state, with chunk
// starts `starts` (sorted; starts[0] = 0, the last entry n_samples)
void par_setup(ParDraw& P, const LegacyRng& g, int64_t n_samples, int n_opt,
               std::vector<int64_t> starts, uint32_t* keys = nullptr) {
    LegacyRng e = g;
    if (e.pos == kMtN) e.twist();
    P.pos0 = e.pos;
    std::memcpy(P.key0, e.key, sizeof(P.key0));
    P.n = n_samples;
    P.n_opt = n_opt;
    P.starts = std::move(starts);
    P.n_chunks = (int64_t)P.starts.size() - 1;
    stream_bounds(P.pos0, n_samples, n_opt, P.max_t, P.max_blocks);
    if (keys) {
        P.snap = keys;
    } else {
        P.snaps.resize((size_t)P.max_blocks * kMtN);
        P.snap = P.snaps.data();
    }
    const int64_t nwords = (P.max_t / 2) / 64 + 2;
    for (int p = 0; p < 2; ++p) {
        std::vector<std::atomic<uint64_t>> v(nwords);
        P.bits[p].swap(v);
        for (auto& a : P.bits[p]) a.store(0, std::memory_order_relaxed);
    }
    {
        std::vector<std::atomic<uint8_t>> v(P.max_blocks);
        P.block_done.swap(v);
        for (auto& a : P.block_done) a.store(0, std::memory_order_relaxed);
        std::vector<std::atomic<uint8_t>> u(std::max<int64_t>(P.n_chunks, 0));
        P.chunk_done.swap(u);
        for (auto& a : P.chunk_done) a.store(0, std::memory_order_relaxed);
    }
    const int64_t nc = std::max<int64_t>(P.n_chunks, 0);
    P.chunk_t.assign(nc, 0);
    P.chunk_hg.assign(nc, 0);
    P.chunk_lp.assign(nc, -1);
    P.chunk_last_gc.assign(nc, NAN);
    P.chunk_fb_i.assign(nc, -1);
    P.chunk_fb_j.assign(nc, -1);
}

// A bit worker (and, with draw, a chunk worker) of the team until the pass is over
void par_worker(ParDraw& P, bool draw, const double* lo, const double* range, double ret_mu,
                double ret_sigma, double noise_sigma, double* params, double* spots,
                double* noise) {
    BitsScratch wbuf;
    ChunkOut out;
    for (;;) {
        if (P.failed.load()) return;
        const bool walking = !P.walk_done.load(std::memory_order_acquire);
        const int64_t b = P.next_block.load(std::memory_order_relaxed);
        if (walking && b < P.snaps_ready.load(std::memory_order_acquire) &&
            b <= P.walker_block.load(std::memory_order_relaxed) + kLookahead) {
            int64_t bb = b;
            if (P.next_block.compare_exchange_weak(bb, b + 1)) par_bits(P, b, wbuf);
            continue;
        }
        if (draw) {
            const int64_t c = P.next_chunk.load(std::memory_order_relaxed);
            if (c < P.chunks_located.load(std::memory_order_acquire)) {
                int64_t cc = c;
                if (P.next_chunk.compare_exchange_weak(cc, c + 1))
                    par_chunk(P, c, lo, range, ret_mu, ret_sigma, noise_sigma, params, spots,
                              noise, out);
                continue;
            }
            if (!walking && c >= P.n_chunks) return;
        } else if (!walking) {
            return;
        }
        spin_pause();
    }
}

// The state the sequential loop leaves after the pass (its walk's end): word n_end = 2 t_end of
// the stream read, has_gauss and the value cached from the last pair (or kept from the entry)
void par_final_state(const ParDraw& P, const LegacyRng& entry, LegacyRng& g) {
    const int64_t n_end = 2 * P.t_end;
    const double entry_gauss = entry.gauss;
    if (n_end > 0) {
        const int64_t last = P.pos0 + n_end - 1;             // the last word read
        P.key_any(last / kMtN, g.key);
        g.pos = (int)(last % kMtN) + 1;                      // 1 .. 624 (624: twist pending)
    } else {
        g = entry;                                           // nothing read: the entry state
    }
    g.has_gauss = P.hg_end;
    g.gauss = P.hg_end ? (P.lp_end >= 0 ? P.pair_cached(P.lp_end) : entry_gauss) : 0.0;
}

// -> 1 done, 0 not applicable / bound exceeded (the caller runs the sequential draw instead)
int gen_draw_parallel(LegacyRng& g, int64_t n_samples, const double* lo, const double* hi,
                      int n_opt, double alpha, double spot0, double ret_mu, double ret_sigma,
                      double noise_sigma, double* params, double* spots, double* noise,
                      const std::function<void(int64_t)>& publish) {
    const int nth = team_size();
    if (nth < 3) return 0;
    ParDraw P;
    std::vector<int64_t> starts;
    for (int64_t i = 0; i < n_samples; i += kParChunk) starts.push_back(i);
    starts.push_back(n_samples);
    par_setup(P, g, n_samples, n_opt, std::move(starts));
    double range[13];
    for (int j = 0; j < 13; ++j) range[j] = hi[j] - lo[j];
    const double beta = 1.0 - alpha;
    double pending = g.gauss;                 // the value cached at entry (used if has_gauss)
    double prev_spot = spot0;
    bool fell_back = false;
    const double t_start = now_s();
    double t_twist = 0.0, t_walk = 0.0;
    Team team(nth);
    team.run([&](int w) {
        if (w == 1) {
            par_twister(P);
            t_twist = now_s() - t_start;
            w = 2;                            // then a worker like the others
        }
        if (w == 0) {
            par_walk(P, g.has_gauss ? 1 : 0);
            t_walk = now_s() - t_start;
            if (P.failed.load()) {
                fell_back = true;
                return;
            }
            // the sweep, in chunk order
            for (int64_t c = 0; c < P.n_chunks; ++c) {
                while (!P.chunk_done[c].load(std::memory_order_acquire)) {
                    if (P.failed.load()) return;
                    spin_pause();
                }
                const int64_t c0 = P.starts[c], c1 = P.starts[c + 1];
                const int64_t fi = P.chunk_fb_i[c];   // served from before the chunk
                if (fi >= 0) {
                    if (P.chunk_fb_j[c] < 0) spots[fi] = ret_mu + ret_sigma * pending;
                    else noise[fi * n_opt + P.chunk_fb_j[c]] = 0.0 + noise_sigma * pending;
                }
                // the value cached after the chunk: its last pair's f x1, or (no new pair) the
                // one from before it
                if (!std::isnan(P.chunk_last_gc[c])) pending = P.chunk_last_gc[c];
                for (int64_t i = c0; i < c1; ++i) {
                    double* p = params + i * 13;
                    if (i > 0) {
                        const double* q = p - 13;
                        for (int j = 0; j < 13; ++j) p[j] = alpha * q[j] + beta * p[j];   // :105-109
                        prev_spot = prev_spot * (1.0 + spots[i]);                         // :112-116
                    }
                    spots[i] = prev_spot;
                }
                publish(c1);
            }
            return;
        }
        par_worker(P, true, lo, range, ret_mu, ret_sigma, noise_sigma, params, spots, noise);
    });
    if (std::getenv("DHCOS_GEN_TIMING"))
        std::fprintf(stderr, "dh_gen_draw (parallel, %d threads): %lld samples: twister %.4f s, "
                     "walk %.4f s, total %.4f s, %lld blocks\n", nth, (long long)n_samples,
                     t_twist, t_walk, now_s() - t_start,
                     (long long)P.snaps_ready.load());
    if (fell_back || P.failed.load()) return 0;
    const LegacyRng entry = g;
    par_final_state(P, entry, g);
    g.gauss = g.has_gauss ? pending : 0.0;    // (par_final_state's value, via the sweep)
    return 1;
}

// ---------------------------------------------------------------------------------------------
// Sharded draw (round 5): one rank locates, every rank draws its own samples.
//   locate:  the serial part of the parallel draw only -- the twister, the acceptance bitmaps
//            and the walk -- recording the generator's state (key, pos, has_gauss, cached value:
//            np.random.get_state()'s fields) at the first sample of each requested chunk;
//   located: a rank draws its chunks from those states (uniforms, accepted pairs, log / sqrt,
//            noise and the spot return's normal; no AR(1), no spot walk);
//   sweep:   the values that carry across samples (the AR(1) blend and the spot walk) over a
//            rank's block, from the previous block's last row (14 doubles passed rank to rank).
// The same words through the same operations in the same order as the sequential loop.
// ---------------------------------------------------------------------------------------------
constexpr int kLocWords = kMtN + 3;           // key[624], pos, has_gauss, cached (as doubles)

void loc_store(const LegacyRng& r, double* out) {
    for (int i = 0; i < kMtN; ++i) out[i] = (double)r.key[i];
    out[kMtN] = r.pos;
    out[kMtN + 1] = r.has_gauss;
    out[kMtN + 2] = r.gauss;
}

bool loc_load(const double* in, LegacyRng& r) {
    for (int i = 0; i < kMtN; ++i) {
        const double v = in[i];
        if (!(v >= 0.0 && v <= 4294967295.0) || v != (double)(uint32_t)v) return false;
        r.key[i] = (uint32_t)v;
    }
    if (!(in[kMtN] >= 0.0 && in[kMtN] <= kMtN) || in[kMtN] != (int)in[kMtN]) return false;
    r.pos = (int)in[kMtN];
    r.has_gauss = in[kMtN + 1] != 0.0 ? 1 : 0;
    r.gauss = in[kMtN + 2];
    return true;
}

// samples [i0, i1) from r's state (positioned at sample i0's first double): raw uniforms into
// params, the spot return's normal (ret_mu + ret_sigma g) into rets for i > 0, noise; rows
// relative to `base`
void draw_raw(LegacyRng r, int64_t i0, int64_t i1, int64_t base, const double* lo,
              const double* range, int n_opt, double ret_mu, double ret_sigma, double noise_sigma,
              double* params, double* rets, double* noise) {
    g_drawn_total.fetch_add(i1 - i0, std::memory_order_relaxed);
    const int kmax = (n_opt + 2) / 2;
    std::vector<double> x1(kmax), x2(kmax), r2(kmax), gn(kmax), gc(kmax);
    int hg = r.has_gauss;
    double cached = r.gauss;
    DoubleStream ds(r);
    for (int64_t i = i0; i < i1; ++i) {
        double* p = params + (i - base) * 13;
        for (int j = 0; j < 13; ++j) p[j] = lo[j] + range[j] * ds.next();   // :100-102
        const int calls = n_opt + (i > 0 ? 1 : 0);                           // :112-116, :141
        const int fresh = calls - hg;
        const int k = fresh > 0 ? (fresh + 1) / 2 : 0;
        ds.pairs(k, x1.data(), x2.data(), r2.data());
        for (int q = 0; q < k; ++q) pair_values(x1[q], x2[q], r2[q], gn[q], gc[q]);
        // gauss call c of this sample: the value cached before it first, then the new pairs,
        // each serving f x2 then f x1
        auto value = [&](int c) {
            if (hg) {
                if (c == 0) return cached;
                --c;
            }
            return (c & 1) ? gc[c / 2] : gn[c / 2];
        };
        const int c00 = i > 0 ? 1 : 0;
        if (i > 0) rets[i - base] = ret_mu + ret_sigma * value(0);
        double* z = noise + (i - base) * n_opt;
        for (int j = 0; j < n_opt; ++j) z[j] = 0.0 + noise_sigma * value(c00 + j);
        if (fresh > 0) {
            hg = fresh & 1;
            if (hg) cached = gc[k - 1];
        } else {
            hg -= calls;
        }
    }
}

}  // namespace

namespace {

int gen_locate(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss, double* cached_gauss,
               int64_t n_samples, int n_opt, const int64_t* starts, int64_t n_starts,
               double* loc) {
    if (!mt_key || !mt_pos || !has_gauss || !cached_gauss) return DH_E_ARG;
    if (n_samples < 0 || n_opt < 0 || n_starts < 0 || (n_starts > 0 && (!starts || !loc)))
        return DH_E_ARG;
    if (*mt_pos < 0 || *mt_pos > kMtN) return DH_E_ARG;
    for (int64_t j = 0; j < n_starts; ++j)
        if (starts[j] < 0 || starts[j] > n_samples || (j > 0 && starts[j] < starts[j - 1]))
            return DH_E_ARG;
    LegacyRng g;
    std::memcpy(g.key, mt_key, sizeof(g.key));
    g.pos = *mt_pos;
    g.has_gauss = *has_gauss ? 1 : 0;
    g.gauss = *cached_gauss;
    const LegacyRng entry = g;
    ParDraw P;
    std::vector<int64_t> st(starts, starts + n_starts);
    st.push_back(n_samples);
    par_setup(P, g, n_samples, n_opt, std::move(st));
    const int nth = std::max(3, team_size());
    {
        Team team(nth);
        team.run([&](int w) {
            if (w == 1) {
                par_twister(P);
                w = 2;
            }
            if (w == 0) {
                par_walk(P, g.has_gauss ? 1 : 0);
                return;
            }
            par_worker(P, false, nullptr, nullptr, 0.0, 0.0, 0.0, nullptr, nullptr, nullptr);
        });
    }
    if (P.failed.load()) return DH_E_ARG;      // past the stream bound (never seen)
    for (int64_t j = 0; j < n_starts; ++j) {
        LegacyRng r;
        P.rng_at(P.chunk_t[j], r);
        r.has_gauss = P.chunk_hg[j];
        r.gauss = r.has_gauss ? (P.chunk_lp[j] >= 0 ? P.pair_cached(P.chunk_lp[j]) : entry.gauss)
                              : 0.0;
        loc_store(r, loc + j * kLocWords);
    }
    par_final_state(P, entry, g);
    std::memcpy(mt_key, g.key, sizeof(g.key));
    *mt_pos = g.pos;
    *has_gauss = g.has_gauss;
    *cached_gauss = g.gauss;
    return DH_OK;
}

}  // namespace

namespace {

// done (optional): the count of leading samples whose params, spot and noise are written, stored
// with release order after each chunk (a concurrent reader may consume those rows)
int gen_draw(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss, double* cached_gauss,
             int64_t n_samples, const double* lo, const double* hi, int n_opt, double alpha,
             double spot0, double ret_mu, double ret_sigma, double noise_sigma, double* params,
             double* spots, double* noise, int64_t* done) {
    auto publish = [done](int64_t v) {
        if (done) __atomic_store_n(done, v, __ATOMIC_RELEASE);
    };
    if (!mt_key || !mt_pos || !has_gauss || !cached_gauss || !lo || !hi) return DH_E_ARG;
    if (n_samples < 0 || n_opt < 0) return DH_E_ARG;
    if (n_samples > 0 && (!params || !spots || (n_opt > 0 && !noise))) return DH_E_ARG;
    if (*mt_pos < 0 || *mt_pos > kMtN) return DH_E_ARG;
    LegacyRng g;
    std::memcpy(g.key, mt_key, sizeof(g.key));
    g.pos = *mt_pos;
    g.has_gauss = *has_gauss ? 1 : 0;
    g.gauss = *cached_gauss;
    double range[13];
    for (int j = 0; j < 13; ++j) range[j] = hi[j] - lo[j];
    const double beta = 1.0 - alpha;                      // (1 - alpha), :108
    double spot = spot0;
    if (n_samples >= kSplitMin &&
        gen_draw_parallel(g, n_samples, lo, hi, n_opt, alpha, spot0, ret_mu, ret_sigma,
                          noise_sigma, params, spots, noise, publish)) {
        std::memcpy(mt_key, g.key, sizeof(g.key));
        *mt_pos = g.pos;
        *has_gauss = g.has_gauss;
        *cached_gauss = g.gauss;
        publish(n_samples);
        return DH_OK;
    }
    g_drawn_total.fetch_add(n_samples, std::memory_order_relaxed);   // (sequential paths)
    if (n_samples < kSplitMin) {
        for (int64_t i = 0; i < n_samples; ++i) {
            double* p = params + i * 13;
            for (int j = 0; j < 13; ++j) p[j] = lo[j] + range[j] * g.next_double();   // :100-102
            if (i > 0) {
                const double* q = p - 13;
                for (int j = 0; j < 13; ++j) p[j] = alpha * q[j] + beta * p[j];       // :105-109
                spot = spot * (1.0 + g.normal(ret_mu, ret_sigma));                     // :112-116
            }
            spots[i] = spot;
            double* z = noise + i * n_opt;
            for (int j = 0; j < n_opt; ++j) z[j] = g.normal(0.0, noise_sigma);        // :141
        }
    } else {
        // Large draws in three passes per chunk of samples, the same operations on the same
        // values in the same order per value (so the same bits):
        //   A (this thread): the MT19937 doubles (DoubleStream), the parameters and their AR(1)
        //     blend, and for every gauss call either the accepted polar pair (x1, x2, r2) or a
        //     reference to the pair whose cached half it returns, exactly as has_gauss toggles;
        //   B (a helper thread): next_gauss's log / sqrt / products per pair;
        //   C (the helper): the noise and the spot walk from the gauss values.
        // A of chunk c + 1 runs while the helper does B and C of chunk c (two chunk slots), so a
        // draw costs about pass A alone.  (A team of 4-16 workers for B / C was measured on the
        // GPU box's EPYC host: B + C 0.05 -> 0.01 s per 1M samples, but pass A of the main
        // thread 0.067 -> 0.12-0.16 s; one overlapped helper keeps A at its single-thread speed.)
        struct Slot {
            std::vector<double> px1, px2, pr2, gn, gc;      // per pair: inputs, f x2, f x1
            // per sample: its first new pair in the chunk, and whether its first gauss call
            // returns the value cached before it (the previous pair's f x1, or `pending`)
            std::vector<int32_t> first;
            std::vector<uint8_t> cached;
            int64_t c0 = 0, c1 = 0;
            int32_t np = 0;
            bool full = false;                              // A done, B + C pending
        };
        const int64_t per = (int64_t)n_opt + 1;             // gauss calls per sample, at most
        const int64_t cs = std::min(n_samples, kChunk);
        Slot slots[2];
        for (Slot& sl : slots) {
            sl.px1.resize(cs * per);
            sl.px2.resize(cs * per);
            sl.pr2.resize(cs * per);
            sl.gn.resize(cs * per);
            sl.gc.resize(cs * per);
            sl.first.resize(cs);
            sl.cached.resize(cs);
        }
        std::mutex mu;
        std::condition_variable cv;
        bool produced = false;
        double pending = g.gauss;                           // the value cached at entry
        double t_a = 0.0;                                   // $DHCOS_GEN_TIMING
        const double t_start = now_s();
        auto consume = [&](Slot& sl) {                      // B and C of one chunk
            for (int32_t k = 0; k < sl.np; ++k)
                pair_values(sl.px1[k], sl.px2[k], sl.pr2[k], sl.gn[k], sl.gc[k]);
            auto value = [&](int64_t r, int c) {            // gauss call c of chunk sample r
                const int32_t f = sl.first[r];
                if (sl.cached[r]) {
                    if (c == 0) return f == 0 ? pending : sl.gc[f - 1];
                    --c;
                }
                return (c & 1) ? sl.gc[f + c / 2] : sl.gn[f + c / 2];
            };
            for (int64_t i = sl.c0; i < sl.c1; ++i) {
                const int64_t r = i - sl.c0;
                if (i > 0) spot = spot * (1.0 + (ret_mu + ret_sigma * value(r, 0)));
                spots[i] = spot;
                const int c00 = i > 0 ? 1 : 0;
                double* z = noise + i * n_opt;
                for (int j = 0; j < n_opt; ++j) z[j] = 0.0 + noise_sigma * value(r, c00 + j);
            }
            if (sl.np > 0) pending = sl.gc[sl.np - 1];      // cached into the next chunk if
        };                                                  // has_gauss is set
        std::thread helper([&] {
            for (int64_t c = 0;; ++c) {
                Slot& sl = slots[c & 1];
                {
                    std::unique_lock<std::mutex> l(mu);
                    cv.wait(l, [&] { return sl.full || produced; });
                    if (!sl.full) return;
                }
                consume(sl);
                publish(sl.c1);                             // rows < c1 complete
                {
                    std::lock_guard<std::mutex> l(mu);
                    sl.full = false;
                }
                cv.notify_all();
            }
        });
        DoubleStream ds(g);
        int64_t c = 0;
        for (int64_t c0 = 0; c0 < n_samples; c0 += kChunk, ++c) {
            Slot& sl = slots[c & 1];
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return !sl.full; });
            }
            const double t0 = now_s();
            sl.c0 = c0;
            sl.c1 = std::min(n_samples, c0 + kChunk);
            int32_t np = 0;
            int hg = g.has_gauss;
            for (int64_t i = sl.c0; i < sl.c1; ++i) {       // A
                double* p = params + i * 13;
                for (int j = 0; j < 13; ++j) p[j] = lo[j] + range[j] * ds.next();   // :100-102
                if (i > 0) {
                    const double* q = p - 13;
                    for (int j = 0; j < 13; ++j) p[j] = alpha * q[j] + beta * p[j]; // :105-109
                }
                // gauss calls: the spot return (i > 0, :112-116), then one per option (:141);
                // the first takes the cached value if there is one, the rest run on new pairs,
                // each serving two calls (f x2 now, f x1 cached for the next)
                const int calls = n_opt + (i > 0 ? 1 : 0);
                const int fresh = calls - hg;
                sl.first[i - sl.c0] = np;
                sl.cached[i - sl.c0] = (uint8_t)hg;
                const int k = (fresh + 1) / 2;
                ds.pairs(k, sl.px1.data() + np, sl.px2.data() + np, sl.pr2.data() + np);
                np += k;
                hg = fresh > 0 ? (fresh & 1) : hg - calls;
            }
            g.has_gauss = hg;
            sl.np = np;
            t_a += now_s() - t0;
            {
                std::lock_guard<std::mutex> l(mu);
                sl.full = true;
            }
            cv.notify_all();
        }
        {
            std::lock_guard<std::mutex> l(mu);
            produced = true;
        }
        cv.notify_all();
        helper.join();
        ds.sync();
        if (std::getenv("DHCOS_GEN_TIMING"))
            std::fprintf(stderr, "dh_gen_draw: %lld samples: pass A %.4f s, total %.4f s\n",
                         (long long)n_samples, t_a, now_s() - t_start);
        g.gauss = g.has_gauss ? pending : 0.0;
    }
    std::memcpy(mt_key, g.key, sizeof(g.key));
    *mt_pos = g.pos;
    *has_gauss = g.has_gauss;
    *cached_gauss = g.gauss;
    publish(n_samples);
    return DH_OK;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// The host part of the device draw (dh_gen_rng.h): the twister, the bit workers and the walk of
// the parallel draw, with the walk's per-sample records (first double, cached-value source) and
// the keys in the caller's buffers, published as they are written.
// ---------------------------------------------------------------------------------------------
namespace dhgen {

void locate_geometry(Located& L) {
    L.pos0 = L.pos == kMtN ? 0 : L.pos;
    stream_bounds(L.pos0, L.n, L.n_opt, L.max_t, L.max_blocks);
}

void locate_run(Located& L) {
    const double t_start = now_s();
    LegacyRng g;
    std::memcpy(g.key, L.key, sizeof(g.key));
    g.pos = L.pos;
    g.has_gauss = L.has_gauss ? 1 : 0;
    g.gauss = L.gauss;
    const LegacyRng entry = g;
    ParDraw P;
    par_setup(P, g, L.n, L.n_opt, std::vector<int64_t>{L.n}, L.keys);
    P.t_out = L.t;
    P.cs_out = L.cs;
    P.located_ext = &L.located;
    P.keys_ready_ext = &L.keys_ready;
    {
        Team team(std::max(3, team_size()));
        team.run([&](int w) {
            if (w == 1) {
                par_twister(P);
                L.s_twister = now_s() - t_start;
                w = 2;
            }
            if (w == 0) {
                par_walk(P, g.has_gauss ? 1 : 0);
                L.s_walk = now_s() - t_start;
                return;
            }
            par_worker(P, false, nullptr, nullptr, 0.0, 0.0, 0.0, nullptr, nullptr, nullptr);
        });
    }
    if (P.failed.load()) {
        L.state.store(-1, std::memory_order_release);
        return;
    }
    par_final_state(P, entry, g);
    std::memcpy(L.key_end, g.key, sizeof(g.key));
    L.pos_end = g.pos;
    L.has_gauss_end = g.has_gauss;
    L.gauss_end = g.gauss;
    L.state.store(1, std::memory_order_release);
}

void locate_extend_keys(Located& L, int64_t blocks) {
    blocks = std::min(blocks, L.max_blocks);
    int64_t b = L.keys_ready.load(std::memory_order_acquire);
    if (b >= blocks) return;
    uint32_t k[kMtN];
    if (b == 0) {
        LegacyRng e;
        std::memcpy(e.key, L.key, sizeof(e.key));
        e.pos = L.pos;
        if (e.pos == kMtN) e.twist();
        std::memcpy(k, e.key, sizeof(k));
        std::memcpy(L.keys, k, sizeof(k));
        b = 1;
    } else {
        std::memcpy(k, L.keys + (b - 1) * kMtN, sizeof(k));
    }
    for (; b < blocks; ++b) {
        for (int i = 0; i < kGensPerBlock; ++i) mt_twist(k);
        std::memcpy(L.keys + b * kMtN, k, sizeof(k));
    }
    L.keys_ready.store(blocks, std::memory_order_release);
}

}  // namespace dhgen

extern "C" int dh_gen_draw(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss,
                           double* cached_gauss, int64_t n_samples, const double* lo,
                           const double* hi, int n_opt, double alpha, double spot0,
                           double ret_mu, double ret_sigma, double noise_sigma, double* params,
                           double* spots, double* noise) {
    return gen_draw(mt_key, mt_pos, has_gauss, cached_gauss, n_samples, lo, hi, n_opt, alpha,
                    spot0, ret_mu, ret_sigma, noise_sigma, params, spots, noise, nullptr);
}

extern "C" int dh_gen_locate(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss,
                             double* cached_gauss, int64_t n_samples, int n_opt,
                             const int64_t* starts, int64_t n_starts, double* loc) {
    return gen_locate(mt_key, mt_pos, has_gauss, cached_gauss, n_samples, n_opt, starts, n_starts,
                      loc);
}

extern "C" int dh_gen_draw_located(const double* loc, const int64_t* starts, int64_t n_starts,
                                   int64_t i_end, const double* lo, const double* hi, int n_opt,
                                   double ret_mu, double ret_sigma, double noise_sigma,
                                   double* params, double* rets, double* noise) {
    if (n_starts < 0 || n_opt < 0 || (n_starts > 0 && (!loc || !starts || !lo || !hi)))
        return DH_E_ARG;
    if (n_starts == 0) return DH_OK;
    for (int64_t j = 0; j < n_starts; ++j)
        if (starts[j] < 0 || (j > 0 && starts[j] < starts[j - 1])) return DH_E_ARG;
    if (i_end < starts[n_starts - 1]) return DH_E_ARG;
    const int64_t base = starts[0], n = i_end - base;
    if (n > 0 && (!params || !rets || (n_opt > 0 && !noise))) return DH_E_ARG;
    std::vector<LegacyRng> rs(n_starts);
    for (int64_t j = 0; j < n_starts; ++j)
        if (!loc_load(loc + j * kLocWords, rs[j])) return DH_E_ARG;
    double range[13];
    for (int j = 0; j < 13; ++j) range[j] = hi[j] - lo[j];
    auto chunk = [&](int64_t j) {
        const int64_t c1 = j + 1 < n_starts ? starts[j + 1] : i_end;
        draw_raw(rs[j], starts[j], c1, base, lo, range, n_opt, ret_mu, ret_sigma, noise_sigma,
                 params, rets, noise);
    };
    if (n_starts == 1 || n < kSplitMin) {
        for (int64_t j = 0; j < n_starts; ++j) chunk(j);
        return DH_OK;
    }
    std::atomic<int64_t> next{0};
    Team team((int)std::min<int64_t>(team_size(), n_starts));
    team.run([&](int) {
        for (int64_t j; (j = next.fetch_add(1)) < n_starts;) chunk(j);
    });
    return DH_OK;
}

extern "C" int dh_gen_sweep(double* params, double* spots, int64_t i0, int64_t n, double alpha,
                            double spot0, double* carry) {
    if (i0 < 0 || n < 0 || !carry || (n > 0 && (!params || !spots))) return DH_E_ARG;
    const double beta = 1.0 - alpha;                       // (1 - alpha), :108
    double prev_spot = i0 > 0 ? carry[13] : spot0;
    for (int64_t r = 0; r < n; ++r) {
        double* p = params + r * 13;
        if (i0 + r > 0) {
            const double* q = r > 0 ? p - 13 : carry;
            for (int j = 0; j < 13; ++j) p[j] = alpha * q[j] + beta * p[j];   // :105-109
            prev_spot = prev_spot * (1.0 + spots[r]);                         // :112-116
        }
        spots[r] = prev_spot;
    }
    if (n > 0) {
        for (int j = 0; j < 13; ++j) carry[j] = params[(n - 1) * 13 + j];
        carry[13] = prev_spot;
    }
    return DH_OK;
}

extern "C" int dh_gen_drawn_samples(int64_t* count) {
    if (!count) return DH_E_ARG;
    *count = g_drawn_total.load(std::memory_order_relaxed);
    return DH_OK;
}

extern "C" int dh_gen_draw_progress(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss,
                                    double* cached_gauss, int64_t n_samples, const double* lo,
                                    const double* hi, int n_opt, double alpha, double spot0,
                                    double ret_mu, double ret_sigma, double noise_sigma,
                                    double* params, double* spots, double* noise, int64_t* done) {
    if (!done) return DH_E_ARG;
    return gen_draw(mt_key, mt_pos, has_gauss, cached_gauss, n_samples, lo, hi, n_opt, alpha,
                    spot0, ret_mu, ret_sigma, noise_sigma, params, spots, noise, done);
}

// ---------------------------------------------------------------------------------------------
// dh_gen_assemble: the generator's per-sample host arithmetic after pricing
// (synthetic_generator.py:141-157), one pass over the batch on a worker team:
//   market = model + noise * model            (:141-142, NumPy's two roundings, no contraction)
//   rel    = (model - market) / market;  loss = mean(rel ** 2)          (:154-157)
//   strike = (K_rel * spot) / 100             (the columnar output's absolute strikes)
// loss is np.mean over a sample's options exactly as NumPy (2.x) forms it: add.reduce's pairwise
// sum of the row (plain below 8 terms, eight accumulators up to 128, halving above), then one
// division by the count (tests/test_generator_rng.py holds it to np.mean bit for bit).
// ---------------------------------------------------------------------------------------------
namespace {

double np_pairwise_sum(const double* a, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_sum(a, n2) + np_pairwise_sum(a + n2, n - n2);
}

}  // namespace

extern "C" int dh_gen_assemble(const double* model, const double* noise, const double* spots,
                               const double* k_rel, int64_t n_samples, int n_opt, double* market,
                               double* loss, double* strikes) {
    if (n_samples < 0 || n_opt < 0) return DH_E_ARG;
    if (n_samples == 0) return DH_OK;
    if (!loss) return DH_E_ARG;
    if (n_opt == 0) {
        for (int64_t i = 0; i < n_samples; ++i) loss[i] = NAN;   // mean of nothing (NumPy: nan)
        return DH_OK;
    }
    if (!model || !noise || !spots || !k_rel || !market || !loss || !strikes) return DH_E_ARG;
    auto sweep = [&](int64_t i0, int64_t i1) {
        std::vector<double> sq(n_opt);
        for (int64_t i = i0; i < i1; ++i) {
            const double* md = model + i * n_opt;
            const double* nz = noise + i * n_opt;
            double* mk = market + i * n_opt;
            double* st = strikes + i * n_opt;
            for (int j = 0; j < n_opt; ++j) {
                const double m = md[j] + nz[j] * md[j];
                const double r = (md[j] - m) / m;
                mk[j] = m;
                sq[j] = r * r;
                st[j] = (k_rel[j] * spots[i]) / 100.0;
            }
            loss[i] = np_pairwise_sum(sq.data(), n_opt) / (double)n_opt;
        }
    };
    if (n_samples < kSplitMin) {
        sweep(0, n_samples);
        return DH_OK;
    }
    Team team(team_size());
    const int nt = team.size();
    team.run([&](int w) { sweep(n_samples * w / nt, n_samples * (w + 1) / nt); });
    return DH_OK;
}

// ---------------------------------------------------------------------------------------------
// dh_gen_dates: the generator's trading dates (synthetic_generator.py:59-67: weekdays from
// 2022-01-03, a Monday, 'YYYY-MM-DD') as UCS-4 code points of a NumPy '<U10' array, one pass on
// a worker team: sample i falls on day first_day + 7 (i / 5) + i % 5 (days since 1970-01-01), and
// the civil date is H. Hinnant's days-to-civil algorithm.  Years past 9999 are the caller's
// (NumPy formats those; the call returns DH_E_ARG).
// ---------------------------------------------------------------------------------------------
extern "C" int dh_gen_dates(int64_t first_day, int64_t n, uint32_t* out) {
    if (n < 0 || (n > 0 && !out)) return DH_E_ARG;
    if (n == 0) return DH_OK;
    auto civil = [](int64_t z, int64_t& y, int& m, int& d) {
        z += 719468;
        const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
        const int64_t doe = z - era * 146097;
        const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
        const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
        const int64_t mp = (5 * doy + 2) / 153;
        d = (int)(doy - (153 * mp + 2) / 5 + 1);
        m = (int)(mp < 10 ? mp + 3 : mp - 9);
        y = yoe + era * 400 + (m <= 2);
    };
    {
        int64_t y;
        int m, d;
        civil(first_day + 7 * ((n - 1) / 5) + (n - 1) % 5, y, m, d);
        if (y > 9999 || first_day < 0) return DH_E_ARG;
    }
    auto sweep = [&](int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            int64_t y;
            int m, d;
            civil(first_day + 7 * (i / 5) + i % 5, y, m, d);
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
    };
    if (n < kSplitMin) {
        sweep(0, n);
        return DH_OK;
    }
    Team team(team_size());
    const int nt = team.size();
    team.run([&](int w) { sweep(n * w / nt, n * (w + 1) / nt); });
    return DH_OK;
}
