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

extern "C" int dh_gen_draw(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss,
                           double* cached_gauss, int64_t n_samples, const double* lo,
                           const double* hi, int n_opt, double alpha, double spot0,
                           double ret_mu, double ret_sigma, double noise_sigma, double* params,
                           double* spots, double* noise) {
    return gen_draw(mt_key, mt_pos, has_gauss, cached_gauss, n_samples, lo, hi, n_opt, alpha,
                    spot0, ret_mu, ret_sigma, noise_sigma, params, spots, noise, nullptr);
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
