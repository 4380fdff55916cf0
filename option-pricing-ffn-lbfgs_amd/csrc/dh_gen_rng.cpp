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
#include <cmath>
#include <cstdint>
#include <cstring>

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

}  // namespace

extern "C" int dh_gen_draw(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss,
                           double* cached_gauss, int64_t n_samples, const double* lo,
                           const double* hi, int n_opt, double alpha, double spot0,
                           double ret_mu, double ret_sigma, double noise_sigma, double* params,
                           double* spots, double* noise) {
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
    std::memcpy(mt_key, g.key, sizeof(g.key));
    *mt_pos = g.pos;
    *has_gauss = g.has_gauss;
    *cached_gauss = g.gauss;
    return DH_OK;
}
