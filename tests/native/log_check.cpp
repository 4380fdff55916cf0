// Host check of csrc/dh_legacy_gauss.h (test infrastructure, loaded only by tests/): the
// restated glibc log against libm's own log, bit for bit, and libm's log over caller arrays (the
// GPU test's reference values).  Built with -ffp-contract=off like the generator's host code.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <initializer_list>

#include "dh_legacy_gauss.h"

namespace {

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

}  // namespace

extern "C" {

// n values of each kind from seed: the polar method's r2 (x1^2 + x2^2 of legacy doubles, kept
// when 0 < r2 < 1: what legacy_gauss passes to log), uniform doubles in (0, 1), and random bit
// patterns of positive finite doubles (every exponent, subnormals included).  Returns the number
// of inputs whose restated log differs from libm's in any bit; *first_bad gets the first one.
int64_t dh_log_mismatches(uint64_t seed, int64_t n, double* first_bad) {
    int64_t bad = 0;
    uint64_t s = seed;
    auto check = [&](double x) {
        const double a = std::log(x), b = dhlog::glibc_log(x);
        if (std::memcmp(&a, &b, 8) != 0) {
            if (bad == 0 && first_bad) *first_bad = x;
            ++bad;
        }
    };
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t w = splitmix(s), v = splitmix(s);
        const double d0 = dhlog::mt_double((uint32_t)w, (uint32_t)(w >> 32));
        const double d1 = dhlog::mt_double((uint32_t)v, (uint32_t)(v >> 32));
        double x1, x2, r2;
        if (dhlog::polar_pair(d0, d1, x1, x2, r2)) check(r2);
        check(d0 > 0.0 ? d0 : 0.5);
        uint64_t u = splitmix(s) & 0x7fffffffffffffffULL;
        if ((u >> 52) == 0x7ff) u &= 0x7fefffffffffffffULL;   // keep it finite
        double x;
        std::memcpy(&x, &u, 8);
        if (x > 0.0) check(x);
    }
    for (double x : {1.0, 1.0 - 0x1p-4, 1.0 + 0x1.09p-4, 0x1p-1074, 0x1p-1022, 0.5, 2.0,
                     1e-300, 1e300, 0x1.fffffffffffffp1023, 0.9375, 0.93749999999999989})
        check(x);
    return bad;
}

// libm's log of x[i] (the reference values of the device restatement's GPU test)
void dh_libm_log(const double* x, int64_t n, double* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = std::log(x[i]);
}

// the restatement on the host (for the same comparison from Python)
void dh_restated_log(const double* x, int64_t n, double* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = dhlog::glibc_log(x[i]);
}

}  // extern "C"
