// dh_legacy_gauss.h -- the per-value arithmetic of NumPy's legacy RandomState draws, for host
// (g++ -ffp-contract=off) and device (hipcc, contraction off in these functions) alike:
//   * the MT19937 tempering and the legacy 53-bit double ((a >> 5) 2^26 + (b >> 6)) / 2^53;
//   * the polar test of a candidate pair (x = 2 d - 1, accepted while 0 < r2 < 1);
//   * the gauss value pair f x2 (returned) / f x1 (cached), f = sqrt(-2 log(r2) / r2), with
//     glibc 2.35's log restated operation for operation (its FMA build, the one libm runs on the
//     build container's and the GPU box's CPUs; constants in dh_glibc_log.h), so the device
//     draws of the generator take NumPy's bits (numpy/random/src/legacy/legacy-distributions.c
//     legacy_gauss; synthetic_generator.py:112-116, :141 call np.random.normal).
// IEEE add / mul / div / sqrt are correctly rounded on both sides; every fused multiply-add below
// is an explicit fma() where glibc's build has one and nowhere else.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#include "dh_glibc_log.h"

#if defined(__HIPCC__)
#define DH_LG __host__ __device__ inline
#else
#define DH_LG inline
#endif

namespace dhlog {

#if defined(__HIPCC__)
__device__ const double kTabDev[256] = DH_LOG_TAB_INIT;
#endif
static const double kTabHost[256] = DH_LOG_TAB_INIT;

DH_LG uint64_t bits_of(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint64_t)__double_as_longlong(x);
#else
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
#endif
}

DH_LG double double_of(uint64_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double((long long)u);
#else
    double d;
    std::memcpy(&d, &u, 8);
    return d;
#endif
}

DH_LG const double* tab() {
#if defined(__HIP_DEVICE_COMPILE__)
    return kTabDev;
#else
    return kTabHost;
#endif
}

// glibc's log(x) (sysdeps/ieee754/dbl-64/e_log.c, FMA build): the operations of its machine
// code in order -- r = fma(z, invc, -1), w = fma(k, ln2hi, logc), ...; see
// tools/gen_glibc_log_table.py for where the constants come from.
DH_LG double glibc_log(double x) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    uint64_t ix = bits_of(x);
    // 1 - 2^-4 <= x < 1 + 0x1.09p-4: log1p(r) by a degree-12 polynomial with an exact-ish head
    if (ix - 0x3fee000000000000ULL < 0x0003090000000000ULL) {
        if (ix == 0x3ff0000000000000ULL) return 0.0;
        const double r = x - 1.0;
        double a = fma(r, DH_LOG_B2, DH_LOG_B1);
        double b = fma(r, DH_LOG_B5, DH_LOG_B4);
        const double r2 = r * r;
        double c = fma(r, DH_LOG_B8, DH_LOG_B7);
        a = fma(r2, DH_LOG_B3, a);
        b = fma(r2, DH_LOG_B6, b);
        const double r3 = r * r2;
        c = fma(r2, DH_LOG_B9, c);
        c = fma(r3, DH_LOG_B10, c);
        const double q = fma(c, r3, b);
        const double pol = fma(q, r3, a);
        const double wq = fma(r, 0x1p27, r);          // r + r 2^27
        const double rhi = fma(-0x1p27, r, wq);       // (r + w) - w, w = r 2^27
        const double rhi2 = rhi * rhi;
        const double rlo = r - rhi;
        const double hi = fma(rhi2, DH_LOG_B0, r);
        const double lo0 = fma(rhi2, DH_LOG_B0, r - hi);
        const double lo = fma(DH_LOG_B0 * rlo, r + rhi, lo0);
        const double y = fma(pol, r3, lo);
        return hi + y;
    }
    const uint32_t top = (uint32_t)(ix >> 48);
    if (top - 0x10u > 0x7fdfu) {                     // zero, subnormal, negative, inf, nan
        if ((ix << 1) == 0) return -HUGE_VAL;
        if (ix == 0x7ff0000000000000ULL) return x;
        if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / (x - x);
        ix = bits_of(x * 0x1p52) + 0xfcc0000000000000ULL;   // subnormal: scale, k -= 52
    }
    const uint64_t tmp = ix + 0xc01a000000000000ULL;         // ix - 0x3fe6000000000000
    const int i = (int)((tmp >> 45) & 127);
    const int32_t k = (int32_t)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & 0xfff0000000000000ULL);
    const double invc = tab()[2 * i], logc = tab()[2 * i + 1];
    const double z = double_of(iz);
    const double kd = (double)k;
    const double r = fma(z, invc, -1.0);
    const double w = fma(kd, DH_LOG_LN2HI, logc);
    const double t1 = fma(r, DH_LOG_A2, DH_LOG_A1);
    const double hi = r + w;
    const double r2 = r * r;
    double lo = (w - hi) + r;
    lo = fma(kd, DH_LOG_LN2LO, lo);
    const double r3 = r * r2;
    const double t2 = fma(r, DH_LOG_A4, DH_LOG_A3);
    const double s = fma(r2, DH_LOG_A0, lo);
    const double p = fma(t2, r2, t1);
    const double y = fma(r3, p, s);
    return y + hi;
}

DH_LG uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// the legacy double of two tempered words (exact in fp64: no rounding anywhere)
DH_LG double mt_double(uint32_t w0, uint32_t w1) {
    const int32_t a = (int32_t)(w0 >> 5), b = (int32_t)(w1 >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

// legacy_gauss's candidate pair: x1 = 2 d0 - 1, x2 = 2 d1 - 1, r2 = x1^2 + x2^2 (two roundings)
DH_LG bool polar_pair(double d0, double d1, double& x1, double& x2, double& r2) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    x1 = 2.0 * d0 - 1.0;
    x2 = 2.0 * d1 - 1.0;
    r2 = x1 * x1 + x2 * x2;
    return r2 < 1.0 && r2 != 0.0;
}

// the two gauss values of an accepted pair: f x2 (returned by the call that drew it) and f x1
// (cached for the next call), f = sqrt(-2 log(r2) / r2)
DH_LG void gauss_values(double x1, double x2, double r2, double& g_new, double& g_cached) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    const double f = sqrt(-2.0 * glibc_log(r2) / r2);
    g_cached = f * x1;
    g_new = f * x2;
}

}  // namespace dhlog
