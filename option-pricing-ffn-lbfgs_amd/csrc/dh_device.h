// dh_device.h -- fp64 device math for the Double-Heston + Merton-jump COS pricer (gfx950).
//
// Every function restates one piece of the reference model (zenthepen/Option-Pricing-FFN-LBFGS,
// src/models/double_heston.py) in the same arithmetic order, so that GPU prices track the
// reference to ~1e-14 relative.  Complex helpers follow the semantics the reference inherits from
// NumPy/CPython: principal-branch sqrt and log, Smith division with a reciprocal scale (NumPy's
// scalar complex division), exp(x)(cos y, sin y).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "dh_exp_table.h"
#include "dh_logatan_table.h"
#include "dh_sincos_table.h"

namespace dh {

constexpr double kPi = 3.141592653589793;  // np.pi

struct cplx {
    double re, im;
};

__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cplx csub(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ cplx cscale(cplx a, double s) { return {a.re * s, a.im * s}; }

// Smith's algorithm with a reciprocal scale factor (NumPy scalar complex division).
__device__ __forceinline__ cplx cdiv(cplx a, cplx b) {
    const double abr = fabs(b.re), abi = fabs(b.im);
    if (abr >= abi) {
        if (abr == 0.0 && abi == 0.0) return {a.re / abr, a.im / abr};
        const double rat = b.im / b.re;
        const double scl = 1.0 / (b.re + b.im * rat);
        return {(a.re + a.im * rat) * scl, (a.im - a.re * rat) * scl};
    }
    const double rat = b.re / b.im;
    const double scl = 1.0 / (b.im + b.re * rat);
    return {(a.re * rat + a.im) * scl, (a.im * rat - a.re) * scl};
}

// Principal square root (Re >= 0), glibc csqrt identity 2 Re Im = Im z for the small half.
__device__ __forceinline__ cplx csqrt_p(cplx z) {
    const double x = z.re, y = z.im;
    if (x == 0.0 && y == 0.0) return {0.0, y};
    const double h = hypot(x, y);
    if (x > 0.0) {
        const double r = sqrt(0.5 * (h + x));
        return {r, 0.5 * (y / r)};
    }
    const double s = sqrt(0.5 * (h - x));
    return {fabs(0.5 * (y / s)), copysign(s, y)};
}

// sin and cos of one argument: 3-part Cody-Waite reduction by pi/2 with FMA, then the fdlibm
// kernel polynomials on [-pi/4, pi/4] (coefficients of __kernel_sin / __kernel_cos).  Max error
// ~2 ulp for |x| < 2^20 (every argument on this path is bounded by N pi plus the CF phases);
// accuracy degrades gracefully beyond, and non-finite x gives NaN like libm.  Replaces ocml's
// sincos, whose inlined Payne-Hanek branch costs ~100 VGPRs per call site.
__device__ __forceinline__ double flip_sign(double v, int neg) {   // neg: 0 or 1
    return __hiloint2double(__double2hiint(v) ^ (neg << 31), __double2loint(v));
}

// c + z * p as one fp64 FMA with the constant c read from an SGPR pair.  The compiler's own
// choice for a polynomial step is v_fmac_f64, whose tied accumulator needs a VGPR copy of c (two
// v_mov_b32 per step, ~30% of a Horner chain's VALU issue).  Here the constant is written into a
// fixed, clobbered SGPR pair (s[96:97]) by two s_mov_b32 inside the same asm statement, then
// read by a VOP3 v_fma_f64: the constant traffic is scalar (it co-issues with other waves' VALU),
// and since each step materialises its own constant the compiler has nothing to hoist -- hoisted
// constants had exhausted the SGPR file and been spilled to VGPR lanes (v_writelane /
// v_readlane, ~5% of the CF loop's VALU).  Same rounding as fma().
template <unsigned long long B>
__device__ __forceinline__ double fma_kc(double z, double p) {
    double r;
    asm("s_mov_b32 s96, %3\n\ts_mov_b32 s97, %4\n\tv_fma_f64 %0, %1, %2, s[96:97]"
        : "=v"(r)
        : "v"(z), "v"(p), "i"((unsigned)(B & 0xffffffffull)), "i"((unsigned)(B >> 32))
        : "s96", "s97");
    return r;
}
#define fma_k(z, p, c) fma_kc<__builtin_bit_cast(unsigned long long, (double)(c))>((z), (p))

__device__ __forceinline__ void dsincos(double x, double* sp, double* cp) {
    const double q = rint(x * 6.36619772367581382433e-01);           // x * 2/pi
    double r = fma(-q, 1.57079632679489655800e+00, x);                 // pi/2, 3 parts
    r = fma(-q, 6.12323399573676588613e-17, r);
    r = fma(-q, -1.49738490485916983089e-33, r);
    const double z = r * r;
    double ps = fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
    ps = fma_k(z, ps, 2.75573137070700676789e-06);
    ps = fma_k(z, ps, -1.98412698298579493134e-04);
    ps = fma_k(z, ps, 8.33333333332248946124e-03);
    ps = fma_k(z, ps, -1.66666666666666324348e-01);
    const double s = fma(r * z, ps, r);
    double pc = fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
    pc = fma_k(z, pc, -2.75573143513906633035e-07);
    pc = fma_k(z, pc, 2.48015872894767294178e-05);
    pc = fma_k(z, pc, -1.38888888888741095749e-03);
    pc = fma_k(z, pc, 4.16666666666666019037e-02);
    pc = z * pc;
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + z * pc);
    // quadrant from the low bits of q (q is an exact integer; |q| < 2^31 on this path)
    const int qi = (int)q;
    const bool swap = qi & 1;
    *sp = flip_sign(swap ? c : s, (qi >> 1) & 1);
    *cp = flip_sign(swap ? s : c, ((qi + 1) >> 1) & 1);
}

// sin and cos by a 128-entry table (the CF loop's form): x = q pi/64 + r with |r| <= pi/128 (the
// 3-part FMA Cody-Waite reduction of dsincos scaled by 2^-5, exact), sin/cos(q pi/64) from an LDS
// copy of kSinCosPi64 (one ds_read_b128; correctly rounded entries), sin r and cos r by Taylor
// polynomials through r^7 / r^8 (the next terms are < 1e-18 relative), then the angle-addition
// formulas.  ~1 ulp for |x| < 2^20; 17 VALU instructions against dsincos's 41.
// Table lookups of the CF loop round their index with the 1.5 * 2^52 shift: qd = fma(x, c, shift)
// is shift + rint(x c) (its ulp is 1) and the low word of qd holds rint(x c) as a two's-
// complement integer, so the index needs no float-to-int conversion (a NaN x gives a defined
// index, masked in range, and a NaN result).  q = qd - shift is exact.
constexpr double kShift52 = 0x1.8p52;

__device__ __forceinline__ void dsincos_t(double x, const double2* __restrict__ tab, double* sp,
                                          double* cp) {
    const double qd = fma(x, 20.371832715762604, kShift52);          // rint(x 64/pi)
    const double q = qd - kShift52;
    double r = fma(-q, 0.04908738521234052, x);                        // pi/64, 3 parts
    r = fma(-q, 1.9135106236677394e-18, r);
    r = fma(-q, -4.6793278276849057e-35, r);
    const double2 sc = tab[__double2loint(qd) & 127];                  // sin, cos (q pi/64)
    const double z = r * r;
    double ps = fma(z, -0.0001984126984126984, 0.008333333333333333);
    ps = fma_k(z, ps, -0.16666666666666666);
    const double sr = fma(r * z, ps, r);                               // sin r
    double pc = fma(z, 2.48015873015873e-05, -0.001388888888888889);
    pc = fma_k(z, pc, 0.041666666666666664);
    const double cr = fma(z * z, pc, fma(z, -0.5, 1.0));               // cos r
    *sp = fma(sc.x, cr, sc.y * sr);
    *cp = fma(sc.y, cr, -(sc.x * sr));
}

// exp(x): restates the ROCm device library's __ocml_exp_f64 operation for operation (same
// reduction constants, degree-11 polynomial and range clamps, so the same bits), with the
// polynomial steps in the fma_k form.
__device__ __forceinline__ double dexp(double x) {
    const double q = rint(x * 0x1.71547652b82fep+0);                 // x log2(e)
    double r = fma(q, -0x1.62e42fefa39efp-1, x);                      // x - q ln2 (2 parts)
    r = fma(q, -0x1.abc9e3b39803fp-56, r);
    double p = fma(0x1.ade156a5dcb37p-26, r, 0x1.28af3fca7ab0cp-22);
    p = fma_k(r, p, 0x1.71dee623fde64p-19);
    p = fma_k(r, p, 0x1.a01997c89e6b0p-16);
    p = fma_k(r, p, 0x1.a01a014761f6ep-13);
    p = fma_k(r, p, 0x1.6c16c1852b7b0p-10);
    p = fma_k(r, p, 0x1.1111111122322p-7);
    p = fma_k(r, p, 0x1.55555555502a1p-5);
    p = fma_k(r, p, 0x1.5555555555511p-3);
    p = fma_k(r, p, 0x1.000000000000bp-1);
    p = fma(r, p, 1.0);
    p = fma(r, p, 1.0);
    double e = ldexp(p, (int)q);
    e = (x > 1024.0) ? INFINITY : e;
    return (x < -1075.0) ? 0.0 : e;
}

// dexp for x <= 0 (or -inf / NaN): the same bits without the overflow select (the CF's
// e^{-Re(d) tau} and Gaussian jump factor e^{-sj^2 u^2 / 2}).
__device__ __forceinline__ double dexp_nonpos(double x) {
    const double q = rint(x * 0x1.71547652b82fep+0);
    double r = fma(q, -0x1.62e42fefa39efp-1, x);
    r = fma(q, -0x1.abc9e3b39803fp-56, r);
    double p = fma(0x1.ade156a5dcb37p-26, r, 0x1.28af3fca7ab0cp-22);
    p = fma_k(r, p, 0x1.71dee623fde64p-19);
    p = fma_k(r, p, 0x1.a01997c89e6b0p-16);
    p = fma_k(r, p, 0x1.a01a014761f6ep-13);
    p = fma_k(r, p, 0x1.6c16c1852b7b0p-10);
    p = fma_k(r, p, 0x1.1111111122322p-7);
    p = fma_k(r, p, 0x1.55555555502a1p-5);
    p = fma_k(r, p, 0x1.5555555555511p-3);
    p = fma_k(r, p, 0x1.000000000000bp-1);
    p = fma(r, p, 1.0);
    p = fma(r, p, 1.0);
    return (x < -1075.0) ? 0.0 : ldexp(p, (int)q);
}

__device__ __forceinline__ cplx cexp_(cplx z) {
    double s, c;
    dsincos(z.im, &s, &c);
    const double e = exp(z.re);
    return {e * c, e * s};
}

// Principal log: arg in (-pi, pi].
__device__ __forceinline__ cplx clog_(cplx z) { return {log(hypot(z.re, z.im)), atan2(z.im, z.re)}; }

// ---- lean fp64 elementary functions for the hot kernels ------------------------------------
// Measured on gfx950 (tools/ubench/fp64_latency.hip, cycles of issue per wave64): IEEE division
// ~70, ocml sqrt ~110, exp ~120, ocml log ~456, ocml atan2 ~255, an fp64 FMA ~5.5.  The COS
// table is issue-bound, so these restate the needed functions with v_rcp_f64 / v_rsq_f64 seeds
// and Newton/Goldschmidt steps (<= ~2 ulp; NaN in gives NaN out; used on finite operands).

// 1/x: v_rcp_f64 seed + two Newton steps.
__device__ __forceinline__ double drcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// sqrt(x) and 1/sqrt(x) together: v_rsq_f64 seed + one Goldschmidt step + residual correction.
__device__ __forceinline__ void dsqrt_rsqrt(double x, double& sq, double& rs) {
    const double y0 = __builtin_amdgcn_rsq(x);
    double g = x * y0, h = 0.5 * y0;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    const double d = fma(-g, g, x);
    sq = fma(h, d, g);
    rs = 2.0 * h;
    if (x == 0.0 || isinf(x)) sq = x;
}

__device__ __forceinline__ double dsqrt(double x) {
    double s, r;
    dsqrt_rsqrt(x, s, r);
    return s;
}

// The same for x finite and > 0 (the CF's |dd|^2 and (|dd| + |Re dd|)/2: dd = beta^2 +
// sigma^2 u (u + i) is never 0 for kappa, sigma > 0), without the 0 / inf special case.
__device__ __forceinline__ void dsqrt_rsqrt_pos(double x, double& sq, double& rs) {
    const double y0 = __builtin_amdgcn_rsq(x);
    double g = x * y0, h = 0.5 * y0;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    const double d = fma(-g, g, x);
    sq = fma(h, d, g);
    rs = 2.0 * h;
}

// log(x): fdlibm e_log.c, x = 2^k (1 + f), sqrt(1/2) <= 1 + f < sqrt(2), s = f / (2 + f).
__device__ __forceinline__ double dlog(double x) {
    int k;
    double m = frexp(x, &k);                         // m in [0.5, 1)
    const bool lo = m < 0.70710678118654752440;
    m = lo ? 2.0 * m : m;
    k = lo ? k - 1 : k;
    const double f = m - 1.0;
    const double s = f * drcp(2.0 + f);
    const double z = s * s, w = z * z;
    double p1 = fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01);
    p1 = fma_k(w, p1, 3.999999999940941908e-01);
    const double t1 = w * p1;
    double p2 = fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01);
    p2 = fma_k(w, p2, 2.857142874366239149e-01);
    p2 = fma_k(w, p2, 6.666666666666735130e-01);
    const double t2 = z * p2;
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double dk = (double)k;
    const double r = dk * 6.93147180369123816490e-01 -
                     ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
    // special values: log(0) = -inf, log(x < 0) = NaN, log(inf) = inf, log(NaN) = NaN
    if (!(x > 0.0) || isinf(x)) return (x == 0.0) ? -INFINITY : (x > 0.0 ? x : NAN + x);
    return r;
}

// atan2(y, x) in (-pi, pi]: t = min/max in [0, 1]; for t > tan(pi/8) use
// atan t = pi/4 + atan((t - 1)/(t + 1)) with (t - 1)/(t + 1) = (mn - mx)/(mn + mx), so one
// reciprocal serves both ranges; the fdlibm s_atan.c polynomial on |t'| <= tan(pi/8).
// Branch-free (every case is a select the compiler keeps as one): zeros need no special case
// (the reciprocal's argument is clamped to the smallest normal, so t = 0 for x = y = 0, and the
// sign bit of x selects pi - a, giving atan2(+-0, -0) = +-pi); the one deviation from libm is
// x = -0 with y != 0, which returns pi/2 one ulp high.
__device__ __forceinline__ double datan2(double y, double x) {
    const double ax = fabs(x), ay = fabs(y);
    const double mx = fmax(ax, ay), mn = fmin(ax, ay);
    const bool big = mn > 0.41421356237309503 * mx;
    const double tr = (big ? mn - mx : mn) * drcp(fmax(big ? mn + mx : mx, 2.2250738585072014e-308));
    const double z = tr * tr, w = z * z;
    double p1 = fma(w, 1.62858201153657823623e-02, 4.97687799461593236017e-02);
    p1 = fma_k(w, p1, 6.66107313738753120669e-02);
    p1 = fma_k(w, p1, 9.09088713343650656196e-02);
    p1 = fma_k(w, p1, 1.42857142725034663711e-01);
    p1 = fma_k(w, p1, 3.33333333333329318027e-01);
    const double s1 = z * p1;
    double p2 = fma(w, -3.65315727442169155270e-02, -5.83357013379057348645e-02);
    p2 = fma_k(w, p2, -7.69187620504482999495e-02);
    p2 = fma_k(w, p2, -1.11111104054623557880e-01);
    p2 = fma_k(w, p2, -1.99999999998764832476e-01);
    const double s2 = w * p2;
    const double at = tr - tr * (s1 + s2);
    double a = big ? 7.85398163397448278999e-01 + (at + 3.06161699786838301793e-17) : at;
    a = (ay > ax) ? (1.57079632679489655800e+00 - a) + 6.12323399573676588613e-17 : a;
    a = signbit(x) ? (3.14159265358979311600e+00 - a) + 1.22464679914735317720e-16 : a;
    a = copysign(a, y);
    return (isnan(x) || isnan(y)) ? x + y : a;
}

// ---- table-driven log, atan2 and exp of the CF loop --------------------------------------------
// The CF's math tables in one LDS array of double2 (load_math_tables): [0, 128) sin / cos of
// j pi/64 (dsincos_t), [128, 256) (invc, logc) of dlog_t, [256, 321) atan(j/64) (hi, lo) of
// datan2_t, [321, 353) 2^(j/64), j = 0..63, two per entry, of dexp_t.
constexpr int kTabLog = 128;
constexpr int kTabAtan = 256;
constexpr int kTabExp = 321;
constexpr int kMathTab = 353;

// log(x) for normal x > 0 (glibc's table layout, tools/gen_logatan_tables.py): x = 2^k z with z
// in [0.6875, 1.375) from the bits, subinterval i by the next 7 bits, r = z invc_i - 1 (one FMA,
// |r| < 2^-8), log x = k ln2 + logc_i + log1p(r) with log1p by its Taylor series through r^7
// (remainder < 2^-67).  Absolute error ~1 ulp of the result's scale (no special path near 1,
// where only absolute accuracy matters here).  ~20 VALU against dlog's ~40.
__device__ __forceinline__ double dlog_t(double x, const double2* __restrict__ tab) {
    // glibc's 64-bit integer steps on the high word only (the constant's low word is 0, so the
    // subtraction never borrows): tmp = hi(x) - 0x3fe60000, i = tmp >> 13 & 127, k = tmp >> 20
    const int hx = __double2hiint(x);
    const int tmp = hx - 0x3fe60000;
    const double kd = (double)(tmp >> 20);
    const double z = __hiloint2double(hx - (tmp & (int)0xfff00000), __double2loint(x));
    const double2 e = tab[kTabLog + ((tmp >> 13) & 127)];            // (invc, logc)
    const double r = fma(z, e.x, -1.0);
    const double w = fma(kd, 0x1.62e42fefa3800p-1, e.y);             // k ln2_hi exact (|k| < 2^11)
    const double hi = w + r;
    const double lo = fma(kd, 0x1.ef35793c76730p-45, (w - hi) + r);  // k ln2_lo
    double p = fma(r, 0.14285714285714285, -0.16666666666666666);
    p = fma_k(r, p, 0.2);
    p = fma_k(r, p, -0.25);
    p = fma_k(r, p, 0.3333333333333333);
    p = fma_k(r, p, -0.5);
    const double y = fma(r * r, p, lo) + hi;
    // positive normal x only (v_cmp_class: class bit 8 = +normal); anything else -- 0, inf, NaN,
    // negative or subnormal, none of which |Q|^2 reaches for finite parameters -- gives NaN, so
    // an out-of-range input surfaces as an invalid price instead of a wrong finite value
    return __builtin_amdgcn_class(x, 1 << 8) ? y : NAN;
}

// atan2(y, x) in (-pi, pi], as datan2 but with the polynomial's range cut to |t'| <= 2^-7 by a
// table: t = min/max(|x|, |y|) in [0, 1] (the v_rcp_f64 seed is enough to pick j = rint(64 t)),
// then atan t = atan(j/64) + atan(t') with t' = (mn - mx s)/(mx + mn s), s = j/64 exact, both
// FMAs; atan t' to t'^7.  Same quadrant rules as datan2.  For the CF only: x, y finite and not
// both 0 (D conj(d)), no NaN handling -- a NaN D makes log|Q|^2 NaN (dlog_t), and so the price.
// ~35 VALU against datan2's ~50.
__device__ __forceinline__ double datan2_t(double y, double x, const double2* __restrict__ tab) {
    const double ax = fabs(x), ay = fabs(y);
    const double mx = fmax(ax, ay), mn = fmin(ax, ay);
    const double t0 = mn * __builtin_amdgcn_rcp(mx);
    // j = rint(64 t0) in 0 .. 64 by the shift (kShift52): a NaN t0 (NaN operands, or D conj(d) =
    // 0) gives a defined index <= 127 (an entry of the next table) and a NaN result, never a NaN
    // converted to int
    const double qd = fma(t0, 64.0, kShift52);
    const double sj = (qd - kShift52) * 0.015625;                     // j / 64, exact
    const double xp = fma(mn, sj, mx), yp = fma(-mx, sj, mn);
    const double tp = yp * drcp(xp);
    const double z = tp * tp;
    double q = fma(z, -0.14285714285714285, 0.2);
    q = fma_k(z, q, -0.3333333333333333);
    const double at = fma(tp * z, q, tp);
    const double2 e = tab[kTabAtan + (__double2loint(qd) & 127)];    // atan(j/64) hi, lo
    double a = e.x + (at + e.y);
    a = (ay > ax) ? (1.57079632679489655800e+00 - a) + 6.12323399573676588613e-17 : a;
    a = signbit(x) ? (3.14159265358979311600e+00 - a) + 1.22464679914735317720e-16 : a;
    return copysign(a, y);
}

// exp(x) by a 64-entry table (tools/gen_exp_table.py): x = (64 e + j) ln2/64 + r with |r| <=
// ln2/128, q = 64 e + j rounded by the 1.5 * 2^52 shift (its low word IS q, so no float-to-int
// conversion: a NaN x indexes a defined entry and stays NaN through r), e^r - 1 by its Taylor
// series through r^5 (remainder < 4e-17 relative), then 2^e (t + t (e^r - 1)) with t = 2^(j/64)
// correctly rounded.  ~1 ulp (a hi + lo table would give ~0.5 ulp but held two more VGPRs live
// across the polynomial: spills in the <= 96-VGPR fused build); 11 fp64 VALU against dexp's 19.
// Finite x <= 709 (the CF's exponents); callers select the overflow / underflow ends.
__device__ __forceinline__ double dexp_t_core(double x, const double2* __restrict__ tab) {
    const double qd = fma(x, 0x1.71547652b82fep+6, kShift52);        // rint(x 64/ln2)
    const double q = qd - kShift52;
    const int qi = __double2loint(qd);                                // q as int32
    double r = fma(q, -0x1.62e42fefa39efp-7, x);                      // ln2/64, 2 parts
    r = fma(q, -0x1.abc9e3b39803fp-62, r);
    double p = fma(r, 0.008333333333333333, 0.041666666666666664);
    p = fma_k(r, p, 0.16666666666666666);
    p = fma_k(r, p, 0.5);
    const double em1 = fma(r * r, p, r);                              // e^r - 1
    const double t = ((const double*)(tab + kTabExp))[qi & 63];       // 2^(j/64)
    return ldexp(fma(t, em1, t), qi >> 6);
}

__device__ __forceinline__ double dexp_t(double x, const double2* __restrict__ tab) {
    const double e = dexp_t_core(x, tab);
    return (x > 709.8) ? INFINITY : ((x < -1075.0) ? 0.0 : e);
}

// dexp_t for x <= 0 (or -inf / NaN): the CF's e^{-Re(d) tau} and Gaussian jump factor.
__device__ __forceinline__ double dexp_t_nonpos(double x, const double2* __restrict__ tab) {
    const double e = dexp_t_core(x, tab);
    return (x < -1075.0) ? 0.0 : e;
}

// z1 / z2 through one reciprocal of |z2|^2 (no Smith scaling: |z2| on this path stays far
// from the fp64 over/underflow thresholds).
__device__ __forceinline__ cplx cdiv_rcp(cplx a, cplx b) {
    const double inv = drcp(fma(b.re, b.re, b.im * b.im));
    return {(a.re * b.re + a.im * b.im) * inv, (a.im * b.re - a.re * b.im) * inv};
}

// Param-set record (DH_PARAM_STRIDE = 16 doubles), double_heston.py:26-46 argument order.
struct Params {
    double v01, k1, t1, s1, r1, v02, k2, t2, s2, r2, lam, muj, sj, S0, r, q;
};

__device__ __forceinline__ Params load_params(const double* __restrict__ p) {
    Params P;
    P.v01 = p[0]; P.k1 = p[1]; P.t1 = p[2]; P.s1 = p[3]; P.r1 = p[4];
    P.v02 = p[5]; P.k2 = p[6]; P.t2 = p[7]; P.s2 = p[8]; P.r2 = p[9];
    P.lam = p[10]; P.muj = p[11]; P.sj = p[12]; P.S0 = p[13]; P.r = p[14]; P.q = p[15];
    return P;
}

// One variance factor of the CF (double_heston.py:64-71 / :73-80 and its A-part :85-91).
// Returns B_j; accumulates the factor's contribution into A.
__device__ __forceinline__ cplx heston_factor(double u, double tau, double kap, double th,
                                              double sig, double rho, cplx& A) {
    const cplx beta = {kap, -((rho * sig) * u)};          // kappa - rho sigma i u
    const double s2 = sig * sig;                          // sigma**2
    const double s2u = s2 * u;
    const cplx quad = {s2u * u, s2u};                     // sigma^2 u (u + i)
    const cplx d = csqrt_p(cadd(cmul(beta, beta), quad)); // :64-65
    const cplx bm = csub(beta, d);
    const cplx g = cdiv(bm, cadd(beta, d));               // :67-68
    const cplx e = cexp_({-d.re * tau, -d.im * tau});     // exp(-d tau)
    const cplx one_m_ge = {1.0 - (g.re * e.re - g.im * e.im), -(g.re * e.im + g.im * e.re)};
    const cplx B = cmul(cdiv(bm, {s2, 0.0}), cdiv({1.0 - e.re, -e.im}, one_m_ge));  // :70-71
    const cplx lg = clog_(cdiv(one_m_ge, {1.0 - g.re, -g.im}));
    const double coef = (kap * th) / s2;                  // kappa theta / sigma^2
    const cplx inner = {bm.re * tau - 2.0 * lg.re, bm.im * tau - 2.0 * lg.im};
    A = cadd(A, cscale(inner, coef));                     // :85-91
    return B;
}

// phi(u; tau) = exp(A + B1 v01 + B2 v02) * phi_jump  (double_heston.py:48-97).
__device__ __forceinline__ cplx cf_eval(const Params& P, double u, double tau) {
    const double comp = exp(P.muj + 0.5 * (P.sj * P.sj)) - 1.0;      // :82
    cplx A = {0.0, ((P.r - P.q - P.lam * comp) * u) * tau};           // :83
    const cplx B1 = heston_factor(u, tau, P.k1, P.t1, P.s1, P.r1, A);
    const cplx B2 = heston_factor(u, tau, P.k2, P.t2, P.s2, P.r2, A);
    const double half_sj2 = 0.5 * (P.sj * P.sj);
    const cplx ej = cexp_({-(half_sj2 * (u * u)), u * P.muj});        // exp(i u mu - sj^2 u^2 / 2)
    const double lt = P.lam * tau;
    const cplx jump = cexp_({lt * (ej.re - 1.0), lt * ej.im});        // :93
    const cplx ex = {A.re + B1.re * P.v01 + B2.re * P.v02, A.im + B1.im * P.v01 + B2.im * P.v02};
    return cmul(cexp_(ex), jump);                                     // :94-96
}

// One variance factor at a complex frequency phi (double_heston.py:64-71 / :73-80, :85-91), in
// the reference's operation order on complex operands: beta = kappa - rho sigma i phi, d =
// sqrt(beta^2 + sigma^2 phi (phi + i)), the same g, B and log terms as heston_factor.
__device__ __forceinline__ cplx heston_factor_z(cplx phi, double tau, double kap, double th,
                                                double sig, double rho, cplx& A) {
    const cplx iphi = {-phi.im, phi.re};                  // i phi
    const cplx beta = csub({kap, 0.0}, cscale(iphi, rho * sig));
    const double s2 = sig * sig;
    const cplx quad = cmul(cscale(phi, s2), {phi.re, phi.im + 1.0});   // sigma^2 phi (phi + i)
    const cplx d = csqrt_p(cadd(cmul(beta, beta), quad));
    const cplx bm = csub(beta, d);
    const cplx g = cdiv(bm, cadd(beta, d));
    const cplx e = cexp_({-(d.re * tau), -(d.im * tau)});
    const cplx ge = cmul(g, e);
    const cplx one_m_ge = {1.0 - ge.re, -ge.im};
    const cplx B = cmul(cdiv(bm, {s2, 0.0}), cdiv({1.0 - e.re, -e.im}, one_m_ge));
    const cplx lg = clog_(cdiv(one_m_ge, {1.0 - g.re, -g.im}));
    const double coef = (kap * th) / s2;
    const cplx inner = {bm.re * tau - 2.0 * lg.re, bm.im * tau - 2.0 * lg.im};
    A = cadd(A, cscale(inner, coef));
    return B;
}

// phi at a complex frequency (double_heston.py:48-97 documents phi : complex): the reference's
// expressions with complex phi throughout, for DoubleHeston.characteristic_function on complex
// input (dh_cf_complex).  Matches the reference to ~1e-14 relative, not bit for bit.
__device__ __forceinline__ cplx cf_eval_z(const Params& P, cplx phi, double tau) {
    const double comp = exp(P.muj + 0.5 * (P.sj * P.sj)) - 1.0;      // :82
    const cplx iphi = {-phi.im, phi.re};
    cplx A = cscale(iphi, (P.r - P.q - P.lam * comp) * tau);         // :83
    const cplx B1 = heston_factor_z(phi, tau, P.k1, P.t1, P.s1, P.r1, A);
    const cplx B2 = heston_factor_z(phi, tau, P.k2, P.t2, P.s2, P.r2, A);
    const cplx phi2 = cmul(phi, phi);
    const cplx arg = csub(cscale(iphi, P.muj), cscale(phi2, 0.5 * (P.sj * P.sj)));
    const cplx ej = cexp_(arg);                                       // e^{i phi mu - sj^2 phi^2/2}
    const double lt = P.lam * tau;
    const cplx jump = cexp_({lt * (ej.re - 1.0), lt * ej.im});        // :93
    const cplx ex = {A.re + (B1.re * P.v01) + (B2.re * P.v02), A.im + (B1.im * P.v01) + (B2.im * P.v02)};
    return cmul(cexp_(ex), jump);                                     // :94-96
}

// ---- fast CF for the COS table: exponent form ----------------------------------------------
// phi(u) = exp(E) with E = A + B1 v01 + B2 v02 + lambda tau (e^{i u mu - sj^2 u^2/2} - 1); the
// table only needs Re(phi e^{-i u a}) = e^{Re E} cos(Im E - u a), so the three final complex
// exponentials and two complex products of cf_eval collapse into one exp and one cos.  Per factor,
// g = (beta - d)/(beta + d) is eliminated algebraically:
//   (1 - e)/(1 - g e) = (1 - e)(beta + d) / D,   (1 - g e)/(1 - g) = D / (2 d),
//   D = (beta + d) - (beta - d) e,  e = exp(-d tau)
// which is the same 'little Heston trap' quantity, with two complex divisions instead of three.
struct FactorC {
    double kap, rs, s2, inv_s2, coef, v0;   // kappa, rho sigma, sigma^2, 1/sigma^2, k th/s^2, v0
};

__device__ __forceinline__ FactorC factor_consts(double v0, double kap, double th, double sig,
                                                 double rho) {
#pragma clang fp contract(off)   // the same bits in every prologue form (table, fused)
    FactorC F;
    F.kap = kap;
    F.rs = rho * sig;
    F.s2 = sig * sig;
    F.inv_s2 = 1.0 / F.s2;
    F.coef = (kap * th) / F.s2;
    F.v0 = v0;
    return F;
}

// One factor's contribution X to the exponent E: kappa theta / sigma^2 ((beta - d) tau - 2 log Q)
// + B v0.  E = ((D + X1) + X2) + J with D = (0, drift u) and J the jump part, in that order in every
// path, so every path agrees.
__device__ __forceinline__ cplx factor_x(const FactorC& F, double u, double tau,
                                         const double2* __restrict__ sct) {
    const cplx beta = {F.kap, -(F.rs * u)};
    const double s2u = F.s2 * u;
    const cplx dd = {fma(beta.re, beta.re, -beta.im * beta.im) + s2u * u,
                     2.0 * beta.re * beta.im + s2u};
    // principal sqrt: |dd|, then sqrt((|dd| + |Re|)/2) and its reciprocal (no division)
    double h, rh, sq, rs;                            // h = |dd| = |d|^2, rh = 1/|dd|
    dsqrt_rsqrt_pos(fma(dd.re, dd.re, dd.im * dd.im), h, rh);
    dsqrt_rsqrt_pos(0.5 * (h + fabs(dd.re)), sq, rs);
    const double other = 0.5 * dd.im * rs;
    const double dre = dd.re > 0.0 ? sq : fabs(other);
    const double dim = dd.re > 0.0 ? other : copysign(sq, dd.im);
    const cplx bm = {beta.re - dre, beta.im - dim};
    const cplx bp = {beta.re + dre, beta.im + dim};
    double es, ec;
    dsincos_t(-dim * tau, sct, &es, &ec);
    const double em = dexp_t_nonpos(-dre * tau, sct);
    const cplx e = {em * ec, em * es};
    const cplx D = {bp.re - (bm.re * e.re - bm.im * e.im), bp.im - (bm.re * e.im + bm.im * e.re)};
    const cplx ome = {1.0 - e.re, -e.im};
    const cplx num = cmul(cscale(bm, F.inv_s2), cmul(ome, bp));
    const cplx B = cdiv_rcp(num, D);
    // log Q, Q = D / (2d), without the division: |Q|^2 = |D|^2 / (4 |dd|) (|d|^2 = |dd|, and 1/|dd|
    // came with the first square root), arg Q = arg(D conj(d)) (a positive real factor apart)
    const double lq2 = dlog_t(fma(D.re, D.re, D.im * D.im) * (0.25 * rh), sct);   // log |Q|^2
    const double aq = datan2_t(fma(D.im, dre, -(D.re * dim)), fma(D.re, dre, D.im * dim), sct);
    return {F.coef * (bm.re * tau - lq2) + B.re * F.v0,
            F.coef * (bm.im * tau - 2.0 * aq) + B.im * F.v0};
}

// Per-(param set, T) constants of the fast CF.
struct CfConsts {
    FactorC f1, f2;
    double drift;      // (r - q - lambda (e^{mu + sj^2/2} - 1)) tau
    double half_sj2, muj, lt;
};

__device__ __forceinline__ CfConsts cf_consts(const Params& P, double tau) {
#pragma clang fp contract(off)   // the same bits in every prologue form (table, fused)
    CfConsts C;
    C.f1 = factor_consts(P.v01, P.k1, P.t1, P.s1, P.r1);
    C.f2 = factor_consts(P.v02, P.k2, P.t2, P.s2, P.r2);
    const double comp = exp(P.muj + 0.5 * (P.sj * P.sj)) - 1.0;
    C.drift = (P.r - P.q - P.lam * comp) * tau;
    C.half_sj2 = 0.5 * (P.sj * P.sj);
    C.muj = P.muj;
    C.lt = P.lam * tau;
    return C;
}

// jump part J of the exponent: lambda tau (e^{i u mu - sj^2 u^2 / 2} - 1)  (double_heston.py:93)
__device__ __forceinline__ cplx jump_x(const CfConsts& C, double u,
                                       const double2* __restrict__ sct) {
    double js, jc;
    dsincos_t(u * C.muj, sct, &js, &jc);
    const double jm = dexp_t_nonpos(-(C.half_sj2 * (u * u)), sct);
    return {C.lt * (jm * jc - 1.0), C.lt * (jm * js)};
}

// Re(phi(u) e^{-i u a}) = e^{Re E} cos(Im E - u a) from the exponent's parts.
__device__ __forceinline__ double cf_phase_from(const CfConsts& C, double u, double a, cplx X1,
                                                cplx X2, cplx J, const double2* __restrict__ sct) {
    cplx E = {0.0, C.drift * u};
    E = cadd(E, X1);
    E = cadd(E, X2);
    E = cadd(E, J);
    double ps, pc;
    dsincos_t(E.im - u * a, sct, &ps, &pc);
    return dexp_t(E.re, sct) * pc;
}

// Re(phi(u) e^{-i u a}) via the exponent form, one lane per entry; sct = LDS copy of kSinCosPi64
// (load_sincos_table).
__device__ __forceinline__ double cf_phase_re(const CfConsts& C, double u, double tau, double a,
                                              const double2* __restrict__ sct) {
    const cplx X1 = factor_x(C.f1, u, tau, sct);
    const cplx X2 = factor_x(C.f2, u, tau, sct);
    return cf_phase_from(C, u, a, X1, X2, jump_x(C, u, sct), sct);
}

// Copy of the CF's math tables (kMathTab double2: sin/cos, log, atan) into LDS by the block's
// threads from t_first on (the caller synchronises before use).
__device__ __forceinline__ void load_math_tables(double2* sct, int t_first) {
    for (int i = (int)threadIdx.x - t_first; i < kMathTab; i += (int)blockDim.x - t_first) {
        if (i < 0) break;
        const double* src = i < kTabLog ? kSinCosPi64 + 2 * i
                          : (i < kTabAtan ? kLogInvcLogc + 2 * (i - kTabLog)
                          : (i < kTabExp ? kAtanJ64 + 2 * (i - kTabAtan)
                                         : kExp2J64 + 2 * (i - kTabExp)));
        sct[i] = make_double2(src[0], src[1]);
    }
}

__device__ __forceinline__ void load_sincos_table(double2* sct) { load_math_tables(sct, 0); }

// First two cumulants of one factor (double_heston.py:101-118).  Q1: c1 includes r*tau.
__device__ __forceinline__ void factor_cumulants(double tau, double r, double v0, double lm,
                                                 double vb, double vv, double rho, double& c1,
                                                 double& c2) {
#pragma clang fp contract(off)   // the same bits in every prologue form (table, fused)
    const double ek = exp(-lm * tau);
    c1 = r * tau + (1.0 - ek) * (vb - v0) / (2.0 * lm) - vb * tau / 2.0;
    const double lm2 = lm * lm, lm3 = lm2 * lm, vv2 = vv * vv;   // np.power(lm, 3) ~ lm*lm*lm
    c2 = 1.0 / (8.0 * lm3) *
         (vv * tau * lm * ek * (v0 - vb) * (8.0 * lm * rho - 4.0 * vv) +
          lm * rho * vv * (1.0 - ek) * (16.0 * vb - 8.0 * v0) +
          2.0 * vb * lm * tau * (-4.0 * lm * rho * vv + vv2 + 4.0 * lm2) +
          vv2 * ((vb - 2.0 * v0) * exp(-2.0 * lm * tau) + vb * (6.0 * ek - 7.0) + 2.0 * v0) +
          8.0 * lm2 * (v0 - vb) * (1.0 - ek));
}

// Un-clamped truncation range c1 -/+ L sqrt|c2| (double_heston.py:120-132).
__device__ __forceinline__ void trunc_unclamped(const Params& P, double T, double L, double& a,
                                                double& b) {
#pragma clang fp contract(off)
    double c1a, c2a, c1b, c2b;
    factor_cumulants(T, P.r, P.v01, P.k1, P.t1, P.s1, P.r1, c1a, c2a);
    factor_cumulants(T, P.r, P.v02, P.k2, P.t2, P.s2, P.r2, c1b, c2b);
    const double c1 = c1a + c1b + P.lam * T * P.muj;
    const double c2 = c2a + c2b + P.lam * T * (P.sj * P.sj + P.muj * P.muj);
    const double h = L * sqrt(fabs(c2));
    a = c1 - h;
    b = c1 + h;
}

// chi_k / psi_k on [c, d] inside [a, b] (double_heston.py:141-158), generic form.
__device__ __forceinline__ void cos_coeffs(int k, double c, double d, double a, double b,
                                           double& chi, double& psi) {
    if (k == 0) {
        chi = exp(d) - exp(c);
        psi = d - c;
        return;
    }
    const double u = k * kPi / (b - a);
    double sd, cd, sc, cc;
    dsincos(u * (d - a), &sd, &cd);
    dsincos(u * (c - a), &sc, &cc);
    const double ed = exp(d), ec = exp(c);
    chi = (1.0 / (1.0 + u * u)) * (cd * ed - cc * ec + u * sd * ed - u * sc * ec);
    psi = (1.0 / u) * (sd - sc);
}

}  // namespace dh
