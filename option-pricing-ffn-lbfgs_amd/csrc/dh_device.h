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

__device__ __forceinline__ cplx cexp_(cplx z) {
    double s, c;
    sincos(z.im, &s, &c);
    const double e = exp(z.re);
    return {e * c, e * s};
}

// Principal log: arg in (-pi, pi].
__device__ __forceinline__ cplx clog_(cplx z) { return {log(hypot(z.re, z.im)), atan2(z.im, z.re)}; }

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

// First two cumulants of one factor (double_heston.py:101-118).  Q1: c1 includes r*tau.
__device__ __forceinline__ void factor_cumulants(double tau, double r, double v0, double lm,
                                                 double vb, double vv, double rho, double& c1,
                                                 double& c2) {
    const double ek = exp(-lm * tau);
    c1 = r * tau + (1.0 - ek) * (vb - v0) / (2.0 * lm) - vb * tau / 2.0;
    const double lm2 = lm * lm, lm3 = pow(lm, 3.0), vv2 = vv * vv;
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
    sincos(u * (d - a), &sd, &cd);
    sincos(u * (c - a), &sc, &cc);
    const double ed = exp(d), ec = exp(c);
    chi = (1.0 / (1.0 + u * u)) * (cd * ed - cc * ec + u * sd * ed - u * sc * ec);
    psi = (1.0 / u) * (sd - sc);
}

}  // namespace dh
