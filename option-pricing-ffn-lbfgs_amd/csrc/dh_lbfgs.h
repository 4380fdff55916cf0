// dh_lbfgs.h -- L-BFGS-B without bounds as a resumable state machine, for the device-resident
// calibration driver (dh_calibrate_lbfgs).  One calibration start = one LbCore<V>.  The code is
// generic in the vector type V: the step kernel instantiates it with one vector component per
// lane (dh_kernels.hip WaveVec: a 13-vector lives in lanes 0..12 of a wave, dot products are
// xor butterflies over 16 lanes), the CPU check build (tests/native/lb_host.cpp) with a plain
// 16-double array whose dot product sums in the same pairwise order -- so both give the same
// bits.  V provides +, -, * (elementwise), double * V, dot(a, b), amax(a), equal(a, b).  The
// pair memory is a separate type R (LDS-resident on the device) with s(j), y(j), rho(j) (1 / dr),
// a(j) (the two-loop's alpha scratch), put(j, s, y, rho) and shift() (drop the oldest pair).
//
// Attribution: the algorithm restated here is L-BFGS-B 3.0 (Ciyou Zhu, Richard Byrd, Jorge Nocedal,
// Jose Luis Morales; BSD-3-Clause, as distributed with SciPy) and its MINPACK-2 line search
// dcsrch / dcstep (Brett M. Averick, Jorge J. More; MINPACK-2 license, BSD-style), both via SciPy's
// C translation (scipy/optimize/_lbfgsb, BSD-3-Clause).  No source text is copied; the logic is
// restated for a wave-parallel state machine.
//
// What it restates (SciPy 1.15.3, the optimizer the reference calls at lbfgs_calibrator.py:259-269
// as minimize(method='L-BFGS-B', options={maxiter, ftol: 1e-9, gtol: 1e-6}) without bounds):
//   * the driver loop of scipy/optimize/_lbfgsb_py.py:_minimize_lbfgsb (:410-470) with
//     ScalarFunction's evaluation rule (a requested x equal to the last evaluated x is not
//     re-evaluated; nfev counts evaluations, x0 included), the maxiter / maxfun stops on NEW_X and
//     the returned fun = f of the LAST evaluation (which differs from f(x) after an abnormal
//     line search, as the reference's own run shows: SURVEY.md 8(c) test 4.1);
//   * setulb / mainlb of L-BFGS-B 3.0 for nbd = 0 (no bounds): cnstnd = false, so the
//     generalized Cauchy point is computed only while the memory is empty (col = 0; it is then
//     x - g / theta), the subspace step otherwise; projgr = max |g_i|; the termination tests
//     (pgtol, then (fold - f) <= factr * epsmch * max(|fold|, |f|, 1)); the update skip
//     dr <= epsmch * ddum; theta = y'y / dr; restart of the memory when a line search fails
//     with col > 0, ABNORMAL termination when it fails with col = 0;
//   * lnsrlb (first step 1 / ||d|| at iter 0, else 1; stpmax = 1e10; ascent-direction check;
//     maxls trial points; x = z when stp = 1 else x = stp d + t) and MINPACK-2 dcsrch / dcstep
//     with ftol = 1e-3, gtol = 0.9, xtol = 0.1, stpmin = 0 (as in scipy/optimize/_dcsrch.py).
// What differs: the subspace step B^-1 (-g) of the compact representation (formk / subsm with
// every variable free) is formed by the two-loop recursion over the same pairs (s_i, y_i), the
// same theta and rho_i = 1 / dr (dr = L-BFGS-B's s_i'y_i), which is the same matrix (Byrd, Nocedal and Schnabel,
// 1994) rounded differently.  Dot products are pairwise (butterfly) sums of rounded products,
// and nothing is contracted into FMAs, so the host and device builds give the same bits.  The
// pairs are kept oldest-first in slots 0..col-1 (shifted down when the memory is full) instead of
// L-BFGS-B's circular head/itail.
#ifndef DH_LBFGS_H
#define DH_LBFGS_H

#include <math.h>

#ifndef DH_HD
#define DH_HD __host__ __device__
#endif

namespace dhlb {

constexpr int kN = 13;          // parameters (lbfgs_calibrator.py:53-57)
constexpr int kM = 10;          // maxcor (SciPy default, scipy/_lbfgsb_py.py:290)
constexpr int kPts = kN + 1;    // points per function+gradient request: x, x + h_i e_i
constexpr int kLanes = 16;      // vector width (13 components + zero padding)
constexpr double kEpsMch = 2.220446049250313e-16;
constexpr double kBig = 1.0e10;

// SciPy task codes (scipy/optimize/_lbfgsb_py.py:49-80): status * 1000 + message
enum : int {
    kStart = 0, kNewX = 1, kFgSt = 2, kFgLn = 3,        // internal (not terminal)
    kConvPgtol = 4401, kConvFactr = 4402, kStopMaxfun = 5502, kStopMaxiter = 5504,
    kAbnormal = 8000, kErrorLs = 7000
};

struct LbConfig {
    int maxiter;
    int maxfun;                 // compared with nfev (requests) exactly as SciPy: nfev > maxfun
    int maxls;
    int pad;
    double factr_epsmch;        // tol = factr * epsmch with factr = ftol / eps
    double pgtol;
};

// dcsrch work variables (MINPACK-2 isave / dsave)
struct LsState {
    double finit, ginit, gtest, gx, gy, fx, fy, stx, sty, stmin, stmax, width, width1;
    int stage, brackt, task, pad;
};

enum : int { kLsStart = 0, kLsFg = 1, kLsConv = 2, kLsWarn = 3, kLsError = 4 };

// the uniform (scalar) part of a start's state
struct LbScalars {
    double f, theta, fold, gd, gdold, stp, dnorm, sbgnrm;
    double fe;                   // f of the last evaluated point (ScalarFunction)
    double best_loss;            // per-start best valid loss (lbfgs_calibrator.py:171-172)
    LsState ls;
    int col, iupdat, iter, ifun, iback, info, task;
    int nit, nfev, warnflag, done;
    int n_calls;                 // loss evaluations of this start (:120)
};

template <class V, class R>
struct LbCore {
    V x, g, z, d, t, r;          // mainlb vectors
    V xe, ge;                    // ScalarFunction: last evaluated point and gradient
    R pairs;                     // (s_i, y_i, 1 / dr_i with dr = L-BFGS-B's s_i'y_i), oldest first
    LbScalars s;
};

// MINPACK-2 dcstep (scipy/optimize/_dcsrch.py dcstep)
DH_HD inline void dcstep(double& stx, double& fx, double& dx, double& sty, double& fy, double& dy,
                         double& stp, double fp, double dp, int& brackt, double stpmin,
                         double stpmax) {
#pragma clang fp contract(off)
    const double sgn_dp = dp > 0 ? 1.0 : (dp < 0 ? -1.0 : 0.0);
    const double sgn_dx = dx > 0 ? 1.0 : (dx < 0 ? -1.0 : 0.0);
    const double sgnd = sgn_dp * sgn_dx;
    double stpf;
    if (fp > fx) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
        double gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
        if (stp < stx) gamma = -gamma;
        const double p = (gamma - dx) + theta;
        const double q = ((gamma - dx) + gamma) + dp;
        const double r = p / q;
        const double stpc = stx + r * (stp - stx);
        const double stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
        if (fabs(stpc - stx) <= fabs(stpq - stx)) stpf = stpc;
        else stpf = stpc + (stpq - stpc) / 2.0;
        brackt = 1;
    } else if (sgnd < 0.0) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
        double gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
        if (stp > stx) gamma = -gamma;
        const double p = (gamma - dp) + theta;
        const double q = ((gamma - dp) + gamma) + dx;
        const double r = p / q;
        const double stpc = stp + r * (stx - stp);
        const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
        stpf = (fabs(stpc - stp) > fabs(stpq - stp)) ? stpc : stpq;
        brackt = 1;
    } else if (fabs(dp) < fabs(dx)) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
        const double disc = (theta / s) * (theta / s) - (dx / s) * (dp / s);
        double gamma = s * sqrt(disc > 0.0 ? disc : 0.0);
        if (stp > stx) gamma = -gamma;
        const double p = (gamma - dp) + theta;
        const double q = (gamma + (dx - dp)) + gamma;
        const double r = p / q;
        double stpc;
        if (r < 0.0 && gamma != 0.0) stpc = stp + r * (stx - stp);
        else if (stp > stx) stpc = stpmax;
        else stpc = stpmin;
        const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
        if (brackt) {
            stpf = (fabs(stpc - stp) < fabs(stpq - stp)) ? stpc : stpq;
            if (stp > stx) stpf = fmin(stp + 0.66 * (sty - stp), stpf);
            else stpf = fmax(stp + 0.66 * (sty - stp), stpf);
        } else {
            stpf = (fabs(stpc - stp) > fabs(stpq - stp)) ? stpc : stpq;
            stpf = fmin(fmax(stpf, stpmin), stpmax);
        }
    } else {
        if (brackt) {
            const double theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
            const double s = fmax(fmax(fabs(theta), fabs(dy)), fabs(dp));
            double gamma = s * sqrt((theta / s) * (theta / s) - (dy / s) * (dp / s));
            if (stp > sty) gamma = -gamma;
            const double p = (gamma - dp) + theta;
            const double q = ((gamma - dp) + gamma) + dy;
            const double r = p / q;
            stpf = stp + r * (sty - stp);
        } else if (stp > stx) {
            stpf = stpmax;
        } else {
            stpf = stpmin;
        }
    }
    // the interval update as selects with every output written once (conditional stores to
    // different references are sunk by the compiler into a store through a selected pointer,
    // which keeps the line-search state in scratch memory on the device)
    const bool hi = fp > fx;
    const bool swap = !hi && sgnd < 0.0;
    const double nsty = hi ? stp : (swap ? stx : sty);
    const double nfy = hi ? fp : (swap ? fx : fy);
    const double ndy = hi ? dp : (swap ? dx : dy);
    const double nstx = hi ? stx : stp;
    const double nfx = hi ? fx : fp;
    const double ndx = hi ? dx : dp;
    sty = nsty;
    fy = nfy;
    dy = ndy;
    stx = nstx;
    fx = nfx;
    dx = ndx;
    stp = stpf;
}

// MINPACK-2 dcsrch (scipy/optimize/_dcsrch.py DCSRCH._iterate) with L-BFGS-B's constants.
// ls.task on entry: kLsStart or kLsFg; on exit kLsFg (evaluate at stp), kLsConv, kLsWarn or
// kLsError.
DH_HD inline void dcsrch(LsState& ls, double f, double g, double& stp, double stpmax) {
#pragma clang fp contract(off)
    constexpr double ftol = 1.0e-3, gtol = 0.9, xtol = 0.1, stpmin = 0.0;
    constexpr double p5 = 0.5, p66 = 0.66, xtrapl = 1.1, xtrapu = 4.0;
    if (ls.task == kLsStart) {
        if (stp < stpmin || stp > stpmax || g >= 0.0) {
            ls.task = kLsError;
            return;
        }
        ls.brackt = 0;
        ls.stage = 1;
        ls.finit = f;
        ls.ginit = g;
        ls.gtest = ftol * ls.ginit;
        ls.width = stpmax - stpmin;
        ls.width1 = ls.width / p5;
        ls.stx = 0.0;
        ls.fx = ls.finit;
        ls.gx = ls.ginit;
        ls.sty = 0.0;
        ls.fy = ls.finit;
        ls.gy = ls.ginit;
        ls.stmin = 0.0;
        ls.stmax = stp + xtrapu * stp;
        ls.task = kLsFg;
        return;
    }
    const double ftest = ls.finit + stp * ls.gtest;
    if (ls.stage == 1 && f <= ftest && g >= 0.0) ls.stage = 2;
    int task = kLsFg;
    if (ls.brackt && (stp <= ls.stmin || stp >= ls.stmax)) task = kLsWarn;
    if (ls.brackt && ls.stmax - ls.stmin <= xtol * ls.stmax) task = kLsWarn;
    if (stp == stpmax && f <= ftest && g <= ls.gtest) task = kLsWarn;
    if (stp == stpmin && (f > ftest || g >= ls.gtest)) task = kLsWarn;
    if (f <= ftest && fabs(g) <= gtol * (-ls.ginit)) task = kLsConv;
    if (task != kLsFg) {
        ls.task = task;
        return;
    }
    // one dcstep call site on locals (two call sites binding different references were merged
    // by the compiler into one through pointer selects, which kept the line-search state in
    // scratch memory on the device)
    const bool modified = ls.stage == 1 && f <= ls.fx && f > ftest;
    double fm, gm, fxm, gxm, fym, gym;
    if (modified) {                      // the modified function psi = f - stp gtest
        fm = f - stp * ls.gtest;
        fxm = ls.fx - ls.stx * ls.gtest;
        fym = ls.fy - ls.sty * ls.gtest;
        gm = g - ls.gtest;
        gxm = ls.gx - ls.gtest;
        gym = ls.gy - ls.gtest;
    } else {
        fm = f;
        fxm = ls.fx;
        fym = ls.fy;
        gm = g;
        gxm = ls.gx;
        gym = ls.gy;
    }
    dcstep(ls.stx, fxm, gxm, ls.sty, fym, gym, stp, fm, gm, ls.brackt, ls.stmin, ls.stmax);
    if (modified) {
        ls.fx = fxm + ls.stx * ls.gtest;
        ls.fy = fym + ls.sty * ls.gtest;
        ls.gx = gxm + ls.gtest;
        ls.gy = gym + ls.gtest;
    } else {
        ls.fx = fxm;
        ls.fy = fym;
        ls.gx = gxm;
        ls.gy = gym;
    }
    if (ls.brackt) {
        if (fabs(ls.sty - ls.stx) >= p66 * ls.width1) stp = ls.stx + p5 * (ls.sty - ls.stx);
        ls.width1 = ls.width;
        ls.width = fabs(ls.sty - ls.stx);
    }
    if (ls.brackt) {
        ls.stmin = fmin(ls.stx, ls.sty);
        ls.stmax = fmax(ls.stx, ls.sty);
    } else {
        ls.stmin = stp + xtrapl * (stp - ls.stx);
        ls.stmax = stp + xtrapu * (stp - ls.stx);
    }
    stp = fmin(fmax(stp, stpmin), stpmax);
    if ((ls.brackt && (stp <= ls.stmin || stp >= ls.stmax)) ||
        (ls.brackt && ls.stmax - ls.stmin <= xtol * ls.stmax))
        stp = ls.stx;
    ls.task = kLsFg;
}

// z = x + H (-g): the two-loop recursion over the stored pairs, H0 = I / theta
template <class V, class R>
DH_HD inline void subspace_step(LbCore<V, R>& c) {
#pragma clang fp contract(off)
    R& m = c.pairs;
    V q = -c.g;
    for (int j = c.s.col - 1; j >= 0; --j) {           // newest -> oldest
        const double a = m.rho(j) * dot(m.s(j), q);
        m.a(j) = a;
        q = q - a * m.y(j);
    }
    q = (1.0 / c.s.theta) * q;
    for (int j = 0; j < c.s.col; ++j) {                // oldest -> newest
        const double b = m.rho(j) * dot(m.y(j), q);
        q = q + (m.a(j) - b) * m.s(j);
    }
    c.z = c.x + q;
}

// Generalized Cauchy point with an empty memory and no bounds (cauchy with nbreak = 0):
// d = -g, f1 = -|g|^2, f2 = -theta f1, z = x + (-f1 / f2) d.
template <class V, class R>
DH_HD inline void cauchy_point(LbCore<V, R>& c) {
#pragma clang fp contract(off)
    c.z = c.x;
    if (c.s.sbgnrm <= 0.0) return;
    c.d = -c.g;
    const double f1 = -dot(c.g, c.g);
    const double f2 = -c.s.theta * f1;
    double dtm = -f1 / f2;
    if (dtm <= 0.0) dtm = 0.0;
    const double tsum = 0.0 + dtm;
    c.z = c.z + tsum * c.d;
}

// setulb for nbd = 0: advances task from START / FG_ST / FG_LN / NEW_X using (f, g) at x
template <class V, class R>
DH_HD inline void setulb(LbCore<V, R>& c, const LbConfig& cf) {
#pragma clang fp contract(off)
    LbScalars& s = c.s;
    double ddum, rr, dr, gd;
    switch (s.task) {
        case kStart:
            s.col = 0;
            s.theta = 1.0;
            s.iupdat = 0;
            s.iback = 0;
            s.fold = 0.0;
            s.dnorm = 0.0;
            s.gd = 0.0;
            s.stp = 0.0;
            s.gdold = 0.0;
            s.sbgnrm = 0.0;
            s.iter = 0;
            s.ifun = 0;
            s.info = 0;
            s.task = kFgSt;
            return;
        case kFgSt: goto L111;
        case kFgLn: goto L556;
        case kNewX: goto L777;
        default: return;
    }
L111:
    s.sbgnrm = amax(c.g);
    if (s.sbgnrm <= cf.pgtol) {
        s.task = kConvPgtol;
        return;
    }
L222:
    if (s.col > 0) {
        subspace_step(c);
    } else {
        cauchy_point(c);
    }
    c.d = c.z - c.x;
    // lnsrlb, first entry
    s.dnorm = sqrt(dot(c.d, c.d));
    s.stp = (s.iter == 0) ? fmin(1.0 / s.dnorm, kBig) : 1.0;
    c.t = c.x;
    c.r = c.g;
    s.fold = s.f;
    s.ifun = 0;
    s.iback = 0;
    s.ls.task = kLsStart;
L556:
    gd = dot(c.g, c.d);
    s.gd = gd;
    if (s.ifun == 0) {
        s.gdold = gd;
        if (gd >= 0.0) s.info = -4;        // ascent direction: line search impossible
    }
    if (s.info == 0) {
        dcsrch(s.ls, s.f, gd, s.stp, kBig);
        if (s.ls.task == kLsError) {
            s.task = kErrorLs;
            return;
        }
        if (s.ls.task == kLsFg) {
            s.ifun += 1;
            s.iback = s.ifun - 1;
            if (s.iback < cf.maxls) {
                if (s.stp == 1.0) c.x = c.z;
                else c.x = s.stp * c.d + c.t;
                s.task = kFgLn;
                return;                            // evaluate f, g at x
            }
        } else {
            s.task = kNewX;
        }
    }
    if (s.info != 0 || s.iback >= cf.maxls) {
        c.x = c.t;
        c.g = c.r;
        s.f = s.fold;
        if (s.col == 0) {
            if (s.info == 0) {
                s.info = -9;
                s.ifun -= 1;
                s.iback -= 1;
            }
            s.task = kAbnormal;
            s.iter += 1;
            return;
        }
        s.info = 0;                                // refresh the memory and restart
        s.col = 0;
        s.theta = 1.0;
        s.iupdat = 0;
        goto L222;
    }
    s.iter += 1;
    s.sbgnrm = amax(c.g);
    return;                                        // task NEW_X
L777:
    if (s.sbgnrm <= cf.pgtol) {
        s.task = kConvPgtol;
        return;
    }
    ddum = fmax(fmax(fabs(s.fold), fabs(s.f)), 1.0);
    if ((s.fold - s.f) <= cf.factr_epsmch * ddum) {
        s.task = kConvFactr;
        return;
    }
    c.r = c.g - c.r;
    rr = dot(c.r, c.r);
    if (s.stp == 1.0) {
        dr = s.gd - s.gdold;
        ddum = -s.gdold;
    } else {
        dr = (s.gd - s.gdold) * s.stp;
        c.d = s.stp * c.d;
        ddum = -s.gdold * s.stp;
    }
    if (dr <= kEpsMch * ddum) goto L222;           // skip the update
    s.iupdat += 1;                                 // matupd
    if (s.col == kM) c.pairs.shift();              // drop the oldest pair
    else s.col += 1;
    c.pairs.put(s.col - 1, c.d, c.r, 1.0 / dr);
    s.theta = rr / dr;
    goto L222;
}

DH_HD inline int lb_finish(LbScalars& s) {
    if (s.task / 1000 == 4) s.warnflag = 0;
    else if (s.task == kStopMaxfun || s.task == kStopMaxiter) s.warnflag = 1;
    else s.warnflag = 2;
    s.done = 1;
    return 0;
}

// _minimize_lbfgsb's loop around setulb.  lb_begin starts a run at x0; whenever it or lb_resume
// returns 1, evaluate f and g at xe, store them in s.fe / ge and call lb_resume.  A return of 0
// means the start is finished (s.task, s.warnflag, s.nit, s.nfev, x and s.fe are final).
template <class V, class R>
DH_HD inline int lb_begin(LbCore<V, R>& c, const V& x0) {
    c.x = x0;
    c.xe = x0;
    c.s.task = kStart;
    c.s.nit = 0;
    c.s.nfev = 1;                                  // ScalarFunction evaluates x0 on creation
    c.s.warnflag = 0;
    c.s.done = 0;
    c.s.f = 0.0;
    return 1;
}

template <class V, class R>
DH_HD inline int lb_resume(LbCore<V, R>& c, const LbConfig& cf) {
    LbScalars& s = c.s;
    if (s.done) return 0;
    bool assign = s.task != kStart;                // START ignores f and g
    // Every pass either asks for a new point, records a NEW_X (bounded by maxiter) or finishes;
    // passes that re-request the last evaluated point advance dcsrch, whose interval shrinks.
    // The cap only guarantees the device loop ends whatever the inputs (NaN, say).
    for (int guard = 0;; ++guard) {
        if (guard > 4 * (cf.maxiter + cf.maxls) + 64) {
            s.task = kErrorLs;
            return lb_finish(s);
        }
        if (assign) {
            s.f = s.fe;
            c.g = c.ge;
        }
        setulb(c, cf);
        if (s.task == kFgSt || s.task == kFgLn) {
            assign = true;
            if (!equal(c.x, c.xe)) {
                c.xe = c.x;
                s.nfev += 1;
                return 1;
            }
        } else if (s.task == kNewX) {
            assign = false;
            s.nit += 1;
            if (s.nit >= cf.maxiter) {
                s.task = kStopMaxiter;
                return lb_finish(s);
            }
            if (s.nfev > cf.maxfun) {
                s.task = kStopMaxfun;
                return lb_finish(s);
            }
        } else {
            return lb_finish(s);
        }
    }
}

}  // namespace dhlb

#endif  // DH_LBFGS_H
