/*
 * dhcos.h -- C-ABI of the MI355X-native Double-Heston + Merton-jump COS pricer and calibration
 * objective (libdhcos.so, gfx950).
 *
 * The reference (zenthepen/Option-Pricing-FFN-LBFGS) is pure Python; it has no FFI of its own.
 * Each entry point below replaces one reference call site on the hot path, named per function
 * (file:line in the reference).  The Python host layer (option-pricing-ffn-lbfgs_amd/dhcos) binds
 * these through ctypes; INTEGRATION.md shows the binding a maintainer adds on the reference side.
 *
 * Conventions
 *   - Every function returns 0 on success and a negative DH_E* code on failure; the message of
 *     the last failure on the calling thread is returned by dh_last_error().
 *   - Numeric failures (NaN / inf / non-positive prices) are NOT errors: they are reported in the
 *     outputs exactly as the reference produces them (see dh_surface_loss).
 *   - "host" entry points take host pointers, copy synchronously and return when results are on
 *     the host (the caller may free its buffers on return).  "_dev" entry points take device
 *     pointers and enqueue on the given HIP stream (NULL = the context's own stream) without
 *     synchronising.
 *   - Param-set record: DH_PARAM_STRIDE (16) doubles per set:
 *       [0..12] v01 kappa1 theta1 sigma1 rho1 v02 kappa2 theta2 sigma2 rho2 lambda_j mu_j sigma_j
 *       [13] S0   [14] r   [15] q
 *     (double_heston.py:26-46 constructor arguments, same meaning).
 *   - All arithmetic is IEEE fp64.
 */
#ifndef DHCOS_H
#define DHCOS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DH_PARAM_STRIDE 16
#define DH_MAX_N 2048            /* longest COS series of the table (fast) path: LDS-resident */
#define DH_MAX_N_PER_TERM 65536  /* longest accepted: N > DH_MAX_N runs the per-term path (the
                                    reference's operation order, one wave per option), slower
                                    but any length the reference's pricing(N) takes up to here  */

enum {
    DH_OK = 0,
    DH_E_ARG = -1,               /* invalid argument (null pointer, bad size, N out of range) */
    DH_E_HIP = -2,               /* HIP runtime error (message has the HIP error string) */
    DH_E_NODEV = -3,             /* no usable gfx950 device */
    DH_E_ALLOC = -4,             /* host/device allocation failure */
    DH_E_COMM = -5               /* RCCL failure or librccl not loadable (message has the detail) */
};

/* strike_mode for surfaces */
enum {
    DH_STRIKE_ABSOLUTE = 0,      /* K[m] is the strike */
    DH_STRIKE_PCT_SPOT = 1       /* K[m] is K_relative; strike = K_relative * S0 / 100.0 per param
                                    set (synthetic_generator.py:125) */
};

typedef struct dh_ctx dh_ctx;
typedef struct dh_surface dh_surface;

/* ---- context ------------------------------------------------------------------------------ */
int dh_version(void);
const char* dh_last_error(void);
int dh_device_count(int* count);
/* One context per (device, host thread).  Owns a HIP stream and grow-only device scratch. */
int dh_ctx_create(int device, dh_ctx** out);
int dh_ctx_destroy(dh_ctx* ctx);
int dh_ctx_synchronize(dh_ctx* ctx);
/* The HIP stream the context launches on (hipStream_t as void*). */
void* dh_ctx_stream(dh_ctx* ctx);
/* Validation mode: when on, every option is priced by the per-term path in the reference's
 * operation order (own CF and sincos per COS term) instead of the shared-table fast path.   */
int dh_ctx_set_exact(dh_ctx* ctx, int on);
/* Adaptive tail of the fast path's angle sums (on by default): a table's COS terms past the last
 * one with |T2_k| > 2^-72 S0 / ((b - a)(1 + (b - a)/pi) N) are not summed, which moves no price by
 * more than 2^-64 of its k = 0 term.  Off: every term k < N is summed (A/B, tests). */
int dh_ctx_set_tail_cut(dh_ctx* ctx, int on);
/* Request kernels of the fast path.  AUTO (default): one fused launch per request when every
 * maturity group fits one tile (<= 256 options), except small tiles in large calls (generator
 * grids: a COS-table launch then the lane-per-option-group kernel); otherwise the table launch
 * then an option launch.  FUSED / SPLIT force one of the two where it applies.  Both produce
 * the same bits; the choice only changes speed.                                              */
enum { DH_PATH_AUTO = 0, DH_PATH_SPLIT = 1, DH_PATH_FUSED = 2, DH_PATH_GEN = 3 };
int dh_ctx_set_path(dh_ctx* ctx, int path);
/* DH_PATH_FUSED, DH_PATH_SPLIT or DH_PATH_GEN (AUTO only: generator grids -- every maturity group
 * one tile of <= 16 options in a call of >= 65,536 tasks -- priced by one fused small-tile
 * launch, agreeing with the other paths to ~1e-15): the kernels the last fast-path request ran
 * (0 before any).                                                                              */
int dh_ctx_last_path(dh_ctx* ctx);
/* Diagnostics (only in the DH_STAMPS build, `make stamps`; the production library returns
 * DH_E_ARG): record per-block s_memtime phase stamps of the COS kernels, read the last request's. */
int dh_ctx_debug_stamps(dh_ctx* ctx, int on);
int dh_ctx_read_stamps(dh_ctx* ctx, unsigned long long* out, int64_t cap, int64_t* n);

/* ---- option surfaces ---------------------------------------------------------------------- */
/* Upload an option set once.  Options are grouped by exact maturity on the host; groups are cut
 * into tiles of at most 256 options; every tile shares one COS/CF table per param set.
 *   K, T, is_call: [M]   (is_call resolved by the caller as option_type.upper()[0]=='C',
 *                         double_heston.py:172)
 *   mkt:           [M] market prices, may be NULL (needed only by dh_surface_loss*)
 * Replaces the per-option DoubleHeston construction in lbfgs_calibrator.py:128-150 and
 * synthetic_generator.py:123-138.                                                           */
int dh_surface_create(dh_ctx* ctx, const double* K, const double* T, const int8_t* is_call,
                      const double* mkt, int M, int strike_mode, dh_surface** out);
int dh_surface_destroy(dh_surface* s);
int dh_surface_size(const dh_surface* s, int* M, int* n_tiles);

/* Price every option of the surface under every param set: out[p*M + m], m in the caller's
 * original option order.  Replaces DoubleHeston.pricing(N) (double_heston.py:160-192) called
 * P*M times.  L is the truncation width (truncationRange(L=10), double_heston.py:100).        */
int dh_surface_price(dh_ctx* ctx, const dh_surface* s, const double* params, int64_t P, int N,
                     double L, double* out);

/* The generator's pricing from its sampler's columns (synthetic_generator.py:123-138): params
 * [P][13] model params, spots [P] (each record's S0), one rate r and q = 0 -- the records of
 * dh_surface_price, formed on the device (no host packing pass), then priced into out[P][M].
 * Host buffers; registered ones (dh_host_register) move by DMA without staging copies.         */
int dh_surface_price_cols(dh_ctx* ctx, const dh_surface* s, const double* params,
                          const double* spots, double r, int64_t P, int N, double L, double* out);
/* Page-lock a host range for the copies of the calls above (hipHostRegister) and release it.
 * A range must be unregistered before its memory is freed.                                     */
int dh_host_register(void* ptr, size_t bytes);
int dh_host_unregister(void* ptr);

/* Calibration objective over the surface for S param sets (one FD request = 14 sets):
 *   sse[s]   = sum_m ((price_sm - mkt_m) / mkt_m)^2      (lbfgs_calibrator.py:163, un-normalised)
 *   n_bad[s] = #{m : price_sm is NaN, +-inf or <= 0}      (lbfgs_calibrator.py:152)
 *   prices   = optional [S][M] output (NULL to skip)
 * The host forms loss = n_bad ? 1e10 : sse / M + feller (lbfgs_calibrator.py:118-177).
 * A fused request sums each set's tile partials in its own tail; a sum whose
 * hand-off never completed (bounded wait, never observed) leaves n_bad[s] = -1 and the call
 * returns DH_E_HIP.                                                                            */
int dh_surface_loss(dh_ctx* ctx, const dh_surface* s, const double* params, int S, int N,
                    double L, double* sse, int32_t* n_bad, double* prices);

/* Device-pointer variants: params/out/sse/n_bad are device pointers; enqueue on `stream`
 * (hipStream_t; NULL = context stream).  No synchronisation, no allocation after warm-up.
 * A request is one fused launch or two launches (COS table, then options), dh_ctx_set_path;
 * in loss mode each param set's sum is finalised in a fixed order (n_bad[s] = -1: a hand-off
 * timeout, see dh_surface_loss).
 * Launches through one context share its scratch: issue them on one stream at a time.       */
int dh_surface_price_dev(dh_ctx* ctx, const dh_surface* s, const double* d_params, int64_t P,
                         int N, double L, double* d_out, void* stream);
int dh_surface_loss_dev(dh_ctx* ctx, const dh_surface* s, const double* d_params, int S, int N,
                        double L, double* d_sse, int32_t* d_n_bad, double* d_prices,
                        void* stream);

/* One function+gradient request per start for a host-driven optimizer (the SciPy driver):
 * x0[S][13] unconstrained -> f[S] = compute_loss(x0) (lbfgs_calibrator.py:118-177), g[S][13] =
 * SciPy's 2-point forward difference (loss(x0 + h_i e_i) - f) / ((x0_i + h_i) - x0_i) with
 * h = 1e-8 (scipy/optimize/_numdiff.py:498-511,592-596), low[S] = the smallest valid loss of the
 * 14 points (best_loss, :171-172).  The 14 x S records are formed on the host and priced in one
 * request (dh_surface_loss).
 * model: [2][S][13] model params (transform_params, lbfgs_calibrator.py:62-87) of x0 (block 0)
 * and of x0 + h (block 1, h as above), formed by the caller with the same exp / tanh the
 * reference's NumPy uses, so f equals compute_loss(x0) bit for bit; NULL = libm exp / tanh here. */
int dh_surface_fg(dh_ctx* ctx, const dh_surface* s, const double* x0, const double* model, int S,
                  double S0, double r, int N, double L, double* f, double* g, double* low);
/* The same request in two halves, so a host driver can run one group of starts' optimizer steps
 * while other groups' requests are on the device: begin forms the records into slot (0 ..
 * DH_FG_SLOTS - 1; each slot owns its pinned buffers) and enqueues the request on the context's
 * stream, then returns;
 * end waits for that slot's request and writes f, g, low as dh_surface_fg would (the same bits:
 * a start's values depend only on its own x0).  A slot holds one request at a time; requests
 * run in enqueue order; 14 S <= 1024 (larger: dh_surface_fg).                                   */
#define DH_FG_SLOTS 4
int dh_surface_fg_begin(dh_ctx* ctx, const dh_surface* s, const double* x0, const double* model,
                        int S, double S0, double r, int N, double L, int slot);
/* end: S must be the start count the slot's request was enqueued with, and s its surface
 * (DH_E_ARG otherwise, the request stays in flight): f[S], g[S][13], low[S] are written.
 * cancel: wait for the slot's request (if any) and discard it, so the slot is free again (a
 * driver unwinding from an error); no-op on an idle slot.                                      */
int dh_surface_fg_end(dh_ctx* ctx, const dh_surface* s, int slot, int S, double* f, double* g,
                      double* low);
int dh_surface_fg_cancel(dh_ctx* ctx, int slot);

/* ---- device-resident multi-start L-BFGS-B ------------------------------------------------- */
/* Runs S independent L-BFGS-B starts (no bounds) on the surface's calibration loss without a
 * host round trip per iteration.  Replaces the per-start
 *   minimize(compute_loss, x0, method='L-BFGS-B', options={maxiter, ftol, gtol})
 * of DoubleHestonJumpCalibrator.calibrate (lbfgs_calibrator.py:259-269, SciPy's 2-point
 * forward-difference gradient at h = 1e-8, scipy/optimize/_numdiff.py:498-511,592-596).
 * Each iteration is one loss launch over the 14 x (live starts) points of every live start's
 * pending function+gradient request, then one step launch (one wave per start) that forms
 * loss = n_bad ? 1e10 : sse / M + Feller penalty and the FD gradient, advances the start's
 * L-BFGS-B state (csrc/dh_lbfgs.h) to its next request and writes that request's 14 param
 * records.  The host only checks for finished starts every `chunk` iterations.
 * x0: [S][13] unconstrained start points (lbfgs_calibrator.py:62-87 transform), S0 / r the
 * spot and rate of every record.  Results per start in out[S].                                */
typedef struct {
    int32_t maxiter;             /* NEW_X iterations (minimize's maxiter) */
    int32_t maxfun;              /* stop when requests (x0 included) > maxfun at a NEW_X */
    int32_t maxls;               /* line-search trial points (SciPy default 20) */
    int32_t chunk;               /* iterations enqueued between host checks (<= 0: 8) */
    double ftol;                 /* relative-reduction test: factr = ftol / eps */
    double gtol;                 /* projected-gradient test */
} dh_lb_options;

typedef struct {
    double x[13];                /* final x (restored start of the last line search if ABNORMAL) */
    double fun;                  /* f of the LAST evaluated point, as SciPy's OptimizeResult.fun */
    double best_loss;            /* smallest valid loss this start evaluated (:171-172) */
    double t_done;               /* seconds from the call until the host saw the start finish */
    int32_t nit;                 /* NEW_X iterations */
    int32_t nfev;                /* function+gradient requests, x0 included */
    int32_t task;                /* SciPy status*1000 + message: 4401/4402 CONVERGENCE,
                                    5502/5504 STOP, 8000 ABNORMAL, 7000 ERROR (line search) */
    int32_t warnflag;            /* 0 converged, 1 maxfun/maxiter, 2 other */
    int32_t n_calls;             /* loss evaluations (14 per request) */
    int32_t pad;
} dh_lb_result;

int dh_calibrate_lbfgs(dh_ctx* ctx, const dh_surface* s, const double* x0, int S, double S0,
                       double r, int N, double L, const dh_lb_options* opt, dh_lb_result* out,
                       int32_t* n_launches);
/* Diagnostics (tests): with cap > 0, dh_calibrate_lbfgs records every consumed request as 40
 * doubles [start, request number, f, x[13], g[13], 0 0 0, 6 phase stamps of the step kernel
 * (DH_STAMPS build only, else 0) 0 0] (order across starts arbitrary); dh_ctx_read_lb_trace
 * copies up to cap records of the last call and sets *n to the count.                         */
int dh_ctx_set_lb_trace(dh_ctx* ctx, int64_t cap);
int dh_ctx_read_lb_trace(dh_ctx* ctx, double* out, int64_t cap, int64_t* n);

/* ---- one-shot forms (SURVEY.md 8(b)'s proposed exports; a surface is built per call) ------- */
/* out[p*M + m] = price of option m (K, T, is_call) under params[p] (13 model params, S0, r, q):
 * dh_surface_create + dh_surface_price + dh_surface_destroy.  Replaces P x M calls of
 * DoubleHeston(...).pricing(N) (double_heston.py:160-192).                                      */
int dh_price_batch(dh_ctx* ctx, const double* params, int64_t P, const double* K, const double* T,
                   const int8_t* is_call, int M, int N, double L, double* out);
/* compute_loss (lbfgs_calibrator.py:118-177) of S unconstrained points x[S][13], all on the
 * device: transform (exp / tanh / identity, :62-87), Feller penalty (:113-116), the surface's
 * loss terms, then loss[s] = n_invalid[s] ? 1e10 : sse / M + penalty (:152-166).  M == 0 gives
 * NaN (np.mean([]), :163); a zero market price gives inf.  One FD request = the 14 points
 * x, x + h_i e_i.                                                                               */
int dh_loss_batch(dh_ctx* ctx, const double* x, int S, const double* K, const double* T,
                  const int8_t* is_call, const double* mkt, int M, double S0, double r, int N,
                  double L, double* loss, int32_t* n_invalid);

/* ---- generator batch path: host RNG ------------------------------------------------------ */
/* Draws n_samples samples of generate_synthetic_calibrations (synthetic_generator.py:98-141)
 * from NumPy's legacy RandomState stream, bit for bit, on the host (no device work): per sample
 * 13 uniform(lo[j], hi[j]) (:100-102), the AR(1) blend alpha * prev + (1 - alpha) * draw for
 * i > 0 (:105-109), spot *= 1 + normal(ret_mu, ret_sigma) for i > 0 (:112-116, spot0 at i = 0),
 * then n_opt normal(0, noise_sigma) (:141).  The state is NumPy's get_state() tuple: mt_key[624],
 * mt_pos, has_gauss, cached_gauss -- read and advanced in place (set it back with set_state).
 * Outputs: params [n][13], spots [n], noise [n][n_opt].  The draws replace the reference's
 * per-sample Python loop; pricing then runs on the GPU (dh_surface_price, STRIKE_PCT_SPOT).      */
int dh_gen_draw(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss, double* cached_gauss,
                int64_t n_samples, const double* lo, const double* hi, int n_opt, double alpha,
                double spot0, double ret_mu, double ret_sigma, double noise_sigma, double* params,
                double* spots, double* noise);
/* dh_gen_draw that also publishes its progress: *done (required) is stored, with release order,
 * as the count of leading samples whose params, spot and noise rows are complete (after every
 * chunk of 65,536 samples, and n_samples at the end), so a caller thread can price finished rows
 * while the draw runs.  Same draws, same bits, same final RNG state as dh_gen_draw.           */
int dh_gen_draw_progress(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss,
                         double* cached_gauss, int64_t n_samples, const double* lo,
                         const double* hi, int n_opt, double alpha, double spot0, double ret_mu,
                         double ret_sigma, double noise_sigma, double* params, double* spots,
                         double* noise, int64_t* done);
/* ---- sharded draw (generate_sharded): one rank locates, every rank draws its own samples -- */
/* The serial part of the draw only (the MT19937 twister, the polar method's acceptance bitmaps
 * and the walk over them; no sample is drawn): for each of n_starts sample indices starts[]
 * (non-decreasing, <= n_samples) the generator's state at that sample's first draw, as
 * DH_GEN_LOC_WORDS doubles at loc[j * DH_GEN_LOC_WORDS]: key[624], pos, has_gauss, cached gauss
 * (np.random.get_state()'s fields).  The state arguments are advanced in place to where
 * dh_gen_draw of n_samples would leave them.  Replaces the stream positions the reference's
 * per-sample loop reaches (synthetic_generator.py:98-141).                                      */
#define DH_GEN_LOC_WORDS 627
int dh_gen_locate(uint32_t* mt_key, int32_t* mt_pos, int32_t* has_gauss, double* cached_gauss,
                  int64_t n_samples, int n_opt, const int64_t* starts, int64_t n_starts,
                  double* loc);
/* Draw samples [starts[0], i_end) from located states: chunk j = [starts[j], starts[j + 1]) (the
 * last ends at i_end) from loc[j], chunks in parallel on the host's threads.  Rows relative to
 * starts[0]: params [n][13] the raw uniforms (:100-102, before the AR(1) blend), rets [n] the spot
 * return's normal(0.0003, 0.01) draw (:112-116; sample 0 has none), noise [n][n_opt] (:141).   */
int dh_gen_draw_located(const double* loc, const int64_t* starts, int64_t n_starts,
                        int64_t i_end, const double* lo, const double* hi, int n_opt,
                        double ret_mu, double ret_sigma, double noise_sigma, double* params,
                        double* rets, double* noise);
/* The values that carry across samples, over rows [0, n) = samples [i0, i0 + n): the AR(1) blend
 * params[i] = alpha params[i - 1] + (1 - alpha) raw[i] (:105-109) and the spot walk spot[i] =
 * spot[i - 1] (1 + ret[i]) (:112-116), in place (spots: rets in, spots out).  carry [14] holds
 * the previous sample's blended params and spot (ignored when i0 = 0: spot0 starts the walk)
 * and receives this block's last row: the 14 doubles one rank passes to the next.            */
int dh_gen_sweep(double* params, double* spots, int64_t i0, int64_t n, double alpha, double spot0,
                 double* carry);
/* Samples drawn by this process's draw calls so far (instrumentation of the sharded draw).    */
int dh_gen_drawn_samples(int64_t* count);
/* The generator's trading dates (synthetic_generator.py:59-67: weekdays from a Monday, here
 * 2022-01-03 = day 18995 since 1970-01-01, as 'YYYY-MM-DD'): sample i's date as 10 UCS-4 code
 * points at out[10 i] (a NumPy '<U10' array's buffer).  DH_E_ARG past year 9999.             */
int dh_gen_dates(int64_t first_day, int64_t n, uint32_t* out);

/* The generator's host arithmetic after pricing (synthetic_generator.py:141-157), per sample i
 * and option j of [n_samples][n_opt] row-major arrays: market = model + noise * model, loss[i] =
 * mean_j ((model - market) / market)^2 formed as np.mean forms it (bit for bit), strikes =
 * (k_rel[j] * spots[i]) / 100.  Host code (threads), no device work.                      */
int dh_gen_assemble(const double* model, const double* noise, const double* spots,
                    const double* k_rel, int64_t n_samples, int n_opt, double* market,
                    double* loss, double* strikes);

/* The generator's whole batch path on the device (replaces synthetic_generator.py:98-157's
 * per-sample loop).  The host keeps only the serial part of NumPy's legacy stream
 * -- the MT19937 twister and the walk over the polar acceptances, which give each sample its
 * first double -- on a team of threads; per 65,536-sample chunk the device re-creates the
 * stream's words, draws each sample's uniforms and normals (glibc's log restated), runs the AR(1)
 * blend (alpha; 1 - alpha as the reference forms it) and the spot walk from spot0 (returns
 * normal(ret_mu, ret_sigma)), prices the grid's options (`grid`: strikes in percent of each
 * sample's spot, DH_STRIKE_PCT_SPOT; rate r, COS N, L) and forms market = model + normal(0,
 * noise_sigma) * model, the per-sample loss (np.mean's bits) and strikes = k_rel[j] spot / 100.
 * Every value is the reference loop's bit for bit; the RNG state arguments (np.random.get_state()
 * fields) are advanced in place to where that loop leaves them.  Host outputs (page-locked ones,
 * dh_host_alloc, move by DMA): params [n][13], spots [n], market, model, strikes [n][M], loss [n],
 * and dates [n][10] UCS-4 ('YYYY-MM-DD' weekdays from day first_day, dh_gen_dates) unless null.
 * stats [8] (optional): seconds from the call's start at which the twister and the walk ended,
 * the first chunk was issued and the call returned; AR(1) segments re-run serially; key blocks
 * bounded / used; chunks.  1 <= M <= 128.                                                        */
int dh_gen_device(dh_ctx* ctx, const dh_surface* grid, uint32_t* mt_key, int32_t* mt_pos,
                  int32_t* has_gauss, double* cached_gauss, int64_t n_samples, const double* lo,
                  const double* hi, double alpha, double spot0, double ret_mu, double ret_sigma,
                  double noise_sigma, double r, int N, double L, const double* k_rel,
                  int64_t first_day, double* params, double* spots, double* market,
                  double* model, double* loss, double* strikes, uint32_t* dates, double* stats);
/* The device's restatement of glibc's log (the legacy gauss's, dh_gen_device) over x[n]: its
 * GPU test against libm.                                                                         */
int dh_gen_log(dh_ctx* ctx, const double* x, int64_t n, double* out);
/* Page-locked host memory from a process-wide cache (hipHostMalloc; a freed block serves the next
 * request of up to 1.25x its size): the generator's output arrays.  dh_host_cache_trim releases
 * the cached blocks.                                                                             */
int dh_host_alloc(size_t bytes, void** out);
int dh_host_free(void* p);
int dh_host_cache_trim(void);

/* ---- paired pricing: option i under param set i ------------------------------------------- */
/* out[i] = price of (K[i], T[i], is_call[i]) under params[i]; replaces a loop of single
 * DoubleHeston(...).pricing(N) calls (double_heston.py:160-192).                              */
int dh_price_pairs(dh_ctx* ctx, const double* params, const double* K, const double* T,
                   const int8_t* is_call, int64_t P, int N, double L, double* out);

/* ---- building blocks (exposed for API parity with the reference's public methods) -------- */
/* phi(u_j; tau) for one param set: DoubleHeston.characteristic_function (double_heston.py:48-97) */
int dh_cf(dh_ctx* ctx, const double* params, const double* u, int n, double tau, double* re,
          double* im);
/* The same at complex frequencies phi_j = u_re[j] + i u_im[j] (the reference documents
 * phi : complex, double_heston.py:48-61, and evaluates it with complex arithmetic throughout)  */
int dh_cf_complex(dh_ctx* ctx, const double* params, const double* u_re, const double* u_im,
                  int n, double tau, double* re, double* im);
/* [a_i, b_i] for param set i and option i: DoubleHeston.truncationRange (double_heston.py:100-139) */
int dh_trunc_range(dh_ctx* ctx, const double* params, const double* K, const double* T,
                   int64_t P, double L, double* a, double* b);
/* chi_k / psi_k for integer k_j on [c,d] within [a,b]: double_heston.py:141-158 */
int dh_cos_coeffs(dh_ctx* ctx, const int32_t* k, int n, double c, double d, double a, double b,
                  double* chi, double* psi);

/* ---- multi-GPU: RCCL communicator (SURVEY 8(b) dh_allgather_best, 8(e)) --------------------- */
/* For callers without torch.distributed (the Python layer's dhcos.distributed uses either).  One
 * communicator per rank, on its context's device and stream; RCCL (librccl.so.1, resolved at run
 * time) over xGMI.  Rank 0 makes the id and ships its bytes to the other ranks by any means.
 * Replaces nothing in the reference (single process); it carries the multi-start sharding of
 * lbfgs_calibrator.py:251-299 across GPUs.                                                      */
#define DH_COMM_ID_BYTES 128
typedef struct dh_comm dh_comm;
int dh_comm_id(unsigned char* id /* [DH_COMM_ID_BYTES] */);
/* Collective: every rank of `world` calls it with the same id. */
int dh_comm_create(dh_ctx* ctx, const unsigned char* id, int world, int rank, dh_comm** out);
int dh_comm_destroy(dh_comm* comm);
/* buf[n] (host): root's values on every rank (the start x0s and the RNG state after the draws). */
int dh_comm_broadcast(dh_comm* comm, double* buf, int64_t n, int root);
/* send[n] (host) of every rank -> recv[world][n] in rank order (the generator's price blocks). */
int dh_comm_allgather(dh_comm* comm, const double* send, int64_t n, double* recv);
/* All-gather of fixed-size per-start records: each rank passes rows x width doubles (its starts;
 * rows must be equal on every rank, padding rows carry a negative start index), all receives
 * [world * rows][width] in rank order, and best the winning start index (or -1): the first start,
 * in start order (column col_start), whose col_fun value is strictly below every earlier one's --
 * lbfgs_calibrator.py:271-275's rule (NaN never wins), without its re-pricing step.            */
int dh_allgather_best(dh_comm* comm, const double* rec, int rows, int width, int col_start,
                      int col_fun, double* all, int* best);
/* The same selection over records already on the host (no device work). */
int dh_best_start(const double* all, int64_t rows, int width, int col_start, int col_fun,
                  int* best);

#ifdef __cplusplus
}
#endif
#endif /* DHCOS_H */
