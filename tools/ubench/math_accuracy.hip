// Accuracy of the CF loop's table-driven primitives against the device library (ocml, ~0.5-1
// ulp): dexp_t over [-708, 709] (normal results), dsincos_t over [-2^12, 2^12], dlog_t over (1e-300, 1e300),
// datan2_t over random quadrants.  Prints the max error in units of the reference's last place.
//   hipcc -O3 --offload-arch=gfx950 -I../../option-pricing-ffn-lbfgs_amd/csrc math_accuracy.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include "dh_device.h"

__device__ double ulps(double got, double want) {
    if (got == want) return 0.0;
    if (!isfinite(want) || !isfinite(got)) return isnan(got) == isnan(want) ? 0.0 : 1e9;
    const double u = ldexp(1.0, ilogb(want) - 52);
    return fabs(got - want) / u;
}

__device__ unsigned long long mix(unsigned long long x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    return x ^ (x >> 33);
}

__global__ void check(int n, double* out) {
    __shared__ double2 sct[dh::kMathTab];
    dh::load_math_tables(sct, 0);
    __syncthreads();
    double e_exp = 0, e_sin = 0, e_cos = 0, e_log = 0, e_atan = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const double r = (mix(i) >> 11) * 0x1.0p-53;                   // [0, 1)
        const double r2 = (mix(i + 0x9e3779b97f4a7c15ULL) >> 11) * 0x1.0p-53;
        const double xe = -708.0 + 1417.0 * r;                         // normal results
        e_exp = fmax(e_exp, ulps(dh::dexp_t(xe, sct), exp(xe)));
        const double xs = (r - 0.5) * 8192.0;
        double s, c;
        dh::dsincos_t(xs, sct, &s, &c);
        if (fabs(sin(xs)) > 1e-3) e_sin = fmax(e_sin, ulps(s, sin(xs)));
        if (fabs(cos(xs)) > 1e-3) e_cos = fmax(e_cos, ulps(c, cos(xs)));
        const double xl = exp((r - 0.5) * 1380.0);
        if (fabs(log(xl)) > 1e-3) e_log = fmax(e_log, ulps(dh::dlog_t(xl, sct), log(xl)));
        const double ya = (r - 0.5) * 7.0, xa = (r2 - 0.5) * 5.0;
        e_atan = fmax(e_atan, ulps(dh::datan2_t(ya, xa, sct), atan2(ya, xa)));
    }
    double v[5] = {e_exp, e_sin, e_cos, e_log, e_atan};
    for (int k = 0; k < 5; ++k) {
        for (int off = 32; off > 0; off >>= 1) v[k] = fmax(v[k], __shfl_xor(v[k], off, 64));
        if ((threadIdx.x & 63) == 0) out[(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 5 + k] = v[k];
    }
}

int main() {
    const int blocks = 1024, threads = 256, n = 1 << 24;
    double* d;
    (void)hipMalloc(&d, (size_t)blocks * 4 * 5 * 8);
    hipLaunchKernelGGL(check, dim3(blocks), dim3(threads), 0, 0, n, d);
    static double h[1024 * 4 * 5];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    double m[5] = {0, 0, 0, 0, 0};
    for (int w = 0; w < blocks * 4; ++w)
        for (int k = 0; k < 5; ++k) m[k] = fmax(m[k], h[w * 5 + k]);
    printf("max ulp vs ocml over %d points: exp_t %.2f  sin_t %.2f  cos_t %.2f  log_t %.2f  "
           "atan2_t %.2f\n", n, m[0], m[1], m[2], m[3], m[4]);
    return 0;
}
