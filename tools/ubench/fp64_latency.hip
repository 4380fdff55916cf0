// Microbenchmark: dependent-chain latency and independent throughput (cycles per op, one wave
// per SIMD) of the fp64 primitives the COS kernels are built from, on gfx950.
//   hipcc -O3 --offload-arch=gfx950 -I../../option-pricing-ffn-lbfgs_amd/csrc fp64_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "dh_device.h"

#define CHAIN 256

template <int OP>
__device__ __forceinline__ double op(double x, double y) {
    if (OP == 0) return fma(x, y, 0.5);
    if (OP == 1) return x * y;
    if (OP == 2) return 1.0 / (x + 2.0);
    if (OP == 3) return sqrt(x + 1.5);
    if (OP == 4) return exp(x * 0.001);
    if (OP == 5) return log(x + 1.5);
    if (OP == 6) { double s, c; dh::dsincos(x, &s, &c); return s + c * y; }
    if (OP == 7) return dh::dlog(x + 1.5);
    if (OP == 8) return dh::datan2(x, y + 2.0);
    if (OP == 9) return atan2(x, y + 2.0);
    if (OP == 10) return dh::drcp(x + 2.0);
    if (OP == 11) return dh::dsqrt(x + 1.5);
    return x;
}

template <int OP, int ILP>
__global__ void lat(double* out, long long* cyc, double seed) {
    double x[ILP];
#pragma unroll
    for (int j = 0; j < ILP; ++j) x[j] = seed + threadIdx.x * 1e-3 + j;
    const double y = 0.999;
    long long t0 = clock64();
    for (int i = 0; i < CHAIN; ++i) {
#pragma unroll
        for (int j = 0; j < ILP; ++j) x[j] = op<OP>(x[j], y);
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int j = 0; j < ILP; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void cf_lat(const double* prm, double* out, long long* cyc, int ilp) {
    const dh::Params P = dh::load_params(prm);
    const dh::CfConsts C = dh::cf_consts(P, 1.0);
    __shared__ double2 sct[dh::kMathTab];
    dh::load_sincos_table(sct);
    __syncthreads();
    double u = 1.0 + threadIdx.x * 1e-3, u2 = 2.0 + threadIdx.x * 1e-3;
    long long t0 = clock64();
    for (int i = 0; i < 32; ++i) {
        const double w = dh::cf_phase_re(C, u, 1.0, -1.0, sct);
        u = 1.0 + 0.1 * w;
        if (ilp > 1) { const double w2 = dh::cf_phase_re(C, u2, 1.0, -1.0, sct); u2 = 2.0 + 0.1 * w2; }
    }
    long long t1 = clock64();
    out[threadIdx.x] = u + u2;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int OP, int ILP>
void run(const char* name, int waves) {
    double* out; long long* cyc;
    (void)hipMalloc(&out, 1 << 24); (void)hipMalloc(&cyc, 1 << 16);
    hipLaunchKernelGGL((lat<OP, ILP>), dim3(waves), dim3(64), 0, 0, out, cyc, 0.3);  // warm
    hipLaunchKernelGGL((lat<OP, ILP>), dim3(waves), dim3(64), 0, 0, out, cyc, 0.3);
    long long c; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-10s ilp=%d waves=%4d  %7.2f cycles/op/wave\n", name, ILP, waves,
           (double)c / (CHAIN * ILP));
    (void)hipFree(out); (void)hipFree(cyc);
}

int main() {
    run<0, 1>("fma", 1);   run<0, 8>("fma", 1);
    run<1, 1>("mul", 1);   run<2, 1>("rcp-div", 1); run<2, 4>("rcp-div", 1);
    run<3, 1>("sqrt", 1);  run<4, 1>("exp", 1);     run<4, 4>("exp", 1);
    run<5, 1>("log-ocml", 1); run<7, 1>("dlog", 1); run<6, 1>("dsincos", 1);
    run<6, 4>("dsincos", 1); run<8, 1>("datan2", 1); run<9, 1>("atan2-ocml", 1);
    run<10, 1>("drcp", 1); run<10, 4>("drcp", 1); run<11, 1>("dsqrt", 1);
    double h[16] = {0.04, 2.0, 0.04, 0.3, -0.5, 0.04, 1.5, 0.04, 0.2, -0.3, 0.5, -0.05, 0.1,
                    100.0, 0.05, 0.0};
    double* prm; double* out; long long* cyc;
    (void)hipMalloc(&prm, 128); (void)hipMalloc(&out, 1 << 16); (void)hipMalloc(&cyc, 64);
    (void)hipMemcpy(prm, h, 128, hipMemcpyHostToDevice);
    for (int ilp = 1; ilp <= 2; ++ilp) {
        hipLaunchKernelGGL(cf_lat, dim3(1), dim3(64), 0, 0, prm, out, cyc, ilp);
        hipLaunchKernelGGL(cf_lat, dim3(1), dim3(64), 0, 0, prm, out, cyc, ilp);
        long long c; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("cf_phase_re ilp=%d  %9.1f cycles per CF (latency, one wave)\n", ilp, (double)c / 32);
    }
    return 0;
}
