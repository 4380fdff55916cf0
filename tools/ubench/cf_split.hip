// Microbenchmark: latency of one CF table entry (dh::cf_phase_re) for a lone wave, and what
// spreading one entry over 2 lanes (one Heston factor each) buys.  Prints cycles per entry.
//   hipcc -O3 --offload-arch=gfx950 -I../../option-pricing-ffn-lbfgs_amd/csrc cf_split.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "dh_device.h"

__global__ void cf_one(const double* prm, double* out, long long* cyc, int reps) {
    const dh::Params P = dh::load_params(prm);
    const dh::CfConsts C = dh::cf_consts(P, 1.0);
    __shared__ double2 sct[dh::kMathTab];
    dh::load_sincos_table(sct);
    __syncthreads();
    double u = 1.0 + (threadIdx.x & 63) * 1e-2;
    long long t0 = clock64();
    for (int i = 0; i < reps; ++i) {
        const double w = dh::cf_phase_re(C, u, 1.0, -1.0, sct);
        u = 1.0 + 1e-3 * w + (threadIdx.x & 63) * 1e-2;
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = u;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

__device__ __forceinline__ double shfl_xor1(double v) {
    return __shfl_xor(v, 1, 64);
}

// lane pairs: even lane factor 1 + jump, odd lane factor 2; exchange X by shuffle, both lanes
// finish (the even one's result is kept)
__global__ void cf_pair(const double* prm, double* out, long long* cyc, int reps) {
    const dh::Params P = dh::load_params(prm);
    const dh::CfConsts C = dh::cf_consts(P, 1.0);
    __shared__ double2 sct[dh::kMathTab];
    dh::load_sincos_table(sct);
    __syncthreads();
    const bool odd = threadIdx.x & 1;
    const dh::FactorC F = odd ? C.f2 : C.f1;
    double u = 1.0 + ((threadIdx.x & 63) >> 1) * 1e-2;
    long long t0 = clock64();
    for (int i = 0; i < reps; ++i) {
        const dh::cplx X = dh::factor_x(F, u, 1.0, sct);
        const dh::cplx J = dh::jump_x(C, u, sct);
        const dh::cplx Xo = {shfl_xor1(X.re), shfl_xor1(X.im)};
        const dh::cplx X1 = odd ? Xo : X, X2 = odd ? X : Xo;
        const double w = dh::cf_phase_from(C, u, -1.0, X1, X2, J, sct);
        u = 1.0 + 1e-3 * w + ((threadIdx.x & 63) >> 1) * 1e-2;
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = u;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

template <typename K>
void run(const char* name, K kern, int threads, double per) {
    double *prm, *out; long long* cyc;
    (void)hipMalloc(&prm, 16 * 8); (void)hipMalloc(&out, 1 << 20); (void)hipMalloc(&cyc, 1 << 16);
    double h[16] = {0.04, 2.0, 0.04, 0.3, -0.5, 0.04, 1.5, 0.04, 0.2, -0.3, 0.1, -0.05, 0.1, 100, 0.03, 0};
    (void)hipMemcpy(prm, h, sizeof h, hipMemcpyHostToDevice);
    const int reps = 16;
    for (int it = 0; it < 2; ++it)
        hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, prm, out, cyc, reps);
    (void)hipDeviceSynchronize();
    long long c[16]; (void)hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
    long long mx = 0;
    for (int w = 0; w < threads / 64; ++w) mx = c[w] > mx ? c[w] : mx;
    printf("%-10s threads=%4d  %8.0f cycles per wave-iteration, %8.1f per entry-slot\n", name,
           threads, (double)mx / reps, (double)mx / reps / per);
    (void)hipFree(prm); (void)hipFree(out); (void)hipFree(cyc);
}

int main() {
    for (int th : {64, 256, 512, 1024}) run("cf_one", cf_one, th, 1.0);
    for (int th : {64, 256, 512, 1024}) run("cf_pair", cf_pair, th, 0.5);
    return 0;
}
