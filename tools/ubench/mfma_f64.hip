// Microbenchmark: v_mfma_f64_16x16x4_f64 throughput on gfx950, fp64 VALU FMA throughput, and
// whether the two pipes overlap when MFMA waves and VALU waves share a SIMD (512-thread blocks:
// waves 0-3 one kind, waves 4-7 the other, so every SIMD holds one wave of each).
//   hipcc -O3 --offload-arch=gfx950 mfma_f64.hip -o /tmp/mfma_f64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int kind>   // 0: MFMA only, 1: VALU only, 2: waves < 4 MFMA, waves >= 4 VALU
__global__ __launch_bounds__(512) void mix(double* out, int reps) {
    const int wv = threadIdx.x >> 6;
    const bool do_mfma = kind == 0 || (kind == 2 && wv < 4);
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    if (do_mfma) {
        d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        for (int i = 0; i < reps; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
            }
        }
        out[blockIdx.x * blockDim.x + threadIdx.x] = c0.x + c1.y + c2.z + c3.w;
    } else {
        double x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = a + j;
        for (int i = 0; i < reps; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {   // 64 FMAs per iteration: 64 lane-FMA x 64 = 4096 MAC
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = fma(x[j], b, a);
            }
        }
        double s = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += x[j];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    }
}

template <int kind>
float run(int blocks, int reps, double* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(mix<kind>, dim3(blocks), dim3(512), 0, 0, out, reps);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(mix<kind>, dim3(blocks), dim3(512), 0, 0, out, reps);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    double* out;
    (void)hipMalloc(&out, (size_t)4096 * 512 * 8);
    const int reps = 2000;
    // one 512-thread block per CU (256 CUs): each SIMD holds two waves
    for (int blocks : {256, 512}) {
        const float m0 = run<0>(blocks, reps, out);
        const float m1 = run<1>(blocks, reps, out);
        const float m2 = run<2>(blocks, reps, out);
        // MFMA waves: 16 MFMA x reps, each 16x16x4 = 1024 MAC = 2048 flop
        const double fl_mfma = (double)blocks * 8 * reps * 16 * 2048.0;
        const double fl_valu = (double)blocks * 8 * reps * 64 * 64 * 2.0;
        printf("blocks=%d  mfma-only %.3f ms (%.1f TF)  valu-only %.3f ms (%.1f TF)  "
               "mixed %.3f ms (mfma half %.1f TF + valu half %.1f TF)\n",
               blocks, m0, fl_mfma / m0 / 1e9, m1, fl_valu / m1 / 1e9, m2,
               fl_mfma / 2 / m2 / 1e9, fl_valu / 2 / m2 / 1e9);
    }
    // single-wave issue rate: one 64-thread... (use 512 threads on 1 block: per-SIMD pipes)
    (void)hipFree(out);
    return 0;
}
