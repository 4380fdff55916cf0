// Microbenchmark: issue cost of the fp64 VALU forms the COS kernels are made of, per wave64
// instruction, at 4 waves per SIMD (whole chip, HIP events) and the implied clock-normalised
// rate.  Each kernel runs 8 independent accumulator chains (no dependency stalls) of one form:
//   fma_vvv   v_fma_f64 acc, v, v, acc        (every operand a VGPR pair)
//   fma_vsv   v_fma_f64 acc, v, s[..], acc    (one operand an SGPR pair: the fma_k form)
//   mul / add v_mul_f64 / v_add_f64
//   fma+int   v_fma_f64 interleaved 1:1 with v_add_u32 (does integer VALU cost issue slots?)
//   int       v_add_u32 alone
//   fma_f32   v_fma_f32 (the fp32 rate, for scale)
//   mfma      v_mfma_f64_16x16x4_f64, 4 independent accumulators
//   hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int kIter = 4096;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int kind>
__global__ __launch_bounds__(256) void k(double* out, double sx) {
    const double x = 1.0 + threadIdx.x * 1e-12, y = 1.0 - threadIdx.x * 1e-12;
    double a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
    float f0 = x, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    int i0 = threadIdx.x, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3, i4 = i0 + 4, i5 = i0 + 5,
        i6 = i0 + 6, i7 = i0 + 7;
    double b0 = y, b1 = y + 1, b2 = y + 2, b3 = y + 3, b4 = y + 4, b5 = y + 5, b6 = y + 6, b7 = y + 7;
    d4 c0 = {x, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < kIter; ++it) {
        if constexpr (kind == 0) {
#define S(j) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a##j) : "v"(x), "v"(y));
            REP8(S)
#undef S
        } else if constexpr (kind == 1) {
#define S(j) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a##j) : "v"(x), "s"(sx));
            REP8(S)
#undef S
        } else if constexpr (kind == 2) {
#define S(j) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a##j) : "v"(y));
            REP8(S)
#undef S
        } else if constexpr (kind == 3) {
#define S(j) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a##j) : "v"(y));
            REP8(S)
#undef S
        } else if constexpr (kind == 4) {
#define S(j) asm volatile("v_fma_f64 %0, %2, %3, %0\n\tv_add_u32 %1, %1, %4" \
                          : "+v"(a##j), "+v"(i##j) : "v"(x), "v"(y), "v"(i0));
            REP8(S)
#undef S
        } else if constexpr (kind == 5) {
#define S(j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(i##j) : "v"(i7));
            REP8(S)
#undef S
        } else if constexpr (kind == 6) {
#define S(j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f##j) : "v"((float)x), "v"((float)y));
            REP8(S)
#undef S
        } else if constexpr (kind == 8) {     // 16 chains: two independent FMAs per accumulator
#define S(j) asm volatile("v_fma_f64 %0, %2, %3, %0\n\tv_fma_f64 %1, %3, %2, %1" \
                          : "+v"(a##j), "+v"(b##j) : "v"(x), "v"(y));
            REP8(S)
#undef S
        } else {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, c3, 0, 0, 0);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + f0 + f1 + f2 +
                                          f3 + f4 + f5 + f6 + f7 + i1 + i2 + i3 + i4 + i5 + i6 +
                                          i7 + c0.x + c1.y + c2.z + c3.w + b0 + b1 + b2 + b3 +
                                          b4 + b5 + b6 + b7;
}

template <int kind>
void run(const char* name, int n_inst_per_iter, double* out, int blocks = 1024) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k<kind>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k<kind>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per SIMD: blocks * 4 waves * kIter * n / 1024 SIMDs
    const double wi = (double)blocks * 4 * kIter * n_inst_per_iter / 1024.0;
    printf("%-8s %5d blocks %8.3f ms  %6.2f ns per wave-instruction per SIMD  (= %5.2f cycles "
           "at 2.4 GHz)\n", name, blocks, ms, ms * 1e6 / wi, ms * 1e6 / wi * 2.4);
}

int main() {
    double* out;
    const int blocks = 1024;   // 256 CUs x 4 blocks of 4 waves: 4 waves per SIMD
    (void)hipMalloc(&out, (size_t)4096 * 256 * 8);
    run<0>("fma_vvv", 8, out, blocks);
    run<1>("fma_vsv", 8, out, blocks);
    run<2>("mul", 8, out, blocks);
    run<3>("add", 8, out, blocks);
    run<4>("fma+int", 16, out, blocks);
    run<5>("int", 8, out, blocks);
    run<6>("fma_f32", 8, out, blocks);
    run<7>("mfma", 4, out, blocks);
    run<8>("fma16", 16, out, blocks);
    run<0>("fma_vvv", 8, out, 2048);       // 8 waves per SIMD
    run<8>("fma16", 16, out, 2048);
    run<0>("fma_vvv", 8, out, 256);        // 1 wave per SIMD
    run<8>("fma16", 16, out, 256);
    (void)hipFree(out);
    return 0;
}
