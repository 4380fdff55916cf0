// Microbenchmark: what a kernel pays to fetch straight-line code it has not run yet on gfx950.
// One wave per block runs a 16 KB (4,096 x 4-byte v_add_u32) straight-line body twice; lane 0
// times each pass with clock64 (the shader clock).  The first pass fetches the code into the
// instruction cache (its lines come from L2 after the launch that ran it before), the second runs
// from the cache.  Blocks: 448 (C2's grid) or 1 (a lone wave, no duplicate misses).
//   hipcc -O3 --offload-arch=gfx950 icache_cold.hip -o icache_cold
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void body(int* out, long long* cyc, int seed) {
    int v = threadIdx.x + seed, w = seed * 3 + 1;
    long long t[3];
#pragma clang loop unroll(disable)
    for (int pass = 0; pass < 2; ++pass) {
        t[pass] = clock64();
        asm volatile(".rept 4096\n v_add_u32 %0, %0, %1\n .endr" : "+v"(v) : "v"(w));
    }
    t[2] = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0) {
        cyc[blockIdx.x * 2] = t[1] - t[0];
        cyc[blockIdx.x * 2 + 1] = t[2] - t[1];
    }
}


// 64 taken forward branches, each over a 256-byte gap of code never run, 16 v_add between them:
// what a cold taken branch costs on the first pass against the second
__global__ void jumps(int* out, long long* cyc, int seed) {
    int v = threadIdx.x + seed, w = seed * 3 + 1;
    long long t[3];
#pragma clang loop unroll(disable)
    for (int pass = 0; pass < 2; ++pass) {
        t[pass] = clock64();
        asm volatile(".rept 64\n"
                     " .rept 16\n v_add_u32 %0, %0, %1\n .endr\n"
                     " s_branch 1f\n"
                     " .rept 64\n s_nop 0\n .endr\n"
                     "1:\n"
                     ".endr" : "+v"(v) : "v"(w));
    }
    t[2] = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0) {
        cyc[blockIdx.x * 2] = t[1] - t[0];
        cyc[blockIdx.x * 2 + 1] = t[2] - t[1];
    }
}

int main() {
    int* out;
    long long* cyc;
    CHECK(hipMalloc(&out, 448 * 64 * sizeof(int)));
    CHECK(hipMalloc(&cyc, 448 * 2 * sizeof(long long)));
    std::vector<long long> h(448 * 2);
    for (int blocks : {1, 448}) {
        for (int i = 0; i < 50; ++i) body<<<blocks, 64>>>(out, cyc, i);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(h.data(), cyc, blocks * 2 * sizeof(long long), hipMemcpyDeviceToHost));
        std::vector<long long> a, b;
        for (int k = 0; k < blocks; ++k) { a.push_back(h[2 * k]); b.push_back(h[2 * k + 1]); }
        std::sort(a.begin(), a.end());
        std::sort(b.begin(), b.end());
        std::printf("%3d blocks: 16 KB straight line, first pass median %6lld (max %6lld), "
                    "second pass median %6lld cycles\n", blocks, a[blocks / 2], a[blocks - 1],
                    b[blocks / 2]);
    }
    for (int blocks : {1, 448}) {
        for (int i = 0; i < 50; ++i) jumps<<<blocks, 64>>>(out, cyc, i);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(h.data(), cyc, blocks * 2 * sizeof(long long), hipMemcpyDeviceToHost));
        std::vector<long long> a, b;
        for (int k = 0; k < blocks; ++k) { a.push_back(h[2 * k]); b.push_back(h[2 * k + 1]); }
        std::sort(a.begin(), a.end());
        std::sort(b.begin(), b.end());
        std::printf("%3d blocks: 64 taken branches over 256-byte gaps, first pass median %6lld "
                    "(max %6lld), second pass median %6lld cycles\n", blocks, a[blocks / 2],
                    a[blocks - 1], b[blocks / 2]);
    }
    return 0;
}
