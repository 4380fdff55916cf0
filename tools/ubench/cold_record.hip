// Microbenchmark: a request's first read of its parameter record on gfx950.  A calibration
// request's records sit in rows of a device buffer written once by the host and never read before
// that request (bench.py's request_bench, or the device driver's step kernel just wrote them).
// Launch i reads row i (cold) and row i + 512 (cold); lane 0 times with s_memtime:
//   a) s_load_dwordx16 of the row's first 64 bytes (the scalar path the fused kernel's prologue uses),
//   b) the same line again (scalar cache hit),
//   c) a vector load (global_load_dwordx2, every lane of the wave) of the other cold row,
//   d) a scalar load of a line the previous launch loaded (L2-warm).
//   hipcc -O3 --offload-arch=gfx950 cold_record.hip -o cold_record
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned u32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ void probe(const double* rows, int i, long long* out) {
    const double* row = rows + (size_t)i * 256;              // 2 KB rows
    const double* other = rows + (size_t)(i + 512) * 256;
    const double* prev = rows + (size_t)(i > 0 ? i - 1 : 0) * 256;
    const unsigned long long t0 = now();
    u32x16 a;
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(a) : "s"(row) : "memory");
    const unsigned long long t1 = now();
    u32x16 b;
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(b) : "s"(row) : "memory");
    const unsigned long long t2 = now();
    double v;
    const double* vp = other + (threadIdx.x & 15);
    asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(vp) : "memory");
    const unsigned long long t3 = now();
    u32x16 c;
    asm volatile("s_load_dwordx16 %0, %1, 0x40\n\ts_waitcnt lgkmcnt(0)" : "=s"(c) : "s"(prev) : "memory");
    const unsigned long long t4 = now();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        long long* o = out + (size_t)i * 5;
        o[0] = (long long)(t1 - t0);
        o[1] = (long long)(t2 - t1);
        o[2] = (long long)(t3 - t2);
        o[3] = (long long)(t4 - t3);
        o[4] = (long long)(a[0] + b[1] + c[2]) + (long long)v;
    }
}

int main() {
    const int n = 400;
    double* rows;
    long long* out;
    CHECK(hipMalloc(&rows, (size_t)1024 * 2048));
    CHECK(hipMalloc(&out, n * 5 * sizeof(long long)));
    std::vector<double> h((size_t)1024 * 256, 1.0);
    CHECK(hipMemcpy(rows, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep) {
        // rep 0: 448 blocks per launch (C2's grid, every block reading the same cold row); rep 1: 1
        const int blocks = rep == 0 ? 448 : 1;
        if (rep == 1) CHECK(hipMemcpy(rows, h.data(), h.size() * 8, hipMemcpyHostToDevice));
        for (int i = 0; i < n; ++i) probe<<<blocks, 64>>>(rows, i + (rep == 1 ? 0 : 0), out);
        CHECK(hipDeviceSynchronize());
        std::vector<long long> o(n * 5);
        CHECK(hipMemcpy(o.data(), out, o.size() * 8, hipMemcpyDeviceToHost));
        const char* names[4] = {"scalar, cold row     ", "scalar, same line    ",
                                "vector, cold row     ", "scalar, previous row "};
        for (int c = 0; c < 4; ++c) {
            std::vector<long long> v;
            for (int k = 8; k < n; ++k) v.push_back(o[k * 5 + c]);
            std::sort(v.begin(), v.end());
            std::printf("%3d blocks  %s median %6lld  p10 %6lld  p90 %6lld cycles\n", blocks, names[c],
                        v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10]);
        }
    }
    return 0;
}
