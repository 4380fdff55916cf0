// Microbenchmark: how long a kernel's first global loads take on gfx950, launched back to back the
// way a calibration request is (C2's fused kernel waits ~6.8k cycles for its parameter record).
// One wave per block; lane 0 times (s_memtime, 100 MHz) and (clock64, shader clock):
//   a) the first load of the request's record (a 2 KB device buffer the previous launch also read),
//   b) a second load from the same 4 KB page (translation now cached),
//   c) a load from a second allocation 64 MB away (another page),
//   d) the same loads on a 4 KB page no launch has touched since the host wrote it.
//   hipcc -O3 --offload-arch=gfx950 entry_latency.hip -o entry_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ long long clk() { return clock64(); }

__global__ void probe(const double* rec, const double* far, long long* out, int stride) {
    if (threadIdx.x != 0) return;
    const long long t0 = clk();
    double v = __builtin_nontemporal_load(rec + (blockIdx.x % 14) * 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t1 = clk();
    double w = __builtin_nontemporal_load(rec + 224 + (blockIdx.x % 14) * 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t2 = clk();
    double x = __builtin_nontemporal_load(far + (size_t)(blockIdx.x % 8) * stride);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t3 = clk();
    long long* o = out + blockIdx.x * 4;
    o[0] = t1 - t0;
    o[1] = t2 - t1;
    o[2] = t3 - t2;
    o[3] = (long long)(v + w + x);
}

static void report(const char* what, const std::vector<long long>& h, int blocks) {
    for (int c = 0; c < 3; ++c) {
        std::vector<long long> v;
        for (int b = 0; b < blocks; ++b) v.push_back(h[b * 4 + c]);
        std::sort(v.begin(), v.end());
        std::printf("%-34s %s  median %6lld  p10 %6lld  p90 %6lld cycles\n", what,
                    c == 0 ? "first load " : (c == 1 ? "same page  " : "other alloc"),
                    v[blocks / 2], v[blocks / 10], v[blocks * 9 / 10]);
    }
}

int main() {
    const int blocks = 448;                 // C2's grid
    double *rec, *far;
    long long* out;
    CHECK(hipMalloc(&rec, 4096));
    CHECK(hipMalloc(&far, (size_t)512 << 20));
    CHECK(hipMalloc(&out, blocks * 4 * sizeof(long long)));
    std::vector<double> hr(512, 1.0);
    CHECK(hipMemcpy(rec, hr.data(), 4096, hipMemcpyHostToDevice));
    CHECK(hipMemset(far, 0, (size_t)512 << 20));
    std::vector<long long> h(blocks * 4);
    const int stride = (64 << 20) / 8;      // 64 MB apart: a page per block group
    // back to back, the request pattern: the last of 200 launches
    for (int i = 0; i < 200; ++i) probe<<<blocks, 64>>>(rec, far, out, stride);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
    report("back-to-back (warm)", h, blocks);
    // after the host rewrote the record (a new request's parameters)
    for (int i = 0; i < 20; ++i) {
        hr[0] = i;
        CHECK(hipMemcpy(rec, hr.data(), 4096, hipMemcpyHostToDevice));
        probe<<<blocks, 64>>>(rec, far, out, stride);
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
    report("after a host copy of the record", h, blocks);
    // a fresh far page each launch (never touched since the memset)
    for (int i = 0; i < 8; ++i) {
        probe<<<blocks, 64>>>(rec, far + (size_t)(i + 1) * 4096 * 64, out, stride);
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
    report("fresh pages", h, blocks);
    int clk_khz = 0;
    CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    std::printf("clock64 rate attribute: %d kHz\n", clk_khz);
    return 0;
}
