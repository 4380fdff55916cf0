// Microbenchmark: the first scalar read of a launch's kernel-argument segment on gfx950 (HIP puts
// kernel arguments in device memory; the fused kernel reads PriceArgs in place through the segment
// pointer).  Lane 0 of each block times, with s_memtime (shader clock):
//   a) an s_load from the segment at byte 256 (past the preloaded arguments),
//   b) a second s_load 256 bytes further (another line),
//   c) the same line again (a scalar-cache hit).
//   hipcc -O3 --offload-arch=gfx950 kernarg_latency.hip -o kernarg_latency
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct Big {
    long long* out;
    unsigned pad[254];
};

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int OFF>
__device__ __forceinline__ unsigned kload_at(const char* base) {
    unsigned v;
    asm volatile("s_load_dword %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(v) : "s"(base), "n"(OFF) : "memory");
    return v;
}

__global__ void probe(Big b) {
    const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned long long t0 = now();
    const unsigned a = kload_at<512>(ka);
    const unsigned long long t1 = now();
    const unsigned c = kload_at<768>(ka);
    const unsigned long long t2 = now();
    const unsigned d = kload_at<516>(ka);
    const unsigned long long t3 = now();
    if (threadIdx.x == 0) {
        long long* o = b.out + blockIdx.x * 4;
        o[0] = (long long)(t1 - t0);
        o[1] = (long long)(t2 - t1);
        o[2] = (long long)(t3 - t2);
        o[3] = a + c + d;
    }
}

int main() {
    const int blocks = 448;
    Big b{};
    CHECK(hipMalloc(&b.out, blocks * 4 * sizeof(long long)));
    for (int i = 0; i < 254; ++i) b.pad[i] = i;
    for (int i = 0; i < 200; ++i) {
        b.pad[0] = i;
        probe<<<blocks, 64>>>(b);
    }
    CHECK(hipDeviceSynchronize());
    std::vector<long long> h(blocks * 4);
    CHECK(hipMemcpy(h.data(), b.out, h.size() * 8, hipMemcpyDeviceToHost));
    const char* names[3] = {"first kernarg line ", "second kernarg line", "same line again    "};
    for (int c = 0; c < 3; ++c) {
        std::vector<long long> v;
        for (int k = 0; k < blocks; ++k) v.push_back(h[k * 4 + c]);
        std::sort(v.begin(), v.end());
        std::printf("%s median %6lld  p10 %6lld  p90 %6lld  max %6lld cycles\n", names[c],
                    v[blocks / 2], v[blocks / 10], v[blocks * 9 / 10], v[blocks - 1]);
    }
    return 0;
}
