// probe_launch.hip -- floor of a graph-replayed launch on this box: the per-launch time of
// (a) an empty kernel, (b) a 1-workgroup kernel, (c) a streaming read of B bytes (plain
// dwordx4 loads, one partial sum per workgroup) for a few B, each replayed 200x in one
// hipGraph, plus s_memtime ticks per s_memrealtime tick (shader clock / 100 MHz).
// Build: hipcc -O3 --offload-arch=gfx950 -o probe_launch tools/probes/probe_launch.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void empty_kernel() {}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_kernel(const u32x4 *__restrict__ p, long n16, unsigned *__restrict__ out)
{
    unsigned acc = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc; // keeps the loads; practically never stores
}

__global__ void clock_kernel(unsigned long long *out)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long r = r0;
    while (r - r0 < 10000) r = __builtin_amdgcn_s_memrealtime(); // 100 us
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r - r0;
    }
}

template <class F>
static float per_launch(hipStream_t s, int reps, F launch)
{
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < reps; ++i) launch(i);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int t = 0; t < 5; ++t) {
        hipEventRecord(a, s);
        hipGraphLaunch(ge, s);
        hipEventRecord(b, s);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return best * 1000.f / reps;
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long *clk;
    CK(hipMalloc(&clk, 16));
    clock_kernel<<<1, 64, 0, s>>>(clk);
    unsigned long long h[2];
    CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    printf("s_memtime ticks per us: %.1f (over %llu realtime ticks)\n", (double)h[0] / (h[1] / 100.0), h[1]);
    const int reps = 200;
    printf("empty kernel, 1 wg      : %.2f us/launch\n",
           per_launch(s, reps, [&](int) { empty_kernel<<<1, 64, 0, s>>>(); }));
    printf("empty kernel, 2048 wg   : %.2f us/launch\n",
           per_launch(s, reps, [&](int) { empty_kernel<<<2048, 512, 0, s>>>(); }));
    // rotating buffers, >= 1 GiB in total, so reads come from HBM
    const size_t sizes[] = {4u << 20, 9437184, 24772608, 67108864, 268435456};
    unsigned *out;
    CK(hipMalloc(&out, 1 << 20));
    for (size_t B : sizes) {
        const int copies = (int)((1ull << 30) / B + 1 < 64 ? (1ull << 30) / B + 1 : 64);
        std::vector<u32x4 *> bufs(copies);
        for (auto &b : bufs) {
            CK(hipMalloc(&b, B));
            CK(hipMemset(b, 1, B));
        }
        for (int grid : {256, 1024, 2048}) {
            const float us = per_launch(s, reps, [&](int i) {
                read_kernel<<<grid, 256, 0, s>>>(bufs[i % copies], (long)(B / 16), out);
            });
            printf("read %9zu B grid %4d: %.2f us/launch  %.0f GB/s\n", B, grid, us, B / us / 1e3);
        }
        for (auto &b : bufs) CK(hipFree(b));
    }
    return 0;
}
