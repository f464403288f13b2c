// Probe 3: warp-specialized LDS-DMA streaming.  Workgroup = 8 reader waves (16 ds_read_b128
// each per sub-stage, like the GEMM's activation fragments) + L loader waves that issue every
// DMA of the planned GEMM stages (W: 128 rows x 224 B per 4 sub-stages, A: 16 KiB per sub-stage).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) void lds_void;
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
constexpr int ROWB = 6720, BM = 128, WSTAGES = 32;

__global__ __launch_bounds__(1024) void wk(const uint8_t *W, const uint8_t *X, uint32_t *out, uint32_t wbytes,
                                                  uint32_t xbytes, int L, int READS)
{
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * 32 * 1024 + 4 * 16 * 1024];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void *)W, 0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, (int)xbytes, 0x00020000);
    const int NWI = 32 / L, NAI = 16 / L; // per loader wave
    const int lw = wave - 8;
    uint32_t wv[16], xv[8];
    if (wave >= 8) {
        for (int i = 0; i < NWI; ++i) {
            const int p = 64 * (lw + L * i) + lane, r = p / 14, j = p - 14 * r;
            wv[i] = p < 128 * 14 ? (blockIdx.x * BM + r) * ROWB + 16 * j : 0xfffffff0u;
        }
        for (int i = 0; i < NAI; ++i) {
            const int p = 64 * (lw + L * i) + lane, r = p >> 3, q = p & 7;
            xv[i] = r * 16384 + 16 * q;
        }
    }
    auto issueW = [&](int s) {
        uint8_t *d = lds + (s & 1) * 32768;
        for (int i = 0; i < NWI; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void *)(d + 1024 * (lw + L * i)), 16, wv[i],
                                                     224 * (s % WSTAGES), 0, 0);
    };
    auto issueA = [&](int a) {
        uint8_t *d = lds + 65536 + (a & 3) * 16384;
        for (int i = 0; i < NAI; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void *)(d + 1024 * (lw + L * i)), 16, xv[i],
                                                     128 * (a % 128), 0, 0);
    };
    uint32_t x = 0;
    if (wave >= 8) {
        issueW(0);
        issueA(0);
        issueA(1);
        issueA(2);
    }
    const int NA = 4 * WSTAGES;
    for (int a = 0; a < NA; ++a) {
        const int s4 = a & 3;
        if (wave >= 8) {
            const int n = s4 != 0 ? 2 * NAI + NWI : 2 * NAI;
            if (n == 16) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
            else if (n == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
            else if (n == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
            else if (n == 32) asm volatile("s_waitcnt vmcnt(32)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            issueA(a + 3);
            if (s4 == 0) issueW(a / 4 + 1);
        } else {
            asm volatile("s_barrier" ::: "memory");
            const uint8_t *xs = lds + 65536 + (a & 3) * 16384;
            u4 v[16];
            if (READS) {
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = *(const u4 *)(xs + ((lane * 16 + i * 1024) & 16383));
#pragma unroll
                for (int i = 0; i < 16; ++i) x += v[i].x ^ v[i].w;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[blockIdx.x * 768 + tid] = x;
}

void run(int L, int R, const char *name, const uint8_t *W, const uint8_t *X, uint32_t *out, size_t wbytes, size_t xbytes)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(wk, dim3(256), dim3(64 * (8 + L)), 0, 0, W, X, out, (uint32_t)wbytes, (uint32_t)xbytes, L, R);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double wb = 256.0 * BM * 224 * WSTAGES, xb = 256.0 * 16384 * 4 * WSTAGES;
    printf("%-28s %8.1f us  W %7.1f GB/s  A %7.1f GB/s  total/CU %.1f GB/s (%s)\n", name, best * 1e3, wb / best / 1e6,
           xb / best / 1e6, (wb + xb) / best / 1e6 / 256, hipGetErrorString(hipGetLastError()));
}

int main()
{
    const size_t wbytes = (size_t)256 * BM * ROWB, xbytes = 128 * 16384;
    uint8_t *W, *X;
    uint32_t *out;
    (void)hipMalloc(&W, wbytes);
    (void)hipMalloc(&X, xbytes);
    (void)hipMalloc(&out, 256 * 1024 * 4);
    (void)hipMemset(W, 1, wbytes);
    (void)hipMemset(X, 1, xbytes);
    run(4, 0, "4 loaders, no reads", W, X, out, wbytes, xbytes);
    run(4, 16, "4 loaders, 16 reads", W, X, out, wbytes, xbytes);
    run(8, 16, "8 loaders, 16 reads", W, X, out, wbytes, xbytes);
    run(2, 16, "2 loaders, 16 reads", W, X, out, wbytes, xbytes);
    return 0;
}
