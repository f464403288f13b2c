// Probe 2: LDS-DMA rates of the planned GEMM stage shapes (no compute), 256 WGs x 512 threads.
//   W: each WG streams 128 rows x 224 contiguous (16-B aligned) bytes per super-block stage
//      (Q6_K-like rows of 6720 B, K = 8192: 32 stages), 28 DMA instr/stage padded to 32
//   A: activation sub-stages: 8 tokens x 128 B per instruction, 16 instr per sub-stage, from a
//      2 MiB buffer every WG re-reads (L2 resident), 4 sub-stages per W stage
// mode 0 = W only, 1 = A only, 2 = W + A, 3 = W linear (1 KiB per instr) + A, 5 = W + A + reads; depth = sub-stages in flight for A (W: 1 ahead)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) void lds_void;

constexpr int ROWB = 6720, BM = 128, WSTAGES = 32;

template <int MODE>
__global__ __launch_bounds__(512) void pk(const uint8_t *W, const uint8_t *X, uint32_t *out, uint32_t wbytes,
                                          uint32_t xbytes)
{
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * 32 * 1024 + 4 * 16 * 1024];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void *)W, 0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, (int)xbytes, 0x00020000);
    uint32_t wv[4];
    for (int i = 0; i < 4; ++i) {
        const int p = 64 * (wave + 8 * i) + lane; // piece of the 128 x 14 tile (padded to 2048)
        const int r = p / 14, j = p - 14 * r;
        wv[i] = p < 128 * 14 ? (blockIdx.x * BM + r) * ROWB + 16 * j : 0xfffffff0u;
    }
    uint32_t xv[2];
    for (int i = 0; i < 2; ++i) {
        const int p = 64 * (wave + 8 * i) + lane, r = p >> 3, q = p & 7;
        xv[i] = r * 16384 + 16 * q; // token rows of 8192 fp16
    }
    auto issueW = [&](int s) {
        if (MODE == 1) return;
        uint8_t *d = lds + (s & 1) * 32768;
        for (int i = 0; i < 4; ++i) {
            const uint32_t lin = (uint32_t)blockIdx.x * BM * ROWB + (uint32_t)(s % WSTAGES) * 32768u +
                                 1024u * (wave + 8 * i) + 16u * lane;
            if (MODE == 7) {
                const uint32_t p = 64 * (wave + 8 * i) + lane, r = p / 14, j = p - 14 * r;
                const uint32_t vo = p < 128 * 14 ? (((blockIdx.x * BM + r) * ROWB + 210u * (s % WSTAGES)) & ~15u) + 16 * j
                                                 : 0xfffffff0u;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void *)(d + 1024 * (wave + 8 * i)), 16, vo, 0, 0, 0);
            } else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void *)(d + 1024 * (wave + 8 * i)), 16,
                                                     MODE == 3 ? lin : wv[i], MODE == 3 ? 0 : 224 * (s % WSTAGES), 0, 0);
        }
    };
    auto issueA = [&](int a) {
        if (MODE == 0) return;
        uint8_t *d = lds + 65536 + (a & 3) * 16384;
        for (int i = 0; i < (MODE == 7 ? 1 : 2); ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void *)(d + 1024 * (wave + 8 * i)), 16, xv[i],
                                                     128 * (a % 128), 0, 0);
    };
    uint32_t x = 0;
    issueW(0);
    issueA(0);
    issueA(1);
    issueA(2);
    const int NA = 4 * WSTAGES;
    for (int a = 0; a < NA; ++a) {
        const int s4 = a & 3;
        // outstanding allowed: A(a+1), A(a+2) and W(a/4+1) when issued after A(a)
        if (MODE == 7) {
            if (s4 == 2 || s4 == 3) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
        } else if (MODE == 6 || MODE == 3) {
            if (s4 == 2 || s4 == 3) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
        } else if (MODE == 0) {
            if (s4 == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
        } else if (MODE == 1) {
            asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
        } else {
            if (s4 == 2 || s4 == 3) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
        }
        if (s4 == 1) issueW(a / 4 + 1);
        issueA(a + 3);
        if (MODE >= 5) { // the GEMM's activation fragment reads: 16 ds_read_b128 per wave
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            const uint8_t *xs = MODE == 5 ? lds + 65536 + (a & 3) * 16384 : lds + 65536 + ((a + 2) & 3) * 16384;
            u4 v[16];
            for (int i = 0; i < 16; ++i) v[i] = *(const u4 *)(xs + ((lane * 16 + i * 1024) & 16383));
            for (int i = 0; i < 16; ++i) x += v[i].x ^ v[i].w;
        } else {
            x += lds[(tid * 4 + a * 64) & 0x1ffff];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[blockIdx.x * 512 + tid] = x;
}

int main()
{
    const size_t wbytes = (size_t)256 * BM * ROWB, xbytes = 128 * 16384;
    uint8_t *W, *X;
    uint32_t *out;
    uint8_t *Wc[6];
    for (int c = 0; c < 6; ++c) { (void)hipMalloc(&Wc[c], wbytes); (void)hipMemset(Wc[c], 1, wbytes); }
    W = Wc[0];
    (void)hipMalloc(&X, xbytes);
    (void)hipMalloc(&out, 256 * 512 * 4);
    (void)hipMemset(W, 1, wbytes);
    (void)hipMemset(X, 1, xbytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int mode = 0; mode < 8; ++mode) {
        if (mode == 4 || mode == 6) continue;
        float best = 1e9;
        for (int rep = 0; rep < 6; ++rep) {
            W = Wc[rep];
            (void)hipEventRecord(e0);
            if (mode == 0) pk<0><<<256, 512>>>(W, X, out, (uint32_t)wbytes, (uint32_t)xbytes);
            if (mode == 1) pk<1><<<256, 512>>>(W, X, out, (uint32_t)wbytes, (uint32_t)xbytes);
            if (mode == 7) pk<7><<<224, 512>>>(W, X, out, (uint32_t)wbytes, (uint32_t)xbytes);
            if (mode == 3) pk<3><<<256, 512>>>(W, X, out, (uint32_t)wbytes, (uint32_t)xbytes);
            if (mode == 2) pk<2><<<256, 512>>>(W, X, out, (uint32_t)wbytes, (uint32_t)xbytes);
            if (mode == 5) pk<5><<<256, 512>>>(W, X, out, (uint32_t)wbytes, (uint32_t)xbytes);
            if (mode == 6) pk<6><<<256, 512>>>(W, X, out, (uint32_t)wbytes, (uint32_t)xbytes);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double wb = mode == 7 ? 224.0 * BM * 210 * WSTAGES : (mode != 1) ? 256.0 * BM * 224 * WSTAGES : 0, xb = mode != 0 ? 256.0 * 16384 * 4 * WSTAGES : 0;
        printf("mode %d: %8.1f us  W %7.1f GB/s (%.1f GB/s/CU)  A %7.1f GB/s (%.1f GB/s/CU)  total/CU %.1f GB/s (%s)\n",
               mode, best * 1e3, wb / best / 1e6, wb / best / 1e6 / 256, xb / best / 1e6, xb / best / 1e6 / 256,
               (wb + xb) / best / 1e6 / 256, hipGetErrorString(hipGetLastError()));
    }
    return 0;
}
