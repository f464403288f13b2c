// Probe: does global_load_lds_dwordx4 accept global addresses that are only 2-byte aligned?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>

__global__ void k(const uint8_t *g, uint8_t *out, int shift)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
    const int t = threadIdx.x;
    __builtin_amdgcn_global_load_lds((const void *)(g + shift + 16 * t), (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int i = t; i < 1024; i += 64) out[i] = lds[i];
}

// Probe 2: ds_read_b64 / ds_read_b32 at 2-byte aligned LDS addresses (inline asm, so the
// compiler cannot split them).
__global__ void k2(const uint8_t *g, uint8_t *out, int shift)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[2048];
    const int t = threadIdx.x;
    for (int i = t; i < 2048; i += 64) lds[i] = g[i];
    __syncthreads();
    uint32_t a = (uint32_t)(uintptr_t)(lds) + 16 * t + shift;
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    u2 v;
    uint32_t w;
    asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    asm volatile("ds_read_b32 %0, %1 offset:8\n s_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(a) : "memory");
    memcpy(out + 12 * t, &v, 8);
    memcpy(out + 12 * t + 8, &w, 4);
}

int main()
{
    uint8_t *g, *o;
    hipMalloc(&g, 4096);
    hipMalloc(&o, 1024);
    uint8_t h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 7 + 3);
    hipMemcpy(g, h, 4096, hipMemcpyHostToDevice);
    int bad_total = 0;
    for (int shift = 0; shift < 16; ++shift) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, g, o, shift);
        hipError_t e = hipDeviceSynchronize();
        uint8_t r[1024];
        hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 1024; ++i) bad += r[i] != h[shift + i];
        printf("shift %2d: err=%s mismatches=%d first=%02x want=%02x\n", shift, hipGetErrorString(e), bad, r[0], h[shift]);
        bad_total += bad;
    }
    printf("PROBE_DMA %s\n", bad_total ? "UNALIGNED_BROKEN" : "UNALIGNED_OK");
    bad_total = 0;
    for (int shift = 0; shift < 8; shift += 1) {
        hipLaunchKernelGGL(k2, dim3(1), dim3(64), 0, 0, g, o, shift);
        hipError_t e = hipDeviceSynchronize();
        uint8_t r[1024];
        hipMemcpy(r, o, 768, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int t = 0; t < 64; ++t)
            for (int i = 0; i < 12; ++i) bad += r[12 * t + i] != h[16 * t + shift + i];
        printf("lds shift %d: err=%s mismatches=%d\n", shift, hipGetErrorString(e), bad);
        bad_total += bad;
    }
    printf("PROBE_LDS %s\n", bad_total ? "UNALIGNED_BROKEN" : "UNALIGNED_OK");
    return 0;
}
