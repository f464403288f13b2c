// Probe: LDS-DMA streaming rate for the GEMM's weight-tile access shapes (no compute).
// 256 workgroups x 512 threads, each owns 256 rows of a [rows][6720 B] Q6_K-like tensor
// (K = 8192) and walks K in stages through a 4-slot LDS ring, 3 stages in flight.
//   mode 0: Q6_K stage pieces (6 x 16 B per row per 64 elements, 2-byte aligned)
//   mode 1: same offsets rounded down to 16 B
//   mode 2: 6 contiguous 16-B pieces per row per stage (96 B runs, aligned)
//   mode 3: every DMA instruction reads 1 KiB contiguous (tile streamed linearly)
//   mode 4: mode 0 pattern but global_load_dwordx4 into VGPRs (no LDS)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) void lds_void;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int ROWB = 6720, BM = 256, NP = 6, NI = BM * NP / 64; // 24 DMA instr per stage
constexpr int STAGES = 128;

__device__ uint32_t soff_q6(int c, int j) {
    const int h = (c >> 1) & 1, v = c & 1;
    const int o = j < 2 ? 64 * h + 32 * v + 16 * j : (j < 4 ? 128 + 32 * h + 16 * (j - 2) : (j == 4 ? 192 : 194));
    return 210 * (c >> 2) + o;
}

__global__ __launch_bounds__(512) void stream_kernel(const uint8_t *A, uint32_t *out, uint32_t nbytes, int MODE) {
    __shared__ __attribute__((aligned(1024))) uint8_t lds[4 * NI * 1024];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, (int)nbytes, 0x00020000);
    const uint32_t r0 = blockIdx.x * BM;
    uint32_t voff[3];
    int kj[3];
    for (int i = 0; i < 3; ++i) {
        const int kk = wave + 8 * i;
        kj[i] = kk / 4;
        voff[i] = (r0 + 64 * (kk % 4) + lane) * ROWB;
    }
    u32x4 x = {0, 0, 0, 0};
    auto so = [&](int c, int i) -> uint32_t {
        if (MODE == 0 || MODE == 4) return soff_q6(c, kj[i]);
        if (MODE == 1) return soff_q6(c, kj[i]) & ~15u;
        if (MODE == 2) return 52 * c + 16 * kj[i];
        return 0;
    };
    auto issue = [&](int c, int buf) {
        for (int i = 0; i < 3; ++i) {
            const int kk = wave + 8 * i;
            uint8_t *dst = lds + buf * NI * 1024 + 1024 * kk;
            if (MODE == 3) {
                const uint32_t off = (blockIdx.x * STAGES + c) * NI * 1024 + kk * 1024 + lane * 16;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)dst, 16, off, 0, 0, 0);
            } else if (MODE == 4) {
                x ^= __builtin_amdgcn_raw_buffer_load_b128(rs, voff[i], so(c, i), 0);
            } else {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)dst, 16, voff[i], so(c, i), 0, 0);
            }
        }
    };
    for (int i = 0; i < 3; ++i) issue(i, i);
    int buf = 0;
    for (int c = 0; c < STAGES; ++c) {
        if (MODE == 4) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
        issue(c + 3 < STAGES ? c + 3 : STAGES - 1, buf == 0 ? 3 : buf - 1);
        x.x += lds[(buf * NI * 1024 + tid * 4) % sizeof(lds)];
        buf = (buf + 1) & 3;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[blockIdx.x * 512 + tid] = x.x ^ x.y ^ x.z ^ x.w;
}

int main() {
    const size_t rows = 256 * 256;
    const size_t bytes = rows * ROWB; // 440 MB
    uint8_t *A;
    uint32_t *out;
    (void)hipMalloc(&A, bytes);
    (void)hipMalloc(&out, 256 * 512 * 4);
    (void)hipMemset(A, 1, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double useful = rows * 52.5 * STAGES; // Q6_K bytes for 128 stages x 64 elements
    const double dma = rows * 96.0 * STAGES;
    for (int mode = 0; mode < 5; ++mode) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipEventRecord(e0);
            switch (mode) {
            case 0: stream_kernel<<<256, 512>>>(A, out, (uint32_t)bytes, 0); break;
            case 1: stream_kernel<<<256, 512>>>(A, out, (uint32_t)bytes, 1); break;
            case 2: stream_kernel<<<256, 512>>>(A, out, (uint32_t)bytes, 2); break;
            case 3: stream_kernel<<<256, 512>>>(A, out, (uint32_t)bytes, 3); break;
            case 4: stream_kernel<<<256, 512>>>(A, out, (uint32_t)bytes, 4); break;
            }
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("mode %d: %8.1f us  useful %7.1f GB/s  dma %7.1f GB/s (%s)\n", mode, best * 1e3,
               useful / best / 1e6, dma / best / 1e6, hipGetErrorString(hipGetLastError()));
    }
    return 0;
}
