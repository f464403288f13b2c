// Probe: load-side ceiling of the decode GEMV on a Q6_K 28672 x 8192 weight (192.7 MB),
// no arithmetic (every loaded word is xor-folded so no load is dead).
//   mode 0: the decode kernel's unit loads (UnitLoad<Q6_K>: 4 x 16 B + 8 B + 2 B per lane-unit),
//           R=2 rows per wave task, next task prefetched, grid 512 x 256
//   mode 1: same bytes as a flat stream: each wave-instruction reads 1 KiB contiguous,
//           U instructions in flight per wave, grid-strided over the tensor
//   mode 2: flat stream via LDS-DMA (buffer_load ... lds), 4 waves x 4 KiB per step, ring of 6 steps
//   mode 3: mode 1 with nt loads
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int64_t M = 28672, K = 8192, RB = K / 256 * 210;

__device__ __forceinline__ u32x4 ld16(const uint8_t *p) { return *(const u32x4 *)p; }

template <int MODE>
__global__ __launch_bounds__(256) void pk(const uint8_t *__restrict__ A, uint32_t *out, int64_t nbytes)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t x = 0;
    if constexpr (MODE == 0) {
        const int nunits = K / 64, niter = nunits / 64;
        const int64_t ngroups = M / 2, gstride = (int64_t)gridDim.x * 4;
        for (int64_t g = blockIdx.x * 4 + wave; g < ngroups; g += gstride) {
            for (int it = 0; it < niter; ++it) {
                const int u = lane + 64 * it;
                for (int r = 0; r < 2; ++r) {
                    const uint8_t *p = A + (g * 2 + r) * RB + 210 * (u >> 2);
                    const int h = (u >> 1) & 1, v = u & 1;
                    u32x4 l0 = ld16(p + 64 * h + 32 * v), l1 = ld16(p + 64 * h + 32 * v + 16);
                    u32x4 g0 = ld16(p + 128 + 32 * h), g1 = ld16(p + 144 + 32 * h);
                    u32x2 sc = *(const u32x2 *)(p + 192 + 8 * h);
                    uint32_t d = *(const uint16_t *)(p + 208);
                    x ^= l0.x ^ l0.w ^ l1.y ^ l1.z ^ g0.x ^ g0.w ^ g1.y ^ g1.z ^ sc.x ^ sc.y ^ d;
                }
            }
        }
    } else if constexpr (MODE == 4 || MODE == 5) {
        // lane = one 210-B superblock (14 x 16 B from its start), 16 lanes per row, 4 rows per
        // wave pass; rows grid-strided by wave; the next pass's loads issued before folding
        constexpr int NSB = K / 256, IT = NSB / 16;
        const int64_t nrows = M, wstride = (int64_t)gridDim.x * 4 * 4;
        const int li = lane & 15, lr = lane >> 4;
        for (int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 4; r0 < nrows; r0 += wstride) {
            const uint8_t *rowp = A + (r0 + lr) * RB;
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const uint8_t *p = rowp + 210 * (li + 16 * it);
                u32x4 v[14];
#pragma unroll
                for (int i = 0; i < 14; ++i) {
                    if constexpr (MODE == 5) v[i] = __builtin_nontemporal_load((const u32x4 *)(p + 16 * i));
                    else v[i] = ld16(p + 16 * i);
                }
#pragma unroll
                for (int i = 0; i < 14; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
            }
        }
    } else if constexpr (MODE == 1 || MODE == 3) {
        constexpr int U = 8;
        const int64_t step = (int64_t)gridDim.x * 4 * U * 1024;
        for (int64_t base = ((int64_t)blockIdx.x * 4 + wave) * U * 1024; base < nbytes; base += step) {
            u32x4 v[U];
#pragma unroll
            for (int i = 0; i < U; ++i) {
                const int64_t o = base + i * 1024 + lane * 16;
                const uint8_t *p = A + (o < nbytes ? o : 0);
                if constexpr (MODE == 3) v[i] = __builtin_nontemporal_load((const u32x4 *)p);
                else v[i] = ld16(p);
            }
#pragma unroll
            for (int i = 0; i < U; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        }
    } else {
        __shared__ __attribute__((aligned(1024))) uint8_t lds[6 * 16384];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, 0x7fffffff, 0x00020000);
        // WG b streams chunk c = b, b + grid, ...; chunk = 16 KiB; 6-slot ring, 4 in flight
        const int64_t nchunks = nbytes / 16384;
        const int64_t my = (nchunks - blockIdx.x + gridDim.x - 1) / gridDim.x;
        auto issue = [&](int64_t j) {
            const int64_t c = blockIdx.x + (j < my ? j : my - 1) * (int64_t)gridDim.x;
            uint8_t *dst = lds + (j % 6) * 16384;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(dst + 1024 * (4 * i + wave)), 16,
                                                         (uint32_t)(c * 16384 + 1024 * (4 * i + wave) + 16 * lane), 0, 0, 0);
        };
        for (int j = 0; j < 4; ++j) issue(j);
        for (int64_t j = 0; j < my; ++j) {
            asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
            issue(j + 4);
            const u32x4 *s = (const u32x4 *)(lds + (j % 6) * 16384);
            if constexpr (MODE == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const u32x4 v = s[256 * i + tid];
                    x ^= v.x ^ v.y ^ v.z ^ v.w;
                }
            } else { // Q6_K unit-pattern reads of the chunk: 78 superblocks = 312 units, 256 lanes
                const uint8_t *c = lds + (j % 6) * 16384;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int u = tid + 256 * i;
                    if (u < 312) {
                        uint32_t o = 210 * (u >> 2) + 64 * ((u >> 1) & 1) + 32 * (u & 1);
                        uint32_t oq = 210 * (u >> 2) + 128 + 32 * ((u >> 1) & 1);
                        if constexpr (MODE == 7) { o &= ~15u; oq &= ~15u; }
                        const u32x4 a = *(const u32x4 *)(c + o), b = *(const u32x4 *)(c + o + 16);
                        const u32x4 g = *(const u32x4 *)(c + oq), h = *(const u32x4 *)(c + oq + 16);
                        x ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ g.x ^ g.y ^ g.z ^ g.w ^ h.x ^ h.y ^ h.z ^ h.w;
                    }
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    out[blockIdx.x * 256 + tid] = x;
}

int main()
{
    const int64_t nbytes = M * RB;
    const int NC = 6;
    uint8_t *W[NC];
    uint32_t *out;
    for (int c = 0; c < NC; ++c) {
        (void)hipMalloc(&W[c], nbytes);
        (void)hipMemset(W[c], c + 1, nbytes);
    }
    (void)hipMalloc(&out, 4096 * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int grids[] = {256, 512, 1024, 2048};
    for (int mode = 2; mode < 8; ++mode) {
        for (int gi = 0; gi < 4; ++gi) {
            const int grid = mode == 0 ? (gi == 0 ? 512 : 0) : grids[gi];
            if (mode == 3 || mode == 4 || mode == 5) continue;
            if (!grid) continue;
            float best = 1e9;
            for (int rep = 0; rep < 3 * NC; ++rep) {
                (void)hipEventRecord(e0);
                if (mode == 0) pk<0><<<grid, 256>>>(W[rep % NC], out, nbytes);
                if (mode == 1) pk<1><<<grid, 256>>>(W[rep % NC], out, nbytes);
                if (mode == 2) pk<2><<<grid, 256>>>(W[rep % NC], out, nbytes);
                if (mode == 3) pk<3><<<grid, 256>>>(W[rep % NC], out, nbytes);
                if (mode == 4) pk<4><<<grid, 256>>>(W[rep % NC], out, nbytes);
                if (mode == 5) pk<5><<<grid, 256>>>(W[rep % NC], out, nbytes);
                if (mode == 6) pk<6><<<grid, 256>>>(W[rep % NC], out, nbytes);
                if (mode == 7) pk<7><<<grid, 256>>>(W[rep % NC], out, nbytes);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (rep >= NC && ms < best) best = ms;
            }
            printf("mode %d grid %5d: %8.1f us  %7.1f GB/s (%s)\n", mode, grid, best * 1e3, nbytes / best / 1e6,
                   hipGetErrorString(hipGetLastError()));
        }
    }
    return 0;
}
