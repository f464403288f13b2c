// probe_gemm_ingest.hip -- where does the MMQ GEMM's per-CU LDS-DMA ingest rate go?
//
// Diagnostic probe (never the product).  One 128-row x 128-token tile per workgroup, the exact
// DMA pattern of gemm_kernel<Q8_0, NB=8> (mmq_gemm.hip): weight stages of one super-block per
// row (128 rows x 17 pieces of 16 B, 272-B rows), activation sub-stages of 64 elements (128
// token rows x 128 B, source-swizzled pieces), NAS activation slots + NWS weight slots in LDS.
// Features are switched on one at a time:
//   STREAMS   1 activations only (L2-served: every workgroup of a split reads the same slab),
//             2 weights only (HBM: a fresh region of a 1.25 GB buffer per launch), 3 both
//   WLAY      weight DMA addresses: 0 the GEMM's row pieces, 1 one contiguous run per stage
//   SYNC      0 loaders free-run on their own vmcnt (ring reuse unchecked -- no consumer),
//             1 the GEMM's s_barrier per sub-stage with NC consumer waves
//   CW        consumer work per sub-stage: 0 none, 1 the fragment reads (16 ds_read_b128 of
//             activations + the Q8_0 weight reads), 2 + 16 fp16 MFMAs, 3 + the Q8_0 dequant
// Rates are per CU: bytes one workgroup moves / kernel span (s_memrealtime, 100 MHz, first
// workgroup start to last workgroup end), and event time over back-to-back launches.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o /tmp/probe_gemm_ingest tools/probes/probe_gemm_ingest.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

#define CHECK(x)                                                                                       \
    do {                                                                                               \
        hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) {                                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                  \
            exit(1);                                                                                   \
        }                                                                                              \
    } while (0)

constexpr int BM = 128, BN = 128, NB = 8, NPW = 17, RBW = 272, SPW = 4;
constexpr int W_REAL = BM * NPW / 64; // 34 DMA instructions per weight stage
constexpr int A_REAL = BN * 8 / 64;   // 16 per activation sub-stage
constexpr int W_SLOT = W_REAL * 1024, A_SLOT = A_REAL * 1024;

template <int MAXN> __device__ __attribute__((always_inline)) inline void vm_wait(int n)
{
    if constexpr (MAXN <= 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        if (n >= MAXN) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MAXN) : "memory");
        else vm_wait<MAXN - 1>(n);
    }
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint8_t *dst, uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)dst, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ h2 as_h2(uint32_t v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ uint32_t as_u32(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2 pair02(uint32_t c) { return as_h2(__builtin_amdgcn_perm(0x64646464u, c, 0x04020400u)); }
__device__ __forceinline__ h2 pair13(uint32_t c) { return as_h2(__builtin_amdgcn_perm(0x64646464u, c, 0x04030401u)); }
__device__ __forceinline__ f16x8 frag4(h2 a, h2 b, h2 c, h2 d)
{
    u32x4 v = {as_u32(a), as_u32(b), as_u32(c), as_u32(d)};
    return __builtin_bit_cast(f16x8, v);
}
__device__ __forceinline__ int act_swz(int r) { return (r >> 1) & 7; }

// Q8_0 fragments of sub-stage u (the GEMM's stage_frags<Q8_0>, aligned-read form)
template <bool DEQ>
__device__ __forceinline__ void q8_frags(const uint8_t *wr, int g, int u, f16x8 (&frag)[2])
{
    const h2 bias = {(_Float16)-1152.f, (_Float16)-1152.f};
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const uint8_t *blk = wr + 34 * (2 * u + b);
        const int off = 34 * (2 * u + b) + 2, sh = off & 7;
        const uint8_t *al = wr + (off & ~7) + 8 * g;
        const u32x2 lo = *(const u32x2 *)al, hi = *(const u32x2 *)(al + 8);
        if constexpr (!DEQ) {
            frag[b] = __builtin_bit_cast(f16x8, (u32x4){lo.x, lo.y, hi.x, hi.y});
            continue;
        }
        const _Float16 dh = __builtin_bit_cast(_Float16, *(const uint16_t *)blk);
        const h2 d = {dh, dh};
        u32x2 q;
        if (sh == 0) q = lo;
        else if (sh < 4) q = (u32x2){__builtin_amdgcn_alignbyte(lo.y, lo.x, sh), __builtin_amdgcn_alignbyte(hi.x, lo.y, sh)};
        else if (sh == 4) q = (u32x2){lo.y, hi.x};
        else q = (u32x2){__builtin_amdgcn_alignbyte(hi.x, lo.y, sh - 4), __builtin_amdgcn_alignbyte(hi.y, hi.x, sh - 4)};
        const uint32_t c0 = q.x ^ 0x80808080u, c1 = q.y ^ 0x80808080u;
        frag[b] = frag4((pair02(c0) + bias) * d, (pair13(c0) + bias) * d, (pair02(c1) + bias) * d, (pair13(c1) + bias) * d);
    }
}

struct Args {
    const uint8_t *W;   // weights of this launch (row-major Q8_0 rows, M x row_bytes)
    const uint8_t *X;   // fp16 activations [128][K]
    int64_t M, K;
    int sps;            // super-blocks (weight stages) per split
    unsigned long long *st; // per workgroup: realtime start, realtime end, memtime first-landed, memtime end
    float *sink;
};

template <int NL, int NC, int NAS, int NWS, int SYNC, int CW, int STREAMS, int WLAY, int WPRE = -1, int PRIO = 0>
__global__ __launch_bounds__(64 * (NL + NC)) void probe(Args p)
{
    constexpr int NW = (W_REAL + NL - 1) / NL, NA = (A_REAL + NL - 1) / NL;
    constexpr bool PAD = W_REAL % NL != 0 || A_REAL % NL != 0;
    constexpr int A_BASE = NWS * W_SLOT, SCRATCH = A_BASE + NAS * A_SLOT;
    constexpr int LDS_BYTES = SCRATCH + (PAD ? 1024 : 0);
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
    constexpr bool DO_A = STREAMS & 1, DO_W = STREAMS & 2;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];

    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), mt0 = __builtin_amdgcn_s_memtime();
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, l16 = lane & 15;
    const int64_t m0 = (int64_t)blockIdx.x * BM;
    const int64_t nsb = p.K / 256, row_bytes = p.K / 32 * 34;
    const int64_t sb0 = (int64_t)blockIdx.z * p.sps, sb1 = sb0 + p.sps < nsb ? sb0 + p.sps : nsb;
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)p.W, 0, (int)(uint32_t)(p.M * row_bytes), 0x00020000);
    const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void *)p.X, 0, (int)(uint32_t)(BN * p.K * 2), 0x00020000);
    unsigned long long mt_first = 0;
    float sacc = 0.f;

    if (wave < NL) {
        const int iw = wave;
        uint32_t wv[NW];
        int wpc[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int pp = 64 * (iw + NL * i) + lane, r = pp / NPW;
            wpc[i] = pp - r * NPW;
            wv[i] = r < BM ? (uint32_t)((m0 + r) * row_bytes) : 0u;
        }
        uint32_t av[NA];
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int k = iw + NL * i, pp = 64 * k + lane, r = pp >> 3, q = pp & 7;
            av[i] = r < BN ? (uint32_t)(r * p.K * 2) + 16u * (uint32_t)(q ^ act_swz(r)) : 0u;
        }
        auto issue_w = [&](int64_t w) {
            if constexpr (!DO_W) return;
            uint8_t *dst = lds + (int)(w % NWS) * W_SLOT;
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int k = iw + NL * i;
                uint32_t vo, so;
                if constexpr (WLAY == 1) {
                    vo = (uint32_t)(m0 * row_bytes) + 16u * (uint32_t)(64 * k + lane);
                    so = (uint32_t)(w * W_SLOT);
                } else {
                    vo = wv[i] + 16u * wpc[i];
                    so = (uint32_t)(RBW * w);
                }
                dma16(wrs, k < W_REAL ? dst + 1024 * k : lds + SCRATCH, vo, so);
            }
        };
        auto issue_a = [&](int64_t a) {
            if constexpr (!DO_A) return;
            uint8_t *dst = lds + A_BASE + (int)(a % NAS) * A_SLOT;
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int k = iw + NL * i;
                dma16(ars, k < A_REAL ? dst + 1024 * k : lds + SCRATCH, av[i], (uint32_t)(128 * a));
            }
        };
        const int64_t w0 = sb0, w1 = sb1, a0 = 4 * sb0, a1 = 4 * sb1;
        const int nrel = (int)(a1 - a0), nws = (int)(w1 - w0);
        constexpr int WP = WPRE < 0 ? NWS - 1 : WPRE; // weight stages in flight ahead
        static_assert(WP <= NWS, "weight prologue");
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(PRIO);
#pragma unroll
        for (int i = 0; i < WP; ++i)
            if (w0 + i < w1) issue_w(w0 + i);
#pragma unroll
        for (int i = 0; i < NAS - 1; ++i)
            if (a0 + i < a1) issue_a(a0 + i);
        constexpr int LA = CW == 6 ? 1 : 0; // sub-stages read ahead of the multiply
        for (int64_t a = a0; a < a1; ++a) {
            const int it = (int)(a - a0), rel = it + LA < nrel ? it + LA : nrel - 1;
            // "A(rel) landed" (and so W(rel/4)) at iteration it: the ops issued after it -- the
            // younger A's (issued up to iteration it-1) and the W's of iterations after A(rel)'s
            constexpr int na = DO_A ? NA : 0, nw = DO_W ? NW : 0;
            const int ya = (it + NAS - 2 < nrel - 1 ? it + NAS - 2 : nrel - 1) - rel;
            const int lo = rel - NAS + 1 > 0 ? rel - NAS + 1 : 0;
            const int hi = it - 1 < SPW * (nws - WP) - 1 ? it - 1 : SPW * (nws - WP) - 1;
            const int w_after = hi >= lo ? hi / SPW - (lo + SPW - 1) / SPW + 1 : 0;
            if constexpr (!DO_A) {
                const int w = rel / SPW, yw = WP - 1 < nws - 1 - w ? WP - 1 : nws - 1 - w;
                if (rel % SPW == 0) vm_wait<(WP - 1) * nw>(yw * nw);
            } else {
                vm_wait<(NAS - 2) * na + ((NAS - 1 + SPW - 1) / SPW) * nw>(ya * na + w_after * nw);
            }
            if (it == 0) mt_first = __builtin_amdgcn_s_memtime() - mt0;
            if constexpr (SYNC) asm volatile("s_barrier" ::: "memory");
            if (a + NAS - 1 < a1) issue_a(a + NAS - 1);
            if (a % SPW == 0 && a / SPW + WP < w1) issue_w(a / SPW + WP);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (SYNC) {
        constexpr int RGC = 8 / NC; // row groups per consumer wave (128 rows)
        const int cw = wave - NL;   // consumer wave: rows 16*(RGC*cw + rg) + [0, 16)
        f32x4 acc[RGC][NB];
#pragma unroll
        for (int rg = 0; rg < RGC; ++rg)
#pragma unroll
            for (int t = 0; t < NB; ++t) acc[rg][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
        uint32_t x = 0;
        f16x8 kf = __builtin_bit_cast(f16x8, (u32x4){0x3c003c00u + lane, 0x3c003c00u, 0x3c003c00u, 0x3c003c00u});
        f16x8 bfr[2][NB], af[RGC][2];
        auto read_frags = [&](int64_t a) __attribute__((always_inline)) {
            const int s4 = (int)(a % SPW);
            const uint8_t *xs = lds + A_BASE + (int)(a % NAS) * A_SLOT;
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const int r = 16 * t + l16;
                    bfr[s][t] = *(const f16x8 *)(xs + 128 * r + 16 * ((4 * s + g) ^ act_swz(r)));
                }
#pragma unroll
            for (int rg = 0; rg < RGC; ++rg) {
                const uint8_t *wr = lds + (int)((a / SPW) % NWS) * W_SLOT + RBW * (16 * (RGC * cw + rg) + l16);
                if constexpr (CW >= 3) q8_frags<true>(wr, g, s4, af[rg]);
                else q8_frags<false>(wr, g, s4, af[rg]);
            }
        };
        auto mma_all = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int rg = 0; rg < RGC; ++rg)
#pragma unroll
                    for (int t = 0; t < NB; ++t) acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[rg][s], bfr[s][t], acc[rg][t], 0, 0, 0);
        };
        for (int64_t a = 4 * sb0; a < 4 * sb1; ++a) {
            asm volatile("s_barrier" ::: "memory");
            if constexpr (CW == 0) continue;
            if constexpr (CW == 4) { // MFMAs only, operands in registers
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int rg = 0; rg < RGC; ++rg)
#pragma unroll
                        for (int t = 0; t < NB; ++t) acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, kf, acc[rg][t], 0, 0, 0);
                continue;
            }
            if constexpr (CW == 5 || CW == 6) {
                // 5: waves of the second half lag one sub-stage (their MFMAs of a-1 before their
                //    reads of a), so on every SIMD one wave reads LDS while its partner multiplies;
                // 6: every wave reads sub-stage a+1's fragments before multiplying a (the loaders
                //    wait for A(a+1) at barrier a: LA = 1)
                const bool lag = CW == 5 ? cw >= NC / 2 : true;
                const int64_t ra = CW == 6 ? a + 1 : a; // the sub-stage read in this interval
                if (lag && a > 4 * sb0) mma_all();
                if (ra < 4 * sb1) read_frags(ra);
                if (!lag) mma_all();
                continue;
            }
            read_frags(a);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (CW == 1) {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const u32x4 w = __builtin_bit_cast(u32x4, af[0][s]);
                    x ^= w.x ^ w.y ^ w.z ^ w.w;
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        const u32x4 v = __builtin_bit_cast(u32x4, bfr[s][t]);
                        x += v.x ^ v.y ^ v.z ^ v.w;
                    }
                }
            } else {
                mma_all();
            }
        }
        if constexpr (CW == 5 || CW == 6) {
            if (CW == 6 || cw >= NC / 2) mma_all(); // the lagging multiply of the last sub-stage
        }
#pragma unroll
        for (int rg = 0; rg < RGC; ++rg)
#pragma unroll
            for (int t = 0; t < NB; ++t) sacc += acc[rg][t][0] + acc[rg][t][3];
        sacc += (float)(x & 1);
    }
    if (sacc == 1234.5f) p.sink[0] = sacc;
    if (tid == 0) {
        const int64_t wg = (int64_t)blockIdx.z * gridDim.x + blockIdx.x;
        p.st[4 * wg + 0] = rt0;
        p.st[4 * wg + 1] = __builtin_amdgcn_s_memrealtime();
        p.st[4 * wg + 2] = mt_first;
        p.st[4 * wg + 3] = __builtin_amdgcn_s_memtime() - mt0;
    }
}

__global__ void touch(uint16_t *x, int64_t n, int v)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        x[i] = (uint16_t)(0x3c00 + ((i + v) & 0xff));
}

struct Buf {
    uint8_t *W;
    size_t wbytes;
    uint8_t *X;
    unsigned long long *st;
    float *sink;
};

template <int NL, int NC, int NAS, int NWS, int SYNC, int CW, int STREAMS, int WLAY, int WPRE = -1, int PRIO = 0>
void run(const char *name, Buf &b, int64_t M, int64_t K, int splits, bool prewrite, int reps = 24)
{
    const int64_t row_bytes = K / 32 * 34, wlaunch = M * row_bytes;
    const int sps = (int)(K / 256 / splits);
    const int ncopies = (int)std::max<int64_t>(1, (int64_t)(b.wbytes / wlaunch));
    const dim3 grid((unsigned)(M / BM), 1, (unsigned)splits);
    const int nwg = (int)(grid.x * grid.z);
    auto launch = [&](int i) {
        Args a{b.W + (size_t)(i % ncopies) * wlaunch, b.X, M, K, sps, b.st, b.sink};
        probe<NL, NC, NAS, NWS, SYNC, CW, STREAMS, WLAY, WPRE, PRIO><<<grid, 64 * (NL + NC)>>>(a);
    };
    const int64_t xn = (int64_t)BN * K;
    for (int i = 0; i < 3; ++i) {
        if (prewrite) touch<<<256, 256>>>((uint16_t *)b.X, xn, i);
        launch(i);
    }
    CHECK(hipDeviceSynchronize());
    std::vector<double> span, first, per;
    std::vector<unsigned long long> h(4 * (size_t)nwg);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float ev_ms = 0.f;
    if (!prewrite) { // event time over back-to-back launches
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch(3 + i);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ev_ms, e0, e1));
    }
    for (int i = 0; i < 9; ++i) { // spans from the stamps, one launch at a time
        if (prewrite) touch<<<256, 256>>>((uint16_t *)b.X, xn, 7 + i);
        launch(100 + i);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(h.data(), b.st, h.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long s0 = ~0ull, s1 = 0;
        double fsum = 0, tsum = 0;
        for (int w = 0; w < nwg; ++w) {
            s0 = std::min(s0, h[4 * w]);
            s1 = std::max(s1, h[4 * w + 1]);
            fsum += (double)h[4 * w + 2];
            tsum += (double)h[4 * w + 3];
        }
        span.push_back((double)(s1 - s0) / 100.0); // us
        first.push_back(fsum / nwg);
        per.push_back(tsum / nwg);
    }
    std::sort(span.begin(), span.end());
    std::sort(first.begin(), first.end());
    std::sort(per.begin(), per.end());
    const double sp = span[span.size() / 2];
    const double bytes_wg = (double)sps * 4 * (((STREAMS & 1) ? A_SLOT : 0)) + (double)sps * (((STREAMS & 2) ? W_SLOT : 0));
    const double ev_us = prewrite ? 0.0 : ev_ms * 1e3 / reps;
    if (bytes_wg == 0) { // consumer-only runs: time per sub-stage
        printf("%-44s grid %4d  sub %3d | span %7.2f us = %6.3f us per sub-stage | event %7.2f us\n", name, nwg, 4 * sps, sp,
               sp / (4 * sps), ev_us);
        fflush(stdout);
        CHECK(hipEventDestroy(e0));
        CHECK(hipEventDestroy(e1));
        return;
    }
    printf("%-44s grid %4d  sub %3d  KB/CU %6.1f | span %7.2f us  %6.1f GB/s/CU | event %7.2f us %6.1f GB/s/CU | "
           "first-landed %6.0f ticks  wg life %7.0f ticks\n",
           name, nwg, 4 * sps, bytes_wg / 1024, sp, bytes_wg / (sp * 1e3), ev_us, ev_us > 0 ? bytes_wg / (ev_us * 1e3) : 0.0,
           first[first.size() / 2], per[per.size() / 2]);
    fflush(stdout);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main()
{
    Buf b;
    b.wbytes = (size_t)1250 << 20;
    CHECK(hipMalloc(&b.W, b.wbytes));
    CHECK(hipMemset(b.W, 0x11, b.wbytes));
    CHECK(hipMalloc(&b.X, (size_t)BN * 16384 * 2));
    touch<<<256, 256>>>((uint16_t *)b.X, (int64_t)BN * 16384, 0);
    CHECK(hipMalloc(&b.st, 4 * 8 * 4096));
    CHECK(hipMalloc(&b.sink, 64));
    CHECK(hipDeviceSynchronize());
    printf("# per-CU ingest probe: one 512-768-thread workgroup per CU; 'span' = first start to last end\n");
    printf("# E. the consumer side alone (no DMA: loaders only keep the barriers), 64 sub-stages\n");
    run<4, 8, 4, 2, 1, 0, 0, 0>("E0 barriers only", b, 32768, 4096, 1, false);
    run<4, 8, 4, 2, 1, 1, 0, 0>("E1 fragment reads (b128 x16 + weights)", b, 32768, 4096, 1, false);
    run<4, 8, 4, 2, 1, 4, 0, 0>("E2 MFMA only", b, 32768, 4096, 1, false);
    run<4, 8, 4, 2, 1, 2, 0, 0>("E3 reads + MFMA", b, 32768, 4096, 1, false);
    run<4, 8, 4, 2, 1, 3, 0, 0>("E4 reads + dequant + MFMA", b, 32768, 4096, 1, false);
    run<4, 8, 4, 2, 1, 5, 0, 0>("E5 = E4, waves 4-7 lag", b, 32768, 4096, 1, false);
    run<4, 4, 4, 2, 1, 3, 0, 0>("E6 = E4, 4 waves x 2 row groups", b, 32768, 4096, 1, false);
    run<4, 4, 4, 2, 1, 2, 0, 0>("E7 = E3, 4 waves x 2 row groups", b, 32768, 4096, 1, false);
    return 0;
}
