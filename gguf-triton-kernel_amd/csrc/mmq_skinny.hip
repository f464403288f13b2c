// mmq_skinny.hip -- MMQ for 5..32 tokens: the weight matrix streamed once, in one launch with no
// split-K partials and no reduce launch, on v_mfma_f32_16x16x32_f16.
//
// C[t][m] = sum_k W[m][k] * x~[t][k] (fp32 accumulate), x~ = fp16(d*q) the q8_1-quantized
// activation (act_quant.hip DEQ form, the integers kernels/cpu_impls multiplies), W dequantized
// to fp16 in registers (gguf_wfrag.hpp).  Replaces, for 5..32 tokens, the reference's Triton
// loops kernels/mmq_q4_k.py:240-289 (and mmq_q8_0.py / mmq_q6_k.py alike).
//
// Shape.  Too few tokens for a GEMM tile to reuse the weights, too many for the decode kernel's
// per-lane int8 dots: the work is a weight stream with a 16- or 32-column MFMA on it.  A
// workgroup owns RG 16-row fragments (16*RG rows, whole K) and NT 16-token column tiles; its 8
// waves are 8/NT contiguous K ranges x NT token tiles (a wave always multiplies one 16-token
// tile: its registers hold one tile's activation fragments; the NT waves of a K range load the
// same weight bytes, the second from the cache).  8/NT independent weight streams per
// workgroup keep bytes in flight; each wave sums its range into 16*RG x 16 fp32 accumulators
// and the ranges' partial tiles are added in LDS at the end (fixed order: deterministic, and a
// row's arithmetic does not depend on which workgroup or launch it lands in).
//
// Per wave, per super-block: the lane's weight bytes straight into registers (WB<F>::load), and
// its token tile's 16 x 256 activations (x~, L2 hits: every workgroup reads all of x~) by
// LDS-DMA into the wave's private LDS ring -- 8 instructions of 1 KiB, two tokens' contiguous
// 512-byte runs each (16-byte loads scattered over 16 token rows ran the texture addresser at
// ~55 cycles per instruction: profiles/r03/skinny_v1_pmc.txt) -- read back as B fragments by
// ds_read_b128 (piece p of token n stored at p ^ n: 16 tokens, 16 distinct bank groups).  A ring
// of D super-blocks holds both; super-block sb + D's weight and activation loads are issued
// together after super-block sb is multiplied, so waiting for the activations never waits for
// younger weight loads (a wave's returns come back in issue order) and the weights keep D - 1
// super-blocks of lead.
//
// MFMA 16x16x32 f16 (gfx950): lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15];
// D[row 4(l>>4)+i][col l&15] in acc element i.  Weight rows are A rows, tokens B columns.
#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_wfrag.hpp"

namespace gq {
namespace {

typedef __attribute__((address_space(3))) void lds_void;

// Diagnostic ablations (-DGQ_SKINNY_ABL in a separate build, never the product): 1 = every
// activation DMA re-reads the wave's first super-block (cache hits: the activation stream
// without its traffic), 2 = every weight load re-reads the first fragment's first super-block,
// 4 = one activation DMA instruction per super-block instead of 8 (garbage results).
#ifndef GQ_SKINNY_ABL
#define GQ_SKINNY_ABL 0
#endif
constexpr int SABL = GQ_SKINNY_ABL;

constexpr int SW = 8;     // waves per workgroup, each a contiguous K range of the workgroup's rows
// compute units: num_cus() (the device attribute, queried once per device)

template <int F> constexpr int w_loads() { return F == Q4_K ? 3 : (F == Q6_K ? 10 : 5); } // per fragment

template <int F, int NT, int RG, int D>
__global__ __launch_bounds__(64 * SW) void skinny_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                         uint16_t *__restrict__ C, int M, int N, int K, int ldc,
                                                         int nunits)
{
    using W = WB<F>;
    constexpr int KR = SW / NT;                                // K ranges
    constexpr int XSLOT = 16 * 512;                            // one super-block of a 16-token tile
    __shared__ __attribute__((aligned(1024))) uint8_t xlds[SW * D * XSLOT];
    __shared__ __attribute__((aligned(16))) float red[SW * RG * 256];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tt = wave % NT, kr = wave / NT; // this wave's token tile and K range
    const int g = lane >> 4, c = lane & 15;
    // this workgroup's contiguous range of units (16*RG rows each)
    const int u0 = (int)((int64_t)blockIdx.x * nunits / gridDim.x);
    const int u1 = (int)((int64_t)(blockIdx.x + 1) * nunits / gridDim.x);
    const int nsb = K / 256;
    const int sb0 = kr * nsb / KR, nsw = (kr + 1) * nsb / KR - sb0; // this wave's super-blocks per unit
    const int row_bytes = (K / Layout<F>::QK) * Layout<F>::BYTES;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, M * row_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, N * K * 2, 0x00020000);
    uint8_t *ring = xlds + wave * (D * XSLOT);
    // DMA instruction i of a slot: tokens 2i, 2i+1; lane l -> token 2i + (l>>5), position q = l&31
    // holding source piece q ^ token (clamped token: past N, garbage that is never stored)
    uint32_t xsrc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int n = 2 * i + (lane >> 5), q = lane & 31;
        const int tok = 16 * tt + n < N ? 16 * tt + n : N - 1;
        xsrc[i] = (uint32_t)tok * (uint32_t)K * 2u + 16u * (uint32_t)(q ^ n);
    }
    f32x4 acc[RG];
#pragma unroll
    for (int rf = 0; rf < RG; ++rf) acc[rf] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // unit u done: the K ranges' partial tiles summed in range order (slot (wave, rf) =
    // ((kr*NT + tt)*RG + rf)) and stored.  Every wave calls it once per unit, in unit order.
    auto finish = [&](int u) __attribute__((always_inline)) {
        const int m0 = u * 16 * RG;
#pragma unroll
        for (int rf = 0; rf < RG; ++rf) {
            *(f32x4 *)(red + (wave * RG + rf) * 256 + 4 * lane) = acc[rf];
            acc[rf] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (int q = tid; q < NT * RG * 64; q += 64 * SW) {
            const int rt = q >> 6, l = q & 63, t = rt / RG, rf = rt % RG; // rt = t*RG + rf: kr = 0's slot
            f32x4 v = *(const f32x4 *)(red + rt * 256 + 4 * l);
#pragma unroll
            for (int k = 1; k < KR; ++k) v += *(const f32x4 *)(red + (k * NT * RG + rt) * 256 + 4 * l);
            const int row = m0 + 16 * rf + 4 * (l >> 4), tok = 16 * t + (l & 15);
            if (row >= M || tok >= N) continue;
            uint16_t *dst = C + (size_t)tok * ldc + row;
            if (row + 4 <= M) {
                *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                        (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)};
            } else {
                for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(v[i]);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); // red may be rewritten
    };

    if (nsw > 0) {
        // the wave's stream: item j = (unit u0 + j / nsw, super-block sb0 + j % nsw), one ring
        // across the unit boundaries (the next unit's first super-blocks load under this one's
        // last); nothing is loaded past the end (a wave often has only 2-4 items: surplus loads
        // would double its activation traffic and hold the wave until they land)
        const int total = (u1 - u0) * nsw;
        W wb[D][RG];
        auto load = [&](int b, int j) __attribute__((always_inline)) {
            const int u = u0 + j / nsw, sb = sb0 + j % nsw;
#pragma unroll
            for (int rf = 0; rf < RG; ++rf) {
                const int row = SABL & 2 ? c : u * 16 * RG + 16 * rf + c;
                wb[b][rf].load(wrs, (uint32_t)((row < M ? row : M - 1) * row_bytes), g,
                               (uint32_t)((SABL & 2 ? sb0 : sb) * W::SB));
            }
            uint8_t *dst = ring + b * XSLOT;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (!(SABL & 4) || i == 0)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void *)(dst + 1024 * i), 16, xsrc[i],
                                                             (uint32_t)(512 * (SABL & 1 ? sb0 : sb)), 0, 0);
        };
        auto compute = [&](int b) __attribute__((always_inline)) {
            const uint8_t *xs = ring + b * XSLOT + c * 512;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const f16x8 bf = *(const f16x8 *)(xs + 16 * ((W::e(s, g) >> 3) ^ c));
#pragma unroll
                for (int rf = 0; rf < RG; ++rf)
                    acc[rf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wb[b][rf].frag(s, g), bf, acc[rf], 0, 0, 0);
            }
        };
        // item j sits in slot j % D; D bodies per loop iteration (static slots), the last < D items
        // after it, so the loop's back edge always follows the same code.  The slot's DMA has
        // landed when at most the younger items' loads are outstanding: D - 1 items', fewer in
        // the last D - 1 (loads return in order; a unit's output stores, issued in between, can
        // only make this wait longer).
        constexpr int PER_SB = RG * w_loads<F>() + 8;
        static_assert((D - 1) * PER_SB <= 63, "vmcnt range");
        // (sched_barrier around the waits: register-only work -- the dequantization -- would
        // otherwise move across them)
        auto body = [&](int j, int b) __attribute__((always_inline)) {
            __builtin_amdgcn_sched_barrier(0);
            const int younger = total - 1 - j < D - 1 ? total - 1 - j : D - 1; // items issued after j
            vm_wait<(D - 1) * PER_SB>(younger * PER_SB);
            __builtin_amdgcn_sched_barrier(0);
            compute(b);
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the slot's reads are done: refill it
            __builtin_amdgcn_sched_barrier(0);
            if (j + D < total) load(b, j + D);
            if ((j + 1) % nsw == 0) finish(u0 + j / nsw);
        };
#pragma unroll
        for (int b = 0; b < D; ++b)
            if (b < total) load(b, b);
        int j = 0;
        for (; j + D - 1 < total; j += D) {
#pragma unroll
            for (int b = 0; b < D; ++b) body(j + b, b);
        }
#pragma unroll
        for (int b = 0; b < D - 1; ++b)
            if (j + b < total) body(j + b, b);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // no DMA may land after the wave is done
    } else {
        for (int u = u0; u < u1; ++u) finish(u); // (K shorter than the ranges: zeros, in step)
    }
}

template <int F, int NT, int RG, int D>
hipError_t launch_cfg(const uint8_t *A, const uint16_t *X, uint16_t *C, int64_t M, int64_t N, int64_t K, int64_t ldc,
                      hipStream_t s)
{
    // persistent: one workgroup per CU (the 128 KiB activation ring fills its LDS), each a
    // contiguous range of units
    const int64_t nunits = (M + 16 * RG - 1) / (16 * RG);
    const unsigned grid = (unsigned)(nunits < num_cus() ? nunits : num_cus());
    skinny_kernel<F, NT, RG, D><<<dim3(grid), dim3(64 * SW), 0, s>>>(A, X, C, (int)M, (int)N, (int)K, (int)ldc,
                                                                     (int)nunits);
    return hipGetLastError();
}

// d = 2 (two 8 KiB activation slots per wave: 128 KiB of LDS); rg = 1..4 fragments per
// workgroup, Q6_K 1..3 (its 4-fragment weight ring spills: kernel-resource-usage)
template <int F> constexpr int rg_max() { return F == Q6_K ? 3 : 4; }
int rg_max_of(int fmt) { return fmt == Q6_K ? 3 : 4; }

template <int F, int NT>
hipError_t launch_nt(const uint8_t *A, const uint16_t *X, uint16_t *C, const SkinnyPlan &p, int64_t M, int64_t N,
                     int64_t K, int64_t ldc, hipStream_t s)
{
    if constexpr (rg_max<F>() >= 4)
        if (p.rg >= 4) return launch_cfg<F, NT, 4, 2>(A, X, C, M, N, K, ldc, s);
    switch (p.rg) {
    case 4:
    case 3: return launch_cfg<F, NT, 3, 2>(A, X, C, M, N, K, ldc, s);
    case 2: return launch_cfg<F, NT, 2, 2>(A, X, C, M, N, K, ldc, s);
    default: return launch_cfg<F, NT, 1, 2>(A, X, C, M, N, K, ldc, s);
    }
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const uint16_t *X, uint16_t *C, const SkinnyPlan &p, int64_t M, int64_t N,
                      int64_t K, int64_t ldc, hipStream_t s)
{
    if (p.nb == 1) return launch_nt<F, 1>(A, X, C, p, M, N, K, ldc, s);
    return launch_nt<F, 2>(A, X, C, p, M, N, K, ldc, s);
}

} // namespace

SkinnyPlan plan_skinny(int fmt, int64_t M, int64_t N, int64_t K, int rg, int d)
{
    (void)d;
    SkinnyPlan p;
    p.nb = N <= 16 ? 1 : 2;
    p.d = 2;
    // A unit (16*rg rows) reads all of x~ (N x K fp16): at 16 tokens 2-4x one fragment's weight
    // bytes, so more rows per unit cut the x~ traffic (L2), while the persistent grid's busiest
    // workgroup takes ceil(units / 256) units.  Cost of that workgroup in fragment-streams:
    // ceil(units / 256) * (rg + xr), xr = x~ bytes per fragment's weight bytes, counted at half
    // (L2 serves a CU about twice as fast as its share of HBM); the cheapest rg.  A row's
    // arithmetic is the same for every rg.
    const int64_t frags = (M + 15) / 16;
    const int rmax = rg_max_of(fmt);
    const int64_t row_bytes = fmt == Q8_0 ? K / 32 * 34 : (fmt == Q4_K ? K / 256 * 144 : K / 256 * 210);
    const double xr = 0.5 * (double)(N * K * 2) / (double)(16 * row_bytes);
    double best = 1e300;
    for (int r = 1; r <= rmax; ++r) {
        const int64_t units = (frags + r - 1) / r;
        const double cost = (double)((units + num_cus() - 1) / num_cus()) * (r + xr);
        if (cost < best - 1e-9) {
            best = cost;
            p.rg = r;
        }
    }
    if (rg) p.rg = rg < 1 ? 1 : (rg > rmax ? rmax : rg);
    return p;
}

hipError_t launch_skinny(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, const SkinnyPlan &plan, int64_t M,
                         int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (N < 1 || N > 32 || K % 256 != 0 || M < 1) return hipErrorInvalidValue;
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, X, C, plan, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, X, C, plan, M, N, K, ldc, s);
    default: return launch_fmt<Q6_K>(A, X, C, plan, M, N, K, ldc, s);
    }
}

} // namespace gq
