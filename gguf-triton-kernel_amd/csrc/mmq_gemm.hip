// mmq_gemm.hip -- batched MMQ (many tokens) on the matrix cores, LDS-DMA staged.
//
// C[t][m] = sum_k W[m][k] * x~[t][k]: W dequantized in registers from the packed GGUF bytes,
// x~ = fp16(d*q) the q8_1-quantized activation (act_quant.hip, DEQ form) -- the integer
// activations kernels/cpu_impls multiplies (mmq_*_q8_1_cpu.py) -- into
// v_mfma_f32_16x16x32_f16 with fp32 accumulation.  fp16 rather than bf16: the reference's
// activations are fp16 and bf16 would drop three of their mantissa bits.
//
// Activation forms (template AM, gguf_internal.hpp ActForm):
//   AF_F16: x~ = fp16(d*q), the q8_1 activation dequantized (act_quant DEQ form);
//   AF_I8 (Q8_0 only): the q8_1 codes and the weight codes go into v_mfma_i32_16x16x32_i8 as
//          they are (one 32-element block = one MFMA k-step, the reference's int dot,
//          mmq_q8_0.py:85-88) and every block's int32 tile is scaled by dA[row]*dB[token] into
//          the fp32 accumulators: no weight dequantization, half the activation bytes;
// AF_I8 stages per token and sub-stage 64 code bytes, and the tile's per-block fp32 d from a
// block-major [K/32][ldd] array.  (The fp8 activation variant arrives as AF_F16: act_quant's
// F8DEQ form widens its e4m3 codes to fp16 x~ once; widening them here per fragment -- round 2's
// AF_F8 form -- cost 12-55% more than the q8_1 path and was removed.)
//
// Workgroup = 8 waves = BM = 128*RG weight rows x BN = 16*NB tokens.  Wave w owns rows
// 16*(RG*w + rg) + [0,16) (rg < RG) and every token of the tile: each weight is dequantized
// once per workgroup; the activation tile is shared through LDS.  Large BM matters: every
// stage moves 2*BN bytes of activations per K element beside BM*bytes/weight of weights, and
// the per-CU L2->LDS rate, not the MFMA, is what a small tile runs into.
//
// K advances in activation sub-stages of 64 elements (2 MFMA k-steps of 32) and weight stages
// of one super-block (256 elements, Q8_0: 8 blocks).  Everything is moved HBM/L2 -> LDS by
// LDS-DMA (global_load_lds_dwordx4: no VGPRs, no ds_write):
//   weights     : per row the stage's raw block bytes (WStage<F> below), 16-byte pieces at
//                 whatever (2-byte) alignment the blocks have (gfx950 runs unaligned);
//   activations : BN token rows x 128 B (AF_I8: x 64 B of codes + the tile's scales), 16-byte pieces
//                 XOR-swizzled on the SOURCE side (the DMA destination is lane-linear) so the
//                 MFMA fragment reads of a lane group hit distinct banks.
// Two weight-stage slots and an activation ring of up to 4 slots (Cfg below) keep the next
// sub-stages in flight while one is multiplied; one s_barrier per sub-stage, preceded by a
// counted vmcnt (never vmcnt(0) inside the loop).  The DMAs are issued either by every wave
// (NL = 0) or by NL = 4 extra loader waves that multiply nothing (the fp16 form's default:
// the multiplying waves then never stall on vector-memory issue).
//
// MFMA 16x16x32 (f16 and i8) maps (gfx950): lane l holds A[row l&15][k 8(l>>4)+j] and
// B[k 8(l>>4)+j][col l&15]; D[row 4(l>>4)+i][col l&15] in acc element i.  Weight rows are the
// A rows and tokens the B columns, so lane l ends with 4 consecutive weight rows of one token:
// one 8-byte store per (row group, token group) in the epilogue.
// The 8 k of an f16 fragment are taken in the element order (0,2,1,3,4,6,5,7) in which packed
// dequantization produces them; act_quant's DEQ form stores x~ in the same order.
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_q8_1.hpp"
#include "gguf_mfma.hpp"

namespace gq {

#ifdef GQ_GEMM_STAMPS // diagnostic build: per-wave s_memtime breakdown (never the product)
__device__ unsigned long long g_gstamps[65536][8];
#endif

namespace {

constexpr int LDS_MAX = 160 * 1024;


// multiplying waves per workgroup: 8 = 512 threads, two waves per SIMD (4 waves x two row
// groups was measured slower and removed: DESIGN.md 5)
constexpr int NWAVE = 8;
constexpr int R1 = 1; // row groups per wave of a 128-row tile

// AQ (in-kernel activation quantization, 16- and 32-token tiles): the loader waves q8_1-quantize
// the tile's fp16 activations for the whole split into LDS (every sub-stage resident, AQ_SUB at
// most), so the call needs no act_quant launch and no activation DMA.
#ifndef GQ_GEMM_AQ_SUB
#define GQ_GEMM_AQ_SUB 24
#endif
template <int NB> constexpr int aq_sub() { return NB == 1 ? GQ_GEMM_AQ_SUB : (NB == 2 ? GQ_GEMM_AQ_SUB / 2 : 8); }
int aq_sub_of(int nb) { return nb == 1 ? GQ_GEMM_AQ_SUB : (nb == 2 ? GQ_GEMM_AQ_SUB / 2 : (nb == 4 ? 8 : 0)); }

template <int F, int NB, int RG = 1, int AM = AF_F16, int NL = 0, int AQ = 0>
struct Cfg {
    // 128*RG weight rows x 16*NB tokens; wave w owns rows 16*(RG*w + rg) + [0, 16), rg < RG.
    // NL > 0: NL more waves that only issue the DMAs (loader waves); 0: every wave issues its share
    static constexpr int BN = 16 * NB, BM = 16 * NWAVE * RG;
    static constexpr int ISSUERS = NL > 0 ? NL : NWAVE, THREADS = 64 * (NWAVE + NL);
    // Q6_K 256-row tiles: 224-B row images (14 pieces, no repeated d piece) so that two weight
    // slots and three activation slots fit the 160 KiB; rows 8..15 of every 16 store their
    // pieces pairwise swapped (LDS byte offset ^ 16), which keeps the 56-dword row stride's
    // rows l and l+8 of a fragment read on distinct banks
    static constexpr bool Q6S = F == Q6_K && RG == 2;
    static constexpr int RBW = Q6S ? 224 : WStage<F>::RBW, NPW = RBW / 16, SPW = WStage<F>::SPW;
    static constexpr int W_REAL = BM * NPW / 64;                              // DMA instructions per stage
    // code-form (AF_I8) activation sub-stage: BN x 64 code bytes (CI instructions), then
    // one instruction for the tile's scales of the sub-stage's two blocks (2 x BN floats)
    static constexpr bool CODES = AM != AF_F16;
    static constexpr int CI = BN * 64 / 1024 > 0 ? BN * 64 / 1024 : 1;
    static constexpr int A_REAL = CODES ? CI + 1 : (BN * 8 / 64 > 0 ? BN * 8 / 64 : 1);
    static constexpr int D_OFF = CI * 1024; // code forms: byte offset of the scales in a slot
    static constexpr int NW = (W_REAL + ISSUERS - 1) / ISSUERS, NA = (A_REAL + ISSUERS - 1) / ISSUERS; // per issuer
    static constexpr int W_SLOT = W_REAL * 1024, A_SLOT = A_REAL * 1024;
    // activation sub-stage ring: as deep as the LDS allows, at most 4*NWS-4 slots (W(w) must
    // be issued before A(4w): see the pipeline note below) and GQ_GEMM_NAS_CAP.  Two weight
    // slots (one super-block ahead): at kernel start every workgroup's prologue DMAs are issued
    // together, and a smaller burst lands the first sub-stage sooner (three slots measured
    // 6-9% slower on every K-quant shape; tools/gemm_stamps.py)
#ifndef GQ_GEMM_SMALL_NWS // weight-stage slots for 16- and 32-token tiles (latency-bound: deeper rings)
#define GQ_GEMM_SMALL_NWS 2
#endif
#ifndef GQ_GEMM_SMALL_NAS_CAP
#define GQ_GEMM_SMALL_NAS_CAP 4
#endif
#ifndef GQ_GEMM_NWS // weight-stage slots for 64- and 128-token tiles
#define GQ_GEMM_NWS 2
#endif
#ifndef GQ_GEMM_FINE_NWS // weight-stage slots with one-sub-stage weight stages
#define GQ_GEMM_FINE_NWS 5
#endif
    static constexpr int NWS = SPW == 1 ? GQ_GEMM_FINE_NWS : (NB <= 2 ? GQ_GEMM_SMALL_NWS : GQ_GEMM_NWS);
    // padding DMAs (instruction counts not a multiple of the wave count) land in a scratch KiB
    static constexpr bool PAD = W_REAL % ISSUERS != 0 || A_REAL % ISSUERS != 0;
    static constexpr int NAS_FIT = (LDS_MAX - (PAD ? 1024 : 0) - NWS * W_SLOT) / A_SLOT;
#ifndef GQ_GEMM_NAS_CAP // activation ring depth cap: 4 measured best (Q4_K 4096^2 x128: 6 slots
#define GQ_GEMM_NAS_CAP 4  // 19.6 us, 4 slots 18.8, 3 slots 19.4; Q6_K x128: 3 slots +15%)
#endif
    static constexpr int NAS_CAP = NB <= 2 ? GQ_GEMM_SMALL_NAS_CAP : GQ_GEMM_NAS_CAP;
    static constexpr int NAS_MAX = SPW * (NWS - 1) < NAS_CAP ? SPW * (NWS - 1) : NAS_CAP;
    static constexpr int NAS = AQ ? aq_sub<NB>() : (NAS_FIT < NAS_MAX ? NAS_FIT : NAS_MAX);
    static constexpr int A_BASE = NWS * W_SLOT, SCRATCH = A_BASE + NAS * A_SLOT; // dummy DMAs land there
    static constexpr int LDS_BYTES = SCRATCH + (PAD ? 1024 : 0);
    static_assert((BM * NPW % 64 == 0 && (BN * 8) % 64 == 0) || BN * 8 < 64, "whole DMA instructions");
    static_assert(AM != AF_I8 || (F == Q8_0 && RG == 1), "int8 form: Q8_0, 128-row tiles");
    static_assert(!CODES || BN <= 128, "code forms: <= 128 tokens per tile");
    static_assert(LDS_BYTES <= LDS_MAX, "LDS budget");
    static_assert(NAS >= 3, "activation ring depth");
    static_assert(!AQ || (NB <= 4 && NL > 0 && RG == R1 && AM == AF_F16), "in-kernel quantization: small tiles, loaders");
    static_assert(AQ || (NAS - 2) * NA + ((NAS - 1 + SPW - 1) / SPW) * NW <= 63, "vmcnt range");
};


// Source of the padding DMAs that keep every wave's instruction count equal: the tensor's first
// bytes (an L2 hit), written to a scratch slot.  (Out-of-range buffer offsets would return
// zeros without a memory access, but they were measured to stall the issuing wave's vmcnt.)
constexpr uint32_t DUMMY = 0u;

// ---------------------------------------------------------------------------------------
// Pipeline (per wave; a = activation sub-stage, w = a / SPW = weight stage, NAS activation
// slots, NWS weight slots):
//   prologue  W(0) .. W(NWS-2) A(0) .. A(NAS-2)
//   iteration a: wait until A(a) (and so W(a/SPW)) landed -> barrier -> A(a+NAS-1) ->
//                [a%SPW == 0: W(w+NWS-1)] -> multiply sub-stage a from W slot w%NWS, A slot a%NAS.
// vmcnt counts in issue order, so "A(a) landed" = all but the ops issued after it: the (up to)
// NAS-2 younger activation sub-stages and the W(.) issued in iterations a-NAS+1 .. a-1 with
// index % SPW == 0 (after their A).  W(w) is issued in iteration SPW(w-NWS+1), after
// A(SPW(w-NWS+1)+NAS-1), which is older than A(SPW w) iff NAS <= SPW(NWS-1).  Nothing is
// issued past the split's end (a split is often 2-8 weight stages: clamped re-loads there were
// up to 40% more L2->LDS traffic), so the last NAS-1 waits count fewer younger ops (vm_wait).
// ABL: ablation bitmask for performance diagnosis (diagnostic build -DGQ_ABLATION only; 0 in
// production): 1 = no MFMA, 2 = no weight DMA, 4 = no activation DMA, 8 = no dequantization,
// 16 = no epilogue, 32 = activation DMAs with the addresses of a sub-stage-blocked layout,
// 64 = weight DMAs with the addresses of a stage-contiguous (tiled) layout, 128 = a quarter of
// the activation fragment reads.
// AF_I8: X = codes [N][K], XD = block-major scales [K/32][ldd]; AF_F16: X = fp16 x~.
template <int F, int NB, int RG, int ABL = 0, int AM = AF_F16, int NL = 0, int AQ = 0>
__global__ __launch_bounds__(64 * (NWAVE + NL)) void gemm_kernel(const uint8_t *__restrict__ A, const void *__restrict__ X,
                                                   const float *__restrict__ XD, uint16_t *__restrict__ C,
                                                   float *__restrict__ P, int64_t M, int64_t N, int64_t K,
                                                   int64_t ldc, int64_t ldd, int wstages_per_split, int pf16)
{
    using G = Cfg<F, NB, RG, AM, NL, AQ>;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[G::LDS_BYTES];
#ifdef GQ_GEMM_STAMPS
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    unsigned long long t_first = 0, t_wait = 0, t_loop = 0, t_issued = 0;
#endif

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // DMA issuer index: loader waves NWAVE.. (NL > 0), else every wave
    const bool loader = NL > 0 && wave >= NWAVE;
    const int iw = NL > 0 ? wave - NWAVE : wave;
    const int g = lane >> 4, l16 = lane & 15;
    const int64_t m0 = (int64_t)blockIdx.x * G::BM;
    const int64_t n0 = (int64_t)blockIdx.y * G::BN;
    // the split's super-blocks [sb0, sb1) = sub-stages [a0, a1) = weight stages [w0, w1)
    const int64_t nsb = K / 256;
    const int64_t sb0 = (int64_t)blockIdx.z * wstages_per_split;
    const int64_t sb1 = sb0 + wstages_per_split < nsb ? sb0 + wstages_per_split : nsb;
    constexpr int SPW = G::SPW;
    const int64_t w0 = 4 * sb0 / SPW, w1 = 4 * sb1 / SPW;
    const int64_t row_bytes = (K / Layout<F>::QK) * Layout<F>::BYTES;

    // buffer descriptors (byte offsets are 32-bit: tensors < 4 GiB, checked on the host).  The
    // range check zeroes a whole 16-byte piece that crosses num_records, so the weight range is
    // rounded up to 16 B: a Q6_K window's last piece may run past the tensor's last byte, but
    // never past the 16-byte granule (hence never the page) that byte lives in.
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, (int)(uint32_t)((M * row_bytes + 15) & ~(int64_t)15), 0x00020000);
    const __amdgpu_buffer_rsrc_t ars =
        __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, (int)(uint32_t)(AQ ? ((N - 1) * ldd + K) * 2 : N * K * (G::CODES ? 1 : 2)), 0x00020000);
    // code forms: scales [K/32][ldd] from XD (this launch's first token), the last block's run
    // holding this launch's N tokens
    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)XD, 0, G::CODES ? (int)(uint32_t)(((K / 32 - 1) * ldd + N) * 4) : 0, 0x00020000);

    // weight DMA: instruction k = wave + 8i moves pieces p = 64k + lane: row p / NPW, piece p % NPW
    uint32_t wv[G::NW];
    int wpc[G::NW];
#pragma unroll
    for (int i = 0; i < G::NW; ++i) {
        const int p = 64 * (iw + G::ISSUERS * i) + lane, r = p / G::NPW;
        wpc[i] = (p - r * G::NPW) ^ (G::Q6S ? (r >> 3) & 1 : 0); // the piece that lands at this lane's slot
        const int64_t row = m0 + r < M ? m0 + r : M - 1;
        wv[i] = r < G::BM ? (uint32_t)(row * row_bytes) : DUMMY;
    }
    // activation DMA: instruction k moves pieces p = 64k + lane: token p >> 3, slot p & 7.
    // Code forms: instructions k < CI move pieces p: token p >> 2, piece p & 3 (swizzle i8_swz;
    // Q6_K: pieces 2, 3 are the second 32-element run, 64 elements on); instruction CI moves the
    // scales of the sub-stage's two blocks: lanes [0, BN/4) block 0, the next BN/4 block 1,
    // four tokens per lane.
    uint32_t av[G::NA];
#pragma unroll
    for (int i = 0; i < G::NA; ++i) {
        const int k = iw + G::ISSUERS * i, p = 64 * k + lane;
        if constexpr (G::CODES) {
            if (k < G::CI) {
                const int r = p >> 2, q = p & 3, qs = q ^ i8_swz(r);
                const int64_t tok = n0 + r < N ? n0 + r : N - 1;
                const uint32_t po = F == Q6_K ? 64u * (uint32_t)(qs >> 1) + 16u * (uint32_t)(qs & 1) : 16u * (uint32_t)qs;
                av[i] = r < G::BN ? (uint32_t)(tok * K) + po : DUMMY;
            } else {
                const int b = lane / (G::BN / 4), j = lane - b * (G::BN / 4);
                const int64_t bstride = F == Q6_K ? 2 : 1; // Q6_K: blocks e0/32 and e0/32 + 2
                av[i] = k == G::CI && b < 2 ? (uint32_t)((b * bstride * ldd + n0 + 4 * j) * 4) : DUMMY;
            }
        } else {
            const int r = p >> 3, q = p & 7;
            const int64_t tok = n0 + r < N ? n0 + r : N - 1;
            if constexpr ((ABL & 32) != 0) // diagnostic: the access pattern of a sub-stage-blocked layout
                av[i] = r < G::BN ? (uint32_t)(tok * 128) + 16u * (q ^ act_swz(r)) : DUMMY;
            else
                av[i] = r < G::BN ? (uint32_t)(tok * K * 2) + act_voff<F>(q ^ act_swz(r)) : DUMMY;
        }
    }
    const int myrow = 16 * RG * wave + l16; // the row this lane multiplies (row group 0)

    auto issue_w = [&](int64_t w) {
        if constexpr (ABL & 2) return;
        uint8_t *dst = lds + (int)(w % G::NWS) * G::W_SLOT;
#pragma unroll
        for (int i = 0; i < G::NW; ++i) {
            const int k = iw + G::ISSUERS * i;
            uint32_t vo, so;
            if constexpr ((ABL & 64) != 0) { // diagnostic: the stage as one contiguous run (a tiled layout)
                vo = (uint32_t)(m0 * row_bytes) + 16u * (uint32_t)(64 * k + lane);
                so = (uint32_t)(w * G::BM * G::RBW);
            } else if constexpr (F == Q6_K) { // super-block image: pieces +16i (i < 13) and +194 (d at 222)
                vo = wv[i] + (uint32_t)WStage<F>::SB * (uint32_t)w + (wpc[i] < 13 ? 16u * wpc[i] : 194u); // piece 14 = 13 again
                so = 0;
            } else if constexpr (F == Q8_0 && SPW == 1) { // 5 pieces from the stage's first byte (4-byte aligned)
                vo = wv[i] + 68u * (uint32_t)w + 16u * wpc[i];
                so = 0;
            } else {
                vo = wv[i] + 16u * wpc[i];
                so = (uint32_t)(WStage<F>::SB * w);
            }
            dma16(wrs, k < G::W_REAL ? dst + 1024 * k : lds + G::SCRATCH, vo, so);
        }
    };
    auto issue_a = [&](int64_t a) {
        if constexpr (ABL & 4) return;
        uint8_t *dst = lds + G::A_BASE + (int)(a % G::NAS) * G::A_SLOT;
#pragma unroll
        for (int i = 0; i < G::NA; ++i) {
            const int k = iw + G::ISSUERS * i;
            uint8_t *d = k < G::A_REAL ? dst + 1024 * k : lds + G::SCRATCH;
            if constexpr (G::CODES) {
                const uint32_t e0 = act_soff<F>(a) / 2; // first element of the sub-stage
                if (k < G::CI) dma16(ars, d, av[i], e0);
                else dma16(drs, d, av[i], (uint32_t)((e0 / 32) * ldd * 4)); // scales of its two blocks
            } else if constexpr ((ABL & 32) != 0) {
                dma16(ars, d, av[i], (uint32_t)(a * N * 128));
            } else {
                dma16(ars, d, av[i], act_soff<F>(a));
            }
        }
    };
    // vmcnt for "A(a) landed": the DMA instructions issued after A(a) -- the younger A's
    // (sub-stages a+1 .. a+NAS-2) and the W's issued in iterations a-NAS+1 .. a-1 (each after its
    // iteration's A), nothing past the split's end (nrel sub-stages, nws weight stages)
    auto wait_a = [&](int rel, int nrel, int nws) __attribute__((always_inline)) {
        constexpr int na = ABL & 4 ? 0 : G::NA, nw = ABL & 2 ? 0 : G::NW; // (ablated streams issue nothing)
        const int ya = G::NAS - 2 < nrel - 1 - rel ? G::NAS - 2 : nrel - 1 - rel;
        const int lo = rel - G::NAS + 1 > 0 ? rel - G::NAS + 1 : 0;
        const int hi = rel - 1 < SPW * (nws - G::NWS + 1) - 1 ? rel - 1 : SPW * (nws - G::NWS + 1) - 1;
        const int w_after = hi >= lo ? hi / SPW - (lo + SPW - 1) / SPW + 1 : 0;
        if constexpr ((ABL & 6) == 6) {
        } else if constexpr (ABL & 4) { // weights only: W(w) must land by sub-stage SPW w
            const int w = rel / SPW, yw = G::NWS - 2 < nws - 1 - w ? G::NWS - 2 : nws - 1 - w;
            if (rel % SPW == 0) vm_wait<(G::NWS - 2) * nw>(yw * nw);
        } else {
            vm_wait<(G::NAS - 2) * na + ((G::NAS - 1 + SPW - 1) / SPW) * nw>(ya * na + w_after * nw);
        }
        asm volatile("s_barrier" ::: "memory");
    };
    static_assert(AQ || (G::NAS - 1 + SPW - 1) / SPW <= 4, "W issues after an A: at most 4");

    f32x4 acc[RG][NB];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[rg][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

#ifdef GQ_GEMM_STAMPS
    const unsigned long long t_setup = __builtin_amdgcn_s_memtime() - t_start;
#endif
    if (AQ && loader) { // weights by DMA; the split's activations quantized straight into LDS
        if (w0 < w1) {
            const int64_t a0 = 4 * sb0, a1 = 4 * sb1;
#pragma unroll
            for (int i = 0; i < G::NWS - 1; ++i)
                if (w0 + i < w1) issue_w(w0 + i);
            // 4 lanes per 32-element block (8 fp16 each), 64 blocks per pass over the 4 loader
            // waves; loads unconditional (clamped) and all issued before the first quantization
            constexpr int PMAX = (G::NAS * G::BN * 2 + 63) / 64;
            const int nbk = 2 * (int)(a1 - a0), nblk = G::BN * nbk;
            const __amdgpu_buffer_rsrc_t xr = ars; // raw fp16 activations [N][ldd]
            u32x4 xv[PMAX];
#pragma unroll
            for (int q = 0; q < PMAX; ++q) {
                int b = 64 * q + 16 * iw + (lane >> 2);
                if (b >= nblk) b = 0;
                const int r = b / nbk, kb = b - r * nbk;
                const int64_t tok = n0 + r < N ? n0 + r : N - 1;
                const uint32_t k = (uint32_t)(64 * a0 + 32 * kb + 8 * (lane & 3));
                xv[q] = __builtin_amdgcn_raw_buffer_load_b128(xr, (uint32_t)(tok * ldd) * 2u + 2u * k, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < PMAX; ++q) {
                const Q81Quad qq = q8_1_quad(xv[q]); // every lane: DPP quad groups
                const int b = 64 * q + 16 * iw + (lane >> 2);
                if (b < nblk) {
                    const int r = b / nbk, kb = b - r * nbk;
                    const int k = 32 * kb + 8 * (lane & 3); // element offset from 64 * a0
                    // x~ = fp16(d*q), 4-groups stored (0,2,1,3) as act_quant's DEQ form
                    uint32_t o[4];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        float v4[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) v4[i] = qq.d * (float)(int8_t)((qq.codes[h] >> (8 * i)) & 0xff);
                        o[2 * h] = (uint32_t)f2h_bits(v4[0]) | ((uint32_t)f2h_bits(v4[2]) << 16);
                        o[2 * h + 1] = (uint32_t)f2h_bits(v4[1]) | ((uint32_t)f2h_bits(v4[3]) << 16);
                    }
                    // where the GEMM's fragment reads expect these 8 elements: sub-stage a (its
                    // region a - a0), piece j of the 8 (Q6_K: the permuted run order of act_soff)
                    int ar, j;
                    if constexpr (F == Q6_K) {
                        const int sbk = k >> 8, wsb = k & 255, h = wsb >> 7, n = (wsb >> 6) & 1, v = (wsb >> 5) & 1;
                        ar = 4 * sbk + 2 * h + v;
                        j = 4 * n + ((wsb >> 3) & 3);
                    } else {
                        ar = k >> 6;
                        j = (k & 63) >> 3;
                    }
                    *(u32x4 *)(lds + G::A_BASE + ar * G::A_SLOT + 128 * r + 16 * (j ^ act_swz(r))) =
                        (u32x4){o[0], o[1], o[2], o[3]};
                }
            }
#pragma unroll
            for (int q = 0; q < PMAX; ++q) asm volatile("" ::"v"(xv[q].x), "v"(xv[q].y), "v"(xv[q].z), "v"(xv[q].w));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the image is complete before barrier a0
            for (int64_t a = a0; a < a1; ++a) {
                if ((a & 3) == 0) { // W(w) landed = all but the (<= NWS-2) stages issued after it
                    const int64_t w = a >> 2;
                    const int yw = (int)(G::NWS - 2 < w1 - 1 - w ? G::NWS - 2 : w1 - 1 - w);
                    vm_wait<(G::NWS - 2) * G::NW>(yw * G::NW);
                    asm volatile("s_barrier" ::: "memory");
                    if (w + G::NWS - 1 < w1) issue_w(w + G::NWS - 1);
                } else {
                    asm volatile("s_barrier" ::: "memory");
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        return;
    }
    if (!AQ && loader) { // loader waves: the DMA schedule of the pipeline note, no multiply
        if (w0 < w1) {
            const int64_t a0 = 4 * sb0, a1 = 4 * sb1;
#pragma unroll
            for (int i = 0; i < G::NWS - 1; ++i)
                if (w0 + i < w1) issue_w(w0 + i);
#pragma unroll
            for (int i = 0; i < G::NAS - 1; ++i)
                if (a0 + i < a1) issue_a(a0 + i);
            for (int64_t a = a0; a < a1; ++a) {
                // A(a) landed -> barrier: the compute waves take sub-stage a
                wait_a((int)(a - a0), (int)(a1 - a0), (int)(w1 - w0));
                if (a + G::NAS - 1 < a1) issue_a(a + G::NAS - 1);
                if (a % SPW == 0 && a / SPW + G::NWS - 1 < w1) issue_w(a / SPW + G::NWS - 1);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        return;
    }
    if (w0 < w1) {
        const int64_t a0 = 4 * sb0, a1 = 4 * sb1;
#pragma unroll
        for (int i = 0; i < G::NWS - 1 && NL == 0; ++i)
            if (w0 + i < w1) issue_w(w0 + i);
#pragma unroll
        for (int i = 0; i < G::NAS - 1 && NL == 0; ++i)
            if (a0 + i < a1) issue_a(a0 + i);
#ifdef GQ_GEMM_STAMPS
        t_issued = __builtin_amdgcn_s_memtime() - t_start;
#endif
        for (int64_t a = a0; a < a1; ++a) {
            const int s4 = (int)(a % SPW); // sub-stage within the weight stage
#ifdef GQ_GEMM_STAMPS
            const unsigned long long tw = __builtin_amdgcn_s_memtime();
#endif
            if constexpr (NL > 0) asm volatile("s_barrier" ::: "memory"); // the loaders' wait_a
            else wait_a((int)(a - a0), (int)(a1 - a0), (int)(w1 - w0));
#ifdef GQ_GEMM_STAMPS
            {
                const unsigned long long tn = __builtin_amdgcn_s_memtime();
                if (a == a0) t_first = tn - t_start;
                else t_wait += tn - tw;
            }
#endif
            const int64_t w = a / SPW;
            if constexpr (NL == 0) {
                if (a + G::NAS - 1 < a1) issue_a(a + G::NAS - 1);
                if (s4 == 0 && w + G::NWS - 1 < w1) issue_w(w + G::NWS - 1);
            }

            const uint8_t *wr = lds + (int)(w % G::NWS) * G::W_SLOT + G::RBW * myrow;
            const uint8_t *xs = lds + G::A_BASE + (int)(AQ ? a - a0 : a % G::NAS) * G::A_SLOT;
            if constexpr (AM == AF_I8) {
                // int8 form: per block b of the sub-stage one i8 MFMA per token tile, the int32
                // tile scaled by dA[row] * dB[token] into the fp32 accumulators
                const uint8_t *wq = wr - G::RBW * l16 + G::RBW * 4 * g; // row 16*wave + 4g (+i)
                long aq[2], bq[2][NB];
                float da[2][4], db[2][NB];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const int boff = 34 * (2 * s4 + b);
                    aq[b] = __builtin_bit_cast(long, *(const u32x2 *)(wr + boff + 2 + 8 * g));
#pragma unroll
                    for (int i = 0; i < 4; ++i) da[b][i] = h2f(*(const uint16_t *)(wq + G::RBW * i + boff));
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        const int r = 16 * t + l16;
                        bq[b][t] = __builtin_bit_cast(
                            long, *(const u32x2 *)(xs + 64 * r + 16 * ((2 * b + (g >> 1)) ^ i8_swz(r)) + 8 * (g & 1)));
                        db[b][t] = *(const float *)(xs + G::D_OFF + 4 * (G::BN * b + r));
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        const i32x4 pi = __builtin_amdgcn_mfma_i32_16x16x32_i8(aq[b], bq[b][t], (i32x4){0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
                        for (int i = 0; i < 4; ++i) acc[0][t][i] = __builtin_fmaf((float)pi[i], da[b][i] * db[b][t], acc[0][t][i]);
                    }
                continue;
            }
            if constexpr (RG == 2 && AM == AF_F16 && (ABL & (8 | 128)) == 0) {
                // 256-row tiles (12 waves: at most 168 VGPRs a wave): the weight fragments of both
                // row groups, then per k-step its 8 activation fragments and 16 MFMAs -- holding the
                // whole sub-stage's activation fragments as below spilled 82-114 VGPRs
                f16x8 af[RG][2];
#pragma unroll
                for (int rg = 0; rg < RG; ++rg)
                    stage_frags<F>(wr + 16 * G::RBW * rg, g, s4, af[rg], G::Q6S ? ((l16 >> 3) & 1) << 4 : 0);
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    f16x8 bk[NB];
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        const int r = 16 * t + l16;
                        bk[t] = *(const f16x8 *)(xs + 128 * r + 16 * ((4 * s + g) ^ act_swz(r)));
                    }
#pragma unroll
                    for (int rg = 0; rg < RG; ++rg)
#pragma unroll
                        for (int t = 0; t < NB; ++t) {
                            if constexpr (ABL & 1) acc[rg][t][0] += (float)af[rg][s][t & 7] * (float)bk[t][0];
                            else acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[rg][s], bk[t], acc[rg][t], 0, 0, 0);
                        }
                }
                continue;
            }
            // all of the sub-stage's activation fragments first (one LDS round trip), the
            // dequantization beside them, then the MFMAs
            f16x8 bfr[2][NB];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const int r = 16 * t + l16;
                    if constexpr ((ABL & 128) != 0) { // diagnostic: a quarter of the fragment reads
                        bfr[s][t] = t < NB / 4 || NB < 4 ? *(const f16x8 *)(xs + 128 * r + 16 * ((4 * s + g) ^ act_swz(r)))
                                                         : bfr[s][t % (NB / 4)];
                    } else {
                        bfr[s][t] = *(const f16x8 *)(xs + 128 * r + 16 * ((4 * s + g) ^ act_swz(r)));
                    }
                }
            f16x8 af[RG][2];
#pragma unroll
            for (int rg = 0; rg < RG; ++rg) {
                const uint8_t *wrg = wr + 16 * G::RBW * rg;
                if constexpr (ABL & 8) {
                    af[rg][0] = *(const f16x8 *)(wrg + 0);
                    af[rg][1] = *(const f16x8 *)(wrg + 16);
                } else {
                    stage_frags<F>(wrg, g, s4, af[rg], G::Q6S ? ((l16 >> 3) & 1) << 4 : 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < 2; ++s) {
#pragma unroll
                for (int rg = 0; rg < RG; ++rg)
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        if constexpr (ABL & 1) acc[rg][t][0] += (float)af[rg][s][t & 7] * (float)bfr[s][t][0];
                        else
                            acc[rg][t] =
                                __builtin_amdgcn_mfma_f32_16x16x32_f16(af[rg][s], bfr[s][t], acc[rg][t], 0, 0, 0);
                    }
            }
        }
        if constexpr (NL == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // no DMA may land after the workgroup exits
    }
#ifdef GQ_GEMM_STAMPS
    t_loop = __builtin_amdgcn_s_memtime() - t_start;
    auto stamp_out = [&]() {
        const int64_t wg = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        const int64_t id = wg * NWAVE + wave;
        if (lane == 0 && id < 65536) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            g_gstamps[id][0] = t_first;
            g_gstamps[id][1] = t_wait;
            g_gstamps[id][2] = t_loop;
            g_gstamps[id][3] = __builtin_amdgcn_s_memtime() - t_start;
            g_gstamps[id][4] = (unsigned long long)(sb1 - sb0) * 4;
            g_gstamps[id][5] = 1 + t_setup;
            g_gstamps[id][6] = t_start;
            g_gstamps[id][7] = t_issued;
        }
    };
#endif

    // epilogue: acc[rg][t][i] = D[row 16*(RG*wave + rg) + 4g + i][token 16t + l16]
    if constexpr ((ABL & 16) != 0) { // diagnostic: no epilogue stores
        if (acc[0][0][0] == 1234.5f) C[0] = 0;
        return;
    }
    if (P != nullptr) {
        // split-K partial: the tile's accumulators in register order, one contiguous block per
        // (tile, split): every store instruction writes 1 KiB contiguous.  pf16: fp16 partials
        // (half the bytes; token tiles 2u, 2u+1 side by side in one 16-byte lane store), each
        // wave's values scaled by 2^-e, e = max(0, E - 14) for their largest |value| in
        // [2^E, 2^E+1): stored values stay below 2^15 (no overflow, whatever the magnitudes);
        // e = 0 -- plain fp16 -- whenever every value is below 2^15.  The e's (one int per
        // wave and block, read by the reduce as a scalar) follow the blocks.
        const int64_t tile = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
        if (pf16) {
            const int64_t bidx = tile * gridDim.z + blockIdx.z;
            uint16_t *hb = (uint16_t *)P + bidx * (int64_t)(G::BM * G::BN);
            float mx = 0.f;
#pragma unroll
            for (int rg = 0; rg < RG; ++rg)
#pragma unroll
                for (int t = 0; t < NB; ++t)
#pragma unroll
                    for (int i = 0; i < 4; ++i) mx = fmaxf(mx, fabsf(acc[rg][t][i]));
            // wave max: DPP row shifts, row broadcasts 15 / 31 (values >= 0, so the zeros of
            // out-of-range lanes are harmless), lane 63 holds it
            int m = __builtin_bit_cast(int, mx);
            m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x111, 0xf, 0xf, true))));
            m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x112, 0xf, 0xf, true))));
            m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x114, 0xf, 0xf, true))));
            m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x118, 0xf, 0xf, true))));
            m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x142, 0xa, 0xf, true))));
            m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x143, 0xc, 0xf, true))));
            const uint32_t mb = (uint32_t)__builtin_amdgcn_readlane(m, 63);
            const int E = (int)((mb >> 23) & 0xff) - 127;
            const int e = E - 14 > 0 ? (E - 14 < 127 ? E - 14 : 126) : 0;
            const float down = __builtin_bit_cast(float, (uint32_t)(127 - e) << 23);
            const int64_t nblk = (int64_t)gridDim.x * gridDim.y * gridDim.z;
            int *es = (int *)((uint16_t *)P + nblk * (G::BM * G::BN));
            auto pk = [down](const f32x4 &v) {
                return (u32x2){(uint32_t)f2h_bits(v[0] * down) | ((uint32_t)f2h_bits(v[1] * down) << 16),
                               (uint32_t)f2h_bits(v[2] * down) | ((uint32_t)f2h_bits(v[3] * down) << 16)};
            };
            if (lane == 0) es[bidx * NWAVE + wave] = e; // (its RG row groups share it)
#pragma unroll
            for (int rg = 0; rg < RG; ++rg) {
                if constexpr (NB == 1) {
                    const int q = (RG * wave + rg) * 64 + lane;
                    ((u32x2 *)hb)[q] = pk(acc[rg][0]);
                } else {
#pragma unroll
                    for (int u = 0; u < NB / 2; ++u) {
                        const u32x2 lo = pk(acc[rg][2 * u]), hi = pk(acc[rg][2 * u + 1]);
                        const int q = ((RG * wave + rg) * (NB / 2) + u) * 64 + lane;
                        const u32x4 w = {lo.x, lo.y, hi.x, hi.y};
                        ((u32x4 *)hb)[q] = w;
                    }
                }
            }
        } else {
            f32x4 *blk = (f32x4 *)(P + (tile * gridDim.z + blockIdx.z) * (int64_t)(G::BM * G::BN));
#pragma unroll
            for (int rg = 0; rg < RG; ++rg)
#pragma unroll
                for (int t = 0; t < NB; ++t) blk[((RG * wave + rg) * NB + t) * 64 + lane] = acc[rg][t];
        }
#ifdef GQ_GEMM_STAMPS
        stamp_out();
#endif
        return;
    }
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
        const int64_t row = m0 + 16 * (RG * wave + rg) + 4 * g;
        if (row >= M) continue;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int64_t tok = n0 + 16 * t + l16;
            if (tok >= N) continue;
            const f32x4 v = acc[rg][t];
            uint16_t *dst = C + tok * ldc + row;
            if (row + 4 <= M) {
                const u32x2 o = {(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                 (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)};
                *(u32x2 *)dst = o; // 2-byte aligned when ldc or M is odd: unaligned store
            } else {
                for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(v[i]);
            }
        }
    }
#ifdef GQ_GEMM_STAMPS
    stamp_out();
#endif
}

// C = fp16(sum_s partial_s), summed in split order (deterministic).  Partials are blocked as the
// GEMM epilogue stores them: per (tile, split) a BM*BN-float block in accumulator register order,
// element (q = (wr*NB + t)*64 + lane, i) = D[row 16*wr + 4*(lane>>4) + i][token 16t + (lane&15)]
// (wr = RG*wave + rg, the wave's row group).
// One thread per (tile, q): S coalesced 16-byte loads, one 8-byte fp16 store.
// fp16 partials (pf16): unit q = ((wr*(NB/2) + u)*64 + lane) holds token tiles 2u, 2u+1 of the
// lane's 4 rows (NB = 1: one tile, 8 bytes), scaled by 2^-e (e per (block, wave), an int each
// after all blocks); rescaled and summed in fp32 in split order.
template <int NB, int RG>
__global__ __launch_bounds__(256) void gemm_reduce_f16_kernel(const uint16_t *__restrict__ P, uint16_t *__restrict__ C,
                                                              int64_t M, int64_t N, int64_t ldc, int S, int tiles_x,
                                                              int64_t nq)
{
    // one thread per 8-byte item (a token tile's 4 rows of one lane): twice the threads of
    // 16-byte units, so twice the loads in flight in this latency-bound kernel
    constexpr int TPU = NB == 1 ? 1 : 2;        // token tiles per 16-byte store unit
    constexpr int QPT = NWAVE * RG * NB * 64;   // 8-byte items per tile block
    constexpr int BPT = QPT / 256 > 0 ? QPT / 256 : 1;
    const int64_t ntiles = nq / QPT;
    int64_t tile, chunk;
    if (ntiles % 8 == 0) { // same XCD placement as gemm_reduce_kernel
        const int64_t i = blockIdx.x / 8;
        tile = blockIdx.x % 8 + 8 * (i / BPT);
        chunk = i % BPT;
    } else {
        tile = blockIdx.x / BPT;
        chunk = blockIdx.x % BPT;
    }
    const int it = (int)(chunk * 256 + threadIdx.x);
    if (tile >= ntiles || it >= QPT) return;
    const int q = TPU == 2 ? it >> 1 : it, j = TPU == 2 ? it & 1 : 0; // unit, tile within the unit
    const int lane = q & 63, u = (q >> 6) % (NB / TPU), wr = (q >> 6) / (NB / TPU);
    const int64_t m0 = (tile % tiles_x) * (16 * NWAVE * RG), n0 = (tile / tiles_x) * (16 * NB);
    const int64_t blk = (int64_t)QPT * 4; // halves per (tile, split) block
    const int *es = (const int *)(P + ntiles * S * blk);
    const int wv = __builtin_amdgcn_readfirstlane(wr / RG); // uniform: a reduce wave is one GEMM wave's rows
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < S; s0 += 8) {
        // every load unconditional (split index clamped), the surplus zeroed after: a load
        // under a per-split condition compiles to a branch and a wait per split (8 serialized
        // round trips)
        u32x2 v[8];
        int ev[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int64_t sp = tile * S + (s0 + i < S ? s0 + i : S - 1);
            ev[i] = es[sp * NWAVE + wv];
            v[i] = ((const u32x2 *)(P + sp * blk))[it];
        }
        float up[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            up[i] = __builtin_bit_cast(float, (uint32_t)(127 + ev[i]) << 23);
            if (s0 + i >= S) v[i] = (u32x2){0, 0};
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            acc[0] += h2f(v[i].x & 0xffffu) * up[i];
            acc[1] += h2f(v[i].x >> 16) * up[i];
            acc[2] += h2f(v[i].y & 0xffffu) * up[i];
            acc[3] += h2f(v[i].y >> 16) * up[i];
        }
    }
    const int64_t row = m0 + 16 * wr + 4 * (lane >> 4);
    const int64_t tok = n0 + 16 * (TPU * u + j) + (lane & 15);
    if (row >= M || tok >= N) return;
    uint16_t *dst = C + tok * ldc + row;
    if (row + 4 <= M) {
        const u32x2 o = {(uint32_t)f2h_bits(acc[0]) | ((uint32_t)f2h_bits(acc[1]) << 16),
                         (uint32_t)f2h_bits(acc[2]) | ((uint32_t)f2h_bits(acc[3]) << 16)};
        *(u32x2 *)dst = o;
    } else {
        for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(acc[i]);
    }
}

template <int NB, int RG>
__global__ __launch_bounds__(256) void gemm_reduce_kernel(const float *__restrict__ P, uint16_t *__restrict__ C,
                                                          int64_t M, int64_t N, int64_t ldc, int S, int tiles_x,
                                                          int64_t nq)
{
    constexpr int QPT = NWAVE * RG * NB * 64; // float4s per tile block
    constexpr int BPT = QPT / 256;            // reduce workgroups per tile
    // Workgroup -> tile on the XCD that computed the tile: workgroups are dealt to the 8 XCDs
    // round-robin by linear id, so with tiles % 8 == 0 every split of GEMM tile t ran on XCD
    // t % 8 and its partials are in that XCD's L2; reduce workgroup b (on XCD b % 8) takes
    // one of those tiles.  Otherwise tile-major.
    const int64_t ntiles = nq / QPT;
    int64_t tile, chunk;
    if (ntiles % 8 == 0) {
        const int64_t i = blockIdx.x / 8;
        tile = blockIdx.x % 8 + 8 * (i / BPT);
        chunk = i % BPT;
    } else {
        tile = blockIdx.x / BPT;
        chunk = blockIdx.x % BPT;
    }
    const int q = (int)(chunk * 256 + threadIdx.x);
    if (tile >= ntiles) return;
    const int lane = q & 63, t = (q >> 6) % NB, wave = (q >> 6) / NB;
    const int64_t m0 = (tile % tiles_x) * (16 * NWAVE * RG), n0 = (tile / tiles_x) * (16 * NB);
    const f32x4 *src = (const f32x4 *)P + tile * S * QPT + q;
    // all loads of a group of 8 splits issued before the first add (independent, in flight
    // together); the sum stays in split order
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < S; s0 += 8) {
        f32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = src[(int64_t)(s0 + i < S ? s0 + i : S - 1) * QPT]; // unconditional (see above)
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (s0 + i >= S) v[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += v[i];
    }
    const int64_t row = m0 + 16 * wave + 4 * (lane >> 4), tok = n0 + 16 * t + (lane & 15);
    if (tok >= N || row >= M) return;
    uint16_t *dst = C + tok * ldc + row;
    if (row + 4 <= M) {
        const u32x2 o = {(uint32_t)f2h_bits(acc[0]) | ((uint32_t)f2h_bits(acc[1]) << 16),
                         (uint32_t)f2h_bits(acc[2]) | ((uint32_t)f2h_bits(acc[3]) << 16)};
        *(u32x2 *)dst = o;
    } else {
        for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(acc[i]);
    }
}

template <int F, int NB, int RG, int AM = AF_F16, int NL = 0, int AQ = 0>
hipError_t launch_cfg(const uint8_t *A, const GemmAct &x, uint16_t *C, float *P, const GemmPlan &pl, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    using G = Cfg<F, NB, RG, AM, NL, AQ>;
    dim3 grid((unsigned)((M + G::BM - 1) / G::BM), (unsigned)((N + G::BN - 1) / G::BN), (unsigned)pl.splits);
    float *PP = pl.splits > 1 ? P : nullptr;
    const int cps = pl.chunks_per_split;
    const void *X = AQ ? (const void *)x.xraw : (G::CODES ? (const void *)x.xq : (const void *)x.xdeq);
    const int64_t ldd = AQ ? x.ldx : x.ldd;
#ifdef GQ_ABLATION
    const int abl = tuning().ablate;
#define GQ_ABL_CASE(v) \
    case v: gemm_kernel<F, NB, RG, v, AM, NL, AQ><<<grid, dim3(G::THREADS), 0, s>>>(A, X, x.xd, C, PP, M, N, K, ldc, ldd, cps, pl.pf16); break;
    switch (abl) {
    GQ_ABL_CASE(1) GQ_ABL_CASE(6) GQ_ABL_CASE(8) GQ_ABL_CASE(15) GQ_ABL_CASE(16) GQ_ABL_CASE(31) GQ_ABL_CASE(32)
    GQ_ABL_CASE(33) GQ_ABL_CASE(2) GQ_ABL_CASE(4) GQ_ABL_CASE(64) GQ_ABL_CASE(68) GQ_ABL_CASE(96) GQ_ABL_CASE(128) GQ_ABL_CASE(134)
    default: gemm_kernel<F, NB, RG, 0, AM, NL, AQ><<<grid, dim3(G::THREADS), 0, s>>>(A, X, x.xd, C, PP, M, N, K, ldc, ldd, cps, pl.pf16); break;
    }
#undef GQ_ABL_CASE
#else
    gemm_kernel<F, NB, RG, 0, AM, NL, AQ><<<grid, dim3(G::THREADS), 0, s>>>(A, X, x.xd, C, PP, M, N, K, ldc, ldd, cps, pl.pf16);
#endif
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || pl.splits == 1) return e;
    if (pl.pf16) {
        const int64_t nq = (int64_t)grid.x * grid.y * (NWAVE * RG * NB * 64);
        gemm_reduce_f16_kernel<NB, RG><<<dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s>>>(
            (const uint16_t *)P, C, M, N, ldc, pl.splits, (int)grid.x, nq);
        return hipGetLastError();
    }
    const int64_t nq = (int64_t)grid.x * grid.y * (NWAVE * RG * NB * 64);
    gemm_reduce_kernel<NB, RG><<<dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s>>>(P, C, M, N, ldc, pl.splits,
                                                                                         (int)grid.x, nq);
    return hipGetLastError();
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const GemmAct &x, uint16_t *C, float *P, const GemmPlan &pl, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if constexpr (F == Q4_K || F == Q6_K)
        if (pl.rg == 2 * R1 && pl.nb == 8)
            return pl.loaders == 4 ? launch_cfg<F, 8, 2 * R1, AF_F16, 4>(A, x, C, P, pl, M, N, K, ldc, s)
                                   : launch_cfg<F, 8, 2 * R1>(A, x, C, P, pl, M, N, K, ldc, s);
    if constexpr (F == Q8_0)
        if (pl.act == AF_I8) switch (pl.nb) {
            case 1: return launch_cfg<F, 1, 1, AF_I8>(A, x, C, P, pl, M, N, K, ldc, s);
            case 2: return launch_cfg<F, 2, 1, AF_I8>(A, x, C, P, pl, M, N, K, ldc, s);
            case 4: return launch_cfg<F, 4, 1, AF_I8>(A, x, C, P, pl, M, N, K, ldc, s);
            default: return launch_cfg<F, 8, 1, AF_I8>(A, x, C, P, pl, M, N, K, ldc, s);
            }
    if (pl.aq && pl.loaders == 4 && pl.rg == R1 && pl.act == AF_F16) switch (pl.nb) {
        case 1: return launch_cfg<F, 1, R1, AF_F16, 4, 1>(A, x, C, P, pl, M, N, K, ldc, s);
        case 2: return launch_cfg<F, 2, R1, AF_F16, 4, 1>(A, x, C, P, pl, M, N, K, ldc, s);
        case 4: return launch_cfg<F, 4, R1, AF_F16, 4, 1>(A, x, C, P, pl, M, N, K, ldc, s);
        default: return hipErrorInvalidValue;
        }
    if (pl.loaders == 4) switch (pl.nb) {
        case 1: return launch_cfg<F, 1, R1, AF_F16, 4>(A, x, C, P, pl, M, N, K, ldc, s);
        case 2: return launch_cfg<F, 2, R1, AF_F16, 4>(A, x, C, P, pl, M, N, K, ldc, s);
        case 4: return launch_cfg<F, 4, R1, AF_F16, 4>(A, x, C, P, pl, M, N, K, ldc, s);
        default: return launch_cfg<F, 8, R1, AF_F16, 4>(A, x, C, P, pl, M, N, K, ldc, s);
        }
    switch (pl.nb) {
    case 1: return launch_cfg<F, 1, R1>(A, x, C, P, pl, M, N, K, ldc, s);
    case 2: return launch_cfg<F, 2, R1>(A, x, C, P, pl, M, N, K, ldc, s);
    case 4: return launch_cfg<F, 4, R1>(A, x, C, P, pl, M, N, K, ldc, s);
    default: return launch_cfg<F, 8, R1>(A, x, C, P, pl, M, N, K, ldc, s);
    }
}

int pick_nb(int64_t N) { return N > 64 ? 8 : (N > 32 ? 4 : (N > 16 ? 2 : 1)); }

} // namespace

hipError_t launch_gemm_reduce_f16(int nb, int rg, const uint16_t *P, uint16_t *C, int64_t M, int64_t N, int64_t ldc,
                                  int S, int tiles_x, int tiles_y, hipStream_t s)
{
    const int64_t nq = (int64_t)tiles_x * tiles_y * (NWAVE * rg * nb * 64);
    const dim3 grid((unsigned)((nq + 255) / 256)), block(256);
#define GQ_RED(NB_, RG_)                                                                                                   if (nb == NB_ && rg == RG_) {                                                                                              gemm_reduce_f16_kernel<NB_, RG_><<<grid, block, 0, s>>>(P, C, M, N, ldc, S, tiles_x, nq);                              return hipGetLastError();                                                                                          }
    GQ_RED(1, 2) GQ_RED(2, 2) GQ_RED(4, 2) GQ_RED(8, 2)
#undef GQ_RED
    return hipErrorInvalidValue;
}

bool gemm_supported(int /*fmt*/, int64_t K) { return K > 0 && K % 256 == 0; }

bool gemm_aq_ok(const GemmPlan &p)
{
    if (!tuning().gemm_aq) return false;
    // splits of at most two super-blocks: the quantization (a few passes of the loader waves)
    // then hides under the first weight stage; longer splits measured neutral to 2% slower
    // (Q4_K 4096x11008 x16), shorter ones 4-9% faster (profiles/r02/gemm_aq_ab.txt)
    // 64-token tiles measured 11-14% slower: the loader waves' quantization
    // (32 blocks per lane) no longer hides under the first weight stage
    constexpr int max_nb = 2;
    return p.act == AF_F16 && p.loaders == 4 && p.rg == R1 && p.nb <= max_nb && p.chunks_per_split <= 2 &&
           4 * p.chunks_per_split <= aq_sub_of(p.nb);
}

GemmPlan plan_gemm(int fmt, int64_t M, int64_t N, int64_t K, int act)
{
    GemmPlan p;
    p.act = act == AF_I8 && fmt != Q8_0 ? AF_F16 : act;
    p.nb = pick_nb(N);
    // two 16-row groups per wave (256-row tiles: half the activation traffic per weight) for
    // tall matrices at full token tiles
    // (Q4_K; Q6_K as a 224-B row image, Cfg::Q6S, only on request: half the activation re-reads
    // but a 3-deep activation ring, measured slower -- 28672x8192 x128 116.5 vs 105.7 us,
    // 8192x28672 106.0 vs 103.9, 4096^2 21.9 vs 16.8: profiles/r03/gemm_q6k_rg2_rejected.log;
    // Q8_0's 272-B rows do not fit 256 rows twice)
    const bool rg2_ok = (fmt == Q4_K || fmt == Q6_K) && p.nb == 8;
    p.rg = (fmt == Q4_K && rg2_ok && M >= 8192) ? 2 * R1 : R1; // measured: Q4_K 11008 rows 5% faster
    if (tuning().gemm_rg) p.rg = (rg2_ok && tuning().gemm_rg == 2) ? 2 * R1 : R1;
    if (p.act != AF_F16) p.rg = 1; // the code forms run 128-row tiles
    // four loader waves (DMA issue off the multiplying waves' path) for the 128-row fp16 form:
    // Q6_K 28672x8192x128 116.5 -> 103.7 us, Q4_K 4096^2x128 17.4 -> 16.7, Q8_0 4096^2x128
    // 20.6 -> 20.1 (profiles/r02/loader_tune.txt)
    p.loaders = p.act == AF_F16 && p.rg == R1 ? 4 : 0;
    const int64_t nws = K / 256; // weight stages (super-blocks)
    if (nws == 0) return p;      // not a GEMM shape (gemm_supported() is false): nothing to plan
    const int64_t bm = 16 * NWAVE * p.rg;
    const int64_t tiles = ((M + bm - 1) / bm) * ((N + 16 * p.nb - 1) / (16 * p.nb));
    // one workgroup per CU (LDS-bound): the largest split that keeps tiles * S <= 256 CUs, so no
    // second wave of workgroups (258 workgroups ran 25% slower than 172 at 11008 x 4096 x 128)
    const int64_t cus = num_cus();
    int64_t S = tiles >= cus ? 1 : cus / tiles;
    if (tuning().gemm_splits > 0) S = tuning().gemm_splits; // tuning / test override
    const int64_t max_split = nws / 2 > 0 ? nws / 2 : 1;            // >= 2 super-blocks per split
    if (S > max_split) S = max_split;
    if (S < 1) S = 1;
    int64_t sps = (nws + S - 1) / S;
    S = (nws + sps - 1) / sps;
    p.splits = (int)S;
    p.chunks_per_split = (int)sps;
    // fp16 partials (default; GQ_GEMM_PARTIAL=f32 for fp32): half the round trip, each wave's
    // partial values rounded to fp16 after a power-of-two scale that keeps them below 2^15
    // (Q8_0 4096^2 x128 step 23.2 -> 22.1 us; profiles/r02/pf16_step.txt)
    p.pf16 = 1;
    if (tuning().gemm_partial_f32) p.pf16 = 0;
    // blocked partials: S x (tiles) x 128 rows x 16*nb tokens (padded tiles)
    p.partial_bytes = S > 1 ? (size_t)S * tiles * bm * 16 * p.nb * (p.pf16 ? 2 : sizeof(float)) : 0;
    if (S > 1 && p.pf16) p.partial_bytes += (size_t)S * tiles * NWAVE * sizeof(int); // the per-wave e's
    return p;
}

hipError_t launch_gemm(int fmt, const uint8_t *A, const GemmAct &x, uint16_t *C, float *P, const GemmPlan &plan,
                       int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, x, C, P, plan, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, x, C, P, plan, M, N, K, ldc, s);
    default: return launch_fmt<Q6_K>(A, x, C, P, plan, M, N, K, ldc, s);
    }
}

} // namespace gq

#ifdef GQ_GEMM_STAMPS
extern "C" int gq_debug_gemm_stamps(void *host, size_t bytes)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(gq::g_gstamps), bytes < sizeof(gq::g_gstamps) ? bytes : sizeof(gq::g_gstamps)) == hipSuccess ? 0 : 1;
}
#endif
