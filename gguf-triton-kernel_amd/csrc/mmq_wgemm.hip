// mmq_wgemm.hip -- batched MMQ (many tokens) with the weights streamed straight into registers.
//
// C[t][m] = sum_k W[m][k] * x~[t][k] on v_mfma_f32_16x16x32_f16 (fp32 accumulate), x~ = fp16(d*q)
// the q8_1-quantized activation (act_quant.hip DEQ form: the integers kernels/cpu_impls
// multiplies, mmq_*_q8_1_cpu.py), W dequantized to fp16 in registers from the packed GGUF bytes.
// Replaces the reference's Triton GEMM loops (kernels/mmq_q8_0.py:59-93, mmq_q4_k.py:167-229,
// mmq_q6_k.py:122-186) for 64+ tokens.
//
// Why this shape.  In mmq_gemm.hip both operands went HBM/L2 -> LDS by LDS-DMA and
// the per-CU DMA ingest (~25 GB/s per CU), not the MFMA or HBM, bounded the kernel.  Here a
// wave's A operand -- 16*RG weight rows private to it -- never touches LDS: each lane loads the
// bytes of its own fragment slots with buffer loads one super-block ahead (VGPR double buffer),
// dequantizes in registers and feeds the MFMA.  Only the activations, which all 8 waves share,
// go through LDS: register-staged (a buffer load one sub-stage ahead, ds_write_b128 the next
// sub-stage behind), a two-slot ring, one barrier per 64-element sub-stage.  Every VMEM op is
// an ordinary load the compiler counts (no LDS-DMA, so no vmcnt(0) drains).
//
// Workgroup = 8 waves (two per SIMD, <= 256 VGPRs) = BM = 128*RG weight rows x BN = 16*NB tokens
// x one K split.  Wave w owns rows 16*(RG*w + rf) + [0,16) and every token of the tile, so each
// weight is dequantized once per workgroup and each activation fragment read from LDS feeds RG
// MFMAs.
//
// K order.  An MFMA k-step is one natural 32-element run of K (a Q8_0 block, a Q4_K sub-block,
// two Q6_K scale groups) and lane group g = lane>>4 takes its 8-element piece g, as fp16 pairs in
// the order (0,2,1,3,4,6,5,7) that packed dequantization produces -- exactly act_quant's DEQ
// layout, so a B fragment is one 16-byte LDS read.  Per super-block (256 elements) lane (row r,
// g) therefore needs: Q4_K qs bytes 32j+8g..+8 (j = 0..3, both nibbles) + the 16-byte header;
// Q6_K ql bytes 64h+32v+8g..+8, qh bytes 128+32h+8g..+8, the 16 scale bytes and d; Q8_0 qs bytes
// 34i+2+8g..+8 and d of each of the 8 blocks.  Those are loaded as they lie (gfx950 runs with
// unaligned buffer access: Q6_K/Q8_0 fields are 2-byte aligned).
//
// MFMA 16x16x32 f16 (gfx950): lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15];
// D[row 4(l>>4)+i][col l&15] in acc element i.  Weight rows are A rows, tokens B columns.
#include <type_traits>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"

namespace gq {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NWAVE = 8;
constexpr int THREADS = 64 * NWAVE;

__device__ __forceinline__ h2 as_h2(uint32_t v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ uint32_t as_u32(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2 splat(float f) { return (h2){(_Float16)f, (_Float16)f}; }
__device__ __forceinline__ f16x8 frag4(h2 a, h2 b, h2 c, h2 d)
{
    u32x4 v = {as_u32(a), as_u32(b), as_u32(c), as_u32(d)};
    return __builtin_bit_cast(f16x8, v);
}
// f16 pairs (1024 + code) from codes masked into the low bits of bytes 0 and 2
__device__ __forceinline__ h2 magic(uint32_t v, uint32_t mask) { return as_h2((v & mask) | 0x64006400u); }
// f16 pairs (1024 + byte) of bytes (0,2) and (1,3) of a code word
__device__ __forceinline__ h2 pair02(uint32_t c) { return as_h2(__builtin_amdgcn_perm(0x64646464u, c, 0x04020400u)); }
__device__ __forceinline__ h2 pair13(uint32_t c) { return as_h2(__builtin_amdgcn_perm(0x64646464u, c, 0x04030401u)); }

__device__ __forceinline__ u32x2 bl8(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s)
{
    return __builtin_amdgcn_raw_buffer_load_b64(r, v, s, 0);
}
__device__ __forceinline__ u32x4 bl16(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, v, s, 0);
}
__device__ __forceinline__ uint32_t bl4(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s)
{
    return __builtin_amdgcn_raw_buffer_load_b32(r, v, s, 0);
}

// Diagnostic ablations (GQ_WGEMM_ABL, a -D of a separate build; 0 in the product): 1 = no
// weight loads after the prologue, 2 = no activation staging after the prologue, 4 = no MFMA,
// 8 = no dequantization (raw bits as fp16), 16 = weight loads at 8-byte aligned addresses (wrong
// values: an access-pattern probe).
#ifndef GQ_WGEMM_ABL
#define GQ_WGEMM_ABL 0
#endif
constexpr int ABL = GQ_WGEMM_ABL;
// weight byte offset as loaded (the alignment probe rounds it down)
__device__ __forceinline__ uint32_t wo(uint32_t v) { return ABL & 16 ? v & ~7u : v; }


// ---------------------------------------------------------------------------------------
// One super-block of one 16-row fragment: this lane's bytes (WB<F>::load: back-to-back 16-byte
// loads, so the 4 lanes of a row read 64 contiguous bytes per instruction and a row's lines are
// reused within the burst) and the A fragment of k-step s = 0..7 from them (WB<F>::frag).  The
// k-step -> element map follows what a lane loaded: e(s, g) below = the first of the 8 elements
// (consecutive in K, fragment order (0,2,1,3,4,6,5,7)) that lane group g supplies at k-step s;
// the B fragment reads the same 8 activations.  v = the row's byte offset, s0 = the super-block's
// byte offset in the row (wave-uniform: the buffer's SGPR offset).
template <int F> struct WB;

// Q4_K: lane g loads the 16-byte header and qs bytes 64i + 16g .. +16 (i = 0, 1); qs byte b holds
// elements 64(b/32) + b%32 (low nibble) and +32 (high).  k-step s = 4i + 2nib + half.
template <> struct WB<Q4_K> {
    static constexpr int SB = 144;
    u32x4 hdr;   // d, dmin, 12 scale bytes
    u32x4 qs[2]; // qs bytes 64i + 16g .. +16
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t v, int g, uint32_t s0)
    {
        hdr = bl16(r, wo(v), s0);
        qs[0] = bl16(r, wo(v + 16 + 16 * g), s0);
        qs[1] = bl16(r, wo(v + 80 + 16 * g), s0);
    }
    static __device__ __forceinline__ int e(int s, int g)
    {
        return 64 * (2 * (s >> 2) + (g >> 1)) + 32 * ((s >> 1) & 1) + 16 * (g & 1) + 8 * (s & 1);
    }
    __device__ __forceinline__ f16x8 frag(int s, int g) const
    {
        const int i = s >> 2, nib = (s >> 1) & 1, half = s & 1;
        const int sbk = 4 * i + 2 * (g >> 1) + nib; // sub-block (per lane)
        const float d = h2f(hdr.x & 0xffffu), dmin = h2f(hdr.x >> 16);
        int sc, m;
        if (i == 0) { // sub-blocks 0..3
            sc = (hdr.y >> (8 * sbk)) & 63;
            m = (hdr.z >> (8 * sbk)) & 63;
        } else {
            const int k = 8 * (sbk - 4);
            const uint32_t hi = (hdr.w >> k) & 0xffu;
            sc = (hi & 0x0f) | (((hdr.y >> k) & 0xc0u) >> 2);
            m = (hi >> 4) | (((hdr.z >> k) & 0xc0u) >> 2);
        }
        const h2 ds = splat(d * (float)sc), ndm = splat(-(dmin * (float)m));
        const h2 bias = splat(-1024.f);
        const uint32_t x0 = (half ? qs[i].z : qs[i].x) >> (4 * nib), x1 = (half ? qs[i].w : qs[i].y) >> (4 * nib);
        return frag4(__builtin_elementwise_fma(magic(x0, 0x000f000fu) + bias, ds, ndm),
                     __builtin_elementwise_fma(magic(x0 >> 8, 0x000f000fu) + bias, ds, ndm),
                     __builtin_elementwise_fma(magic(x1, 0x000f000fu) + bias, ds, ndm),
                     __builtin_elementwise_fma(magic(x1 >> 8, 0x000f000fu) + bias, ds, ndm));
    }
};

// Q6_K: lane g loads ql bytes 64h + 16g .. +16, qh bytes 32h + 16(g&1) .. +16 (h = 0, 1), the 16
// scales and d.  ql byte 64h + 16g + t (t < 16) holds elements 128h + 32(g>>1) + 16(g&1) + t (low
// nibble) and +64 (high); its qh bits sit in qh byte 32h + 16(g&1) + t at 2(g>>1) + 4nib.
// k-step s = 4h + 2nib + half; scale index 8h + 4nib + 2(g>>1) + (g&1) = byte g of word 2h + nib.
template <> struct WB<Q6_K> {
    static constexpr int SB = 210;
    u32x4 ql[2], qh[2];
    u32x4 sc;   // the 16 int8 scales
    uint32_t d; // bytes 206..209: d in the high half
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t v, int g, uint32_t s0)
    {
        ql[0] = bl16(r, wo(v + 16 * g), s0);
        ql[1] = bl16(r, wo(v + 64 + 16 * g), s0);
        qh[0] = bl16(r, wo(v + 128 + 16 * (g & 1)), s0);
        qh[1] = bl16(r, wo(v + 160 + 16 * (g & 1)), s0);
        sc = bl16(r, wo(v + 192), s0);
        d = bl4(r, wo(v + 206), s0);
    }
    static __device__ __forceinline__ int e(int s, int g)
    {
        return 128 * (s >> 2) + 64 * ((s >> 1) & 1) + 32 * (g >> 1) + 16 * (g & 1) + 8 * (s & 1);
    }
    __device__ __forceinline__ f16x8 frag(int s, int g) const
    {
        const int h = s >> 2, nib = (s >> 1) & 1, half = s & 1;
        const u32x4 q4 = ql[h], h4 = qh[h];
        const uint32_t qx = half ? q4.z : q4.x, qy = half ? q4.w : q4.y;
        const uint32_t hx = half ? h4.z : h4.x, hy = half ? h4.w : h4.y;
        const int sq = 2 * (g >> 1) + 4 * nib;
        const uint32_t sw = (2 * h + nib) == 0 ? sc.x : ((2 * h + nib) == 1 ? sc.y : ((2 * h + nib) == 2 ? sc.z : sc.w));
        const float scv = (float)(int8_t)((sw >> (8 * g)) & 0xffu);
        const h2 dsc = splat(h2f(d >> 16) * scv);
        const h2 bias = splat(-1056.f); // 1024 + 32
        const uint32_t c0 = ((qx >> (4 * nib)) & 0x0f0f0f0fu) | (((hx >> sq) & 0x03030303u) << 4);
        const uint32_t c1 = ((qy >> (4 * nib)) & 0x0f0f0f0fu) | (((hy >> sq) & 0x03030303u) << 4);
        return frag4((pair02(c0) + bias) * dsc, (pair13(c0) + bias) * dsc, (pair02(c1) + bias) * dsc,
                     (pair13(c1) + bias) * dsc);
    }
};

// Q8_0: lane g loads row bytes 68g .. 68g+68 of the super-block (blocks 2g, 2g+1: d, 32 qs, d,
// 32 qs; 4-byte aligned: the super-block starts 16-byte aligned whenever K % 256 == 0).  k-step
// s = 4blk + p: qs bytes 8p .. 8p+8 of block 2g + blk.
template <> struct WB<Q8_0> {
    static constexpr int SB = 272;
    u32x4 w[4];
    uint32_t w16;
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t v, int g, uint32_t s0)
    {
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = bl16(r, wo(v + 68 * g + 16 * i), s0);
        w16 = bl4(r, wo(v + 68 * g + 64), s0);
    }
    __device__ __forceinline__ uint32_t dw(int k) const // dword k of the lane's 68 bytes
    {
        const u32x4 q = w[k >> 2 < 4 ? k >> 2 : 3];
        if (k == 16) return w16;
        return (k & 3) == 0 ? q.x : ((k & 3) == 1 ? q.y : ((k & 3) == 2 ? q.z : q.w));
    }
    static __device__ __forceinline__ int e(int s, int g) { return 64 * g + 32 * (s >> 2) + 8 * (s & 3); }
    __device__ __forceinline__ f16x8 frag(int s, int) const
    {
        const int blk = s >> 2, p = s & 3;
        uint32_t q0, q1, dv;
        if (blk == 0) { // qs bytes 2 + 8p ..: dwords 2p .. 2p+2 shifted by 2 bytes
            q0 = __builtin_amdgcn_alignbyte(dw(2 * p + 1), dw(2 * p), 2);
            q1 = __builtin_amdgcn_alignbyte(dw(2 * p + 2), dw(2 * p + 1), 2);
            dv = __builtin_amdgcn_perm(dw(0), dw(0), 0x05040504u); // d of block 2g: bytes 0, 1
        } else { // qs bytes 36 + 8p ..: dwords 9 + 2p, 10 + 2p
            q0 = dw(9 + 2 * p);
            q1 = dw(10 + 2 * p);
            dv = __builtin_amdgcn_perm(dw(8), dw(8), 0x07060706u); // d of block 2g+1: bytes 34, 35
        }
        const h2 bias = splat(-1152.f); // codes biased by +128 (xor 0x80)
        const h2 d = as_h2(dv);
        const uint32_t c0 = q0 ^ 0x80808080u, c1 = q1 ^ 0x80808080u;
        return frag4((pair02(c0) + bias) * d, (pair13(c0) + bias) * d, (pair02(c1) + bias) * d,
                     (pair13(c1) + bias) * d);
    }
};

// ---------------------------------------------------------------------------------------
// LDS: two activation slots of one super-block, [k-step s][token n][4 lane groups x 16 bytes]
// (64 bytes per token and k-step); lane group g's piece stored at g ^ kF[(n >> 2) & 3]: the
// 16-lane groups of a ds_read_b128 then hit 16 distinct 16-byte bank slots.
__device__ __forceinline__ int swz(int g, int n)
{
    constexpr uint32_t kF = 0x1320u; // F = {0, 2, 3, 1}
    return g ^ (int)((kF >> (4 * ((n >> 2) & 3))) & 3u);
}

template <int F, int RG, int NB>
struct WCfg {
    static constexpr int BM = 16 * NWAVE * RG, BN = 16 * NB;
    static constexpr int SLOT = BN * 512; // one super-block of BN tokens
    static constexpr int LDS_BYTES = 2 * SLOT;
    // activation staging: BN * 32 pieces of 16 bytes per super-block, NQ per thread (each thread
    // an equal share: a conditional store would let the compiler sink its loads); BN = 16: 8-byte
    // halves of pieces
    static constexpr int U = BN >= 32 ? 16 : 8;
    static constexpr int NQ = BN * 512 / THREADS / U;
    static_assert(NQ >= 1 && NQ * U * THREADS == BN * 512, "whole staging passes");
};

// Block -> (tile, split): the S splits of tile t run on XCD t % 8 when the tile count is a
// multiple of 8 (blocks b and b + 8 share an XCD under round-robin dispatch; a speed choice,
// never correctness), so the split-K reduce finds a tile's partials in one L2.
__device__ __forceinline__ void block_map(int b, int ntiles, int S, int &tile, int &sp)
{
    if (ntiles % 8 == 0) {
        const int j = b >> 3;
        tile = (b & 7) + 8 * (j / S);
        sp = j % S;
    } else {
        tile = b / S;
        sp = b % S;
    }
}

// P (S > 1): fp16 partials per (tile, split) block in accumulator order -- unit
// q = ((wr*(NB/2) + u)*64 + lane) (wr = RG*wave + rf) holds token tiles 2u, 2u+1 of the lane's 4
// rows, scaled by 2^-e (e per (block, wave), ints after all the blocks); NB = 1: 8-byte units of
// one token tile.  wreduce_kernel sums them.
template <int F, int RG, int NB>
__global__ __launch_bounds__(THREADS) void wgemm_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                       uint16_t *__restrict__ C, uint16_t *__restrict__ P, int M, int N,
                                                       int K, int ldc, int tiles_m, int S, int sb_per_split)
{
    using G = WCfg<F, RG, NB>;
    using W = WB<F>;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[G::LDS_BYTES];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c = lane & 15;
    int tile, sp;
    block_map(blockIdx.x, (int)gridDim.x / S, S, tile, sp);
    const int tm = tile % tiles_m, tn = tile / tiles_m;
    const int m0 = tm * G::BM, n0 = tn * G::BN;
    const int nsb = K / 256;
    const int sb0 = sp * sb_per_split;
    const int sb1 = sb0 + sb_per_split < nsb ? sb0 + sb_per_split : nsb;
    const int row_bytes = (K / Layout<F>::QK) * Layout<F>::BYTES;

    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, M * row_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, N * K * 2, 0x00020000);

    // this lane's weight rows (clamped: rows past M compute garbage that is never stored)
    uint32_t wv[RG];
#pragma unroll
    for (int rf = 0; rf < RG; ++rf) {
        const int row = m0 + 16 * (RG * wave + rf) + c;
        wv[rf] = (uint32_t)((row < M ? row : M - 1) * row_bytes);
    }
    // activation staging: pass q moves piece (half) i = q*THREADS + tid: token i / 32, natural
    // piece P = i % 32 of the super-block (U = 8: i / 64, piece (i % 64) / 2, half i % 2), to the
    // LDS position of the (k-step, lane group) that multiplies it
    uint32_t xv[G::NQ];
    int xd[G::NQ];
#pragma unroll
    for (int q = 0; q < G::NQ; ++q) {
        const int i = q * THREADS + tid;
        const int per = 32 * 16 / G::U; // units per token
        const int n = i / per, u = i % per, Pc = u * G::U / 16, b = u * G::U % 16;
        const int tok = n0 + n < N ? n0 + n : N - 1;
        xv[q] = (uint32_t)tok * (uint32_t)K * 2u + 16u * (uint32_t)Pc + (uint32_t)b;
        int ks = 0, kg = 0; // the (k-step, lane group) whose e(s, g) is piece Pc
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg)
                if (W::e(s, gg) == 8 * Pc) ks = s, kg = gg;
        xd[q] = ks * (G::BN * 64) + n * 64 + 16 * swz(kg, n) + b;
    }

    f32x4 acc[RG][NB];
#pragma unroll
    for (int rf = 0; rf < RG; ++rf)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[rf][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

    if (sb1 > sb0) {
        using XU = typename std::conditional<G::U == 16, u32x4, u32x2>::type;
        W wb[2][RG]; // super-block double buffer
        XU xs[G::NQ];
        auto load_w = [&](int b, int sb) { // super-block sb (clamped) into buffer b
            const uint32_t s0 = (uint32_t)((sb < sb1 ? sb : sb1 - 1) * W::SB) & (ABL & 16 ? ~7u : ~0u);
#pragma unroll
            for (int rf = 0; rf < RG; ++rf) wb[b][rf].load(wrs, wv[rf], g, s0);
        };
        auto load_x = [&](int sb) { // super-block sb (clamped) of the tile's tokens
            const uint32_t so = 512u * (uint32_t)(sb < sb1 ? sb : sb1 - 1);
#pragma unroll
            for (int q = 0; q < G::NQ; ++q) {
                if constexpr (G::U == 16) xs[q] = bl16(xrs, xv[q], so);
                else xs[q] = bl8(xrs, xv[q], so);
            }
        };
        auto store_x = [&](int slot) {
#pragma unroll
            for (int q = 0; q < G::NQ; ++q) *(XU *)(lds + slot * G::SLOT + xd[q]) = xs[q];
        };
        auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
        auto pin = [] { __builtin_amdgcn_sched_barrier(0); };
        // multiply one super-block: weights from buffer b, activations from LDS slot `slot`
        auto compute = [&](int b, int slot) {
            const uint8_t *xsl = lds + slot * G::SLOT;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                f16x8 bf[NB];
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const int n = 16 * t + c;
                    bf[t] = *(const f16x8 *)(xsl + s * (G::BN * 64) + n * 64 + 16 * swz(g, n));
                }
                f16x8 af[RG];
#pragma unroll
                for (int rf = 0; rf < RG; ++rf) {
                    if constexpr (ABL & 8) af[rf] = __builtin_bit_cast(f16x8, (u32x4){wv[rf], wv[rf] + 1u, (uint32_t)s, 5u});
                    else af[rf] = wb[b][rf].frag(s, g);
                }
#pragma unroll
                for (int rf = 0; rf < RG; ++rf)
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        if constexpr (ABL & 4) acc[rf][t][0] += (float)af[rf][t & 7] * (float)bf[t][0];
                        else acc[rf][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[rf], bf[t], acc[rf][t], 0, 0, 0);
                    }
            }
        };

        // Super-block i (buffer i & 1, LDS slot i & 1): multiply; ds_write the activations of
        // i + 1 (loaded one super-block ago); load the activations of i + 2, then the weights of
        // i + 2 into buffer i & 1; barrier.  Issue order is what matters to the in-order vmcnt
        // queue: each activation load is issued BEFORE the weight burst of its super-block, so
        // waiting for it never waits for HBM weight bytes younger than one super-block, and every
        // stream has a full super-block of lead.  The prologue issues the same sequence (X, W, X,
        // W), so the compiler's counts at the loop head agree on both paths.  Every load is
        // unconditional (indices clamped: surplus re-reads hit the cache) -- a load under a
        // condition makes the count at the merge the smaller one, i.e. a drain.
        load_x(sb0);
        pin();
        load_w(0, sb0);
        pin();
        store_x(0);
        load_x(sb0 + 1);
        pin();
        load_w(1, sb0 + 1);
        barrier();
        auto body = [&](int sb, int b) {
            compute(b, b);
            pin();
            if constexpr (!(ABL & 2)) store_x(b ^ 1); // (past the end: a slot nobody reads)
            if constexpr (!(ABL & 2)) load_x(sb + 2);
            pin();
            if constexpr (!(ABL & 1)) load_w(b, sb + 2);
            barrier();
        };
        // pairs in the loop (static buffer parity), an odd last super-block after it: the loop's
        // back edge always follows the same two bodies
        int sb = sb0;
        for (; sb + 1 < sb1; sb += 2) {
            body(sb, 0);
            body(sb + 1, 1);
        }
        if (sb < sb1) body(sb, 0);
    }

    // epilogue: acc[rf][t][i] = D[row 16*(RG*wave + rf) + 4g + i][token 16t + c]
    if (S > 1) {
        const int bidx = tile * S + sp;
        uint16_t *hb = P + (size_t)bidx * (G::BM * G::BN);
        float mx = 0.f;
#pragma unroll
        for (int rf = 0; rf < RG; ++rf)
#pragma unroll
            for (int t = 0; t < NB; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) mx = fmaxf(mx, fabsf(acc[rf][t][i]));
        // wave max (values >= 0): DPP row shifts + row broadcasts, lane 63 holds it
        int mm = __builtin_bit_cast(int, mx);
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x111, 0xf, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x112, 0xf, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x114, 0xf, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x118, 0xf, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x142, 0xa, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x143, 0xc, 0xf, true))));
        const uint32_t mb = (uint32_t)__builtin_amdgcn_readlane(mm, 63);
        const int E = (int)((mb >> 23) & 0xff) - 127;
        const int e = E - 14 > 0 ? (E - 14 < 127 ? E - 14 : 126) : 0;
        const float down = __builtin_bit_cast(float, (uint32_t)(127 - e) << 23);
        const int nblk = (int)gridDim.x;
        if (lane == 0) ((int *)(P + (size_t)nblk * (G::BM * G::BN)))[bidx * NWAVE + wave] = e;
        auto pk = [down](const f32x4 &v) {
            return (u32x2){(uint32_t)f2h_bits(v[0] * down) | ((uint32_t)f2h_bits(v[1] * down) << 16),
                           (uint32_t)f2h_bits(v[2] * down) | ((uint32_t)f2h_bits(v[3] * down) << 16)};
        };
#pragma unroll
        for (int rf = 0; rf < RG; ++rf) {
            if constexpr (NB == 1) {
                ((u32x2 *)hb)[(RG * wave + rf) * 64 + lane] = pk(acc[rf][0]);
            } else {
#pragma unroll
                for (int u = 0; u < NB / 2; ++u) {
                    const u32x2 lo = pk(acc[rf][2 * u]), hi = pk(acc[rf][2 * u + 1]);
                    ((u32x4 *)hb)[((RG * wave + rf) * (NB / 2) + u) * 64 + lane] = (u32x4){lo.x, lo.y, hi.x, hi.y};
                }
            }
        }
        return;
    }
#pragma unroll
    for (int rf = 0; rf < RG; ++rf) {
        const int row = m0 + 16 * (RG * wave + rf) + 4 * g;
        if (row >= M) continue;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int tok = n0 + 16 * t + c;
            if (tok >= N) continue;
            const f32x4 v = acc[rf][t];
            uint16_t *dst = C + (size_t)tok * ldc + row;
            if (row + 4 <= M) {
                *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                        (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)};
            } else {
                for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(v[i]);
            }
        }
    }
}

// C = fp16(sum_s 2^e_s * partial_s) in split order (deterministic), one thread per 16-byte
// unit (two token tiles of a lane's 4 rows; NB = 1: one 8-byte unit), every split's load issued
// before the first add.  Reduce block b takes a tile of XCD b % 8 when the tile count allows it
// (block_map's placement), so the partials are read from the L2 that holds them.
template <int RG, int NB>
__global__ __launch_bounds__(256) void wreduce_kernel(const uint16_t *__restrict__ P, uint16_t *__restrict__ C, int M,
                                                      int N, int ldc, int S, int tiles_m, int ntiles)
{
    constexpr int TPU = NB == 1 ? 1 : 2;
    constexpr int UNITS = NWAVE * RG * (NB / TPU) * 64; // per tile block
    constexpr int BPT = (UNITS + 255) / 256;            // reduce blocks per tile
    int tile, chunk;
    if (ntiles % 8 == 0) {
        const int i = blockIdx.x >> 3;
        tile = (blockIdx.x & 7) + 8 * (i / BPT);
        chunk = i % BPT;
    } else {
        tile = blockIdx.x / BPT;
        chunk = blockIdx.x % BPT;
    }
    const int q = chunk * 256 + threadIdx.x;
    if (tile >= ntiles || q >= UNITS) return;
    const int lane = q & 63, u = (q >> 6) % (NB / TPU), wr = (q >> 6) / (NB / TPU);
    const int wv = wr / RG;
    constexpr int BLK = NWAVE * RG * 16 * 16 * NB; // halves per block
    const int *es = (const int *)(P + (size_t)ntiles * S * BLK);
    f32x4 acc[TPU];
#pragma unroll
    for (int j = 0; j < TPU; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < S; s0 += 8) {
        u32x4 v[8];
        float up[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int sp = tile * S + (s0 + i < S ? s0 + i : S - 1); // unconditional loads
            if constexpr (TPU == 2) {
                v[i] = ((const u32x4 *)(P + (size_t)sp * BLK))[q];
            } else {
                const u32x2 w = ((const u32x2 *)(P + (size_t)sp * BLK))[q];
                v[i] = (u32x4){w.x, w.y, 0u, 0u};
            }
            up[i] = __builtin_bit_cast(float, (uint32_t)(127 + es[sp * NWAVE + wv]) << 23);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (s0 + i >= S) break;
#pragma unroll
            for (int j = 0; j < TPU; ++j) {
                const uint32_t lo = j ? v[i].z : v[i].x, hi = j ? v[i].w : v[i].y;
                acc[j][0] += h2f(lo & 0xffffu) * up[i];
                acc[j][1] += h2f(lo >> 16) * up[i];
                acc[j][2] += h2f(hi & 0xffffu) * up[i];
                acc[j][3] += h2f(hi >> 16) * up[i];
            }
        }
    }
    const int tm = tile % tiles_m, tn = tile / tiles_m;
    const int row = tm * (16 * NWAVE * RG) + 16 * wr + 4 * (lane >> 4);
    if (row >= M) return;
#pragma unroll
    for (int j = 0; j < TPU; ++j) {
        const int tok = tn * 16 * NB + 16 * (TPU * u + j) + (lane & 15);
        if (tok >= N) continue;
        uint16_t *dst = C + (size_t)tok * ldc + row;
        if (row + 4 <= M) {
            *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(acc[j][0]) | ((uint32_t)f2h_bits(acc[j][1]) << 16),
                                    (uint32_t)f2h_bits(acc[j][2]) | ((uint32_t)f2h_bits(acc[j][3]) << 16)};
        } else {
            for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(acc[j][i]);
        }
    }
}

template <int F, int RG, int NB>
hipError_t launch_cfg(const uint8_t *A, const uint16_t *X, uint16_t *C, uint16_t *P, const WGemmPlan &pl, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    const int ntiles = pl.tiles_m * pl.tiles_n;
    wgemm_kernel<F, RG, NB><<<dim3((unsigned)(ntiles * pl.splits)), dim3(THREADS), 0, s>>>(
        A, X, C, P, (int)M, (int)N, (int)K, (int)ldc, pl.tiles_m, pl.splits, pl.sb_per_split);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || pl.splits == 1) return e;
    constexpr int TPU = NB == 1 ? 1 : 2;
    constexpr int UNITS = NWAVE * RG * (NB / TPU) * 64, BPT = (UNITS + 255) / 256;
    wreduce_kernel<RG, NB><<<dim3((unsigned)(ntiles * BPT)), dim3(256), 0, s>>>(P, C, (int)M, (int)N, (int)ldc,
                                                                               pl.splits, pl.tiles_m, ntiles);
    return hipGetLastError();
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const uint16_t *X, uint16_t *C, uint16_t *P, const WGemmPlan &pl, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (pl.rg == 1) switch (pl.nb) {
        case 2: return launch_cfg<F, 1, 2>(A, X, C, P, pl, M, N, K, ldc, s);
        case 4: return launch_cfg<F, 1, 4>(A, X, C, P, pl, M, N, K, ldc, s);
        case 8: return launch_cfg<F, 1, 8>(A, X, C, P, pl, M, N, K, ldc, s);
        default: return hipErrorInvalidValue;
        }
    switch (pl.nb) {
    case 2: return launch_cfg<F, 2, 2>(A, X, C, P, pl, M, N, K, ldc, s);
    case 4: return launch_cfg<F, 2, 4>(A, X, C, P, pl, M, N, K, ldc, s);
    case 8: return launch_cfg<F, 2, 8>(A, X, C, P, pl, M, N, K, ldc, s);
    default: return hipErrorInvalidValue;
    }
}

} // namespace

WGemmPlan plan_wgemm(int fmt, int64_t M, int64_t N, int64_t K, int rg, int nb, int splits)
{
    WGemmPlan p;
    (void)fmt;
    p.rg = rg == 1 ? 1 : 2;
    p.nb = nb == 2 || nb == 4 ? nb : 8;
    const int64_t bm = 16 * NWAVE * p.rg, bn = 16 * p.nb;
    p.tiles_m = (int)((M + bm - 1) / bm);
    p.tiles_n = (int)((N + bn - 1) / bn);
    const int64_t nsb = K / 256, tiles = (int64_t)p.tiles_m * p.tiles_n;
    int64_t S = splits > 0 ? splits : (tiles >= 256 ? 1 : 256 / tiles);
    if (S > nsb) S = nsb;
    if (S < 1) S = 1;
    const int64_t sps = (nsb + S - 1) / S;
    S = (nsb + sps - 1) / sps;
    p.splits = (int)S;
    p.sb_per_split = (int)sps;
    p.partial_bytes = S > 1 ? (size_t)S * tiles * bm * bn * 2 + (size_t)S * tiles * NWAVE * sizeof(int) : 0;
    return p;
}

hipError_t launch_wgemm(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, void *partials,
                        const WGemmPlan &plan, int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    uint16_t *P = (uint16_t *)partials;
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, X, C, P, plan, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, X, C, P, plan, M, N, K, ldc, s);
    default: return launch_fmt<Q6_K>(A, X, C, P, plan, M, N, K, ldc, s);
    }
}

} // namespace gq
