// gguf_mfma.hpp -- what the fp16-MFMA GEMM kernels share (mmq_gemm.hip, mmq_rgemm.hip): the
// operand types, the in-register dequantization of one row's weight stage into MFMA A
// fragments (stage_frags), the LDS stage geometry of each format (WStage) and the activation
// sub-stage addressing and swizzle.
//
// MFMA 16x16x32 f16 maps (gfx950): lane l holds A[row l&15][k 8(l>>4)+j] and B[k 8(l>>4)+j]
// [col l&15]; D[row 4(l>>4)+i][col l&15] in acc element i.  The 8 k of an f16 fragment are
// taken in the element order (0,2,1,3,4,6,5,7) in which packed dequantization produces them;
// act_quant's DEQ form stores x~ in the same order.
#pragma once
#include "gguf_blocks.hpp"

namespace gq {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;


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

constexpr int KC = 64; // K elements per activation sub-stage

// ---------------------------------------------------------------------------------------
// Weight stages are one super-block of K (256 elements; Q8_0: 8 blocks) per row, moved as
// the row's contiguous bytes (16-byte pieces from a 16-byte aligned window: full cache lines,
// the shape HBM streams at its full rate).  Activation sub-stages are 64 elements.
// Per format: RBW = LDS bytes per row per weight stage (pieces NPW = RBW / 16), SB = packed
// bytes per stage.  Q6_K super-blocks are only 2-byte aligned: each is moved as 16-byte pieces
// read from its own first byte (2-byte aligned DMA sources) into a 240-B image whose every
// field is aligned (the d piece repeated at 208..223, d at 222).
// SPW = activation sub-stages per weight stage (4: one super-block; one sub-stage per weight
// stage for Q8_0 was measured no faster and removed: profiles/r02/q8_0_fine_stages_ab.txt).
template <int F> struct WStage;
template <> struct WStage<Q4_K> { static constexpr int RBW = 144, SB = 144, SPW = 4; };
// Q6_K rows are padded to 240 B (15 pieces, the last a repeat of the d piece): a 224-B stride
// (56 dwords) put rows l and l+8 of a 16-lane fragment read on the same banks (2-way
// conflicts, ~half of the LDS cycles measured); 60 dwords spread 16 rows over distinct banks.
template <> struct WStage<Q6_K> { static constexpr int RBW = 240, SB = 210, SPW = 4; };
template <> struct WStage<Q8_0> {
    static constexpr int SPW = 4, RBW = 272, SB = SPW * 68;
};

// Activation sub-stage c (64 elements) = sub-stage s4 = c & 3 of super-block c >> 2: the K
// elements whose weights the k-steps read (Q6_K: two 32-element runs, see frags below).
template <int F>
__device__ __forceinline__ uint32_t act_soff(int64_t c)
{
    if constexpr (F == Q6_K) return (uint32_t)(2 * (256 * (c >> 2) + 128 * ((c >> 1) & 1) + 32 * (c & 1)));
    return (uint32_t)(2 * KC * c);
}
template <int F>
__device__ __forceinline__ uint32_t act_voff(int p) // byte offset of piece p (8 elements) in the sub-stage
{
    if constexpr (F == Q6_K) return 2u * (64 * (p >> 2) + 8 * (p & 3));
    return 16u * p;
}

// ---------------------------------------------------------------------------------------
// A fragments of sub-stage s4 for this lane's row: frag[s] = the 8 weights (fragment element
// order) of k-step s, k-group g.  wr = the row's stage bytes in LDS (block byte 0).
// sx: byte-offset XOR of the row's image (Q6_K 256-row tiles, Cfg::Q6S; 0 otherwise).
template <int F>
__device__ __forceinline__ void stage_frags(const uint8_t *wr, int g, int s4, f16x8 (&frag)[2], int sx);

// Q4_K sub-stage q: sub-blocks 2q (low nibbles) and 2q+1 (high nibbles) of qs bytes 32q..+32:
// hdr = the super-block's first 16 bytes (d, dmin, scales), w = qs + 32q.
__device__ __forceinline__ void q4k_frags(const uint8_t *hdrp, const uint8_t *w32, int g, int q, f16x8 (&frag)[2])
{
    const u32x4 hdr = *(const u32x4 *)hdrp;
    const float d = h2f(hdr.x & 0xffffu), dmin = h2f(hdr.x >> 16);
    // 6-bit scales / mins of sub-blocks 2q, 2q+1, one per byte (get_scale_min_k4)
    const uint32_t sc = q < 2 ? (hdr.y & 0x3f3f3f3fu) : ((hdr.w & 0x0f0f0f0fu) | ((hdr.y >> 2) & 0x30303030u));
    const uint32_t mn = q < 2 ? (hdr.z & 0x3f3f3f3fu) : (((hdr.w >> 4) & 0x0f0f0f0fu) | ((hdr.z >> 2) & 0x30303030u));
    const int sh = 16 * (q & 1);
    const u32x2 w = *(const u32x2 *)(w32 + 8 * g);
    const h2 bias = splat(-1024.f);
#pragma unroll
    for (int n = 0; n < 2; ++n) { // n = 0: low nibbles (sub-block 2q), 1: high (2q+1)
        const h2 ds = splat(d * (float)((sc >> (sh + 8 * n)) & 0xffu));
        const h2 ndm = splat(-(dmin * (float)((mn >> (sh + 8 * n)) & 0xffu)));
        // the nibbles as bytes, then (1024 + code) pairs by byte permutes: one mask per word and
        // one v_perm per pair (the same values as masking each pair into 0x6400 0x6400)
        const uint32_t x0 = (w.x >> (4 * n)) & 0x0f0f0f0fu, x1 = (w.y >> (4 * n)) & 0x0f0f0f0fu;
        frag[n] = frag4(__builtin_elementwise_fma(pair02(x0) + bias, ds, ndm),
                        __builtin_elementwise_fma(pair13(x0) + bias, ds, ndm),
                        __builtin_elementwise_fma(pair02(x1) + bias, ds, ndm),
                        __builtin_elementwise_fma(pair13(x1) + bias, ds, ndm));
    }
}
template <>
__device__ __forceinline__ void stage_frags<Q4_K>(const uint8_t *wr, int g, int q, f16x8 (&frag)[2], int)
{
    q4k_frags(wr, wr + 16 + 32 * q, g, q, frag);
}

// Q6_K sub-stage (h, v) from a half-super-block image (mmq_rgemm.hip): ql bytes 64h..64h+63 at
// 0, qh bytes 128+32h.. at 64, scales (bytes 192..207) at 96, bytes 194..209 at 112 (d at 126);
// the arithmetic of stage_frags<Q6_K> below.
__device__ __forceinline__ void q6k_half_frags(const uint8_t *img, int g, int h, int v, f16x8 (&frag)[2])
{
    const float d = h2f(*(const uint16_t *)(img + 126));
    const u32x2 ql = *(const u32x2 *)(img + 32 * v + 8 * g);
    const u32x2 qh = *(const u32x2 *)(img + 64 + 8 * g);
    const h2 bias = splat(-1056.f); // 1024 + 32
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const float scv = (float)*(const int8_t *)(img + 96 + 8 * h + 4 * n + 2 * v + (g >> 1));
        const h2 dsc = splat(d * scv);
        const int sq = 4 * n + 2 * v;
        const uint32_t c0 = ((ql.x >> (4 * n)) & 0x0f0f0f0fu) | (((qh.x >> sq) & 0x03030303u) << 4);
        const uint32_t c1 = ((ql.y >> (4 * n)) & 0x0f0f0f0fu) | (((qh.y >> sq) & 0x03030303u) << 4);
        frag[n] = frag4((pair02(c0) + bias) * dsc, (pair13(c0) + bias) * dsc, (pair02(c1) + bias) * dsc,
                        (pair13(c1) + bias) * dsc);
    }
}

// Q6_K sub-stage s4 = (h, v): k-step 0 = elements 128h+32v+[0,32) (ql[64h+32v..] low nibbles,
// qh bits 2v), k-step 1 = 128h+64+32v+[0,32) (same ql bytes, high nibbles; qh bits 4+2v).
template <>
__device__ __forceinline__ void stage_frags<Q6_K>(const uint8_t *wr, int g, int s4, f16x8 (&frag)[2], int sx)
{
    const int h = s4 >> 1, v = s4 & 1;
    const float d = h2f(*(const uint16_t *)(wr + (222 ^ sx))); // image: d at 222 (see issue_w)
    const u32x2 ql = *(const u32x2 *)(wr + ((64 * h + 32 * v + 8 * g) ^ sx));
    const u32x2 qh = *(const u32x2 *)(wr + ((128 + 32 * h + 8 * g) ^ sx));
    const h2 bias = splat(-1056.f); // 1024 + 32
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        // sub-block of elements 128h + 64n + 32v + 8g..: 8h + 4n + 2v + (g >> 1)
        const float scv = (float)*(const int8_t *)(wr + ((192 + 8 * h + 4 * n + 2 * v + (g >> 1)) ^ sx));
        const h2 dsc = splat(d * scv);
        const int sq = 4 * n + 2 * v;
        const uint32_t c0 = ((ql.x >> (4 * n)) & 0x0f0f0f0fu) | (((qh.x >> sq) & 0x03030303u) << 4);
        const uint32_t c1 = ((ql.y >> (4 * n)) & 0x0f0f0f0fu) | (((qh.y >> sq) & 0x03030303u) << 4);
        frag[n] = frag4((pair02(c0) + bias) * dsc, (pair13(c0) + bias) * dsc, (pair02(c1) + bias) * dsc,
                        (pair13(c1) + bias) * dsc);
    }
}

// Q8_0 sub-stage u: blocks 2u, 2u+1 of the stage's 8.  The 8 code bytes of a lane start 2, 4
// or 6 bytes past an 8-byte boundary (34-byte blocks): unaligned ds_read_b64 stall the LDS
// (SQ_LDS_UNALIGNED_STALL), so two aligned 8-byte reads and a byte shift (the offset is the
// same for every lane of the sub-stage) are used instead (GQ_Q8_UNALIGNED=1: the direct read).
#ifndef GQ_Q8_UNALIGNED
#define GQ_Q8_UNALIGNED 0
#endif
template <>
__device__ __forceinline__ void stage_frags<Q8_0>(const uint8_t *wr, int g, int u, f16x8 (&frag)[2], int)
{
    const h2 bias = splat(-1152.f); // codes biased by +128 (xor 0x80)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const uint8_t *blk = wr + 34 * (2 * u + b);
        const h2 d = splat(h2f(*(const uint16_t *)blk));
#if GQ_Q8_UNALIGNED
        const u32x2 q = *(const u32x2 *)(blk + 2 + 8 * g); // 2-byte aligned: gfx950 LDS runs unaligned
#else
        // wr is 16-byte aligned (RBW = 272): the shift depends on u and b only
        const int off = 34 * (2 * u + b) + 2, sh = off & 7;
        const uint8_t *al = wr + (off & ~7) + 8 * g;
        const u32x2 lo = *(const u32x2 *)al, hi = *(const u32x2 *)(al + 8);
        u32x2 q;
        if (sh == 0) q = lo;
        else if (sh < 4) q = (u32x2){__builtin_amdgcn_alignbyte(lo.y, lo.x, sh), __builtin_amdgcn_alignbyte(hi.x, lo.y, sh)};
        else if (sh == 4) q = (u32x2){lo.y, hi.x};
        else q = (u32x2){__builtin_amdgcn_alignbyte(hi.x, lo.y, sh - 4), __builtin_amdgcn_alignbyte(hi.y, hi.x, sh - 4)};
#endif
        const uint32_t c0 = q.x ^ 0x80808080u, c1 = q.y ^ 0x80808080u;
        frag[b] = frag4((pair02(c0) + bias) * d, (pair13(c0) + bias) * d, (pair02(c1) + bias) * d,
                        (pair13(c1) + bias) * d);
    }
}

// AUX = cache policy of the DMA (2 = nt; nt on the weight stream measured 2-7% slower and was
// removed, as were an activation-first and a serialized prologue: profiles/r02/*_rejected.txt)
template <int AUX = 0>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, uint8_t *lds_dst, uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void *)lds_dst, 16, voff, soff, 0, AUX);
}

__device__ __forceinline__ int act_swz(int r) { return (r >> 1) & 7; }
// Code rows are 64 B (four 16-byte pieces): piece q of token r lands in piece q ^ i8_swz(r),
// so the 8-byte fragment reads of 16 tokens x 2 k-groups cover all 64 banks once.
__device__ __forceinline__ int i8_swz(int r) { return (r >> 2) & 3; }

} // namespace gq
