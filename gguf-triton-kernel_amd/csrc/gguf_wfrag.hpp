// gguf_wfrag.hpp -- GGUF weight fragments straight from HBM into registers, dequantized to the
// A operand of v_mfma_f32_16x16x32_f16 (the skinny-token kernel, mmq_skinny.hip).
//
// WB<F>: one super-block (256 K elements; Q8_0: 8 blocks) of one 16-row fragment -- lane
// (row c = lane&15, group g = lane>>4) loads its bytes with 16-byte buffer loads and produces
// the fp16 A fragment of k-step s = 0..7; WB<F>::e(s, g) is the first of the 8 consecutive
// elements (in act_quant's DEQ order) lane group g supplies at k-step s, so the B fragment is
// the 16 bytes of x~ at that element.
#pragma once

#include "gguf_blocks.hpp"

namespace gq {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));


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

__device__ __forceinline__ u32x4 bl16(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, v, s, 0);
}
__device__ __forceinline__ uint32_t bl4(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s)
{
    return __builtin_amdgcn_raw_buffer_load_b32(r, v, s, 0);
}
__device__ __forceinline__ uint32_t wo(uint32_t v) { return v; } // (the weight byte offset as loaded)

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
    // e(2j + kk, g) = base(j) + off(kk, g)
    static __device__ __forceinline__ int base(int j) { return 128 * (j >> 1) + 32 * (j & 1); }
    static __device__ __forceinline__ int off(int kk, int g) { return 64 * (g >> 1) + 16 * (g & 1) + 8 * kk; }
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
// A 210-byte super-block starts only 2-byte aligned, and 16-byte loads at addresses = 2 mod 4 run
// at ~3/4 of the aligned rate (measured: profiles/r03/wgemm_align_probe.log): every chunk is
// loaded from 4-byte aligned `addr - sh` (sh = addr & 2) with one trailing dword, and realigned
// by v_alignbyte where a word is used; the scales' trailing dword is the one holding d.
template <> struct WB<Q6_K> {
    static constexpr int SB = 210;
    u32x4 ql[2], qh[2];
    uint32_t qle[2], qhe[2]; // the dword after each chunk
    u32x4 sc;                // the 16 int8 scales
    uint32_t d;              // bytes 206..209: d in the high half
    uint32_t sh;             // 0 or 2: the chunks' byte shift
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t v, int g, uint32_t s0)
    {
        // (the shift is folded into the per-lane offset: the buffer's range check applies to the
        // VGPR offset alone, so v - sh must not wrap below 0 at row 0)
        const uint32_t a = v + s0;
        sh = a & 2u;
        const uint32_t vb = a - sh;
        ql[0] = bl16(r, wo(vb + 16 * g), 0);
        qle[0] = bl4(r, wo(vb + 16 * g + 16), 0);
        ql[1] = bl16(r, wo(vb + 64 + 16 * g), 0);
        qle[1] = bl4(r, wo(vb + 80 + 16 * g), 0);
        qh[0] = bl16(r, wo(vb + 128 + 16 * (g & 1)), 0);
        qhe[0] = bl4(r, wo(vb + 144 + 16 * (g & 1)), 0);
        qh[1] = bl16(r, wo(vb + 160 + 16 * (g & 1)), 0);
        qhe[1] = bl4(r, wo(vb + 176 + 16 * (g & 1)), 0);
        sc = bl16(r, wo(vb + 192), 0);
        d = bl4(r, wo(a + 206), 0);
    }
    // word i (0..3) of a chunk loaded sh bytes early, e = the dword after it
    __device__ __forceinline__ uint32_t word(const u32x4 &q, uint32_t e, int i) const
    {
        const uint32_t lo = i == 0 ? q.x : (i == 1 ? q.y : (i == 2 ? q.z : q.w));
        const uint32_t hi = i == 0 ? q.y : (i == 1 ? q.z : (i == 2 ? q.w : e));
        return __builtin_amdgcn_alignbyte(hi, lo, sh);
    }
    static __device__ __forceinline__ int e(int s, int g)
    {
        return 128 * (s >> 2) + 64 * ((s >> 1) & 1) + 32 * (g >> 1) + 16 * (g & 1) + 8 * (s & 1);
    }
    static __device__ __forceinline__ int base(int j) { return 128 * (j >> 1) + 64 * (j & 1); }
    static __device__ __forceinline__ int off(int kk, int g) { return 32 * (g >> 1) + 16 * (g & 1) + 8 * kk; }
    __device__ __forceinline__ f16x8 frag(int s, int g) const
    {
        const int h = s >> 2, nib = (s >> 1) & 1, half = s & 1;
        const uint32_t qx = word(ql[h], qle[h], 2 * half), qy = word(ql[h], qle[h], 2 * half + 1);
        const uint32_t hx = word(qh[h], qhe[h], 2 * half), hy = word(qh[h], qhe[h], 2 * half + 1);
        const int sq = 2 * (g >> 1) + 4 * nib;
        const uint32_t sw = word(sc, d, 2 * h + nib);
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
    static __device__ __forceinline__ int base(int j) { return 32 * (j >> 1) + 16 * (j & 1); }
    static __device__ __forceinline__ int off(int kk, int g) { return 64 * g + 8 * kk; }
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

} // namespace
} // namespace gq
