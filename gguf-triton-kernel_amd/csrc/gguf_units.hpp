// gguf_units.hpp -- per-lane "unit" loaders shared by the GEMV and the MFMA GEMM.
//
// A unit is 64 weights of one row that one lane owns: unit u of a row covers
//   Q8_0 : blocks 2u, 2u+1 (bytes 68u .. 68u+67 of the row)
//   Q4_K : super-block u/4, sub-blocks 2(u%4), 2(u%4)+1 (qs bytes 32(u%4)..+31, both nibbles)
//   Q6_K : super-block u/4, half h=(u>>1)&1, v=u&1: elements 128h+32v+[0,32) ("A") and
//          128h+64+32v+[0,32) ("B") -- ql bytes 64h+32v..+31 (both nibbles), qh 32h..+31
// so two consecutive units (2c, 2c+1) tile K-chunk c of 128 elements.  Every unit needs
// 16-byte loads only (Q8_0/Q6_K fields are 2-byte aligned: unaligned dwordx4, which
// gfx950 serves in unaligned mode).  act_blocks() gives the two 32-element activation
// blocks a unit multiplies with.
#pragma once
#include "gguf_blocks.hpp"

namespace gq {

template <int F>
__device__ __forceinline__ void act_blocks(int u, int &b0, int &b1)
{
    if constexpr (F == Q6_K) {
        const int sb = u >> 2, h = (u >> 1) & 1, v = u & 1;
        b0 = 8 * sb + 4 * h + v;
        b1 = b0 + 2;
    } else {
        b0 = 2 * u;
        b1 = 2 * u + 1;
    }
}

// A unit is handled in two steps so that loads can be issued far ahead of their use:
//   UnitLoad<F>::load()  issues the unit's loads and keeps the raw registers (no arithmetic,
//                        so nothing waits for the loads here);
//   UnitRaw<F>::from()   decodes them (scales, code bytes) when the unit is consumed.
template <int F> struct UnitLoad;
template <int F> struct UnitRaw;

// N dwords starting at a 2-byte aligned LDS address p, read as dword-aligned words and shifted
// into place: an LDS read that is not dword-aligned stalls the LDS pipeline
// (SQ_LDS_UNALIGNED_STALL was ~90% of the Q6_K/Q8_0 decode kernels' LDS cycles).
template <int N>
__device__ __forceinline__ void lds_words(const uint8_t *p, uint32_t (&o)[N])
{
    const uint32_t *a = (const uint32_t *)((uintptr_t)p & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(uintptr_t)p & 3u;
    uint32_t w[N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k) w[k] = a[k];
#pragma unroll
    for (int k = 0; k < N; ++k) o[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
}

// ---- Q8_0: two blocks ----
template <> struct UnitLoad<Q8_0> {
    uint32_t d0b, d1b;
    u32x4 a0, a1, a2, a3;
    __device__ __forceinline__ void load(const uint8_t *__restrict__ rowp, int u, int64_t nb32)
    {
        // unconditional loads: a missing second block re-reads the first (its d is zeroed later)
        const uint8_t *p = rowp + 68 * (int64_t)u;
        const bool has0 = 2 * (int64_t)u < nb32, has1 = 2 * (int64_t)u + 1 < nb32;
        const uint8_t *p0 = has0 ? p : rowp, *p1 = has1 ? p + 34 : p0;
        d0b = ld2(p0);
        d1b = ld2(p1);
        a0 = ld16(p0 + 2);
        a1 = ld16(p0 + 18);
        a2 = ld16(p1 + 2);
        a3 = ld16(p1 + 18);
    }
    // from LDS (the decode ring): the block pair as 17 dword-aligned words (p is 4-byte
    // aligned there); a missing second block reads bytes of no consequence (its d is zeroed)
    __device__ __forceinline__ void load_lds(const uint8_t *__restrict__ rowp, int u, int64_t /*nb32*/)
    {
        const uint32_t *w = (const uint32_t *)(rowp + 68 * u);
        uint32_t x[17];
#pragma unroll
        for (int k = 0; k < 17; ++k) x[k] = w[k];
        d0b = x[0] & 0xffffu;
        d1b = x[8] >> 16;
        uint32_t c[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_alignbyte(x[k + 1], x[k], 2);
        a0 = (u32x4){c[0], c[1], c[2], c[3]};
        a1 = (u32x4){c[4], c[5], c[6], c[7]};
        a2 = (u32x4){x[9], x[10], x[11], x[12]};
        a3 = (u32x4){x[13], x[14], x[15], x[16]};
    }
};

template <> struct UnitRaw<Q8_0> {
    float d0, d1;
    uint32_t w[16]; // int8 codes: w[0..7] block 2u, w[8..15] block 2u+1

    __device__ __forceinline__ static UnitRaw from(const UnitLoad<Q8_0> &l, int u, int64_t nb32)
    {
        UnitRaw r;
        r.d0 = 2 * (int64_t)u < nb32 ? h2f(l.d0b) : 0.f;
        r.d1 = 2 * (int64_t)u + 1 < nb32 ? h2f(l.d1b) : 0.f;
        const u32x4 v[4] = {l.a0, l.a1, l.a2, l.a3};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            r.w[4 * i] = v[i].x;
            r.w[4 * i + 1] = v[i].y;
            r.w[4 * i + 2] = v[i].z;
            r.w[4 * i + 3] = v[i].w;
        }
        return r;
    }
};

// ---- Q4_K: one quarter of a super-block ----
template <> struct UnitLoad<Q4_K> {
    u32x4 hdr, qa, qb;
    __device__ __forceinline__ void load(const uint8_t *__restrict__ rowp, int u, int64_t /*nb32*/)
    {
        const int sb = u >> 2, q = u & 3;
        const uint8_t *p = rowp + 144 * (int64_t)sb;
        hdr = ld16(p);
        qa = ld16(p + 16 + 32 * q);
        qb = ld16(p + 32 + 32 * q);
    }
};

template <> struct UnitRaw<Q4_K> {
    float ds0, dm0, ds1, dm1; // d*sc and dmin*m of the two sub-blocks
    uint32_t w[8];            // 32 qs bytes: low nibbles = first sub-block, high = second

    __device__ __forceinline__ static UnitRaw from(const UnitLoad<Q4_K> &l, int u, int64_t /*nb32*/)
    {
        UnitRaw r;
        const int q = u & 3;
        const float d = h2f(l.hdr.x & 0xffffu), dmin = h2f(l.hdr.x >> 16);
        const uint32_t sw[3] = {l.hdr.y, l.hdr.z, l.hdr.w};
        int sc0, m0, sc1, m1;
        q4k_sc_m(sw, 2 * q, sc0, m0);
        q4k_sc_m(sw, 2 * q + 1, sc1, m1);
        r.ds0 = d * (float)sc0;
        r.dm0 = dmin * (float)m0;
        r.ds1 = d * (float)sc1;
        r.dm1 = dmin * (float)m1;
        r.w[0] = l.qa.x; r.w[1] = l.qa.y; r.w[2] = l.qa.z; r.w[3] = l.qa.w;
        r.w[4] = l.qb.x; r.w[5] = l.qb.y; r.w[6] = l.qb.z; r.w[7] = l.qb.w;
        return r;
    }
};

// ---- Q6_K: two 32-element runs of one super-block half ----
template <> struct UnitLoad<Q6_K> {
    u32x4 l0, l1, g0, g1;
    u32x2 sc8;
    uint32_t dbits;
    __device__ __forceinline__ void load(const uint8_t *__restrict__ rowp, int u, int64_t /*nb32*/)
    {
        const int sb = u >> 2, h = (u >> 1) & 1, v = u & 1;
        const uint8_t *p = rowp + 210 * (int64_t)sb;
        l0 = ld16(p + 64 * h + 32 * v);
        l1 = ld16(p + 64 * h + 32 * v + 16);
        g0 = ld16(p + 128 + 32 * h);
        g1 = ld16(p + 144 + 32 * h);
        sc8 = ld8(p + 192 + 8 * h);
        dbits = ld2(p + 208);
    }
    // from LDS (the decode ring): every field has the block's 2-byte misalignment
    __device__ __forceinline__ void load_lds(const uint8_t *__restrict__ rowp, int u, int64_t /*nb32*/)
    {
        const int sb = u >> 2, h = (u >> 1) & 1, v = u & 1;
        const uint8_t *p = rowp + 210 * (int64_t)sb;
        uint32_t l[8], g[8], s[2];
        lds_words<8>(p + 64 * h + 32 * v, l);
        lds_words<8>(p + 128 + 32 * h, g);
        lds_words<2>(p + 192 + 8 * h, s);
        l0 = (u32x4){l[0], l[1], l[2], l[3]};
        l1 = (u32x4){l[4], l[5], l[6], l[7]};
        g0 = (u32x4){g[0], g[1], g[2], g[3]};
        g1 = (u32x4){g[4], g[5], g[6], g[7]};
        sc8 = (u32x2){s[0], s[1]};
        dbits = *(const uint16_t *)(p + 208);
    }
    // from the decode ring's aligned image (mmq_decode.hip, kImgSB): super-blocks at a 224-byte
    // stride, bytes 0..207 as packed, d at 222 -- every field at its natural alignment
    __device__ __forceinline__ void load_img(const uint8_t *__restrict__ rowp, int u)
    {
        const int sb = u >> 2, h = (u >> 1) & 1, v = u & 1;
        const uint8_t *p = rowp + 224 * sb;
        l0 = *(const u32x4 *)(p + 64 * h + 32 * v);
        l1 = *(const u32x4 *)(p + 64 * h + 32 * v + 16);
        g0 = *(const u32x4 *)(p + 128 + 32 * h);
        g1 = *(const u32x4 *)(p + 144 + 32 * h);
        sc8 = *(const u32x2 *)(p + 192 + 8 * h);
        dbits = *(const uint16_t *)(p + 222);
    }
};

template <> struct UnitRaw<Q6_K> {
    float fa1, fa2, fb1, fb2; // d*sc for the four 16-element sub-blocks (A lo, A hi, B lo, B hi)
    uint32_t ca[8], cb[8];     // 6-bit codes (0..63) of run A and run B, one per byte

    __device__ __forceinline__ static UnitRaw from(const UnitLoad<Q6_K> &l, int u, int64_t /*nb32*/)
    {
        UnitRaw r;
        const int v = u & 1;
        const float d = h2f(l.dbits);
        const uint32_t ql[8] = {l.l0.x, l.l0.y, l.l0.z, l.l0.w, l.l1.x, l.l1.y, l.l1.z, l.l1.w};
        const uint32_t qh[8] = {l.g0.x, l.g0.y, l.g0.z, l.g0.w, l.g1.x, l.g1.y, l.g1.z, l.g1.w};
        const int shA = 2 * v, shB = 4 + 2 * v;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            r.ca[i] = (ql[i] & 0x0f0f0f0fu) | (((qh[i] >> shA) & 0x03030303u) << 4);
            r.cb[i] = ((ql[i] >> 4) & 0x0f0f0f0fu) | (((qh[i] >> shB) & 0x03030303u) << 4);
        }
        const uint32_t sA = v ? (l.sc8.x >> 16) : l.sc8.x;
        const uint32_t sB = v ? (l.sc8.y >> 16) : l.sc8.y;
        r.fa1 = d * (float)(int8_t)(sA & 0xff);
        r.fa2 = d * (float)(int8_t)((sA >> 8) & 0xff);
        r.fb1 = d * (float)(int8_t)(sB & 0xff);
        r.fb2 = d * (float)(int8_t)((sB >> 8) & 0xff);
        return r;
    }
};

} // namespace gq
