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

template <int F> struct UnitRaw;

// ---- Q8_0: two blocks ----
template <> struct UnitRaw<Q8_0> {
    float d0, d1;
    uint32_t w[16]; // int8 codes: w[0..7] block 2u, w[8..15] block 2u+1

    __device__ __forceinline__ void load(const uint8_t *__restrict__ rowp, int u, int64_t nb32)
    {
        const uint8_t *p = rowp + 68 * (int64_t)u;
        const bool has0 = 2 * (int64_t)u < nb32, has1 = 2 * (int64_t)u + 1 < nb32;
        u32x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
        d0 = 0.f;
        d1 = 0.f;
        if (has0) {
            d0 = h2f(ld2(p));
            a0 = ld16(p + 2);
            a1 = ld16(p + 18);
        }
        if (has1) {
            d1 = h2f(ld2(p + 34));
            a2 = ld16(p + 36);
            a3 = ld16(p + 52);
        }
        w[0] = a0.x; w[1] = a0.y; w[2] = a0.z; w[3] = a0.w;
        w[4] = a1.x; w[5] = a1.y; w[6] = a1.z; w[7] = a1.w;
        w[8] = a2.x; w[9] = a2.y; w[10] = a2.z; w[11] = a2.w;
        w[12] = a3.x; w[13] = a3.y; w[14] = a3.z; w[15] = a3.w;
    }
};

// ---- Q4_K: one quarter of a super-block ----
template <> struct UnitRaw<Q4_K> {
    float ds0, dm0, ds1, dm1; // d*sc and dmin*m of the two sub-blocks
    uint32_t w[8];            // 32 qs bytes: low nibbles = first sub-block, high = second

    __device__ __forceinline__ void load(const uint8_t *__restrict__ rowp, int u, int64_t /*nb32*/)
    {
        const int sb = u >> 2, q = u & 3;
        const uint8_t *p = rowp + 144 * (int64_t)sb;
        const u32x4 hdr = ld16(p);
        const u32x4 qa = ld16(p + 16 + 32 * q), qb = ld16(p + 32 + 32 * q);
        const float d = h2f(hdr.x & 0xffffu), dmin = h2f(hdr.x >> 16);
        const uint32_t sw[3] = {hdr.y, hdr.z, hdr.w};
        int sc0, m0, sc1, m1;
        q4k_sc_m(sw, 2 * q, sc0, m0);
        q4k_sc_m(sw, 2 * q + 1, sc1, m1);
        ds0 = d * (float)sc0;
        dm0 = dmin * (float)m0;
        ds1 = d * (float)sc1;
        dm1 = dmin * (float)m1;
        w[0] = qa.x; w[1] = qa.y; w[2] = qa.z; w[3] = qa.w;
        w[4] = qb.x; w[5] = qb.y; w[6] = qb.z; w[7] = qb.w;
    }
};

// ---- Q6_K: two 32-element runs of one super-block half ----
template <> struct UnitRaw<Q6_K> {
    float fa1, fa2, fb1, fb2; // d*sc for the four 16-element sub-blocks (A lo, A hi, B lo, B hi)
    uint32_t ca[8], cb[8];     // 6-bit codes (0..63) of run A and run B, one per byte

    __device__ __forceinline__ void load(const uint8_t *__restrict__ rowp, int u, int64_t /*nb32*/)
    {
        const int sb = u >> 2, h = (u >> 1) & 1, v = u & 1;
        const uint8_t *p = rowp + 210 * (int64_t)sb;
        const u32x4 l0 = ld16(p + 64 * h + 32 * v), l1 = ld16(p + 64 * h + 32 * v + 16);
        const u32x4 g0 = ld16(p + 128 + 32 * h), g1 = ld16(p + 144 + 32 * h);
        const u32x2 sc8 = ld8(p + 192 + 8 * h);
        const float d = h2f(ld2(p + 208));
        const uint32_t ql[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
        const uint32_t qh[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        const int shA = 2 * v, shB = 4 + 2 * v;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            ca[i] = (ql[i] & 0x0f0f0f0fu) | (((qh[i] >> shA) & 0x03030303u) << 4);
            cb[i] = ((ql[i] >> 4) & 0x0f0f0f0fu) | (((qh[i] >> shB) & 0x03030303u) << 4);
        }
        const uint32_t sA = v ? (sc8.x >> 16) : sc8.x;
        const uint32_t sB = v ? (sc8.y >> 16) : sc8.y;
        fa1 = d * (float)(int8_t)(sA & 0xff);
        fa2 = d * (float)(int8_t)((sA >> 8) & 0xff);
        fb1 = d * (float)(int8_t)(sB & 0xff);
        fb2 = d * (float)(int8_t)((sB >> 8) & 0xff);
    }
};

} // namespace gq
