// gguf_q8_1.hpp -- the q8_1 block quantizer as a device routine (eight lanes per block).
//
// Bit-exact with utils/quantize/q8_1.py:18-70: d = fp16(amax/127) (0 for an all-zero
// block), q = clamp(rne(fp16(x / d')), +-127) with d' = 1 where d == 0,
// s = fp16(d * fp16(sum q)); fp16(x/d) equals torch's CPU fp16 division of finite inputs
// (see Division below).  Each of the 8 lanes of an aligned lane group
// holds 4 consecutive fp16 (two dwords); amax and sum(q) are reduced by xor shuffles inside
// the group, so every lane of the group must reach the call together.
//
// Division.  fp16(x / d) for fp16 x and d is computed as q = x*r, r = v_rcp_f32(d), plus one
// residual correction fma(fma(-q, d, x), r, q): an fp16/fp16 quotient lies more than 2^-23
// (relative) from every fp16 rounding midpoint, and the corrected quotient is within ~2^-24
// of it, so both round to the same fp16 value -- checked exhaustively over all fp16 pairs
// with every r within 1 ulp of 1/d by tools/q81_div_check.cpp.  Three VALU ops per element
// instead of the IEEE division sequence (div_scale x2, rcp, 5 fma, div_fmas, div_fixup).
#pragma once
#include "gguf_blocks.hpp"

namespace gq {

// fp16-exact x / d for fp16-valued x, d (see above); r ~ 1/d within 1 ulp
__device__ __forceinline__ float q81_div(float x, float d, float r)
{
    const float q = x * r;
    return __builtin_fmaf(__builtin_fmaf(-q, d, x), r, q);
}

struct Q81Lane {
    uint32_t codes; // this lane's 4 int8 codes, little endian
    float d;        // block scale (fp16 value)
    uint16_t dbits, sbits;
    int s4;         // (decode quantizer only) sum of the codes of this lane's quad
};

__device__ __forceinline__ Q81Lane q8_1_lane(uint32_t w0, uint32_t w1)
{
    const float x[4] = {h2f(w0 & 0xffff), h2f(w0 >> 16), h2f(w1 & 0xffff), h2f(w1 >> 16)};
    float amax = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
    amax = fmaxf(amax, __shfl_xor(amax, 1, 8));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 8));
    amax = fmaxf(amax, __shfl_xor(amax, 4, 8));
    Q81Lane r;
    r.dbits = amax != 0.f ? f2h_bits(q81_div(amax, 127.0f, 1.0f / 127.0f)) : (uint16_t)0;
    r.d = h2f(r.dbits);
    const float div = r.d == 0.f ? 1.0f : r.d;
    const float rdiv = __builtin_amdgcn_rcpf(div);
    int sum = 0;
    r.codes = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float q = __builtin_rintf(h2f(f2h_bits(q81_div(x[i], div, rdiv))));
        q = fminf(127.f, fmaxf(-127.f, q));
        const int qi = (int)q;
        sum += qi;
        r.codes |= (uint32_t)(qi & 0xff) << (8 * i);
    }
    sum += __shfl_xor(sum, 1, 8);
    sum += __shfl_xor(sum, 2, 8);
    sum += __shfl_xor(sum, 4, 8);
    r.sbits = f2h_bits(r.d * h2f(f2h_bits((float)sum)));
    return r;
}

// q8_1 of one 32-element block held by an aligned group of 8 lanes (4 elements each): the
// arithmetic of gguf_q8_1.hpp (bit-exact with utils/quantize/q8_1.py), with the group
// reductions on DPP quad permutes + one ds_swizzle (xor 4) instead of LDS permutes.
__device__ __forceinline__ Q81Lane q8_1_lane_dpp(uint32_t w0, uint32_t w1)
{
    const float x[4] = {h2f(w0 & 0xffff), h2f(w0 >> 16), h2f(w1 & 0xffff), h2f(w1 >> 16)};
    float amax = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax), 0xb1, 0xf, 0xf, false)));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax), 0x4e, 0xf, 0xf, false)));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, amax), 0x101f)));
    Q81Lane r;
    r.dbits = amax != 0.f ? f2h_bits(q81_div(amax, 127.0f, 1.0f / 127.0f)) : (uint16_t)0;
    r.d = h2f(r.dbits);
    const float div = r.d == 0.f ? 1.0f : r.d;
    const float rdiv = __builtin_amdgcn_rcpf(div);
    int sum = 0;
    r.codes = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float q = __builtin_rintf(h2f(f2h_bits(q81_div(x[i], div, rdiv))));
        q = fminf(127.f, fmaxf(-127.f, q));
        const int qi = (int)q;
        sum += qi;
        r.codes |= (uint32_t)(qi & 0xff) << (8 * i);
    }
    sum += __builtin_amdgcn_mov_dpp(sum, 0xb1, 0xf, 0xf, false);
    sum += __builtin_amdgcn_mov_dpp(sum, 0x4e, 0xf, 0xf, false);
    r.s4 = sum; // sum over this lane's quad (Q6_K: quads 0 and 1 = the 16-element halves)
    sum += __builtin_amdgcn_ds_swizzle(sum, 0x101f);
    r.sbits = f2h_bits(r.d * h2f(f2h_bits((float)sum)));
    return r;
}

// q8_1 of one 32-element block held by an aligned group of 4 lanes (8 elements, one 16-byte
// load, each): the same arithmetic again; the group reductions are two DPP quad permutes.
// codes = the lane's 8 codes (2 dwords); s4 = the sum over the lane pair (a 16-element half).
struct Q81Quad {
    uint32_t codes[2];
    float d;
    uint16_t sbits;
    int s4;
};

__device__ __forceinline__ Q81Quad q8_1_quad(u32x4 w)
{
    const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
    float x[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[2 * i] = h2f(wd[i] & 0xffff);
        x[2 * i + 1] = h2f(wd[i] >> 16);
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(x[i]));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax), 0xb1, 0xf, 0xf, false)));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax), 0x4e, 0xf, 0xf, false)));
    Q81Quad r;
    const uint16_t dbits = amax != 0.f ? f2h_bits(q81_div(amax, 127.0f, 1.0f / 127.0f)) : (uint16_t)0;
    r.d = h2f(dbits);
    const float div = r.d == 0.f ? 1.0f : r.d;
    const float rdiv = __builtin_amdgcn_rcpf(div);
    // The per-element tail on packed fp16 (deq_quad's): the fp16-exact quotients packed by one
    // v_cvt_pk_f16_f32 (RNE, = f2h_bits per element), rint + bias as q + 1536 (|q| < 512: the
    // sum's ulp is 1, so its round-to-nearest-even is rintf's), the clamp in the biased domain
    // [1409, 1663]; fp16(1536 + q) is 0x6600 + q, so the int8 code is its low byte (one v_perm
    // per 4 codes) and sum(q) one v_dot4 of the codes with ones -- the scalar loop's exact bits.
#ifdef GQ_Q81_SCALAR // (diagnostic A/B build: the scalar per-element loop)
    int sum = 0;
    r.codes[0] = r.codes[1] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float q = __builtin_rintf(h2f(f2h_bits(q81_div(x[i], div, rdiv))));
        q = fminf(127.f, fmaxf(-127.f, q));
        const int qi = (int)q;
        sum += qi;
        r.codes[i >> 2] |= (uint32_t)(qi & 0xff) << (8 * (i & 3));
    }
#else
    typedef _Float16 h2t __attribute__((ext_vector_type(2)));
    typedef float f2t __attribute__((ext_vector_type(2)));
    const h2t magic = {(_Float16)1536.f, (_Float16)1536.f};
    const h2t lo = {(_Float16)1409.f, (_Float16)1409.f}, hi = {(_Float16)1663.f, (_Float16)1663.f};
    uint32_t t[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const f2t qf = {q81_div(x[2 * p], div, rdiv), q81_div(x[2 * p + 1], div, rdiv)};
        h2t q = __builtin_convertvector(qf, h2t) + magic;
        q = __builtin_elementwise_min(__builtin_elementwise_max(q, lo), hi);
        t[p] = __builtin_bit_cast(uint32_t, q);
    }
    r.codes[0] = __builtin_amdgcn_perm(t[1], t[0], 0x06040200u);
    r.codes[1] = __builtin_amdgcn_perm(t[3], t[2], 0x06040200u);
    int sum = __builtin_amdgcn_sdot4((int)r.codes[1], 0x01010101, __builtin_amdgcn_sdot4((int)r.codes[0], 0x01010101, 0, false), false);
#endif
    sum += __builtin_amdgcn_mov_dpp(sum, 0xb1, 0xf, 0xf, false);
    r.s4 = sum; // lanes (0,1) and (2,3) of the group: the two 16-element halves
    sum += __builtin_amdgcn_mov_dpp(sum, 0x4e, 0xf, 0xf, false);
    r.sbits = f2h_bits(r.d * h2f(f2h_bits((float)sum)));
    return r;
}

// The DEQ form's x~ = fp16(d * q) of one 32-element block held by an aligned group of 4 lanes
// (8 elements each), bit-identical to q8_1_quad + the fp32 product act_quant.hip rounds (the
// same amax, d, fp16-exact quotient and clamp), with the per-element tail on packed fp16: the
// quotient rounded to fp16 by one pack, rint as (q + 1536) - 1536 (|q| < 512: the sum's ulp is
// 1, IEEE round-to-nearest-even = rintf), the clamp by packed min/max, and fp16(d * q) by one
// packed multiply (the exact product rounded once, as the fp32 product rounded to fp16).
// Returns the pairs (x0,x2), (x1,x3), (x4,x6), (x5,x7): the (0,2,1,3) 4-group order.
__device__ __forceinline__ u32x4 deq_quad(u32x4 w)
{
    typedef _Float16 h2t __attribute__((ext_vector_type(2)));
    const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
    float x[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[2 * i] = h2f(wd[i] & 0xffff);
        x[2 * i + 1] = h2f(wd[i] >> 16);
    }
    float amax = fmaxf(fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))),
                       fmaxf(fmaxf(fabsf(x[4]), fabsf(x[5])), fmaxf(fabsf(x[6]), fabsf(x[7]))));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax), 0xb1, 0xf, 0xf, false)));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax), 0x4e, 0xf, 0xf, false)));
    const uint16_t dbits = amax != 0.f ? f2h_bits(q81_div(amax, 127.0f, 1.0f / 127.0f)) : (uint16_t)0;
    const float d = h2f(dbits);
    const float div = d == 0.f ? 1.0f : d;
    const float rdiv = __builtin_amdgcn_rcpf(div);
    const _Float16 dh = __builtin_bit_cast(_Float16, dbits);
    const h2t dd = {dh, dh}, magic = {(_Float16)1536.f, (_Float16)1536.f};
    const h2t lo = {(_Float16)-127.f, (_Float16)-127.f}, hi = {(_Float16)127.f, (_Float16)127.f};
    const int ord[8] = {0, 2, 1, 3, 4, 6, 5, 7};
    uint32_t o[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        h2t q = {(_Float16)q81_div(x[ord[2 * p]], div, rdiv), (_Float16)q81_div(x[ord[2 * p + 1]], div, rdiv)};
        q = (q + magic) - magic;
        q = __builtin_elementwise_min(__builtin_elementwise_max(q, lo), hi);
        o[p] = __builtin_bit_cast(uint32_t, q * dd);
    }
    return (u32x4){o[0], o[1], o[2], o[3]};
}

// The fp8 variant's block quantization (act_quant.hip F8 / F8DEQ; include/gguf_mmq.h states the
// rule) by an aligned group of 4 lanes, 8 elements each: X = 2^e with e the smallest integer
// such that max|x| <= 448 * 2^e (X = 1 for an all-zero block), codes = e4m3(x / X) RNE, stored
// per 4-group in the order (0,2,1,3); x~ = code * X, exact in fp16, as fp16 pairs (0,2), (1,3)
// of each 4-group -- the DEQ layout.
struct F8Quad {
    uint32_t codes[2]; // e4m3 bytes, 4-groups (0,2,1,3)
    uint32_t xt[4];    // x~ pairs: (x0,x2), (x1,x3), (x4,x6), (x5,x7)
    int e;
};

__device__ __forceinline__ F8Quad f8_quad(u32x4 w)
{
    const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
    float x[8], amax = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[2 * i] = h2f(wd[i] & 0xffff);
        x[2 * i + 1] = h2f(wd[i] >> 16);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(x[i]));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax), 0xb1, 0xf, 0xf, false)));
    amax = fmaxf(amax, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, amax), 0x4e, 0xf, 0xf, false)));
    // amax = m * 2^E, m in [0.5, 1): amax <= 448 * 2^e  <=>  e >= E - 9 + (m > 0.875)
    const uint32_t ab = __builtin_bit_cast(uint32_t, amax);
    const int E = (int)((ab >> 23) & 0xff) - 126;
    F8Quad r;
    r.e = amax == 0.f ? 0 : E - 9 + ((ab & 0x7fffffu) > 0x600000u ? 1 : 0);
    const float inv = __builtin_bit_cast(float, (uint32_t)(127 - r.e) << 23); // 2^-e, exact
    const float X = __builtin_bit_cast(float, (uint32_t)(127 + r.e) << 23);
    typedef _Float16 h2t __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int h = 0; h < 2; ++h) { // elements 4h..4h+3 -> bytes (0,2,1,3)
        int c = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * h] * inv, x[4 * h + 2] * inv, 0, false);
        c = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * h + 1] * inv, x[4 * h + 3] * inv, c, true);
        r.codes[h] = (uint32_t)c;
        r.xt[2 * h] = __builtin_bit_cast(uint32_t, (h2t)__builtin_amdgcn_cvt_scalef32_pk_f16_fp8(c, X, false));
        r.xt[2 * h + 1] = __builtin_bit_cast(uint32_t, (h2t)__builtin_amdgcn_cvt_scalef32_pk_f16_fp8(c, X, true));
    }
    return r;
}

} // namespace gq
