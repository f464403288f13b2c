// gguf_q8_1.hpp -- the q8_1 block quantizer as a device routine (eight lanes per block).
//
// Bit-exact with utils/quantize/q8_1.py:18-70: d = fp16(amax/127) (0 for an all-zero
// block), q = clamp(rne(fp16(x / d')), +-127) with d' = 1 where d == 0,
// s = fp16(d * fp16(sum q)).  fp32 division is IEEE correctly rounded (hipcc default), so
// fp16(x/d) equals torch's CPU fp16 division.  Each of the 8 lanes of an aligned lane group
// holds 4 consecutive fp16 (two dwords); amax and sum(q) are reduced by xor shuffles inside
// the group, so every lane of the group must reach the call together.
#pragma once
#include "gguf_blocks.hpp"

namespace gq {

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
    r.dbits = amax != 0.f ? f2h_bits(amax / 127.0f) : (uint16_t)0;
    r.d = h2f(r.dbits);
    const float div = r.d == 0.f ? 1.0f : r.d;
    int sum = 0;
    r.codes = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float q = __builtin_rintf(h2f(f2h_bits(x[i] / div)));
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
    r.dbits = amax != 0.f ? f2h_bits(amax / 127.0f) : (uint16_t)0;
    r.d = h2f(r.dbits);
    const float div = r.d == 0.f ? 1.0f : r.d;
    int sum = 0;
    r.codes = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float q = __builtin_rintf(h2f(f2h_bits(x[i] / div)));
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

} // namespace gq
