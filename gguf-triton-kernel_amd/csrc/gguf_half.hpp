// gguf_half.hpp -- IEEE binary16 <-> binary32 in software (round to nearest even).
// Shared by the format producers (host, and the device quantizers of quant_device.hip, which
// run the host's exact code) and the C-ABI argument checks; the MMQ kernels use the hardware
// conversions (v_cvt_f16_f32 / v_cvt_f32_f16).
#pragma once
#include <cstdint>
#include <cstring>

#ifdef __HIPCC__
#define GQ_HHD __host__ __device__
#else
#define GQ_HHD
#endif

namespace gq {

GQ_HHD inline float h2f(uint16_t h)
{
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu;
    uint32_t man = h & 0x3ffu;
    uint32_t bits;
    if (exp == 0x1fu) {
        bits = sign | 0x7f800000u | (man << 13);
    } else if (exp != 0) {
        bits = sign | ((exp + 112u) << 23) | (man << 13);
    } else if (man == 0) {
        bits = sign;
    } else {
        // subnormal half: value = man * 2^-24, renormalise into an fp32 normal
        int shift = 0;
        while (!(man & 0x400u)) {
            man <<= 1;
            ++shift;
        }
        bits = sign | ((uint32_t)(113 - shift) << 23) | ((man & 0x3ffu) << 13);
    }
    float f;
    __builtin_memcpy(&f, &bits, 4);
    return f;
}

GQ_HHD inline uint16_t f2h(float f)
{
    uint32_t x;
    __builtin_memcpy(&x, &f, 4);
    const uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax != 0x7f800000u ? 0x200u : 0u));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); // >= 65520 rounds to inf
    if (ax < 0x38800000u) {                                   // below the smallest normal half
        if (ax < 0x33000000u) return sign;                      // < 2^-25: rounds to zero
        uint32_t e = ax >> 23, m = (ax & 0x7fffffu) | 0x800000u;
        uint32_t sh = 126u - e, q = m >> sh, r = m & ((1u << sh) - 1u), h = 1u << (sh - 1u);
        q += (r > h || (r == h && (q & 1u))) ? 1u : 0u;
        return (uint16_t)(sign | q);
    }
    uint32_t q = (((ax >> 23) - 112u) << 10) | ((ax >> 13) & 0x3ffu);
    uint32_t r = ax & 0x1fffu;
    q += (r > 0x1000u || (r == 0x1000u && (q & 1u))) ? 1u : 0u;
    return (uint16_t)(sign | q);
}

} // namespace gq
