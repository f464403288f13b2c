// gguf_blocks.hpp -- GGUF packed-block layouts and the device-side helpers that read them.
//
// Layouts (little endian; a weight tensor is rows of K/QK consecutive blocks, no padding):
//   Q8_0  32 elems / 34 B : [0:2] d fp16 | [2:34] qs int8[32]               w = d*q
//   Q4_K 256 elems /144 B : [0:2] d | [2:4] dmin | [4:16] 6-bit sc/m x8 | [16:144] qs nibbles
//                           w = d*sc_j*q - dmin*m_j   (sub-block j = e/32)
//   Q6_K 256 elems /210 B : [0:128] ql | [128:192] qh | [192:208] int8 sc x16 | [208:210] d
//                           w = d*sc_{e/16}*(q - 32)
//   Q8_1 (activations) 36 B: [0:2] d | [2:4] s = d*sum(q) | [4:36] qs int8[32]
// Reference: block docs in kernels/mmq_q4_k.py:1-16, kernels/mmq_q6_k.py:1-14,
// utils/quantize/q8_1.py:1-11; unpack rules kernels/mmq_q4_k.py:30-114, mmq_q6_k.py:28-68.
//
// "Unit" = the 64 consecutive-in-K weights one lane of the GEMV owns (two 32-element
// activation blocks).  Every format is read straight from HBM into registers with 16-byte
// loads: gfx950 runs with unaligned global access enabled, so the 2-byte-aligned Q8_0/Q6_K
// fields are loaded as dwordx4 without byte shuffling.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gq {

enum Fmt : int { Q8_0 = 0, Q4_K = 1, Q6_K = 2 };

template <int F> struct Layout;
template <> struct Layout<Q8_0> { static constexpr int QK = 32, BYTES = 34; };
template <> struct Layout<Q4_K> { static constexpr int QK = 256, BYTES = 144; };
template <> struct Layout<Q6_K> { static constexpr int QK = 256, BYTES = 210; };

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u32x4 ld16(const void *p)
{
#ifdef GQ_ALIGN_TEST // diagnostic only: same access pattern with 16-byte aligned addresses
    p = (const void *)((uintptr_t)p & ~(uintptr_t)15);
#endif
    u32x4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

__device__ __forceinline__ u32x2 ld8(const void *p)
{
#ifdef GQ_ALIGN_TEST
    p = (const void *)((uintptr_t)p & ~(uintptr_t)7);
#endif
    u32x2 v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

__device__ __forceinline__ uint32_t ld4(const void *p)
{
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}

__device__ __forceinline__ uint16_t ld2(const void *p)
{
    uint16_t v;
    __builtin_memcpy(&v, p, 2);
    return v;
}

__device__ __forceinline__ float h2f(uint32_t bits16)
{
    return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
}

__device__ __forceinline__ uint16_t f2h_bits(float f)
{
    return __builtin_bit_cast(uint16_t, (_Float16)f);
}

// v_dot4_i32_i8: c + sum_k a.i8[k] * b.i8[k]
__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c)
{
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

__device__ __forceinline__ uint32_t byte_of(uint32_t w, uint32_t k) { return (w >> (8 * k)) & 0xffu; }

// Q4_K 6-bit scale and min of sub-block j from the 12 scale bytes s0..s11 packed in
// words sw[0..2] (== get_scale_min_k4; kernels/mmq_q4_k.py:30-80).
__device__ __forceinline__ void q4k_sc_m(const uint32_t sw[3], int j, int &sc, int &m)
{
    if (j < 4) {
        sc = byte_of(sw[0], j) & 63;
        m = byte_of(sw[1], j) & 63;
    } else {
        uint32_t hi = byte_of(sw[2], j - 4);
        sc = (hi & 0x0f) | ((byte_of(sw[0], j - 4) >> 6) << 4);
        m = (hi >> 4) | ((byte_of(sw[1], j - 4) >> 6) << 4);
    }
}

// s_waitcnt vmcnt(n) for a wave-uniform n <= MAXN (the immediate is an encoding field): the
// steady-state count is the first compare, the pipeline tails walk down from it
template <int MAXN> __device__ __attribute__((always_inline)) inline void vm_wait(int n)
{
    if constexpr (MAXN <= 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        if (n >= MAXN) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MAXN) : "memory");
        else vm_wait<MAXN - 1>(n);
    }
}

} // namespace gq
