// gguf_dot.hpp -- per-lane unit dot products against q8_1 activations (GEMV / decode).
//
// Per block the reference's arithmetic (kernels/cpu_impls/*):
//   Q8_0 : dA*dB*sum(qA*qB)                                  mmq_q8_0_q8_1_cpu.py:37-54
//   Q4_K : d*sc*dB*sum(q*qB) - dmin*m*sB                     mmq_q4_k_q8_1_cpu.py:94-117
//   Q6_K : dB*(d*sc1*sum((q-32)*qB)_lo + d*sc2*sum(...)_hi)  mmq_q6_k_q8_1_cpu.py:117-150
// with exact int32 dot products (v_dot4_i32_i8) and fp32 accumulation.
#pragma once
#include "gguf_blocks.hpp"
#include "gguf_units.hpp"

namespace gq {

template <int F, int NT>
struct Act {
    uint32_t q[NT][16]; // int8 codes of the two activation blocks
    float d[NT][2];
    float s[NT][2];  // q8_1 s (Q4_K min term)
    int sum[NT][4];  // sum of codes per 16-element quarter (Q6_K -32 offset)
};

template <int F, int NT>
__device__ __forceinline__ void load_act(Act<F, NT> &a, const int8_t *__restrict__ xq, const float *__restrict__ xd,
                                         const float *__restrict__ xs, int64_t tok0, int64_t N, int64_t K, int u)
{
    const int64_t nb = K / 32;
    int b0, b1;
    act_blocks<F>(u, b0, b1);
    const bool has1 = b1 < nb;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int64_t tok = (tok0 + t < N) ? tok0 + t : N - 1;
        const int8_t *base = xq + tok * K;
        u32x4 c0 = ld16(base + 32 * b0), c1 = ld16(base + 32 * b0 + 16);
        u32x4 c2 = {0, 0, 0, 0}, c3 = {0, 0, 0, 0};
        if (has1) {
            c2 = ld16(base + 32 * b1);
            c3 = ld16(base + 32 * b1 + 16);
        }
        a.q[t][0] = c0.x; a.q[t][1] = c0.y; a.q[t][2] = c0.z; a.q[t][3] = c0.w;
        a.q[t][4] = c1.x; a.q[t][5] = c1.y; a.q[t][6] = c1.z; a.q[t][7] = c1.w;
        a.q[t][8] = c2.x; a.q[t][9] = c2.y; a.q[t][10] = c2.z; a.q[t][11] = c2.w;
        a.q[t][12] = c3.x; a.q[t][13] = c3.y; a.q[t][14] = c3.z; a.q[t][15] = c3.w;
        a.d[t][0] = xd[tok * nb + b0];
        a.d[t][1] = has1 ? xd[tok * nb + b1] : 0.f;
        if constexpr (F == Q4_K) {
            a.s[t][0] = xs[tok * nb + b0];
            a.s[t][1] = has1 ? xs[tok * nb + b1] : 0.f;
        }
        if constexpr (F == Q6_K) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int acc = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = dot4(a.q[t][4 * k + i], 0x01010101u, acc);
                a.sum[t][k] = acc;
            }
        }
    }
}

// Adds a loaded unit's contribution for every token into acc[t].
template <int F, int NT>
__device__ __forceinline__ void dot_unit(const UnitRaw<F> &r, const Act<F, NT> &a, float (&acc)[NT])
{
    if constexpr (F == Q8_0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            int i0 = 0, i1 = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                i0 = dot4(r.w[i], a.q[t][i], i0);
                i1 = dot4(r.w[8 + i], a.q[t][8 + i], i1);
            }
            acc[t] += r.d0 * a.d[t][0] * (float)i0 + r.d1 * a.d[t][1] * (float)i1;
        }
    } else if constexpr (F == Q4_K) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            int i0 = 0, i1 = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                i0 = dot4(r.w[i] & 0x0f0f0f0fu, a.q[t][i], i0);
                i1 = dot4((r.w[i] >> 4) & 0x0f0f0f0fu, a.q[t][8 + i], i1);
            }
            acc[t] += r.ds0 * a.d[t][0] * (float)i0 - r.dm0 * a.s[t][0] + r.ds1 * a.d[t][1] * (float)i1 -
                      r.dm1 * a.s[t][1];
        }
    } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            int a1 = 0, a2 = 0, b1 = 0, b2 = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a1 = dot4(r.ca[i], a.q[t][i], a1);
                a2 = dot4(r.ca[4 + i], a.q[t][4 + i], a2);
                b1 = dot4(r.cb[i], a.q[t][8 + i], b1);
                b2 = dot4(r.cb[4 + i], a.q[t][12 + i], b2);
            }
            a1 -= 32 * a.sum[t][0];
            a2 -= 32 * a.sum[t][1];
            b1 -= 32 * a.sum[t][2];
            b2 -= 32 * a.sum[t][3];
            acc[t] += a.d[t][0] * (r.fa1 * (float)a1 + r.fa2 * (float)a2) +
                      a.d[t][1] * (r.fb1 * (float)b1 + r.fb2 * (float)b2);
        }
    }
}

// ---- the fp8 variant's decode (mmq_decode.hip, FP8 = 1) ----
// The unit's activations as fp16 x~ = e4m3 code * 2^e (gguf_q8_1.hpp f8_quad): 64 values as 32
// pair words in the DEQ order (word 2k = (x4k, x4k+2), 2k+1 = (x4k+1, x4k+3); Q6_K: run A then
// run B), and the fp32 sums of x~ over the unit's four 16-element quarters.  The weights' codes
// enter v_dot2_f32_f16 as fp16 pairs 1024 + byte (one v_perm / v_and_or per pair, no bias
// subtraction): sum (1024 + c) x = sum c x + 1024 sum x, taken out with the quarter sums.
template <int NT> struct ActH {
    uint32_t x[NT][32];
    float s[NT][4];
};

typedef _Float16 hh2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float fdot2u(uint32_t a, uint32_t b, float c)
{
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(hh2, a), __builtin_bit_cast(hh2, b), c, false);
}
// fp16 pairs 1024 + byte of bytes (0,2) / (1,3) of a word; 1024 + nibble of bytes (0,2)
__device__ __forceinline__ uint32_t b02(uint32_t c) { return __builtin_amdgcn_perm(0x64646464u, c, 0x04020400u); }
__device__ __forceinline__ uint32_t b13(uint32_t c) { return __builtin_amdgcn_perm(0x64646464u, c, 0x04030401u); }
__device__ __forceinline__ uint32_t n02(uint32_t v) { return (v & 0x000f000fu) | 0x64006400u; }

// NS (two or more tokens): the code pairs made exact (1024 + c - bias as one v_pk_add) so no
// quarter sums are needed -- Q8_0 and Q6_K keep none in LDS, Q4_K only the per-32 x~ sum of its
// min term (a.s[t][0], a.s[t][2]): the 2-token x~ image of an 11008-long row then fits beside
// the ring (the sums were the 384 bytes over)
template <int F, int NT, bool NS = false>
__device__ __forceinline__ void dot_unit_h(const UnitRaw<F> &r, const ActH<NT> &a, float (&acc)[NT])
{
    typedef _Float16 hb2 __attribute__((ext_vector_type(2)));
    auto unbias = [](uint32_t v, float b) {
        const hb2 bb = {(_Float16)b, (_Float16)b};
        return __builtin_bit_cast(uint32_t, __builtin_bit_cast(hb2, v) - bb);
    };
    if constexpr (NS && F == Q8_0) {
        uint32_t p[32];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t c = r.w[i] ^ 0x80808080u;
            p[2 * i] = unbias(b02(c), 1152.f);
            p[2 * i + 1] = unbias(b13(c), 1152.f);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s0 = fdot2u(p[i], a.x[t][i], s0);
                s1 = fdot2u(p[16 + i], a.x[t][16 + i], s1);
            }
            acc[t] += r.d0 * s0 + r.d1 * s1;
        }
    } else if constexpr (NS && F == Q4_K) {
        uint32_t p[32];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            p[2 * i] = unbias(n02(r.w[i]), 1024.f);
            p[2 * i + 1] = unbias(n02(r.w[i] >> 8), 1024.f);
            p[16 + 2 * i] = unbias(n02(r.w[i] >> 4), 1024.f);
            p[16 + 2 * i + 1] = unbias(n02(r.w[i] >> 12), 1024.f);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s0 = fdot2u(p[i], a.x[t][i], s0);
                s1 = fdot2u(p[16 + i], a.x[t][16 + i], s1);
            }
            acc[t] += r.ds0 * s0 - r.dm0 * a.s[t][0] + r.ds1 * s1 - r.dm1 * a.s[t][2];
        }
    } else if constexpr (NS) { // Q6_K: pairs (c - 32)
        uint32_t p[32];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            p[2 * i] = unbias(b02(r.ca[i]), 1056.f);
            p[2 * i + 1] = unbias(b13(r.ca[i]), 1056.f);
            p[16 + 2 * i] = unbias(b02(r.cb[i]), 1056.f);
            p[16 + 2 * i + 1] = unbias(b13(r.cb[i]), 1056.f);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int i = 0; i < 8; ++i) q[k] = fdot2u(p[8 * k + i], a.x[t][8 * k + i], q[k]);
            acc[t] += r.fa1 * q[0] + r.fa2 * q[1] + r.fb1 * q[2] + r.fb2 * q[3];
        }
    } else if constexpr (F == Q8_0) { // codes + 128 (xor 0x80): pairs 1152 + q
        uint32_t p[32];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t c = r.w[i] ^ 0x80808080u;
            p[2 * i] = b02(c);
            p[2 * i + 1] = b13(c);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s0 = fdot2u(p[i], a.x[t][i], s0);
                s1 = fdot2u(p[16 + i], a.x[t][16 + i], s1);
            }
            acc[t] += r.d0 * (s0 - 1152.f * (a.s[t][0] + a.s[t][1])) + r.d1 * (s1 - 1152.f * (a.s[t][2] + a.s[t][3]));
        }
    } else if constexpr (F == Q4_K) { // low nibbles: sub-block A, high: B
        uint32_t p[32];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            p[2 * i] = n02(r.w[i]);
            p[2 * i + 1] = n02(r.w[i] >> 8);
            p[16 + 2 * i] = n02(r.w[i] >> 4);
            p[16 + 2 * i + 1] = n02(r.w[i] >> 12);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s0 = fdot2u(p[i], a.x[t][i], s0);
                s1 = fdot2u(p[16 + i], a.x[t][16 + i], s1);
            }
            const float xa = a.s[t][0] + a.s[t][1], xb = a.s[t][2] + a.s[t][3];
            acc[t] += r.ds0 * (s0 - 1024.f * xa) - r.dm0 * xa + r.ds1 * (s1 - 1024.f * xb) - r.dm1 * xb;
        }
    } else { // Q6_K: codes 0..63, weight (q - 32) * d * sc per 16 elements
        uint32_t p[32];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            p[2 * i] = b02(r.ca[i]);
            p[2 * i + 1] = b13(r.ca[i]);
            p[16 + 2 * i] = b02(r.cb[i]);
            p[16 + 2 * i + 1] = b13(r.cb[i]);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int i = 0; i < 8; ++i) q[k] = fdot2u(p[8 * k + i], a.x[t][8 * k + i], q[k]);
            acc[t] += r.fa1 * (q[0] - 1056.f * a.s[t][0]) + r.fa2 * (q[1] - 1056.f * a.s[t][1]) +
                      r.fb1 * (q[2] - 1056.f * a.s[t][2]) + r.fb2 * (q[3] - 1056.f * a.s[t][3]);
        }
    }
}

template <int F, int NT>
__device__ __forceinline__ void unit_dot(const uint8_t *__restrict__ rowp, int u, int64_t nb, const Act<F, NT> &a,
                                         float (&acc)[NT])
{
    UnitLoad<F> l;
    l.load(rowp, u, nb);
    dot_unit<F, NT>(UnitRaw<F>::from(l, u, nb), a, acc);
}

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Activation image in LDS (decode kernels):
// LDS: codes [NT][KP] (KP = K rounded up to 64) with 16-byte pieces XOR-swizzled so the
// 16-lane ds_read_b128 groups of a unit read hit 16 distinct bank quads, then d [NT][K/32]
// and (Q4_K) s [NT][K/32] as fp32.
template <int F>
__device__ __forceinline__ int swz_piece(int p)
{
    const int x = p >> 4;
    if constexpr (F == Q6_K) return p ^ ((x & 1) | ((x & 2) << 1));
    return p ^ (x & 3);
}

template <int F, int NT>
__device__ __forceinline__ void load_act_lds(Act<F, NT> &a, const uint8_t *codes, const float *sd, const float *ss,
                                             int64_t kp, int64_t nb, int u)
{
    int b0, b1;
    act_blocks<F>(u, b0, b1);
    const bool has1 = b1 < nb;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const uint8_t *row = codes + t * kp;
        const u32x4 c0 = *(const u32x4 *)(row + 16 * swz_piece<F>(2 * b0));
        const u32x4 c1 = *(const u32x4 *)(row + 16 * swz_piece<F>(2 * b0 + 1));
        u32x4 c2 = {0, 0, 0, 0}, c3 = {0, 0, 0, 0};
        if (has1) {
            c2 = *(const u32x4 *)(row + 16 * swz_piece<F>(2 * b1));
            c3 = *(const u32x4 *)(row + 16 * swz_piece<F>(2 * b1 + 1));
        }
        a.q[t][0] = c0.x; a.q[t][1] = c0.y; a.q[t][2] = c0.z; a.q[t][3] = c0.w;
        a.q[t][4] = c1.x; a.q[t][5] = c1.y; a.q[t][6] = c1.z; a.q[t][7] = c1.w;
        a.q[t][8] = c2.x; a.q[t][9] = c2.y; a.q[t][10] = c2.z; a.q[t][11] = c2.w;
        a.q[t][12] = c3.x; a.q[t][13] = c3.y; a.q[t][14] = c3.z; a.q[t][15] = c3.w;
        a.d[t][0] = sd[t * nb + b0];
        a.d[t][1] = has1 ? sd[t * nb + b1] : 0.f;
        if constexpr (F == Q4_K) {
            a.s[t][0] = ss[t * nb + b0];
            a.s[t][1] = has1 ? ss[t * nb + b1] : 0.f;
        }
        if constexpr (F == Q6_K) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int acc = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = dot4(a.q[t][4 * k + i], 0x01010101u, acc);
                a.sum[t][k] = acc;
            }
        }
    }
}

} // namespace gq
