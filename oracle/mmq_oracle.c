/*
 * oracle/mmq_oracle.c -- CPU restatement of the reference's parity oracle.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the gguf-triton-kernel_amd
 * package, include/, the HIP library) may link or call this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker.
 *
 * What it restates (reference = PowerfulGhost/gguf-triton-kernel @ 2025-11-21):
 *   - quantize_to_q8_1   utils/quantize/q8_1.py:18-70
 *   - quantize_to_q8_0   utils/quantize/q8_0.py:4-49
 *   - mmq_q8_0_q8_1_cpu  kernels/cpu_impls/mmq_q8_0_q8_1_cpu.py:5-56
 *   - mmq_q4_k_q8_1_cpu  kernels/cpu_impls/mmq_q4_k_q8_1_cpu.py:61-119 (+ parser :5-58)
 *   - mmq_q6_k_q8_1_cpu  kernels/cpu_impls/mmq_q6_k_q8_1_cpu.py:84-152 (+ parser :5-81)
 *   - dequantize_*       utils/quantize/{q8_0.py:52, q4_k.py:125-158, q6_k.py:117-159}
 *
 * Two accumulation modes for the matmuls:
 *   mode 0 (ORACLE_EXACT): the reference's arithmetic step for step -- per-block term
 *          computed with the same fp16/fp32 roundings torch applies, accumulated into an
 *          fp16 scalar in block order (C[m, n] += term.item(), cpu_impls:*).
 *          Pinned bit-exact against fixtures produced by the reference itself.
 *   mode 1 (ORACLE_IDEAL): the same quantized inputs, every product formed exactly in
 *          double and summed in double, rounded to fp16 once.  This is the value the
 *          reference's formula would give without its own rounding noise; GPU paths
 *          are held to a tight tolerance against it.
 *
 * Output layout: out[n * M + m] (tokens-major, i.e. the (N, M) tensor the reference
 * returns as C.T).  All packed inputs are raw little-endian bytes.
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

/* ---------- IEEE binary16 <-> binary32 (round to nearest even) ---------- */

static float h2f(uint16_t h)
{
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1f;
    uint32_t man = h & 0x3ffu;
    uint32_t bits;
    if (exp == 0) {
        if (man == 0) {
            bits = sign;
        } else { /* subnormal: renormalise */
            int e = -1;
            do { man <<= 1; e++; } while (!(man & 0x400u));
            man &= 0x3ffu;
            bits = sign | ((uint32_t)(127 - 15 - e) << 23) | (man << 13);
        }
    } else if (exp == 0x1f) {
        bits = sign | 0x7f800000u | (man << 13);
    } else {
        bits = sign | ((exp + 127 - 15) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

static uint16_t f2h(float f)
{
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t absx = x & 0x7fffffffu;
    if (absx >= 0x7f800000u) /* inf or nan */
        return (uint16_t)(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0));
    if (absx >= 0x477ff000u) /* rounds to >= 65536 -> inf */
        return (uint16_t)(sign | 0x7c00u);
    if (absx < 0x38800000u) { /* result subnormal or zero: value < 2^-14 */
        if (absx < 0x33000000u) /* < 2^-25 rounds to 0 */
            return (uint16_t)sign;
        uint32_t e = absx >> 23;
        uint32_t m = (absx & 0x7fffffu) | 0x800000u;
        uint32_t shift = 126 - e; /* 14..24 */
        uint32_t q = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (q & 1))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t e = (absx >> 23) - 127 + 15;
    uint32_t m = absx & 0x7fffffu;
    uint32_t q = (e << 10) | (m >> 13);
    uint32_t rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (q & 1))) q++;
    return (uint16_t)(sign | q);
}

static uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static void wr16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }

/* torch.round on an fp16 value: round half to even, result exactly representable */
static float rne(float v) { return nearbyintf(v); }

float oracle_h2f(uint16_t h) { return h2f(h); }
uint16_t oracle_f2h(float f) { return f2h(f); }

/* ---------- activation / weight 8-bit quantizers ---------- */

/* q8_1.py:18-70 : d = fp16(amax / 127) (0 for all-zero block), divisor 1 where d == 0,
 * q = clamp(round(fp16(x / d)), -127, 127), s = fp16(d * fp16(sum q)).
 * Block: [d fp16][s fp16][qs int8 x 32] = 36 bytes. */
void oracle_quantize_q8_1(const uint16_t *x, int64_t n, uint8_t *out)
{
    for (int64_t g = 0; g < n / 32; ++g) {
        const uint16_t *xs = x + g * 32;
        uint8_t *o = out + g * 36;
        float amax = 0.f;
        for (int i = 0; i < 32; ++i) {
            float a = fabsf(h2f(xs[i]));
            if (a > amax) amax = a;
        }
        uint16_t d = 0;
        if (amax != 0.f) d = f2h(amax / 127.0f);
        uint16_t dsafe = (h2f(d) == 0.f) ? (uint16_t)0x3c00u : d;
        float df = h2f(dsafe);
        int32_t sum = 0;
        for (int i = 0; i < 32; ++i) {
            float q = rne(h2f(f2h(h2f(xs[i]) / df)));
            if (q > 127.f) q = 127.f;
            if (q < -127.f) q = -127.f;
            int8_t qi = (int8_t)q;
            o[4 + i] = (uint8_t)qi;
            sum += qi;
        }
        uint16_t sh = f2h((float)sum);
        uint16_t s = f2h(h2f(d) * h2f(sh));
        wr16(o, d);
        wr16(o + 2, s);
    }
}

/* q8_0.py:4-49 : like q8_1 but the all-zero block stores d = 1.0 and no sum.
 * Block: [d fp16][qs int8 x 32] = 34 bytes. */
void oracle_quantize_q8_0(const uint16_t *x, int64_t n, uint8_t *out)
{
    for (int64_t g = 0; g < n / 32; ++g) {
        const uint16_t *xs = x + g * 32;
        uint8_t *o = out + g * 34;
        float amax = 0.f;
        for (int i = 0; i < 32; ++i) {
            float a = fabsf(h2f(xs[i]));
            if (a > amax) amax = a;
        }
        uint16_t d = 0x3c00u;
        if (amax != 0.f) d = f2h(amax / 127.0f);
        float df = h2f(d);
        for (int i = 0; i < 32; ++i) {
            float q = rne(h2f(f2h(h2f(xs[i]) / df)));
            if (q > 127.f) q = 127.f;
            if (q < -127.f) q = -127.f;
            o[2 + i] = (uint8_t)(int8_t)q;
        }
        wr16(o, d);
    }
}

/* ---------- packed-block field access ---------- */

/* Q4_K 6-bit scale/min unpack: mmq_q4_k_q8_1_cpu.py:33-56 (== get_scale_min_k4). */
static void q4k_scale_min(const uint8_t *s12, int j, int *sc, int *mn)
{
    if (j < 4) {
        *sc = s12[j] & 63;
        *mn = s12[j + 4] & 63;
    } else {
        *sc = (s12[j + 4] & 0x0f) | ((s12[j - 4] >> 6) << 4);
        *mn = (s12[j + 4] >> 4) | ((s12[j] >> 6) << 4);
    }
}

/* Q4_K code of element e (0..255): qs[32*(e/64) + e%32] nibble (e/32)&1. */
static int q4k_code(const uint8_t *blk, int e)
{
    const uint8_t *qs = blk + 16;
    int j = e >> 5;
    uint8_t b = qs[32 * (j >> 1) + (e & 31)];
    return (j & 1) ? (b >> 4) : (b & 0x0f);
}

/* Q6_K code (already minus 32) of element e: mmq_q6_k_q8_1_cpu.py:37-79. */
static int q6k_code(const uint8_t *blk, int e)
{
    const uint8_t *ql = blk;
    const uint8_t *qh = blk + 128;
    int h = e >> 7, r = e & 127;
    int lo = (ql[64 * h + (r & 63)] >> (4 * (r >> 6))) & 0x0f;
    int hi = (qh[32 * h + (r & 31)] >> (2 * (r >> 5))) & 0x03;
    return (lo | (hi << 4)) - 32;
}

/* ---------- matmul oracles (out is (N, M) tokens-major, fp16 bits) ---------- */

void oracle_mmq_q8_0_q8_1(const uint8_t *A, const uint8_t *B, int64_t M, int64_t N, int64_t K,
                          uint16_t *out, int mode)
{
    int64_t nb = K / 32;
    for (int64_t m = 0; m < M; ++m) {
        for (int64_t n = 0; n < N; ++n) {
            uint16_t c = 0;
            double acc = 0.0;
            for (int64_t j = 0; j < nb; ++j) {
                const uint8_t *a = A + (m * nb + j) * 34;
                const uint8_t *b = B + (n * nb + j) * 36;
                int32_t idot = 0;
                for (int i = 0; i < 32; ++i) idot += (int8_t)a[2 + i] * (int8_t)b[4 + i];
                float dA = h2f(rd16(a)), dB = h2f(rd16(b));
                if (mode == 0) {
                    /* scale_A * scale_B * int_dot : fp16*fp16 -> fp16, then * int -> fp16 */
                    uint16_t p = f2h(h2f(f2h(dA * dB)) * (float)idot);
                    c = f2h(h2f(c) + h2f(p));
                } else {
                    acc += (double)dA * (double)dB * (double)idot;
                }
            }
            out[n * M + m] = mode == 0 ? c : f2h((float)acc);
        }
    }
}

void oracle_mmq_q4_k_q8_1(const uint8_t *A, const uint8_t *B, int64_t M, int64_t N, int64_t K,
                          uint16_t *out, int mode)
{
    int64_t nsb = K / 256, nb = K / 32;
    for (int64_t m = 0; m < M; ++m) {
        for (int64_t n = 0; n < N; ++n) {
            uint16_t c = 0;
            double acc = 0.0;
            for (int64_t kb = 0; kb < nsb; ++kb) {
                const uint8_t *a = A + (m * nsb + kb) * 144;
                float d = h2f(rd16(a)), dmin = h2f(rd16(a + 2));
                for (int s = 0; s < 8; ++s) {
                    const uint8_t *b = B + (n * nb + kb * 8 + s) * 36;
                    int sc, mn;
                    q4k_scale_min(a + 4, s, &sc, &mn);
                    int32_t idot = 0;
                    for (int i = 0; i < 32; ++i) idot += q4k_code(a, 32 * s + i) * (int8_t)b[4 + i];
                    float dB = h2f(rd16(b)), sB = h2f(rd16(b + 2));
                    if (mode == 0) {
                        float t = ((d * (float)sc) * dB) * (float)idot - ((dmin * (float)mn) * sB);
                        /* C[m, n] += t.item(): torch casts the Python scalar to the fp16
                         * tensor's dtype first, then adds in fp32 and rounds again */
                        c = f2h(h2f(c) + h2f(f2h(t)));
                    } else {
                        acc += (double)d * sc * dB * idot - (double)dmin * mn * sB;
                    }
                }
            }
            out[n * M + m] = mode == 0 ? c : f2h((float)acc);
        }
    }
}

void oracle_mmq_q6_k_q8_1(const uint8_t *A, const uint8_t *B, int64_t M, int64_t N, int64_t K,
                          uint16_t *out, int mode)
{
    int64_t nsb = K / 256, nb = K / 32;
    for (int64_t m = 0; m < M; ++m) {
        for (int64_t n = 0; n < N; ++n) {
            uint16_t c = 0;
            double acc = 0.0;
            for (int64_t kb = 0; kb < nsb; ++kb) {
                const uint8_t *a = A + (m * nsb + kb) * 210;
                float d = h2f(rd16(a + 208));
                const int8_t *scales = (const int8_t *)(a + 192);
                for (int j = 0; j < 8; ++j) {
                    const uint8_t *b = B + (n * nb + kb * 8 + j) * 36;
                    int32_t dot1 = 0, dot2 = 0;
                    for (int i = 0; i < 16; ++i) dot1 += q6k_code(a, 32 * j + i) * (int8_t)b[4 + i];
                    for (int i = 0; i < 16; ++i) dot2 += q6k_code(a, 32 * j + 16 + i) * (int8_t)b[20 + i];
                    float dB = h2f(rd16(b));
                    if (mode == 0) {
                        float s1 = d * (float)scales[2 * j];
                        float s2 = d * (float)scales[2 * j + 1];
                        float r = dB * (s1 * (float)dot1 + s2 * (float)dot2);
                        c = f2h(h2f(c) + h2f(f2h(r))); /* scalar cast to fp16 first */
                    } else {
                        acc += (double)dB * ((double)d * scales[2 * j] * dot1 + (double)d * scales[2 * j + 1] * dot2);
                    }
                }
            }
            out[n * M + m] = mode == 0 ? c : f2h((float)acc);
        }
    }
}

/* ---------- dequantizers (fp32 out, element order of the original row) ---------- */

void oracle_dequant_q8_0(const uint8_t *A, int64_t nblocks, float *out)
{
    for (int64_t b = 0; b < nblocks; ++b) {
        const uint8_t *a = A + b * 34;
        float d = h2f(rd16(a));
        for (int i = 0; i < 32; ++i) out[b * 32 + i] = d * (float)(int8_t)a[2 + i];
    }
}

void oracle_dequant_q8_1(const uint8_t *A, int64_t nblocks, float *out)
{
    for (int64_t b = 0; b < nblocks; ++b) {
        const uint8_t *a = A + b * 36;
        float d = h2f(rd16(a));
        for (int i = 0; i < 32; ++i) out[b * 32 + i] = d * (float)(int8_t)a[4 + i];
    }
}

/* q4_k.py:125-158 : w = fp32(d)*sc*q - fp32(dmin)*m */
void oracle_dequant_q4_k(const uint8_t *A, int64_t nblocks, float *out)
{
    for (int64_t b = 0; b < nblocks; ++b) {
        const uint8_t *a = A + b * 144;
        float d = h2f(rd16(a)), dmin = h2f(rd16(a + 2));
        for (int s = 0; s < 8; ++s) {
            int sc, mn;
            q4k_scale_min(a + 4, s, &sc, &mn);
            float ds = d * (float)sc, dm = dmin * (float)mn;
            for (int i = 0; i < 32; ++i) out[b * 256 + 32 * s + i] = ds * (float)q4k_code(a, 32 * s + i) - dm;
        }
    }
}

/* q6_k.py:117-159 : w = fp32(d)*scales[e/16]*q */
void oracle_dequant_q6_k(const uint8_t *A, int64_t nblocks, float *out)
{
    for (int64_t b = 0; b < nblocks; ++b) {
        const uint8_t *a = A + b * 210;
        float d = h2f(rd16(a + 208));
        const int8_t *scales = (const int8_t *)(a + 192);
        for (int e = 0; e < 256; ++e) out[b * 256 + e] = (d * (float)scales[e >> 4]) * (float)q6k_code(a, e);
    }
}
