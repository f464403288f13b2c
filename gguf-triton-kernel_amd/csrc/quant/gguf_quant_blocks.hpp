// gguf_quant_blocks.hpp -- the GGUF block producers, one block at a time, for the host
// (gguf_quant.cpp, g++ -ffp-contract=off) and the device (quant_device.hip: one thread per
// block, the on-device requantization of SURVEY 8(f)2).  Every multiply/add is kept separately
// rounded in the reference's order (contraction off in both compilers), divisions and sqrt are
// IEEE (HIP's default correctly rounded fp32 divide/sqrt), so both give the reference's bytes;
// tests/golden/golden_quant.npz pins the host, tests/test_gpu_quant_device.py the device.
//
//   q4k_block  <- (GGML) quantize_row_q4_K_ref / make_qkx2_quants, q4_k_ref.c:188-368
//   q6k_block  <- (GGML) quantize_row_q6_K_ref / make_qx_quants, q6_k_ref.c:153-340
//   q8_block   <- utils/quantize/q8_0.py:4-49 (Q8_0), utils/quantize/q8_1.py:18-70 (Q8_1)
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>

#include "../gguf_half.hpp"

#ifdef __HIPCC__
#define GQ_QHD __host__ __device__
#else
#define GQ_QHD
#endif

#ifdef __clang__
#pragma clang fp contract(off)
#endif

namespace gq {
namespace qblk {

using gq::f2h;
using gq::h2f;

constexpr int QK = 256;
constexpr float kGroupMaxEps = 1e-15f;

// Round-to-nearest-even through the 1.5*2^23 magic constant; valid for |v| <= 2^22.
GQ_QHD inline int round_magic(float v)
{
    float t = v + 12582912.f;
    int32_t bits;
    __builtin_memcpy(&bits, &t, 4);
    return (bits & 0x007fffff) - 0x00400000;
}

GQ_QHD inline void put16(uint8_t *p, uint16_t v)
{
    p[0] = (uint8_t)(v & 0xff);
    p[1] = (uint8_t)(v >> 8);
}

GQ_QHD inline uint16_t get16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// ---------------- Q4_K ----------------
// Weighted fit of x ~ scale * L + min over L in [0, nmax] (GGML make_qkx2_quants with
// rmin=-1, rdelta=0.1, nstep=20, squared error).  Returns scale, writes -min to *neg_min.
GQ_QHD inline float fit_scale_min(const float *x, const float *w, uint8_t *L, uint8_t *Ltmp, float *neg_min)
{
    constexpr int n = 32, nmax = 15, nstep = 20;
    constexpr float rmin = -1.f, rdelta = 0.1f;
    float lo = x[0], hi = x[0];
    float sw = w[0];
    float swx = sw * x[0];
    for (int i = 1; i < n; ++i) {
        lo = x[i] < lo ? x[i] : lo;
        hi = x[i] > hi ? x[i] : hi;
        float wi = w[i];
        sw += wi;
        swx += wi * x[i];
    }
    if (lo > 0) lo = 0;
    if (hi == lo) {
        __builtin_memset(L, 0, n);
        *neg_min = -lo;
        return 0.f;
    }
    float inv = nmax / (hi - lo);
    float scale = 1 / inv;
    float best = 0;
    for (int i = 0; i < n; ++i) {
        int l = round_magic(inv * (x[i] - lo));
        L[i] = (uint8_t)std::max(0, std::min(nmax, l));
        float e = scale * L[i] + lo - x[i];
        best += w[i] * (e * e);
    }
    for (int step = 0; step <= nstep; ++step) {
        float cand = (rmin + rdelta * step + nmax) / (hi - lo);
        float sl = 0, sl2 = 0, sxl = 0;
        for (int i = 0; i < n; ++i) {
            int l = round_magic(cand * (x[i] - lo));
            l = std::max(0, std::min(nmax, l));
            Ltmp[i] = (uint8_t)l;
            float wi = w[i];
            sl += wi * l;
            sl2 += wi * l * l;
            sxl += wi * l * x[i];
        }
        float det = sw * sl2 - sl * sl;
        if (det > 0) {
            float s = (sw * sxl - swx * sl) / det;
            float m = (sl2 * swx - sl * sxl) / det;
            if (m > 0) {
                m = 0;
                s = sxl / sl2;
            }
            float err = 0;
            for (int i = 0; i < n; ++i) {
                float e = s * Ltmp[i] + m - x[i];
                err += w[i] * (e * e);
            }
            if (err < best) {
                __builtin_memcpy(L, Ltmp, n);
                best = err;
                scale = s;
                lo = m;
            }
        }
    }
    *neg_min = -lo;
    return scale;
}

GQ_QHD inline void q4k_block(const float *x, uint8_t *blk)
{
    uint8_t L[QK], Ltmp[32];
    float w[32], sub_scale[8], sub_min[8];
    float max_scale = 0, max_min = 0;
    for (int j = 0; j < 8; ++j) {
        const float *xs = x + 32 * j;
        float ss = 0;
        for (int l = 0; l < 32; ++l) ss += xs[l] * xs[l];
        float rms = std::sqrt(ss / 32);
        for (int l = 0; l < 32; ++l) w[l] = rms + std::fabs(xs[l]);
        sub_scale[j] = fit_scale_min(xs, w, L + 32 * j, Ltmp, &sub_min[j]);
        if (sub_scale[j] > max_scale) max_scale = sub_scale[j];
        if (sub_min[j] > max_min) max_min = sub_min[j];
    }
    float inv_s = max_scale > 0 ? 63.f / max_scale : 0.f;
    float inv_m = max_min > 0 ? 63.f / max_min : 0.f;
    uint8_t *sc = blk + 4;
    __builtin_memset(sc, 0, 12);
    for (int j = 0; j < 8; ++j) {
        uint8_t ls = (uint8_t)round_magic(inv_s * sub_scale[j]);
        uint8_t lm = (uint8_t)round_magic(inv_m * sub_min[j]);
        ls = std::min<uint8_t>(63, ls);
        lm = std::min<uint8_t>(63, lm);
        if (j < 4) {
            sc[j] = ls;
            sc[j + 4] = lm;
        } else {
            sc[j + 4] = (uint8_t)((ls & 0x0f) | ((lm & 0x0f) << 4));
            sc[j - 4] |= (uint8_t)((ls >> 4) << 6);
            sc[j] |= (uint8_t)((lm >> 4) << 6);
        }
    }
    uint16_t dh = f2h(max_scale / 63.f), mh = f2h(max_min / 63.f);
    put16(blk, dh);
    put16(blk + 2, mh);
    for (int j = 0; j < 8; ++j) {
        int s6, m6;
        if (j < 4) {
            s6 = sc[j] & 63;
            m6 = sc[j + 4] & 63;
        } else {
            s6 = (sc[j + 4] & 0x0f) | ((sc[j - 4] >> 6) << 4);
            m6 = (sc[j + 4] >> 4) | ((sc[j] >> 6) << 4);
        }
        float d = h2f(dh) * s6;
        if (!d) continue;
        float dm = h2f(mh) * m6;
        for (int i = 0; i < 32; ++i) {
            int l = round_magic((x[32 * j + i] + dm) / d);
            L[32 * j + i] = (uint8_t)std::max(0, std::min(15, l));
        }
    }
    uint8_t *qs = blk + 16;
    for (int c = 0; c < 4; ++c)
        for (int l = 0; l < 32; ++l) qs[32 * c + l] = (uint8_t)(L[64 * c + l] | (L[64 * c + 32 + l] << 4));
}

// ---------------- Q6_K ----------------
// Symmetric fit x ~ scale * l, l in [-32, 31], squared-x weights
// (GGML make_qx_quants with nmax=32, rmse_type=1).  L receives l + 32.
GQ_QHD inline float fit_scale_sym(const float *x, int8_t *L)
{
    constexpr int n = 16, nmax = 32;
    float peak = 0, amax = 0;
    for (int i = 0; i < n; ++i) {
        float a = std::fabs(x[i]);
        if (a > amax) {
            amax = a;
            peak = x[i];
        }
    }
    if (amax < kGroupMaxEps) {
        __builtin_memset(L, 0, n);
        return 0.f;
    }
    float inv = -nmax / peak;
    float sxl = 0, sl2 = 0;
    for (int i = 0; i < n; ++i) {
        int l = round_magic(inv * x[i]);
        l = std::max(-nmax, std::min(nmax - 1, l));
        L[i] = (int8_t)(l + nmax);
        float w = x[i] * x[i];
        sxl += w * x[i] * l;
        sl2 += w * l * l;
    }
    float scale = sl2 ? sxl / sl2 : 0.0f;
    float best = scale * sxl;
    for (int step = -9; step <= 9; ++step) {
        if (step == 0) continue;
        float cand = -(nmax + 0.1f * step) / peak;
        float a = 0, b = 0;
        for (int i = 0; i < n; ++i) {
            int l = round_magic(cand * x[i]);
            l = std::max(-nmax, std::min(nmax - 1, l));
            float w = x[i] * x[i];
            a += w * x[i] * l;
            b += w * l * l;
        }
        if (b > 0 && a * a > best * b) {
            for (int i = 0; i < n; ++i) {
                int l = round_magic(cand * x[i]);
                L[i] = (int8_t)(nmax + std::max(-nmax, std::min(nmax - 1, l)));
            }
            scale = a / b;
            best = scale * a;
        }
    }
    return scale;
}

GQ_QHD inline void q6k_block(const float *x, uint8_t *blk)
{
    int8_t L[QK];
    float sub[16];
    float max_scale = 0, max_abs = 0;
    for (int ib = 0; ib < 16; ++ib) {
        sub[ib] = fit_scale_sym(x + 16 * ib, L + 16 * ib);
        float a = std::fabs(sub[ib]);
        if (a > max_abs) {
            max_abs = a;
            max_scale = sub[ib];
        }
    }
    __builtin_memset(blk, 0, 210);
    if (max_abs < kGroupMaxEps) {
        put16(blk + 208, f2h(0.f));
        return;
    }
    float inv = -128.f / max_scale;
    uint16_t dh = f2h(1 / inv);
    put16(blk + 208, dh);
    int8_t *scales = (int8_t *)(blk + 192);
    for (int ib = 0; ib < 16; ++ib) scales[ib] = (int8_t)std::min(127, round_magic(inv * sub[ib]));
    for (int j = 0; j < 16; ++j) {
        float d = h2f(dh) * scales[j];
        if (!d) continue;
        for (int i = 0; i < 16; ++i) {
            int l = round_magic(x[16 * j + i] / d);
            L[16 * j + i] = (int8_t)(std::max(-32, std::min(31, l)) + 32);
        }
    }
    uint8_t *ql = blk, *qh = blk + 128;
    for (int half = 0; half < 2; ++half) {
        const int8_t *Lh = L + 128 * half;
        for (int l = 0; l < 32; ++l) {
            uint8_t a = (uint8_t)Lh[l], b = (uint8_t)Lh[l + 32], c = (uint8_t)Lh[l + 64], d = (uint8_t)Lh[l + 96];
            ql[64 * half + l] = (uint8_t)((a & 0x0f) | ((c & 0x0f) << 4));
            ql[64 * half + l + 32] = (uint8_t)((b & 0x0f) | ((d & 0x0f) << 4));
            qh[32 * half + l] = (uint8_t)((a >> 4) | ((b >> 4) << 2) | ((c >> 4) << 4) | ((d >> 4) << 6));
        }
    }
}

// ---------------- Q8_0 / Q8_1 (the reference's torch producers, fp16 arithmetic) ----------------
// d = fp16(amax / 127); q = clamp(rne(fp16(x / d)), +-127).  Q8_0 stores d = 1 for an all-zero
// block; Q8_1 stores d = 0 there (dividing by 1) and s = fp16(d * fp16(sum q)).
template <bool WITH_SUM>
GQ_QHD inline void q8_block(const uint16_t *x, uint8_t *blk)
{
    float amax = 0.f;
    for (int i = 0; i < 32; ++i) amax = std::max(amax, std::fabs(h2f(x[i])));
    uint16_t d = WITH_SUM ? (uint16_t)0 : (uint16_t)0x3c00;
    if (amax != 0.f) d = f2h(amax / 127.0f);
    float div = h2f(d);
    if (WITH_SUM && div == 0.f) div = 1.f;
    uint8_t *qs = blk + (WITH_SUM ? 4 : 2);
    int32_t sum = 0;
    for (int i = 0; i < 32; ++i) {
        float q = std::nearbyint(h2f(f2h(h2f(x[i]) / div)));
        if (q != q) q = 0.f; // 0/0 when d underflowed to 0 (tiny Q8_0 block): torch's int8 cast gives 0
        q = std::min(127.f, std::max(-127.f, q));
        int8_t qi = (int8_t)q;
        qs[i] = (uint8_t)qi;
        sum += qi;
    }
    put16(blk, d);
    if (WITH_SUM) put16(blk + 2, f2h(h2f(d) * h2f(f2h((float)sum))));
}


} // namespace qblk
} // namespace gq
