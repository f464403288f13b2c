// gguf_quant.cpp -- host-side GGUF block producers (the packed layouts the MMQ kernels read).
//
// Drop-in for the reference's format producers:
//   quantize_to_q4_k  utils/quantize/q4_k.py:87-91  -> (GGML) quantize_row_q4_K_ref, q4_k_ref.c:281-368
//   quantize_to_q6_k  utils/quantize/q6_k.py:97-110 -> (GGML) quantize_row_q6_K_ref, q6_k_ref.c:243-340
//   quantize_to_q8_0  utils/quantize/q8_0.py:4-49
//   quantize_to_q8_1  utils/quantize/q8_1.py:18-70
//   dequantize_*      utils/quantize/{q8_0.py:52, q8_1.py:73, q4_k.py:146, q6_k.py:138}
//
// The K-quant producers restate GGML's published reference algorithm (make_qkx2_quants /
// make_qx_quants: weighted least-squares search over candidate inverse scales, 6-bit
// scale/min packing, ql/qh split).  Every multiply/add is kept separately rounded in the
// same order (build with -ffp-contract=off) so the bytes equal the reference's; the
// golden vectors in tests/golden/golden_quant.npz pin that.
//
// Plain C ABI, host only, no GPU and no torch.  Large inputs are split over threads by
// whole super-blocks (results do not depend on the thread count).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>
#include <algorithm>

#include "../gguf_half.hpp"

namespace {

using gq::f2h;
using gq::h2f;

constexpr int QK = 256;
constexpr float kGroupMaxEps = 1e-15f;

// Round-to-nearest-even through the 1.5*2^23 magic constant; valid for |v| <= 2^22.
inline int round_magic(float v)
{
    float t = v + 12582912.f;
    int32_t bits;
    std::memcpy(&bits, &t, 4);
    return (bits & 0x007fffff) - 0x00400000;
}

inline void put16(uint8_t *p, uint16_t v)
{
    p[0] = (uint8_t)(v & 0xff);
    p[1] = (uint8_t)(v >> 8);
}

inline uint16_t get16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }

template <typename F>
void parallel_blocks(int64_t nblocks, F &&fn)
{
    unsigned hw = std::thread::hardware_concurrency();
    int64_t nthreads = std::min<int64_t>(hw ? hw : 1, 32);
    const int64_t min_per_thread = 512;
    nthreads = std::max<int64_t>(1, std::min<int64_t>(nthreads, nblocks / min_per_thread));
    if (nthreads <= 1) {
        fn(0, nblocks);
        return;
    }
    std::vector<std::thread> pool;
    int64_t per = (nblocks + nthreads - 1) / nthreads;
    for (int64_t t = 0; t < nthreads; ++t) {
        int64_t b0 = t * per, b1 = std::min(nblocks, b0 + per);
        if (b0 >= b1) break;
        pool.emplace_back([=, &fn] { fn(b0, b1); });
    }
    for (auto &th : pool) th.join();
}

// ---------------- Q4_K ----------------
// Weighted fit of x ~ scale * L + min over L in [0, nmax] (GGML make_qkx2_quants with
// rmin=-1, rdelta=0.1, nstep=20, squared error).  Returns scale, writes -min to *neg_min.
float fit_scale_min(const float *x, const float *w, uint8_t *L, uint8_t *Ltmp, float *neg_min)
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
        std::memset(L, 0, n);
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
                std::memcpy(L, Ltmp, n);
                best = err;
                scale = s;
                lo = m;
            }
        }
    }
    *neg_min = -lo;
    return scale;
}

void q4k_block(const float *x, uint8_t *blk)
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
    std::memset(sc, 0, 12);
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
float fit_scale_sym(const float *x, int8_t *L)
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
        std::memset(L, 0, n);
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

void q6k_block(const float *x, uint8_t *blk)
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
    std::memset(blk, 0, 210);
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
void q8_block(const uint16_t *x, uint8_t *blk)
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

} // namespace

extern "C" {

// x: n fp32 values (n % 256 == 0), y: n/256 * 144 bytes.
void gq_quantize_q4_k(const float *x, void *y, int64_t n)
{
    parallel_blocks(n / QK, [&](int64_t b0, int64_t b1) {
        for (int64_t b = b0; b < b1; ++b) q4k_block(x + b * QK, (uint8_t *)y + b * 144);
    });
}

// x: n fp32 values (n % 256 == 0), y: n/256 * 210 bytes.
void gq_quantize_q6_k(const float *x, void *y, int64_t n)
{
    parallel_blocks(n / QK, [&](int64_t b0, int64_t b1) {
        for (int64_t b = b0; b < b1; ++b) q6k_block(x + b * QK, (uint8_t *)y + b * 210);
    });
}

// x: n fp16 bit patterns (n % 32 == 0), y: n/32 * 34 bytes.
void gq_quantize_q8_0(const uint16_t *x, void *y, int64_t n)
{
    parallel_blocks(n / 32, [&](int64_t b0, int64_t b1) {
        for (int64_t b = b0; b < b1; ++b) q8_block<false>(x + b * 32, (uint8_t *)y + b * 34);
    });
}

// x: n fp16 bit patterns (n % 32 == 0), y: n/32 * 36 bytes.
void gq_quantize_q8_1(const uint16_t *x, void *y, int64_t n)
{
    parallel_blocks(n / 32, [&](int64_t b0, int64_t b1) {
        for (int64_t b = b0; b < b1; ++b) q8_block<true>(x + b * 32, (uint8_t *)y + b * 36);
    });
}

void gq_dequantize_q8_0(const void *y, float *out, int64_t nblocks)
{
    const uint8_t *p = (const uint8_t *)y;
    for (int64_t b = 0; b < nblocks; ++b, p += 34) {
        float d = h2f(get16(p));
        for (int i = 0; i < 32; ++i) out[32 * b + i] = d * (float)(int8_t)p[2 + i];
    }
}

void gq_dequantize_q8_1(const void *y, float *out, int64_t nblocks)
{
    const uint8_t *p = (const uint8_t *)y;
    for (int64_t b = 0; b < nblocks; ++b, p += 36) {
        float d = h2f(get16(p));
        for (int i = 0; i < 32; ++i) out[32 * b + i] = d * (float)(int8_t)p[4 + i];
    }
}

void gq_dequantize_q4_k(const void *y, float *out, int64_t nblocks)
{
    const uint8_t *p = (const uint8_t *)y;
    for (int64_t b = 0; b < nblocks; ++b, p += 144) {
        float d = h2f(get16(p)), dmin = h2f(get16(p + 2));
        const uint8_t *sc = p + 4, *qs = p + 16;
        for (int j = 0; j < 8; ++j) {
            int s6, m6;
            if (j < 4) {
                s6 = sc[j] & 63;
                m6 = sc[j + 4] & 63;
            } else {
                s6 = (sc[j + 4] & 0x0f) | ((sc[j - 4] >> 6) << 4);
                m6 = (sc[j + 4] >> 4) | ((sc[j] >> 6) << 4);
            }
            float ds = d * (float)s6, dm = dmin * (float)m6;
            for (int i = 0; i < 32; ++i) {
                uint8_t byte = qs[32 * (j >> 1) + i];
                int q = (j & 1) ? (byte >> 4) : (byte & 0x0f);
                out[256 * b + 32 * j + i] = ds * (float)q - dm;
            }
        }
    }
}

void gq_dequantize_q6_k(const void *y, float *out, int64_t nblocks)
{
    const uint8_t *p = (const uint8_t *)y;
    for (int64_t b = 0; b < nblocks; ++b, p += 210) {
        float d = h2f(get16(p + 208));
        const int8_t *scales = (const int8_t *)(p + 192);
        for (int e = 0; e < 256; ++e) {
            int h = e >> 7, r = e & 127;
            int lo = (p[64 * h + (r & 63)] >> (4 * (r >> 6))) & 0x0f;
            int hi = (p[128 + 32 * h + (r & 31)] >> (2 * (r >> 5))) & 0x03;
            out[256 * b + e] = (d * (float)scales[e >> 4]) * (float)((lo | (hi << 4)) - 32);
        }
    }
}

} // extern "C"
