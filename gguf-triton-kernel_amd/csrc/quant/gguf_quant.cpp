// gguf_quant.cpp -- host-side GGUF block producers (the packed layouts the MMQ kernels read).
//
// Drop-in for the reference's format producers:
//   quantize_to_q4_k  utils/quantize/q4_k.py:87-91  -> (GGML) quantize_row_q4_K_ref, q4_k_ref.c:281-368
//   quantize_to_q6_k  utils/quantize/q6_k.py:97-110 -> (GGML) quantize_row_q6_K_ref, q6_k_ref.c:243-340
//   quantize_to_q8_0  utils/quantize/q8_0.py:4-49
//   quantize_to_q8_1  utils/quantize/q8_1.py:18-70
//   dequantize_*      utils/quantize/{q8_0.py:52, q8_1.py:73, q4_k.py:146, q6_k.py:138}
//
// The per-block producers live in gguf_quant_blocks.hpp (shared with the device quantizers of
// quant_device.hip).  The K-quant producers restate GGML's published reference algorithm
// (make_qkx2_quants / make_qx_quants: weighted least-squares search over candidate inverse
// scales, 6-bit scale/min packing, ql/qh split).  Every multiply/add is kept separately rounded
// in the same order (build with -ffp-contract=off) so the bytes equal the reference's; the
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
#include "gguf_quant_blocks.hpp"

namespace {

using gq::f2h;
using gq::h2f;
using namespace gq::qblk;

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
