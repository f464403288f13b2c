/*
 * gguf_quant.h -- C ABI of the host-side GGUF block producers (libgguf_quant.so).
 *
 * Host memory only, no GPU required.  Outputs are byte-identical to the reference's
 * producers (pinned by tests/golden/golden_quant.npz):
 *   gq_quantize_q4_k   <- utils/quantize/q4_k.py:87   quantize_to_q4_k (GGML quantize_row_q4_K_ref)
 *   gq_quantize_q6_k   <- utils/quantize/q6_k.py:97   quantize_to_q6_k (GGML quantize_row_q6_K_ref)
 *   gq_quantize_q8_0   <- utils/quantize/q8_0.py:4    quantize_to_q8_0
 *   gq_quantize_q8_1   <- utils/quantize/q8_1.py:18   quantize_to_q8_1
 *   gq_dequantize_*    <- utils/quantize/{q8_0.py:52, q8_1.py:73, q4_k.py:146, q6_k.py:138}
 */
#ifndef GGUF_QUANT_H
#define GGUF_QUANT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* x: n fp32 (n % 256 == 0) -> y: n/256 blocks of 144 (Q4_K) / 210 (Q6_K) bytes */
void gq_quantize_q4_k(const float *x, void *y, int64_t n);
void gq_quantize_q6_k(const float *x, void *y, int64_t n);

/* x: n fp16 bit patterns (n % 32 == 0) -> y: n/32 blocks of 34 (Q8_0) / 36 (Q8_1) bytes */
void gq_quantize_q8_0(const uint16_t *x, void *y, int64_t n);
void gq_quantize_q8_1(const uint16_t *x, void *y, int64_t n);

/* y: nblocks packed blocks -> out: nblocks * QK fp32 values in element order */
void gq_dequantize_q8_0(const void *y, float *out, int64_t nblocks);
void gq_dequantize_q8_1(const void *y, float *out, int64_t nblocks);
void gq_dequantize_q4_k(const void *y, float *out, int64_t nblocks);
void gq_dequantize_q6_k(const void *y, float *out, int64_t nblocks);

#ifdef __cplusplus
}
#endif

#endif /* GGUF_QUANT_H */
