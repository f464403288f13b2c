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
 *   gq_cpu_mmq         <- kernels/cpu_impls/mmq_q8_0_q8_1_cpu.py:5, mmq_q4_k_q8_1_cpu.py:61,
 *                         mmq_q6_k_q8_1_cpu.py:84 (same outputs bit for bit: fp16 running sum)
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

/* C (M, N) fp16 bits, row-major = the reference CPU MMQ of packed weights A (type 0 Q8_0,
 * 1 Q4_K, 2 Q6_K; M rows of K) and packed q8_1 activations B (N rows of K).  threads <= 0:
 * every hardware thread (the result does not depend on it).  0 = OK, -1 = bad type or K. */
int gq_cpu_mmq(int type, const void *A, const void *B, int64_t M, int64_t N, int64_t K, uint16_t *C, int threads);

#ifdef __cplusplus
}
#endif

#endif /* GGUF_QUANT_H */
