// mmq_gemv.hip -- decode-shaped MMQ (few tokens): weight rows streamed once from HBM.
//
// Computes C[t][m] = sum_k W[m][k] * x~[t][k] for t < N_tok (<= 4 per launch column) where
// x~ is the q8_1-quantized activation (act_quant.hip, SOA form) and W is the packed GGUF
// row m.  The per-block arithmetic is the reference's (kernels/cpu_impls/*):
//   Q8_0 : dA*dB*sum(qA*qB)                                  mmq_q8_0_q8_1_cpu.py:37-54
//   Q4_K : d*sc*dB*sum(q*qB) - dmin*m*sB                     mmq_q4_k_q8_1_cpu.py:94-117
//   Q6_K : dB*(d*sc1*sum((q-32)*qB)_lo + d*sc2*sum(...)_hi)  mmq_q6_k_q8_1_cpu.py:117-150
// with exact int32 dot products (v_dot4_i32_i8) and fp32 accumulation (the reference
// accumulates in fp16), one fp16 rounding at the store.
//
// Mapping (wave64, no LDS): a wave owns R weight rows at a time; lane l owns "unit" u
// (64 consecutive K elements) u = l, l+64, ...  Per unit and row a lane issues 16-byte
// loads straight to registers (Q4_K: header + 32 qs bytes; Q6_K: 32 ql + 32 qh + 8
// scales + d; Q8_0: two 34-byte blocks), dequantizes nothing -- the integer codes go
// straight into dot4 against the int8 activation codes, which the lane loads once per
// unit and reuses for its R rows.  A 6-step xor-shuffle reduction per (row, token) ends
// the row group.  Loop over row groups is grid-strided.
#include <cstdlib>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_units.hpp"
#include "gguf_dot.hpp"

namespace gq {

namespace {

template <int F, int NT, int R>
__global__ __launch_bounds__(256) void gemv_kernel(const uint8_t *__restrict__ A, const int8_t *__restrict__ xq,
                                                   const float *__restrict__ xd, const float *__restrict__ xs,
                                                   uint16_t *__restrict__ C, int64_t M, int64_t N, int64_t K,
                                                   int64_t ldc)
{
    using L = Layout<F>;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t tok0 = (int64_t)blockIdx.y * NT;
    const int64_t nb = K / 32;
    const int64_t row_bytes = (K / L::QK) * L::BYTES;
    const int nunits = (int)((K + 63) / 64);

    for (int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * R; row0 < M; row0 += (int64_t)gridDim.x * 4 * R) {
        float acc[R][NT];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[r][t] = 0.f;

        for (int u = lane; u < nunits; u += 64) {
            Act<F, NT> a;
            load_act<F, NT>(a, xq, xd, xs, tok0, N, K, u);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int64_t row = row0 + r < M ? row0 + r : M - 1;
                unit_dot<F, NT>(A + row * row_bytes, u, nb, a, acc[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float v = wave_sum(acc[r][t]);
                if (lane == 0 && row0 + r < M && tok0 + t < N) C[(tok0 + t) * ldc + row0 + r] = f2h_bits(v);
            }
        }
    }
}

template <int F, int NT, int R>
hipError_t launch_one(const uint8_t *A, const int8_t *xq, const float *xd, const float *xs, uint16_t *C, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    const int64_t groups = (M + 4 * R - 1) / (4 * R);
    const int64_t cap = 2048;
    dim3 grid((unsigned)(groups < cap ? groups : cap), (unsigned)((N + NT - 1) / NT)), block(256);
    gemv_kernel<F, NT, R><<<grid, block, 0, s>>>(A, xq, xd, xs, C, M, N, K, ldc);
    return hipGetLastError();
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const int8_t *xq, const float *xd, const float *xs, uint16_t *C, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    // rows per wave (profiles/r02/gemv_rows_tune.txt): 1-2 tokens Q8_0 4, Q4_K / Q6_K 2
    // (Q4_K 4096x28672 x2 30.3 -> 23.9 us, Q6_K 8192x28672 x2 64.9 -> 58.3); 3-4 tokens 2,
    // Q6_K 4 (x4 81.7 -> 72.9)
    const int r = N <= 2 ? (F == Q8_0 ? 4 : 2) : (F == Q6_K ? 4 : 2);
    if (N == 1) return r == 8 ? launch_one<F, 1, 8>(A, xq, xd, xs, C, M, N, K, ldc, s)
                              : r == 2 ? launch_one<F, 1, 2>(A, xq, xd, xs, C, M, N, K, ldc, s)
                                       : launch_one<F, 1, 4>(A, xq, xd, xs, C, M, N, K, ldc, s);
    if (N == 2) return r == 8 ? launch_one<F, 2, 8>(A, xq, xd, xs, C, M, N, K, ldc, s)
                              : r == 2 ? launch_one<F, 2, 2>(A, xq, xd, xs, C, M, N, K, ldc, s)
                                       : launch_one<F, 2, 4>(A, xq, xd, xs, C, M, N, K, ldc, s);
    return r == 4 ? launch_one<F, 4, 4>(A, xq, xd, xs, C, M, N, K, ldc, s)
                  : r == 1 ? launch_one<F, 4, 1>(A, xq, xd, xs, C, M, N, K, ldc, s)
                           : launch_one<F, 4, 2>(A, xq, xd, xs, C, M, N, K, ldc, s);
}

} // namespace

hipError_t launch_gemv(int fmt, const uint8_t *A, const int8_t *xq, const float *xd, const float *xs, uint16_t *C,
                       int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, xq, xd, xs, C, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, xq, xd, xs, C, M, N, K, ldc, s);
    default: return launch_fmt<Q6_K>(A, xq, xd, xs, C, M, N, K, ldc, s);
    }
}

} // namespace gq
