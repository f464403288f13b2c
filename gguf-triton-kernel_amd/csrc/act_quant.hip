// act_quant.hip -- q8_1 activation quantizer on the GPU.
//
// Bit-exact with the reference's producer utils/quantize/q8_1.py:18-70:
//   d = fp16(amax/127) (0 for an all-zero block), q = clamp(rne(fp16(x / d')), +-127) with
//   d' = 1 where d == 0, s = fp16(d * fp16(sum q)).
// The reference's Triton kernels fuse an fp32 variant of this step (kernels/mmq_q4_k.py:202-207,
// x*127/amax, no fp16 rounding); this build keeps the oracle's exact q8_1 semantics so the
// GPU path and kernels/cpu_impls see identical integer activations.
//
// Four lanes own one 32-element block (8 fp16, one 16-byte load each): gguf_q8_1.hpp's
// q8_1_quad (DPP quad reductions).
//
// Output forms (one kernel template, chosen by the caller):
//   AOS  : the q8_1 byte layout itself (36 B per block) -- gq_quantize_q8_1 / tests
//   SOA  : codes int8 [rows][K] + d float [rows][K/32] + s float [rows][K/32] -- GEMV input
//   DEQ  : x~ = fp16(d * q) [rows][K] -- the dequantized activation fed to the fp16 MFMA GEMM,
//          each 4-element group stored in the order (0,2,1,3) (see mmq_gemm.hip)
//   I8   : codes int8 [rows][K] + d float BLOCK-major [K/32][ld] (ld = rows rounded up to 4) --
//          the int8-MFMA GEMM's input: one tile's d of a K block is one contiguous run
//   F8   : not q8_1 -- the fp8 activation variant (BASELINE configs[4]): per 32-element block
//          X = 2^e, e the smallest integer with max|x| <= 448 * 2^e (X = 1 for an all-zero
//          block), codes = OCP e4m3 (e4m3fn) of x / X, round to nearest even; codes [rows][K]
//          with each 4-group stored (0,2,1,3) (the GEMM's fragment order), X as float in the
//          I8 form's block-major layout
//   F8DEQ: the fp8 variant's x~ = fp16(code * X) in the DEQ layout: the F8 codes widened by
//          v_cvt_scalef32_pk_f16_fp8 (code * 2^e is exact in fp16), so every fp16-activation
//          kernel (skinny, GEMMs, hipBLASLt) runs the fp8 variant unchanged
#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_q8_1.hpp"

namespace gq {

// workgroup wg of a launch over one (rows, K) activation tensor: blocks 64 wg .. 64 wg + 63
template <int MODE>
__device__ __forceinline__ void act_quant_body(const uint16_t *__restrict__ X, int64_t ldx, int64_t rows, int64_t K,
                                               uint8_t *__restrict__ out, int8_t *__restrict__ codes,
                                               float *__restrict__ dout, float *__restrict__ sout,
                                               uint16_t *__restrict__ xdeq, int64_t wg)
{
    const int64_t nb = K / 32;
    const int64_t blk = wg * 64 + (threadIdx.x >> 2);
    const int sub = threadIdx.x & 3; // elements 8*sub .. 8*sub+7 of the block
    const bool live = blk < rows * nb;
    const int64_t row = live ? blk / nb : 0;
    const int64_t j = live ? blk - row * nb : 0;

    u32x4 v = {0, 0, 0, 0};
    if (live) v = ld16(X + row * ldx + 32 * j + 8 * sub);
    if constexpr (MODE == ACT_F8 || MODE == ACT_F8DEQ) {
        const F8Quad f = f8_quad(v); // (every lane: DPP quad groups)
        if (!live) return;
        if constexpr (MODE == ACT_F8DEQ) {
            *(u32x4 *)(xdeq + row * K + 32 * j + 8 * sub) = (u32x4){f.xt[0], f.xt[1], f.xt[2], f.xt[3]};
            return;
        }
        *(u32x2 *)(codes + row * K + 32 * j + 8 * sub) = (u32x2){f.codes[0], f.codes[1]};
        if (sub == 0) dout[j * ((rows + 3) & ~(int64_t)3) + row] = __builtin_bit_cast(float, (uint32_t)(127 + f.e) << 23);
        return;
    }
    const Q81Quad q = q8_1_quad(v);
    if (!live) return;

    if constexpr (MODE == ACT_AOS) {
        uint8_t *o = out + blk * 36;
        __builtin_memcpy(o + 4 + 8 * sub, q.codes, 8);
        if (sub == 0) {
            const uint32_t ds = (uint32_t)f2h_bits(q.d) | ((uint32_t)q.sbits << 16);
            __builtin_memcpy(o, &ds, 4);
        }
    } else if constexpr (MODE == ACT_SOA) {
        *(u32x2 *)(codes + row * K + 32 * j + 8 * sub) = (u32x2){q.codes[0], q.codes[1]};
        if (sub == 0) {
            dout[row * nb + j] = q.d;
            sout[row * nb + j] = h2f(q.sbits);
        }
    } else if constexpr (MODE == ACT_I8) {
        *(u32x2 *)(codes + row * K + 32 * j + 8 * sub) = (u32x2){q.codes[0], q.codes[1]};
        if (sub == 0) {
            dout[j * ((rows + 3) & ~(int64_t)3) + row] = q.d;
            if (sout) sout[j * ((rows + 3) & ~(int64_t)3) + row] = h2f(q.sbits); // (the integer-MFMA skinny kernel's s)
        }
    } else {
        // x~ = fp16(d*q); each 4-element group in the order (0,2,1,3): the order mmq_gemm.hip's
        // packed dequantization produces weight pairs in (its k-permutation; the MFMA k-sum is
        // unchanged)
        uint32_t o[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float v4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v4[i] = q.d * (float)(int8_t)((q.codes[h] >> (8 * i)) & 0xff);
            o[2 * h] = (uint32_t)f2h_bits(v4[0]) | ((uint32_t)f2h_bits(v4[2]) << 16);
            o[2 * h + 1] = (uint32_t)f2h_bits(v4[1]) | ((uint32_t)f2h_bits(v4[3]) << 16);
        }
        *(u32x4 *)(xdeq + row * K + 32 * j + 8 * sub) = (u32x4){o[0], o[1], o[2], o[3]};
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void act_quant_kernel(const uint16_t *__restrict__ X, int64_t ldx, int64_t rows,
                                                        int64_t K, uint8_t *__restrict__ out, int8_t *__restrict__ codes,
                                                        float *__restrict__ dout, float *__restrict__ sout,
                                                        uint16_t *__restrict__ xdeq)
{
    act_quant_body<MODE>(X, ldx, rows, K, out, codes, dout, sout, xdeq, (int64_t)blockIdx.x);
}

// Several tensors' DEQ (q8_1) or F8DEQ (fp8 variant) forms in one launch (gq_act_prepare_grouped):
// segment i owns workgroups [wg0, wg0 + its blocks / 64), each running the one-tensor body --
// bit-identical to its own launch.
struct DeqSegs {
    int n;
    DeqSeg s[kMaxDeqSegs];
};

template <int MODE>
__global__ __launch_bounds__(256) void act_quant_deq_grouped_kernel(const DeqSegs a)
{
    const int64_t b = (int64_t)blockIdx.x;
    int i = 0;
    while (i + 1 < a.n && b >= a.s[i + 1].wg0) ++i;
    const DeqSeg &q = a.s[i];
    act_quant_body<MODE>(q.X, q.ldx, q.rows, q.K, nullptr, nullptr, nullptr, nullptr, q.xdeq, b - q.wg0);
}

hipError_t launch_act_quant_deq_grouped(const DeqSeg *segs, int n, hipStream_t s, int mode)
{
    if (n < 1 || n > kMaxDeqSegs || (mode != ACT_DEQ && mode != ACT_F8DEQ)) return hipErrorInvalidValue;
    DeqSegs a{};
    a.n = n;
    int64_t wg = 0;
    for (int i = 0; i < n; ++i) {
        a.s[i] = segs[i];
        a.s[i].wg0 = wg;
        wg += (segs[i].rows * (segs[i].K / 32) + 63) / 64;
    }
    if (wg == 0) return hipSuccess;
    if (mode == ACT_F8DEQ) act_quant_deq_grouped_kernel<ACT_F8DEQ><<<dim3((unsigned)wg), dim3(256), 0, s>>>(a);
    else act_quant_deq_grouped_kernel<ACT_DEQ><<<dim3((unsigned)wg), dim3(256), 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_act_quant(int mode, const uint16_t *X, int64_t ldx, int64_t rows, int64_t K, void *out0,
                            void *out1, void *out2, hipStream_t s)
{
    const int64_t nblk = rows * (K / 32);
    if (nblk == 0) return hipSuccess;
    dim3 grid((unsigned)((nblk + 63) / 64)), block(256);
    switch (mode) {
    case ACT_AOS:
        act_quant_kernel<ACT_AOS><<<grid, block, 0, s>>>(X, ldx, rows, K, (uint8_t *)out0, nullptr, nullptr,
                                                          nullptr, nullptr);
        break;
    case ACT_SOA:
        act_quant_kernel<ACT_SOA><<<grid, block, 0, s>>>(X, ldx, rows, K, nullptr, (int8_t *)out0, (float *)out1,
                                                          (float *)out2, nullptr);
        break;
    case ACT_F8:
        act_quant_kernel<ACT_F8><<<grid, block, 0, s>>>(X, ldx, rows, K, nullptr, (int8_t *)out0, (float *)out1,
                                                         nullptr, nullptr);
        break;
    case ACT_F8DEQ:
        act_quant_kernel<ACT_F8DEQ><<<grid, block, 0, s>>>(X, ldx, rows, K, nullptr, nullptr, nullptr, nullptr,
                                                            (uint16_t *)out0);
        break;
    case ACT_I8:
        act_quant_kernel<ACT_I8><<<grid, block, 0, s>>>(X, ldx, rows, K, nullptr, (int8_t *)out0, (float *)out1,
                                                         (float *)out2, nullptr);
        break;
    default:
        act_quant_kernel<ACT_DEQ><<<grid, block, 0, s>>>(X, ldx, rows, K, nullptr, nullptr, nullptr, nullptr,
                                                          (uint16_t *)out0);
        break;
    }
    return hipGetLastError();
}

} // namespace gq
