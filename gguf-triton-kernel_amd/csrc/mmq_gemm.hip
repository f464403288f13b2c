// mmq_gemm.hip -- batched MMQ (many tokens) on the fp16 matrix cores.
//
// C[t][m] = sum_k W[m][k] * x~[t][k], W dequantized in registers from the packed GGUF
// blocks, x~ = fp16(d*q) the q8_1-quantized activation (act_quant.hip, DEQ form), both fed
// to v_mfma_f32_16x16x32_f16 with fp32 accumulation.  fp16 (not bf16) operands: the
// reference's activations are fp16, and bf16 would drop three of their mantissa bits.
//
// Tile: a 256-thread workgroup owns BM=64 weight rows x BN=64 tokens; its 4 waves split
// that 2x2 into 32x32 sub-tiles (2x2 MFMA tiles of 16x16 each).  K advances one 256-wide
// step at a time (one Q4_K/Q6_K super-block, eight Q8_0 blocks):
//   1. the 64-token x 256-k activation tile is copied to LDS (16-byte loads / ds_write_b128,
//      rows padded by 16 B so the 16-lane ds_read_b128 groups hit distinct banks);
//   2. every lane loads ITS weight bytes for the step straight from HBM -- lane (r, kg)
//      needs elements 32s+8kg..+7 of row r for s = 0..7 -- and dequantizes them to 8
//      fp16 fragments per row tile (w = d*q, d*sc*q - dmin*m, d*sc*(q-32));
//   3. 8 sub-steps x 2x2 MFMAs, B fragments read from LDS.
// MFMA operand maps (gfx950 16x16x32 f16): lane l holds A[row l&15][k 8(l>>4)+j] and
// B[k 8(l>>4)+j][col l&15]; D[row 4(l>>4)+i][col l&15] in acc element i.
#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"

namespace gq {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64, BN = 64, KS = 256;
constexpr int LDS_ROW = KS * 2 + 16; // bytes per token row in LDS (padded)

// Eight sub-step fragments of one weight row for K-step kb: frag[s][j] = W[row][256kb+32s+8kg+j].
template <int F>
__device__ __forceinline__ void load_afrag(const uint8_t *__restrict__ rowp, int64_t kb, int kg, int64_t nb32,
                                           f16x8 (&frag)[8])
{
    if constexpr (F == Q8_0) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int64_t blk = 8 * kb + s;
            if (blk < nb32) {
                const uint8_t *p = rowp + 34 * blk;
                const float d = h2f(ld2(p));
                const u32x2 q = ld8(p + 2 + 8 * kg);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t w = j < 4 ? q.x : q.y;
                    const int v = (int)(int8_t)((w >> (8 * (j & 3))) & 0xff);
                    frag[s][j] = (_Float16)(d * (float)v);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) frag[s][j] = (_Float16)0.f;
            }
        }
    } else if constexpr (F == Q4_K) {
        const uint8_t *p = rowp + 144 * kb;
        const u32x4 hdr = ld16(p);
        const float d = h2f(hdr.x & 0xffffu), dmin = h2f(hdr.x >> 16);
        const uint32_t sw[3] = {hdr.y, hdr.z, hdr.w};
#pragma unroll
        for (int pch = 0; pch < 4; ++pch) {
            const u32x2 q = ld8(p + 16 + 32 * pch + 8 * kg);
#pragma unroll
            for (int hi = 0; hi < 2; ++hi) {
                const int s = 2 * pch + hi;
                int sc, m;
                q4k_sc_m(sw, s, sc, m);
                const float ds = d * (float)sc, dm = dmin * (float)m;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t w = j < 4 ? q.x : q.y;
                    const int v = (int)((w >> (8 * (j & 3) + 4 * hi)) & 0xf);
                    frag[s][j] = (_Float16)(ds * (float)v - dm);
                }
            }
        }
    } else {
        const uint8_t *p = rowp + 210 * kb;
        const float d = h2f(ld2(p + 208));
        const u32x4 sc = ld16(p + 192);
        const uint32_t scw[4] = {sc.x, sc.y, sc.z, sc.w};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const u32x2 qh = ld8(p + 128 + 32 * h + 8 * kg);
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const u32x2 ql = ld8(p + 64 * h + 32 * c + 8 * kg);
#pragma unroll
                for (int nib = 0; nib < 2; ++nib) {
                    const int s = 4 * h + 2 * nib + c; // s&1 = c, (s>>1)&1 = nib, s>>2 = h
                    const int si = 2 * s + (kg >> 1);
                    const float ds = d * (float)(int8_t)((scw[si >> 2] >> (8 * (si & 3))) & 0xff);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t lw = j < 4 ? ql.x : ql.y;
                        const uint32_t hw = j < 4 ? qh.x : qh.y;
                        const int lo = (int)((lw >> (8 * (j & 3) + 4 * nib)) & 0xf);
                        const int hb = (int)((hw >> (8 * (j & 3) + 2 * (s & 3))) & 0x3);
                        frag[s][j] = (_Float16)(ds * (float)((lo | (hb << 4)) - 32));
                    }
                }
            }
        }
    }
}

template <int F>
__global__ __launch_bounds__(256) void gemm_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                   uint16_t *__restrict__ C, int64_t M, int64_t N, int64_t K,
                                                   int64_t ldc)
{
    using L = Layout<F>;
    __shared__ __attribute__((aligned(16))) uint8_t Bs[BN * LDS_ROW];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
    const int64_t row_bytes = (K / L::QK) * L::BYTES;
    const int64_t nb32 = K / 32;
    const int64_t ksteps = (K + KS - 1) / KS;
    const int r16 = lane & 15, kg = lane >> 4;

    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const uint8_t *rowp[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int64_t r = m0 + 32 * wm + 16 * i + r16;
        rowp[i] = A + (r < M ? r : M - 1) * row_bytes;
    }

    for (int64_t kb = 0; kb < ksteps; ++kb) {
        // 1. activation tile -> LDS: 64 tokens x 512 B; thread handles 8 x 16 B
        __syncthreads();
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int idx = it * 256 + tid; // 2048 chunks of 16 B
            const int trow = idx >> 5, chunk = idx & 31;
            const int64_t tok = n0 + trow;
            const int64_t k = kb * KS + 8 * chunk;
            u32x4 v = {0, 0, 0, 0};
            if (tok < N && k < K) v = ld16(X + tok * K + k);
            *(u32x4 *)(Bs + trow * LDS_ROW + 16 * chunk) = v;
        }
        __syncthreads();

        // 2. weight fragments for this step
        f16x8 fa[2][8];
#pragma unroll
        for (int i = 0; i < 2; ++i) load_afrag<F>(rowp[i], kb, kg, nb32, fa[i]);

        // 3. MFMAs
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            f16x8 fb[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int trow = 32 * wn + 16 * j + r16;
                fb[j] = *(const f16x8 *)(Bs + trow * LDS_ROW + 2 * (32 * s + 8 * kg));
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i][s], fb[j], acc[i][j], 0, 0, 0);
        }
    }

    // epilogue: lane holds rows 4kg..4kg+3 of token column r16 -> 8 contiguous bytes of C
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int64_t tok = n0 + 32 * wn + 16 * j + r16;
            const int64_t row = m0 + 32 * wm + 16 * i + 4 * kg;
            if (tok >= N) continue;
            uint16_t *cp = C + tok * ldc + row;
            if (row + 3 < M) {
                u32x2 o;
                o.x = (uint32_t)f2h_bits(acc[i][j][0]) | ((uint32_t)f2h_bits(acc[i][j][1]) << 16);
                o.y = (uint32_t)f2h_bits(acc[i][j][2]) | ((uint32_t)f2h_bits(acc[i][j][3]) << 16);
                __builtin_memcpy(cp, &o, 8);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (row + e < M) cp[e] = f2h_bits(acc[i][j][e]);
            }
        }
    }
}

} // namespace

hipError_t launch_gemm(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, int64_t M, int64_t N, int64_t K,
                       int64_t ldc, hipStream_t s)
{
    dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((N + BN - 1) / BN)), block(256);
    switch (fmt) {
    case Q8_0: gemm_kernel<Q8_0><<<grid, block, 0, s>>>(A, X, C, M, N, K, ldc); break;
    case Q4_K: gemm_kernel<Q4_K><<<grid, block, 0, s>>>(A, X, C, M, N, K, ldc); break;
    default: gemm_kernel<Q6_K><<<grid, block, 0, s>>>(A, X, C, M, N, K, ldc); break;
    }
    return hipGetLastError();
}

} // namespace gq
