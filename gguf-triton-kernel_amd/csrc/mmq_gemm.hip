// mmq_gemm.hip -- batched MMQ (many tokens) on the fp16 matrix cores.
//
// C[t][m] = sum_k W[m][k] * x~[t][k]: W dequantized in registers from the packed GGUF
// blocks, x~ = fp16(d*q) the q8_1-quantized activation (act_quant.hip, DEQ form) -- the same
// integer activations kernels/cpu_impls multiplies (mmq_*_q8_1_cpu.py) -- fed to
// v_mfma_f32_32x32x16_f16 with fp32 accumulation.  fp16 operands, not bf16: the reference's
// activations are fp16 and bf16 would drop three of their mantissa bits.
//
// Work decomposition
//   workgroup = 4 waves = 128 weight rows x 32*NT tokens (NT = 1..4 token tiles of 32);
//   wave w owns rows 32w..32w+31 of the tile and all NT token tiles (NT accumulators of
//   32x32 f32).  K advances in 128-element chunks; grid.z splits the chunks (split-K) when
//   the row x token tiles alone would not fill the chip -- fp32 partial slabs, summed in
//   fixed order by gemm_reduce_kernel (deterministic).
// Per chunk
//   B (activations): the 32*NT x 128 fp16 tile goes HBM/L2 -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, no VGPRs), double-buffered so chunk c+1 streams in while
//     chunk c is multiplied.  LDS rows are 256 B; 16-byte pieces are XOR-swizzled by
//     (row & 15) on the SOURCE address (the DMA destination is lane-linear), and reads apply
//     the same XOR, so each 16-lane ds_read_b128 group touches 16 distinct bank quads.
//   A (weights): lane (row = lane&31, half = lane>>5) loads its 64-weight "unit" u = 2c+half
//     straight from HBM with 16-byte loads (gguf_units.hpp), one chunk ahead, and
//     dequantizes 8 weights per MFMA k-step into fp16 in registers.  The 64 weights of a
//     unit are mapped onto the 8 k-steps of the chunk in whatever order the unit stores
//     them; the B fragment is read from LDS with the same permutation (MFMA sums over k,
//     so any consistent permutation is exact).
// MFMA 32x32x16 f16 operand maps (gfx950): lane l holds A[row l&31][k 8(l>>5)+j] and
// B[k 8(l>>5)+j][col l&31]; D[row (i&3)+8(i>>2)+4(l>>5)][col l&31] in acc element i.
#include <cstdlib>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_units.hpp"

namespace gq {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int KC = 128;         // K elements per chunk
constexpr int ROW_B = KC * 2;   // LDS bytes per token row of a chunk
constexpr int BM = 128;         // weight rows per workgroup

__device__ __forceinline__ uint32_t pk_f16(float a, float b)
{
    return (uint32_t)f2h_bits(a) | ((uint32_t)f2h_bits(b) << 16);
}

__device__ __forceinline__ f16x8 as_f16x8(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    u32x4 v = {a, b, c, d};
    return __builtin_bit_cast(f16x8, v);
}

// fp16 fragment for k-step t (0..7) of a unit: 8 weights.
template <int F>
__device__ __forceinline__ f16x8 unit_frag(const UnitRaw<F> &r, int t);

template <>
__device__ __forceinline__ f16x8 unit_frag<Q8_0>(const UnitRaw<Q8_0> &r, int t)
{
    const float d = t < 4 ? r.d0 : r.d1;
    const uint32_t w0 = r.w[2 * t], w1 = r.w[2 * t + 1];
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = d * (float)(int8_t)((w0 >> (8 * j)) & 0xff);
        v[4 + j] = d * (float)(int8_t)((w1 >> (8 * j)) & 0xff);
    }
    return as_f16x8(pk_f16(v[0], v[1]), pk_f16(v[2], v[3]), pk_f16(v[4], v[5]), pk_f16(v[6], v[7]));
}

template <>
__device__ __forceinline__ f16x8 unit_frag<Q4_K>(const UnitRaw<Q4_K> &r, int t)
{
    const int tt = t & 3, sh = t < 4 ? 0 : 4;
    const float ds = t < 4 ? r.ds0 : r.ds1, dm = t < 4 ? r.dm0 : r.dm1;
    const uint32_t w0 = r.w[2 * tt] >> sh, w1 = r.w[2 * tt + 1] >> sh;
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = ds * (float)((w0 >> (8 * j)) & 0xf) - dm;
        v[4 + j] = ds * (float)((w1 >> (8 * j)) & 0xf) - dm;
    }
    return as_f16x8(pk_f16(v[0], v[1]), pk_f16(v[2], v[3]), pk_f16(v[4], v[5]), pk_f16(v[6], v[7]));
}

template <>
__device__ __forceinline__ f16x8 unit_frag<Q6_K>(const UnitRaw<Q6_K> &r, int t)
{
    const int tt = t & 3;
    const uint32_t *c = t < 4 ? r.ca : r.cb;
    const float s = t < 4 ? (tt < 2 ? r.fa1 : r.fa2) : (tt < 2 ? r.fb1 : r.fb2);
    const uint32_t w0 = c[2 * tt], w1 = c[2 * tt + 1];
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = s * (float)((int)((w0 >> (8 * j)) & 0xff) - 32);
        v[4 + j] = s * (float)((int)((w1 >> (8 * j)) & 0xff) - 32);
    }
    return as_f16x8(pk_f16(v[0], v[1]), pk_f16(v[2], v[3]), pk_f16(v[4], v[5]), pk_f16(v[6], v[7]));
}

// Which 8-element piece (0..15) of the 128-wide chunk k-step t of half h multiplies.
template <int F>
__device__ __forceinline__ int piece_of(int h, int t)
{
    if constexpr (F == Q6_K) return t < 4 ? 4 * h + t : 8 + 4 * h + (t - 4);
    return 8 * h + t;
}

// Issue the LDS-DMA for chunk c of the activation tile into `buf` (tokens n0.., 32*NT rows).
template <int NT>
__device__ __forceinline__ void stage_b(uint8_t *buf, const uint16_t *__restrict__ X, int64_t n0, int64_t N,
                                        int64_t K, int64_t c, int wave, int lane)
{
    constexpr int INSTR = 8 * NT; // 1 KiB (4 token rows) per wave-instruction
#pragma unroll
    for (int q = wave; q < INSTR; q += 4) {
        const int row = 4 * q + (lane >> 4);
        const int piece = (lane & 15) ^ (row & 15);
        int64_t tok = n0 + row;
        tok = tok < N ? tok : N - 1;
        int64_t k = c * KC + 8 * piece;
        k = k < K - 8 ? k : K - 8;
        __builtin_amdgcn_global_load_lds((const void *)(X + tok * K + k), (lds_void *)(buf + q * 1024), 16, 0, 0);
    }
}

template <int F, int NT>
__global__ __launch_bounds__(256) void gemm_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                   uint16_t *__restrict__ C, float *__restrict__ P, int64_t M,
                                                   int64_t N, int64_t K, int64_t ldc, int chunks_per_split)
{
    using L = Layout<F>;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * 32 * NT * ROW_B];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, r32 = lane & 31;
    const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * 32 * NT;
    const int64_t nchunks = (K + KC - 1) / KC;
    const int64_t c0 = (int64_t)blockIdx.z * chunks_per_split;
    const int64_t c1 = c0 + chunks_per_split < nchunks ? c0 + chunks_per_split : nchunks;
    const int64_t row_bytes = (K / L::QK) * L::BYTES;
    const int64_t nb32 = K / 32;

    int64_t row = m0 + 32 * wave + r32;
    const uint8_t *rowp = A + (row < M ? row : M - 1) * row_bytes;

    f32x16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

    UnitRaw<F> nxt;
    if (c0 < c1) {
        stage_b<NT>(lds, X, n0, N, K, c0, wave, lane);
        nxt.load(rowp, (int)(2 * c0 + h), nb32);
    }
    __syncthreads();

    for (int64_t c = c0; c < c1; ++c) {
        const UnitRaw<F> cur = nxt;
        uint8_t *buf = lds + ((c - c0) & 1) * (32 * NT * ROW_B);
        if (c + 1 < c1) {
            stage_b<NT>(lds + ((c + 1 - c0) & 1) * (32 * NT * ROW_B), X, n0, N, K, c + 1, wave, lane);
            nxt.load(rowp, (int)(2 * (c + 1) + h), nb32);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f16x8 a = unit_frag<F>(cur, t);
            const int piece = piece_of<F>(h, t);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int trow = 32 * nt + r32;
                const f16x8 b = *(const f16x8 *)(buf + trow * ROW_B + 16 * (piece ^ (trow & 15)));
                acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[nt], 0, 0, 0);
            }
        }
        __syncthreads();
    }

    // epilogue: acc[nt][i] = D[row 32w + (i&3) + 8(i>>2) + 4h][token 32nt + r32]
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int64_t tok = n0 + 32 * nt + r32;
        if (tok >= N) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t rr = m0 + 32 * wave + 8 * g + 4 * h;
            const float v0 = acc[nt][4 * g], v1 = acc[nt][4 * g + 1], v2 = acc[nt][4 * g + 2], v3 = acc[nt][4 * g + 3];
            if (P == nullptr) {
                uint16_t *cp = C + tok * ldc + rr;
                if (rr + 3 < M) {
                    u32x2 o = {pk_f16(v0, v1), pk_f16(v2, v3)};
                    __builtin_memcpy(cp, &o, 8);
                } else {
                    const float vv[4] = {v0, v1, v2, v3};
                    for (int e = 0; e < 4; ++e)
                        if (rr + e < M) cp[e] = f2h_bits(vv[e]);
                }
            } else {
                float *pp = P + ((int64_t)blockIdx.z * N + tok) * M + rr;
                const float vv[4] = {v0, v1, v2, v3};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (rr + e < M) pp[e] = vv[e];
            }
        }
    }
}

// C[t][m] = fp16(sum_s P[s][t][m]), summed in split order (deterministic).
__global__ __launch_bounds__(256) void gemm_reduce_kernel(const float *__restrict__ P, uint16_t *__restrict__ C,
                                                          int64_t M, int64_t N, int64_t ldc, int S)
{
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= N * M) return;
    const int64_t tok = idx / M, m = idx - tok * M;
    float acc = 0.f;
    for (int s = 0; s < S; ++s) acc += P[((int64_t)s * N + tok) * M + m];
    C[tok * ldc + m] = f2h_bits(acc);
}

template <int F, int NT>
hipError_t launch_nt(const uint8_t *A, const uint16_t *X, uint16_t *C, float *P, int S, int cps, int64_t M, int64_t N,
                     int64_t K, int64_t ldc, hipStream_t s)
{
    dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((N + 32 * NT - 1) / (32 * NT)), (unsigned)S), block(256);
    gemm_kernel<F, NT><<<grid, block, 0, s>>>(A, X, C, S > 1 ? P : nullptr, M, N, K, ldc, cps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || S == 1) return e;
    const int64_t work = N * M;
    gemm_reduce_kernel<<<dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s>>>(P, C, M, N, ldc, S);
    return hipGetLastError();
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const uint16_t *X, uint16_t *C, float *P, int S, int cps, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    const int nt = N >= 97 ? 4 : (N >= 65 ? 3 : (N >= 33 ? 2 : 1));
    switch (nt) {
    case 1: return launch_nt<F, 1>(A, X, C, P, S, cps, M, N, K, ldc, s);
    case 2: return launch_nt<F, 2>(A, X, C, P, S, cps, M, N, K, ldc, s);
    case 3: return launch_nt<F, 3>(A, X, C, P, S, cps, M, N, K, ldc, s);
    default: return launch_nt<F, 4>(A, X, C, P, S, cps, M, N, K, ldc, s);
    }
}

} // namespace

GemmPlan plan_gemm(int64_t M, int64_t N, int64_t K)
{
    GemmPlan p;
    const int nt = N >= 97 ? 4 : (N >= 65 ? 3 : (N >= 33 ? 2 : 1));
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + 32 * nt - 1) / (32 * nt));
    const int64_t nchunks = (K + KC - 1) / KC;
    const int64_t target = 256; // one workgroup per CU
    int64_t S = tiles >= target ? 1 : (target + tiles / 2) / tiles;
    if (const char *env = getenv("GQ_GEMM_SPLITS")) S = atoll(env); // tuning / test override
    const int64_t max_split = nchunks / 4 > 0 ? nchunks / 4 : 1; // >= 4 chunks per split
    if (S > max_split) S = max_split;
    if (S < 1) S = 1;
    int64_t cps = (nchunks + S - 1) / S;
    S = (nchunks + cps - 1) / cps;
    p.splits = (int)S;
    p.chunks_per_split = (int)cps;
    p.partial_bytes = S > 1 ? (size_t)S * N * M * sizeof(float) : 0;
    return p;
}

hipError_t launch_gemm(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, float *P, const GemmPlan &plan,
                       int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, X, C, P, plan.splits, plan.chunks_per_split, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, X, C, P, plan.splits, plan.chunks_per_split, M, N, K, ldc, s);
    default: return launch_fmt<Q6_K>(A, X, C, P, plan.splits, plan.chunks_per_split, M, N, K, ldc, s);
    }
}

} // namespace gq
