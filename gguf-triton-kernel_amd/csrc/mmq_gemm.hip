// mmq_gemm.hip -- batched MMQ (many tokens) on the fp16 matrix cores, LDS-DMA staged.
//
// C[t][m] = sum_k W[m][k] * x~[t][k]: W dequantized in registers from the packed GGUF bytes,
// x~ = fp16(d*q) the q8_1-quantized activation (act_quant.hip, DEQ form) -- the integer
// activations kernels/cpu_impls multiplies (mmq_*_q8_1_cpu.py) -- into
// v_mfma_f32_16x16x32_f16 with fp32 accumulation.  fp16 rather than bf16: the reference's
// activations are fp16 and bf16 would drop three of their mantissa bits.
//
// Workgroup = 4 waves = BM = 64*RG weight rows x BN = 16*NB tokens.  Wave w owns rows
// 16*(RG*w + rg) + [0,16) (rg < RG) and every token of the tile: each weight is dequantized
// once per workgroup; the activation tile is shared through LDS.  Large BM matters: every
// stage moves 2*BN bytes of activations per K element beside BM*bytes/weight of weights, and
// the per-CU L2->LDS rate, not the MFMA, is what a small tile runs into.
//
// K advances in stages of 64 elements (2 MFMA k-steps of 32).  Everything a stage needs is
// moved HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no ds_write):
//   weights     : per row the stage's raw block bytes (Stage<F> below), 16-byte pieces at
//                 whatever (2-byte) alignment the blocks have (gfx950 runs unaligned);
//   activations : BN token rows x 128 B, 16-byte pieces XOR-swizzled by ((row >> 1) & 7) on
//                 the SOURCE side (the DMA destination is lane-linear) so the MFMA
//                 fragment ds_read_b128s of a 16-lane group hit 16 distinct bank quads.
// A ring of 4 stage buffers keeps three stages in flight while one is multiplied; one
// s_barrier per stage, preceded by a counted vmcnt (never vmcnt(0) inside the loop).
//
// MFMA 16x16x32 f16 maps (gfx950): lane l holds A[row l&15][k 8(l>>4)+j] and
// B[k 8(l>>4)+j][col l&15]; D[row 4(l>>4)+i][col l&15] in acc element i.  Weight rows are the
// A rows and tokens the B columns, so lane l ends with 4 consecutive weight rows of one token:
// one 8-byte store per (row group, token group) in the epilogue.
// The 8 k of a fragment are taken in the element order (0,2,1,3,4,6,5,7) in which packed
// dequantization produces them; act_quant's DEQ form stores x~ in the same order.
#include <cstdlib>
#include <type_traits>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"

namespace gq {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int KC = 64;     // K elements per stage
constexpr int NSTAGE = 4;  // ring depth (3 stages in flight)
constexpr int LDS_MAX = 160 * 1024;

__device__ __forceinline__ h2 as_h2(uint32_t v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ uint32_t as_u32(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2 splat(float f) { return (h2){(_Float16)f, (_Float16)f}; }
__device__ __forceinline__ f16x8 frag4(h2 a, h2 b, h2 c, h2 d)
{
    u32x4 v = {as_u32(a), as_u32(b), as_u32(c), as_u32(d)};
    return __builtin_bit_cast(f16x8, v);
}
// f16 pairs (1024 + code) from codes masked into the low bits of bytes 0 and 2
__device__ __forceinline__ h2 magic(uint32_t v, uint32_t mask) { return as_h2((v & mask) | 0x64006400u); }
// f16 pairs (1024 + byte) of bytes (0,2) and (1,3) of a code word
__device__ __forceinline__ h2 pair02(uint32_t c) { return as_h2(__builtin_amdgcn_perm(0x64646464u, c, 0x04020400u)); }
__device__ __forceinline__ h2 pair13(uint32_t c) { return as_h2(__builtin_amdgcn_perm(0x64646464u, c, 0x04030401u)); }

// ---------------------------------------------------------------------------------------
// Per-format stage geometry.  A stage's weight bytes arrive as NP 16-byte pieces per row.
// Q4_K/Q6_K pieces are stored piece-major in LDS ([j][row][16 B]) so that one DMA
// instruction moves piece j of 64 consecutive rows and the stage-dependent part of its source
// offset is wave-uniform (SGPR soffset); Q8_0 pieces are row-major ([row][5 x 16 B]) because
// its stage offset (68 B per stage) is the same for every piece.
template <int F> struct Stage;

// Q4_K: stage c = quarter q = c&3 of super-block c>>2 = sub-blocks 2q (low nibbles) and 2q+1
// (high nibbles) of qs bytes 32q..32q+31.  Pieces: 0 = d,dmin,scales | 1,2 = qs[32q..+32).
template <> struct Stage<Q4_K> {
    static constexpr int NP = 3;
    __device__ static uint32_t soff(int64_t c, int j)
    {
        return (uint32_t)(144 * (c >> 2)) + (j == 0 ? 0u : (uint32_t)(16 * j + 32 * (c & 3)));
    }
    __device__ static uint32_t act_soff(int64_t c) { return (uint32_t)(2 * KC * c); }
    __device__ static uint32_t act_voff(int p) { return 16u * p; }
};

// Q6_K: stage c = (super-block c>>2, half h = (c>>1)&1, v = c&1): k-step 0 = elements
// 128h+32v+[0,32) (ql low nibbles, qh bits 2v), k-step 1 = 128h+64+32v+[0,32) (ql high
// nibbles, qh bits 4+2v).  Pieces: 0,1 = ql[64h+32v..+32) | 2,3 = qh[32h..+32) |
// 4 = scales[0..16) | 5 = block bytes 194..209 (d at offset 14).
template <> struct Stage<Q6_K> {
    static constexpr int NP = 6;
    __device__ static uint32_t soff(int64_t c, int j)
    {
        const int h = (int)(c >> 1) & 1, v = (int)c & 1;
        const int o = j < 2 ? 64 * h + 32 * v + 16 * j : (j < 4 ? 128 + 32 * h + 16 * (j - 2) : (j == 4 ? 192 : 194));
        return (uint32_t)(210 * (c >> 2)) + (uint32_t)o;
    }
    __device__ static uint32_t act_soff(int64_t c)
    {
        return (uint32_t)(2 * (256 * (c >> 2) + 128 * ((c >> 1) & 1) + 32 * (c & 1)));
    }
    __device__ static uint32_t act_voff(int p) { return 2u * (64 * (p >> 2) + 8 * (p & 3)); }
};

// Q8_0: stage c = blocks 2c, 2c+1 (68 B).  Row-major pieces: [0,64) bytes 0..63 | [64,80)
// bytes 52..67 (a read of bytes [x, x+8) with x+8 > 64 goes to LDS x + 12).
template <> struct Stage<Q8_0> {
    static constexpr int NP = 5;
    __device__ static uint32_t piece_base(int j) { return j < 4 ? 16u * j : 52u; }
    __device__ static uint32_t act_soff(int64_t c) { return (uint32_t)(2 * KC * c); }
    __device__ static uint32_t act_voff(int p) { return 16u * p; }
};

constexpr int NWAVE = 8; // 512 threads: two waves per SIMD

template <int F, int NB, int RG>
struct Cfg {
    static constexpr int BN = 16 * NB, BM = 16 * RG * NWAVE;
    static constexpr int NP = Stage<F>::NP;
    static constexpr int W_INS = BM * NP / 64;          // weight DMA instructions per stage (workgroup)
    static constexpr int A_INS = BN * 8 / 64;           // activation DMA instructions per stage
    static constexpr int NI = W_INS + A_INS;
    static constexpr int MAXI = (NI + NWAVE - 1) / NWAVE; // per wave (waves w < NI % 8 own one more)
    static constexpr int MINI = NI / NWAVE;
    static constexpr int STAGE_BYTES = NI * 1024;
    static constexpr int LDS_BYTES = NSTAGE * STAGE_BYTES;
    static_assert(BM * NP % 64 == 0 && BN * 8 % 64 == 0, "whole DMA instructions");
    static_assert(LDS_BYTES <= LDS_MAX, "LDS budget");
    static_assert(2 * MAXI <= 63, "vmcnt range");
};

// ---------------------------------------------------------------------------------------
// A fragments of one stage for one 16-row group: frag[s] = the 8 weights (fragment element
// order) of k-step s for this lane's row and k-group g.  pc(j) = the row's piece j in LDS.
template <int F, class PC>
__device__ __forceinline__ void stage_frags(PC pc, int g, int64_t c, f16x8 (&frag)[2]);

template <int F, class PC>
__device__ __forceinline__ typename std::enable_if<F == Q4_K>::type
stage_frags_impl(PC pc, int g, int64_t c, f16x8 (&frag)[2])
{
    const int q = (int)c & 3;
    const u32x4 hdr = *(const u32x4 *)pc(0);
    const float d = h2f(hdr.x & 0xffffu), dmin = h2f(hdr.x >> 16);
    // 6-bit scales / mins of sub-blocks 2q, 2q+1, one per byte (get_scale_min_k4)
    const uint32_t sc = q < 2 ? (hdr.y & 0x3f3f3f3fu) : ((hdr.w & 0x0f0f0f0fu) | ((hdr.y >> 2) & 0x30303030u));
    const uint32_t mn = q < 2 ? (hdr.z & 0x3f3f3f3fu) : (((hdr.w >> 4) & 0x0f0f0f0fu) | ((hdr.z >> 2) & 0x30303030u));
    const int sh = 16 * (q & 1);
    const u32x2 w = *(const u32x2 *)(pc(1 + (g >> 1)) + 8 * (g & 1));
    const h2 bias = splat(-1024.f);
#pragma unroll
    for (int n = 0; n < 2; ++n) { // n = 0: low nibbles (sub-block 2q), 1: high (2q+1)
        const h2 ds = splat(d * (float)((sc >> (sh + 8 * n)) & 0xffu));
        const h2 ndm = splat(-(dmin * (float)((mn >> (sh + 8 * n)) & 0xffu)));
        const uint32_t x0 = w.x >> (4 * n), x1 = w.y >> (4 * n);
        frag[n] = frag4(__builtin_elementwise_fma(magic(x0, 0x000f000fu) + bias, ds, ndm),
                        __builtin_elementwise_fma(magic(x0 >> 8, 0x000f000fu) + bias, ds, ndm),
                        __builtin_elementwise_fma(magic(x1, 0x000f000fu) + bias, ds, ndm),
                        __builtin_elementwise_fma(magic(x1 >> 8, 0x000f000fu) + bias, ds, ndm));
    }
}

template <int F, class PC>
__device__ __forceinline__ typename std::enable_if<F == Q6_K>::type
stage_frags_impl(PC pc, int g, int64_t c, f16x8 (&frag)[2])
{
    const int h = (int)(c >> 1) & 1, v = (int)c & 1;
    const float d = h2f(*(const uint16_t *)(pc(5) + 14));
    const u32x2 ql = *(const u32x2 *)(pc(g >> 1) + 8 * (g & 1));
    const u32x2 qh = *(const u32x2 *)(pc(2 + (g >> 1)) + 8 * (g & 1));
    const uint8_t *scp = pc(4);
    const h2 bias = splat(-1056.f); // 1024 + 32
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        // sub-block of elements 128h + 64n + 32v + 8g..: 8h + 4n + 2v + (g >> 1)
        const float scv = (float)*(const int8_t *)(scp + 8 * h + 4 * n + 2 * v + (g >> 1));
        const h2 dsc = splat(d * scv);
        const int sq = 4 * n + 2 * v;
        const uint32_t c0 = ((ql.x >> (4 * n)) & 0x0f0f0f0fu) | (((qh.x >> sq) & 0x03030303u) << 4);
        const uint32_t c1 = ((ql.y >> (4 * n)) & 0x0f0f0f0fu) | (((qh.y >> sq) & 0x03030303u) << 4);
        frag[n] = frag4((pair02(c0) + bias) * dsc, (pair13(c0) + bias) * dsc, (pair02(c1) + bias) * dsc,
                        (pair13(c1) + bias) * dsc);
    }
}

template <int F, class PC>
__device__ __forceinline__ typename std::enable_if<F == Q8_0>::type
stage_frags_impl(PC pc, int g, int64_t /*c*/, f16x8 (&frag)[2])
{
    const uint8_t *wr = pc(0); // row-major: the row's 80 bytes
    const h2 bias = splat(-1152.f); // codes biased by +128 (xor 0x80)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const h2 d = splat(h2f(*(const uint16_t *)(wr + 34 * b)));
        int x = 34 * b + 2 + 8 * g;
        if (b == 1) x = x + 8 > 64 ? x + 12 : x;
        const u32x2 q = *(const u32x2 *)(wr + x); // 2-byte aligned: gfx950 LDS runs unaligned
        const uint32_t c0 = q.x ^ 0x80808080u, c1 = q.y ^ 0x80808080u;
        frag[b] = frag4((pair02(c0) + bias) * d, (pair13(c0) + bias) * d, (pair02(c1) + bias) * d,
                        (pair13(c1) + bias) * d);
    }
}

template <int F, class PC>
__device__ __forceinline__ void stage_frags(PC pc, int g, int64_t c, f16x8 (&frag)[2])
{
    stage_frags_impl<F>(pc, g, c, frag);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, uint8_t *lds_dst, uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void *)lds_dst, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ int act_swz(int r) { return (r >> 1) & 7; }

// ---------------------------------------------------------------------------------------
// ABL: ablation bitmask for performance diagnosis (diagnostic build -DGQ_ABLATION only; 0 in
// production): 1 = no MFMA, 2 = no weight DMA, 4 = no activation DMA, 8 = no dequantization.
template <int F, int NB, int RG, int ABL = 0>
__global__ __launch_bounds__(512) void gemm_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                   uint16_t *__restrict__ C, float *__restrict__ P, int64_t M,
                                                   int64_t N, int64_t K, int64_t ldc, int stages_per_split)
{
    using G = Cfg<F, NB, RG>;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[G::LDS_BYTES];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, l16 = lane & 15;
    const int64_t m0 = (int64_t)blockIdx.x * G::BM;
    const int64_t n0 = (int64_t)blockIdx.y * G::BN;
    const int64_t nstages = K / KC;
    const int64_t c0 = (int64_t)blockIdx.z * stages_per_split;
    const int64_t c1 = c0 + stages_per_split < nstages ? c0 + stages_per_split : nstages;
    const int64_t row_bytes = (K / Layout<F>::QK) * Layout<F>::BYTES;

    // buffer descriptors (byte offsets are 32-bit: tensors < 4 GiB, checked on the host)
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, (int)(uint32_t)(M * row_bytes),
                                                                         0x00020000);
    const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, (int)(uint32_t)(N * K * 2),
                                                                         0x00020000);

    // this wave's DMA instructions k = wave + 8i: weights for k < W_INS, activations after;
    // per instruction a fixed per-lane voffset, the stage part goes to soffset
    uint32_t voff[G::MAXI];
    int kj[G::MAXI]; // weight piece index j (K-quants) of the instruction
#pragma unroll
    for (int i = 0; i < G::MAXI; ++i) {
        const int k = wave + NWAVE * i;
        kj[i] = 0;
        voff[i] = 0;
        if (k < G::W_INS) {
            if constexpr (F == Q8_0) {
                const int p = 64 * k + lane, r = p / 5, j = p - 5 * r; // row-major pieces
                const int64_t row = m0 + r < M ? m0 + r : M - 1;
                voff[i] = (uint32_t)(row * row_bytes) + Stage<F>::piece_base(j);
            } else {
                constexpr int RBLK = G::BM / 64;
                kj[i] = k / RBLK;
                const int64_t r = m0 + 64 * (k - kj[i] * RBLK) + lane;
                voff[i] = (uint32_t)((r < M ? r : M - 1) * row_bytes);
            }
        } else if (k < G::NI) {
            const int p = 64 * (k - G::W_INS) + lane, r = p >> 3, q = p & 7;
            const int64_t tok = n0 + r < N ? n0 + r : N - 1;
            voff[i] = (uint32_t)(tok * K * 2) + Stage<F>::act_voff(q ^ act_swz(r));
        }
    }
    const int my_ins = G::MINI + (wave < G::NI % NWAVE ? 1 : 0);

    auto issue = [&](int64_t c, int buf) {
        uint8_t *base = lds + buf * G::STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < G::MAXI; ++i) {
            const int k = wave + NWAVE * i;
            if (k < G::W_INS) {
                if constexpr (!(ABL & 2)) {
                    uint32_t so;
                    if constexpr (F == Q8_0) so = (uint32_t)(68 * c);
                    else so = Stage<F>::soff(c, kj[i]);
                    dma16(wrs, base + 1024 * k, voff[i], so);
                }
            } else if (k < G::NI) {
                if constexpr (!(ABL & 4)) dma16(ars, base + 1024 * k, voff[i], Stage<F>::act_soff(c));
            }
        }
    };
    auto wait_stage = [&]() { // all but this wave's two youngest stages landed, then barrier
        if constexpr (ABL & 6) {
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        } else if (my_ins == G::MAXI) {
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * G::MAXI) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * G::MINI) : "memory");
        }
    };

    f32x4 acc[RG][NB];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[rg][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

    if (c0 < c1) {
#pragma unroll
        for (int i = 0; i < NSTAGE - 1; ++i) issue(c0 + i < c1 ? c0 + i : c1 - 1, i);
        int buf = 0;
        for (int64_t c = c0; c < c1; ++c) {
            // stage c landed (stages c+1, c+2 may still be in flight); all waves done with c-1
            wait_stage();
            issue(c + NSTAGE - 1 < c1 ? c + NSTAGE - 1 : c1 - 1, buf == 0 ? NSTAGE - 1 : buf - 1);
            const uint8_t *ws = lds + buf * G::STAGE_BYTES;
            const uint8_t *xs = ws + 1024 * G::W_INS;
            f16x8 af[RG][2];
#pragma unroll
            for (int rg = 0; rg < RG; ++rg) {
                const int row = 16 * (RG * wave + rg) + l16;
                if constexpr (ABL & 8) {
                    af[rg][0] = *(const f16x8 *)(ws + 16 * row);
                    af[rg][1] = *(const f16x8 *)(ws + 16 * row + 16 * G::BM);
                } else if constexpr (F == Q8_0) {
                    stage_frags<F>([&](int) { return ws + 80 * row; }, g, c, af[rg]);
                } else {
                    stage_frags<F>([&](int j) { return ws + 16 * (j * G::BM + row); }, g, c, af[rg]);
                }
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const int r = 16 * t + l16;
                    const f16x8 b = *(const f16x8 *)(xs + 128 * r + 16 * ((4 * s + g) ^ act_swz(r)));
#pragma unroll
                    for (int rg = 0; rg < RG; ++rg) {
                        if constexpr (ABL & 1) acc[rg][t][0] += (float)af[rg][s][t & 7] * (float)b[rg & 7];
                        else acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[rg][s], b, acc[rg][t], 0, 0, 0);
                    }
                }
            }
            buf = buf == NSTAGE - 1 ? 0 : buf + 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // no DMA may land after the workgroup exits
    }

    // epilogue: acc[rg][t][i] = D[row 16(RG*wave+rg) + 4g + i][token 16t + l16]
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        const int64_t tok = n0 + 16 * t + l16;
        if (tok >= N) continue;
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
            const int64_t row = m0 + 16 * (RG * wave + rg) + 4 * g;
            if (row >= M) continue;
            const f32x4 v = acc[rg][t];
            if (P == nullptr) {
                uint16_t *dst = C + tok * ldc + row;
                if (row + 4 <= M) {
                    const u32x2 o = {(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                     (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)};
                    *(u32x2 *)dst = o; // 2-byte aligned when ldc or M is odd: unaligned store
                } else {
                    for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(v[i]);
                }
            } else {
                float *dst = P + ((int64_t)blockIdx.z * N + tok) * M + row;
                if (row + 4 <= M) *(f32x4 *)dst = v;
                else
                    for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = v[i];
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

template <int F, int NB, int RG>
hipError_t launch_cfg(const uint8_t *A, const uint16_t *X, uint16_t *C, float *P, const GemmPlan &pl, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    using G = Cfg<F, NB, RG>;
    dim3 grid((unsigned)((M + G::BM - 1) / G::BM), (unsigned)((N + G::BN - 1) / G::BN), (unsigned)pl.splits);
    float *PP = pl.splits > 1 ? P : nullptr;
#ifdef GQ_ABLATION
    const int abl = getenv("GQ_ABLATE") ? atoi(getenv("GQ_ABLATE")) : 0;
    switch (abl) {
    case 1: gemm_kernel<F, NB, RG, 1><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split); break;
    case 2: gemm_kernel<F, NB, RG, 2><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split); break;
    case 4: gemm_kernel<F, NB, RG, 4><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split); break;
    case 6: gemm_kernel<F, NB, RG, 6><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split); break;
    case 8: gemm_kernel<F, NB, RG, 8><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split); break;
    case 9: gemm_kernel<F, NB, RG, 9><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split); break;
    case 14: gemm_kernel<F, NB, RG, 14><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split); break;
    default: gemm_kernel<F, NB, RG><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split); break;
    }
#else
    gemm_kernel<F, NB, RG><<<grid, dim3(512), 0, s>>>(A, X, C, PP, M, N, K, ldc, pl.chunks_per_split);
#endif
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || pl.splits == 1) return e;
    const int64_t work = N * M;
    gemm_reduce_kernel<<<dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s>>>(P, C, M, N, ldc, pl.splits);
    return hipGetLastError();
}

template <int F, int RG>
hipError_t launch_rg(const uint8_t *A, const uint16_t *X, uint16_t *C, float *P, const GemmPlan &pl, int64_t M,
                     int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (pl.nb) {
    case 1: return launch_cfg<F, 1, RG>(A, X, C, P, pl, M, N, K, ldc, s);
    case 2: return launch_cfg<F, 2, RG>(A, X, C, P, pl, M, N, K, ldc, s);
    case 4: return launch_cfg<F, 4, RG>(A, X, C, P, pl, M, N, K, ldc, s);
    default: return launch_cfg<F, 8, RG>(A, X, C, P, pl, M, N, K, ldc, s);
    }
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const uint16_t *X, uint16_t *C, float *P, const GemmPlan &pl, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (pl.rg == 1) return launch_rg<F, 1>(A, X, C, P, pl, M, N, K, ldc, s);
    return launch_rg<F, 2>(A, X, C, P, pl, M, N, K, ldc, s);
}

int pick_nb(int64_t N) { return N > 64 ? 8 : (N > 32 ? 4 : (N > 16 ? 2 : 1)); }

} // namespace

bool gemm_supported(int /*fmt*/, int64_t K) { return K > 0 && K % KC == 0; }

GemmPlan plan_gemm(int fmt, int64_t M, int64_t N, int64_t K)
{
    (void)fmt;
    GemmPlan p;
    p.nb = pick_nb(N);
    if (const char *env = getenv("GQ_GEMM_NB")) p.nb = atoi(env);
    const int64_t nstages = K / KC;
    const int64_t tn = (N + 16 * p.nb - 1) / (16 * p.nb);
    const int64_t target = 256; // one workgroup per CU
    // rows per workgroup: 256 (the activation tile is re-read once per 256 weight rows);
    // 128 only when even split-K cannot fill the chip
    const int64_t max_split = nstages / 16 > 0 ? nstages / 16 : 1; // >= 16 stages per split
    p.rg = ((M + 255) / 256) * tn * max_split < target ? 1 : 2;
    if (const char *env = getenv("GQ_GEMM_RG")) p.rg = atoi(env) == 1 ? 1 : 2;
    const int64_t tiles = ((M + 128 * p.rg - 1) / (128 * p.rg)) * tn;
    int64_t S = tiles >= target ? 1 : (target + tiles / 2) / tiles;
    if (const char *env = getenv("GQ_GEMM_SPLITS")) S = atoll(env); // tuning / test override
    if (S > max_split) S = max_split;
    if (S < 1) S = 1;
    int64_t sps = (nstages + S - 1) / S;
    S = (nstages + sps - 1) / sps;
    p.splits = (int)S;
    p.chunks_per_split = (int)sps;
    p.partial_bytes = S > 1 ? (size_t)S * N * M * sizeof(float) : 0;
    return p;
}

hipError_t launch_gemm(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, float *P, const GemmPlan &plan,
                       int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, X, C, P, plan, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, X, C, P, plan, M, N, K, ldc, s);
    default: return launch_fmt<Q6_K>(A, X, C, P, plan, M, N, K, ldc, s);
    }
}

} // namespace gq
