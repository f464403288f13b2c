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
// The activations are the A operand (MFMA rows = tokens) and the weights the B operand
// (MFMA columns = weight rows), so the accumulator's lane index runs along C's contiguous
// dimension.
#include <cstdlib>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_units.hpp"

namespace gq {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KC = 128;         // K elements per chunk
constexpr int ROW_B = KC * 2;   // LDS bytes per token row of a chunk
constexpr int BM = 128;         // weight rows per workgroup

__device__ __forceinline__ uint32_t pk_f16(float a, float b)
{
    return (uint32_t)f2h_bits(a) | ((uint32_t)f2h_bits(b) << 16);
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ h2 as_h2(uint32_t v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ uint32_t as_u32(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2 splat(float f) { return (h2){(_Float16)f, (_Float16)f}; }

__device__ __forceinline__ f16x8 as_f16x8(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    u32x4 v = {a, b, c, d};
    return __builtin_bit_cast(f16x8, v);
}

// Packed dequantization.  A fragment holds 8 weights of consecutive k in the element order
// (0,2,1,3,4,6,5,7): the pair (byte 0, byte 2) and the pair (byte 1, byte 3) of a code
// dword become one f16x2 each with a single AND-OR / PERM against the exponent pattern
// 0x64 (f16 1024 + v), the bias comes off with one packed add and the scale goes on with one
// packed mul/fma.  act_quant's DEQ form stores x~ in the same element order, so the MFMA's
// k-sum is unchanged.  Rounding: the integer codes are exact in f16; the per-block scales
// are rounded to f16 once (2^-11 relative), then one rounding per product.
__device__ __forceinline__ void bytes_pairs(uint32_t w, uint32_t &p02, uint32_t &p13)
{
    // w holds 4 unsigned byte codes; -> f16 (1024+code) pairs (c0,c2) and (c1,c3)
    p02 = __builtin_amdgcn_perm(0x64646464u, w, 0x04020400u);
    p13 = __builtin_amdgcn_perm(0x64646464u, w, 0x04030401u);
}

// fp16 fragment for k-step t (0..7) of a unit: 8 weights.
template <int F>
__device__ __forceinline__ f16x8 unit_frag(const UnitRaw<F> &r, int t);

template <>
__device__ __forceinline__ f16x8 unit_frag<Q8_0>(const UnitRaw<Q8_0> &r, int t)
{
    const h2 d = splat(t < 4 ? r.d0 : r.d1);
    const h2 bias = splat(-1152.f); // codes were biased by +128 (xor 0x80)
    uint32_t a0, a1, b0, b1;
    bytes_pairs(r.w[2 * t] ^ 0x80808080u, a0, a1);
    bytes_pairs(r.w[2 * t + 1] ^ 0x80808080u, b0, b1);
    return as_f16x8(as_u32((as_h2(a0) + bias) * d), as_u32((as_h2(a1) + bias) * d),
                    as_u32((as_h2(b0) + bias) * d), as_u32((as_h2(b1) + bias) * d));
}

template <>
__device__ __forceinline__ f16x8 unit_frag<Q4_K>(const UnitRaw<Q4_K> &r, int t)
{
    const int tt = t & 3;
    const uint32_t w0 = r.w[2 * tt], w1 = r.w[2 * tt + 1];
    const h2 bias = splat(-1024.f);
    uint32_t a0, a1, b0, b1;
    h2 ds, ndm;
    if (t < 4) { // low nibbles: code at bits 0 / 16 of (w) and of (w >> 8)
        ds = splat(r.ds0);
        ndm = splat(-r.dm0);
        a0 = (w0 & 0x000f000fu) | 0x64006400u;
        a1 = ((w0 >> 8) & 0x000f000fu) | 0x64006400u;
        b0 = (w1 & 0x000f000fu) | 0x64006400u;
        b1 = ((w1 >> 8) & 0x000f000fu) | 0x64006400u;
    } else { // high nibbles: take them at bits 4 / 20, i.e. 16 * code; fold the 1/16 into ds
        ds = splat(r.ds1 * 0.0625f);
        ndm = splat(-r.dm1);
        a0 = (w0 & 0x00f000f0u) | 0x64006400u;
        a1 = ((w0 >> 8) & 0x00f000f0u) | 0x64006400u;
        b0 = (w1 & 0x00f000f0u) | 0x64006400u;
        b1 = ((w1 >> 8) & 0x00f000f0u) | 0x64006400u;
    }
    return as_f16x8(as_u32(__builtin_elementwise_fma(as_h2(a0) + bias, ds, ndm)),
                    as_u32(__builtin_elementwise_fma(as_h2(a1) + bias, ds, ndm)),
                    as_u32(__builtin_elementwise_fma(as_h2(b0) + bias, ds, ndm)),
                    as_u32(__builtin_elementwise_fma(as_h2(b1) + bias, ds, ndm)));
}

template <>
__device__ __forceinline__ f16x8 unit_frag<Q6_K>(const UnitRaw<Q6_K> &r, int t)
{
    const int tt = t & 3;
    const uint32_t *c = t < 4 ? r.ca : r.cb;
    const h2 sc = splat(t < 4 ? (tt < 2 ? r.fa1 : r.fa2) : (tt < 2 ? r.fb1 : r.fb2));
    const h2 bias = splat(-1056.f); // 1024 + 32
    const uint32_t w0 = c[2 * tt], w1 = c[2 * tt + 1];
    const uint32_t a0 = (w0 & 0x003f003fu) | 0x64006400u, a1 = ((w0 >> 8) & 0x003f003fu) | 0x64006400u;
    const uint32_t b0 = (w1 & 0x003f003fu) | 0x64006400u, b1 = ((w1 >> 8) & 0x003f003fu) | 0x64006400u;
    return as_f16x8(as_u32((as_h2(a0) + bias) * sc), as_u32((as_h2(a1) + bias) * sc),
                    as_u32((as_h2(b0) + bias) * sc), as_u32((as_h2(b1) + bias) * sc));
}

// Which 8-element piece (0..15) of the 128-wide chunk k-step t of half h multiplies.
template <int F>
__device__ __forceinline__ int piece_of(int h, int t)
{
    if constexpr (F == Q6_K) return t < 4 ? 4 * h + t : 8 + 4 * h + (t - 4);
    return 8 * h + t;
}

// One pipeline stage in registers: this lane's weight unit for a chunk and its share of the
// chunk's activation tile (BP 16-byte pieces).
template <int F, int BP>
struct Stage {
    UnitLoad<F> a;
    int u;
    u32x4 b[BP];
};

// Activation tile piece p of chunk c (p = tid + i*NTHR): token row p>>4, 16-byte column p&15.
template <int NT, int NTHR, int BP>
__device__ __forceinline__ void load_b(u32x4 (&b)[BP], const uint16_t *__restrict__ X, int64_t n0, int64_t N,
                                       int64_t K, int64_t c, int tid)
{
#pragma unroll
    for (int i = 0; i < BP; ++i) {
        const int p = tid + i * NTHR;
        const int row = p >> 4, col = p & 15;
        int64_t tok = n0 + row;
        tok = tok < N ? tok : N - 1;
        int64_t k = c * KC + 8 * col;
        k = k < K - 8 ? k : K - 8;
        b[i] = ld16(X + tok * K + k);
    }
}

// ... and its store into the LDS image: rows of 256 B, 16-byte pieces XOR-swizzled by row&15
// (the read side applies the same XOR), so each 16-lane ds_read_b128 group of the MFMA's B
// fragment reads 16 distinct bank quads.
template <int NTHR, int BP>
__device__ __forceinline__ void store_b(uint8_t *buf, const u32x4 (&b)[BP], int tid)
{
#pragma unroll
    for (int i = 0; i < BP; ++i) {
        const int p = tid + i * NTHR;
        const int row = p >> 4, col = p & 15;
        *(u32x4 *)(buf + row * ROW_B + 16 * (col ^ (row & 15))) = b[i];
    }
}

// Workgroup = 4*WN waves: wave w owns weight rows 32*(w&3).. of the 128-row tile and token
// tiles [(w>>2)*NTW, (w>>2)*NTW + NTW) of the NT 32-token tiles (NTW = NT/WN).
//
// K pipeline, three register stages deep (all loads ordinary global loads, so the compiler
// counts them with partial vmcnt waits; no LDS-DMA, whose in-flight state would force
// vmcnt(0) at every barrier): in iteration c the wave issues chunk c+2's weight unit and
// activation pieces, writes chunk c+1's activation pieces (loaded one iteration ago) into
// the LDS buffer nobody reads this iteration, multiplies chunk c (weights from the stage
// loaded two iterations ago, activations from the other LDS buffer), then one barrier.
// ABL: ablation bitmask for performance diagnosis only (tools/ablate.sh); 0 in production.
//   1 = no MFMA, 2 = no weight loads, 4 = no activation global loads, 8 = no LDS B reads.
template <int F, int NT, int WN, int ABL = 0>
struct GemmCore {
    static constexpr int NTW = NT / WN, NW = 4 * WN, NTHR = 64 * NW;
    static constexpr int BP = (32 * NT * 16 + NTHR - 1) / NTHR; // 16-byte pieces per thread
    static_assert((32 * NT * 16) % NTHR == 0, "activation tile must split evenly");
    using St = Stage<F, BP>;

    const uint8_t *rowp;
    const uint16_t *X;
    int64_t n0, N, K, nb32;
    int tid, h, r32, wn;
    uint8_t *lds;

    __device__ __forceinline__ void issue(St &st, int64_t c) const
    {
        st.u = (int)(2 * c + h);
        if constexpr (ABL & 2) {
            const uint32_t z = (uint32_t)c * 0x01010101u + (uint32_t)tid;
            __builtin_memset(&st.a, 0, sizeof(st.a));
            *(uint32_t *)&st.a = z;
        } else {
            st.a.load(rowp, st.u, nb32);
        }
        if constexpr (ABL & 4) {
#pragma unroll
            for (int i = 0; i < BP; ++i) st.b[i] = (u32x4){(uint32_t)c, (uint32_t)tid, 1u, 2u};
        } else {
            load_b<NT, NTHR, BP>(st.b, X, n0, N, K, c, tid);
        }
    }

    __device__ __forceinline__ void compute(const St &st, const uint8_t *buf, f32x16 (&acc)[NTW]) const
    {
        const UnitRaw<F> unit = UnitRaw<F>::from(st.a, st.u, nb32);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f16x8 a = unit_frag<F>(unit, t);
            const int piece = piece_of<F>(h, t);
#pragma unroll
            for (int i = 0; i < NTW; ++i) {
                const int trow = 32 * (wn * NTW + i) + r32;
                f16x8 b;
                if constexpr (ABL & 8) b = a;
                else b = *(const f16x8 *)(buf + trow * ROW_B + 16 * (piece ^ (trow & 15)));
                if constexpr (ABL & 1) {
                    acc[i][t] += (float)a[i] + (float)b[t];
                } else {
                    // tokens on the MFMA's M side, weight rows on its N side: D[token][row], so
                    // a lane's outputs are one weight row and consecutive lanes store
                    // consecutive rows of C (coalesced epilogue)
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc[i], 0, 0, 0);
                }
            }
        }
    }

    // one iteration: cur = chunk c, nxt = chunk c+1 (loaded), fut <- chunk c+2.  Branch-free:
    // past the end the chunk index is clamped (a redundant load, a store into the buffer no
    // one reads again) so the compiler's vmcnt counting sees the same loads on every path.
    __device__ __forceinline__ void step(const St &cur, const St &nxt, St &fut, int64_t c, int64_t c0, int64_t c1,
                                         f32x16 (&acc)[NTW]) const
    {
        issue(fut, c + 2 < c1 ? c + 2 : c1 - 1);
        store_b<NTHR, BP>(lds + ((c + 1 - c0) & 1) * (32 * NT * ROW_B), nxt.b, tid);
        compute(cur, lds + ((c - c0) & 1) * (32 * NT * ROW_B), acc);
        __syncthreads();
    }
};

template <int F, int NT, int WN, int ABL = 0>
__global__ __launch_bounds__(256 * WN) void gemm_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                        uint16_t *__restrict__ C, float *__restrict__ P, int64_t M,
                                                        int64_t N, int64_t K, int64_t ldc, int chunks_per_split)
{
    using L = Layout<F>;
    using Core = GemmCore<F, NT, WN, ABL>;
    constexpr int NTW = Core::NTW;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * 32 * NT * ROW_B];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 3;
    const int64_t m0 = (int64_t)blockIdx.x * BM;
    const int64_t nchunks = (K + KC - 1) / KC;
    const int64_t c0 = (int64_t)blockIdx.z * chunks_per_split;
    const int64_t c1 = c0 + chunks_per_split < nchunks ? c0 + chunks_per_split : nchunks;
    const int64_t row_bytes = (K / L::QK) * L::BYTES;
    const int64_t row = m0 + 32 * wm + (lane & 31);

    Core core;
    core.rowp = A + (row < M ? row : M - 1) * row_bytes;
    core.X = X;
    core.n0 = (int64_t)blockIdx.y * 32 * NT;
    core.N = N;
    core.K = K;
    core.nb32 = K / 32;
    core.tid = tid;
    core.h = lane >> 5;
    core.r32 = lane & 31;
    core.wn = wave >> 2;
    core.lds = lds;

    f32x16 acc[NTW];
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

    typename Core::St s0, s1, s2;
    if (c0 < c1) {
        core.issue(s0, c0);
        core.issue(s1, c0 + 1 < c1 ? c0 + 1 : c1 - 1);
        store_b<Core::NTHR, Core::BP>(lds, s0.b, tid);
        __syncthreads();
        int64_t c = c0;
        for (; c + 3 <= c1; c += 3) {
            core.step(s0, s1, s2, c, c0, c1, acc);
            core.step(s1, s2, s0, c + 1, c0, c1, acc);
            core.step(s2, s0, s1, c + 2, c0, c1, acc);
        }
        if (c < c1) core.step(s0, s1, s2, c, c0, c1, acc);
        if (c + 1 < c1) core.step(s1, s2, s0, c + 1, c0, c1, acc);
    }

    // epilogue: acc[i][e] = D[token 32(wn*NTW+i) + (e&3) + 8(e>>2) + 4h][row 32wm + r32]; each
    // store instruction writes two runs of 32 consecutive rows (one per half-wave)
    const int h = lane >> 5, r32 = lane & 31, wn = wave >> 2;
    const int64_t n0 = core.n0;
    const int64_t rr = m0 + 32 * wm + r32;
    if (rr < M) {
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t tok = n0 + 32 * (wn * NTW + i) + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (tok >= N) continue;
                if (P == nullptr) C[tok * ldc + rr] = f2h_bits(acc[i][e]);
                else P[((int64_t)blockIdx.z * N + tok) * M + rr] = acc[i][e];
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

template <int F, int NT, int WN>
hipError_t launch_nt(const uint8_t *A, const uint16_t *X, uint16_t *C, float *P, int S, int cps, int64_t M, int64_t N,
                     int64_t K, int64_t ldc, hipStream_t s)
{
    dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((N + 32 * NT - 1) / (32 * NT)), (unsigned)S),
        block(256 * WN);
#ifdef GQ_ABLATION
    if constexpr (NT == 4) {
        static const int abl = getenv("GQ_ABLATE") ? atoi(getenv("GQ_ABLATE")) : 0;
        float *PP = S > 1 ? P : nullptr;
        switch (abl) {
        case 1: gemm_kernel<F, NT, WN, 1><<<grid, block, 0, s>>>(A, X, C, PP, M, N, K, ldc, cps); break;
        case 2: gemm_kernel<F, NT, WN, 2><<<grid, block, 0, s>>>(A, X, C, PP, M, N, K, ldc, cps); break;
        case 4: gemm_kernel<F, NT, WN, 4><<<grid, block, 0, s>>>(A, X, C, PP, M, N, K, ldc, cps); break;
        case 8: gemm_kernel<F, NT, WN, 8><<<grid, block, 0, s>>>(A, X, C, PP, M, N, K, ldc, cps); break;
        case 6: gemm_kernel<F, NT, WN, 6><<<grid, block, 0, s>>>(A, X, C, PP, M, N, K, ldc, cps); break;
        case 9: gemm_kernel<F, NT, WN, 9><<<grid, block, 0, s>>>(A, X, C, PP, M, N, K, ldc, cps); break;
        case 15: gemm_kernel<F, NT, WN, 15><<<grid, block, 0, s>>>(A, X, C, PP, M, N, K, ldc, cps); break;
        default: gemm_kernel<F, NT, WN><<<grid, block, 0, s>>>(A, X, C, PP, M, N, K, ldc, cps); break;
        }
    } else
#endif
    gemm_kernel<F, NT, WN><<<grid, block, 0, s>>>(A, X, C, S > 1 ? P : nullptr, M, N, K, ldc, cps);
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
    case 1: return launch_nt<F, 1, 1>(A, X, C, P, S, cps, M, N, K, ldc, s);
    case 2: return launch_nt<F, 2, 2>(A, X, C, P, S, cps, M, N, K, ldc, s);
    case 3: return launch_nt<F, 3, 1>(A, X, C, P, S, cps, M, N, K, ldc, s);
    default: return launch_nt<F, 4, 2>(A, X, C, P, S, cps, M, N, K, ldc, s);
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
