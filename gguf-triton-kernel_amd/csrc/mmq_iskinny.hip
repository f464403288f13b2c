// mmq_iskinny.hip -- the skinny-token MMQ (5..16 tokens) on INTEGER MFMA: Q4_K weights as int8
// nibbles x q8_1 activation codes in v_mfma_i32_16x16x32_i8, one 32-element block per MFMA
// k-step, rescaled per block into fp32 -- the reference's own per-block arithmetic
// (kernels/cpu_impls/mmq_q4_k_q8_1_cpu.py: d*sc * sum(q_w q_x) * d_x - dmin*m * s_x), where the
// fp16 skinny kernel (mmq_skinny.hip) dequantizes every weight to fp16 and multiplies the
// activations' fp16 x~.
//
// Shape (the fp16 skinny kernel's): a persistent grid of <= one workgroup per CU, each a
// contiguous range of units of 16*RG weight rows; its 8 waves split K into 8 ranges; per
// super-block of its range a wave loads its lanes' weight bytes straight into registers and
// DMAs the super-block's activation codes (16 tokens x 256 B) and block scales into a private
// LDS ring; the ranges' partial tiles are summed in LDS in fixed order per unit.  The int8
// form moves half the activation bytes of the fp16 one (codes, not x~) and replaces the
// per-weight fp16 dequantization by a per-block rescale of the 16x16 int32 tile.
//
// MFMA roles: A = activations (16 tokens x 32 codes: lane l -> token l&15, codes 8(l>>4)..+7
// of the block), B = weights (32 nibbles x 16 rows: lane l -> row l&15, nibbles 8(l>>4)..+7);
// D[token 4(l>>4)+i][row l&15] in lane l's element i.  So a lane's accumulators are four tokens
// of ONE weight row: the row's d*sc of the block times each token's d_x, and the min term
// -dmin*m (per row, block) x s_x (per token, block) as one v_mfma_f32_16x16x4_f32 per four blocks
// (A = s_x: token x block, B = -dmin*m: block x row).
//
// Activations: act_quant's I8 form -- codes int8 [N][K], d and s fp32 block-major [K/32][ldd].
#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_mfma.hpp"

namespace gq {
namespace {

typedef int i32x4v __attribute__((ext_vector_type(4)));

constexpr int IW = 8;                 // waves per workgroup = K ranges
constexpr int XCODE = 16 * 256;       // one super-block's codes of 16 tokens (4 DMA instructions)
constexpr int XSC = 2 * 8 * 16 * 4;   // its d and s, [2][8 blocks][16 tokens] fp32 (1 instruction)
constexpr int XSLOT = XCODE + XSC;

// Q4_K 6-bit scale / min of sub-block b (get_scale_min_k4) from the header words y, z, w
__device__ __forceinline__ void q4k_scale_min(const u32x4 &h, int b, int &sc, int &m)
{
    if (b < 4) {
        sc = (h.y >> (8 * b)) & 63;
        m = (h.z >> (8 * b)) & 63;
    } else {
        const int k = 8 * (b - 4);
        const uint32_t hi = (h.w >> k) & 0xffu;
        sc = (hi & 0x0f) | (((h.y >> k) & 0xc0u) >> 2);
        m = (hi >> 4) | (((h.z >> k) & 0xc0u) >> 2);
    }
}

// Xd: d [K/32][ldd], then s at Xd + sdelta bytes (the workspace's I8 form: one buffer resource)
template <int RG, int D>
__global__ __launch_bounds__(64 * IW) void iskinny_q4k_kernel(const uint8_t *__restrict__ A, const int8_t *__restrict__ Xq,
                                                             const float *__restrict__ Xd, uint32_t sdelta, int64_t ldd,
                                                             uint16_t *__restrict__ C, int M, int N, int K, int ldc,
                                                             int nunits)
{
    __shared__ __attribute__((aligned(1024))) uint8_t xlds[IW * D * XSLOT + 1024];
    __shared__ __attribute__((aligned(16))) float red[IW * RG * 256];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c = lane & 15;
    const int u0 = (int)((int64_t)blockIdx.x * nunits / gridDim.x);
    const int u1 = (int)((int64_t)(blockIdx.x + 1) * nunits / gridDim.x);
    const int nsb = K / 256, nb = K / 32;
    const int sb0 = wave * nsb / IW, nsw = (wave + 1) * nsb / IW - sb0; // this wave's super-blocks per unit
    const int row_bytes = nsb * 144;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, M * row_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc((void *)Xq, 0, N * K, 0x00020000);
    const __amdgpu_buffer_rsrc_t drs =
        __builtin_amdgcn_make_buffer_rsrc((void *)Xd, 0, (int)(sdelta + (uint32_t)(nb * ldd * 4)), 0x00020000);
    uint8_t *ring = xlds + wave * (D * XSLOT);
    uint8_t *scratch = xlds + IW * D * XSLOT;
    // codes: DMA instruction i moves tokens 4i..4i+3; lane l -> token 4i + (l>>4), LDS piece
    // pp = l&15 of that token's 256 B, holding the token's piece pp ^ token (a block's 16 token
    // reads -- token t, piece 2b + (g>>1) -- land on 16 distinct pieces)
    uint32_t qsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int t = 4 * i + g, q = c ^ t;
        const int tok = t < N ? t : N - 1;
        qsrc[i] = (uint32_t)tok * (uint32_t)K + 16u * (uint32_t)q;
    }
    // scales: lanes 0..31 -> d pieces, 32..63 -> s pieces; piece (b, quad) = 4 tokens of block b
    const int sb_b = (lane & 31) >> 2, sb_q = lane & 3;
    const uint32_t ssrc = (uint32_t)(sb_b * ldd + 4 * sb_q) * 4u + (lane < 32 ? 0u : sdelta); // (+ 8 sb ldd 4: block-major)

    f32x4 acc[RG];
#pragma unroll
    for (int rf = 0; rf < RG; ++rf) acc[rf] = (f32x4){0.f, 0.f, 0.f, 0.f};

    auto finish = [&](int u) __attribute__((always_inline)) {
        const int m0 = u * 16 * RG;
#pragma unroll
        for (int rf = 0; rf < RG; ++rf) {
            *(f32x4 *)(red + (wave * RG + rf) * 256 + 4 * lane) = acc[rf];
            acc[rf] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (int q = tid; q < RG * 64; q += 64 * IW) {
            const int rf = q >> 6, l = q & 63;
            f32x4 v = *(const f32x4 *)(red + rf * 256 + 4 * l);
#pragma unroll
            for (int k = 1; k < IW; ++k) v += *(const f32x4 *)(red + (k * RG + rf) * 256 + 4 * l);
            const int row = m0 + 16 * rf + (l & 15);
            if (row < M) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int tok = 4 * (l >> 4) + i;
                    if (tok < N) C[(size_t)tok * ldc + row] = f2h_bits(v[i]);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); // red may be rewritten
    };

    if (nsw > 0) {
        const int total = (u1 - u0) * nsw;
        u32x4 hdr[D][RG];
        u32x2 qs[D][RG][4];
        auto load = [&](int b, int j) __attribute__((always_inline)) {
            const int u = u0 + j / nsw, sb = sb0 + j % nsw;
#pragma unroll
            for (int rf = 0; rf < RG; ++rf) {
                const int row = u * 16 * RG + 16 * rf + c;
                const uint32_t v = (uint32_t)((row < M ? row : M - 1) * row_bytes), s0 = (uint32_t)(144 * sb);
                hdr[b][rf] = __builtin_amdgcn_raw_buffer_load_b128(wrs, v, s0, 0);
#pragma unroll
                for (int p = 0; p < 4; ++p)
                    qs[b][rf][p] = __builtin_amdgcn_raw_buffer_load_b64(wrs, v + 16u + 32u * p + 8u * g, s0, 0);
            }
            uint8_t *dst = ring + b * XSLOT;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lds_void *)(dst + 1024 * i), 16, qsrc[i], (uint32_t)(256 * sb), 0, 0);
            // scales of blocks 8sb..8sb+7 (lanes 32..63 from s): [d|s][b][16 tokens]
            __builtin_amdgcn_raw_ptr_buffer_load_lds(drs, (lds_void *)(dst + XCODE), 16, ssrc, (uint32_t)(8 * sb * ldd * 4), 0, 0);
        };
        auto compute = [&](int b) __attribute__((always_inline)) {
            const uint8_t *xs = ring + b * XSLOT;
            const float *dx = (const float *)(xs + XCODE), *sx = dx + 128;
            // s_x of this lane's (token c, blocks g and g + 4): the A operand of the min MFMAs
            const float sxa = sx[16 * g + c], sxb = sx[16 * (g + 4) + c];
#pragma unroll
            for (int rf = 0; rf < RG; ++rf) {
                const u32x4 h = hdr[b][rf];
                const float dmin = h2f(h.x >> 16);
                int scg, mg, sch, mh;
                q4k_scale_min(h, g, scg, mg);
                q4k_scale_min(h, g + 4, sch, mh);
                acc[rf] = __builtin_amdgcn_mfma_f32_16x16x4f32(sxa, -(dmin * (float)mg), acc[rf], 0, 0, 0);
                acc[rf] = __builtin_amdgcn_mfma_f32_16x16x4f32(sxb, -(dmin * (float)mh), acc[rf], 0, 0, 0);
            }
#pragma unroll
            for (int blk = 0; blk < 8; ++blk) {
                // A: token c's codes 8g..8g+7 of block blk (piece 2blk + (g>>1), swizzled by token)
                const u32x2 xa = *(const u32x2 *)(xs + 256 * c + 16 * ((2 * blk + (g >> 1)) ^ c) + 8 * (g & 1));
                const f32x4 dxv = *(const f32x4 *)(dx + 16 * blk + 4 * g); // d_x of tokens 4g..4g+3
#pragma unroll
                for (int rf = 0; rf < RG; ++rf) {
                    const u32x2 w = qs[b][rf][blk >> 1];
                    const u32x2 wb = (blk & 1) ? (u32x2){(w.x >> 4) & 0x0f0f0f0fu, (w.y >> 4) & 0x0f0f0f0fu}
                                               : (u32x2){w.x & 0x0f0f0f0fu, w.y & 0x0f0f0f0fu};
                    const i32x4v r = __builtin_amdgcn_mfma_i32_16x16x32_i8(__builtin_bit_cast(long, xa), __builtin_bit_cast(long, wb),
                                                                          (i32x4v){0, 0, 0, 0}, 0, 0, 0);
                    int sc, m;
                    q4k_scale_min(hdr[b][rf], blk, sc, m);
                    const float ds = h2f(hdr[b][rf].x & 0xffffu) * (float)sc;
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[rf][i] = __builtin_fmaf(ds * dxv[i], (float)r[i], acc[rf][i]);
                }
            }
        };
        constexpr int PER_SB = RG * 5 + 5; // weight loads + 4 code DMAs + 1 scale DMA
        static_assert((D - 1) * PER_SB <= 63, "vmcnt range");
        auto body = [&](int j, int b) __attribute__((always_inline)) {
            __builtin_amdgcn_sched_barrier(0);
            const int younger = total - 1 - j < D - 1 ? total - 1 - j : D - 1;
            vm_wait<(D - 1) * PER_SB>(younger * PER_SB);
            __builtin_amdgcn_sched_barrier(0);
            compute(b);
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (j + D < total) load(b, j + D);
            if ((j + 1) % nsw == 0) finish(u0 + j / nsw);
        };
#pragma unroll
        for (int b = 0; b < D; ++b)
            if (b < total) load(b, b);
        int j = 0;
        for (; j + D - 1 < total; j += D) {
#pragma unroll
            for (int b = 0; b < D; ++b) body(j + b, b);
        }
#pragma unroll
        for (int b = 0; b < D - 1; ++b)
            if (j + b < total) body(j + b, b);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int u = u0; u < u1; ++u) finish(u);
    }
    (void)scratch;
}

template <int RG>
hipError_t launch_rg(const uint8_t *A, const int8_t *Xq, const float *Xd, const float *Xs, int64_t ldd, uint16_t *C,
                     int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    const int64_t nunits = (M + 16 * RG - 1) / (16 * RG);
    const unsigned grid = (unsigned)(nunits < num_cus() ? nunits : num_cus());
    const uint32_t sdelta = (uint32_t)((const uint8_t *)Xs - (const uint8_t *)Xd);
    iskinny_q4k_kernel<RG, 2><<<dim3(grid), dim3(64 * IW), 0, s>>>(A, Xq, Xd, sdelta, ldd, C, (int)M, (int)N, (int)K,
                                                                  (int)ldc, (int)nunits);
    return hipGetLastError();
}

} // namespace

int iskinny_rg(int64_t M)
{
    if (tuning().iskinny_rg > 0) return tuning().iskinny_rg;
    // the fewest rows per unit that still give every CU a unit (more rows: fewer code re-reads)
    const int64_t frags = (M + 15) / 16, cus = num_cus();
    int rg = 4;
    while (rg > 1 && (frags + rg - 1) / rg < cus) --rg;
    return rg;
}

hipError_t launch_iskinny(int fmt, const uint8_t *A, const int8_t *Xq, const float *Xd, const float *Xs, int64_t ldd,
                          uint16_t *C, int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (fmt != Q4_K || N < 1 || N > 16 || K % 256 != 0 || M < 1 || Xs < Xd) return hipErrorInvalidValue;
    switch (iskinny_rg(M)) {
    case 1: return launch_rg<1>(A, Xq, Xd, Xs, ldd, C, M, N, K, ldc, s);
    case 2: return launch_rg<2>(A, Xq, Xd, Xs, ldd, C, M, N, K, ldc, s);
    case 3: return launch_rg<3>(A, Xq, Xd, Xs, ldd, C, M, N, K, ldc, s);
    default: return launch_rg<4>(A, Xq, Xd, Xs, ldd, C, M, N, K, ldc, s);
    }
}

} // namespace gq
