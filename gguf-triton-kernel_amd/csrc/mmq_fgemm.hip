// mmq_fgemm.hip -- the full-K tile GEMM: one workgroup per (32*RW weight rows, 16*NB tokens,
// ALL of K), so no split-K partials and no reduce launch.
//
// Why (round 5, profiles/r05/abl.txt): the resident-split GEMM (mmq_rgemm.hip, one super-block
// of K per workgroup) spends most of its time outside the multiply on the M = 128 shapes -- on
// Q8_0 4096^2 x 128 its 16.7 us are 4.9 us of split-K partial stores (16.8 MB, the size of the
// weights), ~3 us of the reduce launch reading them back, and a 5 us floor of two launches; the
// weights' HBM stream is 4.4 us.  Here every output is finished inside one workgroup: the
// workgroup's 8 waves are RW row groups x KW = 8/RW K-interleaved waves, wave (r, k) multiplying
// rows [32r, 32r+32) of the tile against super-blocks k, k+KW, k+2KW, ... and the KW partial
// tiles are summed in LDS (fixed order) at the end.  What it costs instead: each weight byte is
// read by the N/(16*NB) token tiles (the first from HBM, the rest L2 hits: a row tile's token
// tiles are blockIdx.y apart with gridDim.x % 8 == 0, i.e. on one XCD) and each workgroup reads
// its tokens' activations over all of K.
//
// Operands.  A (weights) are private to a wave: its lanes load their bytes of the step's
// super-block straight into VGPRs (gguf_wfrag.hpp WB<F>, 16-byte buffer loads) one step ahead and
// dequantize them in registers.  B (the prepared fp16 x~, act_quant's DEQ form) is shared by the
// RW row groups: each step's KW super-blocks x 16*NB tokens land in one of two LDS slots by
// LDS-DMA (every wave issues 1/8 of the step's 1 KiB instructions: a token's 512-byte run, two
// tokens per instruction, XOR-swizzled on the source as the skinny kernel's ring), read back
// as B fragments by ds_read_b128.  Step j: wait for this wave's loads of step j, one workgroup
// barrier (every wave's DMAs of step j landed; every wave is past step j-1, so its slot is
// free), issue step j+1, multiply step j.
//
// Arithmetic = the skinny kernel's (mmq_skinny.hip) per fragment: WB<F>::frag dequantization,
// v_mfma_f32_16x16x32_f16 over the super-block's 8 k-steps in order, fp32 accumulation per
// wave; the K-waves' sums added in k order.  Replaces, for 17..767 tokens, the reference's
// Triton loops kernels/mmq_q8_0.py:59-93, mmq_q4_k.py:167-229.
#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_wfrag.hpp"

namespace gq {
namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int FW = 8;                // waves per workgroup
constexpr int F_LDS_CAP = 160 * 1024;

template <int F, int RW, int NB> struct FCfg {
    static constexpr int KW = FW / RW;            // K-interleaved waves
    static constexpr int BM = 32 * RW, BN = 16 * NB;
    static constexpr int XT = 16 * 512;           // one super-block of one 16-token tile
    static constexpr int SLOT = KW * NB * XT;     // one step's activations
    static constexpr int XI = SLOT / 1024;        // its DMA instructions
    static constexpr int NXI = XI / FW;           // per wave
    static constexpr int RED = FW * 2 * NB * 1024; // the waves' fp32 tiles at the end
    static constexpr int LDS = 2 * SLOT > RED ? 2 * SLOT : RED;
    static_assert(XI % FW == 0, "whole DMA instructions per wave");
    static_assert(LDS <= F_LDS_CAP, "LDS budget");
};

template <int F, int RW, int NB>
__global__ __launch_bounds__(64 * FW) void fgemm_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                       uint16_t *__restrict__ C, int M, int N, int K, int ldc)
{
    using G = FCfg<F, RW, NB>;
    using W = WB<F>;
    constexpr int KW = G::KW;
    __shared__ __attribute__((aligned(1024))) uint8_t lds_arr[G::LDS];
    uint8_t *const lds = lds_arr;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = wave % RW, k = wave / RW; // row group, K phase
    const int g = lane >> 4, c = lane & 15;
    const int m0 = (int)blockIdx.x * G::BM, n0 = (int)blockIdx.y * G::BN;
    const int nsb = K / 256, steps = (nsb + KW - 1) / KW;
    const int row_bytes = (K / Layout<F>::QK) * Layout<F>::BYTES;
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, (int)(((int64_t)M * row_bytes + 15) & ~(int64_t)15), 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, N * K * 2, 0x00020000);

    // this lane's two weight rows (16-row fragments 2r, 2r+1 of the tile), clamped
    uint32_t wv[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        const int row = m0 + 32 * r + 16 * f + c;
        wv[f] = (uint32_t)((row < M ? row : M - 1) * row_bytes);
    }
    // DMA instruction i = wave + 8u of a step: activation region (kk, t) = i / 8, tokens 2p, 2p+1 of
    // it (p = i % 8); lane l -> token n = 2p + (l >> 5), LDS position q = l & 31 holding source
    // piece q ^ n.  Source offsets without the super-block (added per step in the SGPR offset).
    // (fixed-size arrays: a template-dependent array length captured by the lambdas below made the
    // host pass drop the kernel's launch stub)
    uint32_t xsrc[8];
    int xkk[8];
    static_assert(G::NXI <= 8, "DMA instructions per wave");
#pragma unroll
    for (int u = 0; u < G::NXI; ++u) {
        const int i = wave + FW * u, reg = i >> 3, p = i & 7, kk = reg / NB, t = reg % NB;
        const int n = 2 * p + (lane >> 5), q = lane & 31;
        const int tok = n0 + 16 * t + n < N ? n0 + 16 * t + n : N - 1;
        xsrc[u] = (uint32_t)tok * (uint32_t)K * 2u + 16u * (uint32_t)(q ^ n);
        xkk[u] = kk;
    }

    W wb[2][2];
    auto issue = [&](int j, int b) __attribute__((always_inline)) {
        uint8_t *slot = lds + b * G::SLOT;
#pragma unroll
        for (int u = 0; u < G::NXI; ++u) {
            const int sb = KW * j + xkk[u];
            const int sbc = sb < nsb ? sb : nsb - 1; // (past K: a clamped copy nobody multiplies)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void *)(slot + 1024 * (wave + FW * u)), 16, xsrc[u],
                                                     (uint32_t)(512 * sbc), 0, 0);
        }
        const int sb = KW * j + k, sbc = sb < nsb ? sb : nsb - 1;
#pragma unroll
        for (int f = 0; f < 2; ++f) wb[b][f].load(wrs, wv[f], g, (uint32_t)(sbc * W::SB));
    };

    f32x4 acc[2][NB];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[f][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

    auto body = [&](int j, int b) __attribute__((always_inline)) {
        // this wave's step-j loads landed (the builtin, not inline asm: the compiler's waitcnt pass
        // sees it and knows the step's weight registers are ready -- behind an asm wait it
        // waited again, for the NEXT step's loads, at their first use)
        __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0) (expcnt, lgkmcnt: no wait)
        __builtin_amdgcn_s_barrier();       // everyone's; slot b ^ 1 is free
        if (j + 1 < steps) issue(j + 1, b ^ 1);
        if (KW * j + k >= nsb) return; // (the last step's surplus waves)
        const uint8_t *xs = lds + b * G::SLOT + k * (NB * G::XT) + c * 512;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            f16x8 bk[NB];
#pragma unroll
            for (int t = 0; t < NB; ++t) bk[t] = *(const f16x8 *)(xs + t * G::XT + 16 * ((W::e(s, g) >> 3) ^ c));
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const f16x8 af = wb[b][f].frag(s, g);
#pragma unroll
                for (int t = 0; t < NB; ++t) acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bk[t], acc[f][t], 0, 0, 0);
            }
        }
    };

    issue(0, 0);
    for (int j = 0; j < steps; j += 2) {
        body(j, 0);
        if (j + 1 < steps) body(j + 1, 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // (nothing in flight: the last issue was awaited)

    // the K-waves' tiles summed in k order: slot (k, r, f, t) of 1 KiB
    __builtin_amdgcn_s_barrier(); // every wave's last B reads are done before red overwrites them
    float *red = (float *)lds;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int t = 0; t < NB; ++t) *(f32x4 *)(red + (((k * RW + r) * 2 + f) * NB + t) * 256 + 4 * lane) = acc[f][t];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // (gfx950: no wait in front of a raw barrier)
    __builtin_amdgcn_s_barrier();
    for (int q = tid; q < RW * 2 * NB * 64; q += 64 * FW) {
        const int l = q & 63, rft = q >> 6, t = rft % NB, rf = rft / NB; // rf = r*2 + f
        f32x4 v = *(const f32x4 *)(red + (rf * NB + t) * 256 + 4 * l);
#pragma unroll
        for (int kk = 1; kk < KW; ++kk) v += *(const f32x4 *)(red + ((kk * RW * 2 + rf) * NB + t) * 256 + 4 * l);
        const int row = m0 + 16 * rf + 4 * (l >> 4), tok = n0 + 16 * t + (l & 15);
        if (row >= M || tok >= N) continue;
        uint16_t *dst = C + (int64_t)tok * ldc + row;
        if (row + 4 <= M) {
            *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                    (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)};
        } else {
            for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(v[i]);
        }
    }
}

template <int F, int RW, int NB>
hipError_t launch_cfg(const uint8_t *A, const uint16_t *X, uint16_t *C, int64_t M, int64_t N, int64_t K, int64_t ldc,
                      hipStream_t s)
{
    using G = FCfg<F, RW, NB>;
    const dim3 grid((unsigned)((M + G::BM - 1) / G::BM), (unsigned)((N + G::BN - 1) / G::BN));
    fgemm_kernel<F, RW, NB><<<grid, dim3(64 * FW), 0, s>>>(A, X, C, (int)M, (int)N, (int)K, (int)ldc);
    return hipGetLastError();
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const uint16_t *X, uint16_t *C, const FGemmPlan &p, int64_t M, int64_t N,
                      int64_t K, int64_t ldc, hipStream_t s)
{
    if (p.rw == 2 && p.nb == 2) return launch_cfg<F, 2, 2>(A, X, C, M, N, K, ldc, s);
    if (p.rw == 4 && p.nb == 2) return launch_cfg<F, 4, 2>(A, X, C, M, N, K, ldc, s);
    if (p.rw == 4 && p.nb == 4) return launch_cfg<F, 4, 4>(A, X, C, M, N, K, ldc, s);
    if (p.rw == 8 && p.nb == 4) return launch_cfg<F, 8, 4>(A, X, C, M, N, K, ldc, s);
    return hipErrorInvalidValue;
}

} // namespace

FGemmPlan plan_fgemm(int fmt, int64_t M, int64_t N, int64_t K)
{
    FGemmPlan p;
    if (M < 1 || N < 1 || K < 256 || K % 256 != 0) return p;
    // the tile whose grid is closest to whole rounds of the chip, smaller tiles first
    static const int cand[][2] = {{2, 2}, {4, 2}, {4, 4}, {8, 4}};
    const int64_t cus = num_cus();
    double best = 1e300;
    for (const auto &cd : cand) {
        const int64_t tiles = ((M + 32 * cd[0] - 1) / (32 * cd[0])) * ((N + 16 * cd[1] - 1) / (16 * cd[1]));
        const int64_t rounds = (tiles + cus - 1) / cus;
        // cost ~ rounds x a tile's bytes per K element (weights per row ~1, activations 2 per token)
        const double cost = (double)rounds * (32.0 * cd[0] + 2.0 * 16 * cd[1]);
        if (cost < best) {
            best = cost;
            p.rw = cd[0];
            p.nb = cd[1];
        }
    }
    if (tuning().fgemm_rw > 0) p.rw = tuning().fgemm_rw; // (A/B knobs)
    if (tuning().fgemm_nb > 0) p.nb = tuning().fgemm_nb;
    p.ok = (p.rw == 2 && p.nb == 2) || (p.rw == 4 && (p.nb == 2 || p.nb == 4)) || (p.rw == 8 && p.nb == 4);
    return p;
}

hipError_t launch_fgemm(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, const FGemmPlan &p, int64_t M,
                        int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (!p.ok || N * K * 2 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, X, C, p, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, X, C, p, M, N, K, ldc, s);
    case Q6_K: return launch_fmt<Q6_K>(A, X, C, p, M, N, K, ldc, s);
    default: return hipErrorInvalidValue;
    }
}

} // namespace gq
