// mmq_wgemm.hip -- batched MMQ (33+ tokens): weights streamed into registers, activations by
// LDS-DMA, on v_mfma_f32_16x16x32_f16.
//
// C[t][m] = sum_k W[m][k] * x~[t][k] (fp32 accumulate), x~ = fp16(d*q) the q8_1-quantized
// activation (act_quant.hip DEQ form: the integers kernels/cpu_impls multiplies,
// mmq_*_q8_1_cpu.py), W dequantized to fp16 in registers from the packed GGUF bytes.  Replaces
// the reference's Triton GEMM loops (kernels/mmq_q8_0.py:59-93, mmq_q4_k.py:167-229,
// mmq_q6_k.py:122-186).
//
// Why this shape.  A wave's vector-memory returns are in issue order: a wave that
// streams both the weights (HBM) and the activations (L2, re-read by every row tile) waits for
// the slow stream whenever it needs the fast one.  So the two streams live in different waves:
//   loader waves (NL = 4): the tile's activations, HBM/L2 -> LDS by LDS-DMA (1 KiB per
//     instruction), a ring of R sub-stages (64 K elements each) with L = R - 2 in flight;
//     nothing else in their queues;
//   compute waves (NWC): each owns 16*RG weight rows; its lanes load their own fragment bytes of
//     a super-block (256 K elements) into registers one super-block ahead (double buffer),
//     dequantize in registers, read the activation fragments from the ring, multiply.
// One s_barrier per sub-stage (loaders: before it, wait for sub-stage a to land; after it, issue
// sub-stage a + L into the slot read two sub-stages ago).
//
// K order.  The k-step -> element map follows what a lane loaded (WB<F>::e below): lane group
// g = lane>>4 supplies 8 consecutive elements in the order (0,2,1,3,4,6,5,7) that packed
// dequantization produces -- act_quant's DEQ layout, so a B fragment is one 16-byte LDS read of
// the same 8 activations.
//
// MFMA 16x16x32 f16 (gfx950): lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15];
// D[row 4(l>>4)+i][col l&15] in acc element i.  Weight rows are A rows, tokens B columns.
#include <type_traits>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_wfrag.hpp"

namespace gq {
namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int NL = 4; // loader waves

// one LDS-DMA instruction: 16 bytes per lane from (voff + soff) to lds_dst + 16 * lane
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint8_t *lds_dst, uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)lds_dst, 16, voff, soff, 0, 0);
}

// ---------------------------------------------------------------------------------------
// Activation ring: R slots of one sub-stage (64 K elements = k-steps 2j, 2j+1 of super-block
// sb): per token 128 bytes = 8 pieces, piece kk*4 + g (the 8 activations lane group g reads at
// k-step 2j + kk) stored at position piece ^ swz8(token): a ds_read_b128's 16-lane groups then
// hit 16 distinct 16-byte bank slots.  A DMA instruction fills 1 KiB = 8 tokens' rows (lane l:
// token l>>3, position l&7), its per-lane source address picking the piece.
__device__ __forceinline__ int swz8(int n) { return (n >> 1) & 7; }

template <int NWC, int NB>
struct WCfg {
    static constexpr int BN = 16 * NB;
    static constexpr int SLOT = BN * 128;
    static constexpr int DMA_SUB = SLOT / 1024;                                    // DMA instructions per sub-stage
    static constexpr int DPL = DMA_SUB >= NL ? DMA_SUB / NL : 1;                   // per loader wave
    static constexpr int L = NB >= 8 ? 6 : 8;                                      // sub-stages in flight
    static constexpr int R = L + 2;                                                // ring slots
    static constexpr int LDS_BYTES = R * SLOT;
    static constexpr int THREADS = 64 * (NWC + NL);
    static_assert(DMA_SUB % NL == 0 || DMA_SUB < NL, "loader share");
    static_assert((L - 1) * DPL <= 63, "vmcnt range");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

// Block -> (tile, split): the S splits of tile t run on XCD t % 8 when the tile count is a
// multiple of 8 (blocks b and b + 8 share an XCD under round-robin dispatch; a speed choice,
// never correctness), so the split-K reduce finds a tile's partials in one L2.
__device__ __forceinline__ void block_map(int b, int ntiles, int S, int &tile, int &sp)
{
    if (ntiles % 8 == 0) {
        const int j = b >> 3;
        tile = (b & 7) + 8 * (j / S);
        sp = j % S;
    } else {
        tile = b / S;
        sp = b % S;
    }
}

// s_waitcnt vmcnt(n) for a compile-time n
template <int n> __device__ __forceinline__ void vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory"); }

// P (S > 1): fp16 partials per (tile, split) block in accumulator order -- unit
// q = ((wr*(NB/2) + u)*64 + lane) (wr = RG*wave + rf, wave < NWC) holds token tiles 2u, 2u+1 of
// the lane's 4 rows, scaled by 2^-e (e per (block, compute wave), ints after all the blocks).
// wreduce_kernel sums them.
template <int F, int NWC, int RG, int NB, int WD>
__global__ __launch_bounds__(64 * (NWC + NL)) void wgemm_kernel(
    const uint8_t *__restrict__ A, const uint16_t *__restrict__ X, uint16_t *__restrict__ C, uint16_t *__restrict__ P,
    int M, int N, int K, int ldc, int tiles_m, int S, int sb_per_split)
{
    using G = WCfg<NWC, NB>;
    using W = WB<F>;
    constexpr int BM = 16 * NWC * RG, BN = G::BN;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[G::LDS_BYTES];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int tile, sp;
    block_map(blockIdx.x, (int)gridDim.x / S, S, tile, sp);
    const int tm = tile % tiles_m, tn = tile / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int nsb = K / 256;
    const int sb0 = sp * sb_per_split;
    const int sb1 = sb0 + sb_per_split < nsb ? sb0 + sb_per_split : nsb;
    const int nsub = 4 * (sb1 - sb0);

    if (wave >= NWC) {
        // ---- loader wave: the ring of activation sub-stages, DMA only ----
        if (nsub <= 0) return;
        const int lw = wave - NWC;
        const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, N * K * 2, 0x00020000);
        // instruction i of this wave: DMA k = lw + NL*i (BN = 16: waves 2, 3 repeat 0, 1's -- same
        // bytes to the same place); lane: token 8k + (lane>>3), position lane&7
        uint32_t xv[G::DPL];
        int kd[G::DPL];
#pragma unroll
        for (int i = 0; i < G::DPL; ++i) {
            const int k = G::DMA_SUB >= NL ? lw + NL * i : lw % G::DMA_SUB;
            const int n = 8 * k + (lane >> 3), pc = (lane & 7) ^ swz8(n);
            const int tok = n0 + n < N ? n0 + n : N - 1;
            xv[i] = (uint32_t)tok * (uint32_t)K * 2u + 2u * (uint32_t)W::off(pc >> 2, pc & 3);
            kd[i] = 1024 * k;
        }
        auto issue = [&](int a) __attribute__((always_inline)) { // sub-stage a into slot a % R
            const uint32_t so = 2u * (uint32_t)(256 * (sb0 + (a >> 2)) + W::base(a & 3));
            uint8_t *dst = lds + (a % G::R) * G::SLOT;
#pragma unroll
            for (int i = 0; i < G::DPL; ++i) {
                if constexpr (!(ABL & 2)) dma16(xrs, dst + kd[i], xv[i], so);
            }
        };
        // nothing past the split's end (a split is 8-16 sub-stages: clamped re-loads of the last
        // one were up to 100% more activation DMA), so the last L - 1 waits count fewer younger ones
#pragma unroll
        for (int a = 0; a < G::L; ++a)
            if (a < nsub) issue(a);
        for (int a = 0; a < nsub; ++a) {
            if constexpr (!(ABL & 2)) { // sub-stage a landed: at most the younger sub-stages outstanding
                const int young = G::L - 1 < nsub - 1 - a ? G::L - 1 : nsub - 1 - a;
                vm_wait<(G::L - 1) * G::DPL>(young * G::DPL);
            }
            asm volatile("s_barrier" ::: "memory");
            if (a + G::L < nsub) issue(a + G::L); // into the slot of sub-stage a + L - R = a - 2: read before the last barrier
        }
        vmcnt<0>(); // no DMA may land after the workgroup exits
        return;
    }

    // ---- compute wave ----
    const int g = lane >> 4, c = lane & 15;
    const int row_bytes = (K / Layout<F>::QK) * Layout<F>::BYTES;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, M * row_bytes, 0x00020000);
    // this lane's weight rows (clamped: rows past M compute garbage that is never stored)
    uint32_t wv[RG];
#pragma unroll
    for (int rf = 0; rf < RG; ++rf) {
        const int row = m0 + 16 * (RG * wave + rf) + c;
        wv[rf] = (uint32_t)((row < M ? row : M - 1) * row_bytes);
    }
    f32x4 acc[RG][NB];
#pragma unroll
    for (int rf = 0; rf < RG; ++rf)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[rf][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

    if (nsub > 0) {
        W wb[WD][RG]; // super-block ring: WD - 1 super-blocks of weights in flight
        auto load_w = [&](int b, int sb) __attribute__((always_inline)) { // super-block sb (clamped: the WD - 1 surplus re-reads
            // hit the cache; skipping them -- a branch around register loads -- measured 0-2% slower)
            const uint32_t s0 = (uint32_t)((sb < sb1 ? sb : sb1 - 1) * W::SB) & WMASK;
#pragma unroll
            for (int rf = 0; rf < RG; ++rf) wb[b][rf].load(wrs, wv[rf], g, s0);
        };
        // multiply sub-stage j (k-steps 2j, 2j+1) of the super-block in buffer b from ring slot `slot`
        auto compute = [&](int b, int j, int slot) __attribute__((always_inline)) {
            const uint8_t *xsl = lds + slot * G::SLOT;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                f16x8 bf[NB];
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const int n = 16 * t + c;
                    bf[t] = *(const f16x8 *)(xsl + n * 128 + 16 * ((4 * kk + g) ^ swz8(n)));
                }
                f16x8 af[RG];
#pragma unroll
                for (int rf = 0; rf < RG; ++rf) {
                    if constexpr (ABL & 8) af[rf] = __builtin_bit_cast(f16x8, (u32x4){wv[rf], wv[rf] + 1u, (uint32_t)j, 5u});
                    else af[rf] = wb[b][rf].frag(2 * j + kk, g);
                }
#pragma unroll
                for (int rf = 0; rf < RG; ++rf)
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        if constexpr (ABL & 4) acc[rf][t][0] += (float)af[rf][t & 7] * (float)bf[t][0];
                        else acc[rf][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[rf], bf[t], acc[rf][t], 0, 0, 0);
                    }
            }
        };
        // (sched_barrier on both sides: register-only work -- the dequantization -- would otherwise
        // be hoisted across the asm barrier to the loop head, where it waits for the weight loads
        // just issued)
        auto barrier = [] {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
        };
        // Super-block i (buffer i % WD): 4 sub-stages (barrier: the loaders' sub-stage landed; then
        // multiply), then its buffer is refilled with super-block i + WD -- the weights have WD - 1
        // super-blocks of lead and are the only loads in this wave's queue.  WD bodies per loop
        // iteration (static buffer indices), the last < WD super-blocks after it, so the loop's back
        // edge always follows the same code.
        auto body = [&](int sb, int b) __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int a = 4 * (sb - sb0) + j;
                barrier();
                compute(b, j, a % G::R);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!(ABL & 1)) load_w(b, sb + WD);
        };
#pragma unroll
        for (int b = 0; b < WD; ++b) load_w(b, sb0 + b);
        int sb = sb0;
        for (; sb + WD - 1 < sb1; sb += WD) {
#pragma unroll
            for (int b = 0; b < WD; ++b) body(sb + b, b);
        }
#pragma unroll
        for (int b = 0; b < WD - 1; ++b)
            if (sb + b < sb1) body(sb + b, b);
    }

    // epilogue: acc[rf][t][i] = D[row 16*(RG*wave + rf) + 4g + i][token 16t + c]
    if (S > 1) {
        const int bidx = tile * S + sp;
        uint16_t *hb = P + (size_t)bidx * (BM * BN);
        float mx = 0.f;
#pragma unroll
        for (int rf = 0; rf < RG; ++rf)
#pragma unroll
            for (int t = 0; t < NB; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) mx = fmaxf(mx, fabsf(acc[rf][t][i]));
        // wave max (values >= 0): DPP row shifts + row broadcasts, lane 63 holds it
        int mm = __builtin_bit_cast(int, mx);
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x111, 0xf, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x112, 0xf, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x114, 0xf, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x118, 0xf, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x142, 0xa, 0xf, true))));
        mm = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, mm), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, mm, 0x143, 0xc, 0xf, true))));
        const uint32_t mb = (uint32_t)__builtin_amdgcn_readlane(mm, 63);
        const int E = (int)((mb >> 23) & 0xff) - 127;
        const int e = E - 14 > 0 ? (E - 14 < 127 ? E - 14 : 126) : 0;
        const float down = __builtin_bit_cast(float, (uint32_t)(127 - e) << 23);
        const int nblk = (int)gridDim.x;
        if (lane == 0) ((int *)(P + (size_t)nblk * (BM * BN)))[bidx * NWC + wave] = e;
        auto pk = [down](const f32x4 &v) {
            return (u32x2){(uint32_t)f2h_bits(v[0] * down) | ((uint32_t)f2h_bits(v[1] * down) << 16),
                           (uint32_t)f2h_bits(v[2] * down) | ((uint32_t)f2h_bits(v[3] * down) << 16)};
        };
#pragma unroll
        for (int rf = 0; rf < RG; ++rf) {
#pragma unroll
            for (int u = 0; u < NB / 2; ++u) {
                const u32x2 lo = pk(acc[rf][2 * u]), hi = pk(acc[rf][2 * u + 1]);
                ((u32x4 *)hb)[((RG * wave + rf) * (NB / 2) + u) * 64 + lane] = (u32x4){lo.x, lo.y, hi.x, hi.y};
            }
        }
        return;
    }
#pragma unroll
    for (int rf = 0; rf < RG; ++rf) {
        const int row = m0 + 16 * (RG * wave + rf) + 4 * g;
        if (row >= M) continue;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int tok = n0 + 16 * t + c;
            if (tok >= N) continue;
            const f32x4 v = acc[rf][t];
            uint16_t *dst = C + (size_t)tok * ldc + row;
            if (row + 4 <= M) {
                *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                        (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)};
            } else {
                for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(v[i]);
            }
        }
    }
}

// C = fp16(sum_s 2^e_s * partial_s) in split order (deterministic), one thread per 16-byte unit
// (two token tiles of a lane's 4 rows), every split's load issued before the first add.  Reduce
// block b takes a tile of XCD b % 8 when the tile count allows it (block_map's placement), so
// the partials are read from the L2 that holds them.
template <int NWC, int RG, int NB>
__global__ __launch_bounds__(256) void wreduce_kernel(const uint16_t *__restrict__ P, uint16_t *__restrict__ C, int M,
                                                      int N, int ldc, int S, int tiles_m, int ntiles)
{
    constexpr int UNITS = NWC * RG * (NB / 2) * 64; // per tile block
    constexpr int BPT = (UNITS + 255) / 256;        // reduce blocks per tile
    int tile, chunk;
    if (ntiles % 8 == 0) {
        const int i = blockIdx.x >> 3;
        tile = (blockIdx.x & 7) + 8 * (i / BPT);
        chunk = i % BPT;
    } else {
        tile = blockIdx.x / BPT;
        chunk = blockIdx.x % BPT;
    }
    const int q = chunk * 256 + threadIdx.x;
    if (tile >= ntiles || q >= UNITS) return;
    const int lane = q & 63, u = (q >> 6) % (NB / 2), wr = (q >> 6) / (NB / 2);
    const int wv = wr / RG;
    constexpr int BLK = NWC * RG * 16 * 16 * NB; // halves per block
    const int *es = (const int *)(P + (size_t)ntiles * S * BLK);
    f32x4 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < S; s0 += 8) {
        u32x4 v[8];
        float up[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int sp = tile * S + (s0 + i < S ? s0 + i : S - 1); // unconditional loads
            v[i] = ((const u32x4 *)(P + (size_t)sp * BLK))[q];
            up[i] = __builtin_bit_cast(float, (uint32_t)(127 + es[sp * NWC + wv]) << 23);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (s0 + i >= S) break;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t lo = j ? v[i].z : v[i].x, hi = j ? v[i].w : v[i].y;
                acc[j][0] += h2f(lo & 0xffffu) * up[i];
                acc[j][1] += h2f(lo >> 16) * up[i];
                acc[j][2] += h2f(hi & 0xffffu) * up[i];
                acc[j][3] += h2f(hi >> 16) * up[i];
            }
        }
    }
    const int tm = tile % tiles_m, tn = tile / tiles_m;
    const int row = tm * (16 * NWC * RG) + 16 * wr + 4 * (lane >> 4);
    if (row >= M) return;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int tok = tn * 16 * NB + 16 * (2 * u + j) + (lane & 15);
        if (tok >= N) continue;
        uint16_t *dst = C + (size_t)tok * ldc + row;
        if (row + 4 <= M) {
            *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(acc[j][0]) | ((uint32_t)f2h_bits(acc[j][1]) << 16),
                                    (uint32_t)f2h_bits(acc[j][2]) | ((uint32_t)f2h_bits(acc[j][3]) << 16)};
        } else {
            for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(acc[j][i]);
        }
    }
}

template <int F, int NWC, int RG, int NB>
hipError_t launch_cfg(const uint8_t *A, const uint16_t *X, uint16_t *C, uint16_t *P, const WGemmPlan &pl, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    using G = WCfg<NWC, NB>;
    const int ntiles = pl.tiles_m * pl.tiles_n;
    const dim3 grid((unsigned)(ntiles * pl.splits)), block(G::THREADS);
    // weight super-blocks in registers: 4 only for the one-fragment waves, 3 except where it
    // would spill (Q6_K, two fragments x 8 column blocks)
    constexpr bool wd4 = NWC == 8, wd3 = !(F == Q6_K && RG == 2 && NB == 8);
    const int wd = pl.wd == 4 && !wd4 ? 3 : pl.wd;
    bool done = false;
    if constexpr (wd4) {
        if (wd == 4) {
            wgemm_kernel<F, NWC, RG, NB, 4><<<grid, block, 0, s>>>(A, X, C, P, (int)M, (int)N, (int)K, (int)ldc,
                                                                  pl.tiles_m, pl.splits, pl.sb_per_split);
            done = true;
        }
    }
    if constexpr (wd3) {
        if (!done && wd == 3) {
            wgemm_kernel<F, NWC, RG, NB, 3><<<grid, block, 0, s>>>(A, X, C, P, (int)M, (int)N, (int)K, (int)ldc,
                                                                  pl.tiles_m, pl.splits, pl.sb_per_split);
            done = true;
        }
    }
    if (!done)
        wgemm_kernel<F, NWC, RG, NB, 2><<<grid, block, 0, s>>>(A, X, C, P, (int)M, (int)N, (int)K, (int)ldc, pl.tiles_m,
                                                              pl.splits, pl.sb_per_split);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || pl.splits == 1) return e;
    constexpr int UNITS = NWC * RG * (NB / 2) * 64, BPT = (UNITS + 255) / 256;
    wreduce_kernel<NWC, RG, NB><<<dim3((unsigned)(ntiles * BPT)), dim3(256), 0, s>>>(P, C, (int)M, (int)N, (int)ldc,
                                                                                    pl.splits, pl.tiles_m, ntiles);
    return hipGetLastError();
}

template <int F, int NWC, int RG>
hipError_t launch_nb(const uint8_t *A, const uint16_t *X, uint16_t *C, uint16_t *P, const WGemmPlan &pl, int64_t M,
                     int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (pl.nb) {
    case 2: return launch_cfg<F, NWC, RG, 2>(A, X, C, P, pl, M, N, K, ldc, s);
    case 4: return launch_cfg<F, NWC, RG, 4>(A, X, C, P, pl, M, N, K, ldc, s);
    case 8: return launch_cfg<F, NWC, RG, 8>(A, X, C, P, pl, M, N, K, ldc, s);
    default: return hipErrorInvalidValue;
    }
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const uint16_t *X, uint16_t *C, uint16_t *P, const WGemmPlan &pl, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    // (rg, compute waves): (2, 4) = 128 rows, one compute wave per SIMD; (1, 8) = 128 rows, two
    if (pl.rg == 1) return launch_nb<F, 8, 1>(A, X, C, P, pl, M, N, K, ldc, s);
    return launch_nb<F, 4, 2>(A, X, C, P, pl, M, N, K, ldc, s);
}

} // namespace

WGemmPlan plan_wgemm(int fmt, int64_t M, int64_t N, int64_t K, int rg, int nb, int splits)
{
    WGemmPlan p;
    (void)fmt;
    p.rg = rg == 1 ? 1 : 2;
    p.nb = nb == 2 || nb == 4 ? nb : 8;
    const int64_t bm = 128, bn = 16 * p.nb; // both (rg, waves) shapes are 128 rows
    p.tiles_m = (int)((M + bm - 1) / bm);
    p.tiles_n = (int)((N + bn - 1) / bn);
    const int64_t nsb = K / 256, tiles = (int64_t)p.tiles_m * p.tiles_n;
    const int64_t cus = num_cus();
    int64_t S = splits > 0 ? splits : (tiles >= cus ? 1 : cus / tiles);
    if (S > nsb) S = nsb;
    if (S < 1) S = 1;
    const int64_t sps = (nsb + S - 1) / S;
    S = (nsb + sps - 1) / sps;
    p.splits = (int)S;
    p.sb_per_split = (int)sps;
    p.partial_bytes = S > 1 ? (size_t)S * tiles * bm * bn * 2 + (size_t)S * tiles * 8 * sizeof(int) : 0;
    return p;
}

hipError_t launch_wgemm(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, void *partials,
                        const WGemmPlan &plan, int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    uint16_t *P = (uint16_t *)partials;
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, X, C, P, plan, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, X, C, P, plan, M, N, K, ldc, s);
    default: return launch_fmt<Q6_K>(A, X, C, P, plan, M, N, K, ldc, s);
    }
}

} // namespace gq
