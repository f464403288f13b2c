// mmq_rgemm.hip -- the resident-split MMQ GEMM: one workgroup per (256 weight rows, 16*NB tokens,
// one super-block of K), every operand of the split in LDS at once.
//
// Why this shape (profiles/r04/probe_gemm_ingest.txt): with 16 weight rows per wave the activation
// fragment reads of 8 waves are 128 KiB of LDS per 64-element sub-stage -- 512 LDS cycles, the same
// as the sub-stage's 512 cycles of MFMA per SIMD -- and the waves, in lockstep behind each
// sub-stage barrier, ran the two one after the other (reads + MFMA 0.585 us per sub-stage against
// 0.266 for the MFMAs alone).  Here every wave multiplies 32 rows (two 16-row groups share each
// activation fragment: half the LDS bytes per MFMA), and there is no ring and no barrier in the
// multiply: the split's weights (one super-block per row: 256 x 272 / 144 / 240 B) and its
// activations (16*NB tokens x 256 K as fp16 x~, 64 KiB at 128 tokens) are loaded once, then each
// wave runs its 8 k-steps on its own.  A 4096-row matrix at K = 4096 is 16 row tiles x 16 splits
// = 256 workgroups, one per CU.
//
// Loads: the weights by LDS-DMA first (HBM: the long pole), then the activations -- either the
// prepared x~ (act_quant DEQ / F8DEQ form) by LDS-DMA, or (AQ) the raw fp16 activations into
// registers, q8_1-quantized in-kernel (gguf_q8_1.hpp q8_1_quad: x~ = fp16(d*q), bit-identical to
// act_quant's DEQ form; F8: the fp8 variant's f8_quad) and written to LDS while the weights are
// in flight: no act_quant launch.
//
// Arithmetic = gemm_kernel's (mmq_gemm.hip) for the same rows: stage_frags dequantization, the
// same x~, v_mfma_f32_16x16x32_f16 in the same (sub-stage, k-step) order into fp32 accumulators;
// with one split per super-block the split-K partials are written in gemm_kernel's fp16 form and
// summed by its reduce kernel (launch_gemm_reduce_f16).
#include <type_traits>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_mfma.hpp"
#include "gguf_q8_1.hpp"

namespace gq {

#ifdef GQ_RGEMM_STAMPS // diagnostic build: per-wave timeline of rgemm_kernel (never the product)
// [0] s_memrealtime at entry (100 MHz, chip-wide), [1] s_memtime at entry, then s_memtime at:
// [2] loads issued, [3] x~ written (AQ), [4] past the activation barrier, [5] own half 0 landed,
// [6] half 0 multiplied, [7] half 1 landed, [8] multiply done, [9] partial stores issued,
// [10] stores complete, [11] s_memrealtime at the end; [12] workgroup id, [13] XCC id
__device__ unsigned long long g_rstamps[65536][14];
#define GQ_RST(i) (st[i] = __builtin_amdgcn_s_memtime())
#else
#define GQ_RST(i) ((void)0)
#endif

// polls of the in-launch combine that gave up (ilc_combine; gq_debug_sync_timeouts)
__device__ unsigned int g_ilc_timeouts;

namespace {

// diagnostic ablation builds only (make rabl RABL=n; never the product): 1 = no weight DMA,
// 2 = no activation load, 4 = no multiply (fragments + MFMA; the streaming kernels too),
// 8 = no epilogue stores
#ifndef GQ_RGEMM_ABL
#define GQ_RGEMM_ABL 0
#endif
constexpr int ABL = GQ_RGEMM_ABL;

constexpr int RW = 8;                 // waves per workgroup (two per SIMD)
// Issue priority: waves 4-7 -- dispatched second, so the losers of every VALU / MFMA arbitration
// against their SIMD partners by age (MI355X_MICROARCH.md, two waves per SIMD, item 4) -- run at
// s_setprio 1 in the resident and streaming GEMMs: the 7B layer x64 / x128 / x512 73.9 / 99.4 /
// 331.8 -> 72.3 / 98.3 / 329.0 us, Q4_K 11008x4096x128 33.5 -> 32.8, the headline unchanged
// (16.13), same bits; swapping the halves at the resident GEMM's second half multiply did
// nothing (profiles/r06/gemm_prio_ab.txt).
constexpr int RPRIO_WAVE = RW / 2;
constexpr int RRG = 2;                // 16-row groups per wave
constexpr int RBM = 16 * RW * RRG;    // 256 rows per tile
constexpr int LDS_CAP = 160 * 1024;
constexpr int kSpol = 16; // split-K partial stores write-through (sc1)

// The split's weights as two half-super-block images (K elements 0..127 and 128..255 of every
// row), so that the multiply of the first half runs while the second half is still in flight.
// Per format: NPH 16-byte pieces per row and half (HRB bytes, a row stride that puts the 16 rows
// of a fragment read on distinct banks), piece pc of half h read from super-block byte
// hsrc<F>(h, pc):
//   Q8_0  9 pieces from byte 128h (blocks 4h..4h+3 at image byte 8h..; 8 bytes of overlap)
//   Q4_K  5 pieces: the 16-byte header, then qs bytes 64h..64h+63
//   Q6_K  8 pieces: ql 64h.. (4), qh 128+32h.. (2), bytes 192..207 (scales), 194..209 (d at image
//         byte 126); a 128-B stride is 2 bank sets, so row r's pieces are XOR-permuted by r & 7
//         (hpos_swz).  (Until round 5 a ninth padding piece made the stride 144 B instead; the 8
//         pieces move 11% fewer weight DMA instructions: Q6_K 70B x128 -3%, profiles/r05/q6k_nph8_ab.txt)
template <int F> struct HImg;
template <> struct HImg<Q8_0> { static constexpr int NPH = 9; };
template <> struct HImg<Q4_K> { static constexpr int NPH = 5; };
#ifndef GQ_Q6_NPH
#define GQ_Q6_NPH 8 // (-DGQ_Q6_NPH=9: the padded image, A/B builds)
#endif
template <> struct HImg<Q6_K> { static constexpr int NPH = GQ_Q6_NPH; };
// Q6_K with 8 pieces (no padding piece): the 128-B row stride puts rows r and r+2 on the same
// banks, so piece pc of row r lands at position pc ^ (r & 7) (2-way at most)
template <int F> __device__ __forceinline__ int hpos_swz(int r)
{
    return F == Q6_K && HImg<F>::NPH == 8 ? (r & 7) : 0;
}
template <int F> __device__ __forceinline__ uint32_t hsrc(int h, int pc)
{
    if constexpr (F == Q8_0) return 128u * h + 16u * pc;
    if constexpr (F == Q4_K) return pc == 0 ? 0u : 16u + 64u * h + 16u * (pc - 1);
    return pc < 4 ? 64u * h + 16u * pc : (pc < 6 ? 128u + 32u * h + 16u * (pc - 4) : (pc == 6 ? 192u : 194u));
}

template <int F, int NB> struct RCfg {
    static constexpr int BN = 16 * NB;
    static constexpr int NPH = HImg<F>::NPH, HRB = 16 * NPH, SB = Layout<F>::BYTES * (256 / Layout<F>::QK);
    // each wave's own 32 rows: [half 0 (32 x HRB)][half 1], moved by its own WWI DMA instructions
    // (H0I of them hold half 0 -- the last of those may carry the head of half 1)
    static constexpr int WW = 2 * 32 * HRB, WWI = WW / 1024, H0I = (32 * NPH + 63) / 64;
    static constexpr int X_OFF = RW * WW;                   // then the activation image
    static constexpr int X_BYTES = BN * 512;                // 4 sub-stages x BN tokens x 128 B
    static constexpr int X_INSTR = X_BYTES / 1024;          // prepared form: DMA instructions
    static constexpr int NX = X_INSTR / RW;
    static constexpr int LDS = X_OFF + X_BYTES;
    static_assert(WW % 1024 == 0 && X_INSTR % RW == 0, "whole DMA instructions per wave");
    static_assert(LDS <= LDS_CAP, "LDS budget");
};

// element offset (in the super-block) of piece q (8 elements) of activation sub-stage u: the
// K elements k-steps 2u, 2u+1 multiply (Q6_K: two 32-element runs, as act_soff / act_voff)
template <int F> __device__ __forceinline__ int sub_elem(int u, int q)
{
    if constexpr (F == Q6_K) return 128 * (u >> 1) + 32 * (u & 1) + 64 * (q >> 2) + 8 * (q & 3);
    return 64 * u + 8 * q;
}

// AQ: token r's 32-element block kb of the super-block, lane j of its quad (elements 32kb + 8j..)
// -> the (sub-stage, piece) holding those elements
template <int F> __device__ __forceinline__ void block_piece(int kb, int j, int &u, int &q)
{
    if constexpr (F == Q6_K) {
        const int b4 = kb & 3;
        u = 2 * (kb >> 2) + (b4 & 1);
        q = 4 * (b4 >> 1) + j;
    } else {
        u = kb >> 1;
        q = 4 * (kb & 1) + j;
    }
}

// A fragments of sub-stage u (half h = u >> 1) for the row whose half image starts at img
// (the Q6_K half image's fragments with its pieces at pc ^ sw: q6k_half_frags' arithmetic)
__device__ __forceinline__ void q6k_half_frags_swz(const uint8_t *img, int g, int h, int v, int sw, f16x8 (&frag)[2])
{
    auto at = [sw](int off) { return (((off >> 4) ^ sw) << 4) | (off & 15); };
    const float d = h2f(*(const uint16_t *)(img + at(126)));
    const u32x2 ql = *(const u32x2 *)(img + at(32 * v + 8 * g));
    const u32x2 qh = *(const u32x2 *)(img + at(64 + 8 * g));
    const h2 bias = splat(-1056.f); // 1024 + 32
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const float scv = (float)*(const int8_t *)(img + at(96 + 8 * h + 4 * n + 2 * v + (g >> 1)));
        const h2 dsc = splat(d * scv);
        const int sq = 4 * n + 2 * v;
        const uint32_t c0 = ((ql.x >> (4 * n)) & 0x0f0f0f0fu) | (((qh.x >> sq) & 0x03030303u) << 4);
        const uint32_t c1 = ((ql.y >> (4 * n)) & 0x0f0f0f0fu) | (((qh.y >> sq) & 0x03030303u) << 4);
        frag[n] = frag4((pair02(c0) + bias) * dsc, (pair13(c0) + bias) * dsc, (pair02(c1) + bias) * dsc,
                        (pair13(c1) + bias) * dsc);
    }
}

template <int F> __device__ __forceinline__ void half_frags(const uint8_t *img, int g, int u, int r, f16x8 (&frag)[2])
{
    const int h = u >> 1;
    if constexpr (F == Q8_0) stage_frags<Q8_0>(img - 128 * h, g, u, frag, 0); // (16-byte aligned: HRB = 144)
    else if constexpr (F == Q4_K) q4k_frags(img, img + 16 + 32 * (u & 1), g, u, frag);
    else if constexpr (HImg<F>::NPH == 8) q6k_half_frags_swz(img, g, h, u & 1, hpos_swz<F>(r), frag);
    else q6k_half_frags(img, g, h, u & 1, frag);
}

// The tile's fp32 accumulators out: acc[rg][t][i] = D[row 16*(2*wave + rg) + 4g + i][token
// 16t + l16].  One split: fp16 C.  Split-K (gridDim.z > 1): the partial in gemm_kernel's fp16
// form (its reduce kernel sums it): per (tile, split) a block of 256 x BN halves in accumulator
// order, each wave's values scaled by 2^-e, the e's after all blocks; spol = store cache policy.
// One sub-stage u (64 K elements) of this wave's 32 rows x every token: the A fragments from the
// half image wimg (half u >> 1), the B fragments from the sub-stage's activation image xs
// (rbase: the wave's first row in the image -- 32 * wave in a tile-wide image, 0 in a wave's own)
template <int F, int NB>
__device__ __forceinline__ void mul_substage(const uint8_t *wimg, const uint8_t *xs, int u, f32x4 (&acc)[RRG][NB],
                                             int rbase)
{
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, l16 = lane & 15;
    f16x8 af[RRG][2];
#pragma unroll
    for (int rg = 0; rg < RRG; ++rg)
        half_frags<F>(wimg + (16 * HImg<F>::NPH) * (rbase + 16 * rg + l16), g, u, l16, af[rg]);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        f16x8 bk[NB];
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int r = 16 * t + l16;
            bk[t] = *(const f16x8 *)(xs + 128 * r + 16 * ((4 * s + g) ^ act_swz(r)));
        }
#pragma unroll
        for (int rg = 0; rg < RRG; ++rg)
#pragma unroll
            for (int t = 0; t < NB; ++t)
                acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[rg][s], bk[t], acc[rg][t], 0, 0, 0);
    }
}

struct TileId { // a workgroup's tile: (x, y, z) of a (gx, gy, gz) grid (z = the K split)
    int x, y, z, gx, gy, gz;
};
__device__ __forceinline__ TileId grid_tile()
{
    return TileId{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)gridDim.x, (int)gridDim.y, (int)gridDim.z};
}
// The in-launch combine's 1-D grid (gx > 0): position p = tile * gz + split (tile = y * gx + x,
// the block index store_tile already uses).  Workgroups are dealt to the 8 XCDs round robin by
// launch index b, so with 8 | blocks, p = (b % 8) * (blocks / 8) + b / 8: each XCD runs a
// contiguous run of positions -- a tile's consecutive splits on one XCD, as the 3-D grid had them
// (neighbouring super-blocks of a row share a 128-byte line: Q4_K's 144-byte super-blocks nearly
// all do; split over XCDs the line is fetched into two L2s -- the first 1-D order, tile-major in
// b, measured +3.0 us on Q4_K 4096^2 x128, +0.6 on Q8_0's 272-byte super-blocks,
// profiles/r06/ilc_ab_v1.txt).  Each XCD dispatches its positions in order, so the tiles complete
// in order whatever part of the grid is resident.
__device__ __forceinline__ TileId ilc_tile(int gx, int gy)
{
    const int nb = (int)gridDim.x, gz = nb / (gx * gy), b = (int)blockIdx.x;
    const int p = (nb & 7) == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b, t = p / gz;
    return TileId{t % gx, t / gx, p - t * gz, gx, gy, gz};
}

// ---- In-launch split-K combine (ILC) -------------------------------------------------------
// Replaces the reduce launch where the whole grid is resident at once (one round of the chip):
// every workgroup stores its fp16 partial write-through (sc1), drains its stores, and publishes a
// flag; then the tile's gz workgroups each sum 1/gz of the tile over all gz partials, in split
// order -- gemm_reduce_f16_kernel's arithmetic, so the bits equal the two-launch form's.
// Hand-off (MI355X_MICROARCH.md "visibility", first row of the sc1 table): payload and flags all
// sc1 stores, every storing wave's vmcnt(0) before the workgroup barrier that precedes the flag,
// the flags polled with sc1 loads by one wave that then joins a barrier, every payload load sc1.
// The flags need no zeroed memory: a flag is {nonce + 1, gz, split}, nonce a per-tile word read
// at the start of the launch and advanced by split 0 once its tile's flags are all in, so a flag
// left by an earlier launch (any shape: gz and the split are in it) never matches.  A poll that
// does not complete within kIlcSpins gives up (counted in g_ilc_timeouts, gq_debug_sync_timeouts)
// rather than hang: it cannot happen while the grid is resident, which the launcher ensures.
constexpr int kIlcSpins = 1 << 17;

struct IlcSync {
    uint64_t *flags;  // [tiles * gz]
    uint32_t *nonce;  // [tiles]
};
// the sync words after the partial blocks and their exponents
__host__ __device__ inline size_t ilc_flags_off(int64_t nblk, int BN) { return ((size_t)nblk * (RBM * BN * 2 + RW * 4) + 7) & ~(size_t)7; }
__host__ __device__ inline size_t ilc_sync_bytes(int64_t nblk, int64_t ntiles) { return (size_t)nblk * 8 + (size_t)ntiles * 4; }
__device__ __forceinline__ IlcSync ilc_sync(uint16_t *P, const TileId &id, int BN)
{
    const int64_t nblk = (int64_t)id.gx * id.gy * id.gz;
    uint64_t *f = (uint64_t *)((uint8_t *)P + ilc_flags_off(nblk, BN));
    return IlcSync{f, (uint32_t *)(f + nblk)};
}
__device__ __forceinline__ uint64_t ilc_flag(uint32_t nonce, int gz, int z)
{
    return ((uint64_t)(nonce + 1u) << 32) | ((uint64_t)(uint32_t)gz << 16) | (uint32_t)z;
}

// the tile's nonce word (sc1 load; an empty buffer range without ILC returns 0): loaded
// unconditionally so that nothing waits for it before the epilogue uses it
__device__ __forceinline__ uint32_t ilc_nonce(uint16_t *P, const TileId &id, int BN, bool ilc)
{
    const int64_t t = (int64_t)id.y * id.gx + id.x;
    const __amdgpu_buffer_rsrc_t nrs = __builtin_amdgcn_make_buffer_rsrc(
        ilc ? (void *)(ilc_sync(P, id, BN).nonce + t) : (void *)P, 0, ilc ? 4 : 0, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b32(nrs, 0, 0, 16);
}

// wave 0: poll the S flags of one tile (sc1 loads, s_sleep between rounds, bounded); true when
// all carry {nonce + 1, S, slot}
__device__ __forceinline__ bool ilc_wait(const uint64_t *tf, uint32_t nonce, int S)
{
    const int lane = threadIdx.x & 63;
    bool ok = false;
    for (int it = 0; it < kIlcSpins && !ok; ++it) {
        bool mine = true;
        for (int s = lane; s < S; s += 64)
            mine = mine && __hip_atomic_load(tf + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ilc_flag(nonce, S, s);
        ok = __builtin_amdgcn_ballot_w64(!mine) == 0;
        if (!ok) __builtin_amdgcn_s_sleep(2);
    }
    if (!ok && lane == 0) __hip_atomic_fetch_add(&g_ilc_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return ok;
}

// Share k of nsh of one tile's split-K sum into C: units [k U / nsh, (k+1) U / nsh) of store_tile's
// block order (NB >= 2: 16-byte units = two token tiles of a lane's 4 rows; NB = 1: 8 bytes), the
// partials of slots 0..S-1 of block row `tile` (blocks tile * slots + s, nblk blocks in all, their
// exponents after them) summed in slot order -- gemm_reduce_f16_kernel's / reduce_grouped_kernel's
// arithmetic.  Every load sc1 (the partials were written through by other CUs in this launch).
template <int NB>
__device__ __forceinline__ void ilc_sum(uint16_t *__restrict__ C, const uint16_t *__restrict__ P, int64_t M, int64_t N,
                                        int64_t ldc, int64_t m0, int64_t n0, int64_t tile, int slots, int64_t nblk, int S,
                                        int k, int nsh)
{
    constexpr int BN = 16 * NB;
    constexpr int TPU = NB == 1 ? 1 : 2, UB = 8 * TPU, UPT = RW * RRG * (NB / TPU) * 64;
    const int tid = threadIdx.x;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)P, 0, (int)(uint32_t)(nblk * (RBM * BN * 2 + RW * 4)), 0x00020000);
    const int u0 = (int)((int64_t)k * UPT / nsh), u1 = (int)((int64_t)(k + 1) * UPT / nsh);
    for (int it = u0 + tid; it < u1; it += (int)blockDim.x) {
        const int q = it >> 6, ln = it & 63, u = q % (NB / TPU), wr = q / (NB / TPU), wv = wr / RRG;
        f32x4 acc[TPU];
#pragma unroll
        for (int j = 0; j < TPU; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        constexpr int G = 16; // splits in flight per thread
        for (int s0 = 0; s0 < S; s0 += G) {
            u32x4 v[G];
            float up[G];
#pragma unroll
            for (int g = 0; g < G; ++g) { // unconditional (clamped) loads, the surplus zeroed after
                const uint32_t b = (uint32_t)(tile * slots + (s0 + g < S ? s0 + g : S - 1));
                const uint32_t eo = (uint32_t)(nblk * (RBM * BN * 2)) + (b * RW + (uint32_t)wv) * 4u;
                up[g] = __builtin_bit_cast(float, (127u + __builtin_amdgcn_raw_buffer_load_b32(prs, eo, 0, 16)) << 23);
                const uint32_t vo = b * (uint32_t)(RBM * BN * 2) + (uint32_t)it * UB;
                if constexpr (TPU == 2) {
                    v[g] = __builtin_amdgcn_raw_buffer_load_b128(prs, vo, 0, 16);
                } else {
                    const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(prs, vo, 0, 16);
                    v[g] = (u32x4){w.x, w.y, 0u, 0u};
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                if (s0 + g >= S) v[g] = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
                for (int j = 0; j < TPU; ++j) {
                    const uint32_t x0 = j == 0 ? v[g].x : v[g].z, x1 = j == 0 ? v[g].y : v[g].w;
                    acc[j][0] += h2f(x0 & 0xffffu) * up[g];
                    acc[j][1] += h2f(x0 >> 16) * up[g];
                    acc[j][2] += h2f(x1 & 0xffffu) * up[g];
                    acc[j][3] += h2f(x1 >> 16) * up[g];
                }
            }
        }
        const int64_t row = m0 + 16 * wr + 4 * (ln >> 4);
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < TPU; ++j) {
            const int64_t tok = n0 + 16 * (TPU * u + j) + (ln & 15);
            if (tok >= N) continue;
            uint16_t *dst = C + tok * ldc + row;
            if (row + 4 <= M) {
                *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(acc[j][0]) | ((uint32_t)f2h_bits(acc[j][1]) << 16),
                                        (uint32_t)f2h_bits(acc[j][2]) | ((uint32_t)f2h_bits(acc[j][3]) << 16)};
            } else {
                for (int e = 0; e < 4 && row + e < M; ++e) dst[e] = f2h_bits(acc[j][e]);
            }
        }
    }
}

// after store_tile (split-K partial, stored sc1): publish, wait for the tile, sum this
// workgroup's share of it into C.  nonce: the tile's nonce word as read at the start (wave 0).
template <int NB>
__device__ __forceinline__ void ilc_combine(uint16_t *__restrict__ C, uint16_t *__restrict__ P, int64_t M, int64_t N,
                                            int64_t ldc, const TileId &id, uint32_t nonce)
{
    constexpr int BN = 16 * NB;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gz = id.gz, z = id.z;
    const int64_t tile = (int64_t)id.y * id.gx + id.x;
    const IlcSync sy = ilc_sync(P, id, BN);
    // 1. this wave's partial stores written through, then every wave's (barrier), then the flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave == 0) {
        uint64_t *tf = sy.flags + tile * gz;
        if (lane == 0) __hip_atomic_store(tf + z, ilc_flag(nonce, gz, z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ilc_wait(tf, nonce, gz); // 2. every split's flag
        // every split of the tile has read the nonce (each did before its flag): advance it
        if (lane == 0 && z == 0) __hip_atomic_store(sy.nonce + tile, nonce + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    // 3. this workgroup's share of the tile
    ilc_sum<NB>(C, P, M, N, ldc, (int64_t)id.x * RBM, (int64_t)id.y * BN, tile, gz, (int64_t)id.gx * id.gy * gz, gz, z,
                gz);
}
template <int NB>
__device__ __forceinline__ void store_tile(const f32x4 (&acc)[RRG][NB], uint16_t *__restrict__ C,
                                           uint16_t *__restrict__ P, int64_t M, int64_t N, int64_t ldc, int spol,
                                           const TileId &id)
{
    constexpr int BN = 16 * NB;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, l16 = lane & 15;
    const int64_t m0 = (int64_t)id.x * RBM, n0 = (int64_t)id.y * BN;
    if (id.gz > 1) {
        // split-K partial, gemm_kernel's fp16 form (its reduce kernel sums it): per (tile, split)
        // a block of 256 x BN halves in accumulator order, each wave's values scaled by 2^-e
        const int64_t tile = (int64_t)id.y * id.gx + id.x;
        const int64_t bidx = tile * id.gz + id.z;
        float mx = 0.f;
#pragma unroll
        for (int rg = 0; rg < RRG; ++rg)
#pragma unroll
            for (int t = 0; t < NB; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) mx = fmaxf(mx, fabsf(acc[rg][t][i]));
        int m = __builtin_bit_cast(int, mx);
        m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x111, 0xf, 0xf, true))));
        m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x112, 0xf, 0xf, true))));
        m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x114, 0xf, 0xf, true))));
        m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x118, 0xf, 0xf, true))));
        m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x142, 0xa, 0xf, true))));
        m = __builtin_bit_cast(int, fmaxf(__builtin_bit_cast(float, m), __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, m, 0x143, 0xc, 0xf, true))));
        const uint32_t mb = (uint32_t)__builtin_amdgcn_readlane(m, 63);
        const int E = (int)((mb >> 23) & 0xff) - 127;
        const int e = E - 14 > 0 ? (E - 14 < 127 ? E - 14 : 126) : 0;
        const float down = __builtin_bit_cast(float, (uint32_t)(127 - e) << 23);
        const int64_t nblk = (int64_t)id.gx * id.gy * id.gz;
        const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)P, 0, (int)(uint32_t)(nblk * (RBM * BN * 2 + RW * 4)), 0x00020000);
        const uint32_t bo = (uint32_t)(bidx * (RBM * BN * 2));
        if (lane == 0) {
            const uint32_t eo = (uint32_t)(nblk * (RBM * BN * 2) + (bidx * RW + wave) * 4);
            if (spol == 2) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)e, prs, eo, 0, 2);
            else if (spol == 16) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)e, prs, eo, 0, 16);
            else __builtin_amdgcn_raw_buffer_store_b32((uint32_t)e, prs, eo, 0, 0);
        }
        auto pk = [down](const f32x4 &v) {
            return (u32x2){(uint32_t)f2h_bits(v[0] * down) | ((uint32_t)f2h_bits(v[1] * down) << 16),
                           (uint32_t)f2h_bits(v[2] * down) | ((uint32_t)f2h_bits(v[3] * down) << 16)};
        };
#pragma unroll
        for (int rg = 0; rg < RRG; ++rg) {
            if constexpr (NB == 1) {
                const uint32_t vo = bo + 8u * (uint32_t)((RRG * wave + rg) * 64 + lane);
                if (spol == 2) __builtin_amdgcn_raw_buffer_store_b64(pk(acc[rg][0]), prs, vo, 0, 2);
                else if (spol == 16) __builtin_amdgcn_raw_buffer_store_b64(pk(acc[rg][0]), prs, vo, 0, 16);
                else __builtin_amdgcn_raw_buffer_store_b64(pk(acc[rg][0]), prs, vo, 0, 0);
            } else {
#pragma unroll
                for (int uu = 0; uu < NB / 2; ++uu) {
                    const u32x2 lo = pk(acc[rg][2 * uu]), hi = pk(acc[rg][2 * uu + 1]);
                    const u32x4 w = {lo.x, lo.y, hi.x, hi.y};
                    const uint32_t vo = bo + 16u * (uint32_t)(((RRG * wave + rg) * (NB / 2) + uu) * 64 + lane);
                    if (spol == 2) __builtin_amdgcn_raw_buffer_store_b128(w, prs, vo, 0, 2);
                    else if (spol == 16) __builtin_amdgcn_raw_buffer_store_b128(w, prs, vo, 0, 16);
                    else __builtin_amdgcn_raw_buffer_store_b128(w, prs, vo, 0, 0);
                }
            }
        }
        return;
    }
#pragma unroll
    for (int rg = 0; rg < RRG; ++rg) {
        const int64_t row = m0 + 16 * (RRG * wave + rg) + 4 * g;
        if (row >= M) continue;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int64_t tok = n0 + 16 * t + l16;
            if (tok >= N) continue;
            const f32x4 v = acc[rg][t];
            uint16_t *dst = C + tok * ldc + row;
            if (row + 4 <= M) {
                *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                        (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)};
            } else {
                for (int i = 0; i < 4 && row + i < M; ++i) dst[i] = f2h_bits(v[i]);
            }
        }
    }
}

// AQ: 0 = prepared x~ (X = fp16 [N][K], DEQ layout); 1 = raw fp16 [N][ldx], q8_1 in-kernel;
// 2 = raw fp16, the fp8 variant's e4m3 quantization in-kernel (F8DEQ x~).
// spol: cache policy of the split-K partial stores (0 plain, 2 nt, 16 sc1; kSpol = sc1, measured
// fastest with the reduce in the timed graph: profiles/r05/rgemm_spol_ab_with_reduce.txt).
// ilc_gx > 0: the in-launch combine (1-D grid of ilc_gx x ilc_gy tiles x the splits, ilc_tile;
// P's partials stored sc1 and summed in this launch by ilc_combine); else the 3-D grid, the
// partials summed by the reduce launch.
template <int F, int NB, int AQ>
__global__ __launch_bounds__(64 * RW) void rgemm_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                       int64_t ldx, uint16_t *__restrict__ C, uint16_t *__restrict__ P,
                                                       int64_t M, int64_t N, int64_t K, int64_t ldc, int spol,
                                                       int ilc_gx, int ilc_gy)
{
    using G = RCfg<F, NB>;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[G::LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool ilc = ilc_gx > 0;
    if (wave >= RPRIO_WAVE) __builtin_amdgcn_s_setprio(1);
    const TileId tile = ilc ? ilc_tile(ilc_gx, ilc_gy) : grid_tile();
    const int64_t m0 = (int64_t)tile.x * RBM, n0 = (int64_t)tile.y * G::BN, sb = tile.z;
    const int64_t row_bytes = (K / Layout<F>::QK) * Layout<F>::BYTES;
    uint8_t *const ximg = lds + G::X_OFF;
#ifdef GQ_RGEMM_STAMPS
    unsigned long long st[14] = {};
    st[0] = __builtin_amdgcn_s_memrealtime();
    GQ_RST(1);
#endif
    // (ILC) the tile's nonce word, read first: every wave's oldest memory op, so every counted
    // vmcnt wait below still counts only the DMAs younger than it; unconditional (a buffer load of
    // an empty range returns 0 without ILC) so that nothing waits for it before the epilogue
    const uint32_t nonce = ilc_nonce(P, tile, G::BN, ilc);

    // 1. (AQ) the raw activations into registers first: their loads return ahead of the weight
    //    DMAs in this wave's in-order memory queue, so the quantization overlaps the weights' flight
    //    (BN tokens x 8 blocks of 32, four lanes -- 8 elements, one 16-byte load -- per block)
    u32x4 xv[AQ ? NB : 1];
    if constexpr (AQ != 0 && !(ABL & 2)) {
        const __amdgpu_buffer_rsrc_t xrs =
            __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, (int)(uint32_t)(((N - 1) * ldx + K) * 2), 0x00020000);
#pragma unroll
        for (int ps = 0; ps < NB; ++ps) {
            const int b = 128 * ps + (tid >> 2), r = b >> 3, kb = b & 7;
            const int64_t tok = n0 + r < N ? n0 + r : N - 1;
            xv[ps] = __builtin_amdgcn_raw_buffer_load_b128(
                xrs, (uint32_t)(tok * ldx * 2) + 2u * (uint32_t)(256 * sb + 32 * kb + 8 * (lane & 3)), 0, 0);
        }
    }

    // 2. the weights: this wave's own 32 rows, both half images, instruction i moving pieces
    //    p = 64i + lane of its region (half p / (32 NPH), row, piece) -- only this wave reads them,
    //    so only its own vmcnt orders them: no workgroup barrier on the weights
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, (int)(uint32_t)((M * row_bytes + 15) & ~(int64_t)15), 0x00020000);
    uint8_t *const wimg = lds + wave * G::WW;
    auto issue_w = [&](auto i0c, auto i1c) __attribute__((always_inline)) {
        constexpr int I0 = decltype(i0c)::value, I1 = decltype(i1c)::value;
        if constexpr (ABL & 1) return;
#pragma unroll
        for (int i = I0; i < I1; ++i) {
            const int p = 64 * i + lane, h = p / (32 * G::NPH), rem = p - h * (32 * G::NPH);
            const int r = rem / G::NPH, pc = (rem - r * G::NPH) ^ hpos_swz<F>(r);
            const int64_t row = m0 + 32 * wave + r < M ? m0 + 32 * wave + r : M - 1;
            dma16(wrs, wimg + 1024 * i, (uint32_t)(row * row_bytes) + hsrc<F>(h, pc), (uint32_t)(G::SB * sb)); // (+16 lane)
        }
    };
    // 3. (prepared) the activation image by LDS-DMA, ahead of the weights: image piece P = 64k + lane:
    //    sub-stage u = P / (BN*8), token r, slot qd (source-swizzled)
    auto issue_x = [&]() __attribute__((always_inline)) {
        if constexpr (AQ != 0 || (ABL & 2)) return;
        const __amdgpu_buffer_rsrc_t xrs =
            __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, (int)(uint32_t)(N * K * 2), 0x00020000);
#pragma unroll
        for (int i = 0; i < G::NX; ++i) {
            const int k = wave + RW * i, pp = 64 * k + lane;
            const int u = pp / (G::BN * 8), r = (pp / 8) % G::BN, qd = pp & 7, q = qd ^ act_swz(r);
            const int64_t tok = n0 + r < N ? n0 + r : N - 1;
            const uint32_t vo = (uint32_t)(tok * K * 2) + 2u * (uint32_t)sub_elem<F>(u, q);
            dma16(xrs, lds + G::X_OFF + 1024 * k, vo, (uint32_t)(512 * sb));
        }
    };
    // AQ: two of the wave's weight DMAs go out before the quantization, the rest after it -- the
    // wave's in-order issue stalls on the memory pipeline's back-pressure, and with all of them
    // ahead the quantization (and so the activation barrier) waited behind that stall: Q8_0 4096^2
    // x128 step 16.76 -> 15.77 us, Q4_K 15.83 -> 15.16, Q6_K 17.67 -> 16.52, Q4_K 11008x4096 x16
    // 16.07 -> 15.70 (profiles/r05/rgemm_wpre_ab.txt: 0..4 and all before; A/B builds
    // -DGQ_RGEMM_WPRE=n)
#ifndef GQ_RGEMM_WPRE
#define GQ_RGEMM_WPRE 2
#endif
    constexpr int WPRE = AQ != 0 && GQ_RGEMM_WPRE < G::WWI ? GQ_RGEMM_WPRE : G::WWI;
    issue_x();
    issue_w(std::integral_constant<int, 0>{}, std::integral_constant<int, WPRE>{});
    GQ_RST(2);

    // 4. (AQ) quantize into the image: x~ = fp16(d*q) in act_quant's DEQ order (deq_quad), or the
    //    fp8 variant's F8DEQ x~ (f8_quad) -- the compiler's vmcnt for xv leaves the DMAs in flight
    if constexpr (AQ != 0 && !(ABL & 2)) {
#pragma unroll
        for (int ps = 0; ps < NB; ++ps) {
            const int b = 128 * ps + (tid >> 2), r = b >> 3, kb = b & 7;
            u32x4 o;
            if constexpr (AQ == 2) {
                const F8Quad fq = f8_quad(xv[ps]);
                o = (u32x4){fq.xt[0], fq.xt[1], fq.xt[2], fq.xt[3]};
            } else {
                o = deq_quad(xv[ps]);
            }
            int u, q;
            block_piece<F>(kb, lane & 3, u, q);
            *(u32x4 *)(ximg + u * (G::BN * 128) + 128 * r + 16 * (q ^ act_swz(r))) = o;
        }
    }
    issue_w(std::integral_constant<int, WPRE>{}, std::integral_constant<int, G::WWI>{});
    // the activation image complete (every wave's DMAs, or every wave's quantized pieces): this
    // wave's x loads are older than its weight DMAs, so all but those are awaited
    constexpr int WN = (ABL & 1) ? 0 : G::WWI;
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(WN) : "memory");
    GQ_RST(3);
    __builtin_amdgcn_s_barrier();
    GQ_RST(4);

    // 5. the multiply: the wave's rows 16*rg + [0, 16), every token, 4 sub-stages x 2 k-steps; the
    //    first half as soon as this wave's own half-0 DMAs landed
    f32x4 acc[RRG][NB];
#pragma unroll
    for (int rg = 0; rg < RRG; ++rg)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[rg][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    constexpr int H1N = (ABL & 1) ? 0 : G::WWI - G::H0I;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(H1N) : "memory");
    GQ_RST(5);
#pragma unroll
    for (int u = 0; u < 4 && !(ABL & 4); ++u) {
        if (u == 2) { // the second half
#ifdef GQ_RGEMM_STAMPS
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            for (int rg = 0; rg < RRG; ++rg)
                for (int t = 0; t < NB; ++t) asm volatile("" ::"v"(acc[rg][t]));
#endif
            GQ_RST(6);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            GQ_RST(7);
        }
        mul_substage<F, NB>(wimg + (u >> 1) * (32 * G::HRB), ximg + u * (G::BN * 128), u, acc, 0);
    }
#ifdef GQ_RGEMM_STAMPS
    for (int rg = 0; rg < RRG; ++rg)
        for (int t = 0; t < NB; ++t) asm volatile("" ::"v"(acc[rg][t]));
#endif
    GQ_RST(8);
    if constexpr ((ABL & 4) != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // 6. epilogue
    if constexpr ((ABL & 8) != 0) {
        if (acc[0][0][0] == 1234.5f) C[0] = 0;
        return;
    }
    store_tile<NB>(acc, C, P, M, N, ldc, ilc ? 16 : spol, tile);
    if (ilc && tile.gz > 1) ilc_combine<NB>(C, P, M, N, ldc, tile, nonce);
#ifdef GQ_RGEMM_STAMPS
    GQ_RST(9);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    GQ_RST(10);
    st[11] = __builtin_amdgcn_s_memrealtime();
    const int wg = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    st[12] = (unsigned long long)wg;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    st[13] = xcc & 0xfu;
    const int id = wg * RW + wave;
    if (lane == 0 && id < 65536)
        for (int i = 0; i < 14; ++i) g_rstamps[id][i] = st[i];
#endif
}

// ---------------------------------------------------------------------------------------
// The streaming form (sgemm_kernel): the same 256-row x 16*NB-token tile and multiply over a
// K split of several super-blocks, the split's half-super-block stages (the W half image + the
// activations' half x~ image, prepared by act_quant) through a ring of NS slots in LDS: stage j
// lands -> barrier -> stage j+NS-1 is issued into the slot stage j-1 left -> stage j is multiplied.
// For the matrices whose row tiles x super-blocks exceed one round of the chip (the 70B Q6_K
// matrices, 11008-row Q4_K); split-K partials as rgemm_kernel's.
#ifndef GQ_SGEMM_NSMAX
#define GQ_SGEMM_NSMAX 6
#endif
constexpr int SG_NSMAX = GQ_SGEMM_NSMAX; // ring slots at most (A/B builds: -DGQ_SGEMM_NSMAX=n)
template <int F, int NB> struct SCfg {
    static constexpr int BN = 16 * NB;
    static constexpr int NPH = HImg<F>::NPH, HRB = 16 * NPH, SB = Layout<F>::BYTES * (256 / Layout<F>::QK);
    static constexpr int W_BYTES = RBM * HRB, X_BYTES = BN * 256; // one half stage
    static constexpr int SLOT = W_BYTES + X_BYTES;
    static constexpr int WH_INSTR = (RBM * NPH + 63) / 64, NWH = (WH_INSTR + RW - 1) / RW;
    static constexpr int XH_INSTR = X_BYTES / 1024, NXH = (XH_INSTR + RW - 1) / RW;
    static constexpr int NPS = ((ABL & 1) ? 0 : NWH) + ((ABL & 2) ? 0 : NXH); // DMA instructions per wave and stage
    static constexpr bool PAD = WH_INSTR % RW != 0 || XH_INSTR % RW != 0 || XH_INSTR < RW;
    static constexpr int NS = (LDS_CAP - 1024) / SLOT > SG_NSMAX ? SG_NSMAX : (LDS_CAP - 1024) / SLOT; // ring slots
    static constexpr int SCRATCH = NS * SLOT;
    static constexpr int LDS = SCRATCH + (PAD ? 1024 : 0);
    static_assert(NS >= 2, "two ring slots");
    static_assert(LDS <= LDS_CAP, "LDS budget");
    static_assert((NS - 2) * NPS <= 63, "vmcnt range");
};

constexpr int kMaxSParts = 16;
struct SPart {
    int fmt;
    const uint8_t *A;
    const uint16_t *X;
    uint16_t *C, *P;
    int64_t M, K, ldc;
    int tiles_m, tiles_n, splits, wg0;
    int ustart, scap; // stream-K: the part's first unit (tile-major (tile, super-block) order), partial slots per tile
    int cost, cstart; // stream-K: cost per unit, cost before the part's first unit
    uint64_t *flags;  // in-launch combine: [tile * scap + slot]
    uint32_t *nonce;  // [tile]
};
struct SParts {
    int n;
    int64_t N;
    int spol;
    int streamk, U, W; // stream-K: U units over W workgroups, workgroup w = units [wU/W, (w+1)U/W)
    int full;          // GQ_SGEMM_FULL (Q4_K, NB <= 2: sgemm_full_body)
    int ilc;           // stream-K: the split tiles summed in this launch (no reduce launch)
    SPart p[kMaxSParts];
};
struct RPart {
    const uint16_t *P;
    uint16_t *C;
    int64_t M, ldc;
    int tiles_m, tiles_n, splits, wg0;
    int ustart, nsb, scap;
    int cost, cstart;
};
struct RParts {
    int n;
    int64_t N;
    int streamk, U, W;
    RPart p[kMaxSParts];
};

// stream-K: the workgroups whose unit ranges hold the first and the last unit of [u0, u1)
// (U: the total cost; workgroup w holds the units whose cost start is in [wU/W, (w+1)U/W))
__device__ __forceinline__ int sk_first_wg(int u0, int U, int W) { return (int)(((int64_t)(u0 + 1) * W + U - 1) / U) - 1; }
__device__ __forceinline__ int sk_last_wg(int u1, int U, int W) { return (int)(((int64_t)u1 * W + U - 1) / U) - 1; }
// the workgroup holding unit u of a part (its cost start: cstart + (u - ustart) * cost)
template <typename Q> __device__ __forceinline__ int sk_owner(const Q &q, int u, int U, int W)
{
    return sk_first_wg(q.cstart + (u - q.ustart) * q.cost, U, W);
}

template <int F, int NB>
__device__ __forceinline__ void sgemm_body(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                           uint16_t *__restrict__ C, uint16_t *__restrict__ P, int64_t M, int64_t N,
                                           int64_t K, int64_t ldc, int spol, const TileId &id, int64_t sb0, int64_t sb1,
                                           uint8_t *lds)
{
    using G = SCfg<F, NB>;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (wave >= RPRIO_WAVE) __builtin_amdgcn_s_setprio(1);
    const int64_t m0 = (int64_t)id.x * RBM, n0 = (int64_t)id.y * G::BN;
    const int64_t row_bytes = (K / Layout<F>::QK) * Layout<F>::BYTES;
    // super-blocks [sb0, sb1) of the tile; the partial (or C when id.gz == 1) as split id.z
    const int nst = (int)(2 * (sb1 - sb0)); // half stages
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, (int)(uint32_t)((M * row_bytes + 15) & ~(int64_t)15), 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, (int)(uint32_t)(N * K * 2), 0x00020000);

    auto issue = [&](int j) __attribute__((always_inline)) {
        uint8_t *slot = lds + (j % G::NS) * G::SLOT;
        const int64_t sb = sb0 + (j >> 1);
        const int h = j & 1;
#pragma unroll
        for (int i = 0; i < ((ABL & 1) ? 0 : G::NWH); ++i) {
            const int k = wave + RW * i, p = 64 * k + lane, r = p / G::NPH, pc = (p - r * G::NPH) ^ hpos_swz<F>(r);
            const bool real = k < G::WH_INSTR;
            const int64_t row = m0 + r < M ? m0 + r : M - 1;
            const uint32_t vo = real ? (uint32_t)(row * row_bytes) + hsrc<F>(h, pc) : 0u;
            dma16(wrs, real ? slot + 1024 * k : lds + G::SCRATCH, vo, (uint32_t)(G::SB * sb)); // (+16 lane)
        }
        // activation half image: piece P = 64k + lane: sub-stage ul = P / (BN*8), token r, slot qd
#pragma unroll
        for (int i = 0; i < ((ABL & 2) ? 0 : G::NXH); ++i) {
            const int k = wave + RW * i, pp = 64 * k + lane;
            const bool real = k < G::XH_INSTR;
            const int ul = pp / (G::BN * 8), r = (pp / 8) % G::BN, qd = pp & 7, q = qd ^ act_swz(r);
            const int64_t tok = n0 + r < N ? n0 + r : N - 1;
            const uint32_t vo = real ? (uint32_t)(tok * K * 2) + 2u * (uint32_t)sub_elem<F>(2 * h + ul, q) : 0u;
            dma16(xrs, real ? slot + G::W_BYTES + 1024 * k : lds + G::SCRATCH, vo, (uint32_t)(512 * sb));
        }
    };

    f32x4 acc[RRG][NB];
#pragma unroll
    for (int rg = 0; rg < RRG; ++rg)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[rg][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int issued = G::NS - 1 < nst ? G::NS - 1 : nst;
    for (int i = 0; i < issued; ++i) issue(i);
    for (int j = 0; j < nst; ++j) {
        // stage j landed: all but the (<= NS-2) younger stages this wave issued
        vm_wait<(G::NS - 2) * G::NPS>((issued - 1 - j) * G::NPS);
        __builtin_amdgcn_s_barrier();
        if (issued < nst) issue(issued++); // into the slot stage j-1 left (barrier passed)
        const uint8_t *slot = lds + (j % G::NS) * G::SLOT;
        const int h = j & 1;
        if constexpr ((ABL & 4) != 0) continue; // (ablation builds: no multiply)
#pragma unroll
        for (int ul = 0; ul < 2; ++ul)
            mul_substage<F, NB>(slot, slot + G::W_BYTES + ul * (G::BN * 128), 2 * h + ul, acc, 32 * wave);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // (nothing is in flight here; no DMA outlives the workgroup)
    store_tile<NB>(acc, C, P, M, N, ldc, spol, id);
}

// Q4_K with whole-super-block stages (GQ_SGEMM_FULL; 16 / 32-token tiles; the default for single
// matrices: 11008x4096x16 17.1 vs 22.3 us, 4096x11008x16 15.9 vs 20.0; the grouped layer no
// different, 65.6 vs 65.7 at 8 tokens: profiles/r04/ab15_full_*.txt): a stage is the rows'
// super-block as one 144-byte image per row (gemm_kernel's WStage<Q4_K> layout: the header once,
// each row's bytes one contiguous run, 36 DMA instructions of ~7 rows each instead of 2 x 20 of
// ~13 rows x 80 bytes) and the super-block's four x~ sub-stages.  Same fragments, same MFMA
// sequence as the half stages (q4k_frags on the same bytes): the same bits.
template <int NB> struct SFull {
    static constexpr int BN = 16 * NB, NPW = 9, RBW = 16 * NPW;
    static constexpr int W_BYTES = RBM * RBW, X_BYTES = BN * 512, SLOT = W_BYTES + X_BYTES;
    static constexpr int W_INSTR = RBM * NPW / 64, NW = (W_INSTR + RW - 1) / RW;
    static constexpr int X_INSTR = X_BYTES / 1024, NX = (X_INSTR + RW - 1) / RW;
    static constexpr int NPS = NW + NX;
    static constexpr int NS = (LDS_CAP - 1024) / SLOT > SG_NSMAX ? SG_NSMAX : (LDS_CAP - 1024) / SLOT;
    static constexpr int SCRATCH = NS * SLOT, LDS = SCRATCH + 1024;
    static_assert(RBM * NPW % 64 == 0 && NS >= 2 && LDS <= LDS_CAP && (NS - 2) * NPS <= 63, "SFull");
};

template <int NB>
__device__ __forceinline__ void sgemm_full_body(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                uint16_t *__restrict__ C, uint16_t *__restrict__ P, int64_t M, int64_t N,
                                                int64_t K, int64_t ldc, int spol, const TileId &id, int64_t sb0, int64_t sb1,
                                                uint8_t *lds)
{
    using G = SFull<NB>;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (wave >= RPRIO_WAVE) __builtin_amdgcn_s_setprio(1);
    const int g = lane >> 4, l16 = lane & 15;
    const int64_t m0 = (int64_t)id.x * RBM, n0 = (int64_t)id.y * G::BN;
    const int64_t row_bytes = (K / 256) * 144;
    const int nst = (int)(sb1 - sb0);
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, (int)(uint32_t)((M * row_bytes + 15) & ~(int64_t)15), 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, (int)(uint32_t)(N * K * 2), 0x00020000);
    auto issue = [&](int j) __attribute__((always_inline)) {
        uint8_t *slot = lds + (j % G::NS) * G::SLOT;
        const int64_t sb = sb0 + j;
#pragma unroll
        for (int i = 0; i < ((ABL & 1) ? 0 : G::NW); ++i) {
            const int k = wave + RW * i, p = 64 * k + lane, r = p / G::NPW, pc = p - r * G::NPW;
            const bool real = k < G::W_INSTR;
            const int64_t row = m0 + r < M ? m0 + r : M - 1;
            const uint32_t vo = real ? (uint32_t)(row * row_bytes) + 16u * pc : 0u;
            dma16(wrs, real ? slot + 1024 * k : lds + G::SCRATCH, vo, (uint32_t)(144 * sb));
        }
#pragma unroll
        for (int i = 0; i < G::NX; ++i) {
            const int k = wave + RW * i, pp = 64 * k + lane;
            const bool real = k < G::X_INSTR;
            const int u = pp / (G::BN * 8), r = (pp / 8) % G::BN, qd = pp & 7, q = qd ^ act_swz(r);
            const int64_t tok = n0 + r < N ? n0 + r : N - 1;
            const uint32_t vo = real ? (uint32_t)(tok * K * 2) + 2u * (uint32_t)sub_elem<Q4_K>(u, q) : 0u;
            dma16(xrs, real ? slot + G::W_BYTES + 1024 * k : lds + G::SCRATCH, vo, (uint32_t)(512 * sb));
        }
    };
    f32x4 acc[RRG][NB];
#pragma unroll
    for (int rg = 0; rg < RRG; ++rg)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[rg][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int issued = G::NS - 1 < nst ? G::NS - 1 : nst;
    for (int i = 0; i < issued; ++i) issue(i);
    for (int j = 0; j < nst; ++j) {
        vm_wait<(G::NS - 2) * G::NPS>((issued - 1 - j) * G::NPS);
        __builtin_amdgcn_s_barrier();
        if (issued < nst) issue(issued++);
        const uint8_t *slot = lds + (j % G::NS) * G::SLOT;
        if constexpr ((ABL & 4) != 0) continue;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint8_t *xs = slot + G::W_BYTES + u * (G::BN * 128);
            f16x8 af[RRG][2];
#pragma unroll
            for (int rg = 0; rg < RRG; ++rg) {
                const uint8_t *wr = slot + G::RBW * (16 * (RRG * wave + rg) + l16);
                q4k_frags(wr, wr + 16 + 32 * u, g, u, af[rg]);
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                f16x8 bk[NB];
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const int r = 16 * t + l16;
                    bk[t] = *(const f16x8 *)(xs + 128 * r + 16 * ((4 * s + g) ^ act_swz(r)));
                }
#pragma unroll
                for (int rg = 0; rg < RRG; ++rg)
#pragma unroll
                    for (int t = 0; t < NB; ++t)
                        acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[rg][s], bk[t], acc[rg][t], 0, 0, 0);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_tile<NB>(acc, C, P, M, N, ldc, spol, id);
}

template <int F, int NB> constexpr int sgemm_lds()
{
    if constexpr (F == Q4_K && NB <= 2) return SCfg<F, NB>::LDS > SFull<NB>::LDS ? SCfg<F, NB>::LDS : SFull<NB>::LDS;
    return SCfg<F, NB>::LDS;
}

// The streaming GEMM's default 1-D order (gz1 > 0): split-major positions, dealt to the XCDs in
// contiguous runs (p as ilc_tile's), so that an XCD holds one or two K splits of every row tile
// instead of every split of a few row tiles -- its L2 then holds its splits' activations only
// (8192x28672 x128: one 917 KB slice per XCD instead of all eight, 7.3 MB, against a 4 MB L2)
__device__ __forceinline__ TileId zmajor_tile(int gx, int gy, int gz)
{
    const int nb = (int)gridDim.x, b = (int)blockIdx.x, tiles = gx * gy;
    const int p = (nb & 7) == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b, z = p / tiles, t = p - z * tiles;
    return TileId{t % gx, t / gx, z, gx, gy, gz};
}

// order (1-D grid of gx x gy tiles x the splits): 1 = the in-launch split-K combine, as
// rgemm_kernel's (ilc_tile); 2 = the split-major order (zmajor_tile), partials summed by the
// reduce launch; 0 = the 3-D grid
template <int F, int NB>
__global__ __launch_bounds__(64 * RW) void sgemm_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                       uint16_t *__restrict__ C, uint16_t *__restrict__ P, int64_t M,
                                                       int64_t N, int64_t K, int64_t ldc, int spol, int full, int gx,
                                                       int gy, int order)
{
    __shared__ __attribute__((aligned(1024))) uint8_t lds[sgemm_lds<F, NB>()];
    // split z: super-blocks [z*nsb/S, (z+1)*nsb/S) (split lengths differ by one when S does not divide)
    const bool ilc = order == 1;
    const TileId id = ilc ? ilc_tile(gx, gy) : (order == 2 ? zmajor_tile(gx, gy, (int)gridDim.x / (gx * gy)) : grid_tile());
    const int64_t nsb = K / 256, s0 = id.z * nsb / id.gz, s1 = (id.z + 1) * nsb / id.gz;
    const uint32_t nonce = ilc_nonce(P, id, 16 * NB, ilc); // (the oldest memory op: see rgemm_kernel)
    const int sp = ilc ? 16 : spol;
    bool done = false;
    if constexpr (F == Q4_K && NB <= 2) {
        if (full) {
            sgemm_full_body<NB>(A, X, C, P, M, N, K, ldc, sp, id, s0, s1, lds);
            done = true;
        }
    }
    if (!done) sgemm_body<F, NB>(A, X, C, P, M, N, K, ldc, sp, id, s0, s1, lds);
    if (ilc && id.gz > 1) ilc_combine<NB>(C, P, M, N, ldc, id, nonce);
}

// ---- several matrices in one launch (gq_mmq_grouped_prepared): part i = one matrix's
// (row tile, token tile, split) grid, its workgroups [wg0, wg0 + tiles_m * tiles_n * splits)
template <int NB> constexpr int max_slds()
{
    constexpr int a = SCfg<Q8_0, NB>::LDS, b = sgemm_lds<Q4_K, NB>(), c = SCfg<Q6_K, NB>::LDS;
    return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

template <int NB>
__global__ __launch_bounds__(64 * RW) void sgemm_grouped_kernel(const SParts a);
template <int NB> int grouped_occ()
{
    int n = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, sgemm_grouped_kernel<NB>, 64 * RW, 0) == hipSuccess ? n : 0;
}
template <int NB>
__global__ __launch_bounds__(64 * RW) void sgemm_grouped_kernel(const SParts a)
{
    __shared__ __attribute__((aligned(1024))) uint8_t lds[max_slds<NB>()];
    const int b = (int)blockIdx.x;
    auto run = [&](const SPart &q, const TileId &id, int64_t sb0, int64_t sb1) __attribute__((always_inline)) {
        switch (q.fmt) {
        case Q8_0: sgemm_body<Q8_0, NB>(q.A, q.X, q.C, q.P, q.M, a.N, q.K, q.ldc, a.spol, id, sb0, sb1, lds); return;
        case Q4_K:
            if constexpr (NB <= 2) {
                if (a.full) {
                    sgemm_full_body<NB>(q.A, q.X, q.C, q.P, q.M, a.N, q.K, q.ldc, a.spol, id, sb0, sb1, lds);
                    return;
                }
            }
            sgemm_body<Q4_K, NB>(q.A, q.X, q.C, q.P, q.M, a.N, q.K, q.ldc, a.spol, id, sb0, sb1, lds);
            return;
        default: sgemm_body<Q6_K, NB>(q.A, q.X, q.C, q.P, q.M, a.N, q.K, q.ldc, a.spol, id, sb0, sb1, lds); return;
        }
    };
    if (!a.streamk) { // tile-granular splits: workgroup = (part, tile, split)
        int i = 0;
        while (i + 1 < a.n && b >= a.p[i + 1].wg0) ++i;
        const SPart &q = a.p[i];
        const int l = b - q.wg0, txy = q.tiles_m * q.tiles_n;
        const TileId id{l % q.tiles_m, (l % txy) / q.tiles_m, l / txy, q.tiles_m, q.tiles_n, q.splits};
        const int64_t nsb = q.K / 256;
        run(q, id, id.z * nsb / id.gz, (id.z + 1) * nsb / id.gz);
        return;
    }
    // stream-K: this workgroup's units [u0, u1) of the parts' (tile, super-block) sequence, as
    // segments of at most one tile each; a tile all of whose units one workgroup holds is stored
    // whole, else each of its S_t workgroups writes partial slot k (in workgroup order)
    const int64_t c0 = (int64_t)b * a.U / a.W, c1 = (int64_t)(b + 1) * a.U / a.W;
    bool first = true;
    // (ILC) the split tiles this workgroup wrote a slot of: only its first and its last tile can be
    // split (a tile between them lies wholly in its range), so at most two
    int nsp = 0, sp_part[2], sp_tile[2], sp_k[2], sp_st[2];
    uint32_t sp_nonce[2];
    for (int i = 0; i < a.n; ++i) {
        const SPart &q = a.p[i];
        const int nsb = (int)(q.K / 256), nu = q.tiles_m * q.tiles_n * nsb;
        const int64_t lo = c0 - q.cstart, hi = c1 - q.cstart;
        if (hi <= 0) break; // (parts in cost order)
        int u = q.ustart + (int)(lo <= 0 ? 0 : (lo + q.cost - 1) / q.cost);
        const int64_t k1 = (hi + q.cost - 1) / q.cost;
        const int u1 = q.ustart + (int)(k1 < nu ? k1 : nu);
        while (u < u1) {
            const int local = u - q.ustart, tile = local / nsb, sb = local - tile * nsb;
            const int t0 = q.ustart + tile * nsb, t1 = t0 + nsb;
            const int end = u1 < t1 ? u1 : t1;
            const int wf = sk_owner(q, t0, a.U, a.W), st = sk_owner(q, t1 - 1, a.U, a.W) - wf + 1;
            const TileId id{tile % q.tiles_m, tile / q.tiles_m, st == 1 ? 0 : b - wf, q.tiles_m, q.tiles_n, st == 1 ? 1 : q.scap};
            if (a.ilc && st > 1) { // the tile's nonce word, read before this slot's flag can exist
                if (nsp < 2) {
                    const __amdgpu_buffer_rsrc_t nrs = __builtin_amdgcn_make_buffer_rsrc(q.nonce + tile, 0, 4, 0x00020000);
                    sp_nonce[nsp] = __builtin_amdgcn_raw_buffer_load_b32(nrs, 0, 0, 16);
                    sp_part[nsp] = i;
                    sp_tile[nsp] = tile;
                    sp_k[nsp] = b - wf;
                    sp_st[nsp] = st;
                } else if (threadIdx.x == 0) { // (impossible by the plan; made visible, never silent)
                    __hip_atomic_fetch_add(&g_ilc_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                ++nsp;
            }
            if (!first) __builtin_amdgcn_s_barrier(); // (the previous segment's last stage is read by every wave)
            run(q, id, sb, sb + (end - u));
            first = false;
            u = end;
        }
    }
    if (!a.ilc || nsp == 0) return;
    // in-launch combine (ilc_combine's hand-off): every slot this workgroup wrote is published,
    // then each of its split tiles awaited and this workgroup's share of it (share k of st)
    // summed into C in slot order -- reduce_grouped_kernel's arithmetic, its bits
    if (nsp > 2) nsp = 2;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave == 0) {
        for (int c = 0; c < nsp; ++c) {
            const SPart &q = a.p[sp_part[c]];
            if (lane == 0)
                __hip_atomic_store(q.flags + (int64_t)sp_tile[c] * q.scap + sp_k[c], ilc_flag(sp_nonce[c], sp_st[c], sp_k[c]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int c = 0; c < nsp; ++c) {
            const SPart &q = a.p[sp_part[c]];
            ilc_wait(q.flags + (int64_t)sp_tile[c] * q.scap, sp_nonce[c], sp_st[c]);
            if (lane == 0 && sp_k[c] == 0)
                __hip_atomic_store(q.nonce + sp_tile[c], sp_nonce[c] + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    for (int c = 0; c < nsp; ++c) {
        const SPart &q = a.p[sp_part[c]];
        const int t = sp_tile[c];
        ilc_sum<NB>(q.C, q.P, q.M, a.N, q.ldc, (int64_t)(t % q.tiles_m) * RBM, (int64_t)(t / q.tiles_m) * (16 * NB), t,
                    q.scap, (int64_t)q.tiles_m * q.tiles_n * q.scap, sp_st[c], sp_k[c], sp_st[c]);
    }
}

// The split-K sum of several parts' fp16 partials (store_tile's form): one thread per 16-byte
// unit of a tile block (two token tiles x 4 rows; NB = 1: 8 bytes, one token tile); a part's S
// splits summed in split order in fp32 after each wave's 2^e -- gemm_reduce_f16_kernel's
// arithmetic (the same order, the same trailing +0 for S % 8 != 0), so every part's bits equal
// its own launch's.
template <int NB>
__global__ __launch_bounds__(256) void reduce_grouped_kernel(const RParts a)
{
    constexpr int TPU = NB == 1 ? 1 : 2, UPT = RW * RRG * (NB / TPU) * 64; // units per tile
    constexpr int BPT = (UPT + 255) / 256;
    const int b = (int)blockIdx.x;
    int i = 0;
    while (i + 1 < a.n && b >= a.p[i + 1].wg0) ++i;
    const RPart &q = a.p[i];
    const int l = b - q.wg0, tile = l / BPT, it = (l % BPT) * 256 + (int)threadIdx.x;
    const int ntiles = q.tiles_m * q.tiles_n;
    if (tile >= ntiles || it >= UPT) return;
    int S = q.splits, ss = q.splits; // splits summed, partial slots per tile
    if (a.streamk) {
        const int t0 = q.ustart + tile * q.nsb;
        S = sk_owner(q, t0 + q.nsb - 1, a.U, a.W) - sk_owner(q, t0, a.U, a.W) + 1;
        ss = q.scap;
        if (S == 1) return; // (stored whole by its workgroup)
    }
    const int lane = it & 63, u = (it >> 6) % (NB / TPU), wr = (it >> 6) / (NB / TPU);
    const int wv = __builtin_amdgcn_readfirstlane(wr / RRG);
    const int64_t m0 = (int64_t)(tile % q.tiles_m) * RBM, n0 = (int64_t)(tile / q.tiles_m) * (16 * NB);
    const int64_t blk = (int64_t)RBM * 16 * NB; // halves per (tile, split) block
    const int *es = (const int *)(q.P + (int64_t)ntiles * ss * blk);
    f32x4 acc[TPU];
#pragma unroll
    for (int j = 0; j < TPU; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < S; s0 += 8) {
        u32x4 v[8];
        float up[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { // unconditional (clamped) loads, the surplus zeroed after
            const int64_t sp = (int64_t)tile * ss + (s0 + k < S ? s0 + k : S - 1);
            up[k] = __builtin_bit_cast(float, (uint32_t)(127 + es[sp * RW + wv]) << 23);
            if constexpr (TPU == 2) {
                v[k] = ((const u32x4 *)(q.P + sp * blk))[it];
            } else {
                const u32x2 w = ((const u32x2 *)(q.P + sp * blk))[it];
                v[k] = (u32x4){w.x, w.y, 0u, 0u};
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (s0 + k >= S) v[k] = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < TPU; ++j) {
                const uint32_t x0 = j == 0 ? v[k].x : v[k].z, x1 = j == 0 ? v[k].y : v[k].w;
                acc[j][0] += h2f(x0 & 0xffffu) * up[k];
                acc[j][1] += h2f(x0 >> 16) * up[k];
                acc[j][2] += h2f(x1 & 0xffffu) * up[k];
                acc[j][3] += h2f(x1 >> 16) * up[k];
            }
        }
    }
    const int64_t row = m0 + 16 * wr + 4 * (lane >> 4);
    if (row >= q.M) return;
#pragma unroll
    for (int j = 0; j < TPU; ++j) {
        const int64_t tok = n0 + 16 * (TPU * u + j) + (lane & 15);
        if (tok >= a.N) continue;
        uint16_t *dst = q.C + tok * q.ldc + row;
        if (row + 4 <= q.M) {
            *(u32x2 *)dst = (u32x2){(uint32_t)f2h_bits(acc[j][0]) | ((uint32_t)f2h_bits(acc[j][1]) << 16),
                                    (uint32_t)f2h_bits(acc[j][2]) | ((uint32_t)f2h_bits(acc[j][3]) << 16)};
        } else {
            for (int e = 0; e < 4 && row + e < q.M; ++e) dst[e] = f2h_bits(acc[j][e]);
        }
    }
}

template <int F, int NB>
hipError_t launch_snb(const uint8_t *A, const uint16_t *X, uint16_t *C, void *P, const RGemmPlan &p, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    static const int occ = [] {
        int n = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, sgemm_kernel<F, NB>, 64 * RW, 0) == hipSuccess ? n : 0;
    }();
    const int64_t blocks = (int64_t)p.tiles_m * p.tiles_n * p.splits;
    if (sgemm_ilc(p) && blocks <= (int64_t)num_cus() * occ) { // one kernel
        sgemm_kernel<F, NB><<<dim3((unsigned)blocks), dim3(64 * RW), 0, s>>>(A, X, C, (uint16_t *)P, M, N, K, ldc, 16,
                                                                             tuning().sgemm_full != 0, p.tiles_m, p.tiles_n, 1);
        return hipGetLastError();
    }
    // the split-major order where the activations outgrow an XCD's 4 MiB L2 (each XCD then holds
    // its splits' slices only; 8192x28672 x128: FETCH / algorithmic bytes 1.39 -> 1.07 at the same
    // time, 97.9 vs 98.1 us).  Below that the 3-D grid's refetches are Infinity-Cache hits that
    // cost nothing and the split-major order measured 1.5-5% slower (4096x11008 x128 31.3 vs 30.7 us
    // -- though 1.80 -> 1.12 traffic --, 28672x8192 106.4 vs 104.8; profiles/r06/sgemm_zorder_ab.txt)
#ifndef GQ_SGEMM_ZORDER
#define GQ_SGEMM_ZORDER 1 // (A/B builds: -DGQ_SGEMM_ZORDER=0, the 3-D grid everywhere)
#endif
    if (GQ_SGEMM_ZORDER && p.splits > 1 && (blocks & 7) == 0 && N * K * 2 > ((int64_t)4 << 20)) {
        sgemm_kernel<F, NB><<<dim3((unsigned)blocks), dim3(64 * RW), 0, s>>>(A, X, C, (uint16_t *)P, M, N, K, ldc, kSpol,
                                                                             tuning().sgemm_full != 0, p.tiles_m, p.tiles_n, 2);
    } else {
        const dim3 grid((unsigned)p.tiles_m, (unsigned)p.tiles_n, (unsigned)p.splits);
        sgemm_kernel<F, NB><<<grid, dim3(64 * RW), 0, s>>>(A, X, C, (uint16_t *)P, M, N, K, ldc, kSpol,
                                                            tuning().sgemm_full != 0, 0, 0, 0);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_gemm_reduce_f16(NB, RRG, (const uint16_t *)P, C, M, N, ldc, p.splits, p.tiles_m, p.tiles_n, s);
}

template <int F, int NB, int AQ>
hipError_t launch_nb(const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, void *P, const RGemmPlan &p,
                     int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    // workgroups a CU admits at once (the runtime's answer: registers as well as LDS)
    static const int occ = [] {
        int n = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rgemm_kernel<F, NB, AQ>, 64 * RW, 0) == hipSuccess ? n : 0;
    }();
    const int64_t blocks = (int64_t)p.tiles_m * p.tiles_n * p.splits;
    if (rgemm_ilc(F, p) && blocks <= (int64_t)num_cus() * occ) { // the split-K sum inside the launch: one kernel
        rgemm_kernel<F, NB, AQ><<<dim3((unsigned)blocks), dim3(64 * RW), 0, s>>>(A, X, ldx, C, (uint16_t *)P, M, N, K, ldc,
                                                                                 16, p.tiles_m, p.tiles_n);
        return hipGetLastError();
    }
    const dim3 grid((unsigned)p.tiles_m, (unsigned)p.tiles_n, (unsigned)p.splits);
    rgemm_kernel<F, NB, AQ><<<grid, dim3(64 * RW), 0, s>>>(A, X, ldx, C, (uint16_t *)P, M, N, K, ldc, kSpol,
                                                           0, 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_gemm_reduce_f16(NB, RRG, (const uint16_t *)P, C, M, N, ldc, p.splits, p.tiles_m, p.tiles_n, s);
}

template <int F, int AQ>
hipError_t launch_f(const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, void *P, const RGemmPlan &p,
                    int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (p.nb) {
    case 1: return launch_nb<F, 1, AQ>(A, X, ldx, C, P, p, M, N, K, ldc, s);
    case 2: return launch_nb<F, 2, AQ>(A, X, ldx, C, P, p, M, N, K, ldc, s);
    case 4: return launch_nb<F, 4, AQ>(A, X, ldx, C, P, p, M, N, K, ldc, s);
    case 8: return launch_nb<F, 8, AQ>(A, X, ldx, C, P, p, M, N, K, ldc, s);
    default: return hipErrorInvalidValue;
    }
}

} // namespace

int rgemm_per_cu(int fmt, int nb)
{
#define GQ_RPC(F)                                                                                                      \
    switch (nb) {                                                                                                      \
    case 1: return LDS_CAP / RCfg<F, 1>::LDS;                                                                          \
    case 2: return LDS_CAP / RCfg<F, 2>::LDS;                                                                          \
    case 4: return LDS_CAP / RCfg<F, 4>::LDS;                                                                          \
    default: return LDS_CAP / RCfg<F, 8>::LDS;                                                                         \
    }
    switch (fmt) {
    case Q8_0: GQ_RPC(Q8_0)
    case Q4_K: GQ_RPC(Q4_K)
    default: GQ_RPC(Q6_K)
    }
#undef GQ_RPC
}

RGemmPlan plan_rgemm(int64_t M, int64_t N, int64_t K)
{
    RGemmPlan p;
    if (M < 1 || N < 1 || K < 256 || K % 256 != 0) return p;
    p.nb = N > 64 ? 8 : (N > 32 ? 4 : (N > 16 ? 2 : 1));
    p.tiles_m = (int)((M + RBM - 1) / RBM);
    p.tiles_n = (int)((N + 16 * p.nb - 1) / (16 * p.nb));
    p.splits = (int)(K / 256);
    const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n, nblk = tiles * p.splits;
    // the partial blocks and their exponents, then the in-launch combine's flags and nonces
    p.partial_bytes = p.splits > 1 ? ilc_flags_off(nblk, 16 * p.nb) + ilc_sync_bytes(nblk, tiles) : 0;
    p.ok = true;
    return p;
}

// The in-launch combine (ilc_combine) instead of the reduce launch: split-K plans whose grid the
// chip holds at once (its tile's workgroups wait for each other; launch_nb also checks the
// runtime's occupancy answer).  GQ_RGEMM_ILC=0: the two-launch form everywhere.
bool rgemm_ilc(int fmt, const RGemmPlan &p)
{
    if (!p.ok || p.splits < 2 || tuning().rgemm_ilc == 0) return false;
    return (int64_t)p.tiles_m * p.tiles_n * p.splits <= (int64_t)num_cus() * rgemm_per_cu(fmt, p.nb);
}

bool sgemm_ilc(const RGemmPlan &p)
{
    if (!p.ok || p.splits < 2 || tuning().rgemm_ilc == 0) return false;
    return (int64_t)p.tiles_m * p.tiles_n * p.splits <= (int64_t)num_cus();
}

unsigned int ilc_timeouts()
{
    unsigned int v = 0;
    return hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ilc_timeouts), sizeof(v)) == hipSuccess ? v : ~0u;
}

RGemmPlan plan_sgemm(int64_t M, int64_t N, int64_t K, int splits)
{
    RGemmPlan p;
    if (M < 1 || N < 1 || K < 256 || K % 256 != 0) return p;
    p.nb = N > 64 ? 8 : (N > 32 ? 4 : (N > 16 ? 2 : 1));
    p.tiles_m = (int)((M + RBM - 1) / RBM);
    p.tiles_n = (int)((N + 16 * p.nb - 1) / (16 * p.nb));
    const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n, nsb = K / 256, cus = num_cus();
    // as many splits as keep the grid within one round of the chip (each at least one super-block)
    int64_t S = splits > 0 ? splits : (tiles >= cus ? 1 : cus / tiles);
    if (S > nsb) S = nsb;
    p.splits = (int)(S < 1 ? 1 : S);
    const int64_t nblk = tiles * p.splits;
    p.partial_bytes = p.splits > 1 ? ilc_flags_off(nblk, 16 * p.nb) + ilc_sync_bytes(nblk, tiles) : 0;
    p.ok = true;
    return p;
}

hipError_t launch_sgemm(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, void *partials, const RGemmPlan &p,
                        int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (!p.ok) return hipErrorInvalidValue;
#define GQ_SG_NB(F)                                                                                                       switch (p.nb) {                                                                                                       case 1: return launch_snb<F, 1>(A, X, C, partials, p, M, N, K, ldc, s);                                               case 2: return launch_snb<F, 2>(A, X, C, partials, p, M, N, K, ldc, s);                                               case 4: return launch_snb<F, 4>(A, X, C, partials, p, M, N, K, ldc, s);                                               case 8: return launch_snb<F, 8>(A, X, C, partials, p, M, N, K, ldc, s);                                               default: return hipErrorInvalidValue;                                                                                 }
    switch (fmt) {
    case Q8_0: GQ_SG_NB(Q8_0)
    case Q4_K: GQ_SG_NB(Q4_K)
    default: GQ_SG_NB(Q6_K)
    }
#undef GQ_SG_NB
}

SGroupPlan plan_sgemm_grouped(const SGroupItem *items, int n, int64_t N, int splits)
{
    SGroupPlan g;
    if (n < 1 || n > kMaxSParts || N < 1) return g;
    g.nb = N > 64 ? 8 : (N > 32 ? 4 : (N > 16 ? 2 : 1));
    const int tn = (int)((N + 16 * g.nb - 1) / (16 * g.nb));
    int64_t units = 0, Lmax = 1;
    for (int i = 0; i < n; ++i) {
        if (items[i].M < 1 || items[i].K < 256 || items[i].K % 256 != 0) return g;
        g.tiles_m[i] = (int)((items[i].M + RBM - 1) / RBM);
        const int64_t t = (int64_t)g.tiles_m[i] * tn, nsb = items[i].K / 256;
        units += t * nsb;
        Lmax = nsb > Lmax ? nsb : Lmax;
    }
    // the fewest super-blocks per workgroup L that keeps every part's (tiles x ceil(nsb / L))
    // grid within one round of the chip: the work spread evenly, the splits (partials) fewest.
    // More tiles than the chip holds (a 7B layer from ~200 tokens): not a grouped shape -- the
    // rounds' tails cost more than the launches saved (layer x256 317 vs 211 us per call,
    // profiles/r04/layer.txt)
    const int64_t cus = num_cus();
    int64_t tiles = 0;
    for (int i = 0; i < n; ++i) tiles += (int64_t)g.tiles_m[i] * tn;
    if (tiles > cus) return g;
    g.tiles_n = tn;
    const int sk = tuning().sgemm_streamk;
    if (splits <= 0 && sk != 0 && units < ((int64_t)1 << 30)) {
        // stream-K: the units (tile, super-block), part by part and tile by tile, split evenly
        // over one round of the chip -- every workgroup L or L+1 super-blocks, where whole-tile
        // splits leave the largest part's workgroups up to ceil(nsb / L) (a 7B layer at 128
        // tokens: 16 super-blocks on 198 workgroups vs 12-13 on 256).  The grouped default
        // (a 7B layer at 8 / 32 / 64 / 128 tokens: 64.1 / 67.2 / 80.6 / 102.1 us against 66.3
        // per call / 72.7 / 82.0 / 102.6 whole-tile splits: profiles/r04/ab9_layer.txt); single
        // matrices measured slower (GQ_SGEMM_STREAMK=1 forces it there, gq_capi.hip sgemm_streamk)
        // each unit weighted by its format -- its super-block's bytes (every unit alike, the round-4
        // split, was slower) -- the workgroups splitting the total cost: the
        // 7B layer at 40 / 64 / 128 tokens 77.2 / 78.8 / 100.9 -> 72.2 / 73.4 / 97.8 us
        // (profiles/r05/sgemm_grouped_cost_ab.txt; -55, the K-chunked stream's best, 74.6 / 76.1 / 99.2)
        int64_t ctot = 0;
        for (int i = 0; i < n; ++i) {
            g.cost[i] = items[i].fmt == Q8_0 ? 272 : (items[i].fmt == Q4_K ? 144 : 210);
            g.cstart[i] = (int)ctot;
            ctot += (int64_t)g.tiles_m[i] * tn * (items[i].K / 256) * g.cost[i];
        }
        if (ctot >= ((int64_t)1 << 30)) return g;
        // every workgroup's cost range at least the dearest unit, so that it holds a unit of each
        // tile it spans (no unwritten partial slot between a tile's first and last workgroup)
        int cmax = 1;
        for (int i = 0; i < n; ++i) cmax = g.cost[i] > cmax ? g.cost[i] : cmax;
        int64_t wmax = units < cus ? units : cus;
        if (wmax > ctot / cmax) wmax = ctot / cmax > 0 ? ctot / cmax : 1;
        const int W = (int)wmax, U = (int)ctot;
        auto owner = [&](int i, int64_t u) { // the workgroup holding unit u of part i
            const int64_t c = g.cstart[i] + (u - g.ustart[i]) * g.cost[i];
            return (int)(((c + 1) * W + U - 1) / U) - 1;
        };
        int64_t ust = 0;
        size_t pb = 0;
        for (int i = 0; i < n; ++i) {
            const int64_t nsb = items[i].K / 256, nt = (int64_t)g.tiles_m[i] * tn;
            g.ustart[i] = (int)ust;
            int cap = 1;
            for (int64_t t = 0; t < nt; ++t) {
                const int64_t t0 = ust + t * nsb, st = owner(i, t0 + nsb - 1) - owner(i, t0) + 1;
                cap = st > cap ? (int)st : cap;
            }
            g.scap[i] = cap;
            g.splits[i] = cap;
            g.poff[i] = pb;
            if (cap > 1) pb += ((size_t)cap * nt * (RBM * 16 * g.nb * 2 + RW * 4) + 255) & ~(size_t)255;
            ust += nt * nsb;
        }
        // the in-launch combine's flags [tile * scap + slot] and nonces [tile] of the split parts
        for (int i = 0; i < n; ++i) {
            if (g.scap[i] < 2) continue;
            const int64_t nt = (int64_t)g.tiles_m[i] * tn;
            g.foff[i] = pb;
            pb += (size_t)nt * g.scap[i] * 8;
            g.noff[i] = pb;
            pb = (pb + (size_t)nt * 4 + 255) & ~(size_t)255;
        }
        g.streamk = true;
        g.U = U;
        g.blocks = W;
        g.partial_bytes = pb;
        g.ok = true;
        return g;
    }
    int64_t L = (units + cus - 1) / cus;
    if (L < 1) L = 1;
    for (;; ++L) {
        int64_t wg = 0;
        for (int i = 0; i < n; ++i) wg += (int64_t)g.tiles_m[i] * tn * ((items[i].K / 256 + L - 1) / L);
        if (wg <= cus || L >= Lmax) break;
    }
    int64_t wg0 = 0;
    size_t pb = 0;
    for (int i = 0; i < n; ++i) {
        const int64_t nsb = items[i].K / 256;
        int64_t S = splits > 0 ? splits : (nsb + L - 1) / L;
        if (S > nsb) S = nsb;
        g.splits[i] = (int)S;
        g.wg0[i] = (int)wg0;
        wg0 += (int64_t)g.tiles_m[i] * tn * S;
        g.poff[i] = pb;
        if (S > 1) pb += ((size_t)S * g.tiles_m[i] * tn * (RBM * 16 * g.nb * 2 + RW * 4) + 255) & ~(size_t)255;
    }
    g.tiles_n = tn;
    g.blocks = (int)wg0;
    g.partial_bytes = pb;
    g.ok = true;
    return g;
}

hipError_t launch_sgemm_grouped(const SGroupItem *items, int n, int64_t N, const SGroupPlan &g, void *partials,
                                hipStream_t s)
{
    if (!g.ok) return hipErrorInvalidValue;
    SParts a{};
    RParts r{};
    a.n = n;
    a.N = N;
    a.spol = kSpol;
    a.full = tuning().sgemm_full > 0;
    a.streamk = r.streamk = g.streamk ? 1 : 0;
    static const int occ[4] = {grouped_occ<1>(), grouped_occ<2>(), grouped_occ<4>(), grouped_occ<8>()};
    const int oc = occ[g.nb == 1 ? 0 : (g.nb == 2 ? 1 : (g.nb == 4 ? 2 : 3))];
    a.ilc = g.streamk && tuning().rgemm_ilc != 0 && g.blocks <= num_cus() * oc ? 1 : 0;
    a.U = r.U = g.U;
    a.W = r.W = g.blocks;
    r.N = N;
    int rb = 0;
    constexpr int UPB = 256; // reduce: threads per workgroup
    for (int i = 0; i < n; ++i) {
        uint16_t *P = (uint16_t *)((uint8_t *)partials + g.poff[i]);
        a.p[i] = SPart{items[i].fmt, items[i].A, items[i].X, items[i].C, P, items[i].M, items[i].K, items[i].ldc,
                       g.tiles_m[i], g.tiles_n, g.splits[i], g.wg0[i], g.ustart[i], g.scap[i], g.cost[i], g.cstart[i],
                       (uint64_t *)((uint8_t *)partials + g.foff[i]), (uint32_t *)((uint8_t *)partials + g.noff[i])};
        if (g.splits[i] > 1 && !a.ilc) {
            const int tpu = g.nb == 1 ? 1 : 2, upt = RW * RRG * (g.nb / tpu) * 64, bpt = (upt + UPB - 1) / UPB;
            r.p[r.n++] = RPart{P,         items[i].C, items[i].M, items[i].ldc, g.tiles_m[i], g.tiles_n, g.splits[i], rb,
                               g.ustart[i], (int)(items[i].K / 256), g.scap[i], g.cost[i], g.cstart[i]};
            rb += g.tiles_m[i] * g.tiles_n * bpt;
        }
    }
#define GQ_SGG(NB_)                                                                                                       case NB_:                                                                                                                 sgemm_grouped_kernel<NB_><<<dim3((unsigned)g.blocks), dim3(64 * RW), 0, s>>>(a);                                        if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;                                                    if (r.n > 0) reduce_grouped_kernel<NB_><<<dim3((unsigned)rb), dim3(UPB), 0, s>>>(r);                                   return hipGetLastError();
    switch (g.nb) {
        GQ_SGG(1) GQ_SGG(2) GQ_SGG(4) GQ_SGG(8)
    default: return hipErrorInvalidValue;
    }
#undef GQ_SGG
}

hipError_t launch_rgemm(int fmt, int aq, const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, void *partials,
                        const RGemmPlan &p, int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (!p.ok) return hipErrorInvalidValue;
    if (aq != 0 && ldx % 8 != 0) return hipErrorInvalidValue; // 16-byte activation loads
#define GQ_RG_AQ(F)                                                                                                   \
    switch (aq) {                                                                                                     \
    case 0: return launch_f<F, 0>(A, X, ldx, C, partials, p, M, N, K, ldc, s);                                        \
    case 1: return launch_f<F, 1>(A, X, ldx, C, partials, p, M, N, K, ldc, s);                                        \
    default: return launch_f<F, 2>(A, X, ldx, C, partials, p, M, N, K, ldc, s);                                       \
    }
    switch (fmt) {
    case Q8_0: GQ_RG_AQ(Q8_0)
    case Q4_K: GQ_RG_AQ(Q4_K)
    default: GQ_RG_AQ(Q6_K)
    }
#undef GQ_RG_AQ
}

} // namespace gq

#ifdef GQ_RGEMM_STAMPS
extern "C" int gq_debug_rgemm_stamps(void *host, size_t bytes)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(gq::g_rstamps), bytes < sizeof(gq::g_rstamps) ? bytes : sizeof(gq::g_rstamps)) ==
                   hipSuccess ? 0 : 1;
}
#endif
