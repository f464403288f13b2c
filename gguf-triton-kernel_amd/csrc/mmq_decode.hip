// mmq_decode.hip -- the decode-shaped MMQ (N_tok <= 8): one launch that streams the weight
// matrix once from HBM at the stream rate.
//
// C[t][m] = sum_k W[m][k] * q8_1(x)[t][k] for the NT tokens of blockIdx.y, with the reference's
// per-block arithmetic (gguf_dot.hpp; kernels/cpu_impls/mmq_*_q8_1_cpu.py) and exact int32
// dot products.
//
// Weight stream.  Every wave owns a contiguous range of weight rows, i.e. a contiguous byte
// range of the packed tensor, cut into "tasks" of at most NI KiB: G whole rows when a row fits,
// else a row segment of whole 64-element units.  A task is moved HBM -> LDS by NI LDS-DMA
// instructions (buffer_load_dwordx4 ... lds: one 1 KiB fully coalesced line run per wave
// instruction, nothing through VGPRs) from the 16-byte aligned window around it, into the
// wave's private ring of S slots; S-1 tasks are in flight while one is multiplied.  The ring is
// private, so a wave waits only on its own counted vmcnt -- no workgroup barrier in the loop.
//
// Activations.  The NT tokens are quantized to q8_1 (gguf_q8_1.hpp, bit-exact with
// utils/quantize/q8_1.py) straight into LDS: the fp16 values are loaded into registers (one
// 16-byte load per lane, four lanes per 32-element block) ahead of the first weight DMA,
// quantized by 4-lane DPP groups, written to LDS, and shared by one raw barrier (the second
// ring slot's task is issued before it).  The C ABI routes N <= 4 tokens here (kGemvMaxTokens).
//
// Multiply.  Lane l takes unit u = l % P + P*i of a row (P = 64, or the power of two >= the
// units per row for short rows, several rows per wave pass); it reads the unit's packed bytes
// and its activation block pair from LDS, dots them with v_dot4_i32_i8, and P-lane xor
// shuffles reduce the row.
#include <cstdlib>

#include "gguf_blocks.hpp"
#include "gguf_dot.hpp"
#include "gguf_internal.hpp"
#include "gguf_q8_1.hpp"
#include "gguf_units.hpp"

#ifndef GQ_DECODE_NT
#define GQ_DECODE_NT 1 // weight DMAs with the non-temporal policy (bytes read exactly once)
#endif

namespace gq {

#ifdef GQ_DECODE_STAMPS // diagnostic build: per-wave s_memtime breakdown (never the product)
__device__ unsigned long long g_dstamps[65536][13];
#endif

namespace {

typedef __attribute__((address_space(3))) void lds_void;

#ifndef GQ_DECODE_DW
#define GQ_DECODE_DW 8
#endif
constexpr int DW = GQ_DECODE_DW; // waves per workgroup (two per SIMD)
// (issue priority between a SIMD's two waves -- waves 4-7 lose by age and are every workgroup's
// slowest -- balanced by a swap at the middle of the task list, or favouring waves 4-7 until the
// activation barrier or throughout: the steps move -2.4..+1.6%, the stream sets the time;
// profiles/r06/decode_prio_ab.txt, decode_prio4_ab.txt.  Not kept.)
#ifndef GQ_DECODE_NI
#define GQ_DECODE_NI 7
#endif
#ifndef GQ_DECODE_NS
#define GQ_DECODE_NS 2
#endif
constexpr int NI = GQ_DECODE_NI; // KiB (DMA instructions) per task
constexpr int NS = GQ_DECODE_NS; // ring slots per wave: NS-1 tasks in flight while one is multiplied
constexpr int SLOT = NI * 1024;
constexpr int RING = DW * NS * SLOT;
constexpr int LDS_CAP = 160 * 1024;
// units (64 weights) per lane work item: Q6_K lanes take whole super-block halves (up to two
// tokens: with four, two units' activations at once exceed the register file)
template <int F, int NT> constexpr int UPC_OF = F == Q6_K && NT <= 2 ? 2 : 1;
int upc_of(int fmt, int nt) { return fmt == Q6_K && nt <= 2 ? 2 : 1; }

// Q6_K tasks land in the ring as an aligned image: every 210-byte super-block (2-byte aligned
// in the tensor) becomes 224 bytes -- 13 pieces from its first byte (0..207) and one from byte
// 194 (d at image byte 222) -- so the lanes' ql/qh/scale/d reads are naturally aligned LDS reads
// (read from the packed bytes, ~90% of the kernel's LDS cycles were unaligned-access stalls).
// Each lane's DMA source is per piece (2-byte aligned); a K = 8192 row is exactly 7 KiB.
// Both rings give the same bits, so the choice is by speed alone (profiles/r03/q6_img_ab.log, us
// packed -> image): K <= 4096 at every token count (4096^2 x1 7.1 -> 5.9, 11008x4096 x1/x4
// 12.6 -> 11.4 / 17.3 -> 15.1); longer rows at 2-4 tokens (4096x11008 x2/x4 18.9 -> 17.3 /
// 34.9 -> 32.3) except whole 7 KiB rows (K a multiple of 8192: 28672x8192 x2 39.4 -> 41.1),
// where the packed ring's aligned 16-byte windows stream faster than per-piece misaligned
// sources -- as at one token (4096x11008 12.2 -> 13.1, 28672x8192 36.8 -> 37.3).
// GQ_DECODE_Q6_IMG=0/1 forces it.
constexpr int kImgSB = 224;
bool img_of(int fmt, int64_t K, int nt)
{
    if (fmt != Q6_K) return false;
    if (tuning().decode_q6_img >= 0) return tuning().decode_q6_img == 1;
    return K <= 4096 || (nt >= 2 && K % 8192 != 0);
}

struct DecodeGeom {
    int ngroups; // row groups (nseg == 1) or rows (nseg > 1)
    int G;       // rows per group (nseg == 1)
    int nseg;    // segments per row
    int segu;    // units per segment (nseg > 1; a multiple of 64)
    int lp2;     // log2(P): lanes per row
    int early;   // ring slots 1.. issued: 0 after the quantization, 1 once the activations
                 // arrived (under the quantization), 2 with task 0 (ahead of the arrival)
};

// byte offset of unit u (64 elements) within a row
template <int F>
__device__ __forceinline__ uint32_t unit_byte(int u, int nb32)
{
    if constexpr (F == Q8_0) return 34u * (uint32_t)(2 * u < nb32 ? 2 * u : nb32);
    return (uint32_t)Layout<F>::BYTES * (uint32_t)(u >> 2);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint8_t *lds, uint32_t voff)
{
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)lds, 16, voff, 0, 0, GQ_DECODE_NT ? 2 : 0);
}
__device__ __forceinline__ void dma16x(__amdgpu_buffer_rsrc_t r, uint8_t *lds, uint32_t voff)
{
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)lds, 16, voff, 0, 0, 0);
}

#define GQ_DPP(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xf, 0xf, false))
#define GQ_DPPI(v, ctrl) __builtin_amdgcn_mov_dpp(v, ctrl, 0xf, 0xf, false)
__device__ __forceinline__ float wave_sum_dpp(float v)
{
    v += GQ_DPP(v, 0xb1);  // quad_perm [1,0,3,2]
    v += GQ_DPP(v, 0x4e);  // quad_perm [2,3,0,1]
    v += GQ_DPP(v, 0x124); // row_ror:4
    v += GQ_DPP(v, 0x128); // row_ror:8
    const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    const float b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
    const float c = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
    const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
    return (a + b) + (c + d);
}

// The unit's activations for NT tokens from the LDS image (codes swizzled as swz_piece<F>;
// d, Q4_K s and Q6_K per-16 code sums precomputed by the quantizer).
template <int F, int NT>
__device__ __forceinline__ void act_from_lds(Act<F, NT> &a, const uint8_t *codes, const float *sd, const float *sx,
                                             int kp, int nb, int u)
{
    int b0, b1;
    act_blocks<F>(u, b0, b1);
    const bool has1 = b1 < nb;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const uint8_t *row = codes + t * kp;
        const u32x4 c0 = *(const u32x4 *)(row + 16 * swz_piece<F>(2 * b0));
        const u32x4 c1 = *(const u32x4 *)(row + 16 * swz_piece<F>(2 * b0 + 1));
        u32x4 c2 = {0, 0, 0, 0}, c3 = {0, 0, 0, 0};
        if (has1) {
            c2 = *(const u32x4 *)(row + 16 * swz_piece<F>(2 * b1));
            c3 = *(const u32x4 *)(row + 16 * swz_piece<F>(2 * b1 + 1));
        }
        a.q[t][0] = c0.x; a.q[t][1] = c0.y; a.q[t][2] = c0.z; a.q[t][3] = c0.w;
        a.q[t][4] = c1.x; a.q[t][5] = c1.y; a.q[t][6] = c1.z; a.q[t][7] = c1.w;
        a.q[t][8] = c2.x; a.q[t][9] = c2.y; a.q[t][10] = c2.z; a.q[t][11] = c2.w;
        a.q[t][12] = c3.x; a.q[t][13] = c3.y; a.q[t][14] = c3.z; a.q[t][15] = c3.w;
        a.d[t][0] = sd[t * nb + b0];
        a.d[t][1] = has1 ? sd[t * nb + b1] : 0.f;
        if constexpr (F == Q4_K) {
            a.s[t][0] = sx[t * nb + b0];
            a.s[t][1] = has1 ? sx[t * nb + b1] : 0.f;
        }
        if constexpr (F == Q6_K) { // int32 code sums of the 16-element halves: [t][2*b + h]
            const int *sm = (const int *)sx + t * 2 * nb;
            const u32x2 s0 = *(const u32x2 *)(sm + 2 * b0);
            const u32x2 s1 = has1 ? *(const u32x2 *)(sm + 2 * b1) : (u32x2){0, 0};
            a.sum[t][0] = (int)s0.x; a.sum[t][1] = (int)s0.y;
            a.sum[t][2] = (int)s1.x; a.sum[t][3] = (int)s1.y;
        }
    }
}

// ITC > 0: the lane's activations for its units u = (lane % P) + P*i, i < ITC, are loaded from
// the LDS image once and kept in registers (every row multiplies the same units); ITC == 0:
// read from LDS per unit.
// The kernel body for one matrix: workgroup bx of gx over the matrix's row groups, token group by
// (stream_decode_kernel: the grid itself; stream_decode_grouped_kernel: a slice of a grid shared
// by several matrices).  A row's arithmetic depends on F, NT and K only -- not on bx, gx or the
// geometry's rows per task -- so a matrix computed inside a group gives the same bits as alone.
// FP8 = 1: the fp8 activation variant -- the prologue quantizes x per 32-block to e4m3 codes
// and widens them back (gguf_q8_1.hpp f8_quad: the bytes act_quant's F8DEQ form writes), the
// LDS image is fp16 x~ + the x~ sums of every 16-element quarter, and the units multiply by
// v_dot2_f32_f16 (gguf_dot.hpp dot_unit_h); no register cache of activations (ITC = 0).
template <int F, int NT, int ITC, int IM = 0, int FP8 = 0>
__device__ __forceinline__ void decode_body(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X, int64_t ldx,
                                            uint16_t *__restrict__ C, int M, int64_t N, int K, int64_t ldc,
                                            DecodeGeom geo, int bx, int gx, int by, uint8_t *smem)
{
    using L = Layout<F>;
    constexpr int UPC = UPC_OF<F, NT>;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef GQ_DECODE_STAMPS
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    unsigned long long t_wait = 0, t_w0 = 0, t_c0 = 0;
#endif
    const int64_t tok0 = (int64_t)by * NT;
    const int nb = K / 32;
    const int kp = (K + 63) / 64 * 64;
    const uint32_t RB = (uint32_t)(K / L::QK) * L::BYTES;
    const int upr = (K + 63) / 64;
    const int cpr = upr / UPC; // lane chunks per row
    uint8_t *ring = smem + wave * (NS * SLOT);
    uint8_t *codes = smem + RING;
    float *sd = (float *)(codes + NT * kp * (FP8 ? 2 : 1)); // FP8: quarter sums [NT][2*nb]
    float *sx = sd + NT * nb; // Q4_K: s [NT][nb] (float); Q6_K: code sums [NT][2*nb] (int)
    static_assert(!FP8 || NT == 1 || ITC == 0, "fp8 decode: cached activations at one token only");
    // FP8 at 2+ tokens: exact code pairs, no quarter sums (gguf_dot.hpp dot_unit_h NS; act_lds)
    constexpr bool F8NS = FP8 && NT >= 2;
    // FP8: x~ 16-byte piece P of a token row at piece P ^ ((P >> 4) & 7) (the lanes of a unit
    // read hit distinct banks)
    auto xpiece = [](int P) { return P ^ ((P >> 4) & 7); };

    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, 0, (int)(((uint32_t)M * RB + 15u) & ~15u), 0x00020000);
    constexpr bool IMG = F == Q6_K && IM != 0;
    const uint32_t RBI = IMG ? (uint32_t)(K / 256) * kImgSB : RB; // ring bytes per row
    // IMG: the source offset, from the task's first byte, of the piece this lane moves in DMA
    // instruction k (piece p = 64k + lane: super-block p / 14, piece p % 14)
    uint32_t rel[IMG ? NI : 1];
    if constexpr (IMG) {
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const uint32_t p = 64u * k + (uint32_t)lane, sb = p / 14u, pc = p - 14u * sb;
            rel[k] = 210u * sb + (pc < 13u ? 16u * pc : 194u);
        }
    }

    // this wave's contiguous range of row groups, and its task count
    const int W = gx * DW;
    const int gw = bx * DW + wave;
    const int per = geo.ngroups / W, rem = geo.ngroups % W;
    const int g_begin = gw * per + (gw < rem ? gw : rem);
    const int ntask = (per + (gw < rem ? 1 : 0)) * geo.nseg;

    // task = (row group g, segment s); cursors advance without divisions
    auto window = [&](int g, int s, uint32_t &start, uint32_t &len) {
        if (geo.nseg == 1) {
            const int r0 = g * geo.G;
            const int rows = M - r0 < geo.G ? M - r0 : geo.G;
            start = (uint32_t)r0 * RB;
            len = (uint32_t)rows * RB;
        } else {
            const int u0 = s * geo.segu;
            const int u1 = u0 + geo.segu < upr ? u0 + geo.segu : upr;
            start = (uint32_t)g * RB + unit_byte<F>(u0, nb);
            len = unit_byte<F>(u1, nb) - unit_byte<F>(u0, nb);
        }
    };
    auto next = [&](int &g, int &s) {
        if (++s == geo.nseg) {
            s = 0;
            ++g;
        }
    };
    int gi = g_begin, si = 0; // next task to issue
    auto issue = [&](int j) {
        uint32_t st, len;
        window(gi, si, st, len);
        next(gi, si);
        const uint32_t ws = st & ~15u, we = st + len;
        uint8_t *dst = ring + (j % NS) * SLOT;
        const bool real = j < ntask;
        if constexpr (IMG) {
#pragma unroll
            for (int k = 0; k < NI; ++k) // pieces past the task re-read its first bytes (L2 hit)
                dma16(wrs, dst + 1024 * k, real ? st + (rel[k] < len ? rel[k] : 0u) : 0x80000000u);
            return;
        }
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            uint32_t o = ws + 1024u * k + 16u * lane;
            if (o >= we) o = ws; // past the window: re-read its first line (L2 hit), never past the tensor
            // no task: an offset past the buffer's range (>= 2^31) -- zeros, no memory access
            dma16(wrs, dst + 1024 * k, real ? o : 0x80000000u);
        }
    };

    // ---- prologue: the fp16 activations into registers, then a task into every ring slot ----
    // Activation blocks (32 elements of one token) are dealt to waves round-robin, 16 per pass
    // (4 lanes per block, 8 elements = one 16-byte load per lane), up to XP passes per round.
    // 4 passes (one round) cover K <= 16384 at one token; the instantiations that cache 5+
    // units per lane (K > 16384) take 8 -- more than needed costs redundant loads elsewhere
    constexpr int XP = ITC * UPC >= 5 ? 8 : 4;
    const int xblocks = NT * nb;
    const int xrounds = (xblocks + DW * 16 * XP - 1) / (DW * 16 * XP);
    auto xblock = [&](int r, int pass) { return ((r * XP + pass) * 16 + (lane >> 2)) * DW + wave; };
    auto tok_split = [&](int b, int &t, int &j) { // b = t * nb + j without an integer division
        t = 0;
        j = b;
#pragma unroll
        for (int i = 1; i < NT; ++i)
            if (j >= nb) {
                j -= nb;
                ++t;
            }
    };
    auto npass = [&](int r) { // passes of round r with a block for some lane group of this wave
        const int left = xblocks - (r * XP * 16) * DW - wave;
        const int n = left > 0 ? (left + 16 * DW - 1) / (16 * DW) : 0;
        return n < XP ? n : XP;
    };
    // unconditional (clamped) loads: a load under a branch leaves a phi copy behind it that
    // the compiler waits for (vmcnt(0)) right away, serializing the passes
    auto load_x = [&](int r, u32x4 (&xv)[XP]) {
#pragma unroll
        for (int q = 0; q < XP; ++q) {
            int b = xblock(r, q);
            if (b >= xblocks) b = 0;
            int t, j;
            tok_split(b, t, j);
            const int64_t tok = tok0 + t < N ? tok0 + t : N - 1;
            xv[q] = ld16(X + tok * ldx + 32 * j + 8 * (lane & 3));
        }
    };
    auto store_q = [&](int b, const Q81Quad &qq) {
        int t, j;
        tok_split(b, t, j);
        const int k = 32 * j + 8 * (lane & 3);
        *(u32x2 *)(codes + t * kp + 16 * swz_piece<F>(k >> 4) + (k & 15)) = (u32x2){qq.codes[0], qq.codes[1]};
        if constexpr (F == Q6_K)
            if ((lane & 1) == 0) ((int *)sx)[t * 2 * nb + 2 * j + ((lane >> 1) & 1)] = qq.s4;
        if ((lane & 3) == 0) {
            sd[t * nb + j] = qq.d;
            if constexpr (F == Q4_K) sx[t * nb + j] = h2f(qq.sbits);
        }
    };
    auto store_f = [&](int b, const F8Quad &f, float ls) { // FP8: x~ and the lane pair's quarter sum
        int t, j;
        tok_split(b, t, j);
        const int P = 4 * j + (lane & 3); // 16-byte piece of the token row
        *(u32x4 *)(codes + 2 * t * kp + 16 * xpiece(P)) = (u32x4){f.xt[0], f.xt[1], f.xt[2], f.xt[3]};
        if constexpr (F8NS) { // (Q4_K: the block's sum, two quarters; Q8_0 / Q6_K: no sums)
            if constexpr (F == Q4_K)
                if ((lane & 3) == 0) sd[t * nb + j] = ls;
        } else {
            if ((lane & 1) == 0) sd[t * 2 * nb + 2 * j + ((lane >> 1) & 1)] = ls;
        }
    };
    auto quantize = [&](int r, const u32x4 (&xv)[XP]) {
        const int np = npass(r);
#pragma unroll
        for (int q = 0; q < XP; ++q) {
            if (q < np) { // every lane of the wave computes (DPP groups); stores only real blocks
                const int b = xblock(r, q);
                if constexpr (FP8) {
                    const F8Quad f = f8_quad(xv[q]);
                    float ls = 0.f; // the lane's 8 x~ in fp32, then + the pair lane's (a quarter)
#pragma unroll
                    for (int i = 0; i < 4; ++i) ls += h2f(f.xt[i] & 0xffffu) + h2f(f.xt[i] >> 16);
                    ls += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, ls), 0xb1, 0xf, 0xf, false));
                    if constexpr (F8NS && F == Q4_K) // + the other lane pair's quarter: the 32-block's sum
                        ls += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, ls), 0x4e, 0xf, 0xf, false));
                    if (b < xblocks) store_f(b, f, ls);
                } else {
                    const Q81Quad qq = q8_1_quad(xv[q]);
                    if (b < xblocks) store_q(b, qq);
                }
            }
        }
        // consume every activation register on every path: a load the compiler sees as possibly
        // unconsumed makes it wait vmcnt(0) -- all weight DMAs -- before reusing its register
#pragma unroll
        for (int q = 0; q < XP; ++q) asm volatile("" ::"v"(xv[q].x), "v"(xv[q].y), "v"(xv[q].z), "v"(xv[q].w));
    };

    u32x4 xv[XP];
    load_x(0, xv);
    // Task 0 goes out with the activation loads; by default (early = 0) the rest of the ring
    // once the activations are quantized (issued together, they queue the activations behind
    // twice the weight traffic, and a small matrix waits on exactly that latency); long rows
    // (early = 1, 2) refill under the quantization instead.  Task 0 always issues (past the
    // wave's tasks: an offset beyond the buffer -- zeros, no memory access), so the wait below
    // for the activations, the older loads, is a fixed vmcnt.
#ifndef GQ_DECODE_XFIRST // (diagnostic build -DGQ_DECODE_XFIRST: task 0 only once the activations arrived)
    issue(0);
#endif
    auto issue_rest = [&]() {
#pragma unroll
        for (int j = 1; j < NS; ++j)
            if (j < ntask) issue(j);
    };
    if (geo.early == 2) issue_rest();
#pragma unroll
    for (int q = 0; q < XP; ++q) asm volatile("" ::"v"(xv[q].x), "v"(xv[q].y), "v"(xv[q].z), "v"(xv[q].w)); // waits for the x loads
#ifdef GQ_DECODE_XFIRST
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    issue(0);
#endif
#ifdef GQ_DECODE_STAMPS
    const unsigned long long t_xw = __builtin_amdgcn_s_memtime();
#endif
    if (geo.early == 1) issue_rest();
    quantize(0, xv);
    for (int r = 1; r < xrounds; ++r) { // long activations: further rounds (their loads wait behind the DMAs)
        u32x4 xr[XP];
        load_x(r, xr);
        quantize(r, xr);
    }
    if (geo.early == 0) issue_rest();
    int issued = NS < ntask ? NS : ntask;
    int gc = g_begin, sc = 0; // task being multiplied
#ifdef GQ_DECODE_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t_q = __builtin_amdgcn_s_memtime();
#endif
    // raw barrier: __syncthreads() would also wait vmcnt(0), draining the weight DMAs in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef GQ_DECODE_STAMPS
    const unsigned long long t_pro = __builtin_amdgcn_s_memtime();
#endif

    // ---- main loop ----
    const int P = 1 << geo.lp2;
    const int lrow = lane >> geo.lp2, lunit = lane & (P - 1);
    const int ntok = N - tok0 < NT ? (int)(N - tok0) : NT;
    Act<F, NT> ca[ITC > 0 && !FP8 ? ITC * UPC : 1];
    if constexpr (ITC > 0 && !FP8) {
#pragma unroll
        for (int i = 0; i < ITC; ++i) {
            const int c = lunit + P * i < cpr ? lunit + P * i : cpr - 1;
#pragma unroll
            for (int e = 0; e < UPC; ++e) act_from_lds<F, NT>(ca[UPC * i + e], codes, sd, sx, kp, nb, UPC * c + e);
        }
    }
    float acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = 0.f;

    // FP8: the unit's x~ (two 32-element runs: Q6_K A and B, else elements 64u..64u+63) and quarter sums
    auto act_h = [&](ActH<NT> &a, int u) {
        int e0, e1;
        if constexpr (F == Q6_K) {
            e0 = 256 * (u >> 2) + 128 * ((u >> 1) & 1) + 32 * (u & 1);
            e1 = e0 + 64;
        } else {
            e0 = 64 * u;
            e1 = e0 + 32;
        }
        const bool has1 = F != Q8_0 || 2 * u + 1 < nb; // (Q8_0, K % 64 == 32: no second block)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
#pragma unroll
            for (int rr = 0; rr < 2; ++rr)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    u32x4 v = *(const u32x4 *)(codes + 2 * t * kp + 16 * xpiece(((rr ? e1 : e0) >> 3) + i));
                    if (rr && !has1) v = (u32x4){0, 0, 0, 0};
                    a.x[t][16 * rr + 4 * i] = v.x;
                    a.x[t][16 * rr + 4 * i + 1] = v.y;
                    a.x[t][16 * rr + 4 * i + 2] = v.z;
                    a.x[t][16 * rr + 4 * i + 3] = v.w;
                }
            if constexpr (F8NS) {
                if constexpr (F == Q4_K) { // the two 32-blocks' sums
                    a.s[t][0] = sd[t * nb + (e0 >> 5)];
                    a.s[t][2] = sd[t * nb + (e1 >> 5)];
                }
                continue;
            }
            const float *sq = sd + t * 2 * nb;
            a.s[t][0] = sq[e0 >> 4];
            a.s[t][1] = sq[(e0 >> 4) + 1];
            a.s[t][2] = has1 ? sq[e1 >> 4] : 0.f;
            a.s[t][3] = has1 ? sq[(e1 >> 4) + 1] : 0.f;
        }
    };
    // FP8, ITC > 0 (one token): the lane's units' x~ (32 words each) kept in registers across
    // its rows, as the int8 form's Act cache -- no LDS reads in the row loop
    ActH<NT> ch[FP8 && ITC > 0 ? ITC * UPC : 1];
    if constexpr (FP8 && ITC > 0) {
#pragma unroll
        for (int i = 0; i < ITC; ++i) {
            const int c = lunit + P * i < cpr ? lunit + P * i : cpr - 1;
#pragma unroll
            for (int e = 0; e < UPC; ++e) act_h(ch[UPC * i + e], UPC * c + e);
        }
    }
    // the contribution of unit u (activation slot i when cached) of the row at rowp
    auto unit = [&](const UnitLoad<F> &l, int u, int i, float (&acc)[NT]) {
        if constexpr (FP8 && ITC > 0) {
            dot_unit_h<F, NT, F8NS>(UnitRaw<F>::from(l, u, nb), ch[i], acc);
        } else if constexpr (FP8) {
            ActH<NT> a;
            act_h(a, u);
            dot_unit_h<F, NT, F8NS>(UnitRaw<F>::from(l, u, nb), a, acc);
        } else if constexpr (ITC > 0) {
            dot_unit<F, NT>(UnitRaw<F>::from(l, u, nb), ca[i], acc);
        } else {
            Act<F, NT> a;
            act_from_lds<F, NT>(a, codes, sd, sx, kp, nb, u);
            dot_unit<F, NT>(UnitRaw<F>::from(l, u, nb), a, acc);
        }
    };
    // lane chunk c of the row at rowp (activation slots UPC*i.. when cached).  Q6_K: the half
    // super-block c -- units 2c (v = 0) and 2c+1 (v = 1) share its qh, scale and d bytes, so
    // they are read once (8 LDS reads per 128 weights instead of 12) and the unit's shifts
    // are compile-time constants
    auto chunk = [&](const uint8_t *rowp, int c, int i, float (&acc)[NT]) {
        if constexpr (UPC == 2) {
            // (the shared fields' loads are merged by the compiler; written as two unit loads
            // because direct reads here made the waitcnt pass add a vmcnt(0) before them, i.e.
            // wait for the task DMA just issued -- tools/check_waits.py)
            UnitLoad<Q6_K> l0, l1;
            // (IMG = 0: plain 2-byte aligned reads; the dword-aligned form, UnitLoad::load_lds,
            // cut the unaligned-LDS stalls but measured 7-10% slower -- profiles/r02/decode_lds_align_ab.txt)
            if constexpr (IMG) {
                l0.load_img(rowp, 2 * c);
                l1.load_img(rowp, 2 * c + 1);
            } else {
                l0.load(rowp, 2 * c, nb);
                l1.load(rowp, 2 * c + 1, nb);
            }
            unit(l0, 2 * c, 2 * i, acc);
            unit(l1, 2 * c + 1, 2 * i + 1, acc);
            return;
        }
        const int u = c;
        UnitLoad<F> l;
#ifdef GQ_ABL_NOWLDS
        __builtin_memset(&l, 0, sizeof(l));
        ((uint32_t *)&l)[0] = (uint32_t)(uintptr_t)rowp + u;
        ((uint32_t *)&l)[3] = (uint32_t)u * 77u;
#else
        // Q8_0: dword-aligned reads and a 2-byte shift (4096^2 decode 6.6 -> 5.6 us); Q4_K
        // blocks are 16-byte aligned in the ring; Q6_K: see above
        if constexpr (F == Q8_0) l.load_lds(rowp, u, nb);
        else if constexpr (IMG) l.load_img(rowp, u);
        else l.load(rowp, u, nb);
#endif
#ifdef GQ_ABL_NODOT
        const uint32_t *w = (const uint32_t *)&l;
        uint32_t x = 0;
        for (int q = 0; q < (int)(sizeof(l) / 4); ++q) x ^= w[q];
        acc[0] += (float)x;
        return;
#endif
        unit(l, u, i, acc);
    };

    for (int j = 0; j < ntask; ++j) {
#ifdef GQ_DECODE_STAMPS
        const unsigned long long ta = __builtin_amdgcn_s_memtime();
#endif
        // slot (j - 1) % NS was freed by the previous multiply: refill it, then wait for task j
        // with the tasks issued after it still in flight (counted vmcnt; stores only add to it)
        if (j > 0 && issued < ntask) {
            issue(issued);
            ++issued;
        }
        const int ahead = issued - j - 1;
        static_assert(NS >= 2 && NS <= 4, "ring depth");
        if (ahead >= NS - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1) * NI) : "memory");
        else if (NS > 2 && ahead == NS - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS > 2 ? NS - 2 : 0) * NI) : "memory");
        else if (NS > 3 && ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef GQ_DECODE_STAMPS
        t_wait += __builtin_amdgcn_s_memtime() - ta;
        if (j == 0) t_w0 = __builtin_amdgcn_s_memtime();
        if (j == 1) t_c0 = ta;
#endif

        uint32_t st, len;
        const int g = gc, s = sc;
        window(g, s, st, len);
        next(gc, sc);
        const uint8_t *base = ring + (j % NS) * SLOT + (IMG ? 0u : (st & 15u));
#ifdef GQ_ABL_NOCOMP
        acc[0] += (float)base[lane];
        if (j == ntask - 1 && acc[0] == 1234.5f) C[0] = 0;
        continue;
#endif
        if (geo.nseg == 1) {
            const int r0 = g * geo.G;
            const int nr = M - r0 < geo.G ? M - r0 : geo.G;
            // row pass rp: lane row rp + lrow into a[]; out: reduce over the P lanes and store
            auto pass = [&](int rp, float (&a)[NT]) {
                const int r = rp + lrow;
                const bool valid = r < nr;
                const uint8_t *rowp = base + (uint32_t)(valid ? r : 0) * RBI;
                if constexpr (ITC > 0) {
#pragma unroll
                    for (int i = 0; i < ITC; ++i) {
                        const int c = lunit + P * i;
                        if (valid && c < cpr) chunk(rowp, c, i, a);
                    }
                } else {
                    for (int c = lunit; c < cpr; c += P)
                        if (valid) chunk(rowp, c, 0, a);
                }
            };
            auto out = [&](int rp, float (&a)[NT]) {
                const int r = rp + lrow;
                if (P == 64) {
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        const float v = wave_sum_dpp(a[t]);
                        a[t] = 0.f;
                        if (lane == 0 && t < ntok) C[(tok0 + t) * ldc + r0 + r] = f2h_bits(v);
                    }
                } else {
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        float v = a[t];
                        for (int off = P >> 1; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
                        a[t] = 0.f;
                        if (lunit == 0 && r < nr && t < ntok) C[(tok0 + t) * ldc + r0 + r] = f2h_bits(v);
                    }
                }
            };
            const int RS = 64 >> geo.lp2; // rows per pass
            int rp = 0;
            for (; rp < nr; rp += RS) {
                pass(rp, acc);
                out(rp, acc);
            }
        } else {
            const int u0 = s * geo.segu, c0 = u0 / UPC, c1 = c0 + geo.segu / UPC;
            const uint8_t *rowp = base - (IMG ? (uint32_t)kImgSB * (uint32_t)(u0 >> 2) : unit_byte<F>(u0, nb));
            if constexpr (ITC > 0) {
#pragma unroll
                for (int i = 0; i < ITC; ++i) {
                    const int c = lane + 64 * i;
                    if (c >= c0 && c < c1 && c < cpr) chunk(rowp, c, i, acc);
                }
            } else {
                for (int c = c0 + lane; c < c1; c += 64)
                    if (c < cpr) chunk(rowp, c, 0, acc);
            }
            if (s == geo.nseg - 1) {
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const float v = wave_sum_dpp(acc[t]);
                    acc[t] = 0.f;
                    if (lane == 0 && t < ntok) C[(tok0 + t) * ldc + g] = f2h_bits(v);
                }
            }
        }
    }
    // no DMA may land after the wave exits: every issued task was waited for in the loop, so
    // only a wave without tasks (its task-0 DMA is never waited for) has one in flight; the
    // output stores need no wait
    if (ntask == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef GQ_DECODE_STAMPS
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    const int gw_id = bx * DW + wave;
    if (lane == 0 && gw_id < 65536 && by == 0) {
        g_dstamps[gw_id][0] = t_pro - t_start;
        g_dstamps[gw_id][1] = t_wait;
        g_dstamps[gw_id][2] = t_end - t_pro;
        g_dstamps[gw_id][3] = (unsigned long long)ntask;
        g_dstamps[gw_id][4] = t_xw - t_start;
        g_dstamps[gw_id][5] = t_q - t_start;
        g_dstamps[gw_id][6] = t_start;
        g_dstamps[gw_id][7] = t_end;
        g_dstamps[gw_id][8] = t_w0;
        g_dstamps[gw_id][9] = t_c0 ? t_c0 : t_end;
        g_dstamps[gw_id][10] = t_pro;
        g_dstamps[gw_id][11] = (unsigned long long)bx;
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_dstamps[gw_id][12] = xcc & 0xfu;
    }
#endif
}

template <int F, int NT, int ITC, int IM, int FP8>
__global__ __launch_bounds__(DW * 64) void stream_decode_kernel(const uint8_t *__restrict__ A,
                                                                const uint16_t *__restrict__ X, int64_t ldx,
                                                                uint16_t *__restrict__ C, int M, int64_t N, int K,
                                                                int64_t ldc, DecodeGeom geo)
{
    extern __shared__ __attribute__((aligned(1024))) uint8_t smem[];
    decode_body<F, NT, ITC, IM, FP8>(A, X, ldx, C, M, N, K, ldc, geo, (int)blockIdx.x, (int)gridDim.x, (int)blockIdx.y, smem);
}

struct Pick {
    int nt, itc;
    bool img = false;       // Q6_K: the aligned ring image (kImgSB)
    bool fp8 = false;       // the fp8 activation variant (decode_body FP8; set before pick())
    bool lds_split = false; // fewer tokens per workgroup than wanted: the activations do not fit LDS
    size_t lds;
    DecodeGeom geo;
    int grid;
};

size_t act_lds(int fmt, int nt, int64_t K, bool fp8 = false)
{
    const int64_t kp = (K + 63) / 64 * 64, nb = K / 32;
    if (fp8) // x~ + quarter sums (2+ tokens: Q4_K's block sums only, gguf_dot.hpp dot_unit_h NS)
        return (size_t)nt * kp * 2 + (nt == 1 ? (size_t)nt * nb * 2 * 4 : (fmt == Q4_K ? (size_t)nt * nb * 4 : 0));
    return (size_t)nt * kp + (size_t)nt * nb * 4 * (fmt == Q8_0 ? 1 : (fmt == Q4_K ? 2 : 3));
}

// the largest cached-chunk count ITC instantiated for (format, token tile); the fp8 form caches
// at one token only, at most two units (64 VGPRs of x~ pairs)
int fp8_itc_max(int fmt, int nt) { return nt == 1 ? (fmt == Q6_K ? 1 : 2) : 0; }
int itc_max(int fmt, int nt)
{
    if (nt == 1) return fmt == Q6_K ? 4 : 7;
    if (nt == 2) return fmt == Q6_K ? 1 : 4;
    return 1;
}

int64_t row_bytes(int fmt, int64_t K)
{
    return fmt == Q8_0 ? K / 32 * 34 : (fmt == Q4_K ? K / 256 * 144 : K / 256 * 210);
}

// wgs: the workgroups the matrix gets (0: a launch of its own, the whole chip; a grouped launch
// splits the chip's workgroups by weight bytes)
bool pick(int fmt, int64_t M, int64_t N, int64_t K, Pick &p, int wgs = 0)
{
    // at most 4 tokens per workgroup (NT = 8 spills registers); N = 5..8 runs two token groups,
    // whose second pass over the weights is served largely by the Infinity Cache
    const int nts[3] = {1, 2, 4};
    p.nt = 4;
    for (int i = 0; i < 3; ++i)
        if (nts[i] >= N) { p.nt = nts[i]; break; }
    // Q6_K at 3-4 tokens with K >= 8192: two 2-token groups (super-block-half lanes; the second
    // group re-reads the weights, largely from the Infinity Cache) beat one 4-token group (unit
    // lanes): 28672x8192 x4 79.5 -> 69.4 us, 1024x8192 13.3 -> 8.1; at K = 4096 the 4-token
    // group wins (4096^2 11.1 vs 14.3, 14336x4096 27.4 vs 29.7) -- profiles/r02/decode_maxnt_ab.txt.
    // By K, not by size: row shards of one matrix take the same path (bit-identical results).
    int nt_cap = fmt == Q6_K && K >= 8192 ? 2 : 4;
    while (p.nt > 1 && p.nt > nt_cap) p.nt >>= 1;
    while ((size_t)RING + act_lds(fmt, p.nt, K, p.fp8) > (size_t)LDS_CAP) {
        if (p.nt == 1) return false;
        p.nt >>= 1;
        p.lds_split = true;
    }
    p.lds = (size_t)RING + act_lds(fmt, p.nt, K, p.fp8);
    // ring bytes per row and per task (the 16-byte aligned window of a packed task may start up
    // to 14 bytes before it; the Q6_K image starts at the slot)
    const bool img = p.img = img_of(fmt, K, p.nt);
    const int64_t RB = img ? K / 256 * kImgSB : row_bytes(fmt, K);
    const int64_t upr = (K + 63) / 64;
    const int64_t cpr = upr / upc_of(fmt, p.nt); // lane chunks per row
    const int64_t cap = img ? NI * 1024 : NI * 1024 - 16;
    const int per_cu = (int)(LDS_CAP / p.lds) > 0 ? (int)(LDS_CAP / p.lds) : 1;
    int64_t W = (int64_t)num_cus() * per_cu * DW; // waves the chip holds (or the granted workgroups')
    if (wgs > 0) W = (int64_t)wgs * DW;
    DecodeGeom &g = p.geo;
    if (RB <= cap) {
        const int64_t gmax = cap / RB;
        const int64_t groups_min = (M + gmax - 1) / gmax;
        const int64_t tpw = (groups_min + W - 1) / W;     // tasks per wave at the largest groups
        int64_t G = (M + W * tpw - 1) / (W * tpw);       // smallest groups with that many tasks
        if (G < 1) G = 1;
        if (G > gmax) G = gmax;
        g.G = (int)G;
        g.nseg = 1;
        g.segu = (int)upr;
        g.ngroups = (int)((M + G - 1) / G);
        int lp2 = 0;
        while ((1 << lp2) < cpr && lp2 < 6) ++lp2;
        g.lp2 = lp2;
    } else {
        const int64_t unit64 = fmt == Q8_0 ? 64 * 68 : (fmt == Q4_K ? 64 * 36 : 64 * (img ? kImgSB : 210) / 4);
        if (cap < unit64) return false; // a 64-unit segment must fit one task (tuning builds with small NI)
        g.G = 1;
        g.segu = (int)(64 * (cap / unit64));
        g.nseg = (int)((upr + g.segu - 1) / g.segu);
        g.ngroups = (int)M;
        g.lp2 = 6;
    }
    // activations cached in registers: at most 4 units per lane (Q6_K: 2) and 2 tokens, or 8
    // units and 1 token (K <= 28672: the 70B ffn_down rows) -- no spills (kernel-resource-usage)
    const int64_t itc = (cpr + (1 << g.lp2) - 1) >> g.lp2, units = itc * (upr / cpr);
    p.itc = ((p.nt <= 2 && units <= (fmt == Q6_K ? 2 : 4)) || (p.nt == 1 && units <= 8)) ? (int)itc : 0;
    // only the instantiated chunk counts (launch_f, stream_decode_grouped_kernel): one token
    // 0..7 (Q6_K 0..4), two 0..4 (Q6_K 0..1), four 0..1 -- e.g. K = 29568 at one token gives 8
    if (p.itc > itc_max(fmt, p.nt)) p.itc = 0;
    // four tokens, one unit per lane (K <= 4096): cached too (Q6_K 14336x4096 x4 27.7 -> 20.7 us,
    // profiles/r02/decode_nt4_cache_ab.txt)
    if (p.nt == 4 && units == 1)
        p.itc = 1;
    if (p.fp8) { // (cached x~ at one token: GQ_DECODE_F8_ITC=0 turns it off)
        const int64_t fitc = (cpr + (1 << g.lp2) - 1) >> g.lp2;
        p.itc = p.nt == 1 && tuning().decode_f8_itc && fitc <= fp8_itc_max(fmt, 1) ? (int)fitc : 0;
    }
    g.early = 0; // (1 / 2: the ring refilled under the quantization -- measured slower, profiles/r04/dec_early.txt)
    const int64_t waves = g.ngroups < W ? g.ngroups : W;
    p.grid = (int)((waves + DW - 1) / DW);
    return true;
}

template <int F, int NT, int ITC, int IM = 0, int FP8 = 0>
hipError_t launch_t(const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, int64_t M, int64_t N, int64_t K,
                    int64_t ldc, const Pick &p, hipStream_t s)
{
    static bool attr = false; // raise the dynamic LDS limit once per instantiation
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void *)stream_decode_kernel<F, NT, ITC, IM, FP8>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, LDS_CAP);
        if (e != hipSuccess) return e;
        attr = true;
    }
    dim3 grid((unsigned)p.grid, (unsigned)((N + NT - 1) / NT)), block(DW * 64);
    stream_decode_kernel<F, NT, ITC, IM, FP8><<<grid, block, p.lds, s>>>(A, X, ldx, C, (int)M, N, (int)K, ldc, p.geo);
    return hipGetLastError();
}

template <int F>
hipError_t launch_f(const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, int64_t M, int64_t N, int64_t K,
                    int64_t ldc, const Pick &p, hipStream_t s)
{
#define GQ_LT(nt, itc) launch_t<F, nt, itc>(A, X, ldx, C, M, N, K, ldc, p, s)
#define GQ_LTI(nt, itc) launch_t<F, nt, itc, 1>(A, X, ldx, C, M, N, K, ldc, p, s)
    if (p.fp8) { // (itc: one token only, fp8_itc_max)
        if (p.nt == 1 && p.itc == 1) {
            if constexpr (F == Q6_K)
                if (p.img) return launch_t<F, 1, 1, 1, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
            return launch_t<F, 1, 1, 0, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
        }
        if constexpr (F != Q6_K)
            if (p.nt == 1 && p.itc == 2) return launch_t<F, 1, 2, 0, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
        if (p.itc != 0) return hipErrorInvalidValue;
        if constexpr (F == Q6_K)
            if (p.img) switch (p.nt) {
                case 1: return launch_t<F, 1, 0, 1, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
                case 2: return launch_t<F, 2, 0, 1, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
                default: return launch_t<F, 4, 0, 1, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
                }
        switch (p.nt) {
        case 1: return launch_t<F, 1, 0, 0, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
        case 2: return launch_t<F, 2, 0, 0, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
        default: return launch_t<F, 4, 0, 0, 1>(A, X, ldx, C, M, N, K, ldc, p, s);
        }
    }
    if constexpr (F == Q6_K) { // pick(): at most 8 cached units (4 chunks), 2 with two tokens
        if (p.img) switch (p.nt * 8 + p.itc) {
            case 8: return GQ_LTI(1, 0);
            case 9: return GQ_LTI(1, 1);
            case 10: return GQ_LTI(1, 2);
            case 11: return GQ_LTI(1, 3);
            case 12: return GQ_LTI(1, 4);
            case 16: return GQ_LTI(2, 0);
            case 17: return GQ_LTI(2, 1);
            case 32: return GQ_LTI(4, 0);
            case 33: return GQ_LTI(4, 1);
            default: return hipErrorInvalidValue;
            }
        switch (p.nt * 8 + p.itc) {
        case 8: return GQ_LT(1, 0);
        case 9: return GQ_LT(1, 1);
        case 10: return GQ_LT(1, 2);
        case 11: return GQ_LT(1, 3);
        case 12: return GQ_LT(1, 4);
        case 16: return GQ_LT(2, 0);
        case 17: return GQ_LT(2, 1);
        case 32: return GQ_LT(4, 0);
        case 33: return GQ_LT(4, 1);
        default: return hipErrorInvalidValue;
        }
    } else {
        switch (p.nt * 8 + p.itc) {
        case 8: return GQ_LT(1, 0);
        case 9: return GQ_LT(1, 1);
        case 10: return GQ_LT(1, 2);
        case 11: return GQ_LT(1, 3);
        case 12: return GQ_LT(1, 4);
        case 13: return GQ_LT(1, 5);
        case 14: return GQ_LT(1, 6);
        case 15: return GQ_LT(1, 7);

        case 16: return GQ_LT(2, 0);
        case 17: return GQ_LT(2, 1);
        case 18: return GQ_LT(2, 2);
        case 19: return GQ_LT(2, 3);
        case 20: return GQ_LT(2, 4);
        case 32: return GQ_LT(4, 0);
        case 33: return GQ_LT(4, 1);
        default: return hipErrorInvalidValue; // (pick() caps itc at itc_max)
        }
    }
#undef GQ_LT
#undef GQ_LTI
    return hipErrorInvalidValue;
}

// ---- grouped decode: several matrices (own type, activations, output) in one launch ----
constexpr int kMaxGroup = 16;
struct GroupedProblem {
    const uint8_t *A;
    const uint16_t *X;
    int64_t ldx;
    uint16_t *C;
    int64_t ldc;
    int M, K;
    DecodeGeom geo;
    int code;       // fmt * 16 + itc (+ 8: the Q6_K aligned image)
    int block0, gx; // this (problem, token group)'s workgroups: [block0, block0 + gx)
    int by;         // its token group
};
struct GroupedArgs {
    int n;
    int64_t N;
    GroupedProblem p[kMaxGroup];
};

template <int NT, int FP8 = 0>
__global__ __launch_bounds__(DW * 64) void stream_decode_grouped_kernel(const GroupedArgs args)
{
    extern __shared__ __attribute__((aligned(1024))) uint8_t smem[];
    const int b = (int)blockIdx.x;
    int i = 0;
    while (i + 1 < args.n && b >= args.p[i + 1].block0) ++i;
    const GroupedProblem &q = args.p[i];
    const int bx = b - q.block0;
#define GQ_GB(f, itc)                                                                                                 \
    case f * 16 + itc:                                                                                                 \
        decode_body<f, NT, itc>(q.A, q.X, q.ldx, q.C, q.M, args.N, q.K, q.ldc, q.geo, bx, q.gx, q.by, smem);         \
        return;
#define GQ_GBI(itc)                                                                                                    \
    case Q6_K * 16 + 8 + itc:                                                                                          \
        decode_body<Q6_K, NT, itc, 1>(q.A, q.X, q.ldx, q.C, q.M, args.N, q.K, q.ldc, q.geo, bx, q.gx, q.by, smem);   \
        return;
#define GQ_GF(f, itc, im)                                                                                              \
    case f * 16 + itc + 8 * im:                                                                                        \
        decode_body<f, NT, itc, im, 1>(q.A, q.X, q.ldx, q.C, q.M, args.N, q.K, q.ldc, q.geo, bx, q.gx, q.by, smem);    \
        return;
    if constexpr (FP8 && NT == 1) { // (fp8_itc_max: Q8_0 / Q4_K 0..2, Q6_K 0..1)
        switch (q.code) {
            GQ_GF(Q8_0, 0, 0) GQ_GF(Q8_0, 1, 0) GQ_GF(Q8_0, 2, 0) GQ_GF(Q4_K, 0, 0) GQ_GF(Q4_K, 1, 0) GQ_GF(Q4_K, 2, 0)
            GQ_GF(Q6_K, 0, 0) GQ_GF(Q6_K, 1, 0) GQ_GF(Q6_K, 0, 1) GQ_GF(Q6_K, 1, 1)
        default: return; // (the host checks every code against this set before the launch)
        }
    } else if constexpr (FP8) { // (itc = 0)
        switch (q.code) {
            GQ_GF(Q8_0, 0, 0) GQ_GF(Q4_K, 0, 0) GQ_GF(Q6_K, 0, 0) GQ_GF(Q6_K, 0, 1)
        default: return;
        }
    } else if constexpr (NT == 1) {
        switch (q.code) {
            GQ_GB(Q8_0, 0) GQ_GB(Q8_0, 1) GQ_GB(Q8_0, 2) GQ_GB(Q8_0, 3) GQ_GB(Q8_0, 4) GQ_GB(Q8_0, 5) GQ_GB(Q8_0, 6)
            GQ_GB(Q8_0, 7) GQ_GB(Q4_K, 0) GQ_GB(Q4_K, 1) GQ_GB(Q4_K, 2) GQ_GB(Q4_K, 3) GQ_GB(Q4_K, 4) GQ_GB(Q4_K, 5)
            GQ_GB(Q4_K, 6) GQ_GB(Q4_K, 7) GQ_GB(Q6_K, 0) GQ_GB(Q6_K, 1) GQ_GB(Q6_K, 2) GQ_GB(Q6_K, 3) GQ_GB(Q6_K, 4)
            GQ_GBI(0) GQ_GBI(1) GQ_GBI(2) GQ_GBI(3) GQ_GBI(4)
        default: return;
        }
    } else if constexpr (NT == 2) {
        switch (q.code) {
            GQ_GB(Q8_0, 0) GQ_GB(Q8_0, 1) GQ_GB(Q8_0, 2) GQ_GB(Q8_0, 3) GQ_GB(Q8_0, 4) GQ_GB(Q4_K, 0) GQ_GB(Q4_K, 1)
            GQ_GB(Q4_K, 2) GQ_GB(Q4_K, 3) GQ_GB(Q4_K, 4) GQ_GB(Q6_K, 0) GQ_GB(Q6_K, 1) GQ_GBI(0) GQ_GBI(1)
        default: return;
        }
    } else {
        switch (q.code) {
            GQ_GB(Q8_0, 0) GQ_GB(Q8_0, 1) GQ_GB(Q4_K, 0) GQ_GB(Q4_K, 1) GQ_GB(Q6_K, 0) GQ_GB(Q6_K, 1) GQ_GBI(0) GQ_GBI(1)
        default: return;
        }
    }
#undef GQ_GB
#undef GQ_GBI
#undef GQ_GF
}

template <int NT, int FP8 = 0>
hipError_t launch_grouped_nt(GroupedArgs &a, int blocks, size_t lds, hipStream_t s)
{
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void *)stream_decode_grouped_kernel<NT, FP8>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, LDS_CAP);
        if (e != hipSuccess) return e;
        attr = true;
    }
    stream_decode_grouped_kernel<NT, FP8><<<dim3((unsigned)blocks), dim3(DW * 64), lds, s>>>(a);
    return hipGetLastError();
}

} // namespace

bool decode_fused_ok(int fmt, int64_t N, int64_t K, bool fp8)
{
    Pick p;
    p.fp8 = fp8;
    // 32-bit buffer offsets: the packed tensor must stay below 2 GiB (the C ABI splits larger ones).
    // When the tokens' activations do not fit LDS beside the ring (long K: every extra token
    // group streams the weights again), the GEMV path (activations quantized once to global,
    // weights streamed once) is taken instead: Q6_K 8192x28672 x4 140 -> 82 us, x2 74 -> 67,
    // Q4_K 4096x14336 x4 26.7 -> 22.6 (profiles/r02/decode_vs_gemv_long_k.txt)
    return N <= 8 && pick(fmt, 1, N, K, p) && !p.lds_split;
}

hipError_t launch_decode_fused(int fmt, const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, int64_t M,
                               int64_t N, int64_t K, int64_t ldc, hipStream_t s, bool fp8)
{
    const int64_t RB = row_bytes(fmt, K);
    const int64_t max_rows = ((int64_t)1 << 31) / RB - 1; // rows per launch under 2 GiB
    for (int64_t m0 = 0; m0 < M; m0 += max_rows) {
        const int64_t m = M - m0 < max_rows ? M - m0 : max_rows;
        Pick p;
        p.fp8 = fp8;
        if (!pick(fmt, m, N, K, p)) return hipErrorInvalidValue;
        hipError_t e;
        switch (fmt) {
        case Q8_0: e = launch_f<Q8_0>(A + m0 * RB, X, ldx, C + m0, m, N, K, ldc, p, s); break;
        case Q4_K: e = launch_f<Q4_K>(A + m0 * RB, X, ldx, C + m0, m, N, K, ldc, p, s); break;
        default: e = launch_f<Q6_K>(A + m0 * RB, X, ldx, C + m0, m, N, K, ldc, p, s); break;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

bool decode_grouped_ok(const DecodeItem *items, int n, int64_t N, bool fp8)
{
    if (n < 1 || n > kMaxGroup || N < 1 || N > (fp8 ? 2 : 4)) return false;
    for (int i = 0; i < n; ++i) {
        const DecodeItem &it = items[i];
        if (it.M < 1 || !decode_fused_ok(it.fmt, N, it.K, fp8)) return false;
        if (it.M * row_bytes(it.fmt, it.K) >= ((int64_t)1 << 31)) return false; // 32-bit buffer offsets
    }
    return true;
}

hipError_t launch_decode_grouped(const DecodeItem *items, int n, int64_t N, hipStream_t s, bool fp8)
{
    if (!decode_grouped_ok(items, n, N, fp8)) return hipErrorInvalidValue;
    // every item's token tile as a launch of its own would pick it (bit-identical rows); one
    // launch per distinct tile (a Q6_K long-K item caps it at 2 tokens, so 3-4 tokens can take two)
    Pick solo[kMaxGroup];
    for (int i = 0; i < n; ++i) {
        solo[i].fp8 = fp8;
        if (!pick(items[i].fmt, items[i].M, N, items[i].K, solo[i])) return hipErrorInvalidValue;
    }
    for (int nt : {1, 2, 4}) {
        // the launch's parts: (item, token group); its LDS is the largest part's
        int pi[kMaxGroup], py[kMaxGroup], np = 0;
        size_t lds = 0;
        double bytes[kMaxGroup], total = 0;
        for (int i = 0; i < n; ++i) {
            if (solo[i].nt != nt) continue;
            const int tg = (int)((N + nt - 1) / nt);
            for (int y = 0; y < tg; ++y) {
                if (np == kMaxGroup) return hipErrorInvalidValue;
                pi[np] = i;
                py[np] = y;
                // Q6_K bytes weigh more at 1-2 tokens (their unpacking costs more per byte than
                // Q4_K's): measured on the Q4_K_M 7B layer, profiles/r03/tails/grouped_q6k_weight_ab.log
                // (re-swept after the Q6_K ring image: 0.9-1.75 at one and two tokens, none better,
                // profiles/r03/s3/grouped_q6w_sweep.log)
                // The fp8 form (v_dot2 on fp16 pairs, a different VALU mix): 1.30 / 1.00 at one / two
                // tokens (fp8 layer x1 38.4 -> 37.2 us, x2 53.9 -> 51.2; profiles/r05/decode_q6w_fp8_ab.txt).
                const double q6w = fp8 ? (nt == 1 ? 1.30 : 1.0) : (nt == 1 ? 1.15 : (nt == 2 ? 1.5 : 1.0));
                bytes[np] = (double)items[i].M * (double)row_bytes(items[i].fmt, items[i].K) *
                            (items[i].fmt == Q6_K ? q6w : 1.0);
                total += bytes[np];
                lds = solo[i].lds > lds ? solo[i].lds : lds;
                ++np;
            }
        }
        if (np == 0) continue;
        // The chip's workgroups split by (weighted) weight bytes (all parts finish together), whole
        // workgroups by largest remainder, at least one each: never more than the chip holds at
        // once -- rounding every part up had put a few workgroups into a second round (a 7B layer:
        // 258 of 256), doubling the launch (44.5 -> 30.1 us at one token).  Weighting the bytes by
        // each format's large-matrix streaming rate measured 1-5% slower (grouped_alloc_ab.log).
        const int per_cu = (int)(LDS_CAP / lds) > 0 ? (int)(LDS_CAP / lds) : 1;
        const int budget = num_cus() * per_cu;
        int wg[kMaxGroup], used = 0;
        double frac[kMaxGroup];
        for (int j = 0; j < np; ++j) {
            const double ideal = budget * bytes[j] / total;
            wg[j] = (int)ideal > 1 ? (int)ideal : 1;
            frac[j] = ideal - wg[j];
            used += wg[j];
        }
        while (used < budget) { // the largest remainders get the rest
            int best = 0;
            for (int j = 1; j < np; ++j)
                if (frac[j] > frac[best]) best = j;
            ++wg[best];
            frac[best] -= 1.0;
            ++used;
        }
        while (used > budget) { // (more parts than workgroups cannot happen: np <= 16)
            int best = -1;
            for (int j = 0; j < np; ++j)
                if (wg[j] > 1 && (best < 0 || frac[j] < frac[best])) best = j;
            if (best < 0) break;
            --wg[best];
            frac[best] += 1.0;
            --used;
        }
        GroupedArgs a{};
        a.N = N;
        int blocks = 0;
        for (int j = 0; j < np; ++j) {
            const int i = pi[j];
            Pick p;
            p.fp8 = fp8;
            if (!pick(items[i].fmt, items[i].M, N, items[i].K, p, wg[j]) || p.nt != nt) return hipErrorInvalidValue;
            GroupedProblem &q = a.p[j];
            q.A = items[i].A;
            q.X = items[i].X;
            q.ldx = items[i].ldx;
            q.C = items[i].C;
            q.ldc = items[i].ldc;
            q.M = (int)items[i].M;
            q.K = (int)items[i].K;
            q.geo = p.geo;
            if (p.itc > (fp8 ? fp8_itc_max(items[i].fmt, nt) : itc_max(items[i].fmt, nt)))
                return hipErrorInvalidValue; // no kernel case
            q.code = items[i].fmt * 16 + p.itc + (p.img ? 8 : 0);
            q.block0 = blocks;
            q.gx = p.grid;
            q.by = py[j];
            blocks += p.grid;
        }
        a.n = np;
        hipError_t e = fp8       ? (nt == 1 ? launch_grouped_nt<1, 1>(a, blocks, lds, s) : launch_grouped_nt<2, 1>(a, blocks, lds, s))
                       : nt == 1 ? launch_grouped_nt<1>(a, blocks, lds, s)
                       : nt == 2 ? launch_grouped_nt<2>(a, blocks, lds, s)
                                 : launch_grouped_nt<4>(a, blocks, lds, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

} // namespace gq

#ifdef GQ_DECODE_STAMPS
extern "C" int gq_debug_decode_stamps(void *host, size_t bytes)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(gq::g_dstamps), bytes < sizeof(gq::g_dstamps) ? bytes : sizeof(gq::g_dstamps)) == hipSuccess ? 0 : 1;
}
#endif
