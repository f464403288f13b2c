// mmq_kstream.hip -- the K-chunked streaming MMQ for 5..32 tokens: the weights streamed once at
// the decode kernel's rate, the activations held in registers, one launch, no split-K partials.
//
// C[t][m] = sum_k W[m][k] * x~[t][k] (fp32 accumulate), x~ = fp16(d*q) the q8_1-quantized
// activation (the integers kernels/cpu_impls multiplies; act_quant.hip's DEQ form), W dequantized
// to fp16 in registers, v_mfma_f32_16x16x32_f16.  Replaces, for 5..32 tokens, the reference's
// Triton loops kernels/mmq_q4_k.py:240-289 (and mmq_q8_0.py:102-148 / mmq_q6_k.py:197-246 alike).
//
// Why this shape.  At 16 tokens a GEMM tile reuses each weight byte 16 times only, so the work is
// a weight stream with a small MFMA on it, and the stream must run like the decode kernel's
// (contiguous per-wave LDS-DMA runs, no workgroup barrier, ~4.4 TB/s).  What blocked that in the
// earlier 5..64-token kernels was the activations: a 16-token x~ of K = 4096 is 128 KiB, as large
// as the LDS, so the resident / streaming GEMMs split K over workgroups (split-K partials + a
// reduce launch) and the skinny kernel re-read x~ from L2 for every 16-row unit (~3.5x its weight
// bytes).  Here the x~ lives in VGPRs: a workgroup's 8 waves each own one K chunk of cw <= 4
// super-blocks (NB = 1: 16 tokens, 32 VGPRs per super-block; NB = 2: 32 tokens, cw <= 2) and load
// (or quantize) that chunk of x~ once; the LDS is free for the weight rings.
//
// Work.  An item is a 16-row group of one matrix ("part"; a launch takes up to 16, e.g. a
// transformer block's projections).  Each workgroup takes a contiguous range of items, balanced
// by weight bytes.  For every item each wave streams its chunk of the 16 rows -- tasks of 16 rows
// x 2 (1 from 17 tokens) / 1 / 1 super-blocks (4.5 / 3.75 / 4.25 KiB for Q4_K / Q6_K / Q8_0) -- through a private LDS
// ring of up to 4 slots (the tasks after it in flight while one is multiplied: ~100 KiB per CU;
// the wave waits on its own vmcnt only), and multiplies it into a 16 x 16*NB fp32 tile.  The 8 waves' tiles of an item are summed in LDS in
// wave order by the last wave to arrive (an LDS counter; no workgroup barrier) and stored as fp16.
//
// Determinism.  A row's result depends on its format, K and the token tile only (the wave split
// of K is a function of K): it is the same in any workgroup, in a grouped launch or alone.
//
// MFMA 16x16x32 f16 (gfx950): lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15];
// D[row 4(l>>4)+i][col l&15].  The k-step -> element map: lane group g (= l >> 4) supplies
// "unit" g of the super-block (gguf_units.hpp), 64 elements = two 32-element q8_1 blocks, A
// (k-steps 0..3) and B (4..7) -- so a lane holds whole q8_1 blocks of its token and quantizes
// them without cross-lane reductions.  Fragment element order (0,2,1,3,4,6,5,7) as everywhere.
#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_mfma.hpp"
#include "gguf_q8_1.hpp"

namespace gq {

// hand-off waits of the cross-wave sum that gave up (gq_debug_sync_timeouts; 0 unless broken)
__device__ unsigned int g_kstream_timeouts;

#ifdef GQ_KSTREAM_STAMPS // diagnostic build: per-wave phase ticks (never the product)
__device__ unsigned long long g_kstamps[65536][12];
#endif

namespace {

// diagnostic ablation builds only (make kstamps KS_FLAGS=-DGQ_KSTREAM_ABL=n; never the product):
// 1 = no multiply (LDS reads, dequantization, MFMA), 2 = no cross-wave reduce (nothing stored),
// 4 = no weight DMA (the ring waits return at once)
#ifndef GQ_KSTREAM_ABL
#define GQ_KSTREAM_ABL 0
#endif
constexpr int KABL = GQ_KSTREAM_ABL;

constexpr int KW = 8;        // waves per workgroup
#ifndef GQ_KSTREAM_WPC
#define GQ_KSTREAM_WPC 1
#endif
constexpr int KWPC = GQ_KSTREAM_WPC; // workgroups per CU (2: four waves per SIMD at <= 128 VGPRs -- spills 36-78 VGPRs today, diagnostic builds only)

// LDS image of one super-block of a row: RBW bytes = PPS 16-byte pieces, piece q read from
// super-block byte ksrc<F>(q).  Q6_K: 240-byte aligned image (d at 222), rgemm's / gemm's.
template <int F> struct KImg;
template <> struct KImg<Q4_K> { static constexpr int RBW = 144, PPS = 9; };
template <> struct KImg<Q6_K> { static constexpr int RBW = 240, PPS = 15; };
template <> struct KImg<Q8_0> { static constexpr int RBW = 272, PPS = 17; };
template <int F> __device__ __forceinline__ uint32_t ksrc(int q)
{
    if constexpr (F == Q6_K) return q < 13 ? 16u * (uint32_t)q : 194u;
    return 16u * (uint32_t)q;
}
// A task: 16 rows x TSB super-blocks of the wave's chunk (Q4_K 2 at <= 16 tokens: 4.75 KiB, 1 at
// 17..32: 2.25 KiB; Q6_K / Q8_0 1: 3.75 / 4.25 KiB), as 16 image rows PPR pieces apart (odd
// strides spread a fragment's 16 rows over the banks).  Small tasks, so that a ring of 3-4 slots
// per wave keeps ~100 KiB per CU in flight.  (Q4_K at 17..32 tokens with 2 super-blocks per task:
// 256 VGPRs + 84 bytes of scratch, 8-10% slower on single matrices -- Q4_K 4096^2 x32 11.33 ->
// 10.22 us, 22016x4096 x32 30.96 -> 28.19 -- and the 7B layer within 1%; profiles/r06/kstream_tsb_ab.txt.
// At <= 16 tokens one super-block per task is the slower one: 4096^2 x16 8.46 -> 8.76, 11008x4096
// x16 13.93 -> 14.80, the layer x5-16 49.8-50.1 -> 51.4-52.7; kstream_tsb_nb1_ab.txt.)
template <int F, int NB = 1> struct KTask {
    static constexpr int TSB = F == Q4_K && KWPC == 1 && NB == 1 ? 2 : 1; // super-blocks per task
    static constexpr int PPR0 = TSB * KImg<F>::PPS;    // pieces of a row's task bytes (18 / 15 / 17)
    static constexpr int PPR = PPR0 | 1;               // image row stride in pieces (odd)
    static constexpr int IRS = 16 * PPR;               // image row stride
    static constexpr int NI = (16 * PPR + 63) / 64;    // DMA instructions per task (5 / 4 / 5)
    static constexpr int SLOT = 16 * IRS;              // ring slot bytes (4864 / 3840 / 4352)
};
constexpr int KNSMAX = 4;      // ring slots per wave at most
constexpr int KCWMAX = 2;      // x~ super-blocks per wave at most (a K range: 16 super-blocks)
template <int NB> constexpr int KIP = NB == 1 && KWPC == 1 ? 2 : 1; // items per LDS reduce
// LDS per wave: its weight ring, and the activation staging before it (passes of KSPB super-blocks)
// (a 32 KiB tile scratch -- two buffers, or two items per hand-off at 17..32 tokens -- leaves 15
// KiB rings and one-super-block staging passes: measured slower, profiles/r06/kstream_dbuf_ab.txt,
// kstream_ip2_ab.txt)
constexpr int KRGN = KWPC == 1 ? 16384 : 9200;
constexpr int KSPB = KWPC == 1 ? 2 : 1;
template <int F> constexpr uint32_t sb_bytes() { return Layout<F>::BYTES * (256 / Layout<F>::QK); }

// s_waitcnt vmcnt(n) for a wave-uniform n in [LO, HI] (the immediate is an encoding field): a
// binary search over the immediates, ~log2(HI - LO) scalar compares
template <int LO, int HI> __device__ __attribute__((always_inline)) inline void vm_wait_bs(int n)
{
    if constexpr (LO >= HI) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LO) : "memory");
    } else {
        constexpr int MID = (LO + HI + 1) / 2;
        if (n >= MID) vm_wait_bs<MID, HI>(n);
        else vm_wait_bs<LO, MID - 1>(n);
    }
}

// one matrix of a launch (kernel argument)
struct KPart {
    const uint8_t *A;
    const uint16_t *X;
    uint16_t *C;       // fp16 output (a whole-K part), or
    float *P;          // fp32 partial tile of one K range (a split part; rows ldc apart)
    int64_t ldx, ldc;
    int M, K, fmt, cw; // cw: super-blocks per wave
    int kofs, nsbp;    // the part's K range: super-blocks kofs .. kofs + nsbp - 1
    int64_t wcum;      // weight bytes of the parts before it
    int w;             // weight bytes per item (16 rows)
};
struct KArgs {
    KPart p[kKMaxParts];
    int n, N, aq, slot, ns; // slot: bytes of one ring slot; ns: slots per wave (2..KNSMAX)
    int64_t wtot;
};

// element offset (in the super-block) of lane group g's q8_1 blocks A (k-steps 0..3) and B (4..7)
template <int F> __device__ __forceinline__ int elem_a(int g)
{
    if constexpr (F == Q6_K) return 128 * (g >> 1) + 32 * (g & 1);
    return 64 * g;
}
template <int F> constexpr int elem_b_off() { return F == Q6_K ? 64 : 32; }

// One super-block of the lane's row from the LDS image: the unit's bytes into registers, then
// the A fragments of k-steps (j, j + 4), j = 0..3.
template <int F> struct KL;
// (load() issues every LDS read of the super-block at once; frags() is register arithmetic --
// the same operations as gguf_mfma.hpp q4k_frags / stage_frags<Q6_K>, so the same fp16 weights)
template <> struct KL<Q4_K> {
    u32x4 hdr, qa, qb; // d, dmin, scales; qs bytes 32g .. 32g+31 (sub-blocks 2g, 2g+1)
    int g;
    __device__ __forceinline__ void load(const uint8_t *img, int g_)
    {
        g = g_;
        hdr = *(const u32x4 *)img;
        qa = *(const u32x4 *)(img + 16 + 32 * g);
        qb = *(const u32x4 *)(img + 32 + 32 * g);
    }
    __device__ __forceinline__ void frags(int j, f16x8 (&f)[2]) const
    {
        const float d = h2f(hdr.x & 0xffffu), dmin = h2f(hdr.x >> 16);
        const uint32_t sc = g < 2 ? (hdr.y & 0x3f3f3f3fu) : ((hdr.w & 0x0f0f0f0fu) | ((hdr.y >> 2) & 0x30303030u));
        const uint32_t mn = g < 2 ? (hdr.z & 0x3f3f3f3fu) : (((hdr.w >> 4) & 0x0f0f0f0fu) | ((hdr.z >> 2) & 0x30303030u));
        const int sh = 16 * (g & 1);
        const uint32_t wx = j == 0 ? qa.x : (j == 1 ? qa.z : (j == 2 ? qb.x : qb.z));
        const uint32_t wy = j == 0 ? qa.y : (j == 1 ? qa.w : (j == 2 ? qb.y : qb.w));
        const h2 bias = splat(-1024.f);
#pragma unroll
        for (int n = 0; n < 2; ++n) { // n = 0: low nibbles (sub-block 2g), 1: high (2g+1)
            const h2 ds = splat(d * (float)((sc >> (sh + 8 * n)) & 0xffu));
            const h2 ndm = splat(-(dmin * (float)((mn >> (sh + 8 * n)) & 0xffu)));
            const uint32_t x0 = (wx >> (4 * n)) & 0x0f0f0f0fu, x1 = (wy >> (4 * n)) & 0x0f0f0f0fu;
            f[n] = frag4(__builtin_elementwise_fma(pair02(x0) + bias, ds, ndm),
                         __builtin_elementwise_fma(pair13(x0) + bias, ds, ndm),
                         __builtin_elementwise_fma(pair02(x1) + bias, ds, ndm),
                         __builtin_elementwise_fma(pair13(x1) + bias, ds, ndm));
        }
    }
};
// Q6_K, unit g = (h, v): elements 128h + 32v + [0,32) (A: low nibbles of ql 64h+32v.., qh bits 2v)
// and +64 (B: high nibbles, qh bits 4+2v); from the 240-byte image (d at 222)
template <> struct KL<Q6_K> {
    u32x4 qla, qlb, qha, qhb;
    u32x2 scw; // scale bytes 8h .. 8h+7
    uint32_t dw; // image bytes 220..223 (d in the high half)
    int g;
    __device__ __forceinline__ void load(const uint8_t *img, int g_)
    {
        g = g_;
        const int h = g >> 1, v = g & 1;
        qla = *(const u32x4 *)(img + 64 * h + 32 * v);
        qlb = *(const u32x4 *)(img + 64 * h + 32 * v + 16);
        qha = *(const u32x4 *)(img + 128 + 32 * h);
        qhb = *(const u32x4 *)(img + 144 + 32 * h);
        scw = *(const u32x2 *)(img + 192 + 8 * h);
        dw = *(const uint32_t *)(img + 220);
    }
    __device__ __forceinline__ void frags(int j, f16x8 (&f)[2]) const
    {
        const int v = g & 1;
        const float d = h2f(dw >> 16);
        const uint32_t qx = j == 0 ? qla.x : (j == 1 ? qla.z : (j == 2 ? qlb.x : qlb.z));
        const uint32_t qy = j == 0 ? qla.y : (j == 1 ? qla.w : (j == 2 ? qlb.y : qlb.w));
        const uint32_t hx = j == 0 ? qha.x : (j == 1 ? qha.z : (j == 2 ? qhb.x : qhb.z));
        const uint32_t hy = j == 0 ? qha.y : (j == 1 ? qha.w : (j == 2 ? qhb.y : qhb.w));
        const h2 bias = splat(-1056.f); // 1024 + 32
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            // scale of elements 128h + 64n + 32v + 8j..: byte 4n + 2v + (j >> 1) of the pair
            const int sb = 4 * n + 2 * v + (j >> 1);
            const uint32_t sw = sb < 4 ? scw.x : scw.y;
            const float scv = (float)(int8_t)((sw >> (8 * (sb & 3))) & 0xffu);
            const h2 dsc = splat(d * scv);
            const int sq = 4 * n + 2 * v;
            const uint32_t c0 = ((qx >> (4 * n)) & 0x0f0f0f0fu) | (((hx >> sq) & 0x03030303u) << 4);
            const uint32_t c1 = ((qy >> (4 * n)) & 0x0f0f0f0fu) | (((hy >> sq) & 0x03030303u) << 4);
            f[n] = frag4((pair02(c0) + bias) * dsc, (pair13(c0) + bias) * dsc, (pair02(c1) + bias) * dsc,
                         (pair13(c1) + bias) * dsc);
        }
    }
};
template <> struct KL<Q8_0> {
    uint32_t w[17]; // bytes 68g .. 68g+67 of the super-block image (blocks 2g, 2g+1), 4-byte aligned
    __device__ __forceinline__ void load(const uint8_t *img, int g)
    {
        const uint32_t *q = (const uint32_t *)(img + 68 * g);
#pragma unroll
        for (int k = 0; k < 17; ++k) w[k] = q[k];
    }
    __device__ __forceinline__ void frags(int j, f16x8 (&f)[2]) const
    {
        const h2 bias = splat(-1152.f); // codes biased by +128 (xor 0x80)
        // block 2g: d = bytes 0..1, codes 2 + 8j ..; block 2g+1: d = bytes 34..35, codes 36 + 8j ..
        const uint32_t a0 = __builtin_amdgcn_alignbyte(w[2 * j + 1], w[2 * j], 2);
        const uint32_t a1 = __builtin_amdgcn_alignbyte(w[2 * j + 2], w[2 * j + 1], 2);
        const uint32_t b0 = w[9 + 2 * j], b1 = w[10 + 2 * j];
        const h2 da = as_h2(__builtin_amdgcn_perm(w[0], w[0], 0x05040504u));
        const h2 db = as_h2(__builtin_amdgcn_perm(w[8], w[8], 0x07060706u));
        const uint32_t c0 = a0 ^ 0x80808080u, c1 = a1 ^ 0x80808080u, c2 = b0 ^ 0x80808080u, c3 = b1 ^ 0x80808080u;
        f[0] = frag4((pair02(c0) + bias) * da, (pair13(c0) + bias) * da, (pair02(c1) + bias) * da,
                     (pair13(c1) + bias) * da);
        f[1] = frag4((pair02(c2) + bias) * db, (pair13(c2) + bias) * db, (pair02(c3) + bias) * db,
                     (pair13(c3) + bias) * db);
    }
};

// x~ of one 32-element q8_1 block held by ONE lane (four 16-byte pieces of fp16): deq_quad's
// arithmetic (gguf_q8_1.hpp) with the amax over the lane's 32 values -- the value deq_quad's
// 4-lane reduction forms -- so the bits equal act_quant's DEQ form.  o[i] = piece i in the
// fragment order (0,2,1,3,4,6,5,7).
__device__ __forceinline__ void deq_lane32(const u32x4 (&w)[4], u32x4 (&o)[4])
{
    typedef _Float16 h2t __attribute__((ext_vector_type(2)));
    float x[32];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t wd[4] = {w[i].x, w[i].y, w[i].z, w[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[8 * i + 2 * k] = h2f(wd[k] & 0xffff);
            x[8 * i + 2 * k + 1] = h2f(wd[k] >> 16);
        }
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) amax = fmaxf(amax, fabsf(x[i]));
    const uint16_t dbits = amax != 0.f ? f2h_bits(q81_div(amax, 127.0f, 1.0f / 127.0f)) : (uint16_t)0;
    const float d = h2f(dbits);
    const float div = d == 0.f ? 1.0f : d;
    const float rdiv = __builtin_amdgcn_rcpf(div);
    const _Float16 dh = __builtin_bit_cast(_Float16, dbits);
    const h2t dd = {dh, dh}, magic = {(_Float16)1536.f, (_Float16)1536.f};
    const h2t lo = {(_Float16)-127.f, (_Float16)-127.f}, hi = {(_Float16)127.f, (_Float16)127.f};
    const int ord[8] = {0, 2, 1, 3, 4, 6, 5, 7};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t r[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            h2t q = {(_Float16)q81_div(x[8 * i + ord[2 * p]], div, rdiv), (_Float16)q81_div(x[8 * i + ord[2 * p + 1]], div, rdiv)};
            q = (q + magic) - magic;
            q = __builtin_elementwise_min(__builtin_elementwise_max(q, lo), hi);
            r[p] = __builtin_bit_cast(uint32_t, q * dd);
        }
        o[i] = (u32x4){r[0], r[1], r[2], r[3]};
    }
}

// The fp8 variant's x~ of one 32-element block held by one lane (f8_quad's arithmetic with the
// lane's own amax): codes e4m3(x / 2^e), x~ = code * 2^e, pairs (0,2), (1,3) per 4-group.
__device__ __forceinline__ void f8_lane32(const u32x4 (&w)[4], u32x4 (&o)[4])
{
    float x[32], amax = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t wd[4] = {w[i].x, w[i].y, w[i].z, w[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[8 * i + 2 * k] = h2f(wd[k] & 0xffff);
            x[8 * i + 2 * k + 1] = h2f(wd[k] >> 16);
        }
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) amax = fmaxf(amax, fabsf(x[i]));
    const uint32_t ab = __builtin_bit_cast(uint32_t, amax);
    const int E = (int)((ab >> 23) & 0xff) - 126;
    const int e = amax == 0.f ? 0 : E - 9 + ((ab & 0x7fffffu) > 0x600000u ? 1 : 0);
    const float inv = __builtin_bit_cast(float, (uint32_t)(127 - e) << 23);
    const float X = __builtin_bit_cast(float, (uint32_t)(127 + e) << 23);
    typedef _Float16 h2t __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t r[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float *y = x + 8 * i + 4 * h;
            int c = __builtin_amdgcn_cvt_pk_fp8_f32(y[0] * inv, y[2] * inv, 0, false);
            c = __builtin_amdgcn_cvt_pk_fp8_f32(y[1] * inv, y[3] * inv, c, true);
            r[2 * h] = __builtin_bit_cast(uint32_t, (h2t)__builtin_amdgcn_cvt_scalef32_pk_f16_fp8(c, X, false));
            r[2 * h + 1] = __builtin_bit_cast(uint32_t, (h2t)__builtin_amdgcn_cvt_scalef32_pk_f16_fp8(c, X, true));
        }
        o[i] = (u32x4){r[0], r[1], r[2], r[3]};
    }
}

// One part's items [j0, j1) (16-row groups) on this workgroup.  seq = row groups this workgroup
// reduced before (the scratch protocol's sequence number), advanced here.
// CWM: the x~ super-blocks a wave holds (instantiated per chunk size: 1, 2 or 4; P.cw <= CWM)
template <int F, int NB, int CWM>
__device__ __forceinline__ void kbody(const KPart &P, int j0, int j1, int N, int aq, int slot, int ns, uint8_t *smem,
                                      float *scr, int *sync, int &seq)
{
    using T = KTask<F, NB>;
    constexpr int TSB = T::TSB;
    constexpr int NTG = (CWM + TSB - 1) / TSB; // tasks per row group at most
    constexpr uint32_t SB = sb_bytes<F>();
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l16 = lane & 15, gl = lane >> 4;
    const int M = P.M, nsb = P.K >> 8, cw = P.cw;
    const int sb0 = P.kofs + wave * cw;
    int mysb = P.kofs + P.nsbp - sb0;
    mysb = mysb < 0 ? 0 : (mysb > cw ? cw : mysb);
    const int ntg = (mysb + TSB - 1) / TSB;  // this wave's tasks per row group (0..NTG)
    const int ntask = (j1 - j0) * ntg;
    const uint32_t RB = (uint32_t)nsb * SB;
    uint8_t *ring = smem + wave * KRGN;
#ifdef GQ_KSTREAM_STAMPS
    const unsigned long long t_in = __builtin_amdgcn_s_memtime();
    unsigned long long t_wait = 0, t_red = 0, t_spin = 0, t_sum = 0, n_sum = 0;
#endif

    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)P.A, 0, (int)(((uint32_t)M * RB + 15u) & ~15u), 0x00020000);
    // per-lane source offset of each DMA instruction of a task, relative to the task's first row
    // and super-block (piece p = 64i + lane: row r, super-block s0, image piece q; pad pieces read
    // past the buffer's range -- zeros, no memory access); a task adds one scalar offset
    uint32_t poff[T::NI];
#pragma unroll
    for (int i = 0; i < T::NI; ++i) {
        const int p = 64 * i + lane, r = p / T::PPR, pc = p - r * T::PPR;
        const int s0 = pc / KImg<F>::PPS, q = pc - s0 * KImg<F>::PPS;
        poff[i] = r < 16 && pc < T::PPR0 ? (uint32_t)r * RB + (uint32_t)s0 * SB + ksrc<F>(q) : 0x80000000u;
    }
    // the issue cursor: task (item j0 + igi, sub-chunk isub) into slot islot.  (A super-block past
    // the wave's chunk is read from the next bytes of the row -- or zeros past the tensor -- and
    // never multiplied.)
    constexpr int IP = KIP<NB>; // items per reduce (one LDS hand-off per IP items)
    const int nit = j1 - j0;
    int igi = 0, isub = 0, islot = 0;
    auto issue = [&]() __attribute__((always_inline)) {
        const uint32_t tb = (uint32_t)(16 * (j0 + igi)) * RB + (uint32_t)(sb0 + TSB * isub) * SB;
        uint8_t *dst = ring + islot * slot;
#pragma unroll
        for (int i = 0; i < T::NI; ++i)
            // (the last instruction's lanes past the image stay off: the slot is 16 image rows)
            if (!(KABL & 4) && (i < T::NI - 1 || 64 * i + lane < 16 * T::PPR)) dma16(wrs, dst + 1024 * i, poff[i] + tb, 0);
        if (++isub == ntg) {
            isub = 0;
            ++igi;
        }
        islot = islot + 1 == ns ? 0 : islot + 1;
    };

    // ---- prologue: this wave's chunk of the activations (tokens 16t + l16, super-blocks sb0 + c)
    //      into registers, staged through the wave's ring region: per pass, 16 token rows x 2
    //      super-blocks (1 KiB, one fully coalesced DMA instruction per token row; 16-byte piece Q
    //      of row r at piece Q ^ bitrev4(r), so the fragment reads of 16 rows hit distinct banks),
    //      then the lane's two q8_1 blocks per super-block read back (8 pieces) and quantized
    //      (aq 1 / 2) or taken as they are (aq 0: prepared x~, the fragment order already).
    //      (Loading the prepared x~ straight into the fragments instead -- 16-byte loads, 64-byte
    //      runs per lane group -- is 30-50% slower: profiles/r06/kstream_xdirect_ab.txt; one-
    //      super-block passes with the next in flight leave the prologue's ticks unchanged and the
    //      layer 2-5% slower at 24-32 tokens: kstream_xpipe_ab.txt) ----
    f16x8 xf[CWM][8][NB];
    {
        const uint32_t xbytes = (uint32_t)(((int64_t)(N - 1) * P.ldx + P.K) * 2);
        const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)P.X, 0, (int)xbytes, 0x00020000);
        const int frow = ((l16 & 1) << 3) | ((l16 & 2) << 1) | ((l16 & 4) >> 1) | ((l16 & 8) >> 3); // bitrev4
#pragma unroll
        for (int t = 0; t < NB; ++t)
#pragma unroll
            for (int c0 = 0; c0 < CWM; c0 += KSPB) {
                if (c0 >= mysb) break; // (wave-uniform)
                // a pass: 16 token rows of KSPB super-blocks (RP = 32 * KSPB pieces each)
                constexpr int RP = 32 * KSPB;
#pragma unroll
                for (int i = 0; i < 16 * RP / 64; ++i) {
                    const int r = (64 * i + lane) / RP, pos = (64 * i + lane) % RP;
                    const int tok = 16 * t + r < N ? 16 * t + r : N - 1;
                    const int q = pos ^ (((r & 1) << 3) | ((r & 2) << 1) | ((r & 4) >> 1) | ((r & 8) >> 3));
                    const int sb = sb0 + c0 + (q >> 5);
                    const uint32_t off = 2u * ((uint32_t)tok * (uint32_t)P.ldx +
                                               256u * (uint32_t)(sb < sb0 + mysb ? sb : sb0 + c0) + 8u * (uint32_t)(q & 31));
                    dma16(xrs, ring + 1024 * i, off, 0);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int cs = 0; cs < KSPB && c0 + cs < CWM; ++cs) {
                    const int c = c0 + cs;
                    u32x4 xr[2][4];
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int qp = 32 * cs + (elem_a<F>(gl) + h * elem_b_off<F>()) / 8 + i;
                            xr[h][i] = *(const u32x4 *)(ring + 16 * RP * l16 + 16 * (qp ^ frow));
                        }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        u32x4 o[4];
                        if (aq == 1) deq_lane32(xr[h], o);
                        else if (aq == 2) f8_lane32(xr[h], o);
                        else {
#pragma unroll
                            for (int i = 0; i < 4; ++i) o[i] = xr[h][i];
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i) xf[c][4 * h + i][t] = __builtin_bit_cast(f16x8, o[i]);
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the region is free again
            }
    }
    const int pre = ntask < ns ? ntask : ns; // then the weight ring
    for (int i = 0; i < pre; ++i) issue();
    int issued = pre;
#ifdef GQ_KSTREAM_STAMPS
    const unsigned long long t_pro = __builtin_amdgcn_s_memtime();
#endif

    // ---- IP items' tiles summed over the 8 waves (the last to arrive, in wave order) and stored ----
    // The summing wave issues exactly IP*NB buffer stores (tokens past N: an offset past the
    // buffer's range, dropped), so the ring's waits can count them (stores share vmcnt).
    const __amdgpu_buffer_rsrc_t crs =
        P.P ? __builtin_amdgcn_make_buffer_rsrc((void *)P.P, 0, (int)(uint32_t)(((int64_t)(N - 1) * P.ldc + M) * 4), 0x00020000)
            : __builtin_amdgcn_make_buffer_rsrc((void *)P.C, 0, (int)(uint32_t)(((int64_t)(N - 1) * P.ldc + M) * 2),
                                                0x00020000);
    auto reduce_store = [&](int grp, int np, const f32x4 (&acc)[IP][NB]) __attribute__((always_inline)) -> bool {
        // the scratch is free once the previous hand-off has been summed (a wave is a whole round
        // of items ahead of the summing wave before it waits here)
        // (bounded: a broken hand-off ends the kernel with wrong bits, counted in
        // g_kstream_timeouts -- gq_debug_sync_timeouts -- never hangs the GPU).
#ifdef GQ_KSTREAM_STAMPS
        const unsigned long long ts = __builtin_amdgcn_s_memtime();
#endif
        int spin = 0;
        for (; spin < (1 << 22) && __hip_atomic_load(&sync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < seq; ++spin)
            __builtin_amdgcn_s_sleep(1);
        if (spin == (1 << 22) && lane == 0)
            __hip_atomic_fetch_add(&g_kstream_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef GQ_KSTREAM_STAMPS
        t_spin += __builtin_amdgcn_s_memtime() - ts;
#endif
        // Ordering: a wave's LDS operations execute in issue order, so only the compiler could
        // move the scratch accesses across the hand-off words; an empty asm with a memory clobber
        // at each edge forbids that.  (Not a fence: any acquire / release, even one restricted to
        // LDS, makes the compiler wait vmcnt(0) for the LDS-DMA weight ring and breaks its counted
        // waits -- 19 extra vmcnt(0) in the kstream kernels' ISA.)
        asm volatile("" ::: "memory");
#pragma unroll
        for (int ip = 0; ip < IP; ++ip)
#pragma unroll
            for (int t = 0; t < NB; ++t) *(f32x4 *)(scr + ((wave * IP + ip) * NB + t) * 256 + 4 * lane) = acc[ip][t];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        int old = 0;
        // (the lgkmcnt(0) above: this wave's scratch stores have landed before its arrival; the
        // summing wave's reads below stay after the arrival)
        if (lane == 0) old = __hip_atomic_fetch_add(&sync[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        asm volatile("" ::: "memory");
        old = __builtin_amdgcn_readfirstlane(old);
        ++seq;
        // Issue priority by arrival rank, held until the wave's next arrival: the first half to
        // arrive at 0, the second half at 1, the last -- the summing wave, behind all the others
        // -- at 2.  Without it the waves dispatched second (4-7) lose every arbitration against
        // their SIMD partners, one of them arrives last at every hand-off of the workgroup and
        // sums it, and the other seven wait for it: the 7B layer x16 / x32 50.2 / 61.6 -> 47.5 /
        // 56.3 us with a first form (0 once arrived, 2 last, 1 past the next wait), single
        // matrices 1-2% faster again with the rank form; same bits (profiles/r06/kstream_prio_ab.txt,
        // kstream_prank_ab.txt; a static priority for waves 4-7 did nothing).
        const int rank = old & (KW - 1);
        if (rank != KW - 1) {
            if (rank >= KW / 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
            return false;
        }
        __builtin_amdgcn_s_setprio(2); // (four levels -- rank / 2, the last 3 -- measured no better)
#ifdef GQ_KSTREAM_STAMPS
        const unsigned long long tsum = __builtin_amdgcn_s_memtime();
        ++n_sum;
#endif
#pragma unroll
        for (int ip = 0; ip < IP; ++ip)
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                // the KW tiles read together, one wait (left to itself the compiler waits after
                // every read here -- 14 serialized LDS round trips on the summing wave, which the
                // other waves then wait for at their next hand-off), summed in wave order
                f32x4 r[KW];
#pragma unroll
                for (int w = 0; w < KW; ++w) r[w] = *(const f32x4 *)(scr + ((w * IP + ip) * NB + t) * 256 + 4 * lane);
                asm volatile("" ::"v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]), "v"(r[6]), "v"(r[7]));
                f32x4 v = r[0];
#pragma unroll
                for (int w = 1; w < KW; ++w) v += r[w];
                const int tok = 16 * t + l16, row = 16 * (grp + ip) + 4 * gl; // (M % 16 == 0: 4 rows exist)
                const bool real = tok < N && ip < np;
                if (P.P) { // a split part: its fp32 partial
                    const uint32_t off = real ? 4u * ((uint32_t)tok * (uint32_t)P.ldc + (uint32_t)row) : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), crs, off, 0, 0);
                } else {
                    const uint32_t off = real ? 2u * ((uint32_t)tok * (uint32_t)P.ldc + (uint32_t)row) : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b64(
                        (u32x2){(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)},
                        crs, off, 0, 0);
                }
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the scratch reads are done
        if (lane == 0) __hip_atomic_store(&sync[1], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef GQ_KSTREAM_STAMPS
        t_sum += __builtin_amdgcn_s_memtime() - tsum;
#endif
        return true;
    };

    // ---- main loop: task k = (item j0 + k / ntg, sub-chunk k % ntg) in slot k % ns; items in
    //      groups of IP per reduce ----
    // stq: per slot (8 bits each), the store instructions issued after its in-flight DMA -- the
    // younger ops its wait must allow beside the later tasks' DMAs
    int k = 0, kslot = 0;
    uint32_t stq = 0;
    for (int gi = 0; gi < nit; gi += IP) {
        const int np = nit - gi < IP ? nit - gi : IP;
        f32x4 acc[IP][NB];
#pragma unroll
        for (int ip = 0; ip < IP; ++ip)
#pragma unroll
            for (int t = 0; t < NB; ++t) acc[ip][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ip = 0; ip < IP; ++ip) {
            if (ip >= np) break;
#pragma unroll
            for (int sub = 0; sub < NTG; ++sub) {
                if (sub < ntg) {
#ifdef GQ_KSTREAM_STAMPS
                    const unsigned long long ta = __builtin_amdgcn_s_memtime();
#endif
                    // task k has landed once only younger ops are outstanding: the later tasks'
                    // DMAs and the stores issued after its own (an exact count: rounding it down
                    // would wait on the next task's DMA)
                    vm_wait_bs<0, (KNSMAX - 1) * T::NI + KNSMAX * IP * NB>(
                        (issued - k - 1) * T::NI + (int)((stq >> (8 * kslot)) & 0xffu));
#ifdef GQ_KSTREAM_STAMPS
                    t_wait += __builtin_amdgcn_s_memtime() - ta;
#endif
                    const uint8_t *img = ring + kslot * slot + l16 * T::IRS;
                    // every LDS read of the task first (one latency), then the arithmetic
                    KL<F> w[TSB];
#pragma unroll
                    for (int s = 0; s < TSB; ++s)
                        if (TSB * sub + s < CWM && TSB * sub + s < mysb && !(KABL & 1))
                            w[s].load(img + s * KImg<F>::RBW, gl);
#pragma unroll
                    for (int s = 0; s < TSB; ++s) {
                        const int c = TSB * sub + s;
                        if (c < CWM && c < mysb && !(KABL & 1)) {
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                f16x8 af[2];
                                w[s].frags(j, af);
#pragma unroll
                                for (int t = 0; t < NB; ++t) {
                                    acc[ip][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[0], xf[c][j][t], acc[ip][t], 0, 0, 0);
                                    acc[ip][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[1], xf[c][4 + j][t], acc[ip][t], 0, 0, 0);
                                }
                            }
                        }
                    }
                    // the slot's fragments are in registers: refill it with task k + ns
                    if (issued < ntask) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        issue();
                        ++issued;
                        stq &= ~(0xffu << (8 * kslot));
                    }
                    ++k;
                    kslot = kslot + 1 == ns ? 0 : kslot + 1;
                }
            }
        }
#ifdef GQ_KSTREAM_STAMPS
        const unsigned long long tr = __builtin_amdgcn_s_memtime();
#endif
        if (KABL & 2) { // (every accumulator consumed: the multiply stays)
#pragma unroll
            for (int ip = 0; ip < IP; ++ip)
#pragma unroll
                for (int t = 0; t < NB; ++t) asm volatile("" ::"v"(acc[ip][t]));
        } else if (reduce_store(j0 + gi, np, acc)) {
            stq += (uint32_t)(IP * NB) * 0x01010101u;
        }
#ifdef GQ_KSTREAM_STAMPS
        t_red += __builtin_amdgcn_s_memtime() - tr;
#endif
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // no DMA lands after the wave moves on
#ifdef GQ_KSTREAM_STAMPS
    const unsigned long long t_out = __builtin_amdgcn_s_memtime();
    const int id = (int)blockIdx.x * KW + wave;
    if (lane == 0 && id < 65536) {
        g_kstamps[id][0] += t_pro - t_in;
        g_kstamps[id][1] += t_wait;
        g_kstamps[id][2] += t_red;
        g_kstamps[id][3] += t_out - t_pro;
        g_kstamps[id][4] += (unsigned long long)ntask;
        g_kstamps[id][5] += (unsigned long long)(j1 - j0);
        // this wave's 16-row super-block tasks by format (Q4_K in 6, the others in 7)
        g_kstamps[id][F == Q4_K ? 6 : 7] += (unsigned long long)((j1 - j0) * mysb);
        g_kstamps[id][8] += t_spin; // (of t_red: waiting for the previous hand-off's sum)
        g_kstamps[id][9] += 1;      // parts
        g_kstamps[id][10] += n_sum; // hand-offs this wave summed (the last to arrive)
        g_kstamps[id][11] += t_sum; // and the ticks it spent summing them
    }
#endif
}

template <int NB, int CWM>
__global__ __launch_bounds__(64 * KW, KWPC * KW / 4) void kstream_kernel(const KArgs a)
{
    extern __shared__ __attribute__((aligned(1024))) uint8_t smem[]; // the waves' rings (KRGN each)
    __shared__ __attribute__((aligned(16))) float scr[KW * KIP<NB> * NB * 256]; // the waves' item tiles
    __shared__ int sync[2]; // arrivals, hand-offs summed
    if (threadIdx.x < 2) sync[threadIdx.x] = 0;
    __builtin_amdgcn_s_setprio(1);
    __syncthreads();
    // this workgroup's items: those whose first weight byte (the parts' bytes in order) falls in
    // [t0, t1), an equal share of the launch's cost (weight bytes, weighted per format: launch_kstream)
    const int64_t t0 = a.wtot * blockIdx.x / gridDim.x, t1 = a.wtot * (blockIdx.x + 1) / gridDim.x;
    int seq = 0;
    for (int i = 0; i < a.n; ++i) {
        const KPart &P = a.p[i];
        const int ng = (P.M + 15) / 16;
        const int64_t lo = t0 - P.wcum, hi = t1 - P.wcum;
        const int64_t j0 = lo <= 0 ? 0 : (lo + P.w - 1) / P.w, j1 = hi <= 0 ? 0 : (hi + P.w - 1) / P.w;
        const int b = (int)(j0 < ng ? j0 : ng), e = (int)(j1 < ng ? j1 : ng);
        if (b >= e) continue;
        if (P.fmt == Q4_K) kbody<Q4_K, NB, CWM>(P, b, e, a.N, a.aq, a.slot, a.ns, smem, scr, sync, seq);
        else if (P.fmt == Q6_K) kbody<Q6_K, NB, CWM>(P, b, e, a.N, a.aq, a.slot, a.ns, smem, scr, sync, seq);
        else kbody<Q8_0, NB, CWM>(P, b, e, a.N, a.aq, a.slot, a.ns, smem, scr, sync, seq);
    }
}

// the kernel for a launch's token tiles and largest chunk, its static LDS (the tile scratch)
template <int NB, int CWM> hipError_t run(const KArgs &a, unsigned grid, hipStream_t s)
{
    static bool attr = false;
    if (!attr) {
        hipFuncAttributes fa;
        hipError_t e = hipFuncGetAttributes(&fa, (const void *)kstream_kernel<NB, CWM>);
        if (e != hipSuccess) return e;
        if (KWPC * (fa.sharedSizeBytes + (size_t)KW * KRGN) > 160 * 1024) return hipErrorInvalidValue;
        e = hipFuncSetAttribute((const void *)kstream_kernel<NB, CWM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                KW * KRGN);
        if (e != hipSuccess) return e;
        attr = true;
    }
    kstream_kernel<NB, CWM><<<dim3(grid), dim3(64 * KW), (size_t)KW * KRGN, s>>>(a);
    return hipGetLastError();
}

} // namespace

// K split over the 8 waves: cw super-blocks each (the fewest that cover K), or 0 when K is
// longer than the waves' x~ registers hold (2 super-blocks each: K <= 4096)
// K ranges (split parts) of a matrix: as few as keep each within the 8 waves' x~ registers
// (2 super-blocks per wave: 16 per range); cw = super-blocks per wave of a range
int kstream_splits(int64_t K) { return (int)((K / 256 + 8 * KCWMAX - 1) / (8 * KCWMAX)); }
int kstream_cw(int64_t N, int64_t K)
{
    if (K % 256 != 0 || N < 1 || N > 32) return 0;
    const int64_t S = kstream_splits(K), per = (K / 256 + S - 1) / S;
    return (int)((per + KW - 1) / KW);
}

bool kstream_ok(int fmt, int64_t M, int64_t N, int64_t K)
{
    if (fmt != Q8_0 && fmt != Q4_K && fmt != Q6_K) return false;
    if (M < 16 || M % 16 != 0 || kstream_cw(N, K) == 0) return false; // (whole 16-row items)
    // 32-bit buffer offsets over the weights
    return M * (K / 256) * (int64_t)(fmt == Q8_0 ? 272 : (fmt == Q4_K ? 144 : 210)) < ((int64_t)1 << 31);
}

size_t kstream_partial_bytes(const KItem *items, int n, int64_t N)
{
    size_t b = 0;
    for (int i = 0; i < n; ++i) {
        const int S = kstream_splits(items[i].K);
        if (S > 1) b += ((size_t)S * N * items[i].M * 4 + 255) & ~(size_t)255;
    }
    return b;
}

namespace {
// C[t][m] = fp16(sum over the splits, in order, of the fp32 partials P[z][t][m]); four outputs per
// thread, every split part of a launch in one grid
struct KRed {
    const float *P[kKMaxParts];
    uint16_t *C[kKMaxParts];
    int64_t ldc[kKMaxParts];
    int M[kKMaxParts], S[kKMaxParts], blk0[kKMaxParts + 1];
    int n, N;
};
__global__ __launch_bounds__(256) void kstream_reduce_kernel(const KRed r)
{
    int i = 0;
    while (i + 1 < r.n && (int)blockIdx.x >= r.blk0[i + 1]) ++i;
    const int64_t q = (int64_t)(blockIdx.x - r.blk0[i]) * 256 + threadIdx.x; // 4-output unit
    const int M = r.M[i], m4 = M / 4;
    if (q >= (int64_t)r.N * m4) return;
    const int t = (int)(q / m4), m = 4 * (int)(q % m4);
    const size_t zs = (size_t)r.N * M;
    f32x4 v = *(const f32x4 *)(r.P[i] + (size_t)t * M + m);
    for (int z = 1; z < r.S[i]; ++z) v += *(const f32x4 *)(r.P[i] + z * zs + (size_t)t * M + m);
    *(u32x2 *)(r.C[i] + t * r.ldc[i] + m) = (u32x2){(uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                                    (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16)};
}
} // namespace

hipError_t launch_kstream(const KItem *items, int n, int64_t N, int aq, void *partials, hipStream_t s)
{
    if (n < 1 || n > kKMaxParts || N < 1 || N > 32) return hipErrorInvalidValue;
    KArgs a{};
    KRed rd{};
    a.N = (int)N;
    a.aq = aq;
    rd.N = (int)N;
    int kb = 0, np = 0, cwm = 1;
    int64_t wcum = 0, items_total = 0, rblk = 0;
    uint8_t *pw = (uint8_t *)partials;
    for (int i = 0; i < n; ++i) {
        const KItem &it = items[i];
        if (!kstream_ok(it.fmt, it.M, N, it.K)) return hipErrorInvalidValue;
        const int S = kstream_splits(it.K), nsb = (int)(it.K / 256), per = (nsb + S - 1) / S;
        float *P = nullptr;
        if (S > 1) {
            if (!partials || rd.n == kKMaxParts) return hipErrorInvalidValue;
            P = (float *)pw;
            pw += ((size_t)S * N * it.M * 4 + 255) & ~(size_t)255;
            rd.P[rd.n] = P;
            rd.C[rd.n] = it.C;
            rd.ldc[rd.n] = it.ldc;
            rd.M[rd.n] = (int)it.M;
            rd.S[rd.n] = S;
            rd.blk0[rd.n] = (int)rblk;
            rblk += (N * (it.M / 4) + 255) / 256;
            ++rd.n;
        }
        for (int z = 0; z < S; ++z) {
            if (np == kKMaxParts) return hipErrorInvalidValue;
            KPart &p = a.p[np++];
            p.A = it.A;
            p.X = it.X;
            p.C = it.C;
            p.P = P ? P + (size_t)z * N * it.M : nullptr;
            p.ldx = it.ldx;
            p.ldc = P ? it.M : it.ldc;
            p.M = (int)it.M;
            p.K = (int)it.K;
            p.fmt = it.fmt;
            p.kofs = z * per;
            p.nsbp = nsb - p.kofs < per ? nsb - p.kofs : per;
            p.cw = (p.nsbp + KW - 1) / KW;
            const int64_t sbb = it.fmt == Q8_0 ? 272 : (it.fmt == Q4_K ? 144 : 210);
            // the deal's cost of a 16-row item: per super-block its bytes - 55: Q4_K 89,
            // Q6_K 155, Q8_0 217 -- a Q6_K super-block's dequantization costs more per byte than the
            // bytes alone say; the 7B layer 3-4% faster than a deal by bytes at 5..32 tokens (x16
            // 52.7 -> 50.8 us; profiles/r05/kstream_deal_ab.txt).  Any deal gives the same bits.
#ifndef GQ_KSTREAM_SBW_OFF
#define GQ_KSTREAM_SBW_OFF 55 // (A/B builds: other offsets)
#endif
            p.w = (int)(16 * p.nsbp * (sbb - GQ_KSTREAM_SBW_OFF));
            p.wcum = wcum;
            const int64_t ng = it.M / 16;
            wcum += ng * p.w;
            items_total += ng;
            cwm = p.cw > cwm ? p.cw : cwm;
        }
        const int k = it.fmt == Q4_K ? (N <= 16 ? KTask<Q4_K, 1>::SLOT : KTask<Q4_K, 2>::SLOT)
                                     : (it.fmt == Q6_K ? KTask<Q6_K>::SLOT : KTask<Q8_0>::SLOT);
        kb = k > kb ? k : kb;
    }
    a.n = np;
    a.wtot = wcum;
    a.slot = kb;
    a.ns = KRGN / kb > KNSMAX ? KNSMAX : KRGN / kb; // ring slots per wave (3 or 4)
    const int64_t wgs = num_cus() * KWPC;
    const unsigned grid = (unsigned)(items_total < wgs ? items_total : wgs);
    hipError_t e;
    if (N <= 16) e = cwm <= 1 ? run<1, 1>(a, grid, s) : run<1, 2>(a, grid, s);
    else e = cwm <= 1 ? run<2, 1>(a, grid, s) : run<2, 2>(a, grid, s);
    if (e != hipSuccess || rd.n == 0) return e;
    rd.blk0[rd.n] = (int)rblk;
    kstream_reduce_kernel<<<dim3((unsigned)rblk), dim3(256), 0, s>>>(rd);
    return hipGetLastError();
}

unsigned int kstream_timeouts()
{
    unsigned int v = 0;
    return hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_kstream_timeouts), sizeof(v)) == hipSuccess ? v : ~0u;
}

} // namespace gq

#ifdef GQ_KSTREAM_STAMPS
extern "C" int gq_debug_kstream_stamps(void *host, size_t bytes)
{
    if (bytes > sizeof(gq::g_kstamps)) bytes = sizeof(gq::g_kstamps);
    hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(gq::g_kstamps), bytes, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess) {
        static unsigned long long zeros[65536][12];
        e = hipMemcpyToSymbol(HIP_SYMBOL(gq::g_kstamps), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
    }
    return e == hipSuccess ? 0 : -1;
}
#endif
