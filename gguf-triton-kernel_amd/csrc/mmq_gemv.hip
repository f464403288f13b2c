// mmq_gemv.hip -- decode-shaped MMQ (few tokens): weight rows streamed once from HBM.
//
// Computes C[t][m] = sum_k W[m][k] * x~[t][k] for t < N_tok (<= 4 per launch column) where
// x~ is the q8_1-quantized activation (act_quant.hip, SOA form) and W is the packed GGUF
// row m.  The per-block arithmetic is the reference's (kernels/cpu_impls/*):
//   Q8_0 : dA*dB*sum(qA*qB)                                  mmq_q8_0_q8_1_cpu.py:37-54
//   Q4_K : d*sc*dB*sum(q*qB) - dmin*m*sB                     mmq_q4_k_q8_1_cpu.py:94-117
//   Q6_K : dB*(d*sc1*sum((q-32)*qB)_lo + d*sc2*sum(...)_hi)  mmq_q6_k_q8_1_cpu.py:117-150
// with exact int32 dot products (v_dot4_i32_i8) and fp32 accumulation (the reference
// accumulates in fp16), one fp16 rounding at the store.
//
// Mapping (wave64, no LDS): a wave owns R weight rows at a time; lane l owns "unit" u
// (64 consecutive K elements) u = l, l+64, ...  Per unit and row a lane issues 16-byte
// loads straight to registers (Q4_K: header + 32 qs bytes; Q6_K: 32 ql + 32 qh + 8
// scales + d; Q8_0: two 34-byte blocks), dequantizes nothing -- the integer codes go
// straight into dot4 against the int8 activation codes, which the lane loads once per
// unit and reuses for its R rows.  A 6-step xor-shuffle reduction per (row, token) ends
// the row group.  Loop over row groups is grid-strided.
#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"
#include "gguf_units.hpp"
#include "gguf_q8_1.hpp"

namespace gq {

namespace {

template <int F, int NT>
struct Act {
    uint32_t q[NT][16]; // int8 codes of the two activation blocks
    float d[NT][2];
    float s[NT][2];  // q8_1 s (Q4_K min term)
    int sum[NT][4];  // sum of codes per 16-element quarter (Q6_K -32 offset)
};

template <int F, int NT>
__device__ __forceinline__ void load_act(Act<F, NT> &a, const int8_t *__restrict__ xq, const float *__restrict__ xd,
                                         const float *__restrict__ xs, int64_t tok0, int64_t N, int64_t K, int u)
{
    const int64_t nb = K / 32;
    int b0, b1;
    act_blocks<F>(u, b0, b1);
    const bool has1 = b1 < nb;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int64_t tok = (tok0 + t < N) ? tok0 + t : N - 1;
        const int8_t *base = xq + tok * K;
        u32x4 c0 = ld16(base + 32 * b0), c1 = ld16(base + 32 * b0 + 16);
        u32x4 c2 = {0, 0, 0, 0}, c3 = {0, 0, 0, 0};
        if (has1) {
            c2 = ld16(base + 32 * b1);
            c3 = ld16(base + 32 * b1 + 16);
        }
        a.q[t][0] = c0.x; a.q[t][1] = c0.y; a.q[t][2] = c0.z; a.q[t][3] = c0.w;
        a.q[t][4] = c1.x; a.q[t][5] = c1.y; a.q[t][6] = c1.z; a.q[t][7] = c1.w;
        a.q[t][8] = c2.x; a.q[t][9] = c2.y; a.q[t][10] = c2.z; a.q[t][11] = c2.w;
        a.q[t][12] = c3.x; a.q[t][13] = c3.y; a.q[t][14] = c3.z; a.q[t][15] = c3.w;
        a.d[t][0] = xd[tok * nb + b0];
        a.d[t][1] = has1 ? xd[tok * nb + b1] : 0.f;
        if constexpr (F == Q4_K) {
            a.s[t][0] = xs[tok * nb + b0];
            a.s[t][1] = has1 ? xs[tok * nb + b1] : 0.f;
        }
        if constexpr (F == Q6_K) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int acc = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = dot4(a.q[t][4 * k + i], 0x01010101u, acc);
                a.sum[t][k] = acc;
            }
        }
    }
}

// Adds a loaded unit's contribution for every token into acc[t].
template <int F, int NT>
__device__ __forceinline__ void dot_unit(const UnitRaw<F> &r, const Act<F, NT> &a, float (&acc)[NT])
{
    if constexpr (F == Q8_0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            int i0 = 0, i1 = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                i0 = dot4(r.w[i], a.q[t][i], i0);
                i1 = dot4(r.w[8 + i], a.q[t][8 + i], i1);
            }
            acc[t] += r.d0 * a.d[t][0] * (float)i0 + r.d1 * a.d[t][1] * (float)i1;
        }
    } else if constexpr (F == Q4_K) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            int i0 = 0, i1 = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                i0 = dot4(r.w[i] & 0x0f0f0f0fu, a.q[t][i], i0);
                i1 = dot4((r.w[i] >> 4) & 0x0f0f0f0fu, a.q[t][8 + i], i1);
            }
            acc[t] += r.ds0 * a.d[t][0] * (float)i0 - r.dm0 * a.s[t][0] + r.ds1 * a.d[t][1] * (float)i1 -
                      r.dm1 * a.s[t][1];
        }
    } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            int a1 = 0, a2 = 0, b1 = 0, b2 = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a1 = dot4(r.ca[i], a.q[t][i], a1);
                a2 = dot4(r.ca[4 + i], a.q[t][4 + i], a2);
                b1 = dot4(r.cb[i], a.q[t][8 + i], b1);
                b2 = dot4(r.cb[4 + i], a.q[t][12 + i], b2);
            }
            a1 -= 32 * a.sum[t][0];
            a2 -= 32 * a.sum[t][1];
            b1 -= 32 * a.sum[t][2];
            b2 -= 32 * a.sum[t][3];
            acc[t] += a.d[t][0] * (r.fa1 * (float)a1 + r.fa2 * (float)a2) +
                      a.d[t][1] * (r.fb1 * (float)b1 + r.fb2 * (float)b2);
        }
    }
}

template <int F, int NT>
__device__ __forceinline__ void unit_dot(const uint8_t *__restrict__ rowp, int u, int64_t nb, const Act<F, NT> &a,
                                         float (&acc)[NT])
{
    UnitLoad<F> l;
    l.load(rowp, u, nb);
    dot_unit<F, NT>(UnitRaw<F>::from(l, u, nb), a, acc);
}

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <int F, int NT, int R>
__global__ __launch_bounds__(256) void gemv_kernel(const uint8_t *__restrict__ A, const int8_t *__restrict__ xq,
                                                   const float *__restrict__ xd, const float *__restrict__ xs,
                                                   uint16_t *__restrict__ C, int64_t M, int64_t N, int64_t K,
                                                   int64_t ldc)
{
    using L = Layout<F>;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t tok0 = (int64_t)blockIdx.y * NT;
    const int64_t nb = K / 32;
    const int64_t row_bytes = (K / L::QK) * L::BYTES;
    const int nunits = (int)((K + 63) / 64);

    for (int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * R; row0 < M; row0 += (int64_t)gridDim.x * 4 * R) {
        float acc[R][NT];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[r][t] = 0.f;

        for (int u = lane; u < nunits; u += 64) {
            Act<F, NT> a;
            load_act<F, NT>(a, xq, xd, xs, tok0, N, K, u);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int64_t row = row0 + r < M ? row0 + r : M - 1;
                unit_dot<F, NT>(A + row * row_bytes, u, nb, a, acc[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float v = wave_sum(acc[r][t]);
                if (lane == 0 && row0 + r < M && tok0 + t < N) C[(tok0 + t) * ldc + row0 + r] = f2h_bits(v);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Fused decode kernel: the workgroup quantizes its NT tokens to q8_1 straight into LDS
// (gguf_q8_1.hpp, bit-exact with q8_1.py), so a decode step is ONE launch.  Each wave
// first issues the loads of its first weight task, then joins the quantization (the
// loads are in flight meanwhile), then walks its (row group, unit slice) tasks with the
// next task's weights prefetched into registers while the current one is multiplied.
//
// LDS: codes [NT][KP] (KP = K rounded up to 64) with 16-byte pieces XOR-swizzled so the
// 16-lane ds_read_b128 groups of a unit read hit 16 distinct bank quads, then d [NT][K/32]
// and (Q4_K) s [NT][K/32] as fp32.
template <int F>
__device__ __forceinline__ int swz_piece(int p)
{
    const int x = p >> 4;
    if constexpr (F == Q6_K) return p ^ ((x & 1) | ((x & 2) << 1));
    return p ^ (x & 3);
}

template <int F, int NT>
__device__ __forceinline__ void load_act_lds(Act<F, NT> &a, const uint8_t *codes, const float *sd, const float *ss,
                                             int64_t kp, int64_t nb, int u)
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
            a.s[t][0] = ss[t * nb + b0];
            a.s[t][1] = has1 ? ss[t * nb + b1] : 0.f;
        }
        if constexpr (F == Q6_K) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int acc = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = dot4(a.q[t][4 * k + i], 0x01010101u, acc);
                a.sum[t][k] = acc;
            }
        }
    }
}

template <int F, int R>
__device__ __forceinline__ void load_rows(UnitLoad<F> (&dst)[R], const uint8_t *__restrict__ A, int64_t row_bytes,
                                          int64_t row0, int64_t M, int u, int nunits, int64_t nb)
{
    const int uu = u < nunits ? u : nunits - 1; // unconditional loads; lanes past the end are masked at use
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t row = row0 + r < M ? row0 + r : M - 1;
        dst[r].load(A + row * row_bytes, uu, nb);
    }
}

template <int F, int NT, int R>
__global__ __launch_bounds__(256) void decode_kernel(const uint8_t *__restrict__ A, const uint16_t *__restrict__ X,
                                                     int64_t ldx, uint16_t *__restrict__ C, int64_t M, int64_t N,
                                                     int64_t K, int64_t ldc)
{
    using L = Layout<F>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t tok0 = (int64_t)blockIdx.y * NT;
    const int64_t nb = K / 32;
    const int64_t kp = (K + 63) / 64 * 64;
    uint8_t *codes = smem;
    float *sd = (float *)(smem + NT * kp);
    float *ss = sd + NT * nb;
    const int64_t row_bytes = (K / L::QK) * L::BYTES;
    const int nunits = (int)((K + 63) / 64);
    const int niter = (nunits + 63) / 64;
    const int64_t ngroups = (M + R - 1) / R;
    const int64_t gstride = (int64_t)gridDim.x * 4;

    int64_t g = (int64_t)blockIdx.x * 4 + wave;
    int it = 0;
    UnitLoad<F> cur[R];
    if (g < ngroups) load_rows<F, R>(cur, A, row_bytes, g * R, M, lane, nunits, nb);

    // q8_1-quantize tokens tok0..tok0+NT-1 into LDS (8 lanes per 32-element block)
    for (int64_t blk = tid >> 3; blk < NT * nb; blk += 32) {
        const int t = (int)(blk / nb);
        const int64_t j = blk - (int64_t)t * nb;
        const int sub = tid & 7;
        uint32_t w0 = 0, w1 = 0;
        if (tok0 + t < N) {
            const u32x2 v = ld8(X + (tok0 + t) * ldx + 32 * j + 4 * sub);
            w0 = v.x;
            w1 = v.y;
        }
        const Q81Lane q = q8_1_lane(w0, w1);
        const int e = (int)(32 * j + 4 * sub);
        *(uint32_t *)(codes + t * kp + 16 * swz_piece<F>(e >> 4) + (e & 15)) = q.codes;
        if (sub == 0) {
            sd[t * nb + j] = q.d;
            if constexpr (F == Q4_K) ss[t * nb + j] = h2f(q.sbits);
        }
    }
    __syncthreads();

    float acc[R][NT];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[r][t] = 0.f;

    while (g < ngroups) {
        int64_t g2 = g;
        int it2 = it + 1;
        if (it2 == niter) {
            it2 = 0;
            g2 += gstride;
        }
        UnitLoad<F> nxt[R];
        load_rows<F, R>(nxt, A, row_bytes, (g2 < ngroups ? g2 : g) * R, M, lane + 64 * it2, nunits, nb);
        const int u = lane + 64 * it;
        if (u < nunits) {
            Act<F, NT> a;
            load_act_lds<F, NT>(a, codes, sd, ss, kp, nb, u);
#pragma unroll
            for (int r = 0; r < R; ++r) dot_unit<F, NT>(UnitRaw<F>::from(cur[r], u, nb), a, acc[r]);
        }
        if (it2 == 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const float v = wave_sum(acc[r][t]);
                    acc[r][t] = 0.f;
                    if (lane == 0 && g * R + r < M && tok0 + t < N) C[(tok0 + t) * ldc + g * R + r] = f2h_bits(v);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) cur[r] = nxt[r];
        g = g2;
        it = it2;
    }
}

template <int F, int NT, int R>
hipError_t launch_decode(const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, int64_t M, int64_t N,
                         int64_t K, int64_t ldc, size_t lds, hipStream_t s)
{
    const int64_t groups = (M + R - 1) / R;
    const int64_t wgs = (groups + 3) / 4;
    const int64_t cap = 512;
    dim3 grid((unsigned)(wgs < cap ? wgs : cap), (unsigned)((N + NT - 1) / NT)), block(256);
    decode_kernel<F, NT, R><<<grid, block, lds, s>>>(A, X, ldx, C, M, N, K, ldc);
    return hipGetLastError();
}

template <int F>
constexpr int decode_rows() { return F == Q4_K ? 4 : 2; }

template <int F>
hipError_t decode_fmt(const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, int64_t M, int64_t N, int64_t K,
                      int64_t ldc, hipStream_t s)
{
    const int nt = N == 1 ? 1 : (N == 2 ? 2 : 4);
    const size_t lds = decode_lds_bytes(F, nt, K);
    if (nt == 1) return launch_decode<F, 1, decode_rows<F>()>(A, X, ldx, C, M, N, K, ldc, lds, s);
    if (nt == 2) return launch_decode<F, 2, decode_rows<F>()>(A, X, ldx, C, M, N, K, ldc, lds, s);
    return launch_decode<F, 4, 2>(A, X, ldx, C, M, N, K, ldc, lds, s);
}

template <int F, int NT, int R>
hipError_t launch_one(const uint8_t *A, const int8_t *xq, const float *xd, const float *xs, uint16_t *C, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    const int64_t groups = (M + 4 * R - 1) / (4 * R);
    const int64_t cap = 2048;
    dim3 grid((unsigned)(groups < cap ? groups : cap), (unsigned)((N + NT - 1) / NT)), block(256);
    gemv_kernel<F, NT, R><<<grid, block, 0, s>>>(A, xq, xd, xs, C, M, N, K, ldc);
    return hipGetLastError();
}

template <int F>
hipError_t launch_fmt(const uint8_t *A, const int8_t *xq, const float *xd, const float *xs, uint16_t *C, int64_t M,
                      int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (N == 1) return launch_one<F, 1, 4>(A, xq, xd, xs, C, M, N, K, ldc, s);
    if (N == 2) return launch_one<F, 2, 4>(A, xq, xd, xs, C, M, N, K, ldc, s);
    return launch_one<F, 4, 2>(A, xq, xd, xs, C, M, N, K, ldc, s);
}

} // namespace

size_t decode_lds_bytes(int fmt, int nt, int64_t K)
{
    const int64_t kp = (K + 63) / 64 * 64, nb = K / 32;
    return (size_t)nt * kp + (size_t)nt * nb * 4 * (fmt == Q4_K ? 2 : 1);
}

bool decode_fused_ok(int fmt, int64_t N, int64_t K)
{
    const int nt = N == 1 ? 1 : (N == 2 ? 2 : 4);
    return N <= 8 && decode_lds_bytes(fmt, nt, K) <= 64 * 1024;
}

hipError_t launch_decode_fused(int fmt, const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, int64_t M,
                               int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (fmt) {
    case Q8_0: return decode_fmt<Q8_0>(A, X, ldx, C, M, N, K, ldc, s);
    case Q4_K: return decode_fmt<Q4_K>(A, X, ldx, C, M, N, K, ldc, s);
    default: return decode_fmt<Q6_K>(A, X, ldx, C, M, N, K, ldc, s);
    }
}

hipError_t launch_gemv(int fmt, const uint8_t *A, const int8_t *xq, const float *xd, const float *xs, uint16_t *C,
                       int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    switch (fmt) {
    case Q8_0: return launch_fmt<Q8_0>(A, xq, xd, xs, C, M, N, K, ldc, s);
    case Q4_K: return launch_fmt<Q4_K>(A, xq, xd, xs, C, M, N, K, ldc, s);
    default: return launch_fmt<Q6_K>(A, xq, xd, xs, C, M, N, K, ldc, s);
    }
}

} // namespace gq
