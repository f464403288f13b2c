// gguf_cpu_mmq.cpp -- host MMQ with the reference CPU implementations' exact arithmetic.
//
// Drop-in backend for the reference's CPU products (kernels/cpu_impls):
//   mmq_q8_0_q8_1_cpu  kernels/cpu_impls/mmq_q8_0_q8_1_cpu.py:5-56
//   mmq_q4_k_q8_1_cpu  kernels/cpu_impls/mmq_q4_k_q8_1_cpu.py:61-119
//   mmq_q6_k_q8_1_cpu  kernels/cpu_impls/mmq_q6_k_q8_1_cpu.py:84-152
// Those loop (m, n, block) in Python and add every block's term into an fp16 C[m, n]
// (`C[m, n] += term.item()`); the value of every output therefore depends on the order
// and the fp16/fp32 roundings of that chain, and this file keeps both:
//   Q8_0: term = fp16(fp16(dA*dB) * idot)                 (fp16 tensor * int32 tensor)
//   Q4_K: term = ((d*sc)*dB)*idot - (dmin*m)*sB  in fp32   (the scalar is cast to fp16 first)
//   Q6_K: term = dB*((d*sc_lo)*dot_lo + (d*sc_hi)*dot_hi) in fp32
//   C = fp16(float(C) + float(fp16(term)))
// (build with -ffp-contract=off: no fused multiply-adds).
//
// Layout of the work: a weight row is unpacked ONCE into int8 codes plus its per-32-block
// scale terms, then every token's row of q8_1 blocks is swept against it (the int8 dots
// vectorise); rows are split over threads.  Outputs do not depend on the thread count.
// The GPU product path never calls this (it has no CPU fallback); it exists because the
// reference ships these CPU functions as part of its API.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../gguf_half.hpp"

namespace {

using gq::f2h;
using gq::h2f;

inline uint16_t ld16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// fp16 -> fp32 by table (the conversion is on the innermost chain)
struct HalfTable {
    float v[65536];
    HalfTable()
    {
        for (uint32_t i = 0; i < 65536; ++i) v[i] = h2f((uint16_t)i);
    }
};
const HalfTable &half_table()
{
    static const HalfTable t;
    return t;
}

inline int32_t dot32(const int8_t *a, const int8_t *b, int n)
{
    int32_t s = 0;
    for (int i = 0; i < n; ++i) s += (int32_t)a[i] * (int32_t)b[i];
    return s;
}

// One weight row, unpacked: codes[K] (int8) and per-32-block constants.
struct Row {
    std::vector<int8_t> q;
    std::vector<float> c0, c1; // Q8_0: dA (fp16 bits in c0 as float); Q4_K: d*sc, dmin*m; Q6_K: d*sc_lo, d*sc_hi
    std::vector<uint16_t> h;   // Q8_0: dA fp16 bits
};

void unpack_q8_0(const uint8_t *row, int64_t K, Row &r)
{
    const int64_t nb = K / 32;
    for (int64_t j = 0; j < nb; ++j) {
        const uint8_t *b = row + 34 * j;
        r.h[j] = ld16(b);
        std::memcpy(&r.q[32 * j], b + 2, 32);
    }
}

void unpack_q4_k(const uint8_t *row, int64_t K, Row &r)
{
    const auto &T = half_table();
    for (int64_t sb = 0; sb < K / 256; ++sb) {
        const uint8_t *b = row + 144 * sb;
        const float d = T.v[ld16(b)], dmin = T.v[ld16(b + 2)];
        const uint8_t *s = b + 4, *qs = b + 16;
        for (int j = 0; j < 8; ++j) {
            int sc, mn; // get_scale_min_k4 (mmq_q4_k_q8_1_cpu.py:33-56)
            if (j < 4) {
                sc = s[j] & 63;
                mn = s[j + 4] & 63;
            } else {
                sc = (s[j + 4] & 0x0f) | ((s[j - 4] >> 6) << 4);
                mn = (s[j + 4] >> 4) | ((s[j] >> 6) << 4);
            }
            r.c0[8 * sb + j] = d * (float)sc;
            r.c1[8 * sb + j] = dmin * (float)mn;
            const uint8_t *src = qs + 32 * (j >> 1);
            int8_t *dst = &r.q[256 * sb + 32 * j];
            for (int i = 0; i < 32; ++i) dst[i] = (int8_t)((j & 1) ? (src[i] >> 4) : (src[i] & 0x0f));
        }
    }
}

void unpack_q6_k(const uint8_t *row, int64_t K, Row &r)
{
    const auto &T = half_table();
    for (int64_t sb = 0; sb < K / 256; ++sb) {
        const uint8_t *b = row + 210 * sb;
        const uint8_t *ql = b, *qh = b + 128;
        const int8_t *sc = (const int8_t *)(b + 192);
        const float d = T.v[ld16(b + 208)];
        for (int j = 0; j < 8; ++j) {
            r.c0[8 * sb + j] = d * (float)sc[2 * j];
            r.c1[8 * sb + j] = d * (float)sc[2 * j + 1];
        }
        int8_t *dst = &r.q[256 * sb];
        for (int half = 0; half < 2; ++half)        // 128-element halves
            for (int e = 0; e < 128; ++e) {         // element 128*half + e
                const int lo = (ql[64 * half + (e & 63)] >> (4 * (e >> 6))) & 0x0f;
                const int hi = (qh[32 * half + (e & 31)] >> (2 * (e >> 5))) & 0x03;
                dst[128 * half + e] = (int8_t)((lo | (hi << 4)) - 32);
            }
    }
}

// Token n's q8_1 row: codes and the fp16 d / s of each 32-block.
struct Act {
    std::vector<int8_t> q;
    std::vector<uint16_t> d, s;
};

Act unpack_act(const uint8_t *B, int64_t N, int64_t K)
{
    const int64_t nb = K / 32;
    Act a;
    a.q.resize((size_t)(N * K));
    a.d.resize((size_t)(N * nb));
    a.s.resize((size_t)(N * nb));
    for (int64_t i = 0; i < N * nb; ++i) {
        const uint8_t *b = B + 36 * i;
        a.d[i] = ld16(b);
        a.s[i] = ld16(b + 2);
        std::memcpy(&a.q[32 * i], b + 4, 32);
    }
    return a;
}

// C[m][n] (fp16 bits, (M, N) row-major) for rows [m0, m1)
void rows_q8_0(const uint8_t *A, const Act &x, int64_t m0, int64_t m1, int64_t N, int64_t K, uint16_t *C)
{
    const auto &T = half_table();
    const int64_t nb = K / 32, row_bytes = nb * 34;
    Row r;
    r.q.resize((size_t)K);
    r.h.resize((size_t)nb);
    for (int64_t m = m0; m < m1; ++m) {
        unpack_q8_0(A + m * row_bytes, K, r);
        for (int64_t n = 0; n < N; ++n) {
            const int8_t *xq = &x.q[n * K];
            const uint16_t *xd = &x.d[n * nb];
            uint16_t c = 0;
            for (int64_t j = 0; j < nb; ++j) {
                const int32_t idot = dot32(&r.q[32 * j], xq + 32 * j, 32);
                const uint16_t dd = f2h(T.v[r.h[j]] * T.v[xd[j]]);
                const uint16_t p = f2h(T.v[dd] * (float)idot);
                c = f2h(T.v[c] + T.v[p]);
            }
            C[m * N + n] = c;
        }
    }
}

void rows_q4_k(const uint8_t *A, const Act &x, int64_t m0, int64_t m1, int64_t N, int64_t K, uint16_t *C)
{
    const auto &T = half_table();
    const int64_t nb = K / 32, row_bytes = (K / 256) * 144;
    Row r;
    r.q.resize((size_t)K);
    r.c0.resize((size_t)nb);
    r.c1.resize((size_t)nb);
    for (int64_t m = m0; m < m1; ++m) {
        unpack_q4_k(A + m * row_bytes, K, r);
        for (int64_t n = 0; n < N; ++n) {
            const int8_t *xq = &x.q[n * K];
            const uint16_t *xd = &x.d[n * nb], *xs = &x.s[n * nb];
            uint16_t c = 0;
            for (int64_t j = 0; j < nb; ++j) {
                const int32_t idot = dot32(&r.q[32 * j], xq + 32 * j, 32);
                const float t = (r.c0[j] * T.v[xd[j]]) * (float)idot - r.c1[j] * T.v[xs[j]];
                c = f2h(T.v[c] + T.v[f2h(t)]);
            }
            C[m * N + n] = c;
        }
    }
}

void rows_q6_k(const uint8_t *A, const Act &x, int64_t m0, int64_t m1, int64_t N, int64_t K, uint16_t *C)
{
    const auto &T = half_table();
    const int64_t nb = K / 32, row_bytes = (K / 256) * 210;
    Row r;
    r.q.resize((size_t)K);
    r.c0.resize((size_t)nb);
    r.c1.resize((size_t)nb);
    for (int64_t m = m0; m < m1; ++m) {
        unpack_q6_k(A + m * row_bytes, K, r);
        for (int64_t n = 0; n < N; ++n) {
            const int8_t *xq = &x.q[n * K];
            const uint16_t *xd = &x.d[n * nb];
            uint16_t c = 0;
            for (int64_t j = 0; j < nb; ++j) {
                const int32_t lo = dot32(&r.q[32 * j], xq + 32 * j, 16);
                const int32_t hi = dot32(&r.q[32 * j + 16], xq + 32 * j + 16, 16);
                const float t = T.v[xd[j]] * (r.c0[j] * (float)lo + r.c1[j] * (float)hi);
                c = f2h(T.v[c] + T.v[f2h(t)]);
            }
            C[m * N + n] = c;
        }
    }
}

} // namespace

extern "C" {

// C (M, N) fp16 bits = the reference CPU MMQ of packed weights A (type 0 Q8_0, 1 Q4_K,
// 2 Q6_K) and packed q8_1 activations B.  threads <= 0: all hardware threads.
// Returns 0, or -1 for an unknown type / K not a whole number of blocks.
int gq_cpu_mmq(int type, const void *A, const void *B, int64_t M, int64_t N, int64_t K, uint16_t *C, int threads)
{
    const int qk = type == 0 ? 32 : 256;
    if (type < 0 || type > 2 || K <= 0 || K % qk != 0 || M < 0 || N < 0) return -1;
    if (M == 0 || N == 0) return 0;
    half_table();
    const Act x = unpack_act((const uint8_t *)B, N, K);
    auto run = [&](int64_t m0, int64_t m1) {
        if (type == 0) rows_q8_0((const uint8_t *)A, x, m0, m1, N, K, C);
        else if (type == 1) rows_q4_k((const uint8_t *)A, x, m0, m1, N, K, C);
        else rows_q6_k((const uint8_t *)A, x, m0, m1, N, K, C);
    };
    int64_t nt = threads > 0 ? threads : (int64_t)std::max(1u, std::thread::hardware_concurrency());
    nt = std::max<int64_t>(1, std::min<int64_t>(nt, M));
    if (nt == 1) {
        run(0, M);
        return 0;
    }
    std::vector<std::thread> pool;
    const int64_t per = (M + nt - 1) / nt;
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t m0 = t * per, m1 = std::min(M, m0 + per);
        if (m0 < m1) pool.emplace_back(run, m0, m1);
    }
    for (auto &th : pool) th.join();
    return 0;
}

} // extern "C"
