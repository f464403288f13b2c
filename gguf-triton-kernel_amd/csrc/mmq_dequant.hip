// mmq_dequant.hip -- GGUF -> fp16 dequantization and the library-GEMM path for many tokens.
//
// dequant_kernel<F, PERM>: W[m][k] = fp16(w), the reference's block formulas in fp32
//   Q8_0 w = d*q                                   (utils/quantize/q8_0.py:52-100)
//   Q4_K w = d*sc_j*q - dmin*m_j                   (q4_k_ref.c:358-364, q4_k.py:125-158)
//   Q6_K w = d*sc_{e/16}*(q - 32)                  (q6_k_ref.c:320-336, q6_k.py:117-159)
// one thread per 32-element sub-block, 4 x 16-byte stores.  PERM stores each 4-element group
// in the order (0,2,1,3) -- the order act_quant's DEQ form uses for x~ -- so a GEMM over
// (W_perm, x~) sums the same products as over the natural order.
//
// blas_gemm(): C[n][m] = sum_k W[m][k] * x~[n][k] on hipBLASLt (fp16 in, fp32 compute, fp16
// out): the plain-library GEMM SURVEY.md 8(f)3 names for N_tok >= a few hundred, where a
// dense fp16 GEMM over a dequantized copy of W beats re-streaming the packed blocks once per
// 128-token tile.  Handles and heuristics are created on first use per device and shape (do
// that outside hipGraph capture); the call itself only enqueues work on `stream`.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"

namespace gq {

namespace {

__device__ __forceinline__ void store32(uint16_t *dst, const float (&w)[32], bool perm)
{
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        uint32_t o[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int b = 8 * p + 4 * h;
            const float a0 = w[b], a1 = perm ? w[b + 2] : w[b + 1], a2 = perm ? w[b + 1] : w[b + 2], a3 = w[b + 3];
            o[2 * h] = (uint32_t)f2h_bits(a0) | ((uint32_t)f2h_bits(a1) << 16);
            o[2 * h + 1] = (uint32_t)f2h_bits(a2) | ((uint32_t)f2h_bits(a3) << 16);
        }
        *(u32x4 *)(dst + 8 * p) = (u32x4){o[0], o[1], o[2], o[3]};
    }
}

template <int F, bool PERM>
__global__ __launch_bounds__(256) void dequant_kernel(const uint8_t *__restrict__ A, uint16_t *__restrict__ W,
                                                      int64_t M, int64_t K, int64_t ldw)
{
    using L = Layout<F>;
    const int64_t nsub = K / 32; // 32-element sub-blocks per row
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= M * nsub) return;
    const int64_t row = idx / nsub, j = idx - row * nsub;
    const uint8_t *rowp = A + row * (K / L::QK) * L::BYTES;
    // 16-byte vector loads of the sub-block's fields (global memory runs unaligned on gfx950)
    float w[32];
    if constexpr (F == Q8_0) {
        const uint8_t *b = rowp + 34 * j;
        const float d = h2f(ld2(b));
        const u32x4 q0 = ld16(b + 2), q1 = ld16(b + 18);
        const uint32_t qw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int i = 0; i < 32; ++i) w[i] = d * (float)(int8_t)byte_of(qw[i >> 2], i & 3);
    } else if constexpr (F == Q4_K) {
        const uint8_t *b = rowp + 144 * (j >> 3);
        const int s = (int)(j & 7);
        const u32x4 hdr = ld16(b);
        const float d = h2f(hdr.x & 0xffffu), dmin = h2f(hdr.x >> 16);
        const uint32_t sw[3] = {hdr.y, hdr.z, hdr.w};
        int sc, m;
        q4k_sc_m(sw, s, sc, m);
        const float ds = d * (float)sc, dm = dmin * (float)m;
        const u32x4 q0 = ld16(b + 16 + 32 * (s >> 1)), q1 = ld16(b + 32 + 32 * (s >> 1));
        const uint32_t qw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const int sh = 4 * (s & 1);
#pragma unroll
        for (int i = 0; i < 32; ++i) w[i] = ds * (float)((byte_of(qw[i >> 2], i & 3) >> sh) & 0xf) - dm;
    } else {
        // run jj = j & 7 of the super-block: elements 32*jj + i, i < 32 -> half h = jj >> 2,
        // ql bytes 64h + 32*(jj & 1) (nibble 4*((jj >> 1) & 1)), qh bytes 32h (bits 2*(jj & 3))
        const uint8_t *b = rowp + 210 * (j >> 3);
        const int jj = (int)(j & 7), h = jj >> 2;
        const float d = h2f(ld2(b + 208));
        const u32x4 l0 = ld16(b + 64 * h + 32 * (jj & 1)), l1 = ld16(b + 64 * h + 32 * (jj & 1) + 16);
        const u32x4 g0 = ld16(b + 128 + 32 * h), g1 = ld16(b + 144 + 32 * h);
        const uint32_t lw[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
        const uint32_t gw[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        const uint32_t scw = ld2(b + 192 + 2 * jj);
        const float s0 = d * (float)(int8_t)(scw & 0xff), s1 = d * (float)(int8_t)(scw >> 8);
        const int shl = 4 * ((jj >> 1) & 1), shh = 2 * (jj & 3);
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int lo = (byte_of(lw[i >> 2], i & 3) >> shl) & 0xf;
            const int hi = (byte_of(gw[i >> 2], i & 3) >> shh) & 3;
            w[i] = (i < 16 ? s0 : s1) * (float)((lo | (hi << 4)) - 32);
        }
    }
    store32(W + row * ldw + 32 * j, w, PERM);
}

template <bool PERM>
hipError_t dequant_perm(int fmt, const uint8_t *A, uint16_t *W, int64_t M, int64_t K, int64_t ldw, hipStream_t s)
{
    const int64_t n = M * (K / 32);
    if (n == 0) return hipSuccess;
    dim3 grid((unsigned)((n + 255) / 256)), block(256);
    switch (fmt) {
    case Q8_0: dequant_kernel<Q8_0, PERM><<<grid, block, 0, s>>>(A, W, M, K, ldw); break;
    case Q4_K: dequant_kernel<Q4_K, PERM><<<grid, block, 0, s>>>(A, W, M, K, ldw); break;
    default: dequant_kernel<Q6_K, PERM><<<grid, block, 0, s>>>(A, W, M, K, ldw); break;
    }
    return hipGetLastError();
}

// ---- hipBLASLt plans, cached per (device, M, N, K, ldc) ----
struct Plan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
    hipblasLtMatmulAlgo_t algo{};
    size_t ws = 0;
};

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<std::tuple<int, int64_t, int64_t, int64_t, int64_t>, Plan> g_plans;

bool get_plan(int dev, int64_t M, int64_t N, int64_t K, int64_t ldc, size_t ws_max, hipblasLtHandle_t &h, Plan &out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    auto hit = g_handles.find(dev);
    if (hit == g_handles.end()) {
        hipblasLtHandle_t nh;
        if (hipblasLtCreate(&nh) != HIPBLAS_STATUS_SUCCESS) return false;
        hit = g_handles.emplace(dev, nh).first;
    }
    h = hit->second;
    const auto key = std::make_tuple(dev, M, N, K, ldc);
    auto pit = g_plans.find(key);
    if (pit != g_plans.end()) {
        out = pit->second;
        return out.ws <= ws_max;
    }
    Plan p;
    // column-major view: D (M x N, ld ldc) = op_T(W: K x M, ld K) * x~ (K x N, ld K)
    hipblasOperation_t tA = HIPBLAS_OP_T, tB = HIPBLAS_OP_N;
    if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &tA, sizeof(tA));
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tB, sizeof(tB));
    hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16F, (uint64_t)K, (uint64_t)M, K);
    hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16F, (uint64_t)K, (uint64_t)N, K);
    hipblasLtMatrixLayoutCreate(&p.c, HIP_R_16F, (uint64_t)M, (uint64_t)N, ldc);
    hipblasLtMatmulPreference_t pref;
    hipblasLtMatmulPreferenceCreate(&pref);
    uint64_t wsz = ws_max;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz));
    hipblasLtMatmulHeuristicResult_t res[1];
    int n = 0;
    const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.c, p.c, pref, 1, res, &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || n < 1) return false;
    p.algo = res[0].algo;
    p.ws = res[0].workspaceSize;
    g_plans.emplace(key, p);
    out = p;
    return true;
}

} // namespace

hipError_t launch_dequant(int fmt, const uint8_t *A, uint16_t *W, int64_t M, int64_t K, int64_t ldw, bool perm,
                          hipStream_t s)
{
    return perm ? dequant_perm<true>(fmt, A, W, M, K, ldw, s) : dequant_perm<false>(fmt, A, W, M, K, ldw, s);
}

size_t blas_workspace_bytes() { return (size_t)32 << 20; }

int blas_gemm(const uint16_t *W, const uint16_t *X, uint16_t *C, int64_t M, int64_t N, int64_t K, int64_t ldc,
              void *ws, size_t ws_bytes, hipStream_t s)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    hipblasLtHandle_t h;
    Plan p;
    if (!get_plan(dev, M, N, K, ldc, ws_bytes, h, p)) return -2;
    const float alpha = 1.f, beta = 0.f;
    const hipblasStatus_t st =
        hipblasLtMatmul(h, p.desc, &alpha, W, p.a, X, p.b, &beta, C, p.c, C, p.c, &p.algo, ws, p.ws, s);
    return st == HIPBLAS_STATUS_SUCCESS ? 0 : -3;
}

} // namespace gq
