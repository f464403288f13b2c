// gq_capi.hip -- the C ABI (include/gguf_mmq.h): argument checks, workspace carving,
// path selection (decode GEMV vs MFMA GEMM) and launches.  Stateless and re-entrant.
#include <climits>
#include <cstdio>
#include <dlfcn.h>
#include <mutex>
#include <cstdarg>
#include <cstdlib>
#include <string>

#include <rccl/rccl.h> // types only: the entry point is resolved at run time (shard_allgather)

#include "../../include/gguf_mmq.h"
#include "gguf_blocks.hpp"
#include "gguf_internal.hpp"

namespace gq {
namespace {

Tuning g_tuning;
std::once_flag g_tuning_once;

bool parse_key(Tuning &t, const char *key, long long v)
{
    auto in = [&](std::initializer_list<long long> ok) {
        for (long long o : ok)
            if (v == o) return true;
        return false;
    };
    const std::string k = key;
    if (k == "GQ_BLAS_MIN_TOKENS") t.blas_min_tokens = v;
    else if (k == "GQ_GEMM_MAX_BYTES") {
        if (v <= 0) return false;
        t.gemm_max_bytes = v < (1LL << 31) ? v : (1LL << 31);
    } else if (k == "GQ_GEMM_I8") t.gemm_i8 = v != 0;
    else if (k == "GQ_NO_FUSED_DECODE") t.fused_decode = v == 0;
    else if (k == "GQ_DECODE_F8_ITC") t.decode_f8_itc = v != 0;
    else if (k == "GQ_SGEMM_STREAMK") t.sgemm_streamk = v < 0 ? -1 : (v != 0);
    else if (k == "GQ_DECODE_Q6_IMG") {
        if (!in({-1, 0, 1})) return false;
        t.decode_q6_img = (int)v;
    }
    else if (k == "GQ_GEMM_AQ") t.gemm_aq = v != 0;
    else if (k == "GQ_GEMM_RG") {
        if (!in({0, 1, 2})) return false;
        t.gemm_rg = (int)v;
    } else if (k == "GQ_GEMM_SPLITS") {
        if (v < 0) return false;
        t.gemm_splits = v;
    } else if (k == "GQ_GEMM_PARTIAL") t.gemm_partial_f32 = v != 0; // 1 = f32
    else if (k == "GQ_SKINNY") {
        if (!in({-1, 0, 1})) return false;
        t.skinny = (int)v;
    } else if (k == "GQ_SKINNY_RG") {
        if (!in({0, 1, 2, 3, 4})) return false;
        t.skinny_rg = (int)v;
    } else if (k == "GQ_RGEMM") {
        if (!in({-1, 0, 1})) return false;
        t.rgemm = (int)v;
    } else if (k == "GQ_SGEMM") {
        if (!in({-1, 0, 1})) return false;
        t.sgemm = (int)v;
    } else if (k == "GQ_SGEMM_SPLITS") {
        if (v < 0 || v > 4096) return false;
        t.sgemm_splits = (int)v;
    } else if (k == "GQ_RGEMM_ILC") t.rgemm_ilc = v != 0;
    else if (k == "GQ_SGEMM_FULL") {
        t.sgemm_full = v < 0 ? -1 : (v != 0);
    } else if (k == "GQ_CUS") {
        if (v < 0 || v > 1024) return false;
        t.cus = (int)v;
    } else if (k == "GQ_KSTREAM") {
        if (!in({-1, 0, 1})) return false;
        t.kstream = (int)v;
    } else if (k == "GQ_ABLATE") t.ablate = (int)v;
    else return false;
    return true;
}

void tuning_from_env(Tuning &t)
{
    t = Tuning{};
    static const char *const keys[] = {"GQ_BLAS_MIN_TOKENS", "GQ_GEMM_MAX_BYTES", "GQ_GEMM_I8", "GQ_NO_FUSED_DECODE",
                                       "GQ_DECODE_Q6_IMG", "GQ_DECODE_F8_ITC", "GQ_GEMM_AQ", "GQ_GEMM_RG", "GQ_GEMM_SPLITS",
                                       "GQ_GEMM_PARTIAL", "GQ_SKINNY", "GQ_SKINNY_RG", "GQ_RGEMM", "GQ_SGEMM",
                                       "GQ_SGEMM_SPLITS", "GQ_SGEMM_STREAMK", "GQ_RGEMM_ILC", "GQ_SGEMM_FULL", "GQ_CUS",
                                       "GQ_KSTREAM", "GQ_ABLATE"};
    for (const char *k : keys) {
        const char *e = getenv(k); // the only getenv of the library: once per process
        if (!e || !*e) continue;
        long long v;
        if (std::string(k) == "GQ_GEMM_PARTIAL") v = std::string(e) == "f32";
        else v = atoll(e);
        if (!parse_key(t, k, v)) fprintf(stderr, "gguf_mmq: ignoring %s=%s (out of range)\n", k, e);
    }
}

} // namespace

const Tuning &tuning()
{
    std::call_once(g_tuning_once, [] { tuning_from_env(g_tuning); });
    return g_tuning;
}

int set_tuning(const char *key, long long value)
{
    tuning();
    Tuning t = g_tuning;
    if (!key || !parse_key(t, key, value)) return -1;
    g_tuning = t;
    return 0;
}

void reset_tuning()
{
    tuning();
    Tuning t;
    tuning_from_env(t); // built aside and published by one assignment, as set_tuning does
    g_tuning = t;
}

int num_cus()
{
    if (tuning().cus > 0) return tuning().cus; // test override (GQ_CUS)
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (cached[dev] <= 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    return cached[dev];
}

} // namespace gq

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int block_elems(int t) { return t == GQ_Q8_0 ? 32 : 256; }
int block_bytes(int t) { return t == GQ_Q8_0 ? 34 : (t == GQ_Q4_K ? 144 : 210); }

size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

// Decode path up to this many tokens; beyond it the fp16-MFMA GEMM.
constexpr int64_t kGemvMaxTokens = 4; // 5..8 tokens: the MFMA GEMM (15.9 us at 16 tokens vs 22.3 us decode at 8, Q4_K 4096^2)

// (K % 128 != 0 is only possible for Q8_0, so the choice depends on N and K alone and
// gq_act_prepare, which does not know the weight type, makes the same one.)
bool use_gemv(int64_t N, int64_t K) { return N <= kGemvMaxTokens || !gq::gemm_supported(gq::Q8_0, K); }

// Library-GEMM path (dequantize W to fp16 + hipBLASLt) from this many tokens on; the
// override GQ_BLAS_MIN_TOKENS (0 = never) is for tuning and tests.
int64_t blas_min_tokens()
{
    // default 768: measured crossover (11008x4096 Q4_K 512 tokens 90 vs 121 us, 4096^2 1024 tokens)
    const long long v = gq::tuning().blas_min_tokens;
    return v <= 0 ? INT64_MAX : (int64_t)v;
}
bool use_blas(int64_t N, int64_t K) { return !use_gemv(N, K) && N >= blas_min_tokens(); }

// Q8_0 on the MFMA GEMM path: int8 activations x int8 weights (v_mfma_i32_16x16x32_i8 + per-block
// fp32 scaling) instead of fp16 x~ x dequantized weights.  GQ_GEMM_I8=0/1 overrides.
// The MFMA GEMM addresses its operands with 32-bit buffer offsets: one launch covers at most
// this many weight bytes and this many activation bytes; gemm_chunks() cuts larger calls into
// row / token chunks (launched back to back on the stream, reusing the workspace).
// (GQ_GEMM_MAX_BYTES lowers the limit: tests cut small calls into many chunks.)
int64_t gemm_max_bytes()
{
    const int64_t lim = (int64_t)1 << 31;
    const int64_t v = gq::tuning().gemm_max_bytes;
    return v > 0 && v < lim ? v : lim;
}
int64_t row_bytes_of(int t, int64_t K) { return (K / block_elems(t)) * block_bytes(t); }
int64_t gemm_rows_per_launch(int t, int64_t M, int64_t K)
{
    const int64_t r = gemm_max_bytes() / row_bytes_of(t, K) / 256 * 256; // whole 256-row tiles
    return r < 256 ? 256 : (r < M ? r : M);
}
int64_t gemm_toks_per_launch(int64_t N, int64_t K)
{
    const int64_t n = gemm_max_bytes() / (2 * K) / 128 * 128; // whole 128-token tiles
    return n < 16 ? 16 : (n < N ? n : N);
}

constexpr int64_t kRgemmMinTokens = 5, kRgemmMultiRoundTokens = 32, kRgemmMultiRoundTokensQ4 = 64;
// Skinny-token kernel (mmq_skinny.hip).  By type and token count only (a row subset runs the
// same arithmetic as the whole matrix): by default Q4_K and Q8_0 at 5..16 tokens, where it
// measured faster than the LDS-DMA GEMM (profiles/r03/tails/route_sw.log, step incl. act_quant,
// 16 tokens: Q4_K 4096^2 9.7 vs 12.0 us, 11008x4096 15.3 vs 22.2, 4096x11008 16.5 vs 19.6; Q8_0
// 4096^2 11.3 vs 13.1, 11008x4096 19.4 vs 24.3).  Q6_K stays on the GEMM: faster on 4096-row
// matrices (11.6 vs 13.0) but 28672x8192 72 vs 95, and the choice may not depend on M; 17..32
// tokens: mixed (Q4_K +8% / -5% by shape), the GEMM.  GQ_SKINNY=1: every type at 1..32 tokens
// the GEMM path would take (tests), 0: off.
constexpr int64_t kSkinnyMinTokens = 5, kSkinnyMaxTokens = 16, kSkinnyForcedMax = 32;
bool use_skinny(int t, int form, int64_t N, int act = GQ_ACT_Q8_1)
{
    const int sk = gq::tuning().skinny;
    if (form != gq::AF_F16 || sk == 0) return false;
    if (sk == 1) return N <= kSkinnyForcedMax;
    // the fp8 variant has no decode kernel: its 1..4 tokens take the skinny kernel too
    const int64_t lo = act == GQ_ACT_FP8_E4M3 ? 1 : kSkinnyMinTokens;
    return (t == GQ_Q4_K || t == GQ_Q8_0) && N >= lo && N <= kSkinnyMaxTokens;
}
gq::SkinnyPlan skinny_plan(int t, int64_t M, int64_t N, int64_t K)
{
    const gq::Tuning &tu = gq::tuning();
    return gq::plan_skinny(t, M, N, K, tu.skinny_rg, 0);
}

// Resident-split GEMM (mmq_rgemm.hip: 256 rows x <= 128 tokens x one super-block per workgroup,
// the split's operands loaded once; profiles/r04/).  By default where its grid is one round of
// the chip and at least half of it (a 4096-row matrix at K = 4096: 16 x 16 workgroups) and the
// call needs no 2 GiB chunking; the q8_1 activations are quantized inside it (gq_mmq_ex) or read
// prepared (gq_mmq_prepared).  With split-K over every super-block its partial sums differ from
// gemm_kernel's (other splits), so a forced split factor (GQ_GEMM_SPLITS) keeps gemm_kernel.
// GQ_RGEMM=1: wherever it applies (tests), 0: off.
// A knob of the LDS-DMA GEMM set (tests, A/B of those kernels): the automatic
// resident / streaming routes stand aside so the call reaches the kernel the knob is for.
bool gemm_knob_pinned()
{
    const gq::Tuning &u = gq::tuning();
    return u.gemm_splits > 0 || u.gemm_rg || u.gemm_partial_f32;
}

bool use_rgemm(int t, int form, int64_t M, int64_t N, int64_t K)
{
    const int rg = gq::tuning().rgemm;
    if (rg == 0 || form != gq::AF_F16 || use_gemv(N, K) || use_blas(N, K) || K % 256 != 0) return false;
    if (gemm_rows_per_launch(t, M, K) < M || gemm_toks_per_launch(N, K) < N) return false;
    const gq::RGemmPlan p = gq::plan_rgemm(M, N, K);
    if (!p.ok) return false;
    if (rg == 1) return true;
    if (gemm_knob_pinned() || N < kRgemmMinTokens) return false;
    // one round of the chip at the workgroups a CU holds (Q4_K at 16 tokens: three -- 11008x4096
    // and 4096x11008 at 688 workgroups); up to 32 tokens, up to four rounds (the one-super-block
    // workgroups are short, so later rounds fill in behind the first; step us, default route ->
    // resident, profiles/r04/b6_rg2.txt: Q4_K 22016x4096 x16 27.4 -> 21.6, x8 26.5 -> 20.9,
    // 14336x4096 x16 18.3 -> 14.5, 4096x14336 x16 20.6 -> 14.6, 11008x4096 x32 22.3 -> 15.6;
    // Q6_K 11008x4096 x16 22.2 -> 21.0; Q8_0 11008x4096 x16 20.1 -> 19.4)
    const int64_t grid = (int64_t)p.tiles_m * p.tiles_n * p.splits, cus = gq::num_cus();
    // (Q4_K to 64 tokens: 11008x4096 x48/x64 25.3/25.4 -> 19.5/20.5, 22016x4096 x64 40.6 -> 36.6,
    // 4096x11008 x64 23.1 -> 18.7; not at 128, nor Q6_K at 64: profiles/r04/b7_rg64.txt)
    const int64_t rounds = N <= (t == GQ_Q4_K ? kRgemmMultiRoundTokensQ4 : kRgemmMultiRoundTokens) ? 4 : 1;
    return grid <= rounds * cus * gq::rgemm_per_cu(t, p.nb) && 2 * grid >= cus;
}

// The resident GEMM where it applies, ahead of the skinny kernel (4096^2 x16 step: Q4_K 6.8 vs
// 9.7 us, Q8_0 7.8 vs 11.2, Q6_K 8.1 vs 12.9; x8 Q4_K 6.8 vs 9.3 -- profiles/r04/rg_small.txt)
// unless the skinny kernel is forced (GQ_SKINNY=1)
bool rgemm_route(int t, int form, int64_t M, int64_t N, int64_t K, int act)
{
    if (!use_rgemm(t, form, M, N, K)) return false;
    return gq::tuning().skinny != 1 || !use_skinny(t, form, N, act);
}

// K-chunked streaming MMQ (mmq_kstream.hip): 5..32 tokens (the fp8 variant from 3: its decode
// form covers 1..2), K % 256 == 0, M % 16 == 0; one launch for K <= 4096 (x~ quantized in-kernel
// from the raw activations, or read prepared).  GQ_KSTREAM=1: wherever it applies, 0: off.
// By default on the prepared calls (x~ read as act_quant wrote it; single and grouped) and the
// raw grouped launch: 5..32 tokens measured 7-12% under the routes before it (MMQ us, default -> kstream, round 5
// profiles/r05/ks_ab.txt: Q4_K 4096^2 x16 9.25 -> 7.96, 11008x4096 x16 15.31 -> 13.65,
// 22016x4096 x16 24.23 -> 22.12, x32 30.52 -> 27.72, x8 24.02 -> 21.69; Q6_K 4096^2 x16 10.55 ->
// 9.32; Q8_0 11008x4096 x16 18.05 -> 16.90).  Quantizing in-kernel (gq_mmq_ex) it is slower on the
// small matrices (every workgroup quantizes its whole K of x): a raw call takes it on the tall ones.
// A K longer than 4096 is cut into ranges summed by a second launch (fp32 partials in the
// workspace): by default only inside a grouped launch (the layer's ffn_down beside the K = 4096
// projections); split = false asks for the one-launch form.
bool use_kstream(int t, int form, int64_t M, int64_t N, int64_t K, int act, bool prepared = false,
                 bool split = false)
{
    const int ks = gq::tuning().kstream;
    if (ks == 0 || form != gq::AF_F16 || use_blas(N, K) || !gq::kstream_ok(t, M, N, K)) return false;
    // (q8_1 at 3..4 tokens: the grouped decode -- the prepared workspace holds the decode's SOA
    // q8_1 form there, not the fp16 x~ the stream reads; profiles/r06/kstream_nmin3_ab.txt)
    if (N < (act == GQ_ACT_FP8_E4M3 ? 3 : 5)) return false;
    if (gq::kstream_splits(K) > 1 && !split && ks != 1) return false;
    if (ks == 1) return true;
    if (gemm_knob_pinned()) return false; // (as the resident / streaming routes: the pinned GEMM takes the call)
    if (prepared) return true;
    // a raw call quantizes in-kernel (every workgroup its whole K of x): ahead of the resident GEMM
    // on the tall matrices at 5..16 tokens (Q4_K 11008 / 14336 / 22016 x4096 x16 15.79 / 17.74 /
    // 25.14 -> 15.41 / 17.36 / 23.23 us, Q6_K 11008 19.79 -> 19.15, Q8_0 11008 18.69 -> 18.33, x8
    // 15.61 -> 15.37), behind it on 4096-row matrices (9.27 -> 11.18) and at 32 tokens (18.51 ->
    // 23.98) -- profiles/r05/raw_kstream_ab.txt
    return act == GQ_ACT_Q8_1 && N <= 16 && M >= 8192;
}
size_t kstream_ws(int t, int64_t M, int64_t N, int64_t K)
{
    const gq::KItem it{t, nullptr, nullptr, K, nullptr, M, M, K};
    return gq::kstream_ok(t, M, N, K) && N <= 32 ? gq::kstream_partial_bytes(&it, 1, N) : 0;
}
// its 32-bit buffer offsets over the activations (rows ldx apart) and the output (rows ldc apart)
bool kstream_fits(int64_t M, int64_t N, int64_t K, int64_t ldx, int64_t ldc)
{
    return ((N - 1) * ldx + K) * 2 < ((int64_t)1 << 31) && ((N - 1) * ldc + M) * 4 < ((int64_t)1 << 31) && ldc % 4 == 0;
}

// Streaming 256-row GEMM (mmq_rgemm.hip sgemm_kernel) on the prepared x~, where the resident
// form does not apply (its grid is more than one round of the chip, or under half of one): by
// default from 17 tokens for every type, and Q6_K from 5 (the skinny kernel keeps Q4_K / Q8_0
// at 5..16) -- profiles/r04/sg_v1.txt, sg_n.txt, sg_small.txt (MMQ us, old route -> sgemm): Q6_K
// 28672x8192 x32/x64/x128/x256/x512 73.2/79.9/110.1/207.8/386.5 -> 71.5/78.1/102.2/178.4/342.3,
// 8192x28672 x64/x128 81.1/107.0 -> 75.5/96.5; Q8_0 11008x4096 x64/x128/x256 27.2/36.5/54.9 ->
// 23.8/28.8/45.4; Q4_K 11008x4096 x32/x64/x128 20.8/24.4/30.7 -> 20.0/22.7/28.9 (x256 46.8 vs
// 47.3); Q6_K 11008x4096 x16 23.5 -> 19.8.  GQ_SGEMM=1: wherever it applies (tests, A/B), 0: off.
constexpr int64_t kSgemmMinTokens = 17, kSgemmQ6MinTokens = 5;
bool use_sgemm(int t, int form, int64_t M, int64_t N, int64_t K)
{
    const int sg = gq::tuning().sgemm;
    if (sg == 0 || form != gq::AF_F16 || use_gemv(N, K) || use_blas(N, K) || K % 256 != 0) return false;
    if (gemm_rows_per_launch(t, M, K) < M || gemm_toks_per_launch(N, K) < N) return false;
    if (!gq::plan_sgemm(M, N, K, gq::tuning().sgemm_splits).ok) return false;
    if (sg == 1) return true;
    if (gemm_knob_pinned()) return false;
    return N >= kSgemmMinTokens || (t == GQ_Q6_K && N >= kSgemmQ6MinTokens);
}
gq::RGemmPlan sgemm_plan(int64_t M, int64_t N, int64_t K) { return gq::plan_sgemm(M, N, K, gq::tuning().sgemm_splits); }
// The streaming GEMM of one matrix as the grouped kernel's one-part stream-K plan (GQ_SGEMM_STREAMK=1,
// splits not pinned, tiles within one round of the chip): every workgroup L or L+1 super-blocks
// instead of whole-tile splits (Q6_K 28672x8192 x128: 224 workgroups x 16 super-blocks -> 256 x
// 14).  Measured no faster (104.7 vs 101.9 us there; 11008x4096 x128 33.7 vs 28.9: a workgroup
// of 2-3 super-blocks spanning two tiles fills and drains its ring twice and stores two
// partials; profiles/r04/b4_sk.txt), so off by default.
bool sgemm_streamk(int t, int64_t M, int64_t N, int64_t K, gq::SGroupItem &it, gq::SGroupPlan &g)
{
    if (gq::tuning().sgemm_splits > 0 || gq::tuning().sgemm_streamk <= 0) return false;
    it = gq::SGroupItem{t, nullptr, nullptr, nullptr, M, M, K};
    g = gq::plan_sgemm_grouped(&it, 1, N, 0);
    return g.ok && g.streamk;
}
size_t sgemm_partial_bytes(int t, int64_t M, int64_t N, int64_t K)
{
    gq::SGroupItem it;
    gq::SGroupPlan g;
    return sgemm_streamk(t, M, N, K, it, g) ? g.partial_bytes : sgemm_plan(M, N, K).partial_bytes;
}

bool use_i8(int t, int64_t N, int64_t K)
{
    if (t != GQ_Q8_0 || use_gemv(N, K) || use_blas(N, K)) return false;
    return gq::tuning().gemm_i8 != 0;
}

// Which kernels a call runs.  The q8_1 activations (the reference's semantics) go to the fused
// decode / GEMV (N <= 4), the MFMA GEMMs or, from blas_min_tokens(), dequant + hipBLASLt; the
// fp8 variant (GQ_ACT_FP8_E4M3) is quantized to e4m3 codes and widened to fp16 x~ by act_quant
// (ACT_F8DEQ), then runs every fp16-activation kernel as q8_1's x~ does (skinny from one token:
// there is no fp8 decode kernel).  (Widening the codes inside the GEMM instead, the round-2
// AF_F8 form, cost 12-55% over the q8_1 path: profiles/r03/s3/fp8_deq_route.log.)
struct Route {
    bool gemv = false, blas = false;
    int form = gq::AF_F16; // GEMM activation form
};
Route route(int t, int act, int64_t N, int64_t K)
{
    Route r;
    if (act == GQ_ACT_FP8_E4M3) {
        r.blas = use_blas(N, K);
        return r;
    }
    r.gemv = use_gemv(N, K);
    r.blas = use_blas(N, K);
    r.form = use_i8(t, N, K) ? gq::AF_I8 : gq::AF_F16;
    return r;
}

// GEMM-path activation forms in the workspace: fp16 x~ [N][K], then codes [N][K] and
// block-major scales [K/32][(N+3)&~3] (q8_1: the int8 form; fp8 variant: only these two).
int64_t scale_ld(int64_t N) { return (N + 3) & ~(int64_t)3; }
size_t deq_bytes(int64_t N, int64_t K) { return align_up((size_t)N * K * 2); }
size_t code_bytes(int64_t N, int64_t K) { return align_up((size_t)N * K); }
size_t scale_bytes(int64_t N, int64_t K) { return align_up((size_t)(K / 32) * (size_t)scale_ld(N) * 4); }

// Decode token counts (q8_1: the GEMV tokens, fp8: 1-2): gq_act_prepare also keeps an fp16 copy
// of the activations at the end of the activation part, so that gq_mmq_prepared runs the same
// one-launch decode as gq_mmq (bit-identical to it) instead of the GEMV on the SOA form (Q6_K
// 28672x8192 x1 60.6 -> 35.4 us; profiles/r05/prepared_decode_ab.txt)
// The copy only where a weight type's fused decode can run at (N, K) (gq_act_prepare does not
// know the type; e.g. 4 tokens at K = 11008 fit no type's LDS image: no copy, the GEMV)
bool prep_raw(int act, int64_t N, int64_t K)
{
    const bool fp8 = act == GQ_ACT_FP8_E4M3;
    if (fp8 ? !(N <= 2 && gq::gemm_supported(gq::Q8_0, K)) : !use_gemv(N, K)) return false;
    for (int t : {GQ_Q8_0, GQ_Q4_K, GQ_Q6_K})
        if ((t == GQ_Q8_0 || K % 256 == 0) && gq::decode_fused_ok(t, N, K, fp8)) return true;
    return false;
}
size_t raw_bytes(int act, int64_t N, int64_t K) { return prep_raw(act, N, K) ? align_up((size_t)N * K * 2) : 0; }

// Activation part of the workspace (what gq_act_prepare[_ex] writes); depends on act, N, K only.
size_t act_bytes(int act, int64_t N, int64_t K)
{
    if (act == GQ_ACT_FP8_E4M3) return deq_bytes(N, K) + raw_bytes(act, N, K); // the fp8 variant's x~
    if (use_gemv(N, K)) {
        // SOA q8_1: codes + d + s
        return align_up((size_t)N * K) + 2 * align_up((size_t)N * (K / 32) * sizeof(float)) + raw_bytes(act, N, K);
    }
    return deq_bytes(N, K) + code_bytes(N, K) + 2 * scale_bytes(N, K); // (+ s: the integer skinny kernel)
}

// Whole workspace: activations + (GEMM split-K) fp32 partial slabs / (library path) fp16 W.
size_t ws_bytes(int t, int act, int64_t M, int64_t N, int64_t K)
{
    const Route r = route(t, act, N, K);
    size_t b = act_bytes(act, N, K);
    if (r.blas) b += align_up((size_t)M * K * 2) + gq::blas_workspace_bytes(); // fp16 W + hipBLASLt
    else if (!r.gemv && gq::gemm_supported(t, K) && M > 0 && N > 0) {
        // split-K partials of the largest need over the launch shapes (full and remainder chunks)
        // (the kernel is chosen by the call's token count, so every chunk runs the same arithmetic)
        const bool sk = use_skinny(t, r.form, N, act);
        const int64_t mr = gemm_rows_per_launch(t, M, K), nt = sk ? N : gemm_toks_per_launch(N, K);
        size_t p = use_rgemm(t, r.form, M, N, K) ? gq::plan_rgemm(M, N, K).partial_bytes
                   : use_sgemm(t, r.form, M, N, K) ? sgemm_partial_bytes(t, M, N, K) : 0;
        if (gq::tuning().kstream == 1) p = p > kstream_ws(t, M, N, K) ? p : kstream_ws(t, M, N, K); // (its K ranges)
        for (int64_t mc : {mr, M % mr})
            for (int64_t nc : {nt, N % nt})
                if (mc > 0 && nc > 0) {
                    const size_t q = sk ? 0 : gq::plan_gemm(t, mc, nc, K, r.form).partial_bytes;
                    p = q > p ? q : p;
                }
        b += align_up(p);
    }
    return b;
}

// gq_mmq_ex takes the one-launch fused decode (no workspace) for this call
bool fused_decode_route(int t, int act, int64_t N, int64_t K)
{
    // the fp8 variant's own decode form (mmq_decode.hip FP8: fp16 dot products, 3-4x the int8
    // form's VALU) at 1-2 tokens; at 3-4 the skinny kernel / GEMM is faster (7B layer x4 83 vs
    // 73 us; profiles/r03/s3/fp8_decode.log)
    if (act == GQ_ACT_FP8_E4M3) return N <= 2 && gq::decode_fused_ok(t, N, K, true) && gq::tuning().fused_decode;
    return route(t, act, N, K).gemv && gq::decode_fused_ok(t, N, K) && gq::tuning().fused_decode;
}
// what a gq_mmq_ex call itself needs (gq_act_prepare / gq_mmq_prepared need ws_bytes)
size_t call_ws_bytes(int t, int act, int64_t M, int64_t N, int64_t K)
{
    return fused_decode_route(t, act, N, K) ? 0 : ws_bytes(t, act, M, N, K);
}

// ---- row sharding (gq_mmq_sharded) ----
constexpr int64_t kShardAlign = 64; // dist/row_shard.py shard_rows(align=64)

void shard_geom(int64_t M, int world, int rank, int64_t &row0, int64_t &rows, int64_t &R)
{
    R = (M + world - 1) / world;
    R = (R + kShardAlign - 1) / kShardAlign * kShardAlign;
    row0 = (int64_t)rank * R < M ? (int64_t)rank * R : M;
    const int64_t end = row0 + R < M ? row0 + R : M;
    rows = end - row0;
}

// C[n][m] = G[m / R][n][m % R]; VEC = 8: 8 columns (16 bytes) per thread (R % 8 == 0, so a
// group never straddles two shards; used when C's rows and M allow 16-byte stores)
template <int VEC>
__global__ __launch_bounds__(256) void assemble_kernel(const uint16_t *__restrict__ G, uint16_t *__restrict__ C,
                                                       int64_t N, int64_t R, int64_t M, int64_t ldc)
{
    const int64_t groups = (M + VEC - 1) / VEC;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N * groups;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n = i / groups, m = (i - n * groups) * VEC;
        const int64_t g = m / R, r = m - g * R;
        const uint16_t *src = G + (g * N + n) * R + r;
        uint16_t *dst = C + n * ldc + m;
        if constexpr (VEC == 8) {
            *(uint4 *)dst = *(const uint4 *)src;
        } else {
            *dst = *src;
        }
    }
}

hipError_t launch_assemble(const uint16_t *G, uint16_t *C, int64_t N, int64_t R, int64_t M, int64_t ldc,
                           hipStream_t s)
{
    const bool vec = M % 8 == 0 && ldc % 8 == 0 && ((uintptr_t)C & 15) == 0 && ((uintptr_t)G & 15) == 0;
    const int64_t items = N * (vec ? M / 8 : M);
    const int64_t blocks = (items + 255) / 256 < 4096 ? (items + 255) / 256 : 4096;
    if (vec) assemble_kernel<8><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(G, C, N, R, M, ldc);
    else assemble_kernel<1><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(G, C, N, R, M, ldc);
    return hipGetLastError();
}

// RCCL's all-gather, looked up in the process (the caller's RCCL, whose communicator we are
// handed); librccl.so.1 is opened by soname only if nothing in the process exports it
using AllGatherFn = decltype(&ncclAllGather);
AllGatherFn shard_allgather()
{
    static AllGatherFn fn = nullptr;
    static std::once_flag once;
    std::call_once(once, [] {
        void *sym = dlsym(RTLD_DEFAULT, "ncclAllGather");
        if (!sym) {
            if (void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL)) sym = dlsym(h, "ncclAllGather");
        }
        fn = (AllGatherFn)sym;
    });
    return fn;
}

// every rank's need: the local MMQ's workspace is not monotone in the row count (fewer rows ->
// fewer tiles -> a larger split-K factor -> more partials), so it is the max over the ranks'
// shard sizes, not rank 0's
size_t sharded_ws(int t, int64_t M, int64_t N, int64_t K, int world)
{
    int64_t row0, rows, R;
    size_t local = 0;
    for (int g = 0; g < world; ++g) {
        shard_geom(M, world, g, row0, rows, R);
        const size_t w = ws_bytes(t, GQ_ACT_Q8_1, rows, N, K);
        local = w > local ? w : local;
    }
    return align_up((size_t)N * R * 2) + align_up((size_t)world * N * R * 2) + local;
}

} // namespace

extern "C" {

int gq_debug_set_tuning(const char *key, long long value)
{
    g_err.clear();
    if (gq::set_tuning(key, value) != 0)
        return fail(GQ_EINVAL, "unknown tuning key or value out of range: %s=%lld", key ? key : "(null)", value);
    return GQ_OK;
}
void gq_debug_reset_tuning(void) { gq::reset_tuning(); }


int gq_block_elems(gq_type t) { return block_elems(t); }
int gq_block_bytes(gq_type t) { return block_bytes(t); }
int gq_version(void) { return 105; }

unsigned int gq_debug_sync_timeouts(void) { return gq::ilc_timeouts() + gq::kstream_timeouts(); }
const char *gq_last_error(void) { return g_err.c_str(); }

size_t gq_mmq_call_workspace_size(gq_type t, gq_act act, int64_t M, int64_t N, int64_t K)
{
    if (N <= 0 || K <= 0 || M < 0) return 0;
    return call_ws_bytes(t, act, M, N, K);
}
size_t gq_mmq_workspace_size_ex(gq_type t, gq_act act, int64_t M, int64_t N, int64_t K)
{
    if (N <= 0 || K <= 0 || M < 0) return 0;
    return ws_bytes(t, act, M, N, K);
}
size_t gq_mmq_workspace_size(gq_type t, int64_t M, int64_t N, int64_t K)
{
    return gq_mmq_workspace_size_ex(t, GQ_ACT_Q8_1, M, N, K);
}

static int check_common(gq_type t, int64_t M, int64_t N, int64_t K)
{
    if (t != GQ_Q8_0 && t != GQ_Q4_K && t != GQ_Q6_K) return fail(GQ_EUNSUPPORTED, "unknown gguf type %d", (int)t);
    if (M < 0 || N < 0 || K < 0)
        return fail(GQ_EINVAL, "negative size M=%lld N=%lld K=%lld", (long long)M, (long long)N, (long long)K);
    const int qk = block_elems(t);
    if (K % qk != 0) return fail(GQ_EINVAL, "K=%lld is not a multiple of %d", (long long)K, qk);
    return GQ_OK;
}

static int check_act(int act, int64_t K)
{
    if (act != GQ_ACT_Q8_1 && act != GQ_ACT_FP8_E4M3) return fail(GQ_EUNSUPPORTED, "unknown activation format %d", act);
    if (act == GQ_ACT_FP8_E4M3 && !gq::gemm_supported(gq::Q8_0, K))
        return fail(GQ_EUNSUPPORTED, "fp8 activations need K %% 256 == 0 (K=%lld)", (long long)K);
    return GQ_OK;
}

struct Carved {
    int8_t *xq;       // SOA codes (decode) / GEMM codes (int8 form, fp8 variant)
    float *xd, *xs;   // SOA d, s (decode) / GEMM block-major scales
    uint16_t *xdeq;
    uint16_t *xraw;   // decode token counts: the fp16 activations (rows K apart; prep_raw)
    float *partials;
};

static Carved carve(int act, void *workspace, int64_t N, int64_t K)
{
    uint8_t *ws = (uint8_t *)workspace;
    Carved c{};
    if (prep_raw(act, N, K)) c.xraw = (uint16_t *)(ws + act_bytes(act, N, K) - raw_bytes(act, N, K));
    if (act == GQ_ACT_FP8_E4M3) {
        c.xdeq = (uint16_t *)ws;
    } else if (use_gemv(N, K)) {
        c.xq = (int8_t *)ws;
        c.xd = (float *)(ws + align_up((size_t)N * K));
        c.xs = (float *)((uint8_t *)c.xd + align_up((size_t)N * (K / 32) * sizeof(float)));
        return c;
    } else {
        c.xdeq = (uint16_t *)ws;
        c.xq = (int8_t *)(ws + deq_bytes(N, K));
        c.xd = (float *)(ws + deq_bytes(N, K) + code_bytes(N, K));
        c.xs = (float *)((uint8_t *)c.xd + scale_bytes(N, K));
    }
    c.partials = (float *)(ws + act_bytes(act, N, K));
    return c;
}

// q8_1 forms: bit 0 = fp16 x~ (DEQ), bit 1 = int8 codes + d (I8), bit 2 = with the I8 form, s
// too (the integer skinny kernel); only the GEMM path reads them
static int prepare(int act, const void *B, int64_t N, int64_t K, int64_t ldb, void *workspace,
                   size_t workspace_bytes, hipStream_t s, int forms = 1)
{
    if (!B) return fail(GQ_EINVAL, "null activation pointer");
    if (ldb < K) return fail(GQ_EINVAL, "ldb=%lld < K=%lld", (long long)ldb, (long long)K);
    const size_t need = act_bytes(act, N, K);
    if (!workspace || workspace_bytes < need)
        return fail(GQ_EINVAL, "workspace %zu bytes < required %zu", workspace ? workspace_bytes : (size_t)0, need);
    Carved c = carve(act, workspace, N, K);
    hipError_t e = hipSuccess;
    if (act == GQ_ACT_FP8_E4M3) {
        e = gq::launch_act_quant(gq::ACT_F8DEQ, (const uint16_t *)B, ldb, N, K, c.xdeq, nullptr, nullptr, s);
    } else if (use_gemv(N, K)) {
        e = gq::launch_act_quant(gq::ACT_SOA, (const uint16_t *)B, ldb, N, K, c.xq, c.xd, c.xs, s);
    } else {
        if (forms & 1) e = gq::launch_act_quant(gq::ACT_DEQ, (const uint16_t *)B, ldb, N, K, c.xdeq, nullptr, nullptr, s);
        if (e == hipSuccess && (forms & 2))
            e = gq::launch_act_quant(gq::ACT_I8, (const uint16_t *)B, ldb, N, K, c.xq, c.xd, (forms & 4) ? c.xs : nullptr, s);
    }
    if (e == hipSuccess && c.xraw)
        e = hipMemcpy2DAsync(c.xraw, (size_t)K * 2, B, (size_t)ldb * 2, (size_t)K * 2, (size_t)N, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (act_quant): %s", hipGetErrorString(e));
    return GQ_OK;
}

static int compute(gq_type t, int act, const void *A, void *workspace, size_t workspace_bytes, void *C, int64_t M,
                   int64_t N, int64_t K, int64_t ldc, hipStream_t s)
{
    if (!A || !C || !workspace) return fail(GQ_EINVAL, "null pointer (A=%p C=%p workspace=%p)", A, C, workspace);
    if (ldc < M) return fail(GQ_EINVAL, "ldc=%lld < M=%lld", (long long)ldc, (long long)M);
    const size_t need = ws_bytes(t, act, M, N, K);
    if (workspace_bytes < need) return fail(GQ_EINVAL, "workspace %zu bytes < required %zu", workspace_bytes, need);
    const Route r = route(t, act, N, K);
    Carved c = carve(act, workspace, N, K);
    if (c.xraw && fused_decode_route(t, act, N, K)) { // gq_mmq's one-launch decode on the prepared copy
        const hipError_t e = gq::launch_decode_fused(t, (const uint8_t *)A, c.xraw, K, (uint16_t *)C, M, N, K, ldc, s,
                                                     act == GQ_ACT_FP8_E4M3);
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (decode): %s", hipGetErrorString(e));
        return GQ_OK;
    }
    if (r.blas) {
        uint16_t *W = (uint16_t *)c.partials; // after the activations: fp16 W, then the BLAS workspace
        uint8_t *bws = (uint8_t *)W + align_up((size_t)M * K * 2);
        hipError_t e = gq::launch_dequant(t, (const uint8_t *)A, W, M, K, K, true, s);
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (dequant): %s", hipGetErrorString(e));
        const int rc = gq::blas_gemm(W, c.xdeq, (uint16_t *)C, M, N, K, ldc, bws, gq::blas_workspace_bytes(), s);
        if (rc != 0) return fail(GQ_EHIP, "hipBLASLt GEMM failed (code %d)", rc);
        return GQ_OK;
    }
    hipError_t e;
    if (r.gemv) {
        e = gq::launch_gemv(t, (const uint8_t *)A, c.xq, c.xd, c.xs, (uint16_t *)C, M, N, K, ldc, s);
    } else {
        // chunks of < 2 GiB of weights and of activations per launch (32-bit buffer offsets)
        // (the kernel is chosen by the call's token count: every chunk runs the same arithmetic)
        // (<= 32 skinny tokens are never cut: their x~ is far below the guard, and the token
        // count sets the kernel's K split)
        if (use_kstream(t, r.form, M, N, K, act, true) && kstream_fits(M, N, K, K, ldc)) {
            const gq::KItem it{t, (const uint8_t *)A, c.xdeq, K, (uint16_t *)C, ldc, M, K};
            e = gq::launch_kstream(&it, 1, N, 0, c.partials, s);
            if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (kstream): %s", hipGetErrorString(e));
            return GQ_OK;
        }
        if (rgemm_route(t, r.form, M, N, K, act)) {
            e = gq::launch_rgemm(t, 0, (const uint8_t *)A, c.xdeq, K, (uint16_t *)C, c.partials, gq::plan_rgemm(M, N, K),
                                 M, N, K, ldc, s);
            if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (rgemm): %s", hipGetErrorString(e));
            return GQ_OK;
        }
        if (!rgemm_route(t, r.form, M, N, K, act) && !use_skinny(t, r.form, N, act) && use_sgemm(t, r.form, M, N, K)) {
            gq::SGroupItem it;
            gq::SGroupPlan g;
            if (sgemm_streamk(t, M, N, K, it, g)) {
                it.A = (const uint8_t *)A;
                it.X = c.xdeq;
                it.C = (uint16_t *)C;
                it.ldc = ldc;
                e = gq::launch_sgemm_grouped(&it, 1, N, g, c.partials, s);
            } else {
                e = gq::launch_sgemm(t, (const uint8_t *)A, c.xdeq, (uint16_t *)C, c.partials, sgemm_plan(M, N, K), M, N,
                                     K, ldc, s);
            }
            if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (sgemm): %s", hipGetErrorString(e));
            return GQ_OK;
        }
        const bool sk = use_skinny(t, r.form, N, act);
        const int64_t mr = gemm_rows_per_launch(t, M, K), nt = sk ? N : gemm_toks_per_launch(N, K);
        e = hipSuccess;
        for (int64_t n0 = 0; n0 < N && e == hipSuccess; n0 += nt)
            for (int64_t m0 = 0; m0 < M && e == hipSuccess; m0 += mr) {
                const int64_t mc = M - m0 < mr ? M - m0 : mr, nc = N - n0 < nt ? N - n0 : nt;
                if (sk) {
                    e = gq::launch_skinny(t, (const uint8_t *)A + m0 * row_bytes_of(t, K), c.xdeq + n0 * K,
                                          (uint16_t *)C + n0 * ldc + m0, skinny_plan(t, mc, nc, K), mc, nc, K, ldc, s);
                    continue;
                }
                gq::GemmAct x;
                x.xdeq = c.xdeq ? c.xdeq + n0 * K : nullptr;
                x.xq = c.xq ? c.xq + n0 * K : nullptr;
                x.xd = c.xd ? c.xd + n0 : nullptr;
                x.ldd = scale_ld(N);
                e = gq::launch_gemm(t, (const uint8_t *)A + m0 * row_bytes_of(t, K), x, (uint16_t *)C + n0 * ldc + m0,
                                    c.partials, gq::plan_gemm(t, mc, nc, K, r.form), mc, nc, K, ldc, s);
            }
    }
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (mmq): %s", hipGetErrorString(e));
    return GQ_OK;
}

int gq_mmq_ex(gq_type t, gq_act act, const void *A, const void *B, void *C, int64_t M, int64_t N, int64_t K,
              int64_t ldb, int64_t ldc, void *workspace, size_t workspace_bytes, void *stream)
{
    g_err.clear();
    int rc = check_common(t, M, N, K);
    if (rc != GQ_OK) return rc;
    if ((rc = check_act(act, K)) != GQ_OK) return rc;
    if (M == 0 || N == 0) return GQ_OK;
    if (K == 0) return fail(GQ_EINVAL, "K must be positive");
    if (!A || !B || !C) return fail(GQ_EINVAL, "null pointer (A=%p B=%p C=%p)", A, B, C);
    if (ldc < M) return fail(GQ_EINVAL, "ldc=%lld < M=%lld", (long long)ldc, (long long)M);
    if (ldb < K) return fail(GQ_EINVAL, "ldb=%lld < K=%lld", (long long)ldb, (long long)K);
    const size_t need = call_ws_bytes(t, act, M, N, K);
    if (need && (!workspace || workspace_bytes < need))
        return fail(GQ_EINVAL, "workspace %zu bytes < required %zu", workspace ? workspace_bytes : (size_t)0, need);
    const Route r = route(t, act, N, K);
    if (fused_decode_route(t, act, N, K)) {
        // one launch: activation quantization in LDS + decode GEMV
        hipError_t e = gq::launch_decode_fused(t, (const uint8_t *)A, (const uint16_t *)B, ldb, (uint16_t *)C, M, N,
                                               K, ldc, (hipStream_t)stream, act == GQ_ACT_FP8_E4M3);
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (decode): %s", hipGetErrorString(e));
        return GQ_OK;
    }
    if (use_kstream(t, r.form, M, N, K, act) && ldb % 8 == 0 && ((uintptr_t)B & 15) == 0 &&
        kstream_fits(M, N, K, ldb, ldc)) {
        // one launch, no workspace: the activations quantized inside (q8_1, or the fp8 variant's
        // e4m3), bit-identical to the act_quant forms the prepared call reads
        const gq::KItem it{t, (const uint8_t *)A, (const uint16_t *)B, ldb, (uint16_t *)C, ldc, M, K};
        hipError_t e = gq::launch_kstream(&it, 1, N, act == GQ_ACT_FP8_E4M3 ? 2 : 1,
                                          carve(act, workspace, N, K).partials, (hipStream_t)stream);
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (kstream): %s", hipGetErrorString(e));
        return GQ_OK;
    }
    if (rgemm_route(t, r.form, M, N, K, act) && ldb % 8 == 0 &&
        ((uintptr_t)B & 15) == 0) {
        // one launch (+ the split-K reduce): the activations quantized inside the GEMM (q8_1, or
        // the fp8 variant's e4m3), bit-identical to the act_quant forms it would read
        Carved c = carve(act, workspace, N, K);
        hipError_t e = gq::launch_rgemm(t, act == GQ_ACT_FP8_E4M3 ? 2 : 1, (const uint8_t *)A, (const uint16_t *)B, ldb,
                                        (uint16_t *)C, c.partials, gq::plan_rgemm(M, N, K), M, N, K, ldc,
                                        (hipStream_t)stream);
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (rgemm): %s", hipGetErrorString(e));
        return GQ_OK;
    }
    if (!r.gemv && !r.blas && act == GQ_ACT_Q8_1 && r.form == gq::AF_F16 && !use_skinny(t, r.form, N) &&
        !use_sgemm(t, r.form, M, N, K) &&
        gemm_rows_per_launch(t, M, K) >= M &&
        gemm_toks_per_launch(N, K) >= N) {
        // 16/32-token tiles whose split fits LDS: the GEMM quantizes the activations itself (no
        // act_quant launch; bit-identical to the DEQ form it would read)
        gq::GemmPlan plan = gq::plan_gemm(t, M, N, K, r.form);
        if (gq::gemm_aq_ok(plan)) {
            plan.aq = 1;
            gq::GemmAct x;
            x.xraw = (const uint16_t *)B;
            x.ldx = ldb;
            Carved c = carve(act, workspace, N, K);
            hipError_t e = gq::launch_gemm(t, (const uint8_t *)A, x, (uint16_t *)C, c.partials, plan, M, N, K, ldc,
                                           (hipStream_t)stream);
            if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (mmq): %s", hipGetErrorString(e));
            return GQ_OK;
        }
    }
    rc = prepare(act, B, N, K, ldb, workspace, workspace_bytes, (hipStream_t)stream, r.form == gq::AF_I8 ? 2 : 1);
    if (rc != GQ_OK) return rc;
    return compute(t, act, A, workspace, workspace_bytes, C, M, N, K, ldc, (hipStream_t)stream);
}

int gq_mmq(gq_type t, const void *A, const void *B, void *C, int64_t M, int64_t N, int64_t K, int64_t ldb,
           int64_t ldc, void *workspace, size_t workspace_bytes, void *stream)
{
    return gq_mmq_ex(t, GQ_ACT_Q8_1, A, B, C, M, N, K, ldb, ldc, workspace, workspace_bytes, stream);
}

int gq_act_prepare_ex(gq_act act, const void *B, int64_t N, int64_t K, int64_t ldb, void *workspace,
                      size_t workspace_bytes, void *stream)
{
    g_err.clear();
    if (N < 0 || K < 0) return fail(GQ_EINVAL, "negative size");
    if (K % 32 != 0) return fail(GQ_EINVAL, "K=%lld is not a multiple of 32", (long long)K);
    int rc = check_act(act, K);
    if (rc != GQ_OK) return rc;
    if (N == 0 || K == 0) return GQ_OK;
    // the weight type is not known here: write every form a later gq_mmq_prepared may read
    // (the int8 form only when Q8_0 would use it)
    return prepare(act, B, N, K, ldb, workspace, workspace_bytes, (hipStream_t)stream,
                   use_i8(GQ_Q8_0, N, K) ? 3 : 1);
}

int gq_act_prepare(const void *B, int64_t N, int64_t K, int64_t ldb, void *workspace, size_t workspace_bytes,
                   void *stream)
{
    return gq_act_prepare_ex(GQ_ACT_Q8_1, B, N, K, ldb, workspace, workspace_bytes, stream);
}

int gq_act_prepare_grouped(gq_act act, const gq_prep_item *items, int n, void *stream)
{
    g_err.clear();
    if (n < 0 || (n > 0 && !items)) return fail(GQ_EINVAL, "bad item list (n=%d, items=%p)", n, (const void *)items);
    // every item checked first (gq_act_prepare_ex's checks, in its order): a bad item launches nothing
    for (int i = 0; i < n; ++i) {
        const gq_prep_item &it = items[i];
        const int64_t N = it.N, K = it.K;
        if (N < 0 || K < 0) return fail(GQ_EINVAL, "item %d: negative size", i);
        if (K % 32 != 0) return fail(GQ_EINVAL, "item %d: K=%lld is not a multiple of 32", i, (long long)K);
        const int rc = check_act(act, K);
        if (rc != GQ_OK) return rc;
        if (N == 0 || K == 0) continue;
        if (!it.B) return fail(GQ_EINVAL, "item %d: null activation pointer", i);
        if (it.ldb < K) return fail(GQ_EINVAL, "item %d: ldb=%lld < K=%lld", i, (long long)it.ldb, (long long)K);
        const size_t need = act_bytes(act, N, K);
        if (!it.workspace || it.workspace_bytes < need)
            return fail(GQ_EINVAL, "item %d: workspace %zu bytes < required %zu", i,
                        it.workspace ? it.workspace_bytes : (size_t)0, need);
    }
    const hipStream_t s = (hipStream_t)stream;
    gq::DeqSeg segs[gq::kMaxDeqSegs];
    int ns = 0;
    auto flush = [&]() -> int {
        if (ns == 0) return GQ_OK;
        const hipError_t e = gq::launch_act_quant_deq_grouped(segs, ns, s, act == GQ_ACT_FP8_E4M3 ? gq::ACT_F8DEQ : gq::ACT_DEQ);
        ns = 0;
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (grouped act_quant): %s", hipGetErrorString(e));
        return GQ_OK;
    };
    for (int i = 0; i < n; ++i) {
        const gq_prep_item &it = items[i];
        const int64_t N = it.N, K = it.K;
        if (N == 0 || K == 0) continue;
        int rc;
        if (act == GQ_ACT_Q8_1 && (use_gemv(N, K) || use_i8(GQ_Q8_0, N, K))) { // its own launch(es), as gq_act_prepare_ex
            if ((rc = prepare(act, it.B, N, K, it.ldb, it.workspace, it.workspace_bytes, s,
                              use_i8(GQ_Q8_0, N, K) ? 3 : 1)) != GQ_OK)
                return rc;
            continue;
        }
        if (ns == gq::kMaxDeqSegs && (rc = flush()) != GQ_OK) return rc;
        // the fp16 x~ form sits at the front of the workspace (carve)
        const Carved c = carve(act, it.workspace, N, K);
        segs[ns++] = gq::DeqSeg{(const uint16_t *)it.B, it.ldb, N, K, c.xdeq, 0};
        if (c.xraw) { // (fp8 at 1-2 tokens: the decode's copy, as prepare())
            const hipError_t e = hipMemcpy2DAsync(c.xraw, (size_t)K * 2, it.B, (size_t)it.ldb * 2, (size_t)K * 2,
                                                  (size_t)N, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return fail(GQ_EHIP, "HIP copy failed (grouped act_quant): %s", hipGetErrorString(e));
        }
    }
    return flush();
}

int gq_mmq_prepared_ex(gq_type t, gq_act act, const void *A, void *workspace, size_t workspace_bytes, void *C,
                       int64_t M, int64_t N, int64_t K, int64_t ldc, void *stream)
{
    g_err.clear();
    int rc = check_common(t, M, N, K);
    if (rc != GQ_OK) return rc;
    if ((rc = check_act(act, K)) != GQ_OK) return rc;
    if (M == 0 || N == 0) return GQ_OK;
    if (K == 0) return fail(GQ_EINVAL, "K must be positive");
    return compute(t, act, A, workspace, workspace_bytes, C, M, N, K, ldc, (hipStream_t)stream);
}

int gq_mmq_prepared(gq_type t, const void *A, void *workspace, size_t workspace_bytes, void *C, int64_t M, int64_t N,
                    int64_t K, int64_t ldc, void *stream)
{
    return gq_mmq_prepared_ex(t, GQ_ACT_Q8_1, A, workspace, workspace_bytes, C, M, N, K, ldc, stream);
}

int gq_dequantize(gq_type t, const void *A, void *W, int64_t M, int64_t K, int64_t ldw, void *stream)
{
    g_err.clear();
    int rc = check_common(t, M, 1, K);
    if (rc != GQ_OK) return rc;
    if (M == 0 || K == 0) return GQ_OK;
    if (!A || !W) return fail(GQ_EINVAL, "null pointer");
    if (ldw < K) return fail(GQ_EINVAL, "ldw=%lld < K=%lld", (long long)ldw, (long long)K);
    hipError_t e = gq::launch_dequant(t, (const uint8_t *)A, (uint16_t *)W, M, K, ldw, false, (hipStream_t)stream);
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed: %s", hipGetErrorString(e));
    return GQ_OK;
}

int gq_quantize_q8_1(const void *X, void *Y, int64_t rows, int64_t K, int64_t ldx, void *stream)
{
    g_err.clear();
    if (rows < 0 || K < 0) return fail(GQ_EINVAL, "negative size");
    if (K % 32 != 0) return fail(GQ_EINVAL, "K=%lld is not a multiple of 32", (long long)K);
    if (rows == 0 || K == 0) return GQ_OK;
    if (!X || !Y) return fail(GQ_EINVAL, "null pointer");
    if (ldx < K) return fail(GQ_EINVAL, "ldx=%lld < K=%lld", (long long)ldx, (long long)K);
    hipError_t e = gq::launch_act_quant(gq::ACT_AOS, (const uint16_t *)X, ldx, rows, K, Y, nullptr, nullptr,
                                        (hipStream_t)stream);
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed: %s", hipGetErrorString(e));
    return GQ_OK;
}

int gq_quantize_weights(gq_type t, const void *X, void *Y, int64_t n, void *stream)
{
    g_err.clear();
    if (t != GQ_Q8_0 && t != GQ_Q4_K && t != GQ_Q6_K) return fail(GQ_EUNSUPPORTED, "unknown gguf type %d", (int)t);
    if (n < 0) return fail(GQ_EINVAL, "negative size");
    const int qk = block_elems(t);
    if (n % qk != 0) return fail(GQ_EINVAL, "n=%lld is not a multiple of %d", (long long)n, qk);
    if (n == 0) return GQ_OK;
    if (!X || !Y) return fail(GQ_EINVAL, "null pointer");
    const int kind = t == GQ_Q8_0 ? 0 : (t == GQ_Q4_K ? 1 : 2);
    hipError_t e = gq::launch_quant_blocks(kind, X, Y, n / qk, (hipStream_t)stream);
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (weight quantizer): %s", hipGetErrorString(e));
    return GQ_OK;
}

int gq_quantize_fp8(const void *X, void *codes, void *scales, int64_t rows, int64_t K, int64_t ldx, void *stream)
{
    g_err.clear();
    if (rows < 0 || K < 0) return fail(GQ_EINVAL, "negative size");
    if (K % 32 != 0) return fail(GQ_EINVAL, "K=%lld is not a multiple of 32", (long long)K);
    if (rows == 0 || K == 0) return GQ_OK;
    if (!X || !codes || !scales) return fail(GQ_EINVAL, "null pointer");
    if (ldx < K) return fail(GQ_EINVAL, "ldx=%lld < K=%lld", (long long)ldx, (long long)K);
    hipError_t e = gq::launch_act_quant(gq::ACT_F8, (const uint16_t *)X, ldx, rows, K, codes, scales, nullptr,
                                        (hipStream_t)stream);
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed: %s", hipGetErrorString(e));
    return GQ_OK;
}

int gq_shard_rows(int64_t M, int world, int rank, int64_t *row0, int64_t *rows, int64_t *R)
{
    g_err.clear();
    if (M < 0 || world < 1 || rank < 0 || rank >= world)
        return fail(GQ_EINVAL, "bad shard (M=%lld world=%d rank=%d)", (long long)M, world, rank);
    if (!row0 || !rows || !R) return fail(GQ_EINVAL, "null output pointer");
    shard_geom(M, world, rank, *row0, *rows, *R);
    return GQ_OK;
}

int gq_assemble_shards(const void *gathered, void *C, int world, int64_t N, int64_t R, int64_t M, int64_t ldc,
                       void *stream)
{
    g_err.clear();
    if (world < 1 || N < 0 || R < 0 || M < 0) return fail(GQ_EINVAL, "negative size or world < 1");
    if (M > (int64_t)world * R) return fail(GQ_EINVAL, "M=%lld > world*R=%lld", (long long)M, (long long)world * R);
    if (R % 8 != 0) return fail(GQ_EINVAL, "R=%lld is not a multiple of 8", (long long)R);
    if (ldc < M) return fail(GQ_EINVAL, "ldc=%lld < M=%lld", (long long)ldc, (long long)M);
    if (N == 0 || M == 0) return GQ_OK;
    if (!gathered || !C) return fail(GQ_EINVAL, "null pointer");
    hipError_t e = launch_assemble((const uint16_t *)gathered, (uint16_t *)C, N, R, M, ldc, (hipStream_t)stream);
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (assemble): %s", hipGetErrorString(e));
    return GQ_OK;
}

size_t gq_mmq_sharded_workspace_size(gq_type t, int64_t M, int64_t N, int64_t K, int world)
{
    if (N <= 0 || K <= 0 || M < 0 || world < 1) return 0;
    return sharded_ws(t, M, N, K, world);
}

int gq_mmq_grouped(const gq_group_item *items, int n, int64_t N, void *stream)
{
    return gq_mmq_grouped_ex(GQ_ACT_Q8_1, items, n, N, stream);
}

int gq_mmq_grouped_ex(gq_act act, const gq_group_item *items, int n, int64_t N, void *stream)
{
    g_err.clear();
    const bool fp8 = act == GQ_ACT_FP8_E4M3;
    if (n < 0 || (n > 0 && !items)) return fail(GQ_EINVAL, "bad item list (n=%d, items=%p)", n, (const void *)items);
    if (N < 0) return fail(GQ_EINVAL, "negative N");
    gq::DecodeItem di[16];
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const gq_group_item &it = items[i];
        int rc = check_common(it.type, it.M, N, it.K);
        if (rc != GQ_OK) return rc;
        if ((rc = check_act(act, it.K)) != GQ_OK) return rc;
        if (it.M == 0 || N == 0) continue;
        if (it.K == 0) return fail(GQ_EINVAL, "item %d: K must be positive", i);
        if (!it.A || !it.B || !it.C) return fail(GQ_EINVAL, "item %d: null pointer", i);
        if (it.ldb < it.K) return fail(GQ_EINVAL, "item %d: ldb=%lld < K=%lld", i, (long long)it.ldb, (long long)it.K);
        if (it.ldc < it.M) return fail(GQ_EINVAL, "item %d: ldc=%lld < M=%lld", i, (long long)it.ldc, (long long)it.M);
        if (m == 16) return fail(GQ_EUNSUPPORTED, "more than 16 items");
        di[m++] = gq::DecodeItem{it.type, (const uint8_t *)it.A, (const uint16_t *)it.B, it.ldb, (uint16_t *)it.C,
                                 it.ldc, it.M, it.K};
    }
    if (m == 0) return GQ_OK;
    // (3..4 q8_1 tokens stay on the grouped decode: the stream for the K <= 4096 items with the
    // long-K item on its own measured 13% slower on the 7B layer, profiles/r06/kstream_rawg3_ab.txt)
    if (N >= (fp8 ? 3 : 5)) {
        // 5..32 tokens (fp8: 3..32): the K-chunked streaming MMQ, every item in one launch
        gq::KItem ki[16];
        for (int i = 0; i < m; ++i) {
            const gq::DecodeItem &d = di[i];
            // (the grouped launch's own route: the stream wherever it applies, GQ_KSTREAM=0 refuses)
            if (!use_kstream(d.fmt, gq::AF_F16, d.M, N, d.K, act, true) || gq::kstream_splits(d.K) > 1 || d.ldx % 8 != 0 ||
                ((uintptr_t)d.X & 15) != 0 || !kstream_fits(d.M, N, d.K, d.ldx, d.ldc))
                return fail(GQ_EUNSUPPORTED, "item %d: not a grouped K-chunked-stream shape (N=%lld, M=%lld, K=%lld)", i,
                            (long long)N, (long long)d.M, (long long)d.K);
            ki[i] = gq::KItem{d.fmt, d.A, d.X, d.ldx, d.C, d.ldc, d.M, d.K};
        }
        hipError_t e = gq::launch_kstream(ki, m, N, fp8 ? 2 : 1, nullptr, (hipStream_t)stream); // (no K ranges)
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (grouped kstream): %s", hipGetErrorString(e));
        return GQ_OK;
    }
    if (!gq::decode_grouped_ok(di, m, N, fp8))
        return fail(GQ_EUNSUPPORTED, "not a grouped-decode shape (N=%lld; N <= %d and every item a one-launch decode)",
                    (long long)N, fp8 ? 2 : 4);
    hipError_t e = gq::launch_decode_grouped(di, m, N, (hipStream_t)stream, fp8);
    if (e == hipErrorInvalidValue) return fail(GQ_EUNSUPPORTED, "grouped decode: more than 16 parts");
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (grouped decode): %s", hipGetErrorString(e));
    return GQ_OK;
}

// gq_mmq_grouped_prepared: the items as the grouped streaming GEMM takes them, or a GQ_* error
static int grouped_gemm_items(gq_act act, const gq_gemm_item *items, int n, int64_t N, gq::SGroupItem *out)
{
    if (n < 0 || (n > 0 && !items)) return fail(GQ_EINVAL, "bad item list (n=%d, items=%p)", n, (const void *)items);
    if (n > 16) return fail(GQ_EUNSUPPORTED, "more than 16 items");
    if (N < 5) return fail(GQ_EUNSUPPORTED, "grouped GEMM needs N >= 5 (N=%lld): gq_mmq_grouped for decode", (long long)N);
    for (int i = 0; i < n; ++i) {
        const gq_gemm_item &it = items[i];
        int rc = check_common(it.type, it.M, N, it.K);
        if (rc != GQ_OK) return rc;
        if ((rc = check_act(act, it.K)) != GQ_OK) return rc;
        if (it.K % 256 != 0 || it.K == 0) return fail(GQ_EUNSUPPORTED, "item %d: K=%lld is not a multiple of 256", i, (long long)it.K);
        if (it.M > 0 && (!it.A || !it.ws || !it.C)) return fail(GQ_EINVAL, "item %d: null pointer", i);
        if (it.ldc < it.M) return fail(GQ_EINVAL, "item %d: ldc=%lld < M=%lld", i, (long long)it.ldc, (long long)it.M);
        if (gemm_rows_per_launch(it.type, it.M, it.K) < it.M || gemm_toks_per_launch(N, it.K) < N)
            return fail(GQ_EUNSUPPORTED, "item %d: 2 GiB or more in one operand", i);
        out[i] = gq::SGroupItem{it.type, (const uint8_t *)it.A, carve(act, const_cast<void *>(it.ws), N, it.K).xdeq,
                                (uint16_t *)it.C, it.ldc, it.M, it.K};
    }
    return GQ_OK;
}

// gq_mmq_grouped_prepared's split of the items: those the K-chunked streaming MMQ takes (one
// launch, no workspace) and the rest (the grouped streaming GEMM: one launch + its reduce).
// The stream's launch holds at most kKMaxParts (item, K range) parts: an item whose ranges would
// pass that goes to the streaming GEMM (e.g. 16 items at K = 8192 are 32 parts: the first 12 take
// the stream, the other 4 the GEMM).
static void grouped_split(gq_act act, gq::SGroupItem *g, int n, int64_t N, gq::KItem *ks, int &nk, gq::SGroupItem *rest,
                          int &nr)
{
    nk = nr = 0;
    int parts = 0;
    for (int i = 0; i < n; ++i) {
        if (g[i].M <= 0) continue;
        const int np = gq::kstream_splits(g[i].K);
        if (use_kstream(g[i].fmt, gq::AF_F16, g[i].M, N, g[i].K, act, true, true) &&
            kstream_fits(g[i].M, N, g[i].K, g[i].K, g[i].ldc) && parts + np <= gq::kKMaxParts && (parts += np, true))
            ks[nk++] = gq::KItem{g[i].fmt, g[i].A, g[i].X, g[i].K, g[i].C, g[i].ldc, g[i].M, g[i].K};
        else
            rest[nr++] = g[i];
    }
}

size_t gq_mmq_grouped_prepared_workspace_size(gq_act act, const gq_gemm_item *items, int n, int64_t N)
{
    gq::SGroupItem g[16], rest[16];
    gq::KItem ks[16];
    int nk, nr;
    if (n < 1 || grouped_gemm_items(act, items, n, N, g) != GQ_OK) return 0;
    grouped_split(act, g, n, N, ks, nk, rest, nr);
    // [the K-chunked stream's K-range partials][the streaming GEMM's split-K partials]
    const size_t kb = align_up(gq::kstream_partial_bytes(ks, nk, N));
    if (nr == 0) return kb;
    const gq::SGroupPlan p = gq::plan_sgemm_grouped(rest, nr, N, gq::tuning().sgemm_splits);
    return kb + (p.ok ? p.partial_bytes : 0);
}

int gq_mmq_grouped_prepared(gq_act act, const gq_gemm_item *items, int n, int64_t N, void *workspace,
                            size_t workspace_bytes, void *stream)
{
    g_err.clear();
    gq::SGroupItem g[16], rest[16];
    gq::KItem ks[16];
    int nk, nr;
    int rc = grouped_gemm_items(act, items, n, N, g);
    if (rc != GQ_OK) return rc;
    grouped_split(act, g, n, N, ks, nk, rest, nr);
    // [the K-chunked stream's K-range partials][the streaming GEMM's split-K partials]
    const size_t kb = align_up(gq::kstream_partial_bytes(ks, nk, N));
    gq::SGroupPlan p;
    const size_t need = kb + (nr > 0 ? (p = gq::plan_sgemm_grouped(rest, nr, N, gq::tuning().sgemm_splits)).partial_bytes : 0);
    if (nr > 0 && !p.ok) return fail(GQ_EUNSUPPORTED, "not a grouped GEMM shape");
    if (need && (!workspace || workspace_bytes < need))
        return fail(GQ_EINVAL, "workspace %zu bytes < required %zu", workspace ? workspace_bytes : (size_t)0, need);
    if (nk > 0) {
        const hipError_t e = gq::launch_kstream(ks, nk, N, 0, workspace, (hipStream_t)stream);
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (grouped kstream): %s", hipGetErrorString(e));
    }
    if (nr > 0) {
        const hipError_t e = gq::launch_sgemm_grouped(rest, nr, N, p, (uint8_t *)workspace + kb, (hipStream_t)stream);
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (grouped GEMM): %s", hipGetErrorString(e));
    }
    return GQ_OK;
}

int gq_mmq_sharded(gq_type t, const void *A_shard, const void *B, void *C, int64_t M, int64_t N, int64_t K,
                   int64_t ldb, int64_t ldc, int world, int rank, void *nccl_comm, void *workspace,
                   size_t workspace_bytes, void *stream)
{
    g_err.clear();
    int rc = check_common(t, M, N, K);
    if (rc != GQ_OK) return rc;
    if (world < 1 || rank < 0 || rank >= world) return fail(GQ_EINVAL, "bad rank %d of world %d", rank, world);
    if (world > 1 && !nccl_comm) return fail(GQ_EINVAL, "world=%d needs an RCCL communicator", world);
    if (M == 0 || N == 0) return GQ_OK;
    if (K == 0) return fail(GQ_EINVAL, "K must be positive");
    if (!B || !C) return fail(GQ_EINVAL, "null pointer (B=%p C=%p)", B, C);
    if (ldc < M) return fail(GQ_EINVAL, "ldc=%lld < M=%lld", (long long)ldc, (long long)M);
    const size_t need = sharded_ws(t, M, N, K, world);
    if (!workspace || workspace_bytes < need)
        return fail(GQ_EINVAL, "workspace %zu bytes < required %zu", workspace ? workspace_bytes : (size_t)0, need);
    int64_t row0, rows, R;
    shard_geom(M, world, rank, row0, rows, R);
    if (rows > 0 && !A_shard) return fail(GQ_EINVAL, "null A_shard for %lld rows", (long long)rows);
    uint8_t *ws = (uint8_t *)workspace;
    uint16_t *slab = (uint16_t *)ws;                                  // (N, R)
    uint16_t *gathered = (uint16_t *)(ws + align_up((size_t)N * R * 2)); // (world, N, R)
    uint8_t *mws = (uint8_t *)gathered + align_up((size_t)world * N * R * 2);
    const size_t mws_bytes = workspace_bytes - (size_t)(mws - ws);
    hipStream_t s = (hipStream_t)stream;
    if (rows > 0) {
        rc = gq_mmq(t, A_shard, B, slab, rows, N, K, ldb, R, mws, mws_bytes, stream);
        if (rc != GQ_OK) return rc;
    }
    if (world == 1 && !nccl_comm) { // the slab is the output
        hipError_t e = launch_assemble(slab, (uint16_t *)C, N, R, M, ldc, s);
        if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (assemble): %s", hipGetErrorString(e));
        return GQ_OK;
    }
    AllGatherFn ag = shard_allgather();
    if (!ag) return fail(GQ_EUNSUPPORTED, "RCCL (ncclAllGather) not found in the process");
    // (a short or empty last shard sends its slab's pad columns too: assemble never reads them)
    const ncclResult_t nr = ag(slab, gathered, (size_t)N * R, ncclFloat16, (ncclComm_t)nccl_comm, s);
    if (nr != ncclSuccess) return fail(GQ_EHIP, "ncclAllGather failed (%d)", (int)nr);
    hipError_t e = launch_assemble(gathered, (uint16_t *)C, N, R, M, ldc, s);
    if (e != hipSuccess) return fail(GQ_EHIP, "HIP launch failed (assemble): %s", hipGetErrorString(e));
    return GQ_OK;
}

} // extern "C"

const char *gq_debug_route(gq_type t, gq_act act, int64_t M, int64_t N, int64_t K, int prepared)
{
    // the same decisions, in the same order, as gq_mmq_ex (prepared = 0) and compute()
    if (check_common(t, M, N, K) != GQ_OK || check_act(act, K) != GQ_OK || M <= 0 || N <= 0 || K <= 0) return "none";
    g_err.clear();
    const Route r = route(t, act, N, K);
    if (fused_decode_route(t, act, N, K) && (!prepared || prep_raw(act, N, K))) return "stream_decode_kernel";
    if (r.blas) return "dequant_kernel + hipBLASLt";
    if (r.gemv) return "gemv_kernel";
    if (use_kstream(t, r.form, M, N, K, act, prepared != 0))
        return gq::kstream_splits(K) > 1 ? "kstream_kernel + kstream_reduce_kernel" : "kstream_kernel";
    if (rgemm_route(t, r.form, M, N, K, act)) {
        const gq::RGemmPlan p = gq::plan_rgemm(M, N, K);
        return p.splits == 1 ? "rgemm_kernel"
               : gq::rgemm_ilc(t, p) ? "rgemm_kernel (in-launch split-K sum)" : "rgemm_kernel + gemm_reduce_f16_kernel";
    }
    if (use_skinny(t, r.form, N, act)) return "skinny_kernel";
    if (use_sgemm(t, r.form, M, N, K)) {
        gq::SGroupItem it;
        gq::SGroupPlan g;
        if (sgemm_streamk(t, M, N, K, it, g)) return "sgemm_grouped_kernel + reduce_grouped_kernel (stream-K)";
        const gq::RGemmPlan p = sgemm_plan(M, N, K);
        return p.splits == 1 ? "sgemm_kernel"
               : gq::sgemm_ilc(p) ? "sgemm_kernel (in-launch split-K sum)" : "sgemm_kernel + gemm_reduce_f16_kernel";
    }
    return "gemm_kernel + gemm_reduce_f16_kernel";
}
