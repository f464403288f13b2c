// gguf_internal.hpp -- launchers shared between the kernel translation units and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gq {

// Tuning overrides of the measured defaults.  Read ONCE per process from GQ_* environment
// variables (gq_capi.hip, std::call_once) -- the launch path never calls getenv -- and changed
// at run time only through the debug entry point gq_debug_set_tuning (tests, A/B tools; not
// thread-safe against concurrent launches).  0 / -1 = "the default the code measured".
struct Tuning {
    long long blas_min_tokens = 768;          // GQ_BLAS_MIN_TOKENS: library GEMM from this many tokens (<= 0: never)
    long long gemm_max_bytes = 1LL << 31;     // GQ_GEMM_MAX_BYTES: weight / activation bytes per GEMM launch
    int gemm_i8 = 0;                          // GQ_GEMM_I8: Q8_0 int8-MFMA form
    int fused_decode = 1;                     // GQ_NO_FUSED_DECODE=1 -> 0
    int decode_f8_itc = 1;                    // GQ_DECODE_F8_ITC: fp8 decode keeps x~ in registers at one token
    int decode_q6_img = -1;                   // GQ_DECODE_Q6_IMG: Q6_K aligned ring image (-1: K <= 4096)
    int gemm_aq = 1;                          // GQ_GEMM_AQ: in-kernel quantization of 16/32-token tiles
    int gemm_rg = 0;                          // GQ_GEMM_RG: 1 or 2 (0: auto)
    long long gemm_splits = 0;                // GQ_GEMM_SPLITS: split-K factor (0: auto)
    int gemm_partial_f32 = 0;                 // GQ_GEMM_PARTIAL=f32
    int skinny = -1;                          // GQ_SKINNY: 5..32-token kernel (-1 auto, 0 off, 1 every 1..32)
    int skinny_rg = 0;                        // GQ_SKINNY_RG: fragments per workgroup, 1..4 (0: auto)
    int rgemm = -1;                           // GQ_RGEMM: resident-split GEMM -1 auto / 0 off / 1 wherever it applies
    int sgemm = -1;                           // GQ_SGEMM: streaming 256-row GEMM -1 auto / 0 off / 1 wherever it applies
    int sgemm_splits = 0;                     // GQ_SGEMM_SPLITS (0: auto)
    int sgemm_streamk = -1;                   // GQ_SGEMM_STREAMK: stream-K unit split of the auto plan: 1 every
                                              // streaming GEMM, 0 none, -1 the grouped plans (the measured gain)
    int rgemm_ilc = 0;                        // GQ_RGEMM_ILC: split-K sums inside the GEMM launch (measured slower: opt-in)
    int sgemm_full = -1;                      // GQ_SGEMM_FULL: Q4_K 16/32-token tiles stream whole super-blocks:
                                              // 1 every streaming GEMM, 0 none, -1 single matrices (measured gain)
    int kstream = -1;                         // GQ_KSTREAM: K-chunked streaming MMQ -1 auto / 0 off / 1 wherever it applies
    int cus = 0;                              // GQ_CUS: compute units to plan for (0: the device's count)
    int ablate = 0;                           // GQ_ABLATE (GQ_ABLATION diagnostic builds only)
};
const Tuning &tuning();
// key = the environment variable's name ("GQ_GEMM_SPLITS", ...); value validated (an override
// that no kernel is instantiated for is rejected).  Returns 0, or -1 for an unknown key or a
// value out of range.  reset: back to the environment's values.
int set_tuning(const char *key, long long value);
void reset_tuning();
// compute units of the current device (hipDeviceAttributeMultiprocessorCount, queried once per
// device), or the GQ_CUS override: every "one round of the chip" plan sizes its grid by it
int num_cus();

enum ActMode : int { ACT_AOS = 0, ACT_SOA = 1, ACT_DEQ = 2, ACT_I8 = 3, ACT_F8 = 4, ACT_F8DEQ = 5 };
// Activation form the MFMA GEMM reads (mmq_gemm.hip): fp16 x~ (q8_1's, or the fp8 variant's
// widened e4m3 codes) or q8_1 codes (Q8_0 int8 MFMA).
enum ActForm : int { AF_F16 = 0, AF_I8 = 1 };

// Activation quantizer (act_quant.hip).  AOS: out0 = q8_1 bytes.  SOA: out0 = int8 codes
// [rows][K], out1 = float d [rows][K/32], out2 = float s [rows][K/32].  DEQ: out0 = fp16 x~.
// I8: out0 = int8 codes [rows][K], out1 = float d [K/32][(rows + 3) & ~3] (block-major).
// F8 (the fp8 activation variant, not q8_1): out0 = OCP e4m3 codes [rows][K], each 4-element
// group stored (0,2,1,3); out1 = float 2^e [K/32][(rows + 3) & ~3], e the smallest integer with
// max|x| <= 448 * 2^e over the block (2^0 for an all-zero block); code = e4m3(x / 2^e), RNE.
// F8DEQ: out0 = fp16 code * 2^e [rows][K] in the DEQ layout (the fp8 variant's GEMM input).
// Weight quantizers on the device (quant_device.hip): kind 0 Q8_0 (fp16 in), 1 Q4_K (fp32),
// 2 Q6_K (fp32), 3 Q8_1 (fp16); the host producers' bytes.
hipError_t launch_quant_blocks(int kind, const void *x, void *y, int64_t nblocks, hipStream_t s);

hipError_t launch_act_quant(int mode, const uint16_t *X, int64_t ldx, int64_t rows, int64_t K, void *out0,
                            void *out1, void *out2, hipStream_t s);
// The DEQ form of up to kMaxDeqSegs tensors in one launch (wg0 is set by the launcher),
// bit-identical to launch_act_quant(ACT_DEQ, ...) per tensor.
constexpr int kMaxDeqSegs = 8;
struct DeqSeg {
    const uint16_t *X;
    int64_t ldx, rows, K;
    uint16_t *xdeq;
    int64_t wg0;
};
hipError_t launch_act_quant_deq_grouped(const DeqSeg *segs, int n, hipStream_t s, int mode = ACT_DEQ); // or ACT_F8DEQ

// Decode-shaped GEMV (mmq_gemv.hip): C[t][m] for t < N_tok <= 8 from SOA activations.
hipError_t launch_gemv(int fmt, const uint8_t *A, const int8_t *xq, const float *xd, const float *xs, uint16_t *C,
                       int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s);

// Streaming decode (mmq_decode.hip): q8_1 quantization of the N <= 8 tokens in LDS + the
// weight stream, one launch.  decode_fused_ok() says whether the LDS image fits (else:
// act_quant + launch_gemv).  fp8: the fp8 activation variant's form (e4m3-quantized x~ in LDS,
// fp16 dot products).
bool decode_fused_ok(int fmt, int64_t N, int64_t K, bool fp8 = false);
hipError_t launch_decode_fused(int fmt, const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, int64_t M,
                               int64_t N, int64_t K, int64_t ldc, hipStream_t s, bool fp8 = false);

// Batched GEMM on fp16 MFMA (mmq_gemm.hip): C[t][m] from the dequantized activation x~.
struct GemmPlan {
    int nb = 8;                // 16-token groups per workgroup (tile = 16*nb tokens)
    int rg = 2;                // 16-row groups per wave (8 waves: tile = 128*rg weight rows)
    int splits = 1;            // split-K factor (grid.z)
    int chunks_per_split = 1;  // 256-wide K stages (super-blocks) per split
    int act = AF_F16;          // activation form (AF_I8: Q8_0 only)
    int loaders = 0;           // 4: four dedicated DMA-issuing waves beside the 8 multiplying ones
    int pf16 = 0;              // split-K partials stored as fp16 (else fp32)
    int aq = 0;                // activations quantized in-kernel from raw fp16 (GemmAct::xraw)
    size_t partial_bytes = 0;  // fp32 partial slabs needed when splits > 1
};
// Activations as the GEMM reads them: fp16 x~ (act_quant DEQ) or, for the code forms, codes +
// block-major fp32 scales (act_quant I8 / F8).
struct GemmAct {
    const uint16_t *xdeq = nullptr;
    const int8_t *xq = nullptr;
    const float *xd = nullptr;
    int64_t ldd = 0; // row length of the block-major scale array (all the call's tokens)
    const uint16_t *xraw = nullptr; // aq: the fp16 activations themselves, rows ldx apart
    int64_t ldx = 0;
};
// plan.aq is allowed (in-kernel q8_1 of a 16/32-token tile's split, GemmPlan::aq)
bool gemm_aq_ok(const GemmPlan &p);
// The MFMA GEMM needs K in whole 256-element stages (always true for Q4_K/Q6_K).
bool gemm_supported(int fmt, int64_t K);
// act: the activation form (AF_I8 is honoured for Q8_0 only).
GemmPlan plan_gemm(int fmt, int64_t M, int64_t N, int64_t K, int act = AF_F16);
hipError_t launch_gemm(int fmt, const uint8_t *A, const GemmAct &x, uint16_t *C, float *partials,
                       const GemmPlan &plan, int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s);

// The split-K sum of the fp16 partials gemm_kernel (and rgemm_kernel) write: tiles of 16*8*rg
// rows x 16*nb tokens, S splits (mmq_gemm.hip gemm_reduce_f16_kernel).
hipError_t launch_gemm_reduce_f16(int nb, int rg, const uint16_t *P, uint16_t *C, int64_t M, int64_t N, int64_t ldc,
                                  int S, int tiles_x, int tiles_y, hipStream_t s);

// Resident-split GEMM (mmq_rgemm.hip): 256 rows x 16*nb tokens x one super-block per workgroup,
// the split's weights and activations loaded once into LDS; split-K over every super-block
// (fp16 partials + launch_gemm_reduce_f16).  aq: 0 prepared x~ (X = [N][K] DEQ / F8DEQ form),
// 1 raw fp16 activations (X rows ldx apart) q8_1-quantized in-kernel, 2 raw, fp8-quantized.
struct RGemmPlan {
    bool ok = false;
    int nb = 8, tiles_m = 0, tiles_n = 0, splits = 1;
    size_t partial_bytes = 0;
};

RGemmPlan plan_rgemm(int64_t M, int64_t N, int64_t K);
// the split-K partials summed inside the launch (no reduce launch): plans whose grid the chip holds
bool rgemm_ilc(int fmt, const RGemmPlan &p);
// in-launch combine polls that gave up since the library loaded (0 unless a grid was not resident)
unsigned int ilc_timeouts();
// the K-chunked stream's cross-wave hand-off waits that gave up (0 unless broken)
unsigned int kstream_timeouts();
// resident workgroups one CU holds at once (LDS-bound: Q4_K at 16 tokens 3, at 32 two, else one)
int rgemm_per_cu(int fmt, int nb);
hipError_t launch_rgemm(int fmt, int aq, const uint8_t *A, const uint16_t *X, int64_t ldx, uint16_t *C, void *partials,
                        const RGemmPlan &p, int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s);
// Streaming form (mmq_rgemm.hip sgemm_kernel): the same tile over K splits of several
// super-blocks, half-super-block stages through an LDS ring; prepared x~ only (X = [N][K]).
// splits <= 0: as many as keep the grid within one round of the chip.
RGemmPlan plan_sgemm(int64_t M, int64_t N, int64_t K, int splits);
// its split-K sum inside the launch (as rgemm_ilc; the streaming kernel holds one workgroup per CU)
bool sgemm_ilc(const RGemmPlan &p);
hipError_t launch_sgemm(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, void *partials, const RGemmPlan &p,
                        int64_t M, int64_t N, int64_t K, int64_t ldc, hipStream_t s);

// Several streaming GEMMs in one launch (+ one grouped split-K reduce), at most 16 items sharing
// the token count N; X = each item's prepared x~ ([N][K]).  The plan spreads the super-blocks
// over one round of the chip: the fewest per workgroup that fit, every item split accordingly
// (splits > 0: that split factor for every item, as plan_sgemm's).
struct SGroupItem {
    int fmt;
    const uint8_t *A;
    const uint16_t *X;
    uint16_t *C;
    int64_t ldc, M, K;
};
struct SGroupPlan {
    bool ok = false;
    int nb = 8, tiles_n = 1, blocks = 0;
    int tiles_m[16] = {}, splits[16] = {}, wg0[16] = {};
    bool streamk = false;  // (tile, super-block) units spread evenly over the workgroups (auto splits)
    int U = 0;             // stream-K: total cost of the units (each part's units cost[i]); blocks = the workgroups
    int ustart[16] = {}, scap[16] = {};
    int cost[16] = {}, cstart[16] = {}; // stream-K: a part's per-unit cost, the cost before its first unit
    size_t poff[16] = {};
    size_t foff[16] = {}, noff[16] = {}; // stream-K split parts: the in-launch combine's flags, nonces
    size_t partial_bytes = 0;
};
SGroupPlan plan_sgemm_grouped(const SGroupItem *items, int n, int64_t N, int splits);
hipError_t launch_sgemm_grouped(const SGroupItem *items, int n, int64_t N, const SGroupPlan &g, void *partials,
                                hipStream_t s);

// Grouped decode (mmq_decode.hip): several matrices -- each its own type, activations (N x K
// fp16, row stride ldx) and output (N x M, stride ldc) -- in one launch per token tile, the
// chip's waves split by weight bytes; each matrix's rows come out bit-identical to its own
// launch_decode_fused.  N <= 4, every item decode_fused_ok, at most 16 (item, token group) parts.
struct DecodeItem {
    int fmt;
    const uint8_t *A;
    const uint16_t *X;
    int64_t ldx;
    uint16_t *C;
    int64_t ldc;
    int64_t M, K;
};
bool decode_grouped_ok(const DecodeItem *items, int n, int64_t N, bool fp8 = false);
hipError_t launch_decode_grouped(const DecodeItem *items, int n, int64_t N, hipStream_t s, bool fp8 = false);

// K-chunked streaming MMQ (mmq_kstream.hip, 5..32 tokens): x~ in VGPRs (each of a workgroup's
// 8 waves one K chunk), weights streamed per wave through private LDS rings, the waves' tiles
// summed in LDS: one launch, no partials for K <= 4096.  A longer K is cut into ranges of 16
// super-blocks whose fp32 partial tiles (kstream_partial_bytes of workspace) one small launch
// sums in range order.  Up to kKMaxParts matrices x ranges (own type, activations, output; the
// same N) in one launch, workgroups apportioned by weight bytes; a matrix's bits do not depend on
// the launch it is in.  aq: 0 prepared x~ (X = [N][K], ldx = K, act_quant DEQ / F8DEQ), 1 raw fp16
// q8_1-quantized in-kernel, 2 raw fp16 with the fp8 variant's quantization.
// kstream_ok: K % 256 == 0, M % 16 == 0, < 2 GiB of weights.
constexpr int kKMaxParts = 24;
struct KItem {
    int fmt;
    const uint8_t *A;
    const uint16_t *X;
    int64_t ldx;
    uint16_t *C;
    int64_t ldc, M, K;
};
int kstream_splits(int64_t K);
int kstream_cw(int64_t N, int64_t K);
bool kstream_ok(int fmt, int64_t M, int64_t N, int64_t K);
size_t kstream_partial_bytes(const KItem *items, int n, int64_t N);
hipError_t launch_kstream(const KItem *items, int n, int64_t N, int aq, void *partials, hipStream_t s);

// Skinny-token MMQ (mmq_skinny.hip, 1..32 tokens, K % 256 == 0): 16*rg rows x 16*nb tokens per
// workgroup, K split over its 8 waves (8/nb ranges x nb token tiles), weights and activations
// (fp16 x~, DEQ form) streamed into registers through a d-deep super-block ring, one launch, no
// partials.  rg in 1..4, d = 2.
struct SkinnyPlan {
    int rg = 1, nb = 1, d = 3;
};
SkinnyPlan plan_skinny(int fmt, int64_t M, int64_t N, int64_t K, int rg, int d);
hipError_t launch_skinny(int fmt, const uint8_t *A, const uint16_t *X, uint16_t *C, const SkinnyPlan &plan, int64_t M,
                         int64_t N, int64_t K, int64_t ldc, hipStream_t s);

// Dequantization and the library GEMM (mmq_dequant.hip).  perm: store 4-groups as (0,2,1,3),
// matching act_quant's DEQ form.  blas_gemm returns 0 or a negative code.
hipError_t launch_dequant(int fmt, const uint8_t *A, uint16_t *W, int64_t M, int64_t K, int64_t ldw, bool perm,
                          hipStream_t s);
size_t blas_workspace_bytes();
int blas_gemm(const uint16_t *W, const uint16_t *X, uint16_t *C, int64_t M, int64_t N, int64_t K, int64_t ldc,
              void *ws, size_t ws_bytes, hipStream_t s);

} // namespace gq
