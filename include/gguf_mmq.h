/*
 * gguf_mmq.h -- C ABI of the MI355X GGUF mixed-precision matmul library (libgguf_mmq.so).
 *
 * Plain pointers and sizes only: no torch, no HIP types (streams are passed as void*,
 * i.e. a hipStream_t cast to void*; NULL = the default stream).  All device pointers are
 * HIP device memory on the current device.  Calls are asynchronous on `stream`, never
 * synchronise the host and never allocate (graph-capturable).
 *
 * Notation follows the reference: A is the packed weight matrix with M rows (output
 * features), B the fp16 activations with N rows (tokens), C = (A @ B^T)^T is fp16 (N, M).
 *
 * Reference interfaces these replace (PowerfulGhost/gguf-triton-kernel @ 2025-11-21):
 *   gq_mmq(GQ_Q8_0, ...)  <- kernels/mmq_q8_0.py:102  mmq_q8_0(A, B, M, N, K)
 *   gq_mmq(GQ_Q4_K, ...)  <- kernels/mmq_q4_k.py:240  mmq_q4_k(A, B, M, N, K)
 *   gq_mmq(GQ_Q6_K, ...)  <- kernels/mmq_q6_k.py:197  mmq_q6_k(A, B, M, N, K)
 *   gq_quantize_q8_1      <- utils/quantize/q8_1.py:18 quantize_to_q8_1 (on the device)
 *   gq_quantize_weights   <- utils/quantize/{q8_0.py:4, q4_k.py:87, q6_k.py:97} (on the device)
 *   gq_dequantize         <- utils/quantize/q4_k.py:125, q6_k.py:117, q8_0.py:52 dequantize (device)
 * Beyond the reference (no counterpart there):
 *   gq_*_ex(..., GQ_ACT_FP8_E4M3, ...)  the fp8 activation variant (BASELINE.json configs[4])
 *   gq_quantize_fp8                     its activation quantizer
 */
#ifndef GGUF_MMQ_H
#define GGUF_MMQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { GQ_Q8_0 = 0, GQ_Q4_K = 1, GQ_Q6_K = 2 } gq_type;

/* How the activations are quantized before the matmul.
 *   GQ_ACT_Q8_1      the reference's semantics: q8_1 (int8 per 32 elements, utils/quantize/q8_1.py).
 *   GQ_ACT_FP8_E4M3  the fp8 variant: per 32-element block a power-of-two scale X = 2^e (e the
 *                    smallest integer with max|x| <= 448 * X; X = 1 for an all-zero block) and
 *                    OCP e4m3 (e4m3fn) codes of x / X, round to nearest even; the weights stay in
 *                    their GGUF precision (dequantized to fp16 in registers), products exact in
 *                    fp32.  Needs K % 256 == 0.  Inputs with |x| >= 61440 may round to 65536 and
 *                    overflow fp16. */
typedef enum { GQ_ACT_Q8_1 = 0, GQ_ACT_FP8_E4M3 = 1 } gq_act;

enum {
    GQ_OK = 0,
    GQ_EINVAL = 1,      /* bad argument: null pointer, K not a multiple of the block, ld too small ... */
    GQ_EHIP = 2,        /* a HIP launch failed (message in gq_last_error) */
    GQ_EUNSUPPORTED = 3 /* valid but not implemented (unknown type) */
};

/* Elements per block (32 / 256 / 256) and bytes per block (34 / 144 / 210). */
int gq_block_elems(gq_type t);
int gq_block_bytes(gq_type t);

/* Device workspace for this shape (bytes; the activation quantizer's output and split-K
 * partials): enough for gq_mmq and for gq_act_prepare + gq_mmq_prepared. */
size_t gq_mmq_workspace_size(gq_type t, int64_t M, int64_t N, int64_t K);
size_t gq_mmq_workspace_size_ex(gq_type t, gq_act act, int64_t M, int64_t N, int64_t K);
/* The exact need of one gq_mmq_ex call (<= the above): 0 when the call is a one-launch decode
 * (its quantizer works in LDS), and then workspace may be NULL. */
size_t gq_mmq_call_workspace_size(gq_type t, gq_act act, int64_t M, int64_t N, int64_t K);

/*
 * C[n * ldc + m] = sum_k W[m][k] * x~[n][k]  for m < M, n < N (fp16 out, fp32 accumulate)
 *   A : packed `t` weights, M rows of K/QK blocks, row m at byte m*(K/QK)*block_bytes
 *   B : fp16 activations, row n at element n*ldb (ldb >= K)
 *   x~: B quantized exactly as utils/quantize/q8_1.py does (int8 per 32 elements), the
 *       input the reference's parity oracle (kernels/cpu_impls) consumes.
 * K must be a multiple of gq_block_elems(t) (the reference asserts the same).
 * workspace: >= gq_mmq_workspace_size(t, M, N, K) bytes of device memory
 *            (exactly: gq_mmq_call_workspace_size(t, GQ_ACT_Q8_1, M, N, K); NULL when that is 0).
 * Returns GQ_OK or an error code (gq_last_error() has the text; nothing was launched).
 */
int gq_mmq(gq_type t, const void *A, const void *B, void *C, int64_t M, int64_t N, int64_t K, int64_t ldb,
           int64_t ldc, void *workspace, size_t workspace_bytes, void *stream);
/* gq_mmq with the activation format chosen (gq_mmq == gq_mmq_ex(t, GQ_ACT_Q8_1, ...)). */
int gq_mmq_ex(gq_type t, gq_act act, const void *A, const void *B, void *C, int64_t M, int64_t N, int64_t K,
              int64_t ldb, int64_t ldc, void *workspace, size_t workspace_bytes, void *stream);

/*
 * Split form of gq_mmq.  gq_act_prepare quantizes B into the front of `workspace` (that
 * part depends only on N and K); gq_mmq_prepared then runs the matmul for any weight
 * type and M with that K, using the rest of the workspace (which must be at least
 * gq_mmq_workspace_size(t, M, N, K) bytes in total) for split-K partial sums.  One prepare
 * can serve several weight matrices that share an input (Q/K/V, gate/up).
 * Same result as gq_mmq within the stated tolerances, not always the same kernels: for
 * N <= 4 (fp8: N <= 2) gq_act_prepare also keeps an fp16 copy of B in the workspace and
 * gq_mmq_prepared runs gq_mmq's one-launch fused decode on it -- the same kernel and bits as
 * gq_mmq (round 5; the split form ran the decode-shaped GEMV on the SOA q8_1 form before, and
 * still does where the fused decode does not fit, e.g. 4 tokens at K = 11008); at N = 5..32 (K <= 4096,
 * M % 16 == 0) the split form runs the K-chunked streaming MMQ, and gq_mmq does too at N <= 16 on
 * M >= 8192 rows, else the resident GEMM (the same x~ and products, summed over K in another fp32
 * order: within 4e-3, not bit for bit; GQ_KSTREAM=1 puts both on the stream, GQ_KSTREAM=0 both
 * off it, and then the bits match);
 * for Q8_0 with the int8 GEMM form enabled (GQ_GEMM_I8=1) gq_act_prepare writes both activation
 * forms.
 */
int gq_act_prepare(const void *B, int64_t N, int64_t K, int64_t ldb, void *workspace, size_t workspace_bytes,
                   void *stream);
int gq_mmq_prepared(gq_type t, const void *A, void *workspace, size_t workspace_bytes, void *C, int64_t M, int64_t N,
                    int64_t K, int64_t ldc, void *stream);
/* The split form with the activation format chosen (both calls must name the same one). */
int gq_act_prepare_ex(gq_act act, const void *B, int64_t N, int64_t K, int64_t ldb, void *workspace,
                      size_t workspace_bytes, void *stream);
int gq_mmq_prepared_ex(gq_type t, gq_act act, const void *A, void *workspace, size_t workspace_bytes, void *C,
                       int64_t M, int64_t N, int64_t K, int64_t ldc, void *stream);

/*
 * Several gq_act_prepare_ex calls in as few launches as possible, e.g. the four inputs of one
 * transformer block's projections (no reference counterpart: the reference quantizes inside
 * every matmul).  Item i prepares B_i (N_i x K_i fp16, row stride ldb_i) into its own
 * workspace exactly as gq_act_prepare_ex(act, B_i, ...) would -- the same bytes, the same
 * errors.  Items whose prepared form is the fp16 x~ of the GEMM paths (GQ_ACT_Q8_1 at N >= 5;
 * GQ_ACT_FP8_E4M3's widened codes at every N) share one launch per 8 items; the others are
 * prepared one by one.  Every item is checked
 * before anything is launched: a bad item (GQ_EINVAL / GQ_EUNSUPPORTED) launches nothing.
 * No host sync.
 */
typedef struct gq_prep_item {
    const void *B;
    int64_t N, K, ldb;
    void *workspace;
    size_t workspace_bytes;
} gq_prep_item;
int gq_act_prepare_grouped(gq_act act, const gq_prep_item *items, int n, void *stream);

/*
 * Dequantize packed `t` weights to fp16: W[m * ldw + k] = w (the reference's block formulas,
 * utils/quantize/{q8_0,q4_k,q6_k}.py dequantize, evaluated in fp32, rounded once to fp16).
 * M rows of K (a multiple of the block) elements.  gq_mmq uses the same kernel for its
 * library-GEMM path (N >= a few hundred tokens: fp16 W + hipBLASLt).
 */
int gq_dequantize(gq_type t, const void *A, void *W, int64_t M, int64_t K, int64_t ldw, void *stream);

/*
 * q8_1 quantization of fp16 rows on the device, byte-identical to utils/quantize/q8_1.py:
 * rows x K fp16 (row stride ldx elements) -> rows * K/32 blocks of 36 bytes, row-major.
 */
int gq_quantize_q8_1(const void *X, void *Y, int64_t rows, int64_t K, int64_t ldx, void *stream);

/*
 * The fp8 variant's activation quantizer (GQ_ACT_FP8_E4M3 above) on the device: rows x K fp16
 * (row stride ldx) -> codes [rows][K] e4m3fn bytes, each 4-element group stored in the order
 * (0,2,1,3), and scales [K/32][(rows + 3) & ~3] float X = 2^e (block-major).
 */
int gq_quantize_fp8(const void *X, void *codes, void *scales, int64_t rows, int64_t K, int64_t ldx, void *stream);

/*
 * GGUF weight quantization on the device (the reference quantizes on the host only), byte-
 * identical to the reference's producers and to include/gguf_quant.h's gq_quantize_*:
 *   GQ_Q8_0: X = n fp16 values (n % 32 == 0)  -> Y = n/32 blocks of 34 bytes (quantize_to_q8_0)
 *   GQ_Q4_K: X = n fp32 values (n % 256 == 0) -> Y = n/256 blocks of 144 bytes (quantize_to_q4_k)
 *   GQ_Q6_K: X = n fp32 values (n % 256 == 0) -> Y = n/256 blocks of 210 bytes (quantize_to_q6_k)
 * X is read as flat blocks (a row-major (M, K) matrix gives the packed A of gq_mmq).  One thread
 * per block runs the host producer's exact code; no host sync.
 */
int gq_quantize_weights(gq_type t, const void *X, void *Y, int64_t n, void *stream);

/*
 * Row-sharded MMQ over the GPUs of one node (SURVEY.md 8(b) "gq_mmq_sharded", 8(e)).  The
 * reference is single-GPU and has no counterpart; this is the C form of dist/row_shard.py.
 *
 * gq_shard_rows: rank `rank` of `world` owns weight rows [*row0, *row0 + *rows) of M, padded
 * shard size *R = ceil(M / world) rounded up to 64 (the last shards may be short or empty).
 * Its packed bytes are A + row0 * (K / gq_block_elems(t)) * gq_block_bytes(t): no repacking.
 */
int gq_shard_rows(int64_t M, int world, int rank, int64_t *row0, int64_t *rows, int64_t *R);

/*
 * (world, N, R) fp16 slabs, as an all-gather leaves them -> C (N rows of ldc), columns [0, M):
 * C[n][m] = gathered[m / R][n][m % R].  One device copy kernel on `stream`.
 */
int gq_assemble_shards(const void *gathered, void *C, int world, int64_t N, int64_t R, int64_t M, int64_t ldc,
                       void *stream);

/*
 * One rank's row-sharded MMQ: the local gq_mmq of this rank's rows (A_shard, from
 * gq_shard_rows) into an (N, R) slab, an RCCL all-gather of the slabs over `nccl_comm` (an
 * ncclComm_t of this rank, world ranks; RCCL is resolved at run time from the process, so the
 * caller's own RCCL is the one used), and gq_assemble_shards into C (N, ldc) -- every rank ends
 * with the whole output.  All on `stream`, no host sync (graph-capturable as RCCL allows).
 * world == 1 needs no communicator (NULL: no collective; a 1-rank communicator is used as given).  Workspace: at least
 * gq_mmq_sharded_workspace_size(t, M, N, K, world) bytes.
 */
size_t gq_mmq_sharded_workspace_size(gq_type t, int64_t M, int64_t N, int64_t K, int world);
int gq_mmq_sharded(gq_type t, const void *A_shard, const void *B, void *C, int64_t M, int64_t N, int64_t K,
                   int64_t ldb, int64_t ldc, int world, int rank, void *nccl_comm, void *workspace,
                   size_t workspace_bytes, void *stream);

/*
 * Grouped MMQ: several MMQs of the same token count N (1..32) in one launch, e.g. the
 * projections of one transformer block at decode / small-batch time.  The reference has no
 * counterpart (its kernels/mmq_*.py take one matrix per call); this is the launch the layer
 * dispatcher (kernels/layer_mix.py) makes.  Item i: weights A (M x K of `type`),
 * fp16 activations B (N x K, row stride ldb, q8_1-quantized in the kernel as gq_mmq does), fp16
 * output C (N x M, row stride ldc); items may share B.  N = 1..4: the streaming decode kernel,
 * every item's output bit-identical to its own gq_mmq call; N = 5..32: the K-chunked streaming
 * MMQ (every item bit-identical to its own gq_mmq_ex on that kernel, GQ_KSTREAM=1), which needs
 * K % 256 == 0, K <= 4096, M % 16 == 0, B 16-byte aligned and ldb % 8 == 0.  The chip's workgroups are split over the items by weight bytes.  No workspace, no host
 * sync.  GQ_EUNSUPPORTED (nothing launched) when N > 32, or an item is not a shape of that
 * launch (decode: activations that do not fit LDS, >= 2 GiB of weights, more than 16 parts =
 * item x token group; 5..32: the conditions above, more than 16 items): call gq_mmq per item then.
 */
typedef struct gq_group_item {
    gq_type type;
    const void *A;
    const void *B;
    int64_t ldb;
    void *C;
    int64_t ldc;
    int64_t M, K;
} gq_group_item;
int gq_mmq_grouped(const gq_group_item *items, int n, int64_t N, void *stream);
/* The same with an activation format: GQ_ACT_Q8_1 is gq_mmq_grouped; GQ_ACT_FP8_E4M3 (the fp8
 * variant: its decode form at N <= 2, the K-chunked stream at 3..32) gives every item
 * gq_mmq_ex(..., GQ_ACT_FP8_E4M3, ...)'s bits on that kernel. */
int gq_mmq_grouped_ex(gq_act act, const gq_group_item *items, int n, int64_t N, void *stream);

/*
 * Grouped GEMM: several gq_mmq_prepared_ex calls with the same token count N (5 <= N) in ONE
 * launch of the streaming 256-row MFMA GEMM (+ one launch summing the split-K partials), e.g.
 * the seven projections of a transformer block at prefill (BASELINE.json configs[4]; no
 * reference counterpart).  Item i: weights A (M x K of `type`, K % 256 == 0), ws = the
 * workspace its input was prepared into by gq_act_prepare[_ex|_grouped](act, ..., N, K, ...)
 * (items may share one), output C (N x M, row stride ldc).  The chip's workgroups are spread
 * over the items' row tiles x super-blocks (each item split along K so that the whole launch is
 * one round of the chip); with the split factor pinned (GQ_SGEMM_SPLITS) every item's output is
 * bit-identical to its own gq_mmq_prepared_ex call on that kernel (GQ_SGEMM=1).  At N = 5..32
 * the items with M % 16 == 0 go instead to one launch of the K-chunked streaming MMQ (a K over
 * 4096 in ranges of 4096 whose fp32 partials a second launch sums), each item bit-identical to
 * its own gq_mmq_prepared_ex (which takes the same kernel for K <= 4096; GQ_KSTREAM=1 for
 * longer K); GQ_KSTREAM=0 keeps every item on the streaming GEMM.  workspace: the K-range and
 * split-K partials, >= gq_mmq_grouped_prepared_workspace_size() bytes (0 when nothing splits:
 * NULL allowed).  GQ_EUNSUPPORTED (nothing launched) for N < 5, more than 16 items, K % 256 != 0
 * or >= 2 GiB in one item: call gq_mmq_prepared_ex per item then.  No host sync.
 */
typedef struct gq_gemm_item {
    gq_type type;
    const void *A;
    const void *ws;
    void *C;
    int64_t ldc;
    int64_t M, K;
} gq_gemm_item;
size_t gq_mmq_grouped_prepared_workspace_size(gq_act act, const gq_gemm_item *items, int n, int64_t N);
int gq_mmq_grouped_prepared(gq_act act, const gq_gemm_item *items, int n, int64_t N, void *workspace,
                            size_t workspace_bytes, void *stream);

/* Text of the last error on this thread ("" if none). */
const char *gq_last_error(void);

/* Library ABI version (major * 100 + minor).  103: gq_gemm_item, gq_mmq_grouped_prepared[_workspace_size],
 * gq_debug_route, and larger workspace sizes for the GEMM routes (round 4).  104: gq_mmq_grouped[_ex]
 * takes 5..32 tokens (the K-chunked streaming MMQ; round 5).  105: GEMM workspace sizes grow by the
 * in-launch split-K combine's flag words (opt-in GQ_RGEMM_ILC=1: the resident and streaming GEMMs
 * sum their split-K partials inside their own launch; measured slower, off by default) and
 * gq_debug_sync_timeouts (round 6). */
int gq_version(void);

/*
 * Debug / tuning only (no counterpart in the reference; not for production callers).  The
 * library reads its GQ_* tuning variables from the environment ONCE, at first use; this entry
 * overrides one of them by name (e.g. "GQ_GEMM_SPLITS", "GQ_RGEMM_ILC") for later calls in the
 * process.  Values no kernel is instantiated for are rejected (GQ_EINVAL).  Not thread-safe
 * against calls running concurrently on other threads.  reset: back to the environment's values.
 */
int gq_debug_set_tuning(const char *key, long long value);
void gq_debug_reset_tuning(void);
/* The kernel(s) a gq_mmq_ex call (prepared = 0) or a gq_mmq_prepared_ex call (prepared = 1) of
 * this shape would launch under the current tuning ("none" for an invalid shape): what bench.py
 * names as its roofline kernel.  Split-K reduce kernels are listed whether or not the plan
 * splits. */
const char *gq_debug_route(gq_type t, gq_act act, int64_t M, int64_t N, int64_t K, int prepared);
/* How many synchronisation waits inside a kernel gave up since the library was loaded: the
 * resident GEMM's in-launch split-K combine (only possible when another kernel holds CUs its grid
 * needed) and the K-chunked stream's cross-wave hand-off.  A wait gives up after a bounded spin
 * (wrong bits, never a hang).  Tests assert it stays 0. */
unsigned int gq_debug_sync_timeouts(void);

#ifdef __cplusplus
}
#endif

#endif /* GGUF_MMQ_H */
