/*
 * qg/qg.h — C-ABI of the MI355X (gfx950) W4A8 quantized GEMM/GEMV library `libqg_hip.so`.
 *
 * Plain C: raw device pointers, sizes, an opaque HIP stream. Every call is stream-ordered and
 * asynchronous (no host sync — the one exception is the one-time growth of a workspace the library
 * keeps for a stream, see qg_gemm_w4a8_ws / qg_gemm_w4a16_ws, which the _ws forms avoid), reentrant;
 * the caller owns all buffers
 * (destination-passing, schemas/docs/solution.md:27-42). Unlike the reference's `void` launch
 * wrappers (include/gemm_cuda_naive.cuh:285-292 — no error check), every entry point returns a
 * qg_status: 0 on success, a negative code otherwise; nothing is launched on a validation error.
 *
 * Conventions (the two-convention trap):
 *   activation-major  C[M][N] = A_q8_1[M][K] . B_w[N][K]^T   M = tokens, N = weight rows
 *                     (include/gemm_reference.h:7-13, 175-222; include/llama_adapter.h)
 *   weight-major      out[M][N] = W[M][K] . A_q8_1[N][K]^T   M = weight rows, N = tokens
 *                     (kernels/gemm/gemm_quant_formats.cuh:312-334, python/quant_gemm)
 * Block layouts: qg/blocks.h (byte-identical to include/quant_types.h / compat/ggml_types.h).
 */
#ifndef QG_QG_H
#define QG_QG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Binary-compatible with hipStream_t (NULL = the default stream). */
typedef struct ihipStream_t* qg_stream_t;

/* Quantization type ids = ggml_type ids (compat/ggml_types.h:199-215). */
typedef enum {
    QG_TYPE_F32 = 0,
    QG_TYPE_F16 = 1,
    QG_TYPE_Q4_0 = 2,
    QG_TYPE_Q4_1 = 3,
    QG_TYPE_Q5_0 = 6,
    QG_TYPE_Q5_1 = 7,
    QG_TYPE_Q8_0 = 8,
    QG_TYPE_Q8_1 = 9
} qg_type;

typedef enum {
    QG_OK = 0,
    QG_ERR_INVALID_ARG = -1, /* null pointer, negative size, unknown kernel_type */
    QG_ERR_BAD_K = -2,       /* K (or element count) not a positive multiple of 32 */
    QG_ERR_UNSUPPORTED = -3, /* weight type / algorithm not available for this shape */
    QG_ERR_ALIGN = -4,       /* pointer alignment below what the block format allows */
    QG_ERR_HIP = -5          /* HIP launch error (see qg_last_hip_error) */
} qg_status;

/* Kernel family selection for qg_gemm_w4a8_ex (QG_ALGO_AUTO picks by shape). */
typedef enum {
    QG_ALGO_AUTO = 0,
    QG_ALGO_GEMV = 1,    /* M <= 8 (auto: M <= 4): register-resident weight units; Q4_0/Q4_1 nibble-plane
                            v_dot8_u32_u4 / v_dot8_i32_i4, Q5_x/Q8_0 byte decode + v_dot4 */
    QG_ALGO_MFMA = 2,    /* any M (auto: M >= 5), K % 128 == 0: v_mfma_i32_16x16x32_i8 per Q-block */
    QG_ALGO_GENERIC = 3, /* any K % 32 == 0, any alignment: byte loads, one wave per output (cross-check) */
    QG_ALGO_RAGGED = 4   /* any K % 32 == 0 (odd K / 32), 2-B aligned weights: one wave per weight row */
} qg_algo;

/* ---- W4A8 GEMM, activation-major ---------------------------------------------------------
 * Replaces gemm_w4a8_{naive,tiled,dp4a,tiled_dp4a,vectorized_dp4a}(A, B, C, M, N, K, stream)
 * (include/gemm_cuda_naive.cuh:285-292, gemm_cuda_tiled.cuh:293-300, gemm_cuda_dp4a.cuh:409-444)
 * and is the device twin of gemm_w4a8_reference (include/gemm_reference.h:175-222).
 * A: block_q8_1[M][K/32]; B: blocks of `wtype` (Q4_0/Q4_1/Q5_0/Q5_1, or Q8_0 = W8A8) [N][K/32];
 * C: float[M][N], overwritten. M == 0 or N == 0 is a no-op. */
int qg_gemm_w4a8(const void* A_q8_1, const void* B, float* C, int M, int N, int K, int wtype, qg_stream_t stream);
int qg_gemm_w4a8_ex(const void* A_q8_1, const void* B, float* C, int M, int N, int K, int wtype, int algo,
                    qg_stream_t stream);
/* As qg_gemm_w4a8_ex with an output row stride: C[m * ldc + n], ldc >= N floats (e.g. a rank's
 * column slice of a wider buffer in the row-sharded multi-GPU path, quant_gemm/sharded.py). */
int qg_gemm_w4a8_ldc(const void* A_q8_1, const void* B, float* C, int M, int N, int K, int64_t ldc, int wtype,
                     int algo, qg_stream_t stream);

/* The Solution entry point of the definition gemm_q4_0_q8_1_w4a8
 * (schemas/definitions/gemm/gemm_q4_0_q8_1_w4a8.json:35-53: inputs A_q8_1[M][K/32], B_q4_0[N][K/32],
 * output C[M][N]; destination-passing, schemas/docs/solution.md:27-42), in definition order —
 * the role include/gemm_cuda_dp4a.cuh::gemm_q4_0_q8_1_dp4a plays for the reference's CUDA
 * solutions (schemas/solutions/gemm_q4_0_q8_1_cuda_dp4a.json:15). == qg_gemm_w4a8(..., QG_TYPE_Q4_0).
 * Registered by integration/solutions/gemm_q4_0_q8_1_hip_gfx950.json. */
int qg_gemm_q4_0_q8_1_w4a8(const void* A_q8_1, const void* B_q4_0, float* C, int M, int N, int K,
                           qg_stream_t stream);

/* As qg_gemm_w4a8 (QG_ALGO_AUTO) with a caller workspace for the odd-K/32 prefill route (K/32 not a
 * multiple of 8, or 2-B aligned weights, at M >= 32 and N >= 1024): weights and activations are
 * copied into zero-padded rows inside `workspace` (>= qg_gemm_w4a8_workspace_size(M, N, K, wtype)
 * bytes, 256-B aligned; 0 for shapes that never take that route) and the MFMA kernel runs on the
 * copy. Capture-safe (a graph keeps the caller's pointer). Without a workspace, qg_gemm_w4a8 uses
 * a buffer the library keeps per (device, stream) — it grows to the largest N*K'/32*bb +
 * M*K'/32*36 bytes seen on that stream (K' = K rounded up to 256), is held until
 * qg_release_workspaces(), and growing it synchronizes that stream once; during stream capture
 * that buffer is never used and such shapes run the ragged kernel instead (same results to the
 * summation-order bound, not bit for bit). Weights used many times: repack once with
 * qg_repack_weights and call qg_gemm_w4a8_prepacked. */
size_t qg_gemm_w4a8_workspace_size(int M, int N, int K, int wtype);
int qg_gemm_w4a8_ws(const void* A_q8_1, const void* B, float* C, int M, int N, int K, int wtype, void* workspace,
                    size_t workspace_bytes, qg_stream_t stream);

/* (Round 5: for weights reused across calls the tiled layout below — qg_tile_weights +
 * qg_gemm_w4a8_tiled, or qg_gemm_w4a8_tiled_act with tiled activations — is the faster route for odd K/32
 * as well: M = 32, K = 4128 6.1-6.2 us against 7.4 us here and 7.2 us for qg_gemm_w4a8_padded; DESIGN.md §6.
 * The padded rows below stay for callers that keep the reference row layout.)
 * Load-time weight layout for K/32 not a multiple of 8 (e.g. K = 4128): rows of K'/32 blocks,
 * K'/32 = round_up(K/32, 8), the real blocks first and then zero blocks (d = 0: every padded term is
 * an exact +0 of the reference's sum). qg_repack_weights writes B_packed (16-B aligned,
 * qg_repack_weights_bytes(N, K, wtype) bytes) from B [N][K/32]; one streaming kernel.
 * qg_gemm_w4a8_prepacked then computes the SAME product as qg_gemm_w4a8(A, B, ...) (within the
 * summation-order bound; K is the logical K) from B_packed: the activations are padded into
 * `workspace` (>= qg_gemm_w4a8_prepacked_workspace_size(M, K) bytes, 16-B aligned; 0 when K/32 is
 * already a multiple of 8) and the QG_ALGO_AUTO kernel runs on K' — no per-call weight copy. From M = 5
 * (the MFMA kernel) the activations are read in place instead (round 5: one launch, the workspace
 * is not touched). Capture-safe. */
size_t qg_repack_weights_bytes(int N, int K, int wtype);
int qg_repack_weights(const void* B, void* B_packed, int N, int K, int wtype, qg_stream_t stream);
size_t qg_gemm_w4a8_prepacked_workspace_size(int M, int K);
/* The activation side of the same layout, written by the quantizer itself so the product is ONE
 * launch: qg_quantize_q8_1_padded quantizes M rows of K floats (as qg_quantize_q8_1) into rows of
 * K'/32 Q8_1 blocks, zero blocks after the real ones; qg_gemm_w4a8_padded(A_padded, B_packed, ...)
 * then runs the QG_ALGO_AUTO kernel on K' directly (K is the logical K). */
int qg_quantize_q8_1_padded(const float* x, void* y, int M, int K, qg_stream_t stream);
int qg_gemm_w4a8_padded(const void* A_padded, const void* B_packed, float* C, int M, int N, int K, int wtype,
                        qg_stream_t stream);
int qg_gemm_w4a8_prepacked(const void* A_q8_1, const void* B_packed, float* C, int M, int N, int K, int wtype,
                           void* workspace, size_t workspace_bytes, qg_stream_t stream);

/* Load-time TILED weight layout (round 5) — the fast form for weights used many times, any K % 32 == 0.
 * qg_tile_weights writes B_tiled (16-B aligned, qg_tile_weights_bytes(N, K, wtype) bytes) from B
 * [N][K/32]: rows in tiles of 32, K/32 in stages of 4 blocks, each (tile, stage) one contiguous run of
 * 128 * block_bytes bytes whose fields are arranged in the prefill kernel's operand order (qs by MFMA
 * k-slot, then qh, then the f16 scales); rows past N and blocks past K/32 are zero (d = 0: an exact +0
 * term). The layout is specified in llama.cpp-quant-gemm_amd/csrc/qg_mmq_kernel.hpp (tiled_fmt) and
 * restated in oracle/oracle.py (tile_weights); one streaming kernel.
 * qg_gemm_w4a8_tiled then computes the same product as qg_gemm_w4a8(A, B, ...) (activation-major,
 * A: block_q8_1 [M][K/32], 16-B aligned; within the reassociation bound of the MFMA kernel, DESIGN.md
 * §5; for M = 1..2 the tiled decode GEMV, whose per-block terms are the reference's bit for bit, summed in
 * a fixed order; for M = 3..4, and M = 2 at K/32 > 256, the MFMA small-batch decode, within the same
 * reassociation bound) from B_tiled in ONE launch for every M — the prefill's weight stages are one linear
 * stream instead of 32 row segments. K/32 need not be a multiple of 4 or 8 (the kernel windows the plain
 * activation rows). _ldc: output row stride (>= N floats). qg_debug_sumi_tiled / qg_debug_config_tiled
 * are the parity hook and the configuration query of the same instantiation (as qg_debug_sumi /
 * qg_debug_config below). Replaces the tiled-GEMM role of include/gemm_cuda_tiled.cuh:293-300 and the
 * cp.async-staged kernels/gemm/gemm_async_copy.cuh:65-232 for reused weights.
 * DECODE ON THE TILED LAYOUT (measured, one MI355X, N = 4096, profiles/r06_tuning/r6o_ab_tiled_decode_final.txt):
 * at K = 14336 (the reference's published decode shapes) Q4_0 M = 1 / 2 / 3 / 4 / 8 run 7.77 / 8.27 / 9.10 /
 * 9.39 / 9.82 us against 7.65 / 8.84 / 10.45 / 11.31 / 10.11 on the reference rows (Q8_0 M = 4 13.49 vs 18.32)
 * — one tiled copy serves decode and prefill; at N = K = 4096 M = 1 / 2 / 3 / 4 run 3.94 / 4.18 / 4.30 / 4.38
 * against 3.39 / 3.75 / 4.21 / 4.50: a caller bound by single-token decode at such K keeps the rows for M <= 2
 * (qg_gemm_w4a8) and tiles a second copy only if its batched decode or prefill needs it.
 * Limits (QG_ERR_UNSUPPORTED, nothing launched; the tiled layout has no generic kernel): output strides
 * past INT32_MAX; M <= 4 with K > 16384 whose shape the MFMA kernel rejects too; tiled weights of a
 * (tile, stage) run count past 2^31 bytes; plain activation rows of 2 GiB or more under the windowed
 * (odd K/32) MFMA path. */
size_t qg_tile_weights_bytes(int N, int K, int wtype);
int qg_tile_weights(const void* B, void* B_tiled, int N, int K, int wtype, qg_stream_t stream);
int qg_gemm_w4a8_tiled(const void* A_q8_1, const void* B_tiled, float* C, int M, int N, int K, int wtype,
                       qg_stream_t stream);
int qg_gemm_w4a8_tiled_ldc(const void* A_q8_1, const void* B_tiled, float* C, int M, int N, int K, int64_t ldc,
                           int wtype, qg_stream_t stream);
int qg_debug_sumi_tiled(const void* A_q8_1, const void* B_tiled, int32_t* sumi, int M, int N, int K, int wtype,
                        qg_stream_t stream);
int qg_debug_config_tiled(int M, int N, int K, int wtype, int sumi, char* buf, size_t len);

/* TILED ACTIVATIONS (round 5) — the activation side of the tiled layout, for the prefill on tiled weights:
 * tokens in tiles of 16, K/32 in stages of 4 blocks, each (token tile, stage) one contiguous run of 2304 bytes
 * holding the 16 tokens' 4 block_q8_1 (token-major: token t's blocks at t * 144 + j * 36); tiles follow each
 * other tile-major, stages within a tile in order; tokens past M (to a multiple of 16) and blocks past K/32 (to
 * a multiple of 4) are zero blocks. qg_activations_tiled_bytes(M, K) sizes it. qg_quantize_q8_1_tiled writes it
 * straight from FP32 rows (16-B aligned x and A_tiled; each real block's bytes are qg_quantize_q8_1's);
 * qg_tile_activations rearranges existing Q8_1 rows into it. qg_gemm_w4a8_tiled_act(A_tiled, B_tiled, ...)
 * then computes the same product as qg_gemm_w4a8_tiled(A_q8_1, B_tiled, ...) (the same kernels and tile
 * configurations, so the same bits) with every stage of BOTH operands one linear DMA stream. _ldc, the parity
 * hook and the configuration query as for qg_gemm_w4a8_tiled. */
size_t qg_activations_tiled_bytes(int M, int K);
int qg_quantize_q8_1_tiled(const float* x, void* A_tiled, int M, int K, qg_stream_t stream);
int qg_tile_activations(const void* A_q8_1, void* A_tiled, int M, int K, qg_stream_t stream);
int qg_gemm_w4a8_tiled_act(const void* A_tiled, const void* B_tiled, float* C, int M, int N, int K, int wtype,
                           qg_stream_t stream);
int qg_gemm_w4a8_tiled_act_ldc(const void* A_tiled, const void* B_tiled, float* C, int M, int N, int K, int64_t ldc,
                               int wtype, qg_stream_t stream);
int qg_debug_sumi_tiled_act(const void* A_tiled, const void* B_tiled, int32_t* sumi, int M, int N, int K, int wtype,
                            qg_stream_t stream);
int qg_debug_config_tiled_act(int M, int N, int K, int wtype, int sumi, char* buf, size_t len);

/* W8A8: Q8_0 weights x Q8_1 activations, term sumi * d_a * d_w. Replaces gemm_w8a8_{naive,dp4a}
 * (include/gemm_cuda_naive.cuh:294-301, gemm_cuda_dp4a.cuh:418-425); device twin of
 * gemm_w8a8_reference (include/gemm_reference.h:233-267). Same as qg_gemm_w4a8(..., QG_TYPE_Q8_0). */
int qg_gemm_w8a8(const void* A_q8_1, const void* B_q8_0, float* C, int M, int N, int K, qg_stream_t stream);

/* ---- W4A16 / W8A16: FP32 activations, fp32 arithmetic -----------------
 * C[M][N] = A_f32[M][K] . dequant(B)[N][K]^T, activation-major. Replaces gemm_w4a16_{naive,tiled}
 * (include/gemm_cuda_naive.cuh:267-274, gemm_cuda_tiled.cuh:284-291) and gemm_w8a16_naive
 * (gemm_cuda_naive.cuh:276-283); device twin of gemm_w4a16_reference (gemm_reference.h:73-112).
 * Results agree with the reference to fp32 summation order (each block's products are summed,
 * then scaled by d once); the bf16-MFMA prefill (M > 8, K % 256 == 0) represents each activation
 * exactly (three bf16 parts) below K = 1024 and as two round-to-nearest bf16 parts from K = 1024
 * (added error <= 2^-16 sum_k |a_k w_k|, an eighth or less of the fp32 K-term bound
 * 2 (K + 2) 2^-24 sum_k |a_k w_k|; the high part is clamped to the largest finite bf16, so
 * activations up to FLT_MAX keep that bound and an infinite activation gives an infinite, not a NaN,
 * product). A: 4-B aligned floats (16-B for the fast path), any K % 32 == 0.
 * 8 < M <= 32 with 16-B aligned A and B, K % 256 == 0, K <= 8192 and a grid of at most one workgroup
 * per CU runs without split-K and without any workspace (round 4: each workgroup owns all of K; outputs
 * deterministic); qg_gemm_w16_workspace_size still sizes the split-K route those shapes take when the
 * operands are not 16-B aligned.
 * Prefill (M > 8, K % 256 == 0) otherwise splits K across workgroups when that fills the GPU; the partial
 * tiles live in a workspace the library allocates once per (device, stream), on the first such
 * call outside stream capture. Calls made during stream capture never use the library's
 * workspace: they run without split-K (same results to fp32 summation order), so a graph holds
 * no pointer the library may free. qg_release_workspaces() frees them (after a device synchronize;
 * call it when no other thread is inside the library, e.g. at teardown).
 * The _ws forms take the caller's workspace instead (for graphs and multi-stream callers):
 * >= qg_gemm_w16_workspace_size(M, N, K) bytes (0: no split-K for this shape), 256-B aligned,
 * zeroed once before its first use. Its layout is shape-independent: a counter region that every
 * call leaves zeroed again, then scratch partial tiles — so one workspace serves calls of any
 * shapes on one stream. Calls that may run concurrently need distinct workspaces. A smaller or
 * misaligned workspace is not used. */
void qg_release_workspaces(void);
size_t qg_gemm_w16_workspace_size(int M, int N, int K);
int qg_gemm_w4a16_ws(const float* A, const void* B_q4_0, float* C, int M, int N, int K, void* workspace,
                     size_t workspace_bytes, qg_stream_t stream);
int qg_gemm_w8a16_ws(const float* A, const void* B_q8_0, float* C, int M, int N, int K, void* workspace,
                     size_t workspace_bytes, qg_stream_t stream);
int qg_gemm_w4a16(const float* A, const void* B_q4_0, float* C, int M, int N, int K, qg_stream_t stream);
int qg_gemm_w8a16(const float* A, const void* B_q8_0, float* C, int M, int N, int K, qg_stream_t stream);
/* python/quant_gemm/csrc/gemm_ops.cu:431-466 gemm_q4_0_fp32_cuda(weight_q [N][K/32], activation
 * [M][K], M, N, K) -> out[M][N]: the same product, weight-first argument order. */
int qg_gemm_q4_0_fp32(const void* weight_q4_0, const float* activation, float* out, int M, int N, int K,
                      qg_stream_t stream);

/* Strided batch of independent products (e.g. the experts of an MoE layer, or several projections
 * sharing nothing): item i uses A + i*strideA, B + i*strideB (bytes) and C + i*strideC (floats).
 * One launch on the GEMV path (M <= 8), so the per-launch cost is paid once for the batch. */
int qg_gemm_w4a8_strided_batched(const void* A_q8_1, int64_t strideA, const void* B, int64_t strideB, float* C,
                                 int64_t strideC, int batch, int M, int N, int K, int wtype, qg_stream_t stream);

/* Grouped products with independent pointers and row counts (a decoder layer's Q / K / V or
 * gate / up projections; the experts an MoE step selects): item i computes
 * C_i[m * ldc_i + n] = A_i[M][K] . B_i[N_i][K]^T (ldc_i = 0 means N_i). One M, K and weight type for
 * the group. Where QG_ALGO_AUTO picks the GEMV for every item (M <= 4 at aligned shapes), up to 64
 * items go out in ONE launch (the descriptor travels in the kernel arguments: no device
 * allocation, capture-safe, host `items` array read before return); otherwise the items are
 * enqueued one by one. Either way each C_i is bit-identical to qg_gemm_w4a8_ldc(A_i, B_i, C_i, M,
 * N_i, K, ldc_i, wtype, QG_ALGO_AUTO). Items with N_i == 0 are skipped. Replaces a host loop over
 * gemm_q4_0_q8_1_warp-style launches (kernels/gemm/gemm_warp_optimized.cuh:933-1070). */
typedef struct {
    const void* A_q8_1;  /* block_q8_1 [M][K/32] (items may share it) */
    const void* B;       /* weight blocks [N][K/32] of the group's wtype */
    float* C;            /* [M][ldc] */
    int N;
    int ldc;             /* output row stride in floats, 0 = N */
} qg_gemv_item;
int qg_gemm_w4a8_grouped(const qg_gemv_item* items, int count, int M, int K, int wtype, qg_stream_t stream);

/* ---- weight-major twins (kernels/gemm/gemm_quant_formats.cuh:343-428) ---------------------
 * out[M][N] = W[M][K/32] . A[N][K/32]^T, M = weight rows, N = tokens. */
int qg_gemm_q4_0_q8_1(const void* W, const void* A_q8_1, float* out, int M, int N, int K, qg_stream_t stream);
int qg_gemm_q4_1_q8_1(const void* W, const void* A_q8_1, float* out, int M, int N, int K, qg_stream_t stream);
int qg_gemm_q5_0_q8_1(const void* W, const void* A_q8_1, float* out, int M, int N, int K, qg_stream_t stream);
int qg_gemm_q5_1_q8_1(const void* W, const void* A_q8_1, float* out, int M, int N, int K, qg_stream_t stream);
int qg_gemm_q8_0_q8_1(const void* W, const void* A_q8_1, float* out, int M, int N, int K, qg_stream_t stream);

/* ---- fused activation quantization --------------------------------------
 * Activation-major C[M][N] = Q8_1(X)[M][K] . B[N][K]^T for FP32 activations X[M][K] (dense rows),
 * quantized as quantize_row_q8_1_ref (include/quantize.h:165-193): the results are bit-identical to
 * qg_quantize_q8_1(X) followed by qg_gemm_w4a8 on the same stream.
 *   M <= 4 (X 16-B aligned): ONE launch, the quantization runs in the GEMV prologue (the Q8_1
 *     activations never go through HBM);
 *   otherwise (larger M, or a K the GEMV does not take), with workspace_bytes >=
 *     qg_gemm_w4a8_f32_workspace_size(M, K): quantize into the workspace (4-B aligned device
 *     memory), then the QG_ALGO_AUTO product;
 *   larger M without a workspace: the fused GEMV over 8-row chunks (weights streamed per chunk).
 * X only 4-B aligned is served through the workspace; without one it is QG_ERR_ALIGN. */
size_t qg_gemm_w4a8_f32_workspace_size(int M, int K);
int qg_gemm_w4a8_f32(const float* X, const void* B, float* C, int M, int N, int K, int wtype, void* workspace,
                     size_t workspace_bytes, qg_stream_t stream);

/* Replaces gemm_q4_0_fp16_fused(weight, fp16_activation, output, M, N, K, stream)
 * (kernels/gemm/gemm_fused.cuh:311-338), weight-major: out[M][N] = W_q4_0[M][K/32] .
 * Q8_1(act[N][K])^T, act IEEE half [N tokens][K], quantized with the fused kernel's semantics
 * (gemm_fused.cuh:76-143: tree-reduced amax/sum, id = 1/f16(d), q clamped to +-127) — race-free
 * here. Same dispatch as qg_gemm_w4a8_f32 with M <-> N (tokens); the _ws form
 * takes a workspace of qg_gemm_w4a8_f32_workspace_size(N, K) bytes. */
int qg_gemm_q4_0_fp16_fused(const void* W, const void* act_f16, float* out, int M, int N, int K, qg_stream_t stream);
int qg_gemm_q4_0_fp16_fused_ws(const void* W, const void* act_f16, float* out, int M, int N, int K, void* workspace,
                               size_t workspace_bytes, qg_stream_t stream);
/* The fused kernel's FP16 -> Q8_1 quantizer on its own (k halves, multiple of 32). */
int qg_quantize_q8_1_f16_fused(const void* x_f16, void* y, int64_t k, qg_stream_t stream);

/* ---- quantizers (include/quantize.h:343-368; python/quant_gemm/csrc/gemm_ops.cu:146-202) ----
 * x: float[k] (k = total elements, multiple of 32), y: k/32 blocks of the named type.
 * Bytes are identical to the reference CPU quantizers (quantize_row_*_ref, round half away). */
int qg_quantize_q8_1(const float* x, void* y, int64_t k, qg_stream_t stream);
int qg_quantize_q4_0(const float* x, void* y, int64_t k, qg_stream_t stream);
/* Any type; variant 0 = include/quantize.h semantics, variant 1 (Q8_1 only) =
 * tests/framework/test_framework.cuh:195-225 (s = d * sum(q), q clamped to +-127), variant 2
 * (QG_QVAR_DEFINITION, Q8_1 and Q4_0) = the Solution definitions below. Q4_1/Q5_0/Q5_1
 * follow tests/framework/test_framework.cuh:256-367. */
enum { QG_QVAR_REFERENCE = 0, QG_QVAR_FRAMEWORK = 1, QG_QVAR_DEFINITION = 2 };
int qg_quantize(int type, int variant, const float* x, void* y, int64_t k, qg_stream_t stream);
/* The Solution entry points of the definitions quantize_q8_1 / quantize_q4_0
 * (schemas/definitions/quantization/quantize_q8_1.json:26-33,58 and quantize_q4_0.json:25-32,55: input
 * x[num_elements] f32, output y[num_elements/32] blocks, destination-passing), in definition order,
 * with the definitions' semantics where they differ from include/quantize.h: an all-zero block stores
 * d = 1.0 (not 0); q = round-half-to-EVEN(x / d) (torch.round of a true division, not roundf(x * (1/d)));
 * the stored f16 d is the correctly rounded f16 of amax / 127 (/ 7), the definition's Python float
 * converted once. Q8_1 s = the fp32 sum in element order (the definition's torch.sum order is
 * unspecified). Registered by integration/solutions/quantize_q{8_1,4_0}_hip_gfx950.json. */
int qg_quantize_q8_1_definition(const float* x, void* y, int64_t num_elements, qg_stream_t stream);
int qg_quantize_q4_0_definition(const float* x, void* y, int64_t num_elements, qg_stream_t stream);
/* Dequantize k elements (include/quantize.h:84-102 and the per-format formulas). */
int qg_dequantize(int type, const void* x, float* y, int64_t k, qg_stream_t stream);
int qg_dequantize_q4_0(const void* x, float* y, int64_t k, qg_stream_t stream);

/* ---- parity hook: per-block int32 dots sumi[M][N][K/32] (the reference's inner loop,
 * include/gemm_reference.h:202-212), computed by the SAME kernel instantiation qg_gemm_w4a8_ex
 * launches for this shape and algo (same unit loads, operand records / MFMA fragments and integer
 * dot instructions); only the per-block fp32 epilogue is replaced by a store of the int32 dot.
 * The fp32 terms themselves are checked against the oracle to its summation-order bound (the
 * MFMA-assisted prefill epilogue rounds its scale products differently from the reference). */
int qg_debug_sumi(const void* A_q8_1, const void* B, int32_t* sumi, int M, int N, int K, int wtype, int algo,
                  qg_stream_t stream);
/* The kernel instantiation (family + template parameters + grid) that qg_gemm_w4a8_ex (sumi = 0)
 * or qg_debug_sumi (sumi = 1) would launch for this shape on 256-B aligned buffers, as text;
 * nothing is launched. The parity tests assert the two are the same kernel. */
int qg_debug_config(int M, int N, int K, int wtype, int algo, int sumi, char* buf, size_t len);

/* ---- ggml-facing adapter (include/llama_adapter.h:49-76, declared but never defined there) ----
 * A minimal ggml_tensor view: ne[0] = K (contiguous), ne[1] = rows; nb[] byte strides.
 * activation: Q8_1 [K, M]; weights: Q4_0/Q4_1/Q5_0/Q5_1 [K, N]; output: F32 [N, M] (ggml
 * ne-order), i.e. row-major C[M][N]. kernel_type: NULL or any of the reference's names
 * ("naive", "tiled", "dp4a", "tiled_dp4a", "vectorized_dp4a") or "auto"/"gemv"/"mfma"/"generic". */
typedef struct {
    void* data;
    int type;       /* qg_type */
    int64_t ne[4];  /* elements per dim, ne[0] innermost */
    size_t nb[4];   /* byte stride per dim */
} qg_tensor_view;

int qg_gemm_w4a8_from_view(const qg_tensor_view* activation, const qg_tensor_view* weights, qg_tensor_view* output,
                           const char* kernel_type, qg_stream_t stream);
/* gemm_w4a16_from_ggml (llama_adapter.h:78-90): activation F32 [K, M], weights Q4_0 or Q8_0
 * [K, N], output F32 [N, M]; kernel_type NULL / "naive" / "tiled" / "auto". */
int qg_gemm_w4a16_from_view(const qg_tensor_view* activation, const qg_tensor_view* weights, qg_tensor_view* output,
                            const char* kernel_type, qg_stream_t stream);
/* gemm_fp32_from_ggml (llama_adapter.h:92-103): all three F32. */
int qg_gemm_fp32_from_view(const qg_tensor_view* activation, const qg_tensor_view* weights, qg_tensor_view* output,
                           const char* kernel_type, qg_stream_t stream);
/* validate_tensor_types (llama_adapter.h:110-117): 1 if all three types match, else 0. */
int qg_validate_view_types(const qg_tensor_view* activation, const qg_tensor_view* weights,
                           const qg_tensor_view* output, int expected_activation_type, int expected_weight_type,
                           int expected_output_type);

/* ---- FP32 GEMM C[M][N] = A[M][K] . B[N][K]^T: the unquantized baseline the NMSE is quoted against
 * (gemm_fp32_naive, include/gemm_cuda_naive.cuh:258-265; gemm_fp32_reference,
 * gemm_reference.h:38-58). Any K >= 0, 4-B aligned floats. */
int qg_gemm_fp32(const float* A, const float* B, float* C, int M, int N, int K, qg_stream_t stream);

/* ---- GGUF weight files -------------------------------------------------
 * A read-only mapping of a GGUF v2/v3 file: metadata and tensor directory; Q4_0/Q4_1/Q5_0/Q5_1/
 * Q8_0/Q8_1/F16/F32 tensor data are the same bytes the kernels take. Host-side only, except
 * qg_gguf_upload_tensor (a stream-ordered copy, then a stream sync). Every length and offset is
 * checked against the file size; an unreadable or inconsistent file is QG_ERR_INVALID_ARG.
 * Tensor dims follow ggml: ne[0] = K (contiguous), ne[1] = rows; unused dims are 1. */
typedef struct qg_gguf qg_gguf;
int qg_gguf_open(const char* path, qg_gguf** out);
void qg_gguf_close(qg_gguf* file);
int qg_gguf_version(const qg_gguf* file);
int64_t qg_gguf_alignment(const qg_gguf* file);
int64_t qg_gguf_tensor_count(const qg_gguf* file);
int64_t qg_gguf_find_tensor(const qg_gguf* file, const char* name);   /* -1 if absent */
int qg_gguf_tensor_info(const qg_gguf* file, int64_t index, const char** name, int* type, int* n_dims,
                        int64_t ne[4], uint64_t* nbytes);               /* nbytes 0: type not supported */
const void* qg_gguf_tensor_data(const qg_gguf* file, int64_t index);   /* host pointer into the mapping */
int qg_gguf_upload_tensor(const qg_gguf* file, int64_t index, void* device_dst, size_t dst_bytes,
                          qg_stream_t stream);
/* a ggml-ordered view of the tensor's bytes at device_data, for the *_from_view entry points */
int qg_gguf_tensor_view(const qg_gguf* file, int64_t index, void* device_data, qg_tensor_view* out);
int64_t qg_gguf_kv_count(const qg_gguf* file);
int64_t qg_gguf_find_kv(const qg_gguf* file, const char* key);         /* -1 if absent */
/* GGUF value types: 0 u8, 1 i8, 2 u16, 3 i16, 4 u32, 5 i32, 6 f32, 7 bool, 8 string, 9 array,
 * 10 u64, 11 i64, 12 f64 (arrays: element type and count) */
int qg_gguf_kv_info(const qg_gguf* file, int64_t index, const char** key, int* type, uint64_t* array_count,
                    int* array_type);
int qg_gguf_kv_int(const qg_gguf* file, int64_t index, int64_t* value);
int qg_gguf_kv_float(const qg_gguf* file, int64_t index, double* value);
int qg_gguf_kv_string(const qg_gguf* file, int64_t index, const char** str, uint64_t* len);  /* not NUL-terminated */

/* ---- introspection ---- */
const char* qg_status_string(int status);
int qg_last_hip_error(void);                    /* hipError_t of the last QG_ERR_HIP on this thread */
int qg_select_algo(int M, int N, int K, int wtype); /* what QG_ALGO_AUTO dispatches to */
int qg_block_bytes(int type);                   /* 18/20/22/24/34/36, 0 if unknown */
const char* qg_version(void);

#ifdef __cplusplus
}
#endif

#endif /* QG_QG_H */
