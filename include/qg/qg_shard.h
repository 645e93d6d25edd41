/*
 * qg/qg_shard.h — C-ABI of `libqg_shard.so`: the row-sharded multi-GPU W4A8 product over RCCL
 * (SURVEY.md §8e), for C / C++ callers such as llama.cpp that run one process (or one thread) per GPU.
 *
 * The output rows N are independent (C[:, n] depends only on B[n, :] and the replicated activations),
 * so rank r of a G-rank communicator keeps the contiguous weight rows [r * P, min((r + 1) * P, N)),
 * P = ceil(N / G), resident in its own HBM, computes their outputs with the single-GPU kernels of
 * libqg_hip.so (qg_gemm_w4a8_ldc) and ONE ncclAllGather over xGMI assembles C[M][N] on every rank.
 * No other collective: there is no exchange step in this path.
 *
 * The communicator is the CALLER's (SURVEY.md §8b "one communicator per device, created by the
 * caller-side harness"): a ncclComm_t made with ncclCommInitRank / ncclCommInitAll, passed here as
 * an opaque pointer (binary-compatible with ncclComm_t). qg_shard_comm_init_rank and
 * qg_shard_get_unique_id are thin conveniences for callers without RCCL headers (the Python face,
 * quant_gemm/sharded.py), not a second communicator inside the GEMM.
 *
 * Replaces, on the caller side, the reference's single-device llama_adapter.h entry
 * gemm_w4a8_from_ggml (include/llama_adapter.h:71-76) for a weight tensor split by rows over G devices.
 */
#ifndef QG_QG_SHARD_H
#define QG_QG_SHARD_H

#include <stddef.h>
#include <stdint.h>

#include "qg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ncclComm* qg_nccl_comm_t; /* == ncclComm_t (rccl/rccl.h) */

/* Rank's contiguous row range: *row0 = min(rank * P, N), *rows = min(P, N - *row0) (may be 0),
 * P = ceil(N / world) — the same partition as quant_gemm/sharded.py shard_rows. */
int qg_shard_rows(int N, int world, int rank, int* row0, int* rows);

/* Workspace bytes qg_sharded_gemm_w4a8 needs for this shape on a `world`-rank communicator:
 * 0 when M == 1 and N % world == 0 (the all-gather runs in place in C), else the gather buffer
 * world * M * P floats (16-B aligned device memory; not kept between calls). */
size_t qg_sharded_gemm_workspace_size(int M, int N, int world);

/* C[M][N] = A_q8_1[M][K] . B[N][K]^T on every rank of `comm`, B row-sharded as qg_shard_rows:
 * B_shard holds this rank's rows [rows][K/32] (any of the weight types of qg_gemm_w4a8), A_q8_1 the
 * replicated activations [M][K/32] (device memory of this rank's GPU), C the full output [M][N].
 * Stream-ordered on `stream`: the rank's kernel, then the ncclAllGather, then (unless in place) one
 * reorder kernel from the [world][M][P] gather buffer into C. Each rank runs the kernel QG_ALGO_AUTO
 * picks for its shard: on the GEMV path (M <= 4) every output is bit-identical to qg_gemm_w4a8 on the
 * whole B (per-row summation does not depend on N); beyond it the MFMA tiling (how many waves split
 * K) may follow the shard's N, so outputs agree to the kernels' reassociation bound
 * (tests/test_gpu_shard.py).
 * Returns QG_ERR_INVALID_ARG for a null comm / pointer, QG_ERR_BAD_K, QG_ERR_UNSUPPORTED without a
 * large enough workspace, QG_ERR_HIP for a launch or RCCL error (qg_shard_last_nccl_error).
 * Collective safety: errors in the arguments all ranks share (comm, M, N, K, A, C) are returned before
 * anything is enqueued, on every rank alike; so is a missing / short workspace when N % world != 0 (its
 * size is a function of (M, N, world) alone: pass it alike on every rank). An error local to one rank (a
 * null B_shard with rows to compute, a missing or small workspace when N % world == 0, its kernel's
 * launch) does NOT skip the collective, and its error path allocates nothing: that rank enters the
 * ncclAllGather with its slice set to quiet NaN (0x7FC00000; without a workspace it receives into C),
 * sets its own C to NaN and returns the error afterwards, so its peers finish the call instead of
 * waiting forever. The peers return QG_OK with NaN in the failing rank's columns
 * [rank * P, rank * P + rows): a caller that must know detects it with isnan on those columns or, as
 * usual for rank-local errors, by exchanging the return codes (tests/test_sharded.py shows both). */
int qg_sharded_gemm_w4a8(const void* A_q8_1, const void* B_shard, float* C, int M, int N, int K, int wtype,
                         void* workspace, size_t workspace_bytes, qg_nccl_comm_t comm, qg_stream_t stream);

/* The rank's own part alone (no collective): its [M][P] slice written at C_slice with row stride P
 * — what qg_sharded_gemm_w4a8 computes before the gather (for callers that gather themselves). */
int qg_sharded_gemm_w4a8_local(const void* A_q8_1, const void* B_shard, float* C_slice, int M, int N, int K,
                               int wtype, int world, int rank, qg_stream_t stream);

/* One ncclAllGather of `count` floats per rank (recv = world * count floats, rank-major; in place when
 * send == recv + rank * count) on `stream` — the gather of a step of several local products at once
 * (e.g. G independent GEMVs' [G][M][P] slices written by qg_sharded_gemm_w4a8_local). */
int qg_shard_all_gather_f32(const float* send, float* recv, size_t count, qg_nccl_comm_t comm, qg_stream_t stream);

/* Caller-side conveniences over RCCL (ncclGetUniqueId / ncclCommInitRank / ncclCommDestroy) for
 * callers without RCCL headers: the 128-byte id is created on one rank and broadcast by the caller. */
enum { QG_NCCL_UNIQUE_ID_BYTES = 128 };
int qg_shard_get_unique_id(void* id128);
int qg_shard_comm_init_rank(qg_nccl_comm_t* comm, int world, const void* id128, int rank);
int qg_shard_comm_destroy(qg_nccl_comm_t comm);
int qg_shard_comm_count(qg_nccl_comm_t comm, int* world);
int qg_shard_comm_rank(qg_nccl_comm_t comm, int* rank);
int qg_shard_last_nccl_error(void); /* ncclResult_t of the last failing RCCL call on this thread */

#ifdef __cplusplus
}
#endif

#endif /* QG_QG_SHARD_H */
