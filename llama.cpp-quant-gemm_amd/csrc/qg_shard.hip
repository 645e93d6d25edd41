// qg_shard.hip — libqg_shard.so: row-sharded multi-GPU W4A8 product over RCCL (include/qg/qg_shard.h).
//
// One rank per GPU (process or thread), the caller's communicator. Per call, on the caller's stream:
//   1. the rank's rows through libqg_hip.so (qg_gemm_w4a8_ldc, QG_ALGO_AUTO) into its slice of the
//      gather buffer — C itself when M == 1 and N % G == 0 (in-place all-gather), else the
//      [G][M][P] workspace (P = ceil(N / G) rows per rank, equal slices: ONE collective);
//   2. ncclAllGather of the M * P floats (in place: sendbuff = recvbuff + rank * count);
//   3. (workspace form) one reorder kernel [G][M][P] -> C[M][N], dropping the padded columns.
// Nothing else crosses the links: the rows are independent, so there is no exchange
// step. The single-GPU library does not link RCCL; this one does (-lrccl), and calls it only here.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>

#include "qg/qg_shard.h"

namespace {

thread_local int g_last_nccl = 0;

int nccl_status(ncclResult_t r) {
    if (r == ncclSuccess) return QG_OK;
    g_last_nccl = (int)r;
    return QG_ERR_HIP;
}

inline long per_rank(int N, int world) { return ((long)N + world - 1) / world; }

// recv [G][M][P] -> C[M][N]: C[m][g P + j] = recv[g][m][j] for g P + j < N (coalesced along j)
__global__ __launch_bounds__(256) void shard_reorder_kernel(const float* __restrict__ recv, float* __restrict__ C, int M,
                                                            int N, int P) {
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;  // over M * N outputs, n fastest
    if (idx >= (long)M * N) return;
    const int m = (int)(idx / N), n = (int)(idx - (long)m * N);
    const int g = n / P, j = n - g * P;
    C[idx] = recv[((long)g * M + m) * P + j];
}

}  // namespace

extern "C" {

int qg_shard_rows(int N, int world, int rank, int* row0, int* rows) {
    if (N < 0 || world < 1 || rank < 0 || rank >= world || !row0 || !rows) return QG_ERR_INVALID_ARG;
    const long P = per_rank(N, world);
    const long r0 = std::min<long>((long)rank * P, N);
    *row0 = (int)r0;
    *rows = (int)std::min<long>(P, N - r0);
    return QG_OK;
}

size_t qg_sharded_gemm_workspace_size(int M, int N, int world) {
    if (M <= 0 || N <= 0 || world < 1) return 0;
    if (M == 1 && N % world == 0) return 0;
    return (size_t)world * (size_t)M * (size_t)per_rank(N, world) * sizeof(float);
}

int qg_sharded_gemm_w4a8_local(const void* A, const void* B_shard, float* C_slice, int M, int N, int K, int wtype,
                               int world, int rank, qg_stream_t stream) {
    int row0 = 0, rows = 0;
    const int rc = qg_shard_rows(N, world, rank, &row0, &rows);
    if (rc != QG_OK) return rc;
    if (M < 0) return QG_ERR_INVALID_ARG;
    if (M == 0 || rows == 0) return QG_OK;  // an empty shard leaves its (padding) slice untouched
    return qg_gemm_w4a8_ldc(A, B_shard, C_slice, M, rows, K, per_rank(N, world), wtype, QG_ALGO_AUTO, stream);
}

int qg_sharded_gemm_w4a8(const void* A, const void* B_shard, float* C, int M, int N, int K, int wtype, void* ws,
                         size_t ws_bytes, qg_nccl_comm_t comm, qg_stream_t stream) {
    // Arguments every rank passes alike (the communicator, the shape, the replicated activations and the
    // output) are checked before anything is enqueued: on an error here EVERY rank returns before the
    // collective, so none waits for the others.
    if (!comm) return QG_ERR_INVALID_ARG;
    if (M < 0 || N < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (M == 0 || N == 0) return QG_OK;
    if (!A || !C) return QG_ERR_INVALID_ARG;
    int world = 0, rank = 0;
    if (nccl_status(ncclCommCount((ncclComm_t)comm, &world)) != QG_OK) return QG_ERR_HIP;
    if (nccl_status(ncclCommUserRank((ncclComm_t)comm, &rank)) != QG_OK) return QG_ERR_HIP;
    int row0 = 0, rows = 0;
    qg_shard_rows(N, world, rank, &row0, &rows);
    const long P = per_rank(N, world);
    const size_t count = (size_t)M * (size_t)P;
    hipStream_t st = (hipStream_t)stream;
    const bool in_place = M == 1 && N % world == 0;
    const size_t need = qg_sharded_gemm_workspace_size(M, N, world);
    const bool ws_ok = in_place || (ws && ws_bytes >= need && ((uintptr_t)ws & 15) == 0);
    // A missing or short workspace where the gather buffer does not fit in C (N % world != 0) is reported
    // before anything is enqueued: its size depends only on (M, N, world), which every rank shares, so a
    // caller passing the workspace alike on every rank gets this error on every rank (none waits).
    if (!ws_ok && N % world != 0) return QG_ERR_UNSUPPORTED;
    // From here on a failure is RANK-LOCAL (this rank's shard pointer, its workspace, its kernel): the rank
    // still takes part in the one collective — with its slice set to NaN — and returns the error after it,
    // so its peers complete the all-gather (and see NaN columns) instead of blocking in it. The error path
    // allocates nothing: without a usable workspace (N % world == 0 here) the world * M * P =
    // M * N floats of the gather land in C itself, which is then set to NaN.
    int local_rc = ws_ok ? QG_OK : QG_ERR_UNSUPPORTED;
    float* recv = in_place || !ws_ok ? C : static_cast<float*>(ws);
    float* mine = recv + (size_t)rank * count;
    if (local_rc == QG_OK && rows > 0 && !B_shard) local_rc = QG_ERR_INVALID_ARG;
    if (local_rc == QG_OK) local_rc = qg_sharded_gemm_w4a8_local(A, B_shard, mine, M, N, K, wtype, world, rank, stream);
    if (local_rc != QG_OK) (void)hipMemsetD32Async(mine, 0x7FC00000, count, st);  // quiet NaN
    int rc = nccl_status(ncclAllGather(mine, recv, count, ncclFloat32, (ncclComm_t)comm, st));
    if (rc == QG_OK && local_rc == QG_OK && !in_place) {
        const long total = (long)M * N;
        hipLaunchKernelGGL(shard_reorder_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                           (const float*)recv, C, M, N, (int)P);
        if (hipGetLastError() != hipSuccess) rc = QG_ERR_HIP;
    }
    // the failing rank's own C: all NaN (its slice never reached its peers as numbers either)
    if (local_rc != QG_OK) (void)hipMemsetD32Async(C, 0x7FC00000, (size_t)M * N, st);
    return local_rc != QG_OK ? local_rc : rc;
}

int qg_shard_all_gather_f32(const float* send, float* recv, size_t count, qg_nccl_comm_t comm, qg_stream_t stream) {
    if (!comm || !send || !recv) return QG_ERR_INVALID_ARG;
    if (count == 0) return QG_OK;
    return nccl_status(ncclAllGather(send, recv, count, ncclFloat32, (ncclComm_t)comm, (hipStream_t)stream));
}

int qg_shard_get_unique_id(void* id128) {
    if (!id128) return QG_ERR_INVALID_ARG;
    static_assert(sizeof(ncclUniqueId) == QG_NCCL_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    const int rc = nccl_status(ncclGetUniqueId(&id));
    if (rc == QG_OK) memcpy(id128, &id, sizeof(id));
    return rc;
}

int qg_shard_comm_init_rank(qg_nccl_comm_t* comm, int world, const void* id128, int rank) {
    if (!comm || !id128 || world < 1 || rank < 0 || rank >= world) return QG_ERR_INVALID_ARG;
    ncclUniqueId id;
    memcpy(&id, id128, sizeof(id));
    ncclComm_t c = nullptr;
    const int rc = nccl_status(ncclCommInitRank(&c, world, id, rank));
    *comm = rc == QG_OK ? (qg_nccl_comm_t)c : nullptr;
    return rc;
}

int qg_shard_comm_destroy(qg_nccl_comm_t comm) {
    if (!comm) return QG_ERR_INVALID_ARG;
    return nccl_status(ncclCommDestroy((ncclComm_t)comm));
}

int qg_shard_comm_count(qg_nccl_comm_t comm, int* world) {
    if (!comm || !world) return QG_ERR_INVALID_ARG;
    return nccl_status(ncclCommCount((ncclComm_t)comm, world));
}

int qg_shard_comm_rank(qg_nccl_comm_t comm, int* rank) {
    if (!comm || !rank) return QG_ERR_INVALID_ARG;
    return nccl_status(ncclCommUserRank((ncclComm_t)comm, rank));
}

int qg_shard_last_nccl_error(void) { return g_last_nccl; }

}  // extern "C"
