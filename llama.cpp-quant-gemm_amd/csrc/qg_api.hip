// qg_api.hip — the C-ABI (include/qg/qg.h): validation, dispatch, error reporting.
//
// No host synchronisation, no allocation: every entry point only validates, picks a kernel family
// and enqueues on the caller's stream, so callers may capture it into a hipGraph.
#include <string.h>

#include "../../include/qg/qg.h"
#include "qg_kernels.hpp"

using namespace qg;

namespace {
thread_local int g_last_hip = 0;

int hip_status(hipError_t e) {
    if (e == hipSuccess) return QG_OK;
    g_last_hip = (int)e;
    return QG_ERR_HIP;
}

bool is_weight_type(int t) { return t == QG_TYPE_Q4_0 || t == QG_TYPE_Q4_1 || t == QG_TYPE_Q5_0 || t == QG_TYPE_Q5_1; }

int select_algo(const GemmArgs& g) {
    if (gemv_eligible(g)) return QG_ALGO_GEMV;
    if (mfma_eligible(g)) return QG_ALGO_MFMA;
    return QG_ALGO_GENERIC;
}

int run_gemm(GemmArgs& g, int algo, hipStream_t st) {
    if (g.M < 0 || g.N < 0) return QG_ERR_INVALID_ARG;
    if (g.K <= 0 || g.K % 32 != 0) return QG_ERR_BAD_K;
    if (!is_weight_type(g.wtype)) return QG_ERR_UNSUPPORTED;
    if (g.M == 0 || g.N == 0) return QG_OK;
    if (!g.A || !g.B || (!g.C && !g.sumi)) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)g.B & 1) != 0) return QG_ERR_ALIGN;  // fp16 fields: 2-byte alignment is the floor
    if (g.batch < 0) return QG_ERR_INVALID_ARG;
    if (g.batch == 0) return QG_OK;
    if (g.batch > 1 && (((uintptr_t)g.sB & 1) != 0 || (g.sA & 3) != 0)) return QG_ERR_ALIGN;
    if (algo == QG_ALGO_AUTO) algo = select_algo(g);
    if (algo == QG_ALGO_GEMV) {
        if (!gemv_eligible(g) || (g.batch > 1 && (g.sB % 16 != 0))) {
            if (g.batch == 1) return QG_ERR_UNSUPPORTED;
            algo = QG_ALGO_GENERIC;  // batch strides break the vector-load alignment: per-item path
        } else {
            if (g.batch > 65535) return QG_ERR_INVALID_ARG;
            return hip_status(launch_gemv(g, st));
        }
    }
    // MFMA and generic kernels take one product per launch: enqueue the batch item by item.
    for (int i = 0; i < g.batch; ++i) {
        GemmArgs gi = g;
        gi.batch = 1;
        gi.A = (const uint8_t*)g.A + (long)i * g.sA;
        gi.B = (const uint8_t*)g.B + (long)i * g.sB;
        if (g.C) gi.C = g.C + (long)i * g.sC;
        int rc;
        switch (algo) {
            case QG_ALGO_MFMA:
                if (!mfma_eligible(gi)) return QG_ERR_UNSUPPORTED;
                rc = hip_status(launch_mfma(gi, st));
                break;
            case QG_ALGO_GENERIC:
                rc = hip_status(launch_generic(gi, st));
                break;
            default:
                return QG_ERR_INVALID_ARG;
        }
        if (rc != QG_OK) return rc;
    }
    return QG_OK;
}

int block_bytes(int t) {
    switch (t) {
        case QG_TYPE_Q4_0: return 18;
        case QG_TYPE_Q4_1: return 20;
        case QG_TYPE_Q5_0: return 22;
        case QG_TYPE_Q5_1: return 24;
        case QG_TYPE_Q8_0: return 34;
        case QG_TYPE_Q8_1: return 36;
    }
    return 0;
}

int weight_major(int wtype, const void* W, const void* A, float* out, int M, int N, int K, qg_stream_t s) {
    // out[mw][nt] = sum_b dot(W[mw][b], A[nt][b]) -> activation-major (m = nt, n = mw) with
    // output strides ldc_m = 1, ldc_n = Ntok.
    GemmArgs g;
    g.A = A; g.B = W; g.C = out; g.M = N; g.N = M; g.K = K; g.wtype = wtype;
    g.ldc_m = 1; g.ldc_n = N;
    return run_gemm(g, QG_ALGO_AUTO, (hipStream_t)s);
}
}  // namespace

extern "C" {

int qg_gemm_w4a8_ex(const void* A, const void* B, float* C, int M, int N, int K, int wtype, int algo,
                    qg_stream_t stream) {
    GemmArgs g;
    g.A = A; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    return run_gemm(g, algo, (hipStream_t)stream);
}

int qg_gemm_w4a8_strided_batched(const void* A, int64_t strideA, const void* B, int64_t strideB, float* C,
                                 int64_t strideC, int batch, int M, int N, int K, int wtype, qg_stream_t stream) {
    GemmArgs g;
    g.A = A; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    g.batch = batch; g.sA = strideA; g.sB = strideB; g.sC = strideC;
    return run_gemm(g, QG_ALGO_AUTO, (hipStream_t)stream);
}

int qg_gemm_w4a8(const void* A, const void* B, float* C, int M, int N, int K, int wtype, qg_stream_t stream) {
    return qg_gemm_w4a8_ex(A, B, C, M, N, K, wtype, QG_ALGO_AUTO, stream);
}

int qg_gemm_q4_0_q8_1(const void* W, const void* A, float* out, int M, int N, int K, qg_stream_t s) {
    return weight_major(QG_TYPE_Q4_0, W, A, out, M, N, K, s);
}
int qg_gemm_q4_1_q8_1(const void* W, const void* A, float* out, int M, int N, int K, qg_stream_t s) {
    return weight_major(QG_TYPE_Q4_1, W, A, out, M, N, K, s);
}
int qg_gemm_q5_0_q8_1(const void* W, const void* A, float* out, int M, int N, int K, qg_stream_t s) {
    return weight_major(QG_TYPE_Q5_0, W, A, out, M, N, K, s);
}
int qg_gemm_q5_1_q8_1(const void* W, const void* A, float* out, int M, int N, int K, qg_stream_t s) {
    return weight_major(QG_TYPE_Q5_1, W, A, out, M, N, K, s);
}

int qg_quantize(int type, int variant, const float* x, void* y, int64_t k, qg_stream_t stream) {
    if (k < 0 || k % 32 != 0) return QG_ERR_BAD_K;
    if (block_bytes(type) == 0) return QG_ERR_UNSUPPORTED;
    if (variant != 0 && !(variant == 1 && type == QG_TYPE_Q8_1)) return QG_ERR_UNSUPPORTED;
    if (k == 0) return QG_OK;
    if (!x || !y) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)x & 3) != 0) return QG_ERR_ALIGN;
    const uintptr_t need = type == QG_TYPE_Q8_1 ? 3 : 1;
    if (((uintptr_t)y & need) != 0) return QG_ERR_ALIGN;
    return hip_status(launch_quantize(type, variant, x, y, k / 32, (hipStream_t)stream));
}

int qg_quantize_q8_1(const float* x, void* y, int64_t k, qg_stream_t s) { return qg_quantize(QG_TYPE_Q8_1, 0, x, y, k, s); }
int qg_quantize_q4_0(const float* x, void* y, int64_t k, qg_stream_t s) { return qg_quantize(QG_TYPE_Q4_0, 0, x, y, k, s); }

int qg_dequantize(int type, const void* x, float* y, int64_t k, qg_stream_t stream) {
    if (k < 0 || k % 32 != 0) return QG_ERR_BAD_K;
    if (block_bytes(type) == 0) return QG_ERR_UNSUPPORTED;
    if (k == 0) return QG_OK;
    if (!x || !y) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)y & 3) != 0 || ((uintptr_t)x & 1) != 0) return QG_ERR_ALIGN;
    return hip_status(launch_dequantize(type, x, y, k / 32, (hipStream_t)stream));
}

int qg_dequantize_q4_0(const void* x, float* y, int64_t k, qg_stream_t s) { return qg_dequantize(QG_TYPE_Q4_0, x, y, k, s); }

int qg_debug_sumi(const void* A, const void* B, int32_t* sumi, int M, int N, int K, int wtype, int algo,
                  qg_stream_t stream) {
    GemmArgs g;
    g.A = A; g.B = B; g.sumi = sumi; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    return run_gemm(g, algo, (hipStream_t)stream);
}

int qg_gemm_w4a8_from_view(const qg_tensor_view* act, const qg_tensor_view* w, qg_tensor_view* out,
                           const char* kernel_type, qg_stream_t stream) {
    if (!act || !w || !out) return QG_ERR_INVALID_ARG;
    int algo = QG_ALGO_AUTO;
    if (kernel_type) {
        static const char* autos[] = {"naive", "tiled", "dp4a", "tiled_dp4a", "vectorized_dp4a", "auto"};
        bool known = false;
        for (const char* a : autos) known = known || strcmp(kernel_type, a) == 0;
        if (known) algo = QG_ALGO_AUTO;
        else if (strcmp(kernel_type, "gemv") == 0) algo = QG_ALGO_GEMV;
        else if (strcmp(kernel_type, "mfma") == 0) algo = QG_ALGO_MFMA;
        else if (strcmp(kernel_type, "generic") == 0) algo = QG_ALGO_GENERIC;
        else return QG_ERR_INVALID_ARG;
    }
    // Dims as extract_dims_from_tensor (include/llama_adapter.h:49-61): M = act->ne[1],
    // K = act->ne[0], N = w->ne[1].
    if (act->type != QG_TYPE_Q8_1 || out->type != QG_TYPE_F32 || !is_weight_type(w->type)) return QG_ERR_UNSUPPORTED;
    for (int d = 2; d < 4; ++d)
        if ((act->ne[d] != 1 && act->ne[d] != 0) || (w->ne[d] != 1 && w->ne[d] != 0) || (out->ne[d] != 1 && out->ne[d] != 0))
            return QG_ERR_UNSUPPORTED;  // batched (ne[2..3] > 1) views are out of scope
    const int64_t K = act->ne[0], M = act->ne[1], N = w->ne[1];
    if (w->ne[0] != K || out->ne[0] != N || out->ne[1] != M) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    // Rows must be dense (blocks contiguous within and across rows), as the kernels assume.
    if (act->nb[1] != (size_t)(K / 32) * 36 || w->nb[1] != (size_t)(K / 32) * block_bytes(w->type) ||
        out->nb[0] != sizeof(float) || (M > 1 && out->nb[1] != (size_t)N * sizeof(float)))
        return QG_ERR_UNSUPPORTED;
    return qg_gemm_w4a8_ex(act->data, w->data, (float*)out->data, (int)M, (int)N, (int)K, w->type, algo, stream);
}

const char* qg_status_string(int s) {
    switch (s) {
        case QG_OK: return "ok";
        case QG_ERR_INVALID_ARG: return "invalid argument";
        case QG_ERR_BAD_K: return "K must be a positive multiple of 32";
        case QG_ERR_UNSUPPORTED: return "unsupported type or algorithm for this shape";
        case QG_ERR_ALIGN: return "pointer misaligned for the block format";
        case QG_ERR_HIP: return "HIP launch error";
    }
    return "unknown status";
}

int qg_last_hip_error(void) { return g_last_hip; }

int qg_select_algo(int M, int N, int K, int wtype) {
    GemmArgs g;
    g.A = (const void*)256; g.B = (const void*)256; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    if (K <= 0 || K % 32 != 0 || !is_weight_type(wtype)) return -1;
    return select_algo(g);
}

int qg_block_bytes(int type) { return block_bytes(type); }

const char* qg_version(void) { return "qg-mi355x 0.1.0 (gfx950)"; }

}  // extern "C"
