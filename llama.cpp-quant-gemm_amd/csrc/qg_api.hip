// qg_api.hip — the C-ABI (include/qg/qg.h): validation, dispatch, error reporting.
//
// Every entry point validates, picks a kernel family and enqueues on the caller's stream, so
// callers may capture it into a hipGraph. The library's only allocations are the per-(device,
// stream) workspaces of stream_workspace below — slot 0 the W4A16 / W8A16 split-K partials, slot 1
// the odd-K/32 prefill's padded copies — made outside capture, never handed to a captured call
// (captured calls take the non-workspace kernels, or the caller's buffer through the _ws entry
// points), and grown only: growing one synchronizes its stream once (the library's one host sync,
// qg.h), qg_release_workspaces frees them.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <utility>

#include "../../include/qg/qg.h"
#include "qg_kernels.hpp"

using namespace qg;

namespace qg {
namespace {
std::mutex g_ws_mu;  // guards the map; each entry has its own lock for its buffer
struct WsEntry {
    void* p = nullptr;
    size_t n = 0;
    std::mutex mu;
};
// key: (device, stream, slot) — slot 0 the W4A16 split-K workspace (its counters must stay zero
// between calls), slot 1 the padded-repack buffers of the odd-K/32 prefill (qg_repack.hip)
std::map<std::tuple<int, hipStream_t, int>, std::unique_ptr<WsEntry>> g_ws;
}  // namespace

void* stream_workspace(hipStream_t st, size_t bytes, int slot, std::unique_lock<std::mutex>* hold) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    // Never hand the library's buffer to a stream capture: a graph would keep its raw pointer,
    // and a later eager call that grows the buffer (or qg_release_workspaces) would free it under
    // the graph. Captured calls run without it; graphs pass their own workspace
    // through the _ws entry points.
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        (void)hipGetLastError();
        return nullptr;
    }
    WsEntry* e;
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        auto& up = g_ws[std::make_tuple(dev, st, slot)];
        if (!up) up.reset(new WsEntry);
        e = up.get();
    }
    // The entry's lock is held while the buffer grows and, with `hold`, until the caller has
    // enqueued every kernel that uses it (two host threads on one stream must not
    // interleave a multi-kernel sequence on one buffer).
    std::unique_lock<std::mutex> lk(e->mu);
    if (!e->p || e->n < bytes) {
        const size_t sz = std::max(bytes, (size_t)4 << 20);
        void* p = nullptr;
        if (hipMalloc(&p, sz) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        if (hipMemsetAsync(p, 0, sz, st) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(p);
            return nullptr;
        }
        if (e->p) {
            // launches still queued on st may use the old block: the one host sync of the library,
            // once per growth (documented in qg.h; the _ws entry points never reach it)
            (void)hipStreamSynchronize(st);
            (void)hipFree(e->p);
        }
        e->p = p;
        e->n = sz;
    }
    void* p = e->p;
    if (hold) *hold = std::move(lk);
    return p;
}

int device_cus() {
    static std::atomic<int> cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return 256;
    }
    int v = cached[dev].load(std::memory_order_relaxed);
    if (v > 0) return v;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
        (void)hipGetLastError();
        cus = 256;
    }
    cached[dev].store(cus, std::memory_order_relaxed);
    return cus;
}

void describe_kernel(const GemmArgs& g, const char* fmt, ...) {
    if (!g.describe || g.describe_len == 0) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g.describe, g.describe_len, fmt, ap);
    va_end(ap);
}

void release_workspaces() {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    bool synced = false;
    for (auto& kv : g_ws) {
        std::lock_guard<std::mutex> le(kv.second->mu);
        if (kv.second->p) {
            if (!synced) (void)hipDeviceSynchronize();
            synced = true;
            (void)hipFree(kv.second->p);
        }
    }
    g_ws.clear();
}
}  // namespace qg

namespace {
thread_local int g_last_hip = 0;

int hip_status(hipError_t e) {
    if (e == hipSuccess) return QG_OK;
    g_last_hip = (int)e;
    return QG_ERR_HIP;
}

bool is_weight_type(int t) {
    return t == QG_TYPE_Q4_0 || t == QG_TYPE_Q4_1 || t == QG_TYPE_Q5_0 || t == QG_TYPE_Q5_1 || t == QG_TYPE_Q8_0;
}

// Crossover from profiles/tools_archive/mmq_probe.hip (profiles/r01_tuning/mmq_probe_smallm.txt): the dot4 GEMV
// wins up to M = 4 (its LDS activation reads grow with M), the MFMA kernel from M = 5 on.
int select_algo(const GemmArgs& g) {
    if (g.M <= 4 && gemv_eligible(g)) return QG_ALGO_GEMV;
    if (mfma_eligible(g)) return QG_ALGO_MFMA;
    if (gemv_eligible(g)) return QG_ALGO_GEMV;
    // odd K / 32 (rows off dword alignment) or 2-B aligned weights at prefill sizes: the MFMA kernel
    // on a zero-padded copy (qg_repack.hip); below that one wave per weight row (qg_ragged.hip)
    // instead of the byte-load generic kernel's one wave per output
    if (repack_eligible(g)) return QG_ALGO_MFMA;
    if (ragged_eligible(g)) return QG_ALGO_RAGGED;
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
    const bool auto_algo = algo == QG_ALGO_AUTO;
    if (auto_algo) algo = select_algo(g);
    if (algo == QG_ALGO_GEMV) {
        if (!gemv_eligible(g) || (g.batch > 1 && (g.sB % 16 != 0))) {
            if (g.batch == 1) return QG_ERR_UNSUPPORTED;
            algo = QG_ALGO_GENERIC;  // batch strides break the vector-load alignment: per-item path
        } else {
            if (g.batch > 65535) return QG_ERR_INVALID_ARG;
            return hip_status(launch_gemv(g, st));
        }
    }
    // MFMA on a shape the kernel cannot address directly (odd K / 32, 2-B aligned weights): through
    // the zero-padded repack; without a workspace (stream capture) the automatic choice falls back
    if (algo == QG_ALGO_MFMA && !mfma_eligible(g) && repack_eligible(g)) {
        const hipError_t e = launch_repack_mfma(g, st);
        if (e != hipErrorNotReady) return hip_status(e);
        if (!auto_algo) return QG_ERR_UNSUPPORTED;
        algo = ragged_eligible(g) ? QG_ALGO_RAGGED : QG_ALGO_GENERIC;
    }
    // MFMA and generic kernels take one product per launch: enqueue the batch item by item.
    auto item = [&](int i) {
        GemmArgs gi = g;
        gi.batch = 1;
        gi.A = (const uint8_t*)g.A + (long)i * g.sA;
        gi.B = (const uint8_t*)g.B + (long)i * g.sB;
        if (g.C) gi.C = g.C + (long)i * g.sC;
        return gi;
    };
    // Every item is checked before the first is enqueued (a batch stride can break the MFMA
    // kernel's 16-B alignment for later items only): an explicit MFMA request fails with nothing
    // launched, an automatic choice falls back to the generic kernel for the whole batch.
    if (algo == QG_ALGO_MFMA || algo == QG_ALGO_RAGGED) {
        auto ok = [&](const GemmArgs& gi) { return algo == QG_ALGO_MFMA ? mfma_eligible(gi) : ragged_eligible(gi); };
        bool all_ok = true;
        for (int i = 0; i < g.batch && all_ok; ++i) all_ok = ok(item(i));
        if (!all_ok) {
            if (!auto_algo) return QG_ERR_UNSUPPORTED;
            algo = QG_ALGO_GENERIC;
        }
    }
    for (int i = 0; i < g.batch; ++i) {
        const GemmArgs gi = item(i);
        int rc;
        switch (algo) {
            case QG_ALGO_MFMA:
                rc = hip_status(launch_mfma(gi, st));
                break;
            case QG_ALGO_RAGGED:
                rc = hip_status(launch_ragged(gi, st));
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

// The tiled weight layout (qg_tile_weights): the MFMA small-batch decode for M = 3..4 and M = 2 at K/32 > 256
// (qg_gemvm.hip), the tiled decode GEMV for the rest of M <= 4 (qg_gemvt.hip, round 6), the
// MFMA kernels beyond (LAY_TILED; odd K/32 through its activation windows). Shapes neither
// takes (ldc past INT32_MAX, activation windows of 2 GiB or more, K/32 whose records exceed the LDS at
// M <= 4 where the MFMA kernel rejects the shape too) return QG_ERR_UNSUPPORTED: the tiled layout has no
// generic kernel.
int run_tiled(GemmArgs& g, hipStream_t st) {
    if (g.M < 0 || g.N < 0) return QG_ERR_INVALID_ARG;
    if (g.K <= 0 || g.K % 32 != 0) return QG_ERR_BAD_K;
    if (!is_weight_type(g.wtype)) return QG_ERR_UNSUPPORTED;
    if (g.M == 0 || g.N == 0) return QG_OK;
    if (!g.A || !g.B || (!g.C && !g.sumi)) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)g.B & 15) != 0 || ((uintptr_t)g.A & 15) != 0) return QG_ERR_ALIGN;
#ifndef QG_TILED_GEMVM  // (A/B builds: 0 = the round-6 tiled decode GEMV for every M <= 4)
#define QG_TILED_GEMVM 1
#endif
    if (QG_TILED_GEMVM && gemvm_eligible(g)) return hip_status(launch_gemvm(g, st));  // M = 3..4 (2 at long K)
    if (gemvt_eligible(g)) return hip_status(launch_gemvt(g, st));  // M <= 4: the tiled decode GEMV
    if (!mfma_eligible(g)) return QG_ERR_UNSUPPORTED;
    return hip_status(launch_mfma(g, st));
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
int run_w16(int wtype, const float* A, const void* B, float* C, int M, int N, int K, hipStream_t st,
            void* ws = nullptr, size_t ws_bytes = 0) {
    if (M < 0 || N < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (M == 0 || N == 0) return QG_OK;
    if (!A || !B || !C) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)A & 3) != 0 || ((uintptr_t)B & 1) != 0) return QG_ERR_ALIGN;
    GemmArgs g;
    g.A = A; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    g.ws = ws; g.ws_bytes = ws_bytes;
    return hip_status(launch_w16(g, st));
}

// Dims as extract_dims_from_tensor (include/llama_adapter.h:49-61): K = act->ne[0], M = act->ne[1],
// N = w->ne[1]; output [N, M] in ggml ne-order, i.e. row-major C[M][N]. Rows must be dense (the
// kernels' layout); batched views (ne[2..3] > 1) are out of scope. k_mult: K granularity.
size_t row_bytes(int type, int64_t K) {
    if (type == QG_TYPE_F32) return (size_t)K * 4;
    if (type == QG_TYPE_F16) return (size_t)K * 2;
    return (size_t)(K / 32) * (size_t)block_bytes(type);
}

int view_dims(const qg_tensor_view* act, const qg_tensor_view* w, const qg_tensor_view* out, int64_t& M, int64_t& N,
              int64_t& K, int k_mult = 32) {
    for (int d = 2; d < 4; ++d)
        if ((act->ne[d] != 1 && act->ne[d] != 0) || (w->ne[d] != 1 && w->ne[d] != 0) || (out->ne[d] != 1 && out->ne[d] != 0))
            return QG_ERR_UNSUPPORTED;
    K = act->ne[0];
    M = act->ne[1];
    N = w->ne[1];
    if (w->ne[0] != K || out->ne[0] != N || out->ne[1] != M) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % k_mult != 0) return QG_ERR_BAD_K;
    if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return QG_ERR_UNSUPPORTED;
    if ((M > 1 && act->nb[1] != row_bytes(act->type, K)) || (N > 1 && w->nb[1] != row_bytes(w->type, K)) ||
        out->nb[0] != sizeof(float) || (M > 1 && out->nb[1] != (size_t)N * sizeof(float)))
        return QG_ERR_UNSUPPORTED;
    return QG_OK;
}

size_t fused_workspace_bytes(int M, int K) { return M > 0 && K > 0 ? (size_t)M * (size_t)(K / 32) * 36 : 0; }

// FP32 / FP16 activations (g.ain != AIN_Q8_1), dense rows of K elements. Small M: quantization
// fused into the GEMV prologue, one launch. Larger M: quantize into the caller's workspace, then
// the Q8_1 product (same bytes, so the same results); without a workspace, fused GEMV launches
// over row chunks (the weights are streamed once per chunk).
int run_fused(GemmArgs g, void* ws, size_t ws_bytes, hipStream_t st) {
    if (g.M < 0 || g.N < 0) return QG_ERR_INVALID_ARG;
    if (g.K <= 0 || g.K % 32 != 0) return QG_ERR_BAD_K;
    if (!is_weight_type(g.wtype)) return QG_ERR_UNSUPPORTED;
    if (g.M == 0 || g.N == 0) return QG_OK;
    if (!g.A || !g.B || !g.C) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)g.B & 1) != 0) return QG_ERR_ALIGN;
    const size_t es = g.ain == AIN_F32 ? 4 : 2;
    if (((uintptr_t)g.A & (es - 1)) != 0) return QG_ERR_ALIGN;
    const bool vec_ok = ((uintptr_t)g.A & 15) == 0;
    if (g.M <= 4 && vec_ok && gemv_eligible(g)) return hip_status(launch_gemv(g, st));
    if (ws && ws_bytes >= fused_workspace_bytes(g.M, g.K)) {
        if (((uintptr_t)ws & 3) != 0) return QG_ERR_ALIGN;
        const int64_t nblocks = (int64_t)g.M * (g.K / 32);
        const hipError_t e = g.ain == AIN_F32 ? launch_quantize(QG_TYPE_Q8_1, 0, (const float*)g.A, ws, nblocks, st)
                                              : launch_quantize_f16_fused(g.A, ws, nblocks, st);
        if (e != hipSuccess) return hip_status(e);
        GemmArgs q = g;
        q.ain = AIN_Q8_1;
        q.A = ws;
        return run_gemm(q, QG_ALGO_AUTO, st);
    }
    if (!vec_ok) return QG_ERR_ALIGN;
    for (int rows : {8, 4, 2, 1}) {
        GemmArgs c = g;
        c.M = rows < g.M ? rows : g.M;
        if (!gemv_eligible(c)) continue;
        const long row_bytes = (long)g.K * (long)es;
        const int full = g.M / c.M, rem = g.M - full * c.M;
        if (full > 65535) return QG_ERR_UNSUPPORTED;
        c.batch = full;
        c.sA = (long)c.M * row_bytes;
        c.sB = 0;
        c.sC = (long)c.M * g.ldc_m;
        hipError_t e = launch_gemv(c, st);
        if (e != hipSuccess || rem == 0) return hip_status(e);
        c.batch = 1;
        c.A = (const uint8_t*)g.A + (long)full * c.sA;
        c.C = g.C + (long)full * c.sC;
        c.M = rem;
        return hip_status(launch_gemv(c, st));
    }
    return QG_ERR_UNSUPPORTED;
}
}  // namespace

extern "C" {

void qg_release_workspaces(void) { release_workspaces(); }

size_t qg_gemm_w4a8_f32_workspace_size(int M, int K) { return fused_workspace_bytes(M, K); }

int qg_gemm_w4a16(const float* A, const void* B_q4_0, float* C, int M, int N, int K, qg_stream_t stream) {
    return run_w16(QG_TYPE_Q4_0, A, B_q4_0, C, M, N, K, (hipStream_t)stream);
}

int qg_gemm_w8a16(const float* A, const void* B_q8_0, float* C, int M, int N, int K, qg_stream_t stream) {
    return run_w16(QG_TYPE_Q8_0, A, B_q8_0, C, M, N, K, (hipStream_t)stream);
}

size_t qg_gemm_w16_workspace_size(int M, int N, int K) { return M > 0 && N > 0 ? w16_workspace_bytes(M, N, K) : 0; }

int qg_gemm_w4a16_ws(const float* A, const void* B_q4_0, float* C, int M, int N, int K, void* workspace,
                     size_t workspace_bytes, qg_stream_t stream) {
    return run_w16(QG_TYPE_Q4_0, A, B_q4_0, C, M, N, K, (hipStream_t)stream, workspace, workspace_bytes);
}

int qg_gemm_w8a16_ws(const float* A, const void* B_q8_0, float* C, int M, int N, int K, void* workspace,
                     size_t workspace_bytes, qg_stream_t stream) {
    return run_w16(QG_TYPE_Q8_0, A, B_q8_0, C, M, N, K, (hipStream_t)stream, workspace, workspace_bytes);
}

int qg_gemm_q4_0_fp32(const void* weight_q4_0, const float* activation, float* out, int M, int N, int K,
                      qg_stream_t stream) {
    return run_w16(QG_TYPE_Q4_0, activation, weight_q4_0, out, M, N, K, (hipStream_t)stream);
}

int qg_gemm_w4a8_f32(const float* X, const void* B, float* C, int M, int N, int K, int wtype, void* workspace,
                     size_t workspace_bytes, qg_stream_t stream) {
    GemmArgs g;
    g.A = X; g.ain = AIN_F32; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    return run_fused(g, workspace, workspace_bytes, (hipStream_t)stream);
}

int qg_gemm_q4_0_fp16_fused_ws(const void* W, const void* act_f16, float* out, int M, int N, int K, void* workspace,
                               size_t workspace_bytes, qg_stream_t stream) {
    // Weight-major (M weight rows, N tokens) -> activation-major args, as weight_major().
    GemmArgs g;
    g.A = act_f16; g.ain = AIN_F16_FUSED; g.B = W; g.C = out; g.M = N; g.N = M; g.K = K; g.wtype = QG_TYPE_Q4_0;
    g.ldc_m = 1; g.ldc_n = N;
    return run_fused(g, workspace, workspace_bytes, (hipStream_t)stream);
}

int qg_gemm_q4_0_fp16_fused(const void* W, const void* act_f16, float* out, int M, int N, int K, qg_stream_t stream) {
    return qg_gemm_q4_0_fp16_fused_ws(W, act_f16, out, M, N, K, nullptr, 0, stream);
}

int qg_quantize_q8_1_f16_fused(const void* x, void* y, int64_t k, qg_stream_t stream) {
    if (k < 0 || k % 32 != 0) return QG_ERR_BAD_K;
    if (k == 0) return QG_OK;
    if (!x || !y) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)x & 1) != 0 || ((uintptr_t)y & 3) != 0) return QG_ERR_ALIGN;
    return hip_status(launch_quantize_f16_fused(x, y, k / 32, (hipStream_t)stream));
}

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

size_t qg_gemm_w4a8_workspace_size(int M, int N, int K, int wtype) {
    if (M <= 0 || N <= 0 || K <= 0 || K % 32 != 0 || !is_weight_type(wtype)) return 0;
    GemmArgs g;
    g.A = (const void*)256; g.B = (const void*)256; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    return repack_eligible(g) ? repack_workspace_bytes(g) : 0;
}

int qg_gemm_w4a8_ws(const void* A, const void* B, float* C, int M, int N, int K, int wtype, void* workspace,
                    size_t workspace_bytes, qg_stream_t stream) {
    GemmArgs g;
    g.A = A; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    g.ws = workspace; g.ws_bytes = workspace_bytes;
    return run_gemm(g, QG_ALGO_AUTO, (hipStream_t)stream);
}

size_t qg_repack_weights_bytes(int N, int K, int wtype) {
    if (N < 0 || K <= 0 || K % 32 != 0 || !is_weight_type(wtype)) return 0;
    return (size_t)N * (size_t)padded_blocks(K) * (size_t)block_bytes(wtype);
}

int qg_repack_weights(const void* B, void* B_packed, int N, int K, int wtype, qg_stream_t stream) {
    if (N < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (!is_weight_type(wtype)) return QG_ERR_UNSUPPORTED;
    if (N == 0) return QG_OK;
    if (!B || !B_packed) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)B & 1) != 0 || ((uintptr_t)B_packed & 15) != 0) return QG_ERR_ALIGN;
    const int bb = block_bytes(wtype);
    return hip_status(launch_pad_rows(B, B_packed, N, (K / 32) * bb, padded_blocks(K) * bb, (hipStream_t)stream));
}

int qg_quantize_q8_1_padded(const float* x, void* y, int M, int K, qg_stream_t stream) {
    if (M < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (M == 0) return QG_OK;
    if (!x || !y) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)x & 3) != 0 || ((uintptr_t)y & 3) != 0) return QG_ERR_ALIGN;
    return hip_status(launch_quantize_q8_1_padded(x, y, M, K / 32, padded_blocks(K), (hipStream_t)stream));
}

int qg_gemm_w4a8_padded(const void* A_padded, const void* B_packed, float* C, int M, int N, int K, int wtype,
                        qg_stream_t stream) {
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    GemmArgs g;
    g.A = A_padded; g.B = B_packed; g.C = C; g.M = M; g.N = N; g.K = padded_blocks(K) * 32; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    return run_gemm(g, QG_ALGO_AUTO, (hipStream_t)stream);
}

size_t qg_gemm_w4a8_prepacked_workspace_size(int M, int K) {
    if (M <= 0 || K <= 0 || K % 32 != 0 || padded_blocks(K) == K / 32) return 0;
    return (size_t)M * (size_t)padded_blocks(K) * 36;
}

int qg_gemm_w4a8_prepacked(const void* A, const void* B_packed, float* C, int M, int N, int K, int wtype,
                           void* workspace, size_t workspace_bytes, qg_stream_t stream) {
    if (M < 0 || N < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (!is_weight_type(wtype)) return QG_ERR_UNSUPPORTED;
    if (M == 0 || N == 0) return QG_OK;
    if (!A || !B_packed || !C) return QG_ERR_INVALID_ARG;
    const hipStream_t st = (hipStream_t)stream;
    const int nbp = padded_blocks(K);
    GemmArgs g;
    g.A = A; g.B = B_packed; g.C = C; g.M = M; g.N = N; g.K = nbp * 32; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    if (nbp != K / 32) {
        // round 5: where the MFMA kernel runs (M >= 5), it reads the plain activation rows itself
        // (activation windows against the padded weight rows, qg_mmq_kernel.hpp AW): one launch, no
        // workspace touched
        GemmArgs w = g;
        w.K = K;
        w.nbw = nbp;
        if (M > 4 && mfma_eligible(w)) return hip_status(launch_mfma(w, st));
        // otherwise the activations are padded into the caller's workspace, same zero blocks
        if (!workspace || workspace_bytes < qg_gemm_w4a8_prepacked_workspace_size(M, K)) return QG_ERR_INVALID_ARG;
        if (((uintptr_t)A & 1) != 0 || ((uintptr_t)workspace & 15) != 0) return QG_ERR_ALIGN;
        const hipError_t e = launch_pad_rows(A, workspace, M, (K / 32) * 36, nbp * 36, st);
        if (e != hipSuccess) return hip_status(e);
        g.A = workspace;
    }
    return run_gemm(g, QG_ALGO_AUTO, st);
}

size_t qg_tile_weights_bytes(int N, int K, int wtype) {
    if (N < 0 || K <= 0 || K % 32 != 0 || !is_weight_type(wtype)) return 0;
    return tiled_weight_bytes(N, K, wtype);
}

int qg_tile_weights(const void* B, void* B_tiled, int N, int K, int wtype, qg_stream_t stream) {
    if (N < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (!is_weight_type(wtype)) return QG_ERR_UNSUPPORTED;
    if (N == 0) return QG_OK;
    if (!B || !B_tiled) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)B & 1) != 0 || ((uintptr_t)B_tiled & 15) != 0) return QG_ERR_ALIGN;
    return hip_status(launch_tile_weights(B, B_tiled, N, K, wtype, (hipStream_t)stream));
}

int qg_gemm_w4a8_tiled_ldc(const void* A, const void* B_tiled, float* C, int M, int N, int K, int64_t ldc, int wtype,
                           qg_stream_t stream) {
    if (ldc < N || (M > 1 && ldc <= 0)) return QG_ERR_INVALID_ARG;
    GemmArgs g;
    g.A = A; g.B = B_tiled; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = (long)ldc; g.ldc_n = 1;
    g.lay = LAY_TILED;
    return run_tiled(g, (hipStream_t)stream);
}

int qg_gemm_w4a8_tiled(const void* A, const void* B_tiled, float* C, int M, int N, int K, int wtype, qg_stream_t stream) {
    return qg_gemm_w4a8_tiled_ldc(A, B_tiled, C, M, N, K, N, wtype, stream);
}

int qg_debug_sumi_tiled(const void* A, const void* B_tiled, int32_t* sumi, int M, int N, int K, int wtype,
                        qg_stream_t stream) {
    GemmArgs g;
    g.A = A; g.B = B_tiled; g.sumi = sumi; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    g.lay = LAY_TILED;
    return run_tiled(g, (hipStream_t)stream);
}

int qg_debug_config_tiled(int M, int N, int K, int wtype, int sumi, char* buf, size_t len) {
    if (!buf || len == 0) return QG_ERR_INVALID_ARG;
    buf[0] = 0;
    GemmArgs g;
    g.A = (const void*)256; g.B = (const void*)256; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    if (sumi) g.sumi = (int32_t*)256;
    else g.C = (float*)256;
    g.ldc_m = N; g.ldc_n = 1;
    g.lay = LAY_TILED;
    g.describe = buf; g.describe_len = len;
    return run_tiled(g, nullptr);
}

// ---- round 5: tiled activations (LAY_TILED_ACT) -------------------------------------------------------
size_t qg_activations_tiled_bytes(int M, int K) {
    if (M < 0 || K <= 0 || K % 32 != 0) return 0;
    return tiled_act_bytes(M, K);
}

int qg_quantize_q8_1_tiled(const float* x, void* A_tiled, int M, int K, qg_stream_t stream) {
    if (M < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (M == 0) return QG_OK;
    if (!x || !A_tiled) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)x & 15) != 0 || ((uintptr_t)A_tiled & 15) != 0) return QG_ERR_ALIGN;
    return hip_status(launch_quantize_q8_1_tiled(x, A_tiled, M, K, (hipStream_t)stream));
}

int qg_tile_activations(const void* A_q8_1, void* A_tiled, int M, int K, qg_stream_t stream) {
    if (M < 0) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (M == 0) return QG_OK;
    if (!A_q8_1 || !A_tiled) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)A_q8_1 & 3) != 0 || ((uintptr_t)A_tiled & 15) != 0) return QG_ERR_ALIGN;
    return hip_status(launch_tile_activations(A_q8_1, A_tiled, M, K, (hipStream_t)stream));
}

int qg_gemm_w4a8_tiled_act_ldc(const void* A_tiled, const void* B_tiled, float* C, int M, int N, int K, int64_t ldc, int wtype,
                               qg_stream_t stream) {
    if (ldc < N || (M > 1 && ldc <= 0)) return QG_ERR_INVALID_ARG;
    GemmArgs g;
    g.A = A_tiled; g.B = B_tiled; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = (long)ldc; g.ldc_n = 1;
    g.lay = LAY_TILED_ACT;
    return run_tiled(g, (hipStream_t)stream);
}

int qg_gemm_w4a8_tiled_act(const void* A_tiled, const void* B_tiled, float* C, int M, int N, int K, int wtype,
                           qg_stream_t stream) {
    return qg_gemm_w4a8_tiled_act_ldc(A_tiled, B_tiled, C, M, N, K, N, wtype, stream);
}

int qg_debug_sumi_tiled_act(const void* A_tiled, const void* B_tiled, int32_t* sumi, int M, int N, int K, int wtype,
                            qg_stream_t stream) {
    GemmArgs g;
    g.A = A_tiled; g.B = B_tiled; g.sumi = sumi; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = N; g.ldc_n = 1;
    g.lay = LAY_TILED_ACT;
    return run_tiled(g, (hipStream_t)stream);
}

int qg_debug_config_tiled_act(int M, int N, int K, int wtype, int sumi, char* buf, size_t len) {
    if (!buf || len == 0) return QG_ERR_INVALID_ARG;
    buf[0] = 0;
    GemmArgs g;
    g.A = (const void*)256; g.B = (const void*)256; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    if (sumi) g.sumi = (int32_t*)256;
    else g.C = (float*)256;
    g.ldc_m = N; g.ldc_n = 1;
    g.lay = LAY_TILED_ACT;
    g.describe = buf; g.describe_len = len;
    return run_tiled(g, nullptr);
}

int qg_gemm_w4a8_grouped(const qg_gemv_item* items, int count, int M, int K, int wtype, qg_stream_t stream) {
    if (count < 0 || M < 0 || (count > 0 && !items)) return QG_ERR_INVALID_ARG;
    if (K <= 0 || K % 32 != 0) return QG_ERR_BAD_K;
    if (!is_weight_type(wtype)) return QG_ERR_UNSUPPORTED;
    const hipStream_t st = (hipStream_t)stream;
    auto item_args = [&](const qg_gemv_item& it) {
        GemmArgs g;
        g.A = it.A_q8_1; g.B = it.B; g.C = it.C; g.M = M; g.N = it.N; g.K = K; g.wtype = wtype;
        g.ldc_m = it.ldc ? it.ldc : it.N; g.ldc_n = 1;
        return g;
    };
    // validate every item before anything is enqueued; one launch only if AUTO picks the GEMV for all
    bool one_launch = M > 0 && M <= 4;  // the grouped GEMV is instantiated for MT <= 4 (qg_gemv_kernel.hpp)
    for (int i = 0; i < count; ++i) {
        const qg_gemv_item& it = items[i];
        if (it.N < 0 || it.ldc < 0 || (it.ldc != 0 && it.ldc < it.N)) return QG_ERR_INVALID_ARG;
        if (it.N == 0 || M == 0) continue;
        if (!it.A_q8_1 || !it.B || !it.C) return QG_ERR_INVALID_ARG;
        if (((uintptr_t)it.B & 1) != 0) return QG_ERR_ALIGN;
        const GemmArgs g = item_args(it);
        one_launch = one_launch && select_algo(g) == QG_ALGO_GEMV && gemv_eligible(g);
    }
    if (M == 0) return QG_OK;
    if (!one_launch) {
        for (int i = 0; i < count; ++i) {
            if (items[i].N == 0) continue;
            GemmArgs g = item_args(items[i]);
            const int rc = run_gemm(g, QG_ALGO_AUTO, st);
            if (rc != QG_OK) return rc;
        }
        return QG_OK;
    }
    for (int i0 = 0; i0 < count;) {
        GemvGroup grp = {};
        grp.M = M; grp.K = K;
        int maxn = 0;
        for (; i0 < count && grp.count < GEMV_GROUP_MAX; ++i0) {
            const qg_gemv_item& it = items[i0];
            if (it.N == 0) continue;
            grp.it[grp.count++] = GemvItemDesc{it.A_q8_1, it.B, it.C, it.N, it.ldc ? it.ldc : it.N};
            maxn = std::max(maxn, it.N);
        }
        if (grp.count == 0) break;
        GemmArgs g;
        g.A = grp.it[0].A; g.B = grp.it[0].B; g.C = grp.it[0].C; g.M = M; g.N = maxn; g.K = K; g.wtype = wtype;
        g.ldc_m = grp.it[0].ldc; g.ldc_n = 1;
        g.group = &grp;
        const int rc = hip_status(launch_gemv(g, st));
        if (rc != QG_OK) return rc;
    }
    return QG_OK;
}

int qg_gemm_w4a8(const void* A, const void* B, float* C, int M, int N, int K, int wtype, qg_stream_t stream) {
    return qg_gemm_w4a8_ex(A, B, C, M, N, K, wtype, QG_ALGO_AUTO, stream);
}

int qg_gemm_q4_0_q8_1_w4a8(const void* A_q8_1, const void* B_q4_0, float* C, int M, int N, int K,
                           qg_stream_t stream) {
    return qg_gemm_w4a8_ex(A_q8_1, B_q4_0, C, M, N, K, QG_TYPE_Q4_0, QG_ALGO_AUTO, stream);
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
int qg_gemm_q8_0_q8_1(const void* W, const void* A, float* out, int M, int N, int K, qg_stream_t s) {
    return weight_major(QG_TYPE_Q8_0, W, A, out, M, N, K, s);
}

int qg_gemm_w8a8(const void* A, const void* B, float* C, int M, int N, int K, qg_stream_t stream) {
    return qg_gemm_w4a8_ex(A, B, C, M, N, K, QG_TYPE_Q8_0, QG_ALGO_AUTO, stream);
}

int qg_quantize(int type, int variant, const float* x, void* y, int64_t k, qg_stream_t stream) {
    if (k < 0 || k % 32 != 0) return QG_ERR_BAD_K;
    if (block_bytes(type) == 0) return QG_ERR_UNSUPPORTED;
    if (variant != 0 && !(variant == 1 && type == QG_TYPE_Q8_1) &&
        !(variant == 2 && (type == QG_TYPE_Q8_1 || type == QG_TYPE_Q4_0)))
        return QG_ERR_UNSUPPORTED;
    if (k == 0) return QG_OK;
    if (!x || !y) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)x & 3) != 0) return QG_ERR_ALIGN;
    const uintptr_t need = type == QG_TYPE_Q8_1 ? 3 : 1;
    if (((uintptr_t)y & need) != 0) return QG_ERR_ALIGN;
    return hip_status(launch_quantize(type, variant, x, y, k / 32, (hipStream_t)stream));
}

int qg_quantize_q8_1(const float* x, void* y, int64_t k, qg_stream_t s) { return qg_quantize(QG_TYPE_Q8_1, 0, x, y, k, s); }
int qg_quantize_q4_0(const float* x, void* y, int64_t k, qg_stream_t s) { return qg_quantize(QG_TYPE_Q4_0, 0, x, y, k, s); }
int qg_quantize_q8_1_definition(const float* x, void* y, int64_t num_elements, qg_stream_t s) {
    return qg_quantize(QG_TYPE_Q8_1, QG_QVAR_DEFINITION, x, y, num_elements, s);
}
int qg_quantize_q4_0_definition(const float* x, void* y, int64_t num_elements, qg_stream_t s) {
    return qg_quantize(QG_TYPE_Q4_0, QG_QVAR_DEFINITION, x, y, num_elements, s);
}

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

int qg_debug_config(int M, int N, int K, int wtype, int algo, int sumi, char* buf, size_t len) {
    if (!buf || len == 0) return QG_ERR_INVALID_ARG;
    buf[0] = 0;
    // 256-B aligned stand-in pointers: the shape decides, as for a real call on aligned buffers
    GemmArgs g;
    g.A = (const void*)256; g.B = (const void*)256; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    if (sumi) g.sumi = (int32_t*)256;
    else g.C = (float*)256;
    g.ldc_m = N; g.ldc_n = 1;
    g.describe = buf; g.describe_len = len;
    return run_gemm(g, algo, nullptr);
}

int qg_gemm_w4a8_ldc(const void* A, const void* B, float* C, int M, int N, int K, int64_t ldc, int wtype, int algo,
                     qg_stream_t stream) {
    if (ldc < N || (M > 1 && ldc <= 0)) return QG_ERR_INVALID_ARG;
    GemmArgs g;
    g.A = A; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = wtype;
    g.ldc_m = (long)ldc; g.ldc_n = 1;
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
        else if (strcmp(kernel_type, "ragged") == 0) algo = QG_ALGO_RAGGED;
        else return QG_ERR_INVALID_ARG;
    }
    if (act->type != QG_TYPE_Q8_1 || out->type != QG_TYPE_F32 || !is_weight_type(w->type)) return QG_ERR_UNSUPPORTED;
    int64_t M, N, K;
    const int rc = view_dims(act, w, out, M, N, K);
    if (rc != QG_OK) return rc;
    return qg_gemm_w4a8_ex(act->data, w->data, (float*)out->data, (int)M, (int)N, (int)K, w->type, algo, stream);
}

int qg_gemm_w4a16_from_view(const qg_tensor_view* act, const qg_tensor_view* w, qg_tensor_view* out,
                            const char* kernel_type, qg_stream_t stream) {
    if (!act || !w || !out) return QG_ERR_INVALID_ARG;
    if (kernel_type && strcmp(kernel_type, "naive") != 0 && strcmp(kernel_type, "tiled") != 0 &&
        strcmp(kernel_type, "auto") != 0)
        return QG_ERR_INVALID_ARG;
    if (act->type != QG_TYPE_F32 || out->type != QG_TYPE_F32 || (w->type != QG_TYPE_Q4_0 && w->type != QG_TYPE_Q8_0))
        return QG_ERR_UNSUPPORTED;
    int64_t M, N, K;
    const int rc = view_dims(act, w, out, M, N, K);
    if (rc != QG_OK) return rc;
    return run_w16(w->type, (const float*)act->data, w->data, (float*)out->data, (int)M, (int)N, (int)K,
                   (hipStream_t)stream);
}

int qg_gemm_fp32_from_view(const qg_tensor_view* act, const qg_tensor_view* w, qg_tensor_view* out,
                           const char* kernel_type, qg_stream_t stream) {
    if (!act || !w || !out) return QG_ERR_INVALID_ARG;
    if (kernel_type && strcmp(kernel_type, "naive") != 0 && strcmp(kernel_type, "tiled") != 0 &&
        strcmp(kernel_type, "auto") != 0)
        return QG_ERR_INVALID_ARG;
    if (act->type != QG_TYPE_F32 || out->type != QG_TYPE_F32 || w->type != QG_TYPE_F32) return QG_ERR_UNSUPPORTED;
    int64_t M, N, K;
    const int rc = view_dims(act, w, out, M, N, K, 1);
    if (rc != QG_OK) return rc;
    return qg_gemm_fp32((const float*)act->data, (const float*)w->data, (float*)out->data, (int)M, (int)N, (int)K,
                        stream);
}

int qg_validate_view_types(const qg_tensor_view* act, const qg_tensor_view* w, const qg_tensor_view* out,
                           int expected_activation_type, int expected_weight_type, int expected_output_type) {
    return act && w && out && act->type == expected_activation_type && w->type == expected_weight_type &&
           out->type == expected_output_type;
}

int qg_gemm_fp32(const float* A, const float* B, float* C, int M, int N, int K, qg_stream_t stream) {
    if (M < 0 || N < 0 || K < 0) return QG_ERR_INVALID_ARG;
    if (M == 0 || N == 0) return QG_OK;
    if (!A || !B || !C) return QG_ERR_INVALID_ARG;
    if (((uintptr_t)A & 3) != 0 || ((uintptr_t)B & 3) != 0 || ((uintptr_t)C & 3) != 0) return QG_ERR_ALIGN;
    GemmArgs g;
    g.A = A; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K;
    g.ldc_m = N; g.ldc_n = 1;
    return hip_status(launch_fp32(g, (hipStream_t)stream));
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
