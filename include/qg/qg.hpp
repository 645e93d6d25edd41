// qg/qg.hpp — C++ host-side mirror of the reference's launch API over the C-ABI (qg/qg.h).
//
// Source-compatible drop-ins for the reference's inline launch wrappers: same names, argument
// order and meaning, so a call site written against include/gemm_cuda_*.cuh or
// kernels/gemm/gemm_quant_formats.cuh compiles against this header by swapping the include and
// the block type names. Differences: a qg_status is returned (the reference returns void and
// checks nothing, include/gemm_cuda_naive.cuh:285-292) and every "kernel variant" name maps to
// the MI355X dispatcher (the kernel is chosen by shape, not by name).
#ifndef QG_QG_HPP
#define QG_QG_HPP

#include <stdexcept>
#include <string>

#include "blocks.h"
#include "qg.h"

namespace qg {

// include/gemm_cuda_{naive,tiled,dp4a}.cuh: C[M,N] = A_q8_1[M,K] . B_q4_0[N,K]^T (activation-major)
inline int gemm_w4a8(const qg_block_q8_1* A, const qg_block_q4_0* B, float* C, int M, int N, int K,
                     qg_stream_t stream = nullptr) {
    return qg_gemm_w4a8(A, B, C, M, N, K, QG_TYPE_Q4_0, stream);
}
inline int gemm_w4a8_naive(const qg_block_q8_1* A, const qg_block_q4_0* B, float* C, int M, int N, int K,
                           qg_stream_t stream = nullptr) {  // gemm_cuda_naive.cuh:285
    return gemm_w4a8(A, B, C, M, N, K, stream);
}
inline int gemm_w4a8_tiled(const qg_block_q8_1* A, const qg_block_q4_0* B, float* C, int M, int N, int K,
                           qg_stream_t stream = nullptr) {  // gemm_cuda_tiled.cuh:293
    return gemm_w4a8(A, B, C, M, N, K, stream);
}
inline int gemm_w4a8_dp4a(const qg_block_q8_1* A, const qg_block_q4_0* B, float* C, int M, int N, int K,
                          qg_stream_t stream = nullptr) {  // gemm_cuda_dp4a.cuh:409
    return gemm_w4a8(A, B, C, M, N, K, stream);
}
inline int gemm_w4a8_tiled_dp4a(const qg_block_q8_1* A, const qg_block_q4_0* B, float* C, int M, int N, int K,
                                qg_stream_t stream = nullptr) {  // gemm_cuda_dp4a.cuh:421
    return gemm_w4a8(A, B, C, M, N, K, stream);
}
inline int gemm_w4a8_vectorized_dp4a(const qg_block_q8_1* A, const qg_block_q4_0* B, float* C, int M, int N,
                                     int K, qg_stream_t stream = nullptr) {  // gemm_cuda_dp4a.cuh:433
    return gemm_w4a8(A, B, C, M, N, K, stream);
}

// kernels/gemm/gemm_quant_formats.cuh:343-428 — weight-major: out[M,N] = W[M,K] . A[N,K]^T
inline int gemm_q4_0_q8_1(const qg_block_q4_0* W, const qg_block_q8_1* A, float* out, int M, int N, int K,
                          qg_stream_t stream = nullptr) {
    return qg_gemm_q4_0_q8_1(W, A, out, M, N, K, stream);
}
inline int gemm_q4_1_q8_1(const qg_block_q4_1* W, const qg_block_q8_1* A, float* out, int M, int N, int K,
                          qg_stream_t stream = nullptr) {
    return qg_gemm_q4_1_q8_1(W, A, out, M, N, K, stream);
}
inline int gemm_q5_0_q8_1(const qg_block_q5_0* W, const qg_block_q8_1* A, float* out, int M, int N, int K,
                          qg_stream_t stream = nullptr) {
    return qg_gemm_q5_0_q8_1(W, A, out, M, N, K, stream);
}
inline int gemm_q5_1_q8_1(const qg_block_q5_1* W, const qg_block_q8_1* A, float* out, int M, int N, int K,
                          qg_stream_t stream = nullptr) {
    return qg_gemm_q5_1_q8_1(W, A, out, M, N, K, stream);
}

inline int gemm_q8_0_q8_1(const qg_block_q8_0* W, const qg_block_q8_1* A, float* out, int M, int N, int K,
                          qg_stream_t stream = nullptr) {  // gemm_quant_formats.cuh:415
    return qg_gemm_q8_0_q8_1(W, A, out, M, N, K, stream);
}

// W8A8, activation-major (gemm_cuda_naive.cuh:294, gemm_cuda_dp4a.cuh:418)
inline int gemm_w8a8_naive(const qg_block_q8_1* A, const qg_block_q8_0* B, float* C, int M, int N, int K,
                           qg_stream_t stream = nullptr) {
    return qg_gemm_w8a8(A, B, C, M, N, K, stream);
}
inline int gemm_w8a8_dp4a(const qg_block_q8_1* A, const qg_block_q8_0* B, float* C, int M, int N, int K,
                          qg_stream_t stream = nullptr) {
    return qg_gemm_w8a8(A, B, C, M, N, K, stream);
}

// FP32 activations (gemm_cuda_naive.cuh:258-283, gemm_cuda_tiled.cuh:284)
inline int gemm_fp32_naive(const float* A, const float* B, float* C, int M, int N, int K,
                           qg_stream_t stream = nullptr) {
    return qg_gemm_fp32(A, B, C, M, N, K, stream);
}
inline int gemm_w4a16_naive(const float* A, const qg_block_q4_0* B, float* C, int M, int N, int K,
                            qg_stream_t stream = nullptr) {
    return qg_gemm_w4a16(A, B, C, M, N, K, stream);
}
inline int gemm_w4a16_tiled(const float* A, const qg_block_q4_0* B, float* C, int M, int N, int K,
                            qg_stream_t stream = nullptr) {
    return qg_gemm_w4a16(A, B, C, M, N, K, stream);
}
// W4A16 / W8A16 with a caller-owned split-K workspace (no library allocation; capture-safe)
inline size_t gemm_w16_workspace_size(int M, int N, int K) { return qg_gemm_w16_workspace_size(M, N, K); }
inline int gemm_w4a16_ws(const float* A, const qg_block_q4_0* B, float* C, int M, int N, int K, void* ws,
                         size_t ws_bytes, qg_stream_t stream = nullptr) {
    return qg_gemm_w4a16_ws(A, B, C, M, N, K, ws, ws_bytes, stream);
}
inline int gemm_w8a16_naive(const float* A, const qg_block_q8_0* B, float* C, int M, int N, int K,
                            qg_stream_t stream = nullptr) {
    return qg_gemm_w8a16(A, B, C, M, N, K, stream);
}

// kernels/gemm/gemm_fused.cuh:311-338 — FP16 activations quantized inside the product
// (half = IEEE binary16 bits; the reference's `half` type)
inline int gemm_q4_0_fp16_fused(const qg_block_q4_0* weight, const uint16_t* fp16_activation, float* output, int M,
                                int N, int K, qg_stream_t stream = nullptr) {
    return qg_gemm_q4_0_fp16_fused(weight, fp16_activation, output, M, N, K, stream);
}

// include/quantize.h:343-368 — k = number of elements
inline int quantize_q4_0_cuda(const float* x, qg_block_q4_0* y, int64_t k, qg_stream_t stream = nullptr) {
    return qg_quantize_q4_0(x, y, k, stream);
}
inline int quantize_q8_1_cuda(const float* x, qg_block_q8_1* y, int64_t k, qg_stream_t stream = nullptr) {
    return qg_quantize_q8_1(x, y, k, stream);
}
inline int quantize_q8_0_cuda(const float* x, qg_block_q8_0* y, int64_t k, qg_stream_t stream = nullptr) {
    return qg_quantize(QG_TYPE_Q8_0, 0, x, y, k, stream);
}

// Throwing helper for C++ callers that want the TORCH_CHECK-like behaviour of the Python face.
inline void check(int status, const char* what) {
    if (status != QG_OK) throw std::runtime_error(std::string(what) + ": " + qg_status_string(status));
}

}  // namespace qg

#endif  // QG_QG_HPP
