/*
 * qg/qg_host.h — host-only C-ABI twins of the reference's CPU entry points (`libqg_host.so`).
 *
 * SURVEY.md §8(b) "CPU API": the reference's ground-truth functions are inline host functions in
 * include/gemm_reference.h and include/quantize.h. A caller that links them today can link these
 * instead: same argument order, pointer types (as void*), layouts and results — bit-identical
 * outputs on x86-64 (IEEE fp32, no FMA contraction, the reference's operation order). This
 * library is independent of the GPU library (no HIP) and of the test oracle (oracle/), which
 * checks it.
 *
 * Differences, deliberate: the GEMMs return a status (0, or QG_ERR_BAD_K / QG_ERR_INVALID_ARG from
 * qg/qg.h) instead of void, since the reference never validates K % 32 (gemm_reference.h:181);
 * `_mt` forms partition output rows over threads (each output keeps the serial summation order,
 * so results are identical for any thread count).
 */
#ifndef QG_QG_HOST_H
#define QG_QG_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* gemm_w4a8_reference(const block_q8_1* A, const block_q4_0* B, float* C, int M, int N, int K)
 * (include/gemm_reference.h:175-222): C[M][N] overwritten. */
int qg_gemm_w4a8_q4_0_cpu(const void* A_q8_1, const void* B_q4_0, float* C, int M, int N, int K);

/* vec_dot_q4_0_q8_1(int n, float* s, const void* vx, const void* vy)
 * (include/gemm_reference.h:276-306): *s = the dot of n elements, vx Q4_0, vy Q8_1. */
void qg_vec_dot_q4_0_q8_1_cpu(int n, float* s, const void* vx, const void* vy);

/* vec_dot_q8_0_q8_1 (include/gemm_reference.h:311-335) */
void qg_vec_dot_q8_0_q8_1_cpu(int n, float* s, const void* vx, const void* vy);

/* gemm_w8a8_reference (include/gemm_reference.h:233-267): Q8_0 weights. */
int qg_gemm_w8a8_cpu(const void* A_q8_1, const void* B_q8_0, float* C, int M, int N, int K);

/* Every weight format of qg_gemm_w4a8 (qg_type ids Q4_0/Q4_1/Q5_0/Q5_1/Q8_0), the same
 * per-block formulas as the GPU library (qg_common.hpp header), rows over `threads` threads
 * (<= 0: one). */
int qg_gemm_w4a8_cpu_mt(const void* A_q8_1, const void* B, float* C, int M, int N, int K, int wtype, int threads);

/* gemm_fp32_reference (include/gemm_reference.h:38-58): float accumulation in k order. */
int qg_gemm_fp32_cpu(const float* A, const float* B, float* C, int M, int N, int K);

/* quantize_row_q8_1_ref / quantize_row_q4_0_ref (include/quantize.h:165-193, 35-70). */
int qg_quantize_row_q8_1_cpu(const float* x, void* y, int64_t k);
int qg_quantize_row_q4_0_cpu(const float* x, void* y, int64_t k);

/* The measurement recipe of SURVEY.md §8(d) (tests/step4_w4a8_gemm.cu:142-148): glibc
 * srand(seed), then A[M][K] and B[N][K] drawn as 2*rand()/RAND_MAX - 1, A first. Writes A (if a
 * is not NULL) and rows [row0, row1) of B (if b is not NULL; a rank's shard), advancing the
 * generator over the rows it skips. Uses the process-wide libc generator. */
int qg_fill_step4_cpu(unsigned seed, int M, int N, int K, int row0, int row1, float* a, float* b);

#ifdef __cplusplus
}
#endif

#endif /* QG_QG_HOST_H */
