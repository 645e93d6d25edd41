/*
 * qg_oracle.c — CPU restatement of the reference's W4A8 ground truth. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline. The product (libqg_hip.so) never calls it.
 *
 * Every function restates one reference function operation for operation, in plain C11 with
 * IEEE single-precision arithmetic and no FMA contraction (built with -ffp-contract=off), so its
 * results are bit-identical to the reference's CPU path on x86-64:
 *
 *   qgo_fill_uniform_step4   tests/step4_w4a8_gemm.cu:142-148 (glibc srand/rand, A then B)
 *   qgo_quantize_row_q4_0    include/quantize.h:35-70
 *   qgo_quantize_row_q8_0    include/quantize.h:111-135
 *   qgo_quantize_row_q8_1    include/quantize.h:165-193   (s = sum of the original floats)
 *   qgo_quantize_q8_1_fw     tests/framework/test_framework.cuh:195-225 (s = d * sum(q))
 *   qgo_quantize_q4_1/5_0/5_1 tests/framework/test_framework.cuh:256-367
 *   qgo_quantize_q8_1_fused_f16 kernels/gemm/gemm_fused.cuh:76-143 (per-block semantics of the
 *                            fused kernel's smem quantizer: tree-reduced amax/sum, id from the
 *                            f16-rounded d, q clamped to +-127 — race-free restatement)
 *   qgo_gemm_q4_0_fp16_fused kernels/gemm/gemm_fused.cuh:157-338 (weight-major out[M][N], N fp16 tokens)
 *   qgo_dequantize           include/quantize.h:84-102, 140-150, 198-210 + per-format formulas
 *   qgo_gemm_fp32            include/gemm_reference.h:38-58
 *   qgo_gemm_w4a16           include/gemm_reference.h:73-112
 *   qgo_gemm_w8a16           include/gemm_cuda_naive.cuh:120-143 (no CPU reference exists for W8A16)
 *   qgo_gemm_w4a8            include/gemm_reference.h:175-222 (Q4_0) and, for Q4_1/Q5_0/Q5_1, the
 *                            same loop with the corrected block formulas of
 *                            kernels/gemm/gemm_quant_formats.cuh:105-267 (no /4, SURVEY.md §0.2;
 *                            Q4_1 as flashinfer_trace/.../w4_1a8_q4_1_q8_1_n4096_k4096.json:79)
 *   qgo_gemm_w8a8            include/gemm_reference.h:233-267 (also qgo_gemm_w4a8 with t = Q8_0)
 *   qgo_vec_dot_q4_0_q8_1    include/gemm_reference.h:276-306
 *   qgo_dot4                 __dp4a semantics, include/gemm_cuda_dp4a.cuh:67-77
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/qg/blocks.h"

#define T_Q4_0 2
#define T_Q4_1 3
#define T_Q5_0 6
#define T_Q5_1 7
#define T_Q8_0 8
#define T_Q8_1 9

/* ---- IEEE half <-> float (cuda_fp16 __float2half is round-to-nearest-even) ---- */
float qgo_h2f(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31;
    uint32_t e = (h >> 10) & 0x1F, m = h & 0x3FF, u;
    if (e == 0) {
        if (m == 0) u = s;
        else { /* subnormal: normalise */
            e = 127 - 15 + 1;
            while (!(m & 0x400)) { m <<= 1; e--; }
            m &= 0x3FF;
            u = s | (e << 23) | (m << 13);
        }
    } else if (e == 31) u = s | 0x7F800000u | (m << 13);
    else u = s | ((e + 127 - 15) << 23) | (m << 13);
    float f;
    memcpy(&f, &u, 4);
    return f;
}

uint16_t qgo_f2h(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    const uint32_t s = (u >> 16) & 0x8000u;
    const int32_t e = (int32_t)((u >> 23) & 0xFF);
    uint32_t m = u & 0x7FFFFFu;
    if (e == 255) return (uint16_t)(s | 0x7C00u | (m ? 0x200u : 0u));
    int32_t he = e - 127 + 15;
    if (he >= 31) return (uint16_t)(s | 0x7C00u);
    if (he <= 0) {
        if (he < -10) return (uint16_t)s;
        m |= 0x800000u;
        const int shift = 14 - he; /* 24-bit mantissa -> 10-bit subnormal */
        uint32_t hm = m >> shift;
        const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (hm & 1))) hm++;
        return (uint16_t)(s | hm);
    }
    uint32_t hm = m >> 13;
    const uint32_t rem = m & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (hm & 1))) {
        hm++;
        if (hm == 0x400u) { hm = 0; he++; if (he >= 31) return (uint16_t)(s | 0x7C00u); }
    }
    return (uint16_t)(s | ((uint32_t)he << 10) | hm);
}

/* ---- input recipe: tests/step4_w4a8_gemm.cu:142-148 ---- */
void qgo_fill_uniform_step4(unsigned seed, float* a, int64_t na, float* b, int64_t nb) {
    srand(seed);
    for (int64_t i = 0; i < na; i++) a[i] = 2.0f * (float)rand() / RAND_MAX - 1.0f;
    for (int64_t i = 0; i < nb; i++) b[i] = 2.0f * (float)rand() / RAND_MAX - 1.0f;
}

/* ---- quantizers ---- */
void qgo_quantize_row_q4_0(const float* src, void* dstv, int64_t k) {
    qg_block_q4_0* dst = (qg_block_q4_0*)dstv;
    const int64_t nb = k / QG_QK;
    for (int64_t i = 0; i < nb; i++) {
        const float* x = src + i * QG_QK;
        float amax = 0.0f;
        for (int j = 0; j < QG_QK; j++) amax = fmaxf(amax, fabsf(x[j]));
        const float d = amax / 7.0f;
        dst[i].d = qgo_f2h(d);
        const float id = (d > 0) ? 1.0f / d : 0.0f;
        for (int j = 0; j < QG_QK / 2; j++) {
            int q0 = (int)roundf(x[j] * id) + 8;
            int q1 = (int)roundf(x[j + QG_QK / 2] * id) + 8;
            q0 = q0 < 0 ? 0 : (q0 > 15 ? 15 : q0);
            q1 = q1 < 0 ? 0 : (q1 > 15 ? 15 : q1);
            dst[i].qs[j] = (uint8_t)((q1 << 4) | (q0 & 0x0F));
        }
    }
}

static void quant_q8(const float* x, float* d_out, float* sum_out, int8_t* qs, int clamp_lo) {
    float amax = 0.0f, sum = 0.0f;
    for (int j = 0; j < QG_QK; j++) {
        amax = fmaxf(amax, fabsf(x[j]));
        sum += x[j];
    }
    const float d = amax / 127.0f;
    const float id = (d > 0) ? 1.0f / d : 0.0f;
    for (int j = 0; j < QG_QK; j++) {
        int q = (int)roundf(x[j] * id);
        q = q < clamp_lo ? clamp_lo : (q > 127 ? 127 : q);
        qs[j] = (int8_t)q;
    }
    *d_out = d;
    *sum_out = sum;
}

void qgo_quantize_row_q8_0(const float* src, void* dstv, int64_t k) {
    qg_block_q8_0* dst = (qg_block_q8_0*)dstv;
    for (int64_t i = 0; i < k / QG_QK; i++) {
        float d, s;
        quant_q8(src + i * QG_QK, &d, &s, dst[i].qs, -128);
        dst[i].d = qgo_f2h(d);
    }
}

void qgo_quantize_row_q8_1(const float* src, void* dstv, int64_t k) {
    qg_block_q8_1* dst = (qg_block_q8_1*)dstv;
    for (int64_t i = 0; i < k / QG_QK; i++) {
        float d, s;
        quant_q8(src + i * QG_QK, &d, &s, dst[i].qs, -128);
        dst[i].d = qgo_f2h(d);
        dst[i].s = qgo_f2h(s);
    }
}

void qgo_quantize_q8_1_fw(const float* src, void* dstv, int64_t k) {
    qg_block_q8_1* dst = (qg_block_q8_1*)dstv;
    for (int64_t b = 0; b < k / QG_QK; b++) {
        const float* x = src + b * QG_QK;
        float amax = 0.0f;
        for (int i = 0; i < QG_QK; i++) {
            const float a = fabsf(x[i]);
            if (a > amax) amax = a;
        }
        const float scale = amax / 127.0f;
        const float inv = (scale > 0) ? (1.0f / scale) : 0.0f;
        int sum_q = 0;
        for (int i = 0; i < QG_QK; i++) {
            int8_t v = (int8_t)roundf(x[i] * inv);
            v = (v < -127) ? -127 : ((v > 127) ? 127 : v);
            dst[b].qs[i] = v;
            sum_q += v;
        }
        dst[b].d = qgo_f2h(scale);
        dst[b].s = qgo_f2h(sum_q * scale);
    }
}

/* gemm_fused.cuh:76-143. Thread t < 32 holds x[t]; max/sum halve 16, 8, 4, 2 then lanes 0+1. */
void qgo_quantize_q8_1_fused_f16(const uint16_t* src, void* dstv, int64_t k) {
    qg_block_q8_1* dst = (qg_block_q8_1*)dstv;
    for (int64_t b = 0; b < k / QG_QK; b++) {
        float x[32], mx[32], sm[32];
        for (int t = 0; t < 32; t++) {
            x[t] = qgo_h2f(src[b * QG_QK + t]);
            mx[t] = fabsf(x[t]);
            sm[t] = x[t];
        }
        for (int h = 16; h >= 2; h /= 2)
            for (int t = 0; t < h; t++) {
                mx[t] = fmaxf(mx[t], mx[t + h]);
                sm[t] += sm[t + h];
            }
        const float amax = fmaxf(mx[0], mx[1]);
        const float sum = sm[0] + sm[1];
        dst[b].d = qgo_f2h(amax / 127.0f);
        dst[b].s = qgo_f2h(sum);
        const float d = qgo_h2f(dst[b].d);
        const float id = (d != 0.0f) ? 1.0f / d : 0.0f;
        for (int t = 0; t < 32; t++) {
            /* (int8_t)roundf(.) then clamp; |x*id| <= 127 * d/f16(d) < 127.07, so no wrap occurs */
            int q = (int)roundf(x[t] * id);
            q = q < -127 ? -127 : (q > 127 ? 127 : q);
            dst[b].qs[t] = (int8_t)q;
        }
    }
}

static void minmax(const float* x, float* mn, float* mx) {
    float lo = x[0], hi = x[0];
    for (int i = 1; i < QG_QK; i++) {
        if (x[i] < lo) lo = x[i];
        if (x[i] > hi) hi = x[i];
    }
    *mn = lo;
    *mx = hi;
}

void qgo_quantize_q4_1(const float* src, void* dstv, int64_t k) {
    qg_block_q4_1* dst = (qg_block_q4_1*)dstv;
    for (int64_t b = 0; b < k / QG_QK; b++) {
        const float* x = src + b * QG_QK;
        float mn, mx;
        minmax(x, &mn, &mx);
        const float scale = (mx - mn) / 15.0f;
        const float inv = (scale > 0) ? (1.0f / scale) : 0.0f;
        dst[b].d = qgo_f2h(scale);
        dst[b].m = qgo_f2h(mn);
        for (int i = 0; i < 16; i++) {
            int q0 = (int)roundf((x[i] - mn) * inv);
            int q1 = (int)roundf((x[i + 16] - mn) * inv);
            q0 = q0 < 0 ? 0 : (q0 > 15 ? 15 : q0);
            q1 = q1 < 0 ? 0 : (q1 > 15 ? 15 : q1);
            dst[b].qs[i] = (uint8_t)((q1 << 4) | q0);
        }
    }
}

void qgo_quantize_q5_0(const float* src, void* dstv, int64_t k) {
    qg_block_q5_0* dst = (qg_block_q5_0*)dstv;
    for (int64_t b = 0; b < k / QG_QK; b++) {
        const float* x = src + b * QG_QK;
        float amax = 0.0f;
        for (int i = 0; i < QG_QK; i++) {
            const float a = fabsf(x[i]);
            if (a > amax) amax = a;
        }
        const float scale = amax / 15.0f;
        const float inv = (scale > 0) ? (1.0f / scale) : 0.0f;
        dst[b].d = qgo_f2h(scale);
        uint32_t qh = 0;
        for (int i = 0; i < 16; i++) {
            int q0 = (int)roundf(x[i] * inv) + 16;
            int q1 = (int)roundf(x[i + 16] * inv) + 16;
            q0 = q0 < 0 ? 0 : (q0 > 31 ? 31 : q0);
            q1 = q1 < 0 ? 0 : (q1 > 31 ? 31 : q1);
            dst[b].qs[i] = (uint8_t)(((q1 & 0x0F) << 4) | (q0 & 0x0F));
            qh |= (uint32_t)((q0 >> 4) & 1) << i;
            qh |= (uint32_t)((q1 >> 4) & 1) << (i + 16);
        }
        memcpy(dst[b].qh, &qh, 4);
    }
}

void qgo_quantize_q5_1(const float* src, void* dstv, int64_t k) {
    qg_block_q5_1* dst = (qg_block_q5_1*)dstv;
    for (int64_t b = 0; b < k / QG_QK; b++) {
        const float* x = src + b * QG_QK;
        float mn, mx;
        minmax(x, &mn, &mx);
        const float scale = (mx - mn) / 31.0f;
        const float inv = (scale > 0) ? (1.0f / scale) : 0.0f;
        dst[b].d = qgo_f2h(scale);
        dst[b].m = qgo_f2h(mn);
        uint32_t qh = 0;
        for (int i = 0; i < 16; i++) {
            int q0 = (int)roundf((x[i] - mn) * inv);
            int q1 = (int)roundf((x[i + 16] - mn) * inv);
            q0 = q0 < 0 ? 0 : (q0 > 31 ? 31 : q0);
            q1 = q1 < 0 ? 0 : (q1 > 31 ? 31 : q1);
            dst[b].qs[i] = (uint8_t)(((q1 & 0x0F) << 4) | (q0 & 0x0F));
            qh |= (uint32_t)((q0 >> 4) & 1) << i;
            qh |= (uint32_t)((q1 >> 4) & 1) << (i + 16);
        }
        memcpy(dst[b].qh, &qh, 4);
    }
}

int qgo_block_bytes(int t) {
    switch (t) {
        case T_Q4_0: return 18;
        case T_Q4_1: return 20;
        case T_Q5_0: return 22;
        case T_Q5_1: return 24;
        case T_Q8_0: return 34;
        case T_Q8_1: return 36;
    }
    return 0;
}

/* Stored (unsigned) weight values of one block, element order 0..31, plus d and m. */
static void weight_block(int t, const uint8_t* blk, int q[32], float* d, float* m) {
    uint16_t dh, mh = 0;
    memcpy(&dh, blk, 2);
    *d = qgo_h2f(dh);
    if (t == T_Q8_0) { /* signed bytes in element order */
        for (int j = 0; j < 32; j++) q[j] = (int8_t)blk[2 + j];
        *m = 0.0f;
        return;
    }
    int qs_off = 2, qh_off = -1;
    if (t == T_Q4_1) { memcpy(&mh, blk + 2, 2); qs_off = 4; }
    if (t == T_Q5_0) { qh_off = 2; qs_off = 6; }
    if (t == T_Q5_1) { memcpy(&mh, blk + 2, 2); qh_off = 4; qs_off = 8; }
    *m = (t == T_Q4_1 || t == T_Q5_1) ? qgo_h2f(mh) : 0.0f;
    uint32_t qh = 0;
    if (qh_off >= 0) memcpy(&qh, blk + qh_off, 4);
    for (int j = 0; j < 16; j++) {
        int lo = blk[qs_off + j] & 0x0F, hi = blk[qs_off + j] >> 4;
        if (qh_off >= 0) {
            lo |= (int)((qh >> j) & 1) << 4;
            hi |= (int)((qh >> (j + 16)) & 1) << 4;
        }
        q[j] = lo;
        q[j + 16] = hi;
    }
}

void qgo_dequantize(int t, const void* src, float* dst, int64_t k) {
    const uint8_t* p = (const uint8_t*)src;
    const int bb = qgo_block_bytes(t);
    for (int64_t b = 0; b < k / QG_QK; b++) {
        const uint8_t* blk = p + b * bb;
        float* o = dst + b * QG_QK;
        if (t == T_Q8_0 || t == T_Q8_1) {
            uint16_t dh;
            memcpy(&dh, blk, 2);
            const float d = qgo_h2f(dh);
            const int8_t* qs = (const int8_t*)(blk + (t == T_Q8_0 ? 2 : 4));
            for (int j = 0; j < QG_QK; j++) o[j] = qs[j] * d;
            continue;
        }
        int q[32];
        float d, m;
        weight_block(t, blk, q, &d, &m);
        for (int j = 0; j < QG_QK; j++) {
            if (t == T_Q4_0) o[j] = (q[j] - 8) * d;
            else if (t == T_Q5_0) o[j] = (q[j] - 16) * d;
            else o[j] = q[j] * d + m;
        }
    }
}

int32_t qgo_dot4(int32_t a, int32_t b, int32_t c) {
    for (int i = 0; i < 4; i++) c += (int32_t)(int8_t)(a >> (8 * i)) * (int32_t)(int8_t)(b >> (8 * i));
    return c;
}

/* ---- GEMMs ---- */
void qgo_gemm_fp32(const float* A, const float* B, float* C, int M, int N, int K) {
    memset(C, 0, (size_t)M * N * sizeof(float));
    for (int i = 0; i < M; i++)
        for (int j = 0; j < N; j++) {
            float sum = 0.0f;
            for (int k = 0; k < K; k++) sum += A[(size_t)i * K + k] * B[(size_t)j * K + k];
            C[(size_t)i * N + j] = sum;
        }
}

void qgo_gemm_w4a16(const float* A, const void* Bv, float* C, int M, int N, int K) {
    const qg_block_q4_0* B = (const qg_block_q4_0*)Bv;
    const int nb = K / QG_QK;
    memset(C, 0, (size_t)M * N * sizeof(float));
    for (int i = 0; i < M; i++)
        for (int j = 0; j < N; j++) {
            float sum = 0.0f;
            for (int b = 0; b < nb; b++) {
                const qg_block_q4_0* blk = &B[(size_t)j * nb + b];
                const float d = qgo_h2f(blk->d);
                for (int k = 0; k < QG_QK / 2; k++) {
                    const int q0 = blk->qs[k] & 0x0F, q1 = blk->qs[k] >> 4;
                    const float w0 = (q0 - 8) * d, w1 = (q1 - 8) * d;
                    const int k_idx = b * QG_QK;
                    sum += A[(size_t)i * K + k_idx + k] * w0;
                    sum += A[(size_t)i * K + k_idx + k + QG_QK / 2] * w1;
                }
            }
            C[(size_t)i * N + j] = sum;
        }
}

/* include/gemm_cuda_naive.cuh:120-143 (gemm_w8a16_naive_kernel), the W8A16 sum order. */
void qgo_gemm_w8a16(const float* A, const void* Bv, float* C, int M, int N, int K) {
    const qg_block_q8_0* B = (const qg_block_q8_0*)Bv;
    const int nb = K / QG_QK;
    for (int i = 0; i < M; i++)
        for (int j = 0; j < N; j++) {
            float sum = 0.0f;
            for (int b = 0; b < nb; b++) {
                const float d = qgo_h2f(B[(size_t)j * nb + b].d);
                for (int k = 0; k < QG_QK; k++) {
                    const float w = B[(size_t)j * nb + b].qs[k] * d;
                    sum += A[(size_t)i * K + b * QG_QK + k] * w;
                }
            }
            C[(size_t)i * N + j] = sum;
        }
}

static int32_t block_sumi(const int q[32], const int8_t* aq) {
    int32_t sumi = 0;
    /* gemm_reference.h:202-212: pairs (k, k+16) in k order */
    for (int k = 0; k < QG_QK / 2; k++) {
        sumi += (int32_t)aq[k] * q[k];
        sumi += (int32_t)aq[k + QG_QK / 2] * q[k + QG_QK / 2];
    }
    return sumi;
}

static float block_term(int t, int32_t sumi, float dw, float mw, float da, float sa) {
    if (t == T_Q4_0) return dw * (da * sumi - 8.0f * sa);
    if (t == T_Q5_0) return dw * (da * sumi - 16.0f * sa);
    if (t == T_Q8_0) return sumi * da * dw; /* gemm_reference.h:260 */
    return dw * da * sumi + mw * sa; /* Q4_1 / Q5_1 */
}

typedef struct {
    const uint8_t* A;
    const uint8_t* B;
    float* C;
    int32_t* sumi;
    int M, N, K, t, n0, n1;
} gemm_job;

static void* gemm_rows(void* arg) {
    const gemm_job* jb = (const gemm_job*)arg;
    const int nb = jb->K / QG_QK, bb = qgo_block_bytes(jb->t);
    for (int i = 0; i < jb->M; i++)
        for (int j = jb->n0; j < jb->n1; j++) {
            float sum = 0.0f;
            for (int b = 0; b < nb; b++) {
                const qg_block_q8_1* ab = (const qg_block_q8_1*)(jb->A + ((size_t)i * nb + b) * 36);
                const float da = qgo_h2f(ab->d), sa = qgo_h2f(ab->s);
                int q[32];
                float dw, mw;
                weight_block(jb->t, jb->B + ((size_t)j * nb + b) * bb, q, &dw, &mw);
                const int32_t sumi = block_sumi(q, ab->qs);
                if (jb->sumi) jb->sumi[((size_t)i * jb->N + j) * nb + b] = sumi;
                sum += block_term(jb->t, sumi, dw, mw, da, sa);
            }
            if (jb->C) jb->C[(size_t)i * jb->N + j] = sum;
        }
    return NULL;
}

/* C[M][N] = A_q8_1[M][K/32] . B[N][K/32]^T, optional per-block sumi[M][N][K/32]. */
void qgo_gemm_w4a8(const void* A, const void* B, float* C, int32_t* sumi, int M, int N, int K, int t) {
    if (C) memset(C, 0, (size_t)M * N * sizeof(float));
    gemm_job jb = {(const uint8_t*)A, (const uint8_t*)B, C, sumi, M, N, K, t, 0, N};
    gemm_rows(&jb);
}

/* Row-partitioned (N split over nthreads) — the secondary CPU baseline; same per-element order. */
void qgo_gemm_w4a8_mt(const void* A, const void* B, float* C, int M, int N, int K, int t, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    gemm_job jobs[256];
    for (int i = 0; i < nthreads; i++) {
        jobs[i] = (gemm_job){(const uint8_t*)A, (const uint8_t*)B, C, NULL, M, N, K, t,
                             (int)((int64_t)N * i / nthreads), (int)((int64_t)N * (i + 1) / nthreads)};
        pthread_create(&th[i], NULL, gemm_rows, &jobs[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
}

/* gemm_fused.cuh:311-338: out[M][N] = W_q4_0[M][K/32] . quant_fused(act_f16[N][K])^T. The
 * reference sums each output over lane-strided blocks then a warp tree; this sums in block order
 * (same block terms, dw * (da * sumi - 8 * sa) at :265; outputs agree to summation order). */
void qgo_gemm_q4_0_fp16_fused(const void* W, const uint16_t* act, float* out, int M, int N, int K) {
    const int nb = K / QG_QK;
    qg_block_q8_1* aq = (qg_block_q8_1*)malloc((size_t)N * nb * sizeof(qg_block_q8_1));
    qgo_quantize_q8_1_fused_f16(act, aq, (int64_t)N * K);
    float* c = (float*)malloc((size_t)N * M * sizeof(float));
    qgo_gemm_w4a8(aq, W, c, NULL, N, M, K, T_Q4_0); /* c[N][M] activation-major */
    for (int i = 0; i < M; i++)
        for (int j = 0; j < N; j++) out[(size_t)i * N + j] = c[(size_t)j * M + i];
    free(c);
    free(aq);
}

void qgo_gemm_w8a8(const void* Av, const void* Bv, float* C, int M, int N, int K) {
    const qg_block_q8_1* A = (const qg_block_q8_1*)Av;
    const qg_block_q8_0* B = (const qg_block_q8_0*)Bv;
    const int nb = K / QG_QK;
    memset(C, 0, (size_t)M * N * sizeof(float));
    for (int i = 0; i < M; i++)
        for (int j = 0; j < N; j++) {
            float sum = 0.0f;
            for (int b = 0; b < nb; b++) {
                const float da = qgo_h2f(A[(size_t)i * nb + b].d), dw = qgo_h2f(B[(size_t)j * nb + b].d);
                int32_t sumi = 0;
                for (int k = 0; k < QG_QK; k++) sumi += (int32_t)A[(size_t)i * nb + b].qs[k] * (int32_t)B[(size_t)j * nb + b].qs[k];
                sum += sumi * da * dw;
            }
            C[(size_t)i * N + j] = sum;
        }
}

void qgo_vec_dot_q4_0_q8_1(int n, float* s, const void* vx, const void* vy) {
    const qg_block_q4_0* x = (const qg_block_q4_0*)vx;
    const qg_block_q8_1* y = (const qg_block_q8_1*)vy;
    float sum = 0.0f;
    for (int i = 0; i < n / QG_QK; i++) {
        const float dw = qgo_h2f(x[i].d), da = qgo_h2f(y[i].d), sa = qgo_h2f(y[i].s);
        int32_t sumi = 0;
        for (int k = 0; k < QG_QK / 2; k++) {
            sumi += (int32_t)y[i].qs[k] * (x[i].qs[k] & 0x0F);
            sumi += (int32_t)y[i].qs[k + QG_QK / 2] * (x[i].qs[k] >> 4);
        }
        sum += dw * (da * sumi - 8.0f * sa);
    }
    *s = sum;
}
