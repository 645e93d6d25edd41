/*
 * qg/blocks.h — byte-exact llama.cpp block formats (C and C++, host and device).
 *
 * These are the on-HBM layouts the W4A8 path consumes. They are re-declared here as plain
 * POD structs with the fp16 fields stored as raw uint16_t bit patterns, so the header builds
 * with gcc, g++ and hipcc alike and carries no cuda_fp16/hip_fp16 dependency.
 *
 * Reference layouts (byte-identical):
 *   block_q4_0  18 B  include/quant_types.h:59-64   (compat/ggml_types.h:62-67)
 *   block_q8_0  34 B  include/quant_types.h:85-90
 *   block_q8_1  36 B  include/quant_types.h:116-121 (compat/ggml_types.h:186-191)
 *   block_q4_1  20 B  compat/ggml_types.h:90-96
 *   block_q5_0  22 B  compat/ggml_types.h:111-117
 *   block_q5_1  24 B  compat/ggml_types.h:125-132
 *
 * Nibble packing (include/quantize.h:56-67): qs[j] low nibble = x[j], high nibble = x[j+16].
 * Q5 fifth bit (tests/framework/test_framework.cuh:309-325): bit i of the little-endian u32
 * qh holds bit 4 of element i.
 * Q8_1 ds = {d, s} as half2: d = amax/127, s = Σx of the ORIGINAL floats
 * (include/quantize.h:165-193).
 */
#ifndef QG_BLOCKS_H
#define QG_BLOCKS_H

#include <stdint.h>

#define QG_QK 32 /* elements per block, every format on this path */

typedef struct {
    uint16_t d;      /* fp16 scale */
    uint8_t qs[16];  /* 32 x u4, value = (q - 8) * d */
} qg_block_q4_0;

typedef struct {
    uint16_t d;      /* fp16 scale */
    uint16_t m;      /* fp16 min, value = q * d + m */
    uint8_t qs[16];
} qg_block_q4_1;

typedef struct {
    uint16_t d;      /* fp16 scale, value = (q - 16) * d, q in [0, 31] */
    uint8_t qh[4];   /* bit 4 of each element */
    uint8_t qs[16];  /* low 4 bits */
} qg_block_q5_0;

typedef struct {
    uint16_t d;
    uint16_t m;      /* value = q * d + m */
    uint8_t qh[4];
    uint8_t qs[16];
} qg_block_q5_1;

typedef struct {
    uint16_t d;
    int8_t qs[32];
} qg_block_q8_0;

typedef struct {
    uint16_t d;      /* ds.x: fp16 scale */
    uint16_t s;      /* ds.y: fp16 sum of the original values */
    int8_t qs[32];
} qg_block_q8_1;

#ifdef __cplusplus
static_assert(sizeof(qg_block_q4_0) == 18, "block_q4_0 must be 18 bytes");
static_assert(sizeof(qg_block_q4_1) == 20, "block_q4_1 must be 20 bytes");
static_assert(sizeof(qg_block_q5_0) == 22, "block_q5_0 must be 22 bytes");
static_assert(sizeof(qg_block_q5_1) == 24, "block_q5_1 must be 24 bytes");
static_assert(sizeof(qg_block_q8_0) == 34, "block_q8_0 must be 34 bytes");
static_assert(sizeof(qg_block_q8_1) == 36, "block_q8_1 must be 36 bytes");
#else
_Static_assert(sizeof(qg_block_q4_0) == 18, "block_q4_0 must be 18 bytes");
_Static_assert(sizeof(qg_block_q4_1) == 20, "block_q4_1 must be 20 bytes");
_Static_assert(sizeof(qg_block_q5_0) == 22, "block_q5_0 must be 22 bytes");
_Static_assert(sizeof(qg_block_q5_1) == 24, "block_q5_1 must be 24 bytes");
_Static_assert(sizeof(qg_block_q8_0) == 34, "block_q8_0 must be 34 bytes");
_Static_assert(sizeof(qg_block_q8_1) == 36, "block_q8_1 must be 36 bytes");
#endif

#endif /* QG_BLOCKS_H */
