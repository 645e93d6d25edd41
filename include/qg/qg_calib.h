/*
 * qg/qg_calib.h — calibration kernels of `libqg_calib.so` (measurement only, not the product).
 *
 * bench.py times them under the same protocol as the product GEMV (hipGraph of back-to-back launches,
 * HIP events on the launch stream, rotating weight copies) to put the single-launch floor into the
 * bench line (`roofline.floor_us`): an empty kernel with the GEMV's grid, and a pure coalesced read
 * of the GEMV's algorithmic bytes in one launch. Stream-ordered, no host sync; 0 = ok, negative =
 * the qg_status codes of qg/qg.h.
 */
#ifndef QG_QG_CALIB_H
#define QG_QG_CALIB_H

#include <stddef.h>
#include <stdint.h>

#include "qg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* grid x block threads that do nothing (block 64..1024, a multiple of 64). */
int qg_calib_empty(int grid, int block, qg_stream_t stream);
/* Read `bytes` (a multiple of 16, src 16-B aligned) once with 16-B loads: each thread reads
 * `loads_per_thread` (1..8) 16-B pieces, block-contiguous and lane-coalesced; the XOR of everything
 * read is compared against a constant and only then written to *sink (never, in practice), so the
 * loads cannot be removed and the kernel stores nothing. */
int qg_calib_read(const void* src, size_t bytes, int loads_per_thread, int block, uint32_t* sink, qg_stream_t stream);
/* The M = 1 Q4_0 GEMV's load shape (gemv1_kernel<2, 2, 64, 1024>) without its arithmetic: N weight rows of
 * K/64 36-B units (K <= 4096), 16 rows per 1024-thread workgroup, lane l of row r loading unit l with 9
 * dword loads, the GEMV's XCD-aware tile order. out != NULL: each row also stores one float to out[r]
 * (the GEMV's output write); out == NULL: nothing stored (XOR into *sink as qg_calib_read). */
int qg_calib_read_units(const void* B, int N, int K, float* out, uint32_t* sink, qg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* QG_QG_CALIB_H */
