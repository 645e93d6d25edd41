"""CPU oracle for the W4A8 path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker (or the timed CPU baseline). The product path
(``quant_gemm`` over ``libqg_hip.so``) never imports it and has no CPU fallback.

It wraps ``_build/libqg_oracle.so`` (``qg_oracle.c``: an operation-for-operation C restatement
of the reference's CPU ground truth, see the file:line table in its header) with numpy
conveniences. Pinning (``tests/test_oracle.py``):
  * known-answer values held in the reference's own files (TEST_RESULTS.md:113-119, the
    test_cpu_ref.cpp / test_dot.cpp / test_q8_1.cpp programs compiled from the reference tree
    into ``_ref/``, test_dp4a.cu:24-48);
  * golden vectors produced by the reference's runnable Python definitions
    (flashinfer_trace/definitions/**.json ``reference``) via tests/golden/make_golden.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libqg_oracle.so")

Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1 = 2, 3, 6, 7, 8, 9
BLOCK_BYTES = {Q4_0: 18, Q4_1: 20, Q5_0: 22, Q5_1: 24, Q8_0: 34, Q8_1: 36}
TYPE_NAMES = {Q4_0: "q4_0", Q4_1: "q4_1", Q5_0: "q5_0", Q5_1: "q5_1", Q8_0: "q8_0", Q8_1: "q8_1"}

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I, I64, U = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint
        L.qgo_fill_uniform_step4.argtypes = [U, P, I64, P, I64]
        for name in ("qgo_quantize_row_q4_0", "qgo_quantize_row_q8_0", "qgo_quantize_row_q8_1",
                     "qgo_quantize_q8_1_fw", "qgo_quantize_q4_1", "qgo_quantize_q5_0", "qgo_quantize_q5_1"):
            getattr(L, name).argtypes = [P, P, I64]
        L.qgo_quantize_q8_1_fused_f16.argtypes = [P, P, I64]
        L.qgo_gemm_q4_0_fp16_fused.argtypes = [P, P, P, I, I, I]
        L.qgo_dequantize.argtypes = [I, P, P, I64]
        L.qgo_gemm_fp32.argtypes = [P, P, P, I, I, I]
        L.qgo_gemm_w4a16.argtypes = [P, P, P, I, I, I]
        L.qgo_gemm_w8a16.argtypes = [P, P, P, I, I, I]
        L.qgo_gemm_w4a8.argtypes = [P, P, P, P, I, I, I, I]
        L.qgo_gemm_w4a8_mt.argtypes = [P, P, P, I, I, I, I, I]
        L.qgo_gemm_w8a8.argtypes = [P, P, P, I, I, I]
        L.qgo_vec_dot_q4_0_q8_1.argtypes = [I, P, P, P]
        L.qgo_dot4.argtypes = [ctypes.c_int32] * 3
        L.qgo_dot4.restype = ctypes.c_int32
        L.qgo_f2h.argtypes = [ctypes.c_float]
        L.qgo_f2h.restype = ctypes.c_uint16
        L.qgo_h2f.argtypes = [ctypes.c_uint16]
        L.qgo_h2f.restype = ctypes.c_float
        _lib = L
    return _lib


def _p(a: np.ndarray) -> ctypes.c_void_p:
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def fill_uniform_step4(m: int, n: int, k: int, seed: int = 42):
    """A[m,k], B[n,k] ~ U[-1,1] from glibc srand(seed)/rand(), A first (tests/step4_w4a8_gemm.cu:142-148)."""
    a = np.empty((m, k), np.float32)
    b = np.empty((n, k), np.float32)
    lib().qgo_fill_uniform_step4(seed, _p(a), a.size, _p(b), b.size)
    return a, b


_QUANT = {Q4_0: "qgo_quantize_row_q4_0", Q8_0: "qgo_quantize_row_q8_0", Q8_1: "qgo_quantize_row_q8_1",
          Q4_1: "qgo_quantize_q4_1", Q5_0: "qgo_quantize_q5_0", Q5_1: "qgo_quantize_q5_1"}


def quantize(x: np.ndarray, t: int, variant: int = 0) -> np.ndarray:
    """FP32 [..., K] -> uint8 [..., K/32, block_bytes] (reference CPU quantizers; variant 2 = the
    Solution definitions' semantics, quantize_definition)."""
    if variant == 2:
        return quantize_definition(x, t)
    x = np.ascontiguousarray(x, np.float32)
    k = x.shape[-1]
    assert k % 32 == 0
    out = np.empty(x.shape[:-1] + (k // 32, BLOCK_BYTES[t]), np.uint8)
    fn = "qgo_quantize_q8_1_fw" if (t == Q8_1 and variant == 1) else _QUANT[t]
    getattr(lib(), fn)(_p(x), _p(out), x.size)
    return out


def f16_round_exact(num: int, den: int) -> int:
    """f16 bits (RNE, signless) of the exact rational num/den >= 0 — an independent exact reference for
    the single-rounding f16 conversions below (integer arithmetic only)."""
    from fractions import Fraction
    v = Fraction(num, den)
    if v == 0:
        return 0
    e = v.numerator.bit_length() - v.denominator.bit_length()
    if Fraction(2) ** e > v:
        e -= 1
    e = max(e, -14)                       # below 2^-14: subnormal spacing 2^-24
    q = v / Fraction(2) ** (e - 10)       # significand scaled to 11 integer bits
    n, r = divmod(q.numerator, q.denominator)
    if 2 * r > q.denominator or (2 * r == q.denominator and n & 1):
        n += 1
    if n == 2048:                          # carried into the next binade
        n, e = 1024, e + 1
    if e > 15:
        return 0x7C00
    return ((e + 15) << 10 | (n - 1024)) if n >= 1024 else n


def quantize_definition(x: np.ndarray, t: int) -> np.ndarray:
    """The Solution definitions quantize_q8_1 / quantize_q4_0 restated in numpy from their text
    (schemas/definitions/quantization/quantize_q8_1.json:58, quantize_q4_0.json:55):
      amax = max|x|; d = amax / 127.0 (/ 7.0) as a Python float (double), or 1.0 if amax == 0;
      q = round-half-to-even(x / float32(d)) (torch float32 true division by the scalar), + 8 for Q4_0,
      clamped to [-128, 127] / [0, 15]; Q4_0 qs[i] = q[i] | q[i+16] << 4;
      stored d = f16 of the Python float (one correctly rounded conversion, numpy float64 -> float16);
      Q8_1 s = sum(x): the definition's torch.sum order is unspecified — restated as the fp32 sum in
      element order (include/quantize.h:176-179), the order the GPU variant uses.
    PARITY: Q8_1 is pinned by the flashinfer Q8_1 definition's committed output bytes
    (tests/golden/quantize_q8_1_m16k128.npz, same d / q / tie semantics); the Q4_0 definition has no
    reference-generated fixture (executing the reference's code was denied in round 4):
    its bytes are pinned by this restatement and the asserted mismatch set against the pinned
    include/quantize.h quantizer (tests/test_oracle.py)."""
    assert t in (Q8_1, Q4_0)
    x = np.ascontiguousarray(x, np.float32)
    k = x.shape[-1]
    assert k % 32 == 0
    blk = x.reshape(-1, 32)
    amax = np.abs(blk).max(axis=1)
    div = 127.0 if t == Q8_1 else 7.0
    d64 = np.where(amax > 0, amax.astype(np.float64) / div, 1.0)
    d32 = d64.astype(np.float32)
    q = np.rint(blk / d32[:, None])
    with np.errstate(over="ignore"):  # scales beyond the f16 range store inf, as the f32 -> f16 cast
        dh = d64.astype(np.float16).view(np.uint8).reshape(-1, 2)
    if t == Q8_1:
        s = np.zeros(blk.shape[0], np.float32)
        for j in range(32):
            s = (s + blk[:, j]).astype(np.float32)
        out = np.empty((blk.shape[0], 36), np.uint8)
        out[:, 0:2] = dh
        with np.errstate(over="ignore"):
            out[:, 2:4] = s.astype(np.float16).view(np.uint8).reshape(-1, 2)
        out[:, 4:] = np.clip(q, -128, 127).astype(np.int8).view(np.uint8)
    else:
        qq = np.clip(q + 8, 0, 15).astype(np.uint8)
        out = np.empty((blk.shape[0], 18), np.uint8)
        out[:, 0:2] = dh
        out[:, 2:] = qq[:, :16] | (qq[:, 16:] << 4)
    return out.reshape(x.shape[:-1] + (k // 32, out.shape[-1]))


def quantize_q8_1_fused_f16(x: np.ndarray) -> np.ndarray:
    """FP16 [..., K] -> Q8_1 uint8 [..., K/32, 36], kernels/gemm/gemm_fused.cuh:76-143 semantics."""
    x = np.ascontiguousarray(x, np.float16)
    k = x.shape[-1]
    assert k % 32 == 0
    out = np.empty(x.shape[:-1] + (k // 32, 36), np.uint8)
    lib().qgo_quantize_q8_1_fused_f16(_p(x), _p(out), x.size)
    return out


def gemm_q4_0_fp16_fused(w_q: np.ndarray, act: np.ndarray) -> np.ndarray:
    """Weight-major out[M][N] = W[M] . quant_fused(act[N])^T (kernels/gemm/gemm_fused.cuh:311-338)."""
    w_q = np.ascontiguousarray(w_q, np.uint8)
    act = np.ascontiguousarray(act, np.float16)
    m, nb = w_q.shape[0], w_q.shape[1]
    n, k = act.shape
    assert nb * 32 == k and w_q.shape[2] == 18
    out = np.empty((m, n), np.float32)
    lib().qgo_gemm_q4_0_fp16_fused(_p(w_q), _p(act), _p(out), m, n, k)
    return out


def dequantize(q: np.ndarray, t: int) -> np.ndarray:
    q = np.ascontiguousarray(q, np.uint8)
    k = q.shape[-2] * 32
    out = np.empty(q.shape[:-2] + (k,), np.float32)
    lib().qgo_dequantize(t, _p(q), _p(out), out.size)
    return out


def gemm_fp32(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    m, k = a.shape
    n = b.shape[0]
    c = np.empty((m, n), np.float32)
    lib().qgo_gemm_fp32(_p(a), _p(b), _p(c), m, n, k)
    return c


def gemm_w4a8(a_q: np.ndarray, b_q: np.ndarray, t: int = Q4_0, want_sumi: bool = False):
    """C[M,N] (and optionally sumi[M,N,K/32]) — include/gemm_reference.h:175-222 semantics."""
    a_q = np.ascontiguousarray(a_q, np.uint8)
    b_q = np.ascontiguousarray(b_q, np.uint8)
    m, nb = a_q.shape[0], a_q.shape[1]
    n = b_q.shape[0]
    assert a_q.shape[2] == 36 and b_q.shape[1] == nb and b_q.shape[2] == BLOCK_BYTES[t]
    c = np.empty((m, n), np.float32)
    s = np.empty((m, n, nb), np.int32) if want_sumi else None
    lib().qgo_gemm_w4a8(_p(a_q), _p(b_q), _p(c), _p(s) if want_sumi else None, m, n, nb * 32, t)
    return (c, s) if want_sumi else c


def gemm_w4a8_mt(a_q, b_q, t: int = Q4_0, nthreads: int = 1) -> np.ndarray:
    m, nb = a_q.shape[0], a_q.shape[1]
    n = b_q.shape[0]
    c = np.empty((m, n), np.float32)
    lib().qgo_gemm_w4a8_mt(_p(a_q), _p(b_q), _p(c), m, n, nb * 32, t, nthreads)
    return c


def gemm_w8a8(a_q: np.ndarray, b_q: np.ndarray) -> np.ndarray:
    """include/gemm_reference.h:233-267: Q8_1 activations x Q8_0 weights."""
    m, nb = a_q.shape[0], a_q.shape[1]
    n = b_q.shape[0]
    c = np.empty((m, n), np.float32)
    lib().qgo_gemm_w8a8(_p(np.ascontiguousarray(a_q)), _p(np.ascontiguousarray(b_q)), _p(c), m, n, nb * 32)
    return c


def gemm_w4a16(a: np.ndarray, b_q: np.ndarray) -> np.ndarray:
    m, k = a.shape
    n = b_q.shape[0]
    c = np.empty((m, n), np.float32)
    lib().qgo_gemm_w4a16(_p(np.ascontiguousarray(a, np.float32)), _p(b_q), _p(c), m, n, k)
    return c


def gemm_w8a16(a: np.ndarray, b_q: np.ndarray) -> np.ndarray:
    m, k = a.shape
    n = b_q.shape[0]
    c = np.empty((m, n), np.float32)
    lib().qgo_gemm_w8a16(_p(np.ascontiguousarray(a, np.float32)), _p(np.ascontiguousarray(b_q)), _p(c), m, n, k)
    return c


def w16_tol(a: np.ndarray, b_q: np.ndarray, t: int) -> np.ndarray:
    """fp32 summation-order bound for W4A16/W8A16 outputs: 2 * (K + 2) * 2^-24 * sum_k |a_k w_k|
    (K + 2: the K-term sum plus the per-element / per-block scaling roundings)."""
    w = dequantize(b_q, t).astype(np.float64)
    k = a.shape[1]
    return 2.0 * (k + 2) * 2.0 ** -24 * (np.abs(a.astype(np.float64)) @ np.abs(w).T) + 1e-30


def vec_dot_q4_0_q8_1(x_q4: np.ndarray, y_q8: np.ndarray) -> float:
    s = ctypes.c_float()
    n = x_q4.reshape(-1, 18).shape[0] * 32
    lib().qgo_vec_dot_q4_0_q8_1(n, ctypes.byref(s), _p(np.ascontiguousarray(x_q4)), _p(np.ascontiguousarray(y_q8)))
    return s.value


def dot4(a: int, b: int, c: int = 0) -> int:
    return lib().qgo_dot4(ctypes.c_int32(a), ctypes.c_int32(b), ctypes.c_int32(c))


def nmse(out: np.ndarray, ref: np.ndarray) -> float:
    """Sum e^2 / sum ref^2 in fp64 (tests/framework/test_framework.cuh:41-64)."""
    out = np.asarray(out, np.float64)
    ref = np.asarray(ref, np.float64)
    den = float(np.sum(ref * ref))
    num = float(np.sum((out - ref) ** 2))
    return num / den if den > 0 else (0.0 if num == 0 else float("inf"))


def tile_weights(b_q: np.ndarray, t: int) -> np.ndarray:
    """numpy restatement of the tiled weight layout (qg_tile_weights; the device layout is specified
    by tiled_fmt in llama.cpp-quant-gemm_amd/csrc/qg_mmq_kernel.hpp): [N, K/32, BB] block bytes ->
    1-D bytes, rows in tiles of 32, K/32 in stages of 4 blocks, each (tile, stage) one run of
    128 * BB bytes holding the planes
      QS [row tile i (16 rows)][half][q][r][block][4 B]: qs dword q (+ 4 * half: Q8_0) of row 16 i + r,
      QH [row][block][4 B] (Q5_0 / Q5_1), SC [row][d of blocks 0..3][m of blocks 0..3 (Q4_1 / Q5_1)],
    zero bytes for rows past N and blocks past K/32. A layout check for the tests; not an oracle of
    the reference (the reference has no tiled layout)."""
    n, nb, bb = b_q.shape
    assert bb == BLOCK_BYTES[t]
    tiles, stages = -(-n // 32), -(-nb // 4)
    full = np.zeros((tiles * 32, stages * 4, bb), np.uint8)
    full[:n, :nb] = b_q
    blk = full.reshape(tiles, 32, stages, 4, bb).transpose(0, 2, 1, 3, 4)  # [tile][stage][row][block][byte]
    qs_off = {Q4_0: 2, Q4_1: 4, Q5_0: 6, Q5_1: 8, Q8_0: 2}[t]
    nq = 8 if t == Q8_0 else 4
    qs = blk[..., qs_off:qs_off + 4 * nq].reshape(tiles, stages, 2, 16, 4, nq // 4, 4, 4)  # i r b half q byte
    qs = qs.transpose(0, 1, 2, 5, 6, 3, 4, 7)  # [tile][stage][i][half][q][r][block][byte]
    parts = [qs.reshape(tiles, stages, -1)]
    if t in (Q5_0, Q5_1):
        qh_off = 2 if t == Q5_0 else 4
        parts.append(blk[..., qh_off:qh_off + 4].reshape(tiles, stages, -1))
    sc = [blk[..., 0:2]]
    if t in (Q4_1, Q5_1):
        sc.append(blk[..., 2:4])
    parts.append(np.concatenate([x.reshape(tiles, stages, 32, 8) for x in sc], axis=-1).reshape(tiles, stages, -1))
    out = np.concatenate(parts, axis=-1)
    assert out.shape[-1] == 128 * bb
    return np.ascontiguousarray(out).reshape(-1)


def tile_activations(a_q: np.ndarray) -> np.ndarray:
    """numpy restatement of the tiled activation layout (qg_quantize_q8_1_tiled / qg_tile_activations, round 5;
    LAY_TILED_ACT in llama.cpp-quant-gemm_amd/csrc/qg_kernels.hpp): [M, K/32, 36] Q8_1 block bytes -> 1-D
    bytes, tokens in tiles of 16, K/32 in stages of 4 blocks, each (token tile, stage) one 2304-B run
    [token][block][36 B], zero blocks for tokens past M and blocks past K/32. A layout check for the tests;
    not an oracle of the reference (the reference has no tiled layout)."""
    m, nb, bb = a_q.shape
    assert bb == 36
    tiles, stages = -(-m // 16), -(-nb // 4)
    full = np.zeros((tiles * 16, stages * 4, 36), np.uint8)
    full[:m, :nb] = a_q
    out = full.reshape(tiles, 16, stages, 4, 36).transpose(0, 2, 1, 3, 4)  # [tile][stage][token][block][byte]
    return np.ascontiguousarray(out).reshape(-1)


def _h(x: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(x).view(np.float16).astype(np.float32)[..., 0]


def block_terms(a_q: np.ndarray, b_q: np.ndarray, sumi: np.ndarray, t: int = Q4_0) -> np.ndarray:
    """fp32 per-block terms [M,N,nb] in the reference's operation order (numpy fp32, no FMA)."""
    da = _h(a_q[..., 0:2])[:, None, :]
    sa = _h(a_q[..., 2:4])[:, None, :]
    dw = _h(b_q[..., 0:2])[None, :, :]
    fs = sumi.astype(np.float32)
    if t == Q4_0:
        return dw * (da * fs - np.float32(8.0) * sa)
    if t == Q5_0:
        return dw * (da * fs - np.float32(16.0) * sa)
    if t == Q8_0:
        return fs * da * dw
    mw = _h(b_q[..., 2:4])[None, :, :]
    return dw * da * fs + mw * sa


def block_parts(a_q: np.ndarray, b_q: np.ndarray, sumi: np.ndarray, t: int = Q4_0):
    """The two exact parts of each block term (float64 [M,N,nb]): the scaled dot d_w*d_a*sumi and
    the offset part (-8 d_w s_a for Q4_0, -16 d_w s_a for Q5_0, m_w s_a for Q4_1 / Q5_1, 0 for Q8_0);
    term_b = dot_b + off_b in exact arithmetic (include/gemm_reference.h:202-214)."""
    da = _h(a_q[..., 0:2]).astype(np.float64)[:, None, :]
    sa = _h(a_q[..., 2:4]).astype(np.float64)[:, None, :]
    dw = _h(b_q[..., 0:2]).astype(np.float64)[None, :, :]
    dot = dw * da * sumi.astype(np.float64)
    if t == Q4_0:
        off = -8.0 * dw * sa
    elif t == Q5_0:
        off = -16.0 * dw * sa
    elif t == Q8_0:
        off = np.zeros_like(dot)
    else:
        off = _h(b_q[..., 2:4]).astype(np.float64)[None, :, :] * sa
    return dot, off


def reassoc_tol(a_q: np.ndarray, b_q: np.ndarray, sumi: np.ndarray, t: int = Q4_0, waves: int = 8) -> np.ndarray:
    """Bound for a kernel that rounds the two parts of each block term separately and sums them
    on their own (the MFMA prefill's EPI2 epilogue: d_w*d_a*sumi rounded once per block, the offset
    parts summed by an f16 MFMA and combined at the end, `waves` K-split partial tiles added in fixed
    order): to first order both the reference and that kernel lie within (nb + waves + 2) u
    sum_b (|dot_b| + |off_b|) of the exact sum (u = 2^-24), so they differ by at most twice that.
    Unlike summation_tol this does not assume bit-identical per-block terms: where a block's two
    parts nearly cancel, its term is small but both parts' rounding errors remain."""
    dot, off = block_parts(a_q, b_q, sumi, t)
    nb = dot.shape[-1]
    return 2.0 * (nb + waves + 2) * 2.0 ** -24 * (np.abs(dot) + np.abs(off)).sum(axis=-1) + 1e-30


def summation_tol(a_q: np.ndarray, b_q: np.ndarray, sumi: np.ndarray, t: int = Q4_0) -> np.ndarray:
    """Bound on |fl(sum_b term_b) - fl'(sum_b term_b)| for any two fp32 summation orders
    (2 * nb * 2^-24 * sum_b |term_b|) — the only legitimate CPU/GPU difference once the
    per-block terms are bit-identical."""
    terms = block_terms(a_q, b_q, sumi, t).astype(np.float64)
    nb = terms.shape[-1]
    return 2.0 * nb * 2.0 ** -24 * np.abs(terms).sum(axis=-1) + 1e-30
