"""quant_gemm — MI355X (gfx950) W4A8 quantized GEMM, drop-in for the reference's Python face.

Same names, argument meaning, tensor layouts and error behaviour as the reference package
(python/quant_gemm/__init__.py:33-89, python/quant_gemm/csrc/bindings.cpp:19-91):

    weight_q     = quant_gemm.quantize_q4_0(weight)        # f32 [..., K] -> u8 [..., K/32, 18]
    activation_q = quant_gemm.quantize_q8_1(activation)    # f32 [..., K] -> u8 [..., K/32, 36]
    out = quant_gemm.gemm_q4_0_q8_1(weight_q, activation_q, M, N, K)   # f32 [M, N] (weight-major)
    x   = quant_gemm.dequantize_q4_0(weight_q, K)

Differences, all deliberate: kernels run on torch's *current* HIP stream (the reference launches
on the legacy default stream, gemm_ops.cu:250); validation errors raise RuntimeError like
TORCH_CHECK does. Extra entry points expose the rest of the C-ABI: the activation-major
``gemm_w4a8`` (include/gemm_reference.h convention), Q4_1/Q5_0/Q5_1 weights, every quantizer and
the per-block ``debug_sumi`` parity hook. Every call goes to HIP kernels in ``libqg_hip.so``;
there is no CPU path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

__version__ = "0.1.0"

QK4_0 = 32
QK8_1 = 32
BLOCK_Q4_0_BYTES = 18
BLOCK_Q8_1_BYTES = 36

# ggml_type ids (compat/ggml_types.h:199-215)
Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1 = 2, 3, 6, 7, 8, 9
BLOCK_BYTES = {Q4_0: 18, Q4_1: 20, Q5_0: 22, Q5_1: 24, Q8_0: 34, Q8_1: 36}
ALGO_AUTO, ALGO_GEMV, ALGO_MFMA, ALGO_GENERIC, ALGO_RAGGED = 0, 1, 2, 3, 4
WEIGHT_TYPES = (Q4_0, Q4_1, Q5_0, Q5_1, Q8_0)


def _require(cond: bool, msg: str) -> None:
    if not cond:
        raise RuntimeError(msg)


def _stream(dev: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


# ---------------------------------------------------------------------------- quantizers
def quantize(x: torch.Tensor, qtype: int, variant: int = 0) -> torch.Tensor:
    """FP32 [..., K] -> uint8 [..., K/32, block_bytes(qtype)], bytes identical to the reference
    CPU quantizers (include/quantize.h; tests/framework/test_framework.cuh for Q4_1/Q5_x and
    Q8_1 variant 1)."""
    _require(x.is_cuda, "Input must be a CUDA tensor")
    _require(x.dtype == torch.float32, "Input must be float32")
    _require(x.dim() >= 1, "Input must have at least 1 dimension")
    K = x.size(-1)
    _require(K % 32 == 0, f"Last dimension must be divisible by 32, got {K}")
    _require(qtype in BLOCK_BYTES, f"unknown quant type {qtype}")
    x = x.contiguous()
    out = torch.empty(tuple(x.shape[:-1]) + (K // 32, BLOCK_BYTES[qtype]), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        _lib.check(_lib.load().qg_quantize(qtype, variant, _ptr(x), _ptr(out), x.numel(), _stream(x.device)),
                   "quantize")
    return out


def quantize_q4_0(x: torch.Tensor) -> torch.Tensor:
    """Quantize FP32 tensor to Q4_0: [..., K] -> uint8 [..., K//32, 18]."""
    return quantize(x, Q4_0)


def quantize_q8_1(x: torch.Tensor) -> torch.Tensor:
    """Quantize FP32 tensor to Q8_1: [..., K] -> uint8 [..., K//32, 36]."""
    return quantize(x, Q8_1)


def dequantize(x_q: torch.Tensor, qtype: int) -> torch.Tensor:
    _require(x_q.is_cuda, "Input must be a CUDA tensor")
    _require(x_q.dtype == torch.uint8, "Input must be uint8")
    _require(qtype in BLOCK_BYTES, f"unknown quant type {qtype}")
    bb = BLOCK_BYTES[qtype]
    _require(x_q.numel() % bb == 0, f"Input size {x_q.numel()} is not a multiple of {bb}-byte blocks")
    x_q = x_q.contiguous()
    nblocks = x_q.numel() // bb
    shape = tuple(x_q.shape[:-2]) + (x_q.shape[-2] * 32,) if x_q.dim() >= 2 else (nblocks * 32,)
    out = torch.empty(shape, dtype=torch.float32, device=x_q.device)
    with torch.cuda.device(x_q.device):
        _lib.check(_lib.load().qg_dequantize(qtype, _ptr(x_q), _ptr(out), nblocks * 32, _stream(x_q.device)),
                   "dequantize")
    return out


def dequantize_q4_0(x_q: torch.Tensor, K: int) -> torch.Tensor:
    """Dequantize Q4_0 [..., K//32, 18] back to FP32 [..., K]."""
    _require(x_q.is_cuda, "Input must be a CUDA tensor")
    _require(x_q.dtype == torch.uint8, "Input must be uint8")
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    out = dequantize(x_q, Q4_0)
    return out.reshape(tuple(x_q.shape[:-2]) + (K,))


# ---------------------------------------------------------------------------- GEMMs
def _check_blocks(t: torch.Tensor, what: str, rows: int, K: int, bb: int) -> None:
    _require(t.is_cuda, f"{what} must be a CUDA tensor")
    _require(t.dtype == torch.uint8, f"{what} must be uint8")
    expect = rows * (K // 32) * bb
    _require(t.numel() == expect, f"{what} shape mismatch: expected {expect} elements, got {t.numel()}")


def _check_layout(t: torch.Tensor, what: str, nbytes: int, device) -> None:
    """A load-time layout buffer (tiled / packed weights, tiled activations) handed to the C-ABI as a raw
    pointer: the exact byte count, uint8, contiguous, on the product's device (a strided view
    or a non-uint8 tensor of matching numel would otherwise be read as the wrong bytes)."""
    _require(t.dtype == torch.uint8, f"{what} must be a uint8 tensor, got {t.dtype}")
    _require(t.is_contiguous(), f"{what} must be contiguous")
    _require(t.is_cuda and t.device == device, f"{what} must be on {device}, got {t.device}")
    _require(t.numel() == nbytes, f"{what} shape mismatch: expected {nbytes} bytes, got {t.numel()}")


def gemm_w4a8(activation_q: torch.Tensor, weight_q: torch.Tensor, M: int, N: int, K: int,
              wtype: int = Q4_0, algo: int = ALGO_AUTO, out: torch.Tensor | None = None) -> torch.Tensor:
    """Activation-major C[M, N] = A_q8_1[M, K] . B_w[N, K]^T (include/gemm_reference.h:175-222;
    include/llama_adapter.h). M = tokens, N = weight rows.

    ``out``: optional float32 [M, N] destination; its rows may be strided (``out.stride(1) == 1``,
    ``out.stride(0) >= N``, e.g. a column slice of a wider buffer), written through
    ``qg_gemm_w4a8_ldc``."""
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _require(wtype in WEIGHT_TYPES, f"unsupported weight type {wtype}")
    _check_blocks(activation_q, "Activation", M, K, 36)
    _check_blocks(weight_q, "Weight", N, K, BLOCK_BYTES[wtype])
    a = activation_q.contiguous()
    w = weight_q.contiguous()
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=w.device)
    else:
        _require(out.is_cuda and out.dtype == torch.float32 and tuple(out.shape) == (M, N), "bad out tensor")
        _require(out.device == w.device, "out must be on the weights' device")
        _require(M * N == 0 or out.stride(1) == 1 or N == 1, "bad out tensor: rows must be dense")
    ldc = out.stride(0) if M > 1 else N
    _require(ldc >= N, "bad out tensor: row stride below N")
    with torch.cuda.device(w.device):
        _lib.check(_lib.load().qg_gemm_w4a8_ldc(_ptr(a), _ptr(w), _ptr(out), M, N, K, ldc, wtype, algo,
                                                _stream(w.device)), "gemm_w4a8")
    return out


def gemm_w4a8_batched(activation_q: torch.Tensor, weight_q: torch.Tensor, M: int, N: int, K: int,
                      wtype: int = Q4_0) -> torch.Tensor:
    """Strided batch of independent activation-major products: activation_q [B, M, K/32, 36],
    weight_q [B, N, K/32, bb] -> C [B, M, N]. One launch on the GEMV path (M <= 8)."""
    _require(activation_q.is_cuda and weight_q.is_cuda, "Inputs must be CUDA tensors")
    _require(activation_q.dtype == torch.uint8 and weight_q.dtype == torch.uint8, "Inputs must be uint8")
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    B = weight_q.shape[0]
    bb = BLOCK_BYTES[wtype]
    _require(activation_q.shape[0] == B, "batch mismatch")
    _require(activation_q[0].numel() == M * (K // 32) * 36, "Activation shape mismatch")
    _require(weight_q[0].numel() == N * (K // 32) * bb, "Weight shape mismatch")
    a = activation_q.contiguous()
    w = weight_q.contiguous()
    out = torch.empty((B, M, N), dtype=torch.float32, device=w.device)
    with torch.cuda.device(w.device):
        _lib.check(_lib.load().qg_gemm_w4a8_strided_batched(
            _ptr(a), a[0].numel(), _ptr(w), w[0].numel(), _ptr(out), M * N, B, M, N, K, wtype,
            _stream(w.device)), "gemm_w4a8_batched")
    return out


class _GemvItem(ctypes.Structure):
    _fields_ = [("A_q8_1", ctypes.c_void_p), ("B", ctypes.c_void_p), ("C", ctypes.c_void_p),
                ("N", ctypes.c_int), ("ldc", ctypes.c_int)]


def gemm_w4a8_grouped(activations_q, weights_q, Ns, M: int, K: int, wtype: int = Q4_0, outs=None):
    """Grouped activation-major products with independent pointers and row counts
    (qg_gemm_w4a8_grouped): item i = activations_q[i] [M, K/32, 36] (items may share one tensor) x
    weights_q[i] [Ns[i], K/32, bb] -> outs[i] [M, Ns[i]] (allocated unless given; a given out may be
    a row-strided view, e.g. a column slice of a wider buffer). One launch for up to 64 items on the
    GEMV path; each output bit-identical to gemm_w4a8 on its item."""
    n = len(weights_q)
    _require(len(activations_q) == n and len(Ns) == n, "item count mismatch")
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    bb = BLOCK_BYTES[wtype]
    items = (_GemvItem * max(n, 1))()
    res, keep = [], []
    dev = weights_q[0].device if n else torch.device("cuda")
    for i in range(n):
        a, w, N = activations_q[i], weights_q[i], int(Ns[i])
        _require(a.is_cuda and w.is_cuda, "Inputs must be CUDA tensors")
        _require(a.dtype == torch.uint8 and w.dtype == torch.uint8, "Inputs must be uint8")
        _require(a.numel() == M * (K // 32) * 36, "Activation shape mismatch")
        _require(w.numel() == N * (K // 32) * bb, "Weight shape mismatch")
        a, w = a.contiguous(), w.contiguous()
        if outs is None:
            o = torch.empty((M, N), dtype=torch.float32, device=w.device)
        else:
            o = outs[i]
            _require(o.dtype == torch.float32 and o.shape == (M, N) and (N <= 1 or o.stride(1) == 1),
                     "out must be float32 [M, N] with unit column stride")
        keep += [a, w]
        ldc = o.stride(0) if M > 1 else N
        items[i] = _GemvItem(a.data_ptr(), w.data_ptr(), o.data_ptr(), N, ldc)
        res.append(o)
    with torch.cuda.device(dev):
        _lib.check(_lib.load().qg_gemm_w4a8_grouped(items, n, M, K, wtype, _stream(dev)), "gemm_w4a8_grouped")
    return res


def repack_weights(weight_q: torch.Tensor, N: int, K: int, wtype: int = Q4_0) -> torch.Tensor:
    """Load-time layout for K/32 not a multiple of 8 (qg_repack_weights): [N, K'/32, bb] uint8,
    the real blocks then zero blocks (K'/32 = round_up(K/32, 8)). Feed it to gemm_w4a8_prepacked."""
    _require(weight_q.is_cuda and weight_q.dtype == torch.uint8, "weight_q must be a CUDA uint8 tensor")
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    bb = BLOCK_BYTES[wtype]
    _require(weight_q.numel() == N * (K // 32) * bb, "Weight shape mismatch")
    lib = _lib.load()
    nbytes = lib.qg_repack_weights_bytes(N, K, wtype)
    out = torch.empty((N, nbytes // max(N * bb, 1), bb), dtype=torch.uint8, device=weight_q.device)
    w = weight_q.contiguous()
    with torch.cuda.device(w.device):
        _lib.check(lib.qg_repack_weights(_ptr(w), _ptr(out), N, K, wtype, _stream(w.device)), "repack_weights")
    return out


def gemm_w4a8_prepacked(activation_q: torch.Tensor, weight_packed: torch.Tensor, M: int, N: int, K: int,
                        wtype: int = Q4_0) -> torch.Tensor:
    """C [M, N] = the same product as gemm_w4a8(activation_q, weight_q, ...) from
    repack_weights(weight_q) (qg_gemm_w4a8_prepacked; K is the logical K)."""
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _check_blocks(activation_q, "Activation", M, K, 36)
    lib = _lib.load()
    _check_layout(weight_packed, "weight_packed", lib.qg_repack_weights_bytes(N, K, wtype), activation_q.device)
    a = activation_q.contiguous()
    out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    wsb = lib.qg_gemm_w4a8_prepacked_workspace_size(M, K)
    ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=a.device)
    with torch.cuda.device(a.device):
        _lib.check(lib.qg_gemm_w4a8_prepacked(_ptr(a), _ptr(weight_packed), _ptr(out), M, N, K, wtype, _ptr(ws), wsb,
                                              _stream(a.device)), "gemm_w4a8_prepacked")
    return out


def tile_weights(weight_q: torch.Tensor, N: int, K: int, wtype: int = Q4_0) -> torch.Tensor:
    """Load-time tiled layout (qg_tile_weights): 1-D uint8 of qg_tile_weights_bytes(N, K, wtype) —
    rows in tiles of 32, K/32 in stages of 4 blocks, each (tile, stage) one contiguous run in the
    prefill kernel's operand order. Feed it to gemm_w4a8_tiled."""
    _require(weight_q.is_cuda and weight_q.dtype == torch.uint8, "weight_q must be a CUDA uint8 tensor")
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _require(weight_q.numel() == N * (K // 32) * BLOCK_BYTES[wtype], "Weight shape mismatch")
    lib = _lib.load()
    out = torch.empty(lib.qg_tile_weights_bytes(N, K, wtype), dtype=torch.uint8, device=weight_q.device)
    w = weight_q.contiguous()
    with torch.cuda.device(w.device):
        _lib.check(lib.qg_tile_weights(_ptr(w), _ptr(out), N, K, wtype, _stream(w.device)), "tile_weights")
    return out


def gemm_w4a8_tiled(activation_q: torch.Tensor, weight_tiled: torch.Tensor, M: int, N: int, K: int,
                    wtype: int = Q4_0, out: torch.Tensor | None = None) -> torch.Tensor:
    """C [M, N] = the same product as gemm_w4a8(activation_q, weight_q, ...) from
    tile_weights(weight_q) (qg_gemm_w4a8_tiled; any K % 32 == 0)."""
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _check_blocks(activation_q, "Activation", M, K, 36)
    lib = _lib.load()
    _check_layout(weight_tiled, "weight_tiled", lib.qg_tile_weights_bytes(N, K, wtype), activation_q.device)
    a = activation_q.contiguous()
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    _require(out.is_cuda and out.dtype == torch.float32 and out.shape == (M, N) and out.is_contiguous(),
             "out must be a contiguous CUDA float32 [M, N] tensor")
    with torch.cuda.device(a.device):
        _lib.check(lib.qg_gemm_w4a8_tiled(_ptr(a), _ptr(weight_tiled), _ptr(out), M, N, K, wtype, _stream(a.device)),
                   "gemm_w4a8_tiled")
    return out


def quantize_q8_1_tiled(x: torch.Tensor) -> torch.Tensor:
    """FP32 [M, K] -> the tiled activation layout (qg_quantize_q8_1_tiled): 1-D uint8 of
    qg_activations_tiled_bytes(M, K) — 16-token tiles x 4-block stages, each a contiguous 2304-B run, zero
    padded. Feed it to gemm_w4a8_tiled_act."""
    _require(x.is_cuda and x.dtype == torch.float32 and x.dim() == 2, "x must be a 2-D CUDA float32 tensor")
    M, K = x.shape
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    lib = _lib.load()
    xc = x.contiguous()
    out = torch.empty(lib.qg_activations_tiled_bytes(M, K), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        _lib.check(lib.qg_quantize_q8_1_tiled(_ptr(xc), _ptr(out), M, K, _stream(x.device)), "quantize_q8_1_tiled")
    return out


def tile_activations(activation_q: torch.Tensor, M: int, K: int) -> torch.Tensor:
    """Q8_1 rows [M, K/32] -> the tiled activation layout (qg_tile_activations)."""
    _require(activation_q.is_cuda and activation_q.dtype == torch.uint8, "activation_q must be a CUDA uint8 tensor")
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _require(activation_q.numel() == M * (K // 32) * 36, "Activation shape mismatch")
    lib = _lib.load()
    a = activation_q.contiguous()
    out = torch.empty(lib.qg_activations_tiled_bytes(M, K), dtype=torch.uint8, device=a.device)
    with torch.cuda.device(a.device):
        _lib.check(lib.qg_tile_activations(_ptr(a), _ptr(out), M, K, _stream(a.device)), "tile_activations")
    return out


def gemm_w4a8_tiled_act(activation_tiled: torch.Tensor, weight_tiled: torch.Tensor, M: int, N: int, K: int,
                        wtype: int = Q4_0, out: torch.Tensor | None = None) -> torch.Tensor:
    """C [M, N] = gemm_w4a8_tiled's product with the activations in the tiled layout too
    (qg_gemm_w4a8_tiled_act)."""
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    lib = _lib.load()
    _require(weight_tiled.is_cuda, "weight_tiled must be a CUDA tensor")
    _check_layout(activation_tiled, "activation_tiled", lib.qg_activations_tiled_bytes(M, K), weight_tiled.device)
    _check_layout(weight_tiled, "weight_tiled", lib.qg_tile_weights_bytes(N, K, wtype), weight_tiled.device)
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=weight_tiled.device)
    _require(out.is_cuda and out.dtype == torch.float32 and out.shape == (M, N) and out.is_contiguous(),
             "out must be a contiguous CUDA float32 [M, N] tensor")
    with torch.cuda.device(weight_tiled.device):
        _lib.check(lib.qg_gemm_w4a8_tiled_act(_ptr(activation_tiled), _ptr(weight_tiled), _ptr(out), M, N, K, wtype,
                                              _stream(weight_tiled.device)), "gemm_w4a8_tiled_act")
    return out


def quantize_q8_1_padded(x: torch.Tensor) -> torch.Tensor:
    """x float32 [M, K] -> uint8 [M, K'/32, 36] (qg_quantize_q8_1_padded): each row's blocks as
    quantize_q8_1, then zero blocks up to K'/32 = round_up(K/32, 8) — the activation side of the
    repack_weights layout."""
    _require(x.is_cuda and x.dtype == torch.float32 and x.dim() == 2, "x must be a 2-D CUDA float32 tensor")
    M, K = x.shape
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    nbp = (K // 32 + 7) // 8 * 8
    x = x.contiguous()
    out = torch.empty((M, nbp, 36), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        _lib.check(_lib.load().qg_quantize_q8_1_padded(_ptr(x), _ptr(out), M, K, _stream(x.device)), "quantize_q8_1_padded")
    return out


def gemm_w4a8_padded(activation_padded: torch.Tensor, weight_packed: torch.Tensor, M: int, N: int, K: int,
                     wtype: int = Q4_0) -> torch.Tensor:
    """C [M, N] from quantize_q8_1_padded activations and repack_weights weights, one launch
    (qg_gemm_w4a8_padded; K is the logical K)."""
    _require(weight_packed.is_cuda, "weight_packed must be a CUDA tensor")
    nbp = (K // 32 + 7) // 8 * 8
    _check_layout(activation_padded.contiguous(), "activation_padded", M * nbp * 36, weight_packed.device)
    _check_layout(weight_packed, "weight_packed", N * nbp * BLOCK_BYTES[wtype], weight_packed.device)
    out = torch.empty((M, N), dtype=torch.float32, device=weight_packed.device)
    with torch.cuda.device(weight_packed.device):
        _lib.check(_lib.load().qg_gemm_w4a8_padded(_ptr(activation_padded.contiguous()), _ptr(weight_packed), _ptr(out),
                                                   M, N, K, wtype, _stream(weight_packed.device)), "gemm_w4a8_padded")
    return out


def _gemm_weight_major(sym: str, wtype: int, weight_q, activation_q, M, N, K):
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _check_blocks(weight_q, "Weight", M, K, BLOCK_BYTES[wtype])
    _check_blocks(activation_q, "Activation", N, K, 36)
    w = weight_q.contiguous()
    a = activation_q.contiguous()
    out = torch.empty((M, N), dtype=torch.float32, device=w.device)
    with torch.cuda.device(w.device):
        _lib.check(getattr(_lib.load(), sym)(_ptr(w), _ptr(a), _ptr(out), M, N, K, _stream(w.device)), sym)
    return out


def gemm_q4_0_q8_1(weight_q: torch.Tensor, activation_q: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """Quantized GEMM C[M,N] = W[M,K] @ A[N,K]^T (weight-major: M = weight rows, N = tokens).

    weight_q: uint8 [M, K//32, 18]; activation_q: uint8 [N, K//32, 36]; returns f32 [M, N]."""
    return _gemm_weight_major("qg_gemm_q4_0_q8_1", Q4_0, weight_q, activation_q, M, N, K)


def gemm_q4_1_q8_1(weight_q, activation_q, M: int, N: int, K: int) -> torch.Tensor:
    return _gemm_weight_major("qg_gemm_q4_1_q8_1", Q4_1, weight_q, activation_q, M, N, K)


def gemm_q5_0_q8_1(weight_q, activation_q, M: int, N: int, K: int) -> torch.Tensor:
    return _gemm_weight_major("qg_gemm_q5_0_q8_1", Q5_0, weight_q, activation_q, M, N, K)


def gemm_q5_1_q8_1(weight_q, activation_q, M: int, N: int, K: int) -> torch.Tensor:
    return _gemm_weight_major("qg_gemm_q5_1_q8_1", Q5_1, weight_q, activation_q, M, N, K)


# ---------------------------------------------------------------------------- fused activation quantization
def _workspace(rows: int, K: int, dev: torch.device):
    nbytes = _lib.load().qg_gemm_w4a8_f32_workspace_size(rows, K)
    return torch.empty((nbytes,), dtype=torch.uint8, device=dev)


def gemm_w4a8_f32(x: torch.Tensor, weight_q: torch.Tensor, wtype: int = Q4_0, workspace: bool = True,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """Activation-major C[M, N] = Q8_1(x)[M, K] . B_w[N, K]^T for FP32 x [M, K]: identical to
    ``gemm_w4a8(quantize_q8_1(x), weight_q, ...)``. M <= 4: one launch, x quantized in the GEMV
    prologue. Larger M (or a K the GEMV does not take): through a Q8_1 workspace (``workspace=True``, from torch's caching
    allocator) or the fused GEMV per 8-row chunk (``workspace=False``)."""
    _require(x.is_cuda, "Input must be a CUDA tensor")
    _require(x.dtype == torch.float32 and x.dim() == 2, "x must be float32 [M, K]")
    M, K = x.shape
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _require(wtype in WEIGHT_TYPES, f"unsupported weight type {wtype}")
    N = weight_q.numel() // ((K // 32) * BLOCK_BYTES[wtype]) if K else 0
    _check_blocks(weight_q, "Weight", N, K, BLOCK_BYTES[wtype])
    x = x.contiguous()
    w = weight_q.contiguous()
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=w.device)
    else:
        _require(out.is_contiguous() and out.dtype == torch.float32 and out.numel() == M * N, "bad out tensor")
    ws = _workspace(M, K, w.device) if workspace else None
    with torch.cuda.device(w.device):
        _lib.check(_lib.load().qg_gemm_w4a8_f32(_ptr(x), _ptr(w), _ptr(out), M, N, K, wtype,
                                                _ptr(ws) if ws is not None else None,
                                                ws.numel() if ws is not None else 0, _stream(w.device)),
                   "gemm_w4a8_f32")
    return out


def gemm_q4_0_fp16_fused(weight_q: torch.Tensor, fp16_activation: torch.Tensor, M: int, N: int, K: int,
                         workspace: bool = True) -> torch.Tensor:
    """Weight-major out[M, N] = W_q4_0[M, K] . Q8_1(act[N, K])^T with the FP16 activations quantized
    inside the product (kernels/gemm/gemm_fused.cuh:311-338 gemm_q4_0_fp16_fused; quantizer
    semantics of gemm_fused.cuh:76-143)."""
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _check_blocks(weight_q, "Weight", M, K, 18)
    _require(fp16_activation.is_cuda and fp16_activation.dtype == torch.float16, "Activation must be CUDA float16")
    _require(fp16_activation.numel() == N * K, f"Activation shape mismatch: expected {N * K} elements")
    w = weight_q.contiguous()
    a = fp16_activation.contiguous()
    out = torch.empty((M, N), dtype=torch.float32, device=w.device)
    ws = _workspace(N, K, w.device) if workspace else None
    with torch.cuda.device(w.device):
        _lib.check(_lib.load().qg_gemm_q4_0_fp16_fused_ws(_ptr(w), _ptr(a), _ptr(out), M, N, K,
                                                          _ptr(ws) if ws is not None else None,
                                                          ws.numel() if ws is not None else 0, _stream(w.device)),
                   "gemm_q4_0_fp16_fused")
    return out


def quantize_q8_1_f16_fused(x: torch.Tensor) -> torch.Tensor:
    """FP16 [..., K] -> Q8_1 uint8 [..., K/32, 36] with the fused kernel's quantizer semantics."""
    _require(x.is_cuda and x.dtype == torch.float16, "Input must be a CUDA float16 tensor")
    K = x.size(-1)
    _require(K % 32 == 0, f"Last dimension must be divisible by 32, got {K}")
    x = x.contiguous()
    out = torch.empty(tuple(x.shape[:-1]) + (K // 32, 36), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        _lib.check(_lib.load().qg_quantize_q8_1_f16_fused(_ptr(x), _ptr(out), x.numel(), _stream(x.device)),
                   "quantize_q8_1_f16_fused")
    return out


def gemm_q8_0_q8_1(weight_q, activation_q, M: int, N: int, K: int) -> torch.Tensor:
    """W8A8, weight-major (kernels/gemm/gemm_quant_formats.cuh:415-428)."""
    return _gemm_weight_major("qg_gemm_q8_0_q8_1", Q8_0, weight_q, activation_q, M, N, K)


def gemm_w8a8(activation_q: torch.Tensor, weight_q: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """W8A8, activation-major C[M, N] = A_q8_1 . B_q8_0^T (include/gemm_reference.h:233-267)."""
    return gemm_w4a8(activation_q, weight_q, M, N, K, wtype=Q8_0)


# ---------------------------------------------------------------------------- W4A16 / W8A16
def _gemm_w16(sym: str, wtype: int, activation: torch.Tensor, weight_q: torch.Tensor, M: int, N: int, K: int):
    _require(K % 32 == 0, f"K must be divisible by 32, got {K}")
    _require(activation.is_cuda and activation.dtype == torch.float32, "Activation must be a CUDA float32 tensor")
    _require(activation.numel() == M * K, f"Activation shape mismatch: expected {M * K} elements")
    _check_blocks(weight_q, "Weight", N, K, BLOCK_BYTES[wtype])
    a = activation.contiguous()
    w = weight_q.contiguous()
    out = torch.empty((M, N), dtype=torch.float32, device=w.device)
    with torch.cuda.device(w.device):
        _lib.check(getattr(_lib.load(), sym)(_ptr(a), _ptr(w), _ptr(out), M, N, K, _stream(w.device)), sym)
    return out


def gemm_w4a16(activation: torch.Tensor, weight_q: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """C[M, N] = A_f32[M, K] . dequant(W_q4_0[N, K])^T (include/gemm_reference.h:73-112)."""
    return _gemm_w16("qg_gemm_w4a16", Q4_0, activation, weight_q, M, N, K)


def gemm_w8a16(activation: torch.Tensor, weight_q: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """C[M, N] = A_f32[M, K] . dequant(W_q8_0[N, K])^T (include/gemm_cuda_naive.cuh:276-283)."""
    return _gemm_w16("qg_gemm_w8a16", Q8_0, activation, weight_q, M, N, K)


def gemm_q4_0_fp32(weight_q: torch.Tensor, activation: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """python/quant_gemm/csrc/gemm_ops.cu:431-466: weight_q [N, K/32, 18], activation [M, K] -> [M, N]."""
    return _gemm_w16("qg_gemm_w4a16", Q4_0, activation, weight_q, M, N, K)


def debug_sumi(activation_q: torch.Tensor, weight_q: torch.Tensor, M: int, N: int, K: int,
               wtype: int = Q4_0, algo: int = ALGO_AUTO) -> torch.Tensor:
    """Per-block int32 dots [M, N, K/32] through the same decode path as ``algo``."""
    _check_blocks(activation_q, "Activation", M, K, 36)
    _check_blocks(weight_q, "Weight", N, K, BLOCK_BYTES[wtype])
    out = torch.empty((M, N, K // 32), dtype=torch.int32, device=weight_q.device)
    with torch.cuda.device(weight_q.device):
        _lib.check(_lib.load().qg_debug_sumi(_ptr(activation_q.contiguous()), _ptr(weight_q.contiguous()),
                                             _ptr(out), M, N, K, wtype, algo, _stream(weight_q.device)),
                   "debug_sumi")
    return out


def debug_config(M: int, N: int, K: int, wtype: int = Q4_0, algo: int = ALGO_AUTO, sumi: bool = False) -> str:
    """The kernel instantiation ``gemm_w4a8`` (or ``debug_sumi`` with sumi=True) launches for this
    shape on aligned buffers (family, template parameters, grid); nothing is launched."""
    buf = ctypes.create_string_buffer(256)
    _lib.check(_lib.load().qg_debug_config(M, N, K, wtype, algo, int(sumi), buf, 256), "debug_config")
    return buf.value.decode()


def debug_sumi_tiled(activation_q: torch.Tensor, weight_tiled: torch.Tensor, M: int, N: int, K: int,
                     wtype: int = Q4_0) -> torch.Tensor:
    """Per-block int32 dots [M, N, K/32] from the instantiation gemm_w4a8_tiled launches."""
    _check_blocks(activation_q, "Activation", M, K, 36)
    lib = _lib.load()
    _check_layout(weight_tiled, "weight_tiled", lib.qg_tile_weights_bytes(N, K, wtype), activation_q.device)
    out = torch.empty((M, N, K // 32), dtype=torch.int32, device=weight_tiled.device)
    with torch.cuda.device(weight_tiled.device):
        _lib.check(lib.qg_debug_sumi_tiled(_ptr(activation_q.contiguous()), _ptr(weight_tiled), _ptr(out), M, N, K, wtype,
                                           _stream(weight_tiled.device)), "debug_sumi_tiled")
    return out


def debug_sumi_tiled_act(activation_tiled: torch.Tensor, weight_tiled: torch.Tensor, M: int, N: int, K: int,
                         wtype: int = Q4_0) -> torch.Tensor:
    """Per-block int32 dots [M, N, K/32] from the instantiation gemm_w4a8_tiled_act launches."""
    lib = _lib.load()
    _require(weight_tiled.is_cuda, "weight_tiled must be a CUDA tensor")
    _check_layout(activation_tiled, "activation_tiled", lib.qg_activations_tiled_bytes(M, K), weight_tiled.device)
    _check_layout(weight_tiled, "weight_tiled", lib.qg_tile_weights_bytes(N, K, wtype), weight_tiled.device)
    out = torch.empty((M, N, K // 32), dtype=torch.int32, device=weight_tiled.device)
    with torch.cuda.device(weight_tiled.device):
        _lib.check(lib.qg_debug_sumi_tiled_act(_ptr(activation_tiled), _ptr(weight_tiled), _ptr(out), M, N, K, wtype,
                                               _stream(weight_tiled.device)), "debug_sumi_tiled_act")
    return out


def debug_config_tiled_act(M: int, N: int, K: int, wtype: int = Q4_0, sumi: bool = False) -> str:
    """The instantiation gemm_w4a8_tiled_act (or debug_sumi_tiled_act) launches; nothing runs."""
    buf = ctypes.create_string_buffer(256)
    _lib.check(_lib.load().qg_debug_config_tiled_act(M, N, K, wtype, int(sumi), buf, 256), "debug_config_tiled_act")
    return buf.value.decode()


def debug_config_tiled(M: int, N: int, K: int, wtype: int = Q4_0, sumi: bool = False) -> str:
    """The instantiation gemm_w4a8_tiled (or debug_sumi_tiled with sumi=True) launches; nothing runs."""
    buf = ctypes.create_string_buffer(256)
    _lib.check(_lib.load().qg_debug_config_tiled(M, N, K, wtype, int(sumi), buf, 256), "debug_config_tiled")
    return buf.value.decode()


def select_algo(M: int, N: int, K: int, wtype: int = Q4_0) -> int:
    return _lib.load().qg_select_algo(M, N, K, wtype)


def version() -> str:
    return _lib.load().qg_version().decode()


_lib.load()  # fail loudly at import if the HIP library is absent

__all__ = [
    "quantize_q4_0", "quantize_q8_1", "gemm_q4_0_q8_1", "dequantize_q4_0",
    "QK4_0", "QK8_1", "BLOCK_Q4_0_BYTES", "BLOCK_Q8_1_BYTES",
    "quantize", "dequantize", "gemm_w4a8", "gemm_q4_1_q8_1", "gemm_q5_0_q8_1", "gemm_q5_1_q8_1",
    "gemm_w4a8_batched", "debug_sumi", "debug_config", "select_algo", "version",
    "gemm_w4a8_f32", "gemm_q4_0_fp16_fused", "quantize_q8_1_f16_fused", "gemm_w8a8", "gemm_q8_0_q8_1",
    "gemm_w4a16", "gemm_w8a16", "gemm_q4_0_fp32",
    "tile_weights", "gemm_w4a8_tiled", "debug_sumi_tiled", "debug_config_tiled",
    "quantize_q8_1_tiled", "tile_activations", "gemm_w4a8_tiled_act", "debug_sumi_tiled_act", "debug_config_tiled_act",
    "Q4_0", "Q4_1", "Q5_0", "Q5_1", "Q8_0", "Q8_1",
]
