"""ggml-facing adapter (include/llama_adapter.h) and GGUF weight files, over the C-ABI.

    with GGUFFile("model.gguf") as f:
        w = f.to_device("blk.0.attn_q.weight")           # uint8 [N, K/32, 18] for Q4_0, on cuda
        out = gemm_w4a8_from_ggml(act_view, f.view("blk.0.attn_q.weight", w), out_view)

``TensorView`` mirrors ``qg_tensor_view`` (ne[0] = K contiguous, ne[1] = rows, nb[] byte strides),
the part of ggml_tensor the reference adapter reads (llama_adapter.h:49-61). The GGUF reader maps
the file read-only in the library (qg_gguf.hip); nothing in the file is executed.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib

F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1 = 0, 1, 2, 3, 6, 7, 8, 9
_BB = {Q4_0: 18, Q4_1: 20, Q5_0: 22, Q5_1: 24, Q8_0: 34, Q8_1: 36}


class TensorView(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("type", ctypes.c_int), ("ne", ctypes.c_int64 * 4),
                ("nb", ctypes.c_size_t * 4)]


def view_of(t: torch.Tensor, qtype: int, k: int) -> TensorView:
    """ggml-ordered view of a dense row-major tensor holding rows of K elements of ``qtype``."""
    row = k * 4 if qtype == F32 else k * 2 if qtype == F16 else (k // 32) * _BB[qtype]
    rows = t.numel() * t.element_size() // row
    v = TensorView()
    v.data, v.type = t.data_ptr(), qtype
    v.ne[:] = [k, rows, 1, 1]
    v.nb[:] = [4 if qtype == F32 else 2 if qtype == F16 else _BB[qtype], row, row * rows, row * rows]
    return v


def _call(sym: str, act: TensorView, w: TensorView, out: TensorView, kernel_type: str | None) -> None:
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    kt = kernel_type.encode() if kernel_type else None
    _lib.check(getattr(_lib.load(), sym)(ctypes.byref(act), ctypes.byref(w), ctypes.byref(out), kt, st), sym)


def gemm_w4a8_from_ggml(act: TensorView, w: TensorView, out: TensorView, kernel_type: str | None = "naive") -> None:
    """include/llama_adapter.h:63-76: Q8_1 activation [K, M] x quantized weights [K, N] -> F32 [N, M]."""
    _call("qg_gemm_w4a8_from_view", act, w, out, kernel_type)


def gemm_w4a16_from_ggml(act: TensorView, w: TensorView, out: TensorView, kernel_type: str | None = "naive") -> None:
    """include/llama_adapter.h:78-90: F32 activation x Q4_0 / Q8_0 weights -> F32."""
    _call("qg_gemm_w4a16_from_view", act, w, out, kernel_type)


def gemm_fp32_from_ggml(act: TensorView, w: TensorView, out: TensorView, kernel_type: str | None = "naive") -> None:
    """include/llama_adapter.h:92-103: all F32."""
    _call("qg_gemm_fp32_from_view", act, w, out, kernel_type)


def validate_tensor_types(act: TensorView, w: TensorView, out: TensorView, ea: int, ew: int, eo: int) -> bool:
    """include/llama_adapter.h:110-117."""
    return bool(_lib.load().qg_validate_view_types(ctypes.byref(act), ctypes.byref(w), ctypes.byref(out), ea, ew, eo))


class GGUFTensor:
    def __init__(self, index: int, name: str, qtype: int, ne: list[int], nbytes: int):
        self.index, self.name, self.type, self.ne, self.nbytes = index, name, qtype, ne, nbytes

    @property
    def shape(self) -> tuple:
        """torch-order shape of the data: [.., rows, K/32, block bytes] (quantized) or [.., rows, K]."""
        dims = [d for d in reversed(self.ne)]
        while len(dims) > 1 and dims[0] == 1:
            dims = dims[1:]
        if self.type in _BB:
            return tuple(dims[:-1]) + (dims[-1] // 32, _BB[self.type])
        return tuple(dims)

    def __repr__(self) -> str:
        return f"GGUFTensor({self.name!r}, type={self.type}, ne={self.ne}, nbytes={self.nbytes})"


class GGUFFile:
    """Read-only GGUF v2/v3 file (metadata, tensor directory, tensor bytes)."""

    def __init__(self, path: str | os.PathLike):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self._lib.qg_gguf_open(os.fsencode(path), ctypes.byref(h)), f"gguf open {path}")
        self._h = h
        self.version = self._lib.qg_gguf_version(h)
        self.alignment = self._lib.qg_gguf_alignment(h)
        self.tensors: dict[str, GGUFTensor] = {}
        for i in range(self._lib.qg_gguf_tensor_count(h)):
            name, t, nd = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_int()
            ne, nb = (ctypes.c_int64 * 4)(), ctypes.c_uint64()
            _lib.check(self._lib.qg_gguf_tensor_info(h, i, ctypes.byref(name), ctypes.byref(t), ctypes.byref(nd), ne,
                                                     ctypes.byref(nb)), "gguf tensor info")
            n = name.value.decode()
            self.tensors[n] = GGUFTensor(i, n, t.value, list(ne)[:nd.value], nb.value)
        self.metadata: dict[str, object] = {}
        for i in range(self._lib.qg_gguf_kv_count(h)):
            key, t, cnt, et = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_uint64(), ctypes.c_int()
            _lib.check(self._lib.qg_gguf_kv_info(h, i, ctypes.byref(key), ctypes.byref(t), ctypes.byref(cnt),
                                                 ctypes.byref(et)), "gguf kv info")
            self.metadata[key.value.decode()] = self._value(i, t.value, cnt.value, et.value)

    def _value(self, i: int, t: int, count: int, elem: int):
        if t == 8:
            p, n = ctypes.c_void_p(), ctypes.c_uint64()
            _lib.check(self._lib.qg_gguf_kv_string(self._h, i, ctypes.byref(p), ctypes.byref(n)), "gguf kv")
            return ctypes.string_at(p, n.value).decode("utf-8", "replace")
        if t == 9:
            return ("array", elem, count)
        if t in (6, 12):
            v = ctypes.c_double()
            _lib.check(self._lib.qg_gguf_kv_float(self._h, i, ctypes.byref(v)), "gguf kv")
            return v.value
        v = ctypes.c_int64()
        _lib.check(self._lib.qg_gguf_kv_int(self._h, i, ctypes.byref(v)), "gguf kv")
        return bool(v.value) if t == 7 else v.value

    def close(self) -> None:
        if self._h:
            self._lib.qg_gguf_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _t(self, name: str) -> GGUFTensor:
        if name not in self.tensors:
            raise KeyError(name)
        t = self.tensors[name]
        if t.nbytes == 0:
            raise RuntimeError(f"{name}: tensor type {t.type} not supported")
        return t

    def host_bytes(self, name: str) -> np.ndarray:
        """A copy of the tensor's bytes (uint8, torch-order shape)."""
        t = self._t(name)
        p = self._lib.qg_gguf_tensor_data(self._h, t.index)
        raw = np.frombuffer(ctypes.string_at(p, t.nbytes), np.uint8)
        if t.type in _BB:
            return raw.reshape(t.shape)
        return raw.view(np.float32 if t.type == F32 else np.float16).reshape(t.shape)

    def to_device(self, name: str, device: str | torch.device = "cuda") -> torch.Tensor:
        """Upload the tensor (uint8 [.., rows, K/32, bb] for quantized types, float32/float16 otherwise)."""
        t = self._t(name)
        dtype = torch.uint8 if t.type in _BB else torch.float32 if t.type == F32 else torch.float16
        out = torch.empty(t.shape, dtype=dtype, device=device)
        with torch.cuda.device(out.device):
            st = ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)
            _lib.check(self._lib.qg_gguf_upload_tensor(self._h, t.index, ctypes.c_void_p(out.data_ptr()),
                                                       out.numel() * out.element_size(), st), "gguf upload")
        return out

    def view(self, name: str, device_tensor: torch.Tensor) -> TensorView:
        """The ggml-ordered view of ``name``'s bytes held in ``device_tensor``."""
        t = self._t(name)
        v = TensorView()
        _lib.check(self._lib.qg_gguf_tensor_view(self._h, t.index, ctypes.c_void_p(device_tensor.data_ptr()),
                                                 ctypes.byref(v)), "gguf view")
        return v
