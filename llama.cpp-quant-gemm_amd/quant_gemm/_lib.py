"""Loader for the in-tree HIP library ``libqg_hip.so`` (C-ABI: include/qg/qg.h).

There is no fallback: if the library is missing or does not load, importing ``quant_gemm``
raises. ``torch`` is imported first so the library binds to the HIP runtime torch already loaded
(both carry SONAME libamdhip64.so.7) — one runtime per process, torch's streams valid in ours.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libqg_hip.so")
CSRC = os.path.join(os.path.dirname(HERE), "csrc")

QG_OK = 0
STATUS = {0: "ok", -1: "invalid argument", -2: "K must be a positive multiple of 32",
          -3: "unsupported type or algorithm for this shape", -4: "pointer misaligned for the block format",
          -5: "HIP launch error"}

# exported symbols and their signatures (kept in sync with include/qg/qg.h; tests check both ways)
P, I, I64, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
SIGNATURES = {
    "qg_gemm_w4a8": ([P, P, P, I, I, I, I, P], I),
    "qg_gemm_w4a8_ex": ([P, P, P, I, I, I, I, I, P], I),
    "qg_gemm_q4_0_q8_1_w4a8": ([P, P, P, I, I, I, P], I),
    "qg_gemm_w4a8_ldc": ([P, P, P, I, I, I, I64, I, I, P], I),
    "qg_debug_config": ([I, I, I, I, I, I, ctypes.c_char_p, SZ], I),
    "qg_gemm_w4a8_strided_batched": ([P, I64, P, I64, P, I64, I, I, I, I, I, P], I),
    "qg_gemm_w4a8_grouped": ([P, I, I, I, I, P], I),
    "qg_gemm_w4a8_workspace_size": ([I, I, I, I], SZ),
    "qg_gemm_w4a8_ws": ([P, P, P, I, I, I, I, P, SZ, P], I),
    "qg_repack_weights_bytes": ([I, I, I], SZ),
    "qg_repack_weights": ([P, P, I, I, I, P], I),
    "qg_gemm_w4a8_prepacked_workspace_size": ([I, I], SZ),
    "qg_gemm_w4a8_prepacked": ([P, P, P, I, I, I, I, P, SZ, P], I),
    "qg_quantize_q8_1_padded": ([P, P, I, I, P], I),
    "qg_tile_weights_bytes": ([I, I, I], SZ),
    "qg_tile_weights": ([P, P, I, I, I, P], I),
    "qg_gemm_w4a8_tiled": ([P, P, P, I, I, I, I, P], I),
    "qg_gemm_w4a8_tiled_ldc": ([P, P, P, I, I, I, I64, I, P], I),
    "qg_debug_sumi_tiled": ([P, P, P, I, I, I, I, P], I),
    "qg_debug_config_tiled": ([I, I, I, I, I, ctypes.c_char_p, SZ], I),
    "qg_activations_tiled_bytes": ([I, I], SZ),
    "qg_quantize_q8_1_tiled": ([P, P, I, I, P], I),
    "qg_tile_activations": ([P, P, I, I, P], I),
    "qg_gemm_w4a8_tiled_act": ([P, P, P, I, I, I, I, P], I),
    "qg_gemm_w4a8_tiled_act_ldc": ([P, P, P, I, I, I, I64, I, P], I),
    "qg_debug_sumi_tiled_act": ([P, P, P, I, I, I, I, P], I),
    "qg_debug_config_tiled_act": ([I, I, I, I, I, ctypes.c_char_p, SZ], I),
    "qg_gemm_w4a8_padded": ([P, P, P, I, I, I, I, P], I),
    "qg_gemm_q4_0_q8_1": ([P, P, P, I, I, I, P], I),
    "qg_gemm_q4_1_q8_1": ([P, P, P, I, I, I, P], I),
    "qg_gemm_q5_0_q8_1": ([P, P, P, I, I, I, P], I),
    "qg_gemm_q5_1_q8_1": ([P, P, P, I, I, I, P], I),
    "qg_gemm_q8_0_q8_1": ([P, P, P, I, I, I, P], I),
    "qg_gemm_w8a8": ([P, P, P, I, I, I, P], I),
    "qg_gemm_w4a8_f32_workspace_size": ([I, I], SZ),
    "qg_gemm_w4a8_f32": ([P, P, P, I, I, I, I, P, SZ, P], I),
    "qg_gemm_q4_0_fp16_fused": ([P, P, P, I, I, I, P], I),
    "qg_gemm_q4_0_fp16_fused_ws": ([P, P, P, I, I, I, P, SZ, P], I),
    "qg_quantize_q8_1_f16_fused": ([P, P, I64, P], I),
    "qg_gemm_w4a16": ([P, P, P, I, I, I, P], I),
    "qg_gemm_w8a16": ([P, P, P, I, I, I, P], I),
    "qg_gemm_q4_0_fp32": ([P, P, P, I, I, I, P], I),
    "qg_gemm_w16_workspace_size": ([I, I, I], SZ),
    "qg_gemm_w4a16_ws": ([P, P, P, I, I, I, P, SZ, P], I),
    "qg_gemm_w8a16_ws": ([P, P, P, I, I, I, P, SZ, P], I),
    "qg_release_workspaces": ([], None),
    "qg_quantize_q8_1": ([P, P, I64, P], I),
    "qg_quantize_q4_0": ([P, P, I64, P], I),
    "qg_quantize_q8_1_definition": ([P, P, I64, P], I),
    "qg_quantize_q4_0_definition": ([P, P, I64, P], I),
    "qg_quantize": ([I, I, P, P, I64, P], I),
    "qg_dequantize": ([I, P, P, I64, P], I),
    "qg_dequantize_q4_0": ([P, P, I64, P], I),
    "qg_debug_sumi": ([P, P, P, I, I, I, I, I, P], I),
    "qg_gemm_w4a8_from_view": ([P, P, P, ctypes.c_char_p, P], I),
    "qg_gemm_w4a16_from_view": ([P, P, P, ctypes.c_char_p, P], I),
    "qg_gemm_fp32_from_view": ([P, P, P, ctypes.c_char_p, P], I),
    "qg_validate_view_types": ([P, P, P, I, I, I], I),
    "qg_gemm_fp32": ([P, P, P, I, I, I, P], I),
    "qg_gguf_open": ([ctypes.c_char_p, ctypes.POINTER(P)], I),
    "qg_gguf_close": ([P], None),
    "qg_gguf_version": ([P], I),
    "qg_gguf_alignment": ([P], I64),
    "qg_gguf_tensor_count": ([P], I64),
    "qg_gguf_find_tensor": ([P, ctypes.c_char_p], I64),
    "qg_gguf_tensor_info": ([P, I64, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(I), ctypes.POINTER(I),
                             ctypes.POINTER(I64), ctypes.POINTER(ctypes.c_uint64)], I),
    "qg_gguf_tensor_data": ([P, I64], P),
    "qg_gguf_upload_tensor": ([P, I64, P, SZ, P], I),
    "qg_gguf_tensor_view": ([P, I64, P, P], I),
    "qg_gguf_kv_count": ([P], I64),
    "qg_gguf_find_kv": ([P, ctypes.c_char_p], I64),
    "qg_gguf_kv_info": ([P, I64, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(I), ctypes.POINTER(ctypes.c_uint64),
                         ctypes.POINTER(I)], I),
    "qg_gguf_kv_int": ([P, I64, ctypes.POINTER(I64)], I),
    "qg_gguf_kv_float": ([P, I64, ctypes.POINTER(ctypes.c_double)], I),
    "qg_gguf_kv_string": ([P, I64, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64)], I),
    "qg_status_string": ([I], ctypes.c_char_p),
    "qg_last_hip_error": ([], I),
    "qg_select_algo": ([I, I, I, I], I),
    "qg_block_bytes": ([I], I),
    "qg_version": ([], ctypes.c_char_p),
}

_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"quant_gemm: HIP library not built ({LIB_PATH}); run `make -C {CSRC}` "
                              "or __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lib
    return _lib


def check(status: int, what: str) -> None:
    if status != QG_OK:
        extra = ""
        if status == -5:
            extra = f" (hipError {load().qg_last_hip_error()})"
        raise RuntimeError(f"{what}: {STATUS.get(status, status)}{extra}")
