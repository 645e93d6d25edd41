"""W4A16 / W8A16 (FP32 activations x Q4_0 / Q8_0 weights), GPU parity through the C-ABI.

Bar: |C_gpu - C_oracle| <= 2 (K + 2) 2^-24 sum_k |a_k w_k| (oracle.w16_tol) — the fp32
summation-order bound; the reference's own Python definition outputs (tests/golden/w4a16_*.npz)
are met within the same bound; NMSE vs FP32 within the W4A8 bound.
"""
import ctypes
import glob
import os

import numpy as np
import pytest

from test_gpu_parity import GOLD, dev, host

pytestmark = pytest.mark.gpu


def check(O, c, a, bq, t, ref=None):
    ref = (O.gemm_w4a16(a, bq) if t == O.Q4_0 else O.gemm_w8a16(a, bq)) if ref is None else ref
    tol = O.w16_tol(a, bq, t)
    err = np.abs(c.astype(np.float64) - ref)
    assert (err <= tol).all(), f"max err {err.max()}"


@pytest.mark.parametrize("t", [2, 8])
@pytest.mark.parametrize("m,n,k", [(1, 300, 4096), (2, 64, 4096), (3, 130, 2048), (4, 33, 4096), (5, 40, 1024),
                                   (8, 100, 4096), (9, 64, 2048), (33, 50, 1024), (1, 70, 14336), (2, 17, 192),
                                   (3, 9, 96), (1, 5, 32)])
def test_w16_matches_oracle(O, qg, t, m, n, k):
    a, b = O.fill_uniform_step4(m, n, k, seed=m + n)
    bq = O.quantize(b, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    c = host(fn(dev(a), dev(bq), m, n, k))
    check(O, c, a, bq, t)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "w4a16_*.npz"))), ids=os.path.basename)
def test_w4a16_golden(O, qg, path):
    """The reference definition's outputs, with its interleaved dequant order undone on the
    activations (see tests/test_oracle.py::test_golden_w4a16)."""
    g = np.load(path)
    m, n, k = (int(g[x]) for x in ("m", "n", "k"))
    blk = g["a"].reshape(m, k // 32, 32)
    a = np.ascontiguousarray(np.concatenate([blk[..., 0::2], blk[..., 1::2]], axis=-1).reshape(m, k))
    c = host(qg.gemm_q4_0_fp32(dev(g["b_q"]), dev(a), m, n, k))
    check(O, c, a, g["b_q"], 2, ref=g["c_ref"].astype(np.float64))


def test_w4a16_full_size_nmse(O, qg):
    a, b = O.fill_uniform_step4(1, 4096, 4096)
    bq = O.quantize(b, 2)
    c = host(qg.gemm_w4a16(dev(a), dev(bq), 1, 4096, 4096))
    check(O, c, a, bq, 2)
    assert O.nmse(c, O.gemm_fp32(a, b)) <= 5e-3


def test_w4a16_unaligned_activation_generic_path(O, qg):
    import torch
    m, n, k = 2, 24, 1024
    a, b = O.fill_uniform_step4(m, n, k)
    bq = O.quantize(b, 2)
    raw = torch.zeros(a.size + 1, dtype=torch.float32, device="cuda")
    raw[1:] = dev(a.ravel())
    x = raw[1:]
    assert x.data_ptr() % 16 != 0
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")
    lib = qg._lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p
    assert lib.qg_gemm_w4a16(P(x.data_ptr()), P(dev(bq).data_ptr()), P(c.data_ptr()), m, n, k, st) == 0
    check(O, host(c), a, bq, 2)
