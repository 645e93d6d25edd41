"""The W4A16 / W8A16 small-M prefill without split-K (w16d_kernel, round 4): 8 < M <= 32,
K % 256 == 0, K <= 8192, one dispatch round. Each workgroup owns all of K, so it takes no workspace: a
caller workspace filled with a sentinel is left untouched (the dispatch check), outputs are within the
fp32 K-term bound of the oracle (oracle.w16_tol; include/gemm_reference.h:73-112), repeated launches are
bit-identical (fixed-order wave sum), and the two-part bf16 split stays within 2^-16 + (K + 2) 2^-24 of
sum_k |a_k w_k| against the exact float64 product. Shapes: 16- and 32-row tiles, ragged N and M, fewer
K stages than waves (K = 256), the largest K it takes (8192).
"""
import ctypes

import numpy as np
import pytest

from test_gpu_parity import dev, host
from test_gpu_w4a16 import check

pytestmark = pytest.mark.gpu

SHAPES = [(32, 4096, 4096), (16, 4096, 4096), (16, 4100, 2048), (9, 1000, 256), (31, 2050, 1024), (20, 33, 8192),
          (17, 300, 1024), (32, 512, 4096)]


def run_ws(qg, t, a_d, b_d, m, n, k, ws, nbytes):
    import torch
    lib = qg._lib.load()
    P = ctypes.c_void_p
    sym = lib.qg_gemm_w4a16_ws if t == 2 else lib.qg_gemm_w8a16_ws
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")
    st = P(torch.cuda.current_stream().cuda_stream)
    assert sym(P(a_d.data_ptr()), P(b_d.data_ptr()), P(c.data_ptr()), m, n, k, P(ws.data_ptr()), nbytes, st) == 0
    return c


@pytest.mark.parametrize("t", [2, 8])
@pytest.mark.parametrize("m,n,k", SHAPES)
def test_w16d_parity_no_workspace(O, qg, t, m, n, k):
    import torch
    a, b = O.fill_uniform_step4(m, n, k, seed=m * 3 + n)
    bq = O.quantize(b, t)
    a_d, b_d = dev(a), dev(bq)
    lib = qg._lib.load()
    need = max(int(lib.qg_gemm_w16_workspace_size(m, n, k)), 4096)
    ws = torch.full((need // 4,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    c1 = host(run_ws(qg, t, a_d, b_d, m, n, k, ws, need))
    assert bool((ws == 0x5A5A5A5A).all()), "the no-split-K prefill must not touch a workspace"
    check(O, c1, a, bq, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    assert np.array_equal(c1, host(fn(a_d, b_d, m, n, k)))  # library path, same kernel, bit for bit


@pytest.mark.parametrize("t", [2, 8])
@pytest.mark.parametrize("m,n,k", [(32, 4096, 4096), (13, 520, 8192), (24, 1024, 1024)])
def test_w16d_two_part_split_error(O, qg, t, m, n, k):
    """Full 24-bit activations over 13 binades: error vs the exact product within the two-part bound."""
    rng = np.random.default_rng(m * 7 + k)
    a = (rng.standard_normal((m, k)) * np.exp2(rng.integers(-6, 7, (m, 1)))).astype(np.float32)
    b = rng.uniform(-1, 1, (n, k)).astype(np.float32)
    bq = O.quantize(b, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    c = host(fn(dev(a), dev(bq), m, n, k)).astype(np.float64)
    w = O.dequantize(bq, t).astype(np.float64)
    exact = a.astype(np.float64) @ w.T
    mag = np.abs(a.astype(np.float64)) @ np.abs(w).T
    err = np.abs(c - exact)
    assert (err <= (2.0 ** -16 + (k + 2) * 2.0 ** -24) * mag + 1e-30).all()


def test_w16d_repeat_bit_identical(O, qg):
    """Fixed-order sum of the waves' partial tiles (12 or 16 waves, qg_w4a16.hip w16d_launch): repeated launches
    are bit-identical."""
    m, n, k = 32, 4096, 4096
    a, b = O.fill_uniform_step4(m, n, k, seed=9)
    bq = O.quantize(b, 2)
    a_d, b_d = dev(a), dev(bq)
    import torch
    dense = qg.gemm_w4a16(a_d, b_d, m, n, k)
    for _ in range(3):
        assert torch.equal(qg.gemm_w4a16(a_d, b_d, m, n, k), dense)
    check(O, host(dense), a, bq, 2)
