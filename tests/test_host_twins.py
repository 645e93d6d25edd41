"""libqg_host.so — the host-only twins of the reference's CPU API (include/qg/qg_host.h; SURVEY.md
§8(b) "CPU API": gemm_w4a8_reference, vec_dot_q4_0_q8_1, quantize_row_*_ref, gemm_fp32_reference)
checked bit for bit against the oracle's restatement, which is itself pinned by the reference's
golden vectors (tests/test_oracle.py)."""
import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def H():
    import quant_gemm.host as H
    H.load()
    return H


def test_exports_match_header(H):
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "qg", "qg_host.h")).read(), flags=re.S)
    declared = set(re.findall(r"^\s*\w+\s+\**(qg_\w+)\s*\(", src, flags=re.M))
    assert declared == set(H.SIGNATURES)
    for name in declared:
        assert hasattr(H.load(), name)


@pytest.mark.parametrize("m,n,k", [(1, 128, 256), (3, 33, 1024), (1, 4096, 4096)])
def test_fill_step4_matches_oracle(O, H, m, n, k):
    a0, b0 = O.fill_uniform_step4(m, n, k, 42)
    a, b = H.fill_step4(m, n, k, 42)
    assert np.array_equal(a, a0) and np.array_equal(b, b0)
    _, bs = H.fill_step4(m, n, k, 42, row0=n // 3, row1=n // 2)  # a rank's shard of the rows
    assert np.array_equal(bs, b0[n // 3:n // 2])


def test_quantizers_bit_exact(O, H):
    a, b = O.fill_uniform_step4(7, 9, 1024, 3)
    edge = np.stack([np.zeros(64, np.float32), (np.arange(64, dtype=np.float32) - 31.5) / 8.0,
                     np.full(64, -3.0, np.float32)])
    for x in (a, b, edge):
        assert np.array_equal(H.quantize_q8_1(x), O.quantize(x, O.Q8_1))
        assert np.array_equal(H.quantize_q4_0(x), O.quantize(x, O.Q4_0))


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("m,n,k", [(1, 128, 256), (3, 37, 2048), (2, 300, 4096)])
def test_gemm_bit_exact(O, H, t, m, n, k):
    a, b = O.fill_uniform_step4(m, n, k, 42)
    aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, t)
    want = O.gemm_w4a8(aq, bq, t)
    assert np.array_equal(H.gemm_w4a8(aq, bq, m, n, k, t), want)
    assert np.array_equal(H.gemm_w4a8(aq, bq, m, n, k, t, threads=5), want)


def test_reference_signatures(O, H):
    """gemm_w4a8_reference(A, B, C, M, N, K), vec_dot_q4_0_q8_1(n, &s, vx, vy) and the W8A8 pair."""
    lib = H.load()
    m, n, k = 2, 16, 512
    a, b = O.fill_uniform_step4(m, n, k, 42)
    aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, O.Q4_0)
    c = np.empty((m, n), np.float32)
    P = ctypes.c_void_p
    assert lib.qg_gemm_w4a8_q4_0_cpu(P(aq.ctypes.data), P(bq.ctypes.data), P(c.ctypes.data), m, n, k) == 0
    assert np.array_equal(c, O.gemm_w4a8(aq, bq, O.Q4_0))
    s = ctypes.c_float()
    lib.qg_vec_dot_q4_0_q8_1_cpu(k, ctypes.byref(s), P(bq[5].ctypes.data), P(aq[1].ctypes.data))
    assert np.float32(s.value) == np.float32(O.vec_dot_q4_0_q8_1(bq[5], aq[1]))
    assert np.float32(s.value) == c[1, 5]
    b8 = O.quantize(b, O.Q8_0)
    c8 = np.empty((m, n), np.float32)
    assert lib.qg_gemm_w8a8_cpu(P(aq.ctypes.data), P(b8.ctypes.data), P(c8.ctypes.data), m, n, k) == 0
    assert np.array_equal(c8, O.gemm_w8a8(aq, b8))
    lib.qg_vec_dot_q8_0_q8_1_cpu(k, ctypes.byref(s), P(b8[3].ctypes.data), P(aq[0].ctypes.data))
    assert abs(s.value - c8[0, 3]) <= 1e-5 * max(1.0, abs(c8[0, 3]))  # sumi*d_w*d_a vs sumi*d_a*d_w


def test_fp32_reference_bit_exact(O, H):
    a, b = O.fill_uniform_step4(3, 40, 512, 42)
    assert np.array_equal(H.gemm_fp32(a, b), O.gemm_fp32(a, b))


def test_validation(H):
    lib = H.load()
    P = ctypes.c_void_p
    assert lib.qg_gemm_w4a8_q4_0_cpu(P(8), P(8), P(8), 1, 1, 33) == -2
    assert lib.qg_gemm_w4a8_cpu_mt(P(8), P(8), P(8), 1, 1, 64, 9, 1) == -3
    assert lib.qg_gemm_w4a8_q4_0_cpu(None, None, None, 0, 5, 64) == 0
    assert lib.qg_fill_step4_cpu(1, 1, 4, 32, 3, 2, None, None) == -1
