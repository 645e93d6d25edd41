"""Fused activation quantization, GPU parity through the C-ABI.

* qg_gemm_w4a8_f32: FP32 activations quantized inside the product. Bar: BIT-IDENTICAL to the
  two-step path (qg_quantize_q8_1 + qg_gemm_w4a8 with the same kernel family), hence to the oracle
  within the summation-order bound, on every dispatch branch (fused GEMV prologue, workspace,
  chunked fused GEMV without a workspace).
* qg_gemm_q4_0_fp16_fused (kernels/gemm/gemm_fused.cuh:311-338): FP16 activations, the fused
  kernel's quantizer semantics (gemm_fused.cuh:76-143, restated in the oracle as
  qgo_quantize_q8_1_fused_f16). Bar: quantizer bytes bit-exact; outputs within the summation
  bound of the oracle's qgo_gemm_q4_0_fp16_fused (the reference's own kernel is racy, SURVEY.md
  §0.5, and cannot run here: parity for this row is pinned by the restated per-block semantics).
"""
import ctypes

import numpy as np
import pytest

from test_gpu_parity import WTYPES, assert_close_to_oracle, dev, edge_rows, host, make_case

pytestmark = pytest.mark.gpu


def two_step(qg, x_d, w_d, m, n, k, t, algo=0):
    return host(qg.gemm_w4a8(qg.quantize_q8_1(x_d), w_d, m, n, k, t, algo=algo))


@pytest.mark.parametrize("t", WTYPES)
@pytest.mark.parametrize("m", [1, 2, 3, 4, 5, 8, 13, 40])
def test_f32_fused_bit_identical_to_two_step(O, qg, t, m):
    n, k = 200, 4096
    a, _, aq, bq = make_case(O, m, n, k, t, seed=7 + m)
    x_d, w_d = dev(a), dev(bq)
    ref = two_step(qg, x_d, w_d, m, n, k, t)
    got = host(qg.gemm_w4a8_f32(x_d, w_d, t, workspace=True))
    assert np.array_equal(got, ref)
    assert_close_to_oracle(O, got, aq, bq, t)
    # no workspace: M <= 4 is the same single launch; larger M runs the fused GEMV per 8-row chunk,
    # bit-identical to the two-step GEMV on the same chunks
    got_nows = host(qg.gemm_w4a8_f32(x_d, w_d, t, workspace=False))
    if m <= 4:
        assert np.array_equal(got_nows, ref)
    else:
        for r0 in range(0, m, 8):
            r1 = min(m, r0 + 8)
            chunk = two_step(qg, x_d[r0:r1].contiguous(), w_d, r1 - r0, n, k, t, algo=1)
            assert np.array_equal(got_nows[r0:r1], chunk)
        assert_close_to_oracle(O, got_nows, aq, bq, t)


@pytest.mark.parametrize("k", [64, 96, 128, 288, 14336])
def test_f32_fused_edge_rows_and_odd_k(O, qg, k):
    """Quantizer edge cases (zero rows, f16 ties, tiny/huge scales) and K not a multiple of 128."""
    rows = edge_rows()
    x = np.tile(rows, (1, (k + 63) // 64))[:, :k].copy()[:4]
    m, n = x.shape[0], 33
    _, b = O.fill_uniform_step4(1, n, k, seed=3)
    bq = O.quantize(b, O.Q4_0)
    x_d, w_d = dev(x), dev(bq)
    got = host(qg.gemm_w4a8_f32(x_d, w_d, O.Q4_0))
    assert np.array_equal(got, two_step(qg, x_d, w_d, m, n, k, O.Q4_0))
    assert_close_to_oracle(O, got, O.quantize(x, O.Q8_1), bq, O.Q4_0)


def test_f32_fused_full_size(O, qg):
    """BASELINE configs[1] shape (M=1, N=K=4096) through the fused entry point."""
    a, b, aq, bq = make_case(O, 1, 4096, 4096, 2)
    got = host(qg.gemm_w4a8_f32(dev(a), dev(bq), 2))
    assert_close_to_oracle(O, got, aq, bq, 2)
    assert O.nmse(got, O.gemm_fp32(a, b)) <= 5e-3


def test_f32_fused_alignment(O, qg):
    """X only 4-B aligned: served through the workspace, QG_ERR_ALIGN (-4) without one."""
    import torch
    m, n, k = 2, 64, 1024
    a, _, aq, bq = make_case(O, m, n, k, 2)
    raw = torch.zeros(a.size + 1, dtype=torch.float32, device="cuda")
    raw[1:] = dev(a.ravel())
    x = raw[1:]
    assert x.data_ptr() % 16 != 0
    w = dev(bq)
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")
    lib = qg._lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p
    assert lib.qg_gemm_w4a8_f32(P(x.data_ptr()), P(w.data_ptr()), P(c.data_ptr()), m, n, k, 2, None, 0, st) == -4
    ws = torch.empty(lib.qg_gemm_w4a8_f32_workspace_size(m, k), dtype=torch.uint8, device="cuda")
    assert lib.qg_gemm_w4a8_f32(P(x.data_ptr()), P(w.data_ptr()), P(c.data_ptr()), m, n, k, 2,
                                P(ws.data_ptr()), ws.numel(), st) == 0
    assert_close_to_oracle(O, host(c), aq, bq, 2)


# ------------------------------------------------------------------------------- FP16, gemm_fused.cuh
def f16_rows(seed=5):
    rng = np.random.default_rng(seed)
    rows = [edge_rows().astype(np.float16),
            (rng.standard_normal((8, 64)) * np.array([1e-3, 1, 30, 1000, 3000, 0.5, 2, 7])[:, None]).astype(np.float16),
            rng.choice(np.array([-1000.0, 0.25, 3.0, -0.125, 1e-3], np.float16), size=(8, 64))]
    return np.concatenate(rows)


def test_f16_fused_quantizer_bytes(O, qg):
    x = f16_rows()
    want = O.quantize_q8_1_fused_f16(x)
    got = host(qg.quantize_q8_1_f16_fused(dev(x)))
    assert np.array_equal(got, want)
    # the fused semantics really differ from quantize_row_q8_1_ref on these rows (the test would
    # not notice a kernel using the wrong quantizer otherwise)
    assert not np.array_equal(want, O.quantize(x.astype(np.float32), O.Q8_1))


@pytest.mark.parametrize("ntok", [1, 3, 4, 6, 8, 21])
@pytest.mark.parametrize("workspace", [True, False])
def test_f16_fused_gemm_matches_oracle(O, qg, ntok, workspace):
    mw, k = 130, 2048
    _, b = O.fill_uniform_step4(1, mw, k, seed=11)
    wq = O.quantize(b, O.Q4_0)
    act = (np.random.default_rng(ntok).standard_normal((ntok, k)) * 2).astype(np.float16)
    out = host(qg.gemm_q4_0_fp16_fused(dev(wq), dev(act), mw, ntok, k, workspace=workspace))
    assert out.shape == (mw, ntok)
    aq = O.quantize_q8_1_fused_f16(act)
    # oracle weight-major result, and the summation bound through the activation-major view
    want = O.gemm_q4_0_fp16_fused(wq, act)
    assert_close_to_oracle(O, np.ascontiguousarray(out.T), aq, wq, O.Q4_0)
    assert np.allclose(out, want, rtol=1e-4, atol=1e-3)
    # same bytes into the two-step weight-major product
    two = host(qg.gemm_q4_0_q8_1(dev(wq), qg.quantize_q8_1_f16_fused(dev(act)), mw, ntok, k))
    if ntok <= 4 or workspace:
        assert np.array_equal(out, two)


def test_f16_fused_edge_rows(O, qg):
    x = f16_rows()
    ntok, k = x.shape[0], x.shape[1]
    _, b = O.fill_uniform_step4(1, 40, k, seed=2)
    wq = O.quantize(b, O.Q4_0)
    out = host(qg.gemm_q4_0_fp16_fused(dev(wq), dev(x), 40, ntok, k, workspace=False))
    assert_close_to_oracle(O, np.ascontiguousarray(out.T), O.quantize_q8_1_fused_f16(x), wq, O.Q4_0)
