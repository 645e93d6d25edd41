"""ggml-facing adapter over device data (include/llama_adapter.h), GGUF weights end to end, and
the FP32 baseline GEMM — GPU parity through the C-ABI."""
import numpy as np
import pytest

from gguf_writer import STR, U32, as_bytes, write_gguf
from test_gpu_parity import assert_close_to_oracle, dev, host

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G(qg):
    from quant_gemm import ggml
    return ggml


@pytest.mark.parametrize("wt", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("m", [1, 3, 17])
def test_gguf_weights_through_w4a8_adapter(O, qg, G, tmp_path, wt, m):
    """GGUF file -> device -> gemm_w4a8_from_ggml == oracle on the same bytes."""
    import torch
    n, k = 72, 1024
    a, b = O.fill_uniform_step4(m, n, k, seed=wt + m)
    aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, wt)
    p = tmp_path / "w.gguf"
    write_gguf(p, [("general.architecture", STR, "llama"), ("general.alignment", U32, 64)],
               [("blk.0.w", wt, [k, n], as_bytes(bq))], alignment=64)
    with G.GGUFFile(p) as f:
        w = f.to_device("blk.0.w")
        assert np.array_equal(host(w), bq)
        wv = f.view("blk.0.w", w)
    a_t = dev(aq)
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")
    G.gemm_w4a8_from_ggml(G.view_of(a_t, G.Q8_1, k), wv, G.view_of(c, G.F32, n), "dp4a")
    assert_close_to_oracle(O, host(c), aq, bq, wt)
    assert G.validate_tensor_types(G.view_of(a_t, G.Q8_1, k), wv, G.view_of(c, G.F32, n), G.Q8_1, wt, G.F32)
    assert not G.validate_tensor_types(G.view_of(a_t, G.Q8_1, k), wv, G.view_of(c, G.F32, n), G.Q8_1, 99, G.F32)


@pytest.mark.parametrize("wt", [2, 8])
def test_w4a16_adapter(O, qg, G, wt):
    import torch
    m, n, k = 5, 40, 512
    a, b = O.fill_uniform_step4(m, n, k, seed=3)
    bq = O.quantize(b, wt)
    a_t, w_t = dev(a), dev(bq)
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")
    G.gemm_w4a16_from_ggml(G.view_of(a_t, G.F32, k), G.view_of(w_t, wt, k), G.view_of(c, G.F32, n))
    ref = O.gemm_w4a16(a, bq) if wt == 2 else O.gemm_w8a16(a, bq)
    assert (np.abs(host(c).astype(np.float64) - ref) <= O.w16_tol(a, bq, wt)).all()


@pytest.mark.parametrize("m,n,k", [(1, 64, 256), (33, 70, 100), (128, 96, 1024), (7, 5, 3)])
def test_fp32_gemm_matches_reference(O, qg, G, m, n, k):
    """qg_gemm_fp32 vs gemm_fp32_reference (oracle) within the fp32 summation bound."""
    import torch
    a = np.random.default_rng(m).uniform(-1, 1, (m, k)).astype(np.float32)
    b = np.random.default_rng(n).uniform(-1, 1, (n, k)).astype(np.float32)
    a_t, b_t = dev(a), dev(b)
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")
    G.gemm_fp32_from_ggml(G.view_of(a_t, G.F32, k), G.view_of(b_t, G.F32, k), G.view_of(c, G.F32, n))
    ref = O.gemm_fp32(a, b)
    tol = 2.0 * (k + 1) * 2.0 ** -24 * (np.abs(a.astype(np.float64)) @ np.abs(b.astype(np.float64)).T) + 1e-30
    assert (np.abs(host(c).astype(np.float64) - ref) <= tol).all()
