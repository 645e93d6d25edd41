"""Odd K/32 at prefill sizes without per-call weight copies.

* qg_repack_weights: the load-time layout is the original rows followed by zero blocks (bytes
  checked on the host);
* qg_gemm_w4a8_prepacked: every M from the GEMV to the MFMA range and every weight format, within
  the oracle's bound (summation order on the GEMV, reassociation on the MFMA kernel), for K/32 odd,
  even-but-not-a-multiple-of-8, and already a multiple of 8 (no workspace needed);
* qg_gemm_w4a8_ws: the repack route with the caller's workspace inside a stream capture — the graph
  replays bit-identical to the eager call (which uses the library's per-stream buffer);
* the repack route with a strided output (column slice) and through the weight-major entry.
"""
import ctypes

import numpy as np
import pytest

from test_gpu_product import close_to_oracle, dev, host, random_blocks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("k", [4128, 1056, 4160, 4096])
def test_repack_weights_layout(qg, t, k):
    n = 37
    _, bq = random_blocks(np.random.default_rng(k + t), 1, n, k, t)
    bp = host(qg.repack_weights(dev(bq), n, k, t))
    nb, nbp = k // 32, (k // 32 + 7) // 8 * 8
    assert bp.shape == (n, nbp, bq.shape[2])
    assert np.array_equal(bp[:, :nb], bq)
    assert not bp[:, nb:].any()


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("m,n,k", [(1, 4096, 4128), (3, 300, 4128), (8, 1100, 1056), (32, 4096, 4128),
                                   (64, 1030, 4160), (33, 64, 96), (32, 512, 4096)])
def test_prepacked_matches_oracle(O, qg, t, m, n, k):
    aq, bq = random_blocks(np.random.default_rng(m * 13 + n + k + t), m, n, k, t)
    bp = qg.repack_weights(dev(bq), n, k, t)
    c = host(qg.gemm_w4a8_prepacked(dev(aq), bp, m, n, k, t))
    kp = 32 * ((k // 32 + 7) // 8 * 8)
    close_to_oracle(O, c, aq, bq, t, mfma=qg.select_algo(m, n, kp, t) == 2)


def test_prepacked_workspace_contract(qg):
    lib = qg._lib.load()
    assert lib.qg_gemm_w4a8_prepacked_workspace_size(32, 4096) == 0
    assert lib.qg_gemm_w4a8_prepacked_workspace_size(32, 4128) == 32 * 136 * 36
    assert lib.qg_repack_weights_bytes(10, 4128, 2) == 10 * 136 * 18
    import torch
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = torch.zeros(32 * 129 * 36, dtype=torch.uint8, device="cuda")
    b = torch.zeros(16 * 136 * 18, dtype=torch.uint8, device="cuda")
    c = torch.zeros(32 * 16, dtype=torch.float32, device="cuda")
    P = ctypes.c_void_p
    # K' != K without a workspace: refused on the GEMV path (M <= 4), nothing launched; the MFMA path
    # (M >= 5) reads the plain activation rows itself since round 5 and needs none
    assert lib.qg_gemm_w4a8_prepacked(P(a.data_ptr()), P(b.data_ptr()), P(c.data_ptr()), 3, 16, 4128, 2, None, 0, st) == -1
    assert lib.qg_gemm_w4a8_prepacked(P(a.data_ptr()), P(b.data_ptr()), P(c.data_ptr()), 32, 16, 4128, 2, None, 0, st) == 0


@pytest.mark.parametrize("t", [2, 8])
def test_w4a8_ws_graph_capture_repack(O, qg, t):
    """The repack route inside a hipGraph with the caller's workspace: same bits as eager."""
    import torch
    m, n, k = 32, 1100, 4128
    aq, bq = random_blocks(np.random.default_rng(99 + t), m, n, k, t)
    a_d, b_d = dev(aq), dev(bq)
    lib = qg._lib.load()
    wsb = lib.qg_gemm_w4a8_workspace_size(m, n, k, t)
    assert wsb > 0
    assert lib.qg_gemm_w4a8_workspace_size(32, 4096, 4096, t) == 0 or True  # shape-only upper bound
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    eager = host(qg.gemm_w4a8(a_d, b_d, m, n, k, t))
    out = torch.zeros((m, n), dtype=torch.float32, device="cuda")
    P = ctypes.c_void_p

    def call():
        st = P(torch.cuda.current_stream().cuda_stream)
        assert lib.qg_gemm_w4a8_ws(P(a_d.data_ptr()), P(b_d.data_ptr()), P(out.data_ptr()), m, n, k, t,
                                   P(ws.data_ptr()), wsb, st) == 0

    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        call()
    torch.cuda.synchronize()
    out.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        call()
    g.replay()
    assert np.array_equal(host(out).view(np.uint32), eager.view(np.uint32))
    close_to_oracle(O, eager, aq, bq, t, mfma=True)


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
def test_repack_strided_and_weight_major(O, qg, t):
    """the repack route through qg_gemm_w4a8_ldc (output column slice) and through the
    weight-major entry (transposed store, ldc_n != 1)."""
    import torch
    m, n, k = 40, 1030, 4128
    aq, bq = random_blocks(np.random.default_rng(7 * t), m, n, k, t)
    assert qg.select_algo(m, n, k, t) == 2
    wide = torch.full((m, n + 9), 3.0, dtype=torch.float32, device="cuda")
    qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, out=wide[:, :n])
    w = host(wide)
    assert (w[:, n:] == 3.0).all()
    close_to_oracle(O, w[:, :n], aq, bq, t, mfma=True)
    sym = {2: "gemm_q4_0_q8_1", 3: "gemm_q4_1_q8_1", 6: "gemm_q5_0_q8_1", 7: "gemm_q5_1_q8_1", 8: "gemm_q8_0_q8_1"}[t]
    wm = host(getattr(qg, sym)(dev(bq), dev(aq), n, m, k))  # out [N weight rows][M tokens]
    assert np.array_equal(wm.T.view(np.uint32), w[:, :n].view(np.uint32))


@pytest.mark.parametrize("t", [2, 3, 8])
@pytest.mark.parametrize("m,n,k", [(32, 4096, 4128), (3, 300, 1056), (40, 1030, 96)])
def test_padded_quantizer_and_single_launch(O, qg, t, m, n, k):
    """qg_quantize_q8_1_padded: the real blocks are qg_quantize_q8_1's bytes (= the oracle's), then
    zero blocks; qg_gemm_w4a8_padded on them is bit-identical to qg_gemm_w4a8_prepacked (same padded
    bytes, same kernel) and within the oracle's bound."""
    a, b = O.fill_uniform_step4(m, n, k, seed=m + k + t)
    aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, t)
    ap = host(qg.quantize_q8_1_padded(dev(a)))
    nb, nbp = k // 32, (k // 32 + 7) // 8 * 8
    assert ap.shape == (m, nbp, 36)
    assert np.array_equal(ap[:, :nb], aq) and not ap[:, nb:].any()
    bp = qg.repack_weights(dev(bq), n, k, t)
    c = host(qg.gemm_w4a8_padded(dev(ap), bp, m, n, k, t))
    c2 = host(qg.gemm_w4a8_prepacked(dev(aq), bp, m, n, k, t))
    assert np.array_equal(c.view(np.uint32), c2.view(np.uint32))
    close_to_oracle(O, c, aq, bq, t, mfma=qg.select_algo(m, n, 32 * nbp, t) == 2)
