"""Tiled activations (round 5): the activation side of the tiled layout, so both operands of every prefill
stage are one linear DMA stream (LAY_TILED_ACT; qg_quantize_q8_1_tiled, qg_tile_activations,
qg_gemm_w4a8_tiled_act).

* the quantizer's and the repack's bytes equal oracle.tile_activations of the Q8_1 rows (the real blocks'
  bytes are qg_quantize_q8_1's, which tests/test_gpu_product.py pins to the reference quantizer);
* every block's int32 dot from the instantiation gemm_w4a8_tiled_act launches equals the reference's inner
  loop (include/gemm_reference.h:202-212) — bit-exact — for every format, the small-tile kernels (incl. odd
  K/32: the zero-padded fourth blocks), the large-M kernel and the tiled decode GEMV (M <= 4);
* outputs are bit-identical to gemm_w4a8_tiled on the row activations where the two pick the same tile
  configuration (only the activation bytes' source differs) and within the reassociation bound of the oracle.
"""
import numpy as np
import pytest

from test_gpu_product import dev, host, random_blocks

pytestmark = pytest.mark.gpu

TYPES = [2, 3, 6, 7, 8]


@pytest.mark.parametrize("m,k", [(1, 4096), (17, 4128), (32, 4096), (40, 96), (5, 32)])
def test_tiled_activation_bytes(O, qg, m, k):
    import torch
    rng = np.random.default_rng(m + k)
    x = (rng.standard_normal((m, k)) * 3).astype(np.float32)
    xt = torch.from_numpy(x).to("cuda")
    rows = qg.quantize_q8_1(xt)
    want = O.tile_activations(host(rows).reshape(m, k // 32, 36))
    assert np.array_equal(host(qg.quantize_q8_1_tiled(xt)), want)
    assert np.array_equal(host(qg.tile_activations(rows, m, k)), want)


SHAPES = [
    (1, 4096, 4096, "gemvt "),   # the tiled decode GEMV, activations staged from the tiled layout
    (2, 300, 4128, "gemvt "),    # the same at M = 2, odd K/32 (the layout's zero padding blocks)
    (3, 300, 4128, "gemvm "),    # the MFMA small-batch decode at M = 3, odd K/32
    (32, 4096, 4096, "mmq "),    # configs[2]: 32 x 16 tiles, 12 waves
    (5, 300, 1024, "mmq "),      # 16-row tiles, ragged N, one partly filled token tile
    (40, 1000, 512, "mmq "),     # 32 x 32 tiles, a token tile past the last 16-token tile
    (33, 300, 1056, "mmq "),     # odd K/32: the zero fourth blocks of the last stage
    (520, 4096, 1024, "mmql "),  # the large-M kernel, ragged M
]


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("m,n,k,fam", SHAPES)
def test_tiled_act_sumi_and_output(O, qg, t, m, n, k, fam):
    cfg = qg.debug_config_tiled_act(m, n, k, t)
    assert cfg == qg.debug_config_tiled_act(m, n, k, t, sumi=True)
    assert cfg.startswith(fam) and ("LAY=2" in cfg or " TA=1 " in cfg), cfg
    aq, bq = random_blocks(np.random.default_rng(m * 3 + n + k + t), m, n, k, t)
    a, bt = dev(aq), qg.tile_weights(dev(bq), n, k, t)
    at = qg.tile_activations(a, m, k)
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(host(qg.debug_sumi_tiled_act(at, bt, m, n, k, t)), want)
    c = host(qg.gemm_w4a8_tiled_act(at, bt, m, n, k, t))
    # the same tile configuration as the row-activation entry (odd K/32 may pick another one there: Q8_0's
    # windowed rings do not fit the 8-wave tiles) -> the same bits
    same = qg.debug_config_tiled(m, n, k, t).replace("LAY=1", "LAY=2").replace("AW=1", "AW=0").replace(" TA=0 ", " TA=1 ")
    if same == cfg:
        assert np.array_equal(c, host(qg.gemm_w4a8_tiled(a, bt, m, n, k, t)))
    tol = O.summation_tol(aq, bq, want, t) if fam == "gemvt " else O.reassoc_tol(aq, bq, want, t, waves=16)
    assert (np.abs(c.astype(np.float64) - c_ref) <= tol).all()


def test_tiled_act_contract(qg):
    import ctypes
    import torch
    lib = qg._lib.load()
    assert lib.qg_activations_tiled_bytes(17, 4128) == 2 * 33 * 2304
    assert lib.qg_activations_tiled_bytes(16, 4096) == 32 * 2304
    assert lib.qg_activations_tiled_bytes(4, 100) == 0
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p
    x = torch.zeros(64 * 4096 + 16, dtype=torch.float32, device="cuda")
    y = torch.zeros(lib.qg_activations_tiled_bytes(64, 4096) + 16, dtype=torch.uint8, device="cuda")
    assert lib.qg_quantize_q8_1_tiled(P(x.data_ptr() + 4), P(y.data_ptr()), 64, 4096, st) == -4  # x not 16-B aligned
    assert lib.qg_quantize_q8_1_tiled(P(x.data_ptr()), P(y.data_ptr() + 8), 64, 4096, st) == -4
    assert lib.qg_quantize_q8_1_tiled(P(x.data_ptr()), P(y.data_ptr()), 64, 4100, st) == -2
    assert lib.qg_quantize_q8_1_tiled(P(x.data_ptr()), P(y.data_ptr()), 0, 4096, st) == 0


@pytest.mark.parametrize("t", [2, 8])
def test_tiled_act_full_size_configs2(O, qg, t):
    """BASELINE configs[2] (M = 32, N = K = 4096) from FP32 activations quantized straight into the tiled
    layout: bit-identical to the row-activation tiled product, within the reassociation bound of the oracle."""
    import torch
    m, n, k = 32, 4096, 4096
    a, b = O.fill_uniform_step4(m, n, k, 7)
    bq = O.quantize(b, t)
    xt = torch.from_numpy(a.astype(np.float32)).to("cuda")
    rows = qg.quantize_q8_1(xt)
    bt = qg.tile_weights(dev(bq), n, k, t)
    c = host(qg.gemm_w4a8_tiled_act(qg.quantize_q8_1_tiled(xt), bt, m, n, k, t))
    assert np.array_equal(c, host(qg.gemm_w4a8_tiled(rows, bt, m, n, k, t)))
    aq = host(rows).reshape(m, k // 32, 36)
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert (np.abs(c.astype(np.float64) - c_ref) <= O.reassoc_tol(aq, bq, want, t, waves=16)).all()
