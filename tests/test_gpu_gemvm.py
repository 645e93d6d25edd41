"""Small-batch decode on the tiled layout with the matrix cores (qg_gemvm.hip, round 6).

* the sumi hook runs the instantiation qg_gemm_w4a8_tiled launches (same qg_debug_config_tiled string) and
  every block's int32 dot equals the reference's inner loop (include/gemm_reference.h:202-212) — bit-exact;
* the outputs lie within the MFMA epilogue's reassociation bound of the oracle (oracle.reassoc_tol: the
  d_w d_a sumi part and the offset part rounded separately, W partial tiles summed in fixed order);
* every format, 4 / 8 stages per lane, one wave (no cross-wave sum), stages past K/32 (zero padding
  blocks, and stages past the last real one in the last wave), ragged N, 2..4 tokens, both activation forms
  (Q8_1 rows and the tiled activation layout), grids that put several workgroups on a CU (the padding-record
  bug of the first version showed only there: qg_gemvm.hip header);
* deterministic: the same launch twice gives the same bits.
"""
import numpy as np
import pytest

from test_gpu_product import dev, host, random_blocks

pytestmark = pytest.mark.gpu

TYPES = [2, 3, 6, 7, 8]

SHAPES = [
    (2, 4096, 14336),  # the reference's batch-decode shape, M = 2: 8 stages per lane, 14 waves, 2 token columns
    (4, 4096, 14336),  # M = 4: 4 token columns
    (2, 300, 8224),    # M = 2 from K/32 = 257: a padding block, a last wave with stages past H
    (4, 300, 4128),    # K/32 = 129: padding blocks in the last stage, a last wave with stages past H
    (3, 64, 160),      # one wave (H = 2 of its 4 stages), stages past K/32, token 3 of 4 columns repeats token 2
    (3, 1000, 6144),   # 4 stages per lane, ragged N (one half tile past it)
    (4, 32000, 1024),  # many half tiles (linear order), 2 waves, several workgroups per CU
    (3, 48, 96),       # K/32 = 3 < one stage
]


def _cfg(qg, m, n, k, t, act=False):
    f = qg.debug_config_tiled_act if act else qg.debug_config_tiled
    cfg = f(m, n, k, t)
    assert cfg == f(m, n, k, t, sumi=True)
    return cfg


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("m,n,k", SHAPES)
def test_gemvm_sumi_and_output(O, qg, t, m, n, k):
    cfg = _cfg(qg, m, n, k, t)
    assert cfg.startswith(f"gemvm F={t} ") and " TA=0 " in cfg, cfg
    aq, bq = random_blocks(np.random.default_rng(m * 13 + n + k + t), m, n, k, t)
    bt = qg.tile_weights(dev(bq), n, k, t)
    a = dev(aq)
    got = host(qg.debug_sumi_tiled(a, bt, m, n, k, t))
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)
    c = host(qg.gemm_w4a8_tiled(a, bt, m, n, k, t))
    err = np.abs(c.astype(np.float64) - c_ref)
    assert (err <= O.reassoc_tol(aq, bq, want, t, waves=16)).all(), f"max err {err.max()}"
    c2 = host(qg.gemm_w4a8_tiled(a, bt, m, n, k, t))
    assert np.array_equal(c.view(np.uint32), c2.view(np.uint32))


@pytest.mark.parametrize("t", [2, 7, 8])
@pytest.mark.parametrize("m,n,k", [(4, 4096, 14336), (3, 300, 4128)])
def test_gemvm_tiled_activations(O, qg, t, m, n, k):
    """The tiled activation form feeds the same kernel (TA=1): bit-identical to the Q8_1-row form."""
    cfg = _cfg(qg, m, n, k, t, act=True)
    assert cfg.startswith(f"gemvm F={t} ") and " TA=1 " in cfg, cfg
    aq, bq = random_blocks(np.random.default_rng(m + n + k + t), m, n, k, t)
    bt = qg.tile_weights(dev(bq), n, k, t)
    a = dev(aq)
    at = qg.tile_activations(a, m, k)
    c_rows = host(qg.gemm_w4a8_tiled(a, bt, m, n, k, t))
    c_ta = host(qg.gemm_w4a8_tiled_act(at, bt, m, n, k, t))
    assert np.array_equal(c_rows.view(np.uint32), c_ta.view(np.uint32))
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(host(qg.debug_sumi_tiled_act(at, bt, m, n, k, t)), want)
