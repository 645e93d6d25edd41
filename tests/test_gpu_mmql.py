"""The large-M prefill kernel (qg_mmql_kernel.hpp, round 5): 64-row x 64-token workgroup tiles of four
32 x 32 waves (v_mfma_i32_32x32x32_i8), stages ingested cooperatively, XCD-aware tile order.

* the dispatch picks it exactly when its grid fills the CUs twice over (qg_mmq_dispatch.hpp: config);
* every block's int32 dot from the instantiation the product launches equals the reference's inner loop
  (include/gemm_reference.h:202-212) — bit-exact — on the reference rows and on the tiled layout, every
  format, with ragged M and N (rows / tiles past N read the last valid ones, their outputs dropped) and
  fewer stages than the pipeline's depth;
* outputs within the MFMA epilogue's reassociation bound of the oracle (oracle.reassoc_tol, one K
  partial: the waves own disjoint output tiles and accumulate every stage in order);
* the two layouts compute the same bits (same stage order, same arithmetic; only the bytes' source
  differs).
"""
import numpy as np
import pytest

from test_gpu_product import dev, host, random_blocks

pytestmark = pytest.mark.gpu

TYPES = [2, 3, 6, 7, 8]

SHAPES = [
    (2048, 1024, 256, 64),  # 2 stages (< the pipeline's 3 in flight)
    (1000, 2048, 512, 64),  # ragged M
    (520, 4010, 256, 64),   # ragged N within a 32-row tile, grid not a multiple of 8
    (520, 4096, 1024, 64),  # ragged M (9 token tiles), 8 stages
]


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("m,n,k,bm", SHAPES)
@pytest.mark.parametrize("tiled", [False, True])
def test_mmql_sumi_and_output(O, qg, t, m, n, k, bm, tiled):
    aq, bq = random_blocks(np.random.default_rng(m + n + k + t), m, n, k, t)
    a = dev(aq)
    if tiled:
        b = qg.tile_weights(dev(bq), n, k, t)
        cfg, cfg_s = qg.debug_config_tiled(m, n, k, t), qg.debug_config_tiled(m, n, k, t, sumi=True)
    else:
        b = dev(bq)
        cfg, cfg_s = qg.debug_config(m, n, k, t), qg.debug_config(m, n, k, t, sumi=True)
    assert cfg == cfg_s
    assert cfg.startswith("mmql ") and f"BN=64 BM={bm} " in cfg and f"LAY={int(tiled)}" in cfg, cfg
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    got = host(qg.debug_sumi_tiled(a, b, m, n, k, t) if tiled else qg.debug_sumi(a, b, m, n, k, t))
    assert np.array_equal(got, want)
    del got
    c = host(qg.gemm_w4a8_tiled(a, b, m, n, k, t) if tiled else qg.gemm_w4a8(a, b, m, n, k, t))
    err = np.abs(c.astype(np.float64) - c_ref)
    assert (err <= O.reassoc_tol(aq, bq, want, t, waves=1)).all(), f"max err {err.max()}"


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("m,n,k", [(512, 4096, 4096), (1024, 2048, 1024), (512, 14336, 4096)])
def test_mmql_layouts_bit_identical(qg, t, m, n, k):
    """Full-size shapes (configs' M = 512 prefill): reference rows and tiled layout, same bits."""
    aq, bq = random_blocks(np.random.default_rng(3 * m + t), m, n, k, t)
    assert qg.debug_config(m, n, k, t).startswith("mmql ")
    a, b = dev(aq), dev(bq)
    c_rows = host(qg.gemm_w4a8(a, b, m, n, k, t))
    c_tl = host(qg.gemm_w4a8_tiled(a, qg.tile_weights(b, n, k, t), m, n, k, t))
    assert np.isfinite(c_rows).all()
    assert np.array_equal(c_rows, c_tl)
