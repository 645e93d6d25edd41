"""GEMV at K < 4096 (round 3): 2-block units on 32- or 16-lane rows in 16-row workgroups (256
workgroups at N = 4096), where round 2 ran 4-lane rows in 64-row workgroups on a quarter of the CUs
(2-3x slower; profiles/r03_tuning/r03_ab_sk.txt). Pins the dispatch (qg_debug_config) and the
numerics of the new instantiations: every block's int32 dot bit-exact against the reference's inner
loop (include/gemm_reference.h:202-212) through the sumi hook, which runs the same instantiation,
outputs within the oracle's summation-order bound, for every weight format and M = 1..4; and the
W4A16 / W8A16 GEMV at the same K within the fp32 K-term bound.
"""
import numpy as np
import pytest

from test_gpu_product import dev, host, random_blocks

pytestmark = pytest.mark.gpu

SHAPES = [(1, 4096, 2048, 32), (2, 2048, 2048, 32), (4, 4096, 2048, 32), (3, 1000, 3072, 32), (1, 4096, 1024, 16),
          (4, 300, 1024, 16), (1, 77, 2560, 32)]


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("m,n,k,lpr", SHAPES)
def test_small_k_gemv(O, qg, t, m, n, k, lpr):
    cfg = qg.debug_config(m, n, k, t)
    assert cfg.startswith(f"gemv F={t} MT={1 if m == 1 else 2 if m == 2 else 4} BPL=2 LPR={lpr} "), cfg
    assert cfg == qg.debug_config(m, n, k, t, sumi=True)
    for aq, bq in [random_blocks(np.random.default_rng(m * 100 + k + t), m, n, k, t)]:
        got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t))
        c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
        c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
        assert np.array_equal(got, want)
        assert (np.abs(c.astype(np.float64) - c_ref) <= O.summation_tol(aq, bq, want, t)).all()


@pytest.mark.parametrize("t", [2, 8])
@pytest.mark.parametrize("m,n,k", [(1, 4096, 2048), (2, 4096, 2048), (4, 2048, 2048), (1, 4096, 1024),
                                   (3, 500, 3072), (1, 33, 1024)])
def test_small_k_w16_gemv(O, qg, t, m, n, k):
    a, b = O.fill_uniform_step4(m, n, k, seed=m + n + k)
    bq = O.quantize(b, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    c = host(fn(dev(a), dev(bq), m, n, k))
    ref = O.gemm_w4a16(a, bq) if t == O.Q4_0 else O.gemm_w8a16(a, bq)
    assert (np.abs(c.astype(np.float64) - ref) <= O.w16_tol(a, bq, t)).all()


def test_small_k_grouped_bit_identical(O, qg):
    """The grouped entry uses the same instantiation at K = 2048: each item equals its single launch."""
    rng = np.random.default_rng(9)
    m, k, t = 2, 2048, 2
    ns = [2048, 512, 512]
    aq, _ = random_blocks(rng, m, 1, k, t)
    bqs = [random_blocks(rng, m, n, k, t)[1] for n in ns]
    a_d = dev(aq)
    b_d = [dev(b) for b in bqs]
    outs = qg.gemm_w4a8_grouped([a_d] * 3, b_d, ns, m, k, t)
    for i, n in enumerate(ns):
        single = host(qg.gemm_w4a8(a_d, b_d[i], m, n, k, t))
        assert np.array_equal(host(outs[i]).view(np.uint32), single.view(np.uint32))


def test_w16_two_rows_per_wave_bit_identical(O, qg):
    """M = 1 W4A16 from N = 8192 on: two weight rows per wave (w16_gemv1r_kernel) share the lane's
    activation reads; each row keeps its summation order, so the first 4096 rows equal the one-row
    kernel's (N = 4096) bit for bit, and all rows are within the fp32 K-term bound."""
    n, k = 11008, 4096
    a, b = O.fill_uniform_step4(1, n, k, seed=3)
    bq = O.quantize(b, 2)
    a_d, b_d = dev(a), dev(bq)
    c_big = host(qg.gemm_w4a16(a_d, b_d, 1, n, k))
    c_small = host(qg.gemm_w4a16(a_d, b_d[:4096].contiguous(), 1, 4096, k))
    assert np.array_equal(c_big[:, :4096].view(np.uint32), c_small.view(np.uint32))
    assert (np.abs(c_big.astype(np.float64) - O.gemm_w4a16(a, bq)) <= O.w16_tol(a, bq, 2)).all()
