"""Seeded random-shape sweep of the product dispatch (auto kernel choice) against the oracle.

The parametrized suites pin chosen shapes; this one draws M, N, K and the weight format from a
fixed seed, so every kernel family and its edges (GEMV row tails, MFMA token / row tiles, the
ragged kernel for odd K/32, the W16 split-K planner, strided output rows) meet shapes nobody picked.
Bars as elsewhere: W4A8 within the oracle's summation-order bound (oracle.summation_tol) where the
kernel's per-block terms are bit-identical to the oracle's, within oracle.reassoc_tol where the MFMA
prefill served the shape (its epilogue rounds each term's two parts separately — this sweep found a
K = 128 Q5_0 case just outside summation_tol); W4A16 / W8A16 within oracle.w16_tol.
"""
import numpy as np
import pytest

from test_gpu_product import close_to_oracle, dev, host, random_blocks

pytestmark = pytest.mark.gpu

FMTS = [2, 3, 6, 7, 8]


def w4a8_cases(n_cases=40, seed=2026):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        m = int(rng.choice([1, 2, 3, 4, 5, 7, 8, 9, 12, 16, 17, 24, 31, 32, 33, 48, 64, 65, 96]))
        n = int(rng.integers(1, 700))
        nb = int(rng.integers(1, 160))
        if i % 4 == 0:
            nb |= 1  # odd K/32: the ragged kernel
        out.append((i, m, n, 32 * nb, FMTS[i % len(FMTS)]))
    return out


@pytest.mark.parametrize("i,m,n,k,t", w4a8_cases())
def test_w4a8_random_shapes(O, qg, i, m, n, k, t):
    rng = np.random.default_rng(1000 + i)
    if i % 2:
        aq, bq = random_blocks(rng, m, n, k, t)
    else:
        a, b = O.fill_uniform_step4(m, n, k, 7 + i)
        aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, t)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    close_to_oracle(O, c, aq, bq, t, mfma=qg.select_algo(m, n, k, t) == 2)


def repack_cases(n_cases=10, seed=4242):
    """random odd K/32 (and K/32 % 8 != 0) at prefill sizes — the repack + MFMA route."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        m = int(rng.choice([32, 33, 40, 48, 64, 65, 96]))
        n = int(rng.integers(1024, 2300))
        nb = int(rng.integers(3, 140))
        nb = nb | 1 if i % 2 == 0 else (nb // 2) * 2 + (2 if (nb // 2 * 2) % 8 == 0 else 0)
        out.append((i, m, n, 32 * nb, FMTS[i % len(FMTS)]))
    return out


@pytest.mark.parametrize("i,m,n,k,t", repack_cases())
def test_w4a8_random_repack_shapes(O, qg, i, m, n, k, t):
    """Outputs within the reassociation bound and the parity hook's int32 sumi bit-exact through the
    product instantiation (the padded-image MFMA kernel, compacted)."""
    rng = np.random.default_rng(2000 + i)
    aq, bq = random_blocks(rng, m, n, k, t)
    assert qg.select_algo(m, n, k, t) == 2
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    close_to_oracle(O, c, aq, bq, t, mfma=True)
    got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t))
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("i,m,n,k,t", w4a8_cases()[::4])
def test_w4a8_random_shapes_sumi(O, qg, i, m, n, k, t):
    """The parity hook on the sweep's shapes: int32 sumi bit-exact from the product instantiation."""
    rng = np.random.default_rng(3000 + i)
    aq, bq = random_blocks(rng, m, n, k, t)
    got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t))
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("i", range(8))
def test_w4a8_random_shapes_strided_out(O, qg, i):
    """Output rows in a column slice of a wider buffer (qg_gemm_w4a8_ldc), random shapes."""
    import torch
    rng = np.random.default_rng(500 + i)
    m, n, k, t = int(rng.integers(2, 70)), int(rng.integers(1, 400)), 32 * int(rng.integers(1, 100)), FMTS[i % 5]
    a, b = O.fill_uniform_step4(m, n, k, 11 + i)
    aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, t)
    pad = int(rng.integers(1, 40))
    wide = torch.full((m, n + pad), 7.0, dtype=torch.float32, device="cuda")
    qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, out=wide[:, :n])
    w = host(wide)
    assert (w[:, n:] == 7.0).all(), "wrote outside the slice"
    close_to_oracle(O, w[:, :n], aq, bq, t, mfma=qg.select_algo(m, n, k, t) == 2)


def w16_cases(n_cases=16, seed=77):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        m = int(rng.choice([1, 2, 4, 8, 9, 16, 17, 32, 40, 64, 65]))
        n = int(rng.integers(1, 600))
        k = 256 * int(rng.integers(1, 17)) if i % 2 else 32 * int(rng.integers(1, 130))
        out.append((i, m, n, k, (2, 8)[i % 2]))
    return out


@pytest.mark.parametrize("i,m,n,k,t", w16_cases())
def test_w16_random_shapes(O, qg, i, m, n, k, t):
    a, b = O.fill_uniform_step4(m, n, k, seed=300 + i)
    bq = O.quantize(b, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    c = host(fn(dev(a), dev(bq), m, n, k))
    ref = O.gemm_w4a16(a, bq) if t == O.Q4_0 else O.gemm_w8a16(a, bq)
    err = np.abs(c.astype(np.float64) - ref)
    assert (err <= O.w16_tol(a, bq, t)).all(), f"max err {err.max()}"
