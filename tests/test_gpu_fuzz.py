"""Seeded random-shape sweep through the C-ABI's automatic dispatch (GPU).

Each case draws (M, N, K, weight format) from a fixed seed so a failure names a reproducible
shape; the shapes straddle every dispatch boundary (GEMV M <= 8 / prefill, K % 256, K % 128,
ragged N, the W4A16 split-K plans' slice counts), with raw random blocks (every nibble / byte,
activation -128) for W4A8 and step4 fp32 activations for W4A16 / W8A16. Bars as in
test_gpu_parity.py / test_gpu_w4a16.py: sumi bit-exact, outputs within the fp32 summation bound.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_close_to_oracle, dev, host, random_byte_case
from test_gpu_w4a16 import check as check_w16

pytestmark = pytest.mark.gpu

WTYPES = [2, 3, 6, 7, 8]


def w4a8_shapes(n_cases=36, seed=2024):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        t = WTYPES[i % len(WTYPES)]
        m = int(rng.choice([1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 48, 64, 65, 100]))
        n = int(rng.integers(1, 600))
        # K: multiples of 32 of every residue class mod 256 the kernels distinguish
        k = 32 * int(rng.choice([1, 3, 4, 7, 8, 12, 16, 24, 36, 64, 96, 129, 128]))
        while m * n * k > 12_000_000:
            n = max(1, n // 2)
        out.append((m, n, k, t, i))
    return out


@pytest.mark.parametrize("m,n,k,t,i", w4a8_shapes(), ids=lambda v: str(v))
def test_w4a8_auto_dispatch_random(O, qg, m, n, k, t, i):
    aq, bq = random_byte_case(m, n, k, t, seed=100 + i)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    assert_close_to_oracle(O, c, aq, bq, t)
    # the chosen family's integer sums are the reference's, bit for bit
    algo = qg._lib.load().qg_select_algo(m, n, k, t)
    got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t, algo))
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)


def w16_shapes(n_cases=24, seed=77):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        t = (2, 8)[i % 2]
        m = int(rng.choice([1, 3, 4, 8, 9, 12, 17, 24, 32, 40, 63, 64, 65, 80, 128]))
        n = int(rng.choice([1, 16, 33, 64, 100, 257, 512, 1000, 2048, 2100]))
        k = 32 * int(rng.choice([1, 2, 8, 16, 24, 32, 64, 128, 136, 256]))
        while m * n * k > 12_000_000:
            n = max(1, n // 2)
        out.append((m, n, k, t, i))
    return out


@pytest.mark.parametrize("m,n,k,t,i", w16_shapes(), ids=lambda v: str(v))
def test_w16_auto_dispatch_random(O, qg, m, n, k, t, i):
    a, b = O.fill_uniform_step4(m, n, k, seed=300 + i)
    bq = O.quantize(b, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    ad, bd = dev(a), dev(bq)
    c1 = host(fn(ad, bd, m, n, k))
    check_w16(O, c1, a, bq, t)
    # split-K tile counters re-arm: a repeat launch is bit-identical
    assert np.array_equal(c1, host(fn(ad, bd, m, n, k)))
