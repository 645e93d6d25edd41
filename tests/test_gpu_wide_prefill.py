"""The M <= 32 prefill at wide-row shapes (>= 256 tiles of 32 rows x 16 tokens: the 32-row MFMA tile
of BASELINE configs[2]): full-size configs[2] for every weight format, ragged M / N edges at that tile,
K from one to 160 blocks, raw random bytes, strided outputs and repeat determinism. (Written in round 4
for a chunked-ingest variant of the kernel, profiles/tools_archive/mmqc_experiment.hpp, measured slower and not
shipped; the cases stay as parity coverage of the product tile.) Bars as in test_gpu_parity.py: per-block int32
sumi bit-exact through the parity hook (the same instantiation), outputs within oracle.reassoc_tol
(DESIGN.md §5). Oracle contract: include/gemm_reference.h:175-222."""
import numpy as np
import pytest

from test_gpu_parity import WTYPES, assert_close_to_oracle, dev, host, make_case, random_byte_case

pytestmark = pytest.mark.gpu

SHAPES = [(32, 4096, 4096), (20, 8200, 1024), (32, 4100, 5120), (17, 8192, 3072), (9, 16384, 2048)]


@pytest.mark.parametrize("t", WTYPES)
@pytest.mark.parametrize("m,n,k", SHAPES)
def test_wide_prefill_exact(O, qg, t, m, n, k):
    cfg = qg.debug_config(m, n, k, t)
    assert cfg.startswith(f"mmq F={t} BN=32 TT=1 ") and cfg == qg.debug_config(m, n, k, t, sumi=True), cfg
    _, _, aq, bq = make_case(O, m, n, k, t, seed=m + n)
    a_d, b_d = dev(aq), dev(bq)
    got = host(qg.debug_sumi(a_d, b_d, m, n, k, t, 2))
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)
    c = host(qg.gemm_w4a8(a_d, b_d, m, n, k, t))
    assert_close_to_oracle(O, c, aq, bq, t, mfma=True)


@pytest.mark.parametrize("t", WTYPES)
def test_wide_prefill_random_bytes(O, qg, t):
    """Every weight nibble / byte value and activation byte incl. -128 (raw random blocks)."""
    m, n, k = 24, 8192, 2048
    assert qg.debug_config(m, n, k, t).startswith(f"mmq F={t} BN=32 TT=1 ")
    aq, bq = random_byte_case(m, n, k, t, seed=3)
    got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t, 2))
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    assert_close_to_oracle(O, c, aq, bq, t, mfma=True)


def test_wide_prefill_strided_output_and_determinism(O, qg):
    """A column slice of a wider buffer (qg_gemm_w4a8_ldc): the kernel writes only its columns,
    bit-identical to the dense call; repeated launches are bit-identical (fixed-order wave sum)."""
    import torch
    m, n, k, t = 32, 4096, 4096, 2
    _, _, aq, bq = make_case(O, m, n, k, t, seed=5)
    a_d, b_d = dev(aq), dev(bq)
    dense = qg.gemm_w4a8(a_d, b_d, m, n, k, t)
    wide = torch.full((m, n + 96), -7.0, dtype=torch.float32, device="cuda")
    qg.gemm_w4a8(a_d, b_d, m, n, k, t, out=wide[:, 32:32 + n])
    torch.cuda.synchronize()
    assert torch.equal(wide[:, 32:32 + n], dense)
    assert bool((wide[:, :32] == -7.0).all()) and bool((wide[:, 32 + n:] == -7.0).all())
    for _ in range(3):
        assert torch.equal(qg.gemm_w4a8(a_d, b_d, m, n, k, t), dense)


# The 16-row x 16-token tile of one-round grids (M <= 16): 16 waves with one stage slot each for every
# format but Q8_0 (8 waves x 2 slots; qg_gemm_mfma.hip alt_w / alt_nb). Ragged M / N, one stage (4 blocks) to 192 blocks.
S16_SHAPES = [(16, 4096, 4096), (8, 4096, 4096), (5, 4000, 2048), (13, 4088, 6144), (11, 2056, 128)]


@pytest.mark.parametrize("t", WTYPES)
@pytest.mark.parametrize("m,n,k", S16_SHAPES)
def test_s16_prefill_exact(O, qg, t, m, n, k):
    cfg = qg.debug_config(m, n, k, t)
    if (m, n, k) in S16_SHAPES[:2]:
        assert cfg.startswith(f"mmq F={t} BN=16 TT=1 "), cfg
    if cfg.startswith(f"mmq F={t} BN=16 TT=1 ") and (n + 15) // 16 <= 256:
        assert (" W=8 " in cfg and " NB=2 " in cfg) if t == 8 else (" W=16 " in cfg and " NB=1 " in cfg), cfg
    _, _, aq, bq = make_case(O, m, n, k, t, seed=m + 3 * n)
    a_d, b_d = dev(aq), dev(bq)
    got = host(qg.debug_sumi(a_d, b_d, m, n, k, t, 2))
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)
    c = host(qg.gemm_w4a8(a_d, b_d, m, n, k, t))
    assert_close_to_oracle(O, c, aq, bq, t, mfma=True)
    assert np.array_equal(c, host(qg.gemm_w4a8(a_d, b_d, m, n, k, t)))  # repeat: bit-identical
