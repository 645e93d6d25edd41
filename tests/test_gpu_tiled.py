"""The load-time tiled weight layout and its one-launch prefill (round 5).

* qg_tile_weights: bytes identical to the numpy restatement oracle.tile_weights (which
  tests/test_tiled_layout.py pins to the per-block placement formula on CPU), every format, ragged N
  and K/32 not a multiple of 4;
* qg_debug_sumi_tiled runs the instantiation qg_gemm_w4a8_tiled launches (qg_debug_config_tiled
  names the same kernel for both) and every block's int32 dot equals the reference's inner loop
  (include/gemm_reference.h:202-212) — bit-exact — for every format and the tile configurations the
  dispatch picks (32 x 16 tiles with 12 waves, 16-row tiles, 32 x 32 tiles with 8 and 4 waves), with
  and without activation windows (odd K/32);
* qg_gemm_w4a8_tiled within the MFMA kernel's reassociation bound of the oracle (oracle.reassoc_tol);
  the padding blocks of the windowed form contribute nothing even when the caller's activation
  buffer ends exactly at its last block.
"""
import numpy as np
import pytest

from test_gpu_product import dev, host, random_blocks

pytestmark = pytest.mark.gpu

TYPES = [2, 3, 6, 7, 8]


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("n,k", [(37, 4128), (64, 4096), (16, 96), (100, 1056)])
def test_tile_weights_layout(O, qg, t, n, k):
    _, bq = random_blocks(np.random.default_rng(n + k + t), 1, n, k, t)
    bt = host(qg.tile_weights(dev(bq), n, k, t))
    assert np.array_equal(bt, O.tile_weights(bq, t))


SHAPES = [
    (1, 4096, 4096),   # configs[1] on the tiled layout: the tiled decode GEMV (round 6: 16 rows x 4 stages per wave)
    (1, 300, 4128),    # decode GEMV, odd K/32 (padding blocks), ragged N
    (1, 32000, 1024),  # decode GEMV, many row tiles (linear order)
    (1, 4096, 14336),  # decode GEMV, 2 stages per lane, 14 waves
    (2, 300, 4128),    # M = 2 (K/32 <= 256): the tiled decode GEMV too, padding blocks
    (2, 32000, 1024),  # M = 2, many row tiles (linear order)
    (4, 300, 4128),    # M = 3..4 (and 2 at K/32 > 256): the MFMA small-batch decode (qg_gemvm.hip)
    (3, 32000, 1024),  # ... many half tiles (linear order)
    (2, 4096, 14336),  # ... M = 2 at the reference's batch-decode K
    (4, 64, 160),      # ... one wave per workgroup (no cross-wave sum), stages past K/32
    (32, 4096, 4096),  # configs[2]: 32 x 16 tiles, 12 waves, one dispatch round
    (5, 4096, 4096),   # 16-row tiles
    (16, 1000, 512),   # 16-row tiles, ragged N (one half-filled 32-row tile)
    (64, 4096, 1024),  # 32 x 32 tiles, 8 waves
    (96, 4096, 512),   # 32 x 32 tiles, 4 waves
    (1, 64, 128),      # one token
    (32, 4096, 4128),  # odd K/32: activation windows
    (7, 40, 96),       # K/32 = 3 < one stage, windows, ragged N
    (33, 300, 1056),   # windows, ragged M and N
]


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("m,n,k", SHAPES)
def test_tiled_sumi_and_output(O, qg, t, m, n, k):
    assert qg.debug_config_tiled(m, n, k, t) == qg.debug_config_tiled(m, n, k, t, sumi=True)
    cfg = qg.debug_config_tiled(m, n, k, t)
    gemvm = m in (3, 4) or (m == 2 and k // 32 > 256)
    if gemvm:  # the MFMA small-batch decode
        assert cfg.startswith("gemvm ") and " TA=0 " in cfg, cfg
    elif m <= 4:  # the tiled decode GEMV: per-block terms bit-identical to the oracle's
        assert cfg.startswith("gemvt ") and " TA=0 " in cfg, cfg
    else:
        assert "LAY=1" in cfg and f"AW={int((k // 32) % 4 != 0)}" in cfg, cfg
    aq, bq = random_blocks(np.random.default_rng(m * 7 + n + k + t), m, n, k, t)
    bt = qg.tile_weights(dev(bq), n, k, t)
    got = host(qg.debug_sumi_tiled(dev(aq), bt, m, n, k, t))
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)
    c = host(qg.gemm_w4a8_tiled(dev(aq), bt, m, n, k, t))
    tol = O.summation_tol(aq, bq, want, t) if m <= 4 and not gemvm else O.reassoc_tol(aq, bq, want, t, waves=16)
    err = np.abs(c.astype(np.float64) - c_ref)
    assert (err <= tol).all(), f"max err {err.max()}"


@pytest.mark.parametrize("t", [2, 8])
def test_tiled_windows_at_buffer_end(O, qg, t):
    """Odd K/32, the activations in a buffer that ends exactly at the last token's last block: the
    windows of the padding blocks read past it (zeros through the buffer resource), and the padding
    terms stay an exact +0 (outputs equal the plain-layout product to the reassociation bound, sumi
    bit-exact)."""
    import torch
    m, n, k = 17, 256, 4128
    aq, bq = random_blocks(np.random.default_rng(11 + t), m, n, k, t)
    nbytes = aq.size
    pool = torch.empty(nbytes + 4096, dtype=torch.uint8, device="cuda")
    # place the activations so that they end at the pool's end, 16-B aligned start
    start = (pool.numel() - nbytes) // 16 * 16
    a_dev = pool[start:start + nbytes]
    a_dev.copy_(torch.from_numpy(aq.reshape(-1)).to("cuda"))
    pool[start + nbytes:].fill_(0x7E)  # NaN-like f16 bytes right behind the real data
    bt = qg.tile_weights(dev(bq), n, k, t)
    c = host(qg.gemm_w4a8_tiled(a_dev, bt, m, n, k, t))
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.isfinite(c).all()
    assert (np.abs(c.astype(np.float64) - c_ref) <= O.reassoc_tol(aq, bq, want, t, waves=16)).all()
    got = host(qg.debug_sumi_tiled(a_dev, bt, m, n, k, t))
    assert np.array_equal(got, want)


def test_tiled_contract(qg):
    import ctypes
    import torch
    lib = qg._lib.load()
    assert lib.qg_tile_weights_bytes(40, 4128, 2) == 2 * 33 * 128 * 18
    assert lib.qg_tile_weights_bytes(32, 4096, 8) == 32 * 128 * 34
    assert lib.qg_tile_weights_bytes(10, 100, 2) == 0  # K % 32 != 0
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p
    a = torch.zeros(64 * 128 * 36 + 16, dtype=torch.uint8, device="cuda")
    b = torch.zeros(lib.qg_tile_weights_bytes(64, 4096, 2) + 16, dtype=torch.uint8, device="cuda")
    c = torch.zeros(64 * 64, dtype=torch.float32, device="cuda")
    # misaligned tiled weights / activations: refused, nothing launched
    assert lib.qg_gemm_w4a8_tiled(P(a.data_ptr()), P(b.data_ptr() + 8), P(c.data_ptr()), 64, 64, 4096, 2, st) == -4
    assert lib.qg_gemm_w4a8_tiled(P(a.data_ptr() + 4), P(b.data_ptr()), P(c.data_ptr()), 64, 64, 4096, 2, st) == -4
    assert lib.qg_gemm_w4a8_tiled(P(a.data_ptr()), P(b.data_ptr()), P(c.data_ptr()), 64, 64, 4100, 2, st) == -2
    assert lib.qg_gemm_w4a8_tiled(P(a.data_ptr()), P(b.data_ptr()), P(c.data_ptr()), 0, 64, 4096, 2, st) == 0
    assert lib.qg_gemm_w4a8_tiled_ldc(P(a.data_ptr()), P(b.data_ptr()), P(c.data_ptr()), 2, 64, 4096, 32, 2, st) == -1


def test_tiled_ldc_column_slice(O, qg):
    """qg_gemm_w4a8_tiled_ldc writes a column slice of a wider output and nothing else."""
    import ctypes
    import torch
    m, n, k, t = 20, 96, 512, 2
    aq, bq = random_blocks(np.random.default_rng(5), m, n, k, t)
    bt = qg.tile_weights(dev(bq), n, k, t)
    wide = torch.full((m, n + 40), -7.0, dtype=torch.float32, device="cuda")
    lib = qg._lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = dev(aq)
    P = ctypes.c_void_p
    assert lib.qg_gemm_w4a8_tiled_ldc(P(a.data_ptr()), P(bt.data_ptr()), P(wide.data_ptr() + 4 * 40), m, n, k, n + 40, t,
                                      st) == 0
    w = host(wide)
    assert (w[:, :40] == -7.0).all()
    c = host(qg.gemm_w4a8_tiled(a, bt, m, n, k, t))
    assert np.array_equal(w[:, 40:], c)


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("m,n,k", [(32, 4096, 4096), (8, 4096, 1024), (64, 2048, 2048), (20, 1000, 384)])
def test_tiled_bit_identical_to_rows(qg, t, m, n, k):
    """Same tile configuration, same per-block MFMA arithmetic and the same stage -> wave -> partial-tile
    order as the reference-row kernel: the tiled layout changes where the bytes come from, not one bit
    of the result."""
    cr, ct = qg.debug_config(m, n, k, t), qg.debug_config_tiled(m, n, k, t)
    assert cr.startswith("mmq ") and cr.replace("LAY=0", "LAY=1").split(" SIG=")[0].replace("P16=0", "P16=1") == \
        ct.split(" SIG=")[0], (cr, ct)
    aq, bq = random_blocks(np.random.default_rng(m + n + k + t), m, n, k, t)
    a, b = dev(aq), dev(bq)
    c_rows = host(qg.gemm_w4a8(a, b, m, n, k, t))
    c_tiled = host(qg.gemm_w4a8_tiled(a, qg.tile_weights(b, n, k, t), m, n, k, t))
    assert np.array_equal(c_rows.view(np.uint32), c_tiled.view(np.uint32))

