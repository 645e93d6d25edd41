"""W4A16 / W8A16 (FP32 activations x Q4_0 / Q8_0 weights), GPU parity through the C-ABI.

Bar: |C_gpu - C_oracle| <= 2 (K + 2) 2^-24 sum_k |a_k w_k| (oracle.w16_tol) — the fp32
summation-order bound; the reference's own Python definition outputs (tests/golden/w4a16_*.npz)
are met within the same bound; NMSE vs FP32 within the W4A8 bound.
"""
import ctypes
import glob
import os

import numpy as np
import pytest

from test_gpu_parity import GOLD, dev, host

pytestmark = pytest.mark.gpu


def check(O, c, a, bq, t, ref=None):
    ref = (O.gemm_w4a16(a, bq) if t == O.Q4_0 else O.gemm_w8a16(a, bq)) if ref is None else ref
    tol = O.w16_tol(a, bq, t)
    err = np.abs(c.astype(np.float64) - ref)
    assert (err <= tol).all(), f"max err {err.max()}"


@pytest.mark.parametrize("t", [2, 8])
@pytest.mark.parametrize("m,n,k", [(1, 300, 4096), (2, 64, 4096), (3, 130, 2048), (4, 33, 4096), (5, 40, 1024),
                                   (8, 100, 4096), (9, 64, 2048), (33, 50, 1024), (1, 70, 14336), (2, 17, 192),
                                   (3, 9, 96), (1, 5, 32)])
def test_w16_matches_oracle(O, qg, t, m, n, k):
    a, b = O.fill_uniform_step4(m, n, k, seed=m + n)
    bq = O.quantize(b, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    c = host(fn(dev(a), dev(bq), m, n, k))
    check(O, c, a, bq, t)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "w4a16_*.npz"))), ids=os.path.basename)
def test_w4a16_golden(O, qg, path):
    """The reference definition's outputs, with its interleaved dequant order undone on the
    activations (see tests/test_oracle.py::test_golden_w4a16)."""
    g = np.load(path)
    m, n, k = (int(g[x]) for x in ("m", "n", "k"))
    blk = g["a"].reshape(m, k // 32, 32)
    a = np.ascontiguousarray(np.concatenate([blk[..., 0::2], blk[..., 1::2]], axis=-1).reshape(m, k))
    c = host(qg.gemm_q4_0_fp32(dev(g["b_q"]), dev(a), m, n, k))
    check(O, c, a, g["b_q"], 2, ref=g["c_ref"].astype(np.float64))


def test_w4a16_full_size_nmse(O, qg):
    a, b = O.fill_uniform_step4(1, 4096, 4096)
    bq = O.quantize(b, 2)
    c = host(qg.gemm_w4a16(dev(a), dev(bq), 1, 4096, 4096))
    check(O, c, a, bq, 2)
    assert O.nmse(c, O.gemm_fp32(a, b)) <= 5e-3


def test_w4a16_unaligned_activation_generic_path(O, qg):
    import torch
    m, n, k = 2, 24, 1024
    a, b = O.fill_uniform_step4(m, n, k)
    bq = O.quantize(b, 2)
    raw = torch.zeros(a.size + 1, dtype=torch.float32, device="cuda")
    raw[1:] = dev(a.ravel())
    x = raw[1:]
    assert x.data_ptr() % 16 != 0
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")
    lib = qg._lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p
    assert lib.qg_gemm_w4a16(P(x.data_ptr()), P(dev(bq).data_ptr()), P(c.data_ptr()), m, n, k, st) == 0
    check(O, host(c), a, bq, 2)


# Prefill (M > 8, K % 256 == 0): the split-K kernel (w16_sk_kernel) — K slices across workgroups
# meet through the library's per-stream workspace; 16-token tiles (M <= 64) and 64-token tiles,
# 64- and 128-row workgroups, ragged M and N, several slices per chunk count.
@pytest.mark.parametrize("t", [2, 8])
@pytest.mark.parametrize("m,n,k", [(32, 4096, 4096), (17, 300, 1024), (64, 2048, 2048), (100, 256, 2048),
                                   (130, 2100, 512), (40, 640, 14336), (9, 33, 512), (65, 16, 256)])
def test_w16_prefill_split_k(O, qg, t, m, n, k):
    a, b = O.fill_uniform_step4(m, n, k, seed=m * 7 + n)
    bq = O.quantize(b, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    ad, bd = dev(a), dev(bq)
    c1 = host(fn(ad, bd, m, n, k))
    check(O, c1, a, bq, t)
    # the tile counters re-arm themselves: a second launch is bit-identical
    c2 = host(fn(ad, bd, m, n, k))
    assert np.array_equal(c1, c2)


@pytest.mark.parametrize("t", [2, 8])
@pytest.mark.parametrize("m,n,k", [(32, 512, 4096), (16, 256, 1024), (64, 384, 2048), (24, 128, 14336),
                                   (100, 256, 2048), (130, 300, 1024), (257, 64, 4096),
                                   (64, 4096, 1024), (32, 8200, 2048)])  # the last two: 32-token tiles
def test_w16_prefill_two_part_split_error(O, qg, t, m, n, k):
    """From K = 1024 the prefill (w16s_kernel, M <= 64; w16_sk_kernel beyond) splits each activation into two round-to-nearest bf16
    parts: |a - hi - mid| <= 2^-16 |a|. Against the exact (float64) product the error must stay within
    that representation error plus the fp32 accumulation's (K + 2) u share, 2^-16 + (K + 2) 2^-24 of
    sum_k |a_k w_k| (about half of the oracle-vs-kernel bound at K = 4096); a split that dropped the
    second part (2^-8 relative) would exceed it many times over."""
    rng = np.random.default_rng(m * 131 + k)
    a = (rng.standard_normal((m, k)) * np.exp2(rng.integers(-6, 7, (m, 1)))).astype(np.float32)  # full 24-bit values
    b = rng.uniform(-1, 1, (n, k)).astype(np.float32)
    bq = O.quantize(b, t)
    fn = qg.gemm_w4a16 if t == 2 else qg.gemm_w8a16
    c = host(fn(dev(a), dev(bq), m, n, k)).astype(np.float64)
    w = O.dequantize(bq, t).astype(np.float64)
    exact = a.astype(np.float64) @ w.T
    mag = np.abs(a.astype(np.float64)) @ np.abs(w).T
    bound = (2.0 ** -16 + (k + 2) * 2.0 ** -24) * mag + 1e-30
    err = np.abs(c - exact)
    assert (err <= bound).all(), f"max err / bound {(err / bound).max()}"
    check(O, c.astype(np.float32), a, bq, t)


def test_w16_prefill_split_k_second_stream(O, qg):
    """Each stream gets its own workspace; results are bit-identical across streams."""
    import torch
    m, n, k = 32, 1024, 4096
    a, b = O.fill_uniform_step4(m, n, k, seed=5)
    bq = O.quantize(b, 2)
    ad, bd = dev(a), dev(bq)
    c0 = host(qg.gemm_w4a16(ad, bd, m, n, k))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        c1 = qg.gemm_w4a16(ad, bd, m, n, k)
    s.synchronize()
    assert np.array_equal(c0, host(c1))
    check(O, c0, a, bq, 2)


@pytest.mark.parametrize("t", [2, 8])
def test_w16_prefill_caller_workspace(O, qg, t):
    """qg_gemm_w{4,8}a16_ws: the caller's zeroed workspace, left zeroed; too small -> not used."""
    import torch
    m, n, k = 24, 2048, 2048
    a, b = O.fill_uniform_step4(m, n, k, seed=t)
    bq = O.quantize(b, t)
    lib = qg._lib.load()
    need = lib.qg_gemm_w16_workspace_size(m, n, k)
    assert need > 0
    ws = torch.zeros(need // 4 + 64, dtype=torch.int32, device="cuda")
    P = ctypes.c_void_p
    st = P(torch.cuda.current_stream().cuda_stream)
    sym = lib.qg_gemm_w4a16_ws if t == 2 else lib.qg_gemm_w8a16_ws
    ad, bd = dev(a), dev(bq)
    outs = []
    for nbytes in (need, need, 64):
        c = torch.empty((m, n), dtype=torch.float32, device="cuda")
        assert sym(P(ad.data_ptr()), P(bd.data_ptr()), P(c.data_ptr()), m, n, k, P(ws.data_ptr()), nbytes, st) == 0
        torch.cuda.synchronize()
        outs.append(host(c))
        # counters re-armed: every tile counter is zero again after the launch
        assert int(ws[: (need // 4)][:16].abs().sum()) == 0
    check(O, outs[0], a, bq, t)
    assert np.array_equal(outs[0], outs[1])
    check(O, outs[2], a, bq, t)


def test_w16_library_workspace_two_threads_one_stream(O, qg):
    """two host threads on ONE stream, the second asking for a larger split-K workspace
    than the first's (the library's per-stream buffer grows: stream sync + free of the old block).
    The buffer's lock is held until each call's kernel is enqueued, so no launch can run on a freed
    block: every result equals the single-threaded one, bit for bit."""
    import threading

    import torch
    lib = qg._lib.load()
    shapes = [(40, 1024, 4096), (64, 8192, 4096)]  # M > 32: both split K (M <= 32 runs w16d, no workspace)
    need = [lib.qg_gemm_w16_workspace_size(*s) for s in shapes]
    assert need[1] > max(need[0], 4 << 20)  # the second shape must grow the buffer past its first size
    data = []
    for i, (m, n, k) in enumerate(shapes):
        a, b = O.fill_uniform_step4(m, n, k, seed=40 + i)
        bq = O.quantize(b, 2)
        ad, bd = dev(a), dev(bq)
        data.append((ad, bd, host(qg.gemm_w4a16(ad, bd, m, n, k))))
    s = torch.cuda.Stream()
    P = ctypes.c_void_p
    outs = {0: [], 1: []}
    errs = []

    def worker(i, reps):
        m, n, k = shapes[i]
        ad, bd, _ = data[i]
        try:
            for _ in range(reps):
                c = torch.empty((m, n), dtype=torch.float32, device="cuda")
                rc = lib.qg_gemm_w4a16(P(ad.data_ptr()), P(bd.data_ptr()), P(c.data_ptr()), m, n, k, P(s.cuda_stream))
                assert rc == 0
                outs[i].append(c)
        except BaseException as e:  # reported in the main thread
            errs.append(e)

    lib.qg_release_workspaces()
    th = [threading.Thread(target=worker, args=(0, 40)), threading.Thread(target=worker, args=(1, 4))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    s.synchronize()
    assert not errs, errs
    for i in (0, 1):
        assert len(outs[i]) == (40 if i == 0 else 4)
        for c in outs[i]:
            assert np.array_equal(host(c), data[i][2])


@pytest.mark.parametrize("m,k", [(16, 1024), (9, 256), (40, 2048)])
def test_w16_prefill_activations_near_flt_max(O, qg, m, k):
    """a finite activation whose bf16 rounding would overflow ((2 - 2^-8) 2^127 <= |a| <=
    FLT_MAX) keeps a finite product — the high part is clamped to the largest finite bf16 (before the
    clamp: hi = inf, mid = -inf, NaN) — and an infinite activation gives an infinite product, not NaN,
    in the three-part (K < 1024) and the two-part (K >= 1024) prefill. The kernels form each block's
    code dot sum a * (q - 8) before scaling by d, so the weights here keep |q - 8| <= 1 (every partial
    product then stays below FLT_MAX, as the reference's a * w does)."""
    rng = np.random.default_rng(m * 3 + k)
    n, nb = 64, k // 32
    a, _ = O.fill_uniform_step4(m, n, k, seed=m + k)
    a[0, 5] = np.float32(3.4e38)
    a[1, 7] = np.float32(-3.399e38)
    bq = np.zeros((n, nb, 18), np.uint8)
    bq[..., 0:2] = rng.uniform(1e-3, 0.1, (n, nb)).astype(np.float16).view(np.uint8).reshape(n, nb, 2)
    codes = rng.integers(7, 10, (n, nb, 32)).astype(np.uint8)  # q - 8 in {-1, 0, 1}
    bq[..., 2:] = codes[..., :16] | (codes[..., 16:] << 4)
    w = O.dequantize(bq, 2).astype(np.float64)
    c = host(qg.gemm_w4a16(dev(a), dev(bq), m, n, k)).astype(np.float64)
    exact = a.astype(np.float64) @ w.T
    mag = np.abs(a.astype(np.float64)) @ np.abs(w).T
    assert np.isfinite(c).all()
    bound = (2.0 ** -16 + 2 * (k + 2) * 2.0 ** -24) * mag + 1e-30
    assert (np.abs(c - exact) <= bound).all()
    a2 = a.copy()
    a2[2, 3] = np.inf
    c2 = host(qg.gemm_w4a16(dev(a2), dev(bq), m, n, k))
    nz = w[:, 3] != 0
    assert nz.sum() > 10
    assert np.isinf(c2[2, nz]).all() and (np.sign(c2[2, nz]) == np.sign(w[nz, 3])).all()
