"""Grouped GEMV (qg_gemm_w4a8_grouped): independent A / B / C / N per item in one launch.

Bar: every item's output is bit-identical to qg_gemm_w4a8 (QG_ALGO_AUTO) on that item alone — the
grouped kernel runs the same GEMV body per row — and within the oracle's summation-order bound.
Covers mixed row counts (a decoder layer's Q / K / V with grouped-query K / V, gate / up), shared
and per-item activations, row-strided outputs (column slices of one wide buffer), items with
N = 0, more than 64 items (several launches), every weight format, M = 1..4 on the one-launch path
and M = 8 / odd K/32 on the per-item path, stream capture, and the argument checks.
"""
import ctypes

import numpy as np
import pytest

from test_gpu_product import close_to_oracle, dev, host, random_blocks

pytestmark = pytest.mark.gpu


def _case(O, rng, m, ns, k, t, shared=True):
    aqs, bqs = [], []
    a0 = None
    for n in ns:
        aq, bq = random_blocks(rng, m, n, k, t)
        if shared:
            a0 = aq if a0 is None else a0
            aq = a0
        aqs.append(aq)
        bqs.append(bq)
    return aqs, bqs


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("m", [1, 2, 3, 4])
def test_grouped_qkv_bit_identical(O, qg, t, m):
    rng = np.random.default_rng(100 + 10 * t + m)
    ns, k = [4096, 1024, 1024], 4096
    aqs, bqs = _case(O, rng, m, ns, k, t)
    a_d = dev(aqs[0])
    b_d = [dev(b) for b in bqs]
    outs = qg.gemm_w4a8_grouped([a_d] * 3, b_d, ns, m, k, t)
    for i, n in enumerate(ns):
        single = host(qg.gemm_w4a8(a_d, b_d[i], m, n, k, t))
        got = host(outs[i])
        assert np.array_equal(got.view(np.uint32), single.view(np.uint32)), f"item {i}"
        close_to_oracle(O, got, aqs[i], bqs[i], t)


@pytest.mark.parametrize("count,n,m,k,t", [(8, 4096, 1, 4096, 2), (16, 1000, 2, 2048, 6), (24, 300, 1, 1024, 3),
                                           (64, 4096, 1, 4096, 2)])
def test_grouped_uniform_item_per_xcd_order(O, qg, count, n, m, k, t):
    """Uniform groups (same N for every item, count % 8 == 0) take the 1-D item-per-XCD grid; per-item
    activations: every item's output still equals its single launch bit for bit."""
    rng = np.random.default_rng(count * 31 + n)
    items = [random_blocks(rng, m, n, k, t) for _ in range(min(count, 8))]
    a_d = [dev(items[i % len(items)][0]) for i in range(count)]
    b_d = [dev(items[i % len(items)][1]) for i in range(count)]
    outs = qg.gemm_w4a8_grouped(a_d, b_d, [n] * count, m, k, t)
    for i in range(count):
        single = host(qg.gemm_w4a8(a_d[i], b_d[i], m, n, k, t))
        assert np.array_equal(host(outs[i]).view(np.uint32), single.view(np.uint32)), f"item {i}"
    close_to_oracle(O, host(outs[0]), items[0][0], items[0][1], t)


def test_grouped_per_item_activations_strided_outputs(O, qg):
    import torch
    rng = np.random.default_rng(7)
    m, k, t = 2, 2048, 2
    ns = [300, 17, 1000, 64, 0, 5]
    aqs, bqs = _case(O, rng, m, ns, k, t, shared=False)
    wide = torch.full((m, sum(ns) + 7), float("nan"), dtype=torch.float32, device="cuda")
    offs = np.cumsum([0] + ns)
    outs = [wide[:, offs[i]:offs[i] + n] for i, n in enumerate(ns)]
    qg.gemm_w4a8_grouped([dev(a) for a in aqs], [dev(b) for b in bqs], ns, m, k, t, outs=outs)
    w = host(wide)
    for i, n in enumerate(ns):
        if n == 0:
            continue
        got = w[:, offs[i]:offs[i] + n]
        single = host(qg.gemm_w4a8(dev(aqs[i]), dev(bqs[i]), m, n, k, t))
        assert np.array_equal(got.view(np.uint32), single.view(np.uint32))
    assert np.isnan(w[:, sum(ns):]).all()  # nothing written past the last item


def test_grouped_more_than_64_items(O, qg):
    rng = np.random.default_rng(3)
    m, k, t = 1, 1024, 2
    ns = [int(x) for x in rng.integers(1, 300, 150)]
    aqs, bqs = _case(O, rng, m, ns, k, t)
    a_d = dev(aqs[0])
    b_d = [dev(b) for b in bqs]
    outs = qg.gemm_w4a8_grouped([a_d] * len(ns), b_d, ns, m, k, t)
    for i in range(0, len(ns), 7):
        single = host(qg.gemm_w4a8(a_d, b_d[i], m, ns[i], k, t))
        assert np.array_equal(host(outs[i]).view(np.uint32), single.view(np.uint32)), f"item {i}"


@pytest.mark.parametrize("m", [1, 2])
def test_grouped_mixed_config_rows(O, qg, m):
    """A group whose largest item picks another GEMV workgroup shape (M = 1, N >= 16384: 512-thread
    workgroups, qg_gemv_impl.hpp) than its small items alone: the per-row summation order is the
    same, so every item stays bit-identical to its own single launch."""
    rng = np.random.default_rng(40 + m)
    t, k = 2, 4096
    ns = [32000, 4096, 1000]
    aqs, bqs = _case(O, rng, m, ns, k, t)
    a_d = dev(aqs[0])
    b_d = [dev(b) for b in bqs]
    outs = qg.gemm_w4a8_grouped([a_d] * 3, b_d, ns, m, k, t)
    for i, n in enumerate(ns):
        single = host(qg.gemm_w4a8(a_d, b_d[i], m, n, k, t))
        assert np.array_equal(host(outs[i]).view(np.uint32), single.view(np.uint32)), f"item {i}"
    close_to_oracle(O, host(outs[2]), aqs[2], bqs[2], t)


@pytest.mark.parametrize("m,k", [(8, 4096), (1, 4128), (3, 4128), (32, 1024)])
def test_grouped_per_item_path(O, qg, m, k):
    """Shapes AUTO does not send to the GEMV (M > 4, odd K/32): items enqueued one by one, same bits."""
    rng = np.random.default_rng(m + k)
    t = 2
    ns = [256, 96]
    aqs, bqs = _case(O, rng, m, ns, k, t)
    a_d = dev(aqs[0])
    b_d = [dev(b) for b in bqs]
    outs = qg.gemm_w4a8_grouped([a_d] * 2, b_d, ns, m, k, t)
    for i, n in enumerate(ns):
        single = host(qg.gemm_w4a8(a_d, b_d[i], m, n, k, t))
        assert np.array_equal(host(outs[i]).view(np.uint32), single.view(np.uint32))


def test_grouped_graph_capture(O, qg):
    import torch
    rng = np.random.default_rng(11)
    m, k, t = 1, 4096, 2
    ns = [4096, 512, 512]
    aqs, bqs = _case(O, rng, m, ns, k, t)
    a_d = dev(aqs[0])
    b_d = [dev(b) for b in bqs]
    outs = [torch.zeros((m, n), dtype=torch.float32, device="cuda") for n in ns]
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        qg.gemm_w4a8_grouped([a_d] * 3, b_d, ns, m, k, t, outs=outs)
    torch.cuda.synchronize()
    for o in outs:
        o.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        qg.gemm_w4a8_grouped([a_d] * 3, b_d, ns, m, k, t, outs=outs)
    g.replay()
    for i, n in enumerate(ns):
        single = host(qg.gemm_w4a8(a_d, b_d[i], m, n, k, t))
        assert np.array_equal(host(outs[i]).view(np.uint32), single.view(np.uint32))


def test_grouped_argument_checks(qg):
    import torch
    lib = qg._lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    item = qg._GemvItem(0, 0, 0, 16, 0)
    arr = (qg._GemvItem * 1)(item)
    assert lib.qg_gemm_w4a8_grouped(arr, 1, 1, 4096, 2, st) == -1    # null pointers
    assert lib.qg_gemm_w4a8_grouped(arr, 1, 1, 100, 2, st) == -2     # bad K
    assert lib.qg_gemm_w4a8_grouped(arr, 1, 1, 4096, 5, st) == -3    # bad type
    assert lib.qg_gemm_w4a8_grouped(None, 0, 1, 4096, 2, st) == 0    # empty group
    arr[0] = qg._GemvItem(256, 256, 256, 16, 8)
    assert lib.qg_gemm_w4a8_grouped(arr, 1, 1, 4096, 2, st) == -1    # ldc < N
    assert lib.qg_gemm_w4a8_grouped(arr, -1, 1, 4096, 2, st) == -1


@pytest.mark.parametrize("ns", [[11008, 4096, 100], [8200, 17, 4096], [4096, 4096, 4096, 4096], [33, 1, 7]])
@pytest.mark.parametrize("t,m", [(2, 1), (2, 4), (8, 2), (7, 1)])
def test_grouped_workgroup_size_split(O, qg, ns, t, m):
    """Groups whose largest item fits one round of full-size workgroups launch half-size ones
    (qg_gemv_kernel.hpp, QG_GEMVG_WDIV), larger ones full-size: every item bit-identical to its
    single launch either way."""
    rng = np.random.default_rng(sum(ns) + 10 * t + m)
    k = 2048
    aqs, bqs = _case(O, rng, m, ns, k, t, shared=False)
    a_d = [dev(a) for a in aqs]
    b_d = [dev(b) for b in bqs]
    outs = qg.gemm_w4a8_grouped(a_d, b_d, ns, m, k, t)
    for i, n in enumerate(ns):
        single = host(qg.gemm_w4a8(a_d[i], b_d[i], m, n, k, t))
        assert np.array_equal(host(outs[i]).view(np.uint32), single.view(np.uint32)), f"item {i}"
    close_to_oracle(O, host(outs[-1]), aqs[-1], bqs[-1], t)
