"""GPU parity of the product kernels at the BASELINE shapes, the reference's own test shapes, and
the boundary cases VERDICT/ADVICE r01 named.

* int32 sumi bit-exact from the EXACT instantiations that serve configs[1..4] (the parity hook runs
  the product kernel; qg_debug_config proves it is the same instantiation);
* the reference's weight-major test shapes (python/tests/test_gemm_q4_0.py:151-156) and its
  all-quants unit default M=4 N=512 K=1024 (tests/unit/test_gemm_all_quants.cu:418-425);
* a weight tensor beyond 2 GiB on the MFMA prefill (64-bit DMA bases);
* the W4A16 split-K workspace shared by alternating shapes on one stream;
* the row-sharded module with its default HIP compute, ragged N, over gloo ranks sharing the GPU.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FULL = [(1, 4096, 4096), (2, 4096, 4096), (3, 4096, 4096), (4, 4096, 4096), (8, 4096, 4096), (32, 4096, 4096)]


def dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def close_to_oracle(O, c, aq, bq, t, mfma=None):
    """mfma: the MFMA prefill served it (oracle.reassoc_tol; see test_gpu_parity.assert_close_to_oracle)."""
    c_ref, s = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    if mfma is None:  # auto dispatch: the family the product picks for this shape
        import quant_gemm
        mfma = quant_gemm.select_algo(aq.shape[0], bq.shape[0], 32 * aq.shape[1], t) == 2
    tol = O.reassoc_tol(aq, bq, s, t) if mfma else O.summation_tol(aq, bq, s, t)
    err = np.abs(c.astype(np.float64) - c_ref)
    assert (err <= tol).all(), f"max err {err.max()}"


def random_blocks(rng, m, n, k, t):
    nb, bb = k // 32, {2: 18, 3: 20, 6: 22, 7: 24, 8: 34}[t]
    aq = rng.integers(0, 256, (m, nb, 36), dtype=np.uint8)
    bq = rng.integers(0, 256, (n, nb, bb), dtype=np.uint8)
    f16 = lambda lo, hi, shape: rng.uniform(lo, hi, shape).astype(np.float16).view(np.uint8).reshape(shape + (2,))
    aq[..., 0:2] = f16(1e-3, 2e-2, (m, nb))
    aq[..., 2:4] = f16(-5.0, 5.0, (m, nb))
    bq[..., 0:2] = f16(-0.1, 0.1, (n, nb))
    if t in (3, 7):
        bq[..., 2:4] = f16(-0.5, 0.5, (n, nb))
    return aq, bq


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("m,n,k", FULL)
def test_product_kernel_sumi_full_size(O, qg, t, m, n, k):
    """configs[1] (M=1), the M=2..4 GEMV forms, M=8 and configs[2] (M=32) prefill: every block's
    int32 dot from the product instantiation equals the reference's inner loop
    (include/gemm_reference.h:202-212), on quantized step4 data and on raw random bytes."""
    assert qg.debug_config(m, n, k, t) == qg.debug_config(m, n, k, t, sumi=True)
    a, b = O.fill_uniform_step4(m, n, k, 42)
    cases = [(O.quantize(a, O.Q8_1), O.quantize(b, t)), random_blocks(np.random.default_rng(m * 10 + t), m, n, k, t)]
    for aq, bq in cases:
        got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t))
        c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
        c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
        assert np.array_equal(got, want)
        mfma = qg.select_algo(m, n, k, t) == 2  # M = 8 / 32: the MFMA prefill (oracle.reassoc_tol)
        tol = O.reassoc_tol(aq, bq, want, t) if mfma else O.summation_tol(aq, bq, want, t)
        assert (np.abs(c.astype(np.float64) - c_ref) <= tol).all()


@pytest.mark.parametrize("t,sym", [(2, "gemm_q4_0_q8_1"), (3, "gemm_q4_1_q8_1"), (6, "gemm_q5_0_q8_1"),
                                   (7, "gemm_q5_1_q8_1"), (8, "gemm_q8_0_q8_1")])
@pytest.mark.parametrize("mw,ntok,k", [(1, 1, 32), (4, 2, 1024), (128, 8, 4096), (4096, 2, 14336)])
def test_reference_weight_major_shapes(O, qg, t, sym, mw, ntok, k):
    """python/tests/test_gemm_q4_0.py:151-156: gemm_q4_0_q8_1(weight_q, activation_q, M, N, K) with
    (M, N, K) = (1,1,32), (4,2,1024), (128,8,4096), (4096,2,14336) -> out[M_w, N_tok]."""
    import torch
    gen = torch.Generator(device="cuda")
    gen.manual_seed(mw + ntok + k)
    w = torch.randn((mw, k), generator=gen, device="cuda")
    a = torch.randn((ntok, k), generator=gen, device="cuda")
    wq, aq = qg.quantize(w, t), qg.quantize_q8_1(a)
    out = getattr(qg, sym)(wq, aq, mw, ntok, k)
    assert tuple(out.shape) == (mw, ntok)
    close_to_oracle(O, np.ascontiguousarray(host(out).T), host(aq), host(wq), t)
    # the reference test's own bar: relative error vs the FP32 product of the dequantized inputs
    ref = a.double() @ qg.dequantize(wq, t).reshape(mw, k).double().T
    rel = float(torch.linalg.norm(out.T.double() - ref) / torch.linalg.norm(ref))
    assert rel < 0.05, rel


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
def test_reference_allquants_unit_default(O, qg, t):
    """tests/unit/test_gemm_all_quants.cu:418-425 default M=4, N=512, K=1024, every format, both
    conventions (activation-major and the weight-major gemm_q*_q8_1 twin)."""
    m, n, k = 4, 512, 1024
    a, b = O.fill_uniform_step4(m, n, k, 42)
    aq, bq = O.quantize(a, O.Q8_1, 1), O.quantize(b, t)  # the unit test's framework quantizers
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    close_to_oracle(O, c, aq, bq, t)
    sym = {2: "gemm_q4_0_q8_1", 3: "gemm_q4_1_q8_1", 6: "gemm_q5_0_q8_1", 7: "gemm_q5_1_q8_1", 8: "gemm_q8_0_q8_1"}[t]
    wm = host(getattr(qg, sym)(dev(bq), dev(aq), n, m, k))
    assert np.array_equal(wm.T, c)
    for algo in (2, 3):
        close_to_oracle(O, host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=algo)), aq, bq, t, mfma=algo == 2)


def test_mfma_weights_beyond_2gib(O, qg):
    """Q8_0 weights N=70000, K=32768: 2.44 GB in one tensor on the MFMA prefill (M=16). Rows on both
    sides of the 2 GiB byte offset are checked against the oracle."""
    import torch
    m, n, k = 16, 70000, 32768
    nb, bb = k // 32, 34
    assert n * nb * bb > 2 ** 31
    assert qg.select_algo(m, n, k, 8) == 2
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    bq = torch.randint(0, 256, (n, nb, bb), generator=gen, device="cuda", dtype=torch.uint8)
    scales = (torch.rand((n, nb), generator=gen, device="cuda") * 0.02 + 0.001).half()
    bq[:, :, 0:2] = scales.view(torch.uint8).view(n, nb, 2)
    aq = qg.quantize_q8_1(torch.rand((m, k), generator=gen, device="cuda") * 2 - 1)
    c = host(qg.gemm_w4a8(aq, bq, m, n, k, 8))
    first_far = (2 ** 31) // (nb * bb) + 1  # first row whose bytes lie wholly beyond 2 GiB
    rows = np.r_[0:40, first_far - 40:first_far + 40, n - 40:n]
    sub = host(bq[torch.from_numpy(rows).cuda()])
    close_to_oracle(O, np.ascontiguousarray(c[:, rows]), host(aq), sub, 8, mfma=True)


def test_w16_split_k_workspace_alternating_shapes(O, qg):
    """(32, 4096, 4096) and (32, 11008, 4096) alternating on one stream, through
    the library's stream workspace and through one caller workspace sized for the larger shape:
    every call equals a fresh single call bit for bit."""
    import ctypes
    import torch
    k = 4096
    lib = qg._lib.load()
    a, _ = O.fill_uniform_step4(32, 1, k, 3)
    shapes = [4096, 11008]
    ws_bytes = max(lib.qg_gemm_w16_workspace_size(32, n, k) for n in shapes)
    assert ws_bytes > 0
    ad = dev(a)
    wq = {}
    for n in shapes:
        _, b = O.fill_uniform_step4(1, n, k, n)
        wq[n] = (b, O.quantize(b, 2), dev(O.quantize(b, 2)))
    first = {n: host(qg.gemm_w4a16(ad, wq[n][2], 32, n, k)) for n in shapes}
    for n in shapes:
        rows = np.r_[0:64, n - 64:n]
        ref = O.gemm_w4a16(a, wq[n][1][rows])
        tol = O.w16_tol(a, wq[n][1][rows], 2)
        assert (np.abs(first[n][:, rows].astype(np.float64) - ref) <= tol).all()
    for _ in range(3):
        for n in shapes:
            assert np.array_equal(host(qg.gemm_w4a16(ad, wq[n][2], 32, n, k)), first[n])
    ws = torch.zeros(ws_bytes // 4, dtype=torch.int32, device="cuda")
    P = ctypes.c_void_p
    st = P(torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        for n in shapes:
            c = torch.empty((32, n), dtype=torch.float32, device="cuda")
            assert lib.qg_gemm_w4a16_ws(P(ad.data_ptr()), P(wq[n][2].data_ptr()), P(c.data_ptr()), 32, n, k,
                                        P(ws.data_ptr()), ws_bytes, st) == 0
            assert np.array_equal(host(c), first[n])
    assert int(ws[:1024].abs().sum()) == 0  # the counter region is left zeroed


def test_gemm_w4a8_strided_out(O, qg):
    """qg_gemm_w4a8_ldc: a column slice of a wider buffer as the destination (M > 1), padding
    columns untouched, every family."""
    import torch
    for m, n, k, algo in [(3, 130, 4096, 1), (24, 130, 2048, 2), (3, 130, 1024, 3)]:
        a, b = O.fill_uniform_step4(m, n, k, 9)
        aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, 2)
        big = torch.full((m, n + 7), -7.0, device="cuda")
        qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, algo=algo, out=big[:, :n])
        got = host(big)
        assert (got[:, n:] == -7.0).all()
        close_to_oracle(O, np.ascontiguousarray(got[:, :n]), aq, bq, 2, mfma=algo == 2)
        assert np.array_equal(got[:, :n], host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, algo=algo)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_worker(rank, world, port, m, n, k, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import quant_gemm as qg
        from quant_gemm.sharded import RowShardedW4A8, shard_rows
        torch.cuda.set_device(0)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(21)
        aq = qg.quantize_q8_1(torch.rand((m, k), generator=gen, device="cuda") * 2 - 1)
        bq = qg.quantize_q4_0(torch.rand((n, k), generator=gen, device="cuda") * 2 - 1)
        s0, s1 = shard_rows(n, world, rank)
        mod = RowShardedW4A8(bq[s0:s1].contiguous(), n, k, 2)  # default compute: the HIP kernel
        out = mod.local_out(m)
        mod.compute_local(aq, m, out)
        torch.cuda.synchronize()
        g = torch.empty((world, m, mod.rows), dtype=torch.float32)
        mod.gather(out.cpu(), g)  # gloo gathers host tensors
        c = mod.assemble(g, n)
        full = qg.gemm_w4a8(aq, bq, m, n, k)
        q.put((rank, bool(torch.equal(c, full.cpu())), None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, False, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("m", [1, 3])
def test_row_sharded_default_hip_compute(qg, m):
    """quant_gemm.sharded.RowShardedW4A8 with its default compute (the HIP kernel) on ragged N=4097:
    world 1, and 2 gloo ranks sharing the GPU (rank 1 writes a strided column slice when M > 1);
    the reassembled C equals one single-GPU gemm_w4a8 bit for bit (VERDICT r01 missing #1, weak #6)."""
    import torch
    import torch.multiprocessing as mp
    from quant_gemm.sharded import RowShardedW4A8
    n, k = 4097, 4096
    gen = torch.Generator(device="cuda")
    gen.manual_seed(21)
    aq = qg.quantize_q8_1(torch.rand((m, k), generator=gen, device="cuda") * 2 - 1)
    bq = qg.quantize_q4_0(torch.rand((n, k), generator=gen, device="cuda") * 2 - 1)
    mod = RowShardedW4A8(bq, n, k, 2)
    assert torch.equal(mod.forward(aq, m), qg.gemm_w4a8(aq, bq, m, n, k))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, m, n, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
    for rank, ok, err in res:
        assert ok, (rank, err)


# Odd K / 32 (every other weight row 2 bytes off dword alignment for Q4_0 / Q5_0 / Q8_0) and 2-B
# aligned weight tensors: the one-wave-per-weight-row kernel (qg_ragged.hip)
# instead of the byte-load generic kernel's one wave per output.
RAGGED = [(1, 4096, 4128), (3, 100, 4128), (9, 64, 1056), (32, 130, 4128), (1, 33, 32), (17, 50, 96), (5, 7, 14368)]


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("m,n,k", RAGGED)
def test_ragged_odd_blocks(O, qg, t, m, n, k):
    """Auto dispatch takes the ragged kernel for odd K/32; int32 sumi bit-exact through the product
    instantiation, outputs within the summation bound, and the explicit generic kernel agrees."""
    if (k // 32) % 2 == 1:
        assert qg.select_algo(m, n, k, t) == 4
        assert qg.debug_config(m, n, k, t).startswith("ragged ")
    assert qg.debug_config(m, n, k, t, algo=4) == qg.debug_config(m, n, k, t, algo=4, sumi=True)
    aq, bq = random_blocks(np.random.default_rng(m * 31 + n + t), m, n, k, t)
    got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t, algo=4))
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    tol = O.summation_tol(aq, bq, want, t)
    assert (np.abs(c.astype(np.float64) - c_ref) <= tol).all()
    cg = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=3))
    assert (np.abs(cg.astype(np.float64) - c_ref) <= tol).all()


REPACK = [(32, 1100, 4128), (32, 1024, 1056), (40, 1536, 96), (64, 1030, 4128)]


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
@pytest.mark.parametrize("m,n,k", REPACK)
def test_repack_mfma_odd_blocks(O, qg, t, m, n, k):
    """Odd K/32 at prefill sizes (M >= 32, N >= 1024): the MFMA kernel on a zero-padded copy
    (qg_repack.hip). The sumi hook runs that instantiation (padded image compacted to [M][N][K/32])
    and is bit-exact; outputs sit within the summation bound and agree with the ragged kernel's."""
    assert qg.select_algo(m, n, k, t) == 2
    prod = qg.debug_config(m, n, k, t)
    assert prod.startswith("mmq ") and prod == qg.debug_config(m, n, k, t, sumi=True)
    aq, bq = random_blocks(np.random.default_rng(m * 7 + n + k + t), m, n, k, t)
    got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t))
    c_ref, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    tol = O.reassoc_tol(aq, bq, want, t)
    assert (np.abs(c.astype(np.float64) - c_ref) <= tol).all()
    c_rag = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=4))
    assert (np.abs(c_rag.astype(np.float64) - c_ref) <= O.summation_tol(aq, bq, want, t)).all()
    # twice more on the same stream (workspace reused): bit-identical
    assert np.array_equal(host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t)), c)


def test_repack_two_byte_aligned_weights(O, qg):
    """2-B aligned weight tensor at a prefill size: the repack takes it too (Q4_0, even K/32)."""
    import torch
    m, n, k, t = 32, 1024, 4096, 2
    aq, bq = random_blocks(np.random.default_rng(5), m, n, k, t)
    raw = torch.zeros(bq.size + 2, dtype=torch.uint8, device="cuda")
    raw[2:] = dev(bq.ravel())
    bmis = raw[2:].view(bq.shape)
    c_mis = host(qg.gemm_w4a8(dev(aq), bmis, m, n, k, t))
    c_al = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    close_to_oracle(O, c_mis, aq, bq, t)
    close_to_oracle(O, c_al, aq, bq, t)


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
def test_ragged_two_byte_aligned_weights(O, qg, t):
    """A weight tensor starting 2 bytes past a dword (even K/32 too): GEMV / MFMA decline it, the
    ragged kernel takes it, bit-identical to the same bytes at an aligned address."""
    import torch
    m, n, k = 4, 300, 4096
    aq, bq = random_blocks(np.random.default_rng(t), m, n, k, t)
    raw = torch.zeros(bq.size + 2, dtype=torch.uint8, device="cuda")
    raw[2:] = dev(bq.ravel())
    bmis = raw[2:].view(bq.shape)
    assert bmis.data_ptr() % 4 == 2
    c_mis = host(qg.gemm_w4a8(dev(aq), bmis, m, n, k, t))
    c_rag = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=4))
    assert np.array_equal(c_mis, c_rag)
    close_to_oracle(O, c_mis, aq, bq, t)
