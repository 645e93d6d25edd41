"""Row-sharded multi-GPU path (quant_gemm.sharded) over gloo, world_size 2 and 3, on CPU.

The per-shard compute is injected (the oracle, standing in for the HIP kernel that needs a GPU) so
these tests cover exactly the host-side logic that is new in the build: the row partition, the
equal-size padded all-gather and the reassembly into C[M, N].
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_rows_partition():
    from quant_gemm.sharded import shard_rows
    for n, w in [(32000, 8), (4096, 1), (10, 3), (7, 8), (4097, 2)]:
        spans = [shard_rows(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
            assert a1 == b0
        assert max(b - a for a, b in spans) == (n + w - 1) // w


def _worker(rank, world, port, m, n, k, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from quant_gemm.sharded import RowShardedW4A8, shard_rows
        a, b = O.fill_uniform_step4(m, n, k, seed)
        aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, O.Q4_0)
        s0, s1 = shard_rows(n, world, rank)

        def compute(act_q, w_q, M, rows, K, out):
            out.copy_(torch.from_numpy(O.gemm_w4a8(act_q.numpy(), w_q.numpy(), O.Q4_0)))

        mod = RowShardedW4A8(torch.from_numpy(bq[s0:s1].copy()), n, k, 2, compute=compute)
        c = mod.forward(torch.from_numpy(aq), m)
        q.put((rank, c.numpy().copy(), O.gemm_w4a8(aq, bq, O.Q4_0)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,m,n,k", [(2, 1, 64, 256), (2, 3, 33, 512), (3, 2, 50, 256)])
def test_row_sharded_gather_gloo(world, m, n, k):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, m, n, k, 42, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, c, ref in res:
        # every rank holds the full C; each element computed by exactly one rank with the
        # oracle's own order -> bit-identical to the single-process result
        assert c.shape == (m, n)
        assert np.array_equal(c, ref)


def _group_worker(rank, world, port, m, n, k, q):
    """Several sharded products (G independent weight matrices sharing the activations) computed
    with RowShardedW4A8.compute_local_group (an injected compute: the products run in turn) and
    gathered with ONE all-gather of the [G, M, rows] slices, as bench.py's N > 1 legs do."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from quant_gemm.sharded import RowShardedW4A8, shard_rows
        G = 3
        a, _ = O.fill_uniform_step4(m, 0, k, 5)
        aq = O.quantize(a, O.Q8_1)
        bqs = [O.quantize(O.fill_uniform_step4(0, n, k, 10 + g)[1], O.Q4_0) for g in range(G)]
        s0, s1 = shard_rows(n, world, rank)

        def compute(act_q, w_q, M, rows, K, out):
            out.copy_(torch.from_numpy(O.gemm_w4a8(act_q.numpy(), w_q.numpy(), O.Q4_0)))

        mods = [RowShardedW4A8(torch.from_numpy(b[s0:s1].copy()), n, k, 2, compute=compute) for b in bqs]
        outs = torch.zeros((G, m, mods[0].rows), dtype=torch.float32)
        RowShardedW4A8.compute_local_group(mods, torch.from_numpy(aq), m, outs)
        gathered = torch.empty((world, G, m, mods[0].rows), dtype=torch.float32)
        mods[0].gather(outs, gathered)
        res = [RowShardedW4A8.assemble(gathered[:, g], n).numpy().copy() for g in range(G)]
        q.put((rank, res, [O.gemm_w4a8(aq, b, O.Q4_0) for b in bqs]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,m,n,k", [(2, 1, 64, 256), (3, 2, 50, 256)])
def test_row_sharded_group_gather_gloo(world, m, n, k):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, world, port, m, n, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, cs, refs in res:
        for c, ref in zip(cs, refs):
            assert c.shape == (m, n) and np.array_equal(c, ref)


def _fail_worker(rank, world, port, m, n, k, bad, q):
    """Rank `bad`'s own compute raises (a rank-local failure, e.g. its kernel launch): it must still take
    part in the all-gather with a NaN slice and raise afterwards; every peer returns C with NaN exactly in
    the failing rank's columns and the right values elsewhere."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from quant_gemm.sharded import RowShardedW4A8, ShardComputeError, shard_rows
        a, b = O.fill_uniform_step4(m, n, k, 7)
        aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, O.Q4_0)
        s0, s1 = shard_rows(n, world, rank)

        def compute(act_q, w_q, M, rows, K, out):
            if rank == bad:
                raise RuntimeError("injected rank-local failure (status -5)")
            out.copy_(torch.from_numpy(O.gemm_w4a8(act_q.numpy(), w_q.numpy(), O.Q4_0)))

        mod = RowShardedW4A8(torch.from_numpy(bq[s0:s1].copy()), n, k, 2, compute=compute)
        try:
            c = mod.forward(torch.from_numpy(aq), m)
            status = 0
        except ShardComputeError as e:
            c, status = None, str(e)
        # every rank also learns the others' status the usual way (an all-reduce of the return codes)
        flag = torch.tensor([0 if status == 0 else 1 << rank], dtype=torch.int64)
        dist.all_reduce(flag)
        q.put((rank, status, None if c is None else c.numpy().copy(), None if c is None else mod.failed_ranks(c),
               int(flag.item()), O.gemm_w4a8(aq, bq, O.Q4_0)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,m,n,k,bad", [(2, 1, 64, 256, 1), (2, 2, 33, 256, 0), (3, 1, 50, 256, 1)])
def test_row_sharded_rank_local_failure_gloo(world, m, n, k, bad):
    from quant_gemm.sharded import shard_rows
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, m, n, k, bad, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]  # a hang in the collective would time out here
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s0, s1 = shard_rows(n, world, bad)
    for rank, status, c, failed, flag, ref in res:
        assert flag == 1 << bad
        if rank == bad:
            assert isinstance(status, str) and "injected rank-local failure" in status and c is None
            continue
        assert status == 0 and failed == [bad]
        assert np.isnan(c[:, s0:s1]).all()
        keep = np.ones(n, dtype=bool)
        keep[s0:s1] = False
        assert np.array_equal(c[:, keep], ref[:, keep])


# ------------------------------------------------------------------ native path (libqg_shard.so)
SHARD_HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "qg", "qg_shard.h")


def shard_declared():
    import re
    src = re.sub(r"/\*.*?\*/", "", open(SHARD_HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(qg_\w+)\s*\(", src, flags=re.M)))


def test_native_shard_library_exports_header():
    """libqg_shard.so (RCCL) loads without a GPU and exports every function qg_shard.h declares;
    the ctypes table binds exactly those."""
    import subprocess
    import re
    from quant_gemm import sharded
    lib = sharded.shard_lib()
    fns = shard_declared()
    assert "qg_sharded_gemm_w4a8" in fns and "qg_shard_comm_init_rank" in fns
    for f in fns:
        assert hasattr(lib, f), f
    path = os.path.join(os.path.dirname(sharded.__file__), "libqg_shard.so")
    nm = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    assert set(fns) <= set(re.findall(r" T (qg_\w+)", nm))
    need = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    assert "librccl" in need and "libqg_hip.so" in need


@pytest.mark.parametrize("n", [1, 7, 4096, 4097, 32000, 32001])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_native_shard_rows_match_python(n, world):
    from quant_gemm import sharded
    for r in range(world):
        assert sharded.native_shard_rows(n, world, r) == sharded.shard_rows(n, world, r)


def test_native_shard_validation_without_launch():
    """Status codes returned before any HIP / RCCL call (no GPU needed)."""
    import ctypes
    from quant_gemm import sharded
    lib = sharded.shard_lib()
    P = ctypes.c_void_p
    a = (ctypes.c_uint8 * 64)()
    rc = lib.qg_sharded_gemm_w4a8(P(ctypes.addressof(a)), P(ctypes.addressof(a)), P(ctypes.addressof(a)), 1, 8, 64,
                                  2, None, 0, None, None)
    assert rc == -1  # no communicator
    assert lib.qg_shard_rows(10, 0, 0, ctypes.byref(ctypes.c_int()), ctypes.byref(ctypes.c_int())) == -1
    assert lib.qg_shard_rows(10, 2, 2, ctypes.byref(ctypes.c_int()), ctypes.byref(ctypes.c_int())) == -1
    assert lib.qg_sharded_gemm_workspace_size(1, 32000, 8) == 0          # in place
    assert lib.qg_sharded_gemm_workspace_size(1, 32001, 8) == 8 * 4001 * 4
    assert lib.qg_sharded_gemm_workspace_size(3, 4096, 2) == 2 * 3 * 2048 * 4
    assert lib.qg_shard_comm_init_rank(None, 1, None, 0) == -1
