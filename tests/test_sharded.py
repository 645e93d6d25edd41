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
