"""Row-sharded multi-GPU W4A8 GEMV/GEMM — one process per GPU.

The output rows N (weight rows) are independent: C[:, n] depends only on B[n, :] and the
replicated activations. Each rank keeps a contiguous row range of B resident in its HBM, runs
the HIP kernel on it, and the slices are assembled with ONE all-gather (RCCL over xGMI when the
process group is ``nccl``; gloo in the CPU tests). The reference has no multi-GPU code at all;
this is new, MI355X-first.

Shards are equal-sized (the last one zero-padded when N % world != 0) so the gather is a single
``all_gather_into_tensor`` of contiguous [M, rows_per_rank] fp32 slices; the gathered buffer is
[world, M, rows_per_rank] and C is a strided view of it (no extra copy unless asked).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def shard_rows(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, stop) of rank's rows with equal per-rank capacity ceil(N / world)."""
    per = (n_total + world - 1) // world
    start = min(rank * per, n_total)
    return start, min(start + per, n_total)


def rows_per_rank(n_total: int, world: int) -> int:
    return (n_total + world - 1) // world


class RowShardedW4A8:
    """C[M, N] = A_q8_1[M, K] . B[N, K]^T with B row-sharded over the process group.

    ``weight_q_local``: this rank's rows [stop - start, K/32, block_bytes] (uint8, on this rank's
    device). ``compute(act_q, w_q, M, rows, K, out)`` writes out[M, rows]; by default it is the
    HIP kernel (``quant_gemm.gemm_w4a8``) — the CPU tests inject a host function to exercise the
    partition/gather logic over gloo.
    """

    def __init__(self, weight_q_local: torch.Tensor, n_total: int, K: int, wtype: int = 2,
                 group: Optional[dist.ProcessGroup] = None,
                 compute: Optional[Callable[..., None]] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n_total, self.K, self.wtype = n_total, K, wtype
        self.start, self.stop = shard_rows(n_total, self.world, self.rank)
        self.rows = rows_per_rank(n_total, self.world)
        local = self.stop - self.start
        if weight_q_local.shape[0] != local:
            raise RuntimeError(f"rank {self.rank}: expected {local} weight rows, got {weight_q_local.shape[0]}")
        self.weight = weight_q_local
        self._default = compute is None
        if compute is None:
            import quant_gemm

            def compute(act_q, w_q, M, rows, K, out):
                quant_gemm.gemm_w4a8(act_q, w_q, M, rows, K, wtype, out=out)
        self.compute = compute

    def local_out(self, M: int) -> torch.Tensor:
        return torch.zeros((M, self.rows), dtype=torch.float32, device=self.weight.device)

    def gather_buffer(self, M: int) -> torch.Tensor:
        return torch.empty((self.world, M, self.rows), dtype=torch.float32, device=self.weight.device)

    def compute_local(self, act_q: torch.Tensor, M: int, out: torch.Tensor) -> torch.Tensor:
        """out[M, rows]: this rank's slice. A ragged last shard (local < rows) writes the column
        view out[:, :local] — rows strided by ``rows`` floats, which the HIP entry point takes as
        its output row stride (qg_gemm_w4a8_ldc); the padding columns keep their contents."""
        local = self.stop - self.start
        if local > 0:
            self.compute(act_q, self.weight, M, local, self.K, out[:, :local] if local < self.rows else out)
        return out

    @staticmethod
    def compute_local_group(mods: "list[RowShardedW4A8]", act_q: torch.Tensor, M: int, outs: torch.Tensor) -> torch.Tensor:
        """outs[i] = mods[i].compute_local(act_q, M, outs[i]) for several sharded products of one K
        and weight type on this rank (e.g. a batch of independent projections sharing the
        activations): with the default HIP compute, ONE grouped launch (qg_gemm_w4a8_grouped,
        bit-identical outputs) instead of one launch per product; an injected compute runs them in
        turn. outs: [len(mods), M, rows]."""
        if not all(m._default and m.K == mods[0].K and m.wtype == mods[0].wtype and m.start == mods[0].start
                   and m.stop == mods[0].stop for m in mods):
            for m, o in zip(mods, outs):
                m.compute_local(act_q, M, o)
            return outs
        import quant_gemm
        local = mods[0].stop - mods[0].start
        if local > 0:
            quant_gemm.gemm_w4a8_grouped([act_q] * len(mods), [m.weight for m in mods], [local] * len(mods), M,
                                         mods[0].K, mods[0].wtype, outs=[o[:, :local] for o in outs])
        return outs

    def gather(self, out: torch.Tensor, gathered: torch.Tensor, async_op: bool = False):
        """One all-gather of every rank's ``out`` (any leading dims, e.g. [G, M, rows] for G
        independent products) into ``gathered`` [world, *out.shape]."""
        if self.world == 1:
            gathered[0].copy_(out)
            return None
        return dist.all_gather_into_tensor(gathered.view(-1), out.contiguous().view(-1), group=self.group,
                                           async_op=async_op)

    @staticmethod
    def assemble(gathered: torch.Tensor, n_total: int) -> torch.Tensor:
        """[world, M, rows] -> C[M, n_total] (rank-major row order = global row order)."""
        world, M, rows = gathered.shape
        return gathered.permute(1, 0, 2).reshape(M, world * rows)[:, :n_total]

    def forward(self, act_q: torch.Tensor, M: int) -> torch.Tensor:
        out = self.local_out(M)
        self.compute_local(act_q, M, out)
        g = self.gather_buffer(M)
        self.gather(out, g)
        return self.assemble(g, self.n_total)
