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
        """C[M, n_total] on every rank. Collective safety (as libqg_shard.so, include/qg/qg_shard.h): a
        failure of this rank's own compute does not skip the all-gather — the rank contributes a quiet-NaN
        slice, takes part in the collective and raises ShardComputeError afterwards, so its peers return
        (with NaN in this rank's columns, ``failed_ranks`` names them) instead of waiting forever."""
        out = self.local_out(M)
        err = None
        try:
            self.compute_local(act_q, M, out)
        except Exception as e:  # noqa: BLE001  (any rank-local failure: re-raised after the collective)
            out.fill_(float("nan"))
            err = e
        g = self.gather_buffer(M)
        self.gather(out, g)
        if err is not None:
            raise ShardComputeError(f"rank {self.rank}: local compute failed ({err!r}); its slice was sent as NaN") from err
        return self.assemble(g, self.n_total)

    def failed_ranks(self, C: torch.Tensor) -> list:
        """Ranks whose columns of a forward() result are NaN (a peer's rank-local failure)."""
        bad = []
        for r in range(self.world):
            s0, s1 = shard_rows(self.n_total, self.world, r)
            if s1 > s0 and bool(torch.isnan(C[:, s0:s1]).all()):
                bad.append(r)
        return bad


class ShardComputeError(RuntimeError):
    """This rank's own part of a sharded product failed; the collective still ran (peers hold NaN)."""


# ---------------------------------------------------------------------------------------------
# Native path: libqg_shard.so (include/qg/qg_shard.h) — the rank's kernel and ONE ncclAllGather
# over the caller's RCCL communicator, stream-ordered inside the C library (what a C++ caller such as
# llama.cpp links). The communicator is created here from a 128-byte RCCL unique id that rank 0 makes
# and the process group broadcasts (gloo or nccl); the GEMM call itself never creates one.
_shard_lib = None


def shard_lib():
    """ctypes handle of libqg_shard.so (next to libqg_hip.so); raises if it is not built."""
    global _shard_lib
    if _shard_lib is None:
        import ctypes
        import os

        from . import _lib as L
        L.load()  # libqg_hip.so first: libqg_shard.so resolves it next to itself
        path = os.path.join(L.HERE, "libqg_shard.so")
        if not os.path.exists(path):
            raise ImportError(f"quant_gemm: {path} not built; run `make -C {L.CSRC}`")
        lib = ctypes.CDLL(path)
        P, I, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        sig = {
            "qg_shard_rows": ([I, I, I, ctypes.POINTER(I), ctypes.POINTER(I)], I),
            "qg_sharded_gemm_workspace_size": ([I, I, I], SZ),
            "qg_sharded_gemm_w4a8": ([P, P, P, I, I, I, I, P, SZ, P, P], I),
            "qg_sharded_gemm_w4a8_local": ([P, P, P, I, I, I, I, I, I, P], I),
            "qg_shard_all_gather_f32": ([P, P, SZ, P, P], I),
            "qg_shard_get_unique_id": ([P], I),
            "qg_shard_comm_init_rank": ([ctypes.POINTER(P), I, P, I], I),
            "qg_shard_comm_destroy": ([P], I),
            "qg_shard_comm_count": ([P, ctypes.POINTER(I)], I),
            "qg_shard_comm_rank": ([P, ctypes.POINTER(I)], I),
            "qg_shard_last_nccl_error": ([], I),
        }
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes, fn.restype = args, res
        _shard_lib = lib
    return _shard_lib


def native_shard_rows(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """qg_shard_rows through the C-ABI, as [start, stop) (== shard_rows)."""
    import ctypes
    r0, rows = ctypes.c_int(), ctypes.c_int()
    rc = shard_lib().qg_shard_rows(n_total, world, rank, ctypes.byref(r0), ctypes.byref(rows))
    if rc != 0:
        raise RuntimeError(f"qg_shard_rows: status {rc}")
    return r0.value, r0.value + rows.value


class NcclComm:
    """An RCCL communicator made by the caller-side harness: rank 0's unique id is broadcast over
    ``group`` (any backend), then every rank joins with qg_shard_comm_init_rank on its current
    device. ``close()`` destroys it."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None):
        import ctypes
        lib = shard_lib()
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            rc = lib.qg_shard_get_unique_id(ctypes.c_void_p(uid.data_ptr()))
            if rc != 0:
                raise RuntimeError(f"ncclGetUniqueId failed (ncclResult {lib.qg_shard_last_nccl_error()})")
        if world > 1:
            src = uid.cuda() if dist.get_backend(group) == "nccl" else uid
            dist.broadcast(src, 0, group=group)
            uid = src.cpu()
        comm = ctypes.c_void_p()
        rc = lib.qg_shard_comm_init_rank(ctypes.byref(comm), world, ctypes.c_void_p(uid.data_ptr()), rank)
        if rc != 0:
            raise RuntimeError(f"ncclCommInitRank failed (ncclResult {lib.qg_shard_last_nccl_error()})")
        self.handle, self.world, self.rank = comm, world, rank

    def close(self) -> None:
        if self.handle:
            shard_lib().qg_shard_comm_destroy(self.handle)
            self.handle = None


class NativeRowShardedW4A8:
    """C[M, N] = A_q8_1[M, K] . B[N, K]^T through libqg_shard.so: this rank's rows (shard_rows) in
    ``weight_q_local``; ``forward`` returns the full C on every rank (one native all-gather)."""

    def __init__(self, weight_q_local: torch.Tensor, n_total: int, K: int, comm: NcclComm, wtype: int = 2):
        self.comm, self.n_total, self.K, self.wtype = comm, n_total, K, wtype
        self.start, self.stop = native_shard_rows(n_total, comm.world, comm.rank)
        if weight_q_local.shape[0] != self.stop - self.start:
            raise RuntimeError(f"rank {comm.rank}: expected {self.stop - self.start} weight rows, "
                               f"got {weight_q_local.shape[0]}")
        self.weight = weight_q_local.contiguous()
        self._ws = None

    def workspace(self, M: int) -> Optional[torch.Tensor]:
        need = shard_lib().qg_sharded_gemm_workspace_size(M, self.n_total, self.comm.world)
        if need == 0:
            return None
        if self._ws is None or self._ws.numel() * 4 < need:
            self._ws = torch.empty((need + 3) // 4, dtype=torch.float32, device=self.weight.device)
        return self._ws

    def forward(self, act_q: torch.Tensor, M: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        import ctypes
        dev = self.weight.device
        #  everything the C library would read or write through these raw pointers is checked
        # here first: a wrong M or a strided `out` would otherwise be an out-of-bounds device access
        if M < 0:
            raise RuntimeError(f"M must be >= 0, got {M}")
        if not (act_q.is_cuda and act_q.device == dev and act_q.dtype == torch.uint8 and act_q.is_contiguous()):
            raise RuntimeError("act_q must be a contiguous uint8 tensor on the weights' device")
        if act_q.numel() < M * (self.K // 32) * 36:
            raise RuntimeError(f"act_q holds {act_q.numel()} bytes, M={M} needs {M * (self.K // 32) * 36}")
        if out is None:
            out = torch.empty((M, self.n_total), dtype=torch.float32, device=dev)
        elif not (out.is_cuda and out.device == dev and out.dtype == torch.float32 and out.is_contiguous()
                  and tuple(out.shape) == (M, self.n_total)):
            raise RuntimeError(f"out must be a contiguous float32 [{M}, {self.n_total}] tensor on the weights' device")
        ws = self.workspace(M)
        P = ctypes.c_void_p
        st = P(torch.cuda.current_stream(dev).cuda_stream)
        with torch.cuda.device(dev):
            rc = shard_lib().qg_sharded_gemm_w4a8(
                P(act_q.data_ptr()), P(self.weight.data_ptr() if self.weight.numel() else 0), P(out.data_ptr()),
                M, self.n_total, self.K, self.wtype, P(ws.data_ptr() if ws is not None else 0),
                0 if ws is None else ws.numel() * 4, self.comm.handle, st)
        if rc != 0:
            raise RuntimeError(f"qg_sharded_gemm_w4a8: status {rc} (ncclResult {shard_lib().qg_shard_last_nccl_error()})")
        return out
