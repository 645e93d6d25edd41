"""Native row-sharded path (libqg_shard.so over RCCL, include/qg/qg_shard.h) on the GPU.

On the one-GPU test box the communicator has one rank (the caller-side harness of
quant_gemm.sharded.NcclComm with no process group): the rank's kernel, a real ncclAllGather (in place
for M = 1 and N % world == 0, through the gather workspace + reorder kernel otherwise) and the
reorder. Outputs vs the single-GPU entry: bit-identical on the GEMV path (M <= 4), the MFMA path to
the reassociation bound of the oracle. World > 1 is exercised by the C++ driver
(tests/cpp/test_shard.cpp, one thread per visible GPU) and, at 8 GPUs, by the driver's bench run.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_close_to_oracle, dev, host, make_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(qg):
    from quant_gemm.sharded import NcclComm
    c = NcclComm()
    yield c
    c.close()


@pytest.mark.parametrize("m,n,k,t", [(1, 4096, 4096, 2), (1, 32000, 4096, 2), (3, 4097, 1024, 2), (2, 37, 256, 6),
                                     (4, 300, 2048, 3), (12, 1000, 2048, 2), (32, 4096, 4096, 2)])
def test_native_sharded_world1(O, qg, comm, m, n, k, t):
    from quant_gemm.sharded import NativeRowShardedW4A8
    _, _, aq, bq = make_case(O, m, n, k, t)
    a_d, b_d = dev(aq), dev(bq)
    mod = NativeRowShardedW4A8(b_d, n, k, comm, wtype=t)
    c = mod.forward(a_d, m)
    c2 = mod.forward(a_d, m)  # repeated call: same buffers, same bits
    single = host(qg.gemm_w4a8(a_d, b_d, m, n, k, t))
    got = host(c)
    assert np.array_equal(got, host(c2))
    if m <= 4:
        assert np.array_equal(got, single)
    assert_close_to_oracle(O, got, aq, bq, t)


def test_native_local_slice_matches_columns(O, qg):
    """qg_sharded_gemm_w4a8_local (no collective) for each of 3 ranks writes exactly that rank's
    columns of the single-GPU product, with row stride P = ceil(N / 3)."""
    import ctypes

    import torch
    from quant_gemm.sharded import shard_lib, shard_rows
    m, n, k, world = 2, 1001, 1024, 3
    _, _, aq, bq = make_case(O, m, n, k, 2)
    a_d = dev(aq)
    full = host(qg.gemm_w4a8(a_d, dev(bq), m, n, k))
    p = (n + world - 1) // world
    lib = shard_lib()
    P = ctypes.c_void_p
    for r in range(world):
        s0, s1 = shard_rows(n, world, r)
        b_r = dev(np.ascontiguousarray(bq[s0:s1]))
        out = torch.full((m, p), float("nan"), dtype=torch.float32, device="cuda")
        st = P(torch.cuda.current_stream().cuda_stream)
        assert lib.qg_sharded_gemm_w4a8_local(P(a_d.data_ptr()), P(b_r.data_ptr()), P(out.data_ptr()), m, n, k, 2,
                                              world, r, st) == 0
        got = host(out)
        assert np.array_equal(got[:, : s1 - s0], full[:, s0:s1])
        assert np.isnan(got[:, s1 - s0:]).all()  # padding columns untouched


def test_native_rank_local_errors_join_the_collective(O, qg, comm):
    """The error paths of qg_sharded_gemm_w4a8 allocate nothing and still run the one all-gather:
    M > 1 without a workspace (N % world == 0: the gather lands in C) and a null shard with rows to compute
    return their error with C all NaN; the stream stays usable and the next good call is exact."""
    import ctypes

    import torch
    from quant_gemm.sharded import NativeRowShardedW4A8, shard_lib
    m, n, k = 3, 512, 1024
    _, _, aq, bq = make_case(O, m, n, k, 2)
    a_d, b_d = dev(aq), dev(bq)
    lib = shard_lib()
    P = ctypes.c_void_p
    st = P(torch.cuda.current_stream().cuda_stream)
    c = torch.zeros((m, n), dtype=torch.float32, device="cuda")
    assert lib.qg_sharded_gemm_w4a8(P(a_d.data_ptr()), P(b_d.data_ptr()), P(c.data_ptr()), m, n, k, 2, None, 0,
                                    comm.handle, st) == -3  # QG_ERR_UNSUPPORTED: no workspace
    assert torch.isnan(c).all()
    c.zero_()
    ws = torch.empty(lib.qg_sharded_gemm_workspace_size(m, n, 1) // 4, dtype=torch.float32, device="cuda")
    assert lib.qg_sharded_gemm_w4a8(P(a_d.data_ptr()), None, P(c.data_ptr()), m, n, k, 2, P(ws.data_ptr()),
                                    ws.numel() * 4, comm.handle, st) == -1  # QG_ERR_INVALID_ARG: null shard
    assert torch.isnan(c).all()
    good = NativeRowShardedW4A8(b_d, n, k, comm).forward(a_d, m)
    assert np.array_equal(host(good), host(qg.gemm_w4a8(a_d, b_d, m, n, k)))
