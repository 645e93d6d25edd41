"""W4A16 prefill: repeated calls (library workspace, then a caller workspace) must give bit-identical
outputs, within the fp32 bound of a float64 dequantized reference, at the split-K shapes
(w16s_kernel: M = 32, N = 4096 / 11008, K = 4096 / 14336). Not part of the product: a check run on
the GPU box when the A/B tool reports a difference between libraries."""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))
import quant_gemm as qg  # noqa: E402
from quant_gemm import _lib  # noqa: E402

P = ctypes.c_void_p
dev = torch.device("cuda", 0)
lib = _lib.load()
for M, N, K in [(32, 4096, 4096), (32, 11008, 4096), (32, 4096, 14336), (64, 11008, 4096)]:
    g = torch.Generator(device=dev)
    g.manual_seed(M + N + K)
    a = torch.rand((M, K), generator=g, device=dev) * 2 - 1
    wq = qg.quantize_q4_0(torch.rand((N, K), generator=g, device=dev) * 2 - 1)
    outs = [qg.gemm_w4a16(a, wq, M, N, K) for _ in range(4)]
    torch.cuda.synchronize()
    ws = torch.zeros(64 << 18, dtype=torch.int32, device=dev)
    for _ in range(3):
        c = torch.empty((M, N), dtype=torch.float32, device=dev)
        rc = lib.qg_gemm_w4a16_ws(P(a.data_ptr()), P(wq.data_ptr()), P(c.data_ptr()), M, N, K, P(ws.data_ptr()), 64 << 20,
                                  P(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
        outs.append(c)
    torch.cuda.synchronize()
    same = [bool(torch.equal(outs[0], o)) for o in outs[1:]]
    w = qg.dequantize_q4_0(wq, K).double()
    ref = a.double() @ w.T
    err = (outs[0].double() - ref).abs().max().item()
    bound = (2 * (K + 2) * 2.0**-24 * (a.double().abs() @ w.abs().T)).max().item()
    print(f"M={M} N={N} K={K}: repeat-identical {same}  max|err| {err:.3e}  bound {bound:.3e}  {'OK' if err <= bound and all(same) else 'FAIL'}", flush=True)
