#!/usr/bin/env python3
"""Run one product shape L times back to back (weights rotated over > 600 MB) — a target for
rocprofv3 kernel traces and PMC passes of the non-headline configs (e.g. the M=32 prefill,
BASELINE configs[2]).   python tools/gemm_run.py --m 32 --n 4096 --k 4096 [--wtype 2] [--launches 200] [--w16]
"""
import argparse
import ctypes
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))

import torch  # noqa: E402

import quant_gemm as qg  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=32)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--wtype", type=int, default=2)
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--w16", action="store_true", help="FP32 activations through qg_gemm_w4a16_ws (Q4_0) / w8a16 (Q8_0)")
    ap.add_argument("--tiled", action="store_true", help="the tiled weight layout (qg_tile_weights + qg_gemm_w4a8_tiled)")
    ap.add_argument("--tiled-act", action="store_true", help="tiled weights and tiled activations (qg_gemm_w4a8_tiled_act)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    x = torch.rand((a.m, a.k), generator=g, device=dev) * 2 - 1
    w = torch.rand((a.n, a.k), generator=g, device=dev) * 2 - 1
    xq, wq = qg.quantize_q8_1(x), qg.quantize(w, a.wtype)
    if a.tiled_act:
        a.tiled = True
        xt = qg.quantize_q8_1_tiled(x)
    if a.tiled:
        wq = qg.tile_weights(wq, a.n, a.k, a.wtype)
    R = max(2, math.ceil(600e6 / wq.numel()))
    copies = torch.empty((R,) + tuple(wq.shape), dtype=torch.uint8, device=dev)
    copies.copy_(wq.unsqueeze(0).expand_as(copies))
    out = torch.empty((a.m, a.n), dtype=torch.float32, device=dev)
    lib = qg._lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if a.w16:
        wsb = lib.qg_gemm_w16_workspace_size(a.m, a.n, a.k)
        ws = torch.zeros(max(wsb, 16) // 4 + 64, dtype=torch.int32, device=dev)
        fn = lib.qg_gemm_w4a16_ws if a.wtype == 2 else lib.qg_gemm_w8a16_ws
    for i in range(a.launches):
        if a.w16:
            rc = fn(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(copies[i % R].data_ptr()), ctypes.c_void_p(out.data_ptr()),
                    a.m, a.n, a.k, ctypes.c_void_p(ws.data_ptr()), wsb, st)
        elif a.tiled_act:
            rc = lib.qg_gemm_w4a8_tiled_act(ctypes.c_void_p(xt.data_ptr()), ctypes.c_void_p(copies[i % R].data_ptr()),
                                            ctypes.c_void_p(out.data_ptr()), a.m, a.n, a.k, a.wtype, st)
        elif a.tiled:
            rc = lib.qg_gemm_w4a8_tiled(ctypes.c_void_p(xq.data_ptr()), ctypes.c_void_p(copies[i % R].data_ptr()),
                                        ctypes.c_void_p(out.data_ptr()), a.m, a.n, a.k, a.wtype, st)
        else:
            rc = lib.qg_gemm_w4a8(ctypes.c_void_p(xq.data_ptr()), ctypes.c_void_p(copies[i % R].data_ptr()),
                                  ctypes.c_void_p(out.data_ptr()), a.m, a.n, a.k, a.wtype, st)
        assert rc == 0, rc
    torch.cuda.synchronize()
    print(f"ok: {a.launches} launches of M={a.m} N={a.n} K={a.k} wtype={a.wtype}{' W16' if a.w16 else ''}, "
          f"algo {qg.select_algo(a.m, a.n, a.k, a.wtype)}")


if __name__ == "__main__":
    main()
