#!/usr/bin/env python3
"""A/B of libqg_hip.so builds (tuning only; not product): each library is loaded on its own
(RTLD_LOCAL) and times the same shapes the way bench.py does — G launches on distinct resident
weight copies (> 600 MB, so every launch streams from HBM) captured in a hipGraph, HIP events on
the launch stream — in interleaved rounds, so box-to-box noise cancels.

  python tools/ab_lib.py --libs a.so b.so [--shapes 1x4096x4096:2,32x4096x4096:2] [--rounds 7] [--w16]
Outputs must agree bit for bit across the libraries (checked on every shape).
"""
from __future__ import annotations

import argparse
import ctypes
import math
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))

import torch  # noqa: E402

import quant_gemm as qg  # noqa: E402  (the in-tree product library makes the inputs)

P = ctypes.c_void_p


def load(path: str) -> ctypes.CDLL:
    lib = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_NOW)
    lib.qg_gemm_w4a8_ex.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    lib.qg_gemm_w4a8_ex.restype = ctypes.c_int
    lib.qg_gemm_w4a16_ws.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_size_t, P]
    lib.qg_gemm_w4a16_ws.restype = ctypes.c_int
    lib.qg_gemm_w8a16.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    lib.qg_gemm_w8a16.restype = ctypes.c_int
    lib.qg_gemm_w4a8_grouped.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    lib.qg_gemm_w4a8_grouped.restype = ctypes.c_int
    I64 = ctypes.c_int64
    lib.qg_gemm_w4a8_strided_batched.argtypes = [P, I64, P, I64, P, I64] + [ctypes.c_int] * 5 + [P]
    lib.qg_gemm_w4a8_strided_batched.restype = ctypes.c_int
    return lib


class GemvItem(ctypes.Structure):  # qg_gemv_item (include/qg/qg.h)
    _fields_ = [("A_q8_1", P), ("B", P), ("C", P), ("N", ctypes.c_int), ("ldc", ctypes.c_int)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--shapes", default="1x4096x4096:2,32x4096x4096:2")
    ap.add_argument("--algo", type=int, default=0)
    ap.add_argument("--algos", default="", help="one library, several algo ids (e.g. 0,5): variants = algos; "
                    "outputs compared by max relative difference instead of bit for bit")
    ap.add_argument("--G", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--w16", action="store_true", help="time qg_gemm_w4a16 (fp32 activations, Q4_0 weights)")
    ap.add_argument("--grouped", action="store_true", help="one qg_gemm_w4a8_grouped launch of the G GEMVs per step")
    ap.add_argument("--batched", action="store_true", help="one qg_gemm_w4a8_strided_batched launch of the G GEMVs per step")
    a = ap.parse_args()
    libs = [load(p) for p in a.libs]
    algos = [a.algo] * len(libs)
    names = list(a.libs)
    if a.algos:
        algos = [int(x) for x in a.algos.split(",")]
        libs = [libs[0]] * len(algos)
        names = [f"{os.path.basename(a.libs[0])} algo {x}" for x in algos]
    dev = torch.device("cuda", 0)
    for spec in a.shapes.split(","):
        dims, wt = spec.split(":")
        M, N, K = (int(x) for x in dims.split("x"))
        wt = int(wt)
        gen = torch.Generator(device=dev)
        gen.manual_seed(M * 7 + N)
        af = torch.rand((M, K), generator=gen, device=dev) * 2 - 1
        aq = af if a.w16 else qg.quantize_q8_1(af)
        wq = qg.quantize(torch.rand((N, K), generator=gen, device=dev) * 2 - 1, wt)
        R = max(a.G, math.ceil(600e6 / wq.numel()))
        copies = torch.empty((R,) + tuple(wq.shape), dtype=torch.uint8, device=dev)
        copies.copy_(wq.unsqueeze(0).expand_as(copies))
        outs = torch.empty((len(libs), a.G, M, N), dtype=torch.float32, device=dev)
        graphs = []
        WSB = 64 << 20  # W4A16: each library's own caller workspace (zeroed once), capture-safe
        wss = [torch.zeros(WSB // 4, dtype=torch.int32, device=dev) for _ in libs] if a.w16 else []
        for li, lib in enumerate(libs):
            def step(st, li=li, lib=lib):
                if a.batched:
                    assert R >= a.G
                    assert lib.qg_gemm_w4a8_strided_batched(P(aq.data_ptr()), 0, P(copies.data_ptr()), copies[0].numel(),
                                                            P(outs[li].data_ptr()), M * N, a.G, M, N, K, wt, st) == 0
                    return
                if a.grouped:
                    items = (GemvItem * a.G)(*[GemvItem(aq.data_ptr(), copies[j % R].data_ptr(), outs[li, j].data_ptr(), N, 0)
                                               for j in range(a.G)])
                    assert lib.qg_gemm_w4a8_grouped(items, a.G, M, K, wt, st) == 0
                    return
                for j in range(a.G):
                    if a.w16 and wt == 8:
                        rc = lib.qg_gemm_w8a16(P(aq.data_ptr()), P(copies[j % R].data_ptr()),
                                               P(outs[li, j].data_ptr()), M, N, K, st)
                    elif a.w16:
                        rc = lib.qg_gemm_w4a16_ws(P(aq.data_ptr()), P(copies[j % R].data_ptr()),
                                                  P(outs[li, j].data_ptr()), M, N, K, P(wss[li].data_ptr()), WSB, st)
                    else:
                        rc = lib.qg_gemm_w4a8_ex(P(aq.data_ptr()), P(copies[j % R].data_ptr()),
                                                 P(outs[li, j].data_ptr()), M, N, K, wt, algos[li], st)
                    assert rc == 0, rc
            side = torch.cuda.Stream()
            with torch.cuda.stream(side):
                step(P(side.cuda_stream))
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step(P(torch.cuda.current_stream().cuda_stream))
            graphs.append(g)
        for li in range(1, len(libs)):
            if not torch.equal(outs[0], outs[li]):
                rel = ((outs[li] - outs[0]).abs().max() / outs[0].abs().max()).item()
                print(f"  {'!!' if not a.algos else '..'} {names[li]} differs from {names[0]} at {spec} (max rel {rel:.2e})")
        times = [[] for _ in libs]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for li, g in enumerate(graphs):
                g.replay()
                e0.record()
                for _ in range(a.reps):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                times[li].append(e0.elapsed_time(e1) * 1e3 / (a.reps * a.G))
        nb = K // 32
        bb = qg.BLOCK_BYTES[wt]
        nbytes = N * nb * bb + M * K * (4 if a.w16 else 36 / 32) + M * N * 4
        print(f"M={M} N={N} K={K} wtype={wt} ({nbytes} B/launch, {R} copies)")
        for li, p in enumerate(names):
            med = statistics.median(times[li])
            print(f"  {os.path.basename(p):28s} {med:7.3f} us  (min {min(times[li]):.3f} max {max(times[li]):.3f})"
                  f"  {nbytes / med / 1e3:7.1f} GB/s  frac {nbytes / med / 8e6:.3f}")
        sys.stdout.flush()
        del copies, outs, graphs, wss


if __name__ == "__main__":
    main()
