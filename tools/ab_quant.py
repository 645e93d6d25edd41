#!/usr/bin/env python3
"""A/B of the Q8_1 activation quantizer across libqg_hip.so builds (tuning tool, not product): G
qg_quantize_q8_1 launches of an [M, K] fp32 row block in one hipGraph, HIP events, interleaved rounds;
the bytes must agree across the builds.
  python tools/ab_quant.py --libs a.so b.so [--shapes 1x4096,32x4096]"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import quant_gemm  # noqa: E402,F401  (torch's HIP runtime first)
from bench import graph_time_us  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--shapes", default="1x4096,4x4096,32x4096,512x4096")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--G", type=int, default=64)
    a = ap.parse_args()
    P = ctypes.c_void_p
    fns = []
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_NOW)
        f = lib.qg_quantize_q8_1
        f.argtypes = [P, P, ctypes.c_int64, P]
        fns.append((os.path.basename(path), f))
    dev = torch.device("cuda", 0)
    for spec in a.shapes.split(","):
        M, K = (int(x) for x in spec.split("x"))
        x = (torch.rand((a.G, M, K), device=dev) * 2 - 1).contiguous()
        outs = [torch.empty((a.G, M * (K // 32) * 36), dtype=torch.uint8, device=dev) for _ in fns]

        def step_of(i):
            f = fns[i][1]

            def run():
                cs = P(torch.cuda.current_stream().cuda_stream)
                for j in range(a.G):
                    if f(P(x[j].data_ptr()), P(outs[i][j].data_ptr()), M * K, cs) != 0:
                        raise RuntimeError("qg_quantize_q8_1 failed")
            return run
        times = [[] for _ in fns]
        for _ in range(a.rounds):
            for i in range(len(fns)):
                times[i].append(graph_time_us(step_of(i), 10, a.G))
        same = all(torch.equal(outs[0], o) for o in outs[1:])
        print(f"M={M} K={K}: " + "  ".join(f"{fns[i][0]} {statistics.median(t):.3f} us" for i, t in enumerate(times)) +
              f"  bytes identical: {same}", flush=True)


if __name__ == "__main__":
    main()
