#!/usr/bin/env python3
"""Tiled weights with row activations vs tiled activations (round 5), timed by bench.measure_config (G launches
over > 600 MB of rotating weight copies in a hipGraph, HIP events), several interleaved rounds (tuning tool).
  python tools/ab_tiled_act.py [--shapes 32x4096x4096,...] [--rounds 3]"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="32x4096x4096,16x4096x4096,8x4096x4096,64x4096x4096,32x4096x4128,512x4096x4096")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--wtype", default="q4_0")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for spec in a.shapes.split(","):
        M, N, K = (int(x) for x in spec.split("x"))
        t = {"tiled": [], "tiled_act": []}
        for _ in range(a.rounds):
            for r in bench.measure_config(a.wtype, M, N, K, dev, forms=("tiled", "tiled_act")):
                t[r["form"]].append(r["us_per_launch"])
        print(f"{a.wtype} M={M} N={N} K={K}: " + "  ".join(f"{f} {statistics.median(v):.3f} us (min {min(v):.3f})"
                                                          for f, v in t.items()), flush=True)


if __name__ == "__main__":
    main()
