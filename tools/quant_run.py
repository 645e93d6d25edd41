#!/usr/bin/env python3
"""Run the FP32 -> Q8_1 quantizer L times back to back (inputs rotated over > 600 MB for K = 4096 rows... or
over 64 copies for small rows) — a target for rocprofv3 kernel traces of the quantizer.
  python tools/quant_run.py --m 1 --k 4096 [--launches 400]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))

import torch  # noqa: E402

import quant_gemm as qg  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--launches", type=int, default=400)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    xs = [torch.randn((a.m, a.k), device=dev) for _ in range(64)]
    for i in range(a.launches):
        qg.quantize_q8_1(xs[i % 64])
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
