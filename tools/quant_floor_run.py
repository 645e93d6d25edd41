#!/usr/bin/env python3
"""The quantizer's launch floor under rocprofv3: L launches of the M = 1, K = 4096
FP32 -> Q8_1 quantizer (16 workgroups x 64 lanes, 8 lanes per block), then L launches of the calibration
library's empty kernel with the same grid (libqg_calib.so: qg_calib_empty), back to back on one stream.
The trace's average duration of the empty kernel is what any kernel of that grid pays before its first load.
  rocprofv3 --kernel-trace --stats -d gpurun_out/qf -- python3 tools/quant_floor_run.py"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))

import torch  # noqa: E402

import quant_gemm as qg  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--launches", type=int, default=400)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(os.path.join(REPO, "llama.cpp-quant-gemm_amd", "quant_gemm", "libqg_calib.so"))
    lib.qg_calib_empty.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.qg_calib_empty.restype = ctypes.c_int
    xs = [torch.randn((1, a.k), device=dev) for _ in range(64)]
    stream = torch.cuda.current_stream().cuda_stream
    grid = (a.k // 32) * 8 // 64
    for i in range(a.launches):
        qg.quantize_q8_1(xs[i % 64])
    torch.cuda.synchronize()
    for _ in range(a.launches):
        if lib.qg_calib_empty(grid, 64, stream) != 0:
            raise RuntimeError("qg_calib_empty failed")
    torch.cuda.synchronize()
    print(f"quantizer and empty kernel, grid {grid} x 64, {a.launches} launches each")


if __name__ == "__main__":
    main()
