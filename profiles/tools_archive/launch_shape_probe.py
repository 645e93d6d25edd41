"""Empty-kernel cost per back-to-back launch by grid shape (libqg_calib.so qg_calib_empty), hipGraph of
64 launches, HIP events, as bench.py's floor; and the pure read of the GEMV's 9,458,176 B by shape.
Not part of the product."""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import graph_time_us  # noqa: E402

lib = ctypes.CDLL(os.path.join(REPO, "llama.cpp-quant-gemm_amd", "quant_gemm", "libqg_calib.so"))
lib.qg_calib_empty.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.qg_calib_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
G = 64
for grid, block in [(1, 64), (64, 1024), (256, 64), (256, 256), (256, 512), (256, 1024), (512, 1024), (1024, 256), (1024, 512), (2048, 256), (4096, 64)]:
    def fn():
        cs = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(G):
            assert lib.qg_calib_empty(grid, block, cs) == 0
    t = min(graph_time_us(fn, 10, G) for _ in range(3))
    print(f"empty grid {grid:5d} x {block:4d}: {t:6.3f} us per launch", flush=True)
R = 72
nbytes = 9458176
buf = torch.empty(R * 9437184 + 65536, dtype=torch.uint8, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
for p, blk in [(1, 256), (1, 512), (1, 1024), (2, 256), (2, 512), (4, 512), (8, 256)]:
    def fn():
        cs = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for j in range(G):
            assert lib.qg_calib_read(ctypes.c_void_p(buf.data_ptr() + (j % R) * 9437184), nbytes, p, blk,
                                     ctypes.c_void_p(sink.data_ptr()), cs) == 0
    t = min(graph_time_us(fn, 10, G) for _ in range(3))
    print(f"read x4 p{p} wg{blk}: {t:6.3f} us per launch ({nbytes / t / 1e3 / 8000:.3f} of 8 TB/s)", flush=True)
