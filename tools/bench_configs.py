#!/usr/bin/env python3
"""Measure every BASELINE.json config on one MI355X (secondary numbers for DESIGN.md §6).

For each config: weights quantized on-GPU, rotated over enough resident copies to exceed the
256 MB Infinity Cache, G back-to-back launches captured in a hipGraph, timed with HIP events on
the launch stream; plus (GEMV path) the same G products as one strided-batched launch.
Prints one JSON object per config and writes them to --out.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))

import torch  # noqa: E402

import quant_gemm as qg  # noqa: E402

PEAK = 8000.0
CONFIGS = [
    ("q4_0", 1, 4096, 4096), ("q4_1", 1, 4096, 4096), ("q5_0", 1, 4096, 4096), ("q5_1", 1, 4096, 4096),
    ("q4_0", 32, 4096, 4096), ("q4_0", 1, 32000, 4096), ("q4_0", 1, 4000, 4096),
    ("q4_0", 2, 4096, 4096), ("q4_0", 3, 4096, 4096), ("q4_0", 4, 4096, 4096),
    ("q4_0", 8, 4096, 4096), ("q4_0", 1, 4096, 14336), ("q4_0", 2, 4096, 14336), ("q4_0", 64, 4096, 4096),
    ("q4_0", 128, 4096, 4096), ("q4_0", 256, 4096, 4096), ("q4_0", 512, 4096, 4096),
    ("q8_0", 1, 4096, 4096), ("q8_0", 32, 4096, 4096),          # W8A8
    ("w4a16", 1, 4096, 4096), ("w4a16", 4, 4096, 4096), ("w4a16", 16, 4096, 4096), ("w4a16", 32, 4096, 4096),
    ("w4a16", 64, 4096, 4096), ("w4a16", 512, 4096, 4096),
    ("w8a16", 1, 4096, 4096), ("w8a16", 16, 4096, 4096), ("w8a16", 32, 4096, 4096), ("w8a16", 64, 4096, 4096),
]
WT = {"q4_0": 2, "q4_1": 3, "q5_0": 6, "q5_1": 7, "q8_0": 8}
W16 = {"w4a16": 2, "w8a16": 8}


def graph_us(step, reps: int) -> float:
    """Microseconds per replay of a hipGraph capturing step(stream)."""
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        step(ctypes.c_void_p(side.cuda_stream))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    for _ in range(2):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def measure_w16(wname: str, M: int, N: int, K: int, G: int, reps: int) -> dict:
    """FP32 activations x Q4_0 / Q8_0 weights (qg_gemm_w4a16 / qg_gemm_w8a16)."""
    dev = torch.device("cuda", 0)
    wt = W16[wname]
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    a = torch.rand((M, K), generator=gen, device=dev) * 2 - 1
    b = torch.rand((N, K), generator=gen, device=dev) * 2 - 1
    bq = qg.quantize(b, wt)
    fn = qg.gemm_w4a16 if wt == 2 else qg.gemm_w8a16
    c = fn(a, bq, M, N, K)
    ref = a.double() @ b.double().T
    nmse = float(torch.sum((c.double() - ref) ** 2) / torch.sum(ref ** 2))
    del b, ref
    wbytes = bq.numel()
    R = max(2, math.ceil(600e6 / wbytes))
    G = min(G, R)
    copies = torch.empty((R,) + tuple(bq.shape), dtype=torch.uint8, device=dev)
    copies.copy_(bq.unsqueeze(0).expand_as(copies))
    out = torch.empty((G, M, N), dtype=torch.float32, device=dev)
    lib = qg._lib.load()
    sym = lib.qg_gemm_w4a16_ws if wt == 2 else lib.qg_gemm_w8a16_ws
    # the caller-workspace form: a graph captures its own stream, which has no library workspace
    need = lib.qg_gemm_w16_workspace_size(M, N, K)
    ws = torch.zeros(max(need, 256) // 4 + 64, dtype=torch.int32, device=dev)

    def step(stream):
        for j in range(G):
            assert sym(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(copies[j].data_ptr()),
                       ctypes.c_void_p(out[j].data_ptr()), M, N, K, ctypes.c_void_p(ws.data_ptr()), need,
                       stream) == 0

    us = graph_us(step, reps) / G
    byts = wbytes + M * K * 4 + M * N * 4
    flops = 2.0 * M * N * K
    return {"wtype": wname, "M": M, "N": N, "K": K, "algo": "w16 gemv" if M <= 8 else f"w16 mfma split-K ws={need}", "us_per_launch": round(us, 3),
            "gbps": round(byts / us / 1e3, 1), "frac_hbm": round(byts / us / 1e3 / PEAK, 4),
            "tflops": round(flops / us / 1e6, 3), "nmse_vs_fp32": nmse, "algorithmic_bytes": byts, "launches": G}


def measure(wname: str, M: int, N: int, K: int, G: int, reps: int) -> dict:
    if wname in W16:
        return measure_w16(wname, M, N, K, G, reps)
    dev = torch.device("cuda", 0)
    wt = WT[wname]
    bb = qg.BLOCK_BYTES[wt]
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    a = torch.rand((M, K), generator=gen, device=dev) * 2 - 1
    b = torch.rand((N, K), generator=gen, device=dev) * 2 - 1
    aq, bq = qg.quantize_q8_1(a), qg.quantize(b, wt)
    c = qg.gemm_w4a8(aq, bq, M, N, K, wt)
    ref = a.double() @ b.double().T
    nmse = float(torch.sum((c.double() - ref) ** 2) / torch.sum(ref ** 2))
    del b, ref
    wbytes = bq.numel()
    R = max(2, math.ceil(600e6 / wbytes))
    G = min(G, R)
    copies = torch.empty((R,) + tuple(bq.shape), dtype=torch.uint8, device=dev)
    copies.copy_(bq.unsqueeze(0).expand_as(copies))
    out = torch.empty((G, M, N), dtype=torch.float32, device=dev)
    lib = qg._lib.load()
    algo = lib.qg_select_algo(M, N, K, wt)

    def step(stream):
        for j in range(G):
            st = lib.qg_gemm_w4a8(ctypes.c_void_p(aq.data_ptr()), ctypes.c_void_p(copies[j].data_ptr()),
                                  ctypes.c_void_p(out[j].data_ptr()), M, N, K, wt, stream)
            assert st == 0, st

    us = graph_us(step, reps) / G
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    nbk = K // 32
    byts = N * nbk * bb + M * nbk * 36 + M * N * 4
    flops = 2.0 * M * N * K
    res = {"wtype": wname, "M": M, "N": N, "K": K, "algo": {1: "gemv", 2: "mfma", 3: "generic"}.get(algo, algo),
           "us_per_launch": round(us, 3), "gbps": round(byts / us / 1e3, 1), "frac_hbm": round(byts / us / 1e3 / PEAK, 4),
           "tflops": round(flops / us / 1e6, 3), "nmse_vs_fp32": nmse, "algorithmic_bytes": byts, "launches": G}
    if M <= 8:
        # FP32 activations: fused quantization (one launch) vs quantize + product (two launches)
        a_c = a.contiguous()
        ws = torch.empty((lib.qg_gemm_w4a8_f32_workspace_size(M, K),), dtype=torch.uint8, device=dev)
        aq2 = torch.empty_like(aq)

        def fused(stream):
            for j in range(G):
                st = lib.qg_gemm_w4a8_f32(ctypes.c_void_p(a_c.data_ptr()), ctypes.c_void_p(copies[j].data_ptr()),
                                          ctypes.c_void_p(out[j].data_ptr()), M, N, K, wt,
                                          ctypes.c_void_p(ws.data_ptr()), ws.numel(), stream)
                assert st == 0, st

        def two_step(stream):
            for j in range(G):
                assert lib.qg_quantize_q8_1(ctypes.c_void_p(a_c.data_ptr()), ctypes.c_void_p(aq2.data_ptr()),
                                            M * K, stream) == 0
                assert lib.qg_gemm_w4a8(ctypes.c_void_p(aq2.data_ptr()), ctypes.c_void_p(copies[j].data_ptr()),
                                        ctypes.c_void_p(out[j].data_ptr()), M, N, K, wt, stream) == 0

        fbytes = N * nbk * bb + M * K * 4 + M * N * 4
        for name, fn in (("fused_f32", fused), ("quantize_then_gemm", two_step)):
            uf = graph_us(fn, reps) / G
            res[name] = {"us_per_product": round(uf, 3), "gbps": round(fbytes / uf / 1e3, 1),
                         "frac_hbm": round(fbytes / uf / 1e3 / PEAK, 4)}
    if algo == 1:
        bout = torch.empty((G, M, N), dtype=torch.float32, device=dev)
        cs = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        call = lambda: lib.qg_gemm_w4a8_strided_batched(  # noqa: E731
            ctypes.c_void_p(aq.data_ptr()), 0, ctypes.c_void_p(copies.data_ptr()), wbytes,
            ctypes.c_void_p(bout.data_ptr()), M * N, G, M, N, K, wt, cs)
        for _ in range(2):
            assert call() == 0
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        ub = e0.elapsed_time(e1) * 1e3 / (reps * G)
        res["batched"] = {"us_per_gemv": round(ub, 3), "gbps": round(byts / ub / 1e3, 1),
                          "frac_hbm": round(byts / ub / 1e3 / PEAK, 4), "tflops": round(flops / ub / 1e6, 3)}
        assert torch.equal(bout[0], out[0])
    return res


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--gemvs", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None, help="comma-separated weight kinds to run (e.g. w4a16,q8_0)")
    args = ap.parse_args()
    rows = []
    only = set(args.only.split(",")) if args.only else None
    for w, m, n, k in CONFIGS:
        if only and w not in only:
            continue
        r = measure(w, m, n, k, args.gemvs, args.reps)
        print(json.dumps(r), flush=True)
        rows.append(r)
        torch.cuda.empty_cache()
    if args.out:
        json.dump(rows, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
