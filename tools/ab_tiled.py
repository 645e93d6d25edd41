#!/usr/bin/env python3
"""A/B of the prefill on the reference rows (qg_gemm_w4a8) vs the tiled layout (qg_gemm_w4a8_tiled),
timed as bench.py does: G launches over rotating resident weight copies (> 600 MB) in a hipGraph, HIP
events on the launch stream, interleaved rounds (tuning tool, not product).
  python tools/ab_tiled.py [--shapes 32x4096x4096:2,...] [--rounds 7]"""
from __future__ import annotations

import argparse
import math
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import quant_gemm as qg  # noqa: E402
from bench import graph_time_us  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="32x4096x4096:2,16x4096x4096:2,8x4096x4096:2,64x4096x4096:2,128x4096x4096:2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--G", type=int, default=64)
    ap.add_argument("--libs", nargs="*", default=[], help="variant builds of libqg_hip.so: their tiled entry is timed too")
    ap.add_argument("--rows-libs", nargs="*", default=[], help="other builds whose reference-row entry is timed too")
    a = ap.parse_args()
    import ctypes
    P = ctypes.c_void_p
    extra = {}
    for path in a.libs + a.rows_libs:
        lib = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_NOW)
        tag = os.path.basename(path).replace("libqg_", "").replace(".so", "")
        if path in a.libs:
            f = lib.qg_gemm_w4a8_tiled
            f.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
            extra["tiled@" + tag] = ("tiled", f)
        else:
            f = lib.qg_gemm_w4a8_ex
            f.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
            extra["rows@" + tag] = ("rows", f)
    dev = torch.device("cuda", 0)
    for spec in a.shapes.split(","):
        dims, wt = spec.split(":")
        M, N, K = (int(x) for x in dims.split("x"))
        wt = int(wt)
        gen = torch.Generator(device=dev)
        gen.manual_seed(M + N + K)
        aq = qg.quantize_q8_1(torch.rand((M, K), generator=gen, device=dev) * 2 - 1)
        wq = qg.quantize(torch.rand((N, K), generator=gen, device=dev) * 2 - 1, wt)
        wt_t = qg.tile_weights(wq, N, K, wt)
        forms = {}
        if K % 128 == 0:
            forms["rows"] = wq.reshape(-1)
        forms["tiled"] = wt_t
        copies = {}
        for name, w in forms.items():
            R = max(a.G, math.ceil(600e6 / w.numel()))
            c = torch.empty((R, w.numel()), dtype=torch.uint8, device=dev)
            c.copy_(w.unsqueeze(0).expand_as(c))
            copies[name] = c
        out = torch.empty((a.G, M, N), dtype=torch.float32, device=dev)
        ref = qg.gemm_w4a8(aq, wq, M, N, K, wt)

        def step_of(name):
            if name in extra:
                kind, f = extra[name]
                cp = copies[kind]

                def run():
                    cs = P(torch.cuda.current_stream().cuda_stream)
                    for j in range(a.G):
                        args = (P(aq.data_ptr()), P(cp[j].data_ptr()), P(out[j].data_ptr()), M, N, K, wt)
                        rc = f(*args, cs) if kind == "tiled" else f(*args, 0, cs)
                        if rc != 0:
                            raise RuntimeError(f"{name}: status {rc}")
                return run
            cp = copies[name]
            if name == "rows":
                return lambda: [qg.gemm_w4a8(aq, cp[j], M, N, K, wt, out=out[j]) for j in range(a.G)]
            return lambda: [qg.gemm_w4a8_tiled(aq, cp[j], M, N, K, wt, out=out[j]) for j in range(a.G)]

        names = list(forms) + [n for n, (kind, _) in extra.items() if kind in copies]
        times = {n: [] for n in names}
        for _ in range(a.rounds):
            for n in names:
                times[n].append(graph_time_us(step_of(n), 10, a.G))
        same = bool(torch.equal(qg.gemm_w4a8_tiled(aq, wt_t, M, N, K, wt), ref))
        bits = {}
        for name, (kind, f) in extra.items():  # each variant's output against the in-tree reference rows
            if kind not in copies:
                continue
            o = torch.zeros((M, N), dtype=torch.float32, device=dev)
            w = wt_t if kind == "tiled" else wq
            cs = P(torch.cuda.current_stream().cuda_stream)
            args = (P(aq.data_ptr()), P(w.data_ptr()), P(o.data_ptr()), M, N, K, wt)
            rc = f(*args, cs) if kind == "tiled" else f(*args, 0, cs)
            torch.cuda.synchronize()
            bits[name] = "rc%d" % rc if rc else ("==" if torch.equal(o, ref) else "max|d| %.3g" % float((o - ref).abs().max()))
        print(f"M={M} N={N} K={K} wtype={wt}: " + "  ".join(
            f"{n} {statistics.median(v):.3f} us (min {min(v):.3f})" for n, v in times.items()) +
            f"  tiled==rows bitwise: {same}  variants vs rows: {bits}  cfg {qg.debug_config_tiled(M, N, K, wt)}", flush=True)
        del copies, out


if __name__ == "__main__":
    main()
