#!/usr/bin/env python3
"""Probe (tuning only; not product): odd K/32 at prefill sizes — the auto dispatch (ragged kernel, or since
qg_repack.hip the product repack + MFMA at M >= 16, N >= 1024; its kernel family is printed) vs a padded
repack (weights and activations copied into rows of K'/32 = round_up(K/32, --pad) blocks, the extra
blocks all zero: d = 0, s = 0) followed by the MFMA kernel on K'. DESIGN.md §9 "Odd K/32".

Times with HIP events around a hipGraph replay of L back-to-back launches rotating over > 600 MB of
weight copies (as bench.py). The repack here is torch's strided copy, an upper bound for a
dedicated kernel. Also checks that the padded MFMA result equals the MFMA kernel's own result on
the same padded bytes produced another way (bit-identical by construction) and stays within the
oracle-free fp32 bound of the ragged result (max |diff| printed).

  python tools/repack_probe.py [--k 4128] [--ms 8,16,32,64] [--wtype 2]
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


def timed(fn, launches: int) -> float:
    """Per-launch time of `launches` calls captured into one hipGraph (host dispatch excluded)."""
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for i in range(3):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(launches):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    g.replay()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / launches


def timed_eager(fn, launches: int) -> float:
    """Per-call time of eager back-to-back calls (no capture: the library's repack workspace is
    never handed to a stream capture, so captured calls fall back to the ragged kernel)."""
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for i in range(launches):
        fn(i)
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / launches


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=4128)
    ap.add_argument("--ms", default="8,16,32,64")
    ap.add_argument("--wtype", type=int, default=2)
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--pad", type=int, default=4, help="pad K/32 up to a multiple of this")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    N, K, t = a.n, a.k, a.wtype
    nb = K // 32
    nbp = (nb + a.pad - 1) // a.pad * a.pad
    Kp = nbp * 32
    bb = qg.BLOCK_BYTES[t]
    w = qg.quantize(torch.randn(N, K, device=dev), t).view(N, nb * bb)
    R = max(8, math.ceil(600e6 / w.numel()))
    wc = torch.empty((R, N, nb * bb), dtype=torch.uint8, device=dev)
    wc.copy_(w.unsqueeze(0).expand_as(wc))
    wp = torch.zeros((N, nbp * bb), dtype=torch.uint8, device=dev)  # workspace (pad stays zero)
    print(f"N={N} K={K} (K/32={nb}) -> K'={Kp}; wtype {t}; {R} weight copies; {a.launches} launches; "
          f"MFMA config on K': {qg.debug_config(32, N, Kp, t, algo=qg.ALGO_MFMA)}")
    for M in [int(x) for x in a.ms.split(",")]:
        x = qg.quantize_q8_1(torch.randn(M, K, device=dev)).view(M, nb * 36)
        xp = torch.zeros((M, nbp * 36), dtype=torch.uint8, device=dev)
        out = torch.empty((M, N), dtype=torch.float32, device=dev)
        out2 = torch.empty((M, N), dtype=torch.float32, device=dev)

        def ragged(i):
            qg.gemm_w4a8(x, wc[i % R], M, N, K, t, out=out)

        def repack(i):
            wp[:, :nb * bb].copy_(wc[i % R])
            xp[:, :nb * 36].copy_(x)

        def mfma_only(i):
            qg.gemm_w4a8(xp, wp, M, N, Kp, t, algo=qg.ALGO_MFMA, out=out2)

        def both(i):
            repack(i)
            mfma_only(i)

        lib = qg._lib.load()
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        xa, oa = ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr())
        wa = [ctypes.c_void_p(wc[i].data_ptr()) for i in range(R)]

        def auto_eager(i):  # the C-ABI directly (host cost per call well under the GPU time)
            lib.qg_gemm_w4a8_ldc(xa, wa[i % R], oa, M, N, K, N, t, 0, sp)

        t_e = timed_eager(auto_eager, a.launches)
        cfg_r = qg.debug_config(M, N, K, t)
        cfg_p = qg.debug_config(M, N, Kp, t, algo=qg.ALGO_MFMA)
        t_r = timed(ragged, a.launches)
        t_c = timed(repack, a.launches)
        t_m = timed(mfma_only, a.launches)
        t_b = timed(both, a.launches)
        ragged(0)
        both(0)
        torch.cuda.synchronize()
        d = (out - out2).abs().max().item()
        scale = out.abs().max().item()
        print(f"M={M:3d}  auto eager {t_e:7.2f} us  graph {t_r:7.2f} us [{cfg_r.split(' ')[0]}]  repack(torch copy) {t_c:6.2f} us"
              f"  mfma(K') {t_m:6.2f} us [{cfg_p.split(' ')[0]}]  repack+mfma {t_b:7.2f} us"
              f"  max|diff| {d:.3g} (max|C| {scale:.3g})")


if __name__ == "__main__":
    main()
