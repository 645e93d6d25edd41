#!/usr/bin/env python3
"""Benchmark: Q4_0 x Q8_1 W4A8 GEMV on MI355X (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload:
  * N=1: BASELINE configs[1] — M=1, N=4096, K=4096, Q4_0 weights x Q8_1 activations.
  * N>1: row-sharded GEMV, 4000 weight rows per GPU (N=8 -> BASELINE configs[4], N=32000), each
    step's output slices all-gathered over RCCL (xGMI) on torch's NCCL stream, overlapped with the
    next step's kernels. Per-GPU work is fixed -> "scaling": "weak".
  * One step = G (default 64) independent GEMVs, each on a DIFFERENT resident weight copy (64 x
    9.4 MB = 604 MB > the 256 MB Infinity Cache), so every launch streams its weights from HBM
    (the decode situation: a model's layers are read once per token). Activations are one
    replicated Q8_1 vector already in HBM. The step's G launches are captured in a hipGraph.
  * value = effective TFLOPS (2*M*N*K per GEMV, all ranks) over the timed steps; "gbps" is the
    matching algorithmic byte rate (tests/benchmark/benchmark_comparison.cu:138-140 formula).
  * roofline.achieved = algorithmic bytes of ONE launch / its average duration, measured live with
    HIP events on the launch stream over the timed graph replays (so it includes each launch's
    dispatch boundary; rocprofv3's kernel-only durations are committed under profiles/).
  * "batched": the same G GEMVs issued as ONE qg_gemm_w4a8_strided_batched launch per step;
    "grouped": the same through the pointer-array entry qg_gemm_w4a8_grouped (independent B / C
    pointers per item, what a decoder layer's Q / K / V or gate / up projections can use).
  * roofline.floor_us / floor_frac: the single-launch floor under the same protocol (libqg_calib.so:
    an empty kernel with the GEMV's grid, and the best pure coalesced read of the same algorithmic
    bytes per launch over the same rotating copies) — what ONE isolated launch of this size can reach.
  * N=1 side configs: BASELINE configs[2] and [3], and configs[4]'s full N=32000 GEMV on ONE GPU as
    single launches and as one grouped launch of G — the denominators of the strong-scaling ratios.
  * N>1 "strong": the N=32000 GEMV split over the ranks (32000/N rows each), timed per step with
    the all-gather, as G single launches and as one grouped launch per step; the 1-GPU N=32000
    times measured in the same run on each rank's own GPU; strong_speedup_vs_1gpu_n32000 =
    1-GPU time per GEMV / N-GPU time per GEMV, per leg.
  * cpu_baseline (rank 0, N=1): the oracle's restatement of gemm_w4a8_reference
    (include/gemm_reference.h:175-222) on the step4 input recipe, 1 thread pinned, ~10 s sample;
    beside it the product's own host twin (libqg_host.so qg_gemm_w4a8_cpu_mt) at 1 pinned thread
    (cpu_baseline_twin) and row-partitioned over its persistent worker pool at 16 threads and at
    nproc (cpu_baseline_mt), each with median / p10 / p90.
  * data: the reference's step4 recipe (glibc srand(42), A then B, U[-1,1]) — the NMSE printed is
    then comparable to the reference's own 4.56e-3 at configs[1].
  * the kernel launches go through quant_gemm.sharded.RowShardedW4A8.compute_local (the shipped
    module; at N=1 it is the plain C-ABI call) and, for N>1, its gather.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import quant_gemm as qg  # noqa: E402
import quant_gemm.host as qhost  # noqa: E402
from quant_gemm.sharded import RowShardedW4A8, rows_per_rank, shard_rows  # noqa: E402

METRIC = "effective TFLOPS + GB/s, Q4_0×Q8_1 GEMV M=1 N=K=4096; NMSE vs FP32"
REF_GFLOPS = 622.3  # best published Q4_0xQ8_1 GEMV, M=1 N=K=4096 (RTX 5070 Laptop)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
WTYPES = {"q4_0": 2, "q4_1": 3, "q5_0": 6, "q5_1": 7}


def graph_time_us(fn, reps: int = 10, per: int = 1) -> float:
    """fn() enqueues launches on the current stream; captured once as a hipGraph, replayed `reps`
    times between HIP events on the launch stream; returns us per launch (per = launches in fn)."""
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) * 1e3 / (reps * per)


# The reference's published per-shape numbers (RTX 5070 Laptop; weight-major rows x tokens x K in its
# reports, here activation-major M tokens, N weight rows): BASELINE.md §1.
REF_PUBLISHED = {
    (1, 4096, 4096): (622.3, "docs/2d_tiling_final_report.md:70"),
    (1, 4096, 14336): (594.5, "docs/2d_tiling_final_report.md:71"),
    (2, 4096, 14336): (610.4, "docs/2d_tiling_final_report.md:72"),
    (4, 4096, 14336): (623.4, "docs/2d_tiling_final_report.md:73"),
    (2, 8192, 14336): (630.4, "docs/2d_tiling_final_report.md:74"),
    (512, 4096, 4096): (2700.0, "README.md:827-830 (tiled+dp4a, ~2.7 TFLOPS)"),
}
I8_DENSE_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: dense int8/fp8 MFMA ~5 P(FL)OPS (no sparsity)


def load_pmc(cfg_key: str, field: str):
    """A per-config PMC figure recorded by a rocprofv3 --pmc pass (profiles/*pmc*.json), if present."""
    pdir = os.path.join(REPO, "profiles")
    if not os.path.isdir(pdir):
        return None
    for f in sorted(os.listdir(pdir), reverse=True):
        if f.endswith(".json") and "pmc" in f:
            try:
                d = json.load(open(os.path.join(pdir, f)))
            except (OSError, ValueError):
                continue
            v = d.get(cfg_key, {}).get(field)
            if v is not None:
                return {"value": v, "source": f"profiles/{f}"}
    return None


def measure_config(wname: str, M: int, N: int, K: int, dev, G: int = 64, reps: int = 10,
                   forms: tuple = ("single",), label: str = "") -> list:
    """A BASELINE side config on this GPU the way the headline is measured: step4-recipe data,
    G launches of the product dispatch (qg_gemm_w4a8, auto) over rotating resident weight copies
    (> 600 MB, so every launch streams from HBM) in a hipGraph, HIP events around the replays.
    forms: "single" (G launches), "batched" (one qg_gemm_w4a8_grouped launch over the G copies),
    "prepacked" / "padded" (the load-time padded layout), "tiled" (the load-time tiled layout,
    qg_tile_weights + qg_gemm_w4a8_tiled), "tiled_act" (tiled weights and activations quantized into the tiled
    activation layout, qg_quantize_q8_1_tiled + qg_gemm_w4a8_tiled_act), "w16" (qg_gemm_w4a16_ws: FP32 activations). Every row
    carries the NMSE vs an fp64 product of the unquantized inputs of ITS OWN form's output."""
    wt = WTYPES[wname]
    bb = qg.BLOCK_BYTES[wt]
    a_h, b_h = qhost.fill_step4(M, N, K, 42, 0, N)
    a, b = torch.from_numpy(a_h).to(dev), torch.from_numpy(b_h).to(dev)
    del a_h, b_h
    aq, bq = qg.quantize_q8_1(a), qg.quantize(b, wt)
    ref = a.double() @ b.double().T
    den = torch.sum(ref ** 2)
    nmse_of = lambda c: float(torch.sum((c.double() - ref) ** 2) / den)
    af = a if "w16" in forms else None  # W4A16: the FP32 activations themselves
    ap = None
    if "padded" in forms:
        ap = qg.quantize_q8_1_padded(a)
    at = qg.quantize_q8_1_tiled(a) if "tiled_act" in forms else None  # tiled activations (round 5)
    del b
    nbytes = algo_bytes(M, N, K, bb)
    res = []
    lib = qg._lib.load()
    variant_of = {"prepacked": "repacked", "padded": "repacked", "tiled": "tiled", "tiled_act": "tiled"}
    copies, cur = None, None
    for form in forms:
        var = variant_of.get(form, "rows")
        if var != cur:
            del copies
            torch.cuda.empty_cache()
            w = bq if var == "rows" else qg.repack_weights(bq, N, K, wt) if var == "repacked" else qg.tile_weights(bq, N, K, wt)
            R = max(G, math.ceil(600e6 / w.numel()))
            copies = torch.empty((R,) + tuple(w.shape), dtype=torch.uint8, device=dev)
            copies.copy_(w.unsqueeze(0).expand_as(copies))
            cur = var
            del w
        out = torch.empty((G, M, N), dtype=torch.float32, device=dev)
        P = ctypes.c_void_p
        if form == "single":
            def step() -> None:
                for j in range(G):
                    qg.gemm_w4a8(aq, copies[j], M, N, K, wt, out=out[j])
        elif form == "tiled":
            def step() -> None:
                cs = P(torch.cuda.current_stream().cuda_stream)
                for j in range(G):
                    if lib.qg_gemm_w4a8_tiled(P(aq.data_ptr()), P(copies[j].data_ptr()), P(out[j].data_ptr()), M, N, K,
                                              wt, cs) != 0:
                        raise RuntimeError("qg_gemm_w4a8_tiled failed")
        elif form == "tiled_act":
            def step() -> None:
                cs = P(torch.cuda.current_stream().cuda_stream)
                for j in range(G):
                    if lib.qg_gemm_w4a8_tiled_act(P(at.data_ptr()), P(copies[j].data_ptr()), P(out[j].data_ptr()), M, N,
                                                  K, wt, cs) != 0:
                        raise RuntimeError("qg_gemm_w4a8_tiled_act failed")
        elif form == "prepacked":
            wsb = lib.qg_gemm_w4a8_prepacked_workspace_size(M, K)
            ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)

            def step() -> None:
                cs = P(torch.cuda.current_stream().cuda_stream)
                for j in range(G):
                    if lib.qg_gemm_w4a8_prepacked(P(aq.data_ptr()), P(copies[j].data_ptr()), P(out[j].data_ptr()), M, N, K,
                                                  wt, P(ws.data_ptr()), wsb, cs) != 0:
                        raise RuntimeError("qg_gemm_w4a8_prepacked failed")
        elif form == "w16":  # qg_gemm_w4a16 with a caller workspace (the library's is never handed to a capture)
            wsb = lib.qg_gemm_w16_workspace_size(M, N, K)
            ws16 = torch.zeros(max(wsb, 16) // 4 + 64, dtype=torch.int32, device=dev)

            def step() -> None:
                cs = P(torch.cuda.current_stream().cuda_stream)
                for j in range(G):
                    if lib.qg_gemm_w4a16_ws(P(af.data_ptr()), P(copies[j].data_ptr()), P(out[j].data_ptr()), M, N, K,
                                            P(ws16.data_ptr()), wsb, cs) != 0:
                        raise RuntimeError("qg_gemm_w4a16_ws failed")
        elif form == "padded":
            def step() -> None:
                cs = P(torch.cuda.current_stream().cuda_stream)
                for j in range(G):
                    if lib.qg_gemm_w4a8_padded(P(ap.data_ptr()), P(copies[j].data_ptr()), P(out[j].data_ptr()), M, N, K, wt,
                                               cs) != 0:
                        raise RuntimeError("qg_gemm_w4a8_padded failed")
        else:
            def step() -> None:
                qg.gemm_w4a8_grouped([aq] * G, [copies[j] for j in range(G)], [N] * G, M, K, wt,
                                     outs=[out[j] for j in range(G)])
        us = graph_time_us(step, reps, G)
        nmse = nmse_of(out[0])  # this form's own output of the timed launches
        fb = nbytes if form != "w16" else nbytes + M * K * 4 - M * (K // 32) * 36  # FP32 activations
        tops = 2.0 * M * N * K / us / 1e6
        row = {"wtype": wname if form != "w16" else wname + "_fp32_w4a16", "M": M, "N": N, "K": K, "form": form,
               "kernel_algo": int(qg.select_algo(M, N, K, wt)) if form in ("single", "batched") else None,
               "us_per_launch" if form != "batched" else "us_per_gemv": round(us, 3),
               "gbps": round(fb / us / 1e3, 1),
               "frac_hbm": round(fb / us / 1e3 / HBM_PEAK_GBPS, 4), "tops": round(tops, 2),
               "nmse_vs_fp32": nmse}
        if label:
            row["label"] = label
        pub = REF_PUBLISHED.get((M, N, K))
        if pub and form in ("single", "tiled", "tiled_act") and wname == "q4_0":
            row["ref_published_gflops"], row["ref_source"] = pub
            row["vs_ref_published"] = round(tops * 1e3 / pub[0], 2)
        if M >= 128 and form != "w16":
            cfg = f"{wname}_m{M}_n{N}_k{K}" + {"tiled": "_tiled", "tiled_act": "_tiled_act"}.get(form, "")
            row["mfma"] = {"frac_dense_i8_peak": round(tops / I8_DENSE_PEAK_TOPS, 4), "peak_tops": I8_DENSE_PEAK_TOPS,
                           "busy": load_pmc(cfg, "mfma_busy_frac"),
                           "note": "busy = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles) from a recorded --pmc pass "
                                   "of the same kernel (tools/profile_mfma.sh); frac = effective TOPS / dense i8 peak"}
        res.append(row)
        del out
    del copies, ref
    torch.cuda.empty_cache()
    return res


def measure_floor(dev, wcopies: torch.Tensor, G: int, launch_bytes: int, grid: int, block: int,
                  unit_shape=None) -> dict:
    """The single-launch floor under the headline's protocol (hipGraph of G back-to-back launches,
    HIP events on the launch stream): an empty kernel with the GEMV's grid and block, and the
    fastest pure coalesced read of the GEMV's algorithmic bytes per launch over the same rotating
    weight copies (libqg_calib.so, include/qg/qg_calib.h)."""
    lib = ctypes.CDLL(os.path.join(REPO, "llama.cpp-quant-gemm_amd", "quant_gemm", "libqg_calib.so"))
    lib.qg_calib_empty.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.qg_calib_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p]
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    R = wcopies.shape[0]
    stride = wcopies[0].numel()
    nbytes = (launch_bytes + 15) // 16 * 16
    # copies are contiguous: a read of launch_bytes from copy j stays inside the allocation for j < R-1
    bases = [wcopies.data_ptr() + (j % (R - 1)) * stride for j in range(G)]

    def empty() -> None:
        cs = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(G):
            if lib.qg_calib_empty(grid, block, cs) != 0:
                raise RuntimeError("qg_calib_empty failed")

    def reader(p: int, blk: int):
        def fn() -> None:
            cs = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            for j in range(G):
                if lib.qg_calib_read(ctypes.c_void_p(bases[j]), nbytes, p, blk, ctypes.c_void_p(sink.data_ptr()), cs) != 0:
                    raise RuntimeError("qg_calib_read failed")
        return fn

    empty_us = min(graph_time_us(empty, 10, G) for _ in range(3))
    reads = {f"x4 p{p} wg{blk}": min(graph_time_us(reader(p, blk), 10, G) for _ in range(3))
             for (p, blk) in ((1, 512), (1, 1024), (2, 512), (2, 1024), (4, 256))}
    best = min(reads, key=reads.get)
    res = {"empty_us": round(empty_us, 3), "read_us": round(reads[best], 3), "read_config": best,
           "read_all_us": {k: round(v, 3) for k, v in reads.items()}, "grid": grid, "block": block}
    if unit_shape is not None:
        # the GEMV's own load shape: 36-B units per lane, 16 rows per 1024-thread
        # workgroup, XCD tile order — without, then with, its 4-B-per-row output store
        n_rows, k = unit_shape
        lib.qg_calib_read_units.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p]
        ubuf = torch.empty(n_rows, dtype=torch.float32, device=dev)

        def units(store: bool):
            def fn() -> None:
                cs = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
                for j in range(G):
                    if lib.qg_calib_read_units(ctypes.c_void_p(bases[j]), n_rows, k,
                                               ctypes.c_void_p(ubuf.data_ptr()) if store else None,
                                               ctypes.c_void_p(sink.data_ptr()), cs) != 0:
                        raise RuntimeError("qg_calib_read_units failed")
            return fn
        res["units_read_us"] = round(min(graph_time_us(units(False), 10, G) for _ in range(3)), 3)
        res["units_read_store_us"] = round(min(graph_time_us(units(True), 10, G) for _ in range(3)), 3)
    return res


def algo_bytes(m: int, n: int, k: int, bb: int) -> int:
    """N*(K/32)*S_w + M*(K/32)*36 + M*N*4 (tests/benchmark/benchmark_comparison.cu:138-140)."""
    nb = k // 32
    return n * nb * bb + m * nb * 36 + m * n * 4


def load_traffic(cfg_key: str):
    """HBM bytes per launch from the committed PMC profile (profiles/*pmc*.json), if present."""
    pdir = os.path.join(REPO, "profiles")
    if not os.path.isdir(pdir):
        return None
    for f in sorted(os.listdir(pdir), reverse=True):
        if f.endswith(".json") and "pmc" in f:
            try:
                d = json.load(open(os.path.join(pdir, f)))
            except (OSError, ValueError):
                continue
            v = d.get(cfg_key, {}).get("hbm_bytes_per_launch")
            if v:
                return float(v)
    return None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _timed_runs(fn, seconds: float):
    fn()  # warm-up
    times, t0 = [], time.perf_counter()
    while True:
        r0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - r0)
        if time.perf_counter() - t0 >= seconds:
            break
    times.sort()
    n = len(times)
    return times[n // 2], times[n // 10], times[(9 * n) // 10], n, time.perf_counter() - t0


def cgroup_cpu_quota():
    """CPUs the cgroup grants this process (cgroup v2 cpu.max 'quota period', v1 cfs files), rounded
    up; None when unlimited or unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else max(1, -(-q // per))
    except (OSError, ValueError):
        return None


def cpu_baseline(m: int, n: int, k: int, wtype: int, seconds: float):
    """the reference is single-threaded -> the headline baseline is 1 core, pinned
    (sched_setaffinity, as taskset), after 1 warm-up, median of the runs; beside it the product's
    host twin (libqg_host.so) at 1 pinned thread and row-partitioned over its persistent worker pool.
    Bounded to ~`seconds` (+ 2 x seconds/5) of CPU work."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O  # the checker / CPU baseline only
    import numpy as np
    a, b = O.fill_uniform_step4(m, n, k, 42)
    aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, wtype)
    saved = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    core = min(saved) if saved else None
    if core is not None:
        os.sched_setaffinity(0, {core})
    try:
        per, p10, p90, runs, el = _timed_runs(lambda: O.gemm_w4a8(aq, bq, wtype), seconds)
        twin = _timed_runs(lambda: qhost.gemm_w4a8(aq, bq, m, n, k, wtype, 1), seconds / 5)
    finally:
        if saved is not None:
            os.sched_setaffinity(0, saved)
    if not np.array_equal(qhost.gemm_w4a8(aq, bq, m, n, k, wtype, 1), O.gemm_w4a8(aq, bq, wtype)):
        raise RuntimeError("host twin differs from the oracle")
    flops = 2.0 * m * n * k
    model = cpu_model()
    ms3 = lambda t: [round(x * 1e3, 4) for x in t]
    twin_row = {"value": flops / twin[0] / 1e12, "unit": "TFLOPS", "cores": 1, "kind": "port",
                "ms_per_gemv": twin[0] * 1e3, "ms_p10_p90": ms3(twin[1:3]), "cpu": model,
                "sample": f"the product's host twin libqg_host.so qg_gemm_w4a8_cpu_mt (restates "
                          f"include/gemm_reference.h:175-222), 1 thread pinned to core {core}, median of {twin[3]} runs"}
    # row-partitioned runs over the twin's persistent pool: 16 threads (the box's CPU share for one
    # GPU) and every core this process may run on — the affinity set, capped by the
    # cgroup CPU quota (nproc counts the host's cores, the quota is what the process gets)
    nproc = len(saved) if saved else (os.cpu_count() or 1)
    quota = cgroup_cpu_quota()
    usable = min(nproc, quota) if quota else nproc
    mts = []
    for threads in sorted({min(16, usable), usable}):
        mt = _timed_runs(lambda: qhost.gemm_w4a8(aq, bq, m, n, k, wtype, threads), max(1.0, seconds / 5))
        mts.append({"value": flops / mt[0] / 1e12, "unit": "TFLOPS", "cores": threads, "ms_per_gemv": mt[0] * 1e3,
                    "ms_p10_p90": ms3(mt[1:3]), "cpu": model,
                    "sample": f"libqg_host.so row-partitioned over a persistent pool of {threads} threads "
                              f"(nproc {nproc}, cgroup CPU quota {quota or 'none'}), median of {mt[3]} runs"})
    return ({"value": flops / per / 1e12, "unit": "TFLOPS", "cores": 1, "kind": "port",
             "ms_per_gemv": per * 1e3, "ms_p10_p90": ms3((p10, p90)), "cpu": model,
             "sample": f"oracle/qg_oracle.c gemm_w4a8 (restates include/gemm_reference.h:175-222), "
                       f"M={m} N={n} K={k}, median of {runs} runs in {el:.1f} s, 1 thread pinned to core "
                       f"{core}, step4 srand(42) inputs"}, twin_row, mts)


def sharded_leg(mods, aq, M: int, G: int, rows: int, world: int, steps: int, warmup: int, form: str, dev) -> dict:
    """Time one multi-GPU leg: per step G independent GEMVs on this rank's row shard (form
    "per_launch": G launches through RowShardedW4A8.compute_local; "batched": one grouped launch
    through RowShardedW4A8.compute_local_group), captured as a hipGraph, then the step's output
    slices all-gathered asynchronously (overlapping the next step's kernels), double-buffered.
    Returns the wall time per GEMV (max over ranks) and the event-timed launch-stream time."""
    R = len(mods)
    outs = [torch.zeros((G, M, rows), dtype=torch.float32, device=dev) for _ in range(2)]
    gathered = [torch.empty((world, G, M, rows), dtype=torch.float32, device=dev) for _ in range(2)]

    def step(s: int) -> None:
        if form == "per_launch":
            for j in range(G):
                mods[j % R].compute_local(aq, M, outs[s][j])
        else:
            RowShardedW4A8.compute_local_group([mods[j % R] for j in range(G)], aq, M, outs[s])

    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        step(0)
        step(1)
    torch.cuda.synchronize()
    graphs = []
    for s in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step(s)
        graphs.append(g)
    pending = [None, None]

    def run(i: int) -> None:
        s = i % 2
        if pending[s] is not None:
            pending[s].wait()
            pending[s] = None
        graphs[s].replay()
        if world > 1:
            pending[s] = mods[0].gather(outs[s], gathered[s], async_op=True)

    def drain() -> None:
        for s in range(2):
            if pending[s] is not None:
                pending[s].wait()
                pending[s] = None

    for i in range(warmup):
        run(i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for i in range(steps):
        run(i)
    ev1.record()
    drain()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    launch_us = ev0.elapsed_time(ev1) * 1e3 / (steps * G)
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    del graphs
    return {"us_per_gemv": round(elapsed / (steps * G) * 1e6, 3), "launch_stream_us_per_gemv": round(launch_us, 3)}


def native_leg(wc, aq, M: int, G: int, n_total: int, K: int, wt: int, world: int, steps: int, warmup: int, dev) -> dict:
    """The same strong-scaling step through the native C path (libqg_shard.so, include/qg/qg_shard.h):
    per step G local products (qg_sharded_gemm_w4a8_local: the rank's kernel, captured as a hipGraph)
    and ONE qg_shard_all_gather_f32 of the step's [G, M, P] slices over an RCCL communicator the
    harness creates (quant_gemm.sharded.NcclComm) on a side stream, double-buffered so the gather of
    step i overlaps step i + 1's kernels — what a C++ caller of the library does."""
    import ctypes

    from quant_gemm.sharded import NcclComm, shard_lib
    # every rank agrees before the collective communicator init (a rank that cannot load the library
    # must not leave the others waiting inside ncclCommInitRank)
    try:
        lib = shard_lib()
        ok = 1
    except Exception:  # noqa: BLE001
        lib, ok = None, 0
    flag = torch.tensor([ok], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        raise RuntimeError("libqg_shard.so did not load on every rank")
    comm = NcclComm()
    P = ctypes.c_void_p
    rows = rows_per_rank(n_total, world)
    R = wc.shape[0]
    outs = [torch.zeros((G, M, rows), dtype=torch.float32, device=dev) for _ in range(2)]
    gathered = [torch.empty((world, G, M, rows), dtype=torch.float32, device=dev) for _ in range(2)]
    gs = torch.cuda.Stream()
    done = [torch.cuda.Event(), torch.cuda.Event()]
    computed = [torch.cuda.Event(), torch.cuda.Event()]

    def step(s: int) -> None:
        st = P(torch.cuda.current_stream().cuda_stream)
        for j in range(G):
            rc = lib.qg_sharded_gemm_w4a8_local(P(aq.data_ptr()), P(wc[j % R].data_ptr()), P(outs[s][j].data_ptr()),
                                                M, n_total, K, wt, world, comm.rank, st)
            assert rc == 0, rc

    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        step(0)
        step(1)
    torch.cuda.synchronize()
    graphs = []
    for s in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step(s)
        graphs.append(g)
    started = [False, False]

    def run(i: int) -> None:
        s = i % 2
        if started[s]:
            torch.cuda.current_stream().wait_event(done[s])  # the gather that read outs[s] two steps ago
        graphs[s].replay()
        computed[s].record()
        gs.wait_event(computed[s])
        rc = lib.qg_shard_all_gather_f32(P(outs[s].data_ptr()), P(gathered[s].data_ptr()), outs[s].numel(), comm.handle,
                                         P(gs.cuda_stream))
        assert rc == 0, rc
        done[s].record(gs)
        started[s] = True

    try:
        for i in range(warmup):
            run(i)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            run(i)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # every rank's gathered step equals its own slices where they are its rows (spot check)
        ok = bool(torch.equal(gathered[(steps - 1) % 2][comm.rank], outs[(steps - 1) % 2]))
    finally:
        del graphs
        comm.close()
    return {"us_per_gemv": round(elapsed / (steps * G) * 1e6, 3), "own_slice_roundtrip_ok": ok,
            "path": "libqg_shard.so: qg_sharded_gemm_w4a8_local x G (hipGraph) + qg_shard_all_gather_f32 (RCCL) per step"}


def strong_legs(world: int, rank: int, dev, G: int, steps: int, warmup: int, M: int = 1, K: int = 4096,
                n_total: int = 32000, wname: str = "q4_0") -> dict:
    """BASELINE configs[4] as STRONG scaling: the N=32000 GEMV split over the ranks, both legs, and
    the same GEMV on ONE GPU (this rank's own) in the same run as the denominator."""
    wt = WTYPES[wname]
    s0, s1 = shard_rows(n_total, world, rank)
    rows = rows_per_rank(n_total, world)
    a_h, b_h = qhost.fill_step4(M, n_total, K, 42, s0, s1)
    aq = qg.quantize_q8_1(torch.from_numpy(a_h).to(dev))
    bq = qg.quantize(torch.from_numpy(b_h).to(dev), wt)
    del a_h, b_h
    R = max(G, math.ceil(600e6 / max(bq.numel(), 1)))
    wc = torch.empty((R,) + tuple(bq.shape), dtype=torch.uint8, device=dev)
    wc.copy_(bq.unsqueeze(0).expand_as(wc))
    mods = [RowShardedW4A8(wc[i], n_total, K, wt) for i in range(R)]
    legs = {form: sharded_leg(mods, aq, M, G, rows, world, steps, warmup, form, dev)
            for form in ("per_launch", "batched")}
    # the native C path (libqg_shard.so over its own RCCL communicator): one rank per GPU only (RCCL
    # refuses two ranks on one device, so the gloo rehearsal skips it); reported, never fatal
    if dist.get_backend() != "nccl":
        legs["native"] = {"skipped": f"needs one GPU per rank over RCCL (backend {dist.get_backend()})"}
    else:
        try:
            legs["native"] = native_leg(wc, aq, M, G, n_total, K, wt, world, steps, warmup, dev)
        except Exception as e:  # noqa: BLE001
            legs["native"] = {"error": f"{type(e).__name__}: {e}"}
    del mods, wc
    torch.cuda.empty_cache()
    one = measure_config(wname, M, n_total, K, dev, G, forms=("single", "batched"))
    one_single = one[0]["us_per_launch"]
    one_batched = one[1]["us_per_gemv"]
    return {"config": f"{wname} M={M} N={n_total} K={K}: {rows} rows per GPU x {world} GPUs, all-gather per step of {G}",
            "per_launch": legs["per_launch"], "batched": legs["batched"], "native": legs["native"],
            "one_gpu_n32000": {"single_us_per_launch": one_single, "batched_us_per_gemv": one_batched},
            "strong_speedup_vs_1gpu_n32000": {
                "per_launch": round(one_single / legs["per_launch"]["us_per_gemv"], 3),
                "batched": round(one_batched / legs["batched"]["us_per_gemv"], 3),
                "native": (round(one_single / legs["native"]["us_per_gemv"], 3) if "us_per_gemv" in legs["native"] else None),
                "note": "1-GPU us per GEMV / N-GPU us per GEMV (wall clock per step incl. the all-gather, max over "
                        "ranks), like for like per leg; DESIGN.md §7"}}


def compact_summary(out: dict) -> dict:
    """The bench line's figures in ~1.5 KB (the line's last key; see main)."""
    r = out.get("roofline") or {}
    sm = {"us": r.get("us_per_launch"), "frac": r.get("frac"), "floor_us": r.get("floor_us"),
          "units_read_store_us": (r.get("floor") or {}).get("units_read_store_us")}
    for k in ("batched", "grouped"):
        if out.get(k):
            sm[k + "_us"] = out[k]["us_per_gemv"]
            sm[k + "_frac"] = out[k]["frac"]
    if out.get("cpu_baseline"):
        sm["cpu_1core_ms"] = out["cpu_baseline"].get("ms_per_gemv")
    for x in out.get("cpu_baseline_mt") or []:
        sm[f"cpu_{x.get('cores')}t_ms"] = x.get("ms_per_gemv")
    if out.get("strong"):
        sm["strong"] = {k: v for k, v in out["strong"].items() if "speedup" in k}
    # "[wtype:]MxNxK:form=us": wtype omitted for q4_0; forms s(ingle) t(iled) ta (tiled_act) b(atched, per
    # GEMV) pp (prepacked) pd (padded) w16; fractions of HBM / the i8 peak follow from the bytes and flops
    ab = {"single": "s", "tiled": "t", "tiled_act": "ta", "batched": "b", "prepacked": "pp", "padded": "pd", "w16": "w16"}
    rows = []
    for c in out.get("side_configs") or []:
        us = c.get("us_per_launch", c.get("us_per_gemv"))  # (the batched form's rows are per GEMV)
        w = "" if c["wtype"] == "q4_0" else c["wtype"] + ":"
        rows.append(f"{w}{c['M']}x{c['N']}x{c['K']}:{ab.get(c['form'], c['form'])}={us}")
    sm["side"] = rows
    return sm


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--gemvs-per-step", type=int, default=64)
    ap.add_argument("--wtype", default="q4_0", choices=sorted(WTYPES))
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--n", type=int, default=0, help="total weight rows (default 4096 at 1 GPU, 4000/GPU beyond)")
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--algo", type=int, default=0)
    ap.add_argument("--copy-bytes", type=float, default=600e6, help="resident weight bytes to rotate through")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the side measurements of BASELINE configs[2], [3] and [4]-on-1-GPU (N = 1 only)")
    ap.add_argument("--no-floor", action="store_true", help="skip the single-launch floor (roofline.floor_us)")
    ap.add_argument("--no-strong", action="store_true", help="N > 1: skip the strong-scaling N=32000 legs")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # QG_BENCH_BACKEND=gloo with ranks sharing a device: a rehearsal of the N>1 code path on a
    # one-GPU box (the real multi-GPU run is one rank per GPU over RCCL)
    backend = os.environ.get("QG_BENCH_BACKEND", "nccl")
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        # communicator set-up outside every measured region (even with --warmup 0)
        probe = torch.zeros(world, device=dev)
        dist.all_gather_into_tensor(probe, probe[rank:rank + 1].clone())
        dist.barrier()

    wtype = WTYPES[args.wtype]
    bb = qg.BLOCK_BYTES[wtype]
    M, K, G = args.m, args.k, args.gemvs_per_step
    n_total = args.n or (4096 if world == 1 else 4000 * world)
    rows = rows_per_rank(n_total, world)
    s0, s1 = shard_rows(n_total, world, rank)
    local = s1 - s0

    # ---- synthetic data: the reference's measurement recipe (step4: glibc
    #      srand(42), A then B, U[-1,1]) from the product's host library, this rank's rows of the
    #      full N x K matrix; quantized on the GPU by the product's own kernels
    a_h, b_h = qhost.fill_step4(M, n_total, K, 42, s0, s1)
    a = torch.from_numpy(a_h).to(dev)                                   # replicated activations
    b = torch.from_numpy(b_h).to(dev)                                   # this rank's weight rows
    del a_h, b_h
    aq = qg.quantize_q8_1(a)
    bq = qg.quantize(b, wtype)
    shard_bytes = bq.numel()
    R = max(G, math.ceil(args.copy_bytes / max(shard_bytes, 1)))
    wcopies = torch.empty((R,) + tuple(bq.shape), dtype=torch.uint8, device=dev)
    wcopies.copy_(bq.unsqueeze(0).expand_as(wcopies))
    outs = [torch.zeros((G, M, rows), dtype=torch.float32, device=dev) for _ in range(2)]
    gathered = [torch.empty((world, G, M, rows), dtype=torch.float32, device=dev) for _ in range(2)]
    # the shipped multi-GPU module (quant_gemm.sharded) around each resident weight copy: its
    # compute_local is the HIP kernel through the C-ABI, its gather the one RCCL all-gather
    mods = [RowShardedW4A8(wcopies[i], n_total, K, wtype) for i in range(R)]

    # accuracy of this run's data: NMSE vs an fp64 matmul of the unquantized inputs
    c = qg.gemm_w4a8(aq, bq, M, local, K, wtype)
    ref = a.double() @ b.double().T
    num = torch.sum((c.double() - ref) ** 2)
    den = torch.sum(ref ** 2)
    if world > 1:
        nd = torch.stack([num, den])
        dist.all_reduce(nd)
        num, den = nd[0], nd[1]
    nmse = float(num / den)
    del b, ref, c

    lib = qg._lib.load()
    a_ptr = ctypes.c_void_p(aq.data_ptr())
    w_ptrs = [ctypes.c_void_p(wcopies[i].data_ptr()) for i in range(R)]

    def launch(j: int, s: int, copy: int, stream=None) -> None:
        if args.algo == 0:
            mods[copy].compute_local(aq, M, outs[s][j])
        else:  # a forced kernel family (tuning runs): the C-ABI entry with an explicit algo
            qg.gemm_w4a8(aq, wcopies[copy], M, local, K, wtype, algo=args.algo, out=outs[s][j][:, :local])

    def step_eager(s: int, base: int = 0) -> None:
        for j in range(G):
            launch(j, s, (base + j) % R)

    # ---- hipGraph of one step per output buffer
    graphs = None
    if not args.no_graph:
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            step_eager(0)
            step_eager(1)
        torch.cuda.synchronize()
        graphs = []
        for s in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step_eager(s)
            graphs.append(g)

    pending = [None, None]

    def run_step(i: int) -> None:
        s = i % 2
        if pending[s] is not None:
            pending[s].wait()           # the gather that read outs[s] two steps ago
            pending[s] = None
        if graphs is not None:
            graphs[s].replay()
        else:
            step_eager(s)
        if world > 1:
            pending[s] = mods[0].gather(outs[s], gathered[s], async_op=True)

    def drain() -> None:
        for s in range(2):
            if pending[s] is not None:
                pending[s].wait()
                pending[s] = None

    for i in range(args.warmup):
        run_step(i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for i in range(args.steps):
        run_step(i)
    ev1.record()
    drain()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # GEMV stream time on the launch stream (HIP events), per launch: includes each launch's
    # dispatch boundary, i.e. what a stream of back-to-back GEMVs really costs
    launch_us = ev0.elapsed_time(ev1) * 1e3 / (args.steps * G)
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- per-step distribution (median, p10, p90), in its own pass after the
    #      timed region: HIP events around each step's launches on the launch stream
    step_pct = None
    if graphs is not None:
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(max(args.steps, 10))]
        for i, (ea, eb) in enumerate(evs):
            ea.record()
            graphs[i % 2].replay()
            eb.record()
        torch.cuda.synchronize()
        per = sorted(ea.elapsed_time(eb) * 1e3 / G for ea, eb in evs)
        q = lambda f: round(per[min(len(per) - 1, int(f * len(per)))], 3)
        step_pct = {"p10": q(0.1), "p50": q(0.5), "p90": q(0.9), "steps": len(per),
                    "note": "us per launch, per step (HIP events around each step's graph replay)"}

    # ---- the same G GEMVs as ONE strided-batched launch (qg_gemm_w4a8_strided_batched): the
    #      per-launch dispatch cost is paid once per step instead of once per GEMV
    batched_us = None
    if R >= G:
        fnb = lib.qg_gemm_w4a8_strided_batched
        bout = torch.empty((G, M, rows), dtype=torch.float32, device=dev)
        cs = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

        def launch_batched(first: int) -> None:
            st = fnb(a_ptr, 0, w_ptrs[first], shard_bytes, ctypes.c_void_p(bout.data_ptr()), M * rows, G, M,
                     local, K, wtype, cs)
            if st != 0:
                raise RuntimeError(f"qg_gemm_w4a8_strided_batched failed: {st}")

        for _ in range(3):
            launch_batched(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        nrep = 20
        e0.record()
        for r in range(nrep):
            launch_batched(0 if (r % 2 == 0 or R < 2 * G) else G)
        e1.record()
        torch.cuda.synchronize()
        batched_us = e0.elapsed_time(e1) * 1e3 / (nrep * G)
        # parity of the batched launch against the per-launch results of the timed region
        if not torch.equal(bout[0, :, :local], outs[0][0, :, :local]):
            raise RuntimeError("batched GEMV differs from the single-launch GEMV")

    # ---- the same G GEMVs as ONE pointer-array grouped launch (qg_gemm_w4a8_grouped, through the
    #      shipped module's compute_local_group): independent weight / output pointers per item
    grouped_us = None
    if graphs is not None and args.algo == 0:
        gout = torch.zeros((G, M, rows), dtype=torch.float32, device=dev)
        grouped_us = graph_time_us(lambda: RowShardedW4A8.compute_local_group(mods[:G], aq, M, gout), 20, G)
        if not torch.equal(gout[:, :, :local], outs[0][:, :, :local]):
            raise RuntimeError("grouped GEMV differs from the single-launch GEMV")

    # ---- the single-launch floor of this size under the same protocol (roofline.floor_us)
    floor = None
    if graphs is not None and not args.no_floor:
        rpb = 16  # the M = 1 GEMV's rows per 1024-thread workgroup (qg_gemv.hip)
        floor = measure_floor(dev, wcopies, G, algo_bytes(M, local, K, bb), (local + rpb - 1) // rpb, 1024,
                              unit_shape=(local, K) if (M == 1 and wtype == 2 and K <= 4096 and K % 64 == 0) else None)

    # ---- N > 1: the step's all-gather alone (same bytes, no GEMVs beside it), so the per-GPU kernel
    #      time and the gather latency are reported separately (SURVEY.md §7, 8-GPU hard part)
    gather_us = None
    if world > 1:
        for _ in range(3):
            dist.all_gather_into_tensor(gathered[0].view(-1), outs[0].view(-1))
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        ng = 20
        for _ in range(ng):
            dist.all_gather_into_tensor(gathered[0].view(-1), outs[0].view(-1))
        torch.cuda.synchronize()
        gather_us = (time.perf_counter() - g0) / ng * 1e6

    # ---- hot (Infinity-Cache resident) reference point: one copy, same launch count
    hot_us = None
    if graphs is not None:
        g_hot = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_hot):
            for j in range(G):
                launch(j, 0, 0)
        for _ in range(3):
            g_hot.replay()
        torch.cuda.synchronize()
        th = time.perf_counter()
        for _ in range(10):
            g_hot.replay()
        torch.cuda.synchronize()
        hot_us = (time.perf_counter() - th) / (10 * G) * 1e6

    strong = None
    if world > 1 and not args.no_strong and graphs is not None:
        del mods, wcopies
        torch.cuda.empty_cache()
        strong = strong_legs(world, rank, dev, G, args.steps, args.warmup)

    flops_per_gemv = 2.0 * M * n_total * K
    total_flops = flops_per_gemv * G * args.steps
    bytes_per_gemv_all = n_total * (K // 32) * bb + world * M * (K // 32) * 36 + M * n_total * 4
    launch_bytes = algo_bytes(M, local, K, bb)
    value = total_flops / elapsed / 1e12
    achieved = launch_bytes / (launch_us * 1e-6) / 1e9
    cfg_key = f"{args.wtype}_m{M}_n{local}_k{K}"
    traffic = load_traffic(cfg_key)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "TFLOPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value * 1e3 / REF_GFLOPS, 3),
            "dtype": "int8",
            "data": "synthetic: the reference's step4 recipe (glibc srand(42), A then B, U[-1,1]; "
                    "quant_gemm.host.fill_step4), quantized on-GPU to Q8_1 / weights by the product's quantizers",
            "config": {"workload": f"{args.wtype}_q8_1_gemv", "M": M, "N": n_total, "K": K,
                       "rows_per_gpu": local, "gemvs_per_step": G, "weight_copies": R,
                       "parallelism": f"row-shard x{world}" + (
                           (" + RCCL all-gather" if backend == "nccl" else f" + {backend} all-gather") if world > 1 else ""),
                       "launch": "hipGraph" if graphs is not None else "eager",
                       "kernel_algo": int(qg.select_algo(M, local, K, wtype)) if args.algo == 0 else args.algo},
            "gbps": round(bytes_per_gemv_all * G * args.steps / elapsed / 1e9, 1),
            "us_per_gemv": round(elapsed / (args.steps * G) * 1e6, 3),
            "nmse_vs_fp32": nmse,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "us_per_launch": round(launch_us, 3), "bytes_per_launch": launch_bytes,
                         "timing": "HIP events on the launch stream over the timed graph replays, "
                                   "per launch incl. its dispatch boundary",
                         "per_step": step_pct,
                         "floor_us": None if floor is None else floor["read_us"],
                         "floor_frac": None if floor is None else round(launch_bytes / floor["read_us"] / 1e3 / HBM_PEAK_GBPS, 4),
                         "floor": None if floor is None else dict(floor, note=(
                             "single-launch floor, same protocol: empty kernel with the GEMV grid, and the fastest "
                             "pure 16-B coalesced read of bytes_per_launch per launch over the same rotating copies; "
                             "units_read(_store)_us: the GEMV's own 36-B-unit load shape and grid without its "
                             "arithmetic, without / with its output store (libqg_calib.so)"))},
            "batched": None if batched_us is None else {
                "us_per_gemv": round(batched_us, 3),
                "tflops": round(flops_per_gemv / world / batched_us / 1e6, 3),
                "gbps": round(launch_bytes / batched_us / 1e3, 1),
                "frac": round(launch_bytes / batched_us / 1e3 / HBM_PEAK_GBPS, 4),
                "note": f"{G} GEMVs on distinct weight copies per qg_gemm_w4a8_strided_batched launch"},
            "grouped": None if grouped_us is None else {
                "us_per_gemv": round(grouped_us, 3),
                "frac": round(launch_bytes / grouped_us / 1e3 / HBM_PEAK_GBPS, 4),
                "note": f"{G} GEMVs on distinct weight copies per qg_gemm_w4a8_grouped launch (pointer array)"},
            "strong": strong,
            "gather": None if gather_us is None else {
                "us_per_step": round(gather_us, 2), "bytes_per_rank": G * M * rows * 4,
                "note": f"all_gather_into_tensor of one step's {G} output slices alone ({backend})"},
            "hot_l3": None if hot_us is None else {"us_per_gemv": round(hot_us, 3),
                                                   "tflops": round(flops_per_gemv / world / hot_us / 1e6, 3)},
        }
        if world == 1 and not args.no_cpu_baseline:
            one, twin, mt = cpu_baseline(M, n_total, K, wtype, args.cpu_seconds)
            rnd = lambda d: {k: (round(v, 6) if isinstance(v, float) else v) for k, v in d.items()}
            out["cpu_baseline"] = rnd(one)
            out["cpu_baseline_twin"] = rnd(twin)
            out["cpu_baseline_mt"] = [rnd(x) for x in mt]
        else:
            out["cpu_baseline"] = None
        if world == 1 and not args.no_configs and args.wtype == "q4_0" and args.n == 0 and args.m == 1 and args.k == 4096:
            # BASELINE configs[2] (the M=32 prefill) and configs[3] (all-quants GEMV), measured on the
            # same GPU in the same run (parity cases otherwise; not part of `value`)
            torch.cuda.empty_cache()
            # plus configs[4]'s full N=32000 GEMV on this ONE GPU, single launches and one grouped launch
            # of G: the denominators of the N>1 strong-scaling ratios
            del mods, wcopies
            torch.cuda.empty_cache()
            sides = [("q4_0", 32, 4096, 4096, ("single", "tiled", "tiled_act"), "configs[2]"),
                     ("q4_0", 1, 4096, 4096, ("tiled",), "configs[1] on the tiled layout (decode GEMV)"),
                     ("q4_0", 2, 4096, 4096, ("single", "tiled"), "decode M=2, both layouts"),
                     ("q4_0", 4, 4096, 4096, ("single", "tiled"), "decode M=4, both layouts"),
                     ("q4_1", 1, 4096, 4096, ("single",), "configs[3]"),
                     ("q5_0", 1, 4096, 4096, ("single",), "configs[3]"), ("q5_1", 1, 4096, 4096, ("single",), "configs[3]"),
                     ("q4_0", 1, 32000, 4096, ("single", "batched"), "configs[4] on one GPU"),
                     # odd K/32 at a prefill size: the load-time padded layout and the
                     # tiled layout (round 5)
                     ("q4_0", 32, 4096, 4128, ("prepacked", "padded", "tiled", "tiled_act"), "odd K/32"),
                     # row f3: the W4A16 prefill (FP32 activations x Q4_0), M = 32
                     ("q4_0", 32, 4096, 4096, ("w16",), "row f3"),
                     # the reference's published shapes: 2D-tile table
                     # (docs/2d_tiling_final_report.md:70-74, weight-major 4096/8192 x tokens x 14336), the
                     # llama-shape batch-decode sweep (tests/test_llama_shapes.cu:6,256: 1..8 tokens at
                     # 4096 x 14336) and the step4 prefill sizes (tests/step4_w4a8_gemm.cu:278-281)
                     ("q4_0", 1, 4096, 14336, ("single", "tiled"), "published 4096x1x14336"),
                     ("q4_0", 2, 4096, 14336, ("single", "tiled"), "published 4096x2x14336"),
                     ("q4_0", 3, 4096, 14336, ("single", "tiled"), "llama-shape sweep"),
                     ("q4_0", 4, 4096, 14336, ("single", "tiled"), "published 4096x4x14336"),
                     ("q4_0", 5, 4096, 14336, ("single", "tiled"), "llama-shape sweep"),
                     ("q4_0", 8, 4096, 14336, ("single", "tiled"), "llama-shape sweep"),
                     ("q4_0", 2, 8192, 14336, ("single",), "published 8192x2x14336"),
                     ("q4_0", 128, 4096, 4096, ("single", "tiled"), "step4 prefill"),
                     ("q4_0", 512, 4096, 4096, ("single", "tiled", "tiled_act"), "step4 prefill (published ~2.7 TFLOPS)"),
                     ("q4_0", 512, 4096, 14336, ("single", "tiled"), "step4 prefill")]
            out["side_configs"] = [r for (w, m_, n_, k_, f, lab) in sides
                                   for r in measure_config(w, m_, n_, k_, dev, forms=f, label=lab)]
        # LAST key: the driver keeps only the tail of stdout, so a compact restatement of
        # the figures above ends the line — headline, floor, batched / grouped, CPU rows and every side config
        # as "wtype/MxNxK/form=us@frac_hbm"
        out["summary"] = compact_summary(out)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
