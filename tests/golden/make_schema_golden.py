"""Golden fixtures for the Solution registrations (integration/solutions/*.json), generated in the
build container only from the DEFINITIONS those solutions register against:

  /root/reference/schemas/definitions/gemm/gemm_q4_0_q8_1_w4a8.json  (inputs A_q8_1[M,K/QK],
      B_q4_0[N,K/QK] -> C[M,N], :35-53; Python reference `run(A_q8_1, B_q4_0)`, :96)
  /root/reference/schemas/definitions/gemm/gemm_q4_0_w4a16.json      (A f32[M,K], B_q4_0 -> C[M,N])
  /root/reference/schemas/definitions/gemm/gemm_fp32_baseline.json   (A f32[M,K], B f32[N,K] -> C[M,N])

These definitions' Python references read blocks by attribute (`w_block.d`, `a_block.ds.x`,
`a_block.ds.y`, `block.qs[i]`), so the generator hands them small attribute records built from the
packed bytes (d / ds as the float value of the stored f16, qs as the stored codes, Q8_1 qs signed).
The reference code was read and executed at generation time (round 3) and never stored; the
fixtures hold only inputs and outputs. Since round 4 the script refuses to run without the explicit
opt-in flag and runs the code only after the allowlist checks of tests/golden/defexec.py (ADVICE
r03); in round 4 this build environment denied executing the reference's code, so the
committed fixtures are the round-3 ones and no new ones are generated. Inputs follow the step4 recipe (glibc srand, U[-1,1]) through the CPU
oracle's quantizers (the same bytes as include/quantize.h, pinned in tests/test_oracle.py).

Usage:  python tests/golden/make_schema_golden.py --exec-reference-definitions [--ref /root/reference] [--force]
"""
from __future__ import annotations

import argparse
import os
import sys
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402
from defexec import EXEC_FLAG, load_definition_fn, require_opt_in  # noqa: E402


def load_definition(ref_root: str, name: str):
    spec, run, _ = load_definition_fn(os.path.join(ref_root, "schemas", "definitions", "gemm", name + ".json"))
    return spec, run


def _f16(lo: int, hi: int) -> float:
    return float(np.frombuffer(bytes([lo, hi]), dtype=np.float16)[0])


def q4_0_records(q: np.ndarray) -> np.ndarray:
    """uint8 [rows, nb, 18] -> object [rows, nb] of {d, qs[16]} records."""
    rows, nb, _ = q.shape
    out = np.empty((rows, nb), dtype=object)
    for r in range(rows):
        for b in range(nb):
            blk = q[r, b]
            out[r, b] = SimpleNamespace(d=_f16(blk[0], blk[1]), qs=[int(x) for x in blk[2:18]])
    return out


def q8_1_records(q: np.ndarray) -> np.ndarray:
    """uint8 [rows, nb, 36] -> object [rows, nb] of {ds.x, ds.y, qs[32] signed} records."""
    rows, nb, _ = q.shape
    out = np.empty((rows, nb), dtype=object)
    for r in range(rows):
        for b in range(nb):
            blk = q[r, b]
            ds = SimpleNamespace(x=_f16(blk[0], blk[1]), y=_f16(blk[2], blk[3]))
            out[r, b] = SimpleNamespace(ds=ds, qs=[int(x) for x in blk[4:36].view(np.int8)])
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--force", action="store_true")
    ap.add_argument(EXEC_FLAG, dest="exec_ok", action="store_true",
                    help="allow executing the reference's definition code (defexec.py checks)")
    args = ap.parse_args()
    require_opt_in(args.exec_ok, "make_schema_golden.py")
    import torch

    _, run_w4a8 = load_definition(args.ref, "gemm_q4_0_q8_1_w4a8")
    _, run_w4a16 = load_definition(args.ref, "gemm_q4_0_w4a16")
    _, run_fp32 = load_definition(args.ref, "gemm_fp32_baseline")

    cases = {}
    for (m, n, k, seed) in [(2, 8, 128, 42), (3, 5, 96, 7), (1, 8, 4096, 42), (5, 6, 512, 9), (3, 4, 4128, 11)]:
        a, b = O.fill_uniform_step4(m, n, k, seed)
        aq, bq = O.quantize(a, O.Q8_1), O.quantize(b, O.Q4_0)
        c = run_w4a8(q8_1_records(aq), q4_0_records(bq))
        cases[f"schema_w4a8_m{m}n{n}k{k}"] = dict(
            definition="gemm_q4_0_q8_1_w4a8", m=np.int32(m), n=np.int32(n), k=np.int32(k), seed=np.int32(seed),
            A_q8_1=aq, B_q4_0=bq, C=c.numpy().astype(np.float32))
    for (m, n, k, seed) in [(2, 16, 256, 42), (3, 8, 96, 5), (1, 4, 4096, 42), (9, 6, 256, 3)]:
        a, b = O.fill_uniform_step4(m, n, k, seed)
        bq = O.quantize(b, O.Q4_0)
        c = run_w4a16(torch.from_numpy(a), q4_0_records(bq))
        cases[f"schema_w4a16_m{m}n{n}k{k}"] = dict(
            definition="gemm_q4_0_w4a16", m=np.int32(m), n=np.int32(n), k=np.int32(k), seed=np.int32(seed),
            A=a, B_q4_0=bq, C=c.numpy().astype(np.float32))
    for (m, n, k, seed) in [(2, 16, 256, 42), (3, 7, 100, 5)]:
        a, b = O.fill_uniform_step4(m, n, k, seed)
        c = run_fp32(torch.from_numpy(a), torch.from_numpy(b))
        cases[f"schema_fp32_m{m}n{n}k{k}"] = dict(
            definition="gemm_fp32_baseline", m=np.int32(m), n=np.int32(n), k=np.int32(k), seed=np.int32(seed),
            A=a, B=b, C=c.numpy().astype(np.float32))

    for name, d in cases.items():
        path = os.path.join(HERE, f"{name}.npz")
        if os.path.exists(path) and not args.force:
            continue
        np.savez_compressed(path, **d)
        print(f"{name}: C[0,:3]={d['C'].ravel()[:3]}")


if __name__ == "__main__":
    main()
