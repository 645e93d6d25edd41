"""Solution registrations (integration/solutions/*.json) against the definitions they name.

The reference's FlashInfer-Bench-style schema (schemas/docs/solution.md:27-42) binds a Solution to
a Definition through `spec.entry_point = "file::function"`, destination-passing: the harness calls
the function with the definition's inputs in order, then its outputs, then the axes. The three
GEMM definitions registered here (schemas/definitions/gemm/*.json) are all activation-major:

  gemm_q4_0_q8_1_w4a8  inputs A_q8_1[M,K/QK], B_q4_0[N,K/QK]   output C[M,N]  (:35-53)
  gemm_q4_0_w4a16      inputs A[M,K] f32,     B_q4_0[N,K/QK]   output C[M,N]
  gemm_fp32_baseline   inputs A[M,K] f32,     B[N,K] f32       output C[M,N]

and the two quantization definitions (schemas/definitions/quantization/*.json, round 4):

  quantize_q8_1        input x[num_elements] f32   output y[num_elements/QK] q8_1  (:26-33)
  quantize_q4_0        input x[num_elements] f32   output y[num_elements/QK] q4_0  (:25-32)

The quantization Solutions are checked on the GPU byte for byte against oracle.quantize_definition
(the definitions' semantics restated; Q8_1 pinned by the flashinfer definition's committed bytes,
tests/test_oracle.py) — no output of the schema definitions' own code exists as a fixture (executing
it was denied in round 4).

CPU tests: every solution parses, names a known definition, and its entry point is declared in
include/qg/qg.h with exactly that parameter order and exported by libqg_hip.so. GPU tests resolve
each entry point by name from the library (dlsym through ctypes), call it in definition order and
match the definition's own outputs (tests/golden/schema_*.npz, tests/golden/make_schema_golden.py).
"""
import ctypes
import glob
import json
import os
import re

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SOLUTIONS = sorted(glob.glob(os.path.join(REPO, "integration", "solutions", "*.json")))
GOLD = os.path.join(HERE, "golden")
LIB = os.path.join(REPO, "llama.cpp-quant-gemm_amd", "quant_gemm", "libqg_hip.so")

# definition -> (inputs, outputs, var axes) as schemas/definitions/<group>/<name>.json lists them
DEFINITIONS = {
    "gemm_q4_0_q8_1_w4a8": (["A_q8_1", "B_q4_0"], ["C"], ["M", "N", "K"]),
    "gemm_q4_0_w4a16": (["A", "B_q4_0"], ["C"], ["M", "N", "K"]),
    "gemm_fp32_baseline": (["A", "B"], ["C"], ["M", "N", "K"]),
    "quantize_q8_1": (["x"], ["y"], ["num_elements"]),
    "quantize_q4_0": (["x"], ["y"], ["num_elements"]),
}
GROUP = {name: ("quantization" if name.startswith("quantize_") else "gemm") for name in DEFINITIONS}


def header_params(symbol):
    text = open(os.path.join(REPO, "include", "qg", "qg.h")).read()
    m = re.search(r"\bint\s+" + re.escape(symbol) + r"\s*\(([^)]*)\)\s*;", text)
    assert m, f"{symbol} not declared in include/qg/qg.h"
    return [re.split(r"[\s*]+", p.strip())[-1] for p in m.group(1).split(",")]


def load(path):
    with open(path) as f:
        return json.load(f)


def entry_symbol(sol):
    path, fn = sol["spec"]["entry_point"].split("::")
    assert path == "include/qg/qg.h"
    return fn


def test_solutions_present():
    names = {load(p)["definition"] for p in SOLUTIONS}
    assert names == set(DEFINITIONS)


@pytest.mark.parametrize("path", SOLUTIONS, ids=os.path.basename)
def test_solution_entry_point_matches_definition(path):
    sol = load(path)
    assert sol["spec"]["destination_passing_style"] is True
    assert sol["spec"]["target_hardware"] == ["gfx950"]
    for s in sol["sources"]:
        assert os.path.exists(os.path.join(REPO, s["path"])), s["path"]
    inputs, outputs, axes = DEFINITIONS[sol["definition"]]
    fn = entry_symbol(sol)
    assert header_params(fn) == inputs + outputs + axes + ["stream"]
    assert re.sub(r"\s+", " ", sol["spec"]["signature"]).startswith(f"int {fn}(")


@pytest.mark.parametrize("path", SOLUTIONS, ids=os.path.basename)
def test_entry_point_exported(path):
    """dlsym of the registered name in the built library (loading needs no GPU)."""
    lib = ctypes.CDLL(LIB)
    assert hasattr(lib, entry_symbol(load(path)))


@pytest.mark.skipif(not os.path.isdir("/root/reference/schemas"), reason="reference tree only in the build container")
@pytest.mark.parametrize("name", sorted(DEFINITIONS))
def test_definition_table_matches_reference(name):
    """The definitions' declared inputs / outputs / var axes (their JSON data, read as text)."""
    d = load(f"/root/reference/schemas/definitions/{GROUP[name]}/{name}.json")
    var_axes = [a for a, v in d["axes"].items() if v.get("type") == "var"]
    assert (list(d["inputs"]), list(d["outputs"]), var_axes) == DEFINITIONS[name]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "schema_*.npz"))), ids=os.path.basename)
def test_schema_golden_on_oracle(O, path):
    """The definitions' own outputs vs the CPU oracle (pins the fixtures and the bound used on the GPU)."""
    g = np.load(path)
    name = str(g["definition"])
    if name == "gemm_q4_0_q8_1_w4a8":
        ref, s = O.gemm_w4a8(g["A_q8_1"], g["B_q4_0"], O.Q4_0, want_sumi=True)
        tol = O.summation_tol(g["A_q8_1"], g["B_q4_0"], s, O.Q4_0) + 1e-6 * np.abs(g["C"])
    elif name == "gemm_q4_0_w4a16":
        ref = O.gemm_w4a16(g["A"], g["B_q4_0"])
        tol = O.w16_tol(g["A"], g["B_q4_0"], O.Q4_0)
    else:
        ref = O.gemm_fp32(g["A"], g["B"]).astype(np.float64)
        tol = 2 * (g["A"].shape[1] + 2) * 2.0**-24 * (np.abs(g["A"]) @ np.abs(g["B"]).T)
    assert (np.abs(g["C"].astype(np.float64) - ref) <= tol).all()
