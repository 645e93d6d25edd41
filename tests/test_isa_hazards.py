"""MFMA result hazard, checked on the shipped code object (CPU only).

gfx950 needs 8 wait states between an MFMA and the first instruction that touches its destination
registers with a non-MFMA instruction (VALU, LDS, memory): tools/mfma_hazard_probe.hip, run on
an MI355X (profiles/r02_tuning/mfma_hazard_probe.txt), reads v_mfma_i32_16x16x32_i8 and
v_mfma_f32_16x16x16_f16 results after exactly N states inside one asm string — wrong in all 64
lanes at N <= 6, right from N = 8 — and hipcc pads exactly that (`s_nop 7`). The prefill kernel
adds `s_nop 7; s_nop 7` of its own after its MFMA phases (qg_mmq_kernel.hpp). This test
disassembles every gfx950 kernel in libqg_hip.so and asserts that no straight-line path from a
v_mfma to an access of its destination has fewer than 8 wait states (s_nop N counts N + 1, any
other instruction 1), so a compiler update that pads less fails here instead of in the sums.
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "llama.cpp-quant-gemm_amd", "quant_gemm", "libqg_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
REQUIRED = 8
# the 32 x 32 shapes (16 passes; the large-M prefill, qg_mmql_kernel.hpp) are held to 18, the CDNA3 ISA's
# figure for a 16-pass XDL result read by VALU (not probed on gfx950: a margin, not a measurement)
REQUIRED_32 = 18
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")
STOP = ("s_branch", "s_cbranch", "s_setpc", "s_endpgm", "s_barrier")


def regs(text):
    out = set()
    for kind, lo, hi, one in REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


@pytest.fixture(scope="module")
def listing(tmp_path_factory):
    if not (os.path.exists(OBJDUMP) and os.path.exists(LIB)):
        pytest.skip("llvm-objdump or libqg_hip.so missing")
    d = tmp_path_factory.mktemp("co")
    so = shutil.copy(LIB, d / "libqg_hip.so")
    subprocess.run([OBJDUMP, "--offloading", str(so)], cwd=d, capture_output=True, check=True)
    text = []
    for f in sorted(os.listdir(d)):
        if "gfx950" in f:
            text.append(subprocess.run([OBJDUMP, "-d", str(d / f)], capture_output=True, text=True, check=True).stdout)
    assert text, "no gfx950 code object in libqg_hip.so"
    return "\n".join(text)


def instructions(listing):
    """(function, [instruction text]) for every kernel."""
    fn, body = None, []
    for line in listing.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            if fn:
                yield fn, body
            fn, body = m.group(1), []
            continue
        ins = line.strip().split("//")[0].strip()
        if fn and ins:
            body.append(ins)
    if fn:
        yield fn, body


def test_mfma_results_padded(listing):
    checked, violations, mfmas, wide, chained = 0, [], 0, [], 0
    for fn, body in instructions(listing):
        for i, ins in enumerate(body):
            if not ins.startswith("v_mfma"):
                continue
            mfmas += 1
            if "_32x32x" in ins.split()[0]:
                wide.append(ins.split()[0])
            ops = ins.split(None, 1)[1]
            dst = regs(ops.split(",")[0])
            states = 0
            for nxt in body[i + 1:]:
                op = nxt.split()[0]
                if op.startswith(STOP):
                    break
                touched = regs(nxt.split(None, 1)[1]) if " " in nxt else set()
                if touched & dst:
                    if op.startswith("v_mfma"):
                        # MFMA -> MFMA dependencies (accumulator chains, operand forwarding) are the
                        # matrix pipe's own interlock and hipcc's; once another MFMA rewrites these
                        # registers, later readers belong to it (checked from its own position)
                        if regs(nxt.split(None, 1)[1].split(",")[0]) & dst:
                            chained += 1
                            break
                    else:
                        checked += 1
                        need = REQUIRED_32 if "_32x32x" in ins.split()[0] else REQUIRED
                        if states < need:
                            violations.append(f"{fn}: {ins} -> {nxt} after {states} wait states")
                        break
                m = re.match(r"s_nop\s+(\d+)", nxt)
                states += int(m.group(1)) + 1 if m else 1
    assert mfmas > 100, "expected the prefill / W4A16 MFMA kernels in the library"
    assert any("_32x32x" in f for f in wide), "expected the large-M prefill's 32 x 32 MFMAs"
    # (accumulation chains: only the last MFMA of a chain has its result read by another unit)
    assert checked > (mfmas - chained) // 4, (checked, mfmas, chained)
    assert not violations, "\n".join(violations[:20])


# Cross-opcode MFMA register reuse (round 6, qg_gemvm.hip header): an MFMA that writes registers which an
# MFMA of ANOTHER opcode issued shortly before still reads as its accumulator input (into a different
# destination) or writes itself. hipcc emitted `i8 v[22:25] <- C bias; i8 v[14:17] <- C v[22:25]; f16
# v[22:25]` with 0 wait states, and on an MI355X the f16 result came out wrong whenever CUs held several
# workgroups. In-place accumulation (vdst == SrcC, the next MFMA reading the same registers) is the matrix
# pipe's own chain and is allowed.
MFMA_REUSE_STATES = 16


def test_no_cross_opcode_mfma_register_reuse(listing):
    violations, mfmas = [], 0
    for fn, body in instructions(listing):
        for i, ins in enumerate(body):
            if not ins.startswith("v_mfma"):
                continue
            mfmas += 1
            op1 = ins.split()[0]
            ops = [o.strip() for o in ins.split(None, 1)[1].split(",")]
            dst = regs(ops[0])
            srcc = regs(ops[3]) if len(ops) > 3 else set()
            states = 0
            for nxt in body[i + 1:]:
                op = nxt.split()[0]
                if op.startswith(STOP) or states >= MFMA_REUSE_STATES:
                    break
                if op.startswith("v_mfma") and op != op1:
                    d2 = regs(nxt.split(None, 1)[1].split(",")[0])
                    if d2 & (srcc - dst) or d2 & dst:
                        violations.append(f"{fn}: {ins} -> {nxt} after {states} wait states")
                m = re.match(r"s_nop\s+(\d+)", nxt)
                states += int(m.group(1)) + 1 if m else 1
    assert mfmas > 100
    assert not violations, "\n".join(violations[:20])


def test_hot_kernels_use_no_scratch(tmp_path):
    """Every hot-path kernel (GEMV, tiled decode GEMV, MFMA small-batch decode, MFMA prefill, large-M prefill)
    keeps its live values in registers: private_segment_fixed_size 0 in the code object metadata. A spill
    under the 128-VGPR cap of a 1024-thread workgroup (round 6: the small-batch decode's Q5_0 ring at 8 stages
    per lane) turns into scratch traffic on every launch."""
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not (os.path.exists(OBJDUMP) and os.path.exists(readelf) and os.path.exists(LIB)):
        pytest.skip("llvm tools or libqg_hip.so missing")
    so = shutil.copy(LIB, tmp_path / "libqg_hip.so")
    subprocess.run([OBJDUMP, "--offloading", str(so)], cwd=tmp_path, capture_output=True, check=True)
    notes = ""
    for f in sorted(os.listdir(tmp_path)):
        if "gfx950" in f:
            notes += subprocess.run([readelf, "--notes", str(tmp_path / f)], capture_output=True, text=True,
                                    check=True).stdout
    sizes, name = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s*\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name:
            sizes[name] = int(m.group(1))
    hot = {n: v for n, v in sizes.items() if re.search(r"(gemv|gemvt|gemvm|mmq|mmqt|mmql)\w*_kernel", n)}
    assert len(hot) > 100, len(hot)
    spills = sorted(n for n, v in hot.items() if v)
    assert not spills, spills[:20]
