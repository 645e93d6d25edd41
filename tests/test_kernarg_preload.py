"""Kernel-argument preload, checked on the shipped code object (CPU only).

csrc/Makefile builds with `-mllvm -amdgpu-kernarg-preload-count=16`: the dispatch packet's first
kernel-argument dwords arrive in SGPRs, so a wave's first global loads need no s_load of the
kernarg segment (≈0.3 µs of the headline GEMV's 3.3 µs in round 2,
profiles/r02_tuning/ab_kernarg_preload.txt). The flag is an internal LLVM option and the win
depends on argument order, so a toolchain that stops honouring it would silently cost ≈10 % of the
headline. This test reads every gfx950 kernel descriptor (`<kernel>.kd`, 64 bytes; bits 6:0 of the
u16 at byte 58 = KERNARG_PRELOAD_SPEC_LENGTH in dwords, LLVM AMDGPUUsage "Kernel Descriptor") and
asserts that the hot-path kernels preload at least every argument their first loads use.
"""
import glob
import os
import shutil
import struct
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "llama.cpp-quant-gemm_amd", "quant_gemm", "libqg_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

# kernel family (mangled-name prefix) -> dwords its first loads need:
#   gemv1_kernel(A, B, N, K, out): everything (2 + 2 + 1 + 1 + 2)
#   gemvs_kernel(A, B, M, N, K, out, ...): the pointers and sizes before out (2 + 2 + 3)
#   mmq1_kernel(A, B, M, N, K, C, ...): 2 + 2 + 3 + 2
#   mmq_kernel(A, B, C, sumi, M, N, K, ...): 2 + 2 + 2 + 2 + 3
REQUIRED = {
    "_ZN2qg12gemv1_kernel": 8,
    "_ZN2qg12gemvs_kernel": 7,
    "_ZN2qg11mmq1_kernel": 9,
    "_ZN2qg10mmq_kernel": 11,
}


def kernel_descriptors(path):
    """{symbol: 64-byte descriptor} for the .kd symbols of one ELF64 code object."""
    data = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    out = {}
    for s in secs:
        if s[1] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[s[6]]
        for j in range(s[5] // 24):
            name, _, _, shndx, value, _ = struct.unpack_from("<IBBHQQ", data, s[4] + j * 24)
            start = strtab[4] + name
            nm = data[start:data.index(b"\0", start)].decode()
            if nm.endswith(".kd") and 0 < shndx < len(secs):
                sec = secs[shndx]
                off = sec[4] + (value - sec[3])
                out[nm] = data[off:off + 64]
    return out


@pytest.fixture(scope="module")
def descriptors(tmp_path_factory):
    if not (os.path.exists(OBJDUMP) and os.path.exists(LIB)):
        pytest.skip("llvm-objdump or libqg_hip.so missing")
    d = tmp_path_factory.mktemp("kd")
    so = shutil.copy(LIB, d / "libqg_hip.so")
    subprocess.run([OBJDUMP, "--offloading", str(so)], cwd=d, capture_output=True, check=True)
    kds = {}
    for f in glob.glob(str(d / "*gfx950*")):
        kds.update(kernel_descriptors(f))
    assert kds, "no gfx950 kernel descriptors in libqg_hip.so"
    return kds


def preload_dwords(kd):
    return struct.unpack_from("<H", kd, 58)[0] & 0x7F


@pytest.mark.parametrize("family", sorted(REQUIRED))
def test_hot_kernels_preload_kernargs(descriptors, family):
    found = {k: preload_dwords(v) for k, v in descriptors.items() if k.startswith(family)}
    assert found, f"no {family} instantiation in the code object"
    short = {k: n for k, n in found.items() if n < REQUIRED[family]}
    assert not short, f"{len(short)} of {len(found)} {family} kernels preload too few dwords: {sorted(short.items())[:3]}"


def test_preload_does_not_exceed_kernarg_segment(descriptors):
    for k, kd in descriptors.items():
        kernarg_bytes = struct.unpack_from("<I", kd, 8)[0]
        assert preload_dwords(kd) * 4 <= max(kernarg_bytes, 0) + 256, k
