"""The C-ABI drop-in boundary (include/qg/qg.h) — CPU-only checks, no kernel launches.

* libqg_hip.so loads and exports every function include/qg/qg.h declares (and the Python mirror
  binds exactly those);
* argument validation returns the documented status codes before anything is enqueued
  (the reference's wrappers validate nothing, include/gemm_cuda_naive.cuh:285-292; its Python face
  raises via TORCH_CHECK, python/quant_gemm/csrc/bindings.cpp:19-70);
* the Python mirror's error messages match the reference's TORCH_CHECK texts.
"""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "qg", "qg.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(qg_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    import quant_gemm._lib as L
    return L


def test_header_declares_expected_surface():
    fns = declared_functions()
    for must in ("qg_gemm_w4a8", "qg_gemm_q4_0_q8_1", "qg_quantize_q8_1", "qg_quantize_q4_0",
                 "qg_dequantize_q4_0", "qg_gemm_w4a8_from_view", "qg_debug_sumi"):
        assert must in fns


def test_library_exports_every_declared_symbol(lib):
    so = lib.load()
    fns = declared_functions()
    for f in fns:
        assert hasattr(so, f), f
    nm = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (qg_\w+)", nm))
    assert set(fns) <= exported
    assert set(lib.SIGNATURES) == set(fns), "Python bindings out of sync with qg.h"


def test_library_is_gfx950_code_object(lib, tmp_path):
    # llvm-objdump --offloading extracts every bundle next to its input: run it on a copy
    import shutil
    so = shutil.copy(lib.LIB_PATH, tmp_path / "libqg_hip.so")
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(so)],
                         capture_output=True, text=True, cwd=tmp_path)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout


def test_static_queries(lib):
    so = lib.load()
    assert so.qg_version().decode().startswith("qg-mi355x")
    assert [so.qg_block_bytes(t) for t in (2, 3, 6, 7, 8, 9, 0)] == [18, 20, 22, 24, 34, 36, 0]
    assert so.qg_select_algo(1, 4096, 4096, 2) == 1      # decode -> GEMV
    assert so.qg_select_algo(4, 4096, 4096, 6) == 1      # small batch -> GEMV
    assert so.qg_select_algo(8, 4096, 4096, 6) == 2      # M >= 5 -> MFMA
    assert so.qg_select_algo(32, 4096, 4096, 2) == 2     # prefill -> MFMA
    assert so.qg_select_algo(1, 4096, 4128, 2) == 4      # K/32 odd -> one wave per weight row (ragged)
    assert so.qg_select_algo(16, 64, 4128, 7) == 4
    assert so.qg_select_algo(1, 4096, 33, 2) == -1
    assert so.qg_status_string(-2).decode().startswith("K must be")
    # W4A16 prefill split-K workspace (host-side plan): 512 workgroups of 64 rows x 32 tokens x
    # K/8 at M=32, N=K=4096 -> the fixed 4 KB tile-counter region + 64 tiles x 8 slices x 8 KB of
    # partials (the counter region does not move with the shape: ADVICE r01)
    assert so.qg_gemm_w16_workspace_size(32, 4096, 4096) == 4096 + 64 * 8 * 4 * 2 * 4 * 64 * 4
    assert so.qg_gemm_w16_workspace_size(4, 4096, 4096) == 0      # GEMV: no workspace
    assert so.qg_gemm_w16_workspace_size(512, 4096, 4096) == 0    # enough token tiles: no split


def test_validation_codes_without_launch(lib):
    so = lib.load()
    P = ctypes.c_void_p
    fake = P(4096)  # never dereferenced: validation fails first
    assert so.qg_gemm_w4a8(fake, fake, fake, 1, 1, 33, 2, None) == -2        # bad K
    assert so.qg_gemm_w4a8(fake, fake, fake, 1, 1, 0, 2, None) == -2
    assert so.qg_gemm_w4a8(fake, fake, fake, -1, 1, 32, 2, None) == -1       # negative M
    assert so.qg_gemm_w4a8(fake, fake, fake, 1, 1, 32, 9, None) == -3        # Q8_1 weights: not a weight format
    assert so.qg_gemm_w4a8(None, fake, fake, 1, 1, 32, 2, None) == -1        # null
    assert so.qg_gemm_w4a8(None, None, None, 0, 5, 64, 2, None) == 0         # empty: no-op
    assert so.qg_gemm_w4a8(fake, P(4097), fake, 1, 1, 32, 2, None) == -4     # odd weight pointer
    assert so.qg_gemm_w4a8_ex(fake, fake, fake, 1, 1, 288, 2, 1, None) == -3  # GEMV needs K % 256 == 0
    assert so.qg_quantize(2, 0, fake, fake, 33, None) == -2
    assert so.qg_quantize(2, 1, fake, fake, 32, None) == -3                  # variant 1 is Q8_1 only
    assert so.qg_quantize(9, 0, P(4098), fake, 32, None) == -4               # float input misaligned
    assert so.qg_quantize(9, 0, fake, P(4098), 32, None) == -4               # Q8_1 blocks need 4-B alignment
    assert so.qg_quantize(9, 0, None, None, 0, None) == 0
    assert so.qg_dequantize(5, fake, fake, 32, None) == -3
    # W4A16 / W8A16
    assert so.qg_gemm_w4a16(fake, fake, fake, 1, 1, 48, None) == -2
    assert so.qg_gemm_w4a16(P(4098), fake, fake, 1, 1, 64, None) == -4           # floats misaligned
    assert so.qg_gemm_w8a16(fake, P(4097), fake, 1, 1, 64, None) == -4
    assert so.qg_gemm_q4_0_fp32(fake, None, fake, 1, 1, 64, None) == -1
    assert so.qg_gemm_w4a16(None, None, None, 0, 3, 64, None) == 0
    # fused activation quantization
    assert so.qg_gemm_w4a8_f32_workspace_size(3, 4096) == 3 * 128 * 36
    assert so.qg_gemm_w4a8_f32_workspace_size(0, 4096) == 0
    assert so.qg_gemm_w4a8_f32(fake, fake, fake, 1, 1, 33, 2, None, 0, None) == -2
    assert so.qg_gemm_w4a8_f32(fake, fake, fake, 1, 1, 32, 9, None, 0, None) == -3
    assert so.qg_gemm_w4a8_f32(P(4100), fake, fake, 1, 8, 4096, 2, None, 0, None) == -4  # no 16-B X, no workspace
    assert so.qg_gemm_w4a8_f32(P(4098), fake, fake, 1, 8, 4096, 2, None, 0, None) == -4  # floats misaligned
    assert so.qg_gemm_w4a8_f32(None, None, None, 0, 8, 4096, 2, None, 0, None) == 0
    assert so.qg_gemm_q4_0_fp16_fused(fake, fake, fake, 8, 1, 48, None) == -2
    assert so.qg_gemm_q4_0_fp16_fused(fake, P(4097), fake, 8, 1, 64, None) == -4          # odd half pointer
    assert so.qg_quantize_q8_1_f16_fused(fake, fake, 31, None) == -2
    assert so.qg_quantize_q8_1_f16_fused(fake, P(4098), 32, None) == -4


def test_from_view_validation(lib):
    so = lib.load()

    class View(ctypes.Structure):
        _fields_ = [("data", ctypes.c_void_p), ("type", ctypes.c_int), ("ne", ctypes.c_int64 * 4),
                    ("nb", ctypes.c_size_t * 4)]

    def view(t, ne0, ne1, bb):
        v = View()
        v.data, v.type = 4096, t
        v.ne[:] = [ne0, ne1, 1, 1]
        row = (ne0 // 32) * bb if t != 0 else ne0 * 4
        v.nb[:] = [bb if t != 0 else 4, row, row * ne1, row * ne1]
        return v

    act, w = view(9, 4096, 1, 36), view(2, 4096, 8, 18)
    out = View()
    out.data, out.type = 4096, 0
    out.ne[:] = [8, 1, 1, 1]
    out.nb[:] = [4, 32, 32, 32]
    p = ctypes.byref
    assert so.qg_gemm_w4a8_from_view(p(act), p(w), p(out), b"bogus", None) == -1
    bad = View()
    ctypes.pointer(bad)[0] = out
    bad.type = 2
    assert so.qg_gemm_w4a8_from_view(p(act), p(w), p(bad), b"naive", None) == -3  # output must be F32
    assert so.qg_gemm_w4a8_from_view(p(act), p(act), p(out), b"naive", None) == -3  # Q8_1 weights
    w2 = view(2, 2048, 8, 18)
    assert so.qg_gemm_w4a8_from_view(p(act), p(w2), p(out), None, None) == -1     # K mismatch


def test_python_mirror_errors_match_reference():
    import torch
    import quant_gemm as q
    with pytest.raises(RuntimeError, match="Input must be a CUDA tensor"):
        q.quantize_q4_0(torch.zeros(4, 64))
    with pytest.raises(RuntimeError, match="Weight must be a CUDA tensor"):
        q.gemm_q4_0_q8_1(torch.zeros(4, 2, 18, dtype=torch.uint8), torch.zeros(1, 2, 36, dtype=torch.uint8), 4, 1, 64)
    with pytest.raises(RuntimeError, match="K must be divisible by 32"):
        q.gemm_q4_0_q8_1(torch.zeros(1, dtype=torch.uint8), torch.zeros(1, dtype=torch.uint8), 4, 1, 65)


# The sumi parity hook must run the product's own kernel instantiation: the
# configuration query names the kernel qg_gemm_w4a8_ex and qg_debug_sumi would launch.
PRODUCT_SHAPES = [(1, 4096, 4096), (2, 4096, 4096), (3, 4096, 4096), (4, 4096, 4096), (8, 4096, 4096),
                  (32, 4096, 4096), (1, 4000, 4096), (1, 32000, 4096), (5, 4096, 4096), (128, 4096, 4096),
                  (512, 4096, 4096), (1, 4096, 14336), (3, 11008, 4096), (1, 4096, 4128), (32, 4096, 4128)]


@pytest.mark.parametrize("m,n,k", PRODUCT_SHAPES)
@pytest.mark.parametrize("t", [2, 3, 6, 7, 8])
def test_sumi_hook_runs_product_kernel(lib, m, n, k, t):
    import quant_gemm as qg
    prod = qg.debug_config(m, n, k, t)
    assert prod and prod == qg.debug_config(m, n, k, t, sumi=True)
    fam = {1: "gemv", 2: "mmq", 3: "generic", 4: "ragged"}[qg.select_algo(m, n, k, t)]
    # the MFMA family: the small-tile kernel, or the large-M one (qg_mmql_kernel.hpp) when its grid fills
    # the CUs
    assert prod.startswith(fam + " ") or (fam == "mmq" and prod.startswith("mmql ")), prod


def test_headline_configs_kernels(lib):
    """The kernels serving BASELINE configs[1..4] (what DESIGN.md §3 documents)."""
    import quant_gemm as qg
    assert qg.debug_config(1, 4096, 4096, 2).startswith("gemv F=2 MT=1 BPL=2 LPR=64 WGS=1024")
    assert "ONEU=1" in qg.debug_config(1, 4096, 4096, 2)
    # the published 4096 x 1 x 14336 decode shape: Q4_0 M = 1 loop-free with 4 units per lane (round 5);
    # M = 2 and the other formats keep the unit loop (ONEU=0)
    assert "MT=1 " in qg.debug_config(1, 4096, 14336, 2) and "ONEU=4 SIG=m1" in qg.debug_config(1, 4096, 14336, 2)
    assert "ONEU=2 SIG=m1" in qg.debug_config(1, 4096, 8192, 2)
    assert "ONEU=0" in qg.debug_config(2, 4096, 14336, 2) and "ONEU=0" in qg.debug_config(1, 4096, 14336, 3)
    assert qg.debug_config(1, 4096, 14336, 2) == qg.debug_config(1, 4096, 14336, 2, sumi=True)
    assert qg.debug_config(32, 4096, 4096, 2).startswith("mmq F=2 ")
    assert "BN=32 TT=1 W=12 P16=1 NB=1 LAY=0 AW=0" in qg.debug_config(32, 4096, 4096, 2)
    # the tiled layout of the same config: same tile, same waves
    assert "BN=32 TT=1 W=12 P16=1 NB=1 LAY=1 AW=0" in qg.debug_config_tiled(32, 4096, 4096, 2)
    # the step-4 prefill (M = 512): the large-M kernel's 64 x 64 tiles (round 5), both layouts
    assert qg.debug_config(512, 4096, 4096, 2).startswith("mmql F=2 BN=64 BM=64 W=4 NBUF=4 LAY=0 grid=512")
    assert qg.debug_config_tiled(512, 4096, 4096, 2).startswith("mmql F=2 BN=64 BM=64 W=4 NBUF=4 LAY=1 grid=512")
    assert qg.debug_config(256, 4096, 4096, 2).startswith("mmq F=2 ")  # 512 tiles of 64 x 64 needed
    for t in (3, 6, 7):
        assert qg.debug_config(1, 4096, 4096, t).startswith(f"gemv F={t} MT=1 ")
    assert qg.debug_config(1, 4000, 4096, 2).startswith("gemv F=2 MT=1 ")


def test_tiled_decode_routing():
    """The tiled entry's decode routing (round 6; CPU: the configuration query launches nothing):
    M = 1..2 the tiled decode GEMV up to K/32 = 256, M = 3..4 (and M = 2 beyond K/32 = 256) the MFMA small-batch
    decode with 2 / 4 token columns and 4 (K/32 <= 256) or 8 stages per lane, M >= 5 the MFMA prefill kernels;
    the sumi hook names the same instantiation."""
    import quant_gemm as qg
    cases = [((1, 4096, 4096), "gemvt F=2 MT=1 "), ((2, 4096, 4096), "gemvt F=2 MT=2 "),
             ((2, 4096, 8192), "gemvt F=2 MT=2 "), ((2, 4096, 8224), "gemvm F=2 NU=8 MP=2 "),
             ((2, 4096, 14336), "gemvm F=2 NU=8 MP=2 W=14 "), ((3, 4096, 4096), "gemvm F=2 NU=4 MP=4 W=8 "),
             ((4, 4096, 14336), "gemvm F=2 NU=8 MP=4 W=14 "), ((4, 64, 160), "gemvm F=2 NU=4 MP=4 W=1 "),
             ((5, 4096, 14336), "mmq F=2 "), ((8, 4096, 4096), "mmq F=2 ")]
    for (m, n, k), fam in cases:
        cfg = qg.debug_config_tiled(m, n, k, 2)
        assert cfg.startswith(fam), (m, n, k, cfg)
        assert cfg == qg.debug_config_tiled(m, n, k, 2, sumi=True)
        if fam.startswith("gem"):  # the tiled-activation entry: the same kernel, activations from the tiled layout
            cfg_ta = qg.debug_config_tiled_act(m, n, k, 2)
            assert cfg_ta.startswith(fam) and " TA=1 " in cfg_ta, cfg_ta
    # every format takes the small-batch decode; K beyond 16 waves (K > 16384) goes to the MFMA prefill kernel
    for t in (3, 6, 7, 8):
        assert qg.debug_config_tiled(4, 4096, 14336, t).startswith(f"gemvm F={t} NU=8 MP=4 ")
    assert qg.debug_config_tiled(4, 4096, 16416, 2).startswith("mmq ")


def test_ldc_entry_validates(lib):
    so = lib.load()
    P = ctypes.c_void_p
    # ldc below N is an invalid argument, reported before anything is enqueued
    assert so.qg_gemm_w4a8_ldc(P(256), P(256), P(256), 2, 64, 256, 32, 2, 0, None) == -1
    assert so.qg_gemm_w4a8_ldc(P(256), P(256), P(256), 2, 64, 100, 64, 2, 0, None) == -2


def test_layout_buffers_checked_before_launch():
    """the tiled / packed layout buffers the Python face hands to the C-ABI as raw pointers are
    checked for dtype, contiguity, device and exact size first (CPU tensors: refused before any launch)."""
    import pytest
    import torch
    import quant_gemm as qg
    a = torch.zeros(2 * 4 * 36, dtype=torch.uint8)
    w = torch.zeros(64, dtype=torch.uint8)
    for fn, args in [(qg.gemm_w4a8_tiled, (a, w, 2, 32, 128)), (qg.debug_sumi_tiled, (a, w, 2, 32, 128)),
                     (qg.gemm_w4a8_tiled_act, (w, w, 2, 32, 128)), (qg.debug_sumi_tiled_act, (w, w, 2, 32, 128)),
                     (qg.gemm_w4a8_prepacked, (a, w, 2, 32, 128))]:
        with pytest.raises(RuntimeError):
            fn(*args)
    # a float tensor of the right byte count / a strided view: refused by the layout check itself
    with pytest.raises(RuntimeError, match="uint8"):
        qg._check_layout(torch.zeros(16, dtype=torch.float32), "weight_tiled", 16, torch.device("cpu"))
    with pytest.raises(RuntimeError, match="contiguous"):
        qg._check_layout(torch.zeros(32, dtype=torch.uint8)[::2], "weight_tiled", 16, torch.device("cpu"))
