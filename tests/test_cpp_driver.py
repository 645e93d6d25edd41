"""Build and run the C++ host-side driver (tests/cpp/test_capi.cpp) over the C-ABI on the GPU."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "llama.cpp-quant-gemm_amd", "quant_gemm")
ORACLE = os.path.join(REPO, "oracle", "_build")


def build(tmp_path):
    exe = str(tmp_path / "test_capi")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17",
                    "-I", os.path.join(REPO, "include"), os.path.join(REPO, "tests", "cpp", "test_capi.cpp"),
                    "-L", LIBDIR, "-lqg_hip", "-L", ORACLE, "-lqg_oracle",
                    f"-Wl,-rpath,{LIBDIR}", f"-Wl,-rpath,{ORACLE}", "-o", exe], check=True)
    return exe


def test_cpp_driver_compiles(tmp_path):
    """The C++ mirror header + C-ABI link cleanly (CPU-only check)."""
    assert os.path.exists(build(tmp_path))


@pytest.mark.gpu
def test_cpp_driver_runs(tmp_path):
    exe = build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


def build_shard(tmp_path):
    exe = str(tmp_path / "test_shard")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17",
                    "-I", os.path.join(REPO, "include"), os.path.join(REPO, "tests", "cpp", "test_shard.cpp"),
                    "-L", LIBDIR, "-lqg_shard", "-lqg_hip", "-lrccl", "-pthread",
                    f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib", "-o", exe], check=True)
    return exe


def test_cpp_shard_driver_compiles(tmp_path):
    """The native multi-GPU caller (one RCCL communicator per device, libqg_shard.so) links cleanly."""
    assert os.path.exists(build_shard(tmp_path))


@pytest.mark.gpu
def test_cpp_shard_driver_runs(tmp_path):
    """World = the visible GPUs (1 on the test box): every rank's full C vs single-GPU qg_gemm_w4a8."""
    exe = build_shard(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
