"""bench.py's N>1 legs rehearsed on one GPU: two ranks over gloo sharing the
device (QG_BENCH_BACKEND=gloo), a short run — the weak headline leg, the strong-scaling N=32000
legs (per-launch and grouped) with their 1-GPU denominators, and the single-launch floor at N=1.
Numbers from a gloo rehearsal are meaningless (gloo stages CUDA tensors through the host, two
ranks share one GPU); this checks the code paths and the line's fields, not the speed."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _last_json(out):
    for line in reversed(out.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError(out[-2000:])


def test_bench_world2_gloo_rehearsal():
    env = dict(os.environ, QG_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--gemvs-per-step", "8", "--no-floor"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["rows_per_gpu"] == 4000
    st = d["strong"]
    assert st["per_launch"]["us_per_gemv"] > 0 and st["batched"]["us_per_gemv"] > 0
    sp = st["strong_speedup_vs_1gpu_n32000"]
    assert sp["per_launch"] > 0 and sp["batched"] > 0
    assert "skipped" in st["native"]  # two gloo ranks share the one GPU: the RCCL leg is not run
    assert st["one_gpu_n32000"]["single_us_per_launch"] > 0
    assert d["gather"]["us_per_step"] > 0


def test_bench_world1_floor_and_sides():
    cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    rf = d["roofline"]
    assert 0 < rf["floor"]["empty_us"] < rf["floor_us"] and 0 < rf["floor_frac"] < 1
    assert d["grouped"]["us_per_gemv"] > 0
    forms = {(s["N"], s["form"]) for s in d["side_configs"]}
    assert (32000, "single") in forms and (32000, "batched") in forms and (4096, "single") in forms
