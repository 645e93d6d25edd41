#!/bin/bash
# Round-3 full GPU check: the whole -m gpu suite, smoke, one bench line. Each GPU step under its own
# limit; a crash / limit kill stops the chain.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_suite.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03_gpu_suite.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r03_smoke.log
if fatal $rc; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/r03_bench5.json 2> gpurun_out/r03_bench5.err
echo "bench rc=$?"
