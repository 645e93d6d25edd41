#!/bin/bash
# Full GPU suite + smoke after the quantizer arithmetic change (lanes and block quantizers, fused prologues).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5zb
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r5zb/suite.txt 2>&1 || { tail -40 gpurun_out/r5zb/suite.txt; exit 1; }
tail -3 gpurun_out/r5zb/suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5zb/smoke.txt 2>&1 || { cat gpurun_out/r5zb/smoke.txt; exit 2; }
tail -1 gpurun_out/r5zb/smoke.txt
