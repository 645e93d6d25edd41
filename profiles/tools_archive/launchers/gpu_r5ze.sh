#!/bin/bash
# round 5 closing call 1/2: the GPU suite and smoke() on the final tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5ze
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r5ze/suite.txt 2>&1 || { tail -40 gpurun_out/r5ze/suite.txt; exit 1; }
tail -2 gpurun_out/r5ze/suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5ze/smoke.txt 2>&1 || { cat gpurun_out/r5ze/smoke.txt; exit 2; }
tail -1 gpurun_out/r5ze/smoke.txt
