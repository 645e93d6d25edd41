#!/bin/bash
# Quantizer launch floor: the M = 1 quantizer beside an empty kernel of the same grid, one rocprofv3 trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5x
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5x -o run -- python3 tools/quant_floor_run.py > gpurun_out/r5x/log.txt 2>&1 || exit 1
find gpurun_out/r5x -name '*kernel_stats.csv' -exec cp {} gpurun_out/r5x_kernel_stats.csv \;
cut -c1-160 gpurun_out/r5x_kernel_stats.csv
