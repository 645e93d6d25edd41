#!/bin/bash
# Quantizer rewrite (ordered sum as a DPP add chain, 3-instruction roundf, 32-bit indices): the GPU tests
# that cover its bytes, then its rocprofv3 trace beside the empty kernel of the same grid.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5z
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_product.py tests/test_gpu_repack.py tests/test_gpu_tiled_act.py tests/test_00_gpu_baseline.py > gpurun_out/r5z/tests.txt 2>&1 || { tail -30 gpurun_out/r5z/tests.txt; exit 1; }
tail -3 gpurun_out/r5z/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5z -o run -- python3 tools/quant_floor_run.py > gpurun_out/r5z/log.txt 2>&1 || exit 2
cut -c1-120 gpurun_out/r5z/run_kernel_stats.csv
