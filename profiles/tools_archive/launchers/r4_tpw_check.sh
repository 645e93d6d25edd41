#!/bin/bash
# Round-4 GPU call: GEMV tests on the product (2 row tiles per workgroup in the batched / grouped
# launches), the bench line, then the same bench with the 1-tile variant (tools/variants/libqg_tpw1.so)
# copied over the box's in-tree library — batched / grouped per-GEMV times side by side.
set -e
OUT=gpurun_out/r4d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_grouped.py tests/test_gpu_parity.py tests/test_00_gpu_baseline.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
tail -2 $OUT/tests.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_tpw2.json 2> $OUT/bench_tpw2.err
python -c "import json;d=json.load(open('$OUT/bench_tpw2.json'));print('tpw2',d['roofline']['us_per_launch'],d['batched'],d['grouped'],[(s['N'],s['form'],s.get('us_per_gemv',s.get('us_per_launch'))) for s in d['side_configs']])"
cp tools/variants/libqg_tpw1.so llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs > $OUT/bench_tpw1.json 2> $OUT/bench_tpw1.err
python -c "import json;d=json.load(open('$OUT/bench_tpw1.json'));print('tpw1',d['roofline']['us_per_launch'],d['batched'],d['grouped'])"
