#!/bin/bash
# Round-4 GPU call: the whole GPU suite + smoke on the product, its bench line, then the bench with the
# grouped launch at 4 row tiles per workgroup (tools/variants/libqg_gtpw4.so over the box's library).
set -e
OUT=gpurun_out/r4e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/suite.txt 2>&1
tail -2 $OUT/suite.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
tail -1 $OUT/smoke.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('gtpw2',d['roofline']['us_per_launch'],d['batched']['us_per_gemv'],d['grouped']['us_per_gemv'])"
cp tools/variants/libqg_gtpw4.so llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs > $OUT/bench_gtpw4.json 2> $OUT/bench_gtpw4.err
python -c "import json;d=json.load(open('$OUT/bench_gtpw4.json'));print('gtpw4',d['roofline']['us_per_launch'],d['batched']['us_per_gemv'],d['grouped']['us_per_gemv'])"
timeout -k 10 200 python -u -m pytest tests/test_gpu_grouped.py -x -q --timeout 120 --timeout-method thread > $OUT/grouped_gtpw4.txt 2>&1
tail -1 $OUT/grouped_gtpw4.txt
