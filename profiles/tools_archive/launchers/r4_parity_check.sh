#!/bin/bash
# Round-4 GPU call: the MFMA prefill / W4A16 parity tests on the product library, then the bench line.
set -e
OUT=${OUT:-gpurun_out/r4w}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_boundary.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_product.py tests/test_gpu_wide_prefill.py tests/test_gpu_w16d.py tests/test_gpu_w4a16.py tests/test_gpu_repack.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.txt 2>&1 || { tail -30 $OUT/parity.txt; exit 1; }
tail -2 $OUT/parity.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['roofline']['us_per_launch'],d['batched']['us_per_gemv'],d['grouped']['us_per_gemv']);print([(s['wtype'],s['M'],s['N'],s['form'],s.get('us_per_launch',s.get('us_per_gemv'))) for s in d['side_configs']])"
