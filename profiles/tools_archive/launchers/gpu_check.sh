#!/bin/bash
# One GPU call (through gpurun, from the repo root): the GPU test suite, smoke(), the default bench
# line, then optional A/B libraries (tools/ab_lib.py) given as arguments. Each GPU step has its own
# time limit; the chain stops at the first failure.
set -e
OUT=${OUT:-gpurun_out/check}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/suite.txt 2>&1
tail -2 $OUT/suite.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
cat $OUT/smoke.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
if [ $# -gt 0 ]; then
  timeout -k 10 300 python tools/ab_lib.py --libs llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so "$@" \
    --shapes ${AB_SHAPES:-1x4096x4096:2,1x4000x4096:2,1x4096x4096:3,2x4096x4096:2,32x4096x4096:2} --rounds 9 > $OUT/ab.txt 2>&1
  cat $OUT/ab.txt
fi
