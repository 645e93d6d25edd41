#!/bin/bash
# Round-3 A/B (tuning record): the W4A16 / W8A16 prefill with 32-token tiles (W16S_TT2, each weight
# fragment decoded once for two token tiles) now that the activation planes are two, not three.
set -e
O=gpurun_out/tt2
mkdir -p $O
timeout -k 10 300 python tools/ab_lib.py --w16 --libs llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so tools/variants/libqg_tt2.so \
  --shapes 24x4096x4096:2,32x4096x4096:2,48x4096x4096:2,64x4096x4096:2,32x11008x4096:2,32x4096x14336:2,32x4096x4096:8 --rounds 9 > $O/ab.txt 2>&1
cat $O/ab.txt
# the bench line with its new W4A16 side config
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.load(open('$O/bench.json')); print(json.dumps(d['side_configs'][-1]))"
