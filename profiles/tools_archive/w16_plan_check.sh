#!/bin/bash
# Round-3 A/B (tuning record): the W4A16 prefill's ring depth (W16S_R=3) and split-K plan
# (W16S_MINWG=256: fewer, longer K slices; W16S_MINST=2: more slices for small grids) after the
# two-part split, against the product library.
set -e
O=gpurun_out/w16plan
mkdir -p $O
V=tools/variants
timeout -k 10 400 python tools/ab_lib.py --w16 --libs llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so $V/libqg_w16r3.so $V/libqg_w16wg256.so $V/libqg_w16st2.so \
  --shapes 16x4096x4096:2,32x4096x4096:2,64x4096x4096:2,32x11008x4096:2,32x4096x14336:2,16x2048x4096:2 --rounds 9 > $O/ab.txt 2>&1
cat $O/ab.txt
# the product's W4A16 tests with the 32-token-tile rule in
timeout -k 10 300 python -u -m pytest tests/test_gpu_w4a16.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
tail -2 $O/tests.txt
