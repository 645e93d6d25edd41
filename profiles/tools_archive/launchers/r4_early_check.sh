#!/bin/bash
# Round-4 GPU call: MMQ early refill (product) vs without (tools/variants/libqg_noearly.so), A/B over the
# prefill shapes, then the MFMA / parity tests on the product.
set -e
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 400 python tools/ab_lib.py --libs llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so tools/variants/libqg_noearly.so \
  --shapes 32x4096x4096:2,16x4096x4096:2,24x4096x4096:2,32x4096x4096:3,32x4096x4096:8,32x11008x4096:2,12x8192x4096:2,64x4096x4096:2,128x4096x4096:2,512x4096x4096:2,32x4096x14336:2 --rounds 7 > $OUT/ab_early.txt 2>&1
cat $OUT/ab_early.txt
timeout -k 10 400 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_product.py tests/test_gpu_repack.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.txt 2>&1
tail -2 $OUT/parity.txt
