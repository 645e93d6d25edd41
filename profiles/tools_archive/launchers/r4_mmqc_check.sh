#!/bin/bash
# Round-4 GPU call: the chunked cooperative-ingest prefill (qg_mmqc_kernel.hpp) — MFMA parity tests on
# the product library, then A/B against the library without it (tools/variants/libqg_base.so).
set -e
OUT=${OUT:-gpurun_out/r4i}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_boundary.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_product.py tests/test_gpu_wide_prefill.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.txt 2>&1 || { tail -30 $OUT/parity.txt; exit 1; }
tail -2 $OUT/parity.txt
timeout -k 10 400 python tools/ab_lib.py --libs llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so tools/variants/libqg_base.so \
  --shapes ${AB_SHAPES:-32x4096x4096:2,24x4096x4096:2,32x4096x4096:3,32x4096x4096:6,32x4096x4096:7,32x4096x4096:8,32x11008x4096:2,16x8192x4096:2,12x8192x4096:2,32x4096x14336:2,32x4096x2048:2} --rounds 7 > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
