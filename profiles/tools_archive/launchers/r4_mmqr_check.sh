#!/bin/bash
# Round-4 GPU call: DMA probe (linear variants), grouped GEMV tests + bench (item-per-XCD order),
# A/B of the tile-resident prefill (tools/variants/libqg_mmqr.so, -DQG_MMQR=1) against the product,
# then the variant's parity on the MFMA tests (the variant copied over the box's in-tree library).
set -e
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 150 ./tools/dma_probe2 > $OUT/dma_probe2.txt 2>&1
cat $OUT/dma_probe2.txt
timeout -k 10 300 python tools/ab_lib.py --libs llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so tools/variants/libqg_mmqr.so \
  --shapes 32x4096x4096:2,16x4096x4096:2,24x4096x4096:2,32x4096x4096:3,32x11008x4096:2,32x4096x2048:2,12x8192x4096:2 --rounds 7 > $OUT/ab_mmqr.txt 2>&1
cat $OUT/ab_mmqr.txt
timeout -k 10 200 python -u -m pytest tests/test_gpu_grouped.py -x -q --timeout 120 --timeout-method thread > $OUT/grouped.txt 2>&1
tail -2 $OUT/grouped.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['roofline']['us_per_launch'],d['batched'],d['grouped'])"
cp tools/variants/libqg_mmqr.so llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
timeout -k 10 400 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_boundary.py -x -q --timeout 120 --timeout-method thread > $OUT/mmqr_parity.txt 2>&1
tail -3 $OUT/mmqr_parity.txt
