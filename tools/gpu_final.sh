#!/bin/bash
# Round-3 closing GPU call (through gpurun, from the repo root): the GPU suite, smoke() and the bench
# line (tools/gpu_check.sh), the W4A16 two-part-split A/B against the three-part build
# (tools/variants/libqg_np3.so) at the M > 64 shapes, then the round's profiles (tools/profile_round.sh).
set -e
OUT=gpurun_out/s3 bash tools/gpu_check.sh
timeout -k 10 300 python tools/ab_lib.py --w16 --libs llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so tools/variants/libqg_np3.so \
  --shapes 32x4096x4096:2,96x4096x4096:2,128x4096x4096:2,256x4096x4096:2,512x4096x4096:2,128x11008x4096:2,512x4096x4096:8 --rounds 7 > gpurun_out/s3/ab_w16_large.txt 2>&1
cat gpurun_out/s3/ab_w16_large.txt
bash tools/profile_round.sh > gpurun_out/s3/profile_round.log 2>&1
tail -3 gpurun_out/s3/profile_round.log
