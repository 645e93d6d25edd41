#!/bin/bash
# Round-3 A/B (tuning record): W4A16 two-part split (libqg_np2.so) and the software-pipelined M <= 32
# prefill (libqg_pipe{2,3,4}.so; libqg_base2.so = the refactored product stage), against the in-tree
# product library; then the W4A16 GPU tests on the two-part library. Every GPU step has its own limit.
# Kept as the record of that call: the variant libraries were built by hand (Makefile EXTRA flags,
# -DQG_MMQ_PIPE / -DQG_MMQ_C2D from a since-reverted kernel revision) and are not kept.
set -e
O=gpurun_out/np2
mkdir -p $O
V=tools/variants
P=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
timeout -k 10 300 python tools/ab_lib.py --w16 --libs $P $V/libqg_pipe2.so --shapes 16x4096x4096:2,32x4096x4096:2,64x4096x4096:2,32x11008x4096:2,32x4096x14336:2,32x4096x4096:8,32x4096x1024:2 --rounds 9 > $O/ab_w16.txt 2>&1
cat $O/ab_w16.txt
timeout -k 10 400 python tools/ab_lib.py --libs $P $V/libqg_pipe2.so $V/libqg_pc2d.so --shapes 32x4096x4096:2,24x4096x4096:2,16x4096x4096:2,32x4096x4096:3,32x4096x4096:6,32x4096x4096:8,32x11008x4096:2,32x4096x14336:2 --rounds 9 > $O/ab_pipe.txt 2>&1
cat $O/ab_pipe.txt
cp $V/libqg_pipe2.so $P
timeout -k 10 300 python -u -m pytest tests/test_gpu_w4a16.py tests/test_gpu_fuzz.py tests/test_registration.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
tail -3 $O/tests.txt
