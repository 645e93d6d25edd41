#!/bin/bash
# M = 2..4 decode at K = 14336 (published 4096 x {2,4} x 14336): the multi-unit form for the M tiles and
# 512-thread workgroups, A/B against the product (unit loop, 1024 threads for Q4_0)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
V=tools/variants
timeout -k 10 400 python -u tools/ab_lib.py --libs $L $V/libqg_w512.so $V/libqg_nu2w512.so $V/libqg_nu4w512.so --shapes 2x4096x14336:2,3x4096x14336:2,4x4096x14336:2,2x8192x14336:2,2x4096x4096:2,4x4096x4096:2,2x4096x8192:2 --rounds 7 > gpurun_out/r5zg_ab.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5zg_ab.txt
