#!/bin/bash
# GEMV output stores: nontemporal (libqg_nts.so) vs plain (product), single launches, bench protocol, ABAB rounds
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
V=tools/variants
timeout -k 10 300 python -u tools/ab_lib.py --libs $L $V/libqg_nts.so --shapes 1x4096x4096:2,1x4000x4096:2,2x4096x4096:2,1x4096x4096:3,1x4096x14336:2 --rounds 9 > gpurun_out/r5zi_ab.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5zi_ab.txt
