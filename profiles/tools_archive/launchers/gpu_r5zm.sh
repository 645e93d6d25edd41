#!/bin/bash
# M = 2 multi-unit GEMV with / without per-unit record preloading vs the unit loop (product)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
V=tools/variants
timeout -k 10 300 python -u tools/ab_lib.py --libs $L $V/libqg_nu2p.so $V/libqg_nu2np.so --shapes 2x4096x14336:2,2x8192x14336:2,2x4096x8192:2,2x4096x11008:2 --rounds 7 > gpurun_out/r5zm_ab.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5zm_ab.txt
