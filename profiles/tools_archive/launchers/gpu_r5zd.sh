#!/bin/bash
# Loop-free multi-unit GEMV (ONEU = 2 / 4) for K > 4096 decode: GEMV parity tests, then A/B against the unit
# loop (libqg_nu0.so: QG_GEMV_NU=0) on the reference's published K = 14336 shapes and K = 8192 / 11008.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
V=tools/variants
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_product.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_small_k.py tests/test_00_gpu_baseline.py > gpurun_out/r5zd_tests.txt 2>&1 || { tail -30 gpurun_out/r5zd_tests.txt; exit 1; }
tail -2 gpurun_out/r5zd_tests.txt
timeout -k 10 400 python -u tools/ab_lib.py --libs $V/libqg_nu0.so $L --shapes 1x4096x14336:2,2x4096x14336:2,3x4096x14336:2,4x4096x14336:2,2x8192x14336:2,1x4096x8192:2,1x4096x11008:2,1x4096x14336:8,1x4096x14336:3,4x4096x14336:8 --rounds 7 > gpurun_out/r5zd_ab.txt 2>&1 || exit 2
grep -v amdgpu.ids gpurun_out/r5zd_ab.txt
