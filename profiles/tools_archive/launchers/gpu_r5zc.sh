#!/bin/bash
# Persistent grouped GEMV: parity tests, then A/B against the per-tile grid (libqg_np.so: QG_GEMVG_PERSIST=0)
# and the strided batch as the target.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
V=tools/variants
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grouped.py tests/test_gpu_small_k.py > gpurun_out/r5zc_tests.txt 2>&1 || { tail -30 gpurun_out/r5zc_tests.txt; exit 1; }
tail -2 gpurun_out/r5zc_tests.txt
timeout -k 10 300 python -u tools/ab_lib.py --libs $V/libqg_np.so $L --grouped --shapes 1x4096x4096:2,2x4096x4096:2,4x4096x4096:2,1x4096x4096:8,1x11008x4096:2,1x1024x4096:2 --rounds 7 > gpurun_out/r5zc_ab_grouped.txt 2>&1 || exit 2
timeout -k 10 200 python -u tools/ab_lib.py --libs $L --batched --shapes 1x4096x4096:2,1x4096x4096:8 --rounds 5 > gpurun_out/r5zc_batched.txt 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/r5zc_ab_grouped.txt; grep -v amdgpu.ids gpurun_out/r5zc_batched.txt
