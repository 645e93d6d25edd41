set -o pipefail
mkdir -p gpurun_out
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
V=tools/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiled.py tests/test_00_gpu_baseline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d_suite.txt 2>&1 || { tail -30 gpurun_out/r5d_suite.txt; exit 1; }
tail -2 gpurun_out/r5d_suite.txt
timeout -k 10 300 python -u tools/ab_tiled.py --rounds 7 --shapes 32x4096x4096:2,24x4096x4096:2,32x4096x4096:3,32x4096x4096:8,32x2048x8192:2 --libs $V/libqg_s8w8.so $V/libqg_s8w16.so $V/libqg_s8w12.so > gpurun_out/r5d_ab_tiled.txt 2>&1 || exit 1
cat gpurun_out/r5d_ab_tiled.txt
