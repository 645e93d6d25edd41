set -o pipefail
mkdir -p gpurun_out
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
V=tools/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiled.py tests/test_gpu_grouped.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c_suite.txt 2>&1 || { tail -30 gpurun_out/r5c_suite.txt; exit 1; }
tail -2 gpurun_out/r5c_suite.txt
timeout -k 10 300 python -u tools/ab_tiled.py --rounds 5 --shapes 1x4096x4096:2,2x4096x4096:2,4x4096x4096:2,32x4096x4096:2,32x4096x4096:8 --libs $V/libqg_dmaonly.so $V/libqg_computeonly.so > gpurun_out/r5c_ab_tiled.txt 2>&1 || exit 1
cat gpurun_out/r5c_ab_tiled.txt
timeout -k 10 200 python -u tools/ab_lib.py --libs $V/libqg_r04.so $L $V/libqg_g4.so --grouped --shapes 1x4096x4096:2,2x4096x4096:2 --rounds 7 > gpurun_out/r5c_ab_grouped.txt 2>&1 || exit 1
cat gpurun_out/r5c_ab_grouped.txt
