set -o pipefail
mkdir -p gpurun_out
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
V=tools/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b_suite.txt 2>&1; rc=$?
tail -4 gpurun_out/r5b_suite.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_tiled.py --rounds 5 --shapes 1x4096x4096:2,4x4096x4096:2,32x4096x4096:2,16x4096x4096:2,8x4096x4096:2,64x4096x4096:2,512x4096x4096:2,32x4096x4128:2,32x4096x4096:8 --libs $V/libqg_t8.so $V/libqg_t16.so $V/libqg_t12b.so --rows-libs $V/libqg_r04.so > gpurun_out/r5b_ab_tiled.txt 2>&1 || exit 1
cat gpurun_out/r5b_ab_tiled.txt
timeout -k 10 200 python -u tools/ab_lib.py --libs $V/libqg_r04.so $L --grouped --shapes 1x4096x4096:2,2x4096x4096:2 --rounds 7 > gpurun_out/r5b_ab_grouped.txt 2>&1 || exit 1
cat gpurun_out/r5b_ab_grouped.txt
timeout -k 10 200 python -u tools/ab_quant.py --libs $V/libqg_r04.so $L > gpurun_out/r5b_ab_quant.txt 2>&1 || exit 1
cat gpurun_out/r5b_ab_quant.txt
timeout -k 10 300 python -u bench.py > gpurun_out/r5b_bench.json 2> gpurun_out/r5b_bench.err; echo bench rc=$?
timeout -k 10 200 python -u tools/ab_lib.py --libs $V/libqg_r04.so $L $V/libqg_co.so --shapes 1x4096x4096:2,1x4000x4096:2 --rounds 9 > gpurun_out/r5b_ab_co.txt 2>&1; cat gpurun_out/r5b_ab_co.txt
