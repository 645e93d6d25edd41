# round 5: large-M kernel, zero-seed + v_cvt epilogue (default) vs the biased seed (cvt0); mmql parity
set -o pipefail
mkdir -p gpurun_out
V=tools/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_mmql.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5n_tests.txt 2>&1 || { tail -30 gpurun_out/r5n_tests.txt; exit 1; }
tail -2 gpurun_out/r5n_tests.txt
timeout -k 10 400 python -u tools/ab_tiled.py --rounds 5 --shapes 512x4096x4096:2,1024x4096x4096:2 --libs $V/libqg_nol.so $V/libqg_cvt0.so > gpurun_out/r5n_ab.txt 2>&1 || exit 2
cat gpurun_out/r5n_ab.txt
