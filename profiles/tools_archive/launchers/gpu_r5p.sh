# round 5: tiled activations and the tiled decode on the row GEMV's kernel — parity (new + tiled + mmql
# tests), the M = 1 rows-vs-tiled A/B, the tiled-activation A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled_act.py tests/test_gpu_tiled.py tests/test_gpu_mmql.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p_tests.txt 2>&1 || { tail -40 gpurun_out/r5p_tests.txt; exit 1; }
tail -2 gpurun_out/r5p_tests.txt
timeout -k 10 300 python -u tools/ab_tiled.py --rounds 5 --shapes 1x4096x4096:2,1x4096x4096:3,1x4096x4096:6,1x4096x4096:8,1x4096x14336:2,1x32000x4096:2 > gpurun_out/r5p_ab_m1.txt 2>&1 || { tail -20 gpurun_out/r5p_ab_m1.txt; exit 2; }
grep "M=" gpurun_out/r5p_ab_m1.txt | cut -c1-200
