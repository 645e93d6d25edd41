# round 5: tiled decode GEMV with the row GEMV's records and dot8 — parity, then the M = 1 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled.py tests/test_gpu_tiled_act.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5v_tests.txt 2>&1 || { tail -40 gpurun_out/r5v_tests.txt; exit 1; }
tail -2 gpurun_out/r5v_tests.txt
timeout -k 10 300 python -u tools/ab_tiled.py --rounds 5 --shapes 1x4096x4096:2,1x4096x4096:3,1x4096x4096:6,1x4096x4096:7,1x4096x4096:8,1x4096x14336:2,1x32000x4096:2 > gpurun_out/r5v_ab.txt 2>&1 || exit 2
grep "M=" gpurun_out/r5v_ab.txt | cut -c1-150
