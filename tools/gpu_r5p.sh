# round 5: tiled activations — parity (new + tiled + mmql tests), then the A/B against row activations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled_act.py tests/test_gpu_tiled.py tests/test_gpu_mmql.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p_tests.txt 2>&1 || { tail -40 gpurun_out/r5p_tests.txt; exit 1; }
tail -2 gpurun_out/r5p_tests.txt
timeout -k 10 500 python -u tools/ab_tiled_act.py --rounds 3 > gpurun_out/r5p_ab.txt 2>&1 || { tail -20 gpurun_out/r5p_ab.txt; exit 2; }
cat gpurun_out/r5p_ab.txt
