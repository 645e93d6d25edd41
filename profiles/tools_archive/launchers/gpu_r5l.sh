# round 5: large-M kernel (cleaned) — parity, then A/B against the round-4 dispatch
set -o pipefail
mkdir -p gpurun_out
V=tools/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_mmql.py tests/test_gpu_tiled.py tests/test_isa_hazards.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5l_tests.txt 2>&1 || { tail -30 gpurun_out/r5l_tests.txt; exit 1; }
tail -3 gpurun_out/r5l_tests.txt
timeout -k 10 400 python -u tools/ab_tiled.py --rounds 5 --shapes 512x4096x4096:2,256x4096x4096:2,1024x4096x4096:2,512x4096x4096:8,512x4096x4096:3,512x14336x4096:2,512x4096x14336:2,384x4096x4096:2 --libs $V/libqg_nol.so --rows-libs $V/libqg_nol.so > gpurun_out/r5l_ab.txt 2>&1 || exit 2
cat gpurun_out/r5l_ab.txt
