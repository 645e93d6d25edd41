# round 5: large-M prefill kernel (qg_mmql_kernel.hpp) — parity, then A/B against the round-4 dispatch
set -o pipefail
mkdir -p gpurun_out
V=tools/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_mmql.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5f_mmql_tests.txt 2>&1; rc=$?
tail -5 gpurun_out/r5f_mmql_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_tiled.py --rounds 5 --shapes 512x4096x4096:2,256x4096x4096:2,1024x4096x4096:2,512x4096x4096:8,512x4096x4096:3,512x14336x4096:2,512x4096x14336:2 --rows-libs $V/libqg_nol.so > gpurun_out/r5f_ab_mmql.txt 2>&1; rc=$?
cat gpurun_out/r5f_ab_mmql.txt
exit $rc
