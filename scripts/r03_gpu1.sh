set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_grouped.py tests/test_registration.py tests/test_gpu_bench.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r03_t1.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/r03_bench1.json 2> gpurun_out/r03_bench1.err
echo "bench rc=$?"
