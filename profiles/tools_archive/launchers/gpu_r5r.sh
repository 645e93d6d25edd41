# round 5: GPU suite, smoke, default bench line (one call; each step under its own limit)
set -o pipefail
mkdir -p gpurun_out/r5r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5r/suite.txt 2>&1 || { tail -30 gpurun_out/r5r/suite.txt; exit 1; }
tail -2 gpurun_out/r5r/suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5r/smoke.txt 2>&1 || { cat gpurun_out/r5r/smoke.txt; exit 2; }
tail -1 gpurun_out/r5r/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r5r/bench.json 2> gpurun_out/r5r/bench.err || { tail -20 gpurun_out/r5r/bench.err; exit 3; }
tail -1 gpurun_out/r5r/bench.json | cut -c1-600
