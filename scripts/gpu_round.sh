#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace. Every GPU step has its
# own time limit; a crash/timeout (exit >= 124 or signal) stops the script, plain test failures
# (pytest exit 1) do not stop the measurement steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${TAG:-r01}
STEPS=${STEPS:-all}

fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if fatal $rc; then echo "FATAL: $name rc=$rc, stopping"; exit $rc; fi
  return 0
}

rocm-smi --showproductname > $OUT/gpu_info.log 2>&1 || true
if [[ "$STEPS" == all || "$STEPS" == *tests* ]]; then
  run pytest_gpu 900 python -m pytest tests -m gpu -q -rf
fi
if [[ "$STEPS" == all || "$STEPS" == *smoke* ]]; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ "$STEPS" == all || "$STEPS" == *bench* ]]; then
  run bench 600 python bench.py --steps 50 --warmup 10
fi
if [[ "$STEPS" == all || "$STEPS" == *prof* ]]; then
  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
fi
if [[ "$STEPS" == all || "$STEPS" == *pmc* ]]; then
  # PMC counters in their own passes (kernel trace only beside them), FETCH_SIZE and WRITE_SIZE
  # separately (MI355X_MICROARCH.md: they cannot share a TCC pass)
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
fi
echo done
