#!/bin/bash
# Quick GPU-box check: the GPU parity suite (or a subset: TESTS=...), smoke, one bench line.
# Each GPU step under its own limit; a crash / limit kill stops the chain, test failures do not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -15 $OUT/$name.log
  if fatal $rc; then echo "FATAL: $name rc=$rc, stopping"; exit $rc; fi
  return 0
}
rm -f $OUT/steps.log
run pytest_gpu 1000 python -u -m pytest $TESTS -m gpu -q -rf --timeout 300 --timeout-method thread
[ "${NOSMOKE:-0}" = 1 ] || run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${NOBENCH:-0}" = 1 ] || run bench 400 python bench.py --steps 50 --warmup 10
echo done
