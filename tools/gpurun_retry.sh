#!/bin/bash
# Development helper (not run on the GPU box): re-issue a gpurun call while the pool has no free box.
# usage: gpurun_retry.sh LOG TIMEOUT CMD — retries only while gpurun reports no free box (exit 3)
LOG=$1; T=$2; shift 2
for i in $(seq 1 20); do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout $T -- "$@" > $LOG 2>&1
  rc=$?
  echo "[retry] attempt $i rc=$rc" >> $LOG.attempts
  if [ $rc -ne 3 ] && ! grep -q "no free box\|backing off\|stopped responding while being prepared" $LOG; then break; fi
  sleep 120
done
echo "[retry] done rc=$rc" >> $LOG.attempts
