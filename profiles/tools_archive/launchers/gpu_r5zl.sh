#!/bin/bash
# Decode at K = 14336, M = 1 / 2 / 4 (published shapes): SQ counters of the GEMV (one --pmc pass of 8 SQ
# counters per shape) for the round-6 staging design
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r5zl
mkdir -p $O
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
for m in 1 2 4; do
  P="python3 tools/gemm_run.py --m $m --n 4096 --k 14336 --launches 100"
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/m$m -o run -- $P > $O/m$m.log 2>&1 || exit 1
  python3 tools/summarize_prof.py $O/m$m > $O/sq_m$m.md
  rm -rf $O/m$m
done
for m in 1 2 4; do grep gemv $O/sq_m$m.md | cut -c1-200; done
