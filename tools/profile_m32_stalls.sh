#!/bin/bash
# Where the M = 32 prefill's waves spend their cycles (one MI355X, through gpurun, repo root): one
# PMC pass of 8 SQ counters over tools/gemm_run.py's M = 32 launches, then its summary.
set -e
OUT=gpurun_out/prof_m32_sq
mkdir -p $OUT
export TMPDIR=/tmp
P="python3 tools/gemm_run.py --m 32 --n 4096 --k 4096 --launches 100"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $OUT/sq -o run -- $P > $OUT/sq.log 2>&1
python3 tools/summarize_prof.py $OUT/sq > $OUT/sq.md
rm -rf $OUT/sq
grep mmq $OUT/sq.md
