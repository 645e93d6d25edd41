set -eo pipefail
OUT=gpurun_out/r6t
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "m4:--m 4" "m2:--m 2" "m1:--m 1"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  P="python3 tools/gemm_run.py $args --n 4096 --k 14336 --tiled --launches 100"
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $OUT/${tag}_sq -o run -- $P > $OUT/${tag}_sq.log 2>&1
  python3 tools/summarize_prof.py $OUT/${tag}_sq > $OUT/${tag}_sq.md
  rm -rf $OUT/${tag}_sq
done
