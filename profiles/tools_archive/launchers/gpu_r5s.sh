# round 5: rocprof traces + FETCH / WRITE / matrix-pipe passes of the tiled-activation prefill (M = 32, 512)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_r05b; mkdir -p $OUT
for cfg in "m32_tiled_act:--m 32" "m512_tiled_act:--m 512"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  P="python3 tools/gemm_run.py $args --n 4096 --k 4096 --launches 200 --tiled-act"
  key=q4_0_${tag%%_tiled_act}_n4096_k4096_tiled_act
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $OUT/${tag}_trace -o run -- $P > $OUT/${tag}_trace.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/${tag}_fetch -o run -- $P > $OUT/${tag}_fetch.log 2>&1 || exit 2
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/${tag}_write -o run -- $P > $OUT/${tag}_write.log 2>&1 || exit 3
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/${tag}_mfma -o run -- $P > $OUT/${tag}_mfma.log 2>&1 || exit 4
  python3 tools/summarize_prof.py $OUT/${tag}_trace > $OUT/${tag}_trace.md
  for pass in fetch write mfma; do
    python3 tools/summarize_prof.py $OUT/${tag}_$pass --key $key --pmc-json $OUT/${tag}_$pass.json > $OUT/${tag}_$pass.md
  done
  f=$(find $OUT/${tag}_trace -name "*kernel_stats.csv" | head -1); cp $f $OUT/${tag}_kernel_stats.csv
  rm -rf $OUT/${tag}_trace $OUT/${tag}_fetch $OUT/${tag}_write $OUT/${tag}_mfma
done
grep -h "mmq" $OUT/*_kernel_stats.csv | cut -c1-160
cat $OUT/*_fetch.json $OUT/*_mfma.json | head -40
