#!/bin/bash
# Matrix-pipe utilisation of the dense prefill shapes on one MI355X (through gpurun, repo root):
# W4A8 (v_mfma_i32_16x16x32_i8 + f16 scale MFMAs) and W4A16 (v_mfma_f32_16x16x32_bf16) at M = 512
# and M = 128, N = K = 4096: kernel trace, then SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES /
# GRBM_GUI_ACTIVE in a pass of their own. Each GPU step has its own limit.
set -e
OUT=gpurun_out/prof_mfma
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "w4a8_m512:--m 512" "w4a8_m128:--m 128" "w4a16_m512:--m 512 --w16" "w4a16_m128:--m 128 --w16"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  P="python3 tools/gemm_run.py $args --n 4096 --k 4096 --launches 100"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${tag}_trace -o run -- $P > $OUT/${tag}_trace.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/${tag}_mfma -o run -- $P > $OUT/${tag}_mfma.log 2>&1
  python3 tools/summarize_prof.py $OUT/${tag}_trace > $OUT/${tag}_trace.md
  python3 tools/summarize_prof.py $OUT/${tag}_mfma > $OUT/${tag}_mfma.md
  rm -rf $OUT/${tag}_trace $OUT/${tag}_mfma
done
ls $OUT
