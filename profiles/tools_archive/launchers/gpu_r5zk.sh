#!/bin/bash
# After the quantizer instruction cut: its rocprof stats at M = 1 / 4 / 32 (K = 4096); the multi-unit GEMV at
# 4096 x 1 x 14336: trace stats and HBM read bytes (FETCH_SIZE pass)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r5zk
mkdir -p $O
for m in 1 4 32; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q$m -o run -- python3 tools/quant_run.py --m $m --k 4096 > $O/q$m.log 2>&1 || exit 1
  f=$(find $O/q$m -name "*kernel_stats.csv" | head -1); cp "$f" $O/quant_m${m}_kernel_stats.csv
done
P="python3 tools/gemm_run.py --m 1 --n 4096 --k 14336 --launches 200"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g -o run -- $P > $O/g.log 2>&1 || exit 2
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/gf -o run -- $P > $O/gf.log 2>&1 || exit 3
python3 tools/summarize_prof.py $O/g > $O/gemv_k14336_trace.md
python3 tools/summarize_prof.py $O/gf > $O/gemv_k14336_fetch.md
for d in q1 q4 q32 g gf; do rm -rf $O/$d; done
for m in 1 4 32; do grep quantize $O/quant_m${m}_kernel_stats.csv | cut -c1-200; done
head -8 $O/gemv_k14336_trace.md; head -8 $O/gemv_k14336_fetch.md
