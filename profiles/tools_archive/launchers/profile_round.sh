#!/bin/bash
# Round-end measurement on one MI355X (run through gpurun from the repo root):
#   bench line, rocprofv3 kernel trace + stats of the same bench command, separate PMC passes
#   (FETCH_SIZE, WRITE_SIZE, MFMA busy) for the headline GEMV and the M=32 prefill, summaries.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -e
OUT=gpurun_out/prof_round
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1
# the same trace with dispatches serialised by one harmless counter (the plain trace pass slows each
# dispatch of a 3.3 us kernel)
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $OUT/trace_ser -o run -- $B > $OUT/trace_ser.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1
P="python3 tools/gemm_run.py --m 32 --n 4096 --k 4096 --launches 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/m32_trace -o run -- $P > $OUT/m32_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/m32_fetch -o run -- $P > $OUT/m32_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/m32_mfma -o run -- $P > $OUT/m32_mfma.log 2>&1
python3 tools/summarize_prof.py $OUT/trace > $OUT/bench_trace.md
python3 tools/summarize_prof.py $OUT/trace_ser > $OUT/bench_trace_serialized.md
python3 tools/summarize_prof.py $OUT/pmc_fetch --pmc-json $OUT/pmc_fetch.json > $OUT/pmc_fetch.md
python3 tools/summarize_prof.py $OUT/pmc_write > $OUT/pmc_write.md
python3 tools/summarize_prof.py $OUT/m32_trace > $OUT/m32_trace.md
python3 tools/summarize_prof.py $OUT/m32_fetch --key q4_0_m32_n4096_k4096 --pmc-json $OUT/m32_fetch.json > $OUT/m32_fetch.md
python3 tools/summarize_prof.py $OUT/m32_mfma > $OUT/m32_mfma.md

# keep the summaries and the rocprof stats tables; drop the raw traces (gpurun copies back <= 64 MiB)
for d in trace trace_ser pmc_fetch pmc_write m32_trace m32_fetch m32_mfma; do
  f=$(find $OUT/$d -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" $OUT/${d}_kernel_stats.csv
  rm -rf $OUT/$d
done
cat $OUT/bench.json
