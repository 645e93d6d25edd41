#!/bin/bash
# round 5 closing call 2/2: the default bench line, then rocprofv3 traces of the same bench command
# (plain and dispatch-serialised) with their stats tables; summaries by tools/summarize_prof.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
OUT=gpurun_out/r5zf
mkdir -p $OUT
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-400
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $OUT/trace_ser -o run -- $B > $OUT/trace_ser.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 3
python3 tools/summarize_prof.py $OUT/trace_ser > $OUT/bench_trace_serialized.md
python3 tools/summarize_prof.py $OUT/trace > $OUT/bench_trace.md
for d in trace trace_ser; do
  f=$(find $OUT/$d -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" $OUT/${d}_kernel_stats.csv
  rm -rf $OUT/$d
done
echo done
