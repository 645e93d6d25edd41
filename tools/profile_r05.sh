#!/bin/bash
# Round-5 measurement on one MI355X (through gpurun, repo root): the bench line, rocprofv3 traces and
# separate PMC passes (FETCH_SIZE, WRITE_SIZE, matrix-pipe busy) of the headline GEMV, the M = 32 prefill on
# the reference rows and on the tiled layout, and the M = 128 / 512 prefill (rows and tiled); summaries and
# the per-config PMC record profiles read by bench.py (gpurun_out/prof_r05/r05_pmc.json). Every GPU step
# has its own time limit; the chain stops at the first failure.
set -e
OUT=gpurun_out/prof_r05
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $OUT/trace_ser -o run -- $B > $OUT/trace_ser.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1
python3 tools/summarize_prof.py $OUT/trace_ser > $OUT/bench_trace_serialized.md
python3 tools/summarize_prof.py $OUT/pmc_fetch --key q4_0_m1_n4096_k4096 --pmc-json $OUT/pmc_fetch.json > $OUT/pmc_fetch.md
python3 tools/summarize_prof.py $OUT/pmc_write --key q4_0_m1_n4096_k4096 --pmc-json $OUT/pmc_write.json > $OUT/pmc_write.md
for cfg in "m32:--m 32" "m32_tiled:--m 32 --tiled" "m128:--m 128" "m128_tiled:--m 128 --tiled" "m512:--m 512" "m512_tiled:--m 512 --tiled"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  P="python3 tools/gemm_run.py $args --n 4096 --k 4096 --launches 200"
  key=q4_0_${tag%%_tiled}_n4096_k4096; case $tag in *_tiled) key=${key}_tiled;; esac
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $OUT/${tag}_trace -o run -- $P > $OUT/${tag}_trace.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/${tag}_fetch -o run -- $P > $OUT/${tag}_fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/${tag}_mfma -o run -- $P > $OUT/${tag}_mfma.log 2>&1
  python3 tools/summarize_prof.py $OUT/${tag}_trace > $OUT/${tag}_trace.md
  python3 tools/summarize_prof.py $OUT/${tag}_fetch --key $key --pmc-json $OUT/${tag}_fetch.json > $OUT/${tag}_fetch.md
  python3 tools/summarize_prof.py $OUT/${tag}_mfma --key $key --pmc-json $OUT/${tag}_mfma.json > $OUT/${tag}_mfma.md
done
# one record per config key (bench.py load_pmc / load_traffic)
python3 - <<'PY'
import glob, json, os
out = {}
for f in sorted(glob.glob("gpurun_out/prof_r05/*.json")):
    if f.endswith("bench.json"):
        continue
    for k, v in json.load(open(f)).items():
        if "|" not in k:
            out.setdefault(k, {}).update(v)
h = out.get("q4_0_m1_n4096_k4096", {})
if "hbm_read_bytes_per_launch" in h and "hbm_write_bytes_per_launch" in h:
    h["hbm_bytes_per_launch"] = h["hbm_read_bytes_per_launch"] + h["hbm_write_bytes_per_launch"]
json.dump(out, open("gpurun_out/prof_r05/r05_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
for d in $OUT/*/; do
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" ${d%/}_kernel_stats.csv
  rm -rf $d
done
cat $OUT/bench.json
