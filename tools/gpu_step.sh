#!/bin/bash
# The one GPU launcher (run through gpurun from the repo root): `bash tools/gpu_step.sh TAG STEP...`,
# each STEP under its own time limit, outputs in gpurun_out/TAG/, the chain stopping at the first failure
# (no retries). Steps:
#   suite          pytest -m gpu (the whole GPU suite)
#   tests:F1,F2    pytest of the named test files (tests/F1.py ...)
#   smoke          __graft_entry__.smoke()
#   bench          the default bench line (bench.json)
#   trace          rocprofv3 kernel trace + stats of a short bench run, dispatch-serialised (one harmless
#                  counter) and plain, summarised by tools/summarize_prof.py
#   pmc            separate FETCH_SIZE / WRITE_SIZE passes of the same bench command (per-launch HBM bytes)
#   ab:SHAPES      tools/ab_lib.py rows vs in-tree library (SHAPES = MxNxK:wtype,...)
#   tiled:SHAPES   tools/ab_tiled.py rows vs tiled layout
#   tiled_act:SHAPES  tools/ab_tiled_act.py tiled vs tiled activations
# (The round-1..5 one-off launchers this replaces are kept under profiles/tools_archive/launchers/.)
set -eo pipefail
TAG=${1:?usage: gpu_step.sh TAG STEP...}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs"
for step in "$@"; do
  echo "== $step"
  case $step in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/suite.txt" 2>&1
      tail -3 "$OUT/suite.txt" ;;
    tests:*)
      files=""; for f in $(echo "${step#tests:}" | tr ',' ' '); do files="$files tests/$f.py"; done
      timeout -k 10 900 python -u -m pytest $files -x -q --timeout 120 --timeout-method thread > "$OUT/tests.txt" 2>&1
      tail -3 "$OUT/tests.txt" ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
      cat "$OUT/smoke.txt" ;;
    bench)
      timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      tail -1 "$OUT/bench.json" | cut -c1-600 ;;
    trace)
      timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d "$OUT/trace_ser" -o run -- $B > "$OUT/trace_ser.log" 2>&1
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B > "$OUT/trace.log" 2>&1
      python3 tools/summarize_prof.py "$OUT/trace_ser" > "$OUT/bench_trace_serialized.md"
      python3 tools/summarize_prof.py "$OUT/trace" > "$OUT/bench_trace.md"
      for d in trace trace_ser; do
        f=$(find "$OUT/$d" -name "*kernel_stats.csv" | head -1)
        [ -n "$f" ] && cp "$f" "$OUT/${d}_kernel_stats.csv"
        rm -rf "${OUT:?}/$d"
      done
      head -30 "$OUT/bench_trace_serialized.md" ;;
    pmc)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- $B > "$OUT/pmc_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- $B > "$OUT/pmc_write.log" 2>&1
      python3 tools/summarize_prof.py "$OUT/pmc_fetch" --key q4_0_m1_n4096_k4096 --pmc-json "$OUT/pmc_fetch.json" > "$OUT/pmc_fetch.md"
      python3 tools/summarize_prof.py "$OUT/pmc_write" --key q4_0_m1_n4096_k4096 --pmc-json "$OUT/pmc_write.json" > "$OUT/pmc_write.md"
      rm -rf "${OUT:?}/pmc_fetch" "${OUT:?}/pmc_write"
      cat "$OUT/pmc_fetch.json" "$OUT/pmc_write.json" ;;
    ab:*)
      timeout -k 10 600 python -u tools/ab_lib.py --shapes "${step#ab:}" --rounds 7 > "$OUT/ab.txt" 2>&1
      cut -c1-300 "$OUT/ab.txt" ;;
    tiled:*)
      timeout -k 10 600 python -u tools/ab_tiled.py --shapes "${step#tiled:}" --rounds 5 > "$OUT/tiled.txt" 2>&1
      cut -c1-300 "$OUT/tiled.txt" ;;
    tiled_act:*)
      timeout -k 10 600 python -u tools/ab_tiled_act.py --shapes "${step#tiled_act:}" --rounds 5 > "$OUT/tiled_act.txt" 2>&1
      cut -c1-300 "$OUT/tiled_act.txt" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
