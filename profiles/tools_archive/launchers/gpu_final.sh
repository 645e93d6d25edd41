#!/bin/bash
# Round-3 closing GPU call (through gpurun, from the repo root): the GPU suite, smoke() and the bench
# line (profiles/tools_archive/launchers/gpu_check.sh), the W4A16 prefill decomposition probe (tools/w16s_probe, built in-tree
# by hipcc), then the round's profiles (profiles/tools_archive/launchers/profile_round.sh). Each GPU step has its own limit.
set -e
OUT=gpurun_out/s4 bash profiles/tools_archive/launchers/gpu_check.sh
if [ -x tools/w16s_probe ]; then
  timeout -k 10 300 ./tools/w16s_probe > gpurun_out/s4/w16s_probe.txt 2>&1
  cat gpurun_out/s4/w16s_probe.txt
fi
bash profiles/tools_archive/launchers/profile_round.sh > gpurun_out/s4/profile_round.log 2>&1
tail -3 gpurun_out/s4/profile_round.log
