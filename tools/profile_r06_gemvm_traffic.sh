#!/bin/bash
# HBM traffic of the MFMA small-batch decode (qg_gemvm.hip) at the published 4096 x 4 x 14336 shape on the
# tiled layout: kernel trace, then separate FETCH_SIZE / WRITE_SIZE passes (rocprofv3; gpurun, repo root).
set -eo pipefail
OUT=gpurun_out/r6w
mkdir -p $OUT
export TMPDIR=/tmp
P="python3 tools/gemm_run.py --m 4 --n 4096 --k 14336 --tiled --launches 200"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $P > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- $P > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- $P > $OUT/write.log 2>&1
for d in trace fetch write; do python3 tools/summarize_prof.py $OUT/$d > $OUT/$d.md; rm -rf "${OUT:?}/$d"; done
