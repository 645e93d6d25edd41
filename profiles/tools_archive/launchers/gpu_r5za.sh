#!/bin/bash
# Quantizer A/B in one box: the round-5 lanes quantizer before (libqg_qold.so) and after the instruction cut,
# ABAB, each a rocprofv3 trace of 400 launches beside 400 empty kernels of the same grid.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
cp $L gpurun_out/libqg_new.so || exit 8
mkdir -p gpurun_out/r5za
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp tools/variants/libqg_qold.so $L; else cp gpurun_out/libqg_new.so $L; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5za/${v}$r -o run -- python3 tools/quant_floor_run.py > gpurun_out/r5za/${v}$r.log 2>&1 || exit 1
  done
done
cp gpurun_out/libqg_new.so $L && rm gpurun_out/libqg_new.so
echo done
