# round 5: block-pipelined large-M variants (pipe: 4 buffers; pipe3: 3 buffers, 3 workgroups per CU) and the
# quantizer's rocprof duration at M = 1 / 4 / 32, K = 4096
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5o
V=tools/variants
timeout -k 10 400 python -u tools/ab_tiled.py --rounds 5 --shapes 512x4096x4096:2,1024x4096x4096:2,512x4096x4096:8 --libs $V/libqg_pipe.so $V/libqg_pipe3.so > gpurun_out/r5o/ab.txt 2>&1 || exit 1
cat gpurun_out/r5o/ab.txt
for m in 1 4 32; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5o/q$m -o run -- python3 tools/quant_run.py --m $m --k 4096 --launches 400 > gpurun_out/r5o/q$m.log 2>&1 || exit 2
  f=$(find gpurun_out/r5o/q$m -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r5o/quant_m${m}_kernel_stats.csv; rm -rf gpurun_out/r5o/q$m
  grep quantize gpurun_out/r5o/quant_m${m}_kernel_stats.csv
done
