# round 5: L2 hit / HBM fetch of the large-M kernel, full and DMA-only (variant build copied over the in-tree
# library in this scratch copy only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5i; mkdir -p $O
P="python3 tools/gemm_run.py --m 512 --n 4096 --k 4096 --launches 30 --tiled"
for v in full abl1; do
  if [ $v = abl1 ]; then cp tools/variants/libqg_abl1.so llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so; fi
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/${v}_hit -o run -- $P > $O/${v}_hit.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${v}_fetch -o run -- $P > $O/${v}_fetch.log 2>&1 || exit 2
  timeout -k 10 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/${v}_tcp -o run -- $P > $O/${v}_tcp.log 2>&1 || exit 3
  python3 tools/pmc_dump.py $O --kernel mmql | grep -v "^$" > $O/summary_$v.txt
  rm -rf $O/${v}_hit $O/${v}_fetch $O/${v}_tcp.keep
done
cat $O/summary_full.txt; echo ---; cat $O/summary_abl1.txt
