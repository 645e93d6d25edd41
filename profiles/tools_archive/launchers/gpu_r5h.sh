# round 5: SQ counter passes on the large-M kernel (M=512 tiled), one pass per counter set
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5h
P="python3 tools/gemm_run.py --m 512 --n 4096 --k 4096 --launches 30 --tiled"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/r5h/a -o run -- $P > gpurun_out/r5h/a.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL --kernel-trace --output-format csv -d gpurun_out/r5h/b -o run -- $P > gpurun_out/r5h/b.log 2>&1 || exit 2
python3 tools/pmc_dump.py gpurun_out/r5h --kernel mmql > gpurun_out/r5h/summary.txt
cat gpurun_out/r5h/summary.txt
