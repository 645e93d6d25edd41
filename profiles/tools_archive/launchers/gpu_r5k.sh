# round 5: large-M kernel (64 x 64 tiles, scalar epilogue) — ablations (DMA only / compute only), 3 stage
# buffers at 3 workgroups per CU, and the SQ counters of the default build
set -o pipefail
mkdir -p gpurun_out
V=tools/variants
timeout -k 10 400 python -u tools/ab_tiled.py --rounds 5 --shapes 512x4096x4096:2,256x4096x4096:2,1024x4096x4096:2 --libs $V/libqg_nol.so $V/libqg_c_abl1.so $V/libqg_c_abl2.so $V/libqg_c_n3.so > gpurun_out/r5k_ab.txt 2>&1 || exit 1
cat gpurun_out/r5k_ab.txt
bash profiles/tools_archive/launchers/gpu_r5h.sh
