# round 5: large-M kernel ablations (temporary variant builds: 1 no compute / 2 no DMA / 3 no barrier / 4 no epilogue)
set -o pipefail
mkdir -p gpurun_out
V=tools/variants
timeout -k 10 300 python -u tools/ab_tiled.py --rounds 5 --shapes 512x4096x4096:2 --libs $V/libqg_abl1.so $V/libqg_abl2.so $V/libqg_abl3.so $V/libqg_abl4.so > gpurun_out/r5g_ab_abl.txt 2>&1; rc=$?
cat gpurun_out/r5g_ab_abl.txt
exit $rc
