set -o pipefail
mkdir -p gpurun_out
V=tools/variants
timeout -k 10 300 python -u tools/ab_tiled.py --rounds 7 --shapes 32x4096x4096:2,24x4096x4096:2,32x4096x4096:3,32x4096x4096:8,32x4096x4096:6,20x4096x2048:2 --libs $V/libqg_ra12.so $V/libqg_ra12b.so $V/libqg_ra8.so $V/libqg_ra16.so > gpurun_out/r5e_ab_tiled.txt 2>&1; rc=$?
cat gpurun_out/r5e_ab_tiled.txt
exit $rc
