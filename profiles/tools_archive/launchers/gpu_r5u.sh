# round 5: tiled decode GEMV ablations (temporary variants: 1 no cross-wave reduction, 2 no block compute)
set -o pipefail
mkdir -p gpurun_out
V=tools/variants
timeout -k 10 300 python -u tools/ab_tiled.py --rounds 5 --shapes 1x4096x4096:2 --libs $V/libqg_gt1.so $V/libqg_gt2.so > gpurun_out/r5u_ab.txt 2>&1 || exit 1
grep "M=" gpurun_out/r5u_ab.txt | cut -c1-300
