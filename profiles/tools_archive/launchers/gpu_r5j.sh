# round 5: large-M kernel A/B — round-4 dispatch (nol), 3 stage buffers (n3), 64 x 64 tiles only (f64)
set -o pipefail
mkdir -p gpurun_out
V=tools/variants
timeout -k 10 400 python -u tools/ab_tiled.py --rounds 5 --shapes 512x4096x4096:2,1024x4096x4096:2 --libs $V/libqg_nol.so $V/libqg_b_sc.so $V/libqg_b_f64.so $V/libqg_b_scf64.so $V/libqg_b_stscf64.so > gpurun_out/r5j_ab.txt 2>&1; rc=$?
cat gpurun_out/r5j_ab.txt
exit $rc
