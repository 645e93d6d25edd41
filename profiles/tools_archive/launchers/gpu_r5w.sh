# round 5: wave / slot counts of the 32 x 16 tile on tiled activations (variant libraries copied over the
# in-tree one in this scratch copy only; separate processes, same box)
set -o pipefail
mkdir -p gpurun_out
S=32x4096x4096,16x4096x4096,32x4096x4128
timeout -k 10 300 python -u tools/ab_tiled_act.py --rounds 3 --shapes $S > gpurun_out/r5w_base.txt 2>&1 || exit 1
cp tools/variants/libqg_w12nb2.so llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
timeout -k 10 300 python -u tools/ab_tiled_act.py --rounds 3 --shapes $S > gpurun_out/r5w_w12nb2.txt 2>&1 || exit 2
cp tools/variants/libqg_w16nb2.so llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
timeout -k 10 300 python -u tools/ab_tiled_act.py --rounds 3 --shapes $S > gpurun_out/r5w_w16nb2.txt 2>&1 || exit 3
for f in base w12nb2 w16nb2; do echo "== $f"; grep q4_0 gpurun_out/r5w_$f.txt; done
