# round 5: grouped GEMV — does the kernel-argument segment's placement matter? (the descriptor table travels
# in the kernel arguments; HIP_FORCE_DEV_KERNARG=1 asks HIP to put kernel arguments in device memory)
set -o pipefail
mkdir -p gpurun_out
L=llama.cpp-quant-gemm_amd/quant_gemm/libqg_hip.so
timeout -k 10 200 python -u tools/ab_lib.py --grouped --shapes 1x4096x4096:2 --libs $L > gpurun_out/r5t_default.txt 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python -u tools/ab_lib.py --grouped --shapes 1x4096x4096:2 --libs $L > gpurun_out/r5t_devkernarg.txt 2>&1 || exit 2
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 200 python -u tools/ab_lib.py --grouped --shapes 1x4096x4096:2 --libs $L > gpurun_out/r5t_hostkernarg.txt 2>&1 || exit 3
timeout -k 10 200 python -u tools/ab_lib.py --shapes 1x4096x4096:2 --batched --libs $L > gpurun_out/r5t_batched.txt 2>&1 || true
for f in default devkernarg hostkernarg batched; do echo "== $f"; grep -A2 "M=1" gpurun_out/r5t_$f.txt; done
