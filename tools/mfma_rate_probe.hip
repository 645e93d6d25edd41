// mfma_rate_probe.hip — back-to-back issue cost of the int8 MFMA shapes on one wave (diagnostic).
//   hipcc --offload-arch=gfx950 -O3 -o mfma_rate_probe mfma_rate_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v8i __attribute__((ext_vector_type(8)));
template <int KIND>
__global__ void k(long a0, long b0, int* out, int iters) {
    long a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
    v4i c4[4] = {}; v16i c16[2] = {};
    v4i A4 = {(int)a, (int)b, (int)(a >> 3), (int)(b >> 5)};
    v8i A8 = {(int)a, (int)b, 1, 2, 3, 4, 5, 6};
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (KIND == 0) c4[j] = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c4[j], 0, 0, 0);
            if constexpr (KIND == 1) c4[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A4, A4, c4[j], 0, 0, 0);
            if constexpr (KIND == 2) c16[j & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A4, A4, c16[j & 1], 0, 0, 0);
            if constexpr (KIND == 3) c16[j & 1] = __builtin_amdgcn_mfma_i32_32x32x16_i8(a, b, c16[j & 1], 0, 0, 0);
        }
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    int s = 0;
    for (int j = 0; j < 4; ++j) s += c4[j][0] + c4[j][3];
    for (int j = 0; j < 2; ++j) s += c16[j][0] + c16[j][15];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) out[64] = (int)((t1 - t0) / (iters * 4));
}
int main() {
    int* d; (void)hipMalloc(&d, 1024);
    const char* nm[4] = {"16x16x32_i8", "16x16x64_i8", "32x32x32_i8", "32x32x16_i8"};
    for (int kind = 0; kind < 4; ++kind) {
        for (int rep = 0; rep < 2; ++rep) {
            if (kind == 0) k<0><<<1, 64>>>(3, 5, d, 1000);
            if (kind == 1) k<1><<<1, 64>>>(3, 5, d, 1000);
            if (kind == 2) k<2><<<1, 64>>>(3, 5, d, 1000);
            if (kind == 3) k<3><<<1, 64>>>(3, 5, d, 1000);
            (void)hipDeviceSynchronize();
        }
        int h[65]; (void)hipMemcpy(h, d, 65 * 4, hipMemcpyDeviceToHost);
        printf("%s: %d cycles per MFMA (one wave, independent accumulators)\n", nm[kind], h[64]);
    }
    return 0;
}
