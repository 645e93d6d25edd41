// valu_rate_probe.hip — issue rate of the integer-dot / fp32 VALU instructions the GEMV uses
// (diagnostic, not the product). One workgroup per CU, W waves, each running a long chain of
// independent instructions (8 accumulators) of one kind; reports cycles per wave-instruction per
// SIMD from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o valu_rate_probe valu_rate_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int ITERS = 4096;

template <int KIND>
__global__ __launch_bounds__(1024) void rate(unsigned* out, unsigned long long* cyc, unsigned seed) {
    unsigned a[8], b = seed * 2654435761u + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = b * (i + 3);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0) a[i] = __builtin_amdgcn_udot8(a[i], b, a[i], false);
            if constexpr (KIND == 1) a[i] = (unsigned)__builtin_amdgcn_sdot8((int)a[i], (int)b, (int)a[i], false);
            if constexpr (KIND == 2) a[i] = (unsigned)__builtin_amdgcn_sdot4((int)a[i], (int)b, (int)a[i], false);
            if constexpr (KIND == 3) a[i] = __float_as_uint(__builtin_fmaf(__uint_as_float(a[i]), 1.0001f, 0.5f));
            if constexpr (KIND == 4) a[i] = (a[i] ^ b) + 0x9e3779b9u;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    unsigned* out; unsigned long long* cyc;
    CK(hipMalloc(&out, 256 * 1024 * 4)); CK(hipMalloc(&cyc, 8));
    const char* names[] = {"v_dot8_u32_u4", "v_dot8(c)_i32_i4", "v_dot4(c)_i32_i8", "v_fma_f32", "v_xor + v_add (2 ops)"};
    for (int waves : {4, 8, 16}) {
        for (int k = 0; k < 5; ++k) {
            for (int rep = 0; rep < 2; ++rep) {
                const dim3 g(256), blk(64 * waves);
                if (k == 0) hipLaunchKernelGGL(rate<0>, g, blk, 0, 0, out, cyc, 7u);
                if (k == 1) hipLaunchKernelGGL(rate<1>, g, blk, 0, 0, out, cyc, 7u);
                if (k == 2) hipLaunchKernelGGL(rate<2>, g, blk, 0, 0, out, cyc, 7u);
                if (k == 3) hipLaunchKernelGGL(rate<3>, g, blk, 0, 0, out, cyc, 7u);
                if (k == 4) hipLaunchKernelGGL(rate<4>, g, blk, 0, 0, out, cyc, 7u);
                CK(hipDeviceSynchronize());
            }
            unsigned long long c;
            CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            // s_memtime counts at the shader clock; instructions per SIMD = waves/4 * ITERS * 8
            const double per_simd = (double)waves / 4 * ITERS * 8 * (k == 4 ? 2 : 1);
            printf("%2d waves/CU  %-24s %6.2f cycles per wave-instruction per SIMD\n", waves, names[k], (double)c / per_simd);
        }
    }
    return 0;
}
