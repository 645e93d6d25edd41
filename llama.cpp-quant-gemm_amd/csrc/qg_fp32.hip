// qg_fp32.hip — FP32 GEMM C[M,N] = A[M,K] . B[N,K]^T: the unquantized baseline of the reference
// (gemm_fp32_naive, include/gemm_cuda_naive.cuh:258-265; gemm_fp32_reference,
// include/gemm_reference.h:38-58) used to report NMSE against the quantized paths. Not a hot path:
// a plain LDS-tiled VALU kernel, 64 x 64 outputs per 256-thread workgroup, 4 x 4 per thread, K in
// steps of 16 staged transposed ([k][row]) so the inner loop reads float4 rows of both operands.
#include <hip/hip_runtime.h>

#include "qg_kernels.hpp"

namespace qg {

namespace {
constexpr int TB = 64, TK = 16;

__global__ __launch_bounds__(256) void fp32_gemm_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                        float* __restrict__ C, int M, int N, int K, long ldc_m,
                                                        long ldc_n) {
    __shared__ __attribute__((aligned(16))) float As[TK][TB + 4];
    __shared__ __attribute__((aligned(16))) float Bs[TK][TB + 4];
    const int tid = threadIdx.x;
    const int m0 = blockIdx.y * TB, n0 = blockIdx.x * TB;
    const int tm = (tid / 16) * 4, tn = (tid % 16) * 4;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += TK) {
        // 64 rows x 16 k per operand = 1024 floats: 4 per thread
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + i * 256;
            const int r = e / TK, kk = e % TK;
            const int gm = m0 + r, gn = n0 + r, gk = k0 + kk;
            As[kk][r] = (gm < M && gk < K) ? A[(long)gm * K + gk] : 0.0f;
            Bs[kk][r] = (gn < N && gk < K) ? B[(long)gn * K + gk] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < TK; ++kk) {
            const float4 a = *reinterpret_cast<const float4*>(&As[kk][tm]);
            const float4 b = *reinterpret_cast<const float4*>(&Bs[kk][tn]);
            const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(av[i], bv[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int m = m0 + tm + i, n = n0 + tn + j;
            if (m < M && n < N) C[m * ldc_m + n * ldc_n] = acc[i][j];
        }
}
}  // namespace

hipError_t launch_fp32(const GemmArgs& g, hipStream_t st) {
    if ((g.M + TB - 1) / TB > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fp32_gemm_kernel, dim3((g.N + TB - 1) / TB, (g.M + TB - 1) / TB), dim3(256), 0, st,
                       (const float*)g.A, (const float*)g.B, g.C, g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}

}  // namespace qg
