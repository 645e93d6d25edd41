// qg_generic.hip — shape/alignment-agnostic W4A8 kernel (any K % 32 == 0, any pointer alignment).
//
// Used where the fast paths' preconditions (K % 256 == 0, 16-B aligned weights, LDS budget) do not
// hold, and as the independent cross-check of the fast kernels in the GPU parity tests. One wave
// per output element; lanes stride over Q-blocks and fetch bytes individually, so it has no
// alignment requirement. Block terms and the reduction tree follow the same rules as the fast
// kernels (qg_common.hpp).
#include "qg_common.hpp"
#include "qg_kernels.hpp"

namespace qg {

template <int F>
__device__ __forceinline__ void decode_bytes(const uint8_t* blk, uint32_t (&q)[8], float& d, float& m) {
    using T = wfmt<F>;
    d = h2f((uint32_t)blk[0] | ((uint32_t)blk[1] << 8));
    m = 0.0f;
    if constexpr (T::MOFF >= 0) m = h2f((uint32_t)blk[T::MOFF] | ((uint32_t)blk[T::MOFF + 1] << 8));
    if constexpr (T::Q8) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            q[i] = (uint32_t)blk[T::QS + 4 * i] | ((uint32_t)blk[T::QS + 4 * i + 1] << 8) |
                   ((uint32_t)blk[T::QS + 4 * i + 2] << 16) | ((uint32_t)blk[T::QS + 4 * i + 3] << 24);
        return;
    }
    uint32_t qh = 0;
    if constexpr (T::QH >= 0)
        qh = (uint32_t)blk[T::QH] | ((uint32_t)blk[T::QH + 1] << 8) | ((uint32_t)blk[T::QH + 2] << 16) |
             ((uint32_t)blk[T::QH + 3] << 24);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 4 * i + j;
            uint32_t x = blk[T::QS + e];
            uint32_t l = x & 0xF, h = x >> 4;
            if constexpr (T::QH >= 0) {
                l |= ((qh >> e) & 1u) << 4;
                h |= ((qh >> (e + 16)) & 1u) << 4;
            }
            lo |= l << (8 * j);
            hi |= h << (8 * j);
        }
        q[i] = lo;
        q[4 + i] = hi;
    }
}

template <int F, bool SUMI>
__global__ __launch_bounds__(256) void generic_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                      float* __restrict__ C, int32_t* __restrict__ sumi_out, int M,
                                                      int N, int K, long ldc_m, long ldc_n) {
    using T = wfmt<F>;
    const int nb = K / QK;
    const int lane = threadIdx.x & 63;
    const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int m = blockIdx.y;
    if (n >= N) return;  // wave-uniform
    float acc = 0.0f;
    for (int b = lane; b < nb; b += 64) {
        const uint8_t* wb = B + ((long)n * nb + b) * T::BB;
        const uint8_t* ab = A + ((long)m * nb + b) * Q8_1_BYTES;
        uint32_t q[8];
        float dw, mw;
        decode_bytes<F>(wb, q, dw, mw);
        uint32_t a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            a[i] = (uint32_t)ab[4 + 4 * i] | ((uint32_t)ab[5 + 4 * i] << 8) | ((uint32_t)ab[6 + 4 * i] << 16) |
                   ((uint32_t)ab[7 + 4 * i] << 24);
        const float da = h2f((uint32_t)ab[0] | ((uint32_t)ab[1] << 8));
        const float sa = h2f((uint32_t)ab[2] | ((uint32_t)ab[3] << 8));
        const int sumi = dot_block(q, a);
        if constexpr (SUMI) sumi_out[((long)m * N + n) * nb + b] = sumi;
        else acc += block_term<F>(sumi, dw, mw, da, sa);
    }
    if constexpr (!SUMI) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
        if (lane == 0) C[m * ldc_m + n * ldc_n] = acc;
    }
}

namespace {
template <int F> hipError_t launch_g(const GemmArgs& g, hipStream_t st) {
    dim3 grid((g.N + 3) / 4, g.M);
    if (g.describe) {
        describe_kernel(g, "generic F=%d grid=%ux%u", F, grid.x, grid.y);
        return hipSuccess;
    }
    if (g.sumi)
        hipLaunchKernelGGL((generic_kernel<F, true>), grid, dim3(256), 0, st, (const uint8_t*)g.A,
                           (const uint8_t*)g.B, g.C, g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    else
        hipLaunchKernelGGL((generic_kernel<F, false>), grid, dim3(256), 0, st, (const uint8_t*)g.A,
                           (const uint8_t*)g.B, g.C, g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_generic(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return launch_g<FMT_Q4_0>(g, st);
        case FMT_Q4_1: return launch_g<FMT_Q4_1>(g, st);
        case FMT_Q5_0: return launch_g<FMT_Q5_0>(g, st);
        case FMT_Q5_1: return launch_g<FMT_Q5_1>(g, st);
        case FMT_Q8_0: return launch_g<FMT_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
