// qg_ragged.hip — the W4A8 product for shapes the GEMV / MFMA kernels cannot take: an odd number
// of Q-blocks per row (K / 32 odd, e.g. K = 4128), which leaves every other weight row 2 bytes off
// dword alignment for the 18 / 22 / 34-byte formats, or weight tensors that are only 2-B aligned.
//
// Same contract as the other families: C[m*ldc_m + n*ldc_n] = sum_b term(A[m][b], B[n][b])
// (include/gemm_reference.h:175-222). Round 1 sent these shapes to the byte-load generic kernel
// (qg_generic.hip: one wave per OUTPUT element, so the weights were re-read M times and fetched a
// byte at a time). Here one wave owns one weight row for up to MT tokens (grid.y = chunks of MT):
//  * the workgroup stages its MT activation rows once into LDS records (the GEMV's record,
//    qg_gemv_kernel.hpp make_act_record: nibble planes for Q4_0 / Q4_1, fp32 d / c*s / -1.5*2^23*d);
//    record stride 20 dwords (4 x odd: the 16 lanes of a ds_read_b128 group hit distinct bank slots);
//  * lane l takes blocks l, l + 64, ...: it loads the dwords covering the block's BB bytes from the
//    dword-aligned address at or below the block — every loaded dword holds at least one byte of
//    the block, so none can cross into a page past the tensor — and realigns them with v_alignbyte
//    by the block's 0- or 2-byte offset;
//  * the block dot and term are the GEMV's (block_dot / block_term_rec: bit-identical per-block
//    terms), partials reduced across the wave with DPP (group_sum_last), lane 63 stores.
#include "qg_gemv_kernel.hpp"

#include <algorithm>

namespace qg {

namespace {
constexpr int RG_RS = 20;   // LDS record stride (dwords)
constexpr int RG_WGS = 1024;  // 16 waves = 16 weight rows per workgroup: the activation staging is paid
                              // once per 16 rows (with 4 rows per workgroup it was 4x the weight bytes)

template <int F, int MT, bool SUMI>
__global__ __launch_bounds__(RG_WGS) void ragged_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, int M,
                                                     int N, int K, float* __restrict__ C, long ldc_m, long ldc_n,
                                                     int32_t* __restrict__ sumi_out) {
    using T = wfmt<F>;
    constexpr int LD = (T::BB + 2 + 3) / 4;  // dwords loaded per block (covers a 2-B offset)
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int nb = K / QK;
    const int m0 = blockIdx.y * MT;
    const int mc = min(MT, M - m0);  // tokens of this chunk
    A += (long)m0 * nb * 9;
    const int tid = threadIdx.x, lane = tid & 63;
    const int row = blockIdx.x * (RG_WGS / 64) + (tid >> 6);
    const bool row_ok = row < N;

    for (int g = tid; g < mc * nb; g += RG_WGS) {
        uint32_t ab[9];
        const uint32_t* p = A + (long)g * 9;
#pragma unroll
        for (int i = 0; i < 9; ++i) ab[i] = p[i];
        make_act_record<F>(ab, lds + g * RG_RS);
    }
    __syncthreads();

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;
    const uint8_t* wrow = B + (long)(row_ok ? row : 0) * nb * T::BB;
    for (int b = lane; b < nb; b += 64) {
        const uintptr_t pb = (uintptr_t)(wrow + (long)b * T::BB);
        const uint32_t* pa = reinterpret_cast<const uint32_t*>(pb & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(pb & 3);  // 0 or 2
        uint32_t d[LD], w[LD];
#pragma unroll
        for (int i = 0; i + 1 < LD; ++i) d[i] = pa[i];
        // the last dword holds block bytes only when the block starts 2 bytes into a dword or its
        // size is not a dword multiple (Q4_1 / Q5_1 at offset 0 end exactly on a dword boundary: that
        // dword may lie wholly past the end of the tensor)
        if constexpr (T::BB % 4 == 0) d[LD - 1] = sh ? pa[LD - 1] : 0u;
        else d[LD - 1] = pa[LD - 1];
#pragma unroll
        for (int i = 0; i + 1 < LD; ++i) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
        w[LD - 1] = d[LD - 1] >> (8 * sh);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            if (m < mc) {
                const uint32_t* rec = lds + (m * nb + b) * RG_RS;
                uint4 a[3];
                a[0] = *reinterpret_cast<const uint4*>(rec);
                a[1] = *reinterpret_cast<const uint4*>(rec + 4);
                a[2] = *reinterpret_cast<const uint4*>(rec + 8);
                const uint32_t dot = block_dot<F, 0>(w, a);
                if constexpr (SUMI) {
                    if (row_ok) sumi_out[((long)(m0 + m) * N + row) * nb + b] = (int)(dot - ACC_BIAS);
                } else {
                    acc[m] += block_term_rec<F, 0>(w, dot, a[2]);
                }
            }
        }
    }
    if constexpr (!SUMI) {
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = group_sum_last<64>(acc[m]);
        if (row_ok && lane == 63) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                if (m < mc) C[(long)(m0 + m) * ldc_m + (long)row * ldc_n] = acc[m];
        }
    }
}

constexpr size_t RG_LDS_MAX = 160 * 1024;
inline size_t ragged_lds(int mt, int K) { return (size_t)mt * (K / QK) * RG_RS * 4; }

// tokens per launch chunk: the next power of two >= M (at most 8), halved until the records fit
inline int ragged_mt(const GemmArgs& g) {
    for (int mt = g.M <= 1 ? 1 : g.M <= 2 ? 2 : g.M <= 4 ? 4 : 8; mt >= 1; mt /= 2)
        if (ragged_lds(mt, g.K) <= RG_LDS_MAX && (g.M + mt - 1) / mt <= 65535) return mt;
    return 0;
}

template <int F, int MT> hipError_t launch_mt(const GemmArgs& g, hipStream_t st) {
    const dim3 grid((g.N + RG_WGS / 64 - 1) / (RG_WGS / 64), (g.M + MT - 1) / MT);
    const size_t lds = ragged_lds(std::min(MT, g.M), g.K);
    if (g.describe) {
        describe_kernel(g, "ragged F=%d MT=%d grid=%ux%u", F, MT, grid.x, grid.y);
        return hipSuccess;
    }
    auto k = g.sumi ? ragged_kernel<F, MT, true> : ragged_kernel<F, MT, false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, grid, dim3(RG_WGS), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, g.C,
                       g.ldc_m, g.ldc_n, g.sumi);
    return hipGetLastError();
}

template <int F> hipError_t launch_f(const GemmArgs& g, hipStream_t st) {
    switch (ragged_mt(g)) {
        case 1: return launch_mt<F, 1>(g, st);
        case 2: return launch_mt<F, 2>(g, st);
        case 4: return launch_mt<F, 4>(g, st);
        case 8: return launch_mt<F, 8>(g, st);
    }
    return hipErrorInvalidValue;
}
}  // namespace

// 2-B aligned weights (every format's blocks are whole 2-B fields), 4-B aligned Q8_1 activations,
// the records of at least one token within the LDS.
bool ragged_eligible(const GemmArgs& g) {
    return g.ain == AIN_Q8_1 && g.M >= 1 && g.N >= 1 && ((uintptr_t)g.A & 3) == 0 && ((uintptr_t)g.B & 1) == 0 &&
           ragged_mt(g) > 0;
}

hipError_t launch_ragged(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return launch_f<FMT_Q4_0>(g, st);
        case FMT_Q4_1: return launch_f<FMT_Q4_1>(g, st);
        case FMT_Q5_0: return launch_f<FMT_Q5_0>(g, st);
        case FMT_Q5_1: return launch_f<FMT_Q5_1>(g, st);
        case FMT_Q8_0: return launch_f<FMT_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
