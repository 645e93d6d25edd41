// qg_gemv.hip — W4A8 GEMV / small-batch GEMM (M <= 8 activation rows) for gfx950.
//
// Computes C[m][n] = sum_b term(A_q8_1[m][b], B_w[n][b]) for the reference's activation-major
// contract C[M,N] = A[M,K] * B[N,K]^T (include/gemm_reference.h:175-222); the weight-major entry
// (kernels/gemm/gemm_quant_formats.cuh:343) is the same kernel with transposed output strides.
//
// Design (HBM-bound weight stream):
//  * A weight row of K elements is K/256 "super-blocks" of 8 blocks (144 B for Q4_0). Lane
//    `lir` of a row group owns super-blocks lir, lir+LPR, ... and fetches each with 9..12
//    global_load_dwordx4 (16-B aligned because every super-block is a multiple of 16 B and rows
//    are K/256 super-blocks long). LPR lanes share a row, 64/LPR rows per wave, 4 waves per
//    workgroup; ~one workgroup per CU at the decode shapes, so every weight byte of the launch is
//    requested in the first few hundred cycles.
//  * Blocks are decoded in registers with compile-time v_alignbyte/shift/mask (qg_common.hpp) and
//    dotted against the int8 activations with v_dot4c_i32_i8 (__builtin_amdgcn_sdot4): sumi is the
//    exact int32 of the reference's inner loop (gemm_reference.h:202-212).
//  * The Q8_1 activations (4.6 KB per row at K=4096) are staged once per workgroup into LDS as
//    336-byte records per (row, super-block): 256 B of int8 qs + 8 x float2 (d, s) + 16 B pad. The
//    84-dword record stride makes the 16 different super-blocks a 16-lane ds_read_b128 group touches
//    land on 16 distinct 4-bank slots (conflict-free); lanes of different rows reading the same
//    super-block broadcast.
//  * Per-lane partial sums (block order) are tree-reduced across the LPR lanes of a row with
//    __shfl_xor; lane 0 of the row stores. Fully deterministic.
#include "qg_common.hpp"
#include "qg_kernels.hpp"

namespace qg {

constexpr int AREC_DW = 84;  // 336-byte activation record per (row, super-block)

template <int F, int MT, int LPR, int NSTAGE, bool NT, bool SUMI>
__global__ __launch_bounds__(256) void gemv_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                   float* __restrict__ C, int32_t* __restrict__ sumi_out, int M, int N,
                                                   int K, long ldc_m, long ldc_n) {
    using T = wfmt<F>;
    constexpr int SBB = SB_BLOCKS * T::BB;  // super-block bytes
    constexpr int NV4 = SBB / 16;           // dwordx4 loads per super-block
    constexpr int NW = SBB / 4;
    constexpr int RPW = 64 / LPR;           // rows per wave
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    const int nb = K / QK;
    const int S = K / SB_ELEMS;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int lir = lane % LPR;
    const int row = blockIdx.x * (4 * RPW) + wave * RPW + lane / LPR;
    const bool row_ok = row < N;
    const long row_bytes = (long)S * SBB;

    // 1) activation staging loads (issued first so they do not queue behind the weight stream)
    const int tot = M * nb * 9;
    uint32_t av[NSTAGE];
#pragma unroll
    for (int i = 0; i < NSTAGE; ++i) {
        const int g = tid + i * 256;
        av[i] = g < tot ? A[g] : 0u;
    }

    // 2) first super-block of weights
    const u32x4* wrow = reinterpret_cast<const u32x4*>(B + (long)(row_ok ? row : 0) * row_bytes);
    auto load_sb = [&](u32x4 (&dst)[NV4], int s) {
        const bool ok = row_ok && s < S;
        const u32x4* p = wrow + (long)(ok ? s : 0) * NV4;
#pragma unroll
        for (int v = 0; v < NV4; ++v) {
            if constexpr (NT) dst[v] = __builtin_nontemporal_load(p + v);
            else dst[v] = p[v];
        }
    };
    u32x4 cur[NV4];
    load_sb(cur, lir);

    // 3) scatter activations into the LDS record layout
#pragma unroll
    for (int i = 0; i < NSTAGE; ++i) {
        const int g = tid + i * 256;
        if (g < tot) {
            const int blk = g / 9;
            const int w = g - blk * 9;
            const int m = blk / nb;
            const int b = blk - m * nb;
            const int rec = (m * S + (b >> 3)) * AREC_DW;
            const int bi = b & 7;
            if (w == 0) {
                lds[rec + 64 + 2 * bi] = __float_as_uint(h2f(av[i] & 0xFFFFu));
                lds[rec + 65 + 2 * bi] = __float_as_uint(h2f(av[i] >> 16));
            } else {
                lds[rec + 8 * bi + (w - 1)] = av[i];
            }
        }
    }
    __syncthreads();

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;

    const int spl = (S + LPR - 1) / LPR;
    for (int j = 0; j < spl; ++j) {
        const int s = lir + j * LPR;
        u32x4 nxt[NV4];
        if (j + 1 < spl) load_sb(nxt, s + LPR);
        if (s < S) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(cur);
            static_for<SB_BLOCKS>([&](auto BI) {
                constexpr int bi = decltype(BI)::value;
                const wblock wb = decode_block<F, bi>(w);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    if (m < M) {
                        const uint32_t* rec = lds + (m * S + s) * AREC_DW;
                        const uint4 a0 = *reinterpret_cast<const uint4*>(rec + 8 * bi);
                        const uint4 a1 = *reinterpret_cast<const uint4*>(rec + 8 * bi + 4);
                        const float2 ds = *reinterpret_cast<const float2*>(rec + 64 + 2 * bi);
                        const uint32_t a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                        const int sumi = dot_block(wb.q, a);
                        if constexpr (SUMI) {
                            if (row_ok) sumi_out[((long)m * N + row) * nb + s * SB_BLOCKS + bi] = sumi;
                        } else {
                            acc[m] += block_term<F>(sumi, wb.d, wb.m, ds.x, ds.y);
                        }
                    }
                }
            });
        }
        if (j + 1 < spl) {
#pragma unroll
            for (int v = 0; v < NV4; ++v) cur[v] = nxt[v];
        }
    }
    if constexpr (!SUMI) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
#pragma unroll
            for (int off = LPR / 2; off > 0; off >>= 1) acc[m] += __shfl_xor(acc[m], off);
        }
        if (row_ok && lir == 0) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                if (m < M) C[m * ldc_m + row * ldc_n] = acc[m];
        }
    }
}

// ---- host-side launcher ---------------------------------------------------------------------

namespace {
template <int F, int MT, int LPR, int NSTAGE, bool NT, bool SUMI>
hipError_t launch_one(const GemmArgs& g, hipStream_t st) {
    constexpr int RPW = 64 / LPR;
    const int S = g.K / SB_ELEMS;
    const size_t lds = (size_t)g.M * S * AREC_DW * 4;
    const int grid = (g.N + 4 * RPW - 1) / (4 * RPW);
    auto kfn = gemv_kernel<F, MT, LPR, NSTAGE, NT, SUMI>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(256), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.C, g.sumi,
                       g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}

template <int F, int MT, int LPR, bool SUMI>
hipError_t launch_nt(const GemmArgs& g, hipStream_t st) {
    constexpr int NSTAGE = MT * (LPR == 64 ? 32 : 8);
    if (g.nontemporal) return launch_one<F, MT, LPR, NSTAGE, true, SUMI>(g, st);
    return launch_one<F, MT, LPR, NSTAGE, false, SUMI>(g, st);
}

template <int F, int LPR, bool SUMI>
hipError_t launch_m(const GemmArgs& g, hipStream_t st) {
    if (g.M <= 1) return launch_nt<F, 1, LPR, SUMI>(g, st);
    if (g.M <= 2) return launch_nt<F, 2, LPR, SUMI>(g, st);
    if (g.M <= 4) return launch_nt<F, 4, LPR, SUMI>(g, st);
    return launch_nt<F, 8, LPR, SUMI>(g, st);
}

template <int F, bool SUMI> hipError_t launch_f(const GemmArgs& g, hipStream_t st) {
    const int S = g.K / SB_ELEMS;
    if (S >= 64) return launch_m<F, 64, SUMI>(g, st);
    return launch_m<F, 16, SUMI>(g, st);
}
}  // namespace

static int mt_of(int M) { return M <= 1 ? 1 : M <= 2 ? 2 : M <= 4 ? 4 : 8; }

bool gemv_eligible(const GemmArgs& g) {
    if (g.M < 1 || g.M > 8) return false;
    if (g.K % SB_ELEMS != 0) return false;
    if (((uintptr_t)g.B & 15) != 0 || ((uintptr_t)g.A & 3) != 0) return false;
    const int S = g.K / SB_ELEMS;
    const int LPR = S >= 64 ? 64 : 16;
    const long nstage = (long)mt_of(g.M) * (LPR == 64 ? 32 : 8);
    if ((long)g.M * (g.K / QK) * 9 > nstage * 256) return false;
    if ((long)g.M * S * AREC_DW * 4 > 96 * 1024) return false;
    return true;
}

const char* gemv_kernel_name() { return "gemv_kernel"; }

hipError_t launch_gemv(const GemmArgs& g, hipStream_t st) {
    const bool sumi = g.sumi != nullptr;
    switch (g.wtype) {
        case FMT_Q4_0: return sumi ? launch_f<FMT_Q4_0, true>(g, st) : launch_f<FMT_Q4_0, false>(g, st);
        case FMT_Q4_1: return sumi ? launch_f<FMT_Q4_1, true>(g, st) : launch_f<FMT_Q4_1, false>(g, st);
        case FMT_Q5_0: return sumi ? launch_f<FMT_Q5_0, true>(g, st) : launch_f<FMT_Q5_0, false>(g, st);
        case FMT_Q5_1: return sumi ? launch_f<FMT_Q5_1, true>(g, st) : launch_f<FMT_Q5_1, false>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
