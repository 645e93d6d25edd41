// qg_gemvt.hip — the decode GEMV (M = 1 token) on the tiled weight layout (LAY_TILED,
// qg_tile_weights; tiled_fmt in qg_mmq_kernel.hpp), so weights kept only in that layout serve the decode
// as well as the prefill (qg_gemm_w4a8_tiled). C[M,N] = A_q8_1[M,K] . B[N,K]^T (include/gemm_reference.h:
// 175-222), each block's fp32 term in the reference's operation order (qg_common.hpp block_term_f), i.e.
// bit-identical per block to the oracle, summed in a fixed order (the summation-order bar of the GEMV).
//
// Work: a workgroup of W = 16 waves owns half a tile (16 weight rows) and all of K; wave w takes the
// stages h = w, w + W, ... (4 blocks each). Lane L = 4 r + q of a wave handles row r of the 16 and k-slot q:
// its 16 bytes of the stage's QS plane are piece 16 q + r of the half tile's 64 — one wave instruction
// reads the half tile's 1 KB as one contiguous run (the row-major AoS GEMV's lane unit is 36 B at a 36-B
// stride). The lane's fragment of block b is the MMQ's: qs dword q split into low / high nibbles (+ the
// qh bits, Q5_x; Q8_0: dwords q and 4 + q), dotted with the token's qs dwords q and 4 + q by two
// v_dot4_i32_i8. The four k-slot lanes of a row then reduce-scatter their 4 partial dots over the quad
// (DPP, exact integer adds): lane q ends with block q's exact sumi and computes that block's term. The
// lanes' fp32 partials meet over the quad (DPP) and over the waves (LDS, fixed wave order) at the end.
// Activations are staged into LDS once per workgroup as raw Q8_1 blocks (one thread per 36-B block).
#include "qg_common.hpp"
#include "qg_kernels.hpp"
#include "qg_mmq_kernel.hpp"

namespace qg {

namespace {

constexpr int GT_W = 16;  // waves per workgroup (16 rows)

template <int CTRL> __device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }

template <int F, int MT, bool SUMI, bool TA>
__global__ __launch_bounds__(GT_W * 64) void gemvt_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B, int M, int N,
                                                         int K, void* __restrict__ out, int ldc_m, int ldc_n) {
    using T = wfmt<F>;
    using TF = tiled_fmt<F>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int nb = K / QK, H = (nb + MMQ_SB - 1) / MMQ_SB;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int r = lane >> 2, q = lane & 3;
    const int half = gridDim.x <= 512 ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;  // 16-row tile
    const int n0 = half * 16;
    const int i16 = (n0 % TILE_ROWS) / 16;  // which half of its 32-row tile
    const uint8_t* tb = B + (long)(n0 / TILE_ROWS) * H * TF::STG;
    const int qs_off = i16 * 64 * TF::QSL + (q * 16 + r) * 16;
    const int row_in_tile = i16 * 16 + r;

    struct wst {  // one stage of this lane's weights
        uint4 qs, qs8, qh;
        uint4 sc;
    };
    auto load = [&](int h, wst& s) {
        const uint8_t* st = tb + (long)h * TF::STG;
        s.qs = *reinterpret_cast<const uint4*>(st + qs_off);
        if constexpr (T::Q8) s.qs8 = *reinterpret_cast<const uint4*>(st + qs_off + 1024);
        if constexpr (T::QH >= 0) s.qh = *reinterpret_cast<const uint4*>(st + TF::OQH + row_in_tile * 16);
        if constexpr (T::MOFF >= 0) {
            s.sc = *reinterpret_cast<const uint4*>(st + TF::OSC + row_in_tile * 16);
        } else {
            const uint2 v = *reinterpret_cast<const uint2*>(st + TF::OSC + row_in_tile * 8);
            s.sc = make_uint4(v.x, v.y, 0u, 0u);
        }
    };

    // activations: the M rows' raw Q8_1 blocks into LDS (9 dwords per block), the first issued before
    // the weight stream
    const int totb = M * nb;
    const int tid = threadIdx.x;
    uint32_t ab[9];
    const uint32_t* A32 = reinterpret_cast<const uint32_t*>(A);
    auto load_ablk = [&](int g) {
        long src = (long)g * 9;
        if constexpr (TA) {  // LAY_TILED_ACT: block b of token m inside its tile's 2304-B stage run
            const int m = g / nb, b = g - m * nb;
            src = (((long)(m / ACT_TILE) * H + b / MMQ_SB) * ACT_TILE + m % ACT_TILE) * (MMQ_SB * 9) + (b % MMQ_SB) * 9;
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) ab[i] = A32[src + i];
    };
    if (tid < totb) load_ablk(tid);
    // every stage of this wave (up to NS) in flight before the staging barrier; beyond NS (K > 8192) one
    // stage ahead
    const int nst = wave < H ? (H - 1 - wave) / GT_W + 1 : 0;
    constexpr int NS = 4;
    wst pre[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k)
        if (k < nst) load(wave + k * GT_W, pre[k]);
    for (int g = tid; g < totb; g += GT_W * 64) {
        if (g != tid) load_ablk(g);
#pragma unroll
        for (int i = 0; i < 9; ++i) lds[g * 9 + i] = ab[i];
    }
    __syncthreads();

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;
    const int n = n0 + r;
    auto stage = [&](const wst& cur, int h) {
        const uint32_t qv[4] = {cur.qs.x, cur.qs.y, cur.qs.z, cur.qs.w};
        const uint32_t q8[4] = {cur.qs8.x, cur.qs8.y, cur.qs8.z, cur.qs8.w};
        const uint32_t qhv[4] = {cur.qh.x, cur.qh.y, cur.qh.z, cur.qh.w};
        uint32_t lo[4], hi[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            if constexpr (T::Q8) {
                lo[b] = qv[b];
                hi[b] = q8[b];
            } else {
                lo[b] = qv[b] & 0x0F0F0F0Fu;
                hi[b] = (qv[b] >> 4) & 0x0F0F0F0Fu;
            }
            if constexpr (T::QH >= 0) {
                lo[b] |= spread4_bit4((qhv[b] >> (4 * q)) & 0xFu);
                hi[b] |= spread4_bit4((qhv[b] >> (16 + 4 * q)) & 0xFu);
            }
        }
        const int blk = h * MMQ_SB + q;  // the block this lane finishes
        const uint32_t scd = q < 2 ? cur.sc.x : cur.sc.y;
        const float dw = h2f((q & 1) ? scd >> 16 : scd & 0xFFFFu);
        float mw = 0.0f;
        if constexpr (T::MOFF >= 0) {
            const uint32_t scm = q < 2 ? cur.sc.z : cur.sc.w;
            mw = h2f((q & 1) ? scm >> 16 : scm & 0xFFFFu);
        }
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            if (m >= M) break;
            int p[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int bb = min(h * MMQ_SB + b, nb - 1);  // padding blocks: any real bytes (zero weights)
                const uint32_t* rec = lds + (m * nb + bb) * 9;
                p[b] = __builtin_amdgcn_sdot4((int)hi[b], (int)rec[5 + q], __builtin_amdgcn_sdot4((int)lo[b], (int)rec[1 + q], 0, false),
                                              false);
            }
            // reduce-scatter over the quad: lane q keeps block q
            const bool lo2 = q < 2;
            const int k0 = (lo2 ? p[0] : p[2]) + dpp_i<0x4E>(lo2 ? p[2] : p[0]);  // quad_perm [2,3,0,1]
            const int k1 = (lo2 ? p[1] : p[3]) + dpp_i<0x4E>(lo2 ? p[3] : p[1]);
            const bool odd = q & 1;
            const int s = (odd ? k1 : k0) + dpp_i<0xB1>(odd ? k0 : k1);  // quad_perm [1,0,3,2]
            if (blk < nb) {
                if constexpr (SUMI) {
                    if (n < N) static_cast<int32_t*>(out)[((long)m * N + n) * nb + blk] = s;
                } else {
                    const uint32_t ds = lds[(m * nb + blk) * 9];
                    acc[m] += block_term<F>(s, dw, mw, h2f(ds & 0xFFFFu), h2f(ds >> 16));
                }
            }
        }
    };
    static_for<NS>([&](auto KI) {
        constexpr int k = decltype(KI)::value;
        if (k < nst) stage(pre[k], wave + k * GT_W);
    });
    for (int k = NS; k < nst; ++k) {
        wst c;
        load(wave + k * GT_W, c);
        stage(c, wave + k * GT_W);
    }
    if constexpr (!SUMI) {
        // the row's 4 k-slot lanes, then the waves in fixed order
        float* red = reinterpret_cast<float*>(lds);
        __syncthreads();  // (the activation records are no longer read)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            acc[m] += dpp_f<0xB1>(acc[m]);
            acc[m] += dpp_f<0x4E>(acc[m]);
            if (q == 0 && m < M) red[(m * GT_W + wave) * 16 + r] = acc[m];
        }
        __syncthreads();
        if (tid < 16 * MT) {
            const int m = tid / 16, rr = tid % 16;
            if (m < M && n0 + rr < N) {
                float v = 0.0f;
                for (int w = 0; w < GT_W; ++w) v += red[(m * GT_W + w) * 16 + rr];
                static_cast<float*>(out)[(long)m * ldc_m + (long)(n0 + rr) * ldc_n] = v;
            }
        }
    }
}

template <int F, int MT> hipError_t gemvt_launch(const GemmArgs& g, hipStream_t st) {
    const int grid = (g.N + 15) / 16;
    const size_t lds = std::max((size_t)g.M * (g.K / QK) * 36, (size_t)MT * GT_W * 16 * 4);
    if (g.describe) {
        describe_kernel(g, "gemvt F=%d MT=%d W=%d TA=%d grid=%d", F, MT, GT_W, (int)(g.lay == LAY_TILED_ACT), grid);
        return hipSuccess;
    }
    const bool ta = g.lay == LAY_TILED_ACT;
    auto k = g.sumi ? (ta ? gemvt_kernel<F, MT, true, true> : gemvt_kernel<F, MT, true, false>)
                    : (ta ? gemvt_kernel<F, MT, false, true> : gemvt_kernel<F, MT, false, false>);
    if (lds > 64 * 1024) {
        static std::atomic<unsigned long long> done[4] = {};
        const hipError_t e = set_max_lds_once((const void*)k, 160 * 1024, done[(g.sumi ? 1 : 0) + (ta ? 2 : 0)]);
        if (e != hipSuccess) return e;
    }
    void* out = g.sumi ? (void*)g.sumi : (void*)g.C;
    hipLaunchKernelGGL(k, dim3(grid), dim3(GT_W * 64), lds, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, out,
                       (int)g.ldc_m, (int)g.ldc_n);
    return hipGetLastError();
}

template <int F> hipError_t gemvt_f(const GemmArgs& g, hipStream_t st) {
    switch (g.M) {
        case 1: return gemvt_launch<F, 1>(g, st);
        case 2: return gemvt_launch<F, 2>(g, st);
        default: return gemvt_launch<F, 4>(g, st);
    }
}

}  // namespace

// M = 1 only: against the tiled MFMA kernel (16-row tiles) it measured 4.19-4.26 vs 4.54 us at M = 1 but
// 4.88 vs 4.5 at M = 2 and 5.9-6.4 vs 4.5 at M = 4 (profiles/r05_tuning/r5b_ab_tiled.txt, r5c_ab_tiled.txt: the
// per-token LDS reads and quad reductions grow with M), so M = 2..4 run the MFMA kernel. The activation
// row within the LDS, 32-bit strides (A 4-B aligned, B_tiled 16-B aligned).
bool gemvt_eligible(const GemmArgs& g) {
    return (g.lay == LAY_TILED || g.lay == LAY_TILED_ACT) && g.M == 1 && g.N >= 1 && g.K % QK == 0 && ((uintptr_t)g.B & 15) == 0 &&
           ((uintptr_t)g.A & 3) == 0 && (size_t)g.M * (g.K / QK) * 36 <= 144 * 1024 && g.ldc_m <= INT32_MAX &&
           g.ldc_n <= INT32_MAX && (long)g.M * g.N * (g.K / QK) < (1L << 62);
}

hipError_t launch_gemvt(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return gemvt_f<FMT_Q4_0>(g, st);
        case FMT_Q4_1: return gemvt_f<FMT_Q4_1>(g, st);
        case FMT_Q5_0: return gemvt_f<FMT_Q5_0>(g, st);
        case FMT_Q5_1: return gemvt_f<FMT_Q5_1>(g, st);
        case FMT_Q8_0: return gemvt_f<FMT_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
