// qg_gemm_mfma.hip — W4A8 prefill GEMM (M > 8) on the CDNA4 matrix cores.
//
// v_mfma_i32_32x32x32_i8 has K = 32 = exactly one Q-block, so every MFMA yields the exact int32
// sumi of 32x32 (weight row, token) pairs for one block (include/gemm_reference.h:202-212); the
// per-block scale/compensation epilogue then runs on the VALU with the reference's operation
// order (qg_common.hpp block_term), so the fp32 terms are bit-identical to the CPU oracle's.
//
// Tiling:
//  * Workgroup = 4 waves, output tile 32 weight rows (n) x 32 tokens (m). MFMA A operand = weights
//    (row i = n), B operand = activations (column j = m): the accumulator holds C^T with column
//    m = lane & 31 and rows n = (r&3) + 8(r>>2) + 4(lane>>5), so each lane's token scales are
//    per-lane scalars and only the 16 weight scales per block need an LDS exchange.
//  * The K loop walks 256-element super-blocks; wave w owns blocks 2w and 2w+1 of every
//    super-block and fetches just the 16-B aligned window of its weight rows that covers them
//    (3 dwordx4 for Q4_0/Q4_1/Q5_1, 4 for Q5_0), DEPTH super-blocks ahead. The 4 partial tiles are
//    summed in fixed order through LDS at the end (deterministic).
//  * Operand k-order: both fragments use the same (lane half h, byte j) -> element map
//    e = (j < 8) ? 8h + j : 16 + 8h + (j - 8), so a lane needs only qs bytes [8h, 8h+8) of a block
//    (low nibbles -> j < 8, high nibbles -> j >= 8). Any bijection works because the MFMA pairs
//    A byte (h, j) with B byte (h, j); the integer sum is order-free.
//  * Activations (32 tokens x 8 blocks per super-block) are staged by all 256 threads into
//    double-buffered LDS records of 40 B [block][token]{qs[32], float d, float s}: 10-dword stride
//    -> the ds_read_b64 fragment reads of 32 tokens are bank-conflict-free.
#include "qg_common.hpp"
#include "qg_kernels.hpp"

namespace qg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int F> struct mfma_geom {
    static constexpr int BB = wfmt<F>::BB;
    static constexpr int SBB = 8 * BB;
    static constexpr int nwin() {
        int mx = 0;
        for (int w = 0; w < 4; ++w) {
            const int start = (2 * w * BB) & ~15;
            const int need = 2 * w * BB + 2 * BB - start;
            const int n = (need + 15) / 16;
            mx = n > mx ? n : mx;
        }
        return mx;
    }
    static constexpr int NWIN = nwin();
    static constexpr int wstart(int w) {
        const int s = (2 * w * BB) & ~15;
        const int lim = SBB - NWIN * 16;
        return s < lim ? s : lim;
    }
};

constexpr int ACT_REC = 10;                 // dwords per (block, token) record
constexpr int ACT_DW = 8 * 32 * ACT_REC;    // one super-block stage
constexpr int DWL_DW = 4 * 2 * 2 * 32;      // [wave][block-of-pair][d|m][row]
constexpr int MFMA_DEPTH = 4;               // super-blocks of weights in flight per wave

template <int F, int W, bool SUMI>
__device__ __forceinline__ void mfma_main_loop(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                               int32_t* __restrict__ sumi_out, int M, int N, int K, int n0, int m0,
                                               uint32_t* lds, float (&accf)[16]) {
    using T = wfmt<F>;
    using G = mfma_geom<F>;
    constexpr int NW = G::NWIN;
    constexpr int WS = G::wstart(W);
    const int nb = K / QK;
    const int S = K / SB_ELEMS;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int h = lane >> 5;
    const int l32 = lane & 31;

    // weights: this lane's row (A-operand row n = l32), window WS of every super-block
    const int nrow = min(n0 + l32, N - 1);
    const u32x4* wbase = reinterpret_cast<const u32x4*>(B + (long)nrow * nb * T::BB + WS);
    auto load_win = [&](u32x4 (&dst)[NW], int s) {
        const u32x4* p = wbase + (long)s * (G::SBB / 16);
#pragma unroll
        for (int v = 0; v < NW; ++v) dst[v] = p[v];
    };

    // activation staging: 9 dwords per thread per super-block
    uint32_t st[9];
    auto stage_load = [&](int s) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int g = tid + 256 * i;
            const int t = g / 72;
            const int w72 = g - t * 72;
            const int blk = w72 / 9;
            const int w = w72 - blk * 9;
            const int tok = min(m0 + t, M - 1);
            st[i] = *reinterpret_cast<const uint32_t*>(A + ((long)tok * nb + s * 8 + blk) * Q8_1_BYTES + 4 * w);
        }
    };
    auto stage_store = [&](int buf) {
        uint32_t* act = lds + buf * ACT_DW;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int g = tid + 256 * i;
            const int t = g / 72;
            const int w72 = g - t * 72;
            const int blk = w72 / 9;
            const int w = w72 - blk * 9;
            const int rec = (blk * 32 + t) * ACT_REC;
            if (w == 0) {
                act[rec + 8] = __float_as_uint(h2f(st[i] & 0xFFFFu));
                act[rec + 9] = __float_as_uint(h2f(st[i] >> 16));
            } else {
                act[rec + w - 1] = st[i];
            }
        }
    };

    u32x4 ring[MFMA_DEPTH][NW];
    stage_load(0);
    static_for<MFMA_DEPTH>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if (j < S) load_win(ring[j], j);
    });
    stage_store(0);
    __syncthreads();

    uint32_t* dwl = lds + 2 * ACT_DW + W * (2 * 2 * 32);
    for (int s0 = 0; s0 < S; s0 += MFMA_DEPTH) {
        static_for<MFMA_DEPTH>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const int s = s0 + j;
            if (s < S) {
                if (s + 1 < S) stage_load(s + 1);
                const uint32_t* act = lds + (s & 1) * ACT_DW;
                const uint32_t* w = reinterpret_cast<const uint32_t*>(ring[j]);
                static_for<2>([&](auto BW) {
                    constexpr int bw = decltype(BW)::value;
                    constexpr int b = 2 * W + bw;   // block within the super-block
                    constexpr int o = b * T::BB - WS;  // its byte offset inside the window
                    // ---- A fragment: weights, qs bytes [8h, 8h+8) split into low / high nibbles
                    const uint32_t v0 = vsel(h, ld32<o + T::QS + 8>(w), ld32<o + T::QS>(w));
                    const uint32_t v1 = vsel(h, ld32<o + T::QS + 12>(w), ld32<o + T::QS + 4>(w));
                    uint32_t lo0 = v0 & 0x0F0F0F0Fu, lo1 = v1 & 0x0F0F0F0Fu;
                    uint32_t hi0 = (v0 >> 4) & 0x0F0F0F0Fu, hi1 = (v1 >> 4) & 0x0F0F0F0Fu;
                    if constexpr (T::QH >= 0) {
                        const uint32_t qh = ld32<o + T::QH>(w);
                        const uint32_t bl = (qh >> (8 * h)) & 0xFFu;
                        const uint32_t bh = (qh >> (16 + 8 * h)) & 0xFFu;
                        lo0 |= spread4_bit4(bl & 0xFu);
                        lo1 |= spread4_bit4(bl >> 4);
                        hi0 |= spread4_bit4(bh & 0xFu);
                        hi1 |= spread4_bit4(bh >> 4);
                    }
                    const v4i afrag = {(int)lo0, (int)lo1, (int)hi0, (int)hi1};
                    // ---- B fragment: activations of token l32, same element map
                    const uint32_t* rec = act + (b * 32 + l32) * ACT_REC;
                    const uint2 q0 = *reinterpret_cast<const uint2*>(rec + 2 * h);
                    const uint2 q1 = *reinterpret_cast<const uint2*>(rec + 4 + 2 * h);
                    const float2 ds = *reinterpret_cast<const float2*>(rec + 8);
                    const v4i bfrag = {(int)q0.x, (int)q0.y, (int)q1.x, (int)q1.y};
                    // ---- weight scales of the 16 accumulator rows, exchanged through LDS
                    const float dw_own = h2f(ld16<o>(w));
                    float mw_own = 0.0f;
                    if constexpr (T::MOFF >= 0) mw_own = h2f(ld16<o + T::MOFF>(w));
                    if (h == 0) {
                        dwl[bw * 64 + l32] = __float_as_uint(dw_own);
                        dwl[bw * 64 + 32 + l32] = __float_as_uint(mw_own);
                    }
                    const v16i zero = {};
                    const v16i si = __builtin_amdgcn_mfma_i32_32x32x32_i8(afrag, bfrag, zero, 0, 0, 0);
                    float dws[16], mws[16];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 d4 = *reinterpret_cast<const float4*>(dwl + bw * 64 + 8 * q + 4 * h);
                        dws[4 * q] = d4.x; dws[4 * q + 1] = d4.y; dws[4 * q + 2] = d4.z; dws[4 * q + 3] = d4.w;
                        if constexpr (T::MOFF >= 0) {
                            const float4 m4 = *reinterpret_cast<const float4*>(dwl + bw * 64 + 32 + 8 * q + 4 * h);
                            mws[4 * q] = m4.x; mws[4 * q + 1] = m4.y; mws[4 * q + 2] = m4.z; mws[4 * q + 3] = m4.w;
                        } else {
                            mws[4 * q] = mws[4 * q + 1] = mws[4 * q + 2] = mws[4 * q + 3] = 0.0f;
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        if constexpr (SUMI) {
                            const int n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
                            const int m = m0 + l32;
                            if (n < N && m < M) sumi_out[((long)m * N + n) * nb + s * 8 + b] = si[r];
                        } else {
                            accf[r] += block_term<F>(si[r], dws[r], mws[r], ds.x, ds.y);
                        }
                    }
                });
                if (s + MFMA_DEPTH < S) load_win(ring[j], s + MFMA_DEPTH);
                if (s + 1 < S) stage_store((s + 1) & 1);
                __syncthreads();
            }
        });
    }
}

template <int F, bool SUMI>
__global__ __launch_bounds__(256) void mfma_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                   float* __restrict__ C, int32_t* __restrict__ sumi_out, int M, int N,
                                                   int K, long ldc_m, long ldc_n) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[2 * ACT_DW + DWL_DW];
    const int n0 = blockIdx.x * 32;
    const int m0 = blockIdx.y * 32;
    const int W = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float accf[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) accf[r] = 0.0f;
    switch (W) {
        case 0: mfma_main_loop<F, 0, SUMI>(A, B, sumi_out, M, N, K, n0, m0, lds, accf); break;
        case 1: mfma_main_loop<F, 1, SUMI>(A, B, sumi_out, M, N, K, n0, m0, lds, accf); break;
        case 2: mfma_main_loop<F, 2, SUMI>(A, B, sumi_out, M, N, K, n0, m0, lds, accf); break;
        default: mfma_main_loop<F, 3, SUMI>(A, B, sumi_out, M, N, K, n0, m0, lds, accf); break;
    }
    if constexpr (!SUMI) {
        // fixed-order sum of the 4 waves' partial tiles (the main loop ended on a barrier)
        float* red = reinterpret_cast<float*>(lds);
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int r = 0; r < 16; ++r) red[W * 1024 + r * 64 + lane] = accf[r];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = threadIdx.x + 256 * i;
            const int r = idx >> 6, ln = idx & 63;
            const float v = ((red[idx] + red[1024 + idx]) + red[2048 + idx]) + red[3072 + idx];
            const int n = n0 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
            const int m = m0 + (ln & 31);
            if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v;
        }
    }
}

namespace {
template <int F> hipError_t launch_m(const GemmArgs& g, hipStream_t st) {
    const dim3 grid((g.N + 31) / 32, (g.M + 31) / 32);
    if (g.sumi)
        hipLaunchKernelGGL((mfma_kernel<F, true>), grid, dim3(256), 0, st, (const uint8_t*)g.A, (const uint8_t*)g.B,
                           g.C, g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    else
        hipLaunchKernelGGL((mfma_kernel<F, false>), grid, dim3(256), 0, st, (const uint8_t*)g.A, (const uint8_t*)g.B,
                           g.C, g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}
}  // namespace

bool mfma_eligible(const GemmArgs& g) {
    if (g.M < 1 || g.N < 1 || g.K % SB_ELEMS != 0) return false;
    if (((uintptr_t)g.B & 15) != 0 || ((uintptr_t)g.A & 3) != 0) return false;
    if ((g.M + 31) / 32 > 65535) return false;
    return g.wtype == FMT_Q4_0 || g.wtype == FMT_Q4_1 || g.wtype == FMT_Q5_0 || g.wtype == FMT_Q5_1;
}

hipError_t launch_mfma(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return launch_m<FMT_Q4_0>(g, st);
        case FMT_Q4_1: return launch_m<FMT_Q4_1>(g, st);
        case FMT_Q5_0: return launch_m<FMT_Q5_0>(g, st);
        case FMT_Q5_1: return launch_m<FMT_Q5_1>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
