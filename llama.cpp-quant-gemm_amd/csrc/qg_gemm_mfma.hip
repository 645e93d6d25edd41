// qg_gemm_mfma.hip — W4A8 prefill GEMM (M > 8) on the CDNA4 matrix cores.
//
// v_mfma_i32_32x32x32_i8 has K = 32 = exactly one Q-block, so every MFMA yields the exact int32
// sumi of 32x32 (weight row, token) pairs for one block (include/gemm_reference.h:202-212); the
// per-block term then runs on the VALU in the reference's operation order (qg_common.hpp
// block_term, bit-identical to the CPU oracle), accumulated with one fused multiply-add
// (|fma - (acc + round(d_w * t))| <= half an ulp of the term, inside the summation-order bound).
//
// Tiling:
//  * Workgroup = 8 waves on one 32 (weight rows n) x 32 (tokens m) output tile. MFMA A operand =
//    weights (row i = n), B operand = activations (column j = m): the accumulator holds C^T with
//    column m = lane & 31 and rows n = (r&3) + 8(r>>2) + 4(lane>>5), so the token scales are per-lane
//    scalars and only the 16 weight scales per block go through LDS.
//  * The K dimension is split across the waves: wave w owns 256-element super-blocks w, w+8, ...
//    There is no barrier in the main loop — each wave streams its own weights (the full 144-B
//    super-block of its row, 9 x dwordx4) and its own activations (32 tokens x 288 B, 9 x dwordx4
//    per lane) two super-blocks ahead, stages the activations into a wave-private LDS region and
//    runs 8 MFMAs. The 8 partial tiles are summed in fixed order through LDS at the end.
//  * Operand k-order: both fragments use the same (lane half h, byte j) -> element map
//    e = (j < 8) ? 8h + j : 16 + 8h + (j - 8), so a lane needs only qs bytes [8h, 8h+8) of a block
//    (low nibbles -> j < 8, high nibbles -> j >= 8). The MFMA pairs A byte (h, j) with B byte (h, j),
//    and the integer sum is order-free.
//  * Wave-private activation records [block][token]{qs[32], {d, s} halves, pad}: 10-dword stride ->
//    the ds_read_b64 fragment reads of 32 tokens are bank-conflict-free.
#include "qg_common.hpp"
#include "qg_kernels.hpp"

namespace qg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int MF_WAVES = 8;
constexpr int ACT_REC = 10;                      // dwords per (block, token) record
constexpr int ACT_DW = 8 * 32 * ACT_REC;         // one super-block of one 32-token tile
constexpr int DWL_DW = 8 * 2 * 32;               // [block][d|m][row]
constexpr int WAVE_DW = ACT_DW + DWL_DW;         // per-wave LDS
constexpr int MF_LDS_DW = MF_WAVES * WAVE_DW;    // 96 KB; the end-of-loop reduction reuses it

template <int F, bool SUMI>
__global__ __launch_bounds__(512) void mfma_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                   float* __restrict__ C, int32_t* __restrict__ sumi_out, int M, int N,
                                                   int K, long ldc_m, long ldc_n) {
    using T = wfmt<F>;
    constexpr int SBB = 8 * T::BB;
    constexpr int NV4 = SBB / 16;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    const int n0 = blockIdx.x * 32;
    const int m0 = blockIdx.y * 32;
    const int W = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int nb = K / QK;
    const int S = K / SB_ELEMS;
    uint32_t* act = lds + W * WAVE_DW;
    uint32_t* dwl = act + ACT_DW;

    // this lane's weight row (A-operand row n = l32) and activation pieces (16 B each; piece
    // p = i*64 + lane covers token p/18, bytes 16*(p%18).. of its 288-B super-block run)
    const int nrow = min(n0 + l32, N - 1);
    const u32x4* wrow = reinterpret_cast<const u32x4*>(B + (long)nrow * nb * T::BB);
    auto load_w = [&](u32x4 (&wv)[NV4], int s) {
        const u32x4* p = wrow + (long)s * NV4;
#pragma unroll
        for (int v = 0; v < NV4; ++v) wv[v] = p[v];
    };
    // Activations: lane (token t = lane & 31, half hh = lane >> 5) fetches the 9 x 16 B of its
    // token's 288-B super-block run that hold blocks 4hh..4hh+3 (dwords 36hh..36hh+35), so every
    // source and LDS address is one per-lane base plus a compile-time offset.
    const int hh = lane >> 5;
    const int tok = min(m0 + l32, M - 1);
    const uint8_t* arow = A + (long)tok * nb * Q8_1_BYTES + hh * 144;
    uint32_t* arec = act + (4 * hh * 32 + l32) * ACT_REC;
    auto load_a = [&](u32x4 (&av)[9], int s) {
        const u32x4* p = reinterpret_cast<const u32x4*>(arow + (long)s * 8 * Q8_1_BYTES);
#pragma unroll
        for (int i = 0; i < 9; ++i) av[i] = p[i];
    };
    // dword d of the lane's 36: block d/9, field d%9 (0 = raw {d, s} halves -> slot 8, else qs)
    auto stage = [&](const u32x4 (&av)[9]) {
        static_for<36>([&](auto D) {
            constexpr int d = decltype(D)::value;
            constexpr int bl = d / 9, w = d % 9;
            arec[bl * 32 * ACT_REC + (w == 0 ? 8 : w - 1)] = av[d / 4][d % 4];
        });
    };

    float accf[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) accf[r] = 0.0f;

    // the 8 MFMAs of one staged super-block s, weights in registers wv
    auto compute_sb = [&](const u32x4 (&wv)[NV4], int s) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(wv);
            static_for<8>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
                constexpr int o = b * T::BB;
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
                const uint32_t dsh = rec[8];
            const float2 ds = {h2f(dsh & 0xFFFFu), h2f(dsh >> 16)};
                const v4i bfrag = {(int)q0.x, (int)q0.y, (int)q1.x, (int)q1.y};
                // ---- weight scales of the 16 accumulator rows, exchanged through wave-private LDS
                if (h == 0) {
                    dwl[b * 64 + l32] = __float_as_uint(h2f(ld16<o>(w)));
                    if constexpr (T::MOFF >= 0) dwl[b * 64 + 32 + l32] = __float_as_uint(h2f(ld16<o + T::MOFF>(w)));
                }
                const v16i zero = {};
                const v16i si = __builtin_amdgcn_mfma_i32_32x32x32_i8(afrag, bfrag, zero, 0, 0, 0);
    #pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 d4 = *reinterpret_cast<const float4*>(dwl + b * 64 + 8 * q + 4 * h);
                    float4 m4 = {0.0f, 0.0f, 0.0f, 0.0f};
                    if constexpr (T::MOFF >= 0) m4 = *reinterpret_cast<const float4*>(dwl + b * 64 + 32 + 8 * q + 4 * h);
                    const float dws[4] = {d4.x, d4.y, d4.z, d4.w};
                    const float mws[4] = {m4.x, m4.y, m4.z, m4.w};
    #pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int r = 4 * q + e;
                        if constexpr (SUMI) {
                            const int n = n0 + e + 8 * q + 4 * h;
                            const int m = m0 + l32;
                            if (n < N && m < M) sumi_out[((long)m * N + n) * nb + s * 8 + b] = si[r];
                        } else {
                            accf[r] += block_term<F>(si[r], dws[e], mws[e], ds.x, ds.y);
                        }
                    }
                }
                // Retire this block's epilogue before the next block: without the pin, IR passes sink all
                // eight epilogues below the last MFMA and keep 8 x 16 results live (scratch spills).
                if constexpr (!SUMI)
                    asm volatile("" : "+v"(accf[0]), "+v"(accf[1]), "+v"(accf[2]), "+v"(accf[3]), "+v"(accf[4]),
                                 "+v"(accf[5]), "+v"(accf[6]), "+v"(accf[7]), "+v"(accf[8]), "+v"(accf[9]),
                                 "+v"(accf[10]), "+v"(accf[11]), "+v"(accf[12]), "+v"(accf[13]), "+v"(accf[14]),
                                 "+v"(accf[15]));
                __builtin_amdgcn_sched_barrier(0);
            });
    };

    // Super-blocks of this wave: s = W, W + 8, ... processed in pairs. Both weight super-blocks of a
    // pair are requested at once (at K = 4096 every wave has exactly one pair, so the whole weight
    // tile is in flight from the first cycles); activations are staged one super-block at a time,
    // the second one's loads overlapping the first one's MFMAs.
    u32x4 w0[NV4], w1[NV4], av[9];
    for (int s = W; s < S; s += 2 * MF_WAVES) {
        const int s1 = s + MF_WAVES;
        const bool two = s1 < S;
        load_a(av, s);
        load_w(w0, s);
        if (two) load_w(w1, s1);
        stage(av);
        if (two) load_a(av, s1);
        compute_sb(w0, s);
        if (two) {
            stage(av);
            compute_sb(w1, s1);
        }
    }
    if constexpr (!SUMI) {
        // fixed-order sum of the 8 waves' partial tiles
        __syncthreads();
        float* red = reinterpret_cast<float*>(lds);
#pragma unroll
        for (int r = 0; r < 16; ++r) red[W * 1024 + r * 64 + lane] = accf[r];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int idx = threadIdx.x + 512 * i;
            const int r = idx >> 6, ln = idx & 63;
            float v = red[idx];
#pragma unroll
            for (int ww = 1; ww < MF_WAVES; ++ww) v += red[ww * 1024 + idx];
            const int n = n0 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
            const int m = m0 + (ln & 31);
            if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v;
        }
    }
}

namespace {
template <int F> hipError_t launch_m(const GemmArgs& g, hipStream_t st) {
    const dim3 grid((g.N + 31) / 32, (g.M + 31) / 32);
    const size_t lds = (size_t)MF_LDS_DW * 4;
    auto k = g.sumi ? mfma_kernel<F, true> : mfma_kernel<F, false>;
    static bool attr_set[2] = {false, false};  // once per instantiation (not a stream op: capture-safe)
    if (!attr_set[g.sumi ? 1 : 0]) {
        hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set[g.sumi ? 1 : 0] = true;
    }
    hipLaunchKernelGGL(k, grid, dim3(512), lds, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.C, g.sumi, g.M,
                       g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}
}  // namespace

bool mfma_eligible(const GemmArgs& g) {
    if (g.M < 1 || g.N < 1 || g.K % SB_ELEMS != 0) return false;
    if (((uintptr_t)g.B & 15) != 0 || ((uintptr_t)g.A & 15) != 0) return false;
    if ((g.K / QK) % 4 != 0) return false;  // 16-B aligned activation rows (nb * 36 % 16 == 0)
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
