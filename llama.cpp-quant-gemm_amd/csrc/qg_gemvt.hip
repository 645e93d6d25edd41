// qg_gemvt.hip — the decode GEMV (M <= 4 tokens) on the tiled weight layout (LAY_TILED / LAY_TILED_ACT;
// qg_tile_weights, tiled_fmt in qg_common.hpp), round 6: one resident tiled copy of
// the weights serves decode as fast as the reference rows serve it, and the prefill's MFMA kernels too.
// C[M,N] = A_q8_1[M,K] . B[N,K]^T (include/gemm_reference.h:175-222); every block's fp32 term in the
// reference's operation order (qg_gemv_kernel.hpp block_term_t: bit-identical per block to the oracle),
// summed in a fixed order.
//
// Why this shape. A (tile, stage) run keeps, per 16-row half tile, the k-slot-q pieces of 16 consecutive
// rows as 256 contiguous bytes (QS plane [half tile][q][row][16 B]). A wave of R = 16 rows x SL = 4 stages
// (lane = SL r + s) reads its lane's 4 pieces (dword q of the 4 blocks of row r, stage s) with 4
// global_load_dwordx4: each instruction covers 4 x 256 contiguous bytes, 8 whole 128-B lines — a better
// load shape than the row layout's 36-B units (18 lines per instruction, partly used). The lane then holds
// 4 WHOLE blocks of one row (the gemvt_unit register layout), so the dot is the row kernel's nibble-plane
// v_dot8 pair per qs dword with no cross-lane exchange, and the per-block epilogue is the row kernel's.
// (The first tiled decode kernel, round 5, gave each lane one k-slot of 4 blocks and needed a quad
// reduce-scatter per block: 4.3 us; the row kernel on units gathered from the planes, 32 partly used lines
// per instruction, 4.36 us.)
//  * The W waves of a workgroup split the row group's stages: wave w takes stages w NU SL .. +NU SL
//    (NU per lane, all in flight before anything waits).
//  * Each wave stages ONLY its own stages' activation records (one lane per Q8_1 block) in a wave-private
//    LDS region and reads them back after a wave-local fence: no workgroup barrier in front of the dots.
//  * Row sums: the SL stage lanes of a row by DPP (group_sum_last), the W waves through LDS in fixed wave
//    order after the one workgroup barrier; deterministic.
#include "qg_gemv_kernel.hpp"

namespace qg {

namespace {

// tuning (A/B builds): rows per wave (16: the half tile, 4 stage lanes; 8: 8 stage lanes; 0: per shape, below)
// and stages per lane
#ifndef QG_GEMVT_R
#define QG_GEMVT_R 0
#endif
#ifndef QG_GEMVT_NU
#define QG_GEMVT_NU 0  // 0: per K (gemvt_nu below)
#endif

constexpr int GT_SB = 4;  // blocks per stage (tiled_fmt)

template <int F, int MT, int R, int NU, bool SUMI, bool TA>
__global__ __launch_bounds__(1024) void gemvt_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, int M, int N,
                                                     int K, void* __restrict__ out, int ldc_m, int ldc_n) {
    using T = wfmt<F>;
    using TF = tiled_fmt<F>;
    using TU = gemvt_unit<F, GT_SB>;
    constexpr int SL = 64 / R;                // stage lanes per row
    constexpr int NBW = GT_SB * SL * NU;      // blocks per wave (per token)
    constexpr int UDW = TU::UDW;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    const int nb = K / QK, H = (nb + GT_SB - 1) / GT_SB;
    const int W = blockDim.x >> 6;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int r = lane / SL, s = lane % SL;
    const int tile = gridDim.x <= 512 ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int n = tile * R + r;  // this lane's weight row (rows past N: the layout's zero rows)
    const int rr = n % TILE_ROWS;
    const uint8_t* rowp = B + (long)(n / TILE_ROWS) * H * TF::STG;  // the row's tile, stage 0
    const int oqs = (rr >> 4) * 64 * TF::QSL + (rr & 15) * 16;      // piece q = 0 of the row in a stage run
    const int h0 = wave * (NU * SL);                                // the wave's first stage

    // 1) the lane's first activation block (staging item 0), then every weight unit of the lane
    const int RSTR = 48 * MT + 4;  // record dwords per staged stage (12 per block and token, +4: bank spread)
    uint32_t* wl = lds + wave * (NU * SL) * RSTR;
    constexpr int NIT = (NBW * MT + 63) / 64;  // staging items per lane, ALL loaded before the weight stream
    uint32_t ab[NIT][9];
    auto load_ablk = [&](int it, uint32_t (&d)[9]) {  // staging item it = m * NBW + jb
        const int m = it / NBW, jb = it % NBW, gb = wave * NBW + jb;
        if (m >= M || gb >= (TA ? H * GT_SB : nb)) {
#pragma unroll
            for (int i = 0; i < 9; ++i) d[i] = 0u;
            return;
        }
        long src = ((long)m * nb + gb) * 9;
        if constexpr (TA)  // block gb of token m inside its tile's 2304-B stage run (zero padding blocks)
            src = (((long)(m / ACT_TILE) * H + (gb >> 2)) * ACT_TILE + m % ACT_TILE) * 36 + (gb & 3) * 9;
#pragma unroll
        for (int i = 0; i < 9; ++i) d[i] = A[src + i];
    };
#pragma unroll
    for (int k = 0; k < NIT; ++k)
        if (lane + 64 * k < NBW * MT) load_ablk(lane + 64 * k, ab[k]);

    uint32_t wu[NU][UDW];
#pragma unroll
    for (int j = 0; j < NU; ++j) {
        const int h = min(h0 + j * SL + s, H - 1);  // (stages past H: any real bytes, not accumulated)
        const uint8_t* st = rowp + (long)h * TF::STG;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int hf = 0; hf < (T::Q8 ? 2 : 1); ++hf) {
                const uint4 v = *reinterpret_cast<const uint4*>(st + oqs + 256 * q + 1024 * hf);
                wu[j][0 * TU::QSD + 4 * hf + q] = v.x; wu[j][1 * TU::QSD + 4 * hf + q] = v.y;
                wu[j][2 * TU::QSD + 4 * hf + q] = v.z; wu[j][3 * TU::QSD + 4 * hf + q] = v.w;
            }
        }
        if constexpr (T::QH >= 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(st + TF::OQH + rr * 16);
            wu[j][TU::OQH] = v.x; wu[j][TU::OQH + 1] = v.y; wu[j][TU::OQH + 2] = v.z; wu[j][TU::OQH + 3] = v.w;
        }
        if constexpr (T::MOFF >= 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(st + TF::OSC + rr * TF::SCB);
            wu[j][TU::OD] = v.x; wu[j][TU::OD + 1] = v.y; wu[j][TU::OM] = v.z; wu[j][TU::OM + 1] = v.w;
        } else {
            const uint2 v = *reinterpret_cast<const uint2*>(st + TF::OSC + rr * TF::SCB);
            wu[j][TU::OD] = v.x; wu[j][TU::OD + 1] = v.y;
        }
    }

    // 2) the wave's records: item it -> stage-local block jb = 4 jl + b, token m, at jl * RSTR + (b MT + m) * 12
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
        const int it = lane + 64 * k;
        if (it < NBW * MT) {
            const int m = it / NBW, jb = it % NBW;
            make_act_record<F>(ab[k], wl + (jb >> 2) * RSTR + ((jb & 3) * MT + m) * 12);
        }
    }
    // the records were written by other lanes of this wave: LDS executes a wave's instructions in order, so
    // a fence that keeps the compiler from moving the reads above the writes is all that is needed
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // 3) dots and per-block terms, unit by unit, block by block. The records of step i = (unit j, block b)
    //    are read PD steps ahead (all of unit 0 before the first weight byte is waited for), so the LDS
    //    latency sits under the weight stream instead of between the dots of the tail (4.16 -> 4.07 us at
    //    M = 1, N = K = 4096; K = 14336 8.94 -> 7.76 with 2 stages per lane).
    constexpr int NS = NU * GT_SB;
    // (within the 128 VGPRs of a 1024-thread workgroup; the byte-decode formats need more for the dot)
    constexpr int PD = MT == 1 ? 4 : MT == 2 ? (gemv_planes<F> ? 2 : 1) : 0;
    constexpr int RB = PD + 1;  // ring of record slots (compile-time indices: registers, not scratch)
    uint4 rb[RB][MT][3];
    auto rd = [&](auto IC) {
        constexpr int i = decltype(IC)::value;
        if constexpr (i < NS) {
            const uint32_t* rec = wl + ((i / GT_SB) * SL + s) * RSTR + (i % GT_SB) * MT * 12;
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int x = 0; x < 3; ++x) rb[i % RB][m][x] = *reinterpret_cast<const uint4*>(rec + m * 12 + 4 * x);
        }
    };
    static_for<PD>([&](auto IC) { rd(IC); });
    __builtin_amdgcn_sched_barrier(0);
    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;
    static_for<NS>([&](auto IC) {
        constexpr int i = decltype(IC)::value, j = i / GT_SB, b = i % GT_SB;
        rd(ic<i + PD>{});
        const int h = h0 + j * SL + s;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            if (m < M) {
                const uint4 a[3] = {rb[i % RB][m][0], rb[i % RB][m][1], rb[i % RB][m][2]};
                const uint32_t d = block_dot_t<F, b, GT_SB>(wu[j], a);
                const int gb = h * GT_SB + b;
                if constexpr (SUMI) {
                    if (n < N && h < H && gb < nb) static_cast<int32_t*>(out)[((long)m * N + n) * nb + gb] = (int)(d - ACC_BIAS);
                } else {
                    const float t = block_term_t<F, b, GT_SB>(wu[j], d, a[2]);
                    if (h < H) acc[m] += t;
                }
            }
        }
    });
    if constexpr (!SUMI) {
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = group_sum_last<SL>(acc[m]);
        const bool last = s == SL - 1;
        if (W == 1) {
            if (last && n < N) {
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    if (m < M) static_cast<float*>(out)[(long)m * ldc_m + (long)n * ldc_n] = acc[m];
            }
            return;
        }
        // the waves' partials in fixed wave order (a region past every wave's records)
        float* red = reinterpret_cast<float*>(lds + W * (NU * SL) * RSTR);
        if (last) {
#pragma unroll
            for (int m = 0; m < MT; ++m) red[(m * W + wave) * R + r] = acc[m];
        }
        __syncthreads();
        const int tid = threadIdx.x;
        if (tid < R * MT) {
            const int m = tid / R, rw = tid % R, nn = tile * R + rw;
            if (m < M && nn < N) {
                float v = red[m * W * R + rw];
                for (int w = 1; w < W; ++w) v += red[(m * W + w) * R + rw];
                static_cast<float*>(out)[(long)m * ldc_m + (long)nn * ldc_n] = v;
            }
        }
    }
}

// Rows per wave and stages per lane (profiles/r06_tuning/r6g_ab.txt, N = 4096): 8 rows x 8 stages for M <= 2
// up to K = 4096 (M = 1 4.02 -> 3.83 us, M = 2 4.35 -> 4.13; worse at M = 4 and long K), else the half tile x 4
// stages; 1 stage per lane while 8 waves cover the row group's stages, else 2 (K = 14336 8.94 -> 7.76 us
// against 4 per lane; at most 16 waves: K <= 16384).
struct gemvt_shape {
    int R, NU;
};
inline gemvt_shape gemvt_pick(int M, int H) {
    const int R = QG_GEMVT_R ? QG_GEMVT_R : (M <= 2 && H <= 32) ? 8 : 16, SL = 64 / R;
    return {R, QG_GEMVT_NU ? QG_GEMVT_NU : (H + SL - 1) / SL > 8 ? 2 : 1};
}

template <int F, int MT, int R, int NU> hipError_t gemvt_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int SL = 64 / R;
    const int nb = g.K / QK, H = (nb + GT_SB - 1) / GT_SB;
    const int W = (H + NU * SL - 1) / (NU * SL);
    const int grid = (g.N + R - 1) / R;
    const size_t lds = ((size_t)W * NU * SL * (48 * MT + 4) + (size_t)W * R * MT) * 4;
    const bool ta = g.lay == LAY_TILED_ACT;
    if (g.describe) {
        describe_kernel(g, "gemvt F=%d MT=%d R=%d NU=%d W=%d TA=%d grid=%d", F, MT, R, NU, W, (int)ta, grid);
        return hipSuccess;
    }
    if (W > 16) return hipErrorInvalidValue;
    auto k = g.sumi ? (ta ? gemvt_kernel<F, MT, R, NU, true, true> : gemvt_kernel<F, MT, R, NU, true, false>)
                    : (ta ? gemvt_kernel<F, MT, R, NU, false, true> : gemvt_kernel<F, MT, R, NU, false, false>);
    if (lds > 64 * 1024) {
        static std::atomic<unsigned long long> done[4] = {};
        const hipError_t e = set_max_lds_once((const void*)k, 160 * 1024, done[(g.sumi ? 1 : 0) + (ta ? 2 : 0)]);
        if (e != hipSuccess) return e;
    }
    void* o = g.sumi ? (void*)g.sumi : (void*)g.C;
    hipLaunchKernelGGL(k, dim3(grid), dim3(W * 64), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, o,
                       (int)g.ldc_m, (int)g.ldc_n);
    return hipGetLastError();
}

template <int F, int MT> hipError_t gemvt_m(const GemmArgs& g, hipStream_t st) {
    const gemvt_shape p = gemvt_pick(g.M, (g.K / QK + GT_SB - 1) / GT_SB);
    if (p.R == 8) return p.NU == 1 ? gemvt_launch<F, MT, 8, 1>(g, st) : gemvt_launch<F, MT, 8, 2>(g, st);
    return p.NU == 1 ? gemvt_launch<F, MT, 16, 1>(g, st) : gemvt_launch<F, MT, 16, 2>(g, st);
}

template <int F> hipError_t gemvt_f(const GemmArgs& g, hipStream_t st) {
    switch (g.M) {
        case 1: return gemvt_m<F, 1>(g, st);
        case 2: return gemvt_m<F, 2>(g, st);
        default: return gemvt_m<F, 4>(g, st);
    }
}

}  // namespace

// M <= 4, one product with 32-bit output strides; B_tiled 16-B aligned, A 4-B aligned; at most 16 waves
// per workgroup (K/32 <= 16 waves x 4 stage lanes x 2 stages x 4 blocks: K <= 16384). Beyond, run_tiled takes
// the MFMA kernel.
bool gemvt_eligible(const GemmArgs& g) {
    if (!(g.lay == LAY_TILED || g.lay == LAY_TILED_ACT) || g.M < 1 || g.M > 4 || g.N < 1 || g.K % QK != 0) return false;
    if (g.batch != 1 || g.group || g.ain != AIN_Q8_1 || ((uintptr_t)g.B & 15) != 0 || ((uintptr_t)g.A & 3) != 0) return false;
    if (g.ldc_m > INT32_MAX || g.ldc_n > INT32_MAX || g.ldc_m < 0 || g.ldc_n < 0) return false;
    if (!(g.wtype == FMT_Q4_0 || g.wtype == FMT_Q4_1 || g.wtype == FMT_Q5_0 || g.wtype == FMT_Q5_1 || g.wtype == FMT_Q8_0))
        return false;
    const int H = (g.K / QK + GT_SB - 1) / GT_SB;
    const gemvt_shape p = gemvt_pick(g.M, H);
    const int SL = 64 / p.R;
    return (H + p.NU * SL - 1) / (p.NU * SL) <= 16 && (long)g.M * g.N * (g.K / QK) < (1L << 62);
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
