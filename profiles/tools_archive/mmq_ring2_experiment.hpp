// mmq_ring2_experiment.hpp (round 3, NOT in the product: measured slower, profiles/r03_tuning/README.md) — the M <= 32 prefill as a loader / consumer LDS-DMA ring (VERDICT r02 next #2;
// MI355X_MICROARCH.md "ring-gemm").
//
// Same contract and arithmetic as qg_mmq_kernel.hpp (v_mfma_i32_16x16x32_i8 per Q-block on the stored
// codes, accumulator seeded with the bits of 1.5*2^23, MFMA-assisted EPI2 scale epilogue: per block
// one v_mfma_f32_16x16x16_f16 outer product d_w (x) d_a, per 4 blocks one compensation MFMA), a
// different schedule. A workgroup owns 32 weight rows x 16 tokens x all of K (M = 32, N = 4096:
// 128 x 2 = 256 workgroups, one per CU, a row tile's two token tiles on one XCD) and splits roles:
//  * L loader waves stream the K stages (8 Q-blocks each: 32 row segments of 8*bb bytes + 16 token
//    segments of 288 B, 16-B LDS-DMA pieces, no VGPR staging) into an LDS ring of NS slots, stage h
//    by loader h % L, up to D of a loader's stages in flight; a stage is published by one FULL word
//    per stage in LDS, written after the counted vmcnt that says its DMA landed;
//  * 2*PH consumer waves (the two 16-row halves of the tile x PH fixed K phases: consumer (i, p)
//    takes stages p, p + PH, ...) wait on FULL, read their operand fragments, release the slot by an
//    LDS atomic on its FREE word (a loader refills a slot once both halves released it), then run
//    the MFMAs and the epilogue.
// No workgroup barrier between the first and the last: a consumer computes whatever stage of its
// phase has landed, so no wave waits on DMA that another wave issued late (the product kernel's
// per-wave stage streams left a workgroup's waves finishing up to 2 us apart,
// profiles/r01_tuning/mmq_timeline_r01e.txt). Deterministic: fixed stage sets per consumer, partial
// tiles summed in phase order at the end. Flag traffic is inline-asm LDS ops: an LDS access the
// compiler sees makes it wait for every LDS-DMA in flight (vmcnt(0)).
#pragma once
#include "qg_mmq_kernel.hpp"

namespace qg {

template <int F, int L, int PH, int NS> struct mmqr_geom {
    using T = wfmt<F>;
    static constexpr int SB = 8;                     // blocks per stage
    static constexpr int BN = 32, NTOK = 16;
    static constexpr int RSB = SB * T::BB;           // row segment bytes per stage (16-B multiple)
    static constexpr int PPR = RSB / 16;
    static constexpr int WPC = BN * PPR;             // weight pieces per stage
    static constexpr int APT = SB * Q8_1_BYTES / 16; // 18 pieces per token
    static constexpr int APC = NTOK * APT;
    static constexpr int NI = (WPC + APC + 63) / 64; // DMA instructions per stage
    static constexpr int SLOT = NI * 64 * 16;
    static constexpr int OFF_A = WPC * 16;
    static constexpr int NC = 2 * PH;                // consumer waves
    static constexpr int W = L + NC;
    static constexpr int HMAX = 256;                 // stages (K <= 65536)
    static constexpr int OFF_FLAGS = NS * SLOT;      // FULL[HMAX], FREE[NS]
    static constexpr int OFF_RED = OFF_FLAGS + (HMAX + NS) * 4;
    static constexpr int LDS = OFF_RED + NC * 64 * 16;
    static_assert(RSB % 16 == 0, "16-B row segments");
    static_assert(LDS <= 160 * 1024, "LDS per workgroup");
    static_assert(NS % L == 0, "a loader refills only its own stages' slots");
};

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ uint32_t lds_ld(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return v;
}
__device__ __forceinline__ void lds_st(uint32_t a, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_inc(uint32_t a) {
    asm volatile("ds_add_u32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(1u) : "memory");
}

template <int NI> __device__ __forceinline__ void ring_wait(int younger) {
    if (younger <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NI) : "memory");
}

template <int F, int L, int PH, int NS, int D, bool SUMI, int ABL = 0>
__global__ __launch_bounds__((L + 2 * PH) * 64, 1) void mmqr_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                                     int M, int N, int K, void* __restrict__ out, int ldc_m,
                                                                     int ldc_n) {
    using G = mmqr_geom<F, L, PH, NS>;
    using T = wfmt<F>;
    static_assert(D >= 1 && D <= 4 && D <= NS / L, "loader depth within its slots");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * G::BN, m0 = blockIdx.y * G::NTOK;
    const int nb = K / QK, H = nb / G::SB;
    const long RB = (long)nb * T::BB, AB = (long)nb * Q8_1_BYTES;
    uint32_t* full = reinterpret_cast<uint32_t*>(smem + G::OFF_FLAGS);
    uint32_t* freew = full + G::HMAX;
    for (int i = threadIdx.x; i < G::HMAX + NS; i += G::W * 64) full[i] = 0u;
    __syncthreads();

    if (wave >= G::NC) {
        // ------------------------------------------------------------------ loader wave
        const int l = wave - G::NC;
        const uint8_t* Bw = B + (long)n0 * RB;
        const uint8_t* Aw = A + (long)m0 * AB;
        int coff[G::NI];
        bool isw[G::NI];
#pragma unroll
        for (int i = 0; i < G::NI; ++i) {
            const int p = min(64 * i + lane, G::WPC + G::APC - 1);  // padding lanes refetch the last piece
            isw[i] = p < G::WPC;
            if (isw[i]) {
                const int r = p / G::PPR;
                coff[i] = (min(n0 + r, N - 1) - n0) * (int)RB + (p - r * G::PPR) * 16;
            } else {
                const int pa = p - G::WPC, t = pa / G::APT;
                coff[i] = (min(m0 + t, M - 1) - m0) * (int)AB + (pa - t * G::APT) * 16;
            }
        }
        auto issue = [&](int h) {
            const uint8_t* ws = Bw + (long)h * G::RSB;
            const uint8_t* as = Aw + (long)h * (G::SB * Q8_1_BYTES);
            uint8_t* buf = smem + (h % NS) * G::SLOT;
#pragma unroll
            for (int i = 0; i < G::NI; ++i) glds<16>((isw[i] ? ws : as) + coff[i], buf + 64 * i * 16);
        };
        const int mine = l < H ? (H - 1 - l) / L + 1 : 0;
        int issued = 0;
        for (int pub = 0; pub < mine; ++pub) {
            for (; issued < mine && issued - pub < D; ++issued) {
                const int h = l + issued * L;
                if (h >= NS) {  // slot reuse: both halves of stage h - NS released it
                    const uint32_t fa = lds_addr(freew + h % NS);
                    const uint32_t want = 2u * (uint32_t)(h / NS);
                    while (__builtin_amdgcn_readfirstlane(lds_ld(fa)) < want) __builtin_amdgcn_s_sleep(1);
                }
                issue(h);
            }
            ring_wait<G::NI>(issued - pub - 1);  // stage l + pub * L landed
            if (lane == 0) lds_st(lds_addr(full + l + pub * L), 1u);
        }
    } else {
        // ---------------------------------------------------------------- consumer wave
        const int half = wave & 1, ph = wave >> 1;  // rows 16 half .. +15, stages ph, ph + PH, ...
        const v4i bias = {MMQ_BIAS, MMQ_BIAS, MMQ_BIAS, MMQ_BIAS};
        typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
        typedef float f32x4v __attribute__((ext_vector_type(4)));
        auto h4 = [](unsigned long v) { return __builtin_bit_cast(f16x4, v); };
        constexpr bool HAS_M = T::MOFF >= 0;
        constexpr bool HAS_S = F != FMT_Q8_0;
        constexpr float CFAC = F == FMT_Q4_0 ? -8.0f : F == FMT_Q5_0 ? -16.0f : 1.0f;
        const bool q0 = q == 0;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        f32x4v c2 = {0.f, 0.f, 0.f, 0.f};
        auto u16 = [](const uint8_t* p) { return (uint32_t)*reinterpret_cast<const uint16_t*>(p); };
        auto wfrag = [&](const uint8_t* wr, auto O) -> long {
            constexpr int o = decltype(O)::value;
            uint32_t lo, hi;
            if constexpr (T::Q8) {
                lo = lds32<o + T::QS>(wr + 4 * q);
                hi = lds32<o + T::QS + 16>(wr + 4 * q);
            } else {
                const uint32_t v = lds32<o + T::QS>(wr + 4 * q);
                lo = v & 0x0F0F0F0Fu;
                hi = (v >> 4) & 0x0F0F0F0Fu;
            }
            if constexpr (T::QH >= 0) {
                const uint32_t qh = lds32<o + T::QH>(wr);
                lo |= spread4_bit4((qh >> (4 * q)) & 0xFu);
                hi |= spread4_bit4((qh >> (16 + 4 * q)) & 0xFu);
            }
            return (long)(((unsigned long)hi << 32) | lo);
        };
        for (int h = ph; h < H; h += PH) {
            const uint32_t fa = lds_addr(full + h);
            while (__builtin_amdgcn_readfirstlane(lds_ld(fa)) == 0u) __builtin_amdgcn_s_sleep(1);
            if constexpr (ABL == 1) {  // probe: handshake only
                if (lane == 0) lds_inc(lds_addr(freew + h % NS));
                continue;
            }
            const uint8_t* buf = smem + (h % NS) * G::SLOT;
            const uint8_t* wr = buf + (16 * half + r16) * G::RSB;
            const uint8_t* ar = buf + G::OFF_A + r16 * (G::APT * 16);
            // every LDS read of the stage first (8 blocks), then the slot is released
            long af[8], bf[8];
            uint32_t wdb[8], wmb[8], adb[8];
            static_for<8>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
                constexpr int o = b * T::BB;
                af[b] = wfrag(wr, ic<o>{});
                wdb[b] = u16(wr + o);
                if constexpr (HAS_M) wmb[b] = u16(wr + o + T::MOFF);
                const uint8_t* ab = ar + b * Q8_1_BYTES;
                bf[b] = (long)(((unsigned long)*reinterpret_cast<const uint32_t*>(ab + 20 + 4 * q) << 32) |
                               *reinterpret_cast<const uint32_t*>(ab + 4 + 4 * q));
                adb[b] = *reinterpret_cast<const uint32_t*>(ab);
            });
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) lds_inc(lds_addr(freew + h % NS));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ABL == 2) {  // probe: handshake + operand reads, no MFMA
                uint32_t x = 0;
#pragma unroll
                for (int b = 0; b < 8; ++b) x += (uint32_t)af[b] ^ (uint32_t)bf[b] ^ wdb[b] ^ adb[b];
                acc[0] += (float)(x & 1);
                continue;
            }
            static_for<2>([&](auto HB) {
                constexpr int b0 = 4 * decltype(HB)::value;
                f32x4v dd[4];
                v4i cc[4];
                const f32x4v z4 = {0.f, 0.f, 0.f, 0.f};
                static_for<4>([&](auto BI) {
                    constexpr int b = b0 + decltype(BI)::value;
                    dd[b - b0] = __builtin_amdgcn_mfma_f32_16x16x16f16(h4(q0 ? (unsigned long)(wdb[b] & 0xFFFFu) : 0ul),
                                                                      h4(q0 ? (unsigned long)(adb[b] & 0xFFFFu) : 0ul), z4, 0, 0, 0);
                    cc[b - b0] = __builtin_amdgcn_mfma_i32_16x16x32_i8(af[b], bf[b], bias, 0, 0, 0);
                });
                if constexpr (HAS_S && !SUMI) {
                    const uint32_t* X = HAS_M ? wmb : wdb;
                    const uint32_t x01 = __builtin_amdgcn_perm(X[b0 + 1], X[b0], 0x05040100u);
                    const uint32_t x23 = __builtin_amdgcn_perm(X[b0 + 3], X[b0 + 2], 0x05040100u);
                    const uint32_t s01 = __builtin_amdgcn_perm(adb[b0 + 1], adb[b0], 0x07060302u);
                    const uint32_t s23 = __builtin_amdgcn_perm(adb[b0 + 3], adb[b0 + 2], 0x07060302u);
                    const unsigned long xa = q0 ? (((unsigned long)x23 << 32) | x01) : 0ul;
                    const unsigned long sb = q0 ? (((unsigned long)s23 << 32) | s01) : 0ul;
                    c2 = __builtin_amdgcn_mfma_f32_16x16x16f16(h4(xa), h4(sb), c2, 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (SUMI) {
                    int32_t* so = static_cast<int32_t*>(out);
                    static_for<4>([&](auto BI) {
                        constexpr int b = decltype(BI)::value;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int n = n0 + 16 * half + 4 * q + e, m = m0 + r16;
                            if (n < N && m < M) so[((long)m * N + n) * nb + h * 8 + b0 + b] = cc[b][e] - MMQ_BIAS;
                        }
                    });
                } else {
                    static_for<4>([&](auto BI) {
                        constexpr int b = decltype(BI)::value;
#pragma unroll
                        for (int e = 0; e < 4; e += 2) {
                            const f32x2 sm = f32x2{__int_as_float(cc[b][e]), __int_as_float(cc[b][e + 1])} -
                                             f32x2{MMQ_BIAS_F, MMQ_BIAS_F};  // exact: sumi
                            const f32x2 r = __builtin_elementwise_fma(f32x2{dd[b][e], dd[b][e + 1]}, sm, f32x2{acc[e], acc[e + 1]});
                            acc[e] = r.x;
                            acc[e + 1] = r.y;
                        }
                    });
                }
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        if constexpr (!SUMI) {
            if constexpr (HAS_S) {
                asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // margin: the last compensation MFMA
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(CFAC, c2[e], acc[e]);
            }
            float* red = reinterpret_cast<float*>(smem + G::OFF_RED);
            *reinterpret_cast<f32x4v*>(red + (wave * 64 + lane) * 4) = f32x4v{acc[0], acc[1], acc[2], acc[3]};
        }
    }
    if constexpr (!SUMI) {
        __syncthreads();
        // the PH partial tiles of each half summed in phase order; consumer waves 0 and 1 store
        if (wave < 2) {
            const float* red = reinterpret_cast<const float*>(smem + G::OFF_RED);
            typedef float f32x4v __attribute__((ext_vector_type(4)));
            f32x4v v = *reinterpret_cast<const f32x4v*>(red + (wave * 64 + lane) * 4);
#pragma unroll
            for (int p = 1; p < PH; ++p) v += *reinterpret_cast<const f32x4v*>(red + ((2 * p + wave) * 64 + lane) * 4);
            float* C = static_cast<float*>(out);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int n = n0 + 16 * wave + 4 * q + e, m = m0 + r16;
                if (n < N && m < M) C[(long)m * ldc_m + (long)n * ldc_n] = v[e];
            }
        }
    }
}

template <int F, int L, int PH, int NS> inline bool mmqr_shape_ok(const GemmArgs& g) {
    using G = mmqr_geom<F, L, PH, NS>;
    if (g.M < 1 || g.N < 1 || g.K % (QK * G::SB) != 0 || g.K / QK / G::SB > G::HMAX) return false;
    const long RB = (long)(g.K / QK) * wfmt<F>::BB, AB = (long)(g.K / QK) * Q8_1_BYTES;
    if (((uintptr_t)g.A & 15) != 0 || ((uintptr_t)g.B & 15) != 0 || RB % 16 != 0 || AB % 16 != 0) return false;
    if (RB * G::BN >= (1L << 31) || AB * G::NTOK >= (1L << 31)) return false;
    if (g.ldc_m > INT32_MAX || g.ldc_n > INT32_MAX) return false;
    return true;
}

template <int F, int L, int PH, int NS, int D, bool SUMI, int ABL = 0> hipError_t mmqr_launch(const GemmArgs& g, hipStream_t st) {
    using G = mmqr_geom<F, L, PH, NS>;
    const dim3 grid((g.N + G::BN - 1) / G::BN, (g.M + G::NTOK - 1) / G::NTOK);
    if (g.describe) {
        describe_kernel(g, "mmqr F=%d L=%d PH=%d NS=%d D=%d grid=%ux%u", F, L, PH, NS, D, grid.x, grid.y);
        return hipSuccess;
    }
    auto k = mmqr_kernel<F, L, PH, NS, D, SUMI, ABL>;
    static std::atomic<unsigned long long> attr_done{0};
    const hipError_t e = set_max_lds_once((const void*)k, G::LDS, attr_done);
    if (e != hipSuccess) return e;
    void* out = SUMI ? (void*)g.sumi : (void*)g.C;
    hipLaunchKernelGGL(k, grid, dim3(G::W * 64), G::LDS, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, out,
                       (int)g.ldc_m, (int)g.ldc_n);
    return hipGetLastError();
}

}  // namespace qg
