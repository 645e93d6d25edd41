// mmq_ring_experiment.hpp — (probe only, not product) W4A8 prefill GEMM, cooperative LDS-DMA ring (round 2).
//
// C[M,N] = A_q8_1[M,K] . B_w[N,K]^T (include/gemm_reference.h:175-222), activation-major; the same
// arithmetic as qg_mmq_kernel.hpp (one v_mfma_i32_16x16x32_i8 per Q-block = exact int32 sumi of
// 16 weight rows x 16 tokens, MFMA-assisted scale epilogue), with a different data movement.
//
// Why: at M = 32 the per-wave stage stream of qg_mmq_kernel.hpp
// (each wave DMAs its own 4-block stages: 72-B row segments, 13 rows per DMA instruction) moves the
// workgroup's 147 KB at ~33 GB/s per CU, and the waves finish up to 2 us apart. Here the whole
// workgroup fills ONE stage of SB blocks together (SB = 16: 288-B row segments for Q4_0, 16-B
// aligned for every format, 3-4 rows per DMA instruction) into a ring of NS slots, each wave issuing
// an equal share of the stage's DMA instructions; a raw s_barrier per stage (no __syncthreads: its
// fence would drain every DMA in flight) publishes the slot, and every wave then computes SB / W
// blocks of it for the whole BN x 16*TT tile. Per stage every wave does the same work, so no wave
// trails the others by a whole stage at the end.
//
// Slot layout (lane-linear DMA images, 16-B pieces): [BN rows][RIMG] weights, then
// [16*TT tokens][AIMG] activations; RIMG / AIMG carry one pad piece per row / token (a duplicate
// fetch of the row's first piece) so the 16 rows / tokens of one fragment read hit distinct LDS
// bank groups. Rows / tokens past N / M read the last valid one (results dropped).
//
// Ring protocol per stage s (NS slots, NS - 1 stages in flight):
//   wait own DMAs of stage s (counted vmcnt) -> s_barrier (every wave: stage s landed, stage s-1's
//   reads retired) -> issue stage s + NS - 1 into slot (s - 1) % NS -> compute stage s.
// RAW: DMA data is read only after its issuing wave's vmcnt wait and a barrier the reader passed;
// WAR: a slot is refilled only after the barrier that follows every wave's last read of it (the
// reads' results were consumed before the barrier: s_waitcnt lgkmcnt(0) below).
// End: each wave's partial tile (its SB/W blocks of every stage, in stage order) is summed in fixed
// wave order through LDS: deterministic.
#pragma once
#include "qg_mmq_kernel.hpp"

namespace qg {

template <int F, int BN, int TT, int W, int SB, int NS> struct ring_geom {
    using T = wfmt<F>;
    static_assert(SB % 8 == 0, "stages of whole 8-block groups: 16-B aligned row segments for every format");
    static_assert(SB % W == 0 && (SB / W == 2 || (SB / W) % 4 == 0), "each wave computes 2 or a multiple of 4 of a stage's blocks");
    static_assert(BN % 16 == 0 && BN <= 64 && TT >= 1 && TT <= 2, "row tiles of 16, one or two token tiles");
    static_assert(NS >= 1 && NS <= 5, "ring slots");
    static constexpr int BPW = SB / W;                 // blocks per wave per stage
    static constexpr int GB = BPW < 4 ? BPW : 4;        // blocks per compute group
    static constexpr int RSB = SB * T::BB;              // weight bytes per row per stage
    static constexpr int WPR = RSB / 16;                // weight pieces per row
    static constexpr int WPRP = WPR + 1;                // ... plus the pad piece
    static constexpr int RIMG = WPRP * 16;              // row image stride (bytes)
    static constexpr int ASEG = SB * Q8_1_BYTES;        // activation bytes per token per stage
    static constexpr int APR = ASEG / 16;
    static constexpr int APRP = APR + 1;
    static constexpr int AIMG = APRP * 16;              // token image stride (bytes)
    static constexpr int NTOK = 16 * TT;
    static constexpr int WPC = BN * WPRP;               // weight pieces per stage
    static constexpr int APC = NTOK * APRP;             // activation pieces per stage
    static constexpr int NI = (WPC + APC + 63) / 64;    // DMA instructions per stage
    static constexpr int MAXI = (NI + W - 1) / W;       // per wave (some waves one fewer)
    static constexpr int SLOT = NI * 1024;              // slot bytes (whole instructions)
    static constexpr int OFF_A = WPC * 16;
    static constexpr int RT = BN / 16;
    static constexpr int NACC = RT * TT * 4;            // accumulators per lane
    static constexpr size_t RED = (size_t)W * NACC * 64 * 4;
    static constexpr size_t LDS = (size_t)NS * SLOT > RED ? (size_t)NS * SLOT : RED;
    static_assert(LDS <= 160 * 1024, "LDS per workgroup");
    static_assert(MAXI * (NS > 1 ? NS - 1 : 1) <= 63, "vmcnt range");
    static_assert(RSB % 16 == 0 && ASEG % 16 == 0, "16-B pieces");
};

// OPT (tuning probes; the product uses 0): RING_ROT — workgroup x starts at stage x mod H (the
// grid's workgroups fetch different stages at the same moment); RING_DMA — DMA, waits and barriers
// only, no compute; RING_WONLY / RING_AONLY — only the weight / activation pieces are fetched (the
// other lanes re-fetch the first piece of the stage).
enum : int { RING_ROT = 1, RING_DMA = 2, RING_WONLY = 4, RING_AONLY = 8 };

// s_waitcnt vmcnt(N * k), k in [0, 3] (wave-uniform).
template <int N> __device__ __forceinline__ void ring_wait(int k) {
    if (k <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (k == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    else if (k == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * N) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * N) : "memory");
}

template <int F, int BN, int TT, int W, int SB, int NS, bool SUMI, int OPT = 0>
__global__ __launch_bounds__(W * 64, 1) void mmq_ring_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                             int M, int N, int K, float* __restrict__ C, long ldc_m,
                                                             long ldc_n, int32_t* __restrict__ sumi_out) {
    using G = ring_geom<F, BN, TT, W, SB, NS>;
    using T = wfmt<F>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15;
    const int q = lane >> 4;
    const int n0 = blockIdx.x * BN;
    const int m0 = blockIdx.y * G::NTOK;
    const int nb = K / QK;
    const int H = nb / SB;  // stages
    const long RB = (long)nb * T::BB;
    const long AB = (long)nb * Q8_1_BYTES;
    // 64-bit workgroup bases (tensors beyond 2 GiB), 32-bit per-lane offsets below BN * RB
    const uint8_t* Bw = B + (long)n0 * RB;
    const uint8_t* Aw = A + (long)m0 * AB;

    // this wave's DMA instructions of a stage: i = wave + j W, j < niw
    const int niw = (G::NI - wave + W - 1) / W;
    int coff[G::MAXI];
    bool cisw[G::MAXI];
#pragma unroll
    for (int j = 0; j < G::MAXI; ++j) {
        const int p = min(64 * (wave + j * W) + lane, G::WPC + G::APC - 1);
        cisw[j] = p < G::WPC;
        if constexpr ((OPT & RING_WONLY) != 0) if (!cisw[j]) { cisw[j] = true; coff[j] = 0; continue; }
        if constexpr ((OPT & RING_AONLY) != 0) if (cisw[j]) { cisw[j] = false; coff[j] = 0; continue; }
        if (cisw[j]) {
            const int row = p / G::WPRP, k = p - row * G::WPRP;
            coff[j] = (min(n0 + row, N - 1) - n0) * (int)RB + (k < G::WPR ? k : 0) * 16;
        } else {
            const int pa = p - G::WPC;
            const int tok = pa / G::APRP, k = pa - tok * G::APRP;
            coff[j] = (min(m0 + tok, M - 1) - m0) * (int)AB + (k < G::APR ? k : 0) * 16;
        }
    }
    auto issue = [&](int h, uint8_t* slot) {
        const uint8_t* wsrc = Bw + (long)h * G::RSB;
        const uint8_t* asrc = Aw + (long)h * G::ASEG;
#pragma unroll
        for (int j = 0; j < G::MAXI; ++j)
            if (j < niw) glds<16>((cisw[j] ? wsrc : asrc) + coff[j], slot + (wave + j * W) * 1024);
    };

    float acc[G::NACC];
#pragma unroll
    for (int i = 0; i < G::NACC; ++i) acc[i] = 0.0f;
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    constexpr bool HAS_M = T::MOFF >= 0;
    constexpr bool HAS_S = F != FMT_Q8_0;
    constexpr float CFAC = F == FMT_Q4_0 ? -8.0f : F == FMT_Q5_0 ? -16.0f : 1.0f;
    f32x4v c2[G::RT][TT];
#pragma unroll
    for (int i = 0; i < G::RT; ++i)
#pragma unroll
        for (int t = 0; t < TT; ++t) c2[i][t] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const v4i bias = {MMQ_BIAS, MMQ_BIAS, MMQ_BIAS, MMQ_BIAS};
    const f32x4v z4 = {0.f, 0.f, 0.f, 0.f};
    const bool q0 = q == 0;
    auto h4 = [](unsigned long v) { return __builtin_bit_cast(f16x4, v); };
    auto u16 = [](const uint8_t* p) { return (uint32_t)*reinterpret_cast<const uint16_t*>(p); };

    // this wave's blocks of a stage: bw0 .. bw0 + BPW - 1 (bw0 even, so every block's byte offset
    // parity -- hence the qs dword alignment -- is a compile-time property of its index j)
    const int bw0 = wave * G::BPW;
    auto group = [&](const uint8_t* slot, int h, int gb) {
        const uint8_t* wimg = slot + (bw0 + gb) * T::BB;
        const uint8_t* aimg = slot + G::OFF_A + (bw0 + gb) * Q8_1_BYTES;
        long afrag[G::GB][G::RT], bfrag[G::GB][TT];
        uint32_t wdb[G::GB][G::RT], wmb[G::GB][G::RT], adb[G::GB][TT];
        static_for<G::GB>([&](auto J) {
            constexpr int j = decltype(J)::value;
            constexpr int o = j * T::BB;
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                const uint8_t* wr = wimg + (16 * i + r16) * G::RIMG;
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
                afrag[j][i] = (long)(((unsigned long)hi << 32) | lo);
                wdb[j][i] = u16(wr + o);
                if constexpr (HAS_M) wmb[j][i] = u16(wr + o + T::MOFF);
            }
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                const uint8_t* ar = aimg + (16 * t + r16) * G::AIMG + j * Q8_1_BYTES;
                const uint32_t qa0 = *reinterpret_cast<const uint32_t*>(ar + 4 + 4 * q);
                const uint32_t qa1 = *reinterpret_cast<const uint32_t*>(ar + 20 + 4 * q);
                bfrag[j][t] = (long)(((unsigned long)qa1 << 32) | qa0);
                adb[j][t] = *reinterpret_cast<const uint32_t*>(ar);  // f16 d_a | f16 s_a << 16
            }
        });
        __builtin_amdgcn_sched_barrier(0);
        v4i cc[G::GB][G::RT][TT];
        f32x4v dd[G::GB][G::RT][TT];
        static_for<G::GB>([&](auto J) {
            constexpr int j = decltype(J)::value;
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
                    cc[j][i][t] = __builtin_amdgcn_mfma_i32_16x16x32_i8(afrag[j][i], bfrag[j][t], bias, 0, 0, 0);
            if constexpr (!SUMI) {
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t)  // d_w (x) d_a: k-slot 0 only (lanes q = 0)
                        dd[j][i][t] = __builtin_amdgcn_mfma_f32_16x16x16f16(
                            h4(q0 ? (unsigned long)wdb[j][i] : 0ul), h4(q0 ? (unsigned long)(adb[j][t] & 0xFFFFu) : 0ul), z4, 0,
                            0, 0);
            }
        });
        if constexpr (HAS_S && !SUMI) {
            // compensation sum_b X s_a: k-slots 0 .. BPW-1 = this wave's blocks (lanes q = 0)
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                const auto& X = HAS_M ? wmb : wdb;
                const uint32_t x01 = __builtin_amdgcn_perm(X[1][i], X[0][i], 0x05040100u);
                const uint32_t x23 = G::GB == 4 ? __builtin_amdgcn_perm(X[G::GB - 1][i], X[G::GB / 2][i], 0x05040100u) : 0u;
                const unsigned long xa = q0 ? (((unsigned long)x23 << 32) | x01) : 0ul;
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const uint32_t s01 = __builtin_amdgcn_perm(adb[1][t], adb[0][t], 0x07060302u);
                    const uint32_t s23 = G::GB == 4 ? __builtin_amdgcn_perm(adb[G::GB - 1][t], adb[G::GB / 2][t], 0x07060302u) : 0u;
                    const unsigned long sb = q0 ? (((unsigned long)s23 << 32) | s01) : 0ul;
                    c2[i][t] = __builtin_amdgcn_mfma_f32_16x16x16f16(h4(xa), h4(sb), c2[i][t], 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SUMI) {
            static_for<G::GB>([&](auto J) {
                constexpr int j = decltype(J)::value;
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int n = n0 + 16 * i + 4 * q + e, m = m0 + 16 * t + r16;
                            if (n < N && m < M) sumi_out[((long)m * N + n) * nb + h * SB + bw0 + gb + j] = cc[j][i][t][e] - MMQ_BIAS;
                        }
            });
            return;
        }
        static_for<G::GB>([&](auto J) {
            constexpr int j = decltype(J)::value;
#pragma unroll
            for (int i = 0; i < G::RT; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int e = 0; e < 4; e += 2) {
                        const f32x2 sm = f32x2{__int_as_float(cc[j][i][t][e]), __int_as_float(cc[j][i][t][e + 1])} -
                                         f32x2{MMQ_BIAS_F, MMQ_BIAS_F};  // exact: sumi
                        float* a = &acc[(i * TT + t) * 4 + e];
                        const f32x2 r = __builtin_elementwise_fma(f32x2{dd[j][i][t][e], dd[j][i][t][e + 1]}, sm, f32x2{a[0], a[1]});
                        a[0] = r.x;
                        a[1] = r.y;
                    }
        });
        __builtin_amdgcn_sched_barrier(0);
    };
    auto compute = [&](const uint8_t* slot, int h) {
        for (int gb = 0; gb < G::BPW; gb += G::GB) group(slot, h, gb);
    };

    // ring: NS - 1 stages in flight
    const int rot = (OPT & RING_ROT) ? (int)(blockIdx.x % H) : 0;
    auto stg = [&](int k) { return k + rot < H ? k + rot : k + rot - H; };
#pragma unroll
    for (int k = 0; k < (NS > 1 ? NS - 1 : 1); ++k)
        if (k < H) issue(stg(k), smem + k * G::SLOT);
    for (int s = 0; s < H; ++s) {
        const int younger = NS > 1 ? min(NS - 2, H - 1 - s) : 0;
        if (niw == G::MAXI) ring_wait<G::MAXI>(younger);
        else ring_wait<(G::MAXI > 1 ? G::MAXI - 1 : 1)>(niw == 0 ? 0 : younger);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if constexpr (NS > 1) {
            if (s + NS - 1 < H) issue(stg(s + NS - 1), smem + ((s + NS - 1) % NS) * G::SLOT);
            if constexpr ((OPT & RING_DMA) == 0) compute(smem + (s % NS) * G::SLOT, stg(s));
        } else {  // one slot: the next stage is fetched after every wave has computed this one
            if constexpr ((OPT & RING_DMA) == 0) compute(smem, stg(s));
            if (s + 1 < H) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                issue(stg(s + 1), smem);
            }
        }
    }

    if constexpr (!SUMI) {
        if constexpr (HAS_S) {
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // margin behind the last compensation MFMAs
#pragma unroll
            for (int i = 0; i < G::RT; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        acc[(i * TT + t) * 4 + e] = __builtin_fmaf(CFAC, c2[i][t][e], acc[(i * TT + t) * 4 + e]);
        }
        // fixed-order sum of the W partial tiles through LDS (every DMA has landed: the last
        // iteration waited with vmcnt(0))
        float* red = reinterpret_cast<float*>(smem);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int i = 0; i < G::NACC; ++i) red[(wave * G::NACC + i) * 64 + lane] = acc[i];
        __syncthreads();
        constexpr int TS = G::NACC * 64;  // outputs per tile = BN * NTOK
        const bool nfast = ldc_n == 1;    // consecutive threads along the contiguous output index
        for (int idx = threadIdx.x; idx < TS; idx += W * 64) {
            const int nl = nfast ? idx % BN : idx / G::NTOK;
            const int ml = nfast ? idx / BN : idx % G::NTOK;
            const int i = nl >> 4, qq = (nl >> 2) & 3, e = nl & 3, t = ml >> 4, c = ml & 15;
            const int src = ((i * TT + t) * 4 + e) * 64 + qq * 16 + c;
            float v = red[src];
#pragma unroll
            for (int ww = 1; ww < W; ++ww) v += red[ww * TS + src];
            const int n = n0 + nl, m = m0 + ml;
            if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v;
        }
    }
}

// Preconditions: K a multiple of 32 * SB, 16-B aligned A, B and row strides (whole 16-B pieces),
// one workgroup's rows / tokens within 2 GiB of its 64-bit base.
template <int F, int BN, int TT, int W, int SB, int NS> inline bool ring_shape_ok(const GemmArgs& g) {
    if (g.M < 1 || g.N < 1 || g.K % (QK * SB) != 0 || g.batch != 1) return false;
    const long RB = (long)(g.K / QK) * wfmt<F>::BB, AB = (long)(g.K / QK) * Q8_1_BYTES;
    if (((uintptr_t)g.A & 15) != 0 || ((uintptr_t)g.B & 15) != 0 || RB % 16 != 0 || AB % 16 != 0) return false;
    if (RB * BN >= (1L << 31) || AB * 16 * TT >= (1L << 31)) return false;
    if ((g.M + 16 * TT - 1) / (16 * TT) > 65535) return false;
    return true;
}

template <int F, int BN, int TT, int W, int SB, int NS, bool SUMI, int OPT = 0>
hipError_t ring_launch(const GemmArgs& g, hipStream_t st) {
    using G = ring_geom<F, BN, TT, W, SB, NS>;
    const dim3 grid((g.N + BN - 1) / BN, (g.M + G::NTOK - 1) / G::NTOK);
    auto k = mmq_ring_kernel<F, BN, TT, W, SB, NS, SUMI, OPT>;
    if (g.describe) {  // qg_debug_config: name the instantiation instead of launching it
        describe_kernel(g, "mmq_ring F=%d BN=%d TT=%d W=%d SB=%d NS=%d grid=%ux%u", F, BN, TT, W, SB, NS, grid.x, grid.y);
        return hipSuccess;
    }
    if (G::LDS > 64 * 1024) {
        static bool attr_set = false;  // once per instantiation (not a stream op: capture-safe)
        if (!attr_set) {
            hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
            if (e != hipSuccess) return e;
            attr_set = true;
        }
    }
    hipLaunchKernelGGL(k, grid, dim3(W * 64), G::LDS, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, g.C,
                       g.ldc_m, g.ldc_n, g.sumi);
    return hipGetLastError();
}

}  // namespace qg
