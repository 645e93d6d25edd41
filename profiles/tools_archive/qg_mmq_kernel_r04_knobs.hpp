// qg_mmq_kernel.hpp — W4A8 prefill GEMM (M > 8) on the CDNA4 matrix cores, v_mfma_i32_16x16x32_i8.
//
// C[M,N] = A_q8_1[M,K] . B_w[N,K]^T (include/gemm_reference.h:175-222), activation-major.
//
// One MFMA = one Q-block: v_mfma_i32_16x16x32_i8 has K = 32, so each MFMA returns the exact int32
// sumi of 16 (weight row n) x 16 (token m) pairs for one block. The per-block epilogue runs on the
// VALU and is the kernel's real arithmetic cost at prefill sizes (one per (n, m, block)), so it is
// cut to 3 ops per element: the accumulator is seeded with the bit pattern of 1.5*2^23, so the
// MFMA's integer add leaves cf = 12582912.0f + sumi as a float (|sumi| < 2^22, no v_cvt_f32_i32);
// fma(d_a, cf, -d_a*1.5*2^23) = round(d_a * sumi), bit-identical to the reference's d_a * fs (the
// constant is exact in f32); minus 8 s_a (Q4_0) as in the reference; one fma into the accumulator
// (inside the summation-order bound of the parity tests).
//
// Operand k-order: lane (r = lane&15, q = lane>>4) supplies, for its weight row / token r, the 8
// bytes of k-slot q: elements 4q..4q+3 and 16+4q..16+4q+3 of the block. For the weights that is qs
// dword q split into low / high nibbles (+ the qh bits for Q5_x), for Q8_0 its signed qs dwords q and
// 4+q; for the activations qs dwords q and 4+q. A and B use the same slot -> element map and the
// integer sum is order-free. Q8_0 (W8A8) runs the Q4_0 epilogue with no s_a term.
// C layout (gfx950, dtype-independent): lane holds column m = lane&15, rows n = 4q + e (e < 4), so
// the token's scales are per-lane scalars and the 4 row scales are 4 fp16 reads of the staged rows.
//
// Tiling: a workgroup owns BN weight rows x 16*TT tokens and ALL of K; its W waves
// split K into 128-element stages (4 blocks), wave w taking stages w, w+W, ... With BN = 32,
// TT = 1 the M = 32, N = 4096 prefill is 256 workgroups, one per CU. Each wave streams its stages
// with LDS-DMA (global_load_lds: no VGPR staging, lane-linear LDS images [row][4 blocks] and
// [token][144 B]) into two wave-private LDS buffers, the next stage in flight while the current one
// computes (counted vmcnt). No workgroup barrier in the main loop; the W partial tiles are summed
// in fixed wave order through LDS at the end.
//
// A stage runs in three phases (all LDS reads, all MFMAs, all epilogues) so that each phase's
// latencies overlap. MFMA results -> VALU: gfx950 needs 8 wait states after v_mfma_i32_16x16x32_i8
// and v_mfma_f32_16x16x16_f16 (tools/mfma_hazard_probe.hip on an MI355X: every lane wrong at <= 6
// states, right from 8; profiles/r02_tuning/mfma_hazard_probe.txt) and hipcc pads exactly 8
// (`s_nop 7`); tests/test_isa_hazards.py checks every MFMA of the shipped code object for it. The
// `s_nop 7; s_nop 7` after each MFMA phase below is a margin on top (the round-1 wrong sums that
// first prompted it came from an MFMA result element read through a bit_cast, mmq_probe1-2.txt).
// Only LDS reads in the main loop: an LDS write there makes hipcc wait for every DMA in flight.
#pragma once
#include "qg_common.hpp"
#include "qg_kernels.hpp"

namespace qg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// fma(f16 value in the low half of h, x, c) with one rounding (v_fma_mix_f32).
__device__ __forceinline__ float fma_mix_lo(uint32_t h, float x, float c) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(x), "v"(c));
    return r;
}

constexpr int MMQ_BIAS = 0x4B400000;  // bits of 12582912.0f = 1.5 * 2^23
constexpr float MMQ_BIAS_F = 12582912.0f;
constexpr int MMQ_SB = 4;             // blocks per compute sub-stage (a DMA stage holds SB = 4 or 8)

#ifdef QG_MMQ_STAMPS
// diagnostic build only (profiles/tools_archive/mmq_timeline.hip): per-wave s_memrealtime stamps
__device__ unsigned long long g_mmq_stamps[8 * 65536];
#define MMQ_STAMP(k) stamps[k] = __builtin_amdgcn_s_memrealtime()
#else
#define MMQ_STAMP(k)
#endif

// 32 bits at byte offset (compile-time OFF) of an LDS row, from aligned dword reads.
template <int OFF> __device__ __forceinline__ uint32_t lds32(const uint8_t* base) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(base + (OFF & ~3));
    if constexpr (OFF % 4 == 0) return p[0];
    else return __builtin_amdgcn_alignbyte(p[1], p[0], OFF % 4);
}

// One LDS-DMA instruction: lane's SZ bytes at g -> LDS at (wave-uniform) l + lane * SZ. A __device__
// function: called straight from a lambda inside the kernel, the builtin made the host pass drop
// the kernel's launch stub without a diagnostic (undefined symbol at link time).
template <int SZ> __device__ __forceinline__ void glds(const uint8_t* g, uint8_t* l) {
    auto gp = (const __attribute__((address_space(1))) void*)g;
    auto lp = (__attribute__((address_space(3))) void*)l;
    static_assert(SZ == 4 || SZ == 12 || SZ == 16, "global_load_lds sizes");
    if constexpr (SZ == 16) __builtin_amdgcn_global_load_lds(gp, lp, 16, 0, 0);
    else if constexpr (SZ == 12) __builtin_amdgcn_global_load_lds(gp, lp, 12, 0, 0);
    else __builtin_amdgcn_global_load_lds(gp, lp, 4, 0, 0);
}

// P16: weights DMA'd in 16-B pieces (16-B aligned B and rows; else 4-B pieces). A
// stage's row segment (RSB = 4 * BB bytes) then starts 16-B aligned or 8 bytes past (RSB % 16 == 8
// for Q4_0 / Q5_0 / Q8_0, alternating with the stage parity): each row image is a 16-B aligned
// window of RIMG bytes and the data sits SHIFT(h) = (h * RSB) % 16 bytes into it. With K % 256 == 0
// the stage count is even, so the last stage is an odd one (shift 8) and no window reaches past
// the end of the weight rows.
// NB: stage buffers per wave (the wave keeps up to NB stages in flight; at M = 32, K = 4096 each
// wave owns 4 stages, so NB = 4 issues all of its data at once — the kernel was latency-bound with
// one stage in flight ahead of the one being computed).
// With 16-B weight pieces the weight and activation pieces of a stage share one piece numbering
// (p < WPC: weights, then activations), so only the last DMA instruction carries padding.
// SB: blocks per stage (4 or 8). With 8, every format's stage segment is a 16-B multiple (no
// shifted windows) and each token's activation segment is 288 B (+16 B pad against 2-way LDS bank
// conflicts).
// OPT bit flags (tuning; see mmq_opt below): MMQ_CONTIG — each wave owns a contiguous range of
// K stages (its consecutive stages are adjacent bytes of every row, fetched back to back), instead
// of stages w, w + W, ...; MMQ_ZL — lanes that must feed zeros into the scale MFMAs (k-slots 1..15)
// read their scales from a zeroed per-wave LDS region instead of selecting zeros in VALU.
// MMQ_DYN — stages handed out dynamically: each wave starts with stages w and w + W, then takes the
// next unclaimed stage from an LDS counter after every stage it computes, so waves whose DMA lands
// late take fewer stages (the round-1 timeline had the workgroup's waves finish up to 2 us apart,
// profiles/r01_tuning/mmq_timeline_r01e.txt). Each stage's partial tile goes to its own LDS slot and
// the slots are summed in stage order at the end: bit-identical whichever wave took which stage.
// A tuning option (QG_MMQ_DYN, qg_gemm_mfma.hip): measured slower, off in the product.
// MMQ_EARLY — the refill of a consumed stage buffer (the DMA of the wave's stage k + NB) is issued as
// soon as the buffer's operand reads have returned, before the stage's MFMAs and epilogue, instead of
// after them: the next DMA's latency starts one compute phase earlier (round 4).
// MMQ_RAW — the EPI2 stage's weight fragments are read as raw dwords first (every LDS read of the stage
// in one batch, one lgkmcnt wait) and realigned / split into nibbles afterwards; without it hipcc
// interleaves the realignment with the reads and waits for the LDS twice per stage (round 4).
enum : int { MMQ_CONTIG = 1, MMQ_ZL = 2, MMQ_DYN = 4, MMQ_EARLY = 8, MMQ_RAW = 16 };
constexpr int MMQ_ZB = 1024;  // bytes of the per-wave zero region (covers every scale offset)

template <int F, int BN, int TT, int W, bool P16 = false, int NB = 2, int SB = 4, int OPT = 0> struct mmq_geom {
    using T = wfmt<F>;
    static_assert(SB == 4 || SB == 8 || SB == 16, "4, 8 or 16 blocks per stage");
    static constexpr int RSB = SB * T::BB;                     // weight bytes per row per stage
    static constexpr int WPS = P16 ? 16 : 4;                   // weight DMA piece (bytes)
    static constexpr int RIMG = P16 && RSB % 16 != 0 ? RSB + 8 : RSB;  // row image bytes
    static constexpr int PPR = RIMG / WPS;                     // pieces per row image
    static constexpr int WPC = BN * PPR;                       // weight pieces per stage
    static constexpr int NTOK = 16 * TT;
    static constexpr int APR = 9 * SB / 4;                     // activation 16-B pieces per token
    static constexpr int APT = SB == 4 ? APR : APR + 1;        // ... incl. the pad piece
    static constexpr int ASTR = APT * 16;                      // token image stride (bytes)
    static constexpr int APC = NTOK * APT;                     // activation 16-B pieces per stage
    static constexpr bool CMB = P16;                           // combined piece numbering
    static constexpr int NWI = CMB ? 0 : (WPC + 63) / 64;      // weight-only DMA instructions
    static constexpr int NAI = CMB ? 0 : (APC + 63) / 64;      // activation-only DMA instructions
    static constexpr int NI = CMB ? (WPC + APC + 63) / 64 : NWI + NAI;  // DMA instructions per stage
    static constexpr int RT = BN / 16;                         // row tiles
    // LDS buffer layout (bytes). Every DMA instruction runs on all 64 lanes (see issue()), so the
    // images are padded to whole instructions.
    static constexpr int OFF_A = CMB ? WPC * 16 : NWI * 64 * WPS;
    static constexpr int BUF = CMB ? NI * 64 * 16 : OFF_A + NAI * 64 * 16;
    static constexpr int NACC = RT * TT * 4;                   // accumulators per lane
    // wave buffers; the end-of-kernel partial tiles reuse them (after a barrier)
    static constexpr size_t LDS0 = (size_t)W * (NB * BUF > NACC * 256 ? NB * BUF : NACC * 256);
    static constexpr size_t ZOFF = LDS0;                                   // per-wave zero regions
    static constexpr size_t LDS = LDS0 + ((OPT & MMQ_ZL) ? (size_t)W * MMQ_ZB : 0);
    // MMQ_DYN: the stage counter (16 B), then one partial tile per stage (dynamic LDS beyond LDS)
    static constexpr size_t SLOT = (size_t)NACC * 64 * 4;
    static size_t dyn_lds(int H) { return (OPT & MMQ_DYN) ? LDS + 16 + (size_t)H * SLOT : LDS; }
    static_assert(NB >= 1 && NB <= 4, "1..4 stage buffers per wave");
    static_assert(LDS <= 160 * 1024, "LDS per workgroup");
    static_assert(OFF_A % 16 == 0 && BUF % 16 == 0, "16-B aligned LDS regions");
    static_assert(RSB % 8 == 0, "stage segments are 8-B multiples");
    static_assert(NB * NI <= 63, "vmcnt range");
    __host__ __device__ static constexpr int shift(int h) { return P16 ? (h * RSB) & 15 : 0; }
};

// s_waitcnt vmcnt(younger * NI): the oldest stage's DMA landed, `younger` later stages may still fly.
template <int NI> __device__ __forceinline__ void wait_stage(int younger) {
    if (younger <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NI) : "memory");
}

// ABL (tuning probes only; the product uses 0): 1 = the DMA stream and waits without any compute,
// 2 = operand reads + MFMAs without the VALU epilogue, 3 / 4 = as 1 with only the activation /
// only the weight pieces fetched (the other lanes re-read a line already in flight).
// KS > 1: split-K across workgroups — blockIdx.z = slice of H / KS consecutive stages; each slice's
// fixed-order partial tile goes to the workspace and the last slice to finish (agent-scope counter
// per output tile) sums the KS partials in slice order (deterministic: the same order whichever
// workgroup arrives last) and re-arms the counter to 0 for the next launch.
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB, int ABL, bool ROT, int SB, int KS, bool EPI2, int OPT>
__device__ __forceinline__ void mmq_body(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B, float* __restrict__ C,
                                         int32_t* __restrict__ sumi_out, int M, int N, int K, long ldc_m, long ldc_n,
                                         float* __restrict__ part, unsigned* __restrict__ cnt) {
    using G = mmq_geom<F, BN, TT, W, P16, NB, SB, OPT>;
    using T = wfmt<F>;
    constexpr bool ZL = (OPT & MMQ_ZL) != 0 && EPI2;
    static_assert(BN % 16 == 0 && BN <= 64 && TT >= 1 && TT <= 4, "row tiles of 16, <= 64 tokens");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15;
    const int q = lane >> 4;
#ifndef QG_MMQ_XCDTOK
#define QG_MMQ_XCDTOK 0
#endif
    // (tuning knob) two token tiles on disjoint XCD halves: linear workgroup L runs on XCD L % 8;
    // XCDs 0-3 take token tile 0, XCDs 4-7 token tile 1, so each XCD's L2 serves one activation tile
    int tx = blockIdx.x, ty = blockIdx.y;
    if (QG_MMQ_XCDTOK && gridDim.y == 2 && (gridDim.x & 3) == 0 && gridDim.z == 1) {
        const int L = blockIdx.y * gridDim.x + blockIdx.x, x8 = L & 7;
        ty = x8 >> 2;
        tx = (L >> 3) * 4 + (x8 & 3);
    }
    const int n0 = tx * BN;
    const int m0 = ty * G::NTOK;
    const int nb = K / QK;
    const int H = nb / SB / KS;  // stages of this workgroup's K slice
    const int h0 = KS > 1 ? (int)blockIdx.z * H : 0;
    const long RB = (long)nb * T::BB;
    const long AB = (long)nb * Q8_1_BYTES;
    uint8_t* bufs = smem + wave * NB * G::BUF;
    uint8_t* zb = smem + G::ZOFF + (ZL ? wave * MMQ_ZB : 0);  // this wave's zero region (ZL)
    if constexpr (ZL) {
        static_assert(MMQ_ZB == 64 * 16, "one 16-B store per lane");
        *reinterpret_cast<uint4*>(zb + 16 * lane) = make_uint4(0u, 0u, 0u, 0u);  // read only by this wave
    }
#ifdef QG_MMQ_STAMPS
    unsigned long long stamps[8] = {};
#endif
    MMQ_STAMP(0);

    // per-lane DMA source offsets within a stage (rows / tokens past the edge read the last valid
    // one; their results are dropped), relative to the workgroup's first row / token: the 64-bit
    // bases Bw / Aw carry n0 * RB and m0 * AB, so tensors beyond 2 GiB address correctly and the
    // per-lane offsets stay below BN * RB (mmq_shape_ok)
    const uint8_t* Bw = B + (long)n0 * RB;
    const uint8_t* Aw = A + (long)m0 * AB;
    auto wpiece = [&](int p) {  // weight piece p of a stage: byte offset from Bw
        const int row = p / G::PPR;
        return (min(n0 + row, N - 1) - n0) * (int)RB + (p - row * G::PPR) * G::WPS;
    };
    auto apiece = [&](int p) {  // activation piece p of a stage: byte offset from Aw
        const int tok = p / G::APT;
        return (min(m0 + tok, M - 1) - m0) * (int)AB + min(p - tok * G::APT, G::APR - 1) * 16;
    };
    constexpr int NOFF = G::CMB ? G::NI : 1;
    int woff[G::CMB ? 1 : G::NWI], aoff[G::CMB ? 1 : G::NAI], coff[NOFF];
    bool cisw[NOFF];
    if constexpr (G::CMB) {
#pragma unroll
        for (int i = 0; i < G::NI; ++i) {
            const int p = min(64 * i + lane, G::WPC + G::APC - 1);
            cisw[i] = p < G::WPC;
            coff[i] = cisw[i] ? wpiece(p) : apiece(p - G::WPC);
            if constexpr (ABL == 3) if (cisw[i]) { cisw[i] = false; coff[i] = apiece(min(p, G::APC - 1)); }
            if constexpr (ABL == 4) if (!cisw[i]) { cisw[i] = true; coff[i] = wpiece(0); }
        }
    } else {
#pragma unroll
        for (int i = 0; i < G::NWI; ++i) woff[i] = wpiece(min(64 * i + lane, G::WPC - 1));
#pragma unroll
        for (int i = 0; i < G::NAI; ++i) aoff[i] = apiece(min(64 * i + lane, G::APC - 1));
    }
    // All lanes issue every DMA instruction (lanes past the image fetch a clamped piece into the
    // padding): a lane-predicated global_load_lds let hipcc sink two of them into one block with a
    // per-lane M0 base, read back with v_readfirstlane — wrong destinations for half the wave
    // (found by profiles/tools_archive/mmq_debug.hip on Q4_1, 16 rows x 16 tokens).
    auto issue = [&](int h, uint8_t* buf) {
        const uint8_t* wsrc = Bw + (long)h * G::RSB - G::shift(h);
        const uint8_t* asrc = Aw + (long)h * (SB * Q8_1_BYTES);
        if constexpr (G::CMB) {
#pragma unroll
            for (int i = 0; i < G::NI; ++i) glds<16>((cisw[i] ? wsrc : asrc) + coff[i], buf + 64 * i * 16);
        } else {
#pragma unroll
            for (int i = 0; i < G::NWI; ++i) glds<G::WPS>(wsrc + woff[i], buf + 64 * i * G::WPS);
#pragma unroll
            for (int i = 0; i < G::NAI; ++i) glds<16>(asrc + aoff[i], buf + G::OFF_A + 64 * i * 16);
        }
    };

    float acc[G::NACC];
#pragma unroll
    for (int i = 0; i < G::NACC; ++i) acc[i] = 0.0f;
    const v4i bias = {MMQ_BIAS, MMQ_BIAS, MMQ_BIAS, MMQ_BIAS};

    // Operand fragments of one block, shared by both epilogue forms (so the parity hook's sumi, which
    // runs the product's EPI2 form, covers exactly the product's decode): the weight row's k-slot q
    // (elements 4q..4q+3 | 16+4q..16+4q+3 as low / high nibbles, + qh bits for Q5_x, or Q8_0's
    // signed qs dwords q and 4+q), and the token's qs dwords q and 4+q.
    auto wfrag = [&](const uint8_t* wr, auto O) -> long {
        constexpr int o = decltype(O)::value;  // block's byte offset in the row image
        uint32_t lo, hi;
        if constexpr (T::Q8) {
            lo = lds32<o + T::QS>(wr + 4 * q);
            hi = lds32<o + T::QS + 16>(wr + 4 * q);
        } else {
            const uint32_t v = lds32<o + T::QS>(wr + 4 * q);  // 4q keeps the alignment
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
    auto afrag_of = [&](const uint8_t* ar) -> long {
        const uint32_t qa0 = *reinterpret_cast<const uint32_t*>(ar + 4 + 4 * q);
        const uint32_t qa1 = *reinterpret_cast<const uint32_t*>(ar + 20 + 4 * q);
        return (long)(((unsigned long)qa1 << 32) | qa0);
    };
    // sumi parity hook: the block's int32 dots of this lane's 4 rows x its token
    auto store_sumi = [&](const v4i& c, int i, int t, int h, int b) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int n = n0 + 16 * i + 4 * q + e, m = m0 + 16 * t + r16;
            if (n < N && m < M) sumi_out[((long)m * N + n) * nb + h * SB + b] = c[e] - MMQ_BIAS;
        }
    };


    // Block scales straight from the staged images, per lane: the f16 bits of d_w (and m_w) of the
    // 4 weight rows 16 i + 4 q + e it accumulates (used as f16 by v_fma_mix_f32, no convert), and
    // {d_a, -d_a * 1.5*2^23, -c * s_a} of its token 16 t + r16 with c = 8 (Q4_0), 16 (Q5_0),
    // 0 (Q8_0) or -1 (Q4_1 / Q5_1: + m_w * s_a). Only LDS reads in the main loop: an LDS write
    // there makes hipcc wait for every DMA in flight (vmcnt(0)), which serialised the double buffer.
    constexpr float CS = F == FMT_Q4_0 ? 8.0f : F == FMT_Q5_0 ? 16.0f : F == FMT_Q8_0 ? 0.0f : -1.0f;
    constexpr bool HAS_M = T::MOFF >= 0;
    struct blk_t {
        v4i c[G::RT][TT];
        uint32_t dw[G::RT][4], mw[G::RT][4];
        f32x2 da[TT], nda[TT], ncs[TT];  // token scalars, duplicated for the packed-f32 ops
    };
    auto u16 = [](const uint8_t* p) { return (uint32_t)*reinterpret_cast<const uint16_t*>(p); };
    // Epilogue, two elements (rows e, e+1 of one token) per packed op:
    //   Q4_0 / Q5_0 / Q8_0: acc += d_w * (fma(d_a, cf, -d_a*1.5*2^23) - c*s_a)   [pk_fma, pk_add, fma_mix]
    //   Q4_1 / Q5_1:        acc += (d_w * d_a) * sumi + m_w * s_a   (ncs = +s_a)   [fma_mix, pk_mul, fma_mix, add]
    // fma(d_a, cf, -d_a*1.5*2^23) = round(d_a * sumi) exactly (cf = 1.5*2^23 + sumi, exact constant).
    auto epilogue = [&](const blk_t& p, int h, int b) {
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                if constexpr (SUMI) {
                    store_sumi(p.c[i][t], i, t, h, b);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; e += 2) {
                        const f32x2 cf = {__int_as_float(p.c[i][t][e]), __int_as_float(p.c[i][t][e + 1])};
                        float* a = &acc[(i * TT + t) * 4 + e];
                        if constexpr (!HAS_M) {
                            f32x2 t2 = __builtin_elementwise_fma(p.da[t], cf, p.nda[t]);  // d_a * sumi
                            if constexpr (CS != 0.0f) t2 = t2 + p.ncs[t];                   // - c * s_a
                            a[0] = fma_mix_lo(p.dw[i][e], t2.x, a[0]);
                            a[1] = fma_mix_lo(p.dw[i][e + 1], t2.y, a[1]);
                        } else {
                            const f32x2 x = cf - f32x2{MMQ_BIAS_F, MMQ_BIAS_F};            // exact: sumi
                            const f32x2 dd = {fma_mix_lo(p.dw[i][e], p.da[t].x, -0.0f),
                                              fma_mix_lo(p.dw[i][e + 1], p.da[t].x, -0.0f)};  // d_w * d_a
                            const f32x2 t1 = dd * x;
                            const f32x2 tm = {fma_mix_lo(p.mw[i][e], p.ncs[t].x, t1.x),
                                              fma_mix_lo(p.mw[i][e + 1], p.ncs[t].x, t1.y)};  // + m_w * s_a
                            a[0] += tm.x;
                            a[1] += tm.y;
                        }
                    }
                }
            }
    };

    // The 4 blocks of one staged stage in three phases, so each phase's latencies overlap: every
    // LDS read of the stage (operand fragments and block scales) in flight together, then the
    // 4 x RT x TT MFMAs back to back, then the VALU epilogues (block b's results are read behind
    // the later blocks' MFMAs and epilogues, plus a 16-state margin over the 8 the hardware needs:
    // see the header).
    // EPI2 (!SUMI): the scale arithmetic moves onto the matrix pipe. Per block, one
    // v_mfma_f32_16x16x16_f16 forms the outer product d_w (x) d_a (k-slot 0 only: exact f16 x f16 in
    // f32) in the accumulator layout, so the VALU epilogue is sumi = cf - 1.5*2^23 (exact) and
    // acc += dd * sumi — one packed op per element instead of two; the compensation term
    // sum_b X[n][b] s_a[m][b] (X = d_w, or m_w for Q4_1 / Q5_1) is accumulated over each stage's
    // 4 blocks by one more MFMA per tile into c2 and added once at the end (x -8 / -16 / +1).
    // Each lane reads only its own row's d_w (and m_w): 1 LDS read per row tile and block instead
    // of 4. Within the fp32 summation-order bound of the parity tests (the per-term rounding
    // differs from the reference's d_w * (d_a * sumi - c * s_a)).
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    constexpr bool HAS_S = F != FMT_Q8_0;
    constexpr float CFAC = F == FMT_Q4_0 ? -8.0f : F == FMT_Q5_0 ? -16.0f : 1.0f;
    f32x4v c2[EPI2 ? G::RT : 1][EPI2 ? TT : 1];
    if constexpr (EPI2) {
#pragma unroll
        for (int i = 0; i < G::RT; ++i)
#pragma unroll
            for (int t = 0; t < TT; ++t) c2[i][t] = f32x4v{0.f, 0.f, 0.f, 0.f};
    }
    auto h4 = [](unsigned long v) { return __builtin_bit_cast(f16x4, v); };
    auto compute4_e2 = [&](uint8_t* buf, int h, int sh, auto SUB, auto&& after_reads) {
        constexpr int b0 = 4 * decltype(SUB)::value;
        (void)h;
        long afrag[MMQ_SB][G::RT], bfrag[MMQ_SB][TT];
        uint32_t wdb[MMQ_SB][G::RT], wmb[MMQ_SB][G::RT], adb[MMQ_SB][TT];
        const bool q0 = q == 0;
        constexpr bool RAW = (OPT & MMQ_RAW) != 0;
        // raw weight dwords (MMQ_RAW): [0] / [1] the qs dword(s) at o + QS + 4q (two when not 4-B aligned),
        // [2] / [3] the same 16 bytes on (Q8_0's high dword), [4] / [5] the qh dword (Q5_x)
        uint32_t wraw[RAW ? MMQ_SB : 1][RAW ? G::RT : 1][6];
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            constexpr int o = (b0 + b) * T::BB;
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                const uint8_t* wr = buf + (16 * i + r16) * G::RIMG + sh;
                if constexpr (RAW) {
                    constexpr int qo = o + T::QS, qa = qo % 4;
                    const uint32_t* p = reinterpret_cast<const uint32_t*>(wr + 4 * q + (qo & ~3));
                    wraw[b][i][0] = p[0];
                    if constexpr (qa != 0) wraw[b][i][1] = p[1];
                    if constexpr (T::Q8) {
                        wraw[b][i][2] = p[4];
                        if constexpr (qa != 0) wraw[b][i][3] = p[5];
                    }
                    if constexpr (T::QH >= 0) {
                        constexpr int ho = o + T::QH;
                        const uint32_t* ph = reinterpret_cast<const uint32_t*>(wr + (ho & ~3));
                        wraw[b][i][4] = ph[0];
                        if constexpr (ho % 4 != 0) wraw[b][i][5] = ph[1];
                    }
                } else {
                    afrag[b][i] = wfrag(wr, ic<o>{});
                }
                const uint8_t* ws = ZL ? (q0 ? wr : zb) : wr;  // ZL: lanes q > 0 read zeros
                wdb[b][i] = u16(ws + o);
                if constexpr (HAS_M) wmb[b][i] = u16(ws + o + T::MOFF);
            }
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                const uint8_t* a0 = buf + G::OFF_A + (16 * t + r16) * G::ASTR;
                const uint8_t* ar = a0 + (b0 + b) * Q8_1_BYTES;
                bfrag[b][t] = afrag_of(ar);
                const uint8_t* as = ZL ? (q0 ? a0 : zb) : a0;
                adb[b][t] = *reinterpret_cast<const uint32_t*>(as + (b0 + b) * Q8_1_BYTES);  // f16 d_a | f16 s_a << 16
            }
        });
        __builtin_amdgcn_sched_barrier(0);
        after_reads();  // MMQ_EARLY: the buffer's refill (it waits for the LDS reads itself: WAR on the buffer)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (RAW) {  // realign + nibble split (wfrag's arithmetic) now that every read has returned
            static_for<MMQ_SB>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
                constexpr int o = (b0 + b) * T::BB;
                constexpr int qa = (o + T::QS) % 4;
#pragma unroll
                for (int i = 0; i < G::RT; ++i) {
                    auto al = [&](int k) {
                        if constexpr (qa == 0) return wraw[b][i][k];
                        else return __builtin_amdgcn_alignbyte(wraw[b][i][k + 1], wraw[b][i][k], qa);
                    };
                    uint32_t lo, hi;
                    if constexpr (T::Q8) {
                        lo = al(0);
                        hi = al(2);
                    } else {
                        const uint32_t v = al(0);
                        lo = v & 0x0F0F0F0Fu;
                        hi = (v >> 4) & 0x0F0F0F0Fu;
                    }
                    if constexpr (T::QH >= 0) {
                        constexpr int ha = (o + T::QH) % 4;
                        uint32_t qh;
                        if constexpr (ha == 0) qh = wraw[b][i][4];
                        else qh = __builtin_amdgcn_alignbyte(wraw[b][i][5], wraw[b][i][4], ha);
                        lo |= spread4_bit4((qh >> (4 * q)) & 0xFu);
                        hi |= spread4_bit4((qh >> (16 + 4 * q)) & 0xFu);
                    }
                    afrag[b][i] = (long)(((unsigned long)hi << 32) | lo);
                }
            });
        }
        f32x4v dd[MMQ_SB][G::RT][TT];
        v4i cc[MMQ_SB][G::RT][TT];
        const f32x4v z4 = {0.f, 0.f, 0.f, 0.f};
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int i = 0; i < G::RT; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t)
                    dd[b][i][t] = __builtin_amdgcn_mfma_f32_16x16x16f16(
                        h4(ZL ? (unsigned long)wdb[b][i] : q0 ? (unsigned long)(wdb[b][i] & 0xFFFFu) : 0ul),
                        h4(ZL ? (unsigned long)(adb[b][t] & 0xFFFFu) : q0 ? (unsigned long)(adb[b][t] & 0xFFFFu) : 0ul),
                        z4, 0, 0, 0);
        });
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
                    cc[b][i][t] = __builtin_amdgcn_mfma_i32_16x16x32_i8(afrag[b][i], bfrag[b][t], bias, 0, 0, 0);
        });
        if constexpr (HAS_S) {
            // k-slots 0..3 = the sub-stage's 4 blocks (lanes q = 0 only)
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                const uint32_t* X = HAS_M ? wmb[0] : wdb[0];
                (void)X;
                uint32_t x01, x23;
                if constexpr (HAS_M) {
                    x01 = __builtin_amdgcn_perm(wmb[1][i], wmb[0][i], 0x05040100u);
                    x23 = __builtin_amdgcn_perm(wmb[3][i], wmb[2][i], 0x05040100u);
                } else {
                    x01 = __builtin_amdgcn_perm(wdb[1][i], wdb[0][i], 0x05040100u);
                    x23 = __builtin_amdgcn_perm(wdb[3][i], wdb[2][i], 0x05040100u);
                }
                const unsigned long xa = ZL || q0 ? (((unsigned long)x23 << 32) | x01) : 0ul;
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const uint32_t s01 = __builtin_amdgcn_perm(adb[1][t], adb[0][t], 0x07060302u);
                    const uint32_t s23 = __builtin_amdgcn_perm(adb[3][t], adb[2][t], 0x07060302u);
                    const unsigned long sb = ZL || q0 ? (((unsigned long)s23 << 32) | s01) : 0ul;
                    c2[i][t] = __builtin_amdgcn_mfma_f32_16x16x16f16(h4(xa), h4(sb), c2[i][t], 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SUMI) {
            static_for<MMQ_SB>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t) store_sumi(cc[b][i][t], i, t, h, b0 + b);
            });
            return;
        }
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int i = 0; i < G::RT; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int e = 0; e < 4; e += 2) {
                        const f32x2 sm = f32x2{__int_as_float(cc[b][i][t][e]), __int_as_float(cc[b][i][t][e + 1])} -
                                         f32x2{MMQ_BIAS_F, MMQ_BIAS_F};  // exact: sumi
                        float* a = &acc[(i * TT + t) * 4 + e];
                        const f32x2 r = __builtin_elementwise_fma(f32x2{dd[b][i][t][e], dd[b][i][t][e + 1]}, sm,
                                                                  f32x2{a[0], a[1]});
                        a[0] = r.x;
                        a[1] = r.y;
                    }
        });
        __builtin_amdgcn_sched_barrier(0);
    };

    auto compute4 = [&](uint8_t* buf, int h, int sh, auto SUB) {
        constexpr int b0 = 4 * decltype(SUB)::value;  // first block of this 4-block sub-stage
        blk_t blk[MMQ_SB];
        long afrag[MMQ_SB][G::RT], bfrag[MMQ_SB][TT];
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            constexpr int o = (b0 + b) * T::BB;
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                const uint8_t* wr = buf + (16 * i + r16) * G::RIMG + sh;
                afrag[b][i] = wfrag(wr, ic<o>{});
                const uint8_t* sr = buf + (16 * i + 4 * q) * G::RIMG + sh + o;  // rows 16 i + 4 q + e
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    blk[b].dw[i][e] = u16(sr + e * G::RIMG);
                    if constexpr (HAS_M) blk[b].mw[i][e] = u16(sr + e * G::RIMG + T::MOFF);
                }
            }
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                const uint8_t* ar = buf + G::OFF_A + (16 * t + r16) * G::ASTR + (b0 + b) * Q8_1_BYTES;
                bfrag[b][t] = afrag_of(ar);
                const uint32_t dsh = *reinterpret_cast<const uint32_t*>(ar);
                const float da = h2f(dsh & 0xFFFFu), sa = h2f(dsh >> 16);
                const float nda = -(da * MMQ_BIAS_F), ncs = -(CS * sa);
                blk[b].da[t] = f32x2{da, da};
                blk[b].nda[t] = f32x2{nda, nda};
                blk[b].ncs[t] = f32x2{ncs, ncs};
            }
        });
        __builtin_amdgcn_sched_barrier(0);
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
                    blk[b].c[i][t] = __builtin_amdgcn_mfma_i32_16x16x32_i8(afrag[b][i], bfrag[b][t], bias, 0, 0, 0);
        });
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (ABL == 2) {
            static_for<MMQ_SB>([&](auto BI) {
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t) acc[(i * TT + t) * 4] += __int_as_float(blk[decltype(BI)::value].c[i][t][0]);
            });
        } else {
            static_for<MMQ_SB>([&](auto BI) { epilogue(blk[decltype(BI)::value], h, b0 + decltype(BI)::value); });
        }
        __builtin_amdgcn_sched_barrier(0);
    };

    auto compute = [&](uint8_t* buf, int h, int sh, auto&& after_reads) {
        if constexpr (EPI2 && ABL == 0)
            static_for<SB / 4>([&](auto SUB) {
                if constexpr (decltype(SUB)::value == SB / 4 - 1) compute4_e2(buf, h, sh, SUB, after_reads);
                else compute4_e2(buf, h, sh, SUB, [] {});
            });
        else
            static_for<SB / 4>([&](auto SUB) { compute4(buf, h, sh, SUB); });
    };

    // this wave's stages h = wave + k W (k < nst), up to NB of them in flight. ROT: the workgroups
    // of one XCD (blockIdx.x = c mod 8) start at different rounds of W stages, so they do not all
    // pull the same activation lines through their L2 at the same moment; each wave keeps its set
    // of stages (rotation by a multiple of W when W divides H), only their order changes.
    // MMQ_CONTIG (H % W == 0): wave w owns stages w * H / W .. (w + 1) * H / W - 1 instead.
    constexpr bool CONTIG = (OPT & MMQ_CONTIG) != 0;
    const bool contig = CONTIG && H % W == 0;
    const int nst = contig ? H / W : wave < H ? (H - 1 - wave) / W + 1 : 0;
    const int rot = ROT && H % W == 0 ? (int)(((blockIdx.x >> 3) * W) % H) : 0;
    auto stage = [&](int k) {
        if (contig) return h0 + wave * nst + k;
        const int h = wave + rot + k * W;
        return h0 + (h >= H ? h - H : h);
    };
    constexpr bool DYN = (OPT & MMQ_DYN) != 0;
    if constexpr (DYN) {
        static_assert(NB == 2 && KS == 1 && !CONTIG && !ROT, "dynamic stages: double buffer, no split-K");
        unsigned* ctr = reinterpret_cast<unsigned*>(smem + G::LDS);
        uint8_t* slots = smem + G::LDS + 16;
        if (threadIdx.x == 0) *ctr = 2 * W;  // stages 0 .. 2W - 1 are handed out statically
        __syncthreads();                     // (no DMA in flight yet)
        // LDS atomic and slot stores as inline asm: an LDS write the compiler sees makes it wait for
        // every LDS-DMA in flight (see the header)
        auto grab = [&]() -> int {
            unsigned old = 0;
            if (lane == 0) {
                const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned*)ctr;
                asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(old) : "v"(a), "v"(1u) : "memory");
            }
            return __builtin_amdgcn_readfirstlane((int)old);
        };
        auto put = [&](int h) {
            const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(slots + (size_t)h * G::SLOT) + 16 * lane;
#pragma unroll
            for (int j = 0; j < G::NACC / 4; ++j) {
                const v4i v = {__float_as_int(acc[4 * j]), __float_as_int(acc[4 * j + 1]), __float_as_int(acc[4 * j + 2]),
                               __float_as_int(acc[4 * j + 3])};
                asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(a), "v"(v), "i"(j * 1024) : "memory");
            }
        };
        int ha = wave, hb = wave + W;  // stages in buffers A and B (>= H: none)
        uint8_t* bA = bufs;
        uint8_t* bB = bufs + G::BUF;
        if (ha < H) issue(ha, bA);
        if (hb < H) issue(hb, bB);
        while (ha < H) {
            wait_stage<G::NI>(hb < H ? 1 : 0);  // stage ha's DMA landed
#pragma unroll
            for (int i = 0; i < G::NACC; ++i) acc[i] = 0.0f;
            if constexpr (EPI2) {
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t) c2[i][t] = f32x4v{0.f, 0.f, 0.f, 0.f};
            }
            if constexpr (ABL != 1 && ABL != 3 && ABL != 4) compute(bA, ha, G::shift(ha), [] {});
            if constexpr (!SUMI) {
                if constexpr (EPI2 && HAS_S) {
                    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // margin: the stage's compensation MFMAs
#pragma unroll
                    for (int i = 0; i < G::RT; ++i)
#pragma unroll
                        for (int t = 0; t < TT; ++t)
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                acc[(i * TT + t) * 4 + e] = __builtin_fmaf(CFAC, c2[i][t][e], acc[(i * TT + t) * 4 + e]);
                }
                put(ha);
            }
            const int hn = grab();
            if (hn < H) issue(hn, bA);  // refill the buffer just consumed
            ha = hb;
            hb = hn;
            uint8_t* t = bA;
            bA = bB;
            bB = t;
        }
        MMQ_STAMP(3);
        if constexpr (!SUMI) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's slot stores
            __syncthreads();
            constexpr int TS = G::NACC * 64;
            for (int c = threadIdx.x; c < TS / 4; c += W * 64) {  // 16-B chunk c = (j, ln): acc 4j..4j+3 of lane ln
                const float* p = reinterpret_cast<const float*>(slots) + 4 * c;
                f32x4v v = *reinterpret_cast<const f32x4v*>(p);
                for (int h = 1; h < H; ++h) v += *reinterpret_cast<const f32x4v*>(p + (size_t)h * TS);
                const int j = c >> 6, ln = c & 63;
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                    const int a = 4 * j + e4;
                    const int e = a & 3, t = (a >> 2) % TT, i = (a >> 2) / TT;
                    const int n = n0 + 16 * i + 4 * (ln >> 4) + e;
                    const int m = m0 + 16 * t + (ln & 15);
                    if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v[e4];
                }
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NB; ++k)
            if (k < nst) issue(stage(k), bufs + k * G::BUF);
        for (int k = 0; k < nst; ++k) {
            const int h = stage(k);
            uint8_t* cur = bufs + (k % NB) * G::BUF;
            wait_stage<G::NI>(min(nst - 1 - k, NB - 1));  // this stage's DMA landed
    #ifdef QG_MMQ_STAMPS
            if (k == 0) MMQ_STAMP(1);
    #endif
            constexpr bool early = (OPT & MMQ_EARLY) != 0 && EPI2 && ABL == 0;
            if constexpr (ABL != 1 && ABL != 3 && ABL != 4) {
                // the refill overwrites `cur`: every LDS read of it must have returned first (hipcc does
                // not order a global_load_lds after earlier ds_reads of the same bytes — round 4 found the
                // unwaited form non-deterministic on the GPU, tests/test_gpu_fused.py)
                if constexpr (early)
                    compute(cur, h, G::shift(h), [&] {
                        if (k + NB < nst) {
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            issue(stage(k + NB), cur);
                        }
                    });
                else compute(cur, h, G::shift(h), [] {});
            }
    #ifdef QG_MMQ_STAMPS
            if (k == 0) MMQ_STAMP(2);
    #endif
            if constexpr (!early)
                if (k + NB < nst) issue(stage(k + NB), cur);  // refill the buffer just consumed
        }
        MMQ_STAMP(3);
    
        if constexpr (EPI2 && !SUMI && HAS_S) {
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // margin: the last compensation MFMAs (8 needed, header)
    #pragma unroll
            for (int i = 0; i < G::RT; ++i)
    #pragma unroll
                for (int t = 0; t < TT; ++t)
    #pragma unroll
                    for (int e = 0; e < 4; ++e) acc[(i * TT + t) * 4 + e] = __builtin_fmaf(CFAC, c2[i][t][e], acc[(i * TT + t) * 4 + e]);
        }
        if constexpr (!SUMI) {
            // fixed-order sum of the W partial tiles, in the wave buffers once every wave is done
            float* red = reinterpret_cast<float*>(smem);
            __syncthreads();
    #pragma unroll
            for (int i = 0; i < G::NACC; ++i) red[(wave * G::NACC + i) * 64 + lane] = acc[i];
            __syncthreads();
            constexpr int TS = G::NACC * 64;  // floats per tile
            auto wsum = [&](int idx) {
                float v = red[idx];
    #pragma unroll
                for (int ww = 1; ww < W; ++ww) v += red[ww * TS + idx];
                return v;
            };
            auto store = [&](int idx, float v) {
                const int a = idx >> 6, ln = idx & 63;
                const int e = a & 3, t = (a >> 2) % TT, i = (a >> 2) / TT;
                const int n = n0 + 16 * i + 4 * (ln >> 4) + e;
                const int m = m0 + 16 * t + (ln & 15);
                if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v;
            };
            if constexpr (KS == 1) {
                for (int idx = threadIdx.x; idx < TS; idx += W * 64) store(idx, wsum(idx));
            } else {
                const long tile = (long)blockIdx.y * gridDim.x + blockIdx.x;
                float* pt = part + tile * KS * TS;
                // Partials and counter move with agent-scope (sc1) accesses, coherent across the XCDs'
                // L2s without a release/acquire fence: a fence writes back / invalidates a whole L2,
                // which other workgroups' cached lines pay for (measured 5-40x slower launches).
                for (int idx = threadIdx.x; idx < TS; idx += W * 64)
                    __hip_atomic_store(pt + blockIdx.z * TS + idx, wsum(idx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial is at the coherence point
                __syncthreads();
                int* last = reinterpret_cast<int*>(smem);
                if (threadIdx.x == 0)
                    *last = __hip_atomic_fetch_add(cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == KS - 1;
                __syncthreads();
                if (!*last) return;
                for (int idx = threadIdx.x; idx < TS; idx += W * 64) {
                    float x[KS];  // every slice's load issued before the first add (atomic loads keep order)
    #pragma unroll
                    for (int s = 0; s < KS; ++s) x[s] = __hip_atomic_load(pt + s * TS + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    float v = x[0];
    #pragma unroll
                    for (int s = 1; s < KS; ++s) v += x[s];
                    store(idx, v);
                }
                if (threadIdx.x == 0) __hip_atomic_store(cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
#ifdef QG_MMQ_STAMPS
    MMQ_STAMP(4);
    if (lane == 0) {
        const int wv = (blockIdx.y * gridDim.x + blockIdx.x) * W + wave;
        for (int kk = 0; kk < 5; ++kk) g_mmq_stamps[8 * wv + kk] = stamps[kk];
    }
#endif
}

// General entry (probes: split-K workspace, ablations).
// (4-wave workgroups: at least two per CU, i.e. <= 256 VGPRs — without the cap the EPI2 form took
// 320 and ran one workgroup per CU, 13 % slower at M=512 than with it)
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB = 2, int ABL = 0, bool ROT = false, int SB = 4,
          int KS = 1, bool EPI2 = false, int OPT = 0>
__global__ __launch_bounds__(W * 64, W <= 4 ? 2 : 1) void mmq_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                     float* __restrict__ C, int32_t* __restrict__ sumi_out, int M,
                                                     int N, int K, long ldc_m, long ldc_n, float* __restrict__ part,
                                                     unsigned* __restrict__ cnt) {
    mmq_body<F, BN, TT, W, SUMI, P16, NB, ABL, ROT, SB, KS, EPI2, OPT>(A, B, C, sumi_out, M, N, K, ldc_m, ldc_n, part, cnt);
}

// Short entry (no split-K): (A, B, M, N, K, out, ldc_m, ldc_n) with 32-bit output strides = 10
// kernel-argument dwords, all preloaded into SGPRs (each preloaded dword costs every wave's launch:
// qg_gemv_kernel.hpp, gemv1_kernel). SUMI: out is the parity hook's int32 buffer. Faster for the
// 16-row and the 32 x 32 8-wave tiles, slower for the 32 x 16 8-wave and the 4-wave tiles
// (profiles/r02_tuning/ab_sig2.txt, ab_sig3.txt), so the dispatch picks it per tile.
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB = 2, int SB = 4, bool EPI2 = false, int OPT = 0>
__global__ __launch_bounds__(W * 64, W <= 4 ? 2 : 1) void mmq1_kernel(const uint8_t* __restrict__ A,
                                                      const uint8_t* __restrict__ B, int M, int N, int K,
                                                      void* __restrict__ out, int ldc_m, int ldc_n) {
    mmq_body<F, BN, TT, W, SUMI, P16, NB, 0, false, SB, 1, EPI2, OPT>(A, B, SUMI ? nullptr : (float*)out,
                                                                       SUMI ? (int32_t*)out : nullptr, M, N, K, ldc_m, ldc_n,
                                                                       nullptr, nullptr);
}

// Preconditions: K a multiple of 128 (whole stages), 16-B aligned activation rows and base, weight
// rows and stages aligned to the DMA piece, one workgroup's rows / tokens within 2 GiB (tensors of
// any size otherwise). P16 additionally: a 16-B aligned B
// and rows, and K % 256 == 0 when a stage segment is not a 16-B multiple (see mmq_geom).
// Workspace of a split-K (KS > 1) launch: one counter per output tile (zero before the first
// launch; every launch leaves them zero), then KS partial tiles per output tile.
template <int BN, int TT, int KS> inline size_t mmq_ws_bytes(int M, int N) {
    if (KS == 1) return 0;
    const size_t tiles = (size_t)((N + BN - 1) / BN) * ((M + 16 * TT - 1) / (16 * TT));
    return ((tiles * 4 + 255) & ~(size_t)255) + tiles * KS * (BN / 16) * TT * 4 * 64 * 4;
}

template <int F, int BN, int TT, int W, bool P16, int NB = 2, int SB = 4, int KS = 1>
inline bool mmq_shape_ok(const GemmArgs& g) {
    using G = mmq_geom<F, BN, TT, W, P16, NB, SB>;  // the shape rules do not depend on OPT
    if (g.M < 1 || g.N < 1 || g.K % (QK * SB * KS) != 0) return false;
    if (KS > 1 && (g.sumi || !g.ws || g.ws_bytes < mmq_ws_bytes<BN, TT, KS>(g.M, g.N) || ((uintptr_t)g.ws & 255)))
        return false;
    const long RB = (long)(g.K / QK) * wfmt<F>::BB, AB = (long)(g.K / QK) * Q8_1_BYTES;
    if (((uintptr_t)g.A & 15) != 0 || AB % 16 != 0) return false;
    if (P16 && G::RSB % 16 != 0 && g.K % 256 != 0) return false;
    if (((uintptr_t)g.B % G::WPS) != 0 || RB % G::WPS != 0) return false;
    // per-lane DMA offsets are 32-bit relative to the workgroup's 64-bit row / token base
    if (RB * BN >= (1L << 31) || AB * G::NTOK >= (1L << 31)) return false;
    if (g.ldc_m > INT32_MAX || g.ldc_n > INT32_MAX) return false;  // mmq1_kernel's 32-bit strides
    return true;
}

template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB, int ABL, bool ROT, int SB, int KS, bool EPI2, int OPT>
hipError_t mmq_launch_full(const GemmArgs& g, hipStream_t st, dim3 grid);

// SHORT: launch through mmq1_kernel (10 preloaded argument dwords) instead of the general entry —
// per configuration, as measured (qg_gemm_mfma.hip).
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB = 2, int ABL = 0, bool ROT = false, int SB = 4,
          int KS = 1, bool EPI2 = false, int OPT = 0, bool SHORT = false>
hipError_t mmq_launch(const GemmArgs& g, hipStream_t st) {
    using G = mmq_geom<F, BN, TT, W, P16, NB, SB, OPT>;
    const dim3 grid((g.N + BN - 1) / BN, (g.M + G::NTOK - 1) / G::NTOK, KS);
    if (g.describe) {  // qg_debug_config: name the instantiation instead of launching it
        const bool short_sig = SHORT && KS == 1 && ABL == 0 && !ROT;
        describe_kernel(g, "mmq F=%d BN=%d TT=%d W=%d P16=%d NB=%d ABL=%d ROT=%d SB=%d KS=%d EPI2=%d OPT=%d SIG=%s grid=%ux%ux%u",
                        F, BN, TT, W, (int)P16, NB, ABL, (int)ROT, SB, KS, (int)EPI2, OPT, short_sig ? "short" : "full", grid.x,
                        grid.y, grid.z);
        return hipSuccess;
    }
    if constexpr (SHORT && KS == 1 && ABL == 0 && !ROT) {  // (mmq_shape_ok: 32-bit output strides)
        auto k1 = mmq1_kernel<F, BN, TT, W, SUMI, P16, NB, SB, EPI2, OPT>;
        const size_t lds = G::dyn_lds(g.K / QK / SB);
        if (lds > 64 * 1024) {
            static std::atomic<unsigned long long> attr_done{0};
            const hipError_t e = set_max_lds_once((const void*)k1, 160 * 1024, attr_done);
            if (e != hipSuccess) return e;
        }
        void* out = SUMI ? (void*)g.sumi : (void*)g.C;
        hipLaunchKernelGGL(k1, grid, dim3(W * 64), lds, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, out,
                           (int)g.ldc_m, (int)g.ldc_n);
        return hipGetLastError();
    } else {
        return mmq_launch_full<F, BN, TT, W, SUMI, P16, NB, ABL, ROT, SB, KS, EPI2, OPT>(g, st, grid);
    }
}

template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB, int ABL, bool ROT, int SB, int KS, bool EPI2, int OPT>
hipError_t mmq_launch_full(const GemmArgs& g, hipStream_t st, dim3 grid) {
    using G = mmq_geom<F, BN, TT, W, P16, NB, SB, OPT>;
    auto k = mmq_kernel<F, BN, TT, W, SUMI, P16, NB, ABL, ROT, SB, KS, EPI2, OPT>;
    unsigned* cnt = KS > 1 ? (unsigned*)g.ws : nullptr;
    float* part = KS > 1 ? (float*)((uint8_t*)g.ws + ((((size_t)grid.x * grid.y) * 4 + 255) & ~(size_t)255)) : nullptr;
    const size_t lds = G::dyn_lds(g.K / QK / SB / KS);
    if (lds > 64 * 1024) {
        static std::atomic<unsigned long long> attr_done{0};
        const hipError_t e = set_max_lds_once((const void*)k, 160 * 1024, attr_done);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, grid, dim3(W * 64), lds, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.C, g.sumi, g.M,
                       g.N, g.K, g.ldc_m, g.ldc_n, part, cnt);
    return hipGetLastError();
}

}  // namespace qg
