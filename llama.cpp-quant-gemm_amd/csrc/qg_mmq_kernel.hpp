// qg_mmq_kernel.hpp — W4A8 prefill GEMM (M > 4) on the CDNA4 matrix cores, v_mfma_i32_16x16x32_i8.
//
// C[M,N] = A_q8_1[M,K] . B_w[N,K]^T (include/gemm_reference.h:175-222), activation-major.
//
// One MFMA = one Q-block: v_mfma_i32_16x16x32_i8 has K = 32, so each MFMA returns the exact int32
// sumi of 16 (weight row n) x 16 (token m) pairs for one block. The accumulator is seeded with the
// bit pattern of 1.5*2^23, so the MFMA's integer add leaves cf = 12582912.0f + sumi as a float
// (|sumi| < 2^22, no v_cvt_f32_i32) and cf - 1.5*2^23 = sumi exactly.
//
// Operand k-order: lane (r = lane&15, q = lane>>4) supplies, for its weight row / token r, the 8
// bytes of k-slot q: elements 4q..4q+3 and 16+4q..16+4q+3 of the block. For the weights that is qs
// dword q split into low / high nibbles (+ the qh bits for Q5_x), for Q8_0 its signed qs dwords q and
// 4+q; for the activations qs dwords q and 4+q. A and B use the same slot -> element map and the
// integer sum is order-free. C layout (gfx950, dtype-independent): lane holds column m = lane&15,
// rows n = 4q + e (e < 4).
//
// Scale epilogue on the matrix pipe: per block one v_mfma_f32_16x16x16_f16 with only k-slot 0
// populated forms the outer product d_w (x) d_a (exact f16 x f16 in f32) in the accumulator layout,
// so the VALU work per element is acc += dd * (cf - 1.5*2^23) (one packed op per two elements); the
// compensation term sum_b X[n][b] s_a[m][b] (X = d_w, or m_w for Q4_1 / Q5_1) accumulates over each
// stage's 4 blocks in one more MFMA per tile and is added once at the end (x -8 / -16 / +1). Within the
// reassociation bound of the parity tests (oracle.reassoc_tol; the per-term rounding differs from the
// reference's d_w * (d_a * sumi - c * s_a)).
//
// Tiling: a workgroup owns BN weight rows x 16*TT tokens and ALL of K; its W waves
// split K into 4-block stages, wave w taking stages w, w+W, ... Each wave streams its stages with
// LDS-DMA (global_load_lds / buffer_load ... lds: no VGPR staging) into NB wave-private LDS buffers,
// the next stage in flight while the current one computes (counted vmcnt). No workgroup barrier in
// the main loop; the W partial tiles are summed in fixed wave order through LDS at the end.
//
// Two weight layouts (LAY):
//  * LAY_ROWS — the reference's AoS rows [N][K/32] (drop-in). A stage's weight bytes are BN row
//    segments of 4*BB bytes, 16-B aligned windows of RIMG bytes (P16) or 4-B pieces.
//  * LAY_TILED — the load-time layout of qg_tile_weights (round 5; qg_repack.hip): rows in tiles of 32,
//    K in stages of 4 blocks, each (tile, stage) ONE contiguous run of 128*BB bytes holding the 32 rows'
//    4 blocks as planes in MFMA fragment order (tiled_fmt below). A stage's weights are one linear
//    16-B-per-lane stream (the reference AoS rows scatter it over 32 segments of 72 B, which the LDS-DMA
//    ingests at half the rate: profiles/r04_tuning/dma_probe2_linear.txt), and every lane reads its
//    operand fragment of 4 blocks with ONE ds_read_b128 and its 4 scales with one ds_read_b64.
// AW (activation windows): activation rows of nba blocks with nba % 4 != 0 (K/32 odd, e.g. K = 4128,
// against weights padded to whole stages with zero blocks): a token's stage segment then starts 0, 4, 8
// or 12 bytes into a 16-B aligned 160-B window (the shift depends on the token only), the activation
// DMA goes through a buffer resource over the activation tensor (reads past its end return zeros, so
// no window can fault), and the scales of blocks >= nba are zeroed so the padding blocks' terms are an
// exact +0 whatever bytes their windows caught.
//
// A stage runs in three phases (all LDS reads, all MFMAs, all epilogues) so that each phase's
// latencies overlap. MFMA results -> VALU: gfx950 needs 8 wait states after v_mfma_i32_16x16x32_i8
// and v_mfma_f32_16x16x16_f16 (tools/mfma_hazard_probe.hip on an MI355X: every lane wrong at <= 6
// states, right from 8; profiles/r02_tuning/mfma_hazard_probe.txt) and hipcc pads exactly 8
// (`s_nop 7`); tests/test_isa_hazards.py checks every MFMA of the shipped code object for it. The
// `s_nop 7; s_nop 7` after each MFMA phase below is a margin on top (the round-1 wrong sums that
// first prompted it came from an MFMA result element read through a bit_cast, mmq_probe1-2.txt).
// Only LDS reads in the main loop: an LDS write there makes hipcc wait for every DMA in flight.
// (Rejected round-4 tuning forms — early refill, raw fragment batches, dynamic stage hand-out,
// ablations, timeline stamps — live in profiles/tools_archive/qg_mmq_kernel_r04_knobs.hpp, not here.)
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
constexpr int MMQ_SB = 4;             // blocks per stage

// TILE_ROWS, tiled_fmt: the tiled weight layout, qg_common.hpp (shared with the tiled GEMV)

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
    static_assert(SZ == 4 || SZ == 16, "global_load_lds sizes");
    if constexpr (SZ == 16) __builtin_amdgcn_global_load_lds(gp, lp, 16, 0, 0);
    else __builtin_amdgcn_global_load_lds(gp, lp, 4, 0, 0);
}

// P16 (LAY_ROWS): weights DMA'd in 16-B pieces (16-B aligned B and rows; else 4-B pieces). A stage's
// row segment (RSB = 4 * BB bytes) then starts 16-B aligned or 8 bytes past (RSB % 16 == 8 for Q4_0 /
// Q5_0 / Q8_0, alternating with the stage parity): each row image is a 16-B aligned window of RIMG
// bytes and the data sits SHIFT(h) = (h * RSB) % 16 bytes into it. With K % 256 == 0 the stage count
// is even, so the last stage is an odd one (shift 8) and no window reaches past the end of the rows.
// NB: stage buffers per wave.
// CMB: with 16-B weight pieces and no activation windows, weight and activation pieces share one
// piece numbering (p < WPC: weights, then activations), so only the last DMA instruction carries
// padding. With AW the activation pieces take instructions of their own (buffer loads).
template <int F, int BN, int TT, int W, bool P16, int NB, int LAY, bool AW> struct mmq_geom {
    using T = wfmt<F>;
    using TF = tiled_fmt<F>;
    static constexpr bool TL = LAY != LAY_ROWS;               // tiled weights (LAY_TILED, LAY_TILED_ACT)
    static constexpr bool TA = LAY == LAY_TILED_ACT;          // tiled activations
    static constexpr int RSB = MMQ_SB * T::BB;                 // weight bytes per row per stage
    static constexpr int WPS = (P16 || TL) ? 16 : 4;           // weight DMA piece (bytes)
    static constexpr int RIMG = TL ? RSB : P16 && RSB % 16 != 0 ? RSB + 8 : RSB;  // LAY_ROWS row image bytes
    // LAY_TILED stage image of BN rows: [QS][QH][SC] (offsets within the weight image)
    static constexpr int LQH = (BN / 16) * 64 * TF::QSL;
    static constexpr int LSC = LQH + BN * TF::QHB;
    static constexpr int WIMG = TL ? LSC + BN * TF::SCB : BN * RIMG;
    static constexpr int PPR = RIMG / WPS;                     // LAY_ROWS pieces per row image
    static constexpr int WPC = WIMG / WPS;                     // weight pieces per stage
    static constexpr int NTOK = 16 * TT;
    static constexpr int APR = AW ? 10 : 9;                    // activation 16-B pieces per token
    static constexpr int APT = AW ? 11 : 9;                    // ... incl. a pad piece (AW: 44-dword stride)
    static constexpr int ASTR = APT * 16;                      // token image stride (bytes)
    static constexpr int APC = NTOK * APT;                     // activation 16-B pieces per stage
    static constexpr bool CMB = WPS == 16 && !AW;              // combined piece numbering
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
    static constexpr size_t LDS = (size_t)W * (NB * BUF > NACC * 256 ? NB * BUF : NACC * 256);
    static_assert(NB >= 1 && NB <= 4, "1..4 stage buffers per wave");
    static_assert(!TL || BN == 16 || BN == 32, "tiled layout: 16- or 32-row workgroup tiles");
    static constexpr bool FITS = LDS <= 160 * 1024;            // (mmq_shape_ok refuses the rest)
    static_assert(OFF_A % 16 == 0 && BUF % 16 == 0, "16-B aligned LDS regions");
    static_assert(RSB % 8 == 0, "stage segments are 8-B multiples");
    static_assert(NB * NI <= 63, "vmcnt range");
    __host__ __device__ static constexpr int shift(int h) { return P16 && !TL ? (h * RSB) & 15 : 0; }
};

// s_waitcnt vmcnt(younger * NI): the oldest stage's DMA landed, `younger` later stages may still fly.
template <int NI> __device__ __forceinline__ void wait_stage(int younger) {
    if (younger <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NI) : "memory");
}

// K: the weight side's K (LAY_ROWS: row length; LAY_TILED: 128 x the stage count); nba: activation
// blocks per row (= K / 32 unless AW), also the sumi hook's blocks per (m, n).
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB, int LAY, bool AW>
__device__ __forceinline__ void mmq_body(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B, float* __restrict__ C,
                                         int32_t* __restrict__ sumi_out, int M, int N, int K, int nba, long ldc_m,
                                         long ldc_n) {
    using G = mmq_geom<F, BN, TT, W, P16, NB, LAY, AW>;
    using T = wfmt<F>;
    using TF = tiled_fmt<F>;
    constexpr bool TL = G::TL;
    static_assert(G::FITS, "LDS per workgroup");
    static_assert(BN % 16 == 0 && BN <= 64 && TT >= 1 && TT <= 4, "row tiles of 16, <= 64 tokens");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15;
    const int q = lane >> 4;
    const int n0 = blockIdx.x * BN;
    const int m0 = blockIdx.y * G::NTOK;
    const int nb = K / QK;
    const int H = nb / MMQ_SB;  // stages
    if constexpr (!AW && LAY != LAY_TILED_ACT) nba = nb;  // (tiled activations: nba = the real blocks, sumi hook)
    const long RB = (long)nb * T::BB;
    const long AB = (long)nba * Q8_1_BYTES;
    uint8_t* bufs = smem + wave * NB * G::BUF;

    // per-lane DMA source offsets within a stage (rows / tokens past the edge read the last valid
    // one; their results are dropped), relative to the workgroup's first row / token: the 64-bit
    // bases Bw / Aw carry n0 * RB (tiled: the tile's first stage) and m0 * AB, so tensors beyond 2 GiB
    // address correctly and the per-lane offsets stay small (mmq_shape_ok)
    const int r0 = TL ? n0 % TILE_ROWS : 0;  // LAY_TILED: the workgroup's first row within its tile
    const uint8_t* Bw = TL ? B + (long)(n0 / TILE_ROWS) * H * TF::STG : B + (long)n0 * RB;
    // tiled activations: the workgroup's first 16-token tile (m0 is a multiple of 16); tiles past the last
    // one (TT = 2 at M % 32 in 1..16) read the last tile, their outputs are dropped
    const int nat = (M + ACT_TILE - 1) / ACT_TILE;
    const uint8_t* Aw = G::TA ? A + (long)(m0 / ACT_TILE) * H * ACT_STG : A + (long)m0 * AB;
    auto wpiece = [&](int p) {  // weight piece p of a stage: byte offset from the stage's base
        if constexpr (TL) {
            const int o = 16 * p;  // the image's planes, each a contiguous run of the tile's stage
            if (o < G::LQH) return (r0 / 16) * 64 * TF::QSL + o;
            if (o < G::LSC) return TF::OQH + r0 * TF::QHB + (o - G::LQH);
            return TF::OSC + r0 * TF::SCB + (o - G::LSC);
        } else {
            const int row = p / G::PPR;
            return (min(n0 + row, N - 1) - n0) * (int)RB + (p - row * G::PPR) * G::WPS;
        }
    };
    auto apiece = [&](int p) {  // activation piece p of a stage: byte offset from Aw (+ the stage's)
        const int tok = p / G::APT;
        if constexpr (G::TA) {  // the token's 144-B segment inside its tile's 2304-B stage run
            const int sub = min(m0 / ACT_TILE + tok / ACT_TILE, nat - 1) - m0 / ACT_TILE;
            return sub * H * ACT_STG + (tok % ACT_TILE) * (MMQ_SB * Q8_1_BYTES) + (p - tok * G::APT) * 16;
        }
        const int t0 = (min(m0 + tok, M - 1) - m0) * (int)AB;
        const int j = min(p - tok * G::APT, G::APR - 1);
        if constexpr (AW) return t0 - (t0 & 15) + j * 16;  // the 16-B aligned window around the segment
        else return t0 + j * 16;
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
        }
    } else {
#pragma unroll
        for (int i = 0; i < G::NWI; ++i) woff[i] = wpiece(min(64 * i + lane, G::WPC - 1));
#pragma unroll
        for (int i = 0; i < G::NAI; ++i) aoff[i] = apiece(min(64 * i + lane, G::APC - 1));
    }
    // AW: the activation tile as a raw buffer resource — a window past the tensor's end reads zeros
    // (unused without AW)
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc((void*)Aw, (short)0, (int)min((long)(M - m0) * AB, 0x7FFFFFF0L), 0x00020000);
    // All lanes issue every DMA instruction (lanes past the image fetch a clamped piece into the
    // padding): a lane-predicated global_load_lds let hipcc sink two of them into one block with a
    // per-lane M0 base, read back with v_readfirstlane — wrong destinations for half the wave
    // (found by profiles/tools_archive/mmq_debug.hip on Q4_1, 16 rows x 16 tokens).
    auto issue = [&](int h, uint8_t* buf) {
        const uint8_t* wsrc = TL ? Bw + (long)h * TF::STG : Bw + (long)h * G::RSB - G::shift(h);
        const uint8_t* asrc = Aw + (long)h * (G::TA ? ACT_STG : MMQ_SB * Q8_1_BYTES);
        if constexpr (G::CMB) {
#pragma unroll
            for (int i = 0; i < G::NI; ++i) glds<16>((cisw[i] ? wsrc : asrc) + coff[i], buf + 64 * i * 16);
        } else {
#pragma unroll
            for (int i = 0; i < G::NWI; ++i) glds<G::WPS>(wsrc + woff[i], buf + 64 * i * G::WPS);
#pragma unroll
            for (int i = 0; i < G::NAI; ++i) {
                uint8_t* dst = buf + G::OFF_A + 64 * i * 16;
                if constexpr (AW)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)dst, 16, aoff[i],
                                                             h * (MMQ_SB * Q8_1_BYTES), 0, 0);
                else glds<16>(asrc + aoff[i], dst);
            }
        }
    };

    float acc[G::NACC];
#pragma unroll
    for (int i = 0; i < G::NACC; ++i) acc[i] = 0.0f;
    const v4i bias = {MMQ_BIAS, MMQ_BIAS, MMQ_BIAS, MMQ_BIAS};

    // AW: this lane's tokens' window shifts (bytes into the 16-B aligned window)
    int ash[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) ash[t] = AW ? ((min(m0 + 16 * t + r16, M - 1) - m0) * (int)AB) & 15 : 0;

    // sumi parity hook: the block's int32 dots of this lane's 4 rows x its token
    auto store_sumi = [&](const v4i& c, int i, int t, int blk) {
        if (blk >= nba) return;  // padding blocks (LAY_TILED / AW)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int n = n0 + 16 * i + 4 * q + e, m = m0 + 16 * t + r16;
            if (n < N && m < M) sumi_out[((long)m * N + n) * nba + blk] = c[e] - MMQ_BIAS;
        }
    };

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
    auto h4 = [](unsigned long v) { return __builtin_bit_cast(f16x4, v); };
    auto u16 = [](const uint8_t* p) { return (uint32_t)*reinterpret_cast<const uint16_t*>(p); };

    // The 4 blocks of one staged stage in three phases, so each phase's latencies overlap: every
    // LDS read of the stage (operand fragments and block scales) in flight together, then the MFMAs
    // back to back, then the VALU epilogues (results read behind the later MFMAs plus a 16-state
    // margin over the 8 the hardware needs: see the header).
    auto compute = [&](uint8_t* buf, int h) {
        const int sh = G::shift(h);
        long afrag[MMQ_SB][G::RT], bfrag[MMQ_SB][TT];
        uint32_t wdb[MMQ_SB][G::RT];        // f16 d_w of block b, this lane's row (q = 0 lanes use it)
        uint32_t xs[G::RT][2];              // f16 X of blocks 0..3 (X = d_w, or m_w), packed in pairs
        uint32_t adb[MMQ_SB][TT];           // f16 d_a | f16 s_a << 16
        const bool q0 = q == 0;
        if constexpr (TL) {
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                const uint8_t* qsp = buf + i * 64 * TF::QSL + lane * 16;
                const uint4 v = *reinterpret_cast<const uint4*>(qsp);  // dword q of the 4 blocks
                uint4 v8 = {}, qh = {};
                if constexpr (T::Q8) v8 = *reinterpret_cast<const uint4*>(qsp + 1024);  // dword 4 + q
                if constexpr (T::QH >= 0) qh = *reinterpret_cast<const uint4*>(buf + G::LQH + (16 * i + r16) * 16);
                const uint8_t* scp = buf + G::LSC + (16 * i + r16) * TF::SCB;
                uint32_t sc[4];
                if constexpr (HAS_M) {
                    const uint4 s4 = *reinterpret_cast<const uint4*>(scp);
                    sc[0] = s4.x; sc[1] = s4.y; sc[2] = s4.z; sc[3] = s4.w;
                } else {
                    const uint2 s2 = *reinterpret_cast<const uint2*>(scp);
                    sc[0] = s2.x; sc[1] = s2.y; sc[2] = 0; sc[3] = 0;
                }
                const uint32_t vv[4] = {v.x, v.y, v.z, v.w}, v8v[4] = {v8.x, v8.y, v8.z, v8.w};
                const uint32_t qhv[4] = {qh.x, qh.y, qh.z, qh.w};
#pragma unroll
                for (int b = 0; b < MMQ_SB; ++b) {
                    uint32_t lo, hi;
                    if constexpr (T::Q8) {
                        lo = vv[b];
                        hi = v8v[b];
                    } else {
                        lo = vv[b] & 0x0F0F0F0Fu;
                        hi = (vv[b] >> 4) & 0x0F0F0F0Fu;
                    }
                    if constexpr (T::QH >= 0) {
                        lo |= spread4_bit4((qhv[b] >> (4 * q)) & 0xFu);
                        hi |= spread4_bit4((qhv[b] >> (16 + 4 * q)) & 0xFu);
                    }
                    afrag[b][i] = (long)(((unsigned long)hi << 32) | lo);
                    wdb[b][i] = (b & 1) ? sc[b >> 1] >> 16 : sc[b >> 1] & 0xFFFFu;
                }
                xs[i][0] = HAS_M ? sc[2] : sc[0];
                xs[i][1] = HAS_M ? sc[3] : sc[1];
            }
        } else {
            uint32_t wmb[MMQ_SB][G::RT];
            static_for<MMQ_SB>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
                constexpr int o = b * T::BB;  // block's byte offset in the row image
#pragma unroll
                for (int i = 0; i < G::RT; ++i) {
                    const uint8_t* wr = buf + (16 * i + r16) * G::RIMG + sh;
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
                    afrag[b][i] = (long)(((unsigned long)hi << 32) | lo);
                    wdb[b][i] = u16(wr + o);
                    if constexpr (HAS_M) wmb[b][i] = u16(wr + o + T::MOFF);
                }
            });
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                if constexpr (HAS_M) {
                    xs[i][0] = __builtin_amdgcn_perm(wmb[1][i], wmb[0][i], 0x05040100u);
                    xs[i][1] = __builtin_amdgcn_perm(wmb[3][i], wmb[2][i], 0x05040100u);
                } else {
                    xs[i][0] = __builtin_amdgcn_perm(wdb[1][i], wdb[0][i], 0x05040100u);
                    xs[i][1] = __builtin_amdgcn_perm(wdb[3][i], wdb[2][i], 0x05040100u);
                }
            }
        }
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                const uint8_t* a0 = buf + G::OFF_A + (16 * t + r16) * G::ASTR + ash[t];
                const uint8_t* ar = a0 + b * Q8_1_BYTES;
                const uint32_t qa0 = *reinterpret_cast<const uint32_t*>(ar + 4 + 4 * q);
                const uint32_t qa1 = *reinterpret_cast<const uint32_t*>(ar + 20 + 4 * q);
                bfrag[b][t] = (long)(((unsigned long)qa1 << 32) | qa0);
                adb[b][t] = *reinterpret_cast<const uint32_t*>(ar);
                // AW: blocks past the activation row (the weights' zero padding) contribute an exact +0
                // whatever bytes their window caught (zero d_a and s_a; their weight codes are zero too)
                if constexpr (AW) if (h * MMQ_SB + b >= nba) adb[b][t] = 0u;
            }
        });
        __builtin_amdgcn_sched_barrier(0);
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
                        h4(q0 ? (unsigned long)(wdb[b][i] & 0xFFFFu) : 0ul), h4(q0 ? (unsigned long)(adb[b][t] & 0xFFFFu) : 0ul),
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
            // k-slots 0..3 = the stage's 4 blocks (lanes q = 0 only)
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                const unsigned long xa = q0 ? (((unsigned long)xs[i][1] << 32) | xs[i][0]) : 0ul;
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const uint32_t s01 = __builtin_amdgcn_perm(adb[1][t], adb[0][t], 0x07060302u);
                    const uint32_t s23 = __builtin_amdgcn_perm(adb[3][t], adb[2][t], 0x07060302u);
                    const unsigned long sb = q0 ? (((unsigned long)s23 << 32) | s01) : 0ul;
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
                    for (int t = 0; t < TT; ++t) store_sumi(cc[b][i][t], i, t, h * MMQ_SB + b);
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

    // this wave's stages h = wave + k W (k < nst), up to NB of them in flight
    const int nst = wave < H ? (H - 1 - wave) / W + 1 : 0;
    auto stage = [&](int k) { return wave + k * W; };
#pragma unroll
    for (int k = 0; k < NB; ++k)
        if (k < nst) issue(stage(k), bufs + k * G::BUF);
    for (int k = 0; k < nst; ++k) {
        const int h = stage(k);
        uint8_t* cur = bufs + (k % NB) * G::BUF;
        wait_stage<G::NI>(min(nst - 1 - k, NB - 1));  // this stage's DMA landed
        compute(cur, h);
        if (k + NB < nst) issue(stage(k + NB), cur);  // refill the buffer just consumed
    }

    if constexpr (!SUMI && HAS_S) {
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
        for (int idx = threadIdx.x; idx < TS; idx += W * 64) {
            float v = red[idx];
#pragma unroll
            for (int ww = 1; ww < W; ++ww) v += red[ww * TS + idx];
            const int a = idx >> 6, ln = idx & 63;
            const int e = a & 3, t = (a >> 2) % TT, i = (a >> 2) / TT;
            const int n = n0 + 16 * i + 4 * (ln >> 4) + e;
            const int m = m0 + 16 * t + (ln & 15);
            if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v;
        }
    }
}

// General entry. The two trailing pointers are unused: the argument layout is the one the round-1..4
// tuning measured for the 32 x 16 tiles (profiles/r02_tuning/ab_sig2.txt, ab_sig3.txt).
// (4-wave workgroups: at least two per CU, i.e. <= 256 VGPRs — without the cap the MFMA-assisted
// epilogue took 320 and ran one workgroup per CU, 13 % slower at M=512 than with it)
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB>
__global__ __launch_bounds__(W * 64, W <= 4 ? 2 : 1) void mmq_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                     float* __restrict__ C, int32_t* __restrict__ sumi_out, int M,
                                                     int N, int K, long ldc_m, long ldc_n, float* __restrict__ unused0,
                                                     unsigned* __restrict__ unused1) {
    (void)unused0;
    (void)unused1;
    mmq_body<F, BN, TT, W, SUMI, P16, NB, LAY_ROWS, false>(A, B, C, sumi_out, M, N, K, K / QK, ldc_m, ldc_n);
}

// Short entry: (A, B, M, N, K, out, ldc_m, ldc_n) with 32-bit output strides = 10 kernel-argument
// dwords, all preloaded into SGPRs (each preloaded dword costs every wave's launch:
// qg_gemv_kernel.hpp, gemv1_kernel). SUMI: out is the parity hook's int32 buffer. Faster for the
// 16-row and the 32 x 32 8-wave tiles, slower for the 32 x 16 8-wave and the 4-wave tiles
// (profiles/r02_tuning/ab_sig2.txt, ab_sig3.txt), so the dispatch picks it per tile.
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB>
__global__ __launch_bounds__(W * 64, W <= 4 ? 2 : 1) void mmq1_kernel(const uint8_t* __restrict__ A,
                                                      const uint8_t* __restrict__ B, int M, int N, int K,
                                                      void* __restrict__ out, int ldc_m, int ldc_n) {
    mmq_body<F, BN, TT, W, SUMI, P16, NB, LAY_ROWS, false>(A, B, SUMI ? nullptr : (float*)out, SUMI ? (int32_t*)out : nullptr,
                                                           M, N, K, K / QK, ldc_m, ldc_n);
}

// Tiled-layout and activation-window entry: (A, B, M, N, K, nba, out, ldc_m, ldc_n), K the weight
// side's (stages x 128), nba the activation blocks per row.
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB, int LAY, bool AW>
__global__ __launch_bounds__(W * 64, W <= 4 ? 2 : 1) void mmqt_kernel(const uint8_t* __restrict__ A,
                                                      const uint8_t* __restrict__ B, int M, int N, int K, int nba,
                                                      void* __restrict__ out, int ldc_m, int ldc_n) {
    mmq_body<F, BN, TT, W, SUMI, P16, NB, LAY, AW>(A, B, SUMI ? nullptr : (float*)out, SUMI ? (int32_t*)out : nullptr, M, N, K,
                                                   nba, ldc_m, ldc_n);
}

// Preconditions: K a multiple of 128 (whole stages), 16-B aligned activation base (and rows unless
// AW), weight rows and stages aligned to the DMA piece, one workgroup's rows / tokens within 2 GiB
// (tensors of any size otherwise). P16 additionally: a 16-B aligned B and rows, and K % 256 == 0 when
// a stage segment is not a 16-B multiple (see mmq_geom). LAY_TILED: a 16-B aligned B_tiled.
// g.K is the logical K; LAY_TILED and AW run on the weight side's K (mmq_weight_k).
inline int mmq_weight_k(const GemmArgs& g) {
    const int nb = g.K / QK;
    if (g.lay != LAY_ROWS) return (nb + MMQ_SB - 1) / MMQ_SB * MMQ_SB * QK;
    return g.nbw > 0 ? g.nbw * QK : g.K;
}
template <int F, int BN, int TT, int W, bool P16, int NB = 2, int LAY = LAY_ROWS, bool AW = false>
inline bool mmq_shape_ok(const GemmArgs& g) {
    using G = mmq_geom<F, BN, TT, W, P16, NB, LAY, AW>;
    if (!G::FITS) return false;
    const int K = mmq_weight_k(g), nba = g.K / QK;
    if (g.M < 1 || g.N < 1 || g.K % QK != 0 || K % (QK * MMQ_SB) != 0 || K < g.K) return false;
    if (LAY == LAY_TILED_ACT) {
        if (AW) return false;  // the tiled activations are zero padded to whole stages
    } else if (AW != (nba % MMQ_SB != 0 || K != g.K)) return false;  // windows exactly when the rows differ
    if (LAY != LAY_ROWS) {
        if (g.lay != LAY || ((uintptr_t)g.B & 15) != 0) return false;
        if ((long)tiled_fmt<F>::STG * (K / QK / MMQ_SB) >= (1L << 31)) return false;
    } else {
        if (g.lay != LAY_ROWS) return false;
        const long RB = (long)(K / QK) * wfmt<F>::BB;
        if (P16 && G::RSB % 16 != 0 && K % 256 != 0) return false;
        if (((uintptr_t)g.B % G::WPS) != 0 || RB % G::WPS != 0) return false;
        if (RB * BN >= (1L << 31)) return false;  // per-lane DMA offsets are 32-bit
    }
    const long AB = (long)nba * Q8_1_BYTES;
    if (LAY == LAY_TILED_ACT) {
        if (((uintptr_t)g.A & 15) != 0 || (long)ACT_STG * (K / QK / MMQ_SB) * ((G::NTOK + ACT_TILE - 1) / ACT_TILE) >= (1L << 31))
            return false;
    } else {
        if (((uintptr_t)g.A & 15) != 0 || (!AW && AB % 16 != 0)) return false;
        if (AB * G::NTOK >= (1L << 31) || (AW && AB * g.M >= (1L << 31))) return false;
    }
    if (g.ldc_m > INT32_MAX || g.ldc_n > INT32_MAX) return false;  // the short entries' 32-bit strides
    return true;
}

// SHORT: launch through mmq1_kernel (10 preloaded argument dwords) instead of the general entry —
// per configuration, as measured (qg_gemm_mfma.hip). LAY_TILED / AW: mmqt_kernel.
template <int F, int BN, int TT, int W, bool SUMI, bool P16, int NB = 2, int LAY = LAY_ROWS, bool AW = false, bool SHORT = false>
hipError_t mmq_launch(const GemmArgs& g, hipStream_t st) {
    using G = mmq_geom<F, BN, TT, W, P16, NB, LAY, AW>;
    const dim3 grid((g.N + BN - 1) / BN, (g.M + G::NTOK - 1) / G::NTOK, 1);
    constexpr bool T = LAY != LAY_ROWS || AW;
    if (g.describe) {  // qg_debug_config: name the instantiation instead of launching it
        describe_kernel(g, "mmq F=%d BN=%d TT=%d W=%d P16=%d NB=%d LAY=%d AW=%d SIG=%s grid=%ux%u", F, BN, TT, W, (int)P16, NB,
                        LAY, (int)AW, T ? "tiled" : SHORT ? "short" : "full", grid.x, grid.y);
        return hipSuccess;
    }
    const void* k;
    if constexpr (T) k = (const void*)mmqt_kernel<F, BN, TT, W, SUMI, P16, NB, LAY, AW>;
    else if constexpr (SHORT) k = (const void*)mmq1_kernel<F, BN, TT, W, SUMI, P16, NB>;
    else k = (const void*)mmq_kernel<F, BN, TT, W, SUMI, P16, NB>;
    if (G::LDS > 64 * 1024) {
        static std::atomic<unsigned long long> attr_done{0};
        const hipError_t e = set_max_lds_once(k, 160 * 1024, attr_done);
        if (e != hipSuccess) return e;
    }
    void* out = SUMI ? (void*)g.sumi : (void*)g.C;
    if constexpr (T) {
        hipLaunchKernelGGL((mmqt_kernel<F, BN, TT, W, SUMI, P16, NB, LAY, AW>), grid, dim3(W * 64), G::LDS, st,
                           (const uint8_t*)g.A, (const uint8_t*)g.B, g.M, g.N, mmq_weight_k(g), g.K / QK, out, (int)g.ldc_m,
                           (int)g.ldc_n);
    } else if constexpr (SHORT) {
        hipLaunchKernelGGL((mmq1_kernel<F, BN, TT, W, SUMI, P16, NB>), grid, dim3(W * 64), G::LDS, st, (const uint8_t*)g.A,
                           (const uint8_t*)g.B, g.M, g.N, g.K, out, (int)g.ldc_m, (int)g.ldc_n);
    } else {
        hipLaunchKernelGGL((mmq_kernel<F, BN, TT, W, SUMI, P16, NB>), grid, dim3(W * 64), G::LDS, st, (const uint8_t*)g.A,
                           (const uint8_t*)g.B, g.C, g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n, (float*)nullptr,
                           (unsigned*)nullptr);
    }
    return hipGetLastError();
}

}  // namespace qg
