// qg_mmql_kernel.hpp — W4A8 prefill GEMM for large M (round 5): 64 weight rows x 64 tokens per workgroup,
// four waves each owning a disjoint 32 x 32 output tile, 4-block stages ingested cooperatively into LDS.
//
// Same block arithmetic as qg_mmq_kernel.hpp — the int32 sumi of each Q-block from an integer MFMA seeded with
// the 1.5 * 2^23 bias, d_w (x) d_a as an f16 outer-product MFMA, the m / offset term from one compensation
// MFMA per stage — but on the 32 x 32 shapes: v_mfma_i32_32x32x32_i8 computes a whole 32 x 32 tile of one block
// (K = 32 = one Q-block) at gfx950's full i8 rate, where the small-tile kernel's v_mfma_i32_16x16x32_i8 (the
// CDNA3 form) runs at half of it, and v_mfma_f32_32x32x8_f16 forms the scale products. Per-block sumi are
// bit-identical to the reference's (tests/test_gpu_mmql.py); outputs are within the reassociation bound.
//
// Why a second kernel: the small-tile kernel gives each workgroup a 32 x 32 output tile and ALL of K with its
// waves splitting the stages; at M = 512, N = K = 4096 its 2048 workgroups pull 453 MB through the L2 -> LDS
// path. Here each stage of a 64 x 64 tile is DMA'd once (LDS-DMA, every lane one 16-B piece per instruction,
// weight and activation pieces in wave-uniform instructions) and read by all four waves: 226 MB.
//
// MFMA lanes (32 x 32 shapes): operand row / column r32 = lane & 31, k-half hh = lane >> 5 supplies elements
// 16 hh .. 16 hh + 15 of the block — for the activation its qs bytes 16 hh .., i.e. the same 16 bytes one 16-B
// LDS slot further for hh = 1 (so every activation read is a whole, conflict-free ds_read_b128 at a
// compile-time dword position), for a 4-bit weight nibble hh of its 16 qs bytes, for Q8_0 its qs bytes
// 16 hh ... Result element e of a lane: row 8 (e >> 2) + 4 hh + (e & 3), column r32.
//
// Pipeline: NBUF stage buffers shared by the workgroup, NBUF - 1 stages in flight ahead of the one computed.
// Per stage: each wave waits for its own pieces (counted vmcnt), one s_barrier (all pieces landed; every wave
// done reading the buffer about to be refilled), the refill is issued, then the wave's 4 blocks: LDS reads,
// the MFMAs, the scalar-f32 epilogue. The barrier is a bare s_barrier: __syncthreads()' release fence would
// wait for every DMA in flight. Two workgroups per CU (<= 256 VGPRs, 64 KB LDS each) keep two waves per SIMD.
//
// Grid: one dimension, XCD-aware: workgroup id i runs on XCD i % 8, so tile index (i % 8) * (T / 8) + i / 8
// (T tiles, T % 8 == 0) gives each XCD a contiguous run of tiles in row-tile-major order — the token tiles
// that share a 64-row weight tile sit on one XCD and its L2 (the weight rows are read from HBM about once).
//
// Measured (profiles/r05_tuning/r5l_ab.txt, one MI355X, cold rotating weights): M = 512, N = K = 4096 Q4_0
// 35.7 us on the tiled layout (small tiles 43.1), 41.2 us on the reference rows (46.3); the dispatch takes
// it from two workgroups per CU up (qg_mmq_dispatch.hpp). Where the time goes (r5k_ab.txt): the LDS-DMA
// ingest alone 22.6 us, the compute alone 33.3 us — VALU-bound (the per-element epilogue v_sub + v_fmac and
// the nibble unpack: 39 % of wave cycles issuing VALU, SQ counters in r5h/).
#pragma once
#include "qg_mmq_kernel.hpp"

namespace qg {

// WR x WC waves, each 32 rows x 32 tokens; NBUF shared stage buffers. LAY_ROWS with 16-B windows (the
// P16 row images of mmq_geom) or LAY_TILED (the wave's 32 rows are one tile: its stage run verbatim).
template <int F, int LAY, int WR, int WC, int NBUF> struct mmql_geom {
    using T = wfmt<F>;
    using TF = tiled_fmt<F>;
    static constexpr bool TL = LAY != LAY_ROWS;
    static constexpr bool TA = LAY == LAY_TILED_ACT;
    static constexpr int W = WR * WC, BN = 32 * WR, BM = 32 * WC;
    static constexpr int RSB = MMQ_SB * T::BB;                         // weight bytes per row per stage
    static constexpr int RIMG = RSB % 16 != 0 ? RSB + 8 : RSB;         // LAY_ROWS 16-B aligned row window
    static constexpr int WIMG32 = TL ? TF::STG : 32 * RIMG;            // image of one wave's 32 rows
    static constexpr int PW = WR * WIMG32 / 16;                        // weight pieces per stage
    static constexpr int PPR = RIMG / 16;                              // LAY_ROWS pieces per row
    static constexpr int PPT = WIMG32 / 16;                            // pieces per 32 rows
    static constexpr int APT = 9;                                      // 16-B pieces per token (144 B)
    static constexpr int ASTR = APT * 16;
    static constexpr int PA = BM * APT;                                // activation pieces per stage
    // DMA wave-instructions: the first PWI carry weight pieces, the next PAI activation pieces, so every
    // instruction's source base is wave-uniform; NI per wave (wave-instruction i W + wave)
    static constexpr int PWI = (PW + 63) / 64, PAI = (PA + 63) / 64;
    static constexpr int NI = (PWI + PAI + W - 1) / W;
    static constexpr int OFF_A = PWI * 64 * 16;
    static constexpr int BUF = NI * W * 64 * 16;                       // padded to whole instructions
    static constexpr size_t LDS = (size_t)NBUF * BUF;
    static constexpr bool FITS = LDS <= 160 * 1024;
    static_assert(WIMG32 % 16 == 0 && OFF_A % 16 == 0, "16-B pieces");
    static_assert(NBUF >= 2 && NBUF <= 5 && (NBUF - 2) * NI <= 63, "vmcnt range");
    __host__ __device__ static constexpr int shift(int h) { return TL ? 0 : (h * RSB) & 15; }
    static_assert(TL || RSB % 16 == 0 || RSB % 16 == 8, "window shifts 0 / 8");
};

template <int F, int LAY, int WR, int WC, int NBUF, bool SUMI>
__device__ __forceinline__ void mmql_body(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B, float* __restrict__ C,
                                          int32_t* __restrict__ sumi_out, int M, int N, int K, int ldc_m, int ldc_n) {
    using G = mmql_geom<F, LAY, WR, WC, NBUF>;
    using T = wfmt<F>;
    using TF = tiled_fmt<F>;
    constexpr bool TL = G::TL;
    static_assert(G::FITS, "LDS per workgroup");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave / WC, wc = wave % WC;
    const int lane = threadIdx.x & 63;
    // XCD-aware tile order (header)
    const int NT = (N + G::BN - 1) / G::BN, MT = (M + G::BM - 1) / G::BM, TOT = NT * MT;
    const int id = blockIdx.x;
    const int tidx = TOT % 8 == 0 ? (id % 8) * (TOT / 8) + id / 8 : id;
    const int n0 = (tidx / MT) * G::BN;
    const int m0 = (tidx % MT) * G::BM;
    const int nb = K / QK;
    const int H = nb / MMQ_SB;
    const long RB = (long)nb * T::BB;
    const long AB = (long)nb * Q8_1_BYTES;

    const int ntl = (N + TILE_ROWS - 1) / TILE_ROWS;  // LAY_TILED tiles
    const uint8_t* Bw = TL ? B + (long)(n0 / TILE_ROWS) * H * TF::STG : B + (long)n0 * RB;
    const int nat = (M + ACT_TILE - 1) / ACT_TILE;  // tiled activations: 16-token tiles
    const uint8_t* Aw = G::TA ? A + (long)(m0 / ACT_TILE) * H * ACT_STG : A + (long)m0 * AB;
    // per-lane piece offsets (bytes from Bw / Aw, before the stage's) of wave-instruction gi = i W + wave
    int off[G::NI];
    bool isw[G::NI];  // wave-uniform
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
        const int gi = i * G::W + wave;
        isw[i] = gi < G::PWI;
        if (isw[i]) {
            const int p = min(64 * gi + lane, G::PW - 1);
            const int g32 = p / G::PPT, o = p - g32 * G::PPT;  // wave-row group, piece within it
            if constexpr (TL) {
                const int t = min(n0 / TILE_ROWS + g32, ntl - 1) - n0 / TILE_ROWS;  // tiles past N: the last one
                off[i] = t * H * TF::STG + o * 16;
            } else {
                const int row = o / G::PPR;
                off[i] = (min(n0 + 32 * g32 + row, N - 1) - n0) * (int)RB + (o - row * G::PPR) * 16;
            }
        } else {
            const int pa = min(64 * (gi - G::PWI) + lane, G::PA - 1), tok = pa / G::APT;
            if constexpr (G::TA) {
                const int sub = min(m0 / ACT_TILE + tok / ACT_TILE, nat - 1) - m0 / ACT_TILE;
                off[i] = sub * H * ACT_STG + (tok % ACT_TILE) * (MMQ_SB * Q8_1_BYTES) + (pa - tok * G::APT) * 16;
            } else {
                off[i] = (min(m0 + tok, M - 1) - m0) * (int)AB + (pa - tok * G::APT) * 16;
            }
        }
    }
    auto issue = [&](int h, uint8_t* buf) {
        const uint8_t* wsrc = TL ? Bw + (long)h * TF::STG : Bw + (long)h * G::RSB - G::shift(h);
        const uint8_t* asrc = Aw + (long)h * (G::TA ? ACT_STG : MMQ_SB * Q8_1_BYTES);
#pragma unroll
        for (int i = 0; i < G::NI; ++i) glds<16>((isw[i] ? wsrc : asrc) + off[i], buf + 64 * (i * G::W + wave) * 16);
    };

    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    typedef int i32x16 __attribute__((ext_vector_type(16)));
    constexpr bool HAS_M = T::MOFF >= 0;
    constexpr bool HAS_S = F != FMT_Q8_0;
    constexpr float CFAC = F == FMT_Q4_0 ? -8.0f : F == FMT_Q5_0 ? -16.0f : 1.0f;
    // the integer MFMA's seed: 1.5 * 2^23 (qg_mmq_kernel.hpp). Seeding 0 and converting with v_cvt_f32_i32
    // instead of the v_sub measured 9 % slower (profiles/r05_tuning/mmql/r5n_ab.txt: M = 512 38.7 vs 35.4 us)
    constexpr int SEED = MMQ_BIAS;
    i32x16 bias;
#pragma unroll
    for (int e = 0; e < 16; ++e) bias[e] = SEED;
    float acc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
    f32x16 c2;
#pragma unroll
    for (int e = 0; e < 16; ++e) c2[e] = 0.0f;
    auto h4 = [](unsigned long v) { return __builtin_bit_cast(f16x4, v); };
    auto u16 = [](const uint8_t* p) { return (uint32_t)*reinterpret_cast<const uint16_t*>(p); };
    // 32 x 32 MFMA lanes: operand row / column r32 = lane & 31, k-half hh = lane >> 5 — elements
    // 16 hh .. 16 hh + 15 of the block: the activation's qs bytes 16 hh .. 16 hh + 15 (16 contiguous bytes, one
    // 16-B LDS slot further for hh = 1), the 4-bit weight's nibble hh of its 16 qs bytes (Q8_0: qs bytes
    // 16 hh ..). Result element e of a lane: row 8 (e >> 2) + 4 hh + (e & 3), column r32.
    const int r32 = lane & 31, hh = lane >> 5;
    const int nw0 = n0 + 32 * wr, mw0 = m0 + 32 * wc;  // this wave's first row / token
    auto row_of = [&](int e) { return nw0 + 8 * (e >> 2) + 4 * hh + (e & 3); };

    auto store_sumi = [&](const i32x16& c, int blk) {
        const int m = mw0 + r32;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int n = row_of(e);
            if (n < N && m < M) sumi_out[((long)m * N + n) * nb + blk] = c[e] - SEED;
        }
    };

    // a stage's epilogue: dd = d_w (x) d_a, cc = the biased int32 sumi (MFMA results of compute below)
    auto epi = [&](const f32x16(&dd)[MMQ_SB], const i32x16(&cc)[MMQ_SB], int h) {
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // margin over the 32 x 32 MFMAs' wait states
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SUMI) {
            static_for<MMQ_SB>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
                store_sumi(cc[b], h * MMQ_SB + b);
            });
            return;
        }
        // acc += dd * sumi in scalar f32 (v_sub + v_fmac per element): packed f32 beside the MFMAs measured slower
        // (MI355X_MICROARCH.md: an anti-lever beside MFMAs; r05 A/B: M = 512 39.5 -> 35.1 us)
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = __builtin_fmaf(dd[b][e], __int_as_float(cc[b][e]) - MMQ_BIAS_F, acc[e]);
        });
        __builtin_amdgcn_sched_barrier(0);
    };

    // Activation slots: a token's stage image is 9 slots of 16 B; block b's 16 bytes for half hh start at
    // byte 36 b + 4 + 16 hh, i.e. slot (36 b + 4) / 16 + hh, offset (36 b + 4) % 16 — the same offset for
    // both halves, so a lane reads whole slots (ds_read_b128: conflict-free over the 144-B token stride,
    // MI355X_MICROARCH.md LDS table) and picks dwords at compile-time positions. A lane reads its slots
    // j + hh for j in {0..5, 7}. The d_a | s_a dword of block b (byte 36 b) is in those slots for half
    // HB(b): 0 for block 0, 1 for blocks 1..3; the scale MFMAs take block b's k-slot from that half.
    constexpr int AJ[7] = {0, 1, 2, 3, 4, 5, 7};
    auto aslot = [](int j) { return j == 7 ? 6 : j; };  // index into the 7 slots read
    // one stage's 4 blocks for the wave's 32 x 32 tile: LDS reads, MFMAs, epilogues (qg_mmq_kernel.hpp)
    auto compute = [&](auto SHC, const uint8_t* buf, int h) {
        constexpr int SH = decltype(SHC)::value;  // LAY_ROWS: the stage's window shift (0 or 8)
        const uint8_t* wimg = buf + wr * G::WIMG32;
        const uint8_t* ap = buf + G::OFF_A + (32 * wc + r32) * G::ASTR + 16 * hh;
        v4i afrag[MMQ_SB], bfrag[MMQ_SB];
        uint32_t wdb[MMQ_SB], xw[MMQ_SB], ads[MMQ_SB];
        uint32_t S[7][4];
        {
            // whole slots: the empty asm below "uses" all 16 bytes of each, so hipcc keeps them ds_read_b128
            // (it narrows a partly used slot to ds_read2_b32, whose 32-lane banking conflicts 4-way over the
            // 36-dword token stride) and waits for all seven together
            v4i sv[7];
#pragma unroll
            for (int j = 0; j < 7; ++j) sv[j] = *reinterpret_cast<const v4i*>(ap + 16 * AJ[j]);
            asm volatile("" : "+v"(sv[0]), "+v"(sv[1]), "+v"(sv[2]), "+v"(sv[3]), "+v"(sv[4]), "+v"(sv[5]), "+v"(sv[6]));
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                S[j][0] = sv[j][0]; S[j][1] = sv[j][1]; S[j][2] = sv[j][2]; S[j][3] = sv[j][3];
            }
        }
        auto adw = [&](int byte) {  // dword at token byte `byte` (+ 16 hh), compile-time after unrolling
            const int slot = byte >> 4;
            return S[aslot(slot)][(byte & 15) >> 2];
        };
        if constexpr (TL) {
            // row r32 of the tile: dword k (Q8_0: 4 hh + k) of the 4 blocks, k = 0..3 (planes of tiled_fmt)
            const uint8_t* qsp = wimg + (r32 >> 4) * 64 * TF::QSL + (r32 & 15) * 16 + (T::Q8 ? 1024 * hh : 0);
            uint32_t vq[4][4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = *reinterpret_cast<const uint4*>(qsp + 256 * k);
                vq[k][0] = v.x; vq[k][1] = v.y; vq[k][2] = v.z; vq[k][3] = v.w;
            }
            uint4 qh = {};
            if constexpr (T::QH >= 0) qh = *reinterpret_cast<const uint4*>(wimg + TF::OQH + r32 * 16);
            const uint8_t* scp = wimg + TF::OSC + r32 * TF::SCB;
            uint32_t sc[4];
            if constexpr (HAS_M) {
                const uint4 s4 = *reinterpret_cast<const uint4*>(scp);
                sc[0] = s4.x; sc[1] = s4.y; sc[2] = s4.z; sc[3] = s4.w;
            } else {
                const uint2 s2 = *reinterpret_cast<const uint2*>(scp);
                sc[0] = s2.x; sc[1] = s2.y; sc[2] = 0; sc[3] = 0;
            }
            const uint32_t qhv[4] = {qh.x, qh.y, qh.z, qh.w};
#pragma unroll
            for (int b = 0; b < MMQ_SB; ++b) {
                const uint32_t qb = T::QH >= 0 ? qhv[b] >> (16 * hh) : 0u;
                uint32_t x[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    x[k] = T::Q8 ? vq[k][b] : (vq[k][b] >> (4 * hh)) & 0x0F0F0F0Fu;
                    if constexpr (T::QH >= 0) x[k] |= spread4_bit4((qb >> (4 * k)) & 0xFu);
                }
                afrag[b] = v4i{(int)x[0], (int)x[1], (int)x[2], (int)x[3]};
                wdb[b] = (b & 1) ? sc[b >> 1] >> 16 : sc[b >> 1] & 0xFFFFu;
                xw[b] = HAS_M ? ((b & 1) ? sc[2 + (b >> 1)] >> 16 : sc[2 + (b >> 1)] & 0xFFFFu) : wdb[b];
            }
        } else {
            const uint8_t* wrow = wimg + r32 * G::RIMG;
            static_for<MMQ_SB>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
                constexpr int o = SH + b * T::BB;
                uint32_t x[4];
                if constexpr (T::Q8) {
                    const uint8_t* wq = wrow + 16 * hh;
                    x[0] = lds32<o + T::QS>(wq); x[1] = lds32<o + T::QS + 4>(wq);
                    x[2] = lds32<o + T::QS + 8>(wq); x[3] = lds32<o + T::QS + 12>(wq);
                } else {
                    const uint32_t y[4] = {lds32<o + T::QS>(wrow), lds32<o + T::QS + 4>(wrow), lds32<o + T::QS + 8>(wrow),
                                           lds32<o + T::QS + 12>(wrow)};
#pragma unroll
                    for (int k = 0; k < 4; ++k) x[k] = (y[k] >> (4 * hh)) & 0x0F0F0F0Fu;
                }
                if constexpr (T::QH >= 0) {
                    const uint32_t qb = lds32<o + T::QH>(wrow) >> (16 * hh);
#pragma unroll
                    for (int k = 0; k < 4; ++k) x[k] |= spread4_bit4((qb >> (4 * k)) & 0xFu);
                }
                afrag[b] = v4i{(int)x[0], (int)x[1], (int)x[2], (int)x[3]};
                wdb[b] = u16(wrow + o);
                xw[b] = HAS_M ? u16(wrow + o + T::MOFF) : wdb[b];
            });
        }
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            constexpr int X = 36 * b + 4;  // the block's qs for half 0; half 1's are the next slot's same bytes
            bfrag[b] = v4i{(int)adw(X), (int)adw(X + 4), (int)adw(X + 8), (int)adw(X + 12)};
            ads[b] = adw(36 * b - 16 * (b == 0 ? 0 : 1));  // d_a | s_a, valid in half HB(b) (above)
        });
        __builtin_amdgcn_sched_barrier(0);
        f32x16 dd[MMQ_SB];
        i32x16 cc[MMQ_SB];
        f32x16 z16;
#pragma unroll
        for (int e = 0; e < 16; ++e) z16[e] = 0.0f;
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            const bool on = hh == (b == 0 ? 0 : 1);  // the half that holds block b's d_a
            dd[b] = __builtin_amdgcn_mfma_f32_32x32x8f16(h4(on ? (unsigned long)(wdb[b] & 0xFFFFu) : 0ul),
                                                         h4(on ? (unsigned long)(ads[b] & 0xFFFFu) : 0ul), z16, 0, 0, 0);
        });
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            cc[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(afrag[b], bfrag[b], bias, 0, 0, 0);
        });
        if constexpr (HAS_S) {
            // k-slot 0 (half 0) = block 0, k-slots 4..6 (half 1) = blocks 1..3
            const unsigned long xa = hh == 0 ? (unsigned long)(xw[0] & 0xFFFFu)
                                             : ((unsigned long)(xw[3] & 0xFFFFu) << 32) | (xw[2] << 16) | (xw[1] & 0xFFFFu);
            const unsigned long sb = hh == 0 ? (unsigned long)(ads[0] >> 16)
                                             : ((unsigned long)(ads[3] >> 16) << 32) | (ads[2] & 0xFFFF0000u) | (ads[1] >> 16);
            c2 = __builtin_amdgcn_mfma_f32_32x32x8f16(h4(xa), h4(sb), c2, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        epi(dd, cc, h);
    };
    // the stage pipeline (header): NBUF - 1 stages ahead
#pragma unroll
    for (int k = 0; k < NBUF - 1; ++k)
        if (k < H) issue(k, smem + k * G::BUF);
    for (int h = 0; h < H; ++h) {
        wait_stage<G::NI>(min(H - 1 - h, NBUF - 2));  // this wave's pieces of stage h landed
        asm volatile("s_barrier" ::: "memory");       // ... and every wave's; buffer (h - 1) % NBUF is free
        if (h + NBUF - 1 < H) issue(h + NBUF - 1, smem + ((h + NBUF - 1) % NBUF) * G::BUF);
        // LAY_ROWS: the stage's window shift as a compile-time constant (0, or 8 on odd stages)
        if (G::shift(h) == 0) compute(std::integral_constant<int, 0>{}, smem + (h % NBUF) * G::BUF, h);
        else if constexpr (!TL) compute(std::integral_constant<int, 8>{}, smem + (h % NBUF) * G::BUF, h);
    }
    if constexpr (!SUMI) {
        if constexpr (HAS_S) {
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = __builtin_fmaf(CFAC, c2[e], acc[e]);
        }
        const int m = mw0 + r32;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int n = row_of(e);
            if (n < N && m < M) C[(long)m * ldc_m + (long)n * ldc_n] = acc[e];
        }
    }
}

// (A, B, M, N, K, out, ldc_m, ldc_n): 10 preloaded argument dwords; SUMI: out is the sumi hook's buffer.
// One workgroup per CU (2 waves per SIMD at 8 waves): the accumulators and stage fragments take ~200 VGPRs.
template <int F, int LAY, int WR, int WC, int NBUF, bool SUMI>
__global__ __launch_bounds__(WR * WC * 64, WR * WC <= 4 ? 2 : 1) void mmql_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                               int M, int N, int K, void* __restrict__ out, int ldc_m,
                                                               int ldc_n) {
    mmql_body<F, LAY, WR, WC, NBUF, SUMI>(A, B, SUMI ? nullptr : (float*)out, SUMI ? (int32_t*)out : nullptr, M, N, K, ldc_m,
                                          ldc_n);
}

// Preconditions: whole stages (K % 128 == 0, the activation rows 16-B multiples), 16-B aligned A and B;
// LAY_ROWS: rows 16-B multiples and, when a stage segment is not (Q4_0 / Q5_0 / Q8_0), K % 256 == 0 so no
// window reaches past the rows' end (mmq_geom); per-lane offsets within 2 GiB.
template <int F, int LAY, int WR, int WC, int NBUF> inline bool mmql_shape_ok(const GemmArgs& g) {
    using G = mmql_geom<F, LAY, WR, WC, NBUF>;
    if (!G::FITS || g.nbw > 0 || g.lay != LAY) return false;
    if (g.M < 1 || g.N < 1 || g.K % (QK * MMQ_SB) != 0) return false;
    if (((uintptr_t)g.A & 15) != 0 || ((uintptr_t)g.B & 15) != 0) return false;
    const long nb = g.K / QK, AB = nb * Q8_1_BYTES;
    if (LAY != LAY_ROWS) {
        if ((long)tiled_fmt<F>::STG * (nb / MMQ_SB) * WR >= (1L << 31)) return false;
        if (LAY == LAY_TILED_ACT && (long)ACT_STG * (nb / MMQ_SB) * (G::BM / ACT_TILE) >= (1L << 31)) return false;
    } else {
        const long RB = nb * wfmt<F>::BB;
        if (RB % 16 != 0 || (G::RSB % 16 != 0 && g.K % 256 != 0)) return false;
        if (RB * G::BN >= (1L << 31)) return false;
    }
    if (AB * G::BM >= (1L << 31)) return false;
    if (g.ldc_m > INT32_MAX || g.ldc_n > INT32_MAX) return false;
    return true;
}

template <int F, int LAY, int WR, int WC, int NBUF, bool SUMI> hipError_t mmql_launch(const GemmArgs& g, hipStream_t st) {
    using G = mmql_geom<F, LAY, WR, WC, NBUF>;
    const long tiles = (long)((g.N + G::BN - 1) / G::BN) * ((g.M + G::BM - 1) / G::BM);
    const dim3 grid((unsigned)tiles, 1, 1);
    if (g.describe) {
        describe_kernel(g, "mmql F=%d BN=%d BM=%d W=%d NBUF=%d LAY=%d grid=%u", F, G::BN, G::BM, G::W, NBUF, LAY, grid.x);
        return hipSuccess;
    }
    const void* k = (const void*)mmql_kernel<F, LAY, WR, WC, NBUF, SUMI>;
    if (G::LDS > 64 * 1024) {
        static std::atomic<unsigned long long> attr_done{0};
        const hipError_t e = set_max_lds_once(k, 160 * 1024, attr_done);
        if (e != hipSuccess) return e;
    }
    void* out = SUMI ? (void*)g.sumi : (void*)g.C;
    hipLaunchKernelGGL((mmql_kernel<F, LAY, WR, WC, NBUF, SUMI>), grid, dim3(G::W * 64), G::LDS, st, (const uint8_t*)g.A,
                       (const uint8_t*)g.B, g.M, g.N, g.K, out, (int)g.ldc_m, (int)g.ldc_n);
    return hipGetLastError();
}

}  // namespace qg
