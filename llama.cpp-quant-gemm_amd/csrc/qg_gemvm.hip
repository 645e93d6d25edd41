// qg_gemvm.hip — small-batch decode (M = 2..4 tokens) on the tiled weight layout with the matrix cores,
// round 6 (the reference's published batch-decode shapes, 4096 x M x 14336).
// C[M,N] = A_q8_1[M,K] . B[N,K]^T (include/gemm_reference.h:175-222), activation-major.
//
// Why. The GEMVs (qg_gemv_kernel.hpp, qg_gemvt.hip) compute every (row, token, block) dot on the VALU, so
// their cost grows with M while the weight bytes do not (K = 14336: M = 4 11.2 us against 7.6 at M = 1). On
// the tiled layout a lane's 16-B piece of the QS plane (row r16, k-slot q: dword q of the stage's 4 blocks)
// IS its operand of v_mfma_i32_16x16x32_i8 (the prefill kernels' fragment order, qg_mmq_kernel.hpp), so the
// weights go from HBM straight into MFMA operands, one MFMA per (16 rows, block).
//
// Block-diagonal columns. The prefill's 16 x 16 tile gives 16 token columns; at M <= 8 most would be waste,
// and the per-block scaling (one v_fmac per element and block) would cost 4x-8x the useful VALU. Here the 16
// columns are (block b < BPC, token t < MP) with MP = M rounded up to a power of two and BPC = 16 / MP:
// column j = b MP + t. The BPC MFMAs of a group accumulate into ONE tile, MFMA b seeing the activation
// fragments only in the columns of block b (zeros elsewhere), so column j's int32 result is exactly block
// j / MP's dot for token j % MP (the reference's sumi, bit for bit). The scale products d_w d_a of the whole
// group come from one f16 MFMA with block-diagonal d_a (the A operand: the rows' 4 f16 d of a stage, the
// tiled layout's SC entry as it lies), the offset term d_w c s_a / m_w s_a from one compensation MFMA per
// group; the epilogue is one fma per element and group (4 per lane), every element useful at M = MP. The
// BPC partial columns of a token are summed once, at the end (xor butterfly, fixed order).
//
// Work: a workgroup owns a 16-row half tile and all of K; its W waves split the stages, wave w taking stages
// w NU .. w NU + NU - 1, every weight piece of them in flight before anything waits (a ring of RS stages for
// the formats whose pieces take more registers). Lane (r16, q) loads, per stage, its 16-B piece (the load
// instruction: the half tile's 1 KB of the stage, 8 whole lines) and its row's scales. Each wave stages its
// stages' activation blocks (raw Q8_1, MP tokens) in a wave-private LDS region, in exactly the column order
// (record g 16 + j = group g, column j), behind a wave-local fence; the W partial tiles meet through LDS in
// fixed wave order. Parity: per-block sumi bit-exact (the sumi hook runs this instantiation); outputs within
// the reassociation bound of the MFMA epilogue (oracle.reassoc_tol, as the prefill kernels).
//
// Two things found on the way (round 6, tools/dbg_gemvm*.py on an MI355X). (1) The first version zeroed the
// d|s dword of padding-block records with a v_cndmask right before its ds_write; under load (CUs holding
// several workgroups: rows past the first dispatch round) some records reached the LDS with a wrong d|s
// dword — sumi exact, sum of sumi exact, the scale products (and the compensation) wrong, 40 % of the
// outputs off, some inf — in whichever format / MP the register assignment put that v_cndmask next to
// the store. The records are now stored straight from the load registers and the padding blocks' d|s is
// zeroed where the records are read. (2) hipcc's builtins let an f16 MFMA take the registers an i8 MFMA
// issued just before reads as SrcC (`i8 v[22:25] <- C bias; i8 v[14:17] <- C v[22:25]; f16 v[22:25]`, 0
// wait states); never shown to be wrong by itself, but each group's MFMAs are ONE asm statement all the
// same: dd first, the first i8 MFMA from the bias, the rest accumulating in place (vdst == SrcC), every
// destination early-clobber, 10 wait states before the VALU reads (as fast as the builtins;
// tests/test_isa_hazards.py checks the shipped code object for cross-opcode MFMA register reuse).
#include "qg_mmq_kernel.hpp"

namespace qg {

namespace {

#ifndef QG_GEMVM_LEAN  // (A/B builds: 0 = the first form — cc copied from the bias, s_nop 1 inside the chain,
#define QG_GEMVM_LEAN 1  // 16 wait states at the end; 1-4 % slower, profiles/r06_tuning/r6u_ab_gemvm_lean_groups.txt)
#endif

typedef _Float16 gm_f16x4 __attribute__((ext_vector_type(4)));
typedef float gm_f32x4 __attribute__((ext_vector_type(4)));

template <int F, int NU, int MP, bool SUMI, bool TA>
__global__ __launch_bounds__(1024) void gemvm_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, int M,
                                                     int N, int K, void* __restrict__ out, int ldc_m, int ldc_n) {
    using T = wfmt<F>;
    using TF = tiled_fmt<F>;
    constexpr bool HAS_M = T::MOFF >= 0, HAS_S = F != FMT_Q8_0;
    constexpr float CFAC = F == FMT_Q4_0 ? -8.0f : F == FMT_Q5_0 ? -16.0f : 1.0f;
    constexpr int BPC = 16 / MP;              // blocks per accumulator tile
    constexpr int NBW = NU * MMQ_SB;          // blocks per wave
    constexpr int NG = NBW / BPC;             // tiles (groups) per wave
    constexpr int SPAN = BPC < 4 ? 4 : BPC;   // blocks behind one scale operand (whole stages)
    constexpr int NIT = (NBW * MP + 63) / 64; // staged activation blocks per lane
    static_assert(NBW % BPC == 0 && SPAN <= 16, "groups of whole blocks, scale operand of <= 4 stages");
    // register ring of weight stages: all NU of them under the 128-VGPR cap of 1024-thread workgroups, but 4
    // at NU = 8 for Q5_x (their qh pieces) and for 8 token columns (36 staged dwords): scratch otherwise
    constexpr int RS = (F == FMT_Q5_0 || F == FMT_Q5_1 || MP == 8) && NU > 4 ? 4 : NU;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    const int nb = K / QK, H = (nb + MMQ_SB - 1) / MMQ_SB;
    const int W = blockDim.x >> 6;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int r16 = lane & 15, q = lane >> 4;
    const int cb = r16 / MP, ct = r16 % MP;  // this lane's column: block within the group, token
    const int tile = gridDim.x <= 512 ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int n0 = tile * 16;  // the workgroup's 16 rows: a half tile
    const int rr = n0 % TILE_ROWS + r16;  // this lane's row (A operand) within its 32-row tile
    const uint8_t* tb = B + (long)(n0 / TILE_ROWS) * H * TF::STG;
    const int oqs = (n0 % TILE_ROWS / 16) * 64 * TF::QSL + (q * 16 + r16) * 16;  // piece (q, r16) in a stage run
    const int h0 = wave * NU;
    const int nreal = TA ? H * MMQ_SB : nb;  // blocks with bytes behind them (TA: the layout's zero padding)
    uint32_t* wl = lds + wave * (NBW * MP * 9);  // the wave's records [stage-local block][token][9]

    // 1) this lane's staged activation blocks (item it = block it / MP, token it % MP), then the weights.
    //    Tokens M..MP-1 repeat token M - 1 (columns nobody stores); blocks past the real ones read block 0
    //    and get d = s = 0 where the records are read (an exact +0 term whatever their codes; the records are
    //    stored straight from the load registers, no VALU in between).
    uint32_t ab[NIT][9];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
        const int it = lane + 64 * k, gb = h0 * MMQ_SB + it / MP, t = min(it % MP, M - 1);
        long src = ((long)t * nb + gb) * 9;
        if constexpr (TA) src = (((long)(t / ACT_TILE) * H + (gb >> 2)) * ACT_TILE + t % ACT_TILE) * 36 + (gb & 3) * 9;
        const bool ok = gb < nreal;
        if (!ok) src = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) ab[k][i] = A[src + i];
    }
    struct wst {
        uint4 qs, qs8, qh, sc;
    };
    wst ring[RS];
    auto load = [&](int j, wst& s) {
        const uint8_t* st = tb + (long)min(h0 + j, H - 1) * TF::STG;  // (stages past H: zero activations)
        s.qs = *reinterpret_cast<const uint4*>(st + oqs);
        if constexpr (T::Q8) s.qs8 = *reinterpret_cast<const uint4*>(st + oqs + 1024);
        if constexpr (T::QH >= 0) s.qh = *reinterpret_cast<const uint4*>(st + TF::OQH + rr * 16);
        if constexpr (HAS_M) {
            s.sc = *reinterpret_cast<const uint4*>(st + TF::OSC + rr * 16);
        } else {
            const uint2 v = *reinterpret_cast<const uint2*>(st + TF::OSC + rr * 8);
            s.sc = make_uint4(v.x, v.y, 0u, 0u);
        }
    };
#pragma unroll
    for (int j = 0; j < RS; ++j) load(j, ring[j]);
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
        const int it = lane + 64 * k;
        if (NIT * 64 == NBW * MP || it < NBW * MP) {
            uint32_t* rec = wl + it * 9;
#pragma unroll
            for (int i = 0; i < 9; ++i) rec[i] = ab[k][i];
        }
    }
    // written by other lanes of this wave: a wave's LDS operations execute in order (qg_gemvt.hip)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    const v4i bias = {MMQ_BIAS, MMQ_BIAS, MMQ_BIAS, MMQ_BIAS};
    const gm_f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    gm_f32x4 c2 = z4;
    // 2) per group: operands, the MFMAs, the epilogue
    static_for<NG>([&](auto GC) {
        constexpr int g = decltype(GC)::value;
        constexpr int b0 = g * BPC;               // the group's first block (wave-local)
        constexpr int s0 = b0 / MMQ_SB;           // its stage
        constexpr int kb = b0 % SPAN;             // its first block within the scale operand's span
        constexpr int sp0 = (b0 / SPAN) * (SPAN / MMQ_SB);  // the span's first stage
        constexpr int s1 = (b0 + BPC - 1) / MMQ_SB;         // the group's last stage
        // the lane's activation column: record g 16 + r16
        const uint32_t* rec = wl + (g * 16 + r16) * 9;
        const unsigned long bq = ((unsigned long)rec[5 + q] << 32) | rec[1 + q];
        const uint32_t ds = h0 * MMQ_SB + b0 + cb < nreal ? rec[0] : 0u;  // (blocks past the real ones: +0)
        // weight fragments of the group's blocks
        long af[BPC];
#pragma unroll
        for (int b = 0; b < BPC; ++b) {
            const int j = (b0 + b) / MMQ_SB, bb = (b0 + b) % MMQ_SB;
            const wst& s = ring[j % RS];
            const uint32_t qv[4] = {s.qs.x, s.qs.y, s.qs.z, s.qs.w}, q8v[4] = {s.qs8.x, s.qs8.y, s.qs8.z, s.qs8.w};
            const uint32_t qhv[4] = {s.qh.x, s.qh.y, s.qh.z, s.qh.w};
            uint32_t lo, hi;
            if constexpr (T::Q8) {
                lo = qv[bb];
                hi = q8v[bb];
            } else {
                lo = qv[bb] & 0x0F0F0F0Fu;
                hi = (qv[bb] >> 4) & 0x0F0F0F0Fu;
            }
            if constexpr (T::QH >= 0) {
                lo |= spread4_bit4((qhv[bb] >> (4 * q)) & 0xFu);
                hi |= spread4_bit4((qhv[bb] >> (16 + 4 * q)) & 0xFu);
            }
            af[b] = (long)(((unsigned long)hi << 32) | lo);
        }
        // scale operands: A lane q carries span blocks 4q..4q+3 (stage sp0 + q: its 4 f16 d, or m), B the
        // column's d_a / s_a at slot kb + cb (lane group q = slot / 4)
        unsigned long ad = 0, ax = 0;
#pragma unroll
        for (int x = 0; x < SPAN / MMQ_SB; ++x) {
            const uint4 sc = ring[(sp0 + x) % RS].sc;
            const unsigned long d = ((unsigned long)sc.y << 32) | sc.x;
            const unsigned long mm = HAS_M ? (((unsigned long)sc.w << 32) | sc.z) : d;
            ad = q == x ? d : ad;
            ax = q == x ? mm : ax;
        }
        const int kpos = kb + cb;
        const bool mine = q == (kpos >> 2);
        const unsigned long bd = mine ? (unsigned long)(ds & 0xFFFFu) << (16 * (kpos & 3)) : 0ul;
        const unsigned long bs = mine ? (unsigned long)(ds >> 16) << (16 * (kpos & 3)) : 0ul;
        // the ring slots of the stages this group finished take their next stages
#pragma unroll
        for (int j = s0; j <= s1; ++j)
            if ((j + 1) * MMQ_SB <= b0 + BPC && j + RS < NU) load(j + RS, ring[j % RS]);
        __builtin_amdgcn_sched_barrier(0);
        // The group's MFMAs in ONE asm statement (see the header's hazard note): dd first, the BPC i8 MFMAs
        // accumulating into one tile, the compensation MFMA in place, then the wait states before any VALU
        // reads a result; early-clobber dd / cc and in/out c2 keep every destination off every operand.
        long bsel[BPC];
#pragma unroll
        for (int b = 0; b < BPC; ++b) bsel[b] = cb == b ? (long)bq : 0l;
        gm_f32x4 dd;
#if QG_GEMVM_LEAN
        // the chain's first MFMA takes the bias as its SrcC (no per-group copy into cc), the in-place
        // accumulations back to back (the matrix pipe's own SrcC dependency), 10 wait states at the end
        v4i cc;
#define GM_CC0 "v_mfma_i32_16x16x32_i8 %[cc], %[a0], %[b0], %[bias]\n\t"
#define GM_CC(i) "v_mfma_i32_16x16x32_i8 %[cc], %[a" #i "], %[b" #i "], %[cc]\n\t"
#define GM_TAIL "v_mfma_f32_16x16x16_f16 %[c2], %[ax], %[bs], %[c2]\n\ts_nop 7\n\ts_nop 1"
#define GM_OUT [dd] "=&v"(dd), [cc] "=&v"(cc), [c2] "+v"(c2)
#define GM_IN [ad] "v"(ad), [bd] "v"(bd), [ax] "v"(ax), [bs] "v"(bs), [bias] "v"(bias)
#else
        v4i cc = bias;
#define GM_CC(i) "v_mfma_i32_16x16x32_i8 %[cc], %[a" #i "], %[b" #i "], %[cc]\n\ts_nop 1\n\t"
#define GM_CC0 GM_CC(0)
#define GM_TAIL "v_mfma_f32_16x16x16_f16 %[c2], %[ax], %[bs], %[c2]\n\ts_nop 7\n\ts_nop 7"
#define GM_OUT [dd] "=&v"(dd), [cc] "+v"(cc), [c2] "+v"(c2)
#define GM_IN [ad] "v"(ad), [bd] "v"(bd), [ax] "v"(ax), [bs] "v"(bs)
#endif
#define GM_HEAD "s_nop 2\n\tv_mfma_f32_16x16x16_f16 %[dd], %[ad], %[bd], 0\n\t"
        if constexpr (BPC == 4) {
            asm volatile(GM_HEAD GM_CC0 GM_CC(1) GM_CC(2) GM_CC(3) GM_TAIL
                         : GM_OUT
                         : GM_IN, [a0] "v"(af[0]), [b0] "v"(bsel[0]), [a1] "v"(af[1]), [b1] "v"(bsel[1]), [a2] "v"(af[2]),
                           [b2] "v"(bsel[2]), [a3] "v"(af[3]), [b3] "v"(bsel[3]));
        } else if constexpr (BPC == 2) {
            asm volatile(GM_HEAD GM_CC0 GM_CC(1) GM_TAIL
                         : GM_OUT
                         : GM_IN, [a0] "v"(af[0]), [b0] "v"(bsel[0]), [a1] "v"(af[1]), [b1] "v"(bsel[1]));
        } else {
            static_assert(BPC == 8, "MP in {2, 4, 8}");
            asm volatile(GM_HEAD GM_CC0 GM_CC(1) GM_CC(2) GM_CC(3) GM_CC(4) GM_CC(5) GM_CC(6) GM_CC(7) GM_TAIL
                         : GM_OUT
                         : GM_IN, [a0] "v"(af[0]), [b0] "v"(bsel[0]), [a1] "v"(af[1]), [b1] "v"(bsel[1]), [a2] "v"(af[2]),
                           [b2] "v"(bsel[2]), [a3] "v"(af[3]), [b3] "v"(bsel[3]), [a4] "v"(af[4]), [b4] "v"(bsel[4]),
                           [a5] "v"(af[5]), [b5] "v"(bsel[5]), [a6] "v"(af[6]), [b6] "v"(bsel[6]), [a7] "v"(af[7]),
                           [b7] "v"(bsel[7]));
        }
#undef GM_CC
#undef GM_CC0
#undef GM_HEAD
#undef GM_TAIL
#undef GM_OUT
#undef GM_IN
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SUMI) {
            const int gb = (h0 * MMQ_SB) + b0 + cb;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int n = n0 + 4 * q + e;
                if (ct < M && n < N && gb < nb) static_cast<int32_t*>(out)[((long)ct * N + n) * nb + gb] = cc[e] - MMQ_BIAS;
            }
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(dd[e], __int_as_float(cc[e]) - MMQ_BIAS_F, acc[e]);
        }
        __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (!SUMI) {
        if constexpr (HAS_S) {
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(CFAC, c2[e], acc[e]);
        }
        // the BPC block columns of each token (lanes r16 ^ MP, ^ 2 MP, ...: every lane of the set ends with
        // the same bits), then the waves' partial tiles in fixed wave order
#pragma unroll
        for (int o = MP; o < 16; o <<= 1)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] += __shfl_xor(acc[e], o);
        float* red = reinterpret_cast<float*>(lds + W * (NBW * MP * 9));
#pragma unroll
        for (int e = 0; e < 4; ++e) red[(wave * 4 + e) * 64 + lane] = acc[e];
        __syncthreads();
        for (int idx = threadIdx.x; idx < 256; idx += W * 64) {
            const int e = idx >> 6, ln = idx & 63;
            const int m = ln & 15, n = n0 + 4 * (ln >> 4) + e;
            if (m < M && n < N) {  // (m < M <= MP: column m is block 0 of token m)
                float v = red[idx];
                for (int w = 1; w < W; ++w) v += red[(w * 4 + e) * 64 + ln];
                static_cast<float*>(out)[(long)m * ldc_m + (long)n * ldc_n] = v;
            }
        }
    }
}

// Token columns (M rounded up to a power of two) and stages per lane: 4 up to K/32 = 256, then 8 (at most 16
// waves: K <= 16384, as the tiled decode GEMV). 4 rather than 2 stages per lane at K/32 <= 128
// (profiles/r06_tuning/r6q_ab_gemvm_nu_m2.txt): M = 4 N = K = 4096 4.53 -> 4.38 us, M = 3 4.50 -> 4.30, M = 4
// N = 11008 8.20 -> 7.03; M = 2 stays with the tiled decode GEMV up to K/32 = 256 either way (4.14 vs 4.45 at
// K = 4096, 6.03 vs 5.99 at 8192).
#ifndef QG_GEMVM_MAXM  // (A/B builds: 8 = also M = 5..8 with 8 token columns)
#define QG_GEMVM_MAXM 4
#endif
inline int gemvm_mp(int M) { return M <= 2 ? 2 : M <= 4 ? 4 : 8; }
#ifndef QG_GEMVM_NU_SMALL  // (A/B builds: stages per lane up to K/32 = 128)
#define QG_GEMVM_NU_SMALL 4
#endif
#ifndef QG_GEMVM_M2_MIN_NB  // (A/B builds: M = 2 from this K/32 on)
#define QG_GEMVM_M2_MIN_NB 257
#endif
inline int gemvm_nu(int, int H) { return H <= 32 ? QG_GEMVM_NU_SMALL : H <= 64 ? 4 : 8; }
inline size_t gemvm_lds(int M, int H) {
    const int NU = gemvm_nu(M, H), W = (H + NU - 1) / NU;
    return ((size_t)W * NU * MMQ_SB * gemvm_mp(M) * 9 + (size_t)W * 256) * 4;
}

template <int F, int NU, int MP> hipError_t gemvm_launch(const GemmArgs& g, hipStream_t st) {
    const int nb = g.K / QK, H = (nb + MMQ_SB - 1) / MMQ_SB;
    const int W = (H + NU - 1) / NU;
    const int grid = (g.N + 15) / 16;
    const size_t lds = gemvm_lds(g.M, H);
    const bool ta = g.lay == LAY_TILED_ACT;
    if (g.describe) {
        describe_kernel(g, "gemvm F=%d NU=%d MP=%d W=%d TA=%d grid=%d", F, NU, MP, W, (int)ta, grid);
        return hipSuccess;
    }
    if (W > 16 || lds > 160 * 1024) return hipErrorInvalidValue;
    auto k = g.sumi ? (ta ? gemvm_kernel<F, NU, MP, true, true> : gemvm_kernel<F, NU, MP, true, false>)
                    : (ta ? gemvm_kernel<F, NU, MP, false, true> : gemvm_kernel<F, NU, MP, false, false>);
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

template <int F, int NU> hipError_t gemvm_m(const GemmArgs& g, hipStream_t st) {
    switch (gemvm_mp(g.M)) {
        case 2: return gemvm_launch<F, NU, 2>(g, st);
#if QG_GEMVM_MAXM > 4
        case 8: return gemvm_launch<F, NU, 8>(g, st);
#endif
        default: return gemvm_launch<F, NU, 4>(g, st);
    }
}

template <int F> hipError_t gemvm_f(const GemmArgs& g, hipStream_t st) {
    switch (gemvm_nu(g.M, (g.K / QK + MMQ_SB - 1) / MMQ_SB)) {
        case 2: return gemvm_m<F, 2>(g, st);
        case 4: return gemvm_m<F, 4>(g, st);
        default: return gemvm_m<F, 8>(g, st);
    }
}

}  // namespace

// 3 <= M <= 4 tokens, and M = 2 from K/32 > 256 (8 stages per lane), where it beats the tiled decode GEMV
// (profiles/r06_tuning/r6m_gemvm_ab.txt, N = 4096: M = 2 K = 14336 8.66 -> 8.27 us, M = 4 11.38 -> 9.49, Q8_0
// M = 4 14.86 -> 13.53, Q4_1 M = 3 11.69 -> 9.77; M = 2 K = 4096 4.21 -> 4.49 stays with gemvt; M = 5..8 with
// 8 token columns ran 2x the MFMA kernel's time and stay with it). One product with 32-bit output strides;
// B_tiled 16-B and A 4-B aligned; the wave records within the LDS; at most 16 waves.
bool gemvm_eligible(const GemmArgs& g) {
    if (!(g.lay == LAY_TILED || g.lay == LAY_TILED_ACT) || g.M < 2 || g.M > QG_GEMVM_MAXM || g.N < 1 || g.K % QK != 0) return false;
    if (g.M == 2 && g.K / QK < QG_GEMVM_M2_MIN_NB) return false;
    if (g.batch != 1 || g.group || g.ain != AIN_Q8_1 || ((uintptr_t)g.B & 15) != 0 || ((uintptr_t)g.A & 3) != 0) return false;
    if (g.ldc_m > INT32_MAX || g.ldc_n > INT32_MAX || g.ldc_m < 0 || g.ldc_n < 0) return false;
    if (!(g.wtype == FMT_Q4_0 || g.wtype == FMT_Q4_1 || g.wtype == FMT_Q5_0 || g.wtype == FMT_Q5_1 || g.wtype == FMT_Q8_0))
        return false;
    const int H = (g.K / QK + MMQ_SB - 1) / MMQ_SB, NU = gemvm_nu(g.M, H), W = (H + NU - 1) / NU;
    return W <= 16 && gemvm_lds(g.M, H) <= 160 * 1024 && (long)g.M * g.N * (g.K / QK) < (1L << 62);
}

hipError_t launch_gemvm(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return gemvm_f<FMT_Q4_0>(g, st);
        case FMT_Q4_1: return gemvm_f<FMT_Q4_1>(g, st);
        case FMT_Q5_0: return gemvm_f<FMT_Q5_0>(g, st);
        case FMT_Q5_1: return gemvm_f<FMT_Q5_1>(g, st);
        case FMT_Q8_0: return gemvm_f<FMT_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
