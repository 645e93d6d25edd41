// gemv_direct_probe.hip — single-launch GEMV: the staged product kernel (activation records in LDS
// behind one workgroup barrier) vs the direct-activation form (records built in registers from the
// lane's own Q8_1 blocks, no LDS, no barrier), plus a pure read of the same weight bytes in the
// GEMV's own per-lane unit shape. Not part of the product.
// Protocol as bench.py: a hipGraph of 64 launches, each on a different weight copy (> 256 MB
// Infinity Cache -> every launch streams from HBM), 9 interleaved rounds, median per launch.
// Outputs of every variant are compared bit for bit with the staged kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../llama.cpp-quant-gemm_amd/csrc \
//         -o gemv_direct_probe gemv_direct_probe.hip            (add -DQG_STAMPS: per-wave timelines)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "qg_gemv_kernel.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;
void qg::describe_kernel(const GemmArgs&, const char*, ...) {}

namespace qg {
// Direct-activation form (M <= 2, every lane at most one unit: K <= 32 * BPL * LPR). No LDS and no
// workgroup barrier: each lane loads the Q8_1 blocks of ITS unit (BPL * 36 B per activation row,
// contiguous across the lanes of a wave, L2-resident after the first wave of each XCD touches them)
// right before its weight unit, builds the same activation records build_act_record makes for the
// staged kernel in registers while the weight bytes are in flight, then runs the identical per-block
// dot and epilogue (block_dot / block_term_rec) and DPP row reduction. The staged kernel's 16 waves
// per workgroup waited at one barrier for two waves' activation loads and record stores; here each
// wave waits only for its own loads. SUMI: the same instantiation writes the per-block int32 dots
// instead of accumulating (the parity hook runs the product's decode and unit shape).
template <int F, int MT, int BPL, int LPR, int WGS, bool SUMI>
__global__ __launch_bounds__(WGS) void gemv_direct_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                          float* __restrict__ C, int32_t* __restrict__ sumi_out, int M,
                                                          int N, int K, long ldc_m, long ldc_n, long sA, long sB, long sC) {
    using G = gemv_geom<F, BPL>;
    static_assert(MT >= 1 && MT <= 2, "direct activations: M <= 2");
    QG_STAMP(t0);
    QG_CLK(c0);
    A = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(A) + blockIdx.y * sA);
    B += blockIdx.y * sB;
    C += blockIdx.y * sC;
    constexpr int RPW = 64 / LPR;
    constexpr int RPB = (WGS / 64) * RPW;
    const int nb = K / QK;
    const int U = nb / BPL;
    const int lane = threadIdx.x & 63;
    const int u = lane % LPR;  // this lane's unit (U <= LPR)
    const int row = blockIdx.x * RPB + (threadIdx.x >> 6) * RPW + lane / LPR;
    const bool row_ok = row < N;
    const bool u_ok = u < U;
    const int uu = u_ok ? u : 0;

    // 1) this unit's activation blocks of every row m (BPL * 9 dwords each), 2) the weight unit
    uint32_t ab[MT][BPL * 9];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const uint32_t* p = A + ((long)(m < M ? m : 0) * nb + (long)uu * BPL) * 9;
#pragma unroll
        for (int i = 0; i < BPL * 9; ++i) ab[m][i] = p[i];
    }
    uint32_t w[G::UDW];
    {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(B + ((long)(row_ok ? row : 0) * U + uu) * G::UB);
#pragma unroll
        for (int v = 0; v < G::UDW; ++v) w[v] = p[v];
    }
    // 3) activation records in registers (waits only for the activation loads, issued first)
    uint4 rec[BPL][MT][3];
#pragma unroll
    for (int bi = 0; bi < BPL; ++bi)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            uint32_t r[12];
            build_act_record<F>(&ab[m][9 * bi], r);
            rec[bi][m][0] = make_uint4(r[0], r[1], r[2], r[3]);
            rec[bi][m][1] = make_uint4(r[4], r[5], r[6], r[7]);
            rec[bi][m][2] = make_uint4(r[8], r[9], r[10], r[11]);
        }
    QG_STAMP(tb);
    QG_WAIT_STAMP(t1);

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;
    if (u_ok) {
        static_for<BPL>([&](auto BI) {
            constexpr int bi = decltype(BI)::value;
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                if (m < M) {
                    const uint32_t d = block_dot<F, bi>(w, rec[bi][m]);
                    if constexpr (SUMI) {
                        if (row_ok) sumi_out[((long)m * N + row) * nb + u * BPL + bi] = (int)(d - ACC_BIAS);
                    } else {
                        acc[m] += block_term_rec<F, bi>(w, d, rec[bi][m][2]);
                    }
                }
            }
        });
    }
    QG_STAMP(tc);
    if constexpr (!SUMI) {
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = group_sum_last<LPR>(acc[m]);
        if (row_ok && u == LPR - 1) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                if (m < M) C[m * ldc_m + row * ldc_n] = acc[m];
        }
    }
    QG_STAMP(t2);
    QG_CLK(c2);
    QG_STAMP_STORE(t0, tb, t1, tc, t2, c0, c2);
}

// The direct-activation form takes Q8_1 activations, M <= MT <= 2 and one unit per lane.
template <int F, int BPL, int LPR> inline bool gemv_direct_ok(const GemmArgs& g, int MT) {
    return g.ain == AIN_Q8_1 && g.M >= 1 && g.M <= MT && g.K % (QK * BPL) == 0 && g.K / QK / BPL <= LPR &&
           gemv_shape_ok<F, BPL>(g);
}

template <int F, int MT, int BPL, int LPR, int WGS, bool SUMI>
hipError_t gemv_direct_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    if (!gemv_direct_ok<F, BPL, LPR>(g, MT)) return hipErrorInvalidValue;
    const int grid = (g.N + RPB - 1) / RPB;
    hipLaunchKernelGGL((gemv_direct_kernel<F, MT, BPL, LPR, WGS, SUMI>), dim3(grid, g.batch), dim3(WGS), 0, st,
                       (const uint32_t*)g.A, (const uint8_t*)g.B, g.C, g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n, g.sA,
                       g.sB, g.sC);
    return hipGetLastError();
}

}  // namespace qg

// pure read of the weights in the direct kernel's shape: lane (row, u) reads its UB-byte unit
// ST: 0 no store (unless a magic value), 1 one plain store per row (lane 63), 2 nontemporal,
// 3 agent-scope write-through (sc1), 4 DPP row sum + plain store (the GEMV's tail)
template <int UB, int WGS, int ST = 0>
__global__ __launch_bounds__(WGS) void unit_read(const uint8_t* __restrict__ B, int N, int U, float* out) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (WGS / 64) + (threadIdx.x >> 6);
    if (row >= N) return;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(B + ((long)row * U + (lane < U ? lane : 0)) * UB);
    if constexpr (ST == 9) if (lane == 63) out[row] = (float)row;  // the row's store at the START
    uint32_t acc = 0;
#pragma unroll
    for (int v = 0; v < UB / 4; ++v) acc ^= p[v];
    if constexpr (ST == 0) {
        if (acc == 0x12345678u) out[row] = 1.0f;
    } else {
        float f = __uint_as_float(acc & 0x3FFFFFFFu);
        if constexpr (ST == 4 || ST == 5 || ST == 7 || ST == 8 || ST == 9) f = group_sum_last<64>(f);
        if constexpr (ST == 9) {
            if (f == 1.2345f) out[row] = f;
            return;
        }
        if constexpr (ST == 7) {  // one real store in the whole grid (row 0), the rest magic-guarded
            if (lane == 63 && (row == 0 || f == 1.2345f)) out[row] = f;
            return;
        }
        if constexpr (ST == 8) {  // one store per workgroup (its first row)
            if (lane == 63 && ((row & (WGS / 64 - 1)) == 0 || f == 1.2345f)) out[row] = f;
            return;
        }
        if constexpr (ST == 5) {  // DPP sum, no real store
            if (f == 1.2345f) out[row] = f;
            return;
        }
        if constexpr (ST == 6) {  // no reduction: every lane stores its own value to the row's slot
            out[row] = f;
            return;
        }
        if (lane == 63) {
            if constexpr (ST == 2) __builtin_nontemporal_store(f, out + row);
            else if constexpr (ST == 3) __hip_atomic_store(out + row, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else out[row] = f;
        }
    }
}

// the pure read + DPP + store with the product GEMV's kernel signature (13 arguments: the first 14
// dwords preloaded into SGPRs, the rest fetched by s_load)
template <int UB, int WGS>
__global__ __launch_bounds__(WGS) void unit_read_sig(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, long sA,
                                                     long sB, int M, int N, int K, float* __restrict__ C, long sC,
                                                     long ldc_m, long ldc_n, int32_t* __restrict__ sumi_out) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (WGS / 64) + (threadIdx.x >> 6);
    const int U = K / 64;
    if (row >= N) return;
    B += blockIdx.y * sB;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(B + ((long)row * U + (lane < U ? lane : 0)) * UB);
    uint32_t acc = 0;
#pragma unroll
    for (int v = 0; v < UB / 4; ++v) acc ^= p[v];
    float f = group_sum_last<64>(__uint_as_float(acc & 0x3FFFFFFFu));
    if (lane == 63) C[row * ldc_n] = f;
}

// signature probes: V = 1: (A, B, N, K, C) — 8 dwords, all preloaded; V = 2: (A, B, sA, sB, M, N, K, C) —
// 13 dwords, all preloaded, no s_load
template <int UB, int WGS>
__global__ __launch_bounds__(WGS) void unit_read_v1(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, int N,
                                                    int K, float* __restrict__ C) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (WGS / 64) + (threadIdx.x >> 6);
    const int U = K / 64;
    if (row >= N) return;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(B + ((long)row * U + (lane < U ? lane : 0)) * UB);
    uint32_t acc = 0;
#pragma unroll
    for (int v = 0; v < UB / 4; ++v) acc ^= p[v];
    float f = group_sum_last<64>(__uint_as_float(acc & 0x3FFFFFFFu));
    if (lane == 63) C[row] = f;
}
template <int UB, int WGS>
__global__ __launch_bounds__(WGS) void unit_read_v2(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, long sA,
                                                    long sB, int M, int N, int K, float* __restrict__ C) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (WGS / 64) + (threadIdx.x >> 6);
    const int U = K / 64;
    if (row >= N) return;
    B += blockIdx.y * sB;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(B + ((long)row * U + (lane < U ? lane : 0)) * UB);
    uint32_t acc = 0;
#pragma unroll
    for (int v = 0; v < UB / 4; ++v) acc ^= p[v];
    float f = group_sum_last<64>(__uint_as_float(acc & 0x3FFFFFFFu));
    if (lane == 63) C[row] = f;
}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }
static int bbytes(int f) { return f == FMT_Q4_0 ? 18 : f == FMT_Q4_1 ? 20 : f == FMT_Q5_0 ? 22 : f == FMT_Q5_1 ? 24 : 34; }

typedef std::function<hipError_t(const GemmArgs&, hipStream_t)> Fn;
struct Variant { std::string name; Fn fn; bool read; };

#ifdef QG_STAMPS
static void timeline(const char* name, int nwaves) {
    std::vector<unsigned long long> s(8 * (size_t)nwaves);
    CK(hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(g_stamps), s.size() * 8));
    unsigned long long t0 = ~0ull, tend = 0, tland = 0;
    for (int w = 0; w < nwaves; ++w) { t0 = std::min(t0, s[8 * w]); tend = std::max(tend, s[8 * w + 4]); tland = std::max(tland, s[8 * w + 2]); }
    std::vector<double> st, a, l, c, r;
    for (int w = 0; w < nwaves; ++w) {
        const unsigned long long* q = &s[8 * w];
        st.push_back((q[0] - t0) * 0.01); a.push_back((q[1] - q[0]) * 0.01); l.push_back((q[2] - q[1]) * 0.01);
        c.push_back((q[3] - q[2]) * 0.01); r.push_back((q[4] - q[3]) * 0.01);
    }
    auto pct = [](std::vector<double> v, double p) { std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
    auto row = [&](const char* n, const std::vector<double>& v) {
        printf("     %-26s p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f us\n", n, pct(v, .1), pct(v, .5), pct(v, .9), pct(v, 1.));
    };
    printf("   timeline %s: span %.2f us, last weights landed %.2f us after the first entry\n", name, (tend - t0) * 0.01,
           (tland - t0) * 0.01);
    row("entry offset", st);
    row("entry -> records ready", a);
    row("records -> weights landed", l);
    row("compute", c);
    row("reduce + store", r);
}
#endif

static void run_shape(int F, int M, int N, int K, std::vector<Variant>& vs, hipStream_t st) {
    const int nb = K / 32, bb = bbytes(F), L = 64;
    const size_t wb = (size_t)N * nb * bb;
    const int R = std::max(L, (int)((640UL << 20) / wb) + 1);
    std::vector<uint8_t> hw(wb);
    srand(7);
    for (size_t b = 0; b < (size_t)N * nb; ++b) {
        for (int j = 0; j < bb; ++j) hw[b * bb + j] = rand() & 0xFF;
        uint16_t d = f2h(0.01f + 0.09f * (float)rand() / (float)RAND_MAX);
        memcpy(&hw[b * bb], &d, 2);
        if (F == FMT_Q4_1 || F == FMT_Q5_1) { uint16_t m = f2h(-0.5f * (float)rand() / (float)RAND_MAX); memcpy(&hw[b * bb + 2], &m, 2); }
    }
    std::vector<uint8_t> ha((size_t)M * nb * 36);
    for (size_t b = 0; b < (size_t)M * nb; ++b) {
        uint16_t d = f2h(0.008f), s = f2h((rand() % 2000 - 1000) / 100.0f);
        memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &s, 2);
        for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
    }
    std::vector<uint8_t*> W(R);
    for (auto& p : W) { CK(hipMalloc(&p, wb)); CK(hipMemcpy(p, hw.data(), wb, hipMemcpyHostToDevice)); }
    uint8_t* A; float* C;
    CK(hipMalloc(&A, ha.size())); CK(hipMemcpy(A, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&C, (size_t)M * N * 4));
    auto args = [&](int copy) {
        GemmArgs g; g.A = A; g.B = W[copy % R]; g.C = C; g.M = M; g.N = N; g.K = K; g.wtype = F; g.ldc_m = N; g.ldc_n = 1;
        return g;
    };
    // outputs vs the first variant
    std::vector<float> ref((size_t)M * N), out((size_t)M * N);
    for (size_t k = 0; k < vs.size(); ++k) {
        if (vs[k].read) continue;
        CK(hipMemset(C, 0xFF, (size_t)M * N * 4));
        CK(vs[k].fn(args(0), st));
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(k == 0 ? ref.data() : out.data(), C, (size_t)M * N * 4, hipMemcpyDeviceToHost));
        if (k > 0 && memcmp(ref.data(), out.data(), ref.size() * 4) != 0) printf("  !! %s differs from %s\n", vs[k].name.c_str(), vs[0].name.c_str());
    }
    std::vector<hipGraphExec_t> ge(vs.size());
    for (size_t k = 0; k < vs.size(); ++k) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < L; ++i) CK(vs[k].fn(args(i), st));
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge[k], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 11; ++r)
        for (size_t k = 0; k < vs.size(); ++k) {
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge[k], st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t[k].push_back(ms * 1000.f / L);
        }
    const double bytes = (double)wb + (double)M * nb * 36 + (double)M * N * 4;
    printf("fmt=%d M=%d N=%d K=%d  %.0f algorithmic B per launch, graph of %d launches over %d copies\n", F, M, N, K, bytes, L, R);
    for (size_t k = 0; k < vs.size(); ++k) {
        std::sort(t[k].begin(), t[k].end());
        const double med = t[k][t[k].size() / 2];
        printf("  %-34s %7.3f us  (p10 %6.3f p90 %6.3f)  frac %.3f\n", vs[k].name.c_str(), med, t[k][t[k].size() / 10],
               t[k][(t[k].size() * 9) / 10], bytes / med / 1e3 / 8000.0);
    }
#ifdef QG_STAMPS
    for (size_t k = 0; k < vs.size(); ++k) {
        if (vs[k].read) continue;
        for (int i = 0; i < 8; ++i) CK(vs[k].fn(args(i), st));  // the last launch's stamps survive
        CK(hipStreamSynchronize(st));
        const int RPB = vs[k].name.find("wg512") != std::string::npos ? 8 : vs[k].name.find("wg256") != std::string::npos ? 4 : 16;
        timeline(vs[k].name.c_str(), ((N + RPB - 1) / RPB) * RPB);
    }
#endif
    fflush(stdout);
    for (auto x : ge) CK(hipGraphExecDestroy(x));
    for (auto p : W) CK(hipFree(p));
    CK(hipFree(A)); CK(hipFree(C));
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
}

// the product's M = 1 loop-free kernel with its ABL ablation bits (qg_gemv_kernel.hpp)
template <int F, int ABL> static hipError_t abl_launch(const GemmArgs& g, hipStream_t st) {
    const size_t lds = (ABL & 1) ? 0 : gemv_lds_bytes<F, 2>(g.M, g.K);
    hipLaunchKernelGGL((gemv_kernel<F, 1, 2, 64, 1024, false, AIN_Q8_1, false, true, true, ABL>), dim3((g.N + 15) / 16, 1),
                       dim3(1024), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.sA, g.sB, g.M, g.N, g.K, g.C, g.sC,
                       g.ldc_m, g.ldc_n, g.sumi);
    return hipGetLastError();
}

template <int F, int MT> static std::vector<Variant> variants(bool with_read) {
    std::vector<Variant> vs;
    vs.push_back({"staged bpl2 lpr64 wg1024 (product)", gemv_launch<F, MT, 2, 64, 1024, false, AIN_Q8_1, false, true>, false});
    if (MT == 1 && getenv("QG_ABL")) {
        vs.push_back({"product, neither (staging, dot)", abl_launch<F, 3>, false});
        vs.push_back({"product, nt stores", abl_launch<F, 4>, false});
        vs.push_back({"product, sc1 stores", abl_launch<F, 8>, false});
        vs.push_back({"product, neither + nt stores", abl_launch<F, 7>, false});
        constexpr int UB = 2 * wfmt<F>::BB;
#define RD(ST, NAME) vs.push_back({NAME, [](const GemmArgs& g, hipStream_t s) { \
            hipLaunchKernelGGL((unit_read<UB, 1024, ST>), dim3((g.N + 15) / 16), dim3(1024), 0, s, (const uint8_t*)g.B, g.N, g.K / 64, g.C); \
            return hipGetLastError(); }, true});
        RD(0, "pure read (no store)")
        RD(4, "pure read + DPP sum + store")
        RD(5, "pure read + DPP sum, no store")
        RD(6, "pure read + 64-lane store, no DPP")
        RD(7, "pure read + DPP, ONE store per grid")
        RD(8, "pure read + DPP, one store per WG")
        RD(9, "pure read + DPP, per-row store at START")
        vs.push_back({"pure read + DPP + store, product signature", [](const GemmArgs& g, hipStream_t s) {
            hipLaunchKernelGGL((unit_read_sig<UB, 1024>), dim3((g.N + 15) / 16), dim3(1024), 0, s, (const uint32_t*)g.A,
                               (const uint8_t*)g.B, g.sA, g.sB, g.M, g.N, g.K, g.C, g.sC, g.ldc_m, g.ldc_n, g.sumi);
            return hipGetLastError(); }, true});
#undef RD
    }
    vs.push_back({"direct bpl2 lpr64 wg1024", gemv_direct_launch<F, MT, 2, 64, 1024, false>, false});
    vs.push_back({"direct bpl2 lpr64 wg512", gemv_direct_launch<F, MT, 2, 64, 512, false>, false});
    vs.push_back({"direct bpl2 lpr64 wg256", gemv_direct_launch<F, MT, 2, 64, 256, false>, false});
    vs.push_back({"direct bpl2 lpr64 wg128", gemv_direct_launch<F, MT, 2, 64, 128, false>, false});
    vs.push_back({"direct bpl4 lpr32 wg512", gemv_direct_launch<F, MT, 4, 32, 512, false>, false});
    vs.push_back({"direct bpl4 lpr32 wg256", gemv_direct_launch<F, MT, 4, 32, 256, false>, false});
    if (with_read) {
        constexpr int UB = 2 * wfmt<F>::BB;
        vs.push_back({"pure read, unit shape wg1024", [](const GemmArgs& g, hipStream_t s) {
                          hipLaunchKernelGGL((unit_read<UB, 1024>), dim3((g.N + 15) / 16), dim3(1024), 0, s,
                                             (const uint8_t*)g.B, g.N, g.K / 64, g.C);
                          return hipGetLastError(); }, true});
        vs.push_back({"pure read, unit shape wg256", [](const GemmArgs& g, hipStream_t s) {
                          hipLaunchKernelGGL((unit_read<UB, 256>), dim3((g.N + 3) / 4), dim3(256), 0, s,
                                             (const uint8_t*)g.B, g.N, g.K / 64, g.C);
                          return hipGetLastError(); }, true});
        vs.push_back({"read+DPP+store, sig (A,B,N,K,C)", [](const GemmArgs& g, hipStream_t s) {
            hipLaunchKernelGGL((unit_read_v1<UB, 1024>), dim3((g.N + 15) / 16), dim3(1024), 0, s, (const uint32_t*)g.A,
                               (const uint8_t*)g.B, g.N, g.K, g.C);
            return hipGetLastError(); }, true});
        vs.push_back({"read+DPP+store, sig 13 dw preloaded", [](const GemmArgs& g, hipStream_t s) {
            hipLaunchKernelGGL((unit_read_v2<UB, 1024>), dim3((g.N + 15) / 16), dim3(1024), 0, s, (const uint32_t*)g.A,
                               (const uint8_t*)g.B, g.sA, g.sB, g.M, g.N, g.K, g.C);
            return hipGetLastError(); }, true});
    }
    return vs;
}

int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    { auto v = variants<FMT_Q4_0, 1>(true); run_shape(FMT_Q4_0, 1, 4096, 4096, v, st); }
    if (getenv("QG_ABL")) return 0;
    { auto v = variants<FMT_Q4_0, 1>(false); run_shape(FMT_Q4_0, 1, 4000, 4096, v, st); }
    { auto v = variants<FMT_Q4_0, 2>(false); run_shape(FMT_Q4_0, 2, 4096, 4096, v, st); }
    { auto v = variants<FMT_Q4_1, 1>(true); run_shape(FMT_Q4_1, 1, 4096, 4096, v, st); }
    { auto v = variants<FMT_Q5_0, 1>(true); run_shape(FMT_Q5_0, 1, 4096, 4096, v, st); }
    { auto v = variants<FMT_Q5_1, 1>(true); run_shape(FMT_Q5_1, 1, 4096, 4096, v, st); }
    { auto v = variants<FMT_Q4_0, 1>(false); run_shape(FMT_Q4_0, 1, 32000, 4096, v, st); }
    return 0;
}
