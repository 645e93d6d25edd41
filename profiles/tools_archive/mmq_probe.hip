// mmq_probe.hip — tuning sweep for the prefill (M > 8) kernels: the current product kernel
// (qg_gemm_mfma.hip, via the C-ABI dispatch) vs mmq_kernel (qg_mmq_kernel.hpp) configurations.
// Not part of the product. Interleaved rounds, cold (rotating > 256 MB of weights) medians.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../llama.cpp-quant-gemm_amd/csrc \
//         -o mmq_probe mmq_probe.hip -L../llama.cpp-quant-gemm_amd/quant_gemm -lqg_hip \
//         -Wl,-rpath,'$ORIGIN/../llama.cpp-quant-gemm_amd/quant_gemm' && ./mmq_probe
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "qg_mmq_kernel.hpp"
#include "mmq_tile_experiment.hpp"  // measured slower than the product, kept for the record  // round-1 product kernel (A/B baseline)
#include "../include/qg/qg.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }
static int block_bytes(int f) { return f == FMT_Q4_0 ? 18 : f == FMT_Q4_1 ? 20 : f == FMT_Q5_0 ? 22 : f == FMT_Q8_0 ? 34 : 24; }

typedef std::function<hipError_t(const GemmArgs&, hipStream_t)> LaunchFn;
struct Variant { std::string name; LaunchFn fn; };

int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    struct S { int F, M, N, K; };
    const S shapes[] = {{FMT_Q4_0, 64, 4096, 4096}, {FMT_Q4_0, 96, 4096, 4096}, {FMT_Q4_0, 128, 4096, 4096},
                        {FMT_Q4_0, 128, 11008, 4096}, {FMT_Q4_0, 128, 4096, 11008}};
    for (const S& s : shapes) {
        const int nb = s.K / 32, bb = block_bytes(s.F);
        const long wbytes = (long)s.N * nb * bb;
        const int R = (int)std::max(2L, (640L << 20) / wbytes + 1);
        std::vector<uint8_t> hw(wbytes), ha((long)s.M * nb * 36);
        srand(11);
        for (long b = 0; b < (long)s.N * nb; ++b) {
            for (int j = 0; j < bb; ++j) hw[b * bb + j] = rand() & 0xFF;
            uint16_t d = f2h(0.01f + 0.09f * (float)rand() / (float)RAND_MAX);
            memcpy(&hw[b * bb], &d, 2);
            if (s.F == FMT_Q8_0) for (int j = 2; j < bb; ++j) hw[b * bb + j] = (uint8_t)(rand() % 255 - 127);
            if (s.F == FMT_Q4_1 || s.F == FMT_Q5_1) { uint16_t m = f2h(-0.5f * (float)rand() / (float)RAND_MAX); memcpy(&hw[b * bb + 2], &m, 2); }
        }
        for (long b = 0; b < (long)s.M * nb; ++b) {
            uint16_t d = f2h(0.008f), sm = f2h((rand() % 2000 - 1000) / 100.0f);
            memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &sm, 2);
            for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
        }
        std::vector<uint8_t*> w(R);
        for (auto& p : w) { CK(hipMalloc(&p, wbytes)); CK(hipMemcpy(p, hw.data(), wbytes, hipMemcpyHostToDevice)); }
        uint8_t* a; float* c;
        CK(hipMalloc(&a, ha.size())); CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
        CK(hipMalloc(&c, (size_t)s.M * s.N * 4));
        std::vector<Variant> vs;
        vs.push_back({"gemv (C-ABI algo 1)", [](const GemmArgs& g, hipStream_t st) { return qg_gemm_w4a8_ex(g.A, g.B, g.C, g.M, g.N, g.K, g.wtype, 1, (qg_stream_t)st) == 0 ? hipSuccess : hipErrorUnknown; }});
        vs.push_back({"product (C-ABI algo 2)", [](const GemmArgs& g, hipStream_t st) { return qg_gemm_w4a8_ex(g.A, g.B, g.C, g.M, g.N, g.K, g.wtype, 2, (qg_stream_t)st) == 0 ? hipSuccess : hipErrorUnknown; }});
        // Q4_0 configurations only (other formats: the product dispatch above)
#define V(BN, TT, W, P16, NAME) vs.push_back({NAME, [](const GemmArgs& g, hipStream_t st) { \
        return g.wtype == FMT_Q4_0 && mmq_shape_ok<FMT_Q4_0, BN, TT, W, P16>(g) ? mmq_launch<FMT_Q4_0, BN, TT, W, false, P16>(g, st) : hipErrorInvalidValue; }});
#define VN(BN, TT, W, NB, NAME) vs.push_back({NAME, [](const GemmArgs& g, hipStream_t st) { \
        return g.wtype == FMT_Q4_0 && mmq_shape_ok<FMT_Q4_0, BN, TT, W, true, NB>(g) ? mmq_launch<FMT_Q4_0, BN, TT, W, false, true, NB>(g, st) : hipErrorInvalidValue; }});
        VN(32, 1, 8, 2, "v2 bn32 tt1 w8 nb2")
        VN(16, 2, 8, 2, "v2 bn16 tt2 w8 nb2")
        VN(32, 2, 4, 2, "v2 bn32 tt2 w4 nb2")
#define VA(BN, TT, W, ABL, NAME) vs.push_back({NAME, [](const GemmArgs& g, hipStream_t st) { \
        return g.wtype == FMT_Q4_0 && mmq_shape_ok<FMT_Q4_0, BN, TT, W, true, 2>(g) ? mmq_launch<FMT_Q4_0, BN, TT, W, false, true, 2, ABL>(g, st) : hipErrorInvalidValue; }});
        VA(32, 1, 8, 1, "abl1 loads bn32 tt1 w8")
        VA(32, 1, 8, 2, "abl2 no-epi bn32 tt1 w8")
        VA(16, 1, 8, 1, "abl1 loads bn16 tt1 w8")
        VA(32, 2, 4, 1, "abl1 loads bn32 tt2 w4")
        VA(32, 1, 8, 3, "abl3 act-only bn32 tt1 w8")
        VA(32, 1, 8, 4, "abl4 wt-only bn32 tt1 w8")
        VA(16, 2, 8, 1, "abl1 loads bn16 tt2 w8")
        VA(16, 2, 8, 3, "abl3 act-only bn16 tt2 w8")
        VA(16, 2, 8, 4, "abl4 wt-only bn16 tt2 w8")
#define VS(BN, TT, W, NB, SB, ABL, NAME) vs.push_back({NAME, [](const GemmArgs& g, hipStream_t st) { \
        return g.wtype == FMT_Q4_0 && mmq_shape_ok<FMT_Q4_0, BN, TT, W, true, NB, SB>(g) ? mmq_launch<FMT_Q4_0, BN, TT, W, false, true, NB, ABL, false, SB>(g, st) : hipErrorInvalidValue; }});
#undef VS
#define VE(BN, TT, W, NAME) vs.push_back({NAME, [](const GemmArgs& g, hipStream_t st) { \
        return g.wtype == FMT_Q4_0 && mmq_shape_ok<FMT_Q4_0, BN, TT, W, true, 2>(g) ? mmq_launch<FMT_Q4_0, BN, TT, W, false, true, 2, 0, false, 4, 1, true>(g, st) : hipErrorInvalidValue; }});
        VE(32, 1, 8, "EPI2 bn32 tt1 w8")
        VE(16, 1, 8, "EPI2 bn16 tt1 w8")
        VE(32, 2, 8, "EPI2 bn32 tt2 w8")
        VE(32, 2, 4, "EPI2 bn32 tt2 w4")

#undef VE
#undef VA
#undef VN
#undef V
        auto args = [&](int i) { GemmArgs g; g.A = a; g.B = w[i % R]; g.C = c; g.M = s.M; g.N = s.N; g.K = s.K;
                                 g.wtype = s.F; g.ldc_m = s.N; g.ldc_n = 1; return g; };
        std::vector<float> ref((size_t)s.M * s.N), out(ref.size());
        std::vector<double> err(vs.size(), 0.0);
        for (size_t k = 0; k < vs.size(); ++k) {
            CK(hipMemset(c, 0xFF, ref.size() * 4));
            if (vs[k].fn(args(0), st) != hipSuccess) {
                (void)hipGetLastError();
                printf("  %-24s skipped (launch rejected)\n", vs[k].name.c_str());
                vs.erase(vs.begin() + k); err.erase(err.begin() + k); --k;
                continue;
            }
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(k == 0 ? ref.data() : out.data(), c, ref.size() * 4, hipMemcpyDeviceToHost));
            if (k) for (size_t i = 0; i < ref.size(); ++i) err[k] = std::max(err[k], (double)fabs(out[i] - ref[i]) / (1e-2 + fabs(ref[i])));
        }
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        const int L = s.M >= 256 ? 32 : 128, ROUNDS = 3;
        std::vector<std::vector<double>> t(vs.size());
        for (int r = 0; r < ROUNDS; ++r)
            for (size_t k = 0; k < vs.size(); ++k) {
                CK(hipEventRecord(e0, st));
                for (int i = 0; i < L; ++i) CK(vs[k].fn(args(i), st));
                CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                t[k].push_back(ms * 1e3 / L);
            }
        const double bytes = (double)wbytes + (double)s.M * nb * 36 + (double)s.M * s.N * 4;
        const double flops = 2.0 * s.M * s.N * s.K;
        printf("fmt=%d M=%d N=%d K=%d  (%.0f B, %.2f GFLOP)\n", s.F, s.M, s.N, s.K, bytes, flops / 1e9);
        for (size_t k = 0; k < vs.size(); ++k) {
            std::sort(t[k].begin(), t[k].end());
            const double us = t[k][t[k].size() / 2];
            printf("  %-24s %8.3f us  %6.0f GB/s (frac %.3f)  %7.1f TOPS  maxrel %.2e\n", vs[k].name.c_str(), us,
                   bytes / us / 1e3, bytes / us / 1e3 / 8000.0, flops / us / 1e6, err[k]);
        }
        fflush(stdout);
        for (auto p : w) CK(hipFree(p));
        CK(hipFree(a)); CK(hipFree(c));
    }
    return 0;
}
