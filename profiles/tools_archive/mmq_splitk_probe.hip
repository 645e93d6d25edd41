// mmq_splitk_probe.hip — split-K across workgroups (mmq_kernel KS > 1) vs the product dispatch for
// the small-M prefill shapes. Not part of the product. Interleaved rounds, cold weights (rotating
// > 640 MB of copies), medians. Outputs are checked against the product after the timed rounds
// too (the tile counters must re-arm themselves launch after launch).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../llama.cpp-quant-gemm_amd/csrc \
//         -o mmq_splitk_probe mmq_splitk_probe.hip -L../llama.cpp-quant-gemm_amd/quant_gemm -lqg_hip \
//         -Wl,-rpath,'$ORIGIN/../llama.cpp-quant-gemm_amd/quant_gemm' && ./mmq_splitk_probe
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "qg_mmq_kernel.hpp"
#include "../include/qg/qg.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }

typedef std::function<hipError_t(const GemmArgs&, hipStream_t)> LaunchFn;
struct Variant { std::string name; LaunchFn fn; };

int main(int argc, char** argv) {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    struct S { int M, N, K; };
    const S shapes[] = {{32, 4096, 4096}, {8, 4096, 4096}, {16, 4096, 4096}, {64, 4096, 4096}, {32, 4096, 14336},
                        {32, 14336, 4096}, {128, 4096, 4096}};
    const size_t WS = 64 << 20;
    void* ws;
    CK(hipMalloc(&ws, WS));
    CK(hipMemset(ws, 0, WS));
    for (const S& s : shapes) {
        const int nb = s.K / 32, bb = 18;
        const long wbytes = (long)s.N * nb * bb;
        const int R = (int)std::max(2L, (640L << 20) / wbytes + 1);
        std::vector<uint8_t> hw(wbytes), ha((long)s.M * nb * 36);
        srand(11);
        for (long b = 0; b < (long)s.N * nb; ++b) {
            for (int j = 0; j < bb; ++j) hw[b * bb + j] = rand() & 0xFF;
            uint16_t d = f2h(0.01f + 0.09f * (float)rand() / (float)RAND_MAX);
            memcpy(&hw[b * bb], &d, 2);
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
        vs.push_back({"product (C-ABI algo 2)", [](const GemmArgs& g, hipStream_t st) { return qg_gemm_w4a8_ex(g.A, g.B, g.C, g.M, g.N, g.K, g.wtype, 2, (qg_stream_t)st) == 0 ? hipSuccess : hipErrorUnknown; }});
        if (s.M <= 4)
            vs.push_back({"gemv (C-ABI algo 1)", [](const GemmArgs& g, hipStream_t st) { return qg_gemm_w4a8_ex(g.A, g.B, g.C, g.M, g.N, g.K, g.wtype, 1, (qg_stream_t)st) == 0 ? hipSuccess : hipErrorUnknown; }});
#define VK(BN, TT, W, KS, NAME) vs.push_back({NAME, [](const GemmArgs& g, hipStream_t st) { \
        return mmq_shape_ok<FMT_Q4_0, BN, TT, W, true, 2, 4, KS>(g) ? mmq_launch<FMT_Q4_0, BN, TT, W, false, true, 2, 0, false, 4, KS>(g, st) : hipErrorInvalidValue; }});
        VK(32, 1, 8, 1, "bn32 tt1 w8 ks1")
        VK(32, 1, 8, 2, "bn32 tt1 w8 ks2")
        VK(32, 1, 8, 4, "bn32 tt1 w8 ks4")
        VK(64, 1, 8, 4, "bn64 tt1 w8 ks4")
        VK(16, 1, 8, 2, "bn16 tt1 w8 ks2")
        VK(32, 2, 8, 2, "bn32 tt2 w8 ks2")
        VK(32, 2, 8, 4, "bn32 tt2 w8 ks4")
        VK(32, 2, 4, 4, "bn32 tt2 w4 ks4")
        VK(64, 2, 8, 4, "bn64 tt2 w8 ks4")
        VK(64, 2, 8, 2, "bn64 tt2 w8 ks2")
        VK(16, 2, 8, 2, "bn16 tt2 w8 ks2")
        VK(16, 2, 8, 4, "bn16 tt2 w8 ks4")
        VK(32, 4, 4, 4, "bn32 tt4 w4 ks4")
        VK(64, 4, 4, 4, "bn64 tt4 w4 ks4")
#undef VK
        auto args = [&](int i) { GemmArgs g; g.A = a; g.B = w[i % R]; g.C = c; g.M = s.M; g.N = s.N; g.K = s.K;
                                 g.wtype = FMT_Q4_0; g.ldc_m = s.N; g.ldc_n = 1; g.ws = ws; g.ws_bytes = WS; return g; };
        std::vector<float> ref((size_t)s.M * s.N), out(ref.size());
        std::vector<double> err(vs.size(), 0.0), err2(vs.size(), 0.0);
        auto check = [&](size_t k, std::vector<double>& e) {
            CK(hipMemset(c, 0xFF, ref.size() * 4));
            if (vs[k].fn(args(0), st) != hipSuccess) return false;
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(k == 0 ? ref.data() : out.data(), c, ref.size() * 4, hipMemcpyDeviceToHost));
            if (k) for (size_t i = 0; i < ref.size(); ++i) e[k] = std::max(e[k], (double)fabs(out[i] - ref[i]) / (1e-2 + fabs(ref[i])));
            return true;
        };
        for (size_t k = 0; k < vs.size(); ++k) {
            if (!check(k, err)) {
                (void)hipGetLastError();
                vs.erase(vs.begin() + k); err.erase(err.begin() + k); err2.erase(err2.begin() + k); --k;
            }
        }
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        const int L = 128, ROUNDS = 5;
        std::vector<std::vector<double>> t(vs.size());
        for (int r = 0; r < ROUNDS; ++r)
            for (size_t k = 0; k < vs.size(); ++k) {
                CK(hipEventRecord(e0, st));
                for (int i = 0; i < L; ++i) CK(vs[k].fn(args(i), st));
                CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                t[k].push_back(ms * 1e3 / L);
            }
        for (size_t k = 0; k < vs.size(); ++k) check(k, err2);
        const double bytes = (double)wbytes + (double)s.M * nb * 36 + (double)s.M * s.N * 4;
        const double flops = 2.0 * s.M * s.N * s.K;
        printf("Q4_0 M=%d N=%d K=%d  (%.0f B, %.2f GFLOP)\n", s.M, s.N, s.K, bytes, flops / 1e9);
        for (size_t k = 0; k < vs.size(); ++k) {
            std::sort(t[k].begin(), t[k].end());
            const double us = t[k][t[k].size() / 2];
            printf("  %-24s %8.3f us  %6.0f GB/s (frac %.3f)  %7.1f TOPS  maxrel %.2e / after %.2e\n", vs[k].name.c_str(), us,
                   bytes / us / 1e3, bytes / us / 1e3 / 8000.0, flops / us / 1e6, err[k], err2[k]);
        }
        fflush(stdout);
        for (auto p : w) CK(hipFree(p));
        CK(hipFree(a)); CK(hipFree(c));
    }
    return 0;
}
