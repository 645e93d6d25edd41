// mmqc_probe.hip — timing, ablations and per-wave timeline of the chunked prefill
// (qg_mmqc_kernel.hpp) at BASELINE configs[2] (Q4_0, M = 32, N = K = 4096). Tuning only, not product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DQG_MMQC_STAMPS -I. \
//         -mllvm -amdgpu-kernarg-preload-count=16 -I../../llama.cpp-quant-gemm_amd/csrc -o mmqc_probe mmqc_probe.hip
// Timing as bench.py: 64 launches over distinct weight copies (> 600 MB) in one hipGraph, HIP events,
// median of 9 replays. Timeline: one launch after a 640 MB sweep (cold), per-wave stamps.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "mmqc_experiment.hpp"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
namespace qg {
void describe_kernel(const GemmArgs&, const char*, ...) {}
}
using namespace qg;

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }

template <int F, int CB, int ABL> struct Var {
    static void launch(const uint8_t* A, const uint8_t* B, float* C, int M, int N, int K, hipStream_t st) {
        using G = mmqc_geom<F, 32, 1, 8, CB>;
        auto k = mmqc_kernel<F, 32, 1, 8, CB, false, ABL>;
        static bool set = false;
        if (!set) { CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS)); set = true; }
        hipLaunchKernelGGL(k, dim3((N + 31) / 32, (M + 15) / 16), dim3(512), G::LDS, st, A, B, M, N, K, (void*)C, N, 1);
    }
};

int main(int argc, char** argv) {
    const int M = 32, N = 4096, K = argc > 1 ? atoi(argv[1]) : 4096, nb = K / 32;
    const long wbytes = (long)N * nb * 18;
    const int R = (int)((640L << 20) / wbytes) + 1, G = 64;
    std::vector<uint8_t> hw(wbytes), ha((long)M * nb * 36);
    for (long b = 0; b < (long)N * nb; ++b) { for (int j = 0; j < 18; ++j) hw[b * 18 + j] = rand(); uint16_t d = f2h(0.05f); memcpy(&hw[b * 18], &d, 2); }
    for (long b = 0; b < (long)M * nb; ++b) { for (int j = 0; j < 36; ++j) ha[b * 36 + j] = rand(); uint16_t d = f2h(0.01f); memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &d, 2); }
    uint8_t* wall;
    CK(hipMalloc(&wall, wbytes * R));
    for (int i = 0; i < R; ++i) CK(hipMemcpy(wall + wbytes * i, hw.data(), wbytes, hipMemcpyHostToDevice));
    uint8_t* a; float* c;
    CK(hipMalloc(&a, ha.size())); CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&c, (size_t)M * N * 4));
    hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    typedef std::function<void(const uint8_t*, float*)> Fn;
    struct V { std::string name; Fn fn; };
    std::vector<V> vs = {
        {"mmqc CB32", [&](const uint8_t* B, float* C) { Var<FMT_Q4_0, 32, 0>::launch(a, B, C, M, N, K, st); }},
        {"mmqc CB32 DMA+barriers only", [&](const uint8_t* B, float* C) { Var<FMT_Q4_0, 32, 1>::launch(a, B, C, M, N, K, st); }},
        {"mmqc CB32 compute only", [&](const uint8_t* B, float* C) { Var<FMT_Q4_0, 32, 2>::launch(a, B, C, M, N, K, st); }},
    };
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    printf("chunked prefill probe, Q4_0 M=%d N=%d K=%d, us per launch (median of 9 x %d launches, hipGraph)\n", M, N, K, G);
    for (auto& v : vs) {
        for (int i = 0; i < 3; ++i) v.fn(wall + wbytes * i, c);
        CK(hipStreamSynchronize(st));
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < G; ++i) v.fn(wall + wbytes * (i % R), c);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        std::vector<float> t;
        for (int r = 0; r < 9; ++r) {
            CK(hipEventRecord(e0, st)); CK(hipGraphLaunch(ge, st)); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms * 1e3f / G);
        }
        std::sort(t.begin(), t.end());
        printf("  %-32s %7.3f us (min %7.3f)\n", v.name.c_str(), t[4], t[0]);
        // timeline of one launch behind a sweep of the other copies (cold weights)
        for (int i = 8; i < R; ++i) v.fn(wall + wbytes * i, c);
        v.fn(wall, c);
        CK(hipStreamSynchronize(st));
        const int nw = ((N + 31) / 32) * ((M + 15) / 16) * 8;
        std::vector<unsigned long long> s(8 * nw);
        CK(hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(g_mmqc_stamps), s.size() * 8));
        unsigned long long t0 = ~0ull;
        for (int i = 0; i < nw; ++i) t0 = std::min(t0, s[8 * i]);
        const char* names[7] = {"entry (vs first wave)", "entry -> chunk 0 ready", "entry -> chunk 1 ready", "entry -> chunk 2 ready",
                                "entry -> chunk 3 ready", "entry -> loop done", "entry -> exit"};
        auto pct = [](std::vector<double> x, double p) { if (x.empty()) return 0.0; std::sort(x.begin(), x.end()); return x[(size_t)(p * (x.size() - 1))]; };
        for (int k = 0; k < 7; ++k) {
            std::vector<double> x;
            for (int i = 0; i < nw; ++i) {
                const unsigned long long* q = &s[8 * i];
                if (k == 0) x.push_back((q[0] - t0) * 0.01);
                else if (q[k]) x.push_back((q[k] - q[0]) * 0.01);
            }
            printf("     %-26s p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f us\n", names[k], pct(x, .1), pct(x, .5), pct(x, .9), pct(x, 1.0));
        }
    }
    return 0;
}
