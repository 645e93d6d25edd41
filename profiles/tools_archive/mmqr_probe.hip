// mmqr_probe.hip — the loader / consumer ring prefill (tools/mmq_ring2_experiment.hpp) against the product
// prefill (qg_mmq_kernel.hpp, mmq 32 x 16 tile, 8 waves), timed like bench.py: 64 launches over
// distinct weight copies (> 600 MB) in one hipGraph, HIP events, interleaved rounds, median.
// Correctness: int32 sumi bit-exact vs the product's parity hook; fp32 outputs vs the product's.
// Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 \
//         -I../llama.cpp-quant-gemm_amd/csrc -o mmqr_probe mmqr_probe.hip
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "mmq_ring2_experiment.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;
void qg::describe_kernel(const GemmArgs&, const char*, ...) {}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }

typedef std::function<hipError_t(const GemmArgs&, hipStream_t)> LaunchFn;
struct Variant { std::string name; LaunchFn fn, sumi; };

template <int F> Variant prod() {
    return {"product mmq bn32 tt1 w8",
            [](const GemmArgs& g, hipStream_t st) { return mmq_launch<F, 32, 1, 8, false, true, 2, 0, false, 4, 1, true>(g, st); },
            [](const GemmArgs& g, hipStream_t st) { return mmq_launch<F, 32, 1, 8, true, true, 2, 0, false, 4, 1, true>(g, st); }};
}
template <int F, int L, int PH, int NS, int D, int ABL = 0> Variant ring(const char* name) {
    return {name, [](const GemmArgs& g, hipStream_t st) { return mmqr_launch<F, L, PH, NS, D, false, ABL>(g, st); },
            [](const GemmArgs& g, hipStream_t st) { return mmqr_launch<F, L, PH, NS, D, true>(g, st); }};
}

template <int F> void run_shape(int M, int N, int K, int bb, std::vector<Variant> vs) {
    const int nb = K / 32;
    const long wbytes = (long)N * nb * bb;
    const int G = 64;
    const int R = (int)std::max((long)G, (640L << 20) / wbytes + 1);
    std::vector<uint8_t> hw(wbytes), ha((long)M * nb * 36);
    srand(11);
    for (long b = 0; b < (long)N * nb; ++b) {
        for (int j = 0; j < bb; ++j) hw[b * bb + j] = rand() & 0xFF;
        uint16_t d = f2h(0.01f + 0.09f * (float)rand() / (float)RAND_MAX);
        memcpy(&hw[b * bb], &d, 2);
        if (F == FMT_Q4_1 || F == FMT_Q5_1) { uint16_t m = f2h(-0.3f); memcpy(&hw[b * bb + 2], &m, 2); }
    }
    for (long b = 0; b < (long)M * nb; ++b) {
        uint16_t d = f2h(0.008f), sm = f2h((rand() % 2000 - 1000) / 100.0f);
        memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &sm, 2);
        for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
    }
    uint8_t* wall;
    CK(hipMalloc(&wall, wbytes * R));
    for (int r = 0; r < R; ++r) CK(hipMemcpy(wall + wbytes * r, hw.data(), wbytes, hipMemcpyHostToDevice));
    uint8_t* a; float* c; int32_t* s;
    CK(hipMalloc(&a, ha.size())); CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&c, (size_t)M * N * 4));
    CK(hipMalloc(&s, (size_t)M * N * nb * 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto args = [&](int i) { GemmArgs g; g.A = a; g.B = wall + wbytes * (i % R); g.C = c; g.M = M; g.N = N; g.K = K;
                             g.wtype = F; g.ldc_m = N; g.ldc_n = 1; return g; };
    std::vector<float> ref((size_t)M * N), out(ref.size());
    std::vector<int32_t> sref((size_t)M * N * nb), sout(sref.size());
    std::vector<hipGraphExec_t> ge(vs.size());
    printf("F=%d M=%d N=%d K=%d\n", F, M, N, K);
    for (size_t v = 0; v < vs.size(); ++v) {
        CK(hipMemset(c, 0xFF, (size_t)M * N * 4));
        CK(vs[v].fn(args(0), st));
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(v == 0 ? ref.data() : out.data(), c, ref.size() * 4, hipMemcpyDeviceToHost));
        GemmArgs gs = args(0); gs.C = nullptr; gs.sumi = s;
        CK(hipMemset(s, 0x7F, sref.size() * 4));
        CK(vs[v].sumi(gs, st));
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(v == 0 ? sref.data() : sout.data(), s, sref.size() * 4, hipMemcpyDeviceToHost));
        double maxrel = 0, maxabs = 0, scale = 0;
        for (size_t i = 0; i < ref.size(); ++i) scale = std::max(scale, (double)fabsf(ref[i]));
        bool sumi_ok = true;
        if (v > 0) {
            for (size_t i = 0; i < ref.size(); ++i) {
                const double e = fabs((double)out[i] - ref[i]);
                maxabs = std::max(maxabs, e);
                maxrel = std::max(maxrel, e / (scale + 1e-30));
            }
            sumi_ok = memcmp(sref.data(), sout.data(), sref.size() * 4) == 0;
        }
        printf("  %-30s  max|d|/max|C| %.2e  sumi %s\n", vs[v].name.c_str(), maxrel, sumi_ok ? "bit-exact" : "MISMATCH");
        hipGraph_t gr;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < G; ++i) CK(vs[v].fn(args(i), st));
        CK(hipStreamEndCapture(st, &gr));
        CK(hipGraphInstantiate(&ge[v], gr, nullptr, nullptr, 0));
        CK(hipGraphDestroy(gr));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int round = 0; round < 9; ++round)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge[v], st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms * 1e3f / G);
        }
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("  %-30s %7.3f us per launch (min %7.3f)\n", vs[v].name.c_str(), t[v][4], t[v][0]);
        CK(hipGraphExecDestroy(ge[v]));
    }
    CK(hipFree(wall)); CK(hipFree(a)); CK(hipFree(c)); CK(hipFree(s));
    CK(hipStreamDestroy(st));
}

template <int F, int BN, int TT, int W, int ABL> Variant prodabl(const char* name) {
    return {name, [](const GemmArgs& g, hipStream_t st) { return mmq_launch<F, BN, TT, W, false, true, 2, ABL, false, 4, 1, true>(g, st); },
            [](const GemmArgs& g, hipStream_t st) { return mmq_launch<F, BN, TT, W, true, true, 2, 0, false, 4, 1, true>(g, st); }};
}

int main() {
    run_shape<FMT_Q4_0>(32, 4096, 4096, 18, {prod<FMT_Q4_0>(),
                                             prodabl<FMT_Q4_0, 32, 1, 8, 1>("product DMA only (ABL1)"),
                                             ring<FMT_Q4_0, 2, 4, 16, 4>("ring L2 PH4 NS16 D4"),
                                             ring<FMT_Q4_0, 2, 4, 16, 4, 1>("ring handshake only"),
                                             ring<FMT_Q4_0, 2, 4, 16, 4, 2>("ring handshake + reads"),
                                             ring<FMT_Q4_0, 2, 6, 12, 4, 1>("ring PH6 NS12 handshake only"),
                                             ring<FMT_Q4_0, 2, 4, 8, 3, 1>("ring NS8 D3 handshake only")});
    return 0;
}
