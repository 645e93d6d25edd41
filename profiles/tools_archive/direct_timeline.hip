// direct_timeline.hip — per-wave timeline of the direct-load prefill (tools/mmq_direct_experiment.hpp built with
// QG_DIRECT_STAMPS): entry, issue done, weights landed, activations landed, compute done, exit.
// The stamps of the LAST launch of a hipGraph of 64 launches over distinct weight copies (as the
// benches run it). Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 \
//         -DQG_DIRECT_STAMPS -I../llama.cpp-quant-gemm_amd/csrc -I. -o direct_timeline direct_timeline.hip
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "mmq_direct_experiment.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;
void qg::describe_kernel(const GemmArgs&, const char*, ...) {}

template <int TT, int W, int BPC>
void run(const char* name, int M, int N, int K) {
    const int nb = K / 32;
    const long wbytes = (long)N * nb * 18;
    const int G = 64, R = 72;
    uint8_t* wall; uint8_t* a; float* c;
    CK(hipMalloc(&wall, wbytes * R));
    CK(hipMemset(wall, 0x11, wbytes * R));
    CK(hipMalloc(&a, (size_t)M * nb * 36));
    CK(hipMemset(a, 0x01, (size_t)M * nb * 36));
    CK(hipMalloc(&c, (size_t)M * N * 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto args = [&](int i) { GemmArgs g; g.A = a; g.B = wall + wbytes * (i % R); g.C = c; g.M = M; g.N = N; g.K = K;
                             g.wtype = FMT_Q4_0; g.ldc_m = N; g.ldc_n = 1; return g; };
    if (!direct_shape_ok<FMT_Q4_0, TT, W, BPC, 1>(args(0))) { printf("%s: shape rejected\n", name); return; }
    hipGraph_t gr;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < G; ++i) CK((direct_launch<FMT_Q4_0, TT, W, BPC, 1, false>(args(i), st)));
    CK(hipStreamEndCapture(st, &gr));
    hipGraphExec_t x;
    CK(hipGraphInstantiate(&x, gr, nullptr, nullptr, 0));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(x, st));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(x, st));
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const int nwg = ((N + 15) / 16) * ((M + 16 * TT - 1) / (16 * TT)), nw = nwg * W;
    std::vector<unsigned long long> h((size_t)8 * nw);
    CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_direct_stamps), h.size() * 8));
    unsigned long long t0 = ~0ull, tend = 0;
    for (int w = 0; w < nw; ++w) { t0 = std::min(t0, h[8 * w]); tend = std::max(tend, h[8 * w + 5]); }
    auto pct = [&](const char* lbl, auto f) {
        std::vector<double> v(nw);
        for (int w = 0; w < nw; ++w) v[w] = f(&h[8 * w]) * 0.01;  // 100 MHz ticks -> us
        std::sort(v.begin(), v.end());
        printf("   %-26s p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f us\n", lbl, v[nw / 10], v[nw / 2], v[nw * 9 / 10], v[nw - 1]);
    };
    printf("%s M=%d N=%d K=%d: graph %.3f us/launch, last launch span %.2f us, %d waves\n", name, M, N, K, ms * 1e3 / G,
           (tend - t0) * 0.01, nw);
    pct("entry offset", [&](const unsigned long long* s) { return (double)(s[0] - t0); });
    pct("entry -> issue done", [&](const unsigned long long* s) { return (double)(s[1] - s[0]); });
    pct("entry -> weights landed", [&](const unsigned long long* s) { return (double)(s[2] - s[0]); });
    pct("entry -> acts landed", [&](const unsigned long long* s) { return (double)(s[3] - s[0]); });
    pct("compute", [&](const unsigned long long* s) { return (double)(s[4] - s[3]); });
    pct("reduce + store", [&](const unsigned long long* s) { return (double)(s[5] - s[4]); });
    pct("exit offset", [&](const unsigned long long* s) { return (double)(s[5] - t0); });
    CK(hipGraphExecDestroy(x));
    CK(hipFree(wall)); CK(hipFree(a)); CK(hipFree(c));
}

int main() {
    run<2, 8, 8>("direct tt2 w8 bpc8", 32, 4096, 4096);
    run<2, 8, 16>("direct tt2 w8 bpc16", 32, 4096, 4096);
    run<1, 8, 16>("direct tt1 w8 bpc16", 16, 4096, 4096);
    run<1, 16, 8>("direct tt1 w16 bpc8", 8, 4096, 4096);
    return 0;
}
