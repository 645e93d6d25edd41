// gemv_pre_probe.hip — W4A8 GEMV at M = 2..4 (N = K = 4096, Q4_0): activation records preloaded
// into registers after the staging barrier (PRE) or read per block, cold weights (64 copies), graph
// of 64 launches, median of 5. Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../llama.cpp-quant-gemm_amd/csrc \
//         -o gemv_pre_probe gemv_pre_probe.hip
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "qg_gemv_kernel.hpp"
#include "../../include/qg/qg.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;

int main() {
    const int N = 4096, K = 4096, nb = K / 32, L = 64;
    const size_t wb = (size_t)N * nb * 18;
    std::vector<uint8_t> hw(wb);
    for (size_t i = 0; i < wb; ++i) hw[i] = (uint8_t)(i * 2654435761u >> 13);
    for (size_t i = 0; i < wb; i += 18) { hw[i] = 0x00; hw[i + 1] = 0x20; }
    std::vector<uint8_t*> W(L);
    for (auto& p : W) { CK(hipMalloc(&p, wb)); CK(hipMemcpy(p, hw.data(), wb, hipMemcpyHostToDevice)); }
    std::vector<uint8_t> ha((size_t)4 * nb * 36);
    for (size_t i = 0; i < ha.size(); ++i) ha[i] = (uint8_t)(i * 40503u >> 7);
    for (size_t i = 0; i < ha.size(); i += 36) { ha[i] = 0x00; ha[i + 1] = 0x20; ha[i + 2] = 0; ha[i + 3] = 0x3c; }
    uint8_t* A;
    CK(hipMalloc(&A, ha.size()));
    CK(hipMemcpy(A, ha.data(), ha.size(), hipMemcpyHostToDevice));
    float* C;
    CK(hipMalloc(&C, (size_t)4 * N * 4));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    typedef std::function<hipError_t(const GemmArgs&, hipStream_t)> Fn;
    auto run = [&](const char* name, int M, Fn fn) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < L; ++i) {
            GemmArgs a; a.A = A; a.B = W[i]; a.C = C; a.M = M; a.N = N; a.K = K; a.wtype = FMT_Q4_0; a.ldc_m = N; a.ldc_n = 1;
            CK(fn(a, st));
        }
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        std::vector<float> t;
        for (int r = 0; r < 7; ++r) {
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms * 1000.f / L);
        }
        std::sort(t.begin(), t.end());
        printf("  M=%d %-28s %7.3f us\n", M, name, t[2]);
        fflush(stdout);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    };
    for (int M : {2, 3, 4}) {
        if (M == 2) {
            run("MT2 PRE (product)", M, gemv_launch<FMT_Q4_0, 2, 2, 64, 1024, false, AIN_Q8_1, false, true>);
            run("MT2 no PRE", M, gemv_launch<FMT_Q4_0, 2, 2, 64, 1024, false, AIN_Q8_1, false, false>);
        } else {
            run("MT4 no PRE (product)", M, gemv_launch<FMT_Q4_0, 4, 2, 64, 1024, false, AIN_Q8_1, false, false>);
            run("MT4 PRE", M, gemv_launch<FMT_Q4_0, 4, 2, 64, 1024, false, AIN_Q8_1, false, true>);
            run("MT4 PRE 512-thread WG", M, gemv_launch<FMT_Q4_0, 4, 2, 64, 512, false, AIN_Q8_1, false, true>);
        }
    }
    run("MT1 PRE (product)", 1, gemv_launch<FMT_Q4_0, 1, 2, 64, 1024, false, AIN_Q8_1, false, true>);
    for (int M : {5, 8}) {
        run("C-ABI auto (MMQ)", M, [](const GemmArgs& g, hipStream_t s) { return qg_gemm_w4a8(g.A, g.B, g.C, g.M, g.N, g.K, QG_TYPE_Q4_0, s) == 0 ? hipSuccess : hipErrorUnknown; });
        run("MT8 no PRE 1024", M, gemv_launch<FMT_Q4_0, 8, 2, 64, 1024, false, AIN_Q8_1, false, false>);
        run("MT8 PRE 512", M, gemv_launch<FMT_Q4_0, 8, 2, 64, 512, false, AIN_Q8_1, false, true>);
        run("MT8 no PRE 512", M, gemv_launch<FMT_Q4_0, 8, 2, 64, 512, false, AIN_Q8_1, false, false>);
    }
    return 0;
}
