// branch_probe.hip — do independent single GEMV launches overlap their dispatch boundaries when a
// hipGraph holds them on parallel branches? Not part of the product. 64 product GEMVs (Q4_0, M=1,
// N=K=4096, qg_gemm_w4a8 through the C-ABI) on 64 distinct weight copies (604 MB, cold), captured
//   * as one chain (the bench's shape),
//   * as S parallel chains (the capture stream forks onto S streams via events and joins them),
// timed per graph replay with events; us per GEMV = replay time / 64. Outputs of every variant are
// compared with the chain's (bit-identical).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -o branch_probe branch_probe.hip \
//         -L../llama.cpp-quant-gemm_amd/quant_gemm -lqg_hip -Wl,-rpath,'$ORIGIN/../llama.cpp-quant-gemm_amd/quant_gemm'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "qg/qg.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
    const int N = 4096, K = 4096, G = 64, nb = K / 32;
    const size_t wb = (size_t)N * nb * 18, ab = (size_t)nb * 36;
    std::vector<uint8_t> hw(wb), ha(ab);
    for (size_t i = 0; i < wb; ++i) hw[i] = (uint8_t)(i * 2654435761u >> 13);
    for (size_t i = 0; i < wb; i += 18) { hw[i] = 0x00; hw[i + 1] = 0x20; }
    for (size_t i = 0; i < ab; ++i) ha[i] = (uint8_t)(i * 40503u >> 7);
    for (size_t i = 0; i < ab; i += 36) { ha[i] = 0x00; ha[i + 1] = 0x20; ha[i + 2] = 0; ha[i + 3] = 0x3c; }
    std::vector<uint8_t*> W(G);
    for (auto& p : W) { CK(hipMalloc(&p, wb)); CK(hipMemcpy(p, hw.data(), wb, hipMemcpyHostToDevice)); }
    uint8_t* A;
    CK(hipMalloc(&A, ab));
    CK(hipMemcpy(A, ha.data(), ab, hipMemcpyHostToDevice));
    float* C;
    CK(hipMalloc(&C, (size_t)G * N * 4));
    std::vector<float> ref((size_t)G * N), got((size_t)G * N);
    hipStream_t cap;
    CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int S : {1, 2, 4, 8}) {
        std::vector<hipStream_t> br(S);
        std::vector<hipEvent_t> done(S);
        for (int i = 0; i < S; ++i) {
            CK(hipStreamCreateWithFlags(&br[i], hipStreamNonBlocking));
            CK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
        }
        hipEvent_t fork;
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        CK(hipMemset(C, 0, (size_t)G * N * 4));
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(cap, hipStreamCaptureModeGlobal));
        if (S == 1) {
            for (int j = 0; j < G; ++j)
                if (qg_gemm_w4a8(A, W[j], C + (size_t)j * N, 1, N, K, QG_TYPE_Q4_0, cap) != 0) { printf("launch failed\n"); return 1; }
        } else {
            CK(hipEventRecord(fork, cap));
            for (int i = 0; i < S; ++i) {
                CK(hipStreamWaitEvent(br[i], fork, 0));
                for (int j = i; j < G; j += S)
                    if (qg_gemm_w4a8(A, W[j], C + (size_t)j * N, 1, N, K, QG_TYPE_Q4_0, br[i]) != 0) { printf("launch failed\n"); return 1; }
                CK(hipEventRecord(done[i], br[i]));
                CK(hipStreamWaitEvent(cap, done[i], 0));
            }
        }
        CK(hipStreamEndCapture(cap, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        std::vector<float> t;
        for (int r = 0; r < 12; ++r) {
            CK(hipEventRecord(e0, cap));
            CK(hipGraphLaunch(ge, cap));
            CK(hipEventRecord(e1, cap));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms * 1000.f / G);
        }
        std::sort(t.begin(), t.end());
        CK(hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost));
        if (S == 1) ref = got;
        const bool same = memcmp(ref.data(), got.data(), ref.size() * 4) == 0;
        printf("  %d parallel chain(s) of %2d GEMVs: %6.3f us per GEMV (p10 %6.3f, p90 %6.3f)  %s\n", S, G / S,
               t[t.size() / 2], t[t.size() / 10], t[(9 * t.size()) / 10], same ? "bit-identical" : "MISMATCH");
        fflush(stdout);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
