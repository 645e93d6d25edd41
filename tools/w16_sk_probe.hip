// w16_sk_probe.hip — W4A16 split-K prefill plans at M = 32, N = K = 4096 (Q4_0 weights, fp32
// activations). Not part of the product. Cold weights (64 rotating copies, 600 MB), graph of 64
// launches, median of 5. ABL=1: slices store their partials and exit (no reduction).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -I../llama.cpp-quant-gemm_amd/csrc -o w16_sk_probe w16_sk_probe.hip
#include "../llama.cpp-quant-gemm_amd/csrc/qg_w4a16.hip"

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;
namespace qg { void* stream_workspace(hipStream_t, size_t) { return nullptr; } }

template <int RT, int TT, int KB, int ABL>
void run(const char* name, int M, int N, int K, int ks, const float* A, std::vector<uint8_t*>& W, float* C, void* ws,
         hipStream_t st) {
    const int gx = (N + 16 * RT - 1) / (16 * RT), gy = (M + 16 * TT - 1) / (16 * TT);
    const int nb = K / 32;
    if (nb % (ks * KB)) { printf("  %-34s skipped\n", name); return; }
    unsigned* cnt = (unsigned*)ws;
    float* part = (float*)((uint8_t*)ws + ((size_t)gx * gy * 4 + 255) / 256 * 256);
    constexpr size_t lds = (size_t)TT * KB * 3 * 1024;
    auto kfn = w16_sk_kernel<FMT_Q4_0, RT, TT, KB, ABL>;
    CK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int L = 64;
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < L; ++i)
        hipLaunchKernelGGL(kfn, dim3(gx, gy, ks), dim3(RT * 64), lds, st, A, (const uint8_t*)W[i % W.size()], C, M, N, K,
                           (long)N, 1L, nb / ks, part, cnt);
    CK(hipStreamEndCapture(st, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<float> v;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) v.push_back(ms * 1000.f / L);
    }
    std::sort(v.begin(), v.end());
    printf("  %-34s grid %3dx%dx%-2d %7.3f us\n", name, gx, gy, ks, v[2]);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gr));
}

int main() {
    const int M = 32, N = 4096, K = 4096;
    const size_t wb = (size_t)N * (K / 32) * 18;
    std::vector<uint8_t*> W(64);
    std::vector<uint8_t> h(wb);
    for (size_t i = 0; i < wb; ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
    for (size_t i = 0; i < wb; i += 18) { h[i] = 0x00; h[i + 1] = 0x20; }  // d = 2^-7
    for (auto& p : W) { CK(hipMalloc(&p, wb)); CK(hipMemcpy(p, h.data(), wb, hipMemcpyHostToDevice)); }
    float* A;
    CK(hipMalloc(&A, (size_t)M * K * 4));
    std::vector<float> ha((size_t)M * K);
    for (size_t i = 0; i < ha.size(); ++i) ha[i] = (float)((i * 7919) % 2001) / 1000.f - 1.f;
    CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
    float* C;
    CK(hipMalloc(&C, (size_t)M * N * 4));
    void* ws;
    CK(hipMalloc(&ws, 64 << 20));
    CK(hipMemset(ws, 0, 64 << 20));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    printf("W4A16 Q4_0 M=%d N=%d K=%d\n", M, N, K);
    run<8, 2, 16, 0>("product RT8 TT2 KB16 KS8", M, N, K, 8, A, W, C, ws, st);
    run<8, 2, 16, 1>("ABL1 (no reduction) RT8 KS8", M, N, K, 8, A, W, C, ws, st);
    run<8, 2, 16, 0>("RT8 KB16 KS4", M, N, K, 4, A, W, C, ws, st);
    run<8, 2, 8, 0>("RT8 KB8 KS16", M, N, K, 16, A, W, C, ws, st);
    run<8, 2, 8, 1>("ABL1 RT8 KB8 KS16", M, N, K, 16, A, W, C, ws, st);
    run<4, 2, 16, 0>("RT4 KB16 KS4", M, N, K, 4, A, W, C, ws, st);
    run<4, 2, 16, 0>("RT4 KB16 KS8", M, N, K, 8, A, W, C, ws, st);
    run<4, 2, 16, 1>("ABL1 RT4 KB16 KS8", M, N, K, 8, A, W, C, ws, st);
    run<4, 2, 8, 0>("RT4 KB8 KS8", M, N, K, 8, A, W, C, ws, st);
    run<4, 2, 8, 0>("RT4 KB8 KS16", M, N, K, 16, A, W, C, ws, st);
    run<8, 2, 16, 0>("RT8 KB16 KS2", M, N, K, 2, A, W, C, ws, st);
    run<8, 2, 16, 0>("RT8 KB16 KS1", M, N, K, 1, A, W, C, ws, st);
    return 0;
}
