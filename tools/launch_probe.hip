// launch_probe.hip — what one launch costs outside the GEMV's own work (diagnostic; not the product).
// Back-to-back launches on one stream, eager and captured in a hipGraph:
//   * an empty kernel at the GEMV's grid (256 x 512 threads) and at 1 x 64;
//   * a kernel that only reads its kernel arguments (the GEMV's 23 dwords) and stores one value;
//   * the product GEMV (Q4_0, M=1, N=K=4096), weights rotated over > 256 MB (cold) or fixed (hot).
// Built twice by the recipe below: plain, and with the first kernel arguments preloaded into SGPRs
// by the dispatch (-mllvm -amdgpu-kernarg-preload-count=14), to price the kernarg fetch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../llama.cpp-quant-gemm_amd/csrc \
//         -o launch_probe launch_probe.hip
//   hipcc ... -mllvm -amdgpu-kernarg-preload-count=14 -o launch_probe_pl launch_probe.hip
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "qg_gemv_kernel.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;

__global__ void empty_kernel() {}

__global__ __launch_bounds__(512) void args_kernel(const uint32_t* A, const uint8_t* B, float* C, int32_t* s, int M,
                                                   int N, int K, long a, long b, long c, long d, long e) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && M < 0) C[0] = (float)(N + K + a + b + c + d + e) + A[0] + B[0] + s[0];
    if (threadIdx.x == 0 && blockIdx.x == 0) C[1] = (float)M;
}

static double per_launch(const std::function<void(int, hipStream_t)>& fn, hipStream_t st, bool graph, int L) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<double> t;
    hipGraphExec_t ge = nullptr;
    if (graph) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < L; ++i) fn(i, st);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0, st));
        if (graph) CK(hipGraphLaunch(ge, st));
        else for (int i = 0; i < L; ++i) fn(i, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3 / L);
    }
    if (ge) CK(hipGraphExecDestroy(ge));
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int M = 1, N = 4096, K = 4096, nb = K / 32;
    const long wbytes = (long)N * nb * 18;
    const int R = (int)((640L << 20) / wbytes) + 1;
    std::vector<uint8_t> hw(wbytes), ha((long)M * nb * 36);
    srand(3);
    for (auto& x : hw) x = rand();
    for (auto& x : ha) x = rand() % 64;
    std::vector<uint8_t*> w(R);
    for (auto& p : w) { CK(hipMalloc(&p, wbytes)); CK(hipMemcpy(p, hw.data(), wbytes, hipMemcpyHostToDevice)); }
    uint8_t* a; float* c;
    CK(hipMalloc(&a, ha.size())); CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&c, (size_t)M * N * 4 + 64));
    auto gemv = [&](int copy, hipStream_t s) {
        GemmArgs g;
        g.A = a; g.B = w[copy % R]; g.C = c; g.M = M; g.N = N; g.K = K; g.wtype = FMT_Q4_0; g.ldc_m = N; g.ldc_n = 1;
        CK((gemv_launch<FMT_Q4_0, 1, 4, 32, 512, false>(g, s)));
    };
    const int L = 64;
    struct Row { const char* name; std::function<void(int, hipStream_t)> fn; };
    std::vector<Row> rows = {
        {"empty 256x512", [](int, hipStream_t s) { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(512), 0, s); }},
        {"empty 1x64", [](int, hipStream_t s) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); }},
        {"args 256x512", [&](int, hipStream_t s) {
             hipLaunchKernelGGL(args_kernel, dim3(256), dim3(512), 0, s, (const uint32_t*)a, (const uint8_t*)w[0], c,
                                (int32_t*)nullptr, M, N, K, 1L, 2L, 3L, 4L, 5L); }},
        {"gemv cold", gemv},
        {"gemv hot", [&](int, hipStream_t s) { gemv(0, s); }},
    };
    for (auto& r : rows) {
        for (int i = 0; i < R; ++i) r.fn(i, st);  // warm every copy's TLB entries / code
        CK(hipStreamSynchronize(st));
        const double eager = per_launch(r.fn, st, false, L);
        const double graph = per_launch(r.fn, st, true, L);
        printf("  %-16s eager %7.3f us/launch   graph %7.3f us/launch\n", r.name, eager, graph);
    }
    fflush(stdout);
    return 0;
}
