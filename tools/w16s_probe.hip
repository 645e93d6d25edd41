// w16s_probe.hip — the round-2 W4A16 prefill (w16s_kernel) variants: LDS ring slots R, stages per
// slice, DMA-only / compute-only ablations, against the
// round-1 split-K kernel. Not part of the product. Cold weights (64 rotating copies, 600 MB), graph
// of 64 launches, median of 5 replays.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -mllvm -amdgpu-kernarg-preload-count=16 -I../llama.cpp-quant-gemm_amd/csrc -o w16s_probe w16s_probe.hip
#include "../llama.cpp-quant-gemm_amd/csrc/qg_w4a16.hip"

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;
namespace qg { void* stream_workspace(hipStream_t, size_t, int, std::unique_lock<std::mutex>*) { return nullptr; } }

typedef std::function<void(const float*, const uint8_t*, float*, hipStream_t)> Fn;

static double time_graph(const Fn& fn, const float* A, std::vector<uint8_t*>& W, float* C, hipStream_t st) {
    const int L = 64;
    hipGraph_t gr;
    hipGraphExec_t ge;
    fn(A, W[0], C, st);  // warm (and sets attributes outside capture)
    CK(hipStreamSynchronize(st));
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < L; ++i) fn(A, W[i % W.size()], C, st);
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
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gr));
    return v[2];
}

template <int TT, int R, int ABL, int NP = 3> Fn w16s_fn(int M, int N, int K, int ns, int ks, void* ws) {
    return [=](const float* A, const uint8_t* B, float* C, hipStream_t st) {
        auto k = w16s_kernel<TT, R, ABL, FMT_Q4_0, NP>;
        static bool set = false;
        const size_t lds = (size_t)R * w16s_geom<TT, FMT_Q4_0, NP>::SBYTES + w16s_geom<TT, FMT_Q4_0, NP>::PLB;
        if (!set) { CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); set = true; }
        const int gx = (N + 127) / 128, gy = (M + 16 * TT - 1) / (16 * TT);
        hipLaunchKernelGGL(k, dim3(gx, gy, ks), dim3(256), lds, st, A, B, C, M, N, K, (long)N, 1L, ns,
                           (float*)((uint8_t*)ws + 4096), (unsigned*)ws);
    };
}

int main() {
    const int N = 4096;
    std::vector<uint8_t*> W(64);
    const int KMAX = 14336;
    const size_t wbmax = (size_t)N * (KMAX / 32) * 18;
    std::vector<uint8_t> h(wbmax);
    for (size_t i = 0; i < wbmax; ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
    for (size_t i = 0; i < wbmax; i += 18) { h[i] = 0x00; h[i + 1] = 0x20; }  // d = 2^-7
    float* A;
    CK(hipMalloc(&A, (size_t)64 * KMAX * 4));
    std::vector<float> ha((size_t)64 * KMAX);
    for (size_t i = 0; i < ha.size(); ++i) ha[i] = (float)((i * 7919) % 2001) / 1000.f - 1.f;
    CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
    float* C;
    CK(hipMalloc(&C, (size_t)64 * N * 4));
    void* ws;
    CK(hipMalloc(&ws, 64 << 20));
    CK(hipMemset(ws, 0, 64 << 20));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    struct S { int M, K; };
    for (S s : {S{32, 4096}, S{16, 4096}}) {
        const int M = s.M, K = s.K;
        const size_t wb = (size_t)N * (K / 32) * 18;
        for (auto& p : W) { CK(hipMalloc(&p, wb)); CK(hipMemcpy(p, h.data(), wb, hipMemcpyHostToDevice)); }
        printf("W4A16 Q4_0 M=%d N=%d K=%d\n", M, N, K);
        GemmArgs g; g.M = M; g.N = N; g.K = K; g.ldc_m = N; g.ldc_n = 1; g.ws = ws; g.ws_bytes = 64 << 20; g.wtype = FMT_Q4_0;
        const w16_plan op = w16_make_plan(M, N, K);
        auto old = [&](const float* A_, const uint8_t* B_, float* C_, hipStream_t st_) {
            GemmArgs x = g; x.A = A_; x.B = B_; x.C = C_;
            const hipError_t e = w16_sk_launch<FMT_Q4_0, 4, 2, 8>(x, op, ws, st_);
            CK(e);
        };
        printf("  %-40s %8.3f us\n", "round-1 w16_sk RT4 TT2 KB8", time_graph(old, A, W, C, st));
        const int nst = K / 128;
        const int gx = N / 128;
        for (int ns : {8, 4}) {
            const int ks = (nst + ns - 1) / ns;
            char name[96];
#define V(TT, R, ABL, NP, TAG)                                                                                    \
            snprintf(name, sizeof name, "w16s TT%d R%d NP%d %s ns%d ks%d (%d WGs)", TT, R, NP, TAG, ns, ks,         \
                     gx * ((M + 16 * TT - 1) / (16 * TT)) * ks);                                                   \
            printf("  %-50s %8.3f us\n", name, time_graph(w16s_fn<TT, R, ABL, NP>(M, N, K, ns, ks, ws), A, W, C, st));
            // NP: activation parts (3 truncated, exact; 2 round-to-nearest, the product from K = 1024)
            V(1, 2, 0, 3, "full")
            V(1, 2, 0, 2, "full")
            V(1, 2, 1, 2, "DMA only")
            V(1, 2, 2, 2, "compute only")
            V(1, 2, 3, 2, "hand-off only")
            V(2, 2, 0, 2, "full")
#undef V
            fflush(stdout);
        }
        for (auto p : W) CK(hipFree(p));
    }
    return 0;
}
