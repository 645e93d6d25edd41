// gemv_launch_probe.hip — what a single GEMV launch pays besides its bytes (not product code):
// empty kernels and pure reads of the Q4_0 N=K=4096 weights in the product GEMV's per-lane shape
// (row per wave, lane l reads [36 l, 36 l + 36) of its row: dwordx4, dwordx4, dword), with and
// without a dynamic LDS allocation / an LDS write + barrier, beside the product GEMV (C-ABI).
// Timed like bench.py: 64 launches over distinct weight copies (> 600 MB) in one hipGraph, HIP
// events, interleaved rounds, median per launch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-kernarg-preload-count=16 -o gemv_launch_probe \
//         gemv_launch_probe.hip -L../llama.cpp-quant-gemm_amd/quant_gemm -lqg_hip \
//         -Wl,-rpath,'$ORIGIN/../llama.cpp-quant-gemm_amd/quant_gemm'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "../include/qg/qg.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
constexpr int ROWB = 2304, N = 4096;

template <int WGS>
__global__ __launch_bounds__(WGS) void empty_k(unsigned* out) {
    if (threadIdx.x == 0 && blockIdx.x == 100000) out[0] = 1;
}

// MODE 0: pure read; 1: + LDS allocated (dynamic, untouched); 2: + one LDS write per thread and a
// barrier before the reads are consumed (the staged GEMV's structure, no compute)
template <int WGS, int MODE>
__global__ __launch_bounds__(WGS) void read_k(const unsigned char* __restrict__ B, unsigned* out) {
    extern __shared__ unsigned lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int row = blockIdx.x * (WGS / 64) + (tid >> 6);
    const unsigned* p = reinterpret_cast<const unsigned*>(B + (long)row * ROWB + 36 * lane);
    u32x4a4 a = *reinterpret_cast<const u32x4a4*>(p);
    u32x4a4 b = *reinterpret_cast<const u32x4a4*>(p + 4);
    unsigned c = p[8];
    if constexpr (MODE == 2) {
        lds[tid] = tid * 7u;
        __syncthreads();
        c ^= lds[(tid + 64) % WGS];
    }
    unsigned acc = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c;
    // one store per row, as the GEMV (lane 63 after a reduction)
    acc += __shfl_xor(acc, 32);
    if (lane == 63) out[row] = acc;
}

int main() {
    const long bytes = (long)N * ROWB;
    const int G = 64;
    const int R = std::max(G, (int)(640L * 1024 * 1024 / bytes) + 1);
    unsigned char* wall;
    CK(hipMalloc(&wall, bytes * R));
    CK(hipMemset(wall, 0x11, bytes * R));
    unsigned char* act;  // Q8_1 activations, d = 0.01, s = 0, qs = 1
    std::vector<unsigned char> ha(128 * 36, 1);
    for (int b = 0; b < 128; ++b) { ha[b * 36] = 0x1F; ha[b * 36 + 1] = 0x21; ha[b * 36 + 2] = 0; ha[b * 36 + 3] = 0; }
    CK(hipMalloc(&act, ha.size())); CK(hipMemcpy(act, ha.data(), ha.size(), hipMemcpyHostToDevice));
    float* c; CK(hipMalloc(&c, G * N * 4));
    unsigned* out; CK(hipMalloc(&out, 1 << 20));
    hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct V { std::string name; std::function<void(int)> fn; };
    std::vector<V> vs = {
        {"empty 256x1024", [&](int) { hipLaunchKernelGGL(empty_k<1024>, dim3(256), dim3(1024), 0, st, out); }},
        {"empty 256x1024 + 8 KB LDS", [&](int) { hipLaunchKernelGGL(empty_k<1024>, dim3(256), dim3(1024), 8192, st, out); }},
        {"empty 1024x256", [&](int) { hipLaunchKernelGGL(empty_k<256>, dim3(1024), dim3(256), 0, st, out); }},
        {"read 256x1024", [&](int i) { hipLaunchKernelGGL((read_k<1024, 0>), dim3(256), dim3(1024), 0, st, wall + bytes * (i % R), out); }},
        {"read 256x1024 + LDS", [&](int i) { hipLaunchKernelGGL((read_k<1024, 1>), dim3(256), dim3(1024), 8192, st, wall + bytes * (i % R), out); }},
        {"read 256x1024 + LDS + barrier", [&](int i) { hipLaunchKernelGGL((read_k<1024, 2>), dim3(256), dim3(1024), 8192, st, wall + bytes * (i % R), out); }},
        {"read 512x512", [&](int i) { hipLaunchKernelGGL((read_k<512, 0>), dim3(512), dim3(512), 0, st, wall + bytes * (i % R), out); }},
        {"read 1024x256", [&](int i) { hipLaunchKernelGGL((read_k<256, 0>), dim3(1024), dim3(256), 0, st, wall + bytes * (i % R), out); }},
        {"read 1024x256 + LDS + barrier", [&](int i) { hipLaunchKernelGGL((read_k<256, 2>), dim3(1024), dim3(256), 2048, st, wall + bytes * (i % R), out); }},
        {"product GEMV (C-ABI)", [&](int i) { if (qg_gemm_w4a8(act, wall + bytes * (i % R), c + (i % G) * N, 1, N, 4096, QG_TYPE_Q4_0, (qg_stream_t)st)) exit(2); }},
    };
    std::vector<hipGraphExec_t> ge;
    for (auto& v : vs) {
        v.fn(0);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st));
        hipGraph_t gr;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < G; ++i) v.fn(i);
        CK(hipStreamEndCapture(st, &gr));
        hipGraphExec_t x;
        CK(hipGraphInstantiate(&x, gr, nullptr, nullptr, 0));
        ge.push_back(x);
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int ROUNDS = 9, REPS = 10;
    std::vector<std::vector<double>> t(vs.size());
    for (int r = 0; r < ROUNDS; ++r)
        for (size_t k = 0; k < vs.size(); ++k) {
            CK(hipGraphLaunch(ge[k], st));
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < REPS; ++i) CK(hipGraphLaunch(ge[k], st));
            CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[k].push_back(ms * 1e3 / (REPS * G));
        }
    printf("per launch, hipGraph of %d launches over %d weight copies (%ld B each), median of %d rounds\n", G, R, bytes, ROUNDS);
    for (size_t k = 0; k < vs.size(); ++k) {
        std::sort(t[k].begin(), t[k].end());
        printf("  %-32s %7.3f us  (min %.3f max %.3f)\n", vs[k].name.c_str(), t[k][ROUNDS / 2], t[k][0], t[k][ROUNDS - 1]);
    }
    return 0;
}
