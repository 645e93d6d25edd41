// gemv1h_probe.hip — the M = 1 GEMV with ONE Q-block per lane (two waves per weight row, their
// partial sums combined through LDS) against the product GEMV (two blocks per lane, one wave per row):
// the launch floor probe (profiles/r03_tuning/r03_launch_shape.txt) reads the same 9.4 MB fastest
// with ~9,000 waves of one or two 16-B loads each (2.79-2.82 us) and slowest with few waves of many
// loads; the product runs 4,096 waves of 36 B each. Timed like bench.py (64 launches over distinct
// weight copies > 600 MB, one hipGraph, HIP events, interleaved rounds). Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 \
//         -I../llama.cpp-quant-gemm_amd/csrc -I../include -o gemv1h_probe gemv1h_probe.hip \
//         -L../llama.cpp-quant-gemm_amd/quant_gemm -lqg_hip -Wl,-rpath,'$ORIGIN/../llama.cpp-quant-gemm_amd/quant_gemm'
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "qg/qg.h"
#include "qg_gemv_kernel.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace qg {
void describe_kernel(const GemmArgs&, const char*, ...) {}
}
using namespace qg;

// WPR waves per weight row; each lane one block (nb <= 64 * WPR); WGS threads per workgroup.
// EARLY: the lane's weight loads are issued before the activation staging (as the product).
template <int F, int WGS, int WPR, bool EARLY>
__global__ __launch_bounds__(WGS) void gemv1h_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, int N,
                                                     int K, float* __restrict__ C) {
    using T = wfmt<F>;
    constexpr int LD = (T::BB + 2 + 3) / 4;
    constexpr int RPB = (WGS / 64) / WPR;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int nb = K / QK;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int row = blockIdx.x * RPB + wave / WPR, part = wave % WPR;
    const int b = part * 64 + lane;
    const bool ok = row < N && b < nb;
    const uint8_t* pb = B + (long)(row < N ? row : 0) * nb * T::BB + (long)(b < nb ? b : 0) * T::BB;
    const uint32_t* pa = reinterpret_cast<const uint32_t*>((uintptr_t)pb & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)((uintptr_t)pb & 3);
    uint32_t d[LD];
    auto load_w = [&]() {
#pragma unroll
        for (int i = 0; i < LD; ++i) d[i] = pa[i];
    };
    uint32_t ab[9];
    if (tid < nb) {
#pragma unroll
        for (int i = 0; i < 9; ++i) ab[i] = A[(long)tid * 9 + i];
    }
    if constexpr (EARLY) load_w();
    for (int g = tid; g < nb; g += WGS) {
        if (g != tid) {
#pragma unroll
            for (int i = 0; i < 9; ++i) ab[i] = A[(long)g * 9 + i];
        }
        make_act_record<F>(ab, lds + g * 12);
    }
    __syncthreads();
    if constexpr (!EARLY) load_w();
    const uint32_t* rec = lds + (b < nb ? b : 0) * 12;
    uint4 a[3];
    a[0] = *reinterpret_cast<const uint4*>(rec);
    a[1] = *reinterpret_cast<const uint4*>(rec + 4);
    a[2] = *reinterpret_cast<const uint4*>(rec + 8);
    uint32_t w[LD];
#pragma unroll
    for (int i = 0; i + 1 < LD; ++i) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
    w[LD - 1] = d[LD - 1] >> (8 * sh);
    float acc = 0.0f;
    if (ok) acc = block_term_rec<F, 0>(w, block_dot<F, 0>(w, a), a[2]);
    acc = group_sum_last<64>(acc);
    if constexpr (WPR == 1) {
        if (lane == 63 && row < N) C[row] = acc;
    } else {
        float* red = reinterpret_cast<float*>(lds + nb * 12);
        if (lane == 63) red[wave] = acc;
        __syncthreads();
        if (part == 0 && lane == 63 && row < N) {
            float s = red[wave];
#pragma unroll
            for (int p = 1; p < WPR; ++p) s += red[wave + p];
            C[row] = s;
        }
    }
}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t x; memcpy(&x, &h, 2); return x; }

typedef std::function<void(const uint8_t*, const uint8_t*, float*, hipStream_t)> Fn;

template <int F, int WGS, int WPR, bool EARLY> Fn mk(int N, int K) {
    return [=](const uint8_t* A, const uint8_t* B, float* C, hipStream_t st) {
        constexpr int RPB = (WGS / 64) / WPR;
        const size_t lds = (size_t)(K / 32) * 48 + 64 * 4;
        hipLaunchKernelGGL((gemv1h_kernel<F, WGS, WPR, EARLY>), dim3((N + RPB - 1) / RPB), dim3(WGS), lds, st,
                           (const uint32_t*)A, B, N, K, C);
    };
}

int main() {
    const int N = 4096, K = 4096, nb = K / 32, G = 64, R = 72;
    const long wbytes = (long)N * nb * 18;
    std::vector<uint8_t> hw(wbytes), ha(nb * 36);
    srand(3);
    for (long i = 0; i < (long)N * nb; ++i) {
        for (int j = 0; j < 18; ++j) hw[i * 18 + j] = rand() & 0xFF;
        uint16_t dd = f2h(0.01f + 0.05f * (float)rand() / (float)RAND_MAX);
        memcpy(&hw[i * 18], &dd, 2);
    }
    for (int i = 0; i < nb; ++i) {
        uint16_t dd = f2h(0.008f), s = f2h((rand() % 200 - 100) / 10.0f);
        memcpy(&ha[i * 36], &dd, 2); memcpy(&ha[i * 36 + 2], &s, 2);
        for (int j = 0; j < 32; ++j) ha[i * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
    }
    uint8_t *w, *a;
    float* c;
    CK(hipMalloc(&w, wbytes * R));
    for (int r = 0; r < R; ++r) CK(hipMemcpy(w + wbytes * r, hw.data(), wbytes, hipMemcpyHostToDevice));
    CK(hipMalloc(&a, ha.size()));
    CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&c, (size_t)G * N * 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct V { std::string name; Fn fn; };
    std::vector<V> vs = {
        {"product (qg_gemm_w4a8)", [](const uint8_t* A, const uint8_t* B, float* C, hipStream_t s) {
             qg_gemm_w4a8(A, B, C, 1, 4096, 4096, QG_TYPE_Q4_0, (qg_stream_t)s); }},
        {"1h wg512 wpr2 early", mk<FMT_Q4_0, 512, 2, true>(N, K)},
        {"1h wg512 wpr2 late", mk<FMT_Q4_0, 512, 2, false>(N, K)},
        {"1h wg1024 wpr2 early", mk<FMT_Q4_0, 1024, 2, true>(N, K)},
        {"1h wg256 wpr2 early", mk<FMT_Q4_0, 256, 2, true>(N, K)},
    };
    std::vector<float> ref(N), got(N);
    std::vector<hipGraphExec_t> ge(vs.size());
    for (size_t v = 0; v < vs.size(); ++v) {
        CK(hipMemset(c, 0, N * 4));
        vs[v].fn(a, w, c, st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(v == 0 ? ref.data() : got.data(), c, N * 4, hipMemcpyDeviceToHost));
        double mx = 0, sc = 0;
        for (int i = 0; i < N; ++i) { sc = std::max(sc, (double)fabsf(ref[i])); mx = std::max(mx, (double)fabsf(got[i] - ref[i])); }
        if (v) printf("  %-28s max |d| / max |C| = %.2e\n", vs[v].name.c_str(), mx / sc);
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < G; ++i) vs[v].fn(a, w + wbytes * (i % R), c + (size_t)i * N, st);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge[v], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int round = 0; round < 11; ++round)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge[v], st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms * 1e3f / G);
        }
    printf("Q4_0 M=1 N=K=4096 single-launch GEMV, us per launch (median of 11 x %d)\n", G);
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("  %-28s %7.3f us (min %7.3f)  frac %.3f\n", vs[v].name.c_str(), t[v][5], t[v][0], 9458176.0 / t[v][5] / 8e6);
    }
    return 0;
}
