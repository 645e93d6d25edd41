// dma_probe.hip — the L2 -> LDS data movement of the M = 32 prefill (BASELINE configs[2]) alone, by
// dedicated loader waves, to size a loader / consumer ring before building one.
// Not part of the product.
//
// Per workgroup (grid 128 x 2 = 256, one per CU, a row tile's two token tiles on one XCD as in the
// product): 32 weight rows x 16 tokens x all of K = 32 stages of 4 Q-blocks; a stage = 32 rows x 80-B
// weight windows (16-B pieces, shifted 8 B on odd stages) + 16 tokens x 144 B of Q8_1 = 304 pieces of
// 16 B = 5 LDS-DMA instructions. LW loader waves; loader l issues stages l, l + LW, ... keeping DEPTH
// of its stages in flight (counted vmcnt), into NS LDS slots (NS = 32: no slot reuse). MODE 0 = both
// operands, 1 = weights only, 2 = activations only (the other pieces re-read piece 0).
// Timed like bench.py: 64 launches over distinct weight copies (> 600 MB) in one hipGraph, HIP events.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-kernarg-preload-count=16 -o dma_probe dma_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int BN = 32, NTOK = 16, SB = 4, QK = 32;
constexpr int RSB = SB * 18;                        // 72 weight bytes per row per stage
constexpr int PPR = 5;                              // 80-B window = 5 pieces
constexpr int WPC = BN * PPR;                       // 160 weight pieces
constexpr int APT = 9;                              // 144 B per token per stage
constexpr int APC = NTOK * APT;                     // 144 activation pieces
constexpr int NI = (WPC + APC + 63) / 64;           // 5 instructions per stage
constexpr int SLOT = NI * 64 * 16;                  // 5120 B

__device__ __forceinline__ void glds16(const uint8_t* g, uint8_t* l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int LW, int DEPTH, int NS, int MODE, int EXTRA>
__global__ __launch_bounds__((LW + EXTRA) * 64) void dma_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                                 int K, float* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (wave >= LW) return;  // EXTRA waves: idle consumers (occupancy model only)
    const int nb = K / QK, H = nb / SB;
    const long RB = (long)nb * 18, AB = (long)nb * 36;
    const uint8_t* Bw = B + (long)blockIdx.x * BN * RB;
    const uint8_t* Aw = A + (long)blockIdx.y * NTOK * AB;
    int coff[NI];
    bool isw[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        int p = min(64 * i + lane, WPC + APC - 1);
        isw[i] = p < WPC;
        if (MODE == 1) isw[i] = true;
        if (MODE == 2) isw[i] = false;
        if (isw[i]) {
            const int pp = p < WPC ? p : 0;
            coff[i] = (pp / PPR) * (int)RB + (pp % PPR) * 16;
        } else {
            const int pp = p >= WPC ? p - WPC : 0;
            coff[i] = (pp / APT) * (int)AB + (pp % APT) * 16;
        }
    }
    auto issue = [&](int h) {
        const uint8_t* ws = Bw + (long)h * RSB - ((h * RSB) & 15);
        const uint8_t* as = Aw + (long)h * (SB * 36);
        uint8_t* buf = smem + (h % NS) * SLOT;
#pragma unroll
        for (int i = 0; i < NI; ++i) glds16((isw[i] ? ws : as) + coff[i], buf + 64 * i * 16);
    };
    const int mine = (H - 1 - wave) / LW + 1;  // stages wave, wave + LW, ...
    int issued = 0;
    for (; issued < DEPTH && issued < mine; ++issued) issue(wave + issued * LW);
    for (int k = 0; k < mine; ++k) {
        // stage k of this loader landed once at most min(DEPTH, mine - k) - 1 younger stages fly
        const int younger = min(issued - k - 1, DEPTH - 1);
        if (younger >= 7) vm_wait<7 * NI>();
        else if (younger == 6) vm_wait<6 * NI>();
        else if (younger == 5) vm_wait<5 * NI>();
        else if (younger == 4) vm_wait<4 * NI>();
        else if (younger == 3) vm_wait<3 * NI>();
        else if (younger == 2) vm_wait<2 * NI>();
        else if (younger == 1) vm_wait<NI>();
        else vm_wait<0>();
        if (issued < mine) issue(wave + (issued++) * LW);
    }
    vm_wait<0>();
    if (lane == 0 && K < 0) sink[blockIdx.x] = (float)smem[wave];
}

// Split roles: WL waves stream only the weight pieces of the stages (stage h by weight loader h % WL),
// AL waves only the activation pieces (stage h by activation loader h % AL); ORDER 0: both start at
// once; 1: activation loaders first issue ALL their stages (L2-resident lines, 73.7 KB), weights
// stream meanwhile with depth DW.
constexpr int WNI = (WPC + 63) / 64;  // 3 weight instructions per stage (160 pieces)
constexpr int ANI = (APC + 63) / 64;  // 3 activation instructions per stage (144 pieces)
template <int WL, int AL, int DW, int DA>
__global__ __launch_bounds__((WL + AL) * 64) void dma_split_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                                   int K, float* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nb = K / QK, H = nb / SB;
    const long RB = (long)nb * 18, AB = (long)nb * 36;
    const uint8_t* Bw = B + (long)blockIdx.x * BN * RB;
    const uint8_t* Aw = A + (long)blockIdx.y * NTOK * AB;
    const bool wl = wave < WL;
    const int me = wl ? wave : wave - WL, L = wl ? WL : AL;
    const int NIW = wl ? WNI : ANI;
    int coff[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (wl) {
            const int p = min(64 * i + lane, WPC - 1);
            coff[i] = (p / PPR) * (int)RB + (p % PPR) * 16;
        } else {
            const int p = min(64 * i + lane, APC - 1);
            coff[i] = (p / APT) * (int)AB + (p % APT) * 16;
        }
    }
    auto issue = [&](int h) {
        const uint8_t* src = wl ? Bw + (long)h * RSB - ((h * RSB) & 15) : Aw + (long)h * (SB * 36);
        uint8_t* buf = smem + (h % 26) * 6144 + (wl ? 0 : 3072);  // 26 x 6 KB < 160 KB (probe: slot reuse unguarded)
#pragma unroll
        for (int i = 0; i < 3; ++i) glds16(src + coff[i], buf + 64 * i * 16);
    };
    const int D = wl ? DW : DA;
    const int mine = (H - 1 - me) / L + 1;
    int issued = 0;
    for (; issued < D && issued < mine; ++issued) issue(me + issued * L);
    for (int k = 0; k < mine; ++k) {
        const int younger = min(issued - k - 1, D - 1);
        if (younger >= 8) vm_wait<24>();
        else if (younger >= 4) vm_wait<12>();
        else if (younger >= 2) vm_wait<6>();
        else if (younger == 1) vm_wait<3>();
        else vm_wait<0>();
        if (issued < mine) issue(me + (issued++) * L);
    }
    vm_wait<0>();
    (void)NIW;
    if (lane == 0 && K < 0) sink[blockIdx.x] = (float)smem[wave];
}

typedef std::function<void(const uint8_t*, const uint8_t*, hipStream_t)> Fn;

template <int LW, int DEPTH, int NS, int MODE, int EXTRA = 0>
Fn mk(int K, float* sink) {
    return [=](const uint8_t* A, const uint8_t* B, hipStream_t st) {
        auto k = dma_kernel<LW, DEPTH, NS, MODE, EXTRA>;
        const size_t lds = (size_t)NS * SLOT;
        static bool set = false;
        if (!set) { CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); set = true; }
        hipLaunchKernelGGL(k, dim3(128, 2), dim3((LW + EXTRA) * 64), lds, st, A, B, K, sink);
    };
}

template <int WL, int AL, int DW, int DA>
Fn mks(int K, float* sink) {
    return [=](const uint8_t* A, const uint8_t* B, hipStream_t st) {
        auto k = dma_split_kernel<WL, AL, DW, DA>;
        const size_t lds = 32 * 6144;  // 192 KB? no: 32 stages x 6 KB = 192 KB > LDS -> stages reuse mod 26
        static bool set = false;
        if (!set) { CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)); set = true; }
        (void)lds;
        hipLaunchKernelGGL(k, dim3(128, 2), dim3((WL + AL) * 64), 160 * 1024, st, A, B, K, sink);
    };
}

int main() {
    const int M = 32, N = 4096, K = 4096, nb = K / QK;
    const long wbytes = (long)N * nb * 18, abytes = (long)M * nb * 36;
    const int G = 64, R = 72;
    uint8_t *wall, *a;
    float* sink;
    CK(hipMalloc(&wall, wbytes * R + 4096));
    CK(hipMemset(wall, 0x11, wbytes * R + 4096));
    CK(hipMalloc(&a, abytes));
    CK(hipMemset(a, 0x22, abytes));
    CK(hipMalloc(&sink, 4096));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct V { std::string name; Fn fn; };
    std::vector<V> vs = {
        {"lw8 d2 ns32 both", mk<8, 2, 32, 0>(K, sink)},
        {"lw8 d4 ns32 both", mk<8, 4, 32, 0>(K, sink)},
        {"lw4 d2 ns32 both", mk<4, 2, 32, 0>(K, sink)},
        {"lw4 d4 ns32 both", mk<4, 4, 32, 0>(K, sink)},
        {"lw4 d8 ns32 both", mk<4, 8, 32, 0>(K, sink)},
        {"lw4 d3 ns32 both +4idle", mk<4, 3, 32, 0, 4>(K, sink)},
        {"lw2 d4 ns32 both", mk<2, 4, 32, 0>(K, sink)},
        {"lw2 d8 ns32 both", mk<2, 8, 32, 0>(K, sink)},
        {"lw1 d8 ns32 both", mk<1, 8, 32, 0>(K, sink)},
        {"lw16 d2 ns32 both", mk<16, 2, 32, 0>(K, sink)},
        {"lw4 d4 ns32 weights", mk<4, 4, 32, 1>(K, sink)},
        {"lw4 d4 ns32 acts", mk<4, 4, 32, 2>(K, sink)},
        {"lw8 d2 ns32 weights", mk<8, 2, 32, 1>(K, sink)},
        {"lw8 d2 ns32 acts", mk<8, 2, 32, 2>(K, sink)},
        {"split w2 a1 dw4 da8", mks<2, 1, 4, 8>(K, sink)},
        {"split w2 a2 dw4 da8", mks<2, 2, 4, 8>(K, sink)},
        {"split w4 a1 dw4 da16", mks<4, 1, 4, 16>(K, sink)},
        {"split w4 a2 dw2 da8", mks<4, 2, 2, 8>(K, sink)},
        {"split w2 a1 dw8 da16", mks<2, 1, 8, 16>(K, sink)},
        {"split w4 a4 dw4 da4", mks<4, 4, 4, 4>(K, sink)},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<hipGraphExec_t> ge(vs.size());
    for (size_t v = 0; v < vs.size(); ++v) {
        for (int i = 0; i < 3; ++i) vs[v].fn(a, wall + wbytes * i, st);
        CK(hipStreamSynchronize(st));
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < G; ++i) vs[v].fn(a, wall + wbytes * (i % R), st);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge[v], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    std::vector<std::vector<float>> t(vs.size());
    for (int round = 0; round < 7; ++round)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge[v], st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms * 1e3f / G);
        }
    printf("M=32 N=4096 K=4096 prefill data movement only (per CU 73.7 KB weights + 73.7 KB activations), us per launch (median of 7 x %d)\n", G);
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("  %-28s %7.3f us  (min %7.3f)\n", vs[v].name.c_str(), t[v][3], t[v][0]);
    }
    return 0;
}
