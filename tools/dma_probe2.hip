// dma_probe2.hip — L2/HBM -> LDS ingest of the M = 32 prefill's operands (BASELINE configs[2]) by
// LDS-DMA, per tile geometry and fill size (VERDICT r03 next #3b: re-measure the data-movement
// "floor" with ring-gemm-class fills before calling it one). Not part of the product.
//
// A workgroup owns BN weight rows x NT tokens x all of K (grid N/BN x M/NT, one per CU at 256);
// a stage = SB Q-blocks: BN rows x SB*18 B of Q4_0 + NT tokens x SB*36 B of Q8_1, moved in 16-B
// pieces by LW loader waves (stage h by loader h % LW, DEPTH stages in flight per loader, counted
// vmcnt) into NS LDS slots (reused without a guard: movement only, the bytes are not consumed).
// CP: weight cache policy bits of global_load_lds (0 default, 2 = nt). MODE 0 both operands,
// 1 weights only, 2 activations only. Timed like bench.py: 64 launches over distinct weight copies
// (> 600 MB) in one hipGraph, HIP events; reported with the per-CU ingest rate
// (bytes per workgroup / (t - t_empty)) beside the guide's 68-90 GB/s (MI355X_MICROARCH.md ring-gemm).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o dma_probe2 dma_probe2.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int QK = 32;

template <int CP> __device__ __forceinline__ void glds16(const uint8_t* g, uint8_t* l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, CP);
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int BN, int NT, int SB> struct geo {
    static_assert(SB % 8 == 0, "stage rows are 16-B multiples");
    static constexpr int WPR = SB * 18 / 16;               // weight pieces per row
    static constexpr int APT = SB * 36 / 16;               // activation pieces per token
    static constexpr int WP = BN * WPR, AP = NT * APT;
    static constexpr int NI = (WP + AP + 63) / 64;         // DMA instructions per stage
    static constexpr int SLOT = NI * 1024;
};

template <int BN, int NT, int SB, int LW, int DEPTH, int NS, int CP, int MODE>
__global__ __launch_bounds__(LW * 64) void dma2_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B, int K,
                                                       float* __restrict__ sink) {
    using G = geo<BN, NT, SB>;
    static_assert(DEPTH * G::NI <= 63, "vmcnt range");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nb = K / QK, H = nb / SB;
    const long RB = (long)nb * 18, AB = (long)nb * 36;
    const uint8_t* Bw = B + (long)blockIdx.x * BN * RB;
    const uint8_t* Aw = A + (long)blockIdx.y * NT * AB;
    int off[G::NI];
    bool isw[G::NI];
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
        int p = min(64 * i + lane, G::WP + G::AP - 1);
        bool w = p < G::WP;
        if (MODE == 1) { w = true; p = p % G::WP; }
        if (MODE == 2) { w = false; p = G::WP + p % G::AP; }
        isw[i] = w;
        off[i] = w ? (p / G::WPR) * (int)RB + (p % G::WPR) * 16 : ((p - G::WP) / G::APT) * (int)AB + ((p - G::WP) % G::APT) * 16;
    }
    auto issue = [&](int h) {
        const uint8_t* ws = Bw + (long)h * (SB * 18);
        const uint8_t* as = Aw + (long)h * (SB * 36);
        uint8_t* buf = smem + (h % NS) * G::SLOT;
#pragma unroll
        for (int i = 0; i < G::NI; ++i) {
            if (isw[i]) glds16<CP>(ws + off[i], buf + 64 * i * 16);
            else glds16<0>(as + off[i], buf + 64 * i * 16);
        }
    };
    const int mine = wave < H ? (H - 1 - wave) / LW + 1 : 0;
    int issued = 0;
    for (; issued < DEPTH && issued < mine; ++issued) issue(wave + issued * LW);
    for (int k = 0; k < mine; ++k) {
        const int younger = min(issued - k - 1, DEPTH - 1);
        if (younger >= 3) vm_wait<(DEPTH >= 4 ? 3 * G::NI : 0)>();
        else if (younger == 2) vm_wait<(DEPTH >= 3 ? 2 * G::NI : 0)>();
        else if (younger == 1) vm_wait<G::NI>();
        else vm_wait<0>();
        if (issued < mine) issue(wave + (issued++) * LW);
    }
    vm_wait<0>();
    if (lane == 0 && K < 0) sink[blockIdx.x] = (float)smem[wave];
}

// Linear order: a row tile's weights (BN consecutive rows = ONE contiguous BN * RB-byte region) and a
// token tile's activations (NT consecutive rows, contiguous too) moved as lane-linear 1-KB pieces in
// address order (ORDER 0), or the weights chunk-major (ORDER 1: the 1-KB chunk c of every row before
// chunk c + 1 — the order a consumer working along K needs), LW waves taking pieces round-robin.
// MODE as above. LDS destinations wrap at 144 KB (movement only).
template <int BN, int NT, int LW, int ORDER, int MODE, int CP>
__global__ __launch_bounds__(LW * 64) void lin_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B, int K,
                                                      float* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nb = K / QK;
    const long RB = (long)nb * 18, AB = (long)nb * 36;
    const uint8_t* Bw = B + (long)blockIdx.x * BN * RB;
    const uint8_t* Aw = A + (long)blockIdx.y * NT * AB;
    const int WI = MODE == 2 ? 0 : (int)((BN * RB) / 1024);   // 1-KB weight pieces (RB * BN % 1024 == 0 here)
    const int AI = MODE == 1 ? 0 : (int)((NT * AB) / 1024);
    const int cpr = (int)((RB + 1023) / 1024);               // chunks per row (ORDER 1)
    int n = 0;
    for (int i = wave; i < WI + AI; i += LW) {
        const uint8_t* src;
        if (i < WI) {
            long off = (long)i * 1024;
            if (ORDER == 1) {  // chunk-major: i -> (chunk c, row r), 1 KB of row r at c * 1 KB (clamped)
                const int c = i / BN, r = i % BN;
                off = (long)r * RB + std::min<long>((long)c * 1024, RB - 1024);
                (void)cpr;
            }
            src = Bw + off + 16 * lane;
            glds16<CP>(src, smem + ((long)i * 1024) % (144 * 1024));
        } else {
            src = Aw + (long)(i - WI) * 1024 + 16 * lane;
            glds16<0>(src, smem + ((long)i * 1024) % (144 * 1024));
        }
        if (++n == 48) { vm_wait<16>(); n = 16; }
    }
    vm_wait<0>();
    if (lane == 0 && K < 0) sink[blockIdx.x] = (float)smem[wave];
}

__global__ void empty_kernel(float* sink, int K) {
    if (K < 0) sink[0] = 1.0f;
}

typedef std::function<void(const uint8_t*, const uint8_t*, hipStream_t)> Fn;
struct V {
    std::string name;
    Fn fn;
    double bytes_per_wg;
};

template <int BN, int NT, int SB, int LW, int DEPTH, int NS, int CP, int MODE>
V mk(const char* name, int M, int N, int K, float* sink) {
    using G = geo<BN, NT, SB>;
    const double wb = (double)BN * K / 32 * 18, ab = (double)NT * K / 32 * 36;
    const double bytes = MODE == 1 ? wb : MODE == 2 ? ab : wb + ab;
    return {name,
            [=](const uint8_t* A, const uint8_t* B, hipStream_t st) {
                auto k = dma2_kernel<BN, NT, SB, LW, DEPTH, NS, CP, MODE>;
                const size_t lds = (size_t)NS * G::SLOT;
                static bool set = false;
                if (!set) {
                    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                    set = true;
                }
                hipLaunchKernelGGL(k, dim3(N / BN, M / NT), dim3(LW * 64), lds, st, A, B, K, sink);
            },
            bytes};
}

template <int BN, int NT, int LW, int ORDER, int MODE, int CP>
V mkl(const char* name, int M, int N, int K, float* sink) {
    const double wb = (double)BN * K / 32 * 18, ab = (double)NT * K / 32 * 36;
    const double bytes = MODE == 1 ? wb : MODE == 2 ? ab : wb + ab;
    return {name,
            [=](const uint8_t* A, const uint8_t* B, hipStream_t st) {
                auto k = lin_kernel<BN, NT, LW, ORDER, MODE, CP>;
                static bool set = false;
                if (!set) {
                    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024));
                    set = true;
                }
                hipLaunchKernelGGL(k, dim3(N / BN, M / NT), dim3(LW * 64), 144 * 1024, st, A, B, K, sink);
            },
            bytes};
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
    std::vector<V> vs = {
        {"empty 256 wg", [=](const uint8_t*, const uint8_t*, hipStream_t s) { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(512), 0, s, sink, K); }, 0},
        // geometry A (product): 32 rows x 16 tokens, 256 WGs, 73.7 KB + 73.7 KB per WG
        mk<32, 16, 8, 8, 2, 16, 0, 0>("A sb8  lw8 d2", M, N, K, sink),
        mk<32, 16, 8, 8, 2, 16, 2, 0>("A sb8  lw8 d2 nt", M, N, K, sink),
        mk<32, 16, 16, 4, 2, 8, 0, 0>("A sb16 lw4 d2 (18 KB fills)", M, N, K, sink),
        mk<32, 16, 16, 4, 2, 8, 2, 0>("A sb16 lw4 d2 nt", M, N, K, sink),
        mk<32, 16, 16, 2, 3, 8, 0, 0>("A sb16 lw2 d3", M, N, K, sink),
        mk<32, 16, 16, 8, 1, 8, 0, 0>("A sb16 lw8 d1 (all at once)", M, N, K, sink),
        mk<32, 16, 32, 4, 1, 4, 0, 0>("A sb32 lw4 d1 (all at once)", M, N, K, sink),
        mk<32, 16, 16, 4, 2, 8, 0, 1>("A sb16 lw4 d2 weights", M, N, K, sink),
        mk<32, 16, 16, 4, 2, 8, 0, 2>("A sb16 lw4 d2 acts", M, N, K, sink),
        // geometry B: 16 rows x 32 tokens, 256 WGs, 36.9 KB weights (each read once) + 147 KB acts
        mk<16, 32, 8, 8, 2, 12, 0, 0>("B sb8  lw8 d2", M, N, K, sink),
        mk<16, 32, 16, 4, 2, 6, 0, 0>("B sb16 lw4 d2", M, N, K, sink),
        mk<16, 32, 16, 8, 1, 6, 0, 0>("B sb16 lw8 d1", M, N, K, sink),
        mk<16, 32, 16, 4, 2, 6, 0, 1>("B sb16 lw4 d2 weights", M, N, K, sink),
        mk<16, 32, 16, 4, 2, 6, 0, 2>("B sb16 lw4 d2 acts", M, N, K, sink),
        // geometry C: 32 rows x 32 tokens, 128 WGs (half the CUs), 73.7 KB + 147 KB
        mk<32, 32, 16, 4, 2, 5, 0, 0>("C sb16 lw4 d2 (128 WGs)", M, N, K, sink),
        // linear (address-order) ingest of the same bytes
        mkl<32, 16, 8, 0, 1, 0>("A lin lw8 weights", M, N, K, sink),
        mkl<32, 16, 8, 1, 1, 0>("A lin lw8 weights chunk-major", M, N, K, sink),
        mkl<32, 16, 8, 0, 2, 0>("A lin lw8 acts", M, N, K, sink),
        mkl<32, 16, 8, 0, 0, 0>("A lin lw8 both", M, N, K, sink),
        mkl<32, 16, 8, 1, 0, 0>("A lin lw8 both chunk-major", M, N, K, sink),
        mkl<32, 16, 4, 0, 0, 0>("A lin lw4 both", M, N, K, sink),
        mkl<32, 16, 16, 0, 0, 0>("A lin lw16 both", M, N, K, sink),
        mkl<32, 16, 8, 0, 0, 2>("A lin lw8 both nt", M, N, K, sink),
        mkl<16, 32, 8, 0, 1, 0>("B lin lw8 weights", M, N, K, sink),
        mkl<16, 32, 8, 0, 0, 0>("B lin lw8 both", M, N, K, sink),
        mkl<16, 32, 8, 1, 0, 0>("B lin lw8 both chunk-major", M, N, K, sink),
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
    for (auto& x : t) std::sort(x.begin(), x.end());
    const double t_empty = t[0][4];
    printf("M=32 N=4096 K=4096 prefill operand ingest by LDS-DMA only, us per launch (median of 9 x %d launches, hipGraph)\n", G);
    for (size_t v = 0; v < vs.size(); ++v) {
        const double us = t[v][4];
        const double gbs = vs[v].bytes_per_wg > 0 ? vs[v].bytes_per_wg / ((us - t_empty) * 1e-6) / 1e9 : 0;
        printf("  %-30s %7.3f us (min %7.3f)  %6.1f KB/WG  %6.1f GB/s per CU over the empty launch\n", vs[v].name.c_str(), us,
               t[v][0], vs[v].bytes_per_wg / 1024, gbs);
    }
    return 0;
}
