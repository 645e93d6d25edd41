// gemv_coal_probe.hip — the M = 1 GEMV (Q4_0, N = K = 4096) with its weight row fetched by
// COALESCED loads and handed to the lanes through LDS, against the product (each lane loads its own
// 36-B unit as 9 dword loads at a 36-B lane stride: every load instruction touches the whole
// 2,304-B row, 18 cache lines). The round-3 launch-shape probe read the same 9.4 MB in 2.79 us with
// 16-B coalesced loads; the round-2 pure read in the product's unit shape took 2.97-3.03 us.
// Variants (per wave one weight row, 16 waves per workgroup, the product's activation staging,
// records, dot and epilogue — bit-identical outputs):
//   V0  3 x 16-B coalesced loads per lane (lanes 0..15 for the third) -> LDS -> 9 dwords per lane
//   V1  9 x 4-B coalesced loads per lane (dword j * 64 + lane)          -> LDS -> 9 dwords per lane
//   R2  pure read, the product's unit shape (9 dword loads at a 36-B lane stride), no compute
//   R3  pure read, 3 x 16-B coalesced loads per lane, no compute
// Timed like bench.py (64 launches over distinct weight copies > 600 MB, one hipGraph, HIP events,
// interleaved rounds). Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 \
//         -I../llama.cpp-quant-gemm_amd/csrc -I../include -o gemv_coal_probe gemv_coal_probe.hip \
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

// K = 4096 fixed (one 2-block unit per lane, 64 units per row); N % (WGS / 64) == 0.
template <int V, int WGS>
__global__ __launch_bounds__(WGS) void gemvc_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, int N,
                                                    float* __restrict__ C) {
    constexpr int F = FMT_Q4_0;
    using G = gemv_geom<F, 2>;
    constexpr int NB = 128, RDW = NB * 18 / 4;  // row dwords: 576 = 144 x 16 B
    constexpr int RPB = WGS / 64;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tile = gridDim.x <= 512 ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int row = tile * RPB + wave;
    const uint32_t* wr = reinterpret_cast<const uint32_t*>(B + (long)row * NB * 18);
    if constexpr (V >= 2) {
        uint32_t x = 0;
        if constexpr (V == 2) {
#pragma unroll
            for (int i = 0; i < 9; ++i) x ^= wr[lane * 9 + i];
        } else {
            const uint4* w4 = reinterpret_cast<const uint4*>(wr);
            const uint4 p = w4[lane], q = w4[64 + lane];
            const uint4 r = lane < 16 ? w4[128 + lane] : make_uint4(0, 0, 0, 0);
            x = p.x ^ p.y ^ p.z ^ p.w ^ q.x ^ q.y ^ q.z ^ q.w ^ r.x ^ r.y ^ r.z ^ r.w;
        }
        if (x == 0x9E3779B9u) C[row] = 1.0f;
        return;
    }
    // 1) activation loads (thread t: block t), 2) the row's coalesced weight loads, 3) records
    uint32_t ab[9];
    if (tid < NB) {
#pragma unroll
        for (int i = 0; i < 9; ++i) ab[i] = A[(long)tid * 9 + i];
    }
    uint4 v4[3];
    uint32_t v1[9];
    if constexpr (V == 0) {
        const uint4* w4 = reinterpret_cast<const uint4*>(wr);
        v4[0] = w4[lane];
        v4[1] = w4[64 + lane];
        if (lane < 16) v4[2] = w4[128 + lane];
    } else {
#pragma unroll
        for (int j = 0; j < 9; ++j) v1[j] = wr[j * 64 + lane];
    }
    if (tid < NB) make_act_record<F>(ab, lds + (tid / 2) * G::REC_DW + (tid % 2) * 12);
    __syncthreads();
    // 4) the wave's row through its LDS slab, 5) the lane's unit (dwords 9 * lane ..)
    uint32_t* wl = lds + 64 * G::REC_DW + wave * RDW;
    if constexpr (V == 0) {
        uint4* wl4 = reinterpret_cast<uint4*>(wl);
        wl4[lane] = v4[0];
        wl4[64 + lane] = v4[1];
        if (lane < 16) wl4[128 + lane] = v4[2];
    } else {
#pragma unroll
        for (int j = 0; j < 9; ++j) wl[j * 64 + lane] = v1[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t* rec = lds + lane * G::REC_DW;
    uint4 a0[3], a1[3];
#pragma unroll
    for (int x = 0; x < 3; ++x) {
        a0[x] = *reinterpret_cast<const uint4*>(rec + 4 * x);
        a1[x] = *reinterpret_cast<const uint4*>(rec + 12 + 4 * x);
    }
    uint32_t cur[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) cur[i] = wl[lane * 9 + i];
    float acc = 0.0f;
    acc += block_term_rec<F, 0>(cur, block_dot<F, 0>(cur, a0), a0[2]);
    acc += block_term_rec<F, 1>(cur, block_dot<F, 1>(cur, a1), a1[2]);
    acc = group_sum_last<64>(acc);
    if (lane == 63 && row < N) C[row] = acc;
}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t x; memcpy(&x, &h, 2); return x; }

typedef std::function<void(const uint8_t*, const uint8_t*, float*, hipStream_t)> Fn;

template <int V, int WGS> Fn mk(int N) {
    return [=](const uint8_t* A, const uint8_t* B, float* C, hipStream_t st) {
        constexpr int RPB = WGS / 64;
        const size_t lds = V >= 2 ? 0 : (size_t)64 * gemv_geom<FMT_Q4_0, 2>::REC_DW * 4 + (size_t)RPB * 2304;
        hipLaunchKernelGGL((gemvc_kernel<V, WGS>), dim3(N / RPB), dim3(WGS), lds, st, (const uint32_t*)A, B, N, C);
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
    struct Var { std::string name; Fn fn; bool check; };
    std::vector<Var> vs = {
        {"product (qg_gemm_w4a8)", [](const uint8_t* A, const uint8_t* B, float* C, hipStream_t s) {
             qg_gemm_w4a8(A, B, C, 1, 4096, 4096, QG_TYPE_Q4_0, (qg_stream_t)s); }, true},
        {"V0 16-B coalesced + LDS wg1024", mk<0, 1024>(N), true},
        {"V0 16-B coalesced + LDS wg512", mk<0, 512>(N), true},
        {"V0 16-B coalesced + LDS wg256", mk<0, 256>(N), true},
        {"V1 4-B coalesced + LDS wg1024", mk<1, 1024>(N), true},
        {"R2 read, unit shape wg1024", mk<2, 1024>(N), false},
        {"R3 read, 16-B coalesced wg1024", mk<3, 1024>(N), false},
        {"R3 read, 16-B coalesced wg512", mk<3, 512>(N), false},
    };
    std::vector<float> ref(N), got(N);
    std::vector<hipGraphExec_t> ge(vs.size());
    for (size_t v = 0; v < vs.size(); ++v) {
        CK(hipMemset(c, 0, N * 4));
        vs[v].fn(a, w, c, st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(v == 0 ? ref.data() : got.data(), c, N * 4, hipMemcpyDeviceToHost));
        if (v && vs[v].check)
            printf("  %-34s %s\n", vs[v].name.c_str(), memcmp(ref.data(), got.data(), N * 4) ? "OUTPUT DIFFERS" : "bit-identical");
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
        printf("  %-34s %7.3f us (min %7.3f)  frac %.3f\n", vs[v].name.c_str(), t[v][5], t[v][0], 9458176.0 / t[v][5] / 8e6);
    }
    return 0;
}
