// read_shape_probe.hip — how much of the single-launch GEMV time is the shape of its weight loads?
// Not part of the product. Pure reads (xor-reduced, one store per lane so nothing is dead) of the
// Q4_0 M=1 N=K=4096 weight bytes (9,437,184 B) in one launch, cold (rotating over > 600 MB), each
// with the product GEMV's grid (256 workgroups x 512 threads) unless stated:
//   unit72    the GEMV's per-lane 72-B units: lane (row r, lir) reads [r*2304 + 72*lir, +72) as
//             4 x dwordx4 + 1 x dwordx2 (each instruction spreads 64 lanes over 4.6 KB)
//   coal      the same wave span (2 rows = 4608 B) read coalesced: instruction k, lane l reads
//             16 B at span + 1024 k + 16 l (4.5 instructions, lanes 32..63 idle in the last)
//   coal_dpp  coal + the DPP row_shr:1 exchange a coalesced GEMV would need (each lane also
//             receives its left neighbour's 16 B)
//   p1_many   one dwordx4 per lane, 1152 workgroups x 512 threads (the best pure read of round 1)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o read_shape_probe read_shape_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef unsigned int u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));

constexpr int ROWB = 2304;  // Q4_0 row bytes at K = 4096

__global__ __launch_bounds__(512) void unit72(const unsigned char* __restrict__ B, unsigned* out) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int row = blockIdx.x * 16 + (tid >> 6) * 2 + lane / 32;
    const unsigned char* p = B + (long)row * ROWB + 72 * (lane & 31);
    unsigned acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { u32x4a4 v = *reinterpret_cast<const u32x4a4*>(p + 16 * k); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    u32x2a4 v2 = *reinterpret_cast<const u32x2a4*>(p + 64);
    acc ^= v2.x ^ v2.y;
    out[blockIdx.x * 512 + tid] = acc;
}

template <bool DPP>
__global__ __launch_bounds__(512) void coal(const unsigned char* __restrict__ B, unsigned* out) {
    const int tid = threadIdx.x, lane = tid & 63;
    const unsigned char* span = B + ((long)blockIdx.x * 16 + (tid >> 6) * 2) * ROWB;
    unsigned acc = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        if (k < 4 || lane < 32) {
            u32x4 v = *reinterpret_cast<const u32x4*>(span + 1024 * k + 16 * lane);
            if constexpr (DPP) {
                const unsigned n0 = __builtin_amdgcn_update_dpp(0u, v.x, 0x111, 0xF, 0xF, false);
                const unsigned n1 = __builtin_amdgcn_update_dpp(0u, v.y, 0x111, 0xF, 0xF, false);
                const unsigned n2 = __builtin_amdgcn_update_dpp(0u, v.z, 0x111, 0xF, 0xF, false);
                const unsigned n3 = __builtin_amdgcn_update_dpp(0u, v.w, 0x111, 0xF, 0xF, false);
                acc += n0 ^ n1 ^ n2 ^ n3;
            }
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    out[blockIdx.x * 512 + tid] = acc;
}

__global__ __launch_bounds__(512) void p1_many(const u32x4* __restrict__ B, long n16, unsigned* out) {
    const long i = (long)blockIdx.x * 512 + threadIdx.x;
    unsigned acc = 0;
    if (i < n16) { u32x4 v = B[i]; acc = v.x ^ v.y ^ v.z ^ v.w; }
    out[i] = acc;
}

int main() {
    const long bytes = 4096L * ROWB;
    const int R = (int)(640L * 1024 * 1024 / bytes) + 1;
    std::vector<unsigned char*> w(R);
    std::vector<unsigned char> h(bytes);
    for (long i = 0; i < bytes; ++i) h[i] = (unsigned char)(i * 2654435761u >> 13);
    for (auto& p : w) { CK(hipMalloc(&p, bytes + 4096)); CK(hipMemcpy(p, h.data(), bytes, hipMemcpyHostToDevice)); }
    unsigned* out;
    CK(hipMalloc(&out, 1152 * 512 * 4));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const char* names[] = {"unit72 (GEMV loads)", "coal", "coal_dpp", "p1_many (1152 WGs)"};
    auto launch = [&](int v, int i) {
        const unsigned char* b = w[i % R];
        if (v == 0) hipLaunchKernelGGL(unit72, dim3(256), dim3(512), 0, st, b, out);
        if (v == 1) hipLaunchKernelGGL(coal<false>, dim3(256), dim3(512), 0, st, b, out);
        if (v == 2) hipLaunchKernelGGL(coal<true>, dim3(256), dim3(512), 0, st, b, out);
        if (v == 3) hipLaunchKernelGGL(p1_many, dim3((unsigned)(bytes / 16 + 511) / 512), dim3(512), 0, st,
                                       (const u32x4*)b, bytes / 16, out);
    };
    const int L = 256, ROUNDS = 7;
    std::vector<std::vector<double>> cold(4), hot(4);
    for (int v = 0; v < 4; ++v) for (int i = 0; i < R; ++i) launch(v, i);
    CK(hipStreamSynchronize(st));
    for (int r = 0; r < ROUNDS; ++r)
        for (int v = 0; v < 4; ++v)
            for (int hc = 0; hc < 2; ++hc) {
                CK(hipEventRecord(e0, st));
                for (int i = 0; i < L; ++i) launch(v, hc ? 0 : i);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                (hc ? hot : cold)[v].push_back(ms * 1e3 / L);
            }
    printf("pure reads of %ld B (Q4_0 N=K=4096 weights), %d copies, %d rounds x %d launches, median us/launch\n", bytes, R,
           ROUNDS, L);
    for (int v = 0; v < 4; ++v) {
        std::sort(cold[v].begin(), cold[v].end());
        std::sort(hot[v].begin(), hot[v].end());
        const double c = cold[v][ROUNDS / 2];
        printf("  %-22s cold %6.3f us (%5.0f GB/s)  hot %6.3f us\n", names[v], c, bytes / c / 1e3, hot[v][ROUNDS / 2]);
    }
    return 0;
}
