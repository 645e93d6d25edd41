// l2_ingest_probe.hip — how fast can one CU pull bytes that every CU reads (the prefill's
// activations) compared with bytes only it reads (its weight rows)? Not part of the product.
// Every workgroup (one per CU at 256) reads S bytes:
//   shared_reg   the SAME S bytes for every workgroup (L2-resident after the first touch per XCD),
//                dwordx4 per lane into registers (xor-reduced, one store per lane)
//   shared_lds   the same bytes, LDS-DMA (global_load_lds 16 B per lane) into a wave-private ring
//   distinct_reg a distinct S-byte slice per workgroup of a cold buffer (rotating > 600 MB)
//   both_reg     S/2 shared + S/2 distinct (the prefill's mix)
// U = loads issued per lane before the first use (in flight together).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o l2_ingest_probe l2_ingest_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(1024) void rd(const u32x4* __restrict__ sh, const u32x4* __restrict__ ds, int n_sh,
                                           int n_ds, unsigned* out, int mod) {
    // n_sh / n_ds: 16-B pieces per workgroup from the shared / distinct buffer
    const int T = blockDim.x;
    const u32x4* d = ds + (long)(blockIdx.x % mod) * n_ds;
    unsigned acc = 0;
    for (int i0 = threadIdx.x; i0 < n_sh; i0 += U * T) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i0 + u * T < n_sh ? sh[i0 + u * T] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (int i0 = threadIdx.x; i0 < n_ds; i0 += U * T) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i0 + u * T < n_ds ? d[i0 + u * T] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    out[blockIdx.x * T + threadIdx.x] = acc;
}

// both streams interleaved in one loop (shared and distinct pieces in flight together)
template <int U>
__global__ __launch_bounds__(1024) void rd_mix(const u32x4* __restrict__ sh, const u32x4* __restrict__ ds, int n,
                                               unsigned* out) {
    const int T = blockDim.x;
    const u32x4* d = ds + (long)blockIdx.x * n;
    unsigned acc = 0;
    for (int i0 = threadIdx.x; i0 < n; i0 += U * T) {
        u32x4 v[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool ok = i0 + u * T < n;
            v[u] = ok ? sh[i0 + u * T] : u32x4{0, 0, 0, 0};
            w[u] = ok ? d[i0 + u * T] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w ^ w[u].x ^ w[u].y ^ w[u].z ^ w[u].w;
    }
    out[blockIdx.x * T + threadIdx.x] = acc;
}

// LDS-DMA of the shared bytes into a wave-private ring of R x 1 KB; U instructions in flight
template <int U>
__global__ __launch_bounds__(1024) void lds_dma(const unsigned char* __restrict__ sh, int n_sh, unsigned* out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, NW = blockDim.x >> 6;
    unsigned char* ring = lds + wave * U * 1024;
    // wave w takes 1-KB chunks w, w + NW, ...
    const int nch = n_sh / 64;  // 1 KB chunks
    int k = 0;
    for (int c = wave; c < nch; c += NW, ++k) {
        auto gp = (const __attribute__((address_space(1))) void*)(sh + (long)c * 1024 + lane * 16);
        auto lp = (__attribute__((address_space(3))) void*)(ring + (k % U) * 1024);
        __builtin_amdgcn_global_load_lds(gp, lp, 16, 0, 0);
        if (k % U == U - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U / 2) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    out[blockIdx.x * blockDim.x + threadIdx.x] = reinterpret_cast<unsigned*>(lds)[threadIdx.x];
}

// The M=32 prefill's DMA pattern (mmq_kernel BN=32, TT=1, W=8): workgroup (x, y) reads weight rows
// 32x..32x+31 (row 2304 B) and tokens 16y..16y+15 (row 4608 B); wave w takes K-stages of SB blocks
// w, w+8, ...: per stage 32 row segments of SB*18 B and 16 token segments of SB*36 B, glds 16 B per
// lane into an NB-deep wave-private ring (pieces numbered row-major, lane-linear).
template <int SB, int NB>
__global__ __launch_bounds__(512) void mmq_pat(const unsigned char* __restrict__ W, const unsigned char* __restrict__ A,
                                               unsigned* out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int RS = SB * 18, TS = SB * 36;              // segment bytes
    constexpr int WP = (RS + 15) / 16, AP = TS / 16;       // 16-B pieces per segment
    constexpr int NP = 32 * WP + 16 * AP;                  // pieces per stage
    constexpr int NI = (NP + 63) / 64;                     // instructions per stage
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int x = blockIdx.x & 127, y = blockIdx.x >> 7;
    unsigned char* ring = lds + wave * NB * NI * 1024;
    const int H = 128 / SB;
    int k = 0;
    for (int h = wave; h < H; h += 8, ++k) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            int p = i * 64 + lane;
            if (p >= NP) p = NP - 1;
            const unsigned char* g;
            if (p < 32 * WP) g = W + (long)(32 * x + p / WP) * 2304 + h * RS + 16 * (p % WP);
            else { p -= 32 * WP; g = A + (long)(16 * y + p / AP) * 4608 + h * TS + 16 * (p % AP); }
            auto gp = (const __attribute__((address_space(1))) void*)g;
            auto lp = (__attribute__((address_space(3))) void*)(ring + ((k % NB) * NI + i) * 1024);
            __builtin_amdgcn_global_load_lds(gp, lp, 16, 0, 0);
        }
        if (k % NB == NB - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (NB - 1)) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    out[blockIdx.x * 512 + threadIdx.x] = reinterpret_cast<unsigned*>(lds)[threadIdx.x];
}

// The register-weight alternative for the M=32 prefill: workgroup x reads weight rows 32x..32x+31
// (2304 B each; two workgroups per row slice, as the 2 token tiles), wave w takes K-stages w, w+8, ..
// of 4 blocks; per stage and row tile a lane (r = lane & 15, q = lane >> 4) loads what the i8 MFMA
// operand needs: per block pair an 8-B load at 4q and a 4-B load at 20 + 4q (+ the d dwords when
// D), NB stages in flight. XOR-reduced, one store per lane. Weights cold (rotated over > 600 MB).
template <int NB, bool D>
__global__ __launch_bounds__(512) void rw_pat(const unsigned char* __restrict__ W, unsigned* out) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    const int x = blockIdx.x & 127;
    unsigned acc = 0;
    const unsigned char* rows[2] = {W + (long)(32 * x + r) * 2304, W + (long)(32 * x + 16 + r) * 2304};
    for (int h0 = wave; h0 < 32; h0 += 8 * NB) {
        unsigned v[NB][2][2][D ? 5 : 3];
#pragma unroll
        for (int s = 0; s < NB; ++s) {
            const int h = min(h0 + 8 * s, 31);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    const unsigned* pp = reinterpret_cast<const unsigned*>(rows[i] + h * 72 + 36 * p);
                    const uint2 a = *reinterpret_cast<const uint2*>(pp + q);
                    v[s][i][p][0] = a.x; v[s][i][p][1] = a.y;
                    v[s][i][p][2] = pp[5 + q];
                    if constexpr (D) { v[s][i][p][3] = pp[0]; v[s][i][p][4] = pp[4]; }
                }
        }
#pragma unroll
        for (int s = 0; s < NB; ++s)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int k = 0; k < (D ? 5 : 3); ++k) acc ^= v[s][i][p][k];
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

__global__ void empty(unsigned* out) {
    if (threadIdx.x == 1023 && blockIdx.x == 100000) out[0] = 1;
}

int main() {
    const long SH = 147456;                 // M=32 Q8_1 activations at K=4096
    const int G = 256;
    const long DS_PER = 147456;             // distinct bytes per workgroup (max)
    const long DS = (long)G * DS_PER;       // 37.7 MB per launch
    const int R = (int)(640L * 1024 * 1024 / DS) + 1;
    unsigned char* sh;
    CK(hipMalloc(&sh, SH));
    CK(hipMemset(sh, 0x5A, SH));
    std::vector<unsigned char*> ds(R);
    for (auto& p : ds) { CK(hipMalloc(&p, DS)); CK(hipMemset(p, 0x33, DS)); }
    unsigned* out;
    CK(hipMalloc(&out, (size_t)G * 1024 * 4 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int L = 200;
    auto timeit = [&](const char* name, auto launch) {
        std::vector<float> v;
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < L; ++i) launch(i);
        CK(hipStreamEndCapture(st, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        for (int r = 0; r < 7; ++r) {
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.push_back(ms * 1000.f / L);
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(gr));
        std::sort(v.begin(), v.end());
        printf("  %-44s %7.3f us/launch\n", name, v[3]);
        fflush(stdout);
        return v[3];
    };
    CK(hipFuncSetAttribute((const void*)lds_dma<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)lds_dma<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("empty 256x512", [&](int) { hipLaunchKernelGGL(empty, dim3(G), dim3(512), 0, st, out); });
    {
        unsigned char* A32;
        CK(hipMalloc(&A32, 32 * 4608));
        CK(hipMemset(A32, 1, 32 * 4608));
        auto pat = [&](const char* nm, auto kern, int lds) {
            CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            timeit(nm, [&](int i) { hipLaunchKernelGGL(kern, dim3(256), dim3(512), lds, st, ds[i % R], A32, out); });
        };
        // cold weights for the register-weight patterns: rotate over > 600 MB of 9.4-MB weight sets
        const int RW = 72;
        std::vector<unsigned char*> wc(RW);
        for (auto& p : wc) { CK(hipMalloc(&p, 9437184)); CK(hipMemset(p, 0x21, 9437184)); }
        if (0) timeit("rw_pat NB=1 (cold)", [&](int i) { hipLaunchKernelGGL((rw_pat<1, false>), dim3(256), dim3(512), 0, st, wc[i % RW], out); });
        if (0) timeit("rw_pat NB=2 (cold)", [&](int i) { hipLaunchKernelGGL((rw_pat<2, false>), dim3(256), dim3(512), 0, st, wc[i % RW], out); });
        if (0) timeit("rw_pat NB=4 (cold)", [&](int i) { hipLaunchKernelGGL((rw_pat<4, false>), dim3(256), dim3(512), 0, st, wc[i % RW], out); });
        if (0) timeit("rw_pat NB=2 +d loads (cold)", [&](int i) { hipLaunchKernelGGL((rw_pat<2, true>), dim3(256), dim3(512), 0, st, wc[i % RW], out); });
        timeit("mmq_pat SB=4 NB=2 weights cold", [&](int i) { hipLaunchKernelGGL((mmq_pat<4, 2>), dim3(256), dim3(512), 8 * 2 * 5 * 1024, st, wc[i % RW], A32, out); });
        timeit("mmq_pat SB=4 NB=4 weights cold", [&](int i) { hipLaunchKernelGGL((mmq_pat<4, 4>), dim3(256), dim3(512), 8 * 4 * 5 * 1024, st, wc[i % RW], A32, out); });
        timeit("mmq_pat SB=8 NB=2 weights cold", [&](int i) { hipLaunchKernelGGL((mmq_pat<8, 2>), dim3(256), dim3(512), 8 * 2 * 9 * 1024, st, wc[i % RW], A32, out); });
        timeit("mmq_pat SB=16 NB=1 weights cold", [&](int i) { hipLaunchKernelGGL((mmq_pat<16, 1>), dim3(256), dim3(512), 8 * 1 * 18 * 1024, st, wc[i % RW], A32, out); });
        timeit("coalesced sh 73.7K + wt 73.7K/2 cold", [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(512), 0, st, (const u32x4*)A32, (const u32x4*)wc[i % RW], 4608, 4608, out, 128); });
        timeit("coalesced wt 73.7K/2 only cold", [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(512), 0, st, (const u32x4*)A32, (const u32x4*)wc[i % RW], 0, 4608, out, 128); });
        timeit("coalesced wt 36.9K (x1) only cold", [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(512), 0, st, (const u32x4*)A32, (const u32x4*)wc[i % RW], 0, 2304, out, 256); });
        pat("mmq_pat SB=4  NB=2", mmq_pat<4, 2>, 8 * 2 * 5 * 1024);
        pat("mmq_pat SB=4  NB=4", mmq_pat<4, 4>, 8 * 4 * 5 * 1024);
        pat("mmq_pat SB=8  NB=2", mmq_pat<8, 2>, 8 * 2 * 9 * 1024);
        pat("mmq_pat SB=16 NB=1", mmq_pat<16, 1>, 8 * 1 * 18 * 1024);
    }
    // the M=32 prefill's byte pattern: 73.7 KB of shared activations + 73.7 KB of weights per
    // workgroup, each weight slice read by 2 workgroups (9.4 MB unique), one or two passes
    for (int T : {512, 1024}) {
        char nm[128];
        snprintf(nm, sizeof nm, "mmq pattern sh 73.7K + ds 73.7K/2 T=%4d U=4", T);
        timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(T), 0, st, (const u32x4*)sh, (const u32x4*)ds[i % R], 4608, 4608, out, 128); });
        snprintf(nm, sizeof nm, "weights only ds 73.7K/2 T=%4d U=4", T);
        timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(T), 0, st, (const u32x4*)sh, (const u32x4*)ds[i % R], 0, 4608, out, 128); });
        snprintf(nm, sizeof nm, "weights only ds 36.9K    T=%4d U=4", T);
        timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(T), 0, st, (const u32x4*)sh, (const u32x4*)ds[i % R], 0, 2304, out, 256); });
        snprintf(nm, sizeof nm, "sh 36.9K + ds 36.9K (ks2) T=%4d U=4", T);
        timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(T), 0, st, (const u32x4*)sh, (const u32x4*)ds[i % R], 2304, 2304, out, 256); });
    }
    const u32x4* shp = (const u32x4*)sh;
    for (int T : {512, 1024}) {
        for (long S : {73728L, 147456L}) {
            const int n = (int)(S / 16);
            char nm[128];
            snprintf(nm, sizeof nm, "shared_reg  S=%6ld T=%4d U=4", S, T);
            timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(T), 0, st, shp, (const u32x4*)ds[i % R], n, 0, out, G); });
            snprintf(nm, sizeof nm, "shared_reg  S=%6ld T=%4d U=8", S, T);
            timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<8>, dim3(G), dim3(T), 0, st, shp, (const u32x4*)ds[i % R], n, 0, out, G); });
            snprintf(nm, sizeof nm, "distinct_reg S=%6ld T=%4d U=4", S, T);
            timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(T), 0, st, shp, (const u32x4*)ds[i % R], 0, n, out, G); });
            snprintf(nm, sizeof nm, "distinct_reg S=%6ld T=%4d U=8", S, T);
            timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<8>, dim3(G), dim3(T), 0, st, shp, (const u32x4*)ds[i % R], 0, n, out, G); });
            snprintf(nm, sizeof nm, "seq sh+ds S/2+S/2 T=%4d U=4", T);
            timeit(nm, [&](int i) { hipLaunchKernelGGL(rd<4>, dim3(G), dim3(T), 0, st, shp, (const u32x4*)ds[i % R], n / 2, n / 2, out, G); });
            snprintf(nm, sizeof nm, "mix sh+ds S/2+S/2 T=%4d U=4", T);
            timeit(nm, [&](int i) { hipLaunchKernelGGL(rd_mix<4>, dim3(G), dim3(T), 0, st, shp, (const u32x4*)ds[i % R], n / 2, out); });
            snprintf(nm, sizeof nm, "shared_lds  S=%6ld T=%4d U=4", S, T);
            timeit(nm, [&](int) { hipLaunchKernelGGL(lds_dma<4>, dim3(G), dim3(T), (T / 64) * 4 * 1024, st, sh, n, out); });
            snprintf(nm, sizeof nm, "shared_lds  S=%6ld T=%4d U=8", S, T);
            timeit(nm, [&](int) { hipLaunchKernelGGL(lds_dma<8>, dim3(G), dim3(T), (T / 64) * 8 * 1024, st, sh, n, out); });
        }
    }
    return 0;
}
