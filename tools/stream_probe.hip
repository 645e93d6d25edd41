// stream_probe.hip — calibration microbenchmark: how fast can ONE launch stream an N-byte weight
// matrix from HBM on this MI355X? (floor for the W4A8 GEMV). Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip && ./stream_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Each thread reads UNR consecutive-in-wave 16-B chunks (stride = grid threads * 16 B).
template <int UNR, bool NT>
__global__ __launch_bounds__(256) void stream_read(const u32x4* __restrict__ p, long n16, unsigned* out) {
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long nth = (long)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (long base = tid; base < n16; base += nth * UNR) {
        u32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            long i = base + u * nth;
            if (i < n16) v[u] = NT ? __builtin_nontemporal_load(p + i) : p[i];
            else v[u] = u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keep the loads alive
}

template <int UNR, bool NT>
void run(const char* name, std::vector<u32x4*>& bufs, long bytes, int grid, unsigned* out, hipStream_t st) {
    const long n16 = bytes / 16;
    const int R = (int)bufs.size();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 2 * R; ++i) stream_read<UNR, NT><<<grid, 256, 0, st>>>(bufs[i % R], n16, out);
    // cold: rotate through R copies, 256 launches back to back
    const int L = 256;
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < L; ++i) stream_read<UNR, NT><<<grid, 256, 0, st>>>(bufs[i % R], n16, out);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double cold = ms * 1e3 / L;
    // single launch bracketed by events (cold copy), averaged
    double single = 0;
    for (int i = 0; i < 64; ++i) {
        CK(hipEventRecord(e0, st));
        stream_read<UNR, NT><<<grid, 256, 0, st>>>(bufs[(i * 7) % R], n16, out);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        single += ms * 1e3 / 64;
    }
    // hot: same copy
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < L; ++i) stream_read<UNR, NT><<<grid, 256, 0, st>>>(bufs[0], n16, out);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double hot = ms * 1e3 / L;
    printf("%-14s bytes=%9ld grid=%5d unr=%d nt=%d  cold %7.3f us (%6.0f GB/s)  single %7.3f us  hot %7.3f us (%6.0f GB/s)\n",
           name, bytes, grid, UNR, (int)NT, cold, bytes / cold / 1e3, single, hot, bytes / hot / 1e3);
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
}

__global__ void empty_kernel() {}

int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    unsigned* out;
    CK(hipMalloc(&out, 1 << 20));
    // empty-kernel launch floor
    {
        hipEvent_t e0, e1; float ms;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        for (int i = 0; i < 100; ++i) empty_kernel<<<256, 256, 0, st>>>();
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < 1000; ++i) empty_kernel<<<256, 256, 0, st>>>();
        CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        printf("empty kernel (256 WGs) back-to-back: %.3f us/launch\n", ms);
    }
    long sizes[] = {9437184L, 9216000L, 73728000L, 302L << 20};
    for (long bytes : sizes) {
        const int R = (int)((700L << 20) / bytes) + 1;
        std::vector<u32x4*> bufs(R);
        for (auto& b : bufs) { CK(hipMalloc(&b, bytes)); CK(hipMemset(b, 1, bytes)); }
        for (int grid : {256, 512, 1024, 2048}) {
            run<1, true>("unr1_nt", bufs, bytes, grid, out, st);
            run<4, true>("unr4_nt", bufs, bytes, grid, out, st);
            run<4, false>("unr4", bufs, bytes, grid, out, st);
            run<9, true>("unr9_nt", bufs, bytes, grid, out, st);
        }
        for (auto& b : bufs) CK(hipFree(b));
    }
    return 0;
}
