// qg_calib.hip — libqg_calib.so (include/qg/qg_calib.h): the single-launch floor of bench.py.
// Not part of libqg_hip.so: the product library holds only the product's kernels.
#include <hip/hip_runtime.h>

#include "../../include/qg/qg_calib.h"

namespace {

__global__ __launch_bounds__(1024) void calib_empty_kernel() {}

template <int P>
__global__ __launch_bounds__(1024) void calib_read_kernel(const uint4* __restrict__ src, long n16, uint32_t* __restrict__ sink) {
    const long base = (long)blockIdx.x * blockDim.x * P + threadIdx.x;
    uint4 v[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const long i = base + (long)j * blockDim.x;
        v[j] = i < n16 ? src[i] : make_uint4(0, 0, 0, 0);
    }
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) x ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    if (x == 0x9E3779B9u && threadIdx.x == 0x3FF) sink[0] = x;
}

template <int P> hipError_t read_launch(const void* src, long n16, int block, uint32_t* sink, hipStream_t st) {
    const long per = (long)block * P;
    const int grid = (int)((n16 + per - 1) / per);
    hipLaunchKernelGGL(calib_read_kernel<P>, dim3(grid), dim3(block), 0, st, (const uint4*)src, n16, sink);
    return hipGetLastError();
}

}  // namespace

extern "C" {

int qg_calib_empty(int grid, int block, qg_stream_t stream) {
    if (grid <= 0 || block < 64 || block > 1024 || block % 64 != 0) return QG_ERR_INVALID_ARG;
    hipLaunchKernelGGL(calib_empty_kernel, dim3(grid), dim3(block), 0, (hipStream_t)stream);
    return hipGetLastError() == hipSuccess ? QG_OK : QG_ERR_HIP;
}

int qg_calib_read(const void* src, size_t bytes, int loads_per_thread, int block, uint32_t* sink, qg_stream_t stream) {
    if (!src || !sink || bytes == 0 || bytes % 16 != 0 || ((uintptr_t)src & 15) != 0) return QG_ERR_INVALID_ARG;
    if (block < 64 || block > 1024 || block % 64 != 0) return QG_ERR_INVALID_ARG;
    const long n16 = (long)(bytes / 16);
    const hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    switch (loads_per_thread) {
        case 1: e = read_launch<1>(src, n16, block, sink, st); break;
        case 2: e = read_launch<2>(src, n16, block, sink, st); break;
        case 4: e = read_launch<4>(src, n16, block, sink, st); break;
        case 8: e = read_launch<8>(src, n16, block, sink, st); break;
        default: return QG_ERR_INVALID_ARG;
    }
    return e == hipSuccess ? QG_OK : QG_ERR_HIP;
}

}  // extern "C"
