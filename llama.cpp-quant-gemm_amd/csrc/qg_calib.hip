// qg_calib.hip — libqg_calib.so (include/qg/qg_calib.h): the single-launch floor of bench.py.
// Not part of libqg_hip.so: the product library holds only the product's kernels.
#include <hip/hip_runtime.h>

#include "../../include/qg/qg_calib.h"
#include "qg_common.hpp"  // xcd_tile: the GEMV's tile order

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

// The M = 1 GEMV's own load shape without its arithmetic: 1024-thread workgroups
// of 16 weight rows, one wave per row, lane l loading the row's 36-B unit l (9 dword loads, the GEMV's
// 2-block Q4_0 units: gemv1_kernel<2, 2, 64, 1024>), the XCD-aware tile order of grids of one dispatch
// round (qg_common.hpp xcd_tile); STORE: each row's lane 63 stores one float (the GEMV's 4-B output per
// row) — so the floor set separates the unit-shape read and the output write-back from the dot.
template <bool STORE>
__global__ __launch_bounds__(1024) void calib_units_kernel(const uint8_t* __restrict__ B, int N, int units, float* __restrict__ out,
                                                         uint32_t* __restrict__ sink) {
    const int tile = gridDim.x <= 512 ? qg::xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int row = tile * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const bool ok = row < N && lane < units;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(B + ((long)(ok ? row : 0) * units + (ok ? lane : 0)) * 36);
    uint32_t x = 0;
#pragma unroll
    for (int v = 0; v < 9; ++v) x ^= p[v];
    if constexpr (STORE) {
        // every lane's loads feed the stored value (a wave-wide XOR over DPP row ops, as the GEMV's
        // group_sum_last): with only lane 63's value used, the compiler sank the loads under the store's
        // lane predicate and the launch read 1/64 of the bytes
        auto dx = [](uint32_t v, auto ctrl, auto rm) {
            return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, decltype(ctrl)::value, decltype(rm)::value, 0xF, false);
        };
        x ^= dx(x, qg::ic<0xB1>{}, qg::ic<0xF>{});
        x ^= dx(x, qg::ic<0x4E>{}, qg::ic<0xF>{});
        x ^= dx(x, qg::ic<0x114>{}, qg::ic<0xF>{});
        x ^= dx(x, qg::ic<0x118>{}, qg::ic<0xF>{});
        x ^= dx(x, qg::ic<0x142>{}, qg::ic<0xA>{});
        x ^= dx(x, qg::ic<0x143>{}, qg::ic<0xC>{});
        if (row < N && lane == 63) out[row] = __uint_as_float(x & 0x3FFFFFFFu);
    } else {
        if (x == 0x9E3779B9u && threadIdx.x == 0x3FF) sink[0] = x;
    }
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

int qg_calib_read_units(const void* B, int N, int K, float* out, uint32_t* sink, qg_stream_t stream) {
    if (!B || !sink || N <= 0 || K <= 0 || K % 64 != 0 || K / 64 > 64 || ((uintptr_t)B & 3) != 0) return QG_ERR_INVALID_ARG;
    const int grid = (N + 15) / 16, units = K / 64;
    if (out) hipLaunchKernelGGL(calib_units_kernel<true>, dim3(grid), dim3(1024), 0, (hipStream_t)stream, (const uint8_t*)B, N,
                                units, out, sink);
    else hipLaunchKernelGGL(calib_units_kernel<false>, dim3(grid), dim3(1024), 0, (hipStream_t)stream, (const uint8_t*)B, N,
                            units, out, sink);
    return hipGetLastError() == hipSuccess ? QG_OK : QG_ERR_HIP;
}

}  // extern "C"
