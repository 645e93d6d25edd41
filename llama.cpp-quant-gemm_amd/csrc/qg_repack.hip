// qg_repack.hip — odd K / 32 at prefill sizes through the MFMA kernel.
//
// With K/32 odd, every other weight row starts 2 bytes off a dword, which the MFMA kernel's LDS-DMA
// pieces cannot address; the ragged kernel (qg_ragged.hip) serves those shapes with one wave per
// weight row and no matrix cores (K = 4128: 24.6 us at M = 32, 45.9 us at M = 64 against 6-9 us for
// the MFMA kernel on the same bytes; profiles/tools_archive/repack_probe.py, profiles/r02_tuning/repack_probe.txt).
// Here one streaming kernel copies the weights [N][K/32] and the activations [M][K/32] into rows of
// K'/32 = round_up(K/32, 8) blocks in a per-stream workspace, the extra blocks all zero bytes
// (d = 0 and s = 0: each padded term of gemm_reference.h:202-212 is an exact +0), and the MFMA
// kernel runs on K' (8-block rows also give it the 16-B piece form, P16). The sumi parity hook
// runs the same MFMA instantiation into a [M][N][K'/32] image and compacts it to [M][N][K/32].
#include "qg_common.hpp"
#include "qg_kernels.hpp"
#include "qg_mmq_kernel.hpp"  // tiled_fmt: the LAY_TILED planes

namespace qg {

namespace {
constexpr int PADB = 8;  // pad K/32 up to a multiple of this many blocks

int wbytes(int t) {
    switch (t) {
        case FMT_Q4_0: return 18;
        case FMT_Q4_1: return 20;
        case FMT_Q5_0: return 22;
        case FMT_Q5_1: return 24;
        case FMT_Q8_0: return 34;
    }
    return 0;
}

// One thread per 8-byte word of the padded images (weights first, then activations). Sources are
// 2-B aligned (every block size is even, and so is every row's byte length): four u16 loads per
// word, zero past the row's real bytes.
__global__ __launch_bounds__(256) void repack_pad_kernel(const uint16_t* __restrict__ B, uint64_t* __restrict__ Bp,
                                                         long wwords, int rb, int rbp,
                                                         const uint16_t* __restrict__ A, uint64_t* __restrict__ Ap,
                                                         long awords, int ab, int abp) {
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    const uint16_t* src = B;
    uint64_t* dst = Bp;
    int sb = rb, db = rbp;
    if (i >= wwords) {
        i -= wwords;
        if (i >= awords) return;
        src = A; dst = Ap; sb = ab; db = abp;
    }
    const int wpr = db / 8;
    const long row = i / wpr;
    const int off = (int)(i - row * wpr) * 8;  // byte offset in the padded row
    const uint16_t* s = src + (row * sb + off) / 2;
    uint64_t v = 0;
    if (off + 8 <= sb) {
        v = (uint64_t)s[0] | ((uint64_t)s[1] << 16) | ((uint64_t)s[2] << 32) | ((uint64_t)s[3] << 48);
    } else {
#pragma unroll
        for (int h = 0; h < 4; ++h)
            if (off + 2 * h < sb) v |= (uint64_t)s[h] << (16 * h);
    }
    dst[i] = v;
}

// LAY_TILED (qg_tile_weights; the layout is specified with tiled_fmt in qg_mmq_kernel.hpp): one thread per
// block slot (row r of the tile-padded N, block b of the stage-padded K/32) reads its source block (2-B
// aligned: u16 loads; zero bytes for r >= N or b >= nb) and scatters its fields into the planes of its
// (tile, stage) run. A load-time copy: the scattered 4-B stores are not on any per-call path.
template <int F>
__global__ __launch_bounds__(256) void tile_weights_kernel(const uint16_t* __restrict__ B, uint8_t* __restrict__ Bt, int N, int nb,
                                                          int H, long total) {
    using T = wfmt<F>;
    using TF = tiled_fmt<F>;
    const long g = (long)blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    const int nbp = H * MMQ_SB;
    const long r = g / nbp;
    const int b = (int)(g - r * nbp);
    constexpr int HW = T::BB / 2;  // u16 words per block
    uint16_t w[HW];
#pragma unroll
    for (int i = 0; i < HW; ++i) w[i] = 0;
    if (r < N && b < nb) {
        const uint16_t* src = B + (r * nb + b) * HW;
#pragma unroll
        for (int i = 0; i < HW; ++i) w[i] = src[i];
    }
    auto dw = [&](int byte_off) { return (uint32_t)w[byte_off / 2] | ((uint32_t)w[byte_off / 2 + 1] << 16); };
    const int rr = (int)(r % TILE_ROWS), i16 = rr / 16, r16 = rr % 16, h = b / MMQ_SB, bb = b % MMQ_SB;
    uint8_t* st = Bt + ((r / TILE_ROWS) * H + h) * (long)TF::STG;
    constexpr int NQ = T::Q8 ? 8 : 4;  // qs dwords per block
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        const int qq = j % 4, half = j / 4;
        *reinterpret_cast<uint32_t*>(st + i16 * 64 * TF::QSL + half * 1024 + (qq * 16 + r16) * 16 + bb * 4) = dw(T::QS + 4 * j);
    }
    if constexpr (T::QH >= 0) *reinterpret_cast<uint32_t*>(st + TF::OQH + rr * 16 + bb * 4) = dw(T::QH);
    *reinterpret_cast<uint16_t*>(st + TF::OSC + rr * TF::SCB + bb * 2) = w[0];
    if constexpr (T::MOFF >= 0) *reinterpret_cast<uint16_t*>(st + TF::OSC + rr * TF::SCB + 8 + bb * 2) = w[T::MOFF / 2];
}

// sumi image [M][N][nbp] -> [M][N][nb]
__global__ __launch_bounds__(256) void sumi_compact_kernel(const int32_t* __restrict__ src, int32_t* __restrict__ dst,
                                                           long total, int nb, int nbp) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const long r = i / nb;
    dst[i] = src[r * nbp + (i - r * nb)];
}

inline long round256(long x) { return (x + 255) / 256 * 256; }

GemmArgs padded(const GemmArgs& g) {
    GemmArgs g2 = g;
    const int nbp = (g.K / QK + PADB - 1) / PADB * PADB;
    g2.K = nbp * QK;
    return g2;
}
}  // namespace

// Prefill shapes only (M >= 32: at M = 16 the ragged kernel is as fast, 13.9 vs 13.7 us for Q4_0,
// and faster for Q8_0, 15.2 vs 16.5 us; profiles/r02_tuning/repack_probe.txt) and
// enough weight rows to amortise the copy; one product per call; the padded MFMA shape must be
// one the MFMA kernel takes (checked with placeholder 256-B aligned pointers).
bool repack_eligible(const GemmArgs& g) {
    if (g.batch != 1 || g.M < 32 || g.N < 1024 || g.ain != AIN_Q8_1 || g.K % QK != 0) return false;
    if (wbytes(g.wtype) == 0 || ((uintptr_t)g.A & 1) != 0 || ((uintptr_t)g.B & 1) != 0) return false;
    const long nbp = (g.K / QK + PADB - 1) / PADB * PADB;
    if ((long)g.N * nbp * wbytes(g.wtype) >= (1L << 40)) return false;
    GemmArgs g2 = padded(g);
    g2.A = reinterpret_cast<const void*>(256);
    g2.B = reinterpret_cast<const void*>(256);
    return mfma_eligible(g2);
}

int padded_blocks(int K) { return (K / QK + PADB - 1) / PADB * PADB; }

size_t repack_workspace_bytes(const GemmArgs& g) {
    const int nbp = padded_blocks(g.K);
    const long wimg = round256((long)g.N * nbp * wbytes(g.wtype)), aimg = round256((long)g.M * nbp * Q8_1_BYTES);
    return (size_t)(wimg + aimg);
}

hipError_t launch_pad_rows(const void* src, void* dst, long rows, int rb, int rbp, hipStream_t st) {
    const long words = rows * rbp / 8;
    const long blocks = (words + 255) / 256;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(repack_pad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<const uint16_t*>(src),
                       static_cast<uint64_t*>(dst), words, rb, rbp, static_cast<const uint16_t*>(nullptr),
                       static_cast<uint64_t*>(nullptr), 0L, 0, 8);
    return hipGetLastError();
}

size_t tiled_weight_bytes(int N, int K, int wtype) {
    const long tiles = (N + TILE_ROWS - 1) / TILE_ROWS, stages = (K / QK + MMQ_SB - 1) / MMQ_SB;
    return (size_t)(tiles * stages * TILE_ROWS * MMQ_SB * wbytes(wtype));
}

hipError_t launch_tile_weights(const void* B, void* Bt, int N, int K, int wtype, hipStream_t st) {
    const int nb = K / QK, H = (nb + MMQ_SB - 1) / MMQ_SB;
    const long total = (long)(N + TILE_ROWS - 1) / TILE_ROWS * TILE_ROWS * H * MMQ_SB;
    const long blocks = (total + 255) / 256;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffL) return hipErrorInvalidValue;
    const uint16_t* b16 = static_cast<const uint16_t*>(B);
    uint8_t* bt = static_cast<uint8_t*>(Bt);
    switch (wtype) {
        case FMT_Q4_0: hipLaunchKernelGGL(tile_weights_kernel<FMT_Q4_0>, dim3((unsigned)blocks), dim3(256), 0, st, b16, bt, N, nb, H, total); break;
        case FMT_Q4_1: hipLaunchKernelGGL(tile_weights_kernel<FMT_Q4_1>, dim3((unsigned)blocks), dim3(256), 0, st, b16, bt, N, nb, H, total); break;
        case FMT_Q5_0: hipLaunchKernelGGL(tile_weights_kernel<FMT_Q5_0>, dim3((unsigned)blocks), dim3(256), 0, st, b16, bt, N, nb, H, total); break;
        case FMT_Q5_1: hipLaunchKernelGGL(tile_weights_kernel<FMT_Q5_1>, dim3((unsigned)blocks), dim3(256), 0, st, b16, bt, N, nb, H, total); break;
        case FMT_Q8_0: hipLaunchKernelGGL(tile_weights_kernel<FMT_Q8_0>, dim3((unsigned)blocks), dim3(256), 0, st, b16, bt, N, nb, H, total); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_repack_mfma(const GemmArgs& g, hipStream_t st) {
    GemmArgs g2 = padded(g);
    const int nb = g.K / QK, nbp = g2.K / QK;
    const int rb = nb * wbytes(g.wtype), rbp = nbp * wbytes(g.wtype);
    const int ab = nb * Q8_1_BYTES, abp = nbp * Q8_1_BYTES;
    const long wimg = round256((long)g.N * rbp);
    if (g.describe) {  // configuration query: the MFMA instantiation this call would run
        g2.A = reinterpret_cast<const void*>(256);
        g2.B = reinterpret_cast<const void*>(256);
        return launch_mfma(g2, st);
    }
    // the caller's workspace (qg_gemm_w4a8_ws: capture-safe), else the library's per-stream one,
    // its lock held until the last kernel below is enqueued
    const size_t need = repack_workspace_bytes(g);
    std::unique_lock<std::mutex> hold;
    uint8_t* ws = nullptr;
    if (g.ws && g.ws_bytes >= need && ((uintptr_t)g.ws & 255) == 0) ws = static_cast<uint8_t*>(g.ws);
    else ws = static_cast<uint8_t*>(stream_workspace(st, need, 1, &hold));
    if (!ws) return hipErrorNotReady;
    const long wwords = (long)g.N * rbp / 8, awords = (long)g.M * abp / 8;
    const long blocks = (wwords + awords + 255) / 256;
    if (blocks > 0x7fffffffL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(repack_pad_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                       static_cast<const uint16_t*>(g.B), reinterpret_cast<uint64_t*>(ws), wwords, rb, rbp,
                       static_cast<const uint16_t*>(g.A), reinterpret_cast<uint64_t*>(ws + wimg), awords, ab, abp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    g2.B = ws;
    g2.A = ws + wimg;
    g2.ws = nullptr;
    g2.ws_bytes = 0;
    if (!g.sumi) return launch_mfma(g2, st);
    // parity hook only: the padded sumi image is a stream-ordered temporary (not kept in
    // the per-stream buffer), compacted to [M][N][K/32] and freed on the stream
    void* simg = nullptr;
    e = hipMallocAsync(&simg, (size_t)g.M * g.N * nbp * 4, st);
    if (e != hipSuccess) return e;
    g2.sumi = static_cast<int32_t*>(simg);
    e = launch_mfma(g2, st);
    if (e == hipSuccess) {
        const long total = (long)g.M * g.N * nb;
        hipLaunchKernelGGL(sumi_compact_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                           g2.sumi, g.sumi, total, nb, nbp);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(simg, st);
    return e != hipSuccess ? e : f;
}

}  // namespace qg
