// qg_kernels.hpp — host-side view of the kernel families behind the C-ABI (qg_api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>

namespace qg {

// Activation input of a product: Q8_1 blocks, or FP32 / FP16 rows quantized inside the kernel.
enum : int { AIN_Q8_1 = 0, AIN_F32 = 1, AIN_F16_FUSED = 2 };

// Weight layouts of the MFMA kernel (qg_mmq_kernel.hpp): the reference's rows, or qg_tile_weights' tiles.
// LAY_TILED_ACT: tiled weights AND tiled activations (qg_quantize_q8_1_tiled: 16-token tiles, 4-block stages,
// each (token tile, stage) one contiguous 2304-B run of the 16 tokens' 144-B stage segments, zero padded)
enum : int { LAY_ROWS = 0, LAY_TILED = 1, LAY_TILED_ACT = 2 };
constexpr int ACT_TILE = 16;                              // tokens per activation tile (LAY_TILED_ACT)
constexpr int ACT_STG = ACT_TILE * 4 * 36;                // bytes per (token tile, stage): 2304

// One W4A8 product C = A_q8_1 * B_w^T, activation-major indices (m = activation row, n = weight
// row); the output element (m, n) lives at C[m * ldc_m + n * ldc_n].
struct GemmArgs {
    const void* A = nullptr;     // block_q8_1 [M][K/32] (ain == AIN_Q8_1), else float/half [M][K]
    int ain = AIN_Q8_1;
    const void* B = nullptr;     // weight blocks [N][K/32] of type wtype (lay = LAY_ROWS), or the
                                 // qg_tile_weights layout (lay = LAY_TILED, qg_mmq_kernel.hpp)
    int lay = 0;                 // weight layout: 0 the reference's rows, 1 tiled
    int nbw = 0;                 // LAY_ROWS: weight blocks per row when it differs from K/32 (the
                                 // qg_repack_weights rows of qg_gemm_w4a8_prepacked), else 0
    float* C = nullptr;
    int32_t* sumi = nullptr;     // debug: per-block int32 dots [M][N][K/32] instead of C
    int M = 0, N = 0, K = 0;
    int wtype = 0;
    long ldc_m = 0, ldc_n = 1;
    int batch = 1;               // strided batch of independent products (GEMV path)
    long sA = 0, sB = 0, sC = 0; // batch strides: bytes, bytes, floats
    void* ws = nullptr;          // optional device workspace (split-K partials + tile counters)
    size_t ws_bytes = 0;
    const void* group = nullptr; // GEMV path: a GemvGroup descriptor (qg_gemm_w4a8_grouped); M, K, wtype
                                 // shared, N = the largest item's
    char* describe = nullptr;    // qg_debug_config: the leaf launcher writes the kernel it would
    size_t describe_len = 0;     // launch here (family + template parameters) and launches nothing
};

// Descriptor of a grouped GEMV launch (qg_gemm_w4a8_grouped), passed by value as the kernel argument.
constexpr int GEMV_GROUP_MAX = 64;
struct GemvItemDesc {  // 32 B: one s_load_dwordx8 in the kernel
    const void* A;
    const void* B;
    float* C;
    int N, ldc;
};
struct GemvGroup {
    // full: every item has the launch's row-tile count (no workgroup exits early) — gemvg_kernel
    int count, M, K, full;
    GemvItemDesc it[GEMV_GROUP_MAX];
};

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel instantiation, device): `done`
// is that instantiation's atomic device bitmask (a process may drive several GPUs from
// several threads; the attribute is per device). Not a stream operation, so capture-safe.
inline hipError_t set_max_lds_once(const void* fn, int bytes, std::atomic<unsigned long long>& done) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    const unsigned long long bit = dev < 64 ? 1ull << dev : 0ull;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess && bit) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

// Compute units of the current device (hipDeviceAttributeMultiprocessorCount, cached per device; 256 on a
// whole MI355X, and when no device is visible — the qg_debug_config queries of a GPU-less build host).
// "One dispatch round" tile choices compare grids against it (CU-partitioned devices).
int device_cus();

// printf-style description of a kernel instantiation into g.describe (qg_debug_config). SUMI is
// deliberately not part of it: the parity hook must name the product's kernel.
void describe_kernel(const GemmArgs& g, const char* fmt, ...);

// GEMV / small batch (M <= 8): nibble-plane v_dot8 (Q4_0 / Q4_1) or v_dot4 (Q5_x / Q8_0) on
// register-resident weight units, activation records staged in LDS.
bool gemv_eligible(const GemmArgs& g);
hipError_t launch_gemv(const GemmArgs& g, hipStream_t st);

// The decode GEMV (M <= 4) on the tiled layout (qg_gemvt.hip, round 6): waves of 16 rows x 4 stages reading
// whole 256-B plane runs, the row kernel's dot and per-block terms (bit-identical per block to the
// reference's), fixed summation order. run_tiled sends it M = 1..2 up to K/32 = 256; M = 3..4 only in builds
// without the small-batch decode (QG_TILED_GEMVM=0, A/B).
bool gemvt_eligible(const GemmArgs& g);
hipError_t launch_gemvt(const GemmArgs& g, hipStream_t st);

// Small-batch decode (M = 3..4, and 2 at K/32 > 256) on the tiled layout (qg_gemvm.hip, round 6): 16-row half tiles, the QS
// pieces straight from HBM into v_mfma_i32_16x16x32_i8 operands, the prefill's MFMA-assisted epilogue.
bool gemvm_eligible(const GemmArgs& g);
hipError_t launch_gemvm(const GemmArgs& g, hipStream_t st);

// Prefill (M >= 5): LDS-DMA staged weights + activations, one v_mfma_i32_16x16x32_i8 per Q-block,
// MFMA-assisted (v_mfma_f32_16x16x16_f16) scale epilogue.
bool mfma_eligible(const GemmArgs& g);
hipError_t launch_mfma(const GemmArgs& g, hipStream_t st);


// Any shape / alignment with K % 32 == 0 (byte-granular loads); also the debug sumi fallback.
hipError_t launch_generic(const GemmArgs& g, hipStream_t st);

// Odd K / 32 (weight rows off dword alignment) or 2-B aligned weights: one wave per weight row,
// realigned dword loads, the GEMV's records and block terms (qg_ragged.hip).
bool ragged_eligible(const GemmArgs& g);
hipError_t launch_ragged(const GemmArgs& g, hipStream_t st);

// Odd K / 32 at prefill sizes (qg_repack.hip): weights and activations copied into rows padded with
// zero blocks (d = 0, s = 0) to K'/32 = round_up(K/32, 8), then the MFMA kernel on K'. Every padded
// term is an exact +0, so each real block's int32 dot and scale product is what the MFMA kernel
// computes at any aligned K; the sumi hook runs the same MFMA instantiation into a padded image and
// compacts it. repack_eligible: shape rules only (pointers not needed).
bool repack_eligible(const GemmArgs& g);
// returns hipErrorNotReady (nothing enqueued) when no workspace can be had right now (e.g. capture
// without a caller workspace g.ws of >= repack_workspace_bytes(g))
hipError_t launch_repack_mfma(const GemmArgs& g, hipStream_t st);
size_t repack_workspace_bytes(const GemmArgs& g);  // padded weights + activations
// Weights [N][K/32] -> rows of K'/32 = round_up(K/32, 8) blocks, zero blocks after the real ones
// (qg_repack_weights); activations the same (qg_gemm_w4a8_prepacked). Both enqueue one kernel.
int padded_blocks(int K);
// Weights [N][K/32] -> the tiled layout (qg_tile_weights; tiled_fmt in qg_mmq_kernel.hpp): rows in
// tiles of 32, K/32 in stages of 4 blocks, zero blocks / rows as padding. One kernel.
size_t tiled_weight_bytes(int N, int K, int wtype);
hipError_t launch_tile_weights(const void* B, void* B_tiled, int N, int K, int wtype, hipStream_t st);
hipError_t launch_pad_rows(const void* src, void* dst, long rows, int row_bytes, int padded_row_bytes, hipStream_t st);

// W4A16 / W8A16: FP32 activations (A = float[M][K]) x Q4_0 / Q8_0 weights, fp32 arithmetic.
// g.ws / g.ws_bytes: optional caller workspace for the split-K prefill (>= w16_workspace_bytes,
// 256-B aligned, zero before its first use; left zero by every launch).
hipError_t launch_w16(const GemmArgs& g, hipStream_t st);
size_t w16_workspace_bytes(int M, int N, int K);

// FP32 GEMM C = A . B^T (the unquantized baseline), A = float[M][K], B = float[N][K].
hipError_t launch_fp32(const GemmArgs& g, hipStream_t st);

// Device workspace owned by the library for stream st (split-K partials and tile counters):
// at least `bytes`, zeroed when first allocated, reused by every later launch on st (launches on
// one stream are ordered, and every split-K launch leaves its counters zero). nullptr when it
// cannot be allocated right now (e.g. the stream is being captured): callers fall back to a
// kernel without a workspace.
// hold: keep the buffer's lock until the caller has enqueued everything that uses it.
void* stream_workspace(hipStream_t st, size_t bytes, int slot = 0, std::unique_lock<std::mutex>* hold = nullptr);

// Quantizers / dequantizers (one thread per 32-element block, reference rounding semantics).
hipError_t launch_quantize(int type, int variant, const float* x, void* y, int64_t nblocks, hipStream_t st);
// FP16 -> Q8_1 with the fused kernel's semantics (kernels/gemm/gemm_fused.cuh:76-143).
hipError_t launch_quantize_f16_fused(const void* x, void* y, int64_t nblocks, hipStream_t st);
// FP32 rows of nb blocks -> Q8_1 rows of nbp blocks, zero blocks after the real ones.
hipError_t launch_quantize_q8_1_padded(const float* x, void* y, int64_t rows, int nb, int nbp, hipStream_t st);
// the tiled activation layout (LAY_TILED_ACT): its size, the quantizer writing it, the Q8_1-row repack into it
size_t tiled_act_bytes(int M, int K);
hipError_t launch_quantize_q8_1_tiled(const float* x, void* y, int M, int K, hipStream_t st);
hipError_t launch_tile_activations(const void* a, void* y, int M, int K, hipStream_t st);
hipError_t launch_dequantize(int type, const void* x, float* y, int64_t nblocks, hipStream_t st);

}  // namespace qg
