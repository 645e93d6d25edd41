// enqueue_probe.cpp — host cost of one C-ABI call (enqueue only, no sync) per kernel family, and the
// per-launch wall time with a synchronisation after every launch (the reference harness's
// protocol). Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -o enqueue_probe enqueue_probe.cpp \
//         -L../llama.cpp-quant-gemm_amd/quant_gemm -lqg_hip -Wl,-rpath,'$ORIGIN/../llama.cpp-quant-gemm_amd/quant_gemm'
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <functional>
#include <vector>

#include "qg/qg.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
    const int N = 4096, K = 4096;
    float *A, *C;
    void *Aq, *Bq;
    CK(hipMalloc(&A, 32 * K * 4)); CK(hipMalloc(&C, 32 * N * 4));
    CK(hipMalloc(&Aq, 32 * K / 32 * 36)); CK(hipMalloc(&Bq, (size_t)N * K / 32 * 18));
    CK(hipMemset(A, 0, 32 * K * 4)); CK(hipMemset(Aq, 0, 32 * K / 32 * 36)); CK(hipMemset(Bq, 0, (size_t)N * K / 32 * 18));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto probe = [&](const char* name, const std::function<int()>& f) {
        for (int i = 0; i < 50; ++i) f();
        (void)hipDeviceSynchronize();
        const int L = 2000;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < L; ++i) f();
        auto t1 = std::chrono::steady_clock::now();
        (void)hipDeviceSynchronize();
        auto t2 = std::chrono::steady_clock::now();
        const double enq = std::chrono::duration<double, std::micro>(t1 - t0).count() / L;
        const double all = std::chrono::duration<double, std::micro>(t2 - t0).count() / L;
        // synced per launch, event-timed like tests/benchmark/benchmark_comparison.cu
        float tot = 0.f;
        const int S = 500;
        for (int i = 0; i < S; ++i) {
            (void)hipEventRecord(e0, 0);
            f();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            tot += ms;
        }
        printf("  %-26s enqueue %6.2f us/call, back-to-back %6.2f us/launch, synced per launch %6.2f us\n", name, enq, all,
               tot * 1000.f / S);
        fflush(stdout);
    };
    probe("w4a8 M=1 (GEMV)", [&] { return qg_gemm_w4a8(Aq, Bq, C, 1, N, K, QG_TYPE_Q4_0, nullptr); });
    probe("w4a8 M=32 (MMQ)", [&] { return qg_gemm_w4a8(Aq, Bq, C, 32, N, K, QG_TYPE_Q4_0, nullptr); });
    probe("w4a16 M=1 (GEMV)", [&] { return qg_gemm_w4a16(A, Bq, C, 1, N, K, nullptr); });
    probe("w4a8 M=1 again", [&] { return qg_gemm_w4a8(Aq, Bq, C, 1, N, K, QG_TYPE_Q4_0, nullptr); });
    probe("quantize_q8_1 K=4096", [&] { return qg_quantize_q8_1(A, Aq, K, nullptr); });
    return 0;
}
