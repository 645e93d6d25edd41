// benchmark_comparison.cpp — the reference's benchmark harness (tests/benchmark/benchmark_comparison.cu),
// filled in with this library's kernels through the C-ABI. Same test cases (make_test_cases,
// :191-215), same protocol (one warm-up launch, then launches timed one at a time with an event
// pair until min_time is reached, :106-130), same byte formula (:138-140) and table layout
// (:164-183). The reference ships this file with every kernel call commented out.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -o benchmark_comparison benchmark_comparison.cpp \
//         -L../llama.cpp-quant-gemm_amd/quant_gemm -lqg_hip -Wl,-rpath,'$ORIGIN/../llama.cpp-quant-gemm_amd/quant_gemm'
//   ./benchmark_comparison [min_time_ms]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <vector>

#include "qg/qg.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define QK(x) do { int s_ = (x); if (s_ != 0) { fprintf(stderr, "qg error %d (%s) at %d\n", s_, qg_status_string(s_), __LINE__); exit(1); } } while (0)

struct result {
    const char* name;
    int M, N, K;
    double avg_us, gflops, gbps;
    int runs;
};

static result run(const char* name, int M, int N, int K, size_t bytes, const std::function<void()>& launch,
                  float min_ms) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();  // warm-up
    CK(hipDeviceSynchronize());
    int n = 0;
    float total = 0.f;
    while (total < min_ms) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        total += ms;
        ++n;
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    const double s = total / 1e3;
    return {name, M, N, K, total * 1e3 / n, 2.0 * M * N * K * n / s / 1e9, (double)bytes * n / s / 1e9, n};
}

static void print(const result& r) {
    printf("%-30s %6d %6d %6d %12.2f %10.2f %10.2f %8d\n", r.name, r.M, r.N, r.K, r.avg_us, r.gflops, r.gbps, r.runs);
}

int main(int argc, char** argv) {
    const float min_ms = argc > 1 ? (float)atof(argv[1]) : 200.0f;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    printf("GPU: %s (%s), %d CUs\n", prop.name, prop.gcnArchName, prop.multiProcessorCount);
    printf("Memory: %.1f GB\n", prop.totalGlobalMem / 1e9);
    printf("library: %s\n\n", qg_version());
    printf("================================================================================\n");
    printf("  Quantized GEMM Performance Benchmark\n");
    printf("  (Compatible with llama.cpp test-backend-ops format)\n");
    printf("================================================================================\n\n");
    printf("%-30s %6s %6s %6s %12s %10s %10s %8s\n", "Kernel", "M", "N", "K", "Time(us)", "GFLOPS", "GB/s", "Runs");
    printf("--------------------------------------------------------------------------------\n");
    struct tc { int M, N, K; const char* d; };
    const std::vector<tc> cases = {
        {1, 4096, 4096, "Llama-7B decode bs=1"},   {32, 4096, 4096, "Llama-7B decode bs=32"},
        {128, 4096, 4096, "Llama-7B prefill"},     {512, 4096, 4096, "Llama-7B long prefill"},
        {1, 5120, 5120, "Llama-13B decode bs=1"},  {32, 5120, 5120, "Llama-13B decode bs=32"},
        {1, 11008, 4096, "Llama-7B MLP up"},       {1, 4096, 11008, "Llama-7B MLP down"},
        {256, 256, 256, "Small 256x256x256"},      {1024, 1024, 1024, "Medium 1K x 1K x 1K"},
    };
    std::mt19937 rng(1234);
    std::uniform_real_distribution<float> U(0.f, 1.f);  // curandGenerateUniform's (0, 1]
    for (const tc& c : cases) {
        const int M = c.M, N = c.N, K = c.K;
        if (K % 32) { printf("Skipping %s: K=%d not multiple of 32\n", c.d, K); continue; }
        printf("\n--- %s ---\n", c.d);
        std::vector<float> ha((size_t)M * K), hb((size_t)N * K);
        for (auto& v : ha) v = U(rng);
        for (auto& v : hb) v = U(rng);
        float *A, *B, *C;
        void *Aq, *Bq;
        CK(hipMalloc(&A, ha.size() * 4));
        CK(hipMalloc(&B, hb.size() * 4));
        CK(hipMalloc(&C, (size_t)M * N * 4));
        CK(hipMalloc(&Aq, (size_t)M * K / 32 * 36));
        CK(hipMalloc(&Bq, (size_t)N * K / 32 * 18));
        CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(B, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
        QK(qg_quantize_q8_1(A, Aq, (int64_t)M * K, nullptr));
        QK(qg_quantize_q4_0(B, Bq, (int64_t)N * K, nullptr));
        CK(hipDeviceSynchronize());
        const size_t qbytes = (size_t)N * K / 32 * 18 + (size_t)M * K / 32 * 36 + (size_t)M * N * 4;
        const size_t fbytes = ((size_t)N * K + (size_t)M * K + (size_t)M * N) * 4;
        const size_t w16bytes = (size_t)N * K / 32 * 18 + (size_t)M * K * 4 + (size_t)M * N * 4;
        const result r0 = run("FP32 GEMM (qg_gemm_fp32)", M, N, K, fbytes,
                              [&] { QK(qg_gemm_fp32(A, B, C, M, N, K, nullptr)); }, min_ms);
        print(r0);
        const result r1 = run("W4A8 Q4_0xQ8_1 (qg_gemm_w4a8)", M, N, K, qbytes,
                              [&] { QK(qg_gemm_w4a8(Aq, Bq, C, M, N, K, QG_TYPE_Q4_0, nullptr)); }, min_ms);
        print(r1);
        printf("  -> Speedup vs FP32: %.2fx\n", r0.avg_us / r1.avg_us);
        const result r2 = run("W4A16 Q4_0xFP32 (qg_gemm_w4a16)", M, N, K, w16bytes,
                              [&] { QK(qg_gemm_w4a16(A, Bq, C, M, N, K, nullptr)); }, min_ms);
        print(r2);
        CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(Aq)); CK(hipFree(Bq));
    }
    printf("\n================================================================================\n");
    printf("  Benchmark Complete\n");
    printf("================================================================================\n");
    return 0;
}
