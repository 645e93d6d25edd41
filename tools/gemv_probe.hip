// gemv_probe.hip — tuning sweep for the W4A8 GEMV kernel template (qg_gemv_kernel.hpp).
// Not part of the product: it instantiates Q4_0 M=1 variants of (BPL, LPR, WGS, NT) and times each
// with back-to-back launches over rotating weight copies (cold HBM, > 256 MB Infinity Cache) and on
// one copy (hot), checking every variant's output against the first.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../llama.cpp-quant-gemm_amd/csrc \
//         -o gemv_probe gemv_probe.hip && ./gemv_probe [N] [K]
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "qg_gemv_kernel.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;

struct Bufs {
    std::vector<uint8_t*> w;
    uint8_t* a;
    float* c;
    int N, K;
};

static uint16_t f2h(float f) {
    _Float16 h = (_Float16)f;
    uint16_t b;
    memcpy(&b, &h, 2);
    return b;
}

template <int BPL, int LPR, int WGS, bool NT, int ABL = 0, bool DMA = false>
void run(const char* name, Bufs& bf, hipStream_t st, std::vector<float>& ref, bool first) {
    constexpr int NST = (WGS >= 1024 ? 2 : WGS >= 512 ? 4 : WGS == 256 ? 8 : WGS == 128 ? 16 : 32);
    GemmArgs g;
    g.A = bf.a; g.C = bf.c; g.M = 1; g.N = bf.N; g.K = bf.K; g.wtype = FMT_Q4_0; g.ldc_m = bf.N; g.ldc_n = 1;
    if (!gemv_shape_ok<FMT_Q4_0, BPL>(g)) { printf("%-22s skipped (shape)\n", name); return; }
    const int R = (int)bf.w.size();
    auto launch = [&](int i) { g.B = bf.w[i % R]; CK((gemv_launch<FMT_Q4_0, 1, BPL, LPR, WGS, NST, NT, false, ABL, DMA>(g, st))); };
    for (int i = 0; i < 2 * R; ++i) launch(i);
    CK(hipStreamSynchronize(st));
    // correctness vs the first variant (same copy 0)
    launch(0);
    std::vector<float> out(bf.N);
    CK(hipMemcpyAsync(out.data(), bf.c, bf.N * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    double maxd = 0;
    if (first) ref = out;
    else if (ABL) maxd = -1;
    else for (int i = 0; i < bf.N; ++i) maxd = fmax(maxd, fabs((double)out[i] - ref[i]) / (1e-3 + fabs(ref[i])));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int L = 512;
    float ms;
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < L; ++i) launch(i);
    CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    const double cold = ms * 1e3 / L;
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < L; ++i) launch(0);
    CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    const double hot = ms * 1e3 / L;
    const double bytes = (double)bf.N * (bf.K / 32) * 18 + (bf.K / 32) * 36 + bf.N * 4;
    printf("%-22s cold %7.3f us (%5.0f GB/s)  hot %7.3f us (%5.0f GB/s)  relerr %.2e\n", name, cold,
           bytes / cold / 1e3, hot, bytes / hot / 1e3, maxd);
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int K = argc > 2 ? atoi(argv[2]) : 4096;
    const int nb = K / 32;
    const long wbytes = (long)N * nb * 18;
    const int R = (int)((640L << 20) / wbytes) + 1;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    Bufs bf;
    bf.N = N; bf.K = K;
    std::vector<uint8_t> hw(wbytes), ha((long)nb * 36);
    srand(7);
    for (long b = 0; b < (long)N * nb; ++b) {
        uint16_t d = f2h(0.01f + 0.09f * rand() / RAND_MAX);
        memcpy(&hw[b * 18], &d, 2);
        for (int j = 0; j < 16; ++j) hw[b * 18 + 2 + j] = rand() & 0xFF;
    }
    for (int b = 0; b < nb; ++b) {
        uint16_t d = f2h(0.008f), s = f2h((rand() % 2000 - 1000) / 100.0f);
        memcpy(&ha[b * 36], &d, 2);
        memcpy(&ha[b * 36 + 2], &s, 2);
        for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
    }
    bf.w.resize(R);
    for (auto& p : bf.w) { CK(hipMalloc(&p, wbytes)); CK(hipMemcpy(p, hw.data(), wbytes, hipMemcpyHostToDevice)); }
    CK(hipMalloc(&bf.a, ha.size()));
    CK(hipMemcpy(bf.a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&bf.c, N * 4));
    printf("N=%d K=%d weight bytes %.2f MB, %d copies\n", N, K, wbytes / 1e6, R);
    std::vector<float> ref;
    run<4, 32, 512, false>("bpl4_lpr32_wg512", bf, st, ref, true);
    run<2, 64, 512, false>("bpl2_lpr64_wg512", bf, st, ref, false);
    run<4, 32, 512, false, 0, true>("dma bpl4_lpr32_wg512", bf, st, ref, false);
    run<4, 32, 256, false, 0, true>("dma bpl4_lpr32_wg256", bf, st, ref, false);
    run<8, 16, 256, false, 0, true>("dma bpl8_lpr16_wg256", bf, st, ref, false);
    run<8, 16, 512, false, 0, true>("dma bpl8_lpr16_wg512", bf, st, ref, false);
    run<2, 64, 512, false, 0, true>("dma bpl2_lpr64_wg512", bf, st, ref, false);
    run<2, 64, 256, false, 0, true>("dma bpl2_lpr64_wg256", bf, st, ref, false);
    run<4, 32, 128, false, 0, true>("dma bpl4_lpr32_wg128", bf, st, ref, false);
    run<8, 16, 1024, false, 0, true>("dma bpl8_lpr16_wg1024", bf, st, ref, false);
    run<4, 32, 512, false, 2, true>("dma bpl4 abl2(no-dot)", bf, st, ref, false);
    run<4, 32, 512, false, 3, true>("dma bpl4 abl3(loads)", bf, st, ref, false);
    run<4, 32, 512, false, 3>("bpl4 abl3(loads)", bf, st, ref, false);
    return 0;
}
