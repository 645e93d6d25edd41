// mmq_timeline.hip — per-wave timeline of one cold prefill launch (diagnostic; not the product).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DQG_MMQ_STAMPS \
//         -I../llama.cpp-quant-gemm_amd/csrc -o mmq_timeline mmq_timeline.hip
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "qg_mmq_kernel.hpp"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
namespace qg {
void describe_kernel(const GemmArgs&, const char*, ...) {}
}
using namespace qg;
static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }
template <int BN, int TT, int W, bool P16>
static void run(const char* name, int M, int N, int K) {
    const int nb = K / 32;
    const long wbytes = (long)N * nb * 18;
    const int R = (int)((640L << 20) / wbytes) + 1;
    std::vector<uint8_t> hw(wbytes), ha((long)M * nb * 36);
    for (long b = 0; b < (long)N * nb; ++b) { for (int j = 0; j < 18; ++j) hw[b * 18 + j] = rand(); uint16_t d = f2h(0.05f); memcpy(&hw[b * 18], &d, 2); }
    for (long b = 0; b < (long)M * nb; ++b) { for (int j = 0; j < 36; ++j) ha[b * 36 + j] = rand(); uint16_t d = f2h(0.01f); memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &d, 2); }
    std::vector<uint8_t*> w(R);
    for (auto& p : w) { CK(hipMalloc(&p, wbytes)); CK(hipMemcpy(p, hw.data(), wbytes, hipMemcpyHostToDevice)); }
    uint8_t* a; float* c;
    CK(hipMalloc(&a, ha.size())); CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&c, (size_t)M * N * 4));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    GemmArgs g; g.A = a; g.C = c; g.M = M; g.N = N; g.K = K; g.wtype = FMT_Q4_0; g.ldc_m = N; g.ldc_n = 1;
    const int L = 100;
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(e0, 0));
        // the product's instantiation (qg_gemm_mfma.hip run_p: NB 2, SB 4, EPI2, general entry)
        for (int i = 0; i < L; ++i) { g.B = w[i % R]; CK((mmq_launch<FMT_Q4_0, BN, TT, W, false, P16, 2, 0, false, 4, 1, true>(g, 0))); }
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const int nwg = ((N + BN - 1) / BN) * ((M + 16 * TT - 1) / (16 * TT)), nw = nwg * W;
        std::vector<unsigned long long> s(8 * nw);
        CK(hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(g_mmq_stamps), s.size() * 8));
        unsigned long long t0 = ~0ull, tend = 0;
        for (int i = 0; i < nw; ++i) { t0 = std::min(t0, s[8 * i]); tend = std::max(tend, s[8 * i + 4]); }
        std::vector<double> seg[5];
        for (int i = 0; i < nw; ++i) {
            const unsigned long long* q = &s[8 * i];
            seg[0].push_back((q[0] - t0) * 0.01);
            if (q[1]) seg[1].push_back((q[1] - q[0]) * 0.01);
            if (q[2]) seg[2].push_back((q[2] - q[1]) * 0.01);
            seg[3].push_back((q[3] - q[0]) * 0.01);
            seg[4].push_back((q[4] - q[3]) * 0.01);
        }
        auto pct = [](std::vector<double> v, double p) { if (v.empty()) return 0.0; std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
        printf("%s M=%d N=%d K=%d rep%d: event %.2f us/launch, span %.2f us, %d waves\n", name, M, N, K, rep, ms * 1e3 / L, (tend - t0) * 0.01, nw);
        const char* names[5] = {"entry offset", "entry->first data", "first sb compute", "entry->main loop done", "reduction+store"};
        for (int k = 0; k < 5; ++k) printf("   %-22s p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f\n", names[k], pct(seg[k], .1), pct(seg[k], .5), pct(seg[k], .9), pct(seg[k], 1.0));
        // per-CU ingest: one workgroup per CU; its L2 -> LDS bytes (weights BN rows x K, activations
        // 16 TT tokens x K as Q8_1) over its waves' entry -> main-loop-done span
        const double wg_bytes = (double)BN * nb * 18 + 16.0 * TT * nb * 36;
        printf("   per-workgroup L2->LDS bytes %.0f; ingest at the p50 / p90 main-loop span: %.1f / %.1f GB/s per CU\n",
               wg_bytes, wg_bytes / (pct(seg[3], .5) * 1e3), wg_bytes / (pct(seg[3], .9) * 1e3));
    }
    for (auto p : w) CK(hipFree(p));
    CK(hipFree(a)); CK(hipFree(c));
}
int main() {
    run<32, 1, 8, true>("product bn32 tt1 w8 p16 epi2", 32, 4096, 4096);
    return 0;
}
