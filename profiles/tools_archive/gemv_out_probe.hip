// gemv_out_probe.hip — where the single-launch M = 1 GEMV's output goes, and what the end of the
// kernel costs for it. The product GEMV (libqg_hip.so, qg_gemm_w4a8, BASELINE configs[1]) timed like
// bench.py (64 launches over distinct weight copies > 600 MB, one hipGraph, HIP events), its 16 KB
// output in: device memory (hipMalloc), uncached device memory (hipExtMallocWithFlags
// hipDeviceMallocUncached: stores write through, nothing dirty in L2 at the kernel's end),
// fine-grained device memory, and one output buffer per launch vs one shared by all launches.
// Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -o gemv_out_probe gemv_out_probe.hip \
//         -L../llama.cpp-quant-gemm_amd/quant_gemm -lqg_hip -Wl,-rpath,'$ORIGIN/../llama.cpp-quant-gemm_amd/quant_gemm'
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "qg/qg.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }

int main() {
    const int M = 1, N = 4096, K = 4096, nb = K / 32, G = 64, R = 72;
    const long wbytes = (long)N * nb * 18;
    std::vector<uint8_t> hw(wbytes), ha((long)M * nb * 36);
    srand(5);
    for (long b = 0; b < (long)N * nb; ++b) {
        for (int j = 0; j < 18; ++j) hw[b * 18 + j] = rand() & 0xFF;
        uint16_t d = f2h(0.01f + 0.05f * (float)rand() / (float)RAND_MAX);
        memcpy(&hw[b * 18], &d, 2);
    }
    for (long b = 0; b < (long)M * nb; ++b) {
        uint16_t d = f2h(0.008f), s = f2h(1.0f);
        memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &s, 2);
        for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
    }
    uint8_t *w, *a;
    CK(hipMalloc(&w, wbytes * R));
    for (int r = 0; r < R; ++r) CK(hipMemcpy(w + wbytes * r, hw.data(), wbytes, hipMemcpyHostToDevice));
    CK(hipMalloc(&a, ha.size()));
    CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    const size_t ob = (size_t)G * N * 4;
    float *o_dev, *o_unc, *o_fg;
    CK(hipMalloc(&o_dev, ob));
    CK(hipExtMallocWithFlags((void**)&o_unc, ob, hipDeviceMallocUncached));
    CK(hipExtMallocWithFlags((void**)&o_fg, ob, hipDeviceMallocFinegrained));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct V { std::string name; float* out; bool per_launch; };
    std::vector<V> vs = {{"hipMalloc, one buffer", o_dev, false},
                         {"hipMalloc, buffer per launch", o_dev, true},
                         {"uncached, one buffer", o_unc, false},
                         {"uncached, buffer per launch", o_unc, true},
                         {"fine-grained, one buffer", o_fg, false}};
    std::vector<hipGraphExec_t> ge(vs.size());
    std::vector<float> ref(N), got(N);
    for (size_t v = 0; v < vs.size(); ++v) {
        CK(hipMemset(vs[v].out, 0, ob));
        if (qg_gemm_w4a8(a, w, vs[v].out, M, N, K, QG_TYPE_Q4_0, (qg_stream_t)st) != 0) { printf("launch failed\n"); return 1; }
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(v == 0 ? ref.data() : got.data(), vs[v].out, N * 4, hipMemcpyDeviceToHost));
        if (v > 0 && memcmp(ref.data(), got.data(), N * 4) != 0) printf("  %s: OUTPUT DIFFERS\n", vs[v].name.c_str());
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < G; ++i)
            qg_gemm_w4a8(a, w + wbytes * (i % R), vs[v].out + (vs[v].per_launch ? (size_t)i * N : 0), M, N, K, QG_TYPE_Q4_0,
                         (qg_stream_t)st);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge[v], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int round = 0; round < 11; ++round)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge[v], st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms * 1e3f / G);
        }
    printf("Q4_0 GEMV M=1 N=K=4096 (9,458,176 B per launch), us per launch, median of 11 x %d\n", G);
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("  %-32s %7.3f us  (min %7.3f)  frac %.3f\n", vs[v].name.c_str(), t[v][5], t[v][0], 9458176.0 / t[v][5] / 1e3 / 8000.0);
    }
    return 0;
}
