// ring_probe.hip — the cooperative-ring prefill (tools/mmq_ring_experiment.hpp, tools/mmq_direct_experiment.hpp) against the round-1 prefill
// (qg_mmq_kernel.hpp, product instantiation), timed like bench.py: 64 launches over distinct weight
// copies (> 600 MB) in one hipGraph, HIP events, interleaved rounds, median. Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 \
//         -I../llama.cpp-quant-gemm_amd/csrc -I. -o ring_probe ring_probe.hip && ./ring_probe
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "mmq_ring_experiment.hpp"
#include "mmq_direct_experiment.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;
void qg::describe_kernel(const GemmArgs&, const char*, ...) {}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }

typedef std::function<hipError_t(const GemmArgs&, hipStream_t)> LaunchFn;
struct Variant { std::string name; LaunchFn fn; };

template <int BN, int TT, int W>
hipError_t prod(const GemmArgs& g, hipStream_t st) {
    if (!mmq_shape_ok<FMT_Q4_0, BN, TT, W, true>(g)) return hipErrorInvalidValue;
    return mmq_launch<FMT_Q4_0, BN, TT, W, false, true, 2, 0, false, 4, 1, true>(g, st);
}
template <int BN, int TT, int W, int SB, int NS, int OPT = 0>
hipError_t ring(const GemmArgs& g, hipStream_t st) {
    if (!ring_shape_ok<FMT_Q4_0, BN, TT, W, SB, NS>(g)) return hipErrorInvalidValue;
    return ring_launch<FMT_Q4_0, BN, TT, W, SB, NS, false, OPT>(g, st);
}
template <int TT, int W, int BPC, int NBUF>
hipError_t direct(const GemmArgs& g, hipStream_t st) {
    if (!direct_shape_ok<FMT_Q4_0, TT, W, BPC, NBUF>(g)) return hipErrorInvalidValue;
    return direct_launch<FMT_Q4_0, TT, W, BPC, NBUF, false>(g, st);
}
template <int BN, int TT, int W, int ABL>
hipError_t prodabl(const GemmArgs& g, hipStream_t st) {
    if (!mmq_shape_ok<FMT_Q4_0, BN, TT, W, true>(g)) return hipErrorInvalidValue;
    return mmq_launch<FMT_Q4_0, BN, TT, W, false, true, 2, ABL, false, 4, 1, true>(g, st);
}

int main(int argc, char** argv) {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct S { int M, N, K; };
    const S shapes[] = {{32, 4096, 4096}, {16, 4096, 4096}, {8, 4096, 4096}, {64, 4096, 4096}, {32, 4096, 14336}, {32, 11008, 4096}, {64, 11008, 4096}};
    (void)argc; (void)argv;
    for (const S& s : shapes) {
        const int nb = s.K / 32, bb = 18;
        const long wbytes = (long)s.N * nb * bb;
        const int G = 64;
        const int R = (int)std::max((long)G, (640L << 20) / wbytes + 1);
        std::vector<uint8_t> hw(wbytes), ha((long)s.M * nb * 36);
        srand(11);
        for (long b = 0; b < (long)s.N * nb; ++b) {
            for (int j = 0; j < bb; ++j) hw[b * bb + j] = rand() & 0xFF;
            uint16_t d = f2h(0.01f + 0.09f * (float)rand() / (float)RAND_MAX);
            memcpy(&hw[b * bb], &d, 2);
        }
        for (long b = 0; b < (long)s.M * nb; ++b) {
            uint16_t d = f2h(0.008f), sm = f2h((rand() % 2000 - 1000) / 100.0f);
            memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &sm, 2);
            for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
        }
        uint8_t* wall;
        CK(hipMalloc(&wall, wbytes * R));
        for (int r = 0; r < R; ++r) CK(hipMemcpy(wall + wbytes * r, hw.data(), wbytes, hipMemcpyHostToDevice));
        uint8_t* a; float* c;
        CK(hipMalloc(&a, ha.size())); CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
        CK(hipMalloc(&c, (size_t)s.M * s.N * 4));
        std::vector<Variant> vs;
#define P(BN, TT, W, NAME) vs.push_back({NAME, prod<BN, TT, W>});
#define RG(BN, TT, W, SB, NS, NAME) vs.push_back({NAME, ring<BN, TT, W, SB, NS>});
#define RO(BN, TT, W, SB, NS, OPT, NAME) vs.push_back({NAME, ring<BN, TT, W, SB, NS, OPT>});
#define PA(BN, TT, W, ABL, NAME) vs.push_back({NAME, prodabl<BN, TT, W, ABL>});
#define D(TT, W, BPC, NBUF, NAME) vs.push_back({NAME, direct<TT, W, BPC, NBUF>});
        if (s.M == 32) {
            P(32, 1, 8, "product bn32 tt1 w8")
            D(2, 8, 16, 1, "direct tt2 w8 bpc16 nbuf1")
            D(2, 8, 8, 2, "direct tt2 w8 bpc8 nbuf2")
            D(2, 4, 16, 1, "direct tt2 w4 bpc16 nbuf1")
            D(2, 8, 8, 1, "direct tt2 w8 bpc8 nbuf1")
        } else if (s.M <= 16) {
            P(16, 1, 8, "product bn16 w8")
            D(1, 8, 16, 1, "direct tt1 w8 bpc16 nbuf1")
            D(1, 8, 8, 2, "direct tt1 w8 bpc8 nbuf2")
            D(1, 16, 8, 1, "direct tt1 w16 bpc8 nbuf1")
        } else {
            P(32, 2, 8, "product bn32 tt2 w8")
            D(2, 8, 16, 1, "direct tt2 w8 bpc16 nbuf1")
        }
#undef P
#undef RG
#undef D
#undef RO
#undef PA
        auto args = [&](int i) { GemmArgs g; g.A = a; g.B = wall + wbytes * (i % R); g.C = c; g.M = s.M; g.N = s.N; g.K = s.K;
                                 g.wtype = FMT_Q4_0; g.ldc_m = s.N; g.ldc_n = 1; return g; };
        std::vector<float> ref((size_t)s.M * s.N), out(ref.size());
        std::vector<double> err(vs.size(), 0.0);
        std::vector<hipGraphExec_t> ge;
        for (size_t k = 0; k < vs.size(); ++k) {
            CK(hipMemset(c, 0xFF, ref.size() * 4));
            if (vs[k].fn(args(0), st) != hipSuccess) {
                (void)hipGetLastError();
                printf("  %-28s skipped (shape rejected)\n", vs[k].name.c_str());
                vs.erase(vs.begin() + k); err.erase(err.begin() + k); --k;
                continue;
            }
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(k == 0 ? ref.data() : out.data(), c, ref.size() * 4, hipMemcpyDeviceToHost));
            if (k) for (size_t i = 0; i < ref.size(); ++i) {
                const double d = std::isfinite(out[i]) ? fabs(out[i] - ref[i]) / (1e-2 + fabs(ref[i])) : 1e30;
                err[k] = std::max(err[k], d);
            }
            hipGraph_t gr;
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
            for (int i = 0; i < G; ++i) CK(vs[k].fn(args(i), st));
            CK(hipStreamEndCapture(st, &gr));
            hipGraphExec_t x;
            CK(hipGraphInstantiate(&x, gr, nullptr, nullptr, 0));
            ge.push_back(x);
        }
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        const int ROUNDS = 7, REPS = 10;
        std::vector<std::vector<double>> t(vs.size());
        for (int r = 0; r < ROUNDS; ++r)
            for (size_t k = 0; k < vs.size(); ++k) {
                CK(hipGraphLaunch(ge[k], st));
                CK(hipEventRecord(e0, st));
                for (int i = 0; i < REPS; ++i) CK(hipGraphLaunch(ge[k], st));
                CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                t[k].push_back(ms * 1e3 / (REPS * G));
            }
        const double bytes = (double)wbytes + (double)s.M * nb * 36 + (double)s.M * s.N * 4;
        const double flops = 2.0 * s.M * s.N * s.K;
        printf("Q4_0 M=%d N=%d K=%d  (%.0f B, %.2f GFLOP)\n", s.M, s.N, s.K, bytes, flops / 1e9);
        for (size_t k = 0; k < vs.size(); ++k) {
            std::sort(t[k].begin(), t[k].end());
            const double us = t[k][t[k].size() / 2];
            printf("  %-28s %8.3f us  (min %.3f)  frac %.3f  %7.1f TOPS  maxrel %.2e\n", vs[k].name.c_str(), us,
                   t[k][0], bytes / us / 1e3 / 8000.0, flops / us / 1e6, err[k]);
        }
        fflush(stdout);
        for (auto x : ge) CK(hipGraphExecDestroy(x));
        CK(hipFree(wall)); CK(hipFree(a)); CK(hipFree(c));
    }
    return 0;
}
