// gemv_probe.hip — tuning sweep for the GEMV kernels of the product (qg_gemv_kernel.hpp).
// Not part of the product. For each shape, every variant is timed in R interleaved rounds (clock
// and thermal drift hit all alike); a round = L back-to-back launches rotating over enough weight
// copies to exceed the 256 MB Infinity Cache ("cold") or on one copy ("hot"); medians reported.
// Outputs are checked against the first variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../llama.cpp-quant-gemm_amd/csrc \
//         -o gemv_probe gemv_probe.hip && ./gemv_probe
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "gemv_experiments.hpp"  // + the product header qg_gemv_kernel.hpp

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;

__global__ __launch_bounds__(256) void lin_read(const u32x4* __restrict__ p, long n16, unsigned* out) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long nth = (long)gridDim.x * 256;
    unsigned acc = 0;
    for (long j = i; j < n16; j += nth) { u32x4 v = p[j]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678u) out[0] = acc;
}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }

static int block_bytes(int f) { return f == FMT_Q4_0 ? 18 : f == FMT_Q4_1 ? 20 : f == FMT_Q5_0 ? 22 : 24; }

struct Problem {
    int F, M, N, K;
    long wbytes;
    std::vector<uint8_t*> w;
    uint8_t* a;
    float* c;
    unsigned* scratch;
};

static void make(Problem& p, int F, int M, int N, int K, long copy_bytes) {
    p.F = F; p.M = M; p.N = N; p.K = K;
    const int nb = K / 32, bb = block_bytes(F);
    p.wbytes = (long)N * nb * bb;
    const int R = (int)std::max(2L, copy_bytes / p.wbytes + 1);
    std::vector<uint8_t> hw(p.wbytes), ha((long)M * nb * 36);
    srand(7);
    for (long b = 0; b < (long)N * nb; ++b) {
        for (int j = 0; j < bb; ++j) hw[b * bb + j] = rand() & 0xFF;
        uint16_t d = f2h(0.01f + 0.09f * (float)rand() / (float)RAND_MAX);
        memcpy(&hw[b * bb], &d, 2);
        if (F == FMT_Q4_1 || F == FMT_Q5_1) { uint16_t m = f2h(-0.5f * (float)rand() / (float)RAND_MAX); memcpy(&hw[b * bb + 2], &m, 2); }
    }
    for (long b = 0; b < (long)M * nb; ++b) {
        uint16_t d = f2h(0.008f), s = f2h((rand() % 2000 - 1000) / 100.0f);
        memcpy(&ha[b * 36], &d, 2);
        memcpy(&ha[b * 36 + 2], &s, 2);
        for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
    }
    p.w.resize(R);
    for (auto& q : p.w) { CK(hipMalloc(&q, p.wbytes)); CK(hipMemcpy(q, hw.data(), p.wbytes, hipMemcpyHostToDevice)); }
    CK(hipMalloc(&p.a, ha.size()));
    CK(hipMemcpy(p.a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&p.c, (size_t)M * N * 4));
    CK(hipMalloc(&p.scratch, 4096));
}

static void destroy(Problem& p) {
    for (auto q : p.w) CK(hipFree(q));
    CK(hipFree(p.a)); CK(hipFree(p.c)); CK(hipFree(p.scratch));
    p.w.clear();
}

typedef std::function<hipError_t(const GemmArgs&, hipStream_t)> LaunchFn;
struct Variant { std::string name; LaunchFn fn; bool is_read; };

static GemmArgs args(Problem& p, int copy) {
    GemmArgs g;
    g.A = p.a; g.B = p.w[copy % p.w.size()]; g.C = p.c; g.M = p.M; g.N = p.N; g.K = p.K; g.wtype = p.F;
    g.ldc_m = p.N; g.ldc_n = 1;
    return g;
}

static std::vector<float> output(Problem& p, const Variant& v, hipStream_t st) {
    CK(hipMemsetAsync(p.c, 0xFF, (size_t)p.M * p.N * 4, st));
    CK(v.fn(args(p, 0), st));
    std::vector<float> out((size_t)p.M * p.N);
    CK(hipMemcpyAsync(out.data(), p.c, out.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return out;
}

static double time_round(Problem& p, const Variant& v, hipStream_t st, bool cold, int L, hipEvent_t e0, hipEvent_t e1) {
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < L; ++i) CK(v.fn(args(p, cold ? i : 0), st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / L;
}

static void bench(Problem& p, std::vector<Variant>& vs, hipStream_t st, int rounds, int L) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<float> ref = output(p, vs[0], st);
    std::vector<double> err(vs.size(), 0.0);
    for (size_t k = 1; k < vs.size(); ++k) {
        if (vs[k].is_read) { err[k] = -1; continue; }
        std::vector<float> o = output(p, vs[k], st);
        for (size_t i = 0; i < o.size(); ++i)
            err[k] = std::max(err[k], (double)fabs(o[i] - ref[i]) / (1e-2 + fabs(ref[i])));
    }
    std::vector<std::vector<double>> cold(vs.size()), hot(vs.size());
    for (auto& v : vs) for (int i = 0; i < (int)p.w.size(); ++i) CK(v.fn(args(p, i), st));
    CK(hipStreamSynchronize(st));
    for (int r = 0; r < rounds; ++r)
        for (size_t k = 0; k < vs.size(); ++k) {
            cold[k].push_back(time_round(p, vs[k], st, true, L, e0, e1));
            hot[k].push_back(time_round(p, vs[k], st, false, L, e0, e1));
        }
    const double bytes = (double)p.wbytes + (double)p.M * (p.K / 32) * 36 + (double)p.M * p.N * 4;
    printf("fmt=%d M=%d N=%d K=%d  algorithmic %.0f B, %zu copies, %d rounds x %d launches\n", p.F, p.M, p.N, p.K,
           bytes, p.w.size(), rounds, L);
    for (size_t k = 0; k < vs.size(); ++k) {
        auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
        const double c = med(cold[k]), h = med(hot[k]);
        printf("  %-28s cold %7.3f us (%5.0f GB/s, frac %.3f)  hot %7.3f us  maxrel %.2e\n", vs[k].name.c_str(), c,
               bytes / c / 1e3, bytes / c / 1e3 / 8000.0, h, err[k]);
    }
    fflush(stdout);
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
}

#define STAGED(F, MT, BPL, LPR, WGS, NAME) \
    vs.push_back({NAME, [](const GemmArgs& g, hipStream_t s) { return gemv_launch<F, MT, BPL, LPR, WGS, false>(g, s); }, false});
#define STAGED_NT(F, MT, BPL, LPR, WGS, NAME) \
    vs.push_back({NAME, [](const GemmArgs& g, hipStream_t s) { return gemv_launch<F, MT, BPL, LPR, WGS, false, AIN_Q8_1, true>(g, s); }, false});
#define NOPRE(F, MT, BPL, LPR, WGS, NAME) \
    vs.push_back({NAME, [](const GemmArgs& g, hipStream_t s) { return gemv_launch<F, MT, BPL, LPR, WGS, false, AIN_Q8_1, false, false>(g, s); }, false});
#define RAX(F, MT, BPL, LPR, WGS, PF, NAME) \
    vs.push_back({NAME, [](const GemmArgs& g, hipStream_t s) { return gemv_ra_launch<F, MT, BPL, LPR, WGS, PF, false>(g, s); }, false});

static void add_read(std::vector<Variant>& vs, Problem& p) {
    unsigned* scr = p.scratch;
    long n16 = p.wbytes / 16;
    vs.push_back({"pure linear read", [scr, n16](const GemmArgs& g, hipStream_t s) {
                      const long pieces = (n16 + 1) / 2;
                      hipLaunchKernelGGL(lin_read, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, s,
                                         (const u32x4*)g.B, n16, scr);
                      return hipGetLastError(); }, true});
}

template <int F> static void m1(std::vector<Variant>& vs, bool full) {
    STAGED(F, 1, 4, 32, 512, "v2 bpl4 lpr32 wg512")
    STAGED(F, 1, 4, 32, 256, "v2 bpl4 lpr32 wg256")
    STAGED(F, 1, 2, 64, 512, "v2 bpl2 lpr64 wg512")
    STAGED(F, 1, 2, 64, 1024, "v2 bpl2 lpr64 wg1024")
    STAGED(F, 1, 2, 64, 256, "v2 bpl2 lpr64 wg256")
    if (full) {
        RAX(F, 1, 4, 32, 128, false, "ra bpl4 lpr32 wg128")
        RAX(F, 1, 4, 32, 512, false, "ra bpl4 lpr32 wg512")
        RAX(F, 1, 4, 32, 512, true, "ra bpl4 lpr32 wg512 pf")
        RAX(F, 1, 2, 64, 256, false, "ra bpl2 lpr64 wg256")
        RAX(F, 1, 2, 64, 256, true, "ra bpl2 lpr64 wg256 pf")
        RAX(F, 1, 4, 64, 256, true, "ra bpl4 lpr64 wg256 pf")
        RAX(F, 1, 4, 16, 256, false, "ra bpl4 lpr16 wg256")
    }
}

int main(int argc, char** argv) {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const long copy = 640L << 20;
    struct S { int F, M, N, K, rounds; };
    const S shapes[] = {{FMT_Q4_0, 1, 4096, 4096, 7}, {FMT_Q4_0, 1, 4000, 4096, 3}, {FMT_Q4_0, 1, 32000, 4096, 3},
                        {FMT_Q4_0, 1, 4096, 14336, 3}, {FMT_Q4_0, 1, 14336, 4096, 3}, {FMT_Q4_1, 1, 4096, 4096, 3},
                        {FMT_Q5_0, 1, 4096, 4096, 3}, {FMT_Q5_1, 1, 4096, 4096, 3}, {FMT_Q4_0, 2, 4096, 4096, 3},
                        {FMT_Q4_0, 4, 4096, 4096, 3}, {FMT_Q4_0, 8, 4096, 4096, 3}};
    const bool focus = getenv("QG_FOCUS") != nullptr;
    for (const S& s0 : shapes) {
        S s = s0;
        if (focus) {
            if (!(s.K == 4096 && s.N == 4096)) continue;
            s.rounds = 9;
        }
        Problem p;
        make(p, s.F, s.M, s.N, s.K, copy);
        std::vector<Variant> vs;
        if (s.M == 1) {
            const bool full = false;
            if (s.F == FMT_Q4_0) m1<FMT_Q4_0>(vs, full);
            if (s.F == FMT_Q4_1) m1<FMT_Q4_1>(vs, full);
            if (s.F == FMT_Q5_0) m1<FMT_Q5_0>(vs, full);
            if (s.F == FMT_Q5_1) m1<FMT_Q5_1>(vs, full);
            add_read(vs, p);
        } else if (s.M == 2) {
            STAGED(FMT_Q4_0, 2, 4, 32, 512, "v2 pre bpl4 lpr32 wg512")
            STAGED(FMT_Q4_0, 2, 2, 64, 1024, "v2 pre bpl2 lpr64 wg1024")
            STAGED(FMT_Q4_0, 2, 2, 64, 512, "v2 pre bpl2 lpr64 wg512")
            STAGED_NT(FMT_Q4_0, 2, 4, 32, 512, "v2 nt bpl4 lpr32 wg512")
            RAX(FMT_Q4_0, 2, 4, 32, 256, false, "ra bpl4 lpr32 wg256")
            RAX(FMT_Q4_0, 2, 4, 32, 256, true, "ra bpl4 lpr32 wg256 pf")
            RAX(FMT_Q4_0, 2, 2, 64, 256, false, "ra bpl2 lpr64 wg256")
        } else if (s.M == 4) {
            STAGED(FMT_Q4_0, 4, 4, 32, 512, "v2 bpl4 lpr32 wg512")
            STAGED(FMT_Q4_0, 4, 2, 64, 1024, "v2 bpl2 lpr64 wg1024")
            STAGED(FMT_Q4_0, 4, 4, 32, 256, "staged bpl4 lpr32 wg256")
            RAX(FMT_Q4_0, 4, 4, 32, 256, false, "ra bpl4 lpr32 wg256")
            RAX(FMT_Q4_0, 4, 2, 64, 256, false, "ra bpl2 lpr64 wg256")
        } else {
            STAGED(FMT_Q4_0, 8, 4, 32, 512, "v2 bpl4 lpr32 wg512")
            STAGED(FMT_Q4_0, 8, 4, 32, 256, "staged bpl4 lpr32 wg256")
            STAGED(FMT_Q4_0, 8, 2, 64, 512, "staged bpl2 lpr64 wg512")
            RAX(FMT_Q4_0, 8, 2, 64, 256, false, "ra bpl2 lpr64 wg256")
        }
        bench(p, vs, st, s.rounds, s.M == 1 ? 256 : 128);
        destroy(p);
    }
    return 0;
}
