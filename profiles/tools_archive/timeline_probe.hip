// timeline_probe.hip — per-wave timeline of one cold GEMV launch (diagnostic; not the product).
// Each wave stamps s_memrealtime (100 MHz) at entry, after its weight loads have landed, and at exit,
// plus HW_ID / XCC_ID. Compares the GEMV with a pure linear read of the same bytes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DQG_STAMPS \
//         -I../llama.cpp-quant-gemm_amd/csrc -o timeline_probe timeline_probe.hip
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "gemv_experiments.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace qg;

template <int P>
__global__ void rd_stamp(const uint8_t* __restrict__ p, long bytes, unsigned* out) {
    QG_STAMP(t0);
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long nth = (long)gridDim.x * blockDim.x;
    unsigned acc = 0;
    u32x4 v[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const long off = (t + i * nth) * 16;
        v[i] = off < bytes ? *(const u32x4*)(p + off) : u32x4{0u, 0u, 0u, 0u};
    }
    QG_WAIT_STAMP(t1);
#pragma unroll
    for (int i = 0; i < P; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    if (acc == 0x12345678u) out[0] = acc;
    QG_STAMP(t2);
    QG_STAMP_STORE(t0, t0, t1, t1, t2, 0ull, 0ull);
}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }

static void report(const char* name, int nwaves, double event_us) {
    std::vector<unsigned long long> s(8 * nwaves);
    CK(hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(g_stamps), s.size() * 8));
    unsigned long long t0min = ~0ull, t2max = 0, t1max = 0;
    for (int w = 0; w < nwaves; ++w) {
        t0min = std::min(t0min, s[8 * w]);
        t1max = std::max(t1max, s[8 * w + 2]); t2max = std::max(t2max, s[8 * w + 4]);
    }
    std::vector<double> start, seg_b, seg_l, seg_c, seg_r, life, mhz;
    for (int w = 0; w < nwaves; ++w) {
        const unsigned long long* q = &s[8 * w];
        start.push_back((q[0] - t0min) * 0.01);
        seg_b.push_back((q[1] - q[0]) * 0.01);
        seg_l.push_back((q[2] - q[1]) * 0.01);
        seg_c.push_back((q[3] - q[2]) * 0.01);
        seg_r.push_back((q[4] - q[3]) * 0.01);
        life.push_back((q[4] - q[0]) * 0.01);
        if (q[4] > q[0] && q[6] > q[5]) mhz.push_back((double)(q[6] - q[5]) / ((q[4] - q[0]) * 0.01));
    }
    auto pct = [](std::vector<double> v, double p) { if (v.empty()) return 0.0; std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
    auto row = [&](const char* n, const std::vector<double>& v) {
        printf("   %-22s p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f us\n", n, pct(v, .1), pct(v, .5), pct(v, .9), pct(v, 1.0));
    };
    printf("%s: %d waves, event %.3f us/launch; in-kernel span %.2f us; last data landed %.2f us; clock p50 %.0f MHz\n",
           name, nwaves, event_us, (t2max - t0min) * 0.01, (t1max - t0min) * 0.01, pct(mhz, .5));
    row("entry offset", start);
    row("entry->act barrier", seg_b);
    row("barrier->weights in", seg_l);
    row("compute", seg_c);
    row("reduce+store", seg_r);
    row("wave life", life);
    fflush(stdout);
}

int main() {
    const int N = 4096, K = 4096, nb = K / 32;
    const long wbytes = (long)N * nb * 18;
    const int R = (int)((640L << 20) / wbytes) + 1;
    std::vector<uint8_t*> w(R);
    std::vector<uint8_t> hw(wbytes), ha(nb * 36);
    srand(7);
    for (long b = 0; b < (long)N * nb; ++b) {
        uint16_t d = f2h(0.01f + 0.09f * (float)rand() / (float)RAND_MAX);
        memcpy(&hw[b * 18], &d, 2);
        for (int j = 0; j < 16; ++j) hw[b * 18 + 2 + j] = rand() & 0xFF;
    }
    for (int b = 0; b < nb; ++b) {
        uint16_t d = f2h(0.008f), s = f2h(1.0f);
        memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &s, 2);
        for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
    }
    for (auto& q : w) { CK(hipMalloc(&q, wbytes)); CK(hipMemcpy(q, hw.data(), wbytes, hipMemcpyHostToDevice)); }
    uint8_t* a; float* c; unsigned* scr;
    CK(hipMalloc(&a, ha.size())); CK(hipMemcpy(a, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&c, N * 4)); CK(hipMalloc(&scr, 4096));
    hipStream_t st; CK(hipStreamCreate(&st));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));

    auto run = [&](const char* name, int nwaves, std::function<void(const uint8_t*)> fn, bool cold) {
        for (int rep = 0; rep < 3; ++rep) {
            const int L = 200;
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < L; ++i) fn(w[cold ? i % R : 0]);
            CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            char nm[128]; snprintf(nm, sizeof nm, "%s %s rep%d", name, cold ? "cold" : "hot", rep);
            report(nm, nwaves, ms * 1e3 / L);
        }
    };
    GemmArgs g; g.A = a; g.C = c; g.M = 1; g.N = N; g.K = K; g.wtype = FMT_Q4_0; g.ldc_m = N; g.ldc_n = 1;
    // the product kernel (GEMV v2), stamped build
    auto gemv = [&](const uint8_t* B) { g.B = B; CK((gemv_launch<FMT_Q4_0, 1, 4, 32, 512, false>(g, st))); };
    run("gemv v2 bpl4 lpr32 wg512", 256 * 8, gemv, true);
    run("gemv v2 bpl4 lpr32 wg512", 256 * 8, gemv, false);
    const long n16 = wbytes / 16;
    auto rd2 = [&](const uint8_t* B) { hipLaunchKernelGGL(rd_stamp<2>, dim3((unsigned)((n16 / 2 + 255) / 256)), dim3(256), 0, st, B, wbytes, scr); };
    run("read x4 p2 wg256", (int)((n16 / 2 + 255) / 256) * 4, rd2, true);
    auto rd1 = [&](const uint8_t* B) { hipLaunchKernelGGL(rd_stamp<1>, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st, B, wbytes, scr); };
    run("read x4 p1 wg256", (int)((n16 + 255) / 256) * 4, rd1, true);
    auto rd9 = [&](const uint8_t* B) { hipLaunchKernelGGL(rd_stamp<9>, dim3((unsigned)((n16 / 9 + 511) / 512)), dim3(512), 0, st, B, wbytes, scr); };
    run("read x4 p9 wg512", (int)((n16 / 9 + 511) / 512) * 8, rd9, true);
    return 0;
}
