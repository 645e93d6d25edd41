// mmq_debug.hip — small-shape check of mmq_kernel (per-block sumi and outputs) against a host
// loop for Q4_0 and Q4_1. Diagnostic tool, not part of the product.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "qg_mmq_kernel.hpp"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace qg;
static float h2f_host(uint16_t b) { _Float16 h; memcpy(&h, &b, 2); return (float)h; }
static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t b; memcpy(&b, &h, 2); return b; }
template <int F, int BN, int TT, int W>
static void check(int M, int N, int K) {
    const int nb = K / 32, BB = F == FMT_Q4_0 ? 18 : 20, QS = F == FMT_Q4_0 ? 2 : 4;
    std::vector<uint8_t> hw((size_t)N * nb * BB), ha((size_t)M * nb * 36);
    srand(3);
    for (size_t b = 0; b < (size_t)N * nb; ++b) {
        for (int j = 0; j < BB; ++j) hw[b * BB + j] = rand() & 0xFF;
        uint16_t d = f2h(0.05f + 0.01f * (rand() % 5)); memcpy(&hw[b * BB], &d, 2);
        if (F == FMT_Q4_1) { uint16_t m = f2h(-0.3f + 0.01f * (rand() % 7)); memcpy(&hw[b * BB + 2], &m, 2); }
    }
    for (size_t b = 0; b < (size_t)M * nb; ++b) {
        uint16_t d = f2h(0.01f), s = f2h(1.0f + (rand() % 9)); memcpy(&ha[b * 36], &d, 2); memcpy(&ha[b * 36 + 2], &s, 2);
        for (int j = 0; j < 32; ++j) ha[b * 36 + 4 + j] = (uint8_t)(rand() % 255 - 127);
    }
    std::vector<int> want((size_t)M * N * nb);
    for (int m = 0; m < M; ++m) for (int n = 0; n < N; ++n) for (int b = 0; b < nb; ++b) {
        const uint8_t* w = &hw[((size_t)n * nb + b) * BB + QS]; const int8_t* a = (const int8_t*)&ha[((size_t)m * nb + b) * 36 + 4];
        int s = 0; for (int j = 0; j < 16; ++j) s += a[j] * (w[j] & 15) + a[j + 16] * (w[j] >> 4);
        want[((size_t)m * N + n) * nb + b] = s;
    }
    uint8_t *da, *dw; int* ds; float* dc;
    CK(hipMalloc(&da, ha.size())); CK(hipMalloc(&dw, hw.size())); CK(hipMalloc(&ds, want.size() * 4)); CK(hipMalloc(&dc, M * N * 4));
    CK(hipMemcpy(da, ha.data(), ha.size(), hipMemcpyHostToDevice)); CK(hipMemcpy(dw, hw.data(), hw.size(), hipMemcpyHostToDevice));
    CK(hipMemset(ds, 0, want.size() * 4));
    GemmArgs g; g.A = da; g.B = dw; g.C = dc; g.sumi = ds; g.M = M; g.N = N; g.K = K; g.wtype = F; g.ldc_m = N; g.ldc_n = 1;
    if (!mmq_shape_ok<F, BN, TT, W, false>(g)) { printf("shape rejected\n"); return; }
    CK((mmq_launch<F, BN, TT, W, true, false>(g, 0)));
    CK(hipDeviceSynchronize());
    std::vector<int> got(want.size());
    CK(hipMemcpy(got.data(), ds, got.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (size_t i = 0; i < want.size(); ++i) bad += got[i] != want[i];
    g.sumi = nullptr;
    CK((mmq_launch<F, BN, TT, W, false, false>(g, 0)));
    CK(hipDeviceSynchronize());
    std::vector<float> c(M * N);
    CK(hipMemcpy(c.data(), dc, c.size() * 4, hipMemcpyDeviceToHost));
    int badc = 0;
    for (int m = 0; m < M; ++m) for (int n = 0; n < N; ++n) {
        double ref = 0;
        for (int b = 0; b < nb; ++b) {
            const uint8_t* wb = &hw[((size_t)n * nb + b) * BB]; const uint8_t* ab = &ha[((size_t)m * nb + b) * 36];
            float dwf = h2f_host(*(const uint16_t*)wb), daf = h2f_host(*(const uint16_t*)ab), saf = h2f_host(*(const uint16_t*)(ab + 2));
            float fs = (float)want[((size_t)m * N + n) * nb + b];
            if (F == FMT_Q4_0) ref += dwf * (daf * fs - 8.0f * saf);
            else ref += dwf * daf * fs + h2f_host(*(const uint16_t*)(wb + 2)) * saf;
        }
        if (fabs(c[m * N + n] - ref) > 1e-3 * (1 + fabs(ref))) { if (badc < 6) printf("  C m=%d n=%d got %f want %f\n", m, n, c[m * N + n], ref); badc++; }
    }
    printf("fmt %d BN %d TT %d W %d M=%d N=%d K=%d: sumi bad %d / %zu, C bad %d / %d\n", F, BN, TT, W, M, N, K, bad, want.size(), badc, M * N);
    CK(hipFree(da)); CK(hipFree(dw)); CK(hipFree(ds)); CK(hipFree(dc));
}
int main() {
    check<FMT_Q4_0, 16, 2, 8>(32, 16, 512);
    check<FMT_Q4_0, 16, 1, 8>(9, 96, 2048);
    check<FMT_Q4_1, 16, 1, 8>(16, 16, 512);
    check<FMT_Q4_1, 16, 1, 8>(16, 16, 128);
    check<FMT_Q4_1, 16, 1, 1>(16, 16, 128);
    check<FMT_Q4_1, 16, 2, 8>(32, 16, 512);
    check<FMT_Q4_1, 32, 1, 8>(16, 32, 512);
    check<FMT_Q4_1, 32, 4, 4>(64, 32, 512);
    return 0;
}
