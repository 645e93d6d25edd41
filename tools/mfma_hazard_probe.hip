// mfma_hazard_probe.hip — VALU read of a v_mfma_i32_16x16x32_i8 result after N extra wait states (diagnostic).
//   hipcc --offload-arch=gfx950 -O2 -o mfma_hazard_probe mfma_hazard_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
// MFMA, then exactly N wait states (s_nop), then a VALU read of the result (the compiler adds
// nothing when N exceeds its own hazard model). Compare with the value read much later.
template <int N>
__global__ void k(const long* ain, int* out) {
    int l = threadIdx.x;
    long a = ain[l], b = ain[64 + l];
    v4i c = {1000, 2000, 3000, 4000};
    v4i d = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c, 0, 0, 0);
    if constexpr (N > 0) {
        if constexpr (N > 8) asm volatile("s_nop 7\n\ts_nop %1" : "+v"(d) : "i"(N - 9));
        else asm volatile("s_nop %1" : "+v"(d) : "i"(N - 1));
    }
    int early = d[0] + d[1] + d[2] + d[3];
    out[l] = early;
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}
template <int N>
__global__ void late(const long* ain, int* out) {
    int l = threadIdx.x;
    long a = ain[l], b = ain[64 + l];
    v4i c = {1000, 2000, 3000, 4000};
    v4i d = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c, 0, 0, 0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(d));
    out[l] = d[0] + d[1] + d[2] + d[3];
}
int main() {
    long h_a[128];
    for (int i = 0; i < 128; ++i) h_a[i] = 0x0102030405060708L * (i % 7 + 1) ^ (0x1111111111111111L * (i % 3));
    long* d_a; int* dev; (void)hipMalloc(&d_a, sizeof h_a); (void)hipMalloc(&dev, 512);
    (void)hipMemcpy(d_a, h_a, sizeof h_a, hipMemcpyHostToDevice);
    int ref[64], h[64];
    late<0><<<1, 64>>>(d_a, dev); (void)hipDeviceSynchronize(); (void)hipMemcpy(ref, dev, 256, hipMemcpyDeviceToHost);
#define T(N) { k<N><<<1, 64>>>(d_a, dev); (void)hipDeviceSynchronize(); (void)hipMemcpy(h, dev, 256, hipMemcpyDeviceToHost); \
      int bad = 0; for (int l = 0; l < 64; ++l) bad += h[l] != ref[l]; printf("wait states %2d: wrong in %d of 64 lanes\n", N, bad); }
    T(0) T(2) T(4) T(6) T(8) T(10) T(12) T(14) T(16) T(18) T(20) T(24)
    return 0;
}
