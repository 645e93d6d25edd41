// mfma_hazard_probe.hip — how many wait states must separate an MFMA from a VALU read of its result
// on gfx950 (diagnostic; the prefill's epilogue depends on it, qg_mmq_kernel.hpp). The MFMA, exactly
// N wait states (s_nop) and the VALU read of its result are ONE inline-asm string (the compiler pads
// nothing inside it), so N is exact; the value is compared with a read after 64 states. The
// compiler's own pad for the same pair (hipcc --save-temps of an intrinsic version) is `s_nop 7` =
// 8 states for both instructions.
//   hipcc --offload-arch=gfx950 -O2 -o mfma_hazard_probe mfma_hazard_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define NOPS(N) (N >= 1 ? "s_nop 0\n" : ""), (N >= 2 ? "s_nop 0\n" : "")
template <int N> struct nops;
#define NOPSTR_0 ""
#define NOPSTR_4 "s_nop 3\n"
#define NOPSTR_6 "s_nop 5\n"
#define NOPSTR_8 "s_nop 7\n"
#define NOPSTR_9 "s_nop 7\ns_nop 0\n"
#define NOPSTR_10 "s_nop 7\ns_nop 1\n"
#define NOPSTR_11 "s_nop 7\ns_nop 2\n"
#define NOPSTR_12 "s_nop 7\ns_nop 3\n"
#define NOPSTR_14 "s_nop 7\ns_nop 5\n"
#define NOPSTR_16 "s_nop 7\ns_nop 7\n"
#define NOPSTR_20 "s_nop 7\ns_nop 7\ns_nop 3\n"
#define NOPSTR_64 "s_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\n"

#define KERNEL(NAME, OP, NSTR)                                                                      \
    __global__ void NAME(const long* ain, int* out) {                                              \
        const int l = threadIdx.x;                                                                 \
        const long a = ain[l], b = ain[64 + l];                                                    \
        int r;                                                                                     \
        asm volatile("v_mov_b32 v40, 1000\n v_mov_b32 v41, 2000\n v_mov_b32 v42, 3000\n"          \
                     " v_mov_b32 v43, 4000\n s_nop 4\n " OP " v[40:43], %1, %2, v[40:43]\n" NSTR   \
                     " v_add3_u32 %0, v40, v41, v42\n s_nop 0\n v_xor_b32 %0, %0, v43\n"            \
                     : "=&v"(r) : "v"(a), "v"(b) : "v40", "v41", "v42", "v43");                   \
        out[l] = r;                                                                                \
    }
#define I8 "v_mfma_i32_16x16x32_i8"
#define F16 "v_mfma_f32_16x16x16_f16"
KERNEL(i8_ref, I8, NOPSTR_64) KERNEL(i8_0, I8, NOPSTR_0) KERNEL(i8_4, I8, NOPSTR_4) KERNEL(i8_6, I8, NOPSTR_6)
KERNEL(i8_8, I8, NOPSTR_8) KERNEL(i8_9, I8, NOPSTR_9) KERNEL(i8_10, I8, NOPSTR_10) KERNEL(i8_11, I8, NOPSTR_11)
KERNEL(i8_12, I8, NOPSTR_12) KERNEL(i8_14, I8, NOPSTR_14) KERNEL(i8_16, I8, NOPSTR_16) KERNEL(i8_20, I8, NOPSTR_20)
KERNEL(f16_ref, F16, NOPSTR_64) KERNEL(f16_0, F16, NOPSTR_0) KERNEL(f16_4, F16, NOPSTR_4) KERNEL(f16_6, F16, NOPSTR_6)
KERNEL(f16_8, F16, NOPSTR_8) KERNEL(f16_9, F16, NOPSTR_9) KERNEL(f16_10, F16, NOPSTR_10) KERNEL(f16_11, F16, NOPSTR_11)
KERNEL(f16_12, F16, NOPSTR_12) KERNEL(f16_14, F16, NOPSTR_14) KERNEL(f16_16, F16, NOPSTR_16) KERNEL(f16_20, F16, NOPSTR_20)

int main() {
    long h_a[128];
    for (int i = 0; i < 128; ++i) h_a[i] = (0x0102030405060708L * (i % 7 + 1) ^ (0x1111111111111111L * (i % 3))) & 0x3F7F3F7F3F7F3F7FL;
    long* d_a; int* dev; (void)hipMalloc(&d_a, sizeof h_a); (void)hipMalloc(&dev, 512);
    (void)hipMemcpy(d_a, h_a, sizeof h_a, hipMemcpyHostToDevice);
    int ref[64], h[64];
    typedef void (*K)(const long*, int*);
    struct { const char* name; K ref; K k[11]; } fam[2] = {
        {I8, i8_ref, {i8_0, i8_4, i8_6, i8_8, i8_9, i8_10, i8_11, i8_12, i8_14, i8_16, i8_20}},
        {F16, f16_ref, {f16_0, f16_4, f16_6, f16_8, f16_9, f16_10, f16_11, f16_12, f16_14, f16_16, f16_20}}};
    const int ns[11] = {0, 4, 6, 8, 9, 10, 11, 12, 14, 16, 20};
    for (int rep = 0; rep < 3; ++rep)
        for (auto& f : fam) {
            f.ref<<<1, 64>>>(d_a, dev); (void)hipDeviceSynchronize(); (void)hipMemcpy(ref, dev, 256, hipMemcpyDeviceToHost);
            printf("%s rep %d:", f.name, rep);
            for (int i = 0; i < 11; ++i) {
                f.k[i]<<<1, 64>>>(d_a, dev); (void)hipDeviceSynchronize(); (void)hipMemcpy(h, dev, 256, hipMemcpyDeviceToHost);
                int bad = 0; for (int l = 0; l < 64; ++l) bad += h[l] != ref[l];
                printf("  N=%d:%d", ns[i], bad);
            }
            printf("   (lanes wrong of 64 after N wait states)\n");
        }
    return 0;
}
