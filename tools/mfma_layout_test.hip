// mfma_layout_test.hip — operand / accumulator lane layout of v_mfma_i32_16x16x32_i8 (diagnostic).
//   hipcc --offload-arch=gfx950 -O2 -o mfma_layout_test mfma_layout_test.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
// A[i][k] = i+1 at k == kk only; B[k][j] = j+1 at k == kk only -> C[i][j] = (i+1)(j+1)
__global__ void k(int kk, int* out) {
    int l = threadIdx.x, r = l & 15, q = l >> 4;
    long a = 0, b = 0;
    if (kk / 8 == q) { a = (long)(r + 1) << (8 * (kk % 8)); b = (long)(r + 1) << (8 * (kk % 8)); }
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c, 0, 0, 0);
    for (int e = 0; e < 4; ++e) out[l * 4 + e] = c[e];
}
int main() {
    int* d; hipMalloc(&d, 256 * 4); int h[256];
    for (int kk : {0, 9, 31}) {
        k<<<1, 64>>>(kk, d); hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l) for (int e = 0; e < 4; ++e) {
            int col = l & 15, row = 4 * (l >> 4) + e;
            if (h[l * 4 + e] != (row + 1) * (col + 1)) { if (bad < 5) printf("kk=%d lane %d e %d got %d want %d\n", kk, l, e, h[l*4+e], (row+1)*(col+1)); bad++; }
        }
        printf("kk=%d bad=%d\n", kk, bad);
    }
    return 0;
}
