// Checks the assumed lane maps of v_mfma_i32_16x16x64_i8 on gfx950 with asymmetric integer data:
//   A: lane l holds A[row l&15][k = 16(l>>4) + j], j = 0..15 (4 VGPRs of packed int8)
//   B: lane l holds B[k = 16(l>>4) + j][col l&15]
//   C/D: lane l, reg r holds C[row 4(l>>4) + r][col l&15]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ int8_t Aval(int i, int k) { return (int8_t)((i * 3 + (k % 7) * 5 - 20) % 100); }
__device__ int8_t Bval(int k, int n) { return (int8_t)(((k * 5 + n * 11) % 13) - 6); }

__global__ void k(int* out) {
    const int l = threadIdx.x;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; j++) {
        a[j] = Aval(l & 15, 16 * (l >> 4) + j);
        b[j] = Bval(16 * (l >> 4) + j, l & 15);
    }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
    int bad = 0;
    for (int r = 0; r < 4; r++) {
        const int row = 4 * (l >> 4) + r, col = l & 15;
        int ref = 0;
        for (int kk = 0; kk < 64; kk++) ref += (int)Aval(row, kk) * (int)Bval(kk, col);
        bad += (c[r] != ref);
    }
    atomicAdd(out, bad);
}

int main() {
    int* d;
    hipMalloc(&d, 4);
    hipMemset(d, 0, 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h = -1;
    hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("mfma_i32_16x16x64_i8 layout mismatches: %d\n", h);
    return h != 0;
}
