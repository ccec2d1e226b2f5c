// Checks the lane layout of v_mfma_i32_32x32x32_i8 with exact integer data:
// hypothesis: lane l holds A[l & 31][16 (l >> 5) + j] and B[16 (l >> 5) + j][l & 31]
// in byte j of its 16-byte operand; D[row][col] with col = l & 31,
// row = (r & 3) + 8 (r >> 2) + 4 (l >> 5) for accumulator register r.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const signed char *A, const signed char *B, int *D, int layout) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    signed char a[16], b[16];
    for (int j = 0; j < 16; j++) {
        const int kk = layout == 0 ? 16 * h + j : 8 * h + (j & 7) + 16 * (j >> 3);
        a[j] = A[r * 32 + kk];
        b[j] = B[kk * 32 + r];
    }
    v4i va, vb;
    __builtin_memcpy(&va, a, 16);
    __builtin_memcpy(&vb, b, 16);
    v16i c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(va, vb, c, 0, 0, 0);
    for (int q = 0; q < 16; q++) {
        const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
        D[row * 32 + r] = c[q];
    }
}

int main() {
    signed char hA[1024], hB[1024];
    int ref[1024], got[1024];
    srand(7);
    for (int i = 0; i < 1024; i++) { hA[i] = (signed char)(rand() % 255 - 127); hB[i] = (signed char)(rand() % 255 - 127); }
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) {
            int s = 0;
            for (int kk = 0; kk < 32; kk++) s += hA[i * 32 + kk] * hB[kk * 32 + j];
            ref[i * 32 + j] = s;
        }
    signed char *dA, *dB;
    int *dD;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 4096);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    for (int layout = 0; layout < 2; layout++) {
        hipMemset(dD, 0, 4096);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD, layout);
        hipMemcpy(got, dD, 4096, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 1024; i++) bad += got[i] != ref[i];
        printf("layout %d: %d of 1024 differ\n", layout, bad);
    }
    return 0;
}
