// Layout probe for v_mfma_i32_32x32x32_i8 on gfx950 (tools only): checks that
// lane l feeds A row (l & 31) / B column (l & 31) with a 16-byte k-slice, that
// A and B pair their k-slices element by element, and the C map
// col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k(const signed char* A, const signed char* B, int* C) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    v4i a, b;
    signed char* pa = (signed char*)&a; signed char* pb = (signed char*)&b;
    for (int e = 0; e < 16; ++e) { pa[e] = A[r * 32 + 16 * h + e]; pb[e] = B[r * 32 + 16 * h + e]; }
    v16i acc = {};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
    for (int g = 0; g < 16; ++g) C[l * 16 + g] = acc[g];
}
int main() {
    signed char hA[32 * 32], hB[32 * 32];   // hA[row][k], hB[col][k]
    srand(7);
    for (int i = 0; i < 1024; ++i) { hA[i] = (signed char)(rand() % 255 - 127); hB[i] = (signed char)(rand() % 255 - 127); }
    signed char *dA, *dB; int* dC;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 64 * 16 * 4);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    int hC[64 * 16];
    hipMemcpy(hC, dC, sizeof(hC), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int g = 0; g < 16; ++g) {
            const int col = l & 31, row = (g & 3) + 8 * (g >> 2) + 4 * (l >> 5);
            int ref = 0;
            for (int kk = 0; kk < 32; ++kk) ref += hA[row * 32 + kk] * hB[col * 32 + kk];
            if (ref != hC[l * 16 + g]) ++bad;
        }
    printf("mfma_i32_32x32x32_i8 layout probe: %d of 1024 mismatched\n", bad);
    return bad != 0;
}
