// Checks the operand / result layout of v_mfma_f32_16x16x32_bf16 assumed by the 16x16x32 form of the 256-query
// FILTER: A (16 x 32): lane l holds row l % 16, k = 8 (l / 16) .. + 7; B (32 x 16): lane l holds column l % 16, the
// same k; D (16 x 16): lane l holds column l % 16, rows 4 (l / 16) + r in register r.  Prints PASS / FAIL.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const float* A, const float* B, float* D) {
    const int l = threadIdx.x;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)A[(l % 16) * 32 + 8 * (l / 16) + j];
        b[j] = (__bf16)B[(8 * (l / 16) + j) * 16 + (l % 16)];
    }
    f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, f32x4{0, 0, 0, 0}, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + (l % 16)] = d[r];
}

int main() {
    float A[16 * 32], B[32 * 16], D[256], ref[256];
    for (int i = 0; i < 16 * 32; ++i) A[i] = (float)((i * 7) % 13 - 6);
    for (int i = 0; i < 32 * 16; ++i) B[i] = (float)((i * 5) % 11 - 5);
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            float s = 0;
            for (int kk = 0; kk < 32; ++kk) s += A[m * 32 + kk] * B[kk * 16 + n];
            ref[m * 16 + n] = s;
        }
    float *dA, *dB, *dD;
    hipMalloc(&dA, sizeof(A));
    hipMalloc(&dB, sizeof(B));
    hipMalloc(&dD, sizeof(D));
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(D, dD, sizeof(D), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += D[i] != ref[i];
    printf("%s (%d of 256 differ)\n", bad ? "FAIL" : "PASS", bad);
    return bad != 0;
}
