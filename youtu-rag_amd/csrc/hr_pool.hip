// hr_pool.hip -- K7: the embedding server's pooling epilogue on the GPU.
// Restates LLMEmbeddingModel.encode (docs/content/docs/en/youtu-embedding/deploying-locally.mdx:81-116):
// the first len(instruction tokens) positions of the attention mask are zeroed (:98-112),
// masked mean over the sequence (mean_pooling :75-79), then F.normalize (x / max(||x||, 1e-12), :115).
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/hiprag.h"
#include "hr_common.hpp"

namespace {

template <int DT>
__device__ inline float ld(const void* p, int64_t i) {
    if (DT == hr::F32) return ((const float*)p)[i];
    const uint16_t v = ((const uint16_t*)p)[i];
    return DT == hr::BF16 ? hr::bf16_to_f32(v) : hr::f16_to_f32(v);
}

// grid (B, ceil(H/256)): thread owns one hidden column, sums over the sequence (coalesced over H)
template <int DT>
__global__ __launch_bounds__(256) void k_pool_sum(const void* __restrict__ hidden, const int32_t* __restrict__ mask,
                                                  int T, int H, int n_instr, float* __restrict__ out) {
    const int b = blockIdx.x;
    const int h = blockIdx.y * 256 + threadIdx.x;
    if (h >= H) return;
    float s = 0.f, d = 0.f;
    for (int t = 0; t < T; ++t) {
        const float m = (t < n_instr) ? 0.f : (float)mask[(int64_t)b * T + t];
        s += ld<DT>(hidden, ((int64_t)b * T + t) * H + h) * m;
        d += m;
    }
    out[(int64_t)b * H + h] = s / d;
}

__global__ __launch_bounds__(256) void k_l2norm(float* __restrict__ x, int H) {
    __shared__ float red[4];
    const int b = blockIdx.x;
    float p = 0.f;
    for (int h = threadIdx.x; h < H; h += 256) {
        const float v = x[(int64_t)b * H + h];
        p += v * v;
    }
    for (int off = 32; off >= 1; off >>= 1) p += __shfl_xor(p, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = p;
    __syncthreads();
    const float n = sqrtf(red[0] + red[1] + red[2] + red[3]);
    const float inv = 1.f / fmaxf(n, 1e-12f);
    for (int h = threadIdx.x; h < H; h += 256) x[(int64_t)b * H + h] *= inv;
}

}  // namespace

extern "C" int hr_pool_normalize(const void* hidden_dev, int dtype, const int32_t* mask_dev, int B, int T, int H,
                                 int n_instr, float* out_dev, void* stream) {
    if (!hidden_dev || !mask_dev || !out_dev || B <= 0 || T <= 0 || H <= 0 || n_instr < 0) return HR_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((unsigned)B, (unsigned)((H + 255) / 256));
    switch (dtype) {
        case HR_F32: hipLaunchKernelGGL(k_pool_sum<hr::F32>, grid, dim3(256), 0, st, hidden_dev, mask_dev, T, H, n_instr, out_dev); break;
        case HR_BF16: hipLaunchKernelGGL(k_pool_sum<hr::BF16>, grid, dim3(256), 0, st, hidden_dev, mask_dev, T, H, n_instr, out_dev); break;
        case HR_F16: hipLaunchKernelGGL(k_pool_sum<hr::F16>, grid, dim3(256), 0, st, hidden_dev, mask_dev, T, H, n_instr, out_dev); break;
        default: return HR_E_INVALID;
    }
    hipLaunchKernelGGL(k_l2norm, dim3((unsigned)B), dim3(256), 0, st, out_dev, H);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}
