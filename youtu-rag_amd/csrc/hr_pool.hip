// hr_pool.hip -- K7: the embedding server's pooling epilogue on the GPU; K8: the encoder layers'
// fused residual add + LayerNorm (embedder and cross-encoder forwards).
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

// packed (unpadded) hidden states: sequence b is rows [cu[b], cu[b+1]) of an (N, H) matrix, every row a
// real token; the first n_instr of them are masked out.  Same sums, in the same order, as k_pool_sum
// over the padded batch (whose masked positions add exact zeros).
template <int DT>
__global__ __launch_bounds__(256) void k_pool_sum_packed(const void* __restrict__ hidden, const int32_t* __restrict__ cu,
                                                         int H, int n_instr, float* __restrict__ out) {
    const int b = blockIdx.x;
    const int h = blockIdx.y * 256 + threadIdx.x;
    if (h >= H) return;
    const int64_t t1 = cu[b + 1];
    float s = 0.f, d = 0.f;
    for (int64_t t = (int64_t)cu[b] + n_instr; t < t1; ++t) {
        s += ld<DT>(hidden, t * H + h);
        d += 1.f;
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

template <int DT>
__device__ inline void st1(void* p, int64_t i, float v) {
    if (DT == hr::F32) {
        ((float*)p)[i] = v;
    } else {
        ((uint16_t*)p)[i] = DT == hr::BF16 ? hr::f32_to_bf16_rne(v) : hr::f32_to_f16_rne(v);
    }
}
template <int DT>
__device__ inline float round_to(float v) {  // the value a tensor of this dtype holds
    if (DT == hr::F32) return v;
    return DT == hr::BF16 ? hr::bf16_to_f32(hr::f32_to_bf16_rne(v)) : hr::f16_to_f32(hr::f32_to_f16_rne(v));
}

// K8: y = LayerNorm(x + r) * gamma + beta for one row per workgroup (BertSelfOutput / BertOutput /
// XLMRobertaSelfOutput / XLMRobertaOutput after their dense layer, modeling_bert.py).  Same values as
// PyTorch's two kernels: the sum is rounded to the tensor dtype (the elementwise add's output), the
// statistics are fp32 (mean, then the biased variance of the deviations), rstd = rsqrt(var + eps),
// the affine map in fp32, one rounding to the dtype.  One read of x and r and one write instead of
// the add's write + LayerNorm's re-read (the residual-add kernel disappears).  H <= 256 * kLnE.
constexpr int kLnE = 16;
template <int DT>
__global__ __launch_bounds__(256) void k_add_layernorm(const void* __restrict__ x, const void* __restrict__ r,
                                                       const void* __restrict__ g, const void* __restrict__ bta,
                                                       void* __restrict__ y, int H, float eps) {
    __shared__ float red[4];
    const int64_t row = blockIdx.x;
    const int tid = threadIdx.x;
    float v[kLnE];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kLnE; ++j) {
        const int h = tid + 256 * j;
        v[j] = h < H ? round_to<DT>(ld<DT>(x, row * H + h) + ld<DT>(r, row * H + h)) : 0.f;
        s += v[j];
    }
    auto block_sum = [&](float p) {
        for (int off = 32; off >= 1; off >>= 1) p += __shfl_xor(p, off, 64);
        __syncthreads();  // red[] may still be read by the previous reduction
        if ((tid & 63) == 0) red[tid >> 6] = p;
        __syncthreads();
        return (red[0] + red[1]) + (red[2] + red[3]);
    };
    const float mean = block_sum(s) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < kLnE; ++j)
        if (tid + 256 * j < H) {
            const float d = v[j] - mean;
            q += d * d;
        }
    const float rstd = rsqrtf(block_sum(q) / (float)H + eps);
#pragma unroll
    for (int j = 0; j < kLnE; ++j) {
        const int h = tid + 256 * j;
        if (h < H) st1<DT>(y, row * H + h, (v[j] - mean) * rstd * ld<DT>(g, h) + ld<DT>(bta, h));
    }
}

// Wave-per-row K8 for the common widths (H = 64*C*N: 768 = 64*4*3, 1024 = 64*8*2, ...): each lane
// loads N vectors of C contiguous elements (8 or 16 bytes; a wave instruction reads 64*C elements
// in one contiguous run), both statistics reduce with wave shuffles only (no LDS, no barrier), four
// rows per 256-thread workgroup.  Same arithmetic as the generic kernel.
template <int DT, int C>
__device__ inline void ld_vec(const void* p, int64_t i, float* o) {
    if constexpr (DT == hr::F32) {
        static_assert(C == 4, "fp32: 16-byte vectors of 4");
        const float4 v = *(const float4*)((const float*)p + i);
        o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
    } else if constexpr (C == 8) {
        const uint4 v = *(const uint4*)((const uint16_t*)p + i);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint16_t lo = (uint16_t)(w[c] & 0xFFFFu), hi = (uint16_t)(w[c] >> 16);
            o[2 * c] = DT == hr::BF16 ? hr::bf16_to_f32(lo) : hr::f16_to_f32(lo);
            o[2 * c + 1] = DT == hr::BF16 ? hr::bf16_to_f32(hi) : hr::f16_to_f32(hi);
        }
    } else {
        static_assert(C == 4, "16-bit: vectors of 4 or 8");
        const uint2 v = *(const uint2*)((const uint16_t*)p + i);
        const uint32_t w[2] = {v.x, v.y};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint16_t lo = (uint16_t)(w[c] & 0xFFFFu), hi = (uint16_t)(w[c] >> 16);
            o[2 * c] = DT == hr::BF16 ? hr::bf16_to_f32(lo) : hr::f16_to_f32(lo);
            o[2 * c + 1] = DT == hr::BF16 ? hr::bf16_to_f32(hi) : hr::f16_to_f32(hi);
        }
    }
}
template <int DT, int C>
__device__ inline void st_vec(void* p, int64_t i, const float* v) {
    if constexpr (DT == hr::F32) {
        *(float4*)((float*)p + i) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
        uint32_t w[C / 2];
#pragma unroll
        for (int c = 0; c < C / 2; ++c) {
            const uint16_t lo = DT == hr::BF16 ? hr::f32_to_bf16_rne(v[2 * c]) : hr::f32_to_f16_rne(v[2 * c]);
            const uint16_t hi = DT == hr::BF16 ? hr::f32_to_bf16_rne(v[2 * c + 1]) : hr::f32_to_f16_rne(v[2 * c + 1]);
            w[c] = (uint32_t)lo | ((uint32_t)hi << 16);
        }
        if constexpr (C == 8)
            *(uint4*)((uint16_t*)p + i) = make_uint4(w[0], w[1], w[2], w[3]);
        else
            *(uint2*)((uint16_t*)p + i) = make_uint2(w[0], w[1]);
    }
}

template <int DT, int C, int N>
__global__ __launch_bounds__(256) void k_add_layernorm_w(const void* __restrict__ x, const void* __restrict__ r,
                                                         const void* __restrict__ g, const void* __restrict__ bta,
                                                         void* __restrict__ y, int64_t rows, float eps) {
    constexpr int H = 64 * C * N;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    float v[N][C];
    float s = 0.f;
    // gamma / beta loaded with x and r (one memory round trip, not one after the reductions)
    float gg[N][C], bb[N][C];
#pragma unroll
    for (int n = 0; n < N; ++n) {
        const int col = (n * 64 + lane) * C;
        ld_vec<DT, C>(g, col, gg[n]);
        ld_vec<DT, C>(bta, col, bb[n]);
    }
#pragma unroll
    for (int n = 0; n < N; ++n) {
        const int64_t off = row * H + (int64_t)(n * 64 + lane) * C;
        float a[C], b[C];
        ld_vec<DT, C>(x, off, a);
        ld_vec<DT, C>(r, off, b);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            v[n][c] = round_to<DT>(a[c] + b[c]);
            s += v[n][c];
        }
    }
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)H;
    float q = 0.f;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const float d = v[n][c] - mean;
            q += d * d;
        }
    for (int o = 32; o >= 1; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q / (float)H + eps);
#pragma unroll
    for (int n = 0; n < N; ++n) {
        const int col = (n * 64 + lane) * C;
        float o_[C];
#pragma unroll
        for (int c = 0; c < C; ++c) o_[c] = (v[n][c] - mean) * rstd * gg[n][c] + bb[n][c];
        st_vec<DT, C>(y, row * H + col, o_);
    }
}

template <int DT>
int launch_add_ln(const void* x, const void* r, const void* g, const void* b, void* y, int64_t rows, int H, float eps,
                  hipStream_t st) {
    const dim3 gw((unsigned)((rows + 3) / 4));
#define HR_LN_CASE(Cv, Nv) \
    if (H == 64 * (Cv) * (Nv)) { \
        hipLaunchKernelGGL((k_add_layernorm_w<DT, Cv, Nv>), gw, dim3(256), 0, st, x, r, g, b, y, rows, eps); \
        return HR_OK; \
    }
    if constexpr (DT == hr::F32) {
        HR_LN_CASE(4, 1) HR_LN_CASE(4, 2) HR_LN_CASE(4, 3) HR_LN_CASE(4, 4) HR_LN_CASE(4, 6) HR_LN_CASE(4, 8)
    } else {
        HR_LN_CASE(8, 1) HR_LN_CASE(4, 3) HR_LN_CASE(8, 2) HR_LN_CASE(8, 3) HR_LN_CASE(8, 4) HR_LN_CASE(4, 1)
    }
#undef HR_LN_CASE
    hipLaunchKernelGGL(k_add_layernorm<DT>, dim3((unsigned)rows), dim3(256), 0, st, x, r, g, b, y, H, eps);
    return HR_OK;
}

}  // namespace

extern "C" int hr_add_layernorm(const void* x_dev, const void* r_dev, const void* gamma_dev, const void* beta_dev,
                                void* out_dev, int64_t rows, int H, float eps, int dtype, void* stream) {
    if (!x_dev || !r_dev || !gamma_dev || !beta_dev || !out_dev || rows < 0 || H <= 0 || H > 256 * kLnE)
        return HR_E_INVALID;
    if (rows == 0) return HR_OK;
    hipStream_t st = (hipStream_t)stream;
    // the vector kernels need 16-byte aligned rows (torch allocations are; views might not be)
    const bool aligned = (((uintptr_t)x_dev | (uintptr_t)r_dev | (uintptr_t)gamma_dev | (uintptr_t)beta_dev |
                           (uintptr_t)out_dev) & 15u) == 0;
    int rc = HR_E_INVALID;
    switch (dtype) {
        case HR_F32: rc = aligned ? launch_add_ln<hr::F32>(x_dev, r_dev, gamma_dev, beta_dev, out_dev, rows, H, eps, st) : -100; break;
        case HR_BF16: rc = aligned ? launch_add_ln<hr::BF16>(x_dev, r_dev, gamma_dev, beta_dev, out_dev, rows, H, eps, st) : -100; break;
        case HR_F16: rc = aligned ? launch_add_ln<hr::F16>(x_dev, r_dev, gamma_dev, beta_dev, out_dev, rows, H, eps, st) : -100; break;
        default: return HR_E_INVALID;
    }
    if (rc == -100) {  // unaligned: the generic row-per-workgroup kernel (scalar loads)
        const dim3 grid((unsigned)rows);
        if (dtype == HR_F32) hipLaunchKernelGGL(k_add_layernorm<hr::F32>, grid, dim3(256), 0, st, x_dev, r_dev, gamma_dev, beta_dev, out_dev, H, eps);
        else if (dtype == HR_BF16) hipLaunchKernelGGL(k_add_layernorm<hr::BF16>, grid, dim3(256), 0, st, x_dev, r_dev, gamma_dev, beta_dev, out_dev, H, eps);
        else hipLaunchKernelGGL(k_add_layernorm<hr::F16>, grid, dim3(256), 0, st, x_dev, r_dev, gamma_dev, beta_dev, out_dev, H, eps);
    } else if (rc) {
        return rc;
    }
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}

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

extern "C" int hr_pool_normalize_packed(const void* hidden_dev, int dtype, const int32_t* cu_dev, int B, int H,
                                        int n_instr, float* out_dev, void* stream) {
    if (!hidden_dev || !cu_dev || !out_dev || B <= 0 || H <= 0 || n_instr < 0) return HR_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((unsigned)B, (unsigned)((H + 255) / 256));
    switch (dtype) {
        case HR_F32: hipLaunchKernelGGL(k_pool_sum_packed<hr::F32>, grid, dim3(256), 0, st, hidden_dev, cu_dev, H, n_instr, out_dev); break;
        case HR_BF16: hipLaunchKernelGGL(k_pool_sum_packed<hr::BF16>, grid, dim3(256), 0, st, hidden_dev, cu_dev, H, n_instr, out_dev); break;
        case HR_F16: hipLaunchKernelGGL(k_pool_sum_packed<hr::F16>, grid, dim3(256), 0, st, hidden_dev, cu_dev, H, n_instr, out_dev); break;
        default: return HR_E_INVALID;
    }
    hipLaunchKernelGGL(k_l2norm, dim3((unsigned)B), dim3(256), 0, st, out_dev, H);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}
