// hr_attn.hip -- the query embedder's encoder layers at query shapes (PyTorch-ROCm runs the GEMMs; these are the
// small memory / latency-bound pieces between them).
//
// A 64-query batch at the bge-large shape is ~1,900 tokens in ~64 sequences of ~30 tokens.  Per layer torch's
// variable-length flash attention took 19 us plus a 5 us fill of its own (profiles/r06_embed_forward_kernels.json),
// for work that is ~110 MFLOP and ~15 MB of traffic: its tiles are sized for long sequences.  Here:
//  * k_attn_short: one workgroup per (sequence, head), the sequence's K and V rows staged in LDS as fp32, one
//    thread per query row with its scaled q row and the output accumulator in registers, an online softmax over
//    the keys (running max, rescaled sum) -- the function of scaled_dot_product_attention on each sequence (every
//    token attends to its own sequence only, no mask inside it), fp32 throughout from the bf16 / f16 projections,
//    the output rounded once (RNE).  Sequences up to kMaxL tokens (query and short-passage batches); longer ones
//    are the flash kernel's (hr_attn_varlen returns HR_E_UNSUPPORTED and the caller takes that path).
//  * k_gelu_erf: BertIntermediate's exact (erf) GELU in place, 0.5 x (1 + erf(x / sqrt 2)) in fp32 per element,
//    rounded once -- torch's GeluCUDAKernelImpl's formula and opmath; 16-byte vectors, a grid sized to the tensor.
#include <hip/hip_runtime.h>

#include "../../include/hiprag.h"
#include "hr_common.hpp"

namespace {

constexpr int kMaxL = 64;  // longest sequence the short-sequence attention takes (two 32-key MFMA tiles)

template <int DT>
__device__ inline float ld1(const uint16_t* p) {
    return DT == HR_BF16 ? hr::bf16_to_f32(*p) : hr::f16_to_f32(*p);
}
// (f16: the hardware conversion, as torch's static_cast<at::Half> -- the integer recipe of hr_common.hpp rounds
// subnormal results differently in a few cases; bf16: RNE on the bits, as c10::BFloat16)
template <int DT>
__device__ inline uint16_t st1(float f) {
    return DT == HR_BF16 ? hr::f32_to_bf16_rne(f) : __builtin_bit_cast(uint16_t, (_Float16)f);
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int DT>
__device__ inline f32x16 mfma(const u32x4_t& a, const u32x4_t& b, const f32x16& c) {
    if constexpr (DT == HR_BF16)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(hr::bf16x8, a), __builtin_bit_cast(hr::bf16x8, b),
                                                       c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(hr::f16x8, a), __builtin_bit_cast(hr::f16x8, b), c,
                                                      0, 0, 0);
}

constexpr int kPadK = 8;  // LDS row padding (bf16 elements) of the transposed V and P tiles: 16-byte rows, fewer conflicts

// One workgroup per (head, sequence), two waves; wave w takes the query rows [32 w, 32 w + 32) of the sequence.
// qkv: [N][3][nH][64] (the fused QKV GEMM's output); cu: B + 1 int32 offsets; out: [N][nH][64].
// MFMA operand layout (v_mfma_f32_32x32x16, as hr_kernels.hpp): lane l = r + 32 u holds elements [8 u, 8 u + 8) of
// the k-step of row r; the 32 x 32 result holds column l % 32 in lane l and row 8 (v / 4) + 4 (l / 32) + v % 4 in
// register v.  So:
//  * S^T = K Q^T per 32-key tile (A = K rows, B = Q rows, straight 16-byte loads of the projections, 4 k-steps over
//    d = 64): a lane holds ONE query's scores against 16 keys, its lane partner l ^ 32 the other 16;
//  * the softmax of a query is in-lane (16 registers per key tile) plus one exchange with the partner; P (rounded to
//    the input type, as the flash kernel feeds its P V product) goes to LDS as P^T rows [query][key];
//  * O^T = V^T P^T per 32-column tile (A = V^T rows from LDS, staged transposed once per workgroup; B = P^T rows);
//    a lane then holds one query's outputs in 4 runs of 4 columns, divided by the fp32 row sum, rounded, stored.
template <int DT>
__global__ __launch_bounds__(128) void k_attn_mfma(const uint16_t* __restrict__ qkv, const int32_t* __restrict__ cu,
                                                   int nH, float scale, uint16_t* __restrict__ out) {
    constexpr int D = 64, NKT = 2;  // head dim; key tiles (sequences up to 64 tokens)
    constexpr int LK = 32 * NKT + kPadK;
    __shared__ __attribute__((aligned(16))) uint16_t vt[D][LK];        // V^T: [column][key]
    __shared__ __attribute__((aligned(16))) uint16_t pt[2][32][LK];    // P^T per wave: [query][key]
    const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int s0 = cu[b], L = cu[b + 1] - s0;
    if (L <= 0) return;
    const int64_t rs = (int64_t)3 * nH * D;  // token row stride
    const uint16_t* qbase = qkv + (int64_t)s0 * rs + (int64_t)h * D;
    const uint16_t* kbase = qkv + (int64_t)s0 * rs + (int64_t)(nH + h) * D;
    const uint16_t* vbase = qkv + (int64_t)s0 * rs + (int64_t)(2 * nH + h) * D;
    const int nkt = (L + 31) / 32;
    const int r = lane & 31, u = lane >> 5;
    const int qrow = 32 * w + r;
    const bool active = 32 * w < L;
    // ---- every global load first (one memory round trip): this thread's 4 (key, 8-column) pieces of V, then the
    // wave's Q and K fragments (rows past L: zeros)
    uint4 vr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = tid + 128 * i, j = e / (D / 8), c8 = (e % (D / 8)) * 8;  // keys 0..63
        vr[i] = make_uint4(0u, 0u, 0u, 0u);
        if (j < L) vr[i] = *(const uint4*)(vbase + (int64_t)j * rs + c8);
    }
    u32x4_t qf[4], kf[NKT][4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        qf[s] = u32x4_t{0u, 0u, 0u, 0u};
        if (active && qrow < L) qf[s] = *(const u32x4_t*)(qbase + (int64_t)qrow * rs + 16 * s + 8 * u);
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
            const int krow = 32 * kt + r;
            kf[kt][s] = u32x4_t{0u, 0u, 0u, 0u};
            if (active && krow < L) kf[kt][s] = *(const u32x4_t*)(kbase + (int64_t)krow * rs + 16 * s + 8 * u);
        }
    }
    // ---- V^T into LDS (both waves; keys past L are zeros)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = tid + 128 * i, j = e / (D / 8), c8 = (e % (D / 8)) * 8;
        if (j < 32 * nkt) {
            const uint16_t* v8 = (const uint16_t*)&vr[i];
#pragma unroll
            for (int t = 0; t < 8; ++t) vt[c8 + t][j] = v8[t];
        }
    }
    f32x16 st[NKT];
    if (active) {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
            st[kt] = f32x16{};
            if (kt < nkt) {
#pragma unroll
                for (int s = 0; s < 4; ++s) st[kt] = mfma<DT>(kf[kt][s], qf[s], st[kt]);
            }
        }
        // ---- softmax of query `r` (this lane: keys 32 kt + 8 (v / 4) + 4 u + v % 4; the partner lane ^ 32 the rest)
        float m = -__builtin_inff();
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int key = 32 * kt + 8 * (v >> 2) + 4 * u + (v & 3);
                if (key < L) m = fmaxf(m, st[kt][v]);
            }
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        float l = 0.f;
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                uint16_t p4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int v = 4 * g + e;
                    const int key = 32 * kt + 8 * g + 4 * u + e;
                    const float p = key < L ? expf((st[kt][v] - m) * scale) : 0.f;
                    l += p;
                    p4[e] = st1<DT>(p);
                }
                if (kt < nkt) *(uint2*)&pt[w][r][32 * kt + 8 * g + 4 * u] = *(const uint2*)p4;
            }
        }
        l += __shfl_xor(l, 32, 64);
        st[0][0] = l;  // (kept: the row sum, read back below)
    }
    __syncthreads();  // V^T staged by both waves; this wave's P^T written
    if (!active) return;
    const float inv = 1.0f / st[0][0];
    // ---- O^T = V^T P^T, two 32-column tiles, 2 nkt k-steps of 16 keys
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
        f32x16 o = f32x16{};
        for (int s = 0; s < 2 * nkt; ++s) {
            const u32x4_t a = *(const u32x4_t*)&vt[32 * ct + r][16 * s + 8 * u];
            const u32x4_t bb = *(const u32x4_t*)&pt[w][r][16 * s + 8 * u];
            o = mfma<DT>(a, bb, o);
        }
        if (qrow < L) {
            uint16_t* op = out + (int64_t)(s0 + qrow) * nH * D + (int64_t)h * D + 32 * ct;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                uint16_t o4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) o4[e] = st1<DT>(o[4 * g + e] * inv);
                *(uint2*)(op + 8 * g + 4 * u) = *(const uint2*)o4;
            }
        }
    }
}

template <int DT>
__global__ __launch_bounds__(256) void k_gelu_erf(uint16_t* __restrict__ x, int64_t n) {
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i + 8 <= n) {
        uint4 r = *(const uint4*)(x + i);
        uint16_t* r8 = (uint16_t*)&r;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float v = ld1<DT>(r8 + u);
            r8[u] = st1<DT>(0.5f * v * (1.0f + erff(v * 0.70710678118654752440f)));
        }
        *(uint4*)(x + i) = r;
    } else {
        for (int64_t k = i; k < n; ++k) {
            const float v = ld1<DT>(x + k);
            x[k] = st1<DT>(0.5f * v * (1.0f + erff(v * 0.70710678118654752440f)));
        }
    }
}

}  // namespace

extern "C" int hr_attn_varlen(const void* qkv_dev, int dtype, const int32_t* cu_dev, int B, int nH, int d, int max_len,
                              float scale, void* out_dev, void* stream) {
    if (!qkv_dev || !cu_dev || !out_dev || B <= 0 || nH <= 0 || d <= 0 || max_len < 0) return HR_E_INVALID;
    if ((dtype != HR_BF16 && dtype != HR_F16) || d != 64 || max_len > kMaxL || B > 65535) return HR_E_UNSUPPORTED;
    if (((uintptr_t)qkv_dev | (uintptr_t)out_dev) & 15u) return HR_E_UNSUPPORTED;  // 16-byte rows
    if (max_len == 0) return HR_OK;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)nH, (unsigned)B);
    if (dtype == HR_BF16)
        hipLaunchKernelGGL(k_attn_mfma<HR_BF16>, grid, dim3(128), 0, st, (const uint16_t*)qkv_dev, cu_dev, nH, scale,
                           (uint16_t*)out_dev);
    else
        hipLaunchKernelGGL(k_attn_mfma<HR_F16>, grid, dim3(128), 0, st, (const uint16_t*)qkv_dev, cu_dev, nH, scale,
                           (uint16_t*)out_dev);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}

extern "C" int hr_gelu_erf(void* x_dev, int dtype, int64_t n, void* stream) {
    if (!x_dev || n < 0) return HR_E_INVALID;
    if (dtype != HR_BF16 && dtype != HR_F16) return HR_E_UNSUPPORTED;
    if ((uintptr_t)x_dev & 15u) return HR_E_UNSUPPORTED;
    if (n == 0) return HR_OK;
    hipStream_t st = (hipStream_t)stream;
    const int64_t threads = (n + 7) / 8;
    const dim3 grid((unsigned)((threads + 255) / 256));
    if (dtype == HR_BF16) hipLaunchKernelGGL(k_gelu_erf<HR_BF16>, grid, dim3(256), 0, st, (uint16_t*)x_dev, n);
    else hipLaunchKernelGGL(k_gelu_erf<HR_F16>, grid, dim3(256), 0, st, (uint16_t*)x_dev, n);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}
