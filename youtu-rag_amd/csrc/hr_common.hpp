// hr_common.hpp -- types and bit-exact scalar helpers shared by the hiprag kernels.
// The conversion and generator recipes are identical to oracle/hr_oracle.c (the checker).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hr {

enum { F32 = 0, BF16 = 1, F16 = 2 };
enum { COSINE = 0, IP = 1, L2 = 2 };

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Cand {  // exact candidate record exchanged between shards (16 B)
    double score;
    int64_t row;
};

// ---------------------------------------------------------------- scalar helpers
__device__ __host__ inline uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (uint16_t)((u >> 16) | 0x40u);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
__device__ __host__ inline float bf16_to_f32(uint16_t h) { return __builtin_bit_cast(float, (uint32_t)h << 16); }

__device__ __host__ inline uint16_t f32_to_f16_rne(float f) {  // same bit recipe as oracle hro_f32_to_f16
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    uint32_t sign = (u >> 16) & 0x8000u;
    uint32_t a = u & 0x7FFFFFFFu;
    if (a >= 0x7F800000u) return (uint16_t)(sign | 0x7C00u | (a > 0x7F800000u ? 0x200u : 0u));
    if (a >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);
    if (a < 0x38800000u) {
        int e = (int)(a >> 23);
        if (e < 102) return (uint16_t)sign;
        uint32_t m = (a & 0x7FFFFFu) | 0x800000u;
        int shift = 126 - e;
        uint32_t q = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t r = a - 0x38000000u;
    r += 0xFFFu + ((r >> 13) & 1u);
    return (uint16_t)(sign | (r >> 13));
}
__device__ __host__ inline float f16_to_f32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

template <int MT>
__device__ inline uint16_t quant_mt(float f) {
    return MT == BF16 ? f32_to_bf16_rne(f) : f32_to_f16_rne(f);
}
template <int MT>
__device__ inline float dequant_mt(uint16_t h) {
    return MT == BF16 ? bf16_to_f32(h) : f16_to_f32(h);
}

// order-preserving float <-> uint32 key (larger key = larger float); -0 and +0 share a key, as
// they compare equal (the oracle orders with IEEE comparisons)
__device__ __host__ inline uint32_t f2key(float f) {
    uint32_t u = __builtin_bit_cast(uint32_t, f == 0.0f ? 0.0f : f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __host__ inline float key2f(uint32_t k) {
    uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    return __builtin_bit_cast(float, u);
}
#define HR_KEY_NEG_INF 0x007FFFFFu  // f2key(-inf)

__device__ __host__ inline uint64_t d2key(double d) {
    uint64_t u = __builtin_bit_cast(uint64_t, d == 0.0 ? 0.0 : d);
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// inverse of d2key
__device__ __host__ inline double key2d(uint64_t k) {
    uint64_t u = (k & 0x8000000000000000ull) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __builtin_bit_cast(double, u);
}

// byte offset of k-step chunk (tile, s) for lane l; stride 1 KiB (16-bit) / 2 KiB (fp32)
template <int DT>
__device__ __host__ inline size_t chunk_bytes() { return DT == F32 ? 2048 : 1024; }

// Slot swizzle: row r of tile t = r / 32 sits in tile slot (r + tile_rot(t)) % 32, i.e. in the
// MFMA lane / group-max group of that slot.  The per-tile rotation is a Fibonacci hash of the tile,
// so rows that share r % 32 (a document's k-th chunks, a cluster inserted with a period that is a
// multiple of 32, ...) spread over all 32 groups instead of collapsing into one, which would leave
// the other 31 group maxima to background rows and the scan threshold far below the top-k.
__device__ __host__ inline int tile_rot(int64_t t) { return (int)((uint32_t)((uint64_t)t * 0x9E3779B1ull) >> 27); }
__device__ __host__ inline int row_slot(int64_t r) { return (int)((r + tile_rot(r >> 5)) & 31); }
__device__ __host__ inline int slot_row(int64_t t, int slot) { return (slot - tile_rot(t)) & 31; }  // row % 32

// Multi-device handles stripe rows over G shards by 32-row tile: handle row H lives in shard
// (H/32) % G at local row ((H/32)/G)*32 + H%32.  Every shard's rows stay an append-only
// contiguous range (the tiles of one shard fill in order), and the global row of shard s's local
// row L is stripe_row(L, G, s) -- G = 1 is the identity.
__device__ __host__ inline int64_t stripe_row(int64_t L, int G, int s) {
    return G == 1 ? L : ((((L >> 5) * G) + s) << 5) | (L & 31);
}

// element (row r, column d) of the tiled corpus, as float
template <int DT>
__device__ inline float load_elem(const uint8_t* base, int S, int64_t r, int d) {
    int64_t chunk = (r >> 5) * S + (d >> 4);
    int lane = row_slot(r) + 32 * ((d >> 3) & 1);
    int j = d & 7;
    if (DT == F32) {
        const float* p = (const float*)(base + chunk * 2048 + (j >> 2) * 1024 + lane * 16);
        return p[j & 3];
    } else {
        const uint16_t* p = (const uint16_t*)(base + chunk * 1024 + lane * 16);
        return DT == BF16 ? bf16_to_f32(p[j]) : f16_to_f32(p[j]);
    }
}

__device__ inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ inline float gen_elem(uint64_t seed, int64_t row, int dim, int d) {
    uint64_t z = mix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)row * (uint64_t)dim + (uint64_t)d);
    int64_t v = (int64_t)(z & 0xFFFF) + (int64_t)((z >> 16) & 0xFFFF) + (int64_t)((z >> 32) & 0xFFFF) +
                (int64_t)(z >> 48) - 131070;
    return (float)v;
}

// Guard bound on |approx - exact| of the scan score of query q (DESIGN.md "Exactness guard"):
// inner product E = max|x| (|q - q̂| + (gamma + u_x) |q̂|); euclidean (scan score 2 q̂.x - |x|^2 in
// fp32) adds the doubled dot error, the fp32 rounding of |x|^2 and of the fused multiply-add.
__device__ __host__ inline double guard_e(const double* qe, double max_norm, double gamma, double u_x, int metric) {
    const double E = max_norm * (qe[0] * (1.0 + 1e-6) + (gamma + u_x) * qe[1]) + 1e-9;
    if (metric != L2) return E;
    return 2.0 * E + 0x1p-22 * (max_norm * max_norm + 2.0 * max_norm * qe[1]) + 1e-9;
}

// Exact euclidean similarity 1 - ((|q|^2 - 2 q.x) + |x|^2) from the canonical terms (oracle
// row_score); monotone in s = 2 q.x - |x|^2 up to fp64 rounding, whose size euclid_slack bounds.
__device__ __host__ inline double euclid_score(double qn2, double dot, double xn2) {
    return 1.0 - ((qn2 - 2.0 * dot) + xn2);
}
__device__ __host__ inline double euclid_slack(double qn2, double max_norm) {
    return 0x1p-50 * (1.0 + qn2 + max_norm * max_norm + 2.0 * max_norm * __builtin_sqrt(qn2));
}

__device__ inline double wave_butterfly_sum(double p) {  // canonical: p[i] + p[i ^ off], off = 32..1
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        double o = __shfl_xor(p, off, 64);
        int lane = threadIdx.x & 63;
        p = (lane & off) ? (o + p) : (p + o);  // keep p[i] + p[i+off] operand order for i < off
    }
    return p;
}

}  // namespace hr
