// stream_ceiling.hip -- the practical read-only HBM streaming ceiling of one MI355X, for the scan's
// roofline.  Reads a buffer of the scan's size (default 20.48 GB = 10M x 1024 bf16)
// once per launch with the scan's access shape: every wave streams a contiguous range of 1 KiB
// chunks, one 16-byte load per lane, a ring of P loads in flight, a trivial reduction so nothing is
// optimised away.  Variants: non-temporal vs default-policy loads, all CUs vs the scan's n_cu - 32,
// 8 or 16 waves per CU.  Prints one line per variant: bytes / (average launch time from HIP events).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_ceiling.hip -o tools/stream_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                            \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

template <bool NT, int P>
__global__ __launch_bounds__(512) void k_stream(const u32x4* __restrict__ src, long long n_chunks,
                                               unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long long W = (long long)gridDim.x * (blockDim.x >> 6);
    const long long w = (long long)(threadIdx.x >> 6) * gridDim.x + blockIdx.x;  // wave-major, as the scan
    const long long base = n_chunks / W, rem = n_chunks % W;
    const long long c0 = w * base + (w < rem ? w : rem);
    const long long c1 = c0 + base + (w < rem ? 1 : 0);
    u32x4 ring[P];
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < P; ++i)
        ring[i] = (c0 + i < c1) ? (NT ? __builtin_nontemporal_load(src + (c0 + i) * 64 + lane) : src[(c0 + i) * 64 + lane])
                                : u32x4{0u, 0u, 0u, 0u};
    // branch-free main loop while a whole ring of prefetches stays inside the range, then the rest
    long long c = c0;
    for (; c + 2 * P <= c1; c += P) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            acc ^= ring[i];
            ring[i] = NT ? __builtin_nontemporal_load(src + (c + P + i) * 64 + lane) : src[(c + P + i) * 64 + lane];
        }
    }
    for (; c < c1; c += P) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            if (c + i < c1) acc ^= ring[i];
            const long long nx = c + P + i;
            if (nx < c1) ring[i] = NT ? __builtin_nontemporal_load(src + nx * 64 + lane) : src[nx * 64 + lane];
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1u;  // never true in practice
}

// The scan's stream with a pinned slice: chunks of every pin-th 64-KiB tile are loaded with the default
// policy (they allocate in, and after the first pass hit, the Infinity Cache), all others non-temporal.
template <int P>
__global__ __launch_bounds__(512) void k_stream_pin(const u32x4* __restrict__ src, long long n_chunks, int pin,
                                                    unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long long W = (long long)gridDim.x * (blockDim.x >> 6);
    const long long w = (long long)(threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    const long long base = n_chunks / W, rem = n_chunks % W;
    const long long c0 = w * base + (w < rem ? w : rem);
    const long long c1 = c0 + base + (w < rem ? 1 : 0);
    auto ld = [&](long long c) -> u32x4 {
        if (((c >> 6) & (long long)(pin - 1)) == 0) return src[c * 64 + lane];  // pin: a power of two
        return __builtin_nontemporal_load(src + c * 64 + lane);
    };
    u32x4 ring[P];
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < P; ++i) ring[i] = (c0 + i < c1) ? ld(c0 + i) : u32x4{0u, 0u, 0u, 0u};
    long long c = c0;
    // the policy is chosen once per batch of P chunks (P divides a tile's 64): two unrolled copies
    // of the batch, so no branch sits between a load and the use of its ring slot
    for (; c + 2 * P <= c1; c += P) {
        if ((((c + P) >> 6) & (long long)(pin - 1)) == 0) {
#pragma unroll
            for (int i = 0; i < P; ++i) {
                acc ^= ring[i];
                ring[i] = src[(c + P + i) * 64 + lane];
            }
        } else {
#pragma unroll
            for (int i = 0; i < P; ++i) {
                acc ^= ring[i];
                ring[i] = __builtin_nontemporal_load(src + (c + P + i) * 64 + lane);
            }
        }
    }
    for (; c < c1; c += P) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            if (c + i < c1) acc ^= ring[i];
            const long long nx = c + P + i;
            if (nx < c1) ring[i] = ld(nx);
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1u;
}

// The query-group launch's access shape without its arithmetic: ng workgroups per range block (equal
// blockIdx % 8, so one XCD), each streaming the SAME tiles in the same order with default-policy loads
// (the first to touch a line brings it into L2, the others hit or wait on the same fill) -- the memory
// system's own ceiling for B = ng x 64 queries, and how it moves with waves per CU.
template <int P>
__global__ __launch_bounds__(1024) void k_stream_groups(const u32x4* __restrict__ src, long long n_chunks, int ng,
                                                        unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const int bx = blockIdx.x;
    const long long nrb = gridDim.x / ng;
    const long long rb = ng > 1 ? (long long)((bx >> 3) / ng) * 8 + (bx & 7) : bx;
    const long long W = nrb * (blockDim.x >> 6);
    const long long w = (long long)(threadIdx.x >> 6) * nrb + rb;
    const long long base = n_chunks / W, rem = n_chunks % W;
    const long long c0 = w * base + (w < rem ? w : rem);
    const long long c1 = c0 + base + (w < rem ? 1 : 0);
    u32x4 ring[P];
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < P; ++i) ring[i] = (c0 + i < c1) ? src[(c0 + i) * 64 + lane] : u32x4{0u, 0u, 0u, 0u};
    long long c = c0;
    for (; c + 2 * P <= c1; c += P) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            acc ^= ring[i];
            ring[i] = src[(c + P + i) * 64 + lane];
        }
    }
    for (; c < c1; c += P) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            if (c + i < c1) acc ^= ring[i];
            const long long nx = c + P + i;
            if (nx < c1) ring[i] = src[nx * 64 + lane];
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1u;
}

// Lagged groups: as k_stream_groups, but group g walks its range rotated by g * lag chunks (wrapping),
// so a trailing group re-reads what the leading one read lag chunks earlier -- from L2 / the Infinity
// Cache rather than by waiting on the same fill.  ntl: the trailing groups load non-temporal.
template <int P>
__global__ __launch_bounds__(512) void k_stream_lag(const u32x4* __restrict__ src, long long n_chunks, int ng,
                                                    long long lag, int ntl, unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const int bx = blockIdx.x;
    const int grp = ng > 1 ? (bx >> 3) % ng : 0;
    const long long nrb = gridDim.x / ng;
    const long long rb = ng > 1 ? (long long)((bx >> 3) / ng) * 8 + (bx & 7) : bx;
    const long long W = nrb * (blockDim.x >> 6);
    const long long w = (long long)(threadIdx.x >> 6) * nrb + rb;
    const long long base = n_chunks / W, rem = n_chunks % W;
    const long long c0 = w * base + (w < rem ? w : rem);
    const long long len = base + (w < rem ? 1 : 0);
    const long long off = len > 0 ? (grp * lag) % len : 0;
    const bool nt = ntl && grp > 0;
    u32x4 acc = {0u, 0u, 0u, 0u};
    u32x4 ring[P];
    auto at = [&](long long i) -> const u32x4* {
        long long j = i + off;
        if (j >= len) j -= len;
        return src + (c0 + j) * 64 + lane;
    };
#pragma unroll
    for (int i = 0; i < P; ++i) ring[i] = i < len ? (nt ? __builtin_nontemporal_load(at(i)) : *at(i)) : u32x4{0u, 0u, 0u, 0u};
    long long c = 0;
    for (; c + 2 * P <= len; c += P) {
        if (nt) {
#pragma unroll
            for (int i = 0; i < P; ++i) {
                acc ^= ring[i];
                ring[i] = __builtin_nontemporal_load(at(c + P + i));
            }
        } else {
#pragma unroll
            for (int i = 0; i < P; ++i) {
                acc ^= ring[i];
                ring[i] = *at(c + P + i);
            }
        }
    }
    for (; c < len; c += P) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            if (c + i < len) acc ^= ring[i];
            if (c + P + i < len) ring[i] = *at(c + P + i);
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1u;
}

// Tile-strided assignment: wave w streams tiles (64 chunks) w, w + W, w + 2W, ... instead of one
// contiguous range, so at any moment the chip's waves read one ~W x 64 KiB window of the buffer in order.
template <int P>
__global__ __launch_bounds__(512) void k_stream_strided(const u32x4* __restrict__ src, long long n_tiles, int tile_chunks,
                                                        unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long long W = (long long)gridDim.x * (blockDim.x >> 6);
    const long long w = (long long)(threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (long long t = w; t < n_tiles; t += W) {
        const u32x4* base = src + t * tile_chunks * 64 + lane;
        for (int c = 0; c < tile_chunks; c += P) {
            u32x4 ring[P];
#pragma unroll
            for (int i = 0; i < P; ++i) ring[i] = __builtin_nontemporal_load(base + (c + i) * 64);
#pragma unroll
            for (int i = 0; i < P; ++i) acc ^= ring[i];
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1u;
}

// Tile-strided variants: map = 0 wave-major numbering (as the scan), 1 workgroup-major (a workgroup's
// 8 waves take 8 consecutive tiles); pre = 1 keeps the next burst in flight while one is consumed.
template <int P>
__global__ __launch_bounds__(512) void k_stream_strided2(const u32x4* __restrict__ src, long long n_tiles, int tile_chunks,
                                                         int map, int pre, unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long long W = (long long)gridDim.x * (blockDim.x >> 6);
    const long long w = map ? (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)
                            : (long long)(threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    if (!pre) {
        for (long long t = w; t < n_tiles; t += W) {
            const u32x4* base = src + t * tile_chunks * 64 + lane;
            for (int c = 0; c < tile_chunks; c += P) {
                u32x4 ring[P];
#pragma unroll
                for (int i = 0; i < P; ++i) ring[i] = __builtin_nontemporal_load(base + (c + i) * 64);
#pragma unroll
                for (int i = 0; i < P; ++i) acc ^= ring[i];
            }
        }
    } else {
        // chunk sequence of this wave: tiles w, w+W, ..., each tile_chunks long; ring of P prefetched
        const long long nt = w < n_tiles ? (n_tiles - 1 - w) / W + 1 : 0;
        const long long total = nt * tile_chunks;
        auto addr = [&](long long k) { return src + ((w + (k / tile_chunks) * W) * tile_chunks + k % tile_chunks) * 64 + lane; };
        u32x4 ring[P];
#pragma unroll
        for (int i = 0; i < P; ++i) ring[i] = i < total ? __builtin_nontemporal_load(addr(i)) : u32x4{0u, 0u, 0u, 0u};
        for (long long k = 0; k < total; k += P) {
#pragma unroll
            for (int i = 0; i < P; ++i) {
                acc ^= ring[i];
                if (k + P + i < total) ring[i] = __builtin_nontemporal_load(addr(k + P + i));
            }
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1u;
}

template <bool NT, int P>
static double run(const u32x4* buf, long long n_chunks, unsigned* sink, int blocks, int threads, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_stream<NT, P>), dim3(blocks), dim3(threads), 0, 0, buf, n_chunks, sink);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_stream<NT, P>), dim3(blocks), dim3(threads), 0, 0, buf, n_chunks, sink);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 20.48;
    const long long bytes = (long long)(gb * 1e9) / 1024 * 1024;
    const long long n_chunks = bytes / 1024;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int n_cu = prop.multiProcessorCount;
    u32x4* buf = nullptr;
    unsigned* sink = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(buf, 1, bytes));
    CHECK(hipDeviceSynchronize());
    const int reps = 10;
    struct V { const char* name; bool nt; int cus; int threads; };
    for (const V& v : std::vector<V>{{"nt, ring 32, n_cu-32 CUs, 8 waves/CU", true, n_cu - 32, 512}}) {
        const double ms = run<true, 32>(buf, n_chunks, sink, v.cus, v.threads, reps);
        std::printf("{\"variant\": \"%s\", \"bytes\": %lld, \"ms\": %.4f, \"TBps\": %.4f, \"frac_of_8TBps\": %.4f}\n",
                    v.name, bytes, ms, bytes / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 8e12);
    }
    std::vector<V> vs = {{"nt, n_cu-32 CUs, 8 waves/CU (the scan's launch)", true, n_cu - 32, 512},
                         {"nt, all CUs, 8 waves/CU", true, n_cu, 512},
                         {"default policy, n_cu-32 CUs, 8 waves/CU", false, n_cu - 32, 512},
                         {"nt, all CUs, 16 waves/CU (2 blocks/CU)", true, 2 * n_cu, 512}};
    for (const V& v : vs) {
        const double ms = v.nt ? run<true, 16>(buf, n_chunks, sink, v.cus, v.threads, reps)
                               : run<false, 16>(buf, n_chunks, sink, v.cus, v.threads, reps);
        std::printf("{\"variant\": \"%s\", \"bytes\": %lld, \"ms\": %.4f, \"TBps\": %.4f, \"frac_of_8TBps\": %.4f}\n",
                    v.name, bytes, ms, bytes / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 8e12);
    }
    // Infinity Cache residency behind the scan's stream: read a sample-sized table (128 MiB, default
    // policy), stream the big buffer (non-temporal or default loads), then time a re-read of the table.
    // Compared with a re-read right after the first read (resident) and one after a default-policy
    // stream (evicted): tells whether nt streaming leaves a small, repeatedly read set in the L3.
    if (argc > 2 && atoi(argv[2]) == 2) {  // pinned slice: every pin-th tile default-policy, rest nt
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        for (int pin : {1 << 30, 64, 32, 16, 8}) {
            for (int r = 0; r < 3; ++r)  // warm: the pinned slice settles in the cache
                hipLaunchKernelGGL((k_stream_pin<16>), dim3(n_cu - 32), dim3(512), 0, 0, buf, n_chunks, pin, sink);
            CHECK(hipEventRecord(a, 0));
            for (int r = 0; r < reps; ++r)
                hipLaunchKernelGGL((k_stream_pin<16>), dim3(n_cu - 32), dim3(512), 0, 0, buf, n_chunks, pin, sink);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double t = ms / reps;
            const long long pinned = pin >= (1 << 30) ? 0 : (n_chunks / 64 + pin - 1) / pin * 65536ll;
            std::printf("{\"variant\": \"nt stream, every %d-th tile default policy\", \"bytes\": %lld, \"pinned_bytes\": %lld, "
                        "\"ms\": %.4f, \"TBps\": %.4f, \"frac_of_8TBps\": %.4f}\n",
                        pin >= (1 << 30) ? 0 : pin, bytes, pinned, t, bytes / (t * 1e-3) / 1e12, bytes / (t * 1e-3) / 8e12);
        }
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
    if (argc > 2 && atoi(argv[2]) == 3) {  // query-group access shape: ng x waves per CU
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        const int cus = n_cu - 32;
        for (int ng : {1, 2, 4})
            for (int threads : {512, 768, 1024}) {
                const int blocks = std::max(8, cus / ng / 8 * 8) * ng;
                hipLaunchKernelGGL((k_stream_groups<16>), dim3(blocks), dim3(threads), 0, 0, buf, n_chunks, ng, sink);
                CHECK(hipDeviceSynchronize());
                CHECK(hipEventRecord(a, 0));
                for (int r = 0; r < reps; ++r)
                    hipLaunchKernelGGL((k_stream_groups<16>), dim3(blocks), dim3(threads), 0, 0, buf, n_chunks, ng, sink);
                CHECK(hipEventRecord(b, 0));
                CHECK(hipEventSynchronize(b));
                float ms = 0.f;
                CHECK(hipEventElapsedTime(&ms, a, b));
                const double t = ms / reps;
                std::printf("{\"variant\": \"query-group shape, default policy\", \"ng\": %d, \"waves_per_cu\": %d, "
                            "\"blocks\": %d, \"bytes\": %lld, \"ms\": %.4f, \"unique_TBps\": %.4f}\n",
                            ng, threads / 64, blocks, bytes, t, bytes / (t * 1e-3) / 1e12);
            }
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
    if (argc > 2 && atoi(argv[2]) == 4) {  // lagged groups: ng x lag x trailing-group policy
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        const int cus = n_cu - 32;
        for (int ng : {2, 4})
            for (long long lag : {0ll, 16ll, 64ll, 128ll, 256ll, 1024ll})
                for (int ntl : {0, 1}) {
                    if (lag == 0 && ntl) continue;
                    const int blocks = std::max(8, cus / ng / 8 * 8) * ng;
                    hipLaunchKernelGGL((k_stream_lag<16>), dim3(blocks), dim3(512), 0, 0, buf, n_chunks, ng, lag, ntl, sink);
                    CHECK(hipDeviceSynchronize());
                    CHECK(hipEventRecord(a, 0));
                    for (int r = 0; r < reps; ++r)
                        hipLaunchKernelGGL((k_stream_lag<16>), dim3(blocks), dim3(512), 0, 0, buf, n_chunks, ng, lag, ntl, sink);
                    CHECK(hipEventRecord(b, 0));
                    CHECK(hipEventSynchronize(b));
                    float ms = 0.f;
                    CHECK(hipEventElapsedTime(&ms, a, b));
                    const double t = ms / reps;
                    std::printf("{\"variant\": \"lagged groups\", \"ng\": %d, \"lag_KiB\": %lld, \"trailing_nt\": %d, "
                                "\"bytes\": %lld, \"ms\": %.4f, \"unique_TBps\": %.4f}\n",
                                ng, lag, ntl, bytes, t, bytes / (t * 1e-3) / 1e12);
                }
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
    if (argc > 2 && atoi(argv[2]) == 5) {  // contiguous ranges vs tile-strided assignment
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        const int cus = n_cu - 32;
        for (int tc : {16, 64, 256}) {
            const long long n_tiles = n_chunks / tc;
            hipLaunchKernelGGL((k_stream_strided<16>), dim3(cus), dim3(512), 0, 0, buf, n_tiles, tc, sink);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(a, 0));
            for (int r = 0; r < reps; ++r)
                hipLaunchKernelGGL((k_stream_strided<16>), dim3(cus), dim3(512), 0, 0, buf, n_tiles, tc, sink);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double t = ms / reps;
            const long long by = n_tiles * tc * 1024;
            std::printf("{\"variant\": \"tile-strided, nt, n_cu-32 CUs, 8 waves/CU\", \"tile_KiB\": %d, \"bytes\": %lld, "
                        "\"ms\": %.4f, \"TBps\": %.4f}\n", tc, by, t, by / (t * 1e-3) / 1e12);
        }
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
    if (argc > 2 && atoi(argv[2]) == 6) {  // tile-strided variants
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        struct SV { int cus, map, pre; };
        for (SV v : std::vector<SV>{{n_cu - 32, 0, 0}, {n_cu - 32, 1, 0}, {n_cu - 32, 0, 1}, {n_cu, 0, 0}, {n_cu - 32, 0, 0}}) {
            const int tc = 64;
            const long long n_tiles = n_chunks / tc;
            hipLaunchKernelGGL((k_stream_strided2<16>), dim3(v.cus), dim3(512), 0, 0, buf, n_tiles, tc, v.map, v.pre, sink);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(a, 0));
            for (int r = 0; r < reps; ++r)
                hipLaunchKernelGGL((k_stream_strided2<16>), dim3(v.cus), dim3(512), 0, 0, buf, n_tiles, tc, v.map, v.pre, sink);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double t = ms / reps;
            const long long by = n_tiles * tc * 1024;
            std::printf("{\"variant\": \"tile-strided\", \"cus\": %d, \"wg_major\": %d, \"prefetch\": %d, \"bytes\": %lld, "
                        "\"ms\": %.4f, \"TBps\": %.4f}\n", v.cus, v.map, v.pre, by, t, by / (t * 1e-3) / 1e12);
        }
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
    if (argc > 2 && atoi(argv[2]) == 1) {
        const long long tb = 128ll << 20, t_chunks = tb / 1024;
        u32x4* tab = nullptr;
        CHECK(hipMalloc(&tab, tb));
        CHECK(hipMemset(tab, 2, tb));
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        const int blocks = n_cu, threads = 512, R = 20;
        for (int mode = 0; mode < 3; ++mode) {  // 0: nothing between, 1: nt stream between, 2: default stream
            double tot = 0.0;
            for (int r = 0; r < R; ++r) {
                hipLaunchKernelGGL((k_stream<false, 16>), dim3(blocks), dim3(threads), 0, 0, tab, t_chunks, sink);
                if (mode == 1) hipLaunchKernelGGL((k_stream<true, 16>), dim3(n_cu - 32), dim3(512), 0, 0, buf, n_chunks, sink);
                if (mode == 2) hipLaunchKernelGGL((k_stream<false, 16>), dim3(n_cu - 32), dim3(512), 0, 0, buf, n_chunks, sink);
                CHECK(hipEventRecord(a, 0));
                hipLaunchKernelGGL((k_stream<false, 16>), dim3(blocks), dim3(threads), 0, 0, tab, t_chunks, sink);
                CHECK(hipEventRecord(b, 0));
                CHECK(hipEventSynchronize(b));
                float ms = 0.f;
                CHECK(hipEventElapsedTime(&ms, a, b));
                tot += ms;
            }
            const double ms = tot / R;
            static const char* names[3] = {"table re-read, nothing between", "table re-read after nt stream of buffer",
                                           "table re-read after default-policy stream of buffer"};
            std::printf("{\"variant\": \"%s\", \"table_bytes\": %lld, \"stream_bytes\": %lld, \"ms\": %.4f, \"TBps\": %.4f}\n",
                        names[mode], tb, mode ? bytes : 0ll, ms, tb / (ms * 1e-3) / 1e12);
        }
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
        CHECK(hipFree(tab));
    }
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
