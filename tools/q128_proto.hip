// q128_proto.hip -- timing prototype of a one-read-per-tile scan for 128 queries at D = 1024 (DESIGN.md
// "Query groups"): 4 waves per CU (one per SIMD), each streaming its own tiles through a 32-deep register
// ring (two halves of 16 k-steps), the queries' A-fragments re-staged into LDS in depth windows of 16
// k-steps (QB x 16 KiB, double-buffered) that all four waves walk in lock step (one barrier per window),
// MFMA 32x32x16 bf16, and a k_scan-like epilogue (group maxima, threshold ballot).  No candidate output:
// the memory side + arithmetic of the pass only, to decide whether the design reaches the HBM stream.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/q128_proto.hip -o tools/q128_proto
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                            \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int S = 64;   // k-steps per tile (D = 1024)
constexpr int WIN = 16;  // k-steps per query window
constexpr int NWIN = S / WIN;

__device__ inline f32x16 mfma(const u32x4& a, const u32x4& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// mode bit 1: skip the MFMAs (memory + LDS only); bit 2: skip the LDS query reads too
// Addressing keeps registers for data: corpus and query loads are buffer loads (one V# per tile in SGPRs, the
// lane offset in one VGPR, the k-step offset in the scalar offset), LDS reads one base + immediates.
template <int QB, int MODE, int SB, int PD = 1, int ROT = 0, int REP = 1>
__global__ __launch_bounds__(256, 1) void k_q(const u32x4* __restrict__ corpus, const u32x4* __restrict__ qfrag,
                                             long long n_tiles, int mode_unused, unsigned* __restrict__ sink) {
    constexpr int mode = MODE;
    constexpr int WQ = WIN * QB * 64;                            // u32x4 per window
    // static LDS (base address 0): the compiler then folds every fragment offset into the ds_read's
    // immediate (with the dynamic extern array it kept one address VGPR per read)
    __shared__ __attribute__((aligned(16))) u32x4 lds[2 * WQ];  // [2][WIN][QB][64]
    __shared__ __attribute__((aligned(16))) float th_lds[4][QB * 32];  // per wave: the threshold of each query
    constexpr int PER = WQ / 256;                                // staged per thread per window
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long W = (long long)gridDim.x * 4;
    const long long wr = (long long)wv * gridDim.x + blockIdx.x;
    const long long n_rounds = n_tiles / W;
    auto uni = [](long long v) -> long long {  // wave-uniform value in SGPRs
        const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
        const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)((unsigned long long)v >> 32));
        return (long long)(((unsigned long long)hi << 32) | lo);
    };
    auto tile = [&](long long u) -> long long { return uni((u < n_rounds ? u : n_rounds - 1) * W + wr); };
    auto rsrc = [&](long long t) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)corpus + t * (S * 1024)), (short)0, S * 1024, 0x00020000);
    };
    const int voff = lane * 16;
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int kstep) -> u32x4 {
        return __builtin_amdgcn_raw_buffer_load_b128(r, voff, kstep * 1024, 2);  // nt
    };
    // REP > 1: workgroup b reads replica b % REP of the query fragments (L2 hot-spot test)
    const __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)qfrag + (size_t)(blockIdx.x % REP) * S * QB * 1024), (short)0, S * QB * 1024, 0x00020000);
    // ROT: workgroup b walks the windows of every tile starting at window b % 4 (spreads the staging reads
    // of one moment over four windows); any k-step order gives a valid approximate score
    const int rot = ROT ? (int)(blockIdx.x & (NWIN - 1)) : 0;
    auto wk = [&](int w) { return (w + rot) & (NWIN - 1); };

    u32x4 ra[WIN], rb[WIN];
    {
        const auto r0 = rsrc(tile(0));
#pragma unroll
        for (int i = 0; i < WIN; ++i) ra[i] = ld(r0, wk(0) * WIN + i);
#pragma unroll
        for (int i = 0; i < WIN; ++i) rb[i] = ld(r0, wk(1) * WIN + i);
    }
    // window 0 -> buffer 0
#pragma unroll
    for (int j = 0; j < PER; ++j) lds[j * 256 + tid] = __builtin_amdgcn_raw_buffer_load_b128(qr, tid * 16, wk(0) * WQ * 16 + j * 4096, 0);
    __syncthreads();

    float gmax[QB][16];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) gmax[qb][i] = -1e30f;
    if (lane < QB * 32 / 2) {
        th_lds[wv][2 * lane] = __builtin_bit_cast(float, (unsigned)(0x7E000000u + lane));
        th_lds[wv][2 * lane + 1] = __builtin_bit_cast(float, (unsigned)(0x7E000001u + lane));
    }
    unsigned passes = 0;
    for (long long u = 0; u < n_rounds; ++u) {
        const auto rt = rsrc(tile(u)), rn = rsrc(tile(u + 1));
        f32x16 acc[QB];
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[qb][i] = 0.f;
#pragma unroll
        for (int w = 0; w < NWIN; ++w) {
            u32x4(&ring)[WIN] = (w & 1) ? rb : ra;
            if (!(mode & 8) && (w > 0 || u > 0)) {  // window w's queries are in LDS buffer w & 1 (every wave staged its share)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            // next window's query fragments: global -> registers (two halves), -> LDS during / after this
            // window's k-steps
            constexpr int PH = PER / 2;
            u32x4 stg[PH];
            const int wsrc = wk(w + 1) * WQ * 16;
            if (!(mode & 4)) {
#pragma unroll
                for (int j = 0; j < PH; ++j) stg[j] = __builtin_amdgcn_raw_buffer_load_b128(qr, tid * 16, wsrc + j * 4096, 0);
            }
            unsigned doff = (unsigned)(((w + 1) & 1) * WQ + tid);
            asm volatile("" : "+v"(doff));
            u32x4* dst = lds + doff;
            // the window's base address made opaque per window: otherwise the compiler hoists all 16*QB
            // fragment addresses out of the loop into registers instead of using the ds_read immediate
            unsigned qoff = (unsigned)((w & 1) * WQ + lane);
            asm volatile("" : "+v"(qoff));
            const u32x4* qs = lds + qoff;
            // query fragments PD k-steps ahead: the reads of k-step i + PD go out before the MFMAs of k-step i
            u32x4 qf[PD + 1][QB];
            if (!(mode & 2)) {
#pragma unroll
                for (int d = 0; d < PD; ++d)
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) qf[d][qb] = qs[(d * QB + qb) * 64];
            }
#pragma unroll
            for (int i = 0; i < WIN; ++i) {
                if (!(mode & 2) && i + PD < WIN) {
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) qf[(i + PD) % (PD + 1)][qb] = qs[((i + PD) * QB + qb) * 64];
                }
                const u32x4 x = ring[i];
                ring[i] = (w + 2 < NWIN) ? ld(rt, wk(w + 2) * WIN + i) : ld(rn, wk(w + 2 - NWIN) * WIN + i);
                if (!(mode & 2)) {
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        const u32x4 qc = qf[i % (PD + 1)][qb];
                        if (!(mode & 1)) acc[qb] = mfma(qc, x, acc[qb]);
                        else acc[qb][0] += __builtin_bit_cast(float, qc.x ^ x.x);
                    }
                } else {
                    acc[0][i & 15] += __builtin_bit_cast(float, x.x ^ x.y ^ x.z ^ x.w);
                }
                if (SB) __builtin_amdgcn_sched_barrier(0);  // (keeps the next k-step's LDS reads ahead of these MFMAs)
                if (!(mode & 4) && i == WIN / 2 - 1) {  // first half of the staging -> LDS, second half's loads go out
#pragma unroll
                    for (int j = 0; j < PH; ++j) dst[j * 256] = stg[j];
#pragma unroll
                    for (int j = 0; j < PH; ++j)
                        stg[j] = __builtin_amdgcn_raw_buffer_load_b128(qr, tid * 16, wsrc + (PH + j) * 4096, 0);
                }
            }
            if (!(mode & 4)) {
#pragma unroll
                for (int j = 0; j < PH; ++j) dst[(PH + j) * 256] = stg[j];
            }
        }
        // epilogue: group maxima + threshold ballots (k_scan's fast path); thresholds from LDS, four
        // consecutive queries (i & 3) per 16-byte read
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                typedef float f32x4 __attribute__((ext_vector_type(4)));
                const f32x4 t4 = *(const f32x4*)&th_lds[wv][qb * 32 + 8 * r + 4 * (lane >> 5)];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * r + c;
                    const float v = acc[qb][i];
                    gmax[qb][i] = fmaxf(gmax[qb][i], v);
                    passes += __ballot(v >= t4[c]) != 0 ? 1u : 0u;
                }
            }
    }
    float s = 0.f;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) s += gmax[qb][i];
    if (s == 1234.5f || passes == 0xFFFFFFFFu) sink[0] = 1u;
}

// LDS-DMA staging (global_load_lds_dwordx4: L2 -> LDS without VGPRs or ds_write instructions); the two window
// buffers are separate LDS objects, so the compiler can tell the fragment reads of one from the DMA into the other
template <int QB>
__global__ __launch_bounds__(256, 1) void k_qd(const u32x4* __restrict__ corpus, const u32x4* __restrict__ qfrag,
                                              long long n_tiles, int mode_unused, unsigned* __restrict__ sink) {
    constexpr int WQ = WIN * QB * 64;
    constexpr int PER = WQ / 256;
    __shared__ __attribute__((aligned(16))) u32x4 lb0[WQ];
    __shared__ __attribute__((aligned(16))) u32x4 lb1[WQ];
    __shared__ __attribute__((aligned(16))) float th_lds[4][QB * 32];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long W = (long long)gridDim.x * 4;
    const long long wr = (long long)wv * gridDim.x + blockIdx.x;
    const long long n_rounds = n_tiles / W;
    auto uni = [](long long v) -> long long {
        const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
        const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)((unsigned long long)v >> 32));
        return (long long)(((unsigned long long)hi << 32) | lo);
    };
    auto tile = [&](long long u) -> long long { return uni((u < n_rounds ? u : n_rounds - 1) * W + wr); };
    auto rsrc = [&](long long t) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)corpus + t * (S * 1024)), (short)0, S * 1024, 0x00020000);
    };
    const int voff = lane * 16;
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int kstep) -> u32x4 { return __builtin_amdgcn_raw_buffer_load_b128(r, voff, kstep * 1024, 2); };
    // this thread's staging source: chunk j of window w is qfrag[w * WQ + j * 256 + tid]
    const __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc((void*)qfrag, (short)0, S * QB * 1024, 0x00020000);
    auto stage = [&](int w, u32x4* buf) {
        int vo = tid * 16;
        asm volatile("" : "+v"(vo));  // (per call: keeps the offsets out of loop-invariant registers)
#pragma unroll
        for (int j = 0; j < PER; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (__attribute__((address_space(3))) void*)(buf + j * 256 + wv * 64),
                                                     16, vo, w * WQ * 16 + j * 4096, 0, 0);
    };
    u32x4 ra[WIN], rb[WIN];
    {
        const auto r0 = rsrc(tile(0));
#pragma unroll
        for (int i = 0; i < WIN; ++i) ra[i] = ld(r0, i);
#pragma unroll
        for (int i = 0; i < WIN; ++i) rb[i] = ld(r0, WIN + i);
    }
    stage(0, lb0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float gmax[QB][16];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) gmax[qb][i] = -1e30f;
    if (lane < QB * 32 / 2) {
        th_lds[wv][2 * lane] = __builtin_bit_cast(float, (unsigned)(0x7E000000u + lane));
        th_lds[wv][2 * lane + 1] = __builtin_bit_cast(float, (unsigned)(0x7E000001u + lane));
    }
    unsigned passes = 0;
    for (long long u = 0; u < n_rounds; ++u) {
        const auto rt = rsrc(tile(u)), rn = rsrc(tile(u + 1));
        f32x16 acc[QB];
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[qb][i] = 0.f;
#pragma unroll
        for (int w = 0; w < NWIN; ++w) {
            u32x4(&ring)[WIN] = (w & 1) ? rb : ra;
            if (w > 0 || u > 0) {
                // this wave's DMA for window w landed (the 16 ring refills of the previous window were issued
                // after it), then every wave's (barrier); every wave is also done reading the other buffer
                asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            stage((w + 1) % NWIN, (w & 1) ? lb0 : lb1);
            unsigned qoff = (unsigned)lane;
            asm volatile("" : "+v"(qoff));
            const u32x4* qs = ((w & 1) ? lb1 : lb0) + qoff;
            u32x4 qf[2][QB];
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) qf[0][qb] = qs[qb * 64];
#pragma unroll
            for (int i = 0; i < WIN; ++i) {
                if (i + 1 < WIN) {
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) qf[(i + 1) & 1][qb] = qs[((i + 1) * QB + qb) * 64];
                }
                const u32x4 x = ring[i];
                ring[i] = (w + 2 < NWIN) ? ld(rt, (w + 2) * WIN + i) : ld(rn, (w + 2 - NWIN) * WIN + i);
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) acc[qb] = mfma(qf[i & 1][qb], x, acc[qb]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                typedef float f32x4 __attribute__((ext_vector_type(4)));
                const f32x4 t4 = *(const f32x4*)&th_lds[wv][qb * 32 + 8 * r + 4 * (lane >> 5)];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * r + c;
                    const float v = acc[qb][i];
                    gmax[qb][i] = fmaxf(gmax[qb][i], v);
                    passes += __ballot(v >= t4[c]) != 0 ? 1u : 0u;
                }
            }
    }
    float s = 0.f;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) s += gmax[qb][i];
    if (s == 1234.5f || passes == 0xFFFFFFFFu) sink[0] = 1u;
}

// Two tiles per wave per window pass (window = 8 k-steps): every query fragment read from LDS feeds two MFMAs and
// each staged window serves eight tiles per workgroup instead of four -- half the staging and LDS reads per tile
template <int QB>
__global__ __launch_bounds__(256, 1) void k_qd2(const u32x4* __restrict__ corpus, const u32x4* __restrict__ qfrag,
                                               long long n_tiles, int mode_unused, unsigned* __restrict__ sink) {
    constexpr int WN = 8;              // k-steps per window
    constexpr int NW = S / WN;         // windows per tile
    constexpr int WQ = WN * QB * 64;   // u32x4 per window
    constexpr int PER = WQ / 256;
    __shared__ __attribute__((aligned(16))) u32x4 lb0[WQ];
    __shared__ __attribute__((aligned(16))) u32x4 lb1[WQ];
    __shared__ __attribute__((aligned(16))) float th_lds[4][QB * 32];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long W = (long long)gridDim.x * 4;
    const long long wr = (long long)wv * gridDim.x + blockIdx.x;
    const long long n_rounds = n_tiles / (2 * W);
    auto uni = [](long long v) -> long long {
        const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
        const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)((unsigned long long)v >> 32));
        return (long long)(((unsigned long long)hi << 32) | lo);
    };
    auto pair = [&](long long u) -> long long { return uni(2 * ((u < n_rounds ? u : n_rounds - 1) * W + wr)); };
    auto rsrc = [&](long long t) {  // two consecutive tiles
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)corpus + t * (S * 1024)), (short)0, 2 * S * 1024, 0x00020000);
    };
    const int voff = lane * 16;
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int chunk) -> u32x4 { return __builtin_amdgcn_raw_buffer_load_b128(r, voff, chunk * 1024, 2); };
    const __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc((void*)qfrag, (short)0, S * QB * 1024, 0x00020000);
    auto stage = [&](int w, u32x4* buf) {
        int vo = tid * 16;
        asm volatile("" : "+v"(vo));
#pragma unroll
        for (int j = 0; j < PER; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (__attribute__((address_space(3))) void*)(buf + j * 256 + wv * 64),
                                                     16, vo, w * WQ * 16 + j * 4096, 0, 0);
    };
    // ring slot i of a half: tile (i >> 3) of the pair, k-step (i & 7) of the window
    u32x4 ra[2 * WN], rb[2 * WN];
    {
        const auto r0 = rsrc(pair(0));
#pragma unroll
        for (int i = 0; i < 2 * WN; ++i) ra[i] = ld(r0, (i >> 3) * S + (i & 7));
#pragma unroll
        for (int i = 0; i < 2 * WN; ++i) rb[i] = ld(r0, (i >> 3) * S + WN + (i & 7));
    }
    stage(0, lb0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float gmax[QB][16];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) gmax[qb][i] = -1e30f;
    if (lane < QB * 32 / 2) {
        th_lds[wv][2 * lane] = __builtin_bit_cast(float, (unsigned)(0x7E000000u + lane));
        th_lds[wv][2 * lane + 1] = __builtin_bit_cast(float, (unsigned)(0x7E000001u + lane));
    }
    unsigned passes = 0;
    for (long long u = 0; u < n_rounds; ++u) {
        const auto rt = rsrc(pair(u)), rn = rsrc(pair(u + 1));
        f32x16 acc[2][QB];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[h][qb][i] = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            u32x4(&ring)[2 * WN] = (w & 1) ? rb : ra;
            if (w > 0 || u > 0) {
                asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            stage((w + 1) % NW, (w & 1) ? lb0 : lb1);
            unsigned qoff = (unsigned)lane;
            asm volatile("" : "+v"(qoff));
            const u32x4* qs = ((w & 1) ? lb1 : lb0) + qoff;
            u32x4 qf[2][QB];
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) qf[0][qb] = qs[qb * 64];
#pragma unroll
            for (int i = 0; i < WN; ++i) {
                if (i + 1 < WN) {
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) qf[(i + 1) & 1][qb] = qs[((i + 1) * QB + qb) * 64];
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const u32x4 x = ring[h * WN + i];
                    ring[h * WN + i] = (w + 2 < NW) ? ld(rt, h * S + (w + 2) * WN + i) : ld(rn, h * S + (w + 2 - NW) * WN + i);
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) acc[h][qb] = mfma(qf[i & 1][qb], x, acc[h][qb]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    typedef float f32x4 __attribute__((ext_vector_type(4)));
                    const f32x4 t4 = *(const f32x4*)&th_lds[wv][qb * 32 + 8 * r + 4 * (lane >> 5)];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const int i = 4 * r + c;
                        const float v = acc[h][qb][i];
                        gmax[qb][i] = fmaxf(gmax[qb][i], v);
                        passes += __ballot(v >= t4[c]) != 0 ? 1u : 0u;
                    }
                }
    }
    float s = 0.f;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) s += gmax[qb][i];
    if (s == 1234.5f || passes == 0xFFFFFFFFu) sink[0] = 1u;
}

// Eight waves (two per SIMD), one tile per wave, window = 8 k-steps: the same staging per tile as k_qd2 (eight
// tiles per staged window per workgroup) with half the registers per wave, so a wave's epilogue runs beside the
// other wave's MFMAs on its SIMD
template <int QB>
__global__ __launch_bounds__(512, 1) void k_qd8(const u32x4* __restrict__ corpus, const u32x4* __restrict__ qfrag,
                                               long long n_tiles, int mode_unused, unsigned* __restrict__ sink) {
    constexpr int WN = 8;
    constexpr int NW = S / WN;
    constexpr int WQ = WN * QB * 64;
    constexpr int PER = WQ / 512;
    __shared__ __attribute__((aligned(16))) u32x4 lb0[WQ];
    __shared__ __attribute__((aligned(16))) u32x4 lb1[WQ];
    __shared__ __attribute__((aligned(16))) float th_lds[QB * 32];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long W = (long long)gridDim.x * 8;
    const long long wr = (long long)wv * gridDim.x + blockIdx.x;
    const long long n_rounds = n_tiles / W;
    auto uni = [](long long v) -> long long {
        const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
        const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)((unsigned long long)v >> 32));
        return (long long)(((unsigned long long)hi << 32) | lo);
    };
    auto tile = [&](long long u) -> long long { return uni((u < n_rounds ? u : n_rounds - 1) * W + wr); };
    auto rsrc = [&](long long t) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)corpus + t * (S * 1024)), (short)0, S * 1024, 0x00020000);
    };
    const int voff = lane * 16;
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int chunk) -> u32x4 { return __builtin_amdgcn_raw_buffer_load_b128(r, voff, chunk * 1024, 2); };
    const __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc((void*)qfrag, (short)0, S * QB * 1024, 0x00020000);
    auto stage = [&](int w, u32x4* buf) {
        int vo = tid * 16;
        asm volatile("" : "+v"(vo));
#pragma unroll
        for (int j = 0; j < PER; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (__attribute__((address_space(3))) void*)(buf + j * 512 + wv * 64),
                                                     16, vo, w * WQ * 16 + j * 8192, 0, 0);
    };
    u32x4 ra[WN], rb[WN];
    {
        const auto r0 = rsrc(tile(0));
#pragma unroll
        for (int i = 0; i < WN; ++i) ra[i] = ld(r0, i);
#pragma unroll
        for (int i = 0; i < WN; ++i) rb[i] = ld(r0, WN + i);
    }
    stage(0, lb0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid < QB * 32) th_lds[tid] = __builtin_bit_cast(float, (unsigned)(0x7E000000u + tid));
    __syncthreads();
    float gmax[QB][16];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) gmax[qb][i] = -1e30f;
    unsigned passes = 0;
    for (long long u = 0; u < n_rounds; ++u) {
        const auto rt = rsrc(tile(u)), rn = rsrc(tile(u + 1));
        f32x16 acc[QB];
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[qb][i] = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            u32x4(&ring)[WN] = (w & 1) ? rb : ra;
            if (w > 0 || u > 0) {
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            stage((w + 1) % NW, (w & 1) ? lb0 : lb1);
            unsigned qoff = (unsigned)lane;
            asm volatile("" : "+v"(qoff));
            const u32x4* qs = ((w & 1) ? lb1 : lb0) + qoff;
            u32x4 qf[2][QB];
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) qf[0][qb] = qs[qb * 64];
#pragma unroll
            for (int i = 0; i < WN; ++i) {
                if (i + 1 < WN) {
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) qf[(i + 1) & 1][qb] = qs[((i + 1) * QB + qb) * 64];
                }
                const u32x4 x = ring[i];
                ring[i] = (w + 2 < NW) ? ld(rt, (w + 2) * WN + i) : ld(rn, (w + 2 - NW) * WN + i);
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) acc[qb] = mfma(qf[i & 1][qb], x, acc[qb]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                typedef float f32x4 __attribute__((ext_vector_type(4)));
                const f32x4 t4 = *(const f32x4*)&th_lds[qb * 32 + 8 * r + 4 * (lane >> 5)];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * r + c;
                    const float v = acc[qb][i];
                    gmax[qb][i] = fmaxf(gmax[qb][i], v);
                    passes += __ballot(v >= t4[c]) != 0 ? 1u : 0u;
                }
            }
    }
    float s = 0.f;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) s += gmax[qb][i];
    if (s == 1234.5f || passes == 0xFFFFFFFFu) sink[0] = 1u;
}

int main(int argc, char** argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 20.48;
    const long long tile_bytes = (long long)S * 1024;
    const long long n_tiles = (long long)(gb * 1e9) / tile_bytes;
    const long long bytes = n_tiles * tile_bytes;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int n_cu = prop.multiProcessorCount;
    u32x4 *corpus = nullptr, *qf = nullptr;
    unsigned* sink = nullptr;
    CHECK(hipMalloc(&corpus, bytes));
    CHECK(hipMalloc(&qf, (size_t)8 * S * 4 * 64 * 16));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(corpus, 0x11, bytes));
    CHECK(hipMemset(qf, 0x22, (size_t)8 * S * 4 * 64 * 16));
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int reps = 10;
    auto time = [&](auto kern, int qb, int cus, int mode) {
        const int lds = 2 * WIN * qb * 64 * 16;

        hipLaunchKernelGGL(kern, dim3(cus), dim3(256), 0, 0, corpus, qf, n_tiles, mode, sink);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(cus), dim3(256), 0, 0, corpus, qf, n_tiles, mode, sink);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double t = ms / reps;
        std::printf("{\"proto\": \"q%d windowed\", \"cus\": %d, \"mode\": %d, \"bytes\": %lld, \"ms\": %.4f, \"TBps\": %.4f, "
                    "\"qps_equiv\": %.0f}\n", qb * 32, cus, mode, bytes, t, bytes / (t * 1e-3) / 1e12, qb * 32 / (t * 1e-3));
        std::fflush(stdout);
    };
    auto time8 = [&](auto kern, int qb, int cus, int mode) {
        hipLaunchKernelGGL(kern, dim3(cus), dim3(512), 0, 0, corpus, qf, n_tiles, mode, sink);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(cus), dim3(512), 0, 0, corpus, qf, n_tiles, mode, sink);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double t = ms / reps;
        std::printf("{\"proto\": \"q%d 8 waves\", \"cus\": %d, \"mode\": %d, \"bytes\": %lld, \"ms\": %.4f, \"TBps\": %.4f, "
                    "\"qps_equiv\": %.0f}\n", qb * 32, cus, mode, bytes, t, bytes / (t * 1e-3) / 1e12, qb * 32 / (t * 1e-3));
        std::fflush(stdout);
    };
    const int only = argc > 2 ? atoi(argv[2]) : -1;  // one variant (profiling): 0..4 at all CUs
    for (int cus : {n_cu - 32, n_cu}) {
        if (only >= 0 && cus != n_cu) continue;
        if (only < 0 || only == 0) time(k_qd<4>, 4, cus, 1000);                // LDS-DMA staging
        if (only < 0 || only == 1) time(k_qd2<4>, 4, cus, 2000);               // + two tiles per wave
        if (only < 0 || only == 2) time(k_q<4, 12, 1>, 4, cus, 12);           // neither staging nor barriers
        if (only < 0 || only == 3) time8(k_qd8<4>, 4, cus, 3000);              // eight waves, one tile each
    }
    CHECK(hipFree(corpus));
    CHECK(hipFree(qf));
    CHECK(hipFree(sink));
    return 0;
}
