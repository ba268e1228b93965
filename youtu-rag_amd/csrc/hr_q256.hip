// hr_q256.hip -- the 256-query FILTER: one HBM read of every corpus tile for four 64-query groups.
//
// A batch of 129-256 queries was two launches of the 128-query FILTER (hr_wide.hip): two corpus passes, each at
// about half the MFMA pipe (its eight 256-register waves are issue-bound).  Here the MFMA work of all 256 queries
// rides on ONE pass -- 4x the MFMAs per byte of the 64-query k_scan, so a launch is about as much matrix work as
// streaming time (10M x 1024: 2.6 ms of MFMA at the dense peak against 2.9 ms of HBM at the read ceiling):
//  * one workgroup per CU, 4 waves, ONE wave per SIMD with the whole 512-register file: the 2 x 8 x 16 = 256
//    accumulators of two tiles against 8 blocks of 32 queries sit in AGPRs, a 16-deep corpus ring per tile
//    (32 KiB in flight per wave) and the query fragments in VGPRs -- a single wave keeps its SIMD's matrix pipe
//    fed (v_mfma_f32_32x32x16 issues back to back at 32 cycles, MI355X_MICROARCH.md) with 16 independent MFMAs
//    per k-step;
//  * two tiles per wave per round: every query fragment read from LDS serves two MFMAs, and the workgroup's 8 tiles
//    per round share one staging of the query windows;
//  * the queries' fragments (4 x S KiB x 2: 512 KiB at D = 1024) stream through LDS in windows of 2 k-steps
//    (16 KiB), staged by LDS-DMA (buffer_load ... lds: no registers) 8 windows ahead into a ring of 9 buffers
//    (144 KiB).  LDS-DMA completions count in vmcnt, in order with the corpus ring's loads, so a window staged
//    only one window ahead would make every wait on it drain the corpus ring too; staged as far ahead as the ring
//    reaches, the wait that admits it retires only loads already consumed;
//  * the A fragments are read with inline-asm ds_read_b128 and explicit lgkmcnt waits (one k-step ahead), so the
//    compiler's conservative LDS-DMA tracking inserts no vmcnt drain in front of them;
//  * thresholds per query in LDS (shared by the four waves); group maxima raised in the global table with one
//    fire-and-forget atomicMax per passing score (rare: only scores at or above their threshold can raise the
//    minimum over the groups); a refresh re-reads the global keys of the wave's 64-query group (a part of them per
//    round, loaded a round ahead);
//  * candidates go to k_scan's private per-(query group, wave) regions, so k_select reads them unchanged.
// Exactness: the same invariant as the 128-query FILTER -- every row at or above a query's final threshold was
// appended when scanned (thresholds only grow), and each group key is the score of an appended (or SAMPLE) row.
//  * fp32 rows (the drop-in store's default dtype, faiss_store.py:98; Chroma float32): a k-step's chunk is 2 KiB, two
//    16-byte loads per lane, rounded to the MFMA type on use (as k_scan's XFrag<F32> and the 128-query FILTER), so
//    the ring holds half the k-steps in the same registers -- the same 16 KiB in flight per wave -- and the query
//    windows are still staged 8 k-steps ahead.
// Scope: bf16 / f16 / fp32 rows, D = 256 / 512 / 768 / 1024, one row part (k <= 16), no tile list; cosine / ip / l2.
#include "hr_internal.hpp"
#include "hr_kernels.hpp"

namespace hr {

// HR_Q256_DIAG (timing builds only -- results are WRONG with any bit set): 1 no query-window staging in the loop,
// 2 no corpus ring loads, 4 no per-window barrier, 8 no MFMA (operands consumed by a cheap VALU op) and no
// epilogue, 16 no epilogue, 32 no refresh after round 2
#ifndef HR_Q256_DIAG
#define HR_Q256_DIAG 0
#endif
// A/B knobs (results identical): LDS prefetch distance in (k-step, block) pairs, a wave's two tiles adjacent (1;
// +0.7 % against W apart (0) at 10M x 1024, B = 256), the corpus loads' cache policy (2 = nt)
#ifndef HR_Q256_PF
#define HR_Q256_PF 2
#endif
#ifndef HR_Q256_ADJ
#define HR_Q256_ADJ 1
#endif
#ifndef HR_Q256_CLOCK  // diagnostic build: the in-kernel clock (shader cycles / 100 MHz ticks around the round loop)
#define HR_Q256_CLOCK 0
#endif
#ifndef HR_Q256_STAMPS  // diagnostic build: per-wave cycle shares of the round's phases, printed
#define HR_Q256_STAMPS 0
#endif
// the 16x16x32 form (k_filter_q256_m16) for 16-bit rows at D = 512..1024 (0: the 32x32x16 k_filter_q256 for them);
// its A prefetch distance in 16-query blocks and the register rotation that holds them (2 / 4: +0.5-1 %, 6 / 8 kept)
#ifndef HR_Q256_MFMA16
#define HR_Q256_MFMA16 1
#endif
#ifndef HR_Q256_PF16
#define HR_Q256_PF16 6
#endif
#ifndef HR_Q256_SLOTS16
#define HR_Q256_SLOTS16 8
#endif
#ifndef HR_Q256_VMEXACT
#define HR_Q256_VMEXACT 1
#endif
#ifndef HR_Q256_NT
#define HR_Q256_NT 2
#endif

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kQT = 256;              // threads per workgroup: 4 waves, one per SIMD
constexpr int kWin = 2;               // k-steps per query window
constexpr int kWQ = kWin * 8 * 64;    // u32x4 per window buffer: [k-step][block][lane]
constexpr int kDma = kWQ / kQT;       // LDS-DMA instructions per thread per window
// corpus ring depth in k-steps per tile: 8 for 16-bit rows (16 KiB in flight per wave; 16 measured within 1.5 % at
// D = 1024 and its registers are worth more as the partial refresh's: a refresh that drains the ring costs 7 %), 16
// at D = 256.  fp32 rows: 8 k-steps too, twice the registers (128) and 32 KiB in flight per wave -- a k-step's MFMA
// time covers twice the bytes, and 4 k-steps (16 KiB) left the pass latency-bound at 4.6 TB/s; the epilogue then
// reads its thresholds one block at a time to stay within the VGPRs
constexpr int ring_for(int S, int LPC) { return LPC == 2 ? 8 : (S == 16 ? 16 : 8); }
template <int S_, int LPC>
struct Q256Geom {
    static constexpr int kRing = ring_for(S_, LPC);
    // windows a window is staged ahead of its first use: 8 k-steps (the 16-bit ring's reach), 8 windows at D = 256
    // for 16-bit rows (4 for fp32: the wait's count below must fit vmcnt)
    static constexpr int kLook = S_ == 16 ? kRing / kWin : 8 / kWin;
    // a workgroup barrier every kBar windows: with kLook + kBar buffers the DMA at window w refills the buffer of
    // window w - kBar, which every wave has left by the last barrier (kBar = 2: half the barriers; one per window at
    // D = 256, whose 16-deep ring leaves no LDS for two spare buffers)
    static constexpr int kBar = S_ == 16 ? 1 : 2;
    static constexpr int kNB = kLook + kBar;  // window buffers
    // vmcnt at a barrier window that retires this wave's DMAs of the next kBar windows (the windows read before the
    // next barrier).  The last of them, window w + kBar - 1, was staged at the start of window w + kBar - 1 - kLook,
    // ahead of that window's ring loads: younger than it are the ring loads of kLook - kBar + 1 windows (2 tiles x
    // kWin k-steps x LPC loads each) and the DMAs of kLook - kBar windows (anything else issued since -- keys,
    // appends, maxima -- only adds younger operations).  HR_Q256_VMEXACT 0: the earlier count, one window of each
    // fewer, which also retired ring loads a window before their use.
    static constexpr int kVmNext = HR_Q256_VMEXACT ? (kLook - kBar + 1) * 2 * kWin * LPC + (kLook - kBar) * kDma
                                                   : (kLook - kBar) * 2 * kWin * LPC + (kLook - kBar - 1) * kDma;
    static_assert(kVmNext <= 63, "vmcnt field");
};

// f(std::integral_constant<int, 0>{}) ... f(std::integral_constant<int, N - 1>{}): loop indices usable as constants
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}

template <int OFF>
__device__ __forceinline__ u32x4 lds_read(uint32_t base) {  // ds_read_b128 base + OFF, not tracked by the compiler
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF));
    return v;
}

// four ds_read_b128 at base + OFF + 32 r and their wait in ONE asm statement: with the wait in a separate statement
// the compiler may copy an output register between the two (it takes the asm's outputs as ready at once) and the
// copy reads the register before the load has landed
template <int OFF>
__device__ __forceinline__ void lds_read4_wait(uint32_t base, u32x4 (&t)[4]) {
    asm volatile(
        "ds_read_b128 %0, %4 offset:%5\n\t"
        "ds_read_b128 %1, %4 offset:%6\n\t"
        "ds_read_b128 %2, %4 offset:%7\n\t"
        "ds_read_b128 %3, %4 offset:%8\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3])
        : "v"(base), "n"(OFF), "n"(OFF + 32), "n"(OFF + 64), "n"(OFF + 96));
}

// sixteen ds_read_b128 at base + OFF + 32 r (four blocks' thresholds) and ONE wait
template <int OFF>
__device__ __forceinline__ void lds_read16_wait(uint32_t base, u32x4 (&t)[16]) {
    asm volatile(
        "ds_read_b128 %0, %16 offset:%17\n\tds_read_b128 %1, %16 offset:%18\n\tds_read_b128 %2, %16 offset:%19\n\t"
        "ds_read_b128 %3, %16 offset:%20\n\tds_read_b128 %4, %16 offset:%21\n\tds_read_b128 %5, %16 offset:%22\n\t"
        "ds_read_b128 %6, %16 offset:%23\n\tds_read_b128 %7, %16 offset:%24\n\tds_read_b128 %8, %16 offset:%25\n\t"
        "ds_read_b128 %9, %16 offset:%26\n\tds_read_b128 %10, %16 offset:%27\n\tds_read_b128 %11, %16 offset:%28\n\t"
        "ds_read_b128 %12, %16 offset:%29\n\tds_read_b128 %13, %16 offset:%30\n\tds_read_b128 %14, %16 offset:%31\n\t"
        "ds_read_b128 %15, %16 offset:%32\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7]),
          "=&v"(t[8]), "=&v"(t[9]), "=&v"(t[10]), "=&v"(t[11]), "=&v"(t[12]), "=&v"(t[13]), "=&v"(t[14]), "=&v"(t[15])
        : "v"(base), "n"(OFF), "n"(OFF + 32), "n"(OFF + 64), "n"(OFF + 96), "n"(OFF + 128), "n"(OFF + 160),
          "n"(OFF + 192), "n"(OFF + 224), "n"(OFF + 256), "n"(OFF + 288), "n"(OFF + 320), "n"(OFF + 352), "n"(OFF + 384),
          "n"(OFF + 416), "n"(OFF + 448), "n"(OFF + 480));
}

// eight ds_read_b32 at base + 8 j and ONE wait (the thresholds of queries 2 j apart)
__device__ __forceinline__ void lds_read8_stride8_wait(uint32_t base, float (&t)[8]) {
    asm volatile(
        "ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:8\n\tds_read_b32 %2, %8 offset:16\n\t"
        "ds_read_b32 %3, %8 offset:24\n\tds_read_b32 %4, %8 offset:32\n\tds_read_b32 %5, %8 offset:40\n\t"
        "ds_read_b32 %6, %8 offset:48\n\tds_read_b32 %7, %8 offset:56\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7])
        : "v"(base)
        : "memory");
}

template <int OFF>
__device__ __forceinline__ void lds_write_f32(uint32_t addr, float v) {  // ds_write_b32, not tracked
    asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(addr), "v"(v), "n"(OFF) : "memory");
}

// one accumulator register read out of its AGPR at this point of the program (volatile: the register allocator
// would otherwise copy whole 16-register accumulators to VGPRs early and spill them)
template <int I>
__device__ __forceinline__ float acc_read(const f32x16& v) {
    float r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(v[I]));
    return r;
}

template <int OFF>
__device__ __forceinline__ float lds_read_f32o(uint32_t addr) {  // ds_read_b32 at addr + OFF and its wait
    float v;
    asm volatile("ds_read_b32 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
    return v;
}

__device__ __forceinline__ float lds_read_f32(uint32_t addr) {  // ds_read_b32 and its wait, not tracked
    float v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

#if HR_Q256_STAMPS
__device__ __forceinline__ uint64_t q256_stamp() {  // (diagnostic builds only: cycle shares, never run times)
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define HR_STAMP(var) const uint64_t var = q256_stamp()
#else
#define HR_STAMP(var)
#endif

template <int MT, int DT, int S_>
__global__ __launch_bounds__(kQT, 1) void k_filter_q256(ScanArgs a) {
    constexpr int LPC = DT == F32 ? 2 : 1;  // 16-byte loads per lane per k-step chunk
    using Geom = Q256Geom<S_, LPC>;
    constexpr int kRing = Geom::kRing, kLook = Geom::kLook, kNB = Geom::kNB;
    constexpr int kVmNext = Geom::kVmNext, kBar = Geom::kBar;
    static_assert(S_ % kRing == 0 && S_ % kWin == 0, "tile depth");
    __shared__ __attribute__((aligned(16))) u32x4 qw[kNB * kWQ];
    __shared__ __attribute__((aligned(16))) float th_lds[256];
    constexpr int NQ = S_ / kRing;   // ring spans per tile

    const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, g = lane & 31;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t W = (int64_t)gridDim.x * 4;  // waves (candidate regions per query group)
    const int64_t W2 = 2 * W;                  // tiles per round
    const int64_t wr = (int64_t)wv * gridDim.x + blockIdx.x;
    const int64_t n_tiles = a.n_units;
    const int64_t rounds = (n_tiles + W2 - 1) / W2;
    const int64_t full_rounds = n_tiles / W2;
    // round u: tiles [u W2, (u + 1) W2); wave wr takes u W2 + pos and u W2 + W + pos, pos rotated by a hash of u on
    // full rounds (as k_scan / the 128-query FILTER: a period in the rows must not land in the same few waves)
    auto tile_of = [&](int64_t u, int which) -> int64_t {
        if (u >= rounds) return -1;
        int64_t pos = wr;
        if (HR_ROTATE_ROUNDS && u < full_rounds) {
            pos += (int64_t)((uint32_t)((uint64_t)u * 2654435761ull) % (uint32_t)W);
            if (pos >= W) pos -= W;
        }
        const int64_t t = HR_Q256_ADJ ? u * W2 + 2 * pos + which : u * W2 + which * W + pos;
        return wave_uniform(t < n_tiles ? t : -1);
    };
    auto rsrc = [&](int64_t t) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(a.rows + (t < 0 ? 0 : t) * (S_ * 1024 * LPC)), (short)0,
                                                 t < 0 ? 0 : S_ * 1024 * LPC, 0x00020000);
    };
    const int voff = lane * 16;
    // ring slot i (k-step i of a span) holds LPC 16-byte loads: ring[i * LPC + l]
    auto ld = [&](u32x4* ring, int i, __amdgpu_buffer_rsrc_t r, int ks) {
#pragma unroll
        for (int l = 0; l < LPC; ++l)
            ring[i * LPC + l] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, ks * 1024 * LPC + l * 1024, HR_Q256_NT);
    };
    auto xfrag = [&](const u32x4* ring, int i) -> u32x4 {  // the MFMA B operand of ring slot i
        if constexpr (LPC == 1) {
            return ring[i];
        } else {  // fp32: eight elements rounded to the MFMA type (RNE, as k_scan's XFrag<F32>)
            typedef float f32x8 __attribute__((ext_vector_type(8)));
            // pinned to the point of use: left to itself the scheduler converts each load right after issuing it
            // (half the registers while in flight) and so waits for it there -- vmcnt(0) every k-step, no ring
            u32x4 r0 = ring[2 * i], r1 = ring[2 * i + 1];
            asm volatile("" : "+v"(r0), "+v"(r1));
            const f32x8 f = __builtin_shufflevector(__builtin_bit_cast(f32x4, r0), __builtin_bit_cast(f32x4, r1), 0, 1, 2,
                                                    3, 4, 5, 6, 7);
            if constexpr (MT == BF16) return __builtin_bit_cast(u32x4, __builtin_convertvector(f, bf16x8));
            else return __builtin_bit_cast(u32x4, __builtin_convertvector(f, f16x8));
        }
    };
    // query windows: window gw holds k-steps (gw kWin) mod S of every block; qfrag = [group 4][S][2 blocks][64][16 B]
    const __amdgpu_buffer_rsrc_t qr =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.qfrag, (short)0, 4 * S_ * 2048, 0x00020000);
    const uint32_t qw_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)qw;
    auto stage = [&](int bi, int s0) {  // window starting at k-step s0 (of the tile) into buffer bi
        u32x4* buf = qw + bi * kWQ;
#pragma unroll
        for (int j = 0; j < kDma; ++j) {
            const int i = j >> 1, blk = (j & 1) * 4 + wv;  // chunk j * 256 + wv * 64 + lane of the window
            const int soff = (((blk >> 1) * S_ + s0 + i) * 2 + (blk & 1)) * 1024;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (__attribute__((address_space(3))) void*)(buf + j * 256 + wv * 64),
                                                     16, voff, soff, 0, 0);
        }
    };
    // the window buffer bi's base for this lane (byte address in LDS); block blk of k-step i sits at + (i 8 + blk) KiB
    const uint32_t lane_addr = qw_base + (uint32_t)lane * 16u;
    auto qbase = [&](int bi) -> uint32_t { return lane_addr + (uint32_t)(bi * kWQ * 16); };
    // thresholds: th_lds[q] (this lane's half adds 4 queries)
    const uint32_t th_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)th_lds;
    const uint32_t th_lane = th_base + (uint32_t)half * 16u;

    // ---- thresholds: this wave's 64-query group from the global keys (min over the 32 groups)
    // (register-light: the 32 key loads are buffer loads at SGPR offsets from one lane offset and the 32 threshold
    // updates use immediate LDS offsets -- 64-bit addresses per key were hoisted out of the round loop and spilled)
    const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc((void*)a.mkeys, (short)0, kQT * 32 * 4, 0x00020000);
    const uint32_t key_lane = (uint32_t)(((64 * wv + half) * 32 + g) * 4);  // key (query 64 wv + half, group g)
    const uint32_t th_q = th_base + (uint32_t)(64 * wv + half) * 4u;        // threshold of query 64 wv + half
    auto refresh = [&]() {
        uint32_t key[32];
        static_for<32>([&](auto J_) {  // query 64 wv + 2 j + half; sc1 = the agent-coherent load of an atomic
            constexpr int j = decltype(J_)::value;
            key[j] = __builtin_amdgcn_raw_buffer_load_b32(kr, key_lane, j * 256, 16);
        });
        static_for<32>([&](auto J_) {
            constexpr int j = decltype(J_)::value;
            const float f = half_min32(key2f(key[j] > HR_KEY_NEG_INF ? key[j] : HR_KEY_NEG_INF));
            // (every lane of the half holds the minimum: no branch)
            lds_write_f32<8 * j>(th_q, fmaxf(lds_read_f32o<8 * j>(th_q), f));
        });
    };
    // partial refresh: the keys of 2 kKR of the wave's 64 queries (part p), loaded at the START of a round into kKR
    // registers and applied after its epilogue -- their wait then retires only loads issued a round earlier, where a
    // refresh that loads and applies at once waits behind the whole corpus ring (a drain per refresh: 7 % of the
    // launch).  A quarter per round: each query every 4 rounds.
    constexpr int kKR = 8;
    constexpr int kParts = 32 / kKR;
    uint32_t qkey[kKR];
    auto part_load = [&](int p) {
        static_for<kKR>([&](auto J_) {  // query 64 wv + 2 kKR p + 2 j + half, group g
            constexpr int j = decltype(J_)::value;
            qkey[j] = __builtin_amdgcn_raw_buffer_load_b32(kr, key_lane, p * (kKR * 256) + j * 256, 16);
        });
    };
    static_assert(kKR == 8, "lds_read8_stride8_wait");
    auto part_apply = [&](int p) {  // (eight reductions interleaved step by step, one LDS round trip, eight writes)
        const uint32_t base = th_q + (uint32_t)p * (kKR * 8u);
        uint32_t m[kKR];  // order-preserving keys: the minimum over the half's 32 groups in integer compares
        static_for<kKR>([&](auto J_) {
            constexpr int j = decltype(J_)::value;
            m[j] = qkey[j] > HR_KEY_NEG_INF ? qkey[j] : HR_KEY_NEG_INF;
        });
        auto step = [&](auto CTRL_) {
            static_for<kKR>([&](auto J_) {
                constexpr int j = decltype(J_)::value;
                m[j] = min(m[j], dpp_u32<decltype(CTRL_)::value>(m[j]));
            });
        };
        step(std::integral_constant<int, 0xB1>{});   // quad_perm 1,0,3,2
        step(std::integral_constant<int, 0x4E>{});   // quad_perm 2,3,0,1
        step(std::integral_constant<int, 0x141>{});  // row_half_mirror
        step(std::integral_constant<int, 0x140>{});  // row_mirror
        float t[kKR];
        lds_read8_stride8_wait(base, t);
        static_for<kKR>([&](auto J_) {  // lane l with l ^ 16 (v_permlane16_swap; no LDS swizzle and its wait)
            constexpr int j = decltype(J_)::value;
            const auto r = __builtin_amdgcn_permlane16_swap(m[j], m[j], false, false);
            const uint32_t x = r[0], y = r[1];  // (components copied out first: see the bit_cast note in the epilogue)
            lds_write_f32<8 * j>(base, fmaxf(t[j], key2f(min(x, y))));
        });
    };
    th_lds[tid] = a.floor_q[tid];  // (the floors once: thresholds only grow; kQT = 256 queries)
    __syncthreads();
    refresh();

    // ---- prologue: the first kLook windows and the first ring of both tiles of round 0
    u32x4 ra[kRing * LPC], rb[kRing * LPC];
    for (int w = 0; w < kLook; ++w) stage(w, (w * kWin) % S_);  // (window w in buffer w)
    {
        const auto r0 = rsrc(tile_of(0, 0)), r1 = rsrc(tile_of(0, 1));
#pragma unroll
        for (int i = 0; i < kRing; ++i) {
            ld(ra, i, r0, i);
            ld(rb, i, r1, i);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    uint32_t mycnt[4] = {0u, 0u, 0u, 0u};  // lane q: candidates of query q of each 64-query group
    // a passing block's registers one by one (scores parked in this wave's LDS slot): group maxima raised with one
    // fire-and-forget atomicMax per passing score, the candidates appended to the group's private region
    // a passing block's registers (the set bits of regs, one per register holding a passing score), scores and
    // thresholds in registers -- read at a wave-uniform dynamic index (M0-relative register moves, no memory): group
    // maxima raised with one fire-and-forget atomicMax per passing score, candidates appended to the group's region
    auto walk_block = [&](int b, bool ok, uint32_t row, uint32_t& cnt, const f32x16& V, const f32x16& TH, uint32_t regs) {
        const int gq = b >> 1;
        float2* const reg = a.pbuf + ((gq * W + wr) * 64) * a.capw;
        while (regs) {
            const int i = __builtin_amdgcn_readfirstlane(__builtin_ctz(regs));
            regs &= regs - 1u;
            const float v = V[i];
            const int qm = (b & 1) * 32 + (i & 3) + 8 * (i >> 2);  // query (within the group) of half 0
            const bool pass = ok && v >= TH[i];
            const uint64_t msk = __ballot(pass);
            if (pass) atomicMax(a.mkeys + (int64_t)(gq * 64 + qm + 4 * half) * 32 + g, f2key(v));
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const uint32_t mh = (uint32_t)(msk >> (32 * hh));
                if (!mh) continue;
                const int ql = qm + 4 * hh;
                const uint32_t basepos = (uint32_t)__builtin_amdgcn_readlane((int)cnt, ql);
                if (pass && half == hh) {
                    const uint32_t pos = basepos + __builtin_popcount(mh & ((1u << g) - 1u));
                    if (pos < (uint32_t)a.capw) reg[ql * a.capw + pos] = make_float2(v, __builtin_bit_cast(float, row));
                }
                cnt += (lane == ql) ? (uint32_t)__builtin_popcount(mh) : 0u;
            }
        }
    };
    auto allow_word = [&](int64_t t) -> uint32_t {
        if (t < 0) return 0u;
        uint32_t w0 = scalar_word(a.live, t);
        if (a.mask) w0 &= scalar_word(a.mask, t);
        return w0;
    };
    // A fragments stream in (k-step, block) pairs -- pair p = 8 k + b of the running k-step count -- read kPf pairs
    // ahead into a 4-slot rotation (16 VGPRs instead of a whole k-step's 64): the two MFMAs of a pair (64 cycles)
    // cover the LDS latency of the reads behind it
    constexpr int kPf = HR_Q256_PF;
    static_assert(kPf >= 1 && kPf <= 3, "prefetch distance");
    constexpr int kSlots = 4;  // (a power of two dividing the 128 pairs of a span: the rotation runs on across spans)
    u32x4 pf[kSlots];
    static_for<kPf>([&](auto P_) { pf[decltype(P_)::value] = lds_read<decltype(P_)::value * 1024>(qbase(0)); });
    int wb = 0;  // buffer of the current window (window gw lives in buffer gw mod kNB)
    uint32_t qcur = qbase(0), qnext = qbase(1);  // this lane's address in the current / next window's buffer

    uint32_t dsink = 0;  // (HR_Q256_DIAG & 8 timing builds only)
#if HR_Q256_STAMPS
    uint64_t c_loop = 0, c_wait = 0, c_epi = 0, c_ref = 0;
    uint32_t c_blocks = 0, c_regs = 0;  // passing tile-blocks and walked registers
#endif
#if HR_Q256_CLOCK
    // (MI355X_MICROARCH.md "DVFS give-back" item 6: clock = d(s_memtime) / d(s_memrealtime) x 100 MHz; the values go
    // to printf only, never to an output)
    const uint64_t clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
    for (int64_t u = 0; u < rounds; ++u) {
        HR_STAMP(s_r0);
        if (u >= 2 && !(HR_Q256_DIAG & 32)) part_load((int)(u % kParts));
        const int64_t tA = tile_of(u, 0), tB = tile_of(u, 1);
        const int64_t nA = tile_of(u + 1, 0), nB = tile_of(u + 1, 1);
        const uint32_t allowA = allow_word(tA), allowB = allow_word(tB);
        // (euclidean: the rows' |x|^2 loaded now, ahead of this round's ring refills -- a load issued in the epilogue
        // would be the youngest in vmcnt and its wait would drain the whole ring)
        const float xsA = (a.xnorm && tA >= 0) ? a.xnorm[tA * 32 + slot_row(tA, g)] : 0.0f;
        const float xsB = (a.xnorm && tB >= 0) ? a.xnorm[tB * 32 + slot_row(tB, g)] : 0.0f;
        // (every index into acc is a compile-time constant -- static_for, never a loop variable -- so the array is
        // promoted to registers from the start: a runtime index, even one unrolling later resolves, keeps it a stack
        // object that the epilogue reads back from scratch)
        f32x16 acc[2][8];
        static_for<2>([&](auto T_) {
            static_for<8>([&](auto B_) { acc[decltype(T_)::value][decltype(B_)::value] = f32x16{}; });
        });
#pragma unroll
        for (int qs = 0; qs < NQ; ++qs) {
            const bool last = qs + 1 == NQ;
            const auto sA = rsrc(last ? nA : tA), sB = rsrc(last ? nB : tB);
            const int kb = last ? 0 : (qs + 1) * kRing;
            static_for<kRing>([&](auto I_) {
                constexpr int i = decltype(I_)::value;
                if constexpr (i % kWin == 0) {
                    if (i > 0 || qs > 0 || u > 0) wb = wb + 1 == kNB ? 0 : wb + 1;
                    // (windows per span and per round are even, so the span-local parity is the global one)
                    if constexpr ((i / kWin) % kBar == 0) {
                        // this wave's DMAs of the next kBar windows have landed; the barrier makes every wave's
                        // visible and retires every read of the buffers the DMAs of the next kBar windows refill
                        HR_STAMP(s_w0);
                        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kVmNext) : "memory");
                        if (!(HR_Q256_DIAG & 4)) __builtin_amdgcn_s_barrier();
#if HR_Q256_STAMPS
                        HR_STAMP(s_w1);
                        c_wait += s_w1 - s_w0;
#endif
                    }
                    // the window kLook ahead goes into the buffer of window gw - kBar ((wb + kLook) mod kNB)
                    if (!(HR_Q256_DIAG & 1)) stage(wb >= kBar ? wb - kBar : wb - kBar + kNB, (qs * kRing + i + kLook * kWin) % S_);
                    qcur = qbase(wb);
                    qnext = qbase(wb + 1 == kNB ? 0 : wb + 1);
                }
                const u32x4 xa = xfrag(ra, i), xb = xfrag(rb, i);
                if (!(HR_Q256_DIAG & 2)) {
                    ld(ra, i, sA, kb + i);
                    ld(rb, i, sB, kb + i);
                } else {  // (timing build: the ring registers stay live without loads)
                    ra[i * LPC] ^= xb;
                    rb[i * LPC] ^= xa;
                }
                static_for<8>([&](auto B_) {
                    constexpr int b = decltype(B_)::value;
                    constexpr int p = i * 8 + b;  // pair within the span (slot p & 3: 128 pairs per span)
                    constexpr int pn = p + kPf;   // the pair read now, kPf ahead (possibly in the next window / span)
                    constexpr int kn = pn >> 3;   // its k-step within the span (kRing: the next span's first)
                    const uint32_t base = (kn / kWin) != (i / kWin) ? qnext : qcur;
                    pf[pn % kSlots] = lds_read<((kn % kWin) * 8 + (pn & 7)) * 1024>(base);
                    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(pf[p % kSlots]) : "n"(kPf));
                    if constexpr ((HR_Q256_DIAG & 8) != 0) {  // (timing build: operands consumed, no MFMA)
                        dsink ^= pf[p % kSlots].x ^ pf[p % kSlots].w ^ xa.x ^ xb.y;
                    } else {
                        acc[0][b] = mfma32<MT>(pf[p % kSlots], xa, acc[0][b]);
                        acc[1][b] = mfma32<MT>(pf[p % kSlots], xb, acc[1][b]);
                    }
                });
            });
        }

        if constexpr ((HR_Q256_DIAG & 16) != 0) {  // (timing build: no epilogue, the accumulators kept live)
            float z = 0.0f;
            static_for<2>([&](auto T_) {
                static_for<8>([&](auto B_) { z += acc_read<0>(acc[decltype(T_)::value][decltype(B_)::value]); });
            });
            mycnt[0] += __builtin_bit_cast(uint32_t, z) + allowA + allowB;
        }
        HR_STAMP(s_r1);
        // ---- epilogue, block by block: one read of the block's 16 thresholds (inline asm: a compiler-visible LDS read
        // would be fenced behind every LDS-DMA in flight -- vmcnt(0), the whole corpus ring) serves both tiles; per
        // tile the 16 scores against them and one ballot of "any register passes".  A passing block (rare after the
        // first rounds) gets a 16-bit mask of its passing registers and a rolled loop over the set bits reads score and
        // threshold at a dynamic register index, so the unrolled part stays small in code.  Inner product / cosine compare the
        // accumulators themselves; euclidean forms 2 q.x - |x|^2 first (as k_scan).  Every accumulator read has
        // constant indices (static_for).
        auto epilogue = [&](auto EUC_) {
            constexpr bool EUC = decltype(EUC_)::value;
            const int rgA = slot_row(tA < 0 ? 0 : tA, g), rgB = slot_row(tB < 0 ? 0 : tB, g);
            const bool okA = (allowA >> rgA) & 1u, okB = (allowB >> rgB) & 1u;
            const uint32_t rowA = (uint32_t)(tA * 32 + rgA), rowB = (uint32_t)(tB * 32 + rgB);
            // thresholds four blocks at a time (one LDS round trip per four blocks; one per block at D = 256 and for
            // fp32 rows, whose rings leave no room for 64 more registers)
            constexpr int kTB = (S_ == 16 || LPC == 2) ? 1 : 4;
            u32x4 t4b[4 * kTB];
            static_for<8>([&](auto B_) {
                constexpr int b = decltype(B_)::value;
                if constexpr (b % kTB == 0) {
                    if constexpr (kTB == 4) lds_read16_wait<b * 128>(th_lane, t4b);
                    else lds_read4_wait<b * 128>(th_lane, *(u32x4(*)[4])t4b);
                }
                // (bit_cast the whole vector, then index: this clang lowers a bit_cast of ONE component, t4[r][c], to
                // component 0 for every c, and then loads only that dword)
                f32x4 tf[4];
                static_for<4>([&](auto R_) {
                    tf[decltype(R_)::value] = __builtin_bit_cast(f32x4, t4b[(b % kTB) * 4 + decltype(R_)::value]);
                });
                // both tiles' scores and the max of (score - threshold) over the 16 registers first -- independent
                // work and a reduction tree, not a chain of dependent maxima -- then the two ballots
                f32x16 V[2], TH;
                float d[2];
                static_for<16>([&](auto I_) {
                    constexpr int i = decltype(I_)::value;
                    TH[i] = tf[i >> 2][i & 3];
                });
                static_for<2>([&](auto T_) {
                    constexpr int T = decltype(T_)::value;
                    float e[16];
                    static_for<16>([&](auto I_) {
                        constexpr int i = decltype(I_)::value;
                        const float r = acc_read<i>(acc[T][b]);
                        V[T][i] = EUC ? __builtin_fmaf(2.0f, r, -(T ? xsB : xsA)) : r;
                        e[i] = V[T][i] - TH[i];
                    });
                    static_for<8>([&](auto I_) { e[decltype(I_)::value] = fmaxf(e[decltype(I_)::value], e[decltype(I_)::value + 8]); });
                    static_for<4>([&](auto I_) { e[decltype(I_)::value] = fmaxf(e[decltype(I_)::value], e[decltype(I_)::value + 4]); });
                    static_for<2>([&](auto I_) { e[decltype(I_)::value] = fmaxf(e[decltype(I_)::value], e[decltype(I_)::value + 2]); });
                    d[T] = fmaxf(e[0], e[1]);
                });
                static_for<2>([&](auto T_) {
                    constexpr int T = decltype(T_)::value;
                    const bool ok = T ? okB : okA;
                    if (!__ballot(ok && d[T] >= 0.0f)) return;
                    uint32_t regs = 0;  // the registers holding a passing score (wave-uniform bits)
                    static_for<16>([&](auto I_) {
                        constexpr int i = decltype(I_)::value;
                        regs |= (__ballot(ok && V[T][i] >= TH[i]) != 0 ? 1u : 0u) << i;
                    });
                    walk_block(b, ok, T ? rowB : rowA, mycnt[b >> 1], V[T], TH, regs);
#if HR_Q256_STAMPS
                    c_blocks += 1;
                    c_regs += __builtin_popcount(regs);
#endif
                });
            });
        };
        if constexpr ((HR_Q256_DIAG & 24) == 0) {
            if (a.xnorm) epilogue(std::true_type{});
            else epilogue(std::false_type{});
        }
        HR_STAMP(s_r2);
        // thresholds of this wave's group: all of them after rounds 1 and 2 (the early keys rise fast), then a part
        // after every round
        if (u < 2) refresh();
        else if (!(HR_Q256_DIAG & 32)) part_apply((int)(u % kParts));
#if HR_Q256_STAMPS
        HR_STAMP(s_r3);
        c_loop += s_r1 - s_r0;
        c_epi += s_r2 - s_r1;
        c_ref += s_r3 - s_r2;
#endif
    }
#if HR_Q256_CLOCK
    {
        const uint64_t clk_t1 = __builtin_amdgcn_s_memtime(), clk_r1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0 && wv == 0 && (blockIdx.x % 64) == 0)
            printf("q256clock blk %d cycles %lu ticks %lu\n", (int)blockIdx.x, (unsigned long)(clk_t1 - clk_t0),
                   (unsigned long)(clk_r1 - clk_r0));
    }
#endif
    if constexpr ((HR_Q256_DIAG & 8) != 0) mycnt[0] += dsink;
#if HR_Q256_STAMPS
    if (lane == 0 && (blockIdx.x % 32) == 0)
        printf("q256 stamps blk %d wave %d rounds %ld loop %lu (window waits %lu) epilogue %lu refresh %lu blocks %u regs %u\n",
               (int)blockIdx.x, wv, (long)rounds, (unsigned long)c_loop, (unsigned long)c_wait, (unsigned long)c_epi,
               (unsigned long)c_ref, c_blocks, c_regs);
#endif
#pragma unroll
    for (int x = 0; x < 4; ++x) a.pcnt[(x * W + wr) * 64 + lane] = mycnt[x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the look-ahead DMAs land before the workgroup's LDS goes)
}

// ---------------------------------------------------------------------------------------------------------------
// The same FILTER on v_mfma_f32_16x16x32 (HR_Q256_MFMA16; 16-bit rows).  MI355X_MICROARCH.md "DVFS give-back" item 7:
// under the clock this MFMA-dense body holds (~1.63 GHz, measured), the 16x16x32 shape delivers ~1.12-1.15x the
// FLOP/s of 32x32x16 at equal cycles per FLOP.  Same corpus layout, windows, barriers and vmcnt accounting; what
// changes is the operand and accumulator mapping:
//  * a k32 step (= one query window of 2 k-steps) of a tile is two 16-row blocks rb: lane l = n + 16 q loads row slot
//    16 rb + n, k = 8 q .. 8 q + 7 of the k32 step -- from k-step chunk q / 2, lane slot 16 rb + n + 32 (q % 2) of the
//    tiled layout (16-byte loads at per-lane offsets; 4 x 256 contiguous bytes per load instruction);
//  * the A fragment of a 16-query block: lane (m, q) reads query m of the block, the same k -- from the window buffer
//    at k-step q / 2, 32-query block b / 2, lane 16 (b % 2) + m + 32 (q % 2);
//  * 2 tiles x 2 row blocks x 16 query blocks x 4 = 256 accumulators; a lane holds row slot 16 rb + n (its group)
//    against queries 16 b + 4 q + r in register r.
// Measured (10M x 1024 bf16, B = 256, A/B on one box, profiles/r06_q256_m16_ab.jsonl): the chip holds 1.84 GHz
// against 1.60 under the 32x32x16 form (GRBM_GUI_ACTIVE / 8 / duration), but the round takes more cycles -- twice the
// MFMA instructions to issue, and an epilogue of 64 four-register items.  With one ballot per block (the four items of
// a block share their thresholds) and the A fragments 6 blocks ahead it is 2-3 % faster per launch; the pass is then
// bound by the corpus stream (no-ring-load timing build: -0.87 ms of 4.9) more than by the matrix pipe.
template <int OFF>
__device__ __forceinline__ void lds_read4s64_wait(uint32_t base, u32x4 (&t)[4]) {  // 4 x ds_read_b128, 64 B apart
    asm volatile(
        "ds_read_b128 %0, %4 offset:%5\n\t"
        "ds_read_b128 %1, %4 offset:%6\n\t"
        "ds_read_b128 %2, %4 offset:%7\n\t"
        "ds_read_b128 %3, %4 offset:%8\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3])
        : "v"(base), "n"(OFF), "n"(OFF + 64), "n"(OFF + 128), "n"(OFF + 192));
}

template <int I>
__device__ __forceinline__ float acc_read4(const f32x4& v) {
    float r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(v[I]));
    return r;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_sub(f32x2 x, f32x2 y) {  // x - y on both halves (one VALU op; the compiler emits two)
    f32x2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

__device__ __forceinline__ float max3_raw(float x, float y, float z) {  // (no NaN canonicalisation of the inputs)
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    return r;
}

template <int MT>
__device__ __forceinline__ f32x4 mfma16(const u32x4& a, const u32x4& b, const f32x4& c) {
    if constexpr (MT == BF16)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
}

template <int MT, int S_>
__global__ __launch_bounds__(kQT, 1) void k_filter_q256_m16(ScanArgs a) {
    using Geom = Q256Geom<S_, 1>;
    constexpr int kRing = Geom::kRing, kLook = Geom::kLook, kNB = Geom::kNB;
    constexpr int kVmNext = Geom::kVmNext, kBar = Geom::kBar;
    constexpr int kR32 = kRing / kWin;  // k32 steps (windows) per ring span
    static_assert(S_ % kRing == 0 && kRing % kWin == 0 && kWin == 2, "tile depth");
    __shared__ __attribute__((aligned(16))) u32x4 qw[kNB * kWQ];
    __shared__ __attribute__((aligned(16))) float th_lds[256];
    constexpr int NQ = S_ / kRing;

    const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, g = lane & 31;
    const int n16 = lane & 15, q4 = lane >> 4;  // 16x16x32 lane roles: row / column n16, k-group q4
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t W = (int64_t)gridDim.x * 4;
    const int64_t W2 = 2 * W;
    const int64_t wr = (int64_t)wv * gridDim.x + blockIdx.x;
    const int64_t n_tiles = a.n_units;
    const int64_t rounds = (n_tiles + W2 - 1) / W2;
    const int64_t full_rounds = n_tiles / W2;
    auto tile_of = [&](int64_t u, int which) -> int64_t {
        if (u >= rounds) return -1;
        int64_t pos = wr;
        if (HR_ROTATE_ROUNDS && u < full_rounds) {
            pos += (int64_t)((uint32_t)((uint64_t)u * 2654435761ull) % (uint32_t)W);
            if (pos >= W) pos -= W;
        }
        const int64_t t = HR_Q256_ADJ ? u * W2 + 2 * pos + which : u * W2 + which * W + pos;
        return wave_uniform(t < n_tiles ? t : -1);
    };
    auto rsrc = [&](int64_t t) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(a.rows + (t < 0 ? 0 : t) * (S_ * 1024)), (short)0,
                                                 t < 0 ? 0 : S_ * 1024, 0x00020000);
    };
    // per-lane byte offsets of the two row blocks of a k32 step (chunk q4 / 2, lane slot 16 rb + n16 + 32 (q4 % 2))
    const int voff0 = (q4 >> 1) * 1024 + (n16 + 32 * (q4 & 1)) * 16;
    const int voff1 = voff0 + 16 * 16;
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int k32, int rb) -> u32x4 {
        return __builtin_amdgcn_raw_buffer_load_b128(r, rb ? voff1 : voff0, k32 * 2048, HR_Q256_NT);
    };
    const int voff = lane * 16;
    const __amdgpu_buffer_rsrc_t qr =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.qfrag, (short)0, 4 * S_ * 2048, 0x00020000);
    const uint32_t qw_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)qw;
    auto stage = [&](int bi, int s0) {
        u32x4* buf = qw + bi * kWQ;
#pragma unroll
        for (int j = 0; j < kDma; ++j) {
            const int i = j >> 1, blk = (j & 1) * 4 + wv;
            const int soff = (((blk >> 1) * S_ + s0 + i) * 2 + (blk & 1)) * 1024;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (__attribute__((address_space(3))) void*)(buf + j * 256 + wv * 64),
                                                     16, voff, soff, 0, 0);
        }
    };
    // A fragment of 16-query block b in window buffer bi: this lane's address (k-step q4 / 2, lane 32 (q4 % 2) + n16;
    // block b adds (b / 2) KiB + (b % 2) 256 B as an immediate)
    const uint32_t lane_a = qw_base + (uint32_t)((q4 >> 1) * 8 * 1024 + (n16 + 32 * (q4 & 1)) * 16);
    auto qbase = [&](int bi) -> uint32_t { return lane_a + (uint32_t)(bi * kWQ * 16); };
    const uint32_t th_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)th_lds;
    const uint32_t th_lane4 = th_base + (uint32_t)(4 * q4) * 4u;  // thresholds of queries 16 b + 4 q4 .. + 3 at + 64 b

    // ---- thresholds: as k_filter_q256
    const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc((void*)a.mkeys, (short)0, kQT * 32 * 4, 0x00020000);
    const uint32_t key_lane = (uint32_t)(((64 * wv + half) * 32 + g) * 4);
    const uint32_t th_q = th_base + (uint32_t)(64 * wv + half) * 4u;
    auto refresh = [&]() {
        uint32_t key[32];
        static_for<32>([&](auto J_) {
            constexpr int j = decltype(J_)::value;
            key[j] = __builtin_amdgcn_raw_buffer_load_b32(kr, key_lane, j * 256, 16);
        });
        static_for<32>([&](auto J_) {
            constexpr int j = decltype(J_)::value;
            const float f = half_min32(key2f(key[j] > HR_KEY_NEG_INF ? key[j] : HR_KEY_NEG_INF));
            lds_write_f32<8 * j>(th_q, fmaxf(lds_read_f32o<8 * j>(th_q), f));
        });
    };
    constexpr int kKR = 8;
    constexpr int kParts = 32 / kKR;
    uint32_t qkey[kKR];
    auto part_load = [&](int p) {
        static_for<kKR>([&](auto J_) {
            constexpr int j = decltype(J_)::value;
            qkey[j] = __builtin_amdgcn_raw_buffer_load_b32(kr, key_lane, p * (kKR * 256) + j * 256, 16);
        });
    };
    auto part_apply = [&](int p) {
        const uint32_t base = th_q + (uint32_t)p * (kKR * 8u);
        uint32_t m[kKR];
        static_for<kKR>([&](auto J_) {
            constexpr int j = decltype(J_)::value;
            m[j] = qkey[j] > HR_KEY_NEG_INF ? qkey[j] : HR_KEY_NEG_INF;
        });
        auto step = [&](auto CTRL_) {
            static_for<kKR>([&](auto J_) {
                constexpr int j = decltype(J_)::value;
                m[j] = min(m[j], dpp_u32<decltype(CTRL_)::value>(m[j]));
            });
        };
        step(std::integral_constant<int, 0xB1>{});
        step(std::integral_constant<int, 0x4E>{});
        step(std::integral_constant<int, 0x141>{});
        step(std::integral_constant<int, 0x140>{});
        float t[kKR];
        lds_read8_stride8_wait(base, t);
        static_for<kKR>([&](auto J_) {
            constexpr int j = decltype(J_)::value;
            const auto r = __builtin_amdgcn_permlane16_swap(m[j], m[j], false, false);
            const uint32_t x = r[0], y = r[1];
            lds_write_f32<8 * j>(base, fmaxf(t[j], key2f(min(x, y))));
        });
    };
    th_lds[tid] = a.floor_q[tid];
    __syncthreads();
    refresh();

    // ---- prologue
    u32x4 ra[kRing], rb[kRing];  // slot 2 w + rb_: row block rb_ of the span's k32 step w
    for (int w = 0; w < kLook; ++w) stage(w, (w * kWin) % S_);
    {
        const auto r0 = rsrc(tile_of(0, 0)), r1 = rsrc(tile_of(0, 1));
#pragma unroll
        for (int w = 0; w < kR32; ++w)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                ra[2 * w + h] = ld(r0, w, h);
                rb[2 * w + h] = ld(r1, w, h);
            }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    uint32_t mycnt[4] = {0u, 0u, 0u, 0u};
    // a passing (tile, row block, 16-query block)'s registers: rows of this lane's slot against queries 16 b + 4 q4 + r
    auto walk = [&](int b, bool ok, uint32_t row, int slot, const f32x4& V, const f32x4& TH, uint32_t regs) {
        const int gq = b >> 2;
        uint32_t& cnt = mycnt[gq];
        float2* const reg = a.pbuf + ((gq * W + wr) * 64) * a.capw;
        while (regs) {
            const int r = __builtin_amdgcn_readfirstlane(__builtin_ctz(regs));
            regs &= regs - 1u;
            const float v = V[r];
            const int qm = (b & 3) * 16 + r;  // query (within the group) of lane quad 0
            const bool pass = ok && v >= TH[r];
            const uint64_t msk = __ballot(pass);
            if (pass) atomicMax(a.mkeys + (int64_t)(gq * 64 + qm + 4 * q4) * 32 + slot, f2key(v));
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const uint32_t mh = (uint32_t)(msk >> (16 * hh)) & 0xFFFFu;
                if (!mh) continue;
                const int ql = qm + 4 * hh;
                const uint32_t basepos = (uint32_t)__builtin_amdgcn_readlane((int)cnt, ql);
                if (pass && q4 == hh) {
                    const uint32_t pos = basepos + __builtin_popcount(mh & ((1u << n16) - 1u));
                    if (pos < (uint32_t)a.capw) reg[ql * a.capw + pos] = make_float2(v, __builtin_bit_cast(float, row));
                }
                cnt += (lane == ql) ? (uint32_t)__builtin_popcount(mh) : 0u;
            }
        }
    };
    auto allow_word = [&](int64_t t) -> uint32_t {
        if (t < 0) return 0u;
        uint32_t w0 = scalar_word(a.live, t);
        if (a.mask) w0 &= scalar_word(a.mask, t);
        return w0;
    };
    // A fragments kPf blocks ahead (one ds_read_b128 per 4 MFMAs, 64 cycles of matrix work) in a kSlots rotation
    constexpr int kPf = HR_Q256_PF16;
    constexpr int kSlots = HR_Q256_SLOTS16;
    static_assert(kPf >= 1 && kPf < kSlots && (kSlots & (kSlots - 1)) == 0 && 16 % kSlots == 0, "A prefetch");
    u32x4 pf[kSlots];
    static_for<kPf>([&](auto P_) {  // (window 0's first reads: blocks 0 .. kPf - 1)
        constexpr int pn = decltype(P_)::value;
        pf[pn] = lds_read<(pn >> 1) * 1024 + (pn & 1) * 256>(qbase(0));
    });
    int wb = 0;
    uint32_t qcur = qbase(0), qnext = qbase(1);
    uint32_t dsink = 0;  // (HR_Q256_DIAG & 8 timing builds only)
#if HR_Q256_STAMPS
    uint64_t c_loop = 0, c_wait = 0, c_epi = 0, c_ref = 0;
    uint32_t c_blocks = 0, c_regs = 0;
#endif

    for (int64_t u = 0; u < rounds; ++u) {
        HR_STAMP(s_r0);
        if (u >= 2) part_load((int)(u % kParts));
        const int64_t tA = tile_of(u, 0), tB = tile_of(u, 1);
        const int64_t nA = tile_of(u + 1, 0), nB = tile_of(u + 1, 1);
        const uint32_t allowA = allow_word(tA), allowB = allow_word(tB);
        float xs[2][2];  // (euclidean) |x|^2 of this lane's row in each (tile, row block)
        static_for<2>([&](auto T_) {
            constexpr int T = decltype(T_)::value;
            const int64_t t = T ? tB : tA;
            static_for<2>([&](auto R_) {
                constexpr int rb_ = decltype(R_)::value;
                xs[T][rb_] = (a.xnorm && t >= 0) ? a.xnorm[t * 32 + slot_row(t, 16 * rb_ + n16)] : 0.0f;
            });
        });
        f32x4 acc[2][2][16];
        static_for<2>([&](auto T_) {
            static_for<2>([&](auto R_) {
                static_for<16>([&](auto B_) {
                    acc[decltype(T_)::value][decltype(R_)::value][decltype(B_)::value] = f32x4{};
                });
            });
        });
#pragma unroll
        for (int qs = 0; qs < NQ; ++qs) {
            const bool last = qs + 1 == NQ;
            const auto sA = rsrc(last ? nA : tA), sB = rsrc(last ? nB : tB);
            const int kb = last ? 0 : (qs + 1) * kR32;
            static_for<kR32>([&](auto W_) {
                constexpr int w = decltype(W_)::value;  // k32 step (window) within the span
                if (w > 0 || qs > 0 || u > 0) wb = wb + 1 == kNB ? 0 : wb + 1;
                if constexpr (w % kBar == 0) {
                    HR_STAMP(s_w0);
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kVmNext) : "memory");
                    if (!(HR_Q256_DIAG & 4)) __builtin_amdgcn_s_barrier();
#if HR_Q256_STAMPS
                    HR_STAMP(s_w1);
                    c_wait += s_w1 - s_w0;
#endif
                }
                if (!(HR_Q256_DIAG & 1)) stage(wb >= kBar ? wb - kBar : wb - kBar + kNB, (qs * kRing + w * kWin + kLook * kWin) % S_);
                qcur = qbase(wb);
                qnext = qbase(wb + 1 == kNB ? 0 : wb + 1);
                const u32x4 xa0 = ra[2 * w], xa1 = ra[2 * w + 1], xb0 = rb[2 * w], xb1 = rb[2 * w + 1];
                if (!(HR_Q256_DIAG & 2)) {
                    ra[2 * w] = ld(sA, kb + w, 0);
                    ra[2 * w + 1] = ld(sA, kb + w, 1);
                    rb[2 * w] = ld(sB, kb + w, 0);
                    rb[2 * w + 1] = ld(sB, kb + w, 1);
                } else {  // (timing build: the ring registers stay live without loads)
                    ra[2 * w] ^= xb0;
                    rb[2 * w + 1] ^= xa1;
                }
                static_for<16>([&](auto B_) {
                    constexpr int b = decltype(B_)::value;
                    constexpr int p = w * 16 + b;
                    constexpr int pn = p + kPf;
                    constexpr int wn = pn >> 4, bn = pn & 15;  // window (possibly the next span's first) and block read now
                    const uint32_t base = wn != w ? qnext : qcur;
                    pf[pn % kSlots] = lds_read<(bn >> 1) * 1024 + (bn & 1) * 256>(base);
                    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(pf[p % kSlots]) : "n"(kPf));
                    if constexpr ((HR_Q256_DIAG & 8) != 0) {  // (timing build: operands consumed, no MFMA)
                        dsink ^= pf[p % kSlots].x ^ pf[p % kSlots].w ^ xa0.x ^ xb1.y;
                    } else {
                        acc[0][0][b] = mfma16<MT>(pf[p % kSlots], xa0, acc[0][0][b]);
                        acc[0][1][b] = mfma16<MT>(pf[p % kSlots], xa1, acc[0][1][b]);
                        acc[1][0][b] = mfma16<MT>(pf[p % kSlots], xb0, acc[1][0][b]);
                        acc[1][1][b] = mfma16<MT>(pf[p % kSlots], xb1, acc[1][1][b]);
                    }
                });
            });
        }

        // ---- epilogue: per 16-query block, the lane's 4 thresholds (4 blocks per LDS round trip) are the same for both
        // tiles and both row blocks, so the block's 16 scores reduce to one max of (score - threshold) (packed
        // subtracts, max3) and ONE ballot; a passing block (rare after the first rounds) is walked per (tile, row block)
        auto epilogue = [&](auto EUC_) {
            constexpr bool EUC = decltype(EUC_)::value;
            bool ok[2][2];
            float pen[2][2];  // 0 for an allowed row, -inf otherwise: the reduction stays branch-free
            uint32_t rowv[2][2];
            static_for<2>([&](auto T_) {
                constexpr int T = decltype(T_)::value;
                const int64_t t = T ? tB : tA;
                const uint32_t allow = T ? allowB : allowA;
                static_for<2>([&](auto R_) {
                    constexpr int rb_ = decltype(R_)::value;
                    const int rg = slot_row(t < 0 ? 0 : t, 16 * rb_ + n16);
                    ok[T][rb_] = (allow >> rg) & 1u;
                    pen[T][rb_] = ok[T][rb_] ? 0.0f : -__builtin_inff();
                    rowv[T][rb_] = (uint32_t)(t * 32 + rg);
                });
            });
            static_for<4>([&](auto G_) {
                constexpr int gb = decltype(G_)::value;
                u32x4 t4[4];
                lds_read4s64_wait<gb * 256>(th_lane4, t4);
                static_for<4>([&](auto J_) {
                    constexpr int b = 4 * gb + decltype(J_)::value;
                    const f32x4 TH = __builtin_bit_cast(f32x4, t4[decltype(J_)::value]);
                    f32x4 V[2][2];
                    float e = -__builtin_inff();
                    static_for<2>([&](auto T_) {
                        constexpr int T = decltype(T_)::value;
                        static_for<2>([&](auto R_) {
                            constexpr int rb_ = decltype(R_)::value;
                            f32x4 r;
                            static_for<4>([&](auto I_) {
                                constexpr int i = decltype(I_)::value;
                                r[i] = acc_read4<i>(acc[T][rb_][b]);
                            });
                            if constexpr (EUC) r = 2.0f * r - xs[T][rb_];
                            V[T][rb_] = r;
                            const f32x2 d0 = pk_sub(__builtin_shufflevector(r, r, 0, 1), __builtin_shufflevector(TH, TH, 0, 1));
                            const f32x2 d1 = pk_sub(__builtin_shufflevector(r, r, 2, 3), __builtin_shufflevector(TH, TH, 2, 3));
                            const float m = max3_raw(d0[0], d0[1], d1[0]) + pen[T][rb_];
                            e = max3_raw(e, m, d1[1] + pen[T][rb_]);
                        });
                    });
                    if (!__ballot(e >= 0.0f)) return;
                    static_for<2>([&](auto T_) {
                        constexpr int T = decltype(T_)::value;
                        static_for<2>([&](auto R_) {
                            constexpr int rb_ = decltype(R_)::value;
                            const bool okv = ok[T][rb_];
                            uint32_t regs = 0;
                            static_for<4>([&](auto I_) {
                                constexpr int i = decltype(I_)::value;
                                regs |= (__ballot(okv && V[T][rb_][i] >= TH[i]) != 0 ? 1u : 0u) << i;
                            });
                            if (!regs) return;
                            walk(b, okv, rowv[T][rb_], 16 * rb_ + n16, V[T][rb_], TH, regs);
#if HR_Q256_STAMPS
                            c_blocks += 1;
                            c_regs += __builtin_popcount(regs);
#endif
                        });
                    });
                });
            });
        };
        HR_STAMP(s_r1);
        if constexpr ((HR_Q256_DIAG & 24) != 0) {  // (timing build: no epilogue, the accumulators kept live)
            float z = 0.0f;
            static_for<2>([&](auto T_) {
                static_for<2>([&](auto R_) {
                    static_for<16>([&](auto B_) {
                        z += acc_read4<0>(acc[decltype(T_)::value][decltype(R_)::value][decltype(B_)::value]);
                    });
                });
            });
            mycnt[0] += __builtin_bit_cast(uint32_t, z) + allowA + allowB;
        } else {
            if (a.xnorm) epilogue(std::true_type{});
            else epilogue(std::false_type{});
        }
        HR_STAMP(s_r2);
        if (u < 2) refresh();
        else part_apply((int)(u % kParts));
#if HR_Q256_STAMPS
        HR_STAMP(s_r3);
        c_loop += s_r1 - s_r0;
        c_epi += s_r2 - s_r1;
        c_ref += s_r3 - s_r2;
#endif
    }
#if HR_Q256_STAMPS
    if (lane == 0 && (blockIdx.x % 32) == 0)
        printf("q256 stamps blk %d wave %d rounds %ld loop %lu (window waits %lu) epilogue %lu refresh %lu blocks %u regs %u\n",
               (int)blockIdx.x, wv, (long)rounds, (unsigned long)c_loop, (unsigned long)c_wait, (unsigned long)c_epi,
               (unsigned long)c_ref, c_blocks, c_regs);
#endif
    if constexpr ((HR_Q256_DIAG & 8) != 0) mycnt[0] += dsink;
#pragma unroll
    for (int x = 0; x < 4; ++x) a.pcnt[(x * W + wr) * 64 + lane] = mycnt[x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int MT, int S_>
int launch_m16(int cus, const ScanArgs& a, hipStream_t st) {
    hipLaunchKernelGGL((k_filter_q256_m16<MT, S_>), dim3((unsigned)cus), dim3(kQT), 0, st, a);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}

template <int MT, int DT, int S_>
int launch_t(int cus, const ScanArgs& a, hipStream_t st) {
    hipLaunchKernelGGL((k_filter_q256<MT, DT, S_>), dim3((unsigned)cus), dim3(kQT), 0, st, a);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}

}  // namespace

bool q256_filter_ok(int dtype, int S) {
    return (dtype == BF16 || dtype == F16 || dtype == F32) && (S == 16 || S == 32 || S == 48 || S == 64);
}

int launch_filter_q256(int mt, int dtype, int S, int cus, const ScanArgs& a, hipStream_t st) {
    if (!q256_filter_ok(dtype, S)) return HR_E_UNSUPPORTED;
#define HR_Q256_CASE(MTv, DTv, Sv) \
    if (mt == MTv && dtype == DTv && S == Sv) return launch_t<MTv, DTv, Sv>(cus, a, st);
#define HR_Q256_M16(MTv, Sv) \
    if (mt == MTv && dtype == MTv && S == Sv) return launch_m16<MTv, Sv>(cus, a, st);
    // 16-bit rows at D = 512..1024: the 16x16x32 form (HR_Q256_MFMA16 0 builds the 32x32x16 one for them instead);
    // D = 256 keeps the 16-deep-ring 32x32x16 form
#if defined(HR_Q256_ONE_F32)  // (code studies of the fp32 form: that instantiation only)
    HR_Q256_CASE(F16, F32, 64)
#elif HR_Q256_MFMA16
    HR_Q256_M16(BF16, 64)
#else
    HR_Q256_CASE(BF16, BF16, 64)
#endif
#if !defined(HR_Q256_ONE) && !defined(HR_Q256_ONE_F32)  // (register-allocation studies compile one instantiation)
#if HR_Q256_MFMA16
    HR_Q256_M16(BF16, 48) HR_Q256_M16(BF16, 32) HR_Q256_M16(F16, 64) HR_Q256_M16(F16, 48) HR_Q256_M16(F16, 32)
#else
    HR_Q256_CASE(BF16, BF16, 48) HR_Q256_CASE(BF16, BF16, 32)
    HR_Q256_CASE(F16, F16, 64) HR_Q256_CASE(F16, F16, 48) HR_Q256_CASE(F16, F16, 32)
#endif
    HR_Q256_CASE(BF16, BF16, 16) HR_Q256_CASE(F16, F16, 16)
    // fp32 rows: f16 MFMA for cosine (normalised rows), bf16 for raw inner product / euclidean (mfma_type)
    HR_Q256_CASE(F16, F32, 64) HR_Q256_CASE(F16, F32, 48) HR_Q256_CASE(F16, F32, 32) HR_Q256_CASE(F16, F32, 16)
    HR_Q256_CASE(BF16, F32, 64) HR_Q256_CASE(BF16, F32, 48) HR_Q256_CASE(BF16, F32, 32) HR_Q256_CASE(BF16, F32, 16)
#endif
#undef HR_Q256_M16
#undef HR_Q256_CASE
    return HR_E_UNSUPPORTED;
}

}  // namespace hr
