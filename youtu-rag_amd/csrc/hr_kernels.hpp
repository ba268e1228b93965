// hr_kernels.hpp -- CDNA4 (gfx950) kernels of the hiprag vector index.
//
// Corpus layout in HBM ("MFMA-tiled"): rows are grouped in tiles of 32; a tile
// is S = dpad/16 k-steps; k-step s of tile t is one 1 KiB block (2 KiB for an
// fp32 corpus) holding, for lane l = r + 32h (r = row in tile, h = 0/1), the 8
// elements k = 16s + 8h .. 16s + 8h + 7 of row r.  One wave-wide 16-byte load
// of a k-step is therefore both perfectly coalesced (1 KiB contiguous) and
// exactly the B operand of v_mfma_f32_32x32x16_{bf16,f16} for those 32 rows.
// A wave streams its contiguous tile range as one linear byte stream.
//
// Kernels (SURVEY.md §2 kernel inventory):
//   k_store      K1+K2  canonical L2-normalise (cosine) + RNE quantise, tiled write
//   k_prep_q     K1     query normalise + quantise into A-fragment order, error terms
//   k_scan       K3+K6  Q·Xᵀ on MFMA, live/mask predicate, group-max threshold,
//                       ballot-compacted candidate append (SAMPLE / FILTER modes)
//   k_select     K4     per-query candidate compaction + bitonic top-kc
//   k_rescore    K5     exact canonical fp64 rescoring + shard error bound
//   k_merge      K4/C1  (exact desc, row asc) merge over shards + exactness guard
//   k_gather     get_by_id de-tiling
#pragma once
#include "hr_common.hpp"

namespace hr {

// ---------------------------------------------------------------- K1+K2: store rows
// One wave per row.  Phase 1: canonical fp64 norm² (lane-strided + butterfly, exactly the
// oracle's order).  Phase 2: lane c owns 8-element chunks, scales (cosine), quantises
// and writes its 16-byte (32-byte for fp32) slot of the tiled layout.
// SYNTH: local row L = lrow0 + r gets generator row gen_base + stripe_row(L, sG, ss) (the handle row
// of a striped shard; for a single-device index gen_base + L).
template <int DT, bool SYNTH>
__global__ __launch_bounds__(256) void k_store(const float* __restrict__ in, uint64_t seed, int64_t gen_base, int64_t n,
                                               int dim, int S, int metric, int64_t lrow0, uint8_t* __restrict__ rows,
                                               unsigned long long* max_norm2_bits,
                                               const int64_t* __restrict__ dest = nullptr, int sG = 1, int ss = 0) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const int64_t grow = SYNTH ? gen_base + stripe_row(lrow0 + r, sG, ss) : 0;
    auto src = [&](int d) -> float {
        if (d >= dim) return 0.0f;
        return SYNTH ? gen_elem(seed, grow, dim, d) : in[r * dim + d];
    };
    double inv = 1.0;
    bool scale = false;
    if (metric == COSINE) {
        double p = 0.0;
        for (int d = lane; d < dim; d += 64) {
            double x = (double)src(d);
            p = p + x * x;
        }
        double n2 = wave_butterfly_sum(p);
        if (n2 > 0.0) {
            inv = 1.0 / __builtin_sqrt(n2);
            scale = true;
        }
    }
    const int64_t R = dest ? dest[r] : lrow0 + r;  // dest: explicit positions (IVF lists)
    const int nchunk = S * 2;  // 8-element chunks per row
    double sq = 0.0;
    for (int c = lane; c < nchunk; c += 64) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float x = src(8 * c + j);
            v[j] = scale ? (float)((double)x * inv) : x;
        }
        const int s = c >> 1, h = c & 1;
        const int64_t chunk = (R >> 5) * S + s;
        const int sl = row_slot(R) + 32 * h;
        if (DT == F32) {
#pragma unroll
            for (int j = 0; j < 8; ++j) sq += (double)v[j] * (double)v[j];
            float4* p0 = (float4*)(rows + chunk * 2048 + sl * 16);
            float4* p1 = (float4*)(rows + chunk * 2048 + 1024 + sl * 16);
            *p0 = make_float4(v[0], v[1], v[2], v[3]);
            *p1 = make_float4(v[4], v[5], v[6], v[7]);
        } else {
            uint16_t hq[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                hq[j] = DT == BF16 ? f32_to_bf16_rne(v[j]) : f32_to_f16_rne(v[j]);
                float dq = DT == BF16 ? bf16_to_f32(hq[j]) : f16_to_f32(hq[j]);
                sq += (double)dq * (double)dq;
            }
            u32x4 w;
            w[0] = hq[0] | ((uint32_t)hq[1] << 16);
            w[1] = hq[2] | ((uint32_t)hq[3] << 16);
            w[2] = hq[4] | ((uint32_t)hq[5] << 16);
            w[3] = hq[6] | ((uint32_t)hq[7] << 16);
            *(u32x4*)(rows + chunk * 1024 + sl * 16) = w;
        }
    }
    sq = wave_butterfly_sum(sq);
    if (lane == 0) atomicMax(max_norm2_bits, (unsigned long long)__builtin_bit_cast(uint64_t, sq));
}

// ---------------------------------------------------------------- K1b: stored row norms (euclidean)
// One wave per row: |x|^2 of the stored (quantised) row in the canonical order, as fp32.  Used
// only by the approximate scan score 2 q.x - |x|^2 (its rounding is inside the guard's bound);
// the exact rescoring recomputes the canonical fp64 value.
template <int DT>
__global__ __launch_bounds__(256) void k_row_norms(const uint8_t* __restrict__ rows, int S, int dpad, int64_t r0,
                                                   int64_t n, float* __restrict__ xnorm,
                                                   const int64_t* __restrict__ dest = nullptr) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int64_t r = dest ? dest[i] : r0 + i;
    double p = 0.0;
#pragma unroll 8
    for (int d = lane; d < dpad; d += 64) {
        const double x = (double)load_elem<DT>(rows, S, r, d);
        p = p + x * x;
    }
    p = wave_butterfly_sum(p);
    if (lane == 0) xnorm[r] = (float)p;
}

// live bits of explicitly placed rows
static __global__ __attribute__((unused)) void k_mark_live(const int64_t* __restrict__ dest, int64_t n, uint32_t* __restrict__ live) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicOr(&live[dest[i] >> 5], 1u << (dest[i] & 31));
}

// synthetic fp32 rows (the corpus generator of k_store / the oracle), row-major
static __global__ __attribute__((unused)) void k_gen_rows(uint64_t seed, int64_t row0, int64_t n, int dim, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n * dim) out[i] = gen_elem(seed, row0 + i / dim, dim, (int)(i % dim));
}

// ---------------------------------------------------------------- K1: query prep
// One wave per (padded) query.  q32: normalised fp32 queries [Bp][dpad] (exact rescoring
// operand); qfrag: MFMA A-fragments [S][QB][64 lanes][8]; qerr[4b] = ||q - q̂||, [4b+1] = ||q̂||,
// [4b+2] = |q|^2 (canonical fp64 of the processed query: the euclidean score's first term).
// One wave per query.  The wave's whole query row is loaded in ONE batch of independent loads
// (kPrepJ per lane: dim <= 2560) before any arithmetic: the kernel then costs one memory round
// trip instead of one per unrolled group of the two passes (measured 17 -> ? us per launch at
// B=64, D=1024).  Arithmetic order is unchanged (canonical: lane-strided fp64 sum + butterfly).
static constexpr int kPrepJ = 40;  // 40 * 64 = 2560 = the widest query tile the scan's LDS holds
template <int MT>
__global__ __launch_bounds__(256) void k_prep_q(const float* __restrict__ q, int B, int Bp, int dim, int dpad, int S,
                                                int QB, int metric, float* __restrict__ q32,
                                                uint16_t* __restrict__ qfrag, double* __restrict__ qerr,
                                                uint32_t* __restrict__ mkeys, int np, uint32_t* __restrict__ cnt,
                                                float* __restrict__ floor_q, uint32_t* __restrict__ dyn_q) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= Bp) return;
    const bool real = b < B;
    auto src = [&](int d) -> float { return (real && d < dim) ? q[(int64_t)b * dim + d] : 0.0f; };
    float v[kPrepJ];
#pragma unroll
    for (int j = 0; j < kPrepJ; ++j) v[j] = src(lane + 64 * j);
    // per-batch scratch of this query (replaces two memsets and an H2D copy per batch):
    // group maxima -> -inf, candidate count -> 0, floor -> -inf (+inf for padding rows);
    // floor_q == nullptr: the caller uploaded explicit floors (collect mode)
    if (mkeys && lane < 32)
        for (int p = 0; p < np; ++p) mkeys[((int64_t)p * Bp + b) * 32 + lane] = HR_KEY_NEG_INF;
    if (lane == 0) {
        if (dyn_q && (b % (QB * 32)) == 0)  // per query group: one counter per row-part team (<= 16)
            for (int p = 0; p < 16; ++p) dyn_q[(b / (QB * 32)) * 16 + p] = 0;
        if (cnt) cnt[b] = 0;
        if (floor_q) floor_q[b] = real ? -__builtin_inff() : __builtin_inff();
    }
    // elements j >= kPrepJ (dim > 2560: IVF lists only) are read in place, in the same order
    double inv = 1.0;
    bool scale = false;
    if (metric == COSINE) {
        double p = 0.0;
        auto acc = [&](int d, float xf) {
            if (d < dim) {
                const double x = (double)xf;
                p = p + x * x;
            }
        };
#pragma unroll
        for (int j = 0; j < kPrepJ; ++j) acc(lane + 64 * j, v[j]);
        for (int d = lane + 64 * kPrepJ; d < dim; d += 64) acc(d, src(d));
        double n2 = wave_butterfly_sum(p);
        if (n2 > 0.0) {
            inv = 1.0 / __builtin_sqrt(n2);
            scale = true;
        }
    }
    double e1 = 0.0, nh = 0.0, qn = 0.0;
    // A-fragment layout [group][S][QB][64 lanes][8]: a group = the QB*32 queries one scan workgroup stages
    const int qg = (b >> 5) / QB, qb = (b >> 5) % QB;
    auto put = [&](int d, float x) {
        const float y = scale ? (float)((double)x * inv) : x;
        q32[(int64_t)b * dpad + d] = y;
        const uint16_t h = quant_mt<MT>(y);
        const float dq = dequant_mt<MT>(h);
        const int s = d >> 4, sl = (b & 31) + 32 * ((d >> 3) & 1), jj = d & 7;
        qfrag[((((int64_t)qg * S + s) * QB + qb) * 64 + sl) * 8 + jj] = h;
        const double e = (double)y - (double)dq;
        e1 += e * e;
        nh += (double)dq * (double)dq;
        qn = qn + (double)y * (double)y;
    };
#pragma unroll
    for (int j = 0; j < kPrepJ; ++j)
        if (lane + 64 * j < dpad) put(lane + 64 * j, v[j]);
    for (int d = lane + 64 * kPrepJ; d < dpad; d += 64) put(d, src(d));
    e1 = wave_butterfly_sum(e1);
    nh = wave_butterfly_sum(nh);
    qn = wave_butterfly_sum(qn);
    if (lane == 0) {
        qerr[4 * b] = __builtin_sqrt(e1);
        qerr[4 * b + 1] = __builtin_sqrt(nh);
        qerr[4 * b + 2] = qn;
        qerr[4 * b + 3] = 0.0;
    }
}

// ---------------------------------------------------------------- K3: the scan
// s_waitcnt immediate that waits for vmcnt <= n only (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] |
// vmcnt[5:4] in bits 15:14)
constexpr int vmcnt_only(int n) { return 0x0F70 | (n & 15) | (((n >> 4) & 3) << 14); }

// global -> LDS copy of n 16-byte vectors by the whole block, U loads in flight per thread
__device__ inline void stage_lds(u32x4* dst, const u32x4* src, int n) {
    constexpr int U = 8;
    const int st = blockDim.x;
    int i = threadIdx.x;
    for (; i + (U - 1) * st < n; i += U * st) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) v[j] = src[i + j * st];
#pragma unroll
        for (int j = 0; j < U; ++j) dst[i + j * st] = v[j];
    }
    for (; i < n; i += st) dst[i] = src[i];
}

struct ScanArgs {
    const uint8_t* rows;     // tiled corpus
    const uint32_t* live;    // one word per tile
    const uint32_t* mask;    // one word per tile (u64 row bitmap viewed as u32), nullable
    const uint16_t* qfrag;   // [S][QB][64][8]
    int S;
    int64_t n_units;         // tiles (FILTER) or sample tiles (SAMPLE)
    int64_t sample_stride;   // SAMPLE: tile = unit * stride
    // optional sorted list of the tiles to visit (a selective row filter: only tiles holding at
    // least one live, allowed row); unit u then stands for tile_list[u * stride].  nullptr: all tiles
    const uint32_t* tile_list;
    uint32_t* mkeys;         // [np parts][QB*32 queries][32 groups] group-max keys (a wave access spans 2 lines)
    int np;                  // row parts: group (p, g) = rows of tile part p with row % 32 == g (k > 32)
    int64_t part_tiles;      // tiles per part (part of tile t = t / part_tiles)
    int64_t pstride;         // words between parts of mkeys (QB*32*32)
    const float* floor_q;    // [QB*32] per-query floor (collect mode / +inf for padding)
    int use_groups;          // FILTER: threshold = max(floor, min_g M[q][g]) if set, else floor
    uint32_t* cnt;           // [QB*32] candidate counts (shared-buffer mode)
    float2* buf;             // [QB*32][cap] (approx score, row bits)
    int cap;
    int refresh_every;       // tiles between threshold refreshes (FILTER, use_groups)
    int publish;             // FILTER: publish this wave's group maxima at refresh
    // private mode (FILTER): each wave appends into its own region pbuf[w][q][capw] and
    // reports pcnt[w][q]; no atomics on the append path.  The [wave][query] order makes the
    // query index a compile-time offset from a wave-uniform base (no hoisted per-query
    // pointers: those cost ~150 VGPRs of spills in the fully unrolled epilogue).
    int private_bufs;
    int wave_major;          // unit ranges numbered wave-major across workgroups (spreads the tail)
    int strided;             // static units dealt round-robin (wave wr: wr, wr + W, ...) instead of in ranges
    float2* pbuf;
    uint32_t* pcnt;
    int capw;
    // dynamic tail (FILTER): waves run at rates that differ by +-6 % (two waves share a SIMD and
    // are not served fairly), so a static split ends with the slowest wave.  Units [0, dyn_start)
    // are split statically; the rest are handed out in runs of dyn_chunk units from a counter
    // (zeroed by k_prep_q), grabbed while a wave works on the last unit of its current run.
    int64_t dyn_start;       // == n_units: no dynamic part
    int dyn_chunk;
    uint32_t* dyn_q;
    // euclidean: approximate score 2 q̂.x - |x|^2 (fp32 |x|^2 per row); nullptr for cosine / ip
    const float* xnorm;
    // diagnostics (nullable): tiles each wave scanned, [group wave] -- every tile exactly once over a FILTER's waves
    uint32_t* wave_tiles;
    // query groups (more than QB*32 queries per corpus pass): ng workgroups stream the same tile range,
    // each with its own QB*32 queries in LDS; per-query tables hold ng consecutive groups
    int ng;
    int early_refresh;       // FILTER: a refresh's loads go out before the tile's k-loop (0: in its epilogue)
    // FILTER with row parts (np > 1) and round-robin dealing: the waves form np teams, team p (waves with
    // wr % np == p) deals part p's tiles round-robin among its members with a dynamic tail of its own
    // (counter dyn_q[p]) -- every wave stays in one part, every part is read from the start, and the chip
    // reads np windows of consecutive tiles.  0: parts keep contiguous per-wave ranges (tile lists)
    int teams;
    int dyn_pct;             // dynamic-tail percentage the host used (teams recompute their split)
    int stagger;             // FILTER: refreshes staggered over a workgroup's waves (see roff in scan_body)
};


// ---- the persistent FILTER (hr_persist.hip): control words of the instances and one instance's launch
constexpr int kPersistSlots = 3;    // batches in flight between the host and an instance (workspace sets)
constexpr int kPersistRing = 4096;  // per-epoch completion stamps
struct PersistCtl {                 // device memory; initialised once per index
    uint32_t gate;                  // admitted-through epoch (low 31 bits); bit 31: closed (no further admissions)
    uint32_t posted;                // highest epoch whose query prep + SAMPLE are complete
    uint32_t next_epoch;            // first epoch no instance has processed (written by an exiting instance)
    uint32_t stop;                  // a quiesce asked the instances to stop admitting
    uint32_t error;                 // a bounded wait gave up (1: instance, 2: tail)
    uint32_t runs;                  // instances that ran (did not find their batch processed already)
    uint32_t opened;                // the epoch the running instance's leader opened the gate for (release-published)
    uint32_t pad;
    // per slot: the tail's wait for the slot's current batch gave up (k_persist_wait) -- k_select then flags every
    // query of that batch as overflowed, so its guard fails and the exact collect pass answers it (never a partial scan)
    uint32_t slot_fail[4];
    // per epoch (index e % ring): (e << 32) | workgroup arrivals, reset to (e << 32) by the epoch's post.  Tagged
    // rather than a monotonic per-slot count: an epoch that never completed (a failed submit, a timed-out wait) cannot
    // shift the targets of later batches, and the tail's wait cannot match a stale epoch's count
    unsigned long long arr[kPersistRing];
    // per-epoch s_memrealtime stamps (index e % ring; the post resets them): the last arrival (the tail's timing),
    // and for hr_index_persist_trace the post, the first and last workgroup start and the first arrival
    unsigned long long t_end[kPersistRing];
    unsigned long long t_post[kPersistRing], t_start0[kPersistRing], t_start1[kPersistRing], t_end0[kPersistRing];
};
struct PersistLaunch {              // kernel argument of one instance
    ScanArgs a;                     // the FILTER of slot 0's workspace; slot s: every per-batch pointer + s * its stride
    int64_t st_qfrag, st_mkeys, st_floor, st_pbuf, st_pcnt, st_dynq;  // slot strides (bytes)
    PersistCtl* ctl;
    uint32_t* host_err;             // pinned host word mirroring PersistCtl::error (nullable)
    uint32_t e0;                    // the epoch the instance was launched for
    uint32_t idle_ticks;            // s_memrealtime ticks without an admission before the instance exits
};

template <int MT>
__device__ inline f32x16 mfma32(const u32x4& a, const u32x4& b, const f32x16& c) {
    if constexpr (MT == BF16)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                        0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                       0, 0);
}

// X fragment of k-step chunk c (flattened tile*S + s) for this lane, converted to MT.
// NT: non-temporal corpus loads (every byte read once per launch); query groups (ng > 1) use the
// default policy instead, so the other groups of a range block find the tiles in the XCD's L2.
template <int MT, int DT, bool NT = true>
struct XFrag;
// corpus stream loads: every byte is read once per launch, so they go out non-temporal
// (HR_CORPUS_NT=0 builds the default-policy variant for A/B timing)
#ifndef HR_CORPUS_NT
#define HR_CORPUS_NT 1
#endif
// HR_DIAG (timing builds only -- results are WRONG with any bit set; tools/gpu diagnostic A/Bs of where a
// FILTER launch's time goes): 1 no candidate appends, 2 no threshold refreshes after the first, 4 no epilogue at
// all (group maxima, compares), 8 no query staging into LDS, 16 no MFMA (a cheap XOR keeps the operands live)
#ifndef HR_DIAG
#define HR_DIAG 0
#endif
// HR_ROTATE_ROUNDS=0 builds the unrotated round-robin dealing (A/B and the regression check of
// test_periodic_clusters_spread_over_waves only)
#ifndef HR_ROTATE_ROUNDS
#define HR_ROTATE_ROUNDS 1
#endif
// a wave-uniform 64-bit value in scalar registers (the compiler cannot prove threadIdx.x >> 6 uniform)
__device__ inline int64_t wave_uniform(int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// read-only word at a wave-uniform index through the constant address space: a scalar load, counted
// by lgkmcnt -- a vector load here would be counted by vmcnt behind the corpus ring, and reading it
// would wait for every ring load issued after it
__device__ inline uint32_t scalar_word(const uint32_t* p, int64_t i) {
    return ((const __attribute__((address_space(4))) uint32_t*)p)[i];
}
template <bool NT>
__device__ inline u32x4 corpus_load(const uint8_t* p) {
#if HR_CORPUS_NT
    if constexpr (NT) return __builtin_nontemporal_load((const u32x4*)p);
#endif
    return *(const u32x4*)p;
}
template <int MT, bool NT>
struct XFrag<MT, BF16, NT> {
    static constexpr int kLoads = 1;  // 16-byte loads per lane per k-step
    u32x4 v;
    __device__ inline void load(const uint8_t* rows, int64_t c, int lane) {
        v = corpus_load<NT>(rows + c * 1024 + lane * 16);
    }
    __device__ inline u32x4 get() const { return v; }
};
template <int MT, bool NT>
struct XFrag<MT, F16, NT> {
    static constexpr int kLoads = 1;
    u32x4 v;
    __device__ inline void load(const uint8_t* rows, int64_t c, int lane) {
        v = corpus_load<NT>(rows + c * 1024 + lane * 16);
    }
    __device__ inline u32x4 get() const { return v; }
};
template <int MT, bool NT>
struct XFrag<MT, F32, NT> {
    static constexpr int kLoads = 2;
    u32x4 a, b;
    __device__ inline void load(const uint8_t* rows, int64_t c, int lane) {
        a = corpus_load<NT>(rows + c * 2048 + lane * 16);
        b = corpus_load<NT>(rows + c * 2048 + 1024 + lane * 16);
    }
    // fp32 corpus -> MFMA operand: packed hardware RNE conversion (v_cvt_pk_*).  Only the
    // error-bounded approximate score depends on it (the exact rescoring reads fp32).
    // Whole-vector bit casts: hipcc (ROCm 7.2) mis-lowers __builtin_bit_cast of single
    // ext-vector elements here (it re-used one lane value for all eight).
    __device__ inline u32x4 get() const {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        typedef float f32x8 __attribute__((ext_vector_type(8)));
        const f32x4 fa = __builtin_bit_cast(f32x4, a);
        const f32x4 fb = __builtin_bit_cast(f32x4, b);
        const f32x8 f = __builtin_shufflevector(fa, fb, 0, 1, 2, 3, 4, 5, 6, 7);
        if constexpr (MT == BF16) {
            return __builtin_bit_cast(u32x4, __builtin_convertvector(f, bf16x8));
        } else {
            return __builtin_bit_cast(u32x4, __builtin_convertvector(f, f16x8));
        }
    }
};

// query index held by accumulator register i of block qb in this lane's half
__device__ inline int acc_query(int qb, int i, int half) { return qb * 32 + (i & 3) + 8 * (i >> 2) + 4 * half; }

// Cross-lane reductions without LDS round trips (a __shfl_xor is a ds_bpermute, and a 5-step reduction waited for
// each: 40 serialised LDS round trips per refresh): DPP within each row of 16 lanes (xor 1, xor 2, half-mirror,
// mirror), then a ds_swizzle (xor 16 within 32 lanes) or four readlanes across the rows
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
// min over the 32 lanes of each half-wave, in every lane
__device__ __forceinline__ float half_min32(float f) {
    f = fminf(f, __builtin_bit_cast(float, dpp_u32<0xB1>(__builtin_bit_cast(uint32_t, f))));   // quad_perm 1,0,3,2
    f = fminf(f, __builtin_bit_cast(float, dpp_u32<0x4E>(__builtin_bit_cast(uint32_t, f))));   // quad_perm 2,3,0,1
    f = fminf(f, __builtin_bit_cast(float, dpp_u32<0x141>(__builtin_bit_cast(uint32_t, f))));  // row_half_mirror
    f = fminf(f, __builtin_bit_cast(float, dpp_u32<0x140>(__builtin_bit_cast(uint32_t, f))));  // row_mirror
    return fminf(f, __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, f), 0x401F)));
}
// OR over the wave's 64 lanes, wave-uniform
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
    x |= dpp_u32<0xB1>(x);
    x |= dpp_u32<0x4E>(x);
    x |= dpp_u32<0x141>(x);
    x |= dpp_u32<0x140>(x);
    return (uint32_t)(__builtin_amdgcn_readlane((int)x, 0) | __builtin_amdgcn_readlane((int)x, 16) |
                      __builtin_amdgcn_readlane((int)x, 32) | __builtin_amdgcn_readlane((int)x, 48));
}
// the j-th largest of the 32 values of each half-wave (1 <= j <= 32; j wave-uniform), in every lane: the smallest
// is dropped 32 - j times -- one lane per round even among equal values (the lowest such lane of the half), so
// exactly 32 - j values go -- then the minimum of the rest
__device__ __forceinline__ float half_kth_largest(float f, int j) {
    const int lane = __lane_id();
    for (int r = 0; r < 32 - j; ++r) {
        const float m = half_min32(f);
        const uint64_t b = __ballot(f == m);
        const uint32_t bh = lane >= 32 ? (uint32_t)(b >> 32) : (uint32_t)b;
        if ((lane & 31) == __builtin_ctz(bh)) f = __builtin_inff();
    }
    return half_min32(f);
}

// MODE: SCAN_SAMPLE (group maxima only), SCAN_FILTER (threshold + private per-wave
// candidate regions, no atomics on the append path), SCAN_COLLECT (floor-only threshold,
// shared per-query buffer with atomic slot reservation; the exact fallback)
enum { SCAN_SAMPLE = 0, SCAN_FILTER = 1, SCAN_COLLECT = 2 };

// TPB: threads per workgroup (512 = 8 waves, 2 per SIMD, <= 256 registers each).  A 4-wave variant
// with a 32- / 64-deep corpus ring (one wave per SIMD, up to 512 registers) was measured for the
// query-group launches and was slower (B = 128 at 10M rows: 5.7 / 6.3 ms vs 4.6 ms), so it is not built.
// The body is shared; each MODE is its own kernel symbol (k_scan_sample / k_scan_filter / k_scan_collect,
// below), so profiles tell the passes apart by name rather than by grid size or duration.
// LEAN (the persistent FILTER, hr_persist.hip): one query group, one row part, no mask or tile list, round-robin
// units -- fixed at compile time, which frees the scalar registers those cases take (the persistent loop around the
// body needs a few of its own, and this body is at the 256-VGPR limit with SGPRs spilled to VGPR lanes).
template <int MT, int DT, int QB, int P, int MODE, bool NT, int TPB, bool LEAN = false>
__device__ __forceinline__ void scan_body(ScanArgs a) {
    constexpr bool FILTER = MODE != SCAN_SAMPLE;
    constexpr bool priv = MODE == SCAN_FILTER;
    static_assert(!LEAN || MODE == SCAN_FILTER, "the lean body is a FILTER");
    if constexpr (LEAN) {
        a.ng = 1;
        a.np = 1;
        a.part_tiles = (int64_t)1 << 62;
        a.mask = nullptr;
        a.tile_list = nullptr;
        a.strided = 1;
        a.wave_major = 1;
        a.teams = 0;
        a.use_groups = 1;
        a.publish = 1;
    }
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    int tid_ = threadIdx.x;
    // the persistent loop runs this body once per batch: lane-derived values are recomputed each time instead of
    // being hoisted out of the loop into registers held across it (the body is at the 256-VGPR limit)
    if constexpr (LEAN) asm volatile("" : "+v"(tid_));
    const int tid = tid_;
    const int lane = tid & 63;
    const int half = lane >> 5;
    const int g = lane & 31;

    // Query groups: workgroup bx serves group grp of range block rb.  The ng workgroups of one range
    // block have equal bx % 8 -- one XCD under the round-robin dispatch (speed only, never
    // correctness) -- and walk the same tiles in the same order, so each corpus tile comes from HBM
    // once and from that XCD's L2 for the other groups.  ng == 1: rb = bx, grp = 0.
    const int ng = a.ng;
    const int bx = blockIdx.x;
    const int grp = ng > 1 ? (bx >> 3) % ng : 0;
    const int64_t nrb = gridDim.x / ng;
    const int64_t rb = ng > 1 ? (int64_t)((bx >> 3) / ng) * 8 + (bx & 7) : bx;
    {
        constexpr int Bq = QB * 32;
        a.qfrag += (int64_t)grp * a.S * QB * 64 * 8;
        a.mkeys += grp * Bq * 32;
        a.floor_q += grp * Bq;
        if (a.cnt) a.cnt += grp * Bq;
        if (a.buf) a.buf += (int64_t)grp * Bq * a.cap;
        if (a.dyn_q) a.dyn_q += grp * 16;
    }
    const int64_t Wg = nrb * (blockDim.x >> 6);  // waves per group
    const int64_t w = rb * (blockDim.x >> 6) + (tid >> 6);  // slot of this wave's outputs within the group
    const int64_t wg = (int64_t)grp * Wg + w;               // ... over all groups
    // unit range: contiguous per wave, numbered wave-major across workgroups so the waves that
    // get one extra unit sit on different CUs (the tail is then one tile per CU, not a
    // handful of fully loaded CUs finishing a tile after everyone else)
    const int64_t wrg = a.wave_major ? (int64_t)(tid >> 6) * nrb + rb : w;
    // teams (FILTER, row parts, round-robin dealing; ScanArgs::teams): this wave deals part tp's tiles
    // [t_off, t_off + n_units) with the other Wt waves of its team; every index below is team-local
    const bool teams = MODE == SCAN_FILTER && a.np > 1 && a.teams && a.strided;
    const int tp = teams ? (int)(wrg % a.np) : 0;
    const int64_t W = teams ? (Wg - tp + a.np - 1) / a.np : Wg;
    const int64_t wr = teams ? wrg / a.np : wrg;
    const int64_t t_off = teams ? (int64_t)tp * a.part_tiles : 0;
    const int64_t n_units = teams ? std::max<int64_t>(0, std::min<int64_t>(a.n_units - t_off, a.part_tiles)) : a.n_units;
    int64_t dyn_start = a.dyn_start;
    if (teams) {  // the host's split recomputed for this team's share (static runs >= 8 units or no tail)
        const int64_t per_wave = n_units / W;
        dyn_start = n_units;
        if (a.dyn_start < a.n_units && per_wave >= 8)
            dyn_start = (per_wave - std::max<int64_t>(2, per_wave * a.dyn_pct / 100)) * W;
    }
    uint32_t* const dyn_ctr = a.dyn_q ? a.dyn_q + tp : nullptr;
    const bool dyn = MODE == SCAN_FILTER && dyn_start < n_units;  // team-uniform
    const int64_t n_static = dyn ? dyn_start : n_units;
    // static units: a contiguous range per wave, or (strided) every W-th unit from wr, so that at any
    // moment the chip's waves read one window of consecutive tiles; u then counts the wave's own units
    const int64_t base = n_static / W, rem = n_static % W;
    const bool strided = a.strided != 0 && (a.np == 1 || teams);
    const int64_t u0 = strided ? 0 : wr * base + (wr < rem ? wr : rem);
    const int64_t u1 = strided ? (wr < n_static ? (n_static - 1 - wr) / W + 1 : 0) : u0 + base + (wr < rem ? 1 : 0);
    const int64_t stride = FILTER ? 1 : a.sample_stride;
    const int S = a.S;
    // the plan picks P dividing S (make_plan): every k-loop runs at least once, so its ring waits retire
    // whatever was issued before it (the early refresh loads) -- without this the compiler keeps the
    // zero-trip path and waits for the ring again where those loads are used
    __builtin_assume(S >= P);
    bool in_static = true;  // u indexes this wave's static units (else a dynamic unit itself)
    // Round-robin dealing: round j covers units [jW, (j+1)W) and wave wr takes one of them.  The position
    // is rotated by a hash of j (full rounds only; the last, partial round keeps wr): with a fixed
    // position, wave wr would see only tiles = wr (mod W), so any period in the rows that shares factors
    // with W -- every 4096th row in one cluster, a document's k-th chunks -- lands in the same few waves
    // (clustered 6.25M rows: 14 waves held a cluster's candidates, their 32-slot regions overflowed and
    // 45 of 64 queries took the collect pass)
    const int64_t full_rounds = n_static / W;
    auto tile_at = [&](int64_t u) -> int64_t {
        if (strided && in_static) {
            int64_t pos = wr;
            if (HR_ROTATE_ROUNDS && u < full_rounds) {
                const uint32_t rot = (uint32_t)((uint64_t)u * 2654435761ull) % (uint32_t)W;
                pos += rot;
                if (pos >= W) pos -= W;
            }
            u = u * W + pos;
        }
        const int64_t i = wave_uniform(t_off + u * stride);
        return a.tile_list ? (int64_t)scalar_word(a.tile_list, i) : i;
    };

    // The query fragments (QB*S KiB) go to LDS once per launch by LDS-DMA (buffer_load ... lds: L2 -> LDS, no
    // registers, no ds_write), issued BEFORE the corpus ring's first loads: vmcnt retires in issue order, so the
    // wait for the fragments below then leaves the ring loads in flight.  (Staged with loads + ds_writes behind the
    // ring, every workgroup waited out the ring's HBM latency, then the fragments', then the first refresh's before
    // its first MFMA: 8 % of a 1.25M-row FILTER launch and 12 % at 1M x 768 went to that start,
    // profiles/r05_small_shard_filter_diag_builds.jsonl.)  The persistent FILTER (LEAN) restages per batch with the
    // ring already running and keeps the register copy.
    const int n_q16 = a.S * QB * 64;  // 16-byte chunks of the query tile
    if constexpr (!LEAN) {
        if (!(HR_DIAG & 8)) {
            const __amdgpu_buffer_rsrc_t qr =
                __builtin_amdgcn_make_buffer_rsrc((void*)a.qfrag, (short)0, n_q16 * 16, 0x00020000);
            const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
            for (int c = wv * 64; c < n_q16; c += (int)blockDim.x)  // (wave-uniform: 64 chunks per instruction)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (__attribute__((address_space(3))) void*)(lds + c * 16), 16,
                                                         lane * 16, c * 16, 0, 0);
        }
    }
    XFrag<MT, DT, NT> ring[P];
    const bool ring0 = u0 < u1;
    if (ring0) {
        const int64_t c0 = tile_at(u0) * S;
#pragma unroll
        for (int i = 0; i < P; ++i) ring[i].load(a.rows, c0 + i, lane);
    }
    if constexpr (LEAN) {
        stage_lds((u32x4*)lds, (const u32x4*)a.qfrag, n_q16);
    } else {
        // this wave's DMAs have landed (only the ring's loads, issued after them, may be in flight); the barrier
        // below makes every wave's visible
        // (the builtin, not inline asm: the compiler's wait-count pass then knows the DMAs are complete and inserts
        // no drain of its own in front of the k-loop's LDS reads)
        if (ring0) __builtin_amdgcn_s_waitcnt(vmcnt_only(P * XFrag<MT, DT, NT>::kLoads));
        else __builtin_amdgcn_s_waitcnt(vmcnt_only(0));
    }
    __syncthreads();

    if (u0 >= u1 && FILTER) {
        if (priv && lane < QB * 32) {
            if constexpr (LEAN)
                __hip_atomic_store(&a.pcnt[wg * (QB * 32) + lane], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                a.pcnt[wg * (QB * 32) + lane] = 0;
        }
        if (a.wave_tiles && lane == 0) a.wave_tiles[wg] = 0u;
        return;
    }  // an idle SAMPLE wave stays: it takes part in the workgroup reduction below
    uint32_t mycnt = 0;  // private mode: lane q counts the candidates of query q in this wave
    float2* const wave_buf = priv ? a.pbuf + wg * (QB * 32) * a.capw : nullptr;

    const u32x4* qs = (const u32x4*)lds;

    float th[QB][16], gmax[QB][16];
    // this lane's group column of the group-max table, one base per query block; the per-register
    // query offset 32*((i&3) + 8(i>>2)) words stays under the 4 KiB immediate-offset range
    // With np > 1 parts (top-k beyond 32) the groups are (part, row % 32): 32*np disjoint row sets,
    // so min over all of them bounds the (32*np)-th best score; gkq points at this wave's current
    // part and the other parts sit at scalar offsets (p - part) * pstride.
    int64_t part = (u0 < u1 ? tile_at(u0) : 0) / a.part_tiles;
    int64_t part_end = (part + 1) * a.part_tiles;
    uint32_t* gkq[QB];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) gkq[qb] = a.mkeys + part * a.pstride + (qb * 32 + 4 * half) * 32 + g;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            gmax[qb][i] = -__builtin_inff();
            th[qb][i] = -__builtin_inff();
        }

    // Threshold refresh.  All 16*QB group-max loads are issued back to back (one memory round
    // trip per refresh; a load->compare->branch chain costs one round trip PER register and
    // measured 0.6 ms of a 1.0 ms scan at 1.25M rows), then this wave's group max is published
    // only where it beats the global value (a blind atomicMax from every wave piles ~#waves
    // atomics onto each of the 32*B addresses).
    // The loads (refresh_load) and their use (refresh_apply) are split so that the main loop issues a
    // refresh's loads BEFORE a tile's k-loop and applies them in its epilogue: the k-loop's own ring
    // waits retire them, whereas loads issued in the epilogue and used at once made the wave wait for
    // everything issued before them -- the next tile's ring refills included (a drain per refresh).
    auto refresh_load = [&](uint32_t (&key)[QB][16]) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i)
                key[qb][i] = __hip_atomic_load(gkq[qb] + 32 * ((i & 3) + 8 * (i >> 2)), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    };
    // floor: also take the per-query floor (the first refresh; th never drops below it afterwards)
    auto refresh_apply = [&](uint32_t (&key)[QB][16], bool publish, bool floor) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                key[qb][i] = key[qb][i] > HR_KEY_NEG_INF ? key[qb][i] : HR_KEY_NEG_INF;
                if (publish && a.publish && gmax[qb][i] > key2f(key[qb][i])) {
                    atomicMax(gkq[qb] + 32 * ((i & 3) + 8 * (i >> 2)), f2key(gmax[qb][i]));
                    key[qb][i] = f2key(gmax[qb][i]);
                }
            }
        // the other parts' groups of this lane (keys order like floats: min of keys = min of scores).
        // A part's 16*QB keys are loaded back to back before any is used -- one memory round trip per
        // part (a load -> min chain waited for every load in turn: (np - 1) * 32 round trips per refresh)
        for (int p = 0; p < a.np; ++p) {
            if (p == part) continue;
            const int64_t off = (p - part) * a.pstride;
            uint32_t k2[QB][16];
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    k2[qb][i] = __hip_atomic_load(gkq[qb] + off + 32 * ((i & 3) + 8 * (i >> 2)), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const uint32_t v = k2[qb][i] > HR_KEY_NEG_INF ? k2[qb][i] : HR_KEY_NEG_INF;
                    key[qb][i] = key[qb][i] < v ? key[qb][i] : v;
                }
        }
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                // (a ds_bpermute chain: the DPP + ds_swizzle form of half_min32 measured 0.5 % slower at 10M rows,
                // 1.1 % at k = 100, 0.6 % faster at 1.25M -- same box, profiles/r04_kscan_dpp_refresh_ab.jsonl)
                float f = key2f(key[qb][i]);
#pragma unroll
                for (int off = 16; off >= 1; off >>= 1) f = fminf(f, __shfl_xor(f, off, 64));
                gmax[qb][i] = -__builtin_inff();
                if (floor) f = fmaxf(f, a.floor_q[acc_query(qb, i, half)]);
                th[qb][i] = fmaxf(th[qb][i], f);
            }
    };
    auto refresh = [&](bool publish) {
        if (!a.use_groups) {
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    gmax[qb][i] = -__builtin_inff();
                    th[qb][i] = fmaxf(th[qb][i], a.floor_q[acc_query(qb, i, half)]);
                }
            return;
        }
        uint32_t key[QB][16];
        refresh_load(key);
        refresh_apply(key, publish, true);
    };
    // publish the group maxima of the part being left (or at the end of a SAMPLE range)
    auto flush = [&]() {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (gmax[qb][i] > -__builtin_inff())
                    atomicMax(gkq[qb] + 32 * ((i & 3) + 8 * (i >> 2)), f2key(gmax[qb][i]));
                gmax[qb][i] = -__builtin_inff();
            }
    };
    if (FILTER) refresh(false);


    // grab the next dynamic run: first unit, or -1 when the pool is exhausted
    // The grab is issued one unit before its result is needed (runs are >= 2 units long): the
    // returned value then sits behind a whole unit of ring loads, so reading it costs no wait.
    // (Reading it at once makes the compiler drain every outstanding load: vmcnt(0).)
    auto grab_issue = [&]() -> uint32_t {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(dyn_ctr, 1u);
        return v;
    };
    auto grab_resolve = [&](uint32_t v) -> int64_t {
        v = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
        const int64_t u = dyn_start + (int64_t)v * a.dyn_chunk;
        return u < n_units ? u : -1;
    };
    uint32_t rkey[QB][16];  // group-max keys of the refresh due in the current tile's epilogue
    // (LEAN: never -- the 32 keys held across the k-loop cost the registers the persistent loop needs)
    const bool early_refresh = !LEAN && a.early_refresh != 0;
    int64_t u = u0, u_end = u1, pend = -1, done = 0;
    // a.stagger: refreshes staggered over the workgroup's waves (wave v refreshes after tiles with (done + v) % RT
    // == 0) -- each tile some waves publish and read fresh keys instead of all of them every RT-th tile.  Large
    // shards only: 10M rows 2.988-2.993 -> 2.958-2.961 ms/step, k = 100 -0.3 %; 1.25M +0.7 %, 1M x 768 +1.2 %
    // (profiles/r04_refresh_stagger_ab.jsonl, same box)
    const int roff = a.stagger ? __builtin_amdgcn_readfirstlane((tid >> 6) % a.refresh_every) : 0;
    uint32_t graw = 0;
    bool issued = false;  // this run's grab is in flight (exactly one grab per run)
    if (dyn && u0 >= u1) {  // no static units (tiny launches): start in the pool
        in_static = false;
        u = grab_resolve(grab_issue());
        if (u < 0) u = u_end = 0;
        else u_end = std::min<int64_t>(u + a.dyn_chunk, n_units);
    }
    while (u < u_end) {
        if (dyn && !issued && u + 2 >= u_end) {  // a 1-unit run issues and resolves at once
            graw = grab_issue();
            issued = true;
        }
        if (dyn && u + 1 == u_end) pend = grab_resolve(graw);  // this unit's last k-steps prefetch its first unit
        const int64_t t = wave_uniform(tile_at(u));
        int64_t tn = t;
        if (u + 1 < u_end) {
            tn = tile_at(u + 1);
        } else if (pend >= 0) {
            const bool st = in_static;
            in_static = false;  // (pend is a dynamic unit)
            tn = tile_at(pend);
            in_static = st;
        }
        tn = wave_uniform(tn);
        if (t >= part_end) {  // wave-uniform; never taken with one part
            if (MODE != SCAN_COLLECT && a.use_groups) flush();
            const int64_t np_ = t / a.part_tiles;
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) gkq[qb] += (np_ - part) * a.pstride;
            part = np_;
            part_end = (part + 1) * a.part_tiles;
        }
        // a refresh applied in this tile's epilogue: its loads go out now (see refresh_load)
        const bool rdue = MODE == SCAN_FILTER && a.use_groups && early_refresh && !(HR_DIAG & 2) &&
                          ((done + 1 + roff) % a.refresh_every) == 0;
        if (rdue) {
            refresh_load(rkey);
            asm volatile("" ::: "memory");  // keeps the loads here (the compiler would sink them to their use)
        }
        f32x16 acc[QB];
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[qb][i] = 0.0f;
        // row held by this lane's slot (slot swizzle, hr_common.hpp)
        const int rg = slot_row(t, g);

        // this tile's live / mask words, issued before the k-loop: read in the epilogue, they are then
        // older than the ring loads in flight (a load issued after them would make that read wait for
        // the whole ring: vmcnt(0) at every tile)
        uint32_t allow = scalar_word(a.live, t);
        if (a.mask) allow &= scalar_word(a.mask, t);
        for (int sb = 0; sb < S; sb += P) {
            const bool same = sb + P < S;
            const int64_t nc = same ? t * S + sb + P : tn * S;
#pragma unroll
            for (int i = 0; i < P; ++i) {
                const u32x4 xf = ring[i].get();
                ring[i].load(a.rows, nc + i, lane);
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) {
                    const u32x4 qf = qs[((sb + i) * QB + qb) * 64 + lane];
                    if (HR_DIAG & 16)
                        acc[qb][i & 15] += __builtin_bit_cast(float, (qf.x ^ xf.x) & 0x3f000000u);
                    else
                        acc[qb] = mfma32<MT>(qf, xf, acc[qb]);
                }
            }
        }

        if constexpr ((HR_DIAG & 4) != 0) {  // timing build: no epilogue, the accumulators only kept live
            float s = 0.0f;
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int i = 0; i < 16; ++i) s += acc[qb][i];
            if (s == 1234.5f) a.pcnt[wg] = (uint32_t)t;
            ++done;
            if (u + 1 < u_end) {
                ++u;
            } else if (pend >= 0 && done < n_units) {
                in_static = false;
                u = pend;
                u_end = std::min<int64_t>(u + a.dyn_chunk, n_units);
                pend = -1;
                issued = false;
            } else {
                break;
            }
            continue;
        }
        // epilogue: (euclidean) approximate score, predicate, group max, threshold filter
        if (a.xnorm) {
            // euclidean: this tile's row norms, read here and only here -- a vector load issued before
            // the k-loop would make even the cosine path's epilogue wait for the whole ring (vmcnt(0)
            // at the join; the loop's trip count is not known to the compiler)
            const float xs = a.xnorm[t * 32 + rg];
            const float xmul = 2.0f;
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[qb][i] = __builtin_fmaf(xmul, acc[qb][i], -xs);
        }
        const bool ok = (allow >> rg) & 1u;
        const uint32_t row = (uint32_t)(t * 32 + rg);
        // regs: the accumulator registers (bit qb*16+i, wave-uniform) holding a passing score; the
        // append pass below visits only those (a scalar bit test per register instead of a compare +
        // ballot for all 16*QB of them: early in a scan, while the threshold is still loose, most
        // tiles append something)
        uint32_t regs = 0;
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float v = ok ? acc[qb][i] : -__builtin_inff();
                gmax[qb][i] = fmaxf(gmax[qb][i], v);
                if (FILTER) regs |= (__ballot(ok && v >= th[qb][i]) != 0 ? 1u : 0u) << (qb * 16 + i);
            }
        if (FILTER && regs && !(HR_DIAG & 1)) {
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (!((regs >> (qb * 16 + i)) & 1u)) continue;
                    const float v = acc[qb][i];
                    const bool pass = ok && v >= th[qb][i];
                    const uint64_t m = __ballot(pass);
                    if (m) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const uint32_t mh = (uint32_t)(m >> (32 * h));
                            if (priv && mh) {
                                const int q = acc_query(qb, i, h);  // compile-time: readlane is cheap
                                const uint32_t basepos = (uint32_t)__builtin_amdgcn_readlane((int)mycnt, q);
                                if (pass && half == h) {
                                    const uint32_t pos = basepos + __builtin_popcount(mh & ((1u << g) - 1u));
                                    if (pos < (uint32_t)a.capw) {
                                        if constexpr (LEAN)  // write-through (sc1): no release fence per batch
                                            __hip_atomic_store((uint64_t*)&wave_buf[q * a.capw + pos],
                                                               ((uint64_t)row << 32) | __builtin_bit_cast(uint32_t, v),
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                        else
                                            wave_buf[q * a.capw + pos] = make_float2(v, __builtin_bit_cast(float, row));
                                    }
                                }
                                mycnt += (lane == q) ? (uint32_t)__builtin_popcount(mh) : 0u;
                            } else if (!priv && mh) {
                                const int q = acc_query(qb, i, h);
                                const int leader = 32 * h + __builtin_ctz(mh);
                                uint32_t basepos = 0;
                                if (lane == leader) basepos = atomicAdd(&a.cnt[q], (uint32_t)__builtin_popcount(mh));
                                basepos = __shfl(basepos, leader, 64);
                                if (pass && half == h) {
                                    const uint32_t pos = basepos + __builtin_popcount(mh & ((1u << g) - 1u));
                                    if (pos < (uint32_t)a.cap)
                                        a.buf[(int64_t)q * a.cap + pos] = make_float2(v, __builtin_bit_cast(float, row));
                                }
                            }
                        }
                    }
                }
        }
        ++done;
        if (MODE == SCAN_FILTER && !(HR_DIAG & 2) && ((done + roff) % a.refresh_every) == 0) {
            if (rdue) refresh_apply(rkey, true, false);
            else refresh(true);
        }
        if (u + 1 < u_end) {
            ++u;
        } else if (pend >= 0 && done < n_units) {  // (done bound: termination even if the counter were corrupt)
            in_static = false;
            u = pend;
            u_end = std::min<int64_t>(u + a.dyn_chunk, n_units);
            pend = -1;
            issued = false;
        } else {
            break;
        }
    }

    if (priv && lane < QB * 32) {
        if constexpr (LEAN)
            __hip_atomic_store(&a.pcnt[wg * (QB * 32) + lane], mycnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            a.pcnt[wg * (QB * 32) + lane] = mycnt;
    }
    if (a.wave_tiles && lane == 0) a.wave_tiles[wg] = (uint32_t)done;
    if (!FILTER && a.publish) {
        // SAMPLE: publish the group maxima.  The table lives at the memory side (device-scope
        // atomics from 8 XCDs), where same-address atomics serialise, so the workgroup's 8 waves
        // first reduce in LDS (the query tile is no longer needed): one atomic per address per
        // workgroup instead of one per wave.  Waves in different row parts flush on their own.
        constexpr int NE = QB * 16 * 64;  // entries per wave
        float* red = (float*)lds;
        int64_t* partw = (int64_t*)(red + 8 * NE);
        const int wv = tid >> 6;
        __syncthreads();  // every wave is done reading the query fragments
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) red[wv * NE + (qb * 16 + i) * 64 + lane] = gmax[qb][i];
        if (lane == 0) partw[wv] = u0 < u1 ? part : -1;
        __syncthreads();
        int64_t p0 = -1;
        bool same = true;
        const int nw = blockDim.x >> 6;
        for (int v = 0; v < nw; ++v) {
            if (partw[v] < 0) continue;
            if (p0 < 0) p0 = partw[v];
            same = same && partw[v] == p0;
        }
        if (!same) {
            flush();
        } else if (p0 >= 0) {
            for (int e = tid; e < NE; e += blockDim.x) {
                float m = -__builtin_inff();
                for (int v = 0; v < nw; ++v) m = fmaxf(m, red[v * NE + e]);
                if (m > -__builtin_inff()) {
                    const int l = e & 63, ri = (e >> 6) & 15, qb = e >> 10;
                    const int q = qb * 32 + 4 * (l >> 5) + (ri & 3) + 8 * (ri >> 2);
                    atomicMax(a.mkeys + p0 * a.pstride + q * 32 + (l & 31), f2key(m));
                }
            }
        }
    }
}


// (2nd launch bound: min waves per SIMD)
template <int MT, int DT, int QB, int P, bool NT, int TPB>
__global__ __launch_bounds__(TPB, TPB >= 512 ? 2 : 1) void k_scan_sample(ScanArgs a) {
    scan_body<MT, DT, QB, P, SCAN_SAMPLE, NT, TPB>(a);
}
template <int MT, int DT, int QB, int P, bool NT, int TPB>
__global__ __launch_bounds__(TPB, TPB >= 512 ? 2 : 1) void k_scan_filter(ScanArgs a) {
    scan_body<MT, DT, QB, P, SCAN_FILTER, NT, TPB>(a);
}
template <int MT, int DT, int QB, int P, bool NT, int TPB>
__global__ __launch_bounds__(TPB, TPB >= 512 ? 2 : 1) void k_scan_collect(ScanArgs a) {
    scan_body<MT, DT, QB, P, SCAN_COLLECT, NT, TPB>(a);
}
template <int MT, int DT, int QB, int P, int MODE, bool NT, int TPB>
constexpr auto scan_kernel() {
    if constexpr (MODE == SCAN_SAMPLE) return &k_scan_sample<MT, DT, QB, P, NT, TPB>;
    else if constexpr (MODE == SCAN_FILTER) return &k_scan_filter<MT, DT, QB, P, NT, TPB>;
    else return &k_scan_collect<MT, DT, QB, P, NT, TPB>;
}

// ---------------------------------------------------------------- diagnostics
// Approximate (MFMA) scores of every row for the queries in LDS, written densely
// [Bp][n_tiles*32]; one wave per tile.  Same operand path as k_scan (used by the
// error-bound test: |approx - exact| <= E_q for every row).
template <int MT, int DT, int QB>
__global__ __launch_bounds__(256) void k_debug_approx(const uint8_t* __restrict__ rows, const uint16_t* __restrict__ qfrag,
                                                      int S, int64_t n_tiles, const float* __restrict__ xnorm,
                                                      float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    stage_lds((u32x4*)lds, (const u32x4*)qfrag, S * QB * 64);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= n_tiles) return;
    const u32x4* qs = (const u32x4*)lds;
    f32x16 acc[QB];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[qb][i] = 0.0f;
    for (int s = 0; s < S; ++s) {
        XFrag<MT, DT> x;
        x.load(rows, t * S + s, lane);
        const u32x4 xf = x.get();
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) acc[qb] = mfma32<MT>(qs[(s * QB + qb) * 64 + lane], xf, acc[qb]);
    }
    const int64_t ncol = n_tiles * 32;
    const int rg = slot_row(t, lane & 31);
    const float xs = xnorm ? xnorm[t * 32 + rg] : 0.0f;  // euclidean: same score as k_scan
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i)
            out[(int64_t)acc_query(qb, i, lane >> 5) * ncol + t * 32 + rg] =
                xnorm ? __builtin_fmaf(2.0f, acc[qb][i], -xs) : acc[qb][i];
}

// ---------------------------------------------------------------- K4: select top-kc
// One 1024-thread block per query.  Keys (u64) = f2key(score) << 32 | ~row: descending
// key order == (score desc, row asc).
__device__ inline void block_bitonic_desc(uint64_t* s, int n) {  // n power of two
    for (int k = 2; k <= n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    uint64_t x = s[i], y = s[ixj];
                    bool desc = (i & k) == 0;
                    if (desc ? (x < y) : (x > y)) {
                        s[i] = y;
                        s[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// After the SAMPLE, one row part: raise each query's floor to the kj-th largest of its 32 group maxima (one wave per
// query).  The FILTER takes th = max(floor, min over the groups) and k_select thr = max(floor, min over the final
// groups), so this starts every wave's threshold at the kj-th largest sampled group maximum instead of the smallest
// (hr_rank_for: kj = k + margin < 32).  Exact: each key is the score of a row of its group, so kj rows lie at or
// above the floor; with thr = max(floor, min_final) every row at or above thr is appended (th never exceeds thr),
// and at least kj of them (the floor's rows, or one row per group) are candidates -- the guard's premise.
static __global__ __attribute__((unused)) __launch_bounds__(256) void k_floor_kth(const uint32_t* __restrict__ mkeys,
                                                                                   float* __restrict__ floor_q, int B,
                                                                                   int kj) {
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= B) return;  // (wave-uniform)
    const uint32_t k = mkeys[(int64_t)q * 32 + (threadIdx.x & 31)];
    const float t = half_kth_largest(key2f(k > HR_KEY_NEG_INF ? k : HR_KEY_NEG_INF), kj);
    if ((threadIdx.x & 63) == 0) floor_q[q] = fmaxf(floor_q[q], t);
}

// The same with row parts (np > 1: 32 np groups, keys [np][Bp][32]): one 64-thread block per query ranks its
// 32 np <= 256 keys by counting and raises the floor to the kj-th largest.
static __global__ __attribute__((unused)) __launch_bounds__(64) void k_floor_kth_parts(const uint32_t* __restrict__ mkeys,
                                                                                        float* __restrict__ floor_q,
                                                                                        int Bp, int np, int kj) {
    __shared__ float v[256];
    const int q = blockIdx.x, m = np * 32;
    for (int i = threadIdx.x; i < m; i += 64) {
        const uint32_t k = mkeys[((int64_t)(i >> 5) * Bp + q) * 32 + (i & 31)];
        v[i] = key2f(k > HR_KEY_NEG_INF ? k : HR_KEY_NEG_INF);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += 64) {
        int gt = 0, ge = 0;
        for (int j = 0; j < m; ++j) {
            gt += v[j] > v[i];
            ge += v[j] >= v[i];
        }
        if (gt < kj && ge >= kj) floor_q[q] = fmaxf(floor_q[q], v[i]);  // (every such thread holds the same value)
    }
}

constexpr int kRankMax = 1024;  // candidate sets up to this size are ranked by counting, larger ones sorted

static __global__ __attribute__((unused)) __launch_bounds__(1024) void k_select(const uint32_t* __restrict__ cnt, const float2* __restrict__ buf,
                                                 int cap, const uint32_t* __restrict__ pcnt,
                                                 const float2* __restrict__ pbuf, int W, int capw, int Bq, int Bp,
                                                 const uint32_t* __restrict__ mkeys, int np,
                                                 const float* __restrict__ floor_q, int use_groups, int B, int kc,
                                                 uint32_t* __restrict__ sel_rows, int* __restrict__ sel_cnt,
                                                 float* __restrict__ bound_approx, int* __restrict__ overflow,
                                                 const uint32_t* __restrict__ force_ovf = nullptr) {
    // all LDS in the dynamic region (G17): 16 B of scalars, then the sort keys
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int& m_sh = *(int*)smem;
    int& ovf_sh = *(int*)(smem + 4);
    float& thr_sh = *(float*)(smem + 8);
    uint64_t* keys = (uint64_t*)(smem + 16);
    const int q = blockIdx.x;
    if (q >= B) return;
    const int tid = threadIdx.x;
    if (tid < 64) {
        // min over the 32*np group maxima of this query (mkeys [np][Bp][32])
        float f = use_groups ? __builtin_inff() : -__builtin_inff();
        if (use_groups)
            for (int j = tid; j < np * 32; j += 64) {
                uint32_t k = mkeys[((int64_t)(j >> 5) * Bp + q) * 32 + (j & 31)];
                f = fminf(f, key2f(k > HR_KEY_NEG_INF ? k : HR_KEY_NEG_INF));
            }
        for (int off = 32; off >= 1; off >>= 1) f = fminf(f, __shfl_xor(f, off, 64));
        if (tid == 0) {
            thr_sh = fmaxf(f, floor_q[q]);
            m_sh = 0;
            // force_ovf: the persistent FILTER's batch did not complete (k_persist_wait gave up): its candidate
            // regions are partial, so the batch goes to the exact collect pass through the guard
            ovf_sh = (force_ovf && __hip_atomic_load(force_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 1 : 0;
        }
    }
    __syncthreads();
    const float thr = thr_sh;
    bool ovf = false;
    auto push = [&](float2 e) {
        if (e.x >= thr) {
            int p = atomicAdd(&m_sh, 1);
            if (p < cap)
                keys[p] = ((uint64_t)f2key(e.x) << 32) | (uint64_t)(0xFFFFFFFFu - __builtin_bit_cast(uint32_t, e.y));
            else
                ovf = true;
        }
    };
    if (pcnt) {  // private per-wave regions of the FILTER scan: [group][W][Bq] (the query's group only)
        const int64_t gw0 = (int64_t)(q / Bq) * W;
        const int ql = q % Bq;
        for (int w = tid; w < W; w += blockDim.x) {
            const uint32_t c = pcnt[(gw0 + w) * Bq + ql];
            if (c > (uint32_t)capw) ovf = true;
            const int n = c < (uint32_t)capw ? (int)c : capw;
            for (int j = 0; j < n; ++j) push(pbuf[((gw0 + w) * Bq + ql) * capw + j]);
        }
    } else {
        const uint32_t c = cnt[q];
        if (c > (uint32_t)cap) ovf = true;
        const int n = c < (uint32_t)cap ? (int)c : cap;
        for (int i = tid; i < n; i += blockDim.x) push(buf[(int64_t)q * cap + i]);
    }
    if (ovf) atomicOr(&ovf_sh, 1);
    __syncthreads();
    const int m = m_sh < cap ? m_sh : cap;
    const int keep = m < kc ? m : kc;
    if (m <= kRankMax) {
        // rank by counting: keys are distinct (row in the low word), so a key's rank is the number of
        // larger keys; every thread reads the same LDS word per step (broadcast), no sort stages
        uint64_t* kth_sh = (uint64_t*)(smem + 8);  // reuses thr_sh's slot (thr already read)
        for (int i = tid; i < m; i += blockDim.x) {
            const uint64_t key = keys[i];
            int rank = 0;
            for (int j = 0; j < m; ++j) rank += keys[j] > key ? 1 : 0;
            if (rank < kc) sel_rows[q * kc + rank] = 0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFu);
            if (rank == kc - 1) *kth_sh = key;
        }
        for (int i = keep + tid; i < kc; i += blockDim.x) sel_rows[q * kc + i] = 0xFFFFFFFFu;
        __syncthreads();
        if (tid == 0) {
            sel_cnt[q] = keep;
            bound_approx[q] = (m >= kc && kc > 0) ? key2f((uint32_t)(*kth_sh >> 32)) : thr;
            overflow[q] = ovf_sh;
        }
        return;
    }
    int p2 = 1;
    while (p2 < m) p2 <<= 1;
    for (int i = m + tid; i < p2; i += blockDim.x) keys[i] = 0;
    __syncthreads();
    if (p2 > 1) block_bitonic_desc(keys, p2);
    for (int i = tid; i < kc; i += blockDim.x)
        sel_rows[q * kc + i] = i < keep ? 0xFFFFFFFFu - (uint32_t)(keys[i] & 0xFFFFFFFFu) : 0xFFFFFFFFu;
    if (tid == 0) {
        sel_cnt[q] = keep;
        bound_approx[q] = (m >= kc && kc > 0) ? key2f((uint32_t)(keys[kc - 1] >> 32)) : thr;
        overflow[q] = ovf_sh;
    }
}

// ---------------------------------------------------------------- K5: exact rescoring
// One wave per (query, candidate slot): canonical fp64 dot of the stored row and the
// normalised fp32 query.  Slot 0 also writes the shard bound = bound_approx + E_q.
template <int DT>
__global__ __launch_bounds__(256) void k_rescore(const uint8_t* __restrict__ rows, int S, int dpad,
                                                 const float* __restrict__ q32, const uint32_t* __restrict__ sel_rows,
                                                 const int* __restrict__ sel_cnt, int B, int kc, int64_t row_offset,
                                                 const float* __restrict__ bound_approx,
                                                 const double* __restrict__ qerr, double max_norm, double gamma,
                                                 double u_x, int metric, const int* __restrict__ overflow,
                                                 Cand* __restrict__ out, double* __restrict__ bound_out, int sG = 1,
                                                 int ss = 0) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wid >= (int64_t)B * kc) return;
    const int q = (int)(wid / kc), c = (int)(wid % kc);
    const double qn2 = qerr[4 * q + 2];
    if (c == 0 && lane == 0) {
        float ba = bound_approx[q];
        const double E = guard_e(qerr + 4 * q, max_norm, gamma, u_x, metric);
        double bd = (ba == -__builtin_inff()) ? -__builtin_inf() : (double)ba + E;
        // euclidean: scan-score space -> similarity space (+ the rounding slack, an upper bound)
        if (metric == L2 && bd > -__builtin_inf()) bd = (1.0 - qn2) + bd + euclid_slack(qn2, max_norm);
        if (overflow && overflow[q]) bd = __builtin_inf();
        bound_out[q] = bd;
    }
    if (c >= sel_cnt[q]) {
        if (lane == 0) out[wid] = Cand{-__builtin_inf(), -1};
        return;
    }
    const int64_t r = (int64_t)sel_rows[q * kc + c];
    const float* qv = q32 + (int64_t)q * dpad;
    double p = 0.0, x2 = 0.0;
#pragma unroll 8
    for (int d = lane; d < dpad; d += 64) {
        const double x = (double)load_elem<DT>(rows, S, r, d);
        p = p + x * (double)qv[d];
        if (metric == L2) x2 = x2 + x * x;
    }
    p = wave_butterfly_sum(p);
    if (metric == L2) {
        x2 = wave_butterfly_sum(x2);
        p = euclid_score(qn2, p, x2);
    }
    if (lane == 0) out[wid] = Cand{p, stripe_row(r, sG, ss) + row_offset};
}

// ---------------------------------------------------------------- K4/C1: merge shards
// One block per query over G*kc exact candidates.  Sort key: (d2key(score) desc, row asc).
// Rank g's candidates start at cand + g*cstride bytes, its bounds at bounds + g*bstride bytes (one
// packed all-gather record per rank: [B*kc Cand][B double]).
static __global__ __attribute__((unused)) __launch_bounds__(256) void k_merge(const uint8_t* __restrict__ cand, const uint8_t* __restrict__ bounds,
                                               int64_t cstride, int64_t bstride, int G,
                                               int B, int kc, int k, float* __restrict__ scores_out,
                                               int64_t* __restrict__ rows_out, double* __restrict__ kth_out,
                                               int32_t* __restrict__ fail_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int q = blockIdx.x;
    if (q >= B) return;
    const int n = G * kc;
    int p2 = 1;
    while (p2 < n) p2 <<= 1;
    uint64_t* ks = (uint64_t*)smem;  // score keys
    int64_t* rs = (int64_t*)(ks + p2);
    for (int i = threadIdx.x; i < p2; i += blockDim.x) {
        if (i < n) {
            const int gi = i / kc, ci = i % kc;
            Cand e = ((const Cand*)(cand + gi * cstride))[(int64_t)q * kc + ci];
            if (e.row < 0) {
                ks[i] = 0;
                rs[i] = INT64_MAX;
            } else {
                ks[i] = d2key(e.score);
                rs[i] = e.row;
            }
        } else {
            ks[i] = 0;
            rs[i] = INT64_MAX;
        }
    }
    __syncthreads();
    auto key_of = [](uint64_t key) {
        uint64_t u = (key & 0x8000000000000000ull) ? (key & 0x7FFFFFFFFFFFFFFFull) : ~key;
        return __builtin_bit_cast(double, u);
    };
    if (n <= kRankMax) {
        // rank by counting over (score key desc, row asc); invalid slots (key 0, row INT64_MAX) rank last
        // two scalars after the keys/rows (all LDS in the dynamic region, like k_select)
        int& valid_sh = *(int*)(smem + (size_t)p2 * 16);
        uint64_t& kth_key_sh = *(uint64_t*)(smem + (size_t)p2 * 16 + 8);
        if (threadIdx.x == 0) {
            valid_sh = 0;
            kth_key_sh = 0;
        }
        __syncthreads();
        int myvalid = 0;
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const uint64_t a = ks[i];
            const int64_t ra = rs[i];
            if (ra == INT64_MAX) continue;
            ++myvalid;
            int rank = 0;
            for (int j = 0; j < n; ++j) {
                const uint64_t b = ks[j];
                rank += (b > a || (b == a && rs[j] < ra)) ? 1 : 0;
            }
            if (rank < k) {
                scores_out[(int64_t)q * k + rank] = (float)key_of(a);
                rows_out[(int64_t)q * k + rank] = ra;
            }
            if (rank == k - 1) kth_key_sh = a;
        }
        if (myvalid) atomicAdd(&valid_sh, myvalid);
        __syncthreads();
        const int valid = valid_sh;
        for (int i = valid + threadIdx.x; i < k; i += blockDim.x) {
            scores_out[(int64_t)q * k + i] = -__builtin_inff();
            rows_out[(int64_t)q * k + i] = -1;
        }
        if (threadIdx.x == 0) {
            double maxb = -__builtin_inf();
            for (int gi = 0; gi < G; ++gi) maxb = fmax(maxb, ((const double*)(bounds + gi * bstride))[q]);
            double sk = -__builtin_inf();
            if (valid >= k && k > 0) sk = key_of(kth_key_sh);  // fewer than k: every remaining row is a candidate
            kth_out[q] = sk;
            bool fail = maxb > -__builtin_inf() && (valid < k || !(sk > maxb));
            fail_out[q] = fail ? 1 : 0;
        }
        return;
    }
    for (int kk = 2; kk <= p2; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < p2; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    uint64_t a = ks[i], b = ks[ixj];
                    int64_t ra = rs[i], rb = rs[ixj];
                    bool a_first = a > b || (a == b && ra < rb);
                    bool desc = (i & kk) == 0;
                    if (desc ? !a_first : a_first) {
                        ks[i] = b;
                        ks[ixj] = a;
                        rs[i] = rb;
                        rs[ixj] = ra;
                    }
                }
            }
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        int valid = 0;
        for (int i = 0; i < p2 && rs[i] != INT64_MAX; ++i) ++valid;
        double maxb = -__builtin_inf();
        for (int gi = 0; gi < G; ++gi) maxb = fmax(maxb, ((const double*)(bounds + gi * bstride))[q]);
        double sk = -__builtin_inf();
        for (int i = 0; i < k; ++i) {
            if (i < valid) {
                scores_out[(int64_t)q * k + i] = (float)key_of(ks[i]);
                rows_out[(int64_t)q * k + i] = rs[i];
            } else {
                scores_out[(int64_t)q * k + i] = -__builtin_inff();
                rows_out[(int64_t)q * k + i] = -1;
            }
        }
        if (valid >= k && k > 0) sk = key_of(ks[k - 1]);  // fewer than k: every remaining row is a candidate
        kth_out[q] = sk;
        bool fail = maxb > -__builtin_inf() && (valid < k || !(sk > maxb));
        fail_out[q] = fail ? 1 : 0;
    }
}

// ---------------------------------------------------------------- get_by_id: de-tile rows
template <int DT>
__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ rows, int S, int dim,
                                                const int64_t* __restrict__ idx, int64_t n, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= n) return;
    const int64_t r = idx[w];
    for (int d = lane; d < dim; d += 64) out[w * dim + d] = load_elem<DT>(rows, S, r, d);
}

}  // namespace hr
