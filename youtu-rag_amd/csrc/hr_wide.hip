// hr_wide.hip -- the 128-query FILTER pass: one read of every corpus tile for 128 queries (two 64-query groups).
//
// k_scan holds one 64-query group's A-fragments in LDS for the whole depth (128 KiB at D = 1024), so a batch of
// 65-128 queries used to be two groups of workgroups streaming the same tiles, the second reading them from L2
// (query groups): bounded by that access shape at 4.4-4.6 ms per 10M x 1024 batch, 1.13x the HBM
// bytes.  Here ONE workgroup serves 128 queries and every tile is read from HBM once:
//  * 8 waves (two per SIMD), one tile per wave per round; each wave scores its tile against all 128 queries
//    (4 MFMA blocks of 32 queries, 64 accumulators);
//  * the queries' fragments do not fit in LDS (256 KiB at D = 1024), so they stream through it in depth
//    windows of 8 k-steps (2 groups x 8 k-steps x 2 blocks x 1 KiB = 32 KiB, double-buffered) that the eight
//    waves walk in lock step -- one barrier per window; each window is staged by LDS-DMA
//    (buffer_load ... lds: L2 -> LDS with no registers and no ds_write) one window ahead, and the first
//    windows of every tile stay resident in LDS for the whole launch;
//  * the corpus streams through a 16-deep register ring (two halves of 8 k-steps, non-temporal buffer loads,
//    one V# per tile);
//  * per-query thresholds live in LDS, and so do the group maxima: one table per workgroup raised with ds_max,
//    only by scores at or above their query's threshold (nothing below the minimum over the groups can raise
//    it, so these updates are as rare as the appends); at a refresh the waves swap their share of the table
//    out, publish it (atomicMax only where it beats the global key) and recompute the thresholds.  The final
//    keys may then sit below a group's true maximum, which only lowers k_select's threshold: the candidates
//    still hold every row at or above the scan's highest threshold, and 32 of them (one per group) lie at or
//    above it, so the kc-th best candidate bounds every dropped row;
//  * candidates go to k_scan's private per-(group, wave) regions, so k_select reads them unchanged.
// Timing prototype and its measurements: tools/q128_proto.hip.  (A four-wave tile-pair form was built in round 3
// and measured slower, 4.0-4.2 vs 3.58 ms per 10M x 1024 pass: its epilogue ran on the only wave of its SIMD.)
// Scope: bf16 / f16 / fp32 corpora, D a multiple of 256 up to 1024 (S = 16, 32, 48, 64 k-steps), row parts up to
// wide_max_parts, cosine / inner product / euclidean, no tile list -- every other FILTER keeps k_scan's query groups.
#include "hr_internal.hpp"
#include "hr_kernels.hpp"

namespace hr {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWN = 8;       // k-steps per query window
// eight-wave form: depth windows kept resident in LDS for the whole launch (the rest stream): 2 x 32 KiB
constexpr int kResidentWindows = 2;

// Two waves per SIMD, one tile per wave per round: each staged window serves the workgroup's eight tiles, and a
// wave's epilogue runs beside the other wave's MFMAs on its SIMD -- with 128 queries per tile a third of the tiles
// hold a candidate (10M rows, k = 10), so the epilogue is not rare.  A refresh splits each query block's 16
// registers between two waves.
template <int MT, int DT, int S_, bool PARTS = false>
__global__ __launch_bounds__(512, 1) void k_filter_wide8(ScanArgs a) {
    // fp32 rows: 2 KiB k-step chunks (two 16-byte loads per lane, rounded to the MFMA type on use, as k_scan's
    // XFrag<F32>), so a window / ring half is 4 k-steps -- the same 8 loads and 16 KiB in flight per wave
    constexpr int LPC = DT == F32 ? 2 : 1;  // 16-byte loads per lane per k-step chunk
    constexpr int WN = kWN / LPC;           // k-steps per query window and per ring half
    static_assert(S_ % (2 * WN) == 0, "an even number of windows per tile (the ring halves alternate by window)");
    constexpr int NW = S_ / WN;
    constexpr int WQ = WN * 4 * 64;   // u32x4 per window buffer: [group][k-step][block][lane]
    constexpr int PER = WQ / 512;     // LDS-DMA chunks per thread per window
    // rounds between refreshes (k_scan's tiles per refresh: 4).  At 10M rows, B = 128, every 1 / 2 / 4 rounds
    // appended 850 / 897 / 1128 candidates per query and took 3.51 / 3.41 / 3.32 ms: the refresh costs more than
    // the candidates it saves
    const int RT = std::max(1, a.refresh_every);
    // windows [0, NR) stay resident for the whole launch; [NR, NW) stream through lb0 / lb1 (window w in
    // buffer (w - NR) & 1), each staged during the window before it
    // (LDS: (NR + 2) windows + the 16.5 KiB key / threshold tables within 160 KiB: 2 windows of 32 KiB resident,
    // or 6 of 16 KiB for fp32 rows)
    // With row parts (PARTS: kc > 32, np parts of 32 groups each) the per-part key tables take the resident
    // windows' LDS: none stay resident
    constexpr int NR_MAX = PARTS ? 0 : (DT == F32 ? 3 * kResidentWindows : kResidentWindows);
    constexpr int NR = NW < NR_MAX ? NW : NR_MAX;
    constexpr int KP = PARTS ? wide_max_parts(DT) : 1;  // key tables (row parts) in LDS
    __shared__ __attribute__((aligned(16))) u32x4 lres[NR > 0 ? NR : 1][WQ];
    __shared__ __attribute__((aligned(16))) u32x4 lb0[WQ];
    __shared__ __attribute__((aligned(16))) u32x4 lb1[WQ];
    __shared__ __attribute__((aligned(16))) float th_lds[128];
    __shared__ __attribute__((aligned(16))) uint32_t G[KP][4][16][64];
    // row parts: per part the min over its 32 groups' keys at that part's last refresh, per query
    __shared__ __attribute__((aligned(16))) float pmin[KP][128];
    const int np = PARTS ? a.np : 1;

    // wv: wave-uniform (readfirstlane), so every per-wave base below (candidate regions, tile positions) is a scalar
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6), half = lane >> 5,
              g = lane & 31;
    const int64_t W = (int64_t)gridDim.x * 8;
    const int64_t wr = (int64_t)wv * gridDim.x + blockIdx.x;
    const int64_t n_tiles = a.n_units;
    // row parts: deal position s takes tile (s % np) * part_tiles + s / np, so every round spans all parts (a part's
    // group maxima bound nothing until every part has some: parts dealt one after another would leave the
    // threshold at the floor until the last part); positions past the last part's end hold no tile
    const int64_t n_pos = PARTS ? (int64_t)np * a.part_tiles : n_tiles;
    const int64_t rounds = (n_pos + W - 1) / W;
    const int64_t full_rounds = n_pos / W;
    auto tile_at = [&](int64_t u) -> int64_t {  // -1: no tile this round (zero-record V#)
        int64_t pos = wr;
        if (HR_ROTATE_ROUNDS && u < full_rounds) {
            pos += (int64_t)((uint32_t)((uint64_t)u * 2654435761ull) % (uint32_t)W);
            if (pos >= W) pos -= W;
        }
        int64_t t = u * W + pos;
        if constexpr (PARTS) {
            const uint32_t s = (uint32_t)t;
            t = t < n_pos ? (int64_t)(s % (uint32_t)np) * a.part_tiles + (int64_t)(s / (uint32_t)np) : n_tiles;
        }
        return wave_uniform(t < n_tiles ? t : -1);
    };
    auto rsrc = [&](int64_t t) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(a.rows + (t < 0 ? 0 : t) * (S_ * 1024 * LPC)), (short)0,
                                                 t < 0 ? 0 : S_ * 1024 * LPC, 0x00020000);
    };
    const int voff = lane * 16;
    // ring slot i (k-step i of a window) holds LPC 16-byte loads: ring[i * LPC + l]
    auto ld = [&](u32x4* ring, int i, __amdgpu_buffer_rsrc_t r, int chunk) {
#pragma unroll
        for (int l = 0; l < LPC; ++l)
            ring[i * LPC + l] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, chunk * 1024 * LPC + l * 1024, 2);  // nt
    };
    auto xfrag = [&](const u32x4* ring, int i) -> u32x4 {  // the MFMA B operand of ring slot i
        if constexpr (LPC == 1) {
            return ring[i];
        } else {
            typedef float f32x8 __attribute__((ext_vector_type(8)));
            const f32x8 f = __builtin_shufflevector(__builtin_bit_cast(f32x4, ring[2 * i]), __builtin_bit_cast(f32x4, ring[2 * i + 1]),
                                                    0, 1, 2, 3, 4, 5, 6, 7);
            if constexpr (MT == BF16) return __builtin_bit_cast(u32x4, __builtin_convertvector(f, bf16x8));
            else return __builtin_bit_cast(u32x4, __builtin_convertvector(f, f16x8));
        }
    };
    const __amdgpu_buffer_rsrc_t qr =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.qfrag, (short)0, 2 * S_ * 2 * 1024, 0x00020000);
    // chunk c = j * 512 + tid of a window buffer: group j / (PER / 2), position (j % (PER / 2)) * 512 + tid in it
    auto stage = [&](int w, u32x4* buf) {
        int vo = tid * 16;
        asm volatile("" : "+v"(vo));
#pragma unroll
        for (int j = 0; j < PER; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (__attribute__((address_space(3))) void*)(buf + j * 512 + wv * 64), 16, vo,
                                                     (j / (PER / 2)) * S_ * 2048 + w * WN * 2048 + (j % (PER / 2)) * 8192, 0, 0);
    };
    u32x4 ra[WN * LPC], rb[WN * LPC];
    {
        const auto r0 = rsrc(tile_at(0));
#pragma unroll
        for (int i = 0; i < WN; ++i) ld(ra, i, r0, i);
#pragma unroll
        for (int i = 0; i < WN; ++i) ld(rb, i, r0, WN + i);
    }
#pragma unroll
    for (int w = 0; w < NR; ++w) stage(w, lres[w]);
    if constexpr (NR < NW) stage(NR, lb0);

    // refresh share of this wave: block wb = wv & 3, registers [8 * (wv >> 2), + 8)
    const int wb = wv & 3, i0 = 8 * (wv >> 2);
    uint32_t* const keys_w = a.mkeys + (wb * 32 + 4 * half) * 32 + g;
    auto qoff_i = [](int i) { return 32 * ((i & 3) + 8 * (i >> 2)); };
    // refresh of part p (p = 0 without parts): publish this wave's share of G[p] (m) where it beats the global key,
    // the min over the part's 32 groups -> pmin, the threshold = max(old, floor, min over the parts' mins).  With
    // parts, each refresh serves one part in rotation: the other parts' mins are older, hence lower -- still a
    // valid bound on the (32 np)-th best score
    auto publish_refresh = [&](const float (&m)[8], const uint32_t (&key)[8], bool publish, int p) {
        uint32_t* const kp = keys_w + (int64_t)p * a.pstride;
        float th8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = i0 + j;
            uint32_t k = key[j] > HR_KEY_NEG_INF ? key[j] : HR_KEY_NEG_INF;
            if (publish && a.publish && m[j] > key2f(k)) {
                atomicMax(kp + qoff_i(i), f2key(m[j]));
                k = f2key(m[j]);
            }
            float f = key2f(k);
            f = half_min32(f);
            th8[j] = f;
        }
        if (g == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = i0 + j;
                const int q = wb * 32 + (i & 3) + 8 * (i >> 2) + 4 * half;
                float f = th8[j];
                if constexpr (PARTS) {
                    pmin[p][q] = f;
                    for (int p2 = 0; p2 < np; ++p2) f = fminf(f, pmin[p2][q]);
                }
                th_lds[q] = fmaxf(th_lds[q], fmaxf(f, a.floor_q[q]));
            }
        }
    };
    if (tid < 128) th_lds[tid] = -__builtin_inff();
    for (int p = 0; p < KP; ++p) {
#pragma unroll
        for (int j = 0; j < 8; ++j) G[p][wb][i0 + j][lane] = HR_KEY_NEG_INF;
        if (tid < 128) pmin[p][tid] = -__builtin_inff();  // (parts beyond np stay out of the minimum below)
    }
    __syncthreads();
    if constexpr (PARTS) {  // every part's minimum first, then the thresholds from all of them
        if (tid < 128)
            for (int p = np; p < KP; ++p) pmin[p][tid] = __builtin_inff();
    }
    for (int p = 0; p < np; ++p) {
        uint32_t key[8];
        float m[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            key[j] = __hip_atomic_load(keys_w + (int64_t)p * a.pstride + qoff_i(i0 + j), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            m[j] = -__builtin_inff();
        }
        publish_refresh(m, key, false, p);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    uint32_t mycnt[2] = {0u, 0u};
    float2* const reg0 = a.pbuf + (wr * 64) * a.capw;
    float2* const reg1 = a.pbuf + ((W + wr) * 64) * a.capw;
    auto allow_word = [&](int64_t t) -> uint32_t {
        if (t < 0) return 0u;
        uint32_t w0 = scalar_word(a.live, t);
        if (a.mask) w0 &= scalar_word(a.mask, t);
        return w0;
    };
    uint32_t next_allow = allow_word(tile_at(0));
    for (int64_t u = 0; u < rounds; ++u) {
        const int64_t t = tile_at(u), tn = tile_at(u + 1);
        const auto rt = rsrc(t), rn = rsrc(tn);
        const uint32_t allow = next_allow;
        next_allow = allow_word(tn);
        // workgroup-uniform; staggered over the workgroups, so each round a 1 / RT share of them publishes and
        // reads fresh keys instead of all at once (15-17 % fewer candidates at the same refresh rate)
        const bool refresh = u > 0 && ((u + blockIdx.x) % RT) == 0;
        // the part whose keys the refresh prefetches (rotating; a refresh serves every part) and the part of this
        // wave's tile (its G table)
        const int pr = PARTS ? (int)((u / RT) % np) : 0;
        const int pt = PARTS && t >= 0 ? (int)(t / a.part_tiles) : 0;
        f32x16 acc[4];
#pragma unroll
        for (int qb = 0; qb < 4; ++qb)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[qb][i] = 0.0f;
        uint32_t key[8];
        const int rg = slot_row(t < 0 ? 0 : t, g);  // row of the tile held by this lane's slot
        float xs = 0.0f;  // euclidean: the row's fp32 |x|^2 (score 2 q.x - |x|^2, as k_scan)
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            u32x4(&ring)[WN * LPC] = (w & 1) ? rb : ra;
            if (w >= NR && (w > NR || u > 0)) {
                // streamed window w: this wave's DMA for it landed (the previous window's 8 ring refills were
                // issued after it), every wave's (barrier); every wave is also through window w - 1, whose
                // buffer the next staging refills
                asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            // stage window w + 1 when it streams (window NR, the first, is staged during window NR - 1: its
            // buffer was last read by window NW - 2 of the previous tile, which every wave finished before
            // window NW - 1's barrier)
            if (w + 1 >= NR && w + 1 < NW) stage(w + 1, ((w + 1 - NR) & 1) ? lb1 : lb0);
            // no resident windows (row parts): window 0 of the next tile streams too, staged during the last window
            // into lb0 (NW is even: window NW - 2, lb0's last reader, is done everywhere at this window's barrier)
            if constexpr (NR == 0)
                if (w == NW - 1 && u + 1 < rounds) stage(0, lb0);
            if (refresh && w == NW - 1) {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    key[j] = __hip_atomic_load(keys_w + (int64_t)pr * a.pstride + qoff_i(i0 + j), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
            }
            // (issued before the last window's refills, like the keys: read after the k-loop, it waits for nothing
            // newer than itself)
            if (a.xnorm && w == NW - 1 && t >= 0) xs = a.xnorm[t * 32 + rg];
            unsigned qo = (unsigned)lane;
            asm volatile("" : "+v"(qo));
            const u32x4* qs = (w < NR ? lres[w < NR ? w : 0] : (((w - NR) & 1) ? lb1 : lb0)) + qo;
            auto qfrag = [&](int i, int qb) { return qs[((qb >> 1) * WN * 2 + i * 2 + (qb & 1)) * 64]; };
            u32x4 qf[2][4];
#pragma unroll
            for (int qb = 0; qb < 4; ++qb) qf[0][qb] = qfrag(0, qb);
#pragma unroll
            for (int i = 0; i < WN; ++i) {
                if (i + 1 < WN) {
#pragma unroll
                    for (int qb = 0; qb < 4; ++qb) qf[(i + 1) & 1][qb] = qfrag(i + 1, qb);
                }
                const u32x4 x = xfrag(ring, i);
                if (w + 2 < NW) ld(ring, i, rt, (w + 2) * WN + i);
                else ld(ring, i, rn, (w + 2 - NW) * WN + i);
#pragma unroll
                for (int qb = 0; qb < 4; ++qb) acc[qb] = mfma32<MT>(qf[i & 1][qb], x, acc[qb]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }

        // epilogue: fast test (acc - th >= 0 exactly when acc >= th, a flushed denormal difference only adds a
        // false positive), then, for a tile with a
        // hit, the exact per-register compares, group maxima (ds_max, scores at or above their threshold
        // only) and appends
        const bool ok = (allow >> rg) & 1u;
        if (a.xnorm) {
#pragma unroll
            for (int qb = 0; qb < 4; ++qb)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[qb][i] = __builtin_fmaf(2.0f, acc[qb][i], -xs);
        }
        float d = -__builtin_inff();
#pragma unroll
        for (int qb = 0; qb < 4; ++qb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const f32x4 t4 = *(const f32x4*)&th_lds[qb * 32 + 8 * r + 4 * half];
#pragma unroll
                for (int c = 0; c < 4; ++c) d = fmaxf(d, acc[qb][4 * r + c] - t4[c]);
            }
        if (__ballot(ok && d >= 0.0f)) {
            // the registers holding a passing score: per-lane bits, OR-reduced over the wave, then a loop over
            // the set bits only (usually one or two) that reads each register by a uniform dynamic index.  The
            // workgroup's eight waves meet at the next window barrier, so a long epilogue on one wave holds all
            const uint32_t row = (uint32_t)(t * 32 + rg);
            uint32_t bl = 0, bh = 0;
#pragma unroll
            for (int qb = 0; qb < 4; ++qb)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const f32x4 t4 = *(const f32x4*)&th_lds[qb * 32 + 8 * r + 4 * half];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const int b = qb * 16 + 4 * r + c;
                        const bool p = ok && acc[qb][4 * r + c] >= t4[c];
                        if (b < 32) bl |= p ? (1u << b) : 0u;
                        else bh |= p ? (1u << (b - 32)) : 0u;
                    }
                }
            uint64_t bits = ((uint64_t)wave_or(bh) << 32) | wave_or(bl);
            while (bits) {
                const int b = __builtin_ctzll(bits);  // wave-uniform
                bits &= bits - 1;
                const int qb = b >> 4, i = b & 15;
                // register b by uniform selects (16 per read; a dynamic register index spilled)
                float v = 0.0f;
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
                    for (int j = 0; j < 16; ++j) v = (b == q4 * 16 + j) ? acc[q4][j] : v;
                const int ql0 = (qb & 1) * 32 + (i & 3) + 8 * (i >> 2);  // query within its group, half 0
                const bool pass = ok && v >= th_lds[(qb >> 1) * 64 + ql0 + 4 * half];
                const uint64_t msk = __ballot(pass);
                if (pass) atomicMax(&G[pt][qb][i][lane], f2key(v));
                if (!msk) continue;
                const int gq = qb >> 1;
                uint32_t cnt = gq ? mycnt[1] : mycnt[0];
                float2* const reg = gq ? reg1 : reg0;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const uint32_t mh = (uint32_t)(msk >> (32 * hh));
                    if (!mh) continue;
                    const int ql = ql0 + 4 * hh;
                    const uint32_t basepos = (uint32_t)__builtin_amdgcn_readlane((int)cnt, ql);
                    if (pass && half == hh) {
                        const uint32_t pos = basepos + __builtin_popcount(mh & ((1u << g) - 1u));
                        if (pos < (uint32_t)a.capw) reg[ql * a.capw + pos] = make_float2(v, __builtin_bit_cast(float, row));
                    }
                    cnt += (lane == ql) ? (uint32_t)__builtin_popcount(mh) : 0u;
                }
                if (gq) mycnt[1] = cnt;
                else mycnt[0] = cnt;
            }
        }
        if (refresh) {  // this wave's share of block wb, swapped out of G -- every part's (part pr's keys prefetched)
            for (int p = 0; p < np; ++p) {
                const int pp = PARTS ? (pr + p < np ? pr + p : pr + p - np) : 0;
                if (PARTS && p > 0) {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        key[j] = __hip_atomic_load(keys_w + (int64_t)pp * a.pstride + qoff_i(i0 + j), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                }
                float m[8];
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    m[j] = key2f(__hip_atomic_exchange(&G[pp][wb][i0 + j][lane], (uint32_t)HR_KEY_NEG_INF,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                publish_refresh(m, key, true, pp);
            }
        }
    }
    a.pcnt[wr * 64 + lane] = mycnt[0];
    a.pcnt[(W + wr) * 64 + lane] = mycnt[1];
}

template <int MT, int DT, int S_>
int launch_t(int cus, const ScanArgs& a, hipStream_t st) {
    if (a.np > 1) hipLaunchKernelGGL((k_filter_wide8<MT, DT, S_, true>), dim3((unsigned)cus), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((k_filter_wide8<MT, DT, S_>), dim3((unsigned)cus), dim3(512), 0, st, a);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}

}  // namespace

bool wide_filter_ok(int dtype, int S) { return S == 16 || S == 32 || S == 48 || S == 64; }

int launch_filter_wide(int mt, int dtype, int S, int cus, const ScanArgs& a, hipStream_t st) {
#define HR_WIDE_CASE(MTv, DTv, Sv) \
    if (mt == MTv && dtype == DTv && S == Sv) return launch_t<MTv, DTv, Sv>(cus, a, st);
    HR_WIDE_CASE(BF16, BF16, 64) HR_WIDE_CASE(BF16, BF16, 48) HR_WIDE_CASE(BF16, BF16, 32) HR_WIDE_CASE(BF16, BF16, 16)
    HR_WIDE_CASE(F16, F16, 64) HR_WIDE_CASE(F16, F16, 48) HR_WIDE_CASE(F16, F16, 32) HR_WIDE_CASE(F16, F16, 16)
    // fp32 rows: the MFMA type follows the metric (mfma_type: cosine -> f16, inner product -> bf16)
    HR_WIDE_CASE(F16, F32, 64) HR_WIDE_CASE(F16, F32, 48) HR_WIDE_CASE(F16, F32, 32) HR_WIDE_CASE(F16, F32, 16)
    HR_WIDE_CASE(BF16, F32, 64) HR_WIDE_CASE(BF16, F32, 48) HR_WIDE_CASE(BF16, F32, 32) HR_WIDE_CASE(BF16, F32, 16)
#undef HR_WIDE_CASE
    return HR_E_UNSUPPORTED;
}

}  // namespace hr
