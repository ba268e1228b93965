// hr_ivf.hip -- IVF-flat lists search: BASELINE config 5's candidate generation (SURVEY.md
// §8(f) rank 4).  The index is an ordinary hr_index whose rows sit in list order (each list
// starts on a 32-row tile; pad rows are dead), plus fp32 centroids, the tile offset of every
// list and the original id of every stored position.
//
// Search of one batch (<= 64 queries per chunk), all on the caller's stream:
//   k_prep_q     processed fp32 queries (the exact operand), |q|^2
//   k_coarse     exact canonical fp64 score of every (query, centroid) pair
//   k_topk_cand  top-nprobe lists per query, (score desc, list asc)
//   k_ivf_units  per-query unit list: (query, tile) for every tile of its probed lists
//   k_ivf_scan   exact canonical fp64 score of every row of every unit, one wave per unit:
//                the tile's 64 KiB stream is read coalesced exactly as the brute-force scan
//                reads it, and the 64 canonical partial sums of each row live in the lane
//                pair that holds the row (acc[s % 4][j] on lane r + 32h = partial 16(s%4)+8h+j)
//   k_topk_cand  exact top-k per query, (score desc, id asc)
// The candidates are exact over the visible rows (the rows of the probed lists), so every
// shard returns bound = -inf and the usual merge needs no fallback.  Exact scoring costs no
// more than an approximate pass here: each probed tile is read once per query either way
// (lists are rarely probed by two queries of one batch), and 8 fp64 FMAs per 16 bytes keep
// far below the fp64 VALU rate, so the scan stays HBM-bound.
#include "hr_internal.hpp"
#include "hr_kernels.hpp"

namespace {

// ---------------------------------------------------------------- K9: coarse scores
// Exact canonical fp64 score of every (query, centroid) pair (oracle order: lane-strided partial
// sums + butterfly).  A 1024-thread workgroup = 16 waves = 16 centroids; the processed queries
// are staged through LDS up to 32 at a time (128 KiB at dpad 1024), so L2 serves each query once per
// workgroup instead of once per wave.  CJ > 0: the wave's centroid row (CJ = dpad/64 values per lane)
// is held in registers for all queries -- re-loading it from memory inside the query loop made every
// iteration wait one memory round trip (165 us per 64 x 8192 x 1024 batch, latency-bound).
template <int CJ>
__global__ __launch_bounds__(1024) void k_coarse(const float* __restrict__ cent, int nlist, int dpad,
                                                 const float* __restrict__ q32, int B, int qgroup,
                                                 Cand* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float qs[];  // [kCoarseQ][dpad]
    const int lane = threadIdx.x & 63;
    const int l = blockIdx.x * 16 + (threadIdx.x >> 6);
    const float* c = cent + (int64_t)(l < nlist ? l : 0) * dpad;
    double cr[CJ > 0 ? CJ : 1];
    if constexpr (CJ > 0) {
#pragma unroll
        for (int j = 0; j < CJ; ++j) cr[j] = (double)c[lane + 64 * j];
    }
    auto cval = [&](int j, int d) -> double {
        if constexpr (CJ > 0) return cr[j];
        return (double)c[d];
    };
    const int nj = dpad / 64;
    for (int b0 = 0; b0 < B; b0 += qgroup) {
        const int nb = B - b0 < qgroup ? B - b0 : qgroup;
        __syncthreads();  // previous group done with LDS
        for (int i = threadIdx.x; i < nb * dpad / 4; i += blockDim.x)
            ((float4*)qs)[i] = ((const float4*)(q32 + (int64_t)b0 * dpad))[i];
        __syncthreads();
        if (l < nlist) {
            int b = 0;
            for (; b + 4 <= nb; b += 4) {  // four independent sums and butterflies interleave (ILP)
                double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
                for (int j = 0; j < (CJ > 0 ? CJ : 1); ++j) {
                    for (int jj = (CJ > 0 ? j : 0); jj < (CJ > 0 ? j + 1 : nj); ++jj) {
                        const int d = lane + 64 * jj;
                        const double cd = cval(jj, d);
                        p0 = p0 + cd * (double)qs[(b + 0) * dpad + d];
                        p1 = p1 + cd * (double)qs[(b + 1) * dpad + d];
                        p2 = p2 + cd * (double)qs[(b + 2) * dpad + d];
                        p3 = p3 + cd * (double)qs[(b + 3) * dpad + d];
                    }
                }
                p0 = wave_butterfly_sum(p0);
                p1 = wave_butterfly_sum(p1);
                p2 = wave_butterfly_sum(p2);
                p3 = wave_butterfly_sum(p3);
                if (lane == 0) {
                    Cand* o = out + (int64_t)(b0 + b) * nlist + l;
                    o[0] = Cand{p0, l};
                    o[nlist] = Cand{p1, l};
                    o[2 * (int64_t)nlist] = Cand{p2, l};
                    o[3 * (int64_t)nlist] = Cand{p3, l};
                }
            }
            for (; b < nb; ++b) {
                const float* qv = qs + b * dpad;
                double p = 0.0;
                for (int jj = 0; jj < nj; ++jj) {
                    const int d = lane + 64 * jj;
                    p = p + cval(CJ > 0 ? (jj < CJ ? jj : 0) : 0, d) * (double)qv[d];
                }
                p = wave_butterfly_sum(p);
                if (lane == 0) out[(int64_t)(b0 + b) * nlist + l] = Cand{p, l};
            }
        }
    }
}

// ---------------------------------------------------------------- K10: exact top-m per segment
// One 1024-thread block per query.  Order (score desc, id asc); records with id < 0 are absent.
// Radix select of the m-th largest score key (8 passes of 8 bits over the segment, histogram in
// LDS), then, if the m-th place is tied, radix select of the smallest tied ids; the m winners are
// bitonic-sorted in LDS.  Out: m records per query, padded with (-inf, -1).
constexpr int kTopkMax = 1024;
__device__ inline uint64_t cand_key(const Cand& e) { return e.row < 0 ? 0ull : d2key(e.score); }
__device__ inline uint64_t id_key(int64_t id) { return (uint64_t)id ^ 0x8000000000000000ull; }

// f(record) for every record of a segment, this thread's share: U independent loads in flight per
// iteration (one at a time left every radix pass waiting on one L2 round trip per record)
template <class F>
__device__ inline void for_each_record(const Cand* __restrict__ seg, int64_t n, F&& f) {
    constexpr int U = 4;
    const int64_t st = blockDim.x;
    int64_t i = threadIdx.x;
    for (; i + (U - 1) * st < n; i += U * st) {
        Cand e[U];
#pragma unroll
        for (int r = 0; r < U; ++r) e[r] = seg[i + r * st];
#pragma unroll
        for (int r = 0; r < U; ++r) f(e[r]);
    }
    for (; i < n; i += st) f(seg[i]);
}

__global__ __launch_bounds__(1024) void k_topk_cand(const Cand* __restrict__ in, const int64_t* __restrict__ seg_off,
                                                    int seg_scale, int64_t seg_stride, int B, int m,
                                                    Cand* __restrict__ out) {
    __shared__ uint32_t hist[256];
    __shared__ uint64_t sh_prefix;
    __shared__ int64_t sh_need;
    __shared__ int sh_cnt;
    __shared__ uint64_t skey[kTopkMax];
    __shared__ int64_t sid[kTopkMax];
    __shared__ double ssc[kTopkMax];
    const int b = blockIdx.x;
    if (b >= B) return;
    const int tid = threadIdx.x;
    const int64_t lo = seg_off ? seg_off[b] * seg_scale : (int64_t)b * seg_stride;
    const int64_t hi = seg_off ? seg_off[b + 1] * seg_scale : lo + seg_stride;
    const Cand* seg = in + lo;
    const int64_t n = hi - lo;

    // m-th largest key among valid records (radix select, MSB first)
    auto select_key = [&](bool by_id, uint64_t key_eq, int64_t need0) -> uint64_t {
        uint64_t prefix = 0, mask = 0;
        if (tid == 0) sh_need = need0;
        for (int shift = 56; shift >= 0; shift -= 8) {
            for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
            __syncthreads();
            for_each_record(seg, n, [&](const Cand& e) {
                const uint64_t k = cand_key(e);
                if (k == 0 || (by_id && k != key_eq)) return;
                const uint64_t v = by_id ? ~id_key(e.row) : k;  // ids: smallest first = largest complement
                if ((v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255], 1u);
            });
            __syncthreads();
            if (tid == 0) {
                int64_t need = sh_need, above = 0;
                int d = 255;
                for (; d > 0; --d) {
                    if (above + hist[d] >= need) break;
                    above += hist[d];
                }
                sh_need = need - above;
                sh_prefix = prefix | ((uint64_t)d << shift);
            }
            __syncthreads();
            prefix = sh_prefix;
            mask |= (uint64_t)255 << shift;
        }
        return prefix;
    };

    // valid records
    if (tid == 0) sh_cnt = 0;
    __syncthreads();
    int my = 0;
    for_each_record(seg, n, [&](const Cand& e) { my += cand_key(e) != 0; });
    if (my) atomicAdd(&sh_cnt, my);
    __syncthreads();
    const int64_t n_valid = sh_cnt;
    __syncthreads();

    uint64_t kth = 0, id_thr = ~0ull;  // take key > kth, or key == kth with ~id_key >= id_thr
    bool done = n_valid <= m;
    if (!done) {
        // Level 1: the m-th largest of the keys' upper 32 bits (4 radix passes).  Usually only a few
        // records share that prefix, so every record at or above it fits in LDS and one bitonic sort
        // of (key, id) finishes the job; otherwise fall through to the full 64-bit + id selection.
        uint64_t prefix = 0, mask = 0;
        if (tid == 0) sh_need = m;
        for (int shift = 56; shift >= 32; shift -= 8) {
            for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
            __syncthreads();
            for_each_record(seg, n, [&](const Cand& e) {
                const uint64_t k = cand_key(e);
                if (k != 0 && (k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1u);
            });
            __syncthreads();
            if (tid == 0) {
                int64_t need = sh_need, above = 0;
                int d = 255;
                for (; d > 0; --d) {
                    if (above + hist[d] >= need) break;
                    above += hist[d];
                }
                sh_need = need - above;
                sh_prefix = prefix | ((uint64_t)d << shift);
            }
            __syncthreads();
            prefix = sh_prefix;
            mask |= (uint64_t)255 << shift;
        }
        // records with upper key >= the m-th: gather if they fit
        if (tid == 0) sh_cnt = 0;
        __syncthreads();
        for_each_record(seg, n, [&](const Cand& e) {
            const uint64_t k = cand_key(e);
            if (k == 0 || (k & mask) < prefix) return;
            const int p = atomicAdd(&sh_cnt, 1);
            if (p < kTopkMax) {
                skey[p] = k;
                sid[p] = e.row;
                ssc[p] = e.score;
            }
        });
        __syncthreads();
        done = sh_cnt <= kTopkMax;
        __syncthreads();
    }
    if (!done && n_valid > m) {
        kth = select_key(false, 0, m);
        const int64_t need_ties = sh_need;  // winners among records with key == kth
        // are all ties needed?  count them
        __syncthreads();
        if (tid == 0) sh_cnt = 0;
        __syncthreads();
        int t = 0;
        for_each_record(seg, n, [&](const Cand& e) { t += cand_key(e) == kth; });
        if (t) atomicAdd(&sh_cnt, t);
        __syncthreads();
        const int64_t n_ties = sh_cnt;
        __syncthreads();
        if (n_ties > need_ties) id_thr = select_key(true, kth, need_ties);
        else id_thr = 0;
    }
    // gather the winners (exactly min(m, n_valid)) unless level 1 already holds a superset in LDS
    if (!done || n_valid <= m) {
    if (tid == 0) sh_cnt = 0;
    __syncthreads();
    for_each_record(seg, n, [&](const Cand& e) {
        const uint64_t k = cand_key(e);
        if (k == 0) return;
        const bool win = n_valid <= m || k > kth || (k == kth && ~id_key(e.row) >= id_thr);
        if (!win) return;
        const int p = atomicAdd(&sh_cnt, 1);
        if (p < kTopkMax) {
            skey[p] = k;
            sid[p] = e.row;
            ssc[p] = e.score;
        }
    });
    }
    __syncthreads();
    const int cnt = sh_cnt < kTopkMax ? sh_cnt : kTopkMax;
    int p2 = 1;
    while (p2 < cnt) p2 <<= 1;
    for (int i = cnt + tid; i < p2; i += blockDim.x) {
        skey[i] = 0;
        sid[i] = INT64_MAX;
        ssc[i] = -__builtin_inf();
    }
    __syncthreads();
    for (int kk = 2; kk <= p2; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < p2; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const bool a_first = skey[i] > skey[ixj] || (skey[i] == skey[ixj] && sid[i] < sid[ixj]);
                    const bool desc = (i & kk) == 0;
                    if (desc ? !a_first : a_first) {
                        uint64_t tk = skey[i];
                        skey[i] = skey[ixj];
                        skey[ixj] = tk;
                        int64_t ti = sid[i];
                        sid[i] = sid[ixj];
                        sid[ixj] = ti;
                        double ts = ssc[i];
                        ssc[i] = ssc[ixj];
                        ssc[ixj] = ts;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int i = tid; i < m; i += blockDim.x)
        out[(int64_t)b * m + i] = i < cnt ? Cand{ssc[i], sid[i]} : Cand{-__builtin_inf(), -1};
}

// ---------------------------------------------------------------- K11: unit lists
// One block: unit = (query << 26) | tile for every tile of every probed list, query-major;
// uoff[b] = first unit of query b, uoff[B] = total.  Units beyond cap are dropped (the host
// sizes cap from the largest list, so this never happens).
__global__ __launch_bounds__(1024) void k_ivf_units(const Cand* __restrict__ probes, int B, int nprobe,
                                                    const int64_t* __restrict__ list_tiles,
                                                    uint32_t* __restrict__ units, int64_t* __restrict__ uoff,
                                                    int64_t cap) {
    __shared__ int64_t part[1024];
    const int tid = threadIdx.x;
    const int np = B * nprobe;
    const int per = (np + blockDim.x - 1) / blockDim.x;  // pairs per thread, contiguous
    int64_t mine = 0;
    for (int j = 0; j < per; ++j) {
        const int p = tid * per + j;
        if (p >= np) break;
        const int64_t l = probes[p].row;
        mine += l >= 0 ? list_tiles[l + 1] - list_tiles[l] : 0;
    }
    // exclusive scan over the 1024 partials: inclusive scan inside each wave (shuffles), then over
    // the 16 wave totals (a serial scan by one thread cost ~40 us: 1024 dependent LDS round trips)
    int64_t incl = mine;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t o = __shfl_up(incl, off, 64);
        if ((tid & 63) >= off) incl += o;
    }
    if ((tid & 63) == 63) part[tid >> 6] = incl;
    __syncthreads();
    if (tid < 64) {
        int64_t w = tid < (int)(blockDim.x >> 6) ? part[tid] : 0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t o = __shfl_up(w, off, 64);
            if (tid >= off) w += o;
        }
        part[64 + tid] = w;  // inclusive over waves
    }
    __syncthreads();
    int64_t pos = incl - mine + ((tid >> 6) ? part[64 + (tid >> 6) - 1] : 0);
    for (int j = 0; j < per; ++j) {
        const int p = tid * per + j;
        if (p >= np) break;
        const int b = p / nprobe;
        if (p % nprobe == 0) uoff[b] = pos < cap ? pos : cap;
        const int64_t l = probes[p].row;
        if (l < 0) continue;
        const int64_t t0 = list_tiles[l], t1 = list_tiles[l + 1];
        for (int64_t t = t0; t < t1; ++t, ++pos)
            if (pos < cap) units[pos] = ((uint32_t)b << 26) | (uint32_t)t;
    }
    if (tid == (int)blockDim.x - 1) uoff[B] = pos < cap ? pos : cap;
}

// ---------------------------------------------------------------- K12: exact scan of the units
// One wave per unit at a time (static contiguous split of the unit list).  Lane l = r + 32h of a
// k-step chunk holds elements 16s + 8h + j of row r, i.e. canonical partials c = 16(s%4) + 8h + j;
// the oracle's butterfly (off 32, 16: local; 8: lanes r <-> r+32; 4, 2, 1: local) then gives the
// canonical score of row r on lane r.  The chunk stream of a wave (its units back to back) goes
// through a ring of P raw 16-byte loads (the same software pipeline as the brute-force scan), so
// P KiB per wave stay in flight across unit boundaries.
template <int DT>
struct RawChunk {  // one k-step chunk of this lane, undecoded
    u32x4 a, b;
    __device__ inline void load(const uint8_t* rows, int64_t c, int lane) {
        if constexpr (DT == F32) {
            a = __builtin_nontemporal_load((const u32x4*)(rows + c * 2048 + lane * 16));
            b = __builtin_nontemporal_load((const u32x4*)(rows + c * 2048 + 1024 + lane * 16));
        } else {
            a = __builtin_nontemporal_load((const u32x4*)(rows + c * 1024 + lane * 16));
        }
    }
    __device__ inline void get(float (&x)[8]) const {
        if constexpr (DT == F32) {
            // whole-vector bit casts: hipcc (ROCm 7.2) mis-lowers bit casts of single ext-vector
            // elements here (see XFrag<MT, F32> in hr_kernels.hpp)
            typedef float f32x4 __attribute__((ext_vector_type(4)));
            const f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                x[j] = fa[j];
                x[4 + j] = fb[j];
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint16_t lo = (uint16_t)(a[j] & 0xFFFFu), hi = (uint16_t)(a[j] >> 16);
                x[2 * j] = DT == BF16 ? bf16_to_f32(lo) : f16_to_f32(lo);
                x[2 * j + 1] = DT == BF16 ? bf16_to_f32(hi) : f16_to_f32(hi);
            }
        }
    }
};

template <int DT, int P>
__global__ __launch_bounds__(256) void k_ivf_scan(const uint8_t* __restrict__ rows, int S,
                                                  const uint32_t* __restrict__ live, const uint32_t* __restrict__ mask,
                                                  const int64_t* __restrict__ ids, const float* __restrict__ q32,
                                                  int dpad, const uint32_t* __restrict__ units,
                                                  const int64_t* __restrict__ uoff, int B, Cand* __restrict__ out) {
    static_assert(P % 4 == 0, "ring depth is a multiple of the 4-step canonical cycle");
    // the wave's current query lives in LDS (dpad floats per wave): its reads then count against
    // lgkmcnt, not vmcnt, so they never make the corpus ring drain (a global query load after the
    // ring loads would have to wait for all of them)
    extern __shared__ __attribute__((aligned(16))) float qlds[];
    float* const myq = qlds + (int64_t)(threadIdx.x >> 6) * dpad;
    const int lane = threadIdx.x & 63;
    const int r = lane & 31, h = lane >> 5;
    const int64_t W = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t n_units = uoff[B];
    const int64_t base = n_units / W, rem = n_units % W;
    const int64_t u0 = w * base + (w < rem ? w : rem);
    const int64_t u1 = u0 + base + (w < rem ? 1 : 0);
    if (u0 >= u1) return;
    auto stage_query = [&](int b) {  // the wave's own LDS rows; LDS ops of one wave execute in order
        const float4* src = (const float4*)(q32 + (int64_t)b * dpad);
        for (int e = lane; e < dpad / 4; e += 64) ((float4*)myq)[e] = src[e];
        __builtin_amdgcn_wave_barrier();
    };
    // first query before the first ring loads: its wait then leaves the ring in flight
    int cur_b = (int)(units[u0] >> 26);
    stage_query(cur_b);
    RawChunk<DT> ring[P];
    int64_t t_next = units[u0] & 0x3FFFFFFu;
#pragma unroll
    for (int i = 0; i < P; ++i) ring[i].load(rows, t_next * S + i, lane);
    for (int64_t u = u0; u < u1; ++u) {
        const uint32_t pk = units[u];
        const int64_t t = pk & 0x3FFFFFFu;
        const int b = (int)(pk >> 26);
        if (b != cur_b) {  // a query change (units are query-major: about once per wave)
            __builtin_amdgcn_wave_barrier();
            stage_query(b);
            cur_b = b;
        }
        const int64_t tn = u + 1 < u1 ? (int64_t)(units[u + 1] & 0x3FFFFFFu) : t;  // prefetch target after t
        const float* qv = myq + 8 * h;
        double acc[4][8];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[a][j] = 0.0;
        for (int s0 = 0; s0 < S; s0 += P) {
            const int64_t nc = s0 + P < S ? t * S + s0 + P : tn * S;
#pragma unroll
            for (int i = 0; i < P; ++i) {
                float x[8];
                ring[i].get(x);
                ring[i].load(rows, nc + i, lane);
                const float4 q0 = *(const float4*)(qv + 16 * (s0 + i));
                const float4 q1 = *(const float4*)(qv + 16 * (s0 + i) + 4);
                const float qq[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[i % 4][j] = __builtin_fma((double)x[j], (double)qq[j], acc[i % 4][j]);
            }
        }
        // canonical butterfly over partial index c = 16a + 8h + j
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[0][j] = acc[0][j] + acc[2][j];  // off 32
            acc[1][j] = acc[1][j] + acc[3][j];
            acc[0][j] = acc[0][j] + acc[1][j];  // off 16
            const double o = __shfl_xor(acc[0][j], 32, 64);  // off 8: lane r (h=0) takes r+32's
            acc[0][j] = acc[0][j] + o;
        }
        double p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] = acc[0][j];
        p[0] = p[0] + p[4]; p[1] = p[1] + p[5]; p[2] = p[2] + p[6]; p[3] = p[3] + p[7];  // off 4
        p[0] = p[0] + p[2]; p[1] = p[1] + p[3];                                          // off 2
        p[0] = p[0] + p[1];                                                              // off 1
        if (h == 0) {  // lane r holds the row of slot r (slot swizzle, hr_common.hpp)
            const int rr = slot_row(t, r);
            uint32_t allow = live[t];
            if (mask) allow &= mask[t];
            const int64_t pos = t * 32 + rr;
            const bool ok = (allow >> rr) & 1u;
            out[u * 32 + r] = ok ? Cand{p[0], ids[pos]} : Cand{-__builtin_inf(), -1};
        }
    }
}

__global__ void k_fill_f64(double* __restrict__ p, int n, double v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

}  // namespace

// ---------------------------------------------------------------- C ABI
extern "C" int hr_ivf_search(hr_index* h, const float* centroids_dev, int nlist, const int64_t* list_tiles_dev,
                             int64_t max_list_tiles, const int64_t* ids_dev, const float* q_dev, int B, int nprobe,
                             int k, const uint64_t* row_mask_dev, void* cand_out_dev, double* bound_out_dev,
                             void* probes_out_dev, void* stream) {
    if (!h || !centroids_dev || !list_tiles_dev || !ids_dev || !q_dev || !cand_out_dev || !bound_out_dev)
        return set_err(HR_E_INVALID, "null argument");
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "IVF lists need a single-device index");
    if (B <= 0 || nlist <= 0 || nprobe <= 0 || nprobe > nlist || nprobe > kTopkMax || k <= 0 || k > kTopkMax ||
        max_list_tiles < 0)
        return set_err(HR_E_INVALID, "bad sizes (need 1 <= nprobe <= min(nlist, 1024), 1 <= k <= 1024)");
    if (h->metric == L2) return set_err(HR_E_UNSUPPORTED, "IVF lists support cosine and dot (inner product)");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = set_device(h)) return rc;
    hipStream_t st = (hipStream_t)stream;
    Scratch& sc = h->scr[kSyncSet];
    const int dpad = h->dpad;
    for (int b0 = 0; b0 < B; b0 += 64) {
        const int bc = std::min(64, B - b0);
        const int Bp = bc > 32 ? 64 : 32, QB = Bp / 32;
        const int64_t cap = (int64_t)bc * nprobe * std::max<int64_t>(1, max_list_tiles);
        if (cap >= ((int64_t)1 << 31)) return set_err(HR_E_INVALID, "probed lists too large for one batch");
        HIP_TRY(sc.q32.ensure((size_t)Bp * dpad * 4));
        HIP_TRY(sc.qfrag.ensure((size_t)h->S * QB * 1024));
        HIP_TRY(sc.qerr.ensure((size_t)Bp * 4 * 8));
        HIP_TRY(h->ivf_coarse.ensure((size_t)bc * nlist * sizeof(Cand)));
        HIP_TRY(h->ivf_probe.ensure((size_t)bc * nprobe * sizeof(Cand)));
        HIP_TRY(h->ivf_units.ensure((size_t)cap * 4));
        HIP_TRY(h->ivf_uoff.ensure((size_t)(bc + 1) * 8));
        HIP_TRY(h->ivf_out.ensure((size_t)cap * 32 * sizeof(Cand)));
        const float* qb = q_dev + (int64_t)b0 * h->dim;
        if (mfma_type(h) == BF16)
            hipLaunchKernelGGL((k_prep_q<BF16>), dim3((Bp + 3) / 4), dim3(256), 0, st, qb, bc, Bp, h->dim, dpad, h->S,
                               QB, h->metric, sc.q32.as<float>(), sc.qfrag.as<uint16_t>(), sc.qerr.as<double>(),
                               nullptr, 1, nullptr, nullptr, nullptr);
        else
            hipLaunchKernelGGL((k_prep_q<F16>), dim3((Bp + 3) / 4), dim3(256), 0, st, qb, bc, Bp, h->dim, dpad, h->S,
                               QB, h->metric, sc.q32.as<float>(), sc.qfrag.as<uint16_t>(), sc.qerr.as<double>(),
                               nullptr, 1, nullptr, nullptr, nullptr);
        // centroid row in registers for dpad <= 1024 (CJ = dpad / 64 values per lane)
        auto coarse = dpad == 1024 ? k_coarse<16> : dpad == 768 ? k_coarse<12> : dpad == 512 ? k_coarse<8>
                      : dpad == 384 ? k_coarse<6> : dpad == 256 ? k_coarse<4> : dpad == 128 ? k_coarse<2>
                      : dpad == 64 ? k_coarse<1> : k_coarse<0>;
        static bool coarse_attr[64][17] = {};
        const int ci = (dpad == 1024 || dpad == 768 || dpad == 512 || dpad == 384 || dpad == 256 || dpad == 128 ||
                        dpad == 64) ? dpad / 64 : 0;  // the CJ of the instantiation chosen above
        if (!coarse_attr[h->device & 63][ci]) {
            HIP_TRY(hipFuncSetAttribute((const void*)coarse, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            coarse_attr[h->device & 63][ci] = true;
        }
        const int qgroup = std::max(1, std::min(32, (160 * 1024) / (dpad * 4)));  // queries per LDS stage
        hipLaunchKernelGGL(coarse, dim3((nlist + 15) / 16), dim3(1024), (size_t)qgroup * dpad * 4, st,
                           centroids_dev, nlist, dpad, sc.q32.as<float>(), bc, qgroup, h->ivf_coarse.as<Cand>());
        hipLaunchKernelGGL(k_topk_cand, dim3(bc), dim3(1024), 0, st, h->ivf_coarse.as<Cand>(), (const int64_t*)nullptr,
                           1, (int64_t)nlist, bc, nprobe, h->ivf_probe.as<Cand>());
        hipLaunchKernelGGL(k_ivf_units, dim3(1), dim3(1024), 0, st, h->ivf_probe.as<Cand>(), bc, nprobe,
                           list_tiles_dev, h->ivf_units.as<uint32_t>(), h->ivf_uoff.as<int64_t>(), cap);
        HIP_TRY(hipGetLastError());
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((int64_t)h->n_cu * 8, (cap + 3) / 4));
        int rc = dispatch_dt(h->dtype, [&](auto dt) -> int {
            constexpr int DT = decltype(dt)::value;
            // ring depth (chunks in flight per wave): fp32 rows 4 (8 KiB; deeper rings spill), 16-bit
            // rows 16 where the k-steps allow it
            const int ring = DT == F32 ? 4 : (h->S % 16 == 0 ? 16 : (h->S % 8 == 0 ? 8 : 4));
            auto kern = ring == 16 ? k_ivf_scan<DT, 16> : ring == 8 ? k_ivf_scan<DT, 8> : k_ivf_scan<DT, 4>;
            const size_t qbytes = (size_t)4 * dpad * sizeof(float);  // one query per wave
            static bool scan_attr[64][3] = {};
            const int ri = ring == 16 ? 2 : ring == 8 ? 1 : 0;
            if (qbytes > 64 * 1024 && !scan_attr[h->device & 63][ri]) {
                HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
                scan_attr[h->device & 63][ri] = true;
            }
            if (qbytes > 160 * 1024) return set_err(HR_E_UNSUPPORTED, "IVF scan: dim too large for the LDS query");
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), qbytes, st, h->rows, h->S, h->live,
                               (const uint32_t*)row_mask_dev, ids_dev, sc.q32.as<float>(), dpad,
                               h->ivf_units.as<uint32_t>(), h->ivf_uoff.as<int64_t>(), bc, h->ivf_out.as<Cand>());
            HIP_TRY(hipGetLastError());
            return HR_OK;
        });
        if (rc) return rc;
        hipLaunchKernelGGL(k_topk_cand, dim3(bc), dim3(1024), 0, st, h->ivf_out.as<Cand>(), h->ivf_uoff.as<int64_t>(),
                           32, (int64_t)0, bc, k, (Cand*)cand_out_dev + (int64_t)b0 * k);
        HIP_TRY(hipGetLastError());
        if (probes_out_dev)
            HIP_TRY(hipMemcpyAsync((Cand*)probes_out_dev + (int64_t)b0 * nprobe, h->ivf_probe.p,
                                   (size_t)bc * nprobe * sizeof(Cand), hipMemcpyDeviceToDevice, st));
    }
    // exact over the visible rows: nothing unreturned can matter
    hipLaunchKernelGGL(k_fill_f64, dim3((B + 255) / 256), dim3(256), 0, st, bound_out_dev, B, -INFINITY);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}

// Exact top-m records per segment, (score desc, id asc), ids < 0 absent: segment b is
// [seg_off[b], seg_off[b+1]) records if seg_off (int64, in records) is given, else
// [b * seg_stride, (b + 1) * seg_stride).  The reranker's per-query selection and the IVF stages.
extern "C" int hr_topk_records(const void* in_dev, const int64_t* seg_off_records_dev, int64_t seg_stride, int B,
                               int m, void* out_dev, void* stream) {
    if (!in_dev || !out_dev || B <= 0 || m <= 0 || m > kTopkMax || (!seg_off_records_dev && seg_stride < 0))
        return set_err(HR_E_INVALID, "bad arguments (need 1 <= m <= 1024)");
    hipLaunchKernelGGL(k_topk_cand, dim3(B), dim3(1024), 0, (hipStream_t)stream, (const Cand*)in_dev,
                       seg_off_records_dev, 1, seg_stride, B, m, (Cand*)out_dev);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}
