// hr_internal.hpp -- host-side internals shared by the libhiprag.so translation units
// (hr_index.hip: index handles and the exact search; hr_ivf.hip: the IVF lists search).
#pragma once
#include <hip/hip_runtime.h>
#include <unistd.h>
#include <atomic>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hiprag.h"
#include "../../include/hiprag_diag.h"
#include "hr_common.hpp"

using namespace hr;

// ---------------------------------------------------------------- errors
int set_err(int code, const std::string& msg);  // thread-local message for hr_last_error (hr_index.hip)
#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return set_err(HR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
    } while (0)

// ---------------------------------------------------------------- device buffers
// bumped whenever a work buffer is (re)allocated or freed: a captured HIP graph holds raw buffer
// addresses, so a graph captured before the bump is stale (see SyncGraph)
inline std::atomic<uint64_t> g_buf_gen{0};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        g_buf_gen.fetch_add(1);
        hipError_t e = hipMalloc(&p, need);
        if (e == hipSuccess) bytes = need;
        return e;
    }
    void release() {
        if (p) {
            (void)hipFree(p);
            g_buf_gen.fetch_add(1);
        }
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const {
        return (T*)p;
    }
};

namespace hr {  // hr_exhaustive.hip
size_t exhaustive_scratch_bytes(int64_t n);
int exhaustive_topm(const uint8_t* rows, int dtype, int S, int dpad, const float* qv, int metric, double qn2,
                    const uint32_t* live,
                    const uint32_t* mask, int64_t n, int64_t row_offset, int m, Cand* out, void* scratch,
                    size_t scratch_bytes, hipStream_t st, int sG = 1, int ss = 0);
// G ranks' sorted exact top-m lists (rank stride cstride bytes) -> the top-k (score desc, row asc; -inf / -1 padding)
int launch_merge_sorted(const Cand* cand, int64_t cstride, int G, int B, int m, int k, float* s_out, int64_t* r_out,
                        hipStream_t st);
size_t tile_list_scratch_bytes(int64_t n_tiles);
int build_tile_list(const uint32_t* live, const uint32_t* mask, int64_t n_tiles, uint32_t* list, uint32_t* count,
                    void* scratch, size_t scratch_bytes, hipStream_t st);
// hr_wide.hip: the 128-query FILTER (one workgroup per CU, 4 waves; pbuf / pcnt regions [2 groups][4 * cus][64])
struct ScanArgs;
bool wide_filter_ok(int dtype, int S);
int launch_filter_wide(int mt, int dtype, int S, int cus, const ScanArgs& a, hipStream_t st);
// row parts of the eight-wave form (kc > 32): 32 groups per part, one 16 KiB key table each in LDS beside the two
// streamed window buffers (2 x 32 KiB, or 2 x 16 KiB for fp32 rows): at most 5 (bf16 / f16) or 7 (fp32) parts,
// kc <= 160 / 224
constexpr int wide_max_parts(int dtype) { return dtype == F32 ? 7 : 5; }
// hr_q256.hip: the 256-query FILTER (four 64-query groups in one pass; bf16 / f16 rows, D = 256..1024, one row
// part); candidate regions [4 groups][4 * cus waves][64][kCapW] as k_scan's
bool q256_filter_ok(int dtype, int S);
int launch_filter_q256(int mt, int dtype, int S, int cus, const ScanArgs& a, hipStream_t st);
// hr_persist.hip: the persistent FILTER (plans with 64-query tiles: P = 16 for 16-bit rows, 4 for fp32 rows)
struct PersistCtl;
struct PersistLaunch;
int launch_persist(int mt, int dtype, int P, int cus, const PersistLaunch& pa, int lds, hipStream_t st);
int launch_persist_post(PersistCtl* c, uint32_t e, hipStream_t st);
int launch_persist_close(PersistCtl* c, hipStream_t st);
int launch_persist_wait(PersistCtl* c, uint32_t e, uint32_t nwg, uint32_t* host_err, hipStream_t st);
}  // namespace hr

static constexpr int kCap = 8192;       // candidate buffer per query (shared-buffer / collect mode)
static constexpr int kCapW = 32;        // private candidate slots per (wave, query) (FILTER mode)
static constexpr int kScanThreads = 512;

// Per-batch search workspace.  Two sets ping-pong between consecutive pipelined batches
// (hr_index_search_shard_async: batch i's select/rescore on the tail stream overlaps batch
// i+1's scan on the scan stream); a third serves the synchronous and collect paths.
struct Scratch {
    DevBuf q32, qfrag, qerr, mkeys, floor_q, cnt, buf, sel_rows, sel_cnt, bound_approx, overflow, pbuf, pcnt, dyn_q,
        tl, tl_tmp,  // device-mask tile list (+ its count after the list) and its rocPRIM scratch
        wtiles;      // diagnostics: tiles each wave of the most recent FILTER launch scanned (ScanArgs::wave_tiles)
    int64_t last_W = 0, last_Bp = 0;  // waves (per query group) and queries per group of the most recent FILTER
    int last_ng = 1;                  // query groups of that launch
    int last_capw = kCapW;            // candidate slots per (region, query) of that launch
    bool wtiles_valid = false;        // that launch was a k_scan FILTER (it wrote wtiles)
    hipEvent_t scanned = nullptr;     // scan stream: this set's FILTER is done
    hipEvent_t released = nullptr;    // tail stream: this set's select/rescore are done
    hipEvent_t sampled = nullptr;     // pre stream: this set's early query prep + SAMPLE are done
    hipStream_t scan = nullptr;       // early mode: this set's FILTER stream (created on first use)
    bool armed = false;               // `released` has been recorded at least once
    void release_all() {
        for (DevBuf* b : {&q32, &qfrag, &qerr, &mkeys, &floor_q, &cnt, &buf, &sel_rows, &sel_cnt, &bound_approx,
                          &overflow, &pbuf, &pcnt, &dyn_q, &tl, &tl_tmp, &wtiles})
            b->release();
        if (scanned) (void)hipEventDestroy(scanned);
        if (released) (void)hipEventDestroy(released);
        if (sampled) (void)hipEventDestroy(sampled);
        if (scan) (void)hipStreamDestroy(scan);
        scan = nullptr;
        scanned = released = sampled = nullptr;
    }
};
static constexpr int kSyncSet = 2;

struct hr_index {
    int dim = 0, dpad = 0, S = 0, dtype = BF16, metric = COSINE, device = 0;
    int64_t n = 0, cap = 0, n_live = 0;
    double max_norm2 = 0.0;
    uint8_t* rows = nullptr;        // tiled corpus
    // fp32 corpora: a 16-bit copy of the rows in the MFMA type (mfma_type), tiled as a 16-bit corpus, that the
    // approximate passes (SAMPLE, FILTER, collect) stream instead of the fp32 tiles -- the values they round every
    // fragment to anyway, at half the bytes; the exact rescoring and exhaustive passes keep reading the fp32 rows.
    // Maintained lazily: row writers lower shadow_lo (first stale tile) and the next search converts [shadow_lo,
    // tiles).  HIPRAG_F32_SHADOW=0 at create: none (the fp32 tiles are streamed and rounded in the kernels).
    uint8_t* rows16 = nullptr;
    bool shadow = false;
    int64_t shadow_lo = 0;
    uint32_t* live = nullptr;       // one word per tile
    float* xnorm = nullptr;         // euclidean only: fp32 |x|^2 per stored row (approximate scan score)
    std::vector<uint32_t> live_host;
    unsigned long long* norm_bits = nullptr;  // device max stored norm² (as double bits)
    hipStream_t stream = nullptr;
    hipStream_t pre = nullptr;  // early query prep + SAMPLE of pipelined batches (created on first use)
    // per-launch timing of the main (SAMPLE, FILTER) scan pair: events are recorded on the
    // search stream and harvested later, so batches can be pipelined (see hr_index_take_scan_times)
    struct ScanEvents {
        hipEvent_t e[4];  // SAMPLE start, FILTER start (= SAMPLE end unless early), early SAMPLE end, FILTER end
        bool sampled, early;
        uint32_t pepoch;  // persistent FILTER: the batch's epoch (its FILTER time comes from the device's stamps)
    };
    std::vector<ScanEvents> ev_free;
    std::deque<ScanEvents> ev_pending;
    float last_sample_ms = 0.f, last_filter_ms = 0.f;
    int time_every = 0;               // record events around every Nth main pass (0 = never)
    int64_t main_passes = 0;
    bool isolate_next = false;        // dual-stream mode: the next FILTER waits for a timed one
    int n_cu = 256;
    std::mutex mu;
    // tile list of the current selective-filter search (hr_index_search with a row mask that
    // leaves at most half the tiles): sorted tiles holding a live, allowed row; tl_n = -1: none
    // (a device mask builds its own), -2: the host evaluated the mask and chose the full scan
    DevBuf tl;
    int64_t tl_n = -1;
    std::vector<uint32_t> tl_host;
    // search workspace
    DevBuf q_in, cand, bound, kth, fail, fb_cand, fb_bound, fb_q, fb_out, stage, exh;
    DevBuf ivf_coarse, ivf_probe, ivf_units, ivf_uoff, ivf_out;  // IVF lists search (hr_ivf.hip)
    Scratch scr[3];
    int flip = 0;                     // next ping-pong set of the pipelined path
    const Scratch* last_scr = nullptr;  // set of the most recent FILTER launch (diagnostics)
    int64_t n_exhaustive = 0;         // queries that needed the exhaustive exact pass (diagnostics)
    int64_t n_guard_fail = 0;         // queries that failed the exactness guard (collect fallback)
    int64_t n_wide = 0;               // 128-query FILTER launches issued (hr_wide.hip; not graph replays)
    int64_t n_q256 = 0;               // 256-query FILTER launches issued (hr_q256.hip)
    bool q256 = true;                 // hr_index_set_q256: 129-256-query batches take the 256-query FILTER
    std::vector<float> floor_host;
    // ---- hr_index_search (host queries, no mask) replayed as one HIP graph per batch shape: H2D of
    // the queries from pinned staging, prep, SAMPLE, FILTER, select, rescore, merge, D2H of results
    // and guard flags.  Captured on a shape's second use (the first allocates every buffer); stale once
    // the corpus, its buffers or any work buffer changes (address / size snapshot below).
    struct SyncGraph {
        int B = 0, k = 0, uses = 0;
        bool disabled = false;
        int64_t n = -1;
        const void* rows = nullptr;
        const void* live = nullptr;
        const void* xnorm = nullptr;
        const void* pin = nullptr;
        double max_norm2 = 0.0;
        uint64_t buf_gen = 0;
        int chunks = 1;
        hipGraphExec_t exec = nullptr;
    };
    std::vector<SyncGraph> sync_graphs;
    void* pin = nullptr;      // pinned host staging of the graph path (hipHostMalloc)
    size_t pin_bytes = 0;
    DevBuf sync_out;          // device results of the graph path
    int64_t n_graph_replays = 0;
    // ---- asynchronous host-query search (hr_index_search_submit_host / _collect, hr_index.hip): up to two
    // batches in flight; each batch's completion is signalled to a file descriptor (an eventfd the caller's
    // event loop watches) by a host function queued behind its results' copy to pinned memory
    struct AsyncSlot {
        bool busy = false;
        int64_t ticket = 0;
        int B = 0, k = 0;
        uint8_t* pin = nullptr;  // pinned: queries in | scores | rows | guard flags | k-th scores out
        size_t pin_bytes = 0;
        size_t off_s = 0, off_r = 0, off_f = 0, off_k = 0;
        DevBuf q, cand, bound, kth, fail, s, r;
        hipEvent_t q_ready = nullptr, done = nullptr;
        // the batch's notify host function (hipLaunchHostFunc behind `done`) has not returned yet: collect and
        // destroy wait for it, so the caller never closes or reuses the fd number while that write is pending
        std::atomic<int> notify_pending{0};
        int notify_fd = -1;
    } aslot[2];
    int64_t aticket = 1;
    hipStream_t acopy = nullptr, atail = nullptr;
    // ---- multi-device handles (hr_index_create with n_dev > 1, hr_group.hip)
    // A group handle owns G shard handles (one per dev_ids entry, repeats allowed) and stripes its
    // rows over them by 32-row tile (stripe_row, hr_common.hpp); it holds no rows itself.  Its
    // device / stream are the primary's (dev_ids[0]): the shards' candidates are copied there
    // (hipMemcpyPeerAsync, xGMI) and merged by k_merge.  A shard knows its place in the stripe.
    int G = 1;                        // > 1: group handle
    std::vector<hr_index*> shards;
    int stripe_G = 1, stripe_s = 0;   // shard of a group: global row of local row L = stripe_row(L, G, s)
    bool shared_dev = false;          // shard of a group whose GPU also holds another shard of the group
    DevBuf g_cand, g_bound, g_kth, g_fail, g_out, g_q;  // group: gathered candidates / merge outputs (primary)
    DevBuf s_mask;                    // shard of a group: this shard's words of the caller's row mask
    std::vector<hipEvent_t> g_ev;     // group: one per shard (shard stream -> primary stream)
    hipEvent_t g_ev_q = nullptr;      // group: queries ready on the primary stream
    std::vector<char> g_peer;         // group: shard s's device has peer access with the primary
    struct GroupPipe* pipe = nullptr; // group: pipelined search (submit / finalize, hr_group.hip)
    struct Persist* ps = nullptr;     // persistent FILTER state (hr_index.hip; created on first use)
    // hr_index_set_cu_mask: the CUs this index's own streams may use (empty: all).  Every internal stream is then
    // created with hipExtStreamCreateWithCUMask and the launch grids are sized for popcount(mask) CUs
    std::vector<uint32_t> cu_mask;
};

// an internal stream of h: on h's CU mask when one is set (priority is then not available), else high priority or
// the default one (hr_index.hip)
hipError_t index_stream_create(const hr_index* h, hipStream_t* s, bool high_priority);

// group-handle entry points (hr_group.hip); each public hr_index_* call forwards here when h->G > 1
int group_create(int dim, int dtype, int metric, int n_dev, const int* dev_ids, hr_index** out);
void group_destroy(hr_index* g);
int group_reserve(hr_index* g, int64_t rows);
int group_add_host(hr_index* g, const float* rows, int64_t n, int64_t* first);
int group_add_synthetic(hr_index* g, uint64_t seed, int64_t global_row0, int64_t n, int64_t* first);
int group_add_device(hr_index* g, const float* rows_dev, int64_t n, int64_t* first, hipStream_t st);
int group_remove(hr_index* g, const int64_t* rows, int64_t n);
int group_search_host(hr_index* g, const float* q, int B, int k, const uint64_t* mask, float* s_out, int64_t* r_out);
int group_search_device(hr_index* g, const float* q_dev, int B, int k, const uint64_t* mask_dev, float* s_out,
                        int64_t* r_out, hipStream_t st);
int group_get_rows(hr_index* g, const int64_t* rows, int64_t n, float* out);
// pipelined group search: enqueue a batch (every shard submitted by its own host thread), finalize =
// wait for its guard flags and run the exact fallback; group_drain finalizes everything in flight
int group_search_submit(hr_index* g, const float* q_dev, int B, int k, float* s_out, int64_t* r_out, hipStream_t st,
                        int64_t* ticket);
int group_search_finalize(hr_index* g, int64_t ticket);
int group_drain(hr_index* g);
int group_host_us(hr_index* g, double out[3]);
int group_save(hr_index* g, const char* path);
int group_load_into(hr_index* g, FILE* f, int64_t n, int64_t n_live, double max_norm2);
void group_stats(hr_index* g, int64_t out[3]);

// single-shard internals shared with hr_group.hip (hr_index.hip)
int index_grow(hr_index* h, int64_t need_rows);
int index_add_host(hr_index* h, const float* rows, int64_t n, int64_t* first);
int index_add_synthetic(hr_index* h, uint64_t seed, int64_t gen_base, int64_t n);
int index_remove_local(hr_index* h, const int64_t* rows, int64_t n);
int index_get_rows(hr_index* h, const int64_t* rows, int64_t n, float* out);
int index_update_row_norms(hr_index* h, int64_t r0, int64_t n);
// the group-max order statistic of the FILTER's starting threshold and k_select (ScanArgs::kj; hr_index.hip)
int hr_rank_for(int k, int kc, int dim);
int index_finish_load(hr_index* h);
// one batch of queries (device, on this shard's device) through the exact search of one shard:
// candidates (global rows) + bounds into cand_out / bound_out on `st`
int index_shard_search(hr_index* h, const float* q_dev, int B, int kc, int kj, const uint64_t* mask_dev, Cand* cand_out,
                       double* bound_out, hipStream_t st);
// the same, pipelined: scan on st, select + rescore on st_tail (outputs ready in st_tail order), the
// queries ready once q_ready completes (see hr_index_search_shard_async_ev)
int index_shard_search_async(hr_index* h, const float* q_dev, int B, int kc, int kj, Cand* cand_out, double* bound_out,
                             hipStream_t st, hipStream_t st_tail, hipEvent_t q_ready);
int index_shard_collect(hr_index* h, const float* q_dev, int B, const double* kth_host, int cap,
                        const uint64_t* mask_dev, Cand* cand_out, double* bound_out, hipStream_t st);
int index_exact_all(hr_index* h, const float* q_dev, int B, int m, const uint64_t* mask_dev, Cand* out_host,
                    hipStream_t st);
int index_host_tile_list(hr_index* h, const uint32_t* mask_words, hipStream_t st);
int launch_merge(int device, const Cand* cand, const double* bounds, int G, int B, int kc, int k, float* s_out,
                 int64_t* r_out, double* kth_out, int32_t* fail_out, hipStream_t st, int64_t cstride = 0,
                 int64_t bstride = 0);
static constexpr int kFallbackCapMax = 1024;
inline int fallback_cap(int G) { return std::max(64, std::min(kFallbackCapMax, 8192 / std::max(1, G))); }

struct FileHeader {
    char magic[8];
    int32_t version, dim, dtype, metric;
    int64_t n, n_live;
    double max_norm2;
};

inline size_t tile_bytes(const hr_index* h) { return (size_t)h->S * (h->dtype == F32 ? 2048 : 1024); }

inline int set_device(hr_index* h) {
    HIP_TRY(hipSetDevice(h->device));
    return HR_OK;
}

// ---------------------------------------------------------------- dispatch helpers
template <class F>
inline int dispatch_dt(int dt, F&& f) {
    switch (dt) {
        case F32: return f(std::integral_constant<int, F32>{});
        case BF16: return f(std::integral_constant<int, BF16>{});
        case F16: return f(std::integral_constant<int, F16>{});
    }
    return set_err(HR_E_INVALID, "unknown dtype");
}

// MFMA operand type: f16 corpora use the f16 MFMA and bf16 corpora the bf16 one.  fp32 corpora are
// rounded to one of them on the fly: f16 (unit roundoff 2^-11, 8x finer than bf16, so the guard's window
// and the collect fallbacks shrink with it) when the rows are normalised (cosine: every element in
// [-1, 1], far inside f16's range), bf16 (fp32's range) for raw inner-product / euclidean rows
inline int mfma_type(const hr_index* h) {
    return (h->dtype == F16 || (h->dtype == F32 && h->metric == COSINE)) ? F16 : BF16;
}

// what the approximate passes stream: the 16-bit shadow of an fp32 corpus (as a corpus of the MFMA type), else the
// stored rows.  The exactness guard's storage term (storage_u) stays the fp32 one: the shadow holds exactly the
// RNE-rounded values the fp32 kernels would form on the fly.
inline int scan_dtype(const hr_index* h) { return h->rows16 ? mfma_type(h) : h->dtype; }
inline const uint8_t* scan_rows(const hr_index* h) { return h->rows16 ? h->rows16 : h->rows; }
// a row writer touched tiles from t0 on (INT64_MAX: the shadow is current)
inline void shadow_stale(hr_index* h, int64_t t0) {
    if (h->shadow && t0 < h->shadow_lo) h->shadow_lo = t0 < 0 ? 0 : t0;
}
int shadow_update(hr_index* h);

