// hr_index.hip -- host side of libhiprag.so: index handles, launch plumbing, C ABI.
// Declarations and the reference call each entry replaces: include/hiprag.h.
#include "hr_internal.hpp"
#include "hr_kernels.hpp"

// ---------------------------------------------------------------- errors
static thread_local std::string g_err;
int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

static int async_drain(hr_index* h);

// ---------------------------------------------------------------- the persistent FILTER (hr_persist.hip)
// Host state of an index's persistent FILTER: kPersistSlots per-batch workspaces whose buffers the instance reads
// (query fragments, group-max keys, floors, candidate regions, dynamic-tail counters) sit at a constant stride in
// one arena per kind, so an instance finds slot s's buffers as slot 0's + s * stride; the other per-batch buffers
// (select / rescore) are the slots' own.  Configured for one corpus state and plan; re-configured after a quiesce.
struct Persist {
    int mode = 1;                      // hr_index_set_persist: 0 off, 1 where it measured faster (default), 2 always
    bool ready = false;                // configured (for the key below)
    int64_t key_n = -1;
    const void* key_rows = nullptr;
    int key_S = 0, key_P = 0, key_ncu = 0;
    Scratch slot[kPersistSlots];       // qfrag / mkeys / floor_q / pbuf / pcnt / dyn_q are views into the arenas
    DevBuf ar_qfrag, ar_mkeys, ar_floor, ar_pbuf, ar_pcnt, ar_dynq;
    int64_t st_qfrag = 0, st_mkeys = 0, st_floor = 0, st_pbuf = 0, st_pcnt = 0, st_dynq = 0;
    DevBuf ctl;                        // PersistCtl
    uint32_t* host_err = nullptr;      // pinned mirror of PersistCtl::error
    hipStream_t pst = nullptr;         // instances (one launch per batch, gated by the batch's post event)
    hipEvent_t posted[kPersistSlots] = {};
    hipEvent_t closed = nullptr;       // pre stream: behind the last k_persist_close (orders the stop reset after it)
    uint32_t epoch = 0;                // last epoch posted
    bool active = false;               // the gate is open: a running instance may admit further batches
    bool launched = false;             // instances launched since the last quiesce (may still run: close != quiesce)
    int64_t timeouts = 0;              // quiesces that found a bounded wait given up (those batches took the exact pass)
    uint32_t last_err = 0;             // the error word of the latest such quiesce
    int nwg = 0;                       // workgroups of every instance (n_cu - tail CUs): fixed, the tail's targets use it
    uint32_t idle_ticks = 30000;       // 300 us of s_memrealtime (100 MHz) without a batch: the instance exits
    void drop_views() {
        for (auto& sc : slot)
            for (DevBuf* b : {&sc.qfrag, &sc.mkeys, &sc.floor_q, &sc.pbuf, &sc.pcnt, &sc.dyn_q}) {
                b->p = nullptr;
                b->bytes = 0;
            }
    }
};
static int persist_quiesce(hr_index* h);  // blocking: every instance has exited (mutations, destroy)
static int persist_close(hr_index* h);    // non-blocking: the running instance exits once through its batches

// ---------------------------------------------------------------- streams
hipError_t index_stream_create(const hr_index* h, hipStream_t* s, bool high_priority) {
    if (!h->cu_mask.empty())
        return hipExtStreamCreateWithCUMask(s, (uint32_t)h->cu_mask.size(), h->cu_mask.data());
    if (!high_priority) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    int lo = 0, hi = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e != hipSuccess) return e;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
}

// ---------------------------------------------------------------- create / grow
extern "C" int hr_index_create(int dim, int dtype, int metric, int n_dev, const int* dev_ids, hr_index** out) {
    if (!out) return set_err(HR_E_INVALID, "out is null");
    *out = nullptr;
    if (dim <= 0 || dim > 4096) return set_err(HR_E_INVALID, "dim must be in [1, 4096]");
    if (dtype < F32 || dtype > F16) return set_err(HR_E_INVALID, "dtype must be HR_F32, HR_BF16 or HR_F16");
    if (metric != COSINE && metric != IP && metric != L2) return set_err(HR_E_INVALID, "unknown metric");
    if (n_dev < 1 || n_dev > 64) return set_err(HR_E_INVALID, "n_dev must be in [1, 64]");
    if (n_dev > 1) {
        if (!dev_ids) return set_err(HR_E_INVALID, "dev_ids required when n_dev > 1");
        return group_create(dim, dtype, metric, n_dev, dev_ids, out);
    }
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    int dev = dev_ids ? dev_ids[0] : 0;
    if (dev < 0 || dev >= ndev) return set_err(HR_E_INVALID, "device id out of range");
    hr_index* h = new hr_index();
    h->dim = dim;
    h->dpad = (dim + 63) / 64 * 64;
    h->S = h->dpad / 16;
    h->dtype = dtype;
    h->metric = metric;
    h->device = dev;
    {
        const char* e = std::getenv("HIPRAG_F32_SHADOW");
        h->shadow = dtype == F32 && !(e && e[0] == '0');
        h->shadow_lo = INT64_MAX;
    }
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&h->norm_bits, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(h->norm_bits, 0, sizeof(unsigned long long));
    hipDeviceProp_t prop;
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) {
        hr_index_destroy(h);
        return set_err(HR_E_HIP, std::string("hr_index_create: ") + hipGetErrorString(e));
    }
    h->n_cu = prop.multiProcessorCount;
    *out = h;
    return HR_OK;
}

int index_grow(hr_index* h, int64_t need_rows) {
    if (need_rows <= h->cap) return HR_OK;
    int64_t new_cap = std::max<int64_t>({need_rows, h->cap + h->cap / 2, 1024});
    new_cap = (new_cap + 31) / 32 * 32;
    const size_t tb = tile_bytes(h);
    uint8_t* nr = nullptr;
    uint32_t* nl = nullptr;
    HIP_TRY(hipMalloc(&nr, (size_t)(new_cap / 32) * tb));
    HIP_TRY(hipMemsetAsync(nr, 0, (size_t)(new_cap / 32) * tb, h->stream));
    HIP_TRY(hipMalloc(&nl, (size_t)(new_cap / 32) * 4));
    HIP_TRY(hipMemsetAsync(nl, 0, (size_t)(new_cap / 32) * 4, h->stream));
    float* nx = nullptr;
    if (h->metric == L2) {
        HIP_TRY(hipMalloc(&nx, (size_t)new_cap * 4));
        HIP_TRY(hipMemsetAsync(nx, 0, (size_t)new_cap * 4, h->stream));
        if (h->xnorm) HIP_TRY(hipMemcpyAsync(nx, h->xnorm, (size_t)h->cap * 4, hipMemcpyDeviceToDevice, h->stream));
    }
    if (h->rows) {
        HIP_TRY(hipMemcpyAsync(nr, h->rows, (size_t)(h->cap / 32) * tb, hipMemcpyDeviceToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync(nl, h->live, (size_t)(h->cap / 32) * 4, hipMemcpyDeviceToDevice, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        HIP_TRY(hipFree(h->rows));
        HIP_TRY(hipFree(h->live));
    }
    if (h->xnorm) {
        HIP_TRY(hipStreamSynchronize(h->stream));
        HIP_TRY(hipFree(h->xnorm));
    }
    if (h->shadow) {  // the 16-bit shadow grows with the rows (its converted tiles carried over)
        const size_t tb16 = (size_t)h->S * 1024;
        uint8_t* n16 = nullptr;
        if (hipMalloc(&n16, (size_t)(new_cap / 32) * tb16) != hipSuccess) {
            // no room for it beside the fp32 rows (a corpus of more than ~2/3 of the device): the index goes on
            // without a shadow, scanning the fp32 tiles as before (plans follow scan_dtype)
            (void)hipGetLastError();
            HIP_TRY(hipStreamSynchronize(h->stream));
            if (h->rows16) HIP_TRY(hipFree(h->rows16));
            h->rows16 = nullptr;
            h->shadow = false;
            h->shadow_lo = INT64_MAX;
        } else {
            HIP_TRY(hipMemsetAsync(n16, 0, (size_t)(new_cap / 32) * tb16, h->stream));
            if (h->rows16) {
                HIP_TRY(hipMemcpyAsync(n16, h->rows16, (size_t)(h->cap / 32) * tb16, hipMemcpyDeviceToDevice, h->stream));
                HIP_TRY(hipStreamSynchronize(h->stream));
                HIP_TRY(hipFree(h->rows16));
            }
            h->rows16 = n16;
        }
    }
    h->rows = nr;
    h->live = nl;
    h->xnorm = nx;
    h->cap = new_cap;
    h->live_host.resize((size_t)(new_cap / 32), 0u);
    return HR_OK;
}

extern "C" int hr_index_reserve(hr_index* h, int64_t capacity_rows) {
    if (!h || capacity_rows < 0) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = async_drain(h)) return rc;  // asynchronous batches in flight read the rows
    if (h->G > 1) return group_reserve(h, capacity_rows);
    if (int rc = set_device(h)) return rc;
    return index_grow(h, capacity_rows);
}

static int mark_live(hr_index* h, int64_t r0, int64_t n) {
    if (n <= 0) return HR_OK;
    for (int64_t r = r0; r < r0 + n; ++r) h->live_host[(size_t)(r >> 5)] |= 1u << (r & 31);
    const int64_t w0 = r0 >> 5, w1 = (r0 + n - 1) >> 5;
    HIP_TRY(hipMemcpyAsync(h->live + w0, h->live_host.data() + w0, (size_t)(w1 - w0 + 1) * 4, hipMemcpyHostToDevice,
                           h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));  // live_host may be modified again by the caller's next call
    h->n_live += n;
    return HR_OK;
}

static int finish_add(hr_index* h) {
    unsigned long long bits = 0;
    HIP_TRY(hipMemcpyAsync(&bits, h->norm_bits, sizeof(bits), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    double v;
    std::memcpy(&v, &bits, 8);
    h->max_norm2 = std::max(h->max_norm2, v);
    return HR_OK;
}

// euclidean: fp32 |x|^2 of stored rows [r0, r0 + n) for the approximate scan score
int index_update_row_norms(hr_index* h, int64_t r0, int64_t n) {
    if (h->metric != L2 || n <= 0) return HR_OK;
    return dispatch_dt(h->dtype, [&](auto dt) -> int {
        hipLaunchKernelGGL((k_row_norms<decltype(dt)::value>), dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream,
                           h->rows, h->S, h->dpad, r0, n, h->xnorm);
        HIP_TRY(hipGetLastError());
        return HR_OK;
    });
}

// SRC: where the fp32 rows come from (host memory staged through h->stage, the generator, or device memory).
enum { ADD_HOST = 0, ADD_SYNTH = 1, ADD_DEVICE = 2 };

// ADD_SYNTH: local row L gets generator row gen_base + stripe_row(L) (hr_common.hpp)
template <int SRC>
static int add_impl(hr_index* h, const float* rows, uint64_t seed, int64_t gen_base, int64_t n, int64_t* first) {
    constexpr bool SYNTH = SRC == ADD_SYNTH;
    if (int rc = set_device(h)) return rc;
    if (int rc = index_grow(h, h->n + n)) return rc;
    const int64_t r0 = h->n;
    const int64_t chunk = SYNTH ? (int64_t)1 << 22 : std::max<int64_t>(1, ((int64_t)64 << 20) / (4 * h->dim));
    for (int64_t off = 0; off < n; off += chunk) {
        const int64_t m = std::min(chunk, n - off);
        const float* src = nullptr;
        if (SRC == ADD_HOST) {
            HIP_TRY(h->stage.ensure((size_t)m * h->dim * 4));
            HIP_TRY(hipMemcpyAsync(h->stage.p, rows + off * h->dim, (size_t)m * h->dim * 4, hipMemcpyHostToDevice,
                                   h->stream));
            src = h->stage.as<float>();
        } else if (SRC == ADD_DEVICE) {
            src = rows + off * h->dim;
        }
        const dim3 grid((unsigned)((m + 3) / 4));
        int rc = dispatch_dt(h->dtype, [&](auto dt) -> int {
            hipLaunchKernelGGL((k_store<decltype(dt)::value, SYNTH>), grid, dim3(256), 0, h->stream, src, seed,
                               gen_base, m, h->dim, h->S, h->metric, r0 + off, h->rows, h->norm_bits, nullptr,
                               h->stripe_G, h->stripe_s);
            HIP_TRY(hipGetLastError());
            return HR_OK;
        });
        if (rc) return rc;
    }
    h->n = r0 + n;
    shadow_stale(h, r0 / 32);
    if (int rc = index_update_row_norms(h, r0, n)) return rc;
    if (int rc = mark_live(h, r0, n)) return rc;
    if (int rc = finish_add(h)) return rc;
    if (first) *first = r0;
    return HR_OK;
}

int index_add_host(hr_index* h, const float* rows, int64_t n, int64_t* first) {
    return add_impl<ADD_HOST>(h, rows, 0, 0, n, first);
}
int index_add_synthetic(hr_index* h, uint64_t seed, int64_t gen_base, int64_t n) {
    return add_impl<ADD_SYNTH>(h, nullptr, seed, gen_base, n, nullptr);
}

static int64_t max_rows(const hr_index* h) { return (((int64_t)1 << 32) - 64) * h->G; }

extern "C" int hr_index_add(hr_index* h, const float* rows, int64_t n, int64_t* first_row_out) {
    if (!h || n < 0 || (n > 0 && !rows)) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = async_drain(h)) return rc;  // asynchronous batches in flight read the rows
    if (h->n + n > max_rows(h)) return set_err(HR_E_INVALID, "a shard holds at most 2^32 rows");
    if (n == 0) {
        if (first_row_out) *first_row_out = h->n;
        return HR_OK;
    }
    if (h->G > 1) return group_add_host(h, rows, n, first_row_out);
    return add_impl<ADD_HOST>(h, rows, 0, 0, n, first_row_out);
}

extern "C" int hr_index_add_synthetic(hr_index* h, uint64_t seed, int64_t global_row0, int64_t n,
                                      int64_t* first_row_out) {
    if (!h || n < 0 || global_row0 < 0) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = async_drain(h)) return rc;  // asynchronous batches in flight read the rows
    if (h->n + n > max_rows(h)) return set_err(HR_E_INVALID, "a shard holds at most 2^32 rows");
    if (n == 0) {
        if (first_row_out) *first_row_out = h->n;
        return HR_OK;
    }
    if (h->G > 1) return group_add_synthetic(h, seed, global_row0, n, first_row_out);
    return add_impl<ADD_SYNTH>(h, nullptr, seed, global_row0 - h->n, n, first_row_out);
}

extern "C" int hr_index_add_device_at(hr_index* h, const float* rows_dev, int64_t n, const int64_t* dest_dev,
                                      int64_t n_rows_after, void* stream) {
    if (!h || n < 0 || (n > 0 && (!rows_dev || !dest_dev))) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = async_drain(h)) return rc;  // asynchronous batches in flight read the rows
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "explicit row placement (IVF lists) needs a single-device index");
    if (n_rows_after < h->n || n_rows_after > ((int64_t)1 << 32) - 64)
        return set_err(HR_E_INVALID, "n_rows_after must be >= the current size and < 2^32");
    if (int rc = set_device(h)) return rc;
    if (int rc = index_grow(h, n_rows_after)) return rc;
    hipEvent_t ev;  // order after the producer of rows_dev / dest_dev on the caller's stream
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ev, (hipStream_t)stream));
    HIP_TRY(hipStreamWaitEvent(h->stream, ev, 0));
    HIP_TRY(hipEventDestroy(ev));
    if (n > 0) {
        int rc = dispatch_dt(h->dtype, [&](auto dt) -> int {
            hipLaunchKernelGGL((k_store<decltype(dt)::value, false>), dim3((unsigned)((n + 3) / 4)), dim3(256), 0,
                               h->stream, rows_dev, 0, 0, n, h->dim, h->S, h->metric, 0, h->rows, h->norm_bits, dest_dev);
            HIP_TRY(hipGetLastError());
            if (h->metric == L2)
                hipLaunchKernelGGL((k_row_norms<decltype(dt)::value>), dim3((unsigned)((n + 3) / 4)), dim3(256), 0,
                                   h->stream, h->rows, h->S, h->dpad, 0, n, h->xnorm, dest_dev);
            HIP_TRY(hipGetLastError());
            return HR_OK;
        });
        if (rc) return rc;
        hipLaunchKernelGGL(k_mark_live, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, dest_dev, n, h->live);
        HIP_TRY(hipGetLastError());
        shadow_stale(h, 0);  // (rows placed anywhere)
    }
    h->n = n_rows_after;
    const int64_t words = (h->n + 31) / 32;
    HIP_TRY(hipMemcpyAsync(h->live_host.data(), h->live, (size_t)words * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    int64_t live = 0;
    for (int64_t w = 0; w < words; ++w) live += __builtin_popcount(h->live_host[(size_t)w]);
    h->n_live = live;
    return finish_add(h);
}

extern "C" int hr_gen_rows_device(uint64_t seed, int64_t row0, int64_t n, int dim, float* out_dev, void* stream) {
    if (n < 0 || dim <= 0 || (n > 0 && !out_dev)) return set_err(HR_E_INVALID, "bad arguments");
    if (n == 0) return HR_OK;
    const int64_t total = n * dim;
    hipLaunchKernelGGL(k_gen_rows, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, seed, row0,
                       n, dim, out_dev);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}

extern "C" int hr_index_add_device(hr_index* h, const float* rows_dev, int64_t n, int64_t* first_row_out,
                                   void* stream) {
    if (!h || n < 0 || (n > 0 && !rows_dev)) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = async_drain(h)) return rc;  // asynchronous batches in flight read the rows
    if (h->n + n > max_rows(h)) return set_err(HR_E_INVALID, "a shard holds at most 2^32 rows");
    if (n == 0) {
        if (first_row_out) *first_row_out = h->n;
        return HR_OK;
    }
    if (h->G > 1) return group_add_device(h, rows_dev, n, first_row_out, (hipStream_t)stream);
    if (int rc = set_device(h)) return rc;
    // the rows are produced on the caller's stream (e.g. the embedder's pooling kernel): order the store after it.
    // add_impl synchronises h->stream before returning, so the caller may reuse rows_dev afterwards.
    hipEvent_t ev;
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipError_t e = hipEventRecord(ev, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(h->stream, ev, 0);
    (void)hipEventDestroy(ev);
    HIP_TRY(e);
    return add_impl<ADD_DEVICE>(h, rows_dev, 0, 0, n, first_row_out);
}

extern "C" int hr_index_remove(hr_index* h, const int64_t* rows, int64_t n) {
    if (!h || n < 0 || (n > 0 && !rows)) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = async_drain(h)) return rc;  // asynchronous batches in flight read the rows
    if (h->G > 1) return group_remove(h, rows, n);
    return index_remove_local(h, rows, n);
}

int index_remove_local(hr_index* h, const int64_t* rows, int64_t n) {
    if (int rc = set_device(h)) return rc;
    // validate every row before touching anything: a failed call leaves host and device bits as they were
    for (int64_t i = 0; i < n; ++i)
        if (rows[i] < 0 || rows[i] >= h->n) return set_err(HR_E_INVALID, "row out of range");
    int64_t lo = INT64_MAX, hi = -1;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t r = rows[i];
        uint32_t& w = h->live_host[(size_t)(r >> 5)];
        const uint32_t bit = 1u << (r & 31);
        if (w & bit) {
            w &= ~bit;
            h->n_live--;
        }
        lo = std::min(lo, r >> 5);
        hi = std::max(hi, r >> 5);
    }
    if (hi >= 0) {
        HIP_TRY(hipMemcpyAsync(h->live + lo, h->live_host.data() + lo, (size_t)(hi - lo + 1) * 4,
                               hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    return HR_OK;
}

extern "C" int hr_index_size(hr_index* h, int64_t* n_out, int64_t* n_live_out) {
    if (!h) return set_err(HR_E_INVALID, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    if (n_out) *n_out = h->n;
    int64_t live = h->n_live;
    if (h->G > 1) {
        live = 0;
        for (hr_index* s : h->shards) live += s->n_live;
    }
    if (n_live_out) *n_live_out = live;
    return HR_OK;
}

extern "C" int hr_index_info(hr_index* h, int* dim_out, int* dtype_out, int* metric_out, int* n_dev_out) {
    if (!h) return set_err(HR_E_INVALID, "null handle");
    if (dim_out) *dim_out = h->dim;
    if (dtype_out) *dtype_out = h->dtype;
    if (metric_out) *metric_out = h->metric;
    if (n_dev_out) *n_dev_out = h->G;
    return HR_OK;
}

// ---------------------------------------------------------------- search pieces
// A/B knobs of the scan plan, read once (timing studies; the defaults are the measured choices):
// HIPRAG_TAIL_CUS (32), HIPRAG_SAMPLE_MIN (1024: sampled tiles of a shard <= 80k tiles), HIPRAG_DYN_PCT (10),
// HIPRAG_REFRESH_EVERY (0 = by shard size: group-maxima refreshes every 8 tiles on shards of <= 160k tiles, every 4
// above -- 1.25M x 1024: 0.403-0.406 against 0.410-0.418 ms/step; 5M: 1.494-1.497 against 1.516-1.519; 1M x 768 and
// 2.5M unchanged; 10M x 1024: 2.97-3.03 against 2.94-2.95 ms; three alternating repeats each,
// profiles/r06_refresh_every_ab.jsonl)
static int knob(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}
static const int kTailCus = knob("HIPRAG_TAIL_CUS", 32);
static const int kSampleMin = knob("HIPRAG_SAMPLE_MIN", 1024);
static const int kDynPct = knob("HIPRAG_DYN_PCT", 10);
static const int kRefreshEvery = std::max(0, knob("HIPRAG_REFRESH_EVERY", 0));
static int refresh_every(int64_t n_tiles) { return kRefreshEvery ? kRefreshEvery : (n_tiles <= 160 * 1024 ? 8 : 4); }

struct Plan {
    int QB, Bp, P;
    int NG;  // query groups per corpus pass (each QB*32 queries in one workgroup's LDS); Bp = NG*QB*32
};

static int scan_lds_bytes(const hr_index* h, int QB) { return h->S * QB * 1024; }

static int make_plan(const hr_index* h, int B, Plan* p) {
    const int QB = (B > 32 && scan_lds_bytes(h, 2) <= 160 * 1024) ? 2 : 1;
    if (scan_lds_bytes(h, QB) > 160 * 1024)
        return set_err(HR_E_UNSUPPORTED, "dim too large for the LDS-resident query tile (max 2560)");
    p->QB = QB;
    // More than 64 queries: up to 4 groups of 64 share one corpus pass -- each group's workgroups stream the
    // same tiles on one XCD, the others reading them from L2 (DESIGN.md "Query groups").  fp32 corpora (2 KiB
    // k-steps) form groups only at the dims the 128-query FILTER takes (below); elsewhere they keep one group.
    constexpr int max_groups = 4;
    // (fp32 rows form groups only where the 128-query FILTER takes them: its eight-wave form reads fp32 rows)
    const int sdt = scan_dtype(h);
    p->NG = (QB == 2 && (sdt != F32 || wide_filter_ok(sdt, h->S))) ? std::max(1, std::min(max_groups, (B + 63) / 64)) : 1;
    // D > 1280 (Youtu-Embedding's 2048 / 2304 dims) leaves LDS for one 32-query block only: a 64-query
    // batch was two corpus passes; 32-query groups share one (2M x 2304: 3.03 -> 1.98 ms/batch)
    if (QB == 1 && B > 32 && sdt != F32) p->NG = std::max(1, std::min(max_groups, (B + 31) / 32));
    // the 128-query FILTER (hr_wide.hip) serves query groups in pairs: round the group count up to even
    if (p->NG > 1 && QB == 2 && wide_filter_ok(sdt, h->S)) p->NG = (p->NG + 1) & ~1;
    p->Bp = p->NG * QB * 32;
    // ring depth: deepest prefetch that compiles without spills (see `make resource`)
    const int pmax = sdt == F32 ? (QB == 2 ? 4 : 8) : 16;
    p->P = (h->S % 16 == 0 && pmax >= 16) ? 16 : (h->S % 8 == 0 && pmax >= 8 ? 8 : 4);
    return HR_OK;
}

// the FILTER of this plan runs as the 128-query pass (hr_wide.hip): query groups in pairs, D a multiple of 256 up to
// 1024, no tile list, row parts as below
static bool wide_plan(const hr_index* h, const Plan& pl, int np, bool tile_list) {
    // Row parts: fp32 rows up to the LDS's 7 (10M x 1024, B = 128, pipelined: k = 20 / 50 / 100 at 20.0k / 19.0k /
    // 17.3k QPS vs the query groups' 16.2k / 16.0k / 15.7k); 16-bit rows up to 3 parts and one 128-query set
    // (bf16, k = 20 / 50: B = 128 31.9k / 29.6k vs 28.2k / 27.6k QPS, but B = 256 32.4k / 29.8k vs 33.0k / 32.2k,
    // and k = 100's 5 parts FILTER in 5.0 vs 4.5 ms: the appends of its slower-rising thresholds cost more than
    // the L2 re-reads of the groups; profiles/r03_wide_parts_*)
    const bool f32 = scan_dtype(h) == F32;
    const int max_parts = std::min(f32 ? 7 : 3, wide_max_parts(scan_dtype(h)));
    const bool parts_ok = np <= max_parts && (f32 || pl.NG == 2);
    return pl.NG >= 2 && pl.QB == 2 && !tile_list && (np == 1 || parts_ok) && wide_filter_ok(scan_dtype(h), h->S);
}

// dynamic tail of a FILTER over W waves: the last 10 % of the units go out in 2-unit runs from the counter, but
// only when every wave still gets a long static run (DESIGN.md "Dynamic tail"; profiles/r03_shard1.25M_knob_sweep.log)
static void set_dyn_tail(ScanArgs& args, int64_t W, uint32_t* dyn_q) {
    const int pct = kDynPct;
    const int64_t per_wave = args.n_units / W;
    args.dyn_start = args.n_units;
    if (per_wave >= 8 && dyn_q) {
        // static runs and dynamic runs are >= 2 units (the grab is issued one unit early)
        const int64_t s_per = per_wave - std::max<int64_t>(2, per_wave * pct / 100);
        args.dyn_start = s_per * W;
        args.dyn_pct = pct;
        args.dyn_chunk = 2;
        args.dyn_q = dyn_q;
    }
}

template <int MT, int DT, int QB, int P, int MODE, bool NT, int TPB = kScanThreads>
static int launch_scan_t(hr_index* h, Scratch& sc, int cus, const ScanArgs& a, hipStream_t st, int lds) {
    const int ng = std::max(1, a.ng);
    auto kern = scan_kernel<MT, DT, QB, P, MODE, NT, TPB>();
    static std::mutex attr_mu;
    static int attr_lds[64] = {};     // per device: largest dynamic LDS already allowed
    static int occ[64][4] = {};       // per device: blocks/CU for lds buckets (0 = unknown), per instantiation
    const int dev = h->device & 63;
    const int bucket = lds <= 40 * 1024 ? 0 : lds <= 80 * 1024 ? 1 : lds <= 120 * 1024 ? 2 : 3;
    int per_cu;
    {
        std::lock_guard<std::mutex> lk(attr_mu);
        if (attr_lds[dev] < 160 * 1024) {
            HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            attr_lds[dev] = 160 * 1024;
        }
        if (!occ[dev][bucket]) {
            int o = 0;
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, TPB, lds));
            occ[dev][bucket] = std::max(1, o);
        }
        per_cu = occ[dev][bucket];
    }
    // blocks per query group (each group's workgroups cover the whole unit range); with several
    // groups a multiple of 8, so the groups of one range block share blockIdx % 8 (k_scan)
    int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * per_cu / ng, (a.n_units + 7) / 8));
    if (ng > 1) blocks = std::max<int64_t>(8, blocks / 8 * 8);
    ScanArgs args = a;
    args.ng = ng;
    if (MODE == SCAN_FILTER) {
        const int64_t W = blocks * (TPB / 64);  // waves per group
        const int Bq = QB * 32;
        HIP_TRY(sc.pbuf.ensure((size_t)ng * Bq * W * kCapW * sizeof(float2)));
        HIP_TRY(sc.pcnt.ensure((size_t)ng * Bq * W * 4));
        HIP_TRY(sc.wtiles.ensure((size_t)ng * W * 4));
        args.wave_tiles = sc.wtiles.as<uint32_t>();
        sc.wtiles_valid = true;
        args.pbuf = sc.pbuf.as<float2>();
        args.pcnt = sc.pcnt.as<uint32_t>();
        args.capw = kCapW;
        sc.last_W = W;
        sc.last_Bp = Bq;
        sc.last_ng = ng;
        sc.last_capw = kCapW;
        h->last_scr = &sc;
        set_dyn_tail(args, W, sc.dyn_q.as<uint32_t>());
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)(blocks * ng)), dim3(TPB), lds, st, args);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}

template <int MT, int DT, int MODE>
static int launch_scan_p(hr_index* h, Scratch& sc, int cus, const Plan& pl, const ScanArgs& a, hipStream_t st) {
    int lds = scan_lds_bytes(h, pl.QB);
    // SAMPLE reduces its waves' group maxima in LDS: 8 waves x QB*16*64 floats + 8 part ids
    if (MODE == SCAN_SAMPLE) lds = std::max(lds, (kScanThreads / 64) * pl.QB * 16 * 64 * 4 + 64);
    // Default-policy corpus loads for query groups (the other groups read the tiles from L2) and for
    // the SAMPLE pass: its tiles are the same every batch (unit * stride), and the FILTER's
    // non-temporal stream does not evict them from the Infinity Cache, so after the first batch the
    // SAMPLE is served on-die instead of taking HBM time from the FILTER beside it
    // (1.25M rows: 0.442 -> 0.437 ms/step, profiles/r02_sample_policy_ab.jsonl)
    const bool dflt = pl.NG > 1 || MODE == SCAN_SAMPLE;
    // more than 64 queries (query groups) in a plain FILTER: the 128-query pass reads every tile once for
    // two groups (hr_wide.hip) instead of one workgroup per group streaming the same tiles through L2
    if constexpr (MODE == SCAN_FILTER) {
        if (wide_plan(h, pl, a.np, a.tile_list != nullptr) && a.use_groups) {
            // 129-256 queries (four groups), one row part: ONE pass of the 256-query FILTER (hr_q256.hip) instead of
            // two of the 128-query one
            if (pl.NG == 4 && a.np == 1 && h->q256 && q256_filter_ok(scan_dtype(h), h->S)) {
                const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(cus, (a.n_units + 7) / 8));
                const int64_t W = (int64_t)blocks * 4;  // waves: one candidate region per (group, wave)
                HIP_TRY(sc.pbuf.ensure((size_t)4 * 64 * W * kCapW * sizeof(float2)));
                HIP_TRY(sc.pcnt.ensure((size_t)4 * 64 * W * 4));
                sc.last_W = W;
                sc.last_Bp = 64;
                sc.last_ng = 4;
                sc.last_capw = kCapW;
                sc.wtiles_valid = false;
                h->last_scr = &sc;
                ScanArgs b = a;
                b.pbuf = sc.pbuf.as<float2>();
                b.pcnt = sc.pcnt.as<uint32_t>();
                b.capw = kCapW;
                if (int rc = launch_filter_q256(MT, DT, h->S, blocks, b, st)) return set_err(rc, "256-query FILTER launch failed");
                h->n_q256++;
                return HR_OK;
            }
            // waves: one candidate region per (group, wave); a wave takes one tile per round
            constexpr int wpb = 8;
            const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(cus, (a.n_units + wpb - 1) / wpb));
            const int64_t W = (int64_t)blocks * wpb;
            HIP_TRY(sc.pbuf.ensure((size_t)pl.NG * 64 * W * kCapW * sizeof(float2)));
            HIP_TRY(sc.pcnt.ensure((size_t)pl.NG * 64 * W * 4));
            sc.last_W = W;
            sc.last_Bp = 64;
            sc.last_ng = pl.NG;
            sc.last_capw = kCapW;
            sc.wtiles_valid = false;
            h->last_scr = &sc;
            for (int set = 0; set < pl.NG / 2; ++set) {  // two groups per launch
                ScanArgs b = a;
                b.qfrag = a.qfrag + (int64_t)set * 2 * h->S * 2 * 64 * 8;
                b.mkeys = a.mkeys + set * 128 * 32;
                b.floor_q = a.floor_q + set * 128;
                b.pbuf = sc.pbuf.as<float2>() + (int64_t)set * 2 * W * 64 * kCapW;
                b.pcnt = sc.pcnt.as<uint32_t>() + (int64_t)set * 2 * W * 64;
                b.capw = kCapW;
                if (int rc = launch_filter_wide(MT, DT, h->S, blocks, b, st)) return set_err(rc, "wide FILTER launch failed");
                h->n_wide++;
            }
            return HR_OK;
        }
    }
#define HR_SCAN_CASE(QBv, Pv)                                                                     \
    if (pl.QB == QBv && pl.P == Pv)                                                               \
        return dflt ? launch_scan_t<MT, DT, QBv, Pv, MODE, false>(h, sc, cus, a, st, lds)         \
                    : launch_scan_t<MT, DT, QBv, Pv, MODE, true>(h, sc, cus, a, st, lds);
    if constexpr (DT == F32) {
        HR_SCAN_CASE(1, 8) HR_SCAN_CASE(1, 4) HR_SCAN_CASE(2, 4)
    } else {
        HR_SCAN_CASE(1, 16) HR_SCAN_CASE(2, 16) HR_SCAN_CASE(1, 8) HR_SCAN_CASE(2, 8) HR_SCAN_CASE(1, 4)
        HR_SCAN_CASE(2, 4)
    }
#undef HR_SCAN_CASE
    return set_err(HR_E_INVALID, "no scan variant for this plan");
}

static int launch_scan(hr_index* h, Scratch& sc, int cus, const Plan& pl, const ScanArgs& a, int mode,
                       hipStream_t st) {
    return dispatch_dt(scan_dtype(h), [&](auto dt) -> int {
        constexpr int DT = decltype(dt)::value;
        auto go = [&](auto mt) -> int {
            constexpr int MT = decltype(mt)::value;
            if (mode == SCAN_SAMPLE) return launch_scan_p<MT, DT, SCAN_SAMPLE>(h, sc, cus, pl, a, st);
            if (mode == SCAN_FILTER) return launch_scan_p<MT, DT, SCAN_FILTER>(h, sc, cus, pl, a, st);
            return launch_scan_p<MT, DT, SCAN_COLLECT>(h, sc, cus, pl, a, st);
        };
        if constexpr (DT == F32) {  // fp32 rows: the MFMA type follows the metric (mfma_type)
            if (mfma_type(h) == F16) return go(std::integral_constant<int, F16>{});
            return go(std::integral_constant<int, BF16>{});
        } else {
            return go(std::integral_constant<int, DT == F16 ? F16 : BF16>{});
        }
    });
}

// CUs left to the tail stream while a pipelined scan runs: the scan reads HBM at the same rate
// on 224 of the 256 CUs (measured: 6.85 vs 6.81 TB/s at 10M rows, 0.434 vs 0.427 ms at 1.25M),
// so select/rescore, the RCCL all-gather and the merge of the previous batch run beside it
static int tail_cus(const hr_index* h) {
    return std::max(0, std::min(kTailCus, h->n_cu - 8));
}

// ---- persistent FILTER: configuration, quiesce, close
// Waits whenever instances were launched since the last quiesce, whether or not the gate is still open: a close
// (persist_close) only stops admissions, the instance may still be scanning the rows a mutation is about to change
// (ADVICE r04).  A bounded wait that gave up meanwhile is cleared here: the batch it concerned was failed over to the
// exact collect pass (PersistCtl::slot_fail), so it is counted (hr_index_persist_stats), not returned.
static int persist_quiesce(hr_index* h) {
    Persist* ps = h->ps;
    if (!ps || !(ps->active || ps->launched)) return HR_OK;
    if (int rc = set_device(h)) return rc;
    PersistCtl* c = ps->ctl.as<PersistCtl>();
    if (ps->active)
        if (int rc = launch_persist_close(c, h->pre)) return rc;  // behind every post (same stream)
    HIP_TRY(hipStreamSynchronize(h->pre));
    HIP_TRY(hipStreamSynchronize(ps->pst));                   // every instance has exited
    HIP_TRY(hipMemsetAsync(&c->stop, 0, 4, ps->pst));
    HIP_TRY(hipStreamSynchronize(ps->pst));
    ps->active = ps->launched = false;
    if (ps->host_err && *(volatile uint32_t*)ps->host_err) {
        ps->timeouts++;
        ps->last_err = *(volatile uint32_t*)ps->host_err;
        *(volatile uint32_t*)ps->host_err = 0;
        HIP_TRY(hipMemset(&c->error, 0, 4));
    }
    return HR_OK;
}

static int persist_close(hr_index* h) {
    Persist* ps = h->ps;
    if (!ps || !ps->active) return HR_OK;
    if (int rc = set_device(h)) return rc;
    if (int rc = launch_persist_close(ps->ctl.as<PersistCtl>(), h->pre)) return rc;
    // the next batch finds the gate closed and starts an instance of its own, which reopens it.  stop is cleared on
    // the instances' stream -- behind the running instance AND behind the close (event): cleared first, a late close
    // would leave stop set and every later instance serving its own batch only
    HIP_TRY(hipEventRecord(ps->closed, h->pre));
    HIP_TRY(hipStreamWaitEvent(ps->pst, ps->closed, 0));
    HIP_TRY(hipMemsetAsync(&ps->ctl.as<PersistCtl>()->stop, 0, 4, ps->pst));
    ps->active = false;  // (launched stays: a quiesce still waits for the instance)
    return HR_OK;
}

static void persist_free(hr_index* h) {
    Persist* ps = h->ps;
    if (!ps) return;
    (void)persist_quiesce(h);
    ps->drop_views();
    for (auto& sc : ps->slot) sc.release_all();
    for (DevBuf* b : {&ps->ar_qfrag, &ps->ar_mkeys, &ps->ar_floor, &ps->ar_pbuf, &ps->ar_pcnt, &ps->ar_dynq, &ps->ctl})
        b->release();
    for (auto& e : ps->posted)
        if (e) (void)hipEventDestroy(e);
    if (ps->closed) (void)hipEventDestroy(ps->closed);
    if (ps->pst) (void)hipStreamDestroy(ps->pst);
    if (ps->host_err) (void)hipHostFree(ps->host_err);
    delete ps;
    h->ps = nullptr;
}

// The persistent FILTER serves this pipelined batch?  Unmasked, one 64-query tile (one group, one row part: k <= 16),
// not the 128-query FILTER, a plan it is built for, early-SAMPLE conditions met, a single-device index (not a group
// shard), and (mode 1) a shard where it measured faster than per-batch launches: 128k-160k tiles (4.2M-5.1M rows: the
// 5M-row shard of a 10M corpus at G = 2, 1.532-1.558 vs 1.581-1.606 ms/step on two boxes).  Below that the dual
// FILTER streams already hide each launch's ramp and tail and the instance's per-batch hand-off costs more (1.25M
// rows: 0.435 ms device period vs 0.427-0.432 ms/step; 2.5M: 0.794 vs 0.805; 625k: the SAMPLE chain bounds both),
// and the single-stream 10M launch equals it (2.992 vs 3.003 ms; profiles/r04_persist_vs_launches_shard_sweep.jsonl,
// r04_persist_sc1_shard_sweep.jsonl).
static bool persist_wanted(hr_index* h, const Plan& pl, int np, bool early, const uint64_t* mask_dev, int64_t n_tiles) {
    const int mode = h->ps ? h->ps->mode : 1;
    if (mode == 0 || !early || mask_dev || np != 1 || pl.NG != 1 || pl.QB != 2 || h->stripe_G != 1) return false;
    if (!(scan_dtype(h) != F32 ? pl.P == 16 : pl.P == 4)) return false;
    return mode == 2 || (n_tiles >= 128 * 1024 && n_tiles <= 160 * 1024);
}

// (re)configure for the current corpus and plan: arenas sized for one 64-query tile per slot
static int persist_configure(hr_index* h, const Plan& pl) {
    if (!h->ps) h->ps = new Persist();
    Persist& ps = *h->ps;
    const int64_t n_tiles = (h->n + 31) / 32;
    const int nwg = h->n_cu - tail_cus(h);
    if (ps.ready && ps.key_n == h->n && ps.key_rows == h->rows && ps.key_S == h->S && ps.key_P == pl.P &&
        ps.key_ncu == h->n_cu)
        return HR_OK;
    if (int rc = persist_quiesce(h)) return rc;
    if ((n_tiles + 7) / 8 < nwg) return set_err(HR_E_UNSUPPORTED, "shard too small for the persistent FILTER");
    if (!ps.pst) {
        HIP_TRY(index_stream_create(h, &ps.pst, true));
        for (auto& e : ps.posted) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&ps.closed, hipEventDisableTiming));
        HIP_TRY(hipHostMalloc((void**)&ps.host_err, 64));
        *ps.host_err = 0;
        HIP_TRY(ps.ctl.ensure(sizeof(PersistCtl)));
        std::vector<PersistCtl> init(1);  // (value-initialised: zero arrival words and stamps; ~200 KB, not on the stack)
        init[0].gate = 0x80000000u;  // closed: the first batch starts an instance of its own
        init[0].next_epoch = 1;
        HIP_TRY(hipMemcpy(ps.ctl.p, init.data(), sizeof(PersistCtl), hipMemcpyHostToDevice));
    }
    auto up = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    const int64_t W = (int64_t)nwg * (kScanThreads / 64);
    ps.st_qfrag = up((int64_t)h->S * pl.QB * 1024);
    ps.st_mkeys = up((int64_t)pl.Bp * 32 * 4);
    ps.st_floor = up((int64_t)pl.Bp * 4);
    ps.st_pbuf = up((int64_t)pl.Bp * W * kCapW * (int64_t)sizeof(float2));
    ps.st_pcnt = up((int64_t)pl.Bp * W * 4);
    ps.st_dynq = 256;
    ps.drop_views();
    const int R = kPersistSlots;
    HIP_TRY(ps.ar_qfrag.ensure((size_t)(R * ps.st_qfrag)));
    HIP_TRY(ps.ar_mkeys.ensure((size_t)(R * ps.st_mkeys)));
    HIP_TRY(ps.ar_floor.ensure((size_t)(R * ps.st_floor)));
    HIP_TRY(ps.ar_pbuf.ensure((size_t)(R * ps.st_pbuf)));
    HIP_TRY(ps.ar_pcnt.ensure((size_t)(R * ps.st_pcnt)));
    HIP_TRY(ps.ar_dynq.ensure((size_t)(R * ps.st_dynq)));
    for (int s = 0; s < R; ++s) {
        Scratch& sc = ps.slot[s];
        auto view = [&](DevBuf& v, DevBuf& ar, int64_t st) {
            v.p = (uint8_t*)ar.p + s * st;
            v.bytes = (size_t)st;
        };
        view(sc.qfrag, ps.ar_qfrag, ps.st_qfrag);
        view(sc.mkeys, ps.ar_mkeys, ps.st_mkeys);
        view(sc.floor_q, ps.ar_floor, ps.st_floor);
        view(sc.pbuf, ps.ar_pbuf, ps.st_pbuf);
        view(sc.pcnt, ps.ar_pcnt, ps.st_pcnt);
        view(sc.dyn_q, ps.ar_dynq, ps.st_dynq);
        sc.last_W = W;
        sc.last_Bp = pl.Bp;
        sc.last_ng = 1;
        sc.last_capw = kCapW;
    }
    ps.nwg = nwg;
    ps.key_n = h->n;
    ps.key_rows = h->rows;
    ps.key_S = h->S;
    ps.key_P = pl.P;
    ps.key_ncu = h->n_cu;
    ps.ready = true;
    return HR_OK;
}

// fp32 tiles [t0, t1) -> the 16-bit shadow: k-step chunk c of a tile, lane l -> the 8 elements XFrag<MT, F32> forms
// from bytes l*16 of the chunk's two KiB halves, rounded to MT the same way (packed hardware RNE)
template <int MT>
__global__ __launch_bounds__(256) void k_shadow(const uint8_t* __restrict__ rows, uint8_t* __restrict__ rows16, int S,
                                                int64_t t0, int64_t t1) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (tile - t0) * S * 64 + chunk * 64 + lane
    const int64_t per_tile = (int64_t)S * 64;
    if (i >= (t1 - t0) * per_tile) return;
    const int64_t t = t0 + i / per_tile, c = (i % per_tile) >> 6;
    const int lane = (int)(i & 63);
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    typedef float f32x8 __attribute__((ext_vector_type(8)));
    const uint8_t* src = rows + (t * S + c) * 2048 + lane * 16;
    const f32x4 fa = *(const f32x4*)src, fb = *(const f32x4*)(src + 1024);
    const f32x8 f = __builtin_shufflevector(fa, fb, 0, 1, 2, 3, 4, 5, 6, 7);
    u32x4 o;
    if constexpr (MT == BF16) o = __builtin_bit_cast(u32x4, __builtin_convertvector(f, bf16x8));
    else o = __builtin_bit_cast(u32x4, __builtin_convertvector(f, f16x8));
    *(u32x4*)(rows16 + (t * S + c) * 1024 + lane * 16) = o;
}

// bring the shadow up to the rows (h->stream, synchronous; never inside a capture: the graph path calls it first)
int shadow_update(hr_index* h) {
    if (!h->rows16 || h->shadow_lo == INT64_MAX) return HR_OK;
    const int64_t t1 = (h->n + 31) / 32, t0 = std::min(h->shadow_lo, t1);
    if (t1 > t0) {
        if (int rc = set_device(h)) return rc;
        const int64_t work = (t1 - t0) * h->S * 64;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, h->stream, h->rows, h->rows16, h->S,
                               t0, t1);
        };
        if (mfma_type(h) == BF16) go(k_shadow<BF16>);
        else go(k_shadow<F16>);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    h->shadow_lo = INT64_MAX;
    return HR_OK;
}

// error-bound constants for the approximate (MFMA) scores, see DESIGN.md "Exactness guard"
static double acc_gamma(const hr_index* h) { return (double)(h->dpad + 64) * std::ldexp(1.0, -23); }
static double storage_u(const hr_index* h) {
    if (h->dtype != F32) return 0.0;
    if (mfma_type(h) == BF16) return std::ldexp(1.0, -8);
    // f16: relative 2^-11 for normal values; an element below 2^-14 rounds to a subnormal with an absolute
    // error up to 2^-25, which sum_i |q_i| 2^-25 <= sqrt(dpad) |q| 2^-25 bounds -- folded in relative to
    // the largest row norm, as guard_e scales u_x by it
    const double mn = std::sqrt(h->max_norm2);
    return std::ldexp(1.0, -11) + (mn > 0.0 ? std::sqrt((double)h->dpad) * std::ldexp(1.0, -25) / mn : 0.0);
}

// One chunk of <= Bp queries on this shard.  mode 0: top-kc via SAMPLE+FILTER(groups);
// mode 1: collect every row with approx >= floor (exact fallback).
// st_tail: stream of select + rescore (the outputs are ready in its order).  st_tail != st:
// pipelined (mode 0 only) -- ping-pong scratch set, the scan leaves tail_cus() CUs free and the
// tail waits for this batch's FILTER by event; st_tail == st: one stream, the synchronous set.
static int shard_chunk(hr_index* h, const float* q_dev, int B, int kc, int kj, const uint64_t* mask_dev, int64_t row_offset,
                       const double* kth_dev_host /* mode 1: host array of kth, B */, int mode, int cap_out,
                       Cand* cand_out, double* bound_out, hipStream_t st, hipStream_t st_tail,
                       hipEvent_t q_ready = nullptr) {
    if (int rc = shadow_update(h)) return rc;
    Plan pl;
    if (int rc = make_plan(h, B, &pl)) return rc;
    const int Bp = pl.Bp;
    const bool piped = st_tail != st && mode == 0;
    if (!piped) st_tail = st;
    const int64_t n_tiles = (h->n + 31) / 32;
    // SAMPLE size for n units: n/128 tiles (round 2: 128 beat 64 by 0.7 % at 10M; with the kj-th largest floor, n/256
    // on shards beyond 160k tiles), at least 2048 -- or 1024 on shards
    // up to 80k tiles (2.56M rows): with the kj-th largest starting floor (k_floor_kth) 1024 sampled tiles start
    // the FILTER as well there and the early-SAMPLE chain is shorter -- 1M x 768 0.289 -> 0.284 ms/step, 2.5M
    // 0.804 -> 0.800, 1.25M unchanged, 3072 slower; at 5M rows 1024 cost 0.5 % (profiles/
    // r04_small_shard_sample_cadence_ab.jsonl, r04_sample_floor_1024_ab.jsonl).
    // (Capping it at a fraction of a small shard -- at 100k rows a fixed 2048 read 65 % of the shard again --
    // gained nothing: 0.11-0.13 ms/step either way, the per-step host submission bounds such small collections.)
    auto sample_target = [&](int64_t n) {
        // a shard sharing its GPU with other shards of a group samples 512 tiles: the co-located shards'
        // SAMPLEs add up (8 x 1.25M rows on one GPU: 3.387 / 3.308 / 3.297 ms per batch at 2048 / 1024 /
        // 512, profiles/r03_group_scan_streams.log)
        const int64_t smin = h->shared_dev ? 512 : (n <= 80 * 1024 ? kSampleMin : 2048);
        // beyond the dual-FILTER range n/256: the SAMPLE beside the FILTER reads half as much (10M rows 2.958-2.968
        // -> 2.944-2.956 ms/step, k = 100 -0.35 %; profiles/r04_sample_size_10M_ab.jsonl)
        return std::max<int64_t>(smin, n > 160 * 1024 ? n / 256 : n / 128);
    };
    // Early SAMPLE (pipelined, queries ready by event): query prep and the SAMPLE pass run on the
    // index's own "pre" stream over the CUs the previous batch's FILTER leaves free, while that
    // FILTER still runs; this batch's FILTER then waits for them by event.  Only when the shard is
    // large enough (>= 16384 tiles, 524k rows: 8 of round 3's 2048-tile samples) for the narrow SAMPLE to finish
    // inside the previous FILTER (A/B at 16 samples: 1M x 768 0.355 vs 0.325 ms/step; at 4, 300k-row shards lose
    // 10 %); kept in tiles when the sample floor went to 1024
    constexpr int64_t early_min_tiles = 16384;
    // Not for a group shard sharing its GPU with other shards (dev_ids repeated): their early SAMPLEs on
    // high-priority streams then cut into each other's FILTERs -- 8 shards of 1.25M rows on one GPU
    // 4.87 ms/batch with, 3.76 without (profiles/r03_group_shared_gpu.log)
    // (not for the 128-query FILTER, which takes every CU: an early SAMPLE on the spare CUs would only start
    // when the previous FILTER ends, on 32 CUs instead of all of them)
    // CUs the pipelined FILTER leaves to the tail stream and the early SAMPLE: tail_cus(h) for k_scan; none for the
    // 128-query FILTER, whose per-CU rate bounds it (8 / 16 spare CUs: 3.66 / 3.65 vs 3.44 ms at B = 128,
    // profiles/r03_wide_spare_cus_sample_ab.log), so its SAMPLE is not early
    const bool wide_likely = mode == 0 && wide_plan(h, pl, (kc + 31) / 32, h->tl_n >= 0);
    const int spare = wide_likely ? 0 : tail_cus(h);
    const bool early = piped && q_ready && h->tl_n < 0 && spare > 0 && !h->shared_dev &&
                       n_tiles >= std::max<int64_t>(early_min_tiles, 8 * sample_target(n_tiles));
    // the persistent FILTER (hr_persist.hip) takes this batch: its FILTER runs in the instance streaming the
    // batches one after another; prep, SAMPLE, select and rescore are this function's as for any pipelined batch
    const bool persist = mode == 0 && !wide_likely && persist_wanted(h, pl, (kc + 31) / 32, early, mask_dev, n_tiles);
    uint32_t pepoch = 0;
    int pslot = 0;
    if (persist) {
        if (int rc = persist_configure(h, pl)) return rc;
        pepoch = h->ps->epoch + 1;  // committed to h->ps->epoch once its post is enqueued (below)
        pslot = (int)((pepoch - 1) % kPersistSlots);
    } else if (piped && h->ps && h->ps->active) {
        if (int rc = persist_close(h)) return rc;  // another kind of batch: let the running instance go
    }
    Scratch& sc = persist ? h->ps->slot[pslot] : (piped ? h->scr[h->flip] : h->scr[kSyncSet]);
    hipStream_t sp = st;  // stream of query prep + SAMPLE
    if (early) {
        if (!h->pre) {
            // highest priority: a stream of its own priority class gets its own hardware queue even
            // when the (GPU_MAX_HW_QUEUES = 4) normal-priority queues are shared by many streams --
            // sharing one with the scan stream would serialise the early SAMPLE behind the FILTER
            HIP_TRY(index_stream_create(h, &h->pre, true));
        }
        sp = h->pre;
    }
    if (piped) {
        if (!persist) h->flip ^= 1;
        if (!sc.scanned) HIP_TRY(hipEventCreateWithFlags(&sc.scanned, hipEventDisableTiming));
        if (!sc.released) HIP_TRY(hipEventCreateWithFlags(&sc.released, hipEventDisableTiming));
        if (early && !sc.sampled) HIP_TRY(hipEventCreateWithFlags(&sc.sampled, hipEventDisableTiming));
        // the set's previous batch must be through select/rescore before its buffers are rewritten
        // (skipped when it has already happened -- in the pipelined flow the host finalized that
        // batch before submitting this one -- a stream wait costs a bubble on the stream)
        if (sc.armed && hipEventQuery(sc.released) != hipSuccess) HIP_TRY(hipStreamWaitEvent(sp, sc.released, 0));
    }
    if (early) HIP_TRY(hipStreamWaitEvent(sp, q_ready, 0));  // the caller's queries
    // Units the scans visit: every tile, or (selective filter) only the tiles holding a live, allowed
    // row -- from the host-mask path (hr_index_search built h->tl), or built here for a device mask
    // (rocPRIM select on the prep stream; the count is read back, so a masked batch costs one host
    // wait for the prep stream).  A dense mask (more than half the tiles) keeps the full scan.
    const uint32_t* tl_ptr = nullptr;
    int64_t n_vis = n_tiles;
    if (h->tl_n >= 0) {
        tl_ptr = h->tl.as<uint32_t>();
        n_vis = h->tl_n;
    } else if (h->tl_n == -1 && mask_dev && n_tiles > 0) {  // (-2: the host already chose the full scan)
        HIP_TRY(sc.tl.ensure((size_t)n_tiles * 4 + 64));
        HIP_TRY(sc.tl_tmp.ensure(std::max<size_t>(64, tile_list_scratch_bytes(n_tiles))));
        uint32_t* list = sc.tl.as<uint32_t>();
        uint32_t* cnt_dev = list + n_tiles;
        if (int rc = build_tile_list(h->live, (const uint32_t*)mask_dev, n_tiles, list, cnt_dev, sc.tl_tmp.p,
                                     sc.tl_tmp.bytes, sp))
            return set_err(rc, "tile list build failed");
        uint32_t cnt_h = 0;
        HIP_TRY(hipMemcpyAsync(&cnt_h, cnt_dev, 4, hipMemcpyDeviceToHost, sp));
        HIP_TRY(hipStreamSynchronize(sp));
        if ((int64_t)cnt_h * 2 <= n_tiles) {
            tl_ptr = list;
            n_vis = cnt_h;
        }
    }
    const int64_t s_target = sample_target(n_vis);
    // Early mode on a small shard also runs each workspace's FILTER on a scan stream of its own:
    // consecutive batches use different workspaces, so batch i+1's FILTER has no dependency on
    // batch i's and its workgroups take the CUs batch i's FILTER frees during its tail (measured
    // 0.482 -> 0.462 ms/step at 1.25M rows, 0.873 -> 0.835 at 2.5M, 1.625 -> 1.607 at 5M, no gain
    // at 10M)
    const bool dual = early && !persist && n_tiles <= 160 * 1024;
    hipStream_t sf = st;  // stream of the FILTER scan
    if (dual) {
        if (!sc.scan) {
            HIP_TRY(index_stream_create(h, &sc.scan, true));
        }
        sf = sc.scan;
    }
    // the 128-query FILTER takes every CU even when pipelined (by default): with two of its 512-thread
    // workgroups' waves per SIMD (248 registers each) no tail kernel fits beside it anyway, and its per-CU rate,
    // not HBM, bounds it (10M x 1024, B = 128: 3.60 -> 3.43 ms per batch, B = 256: 7.19 -> 6.81 ms)
    const bool wide = mode == 0 && wide_plan(h, pl, (kc + 31) / 32, tl_ptr != nullptr);
    const int cus = piped && !wide ? h->n_cu - tail_cus(h) : h->n_cu;
    HIP_TRY(sc.q32.ensure((size_t)Bp * h->dpad * 4));
    HIP_TRY(sc.qfrag.ensure((size_t)pl.NG * h->S * pl.QB * 1024));
    HIP_TRY(sc.qerr.ensure((size_t)Bp * 4 * 8));
    // row parts for the group-max bound: 32 groups bound the 32nd best, so kc > 32 needs ceil(kc/32) parts
    const int np = mode == 0 ? (kc + 31) / 32 : 1;
    HIP_TRY(sc.mkeys.ensure((size_t)np * Bp * 32 * 4));
    HIP_TRY(sc.floor_q.ensure((size_t)Bp * 4));
    HIP_TRY(sc.cnt.ensure((size_t)Bp * 4));
    HIP_TRY(sc.buf.ensure((size_t)Bp * kCap * 8));
    HIP_TRY(sc.sel_rows.ensure((size_t)Bp * std::max(kc, cap_out) * 4));
    HIP_TRY(sc.sel_cnt.ensure((size_t)Bp * 4));
    HIP_TRY(sc.bound_approx.ensure((size_t)Bp * 4));
    HIP_TRY(sc.overflow.ensure((size_t)Bp * 4));
    HIP_TRY(sc.dyn_q.ensure((size_t)std::max(4, pl.NG) * 64));

    const int MT = mfma_type(h);
    float* fl = mode == 0 ? sc.floor_q.as<float>() : nullptr;  // else uploaded below
    if (MT == BF16)
        hipLaunchKernelGGL((k_prep_q<BF16>), dim3((Bp + 3) / 4), dim3(256), 0, sp, q_dev, B, Bp, h->dim, h->dpad,
                           h->S, pl.QB, h->metric, sc.q32.as<float>(), sc.qfrag.as<uint16_t>(), sc.qerr.as<double>(),
                           sc.mkeys.as<uint32_t>(), np, sc.cnt.as<uint32_t>(), fl, sc.dyn_q.as<uint32_t>());
    else
        hipLaunchKernelGGL((k_prep_q<F16>), dim3((Bp + 3) / 4), dim3(256), 0, sp, q_dev, B, Bp, h->dim, h->dpad, h->S,
                           pl.QB, h->metric, sc.q32.as<float>(), sc.qfrag.as<uint16_t>(), sc.qerr.as<double>(),
                           sc.mkeys.as<uint32_t>(), np, sc.cnt.as<uint32_t>(), fl, sc.dyn_q.as<uint32_t>());
    HIP_TRY(hipGetLastError());

    // floors: padded queries never collect; mode 1 uses kth - E (computed on the host from qerr)
    h->floor_host.assign((size_t)Bp, -INFINITY);
    for (int b = B; b < Bp; ++b) h->floor_host[(size_t)b] = INFINITY;
    const double max_norm = std::sqrt(h->max_norm2) * (1.0 + 1e-12);
    if (mode == 1) {
        std::vector<double> qerr((size_t)Bp * 4);
        HIP_TRY(hipMemcpyAsync(qerr.data(), sc.qerr.p, qerr.size() * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        for (int b = 0; b < B; ++b) {
            const double kth = kth_dev_host[b];
            if (std::isnan(kth)) {
                h->floor_host[(size_t)b] = INFINITY;  // query not in the fallback
                continue;
            }
            const double E = guard_e(&qerr[4 * (size_t)b], max_norm, acc_gamma(h), storage_u(h), h->metric);
            double lo = kth - E;
            if (h->metric == L2) {  // similarity -> scan-score space, minus the rounding slack
                const double qn2 = qerr[4 * (size_t)b + 2];
                lo = (kth - (1.0 - qn2)) - E - euclid_slack(qn2, max_norm);
            }
            float f = (float)lo;
            if ((double)f > lo) f = std::nextafter(f, -INFINITY);
            h->floor_host[(size_t)b] = f;
        }
    }
    if (!fl) {
        HIP_TRY(hipMemcpyAsync(sc.floor_q.p, h->floor_host.data(), (size_t)Bp * 4, hipMemcpyHostToDevice, st));
    }

    ScanArgs a{};
    a.rows = scan_rows(h);
    a.xnorm = h->metric == L2 ? h->xnorm : nullptr;
    a.live = h->live;
    a.mask = (const uint32_t*)mask_dev;
    a.qfrag = sc.qfrag.as<uint16_t>();
    a.S = h->S;
    a.mkeys = sc.mkeys.as<uint32_t>();
    a.np = np;
    a.part_tiles = np > 1 ? std::max<int64_t>(1, (n_tiles + np - 1) / np) : ((int64_t)1 << 62);
    a.pstride = (int64_t)Bp * 32;
    a.floor_q = sc.floor_q.as<float>();
    a.cnt = sc.cnt.as<uint32_t>();
    a.buf = sc.buf.as<float2>();
    a.cap = kCap;
    a.publish = 1;
    a.private_bufs = mode == 0 ? 1 : 0;
    a.wave_major = 1;
    // round-robin units make the chip sweep the tiles in order, so with row parts (k > 32) the last part
    // would keep its SAMPLE-level group maxima until the sweep reaches it, and the threshold (min over all
    // parts) with them: 50M rows at k = 100 then appended 78k candidates per query, overflowed every
    // private region and sent every query to the collect pass (33.8 ms/batch).  So with parts the FILTER
    // deals in teams (ScanArgs::teams): team p = every np-th wave, dealing part p's tiles round-robin, so
    // every part is read from the start and each wave stays in its part; over a tile list (units are list
    // positions, not tiles) parts keep contiguous per-wave ranges, as does the SAMPLE pass.
    a.strided = 1;
    a.teams = tl_ptr ? 0 : 1;
    a.refresh_every = refresh_every(n_tiles);
    // refresh loads issued before the tile's k-loop (ScanArgs::early_refresh): on small shards (the dual
    // FILTER streams' range, <= 5.1M rows) 1.25M rows 0.425 -> 0.421 ms/step; at 10M rows 2.99-3.03 ->
    // 3.05-3.07 ms (two alternating repeats on one box), so big shards keep the epilogue loads ...
    // ... except with 4+ row parts (k >= 75: a refresh then also reads the other parts' maxima), where the
    // early loads pay at 10M too: k = 100 3.217 -> 3.190 ms (profiles/r03_rowpart_knobs_10M.log)
    a.early_refresh = (dual || persist || np >= 4) ? 1 : 0;
    // staggered refreshes pay on shards beyond the dual-FILTER range (scan_body: roff)
    a.stagger = n_tiles > 160 * 1024 ? 1 : 0;
    const bool groups = mode == 0;
    a.use_groups = groups ? 1 : 0;
    a.tile_list = tl_ptr;
    a.ng = pl.NG;
    if (n_vis > 0) {
        hr_index::ScanEvents ev{};
        // time the main pass only, not fallbacks, and only every time_every-th one: each event
        // record costs a ~6 us bubble between kernels on the stream
        const bool timed = groups && h->time_every > 0 && (h->main_passes % h->time_every) == 0;
        if (groups) h->main_passes++;
        if (timed) {
            if (h->ev_free.empty()) {
                for (auto& x : ev.e) HIP_TRY(hipEventCreate(&x));
            } else {
                ev = h->ev_free.back();
                h->ev_free.pop_back();
            }
            ev.sampled = false;
            ev.early = early;
            ev.pepoch = pepoch;
        }
        if (groups) {
            a.sample_stride = std::max<int64_t>(1, n_vis / s_target);
            a.n_units = (n_vis + a.sample_stride - 1) / a.sample_stride;
            if (timed) HIP_TRY(hipEventRecord(ev.e[0], sp));
            if (int rc = launch_scan(h, sc, early ? spare : cus, pl, a, SCAN_SAMPLE, sp)) return rc;
            // a strided sample: start the thresholds at the kj-th largest sampled group maximum (k_floor_kth; a
            // sample of every tile -- small shards -- leaves the floor)
            if (kj > 0 && a.sample_stride > 1) {
                if (np == 1)
                    hipLaunchKernelGGL(k_floor_kth, dim3((Bp + 3) / 4), dim3(256), 0, sp, sc.mkeys.as<uint32_t>(),
                                       sc.floor_q.as<float>(), Bp, kj);
                else
                    hipLaunchKernelGGL(k_floor_kth_parts, dim3(Bp), dim3(64), 0, sp, sc.mkeys.as<uint32_t>(),
                                       sc.floor_q.as<float>(), Bp, np, kj);
                HIP_TRY(hipGetLastError());
            }
            ev.sampled = true;
            if (early) {  // the FILTER (scan stream) waits for the early prep + SAMPLE
                if (timed) HIP_TRY(hipEventRecord(ev.e[2], sp));
                if (!persist) {
                    HIP_TRY(hipEventRecord(sc.sampled, sp));
                    HIP_TRY(hipStreamWaitEvent(sf, sc.sampled, 0));
                }
            }
        }
        a.sample_stride = 1;
        a.n_units = n_vis;
        // one event between SAMPLE and FILTER ends the one and starts the other (each record is a
        // ~6 us bubble on the stream)
        // dual-stream mode: a timed FILTER waits for the previous FILTER and the FILTER after it waits
        // for the timed one, so the timed launch's events bracket that launch alone (not the tail of
        // the launch before it, nor the head of the one after)
        if (dual && (timed || h->isolate_next)) {
            const Scratch& other = h->scr[h->flip];  // (flipped above: the previous batch's set)
            if (other.armed && other.scanned) HIP_TRY(hipStreamWaitEvent(sf, other.scanned, 0));
        }
        h->isolate_next = dual && timed;
        if (persist) {
            // post the batch (admits it to a running instance), then an instance behind it on the instances'
            // stream: it runs only if the running one has exited before admitting this batch (else it exits at once)
            Persist& ps = *h->ps;
            PersistLaunch pa{};
            pa.a = a;
            pa.a.qfrag = ps.ar_qfrag.as<uint16_t>();  // slot 0's buffers; slot s = + s * stride
            pa.a.mkeys = ps.ar_mkeys.as<uint32_t>();
            pa.a.floor_q = ps.ar_floor.as<float>();
            pa.a.pbuf = ps.ar_pbuf.as<float2>();
            pa.a.pcnt = ps.ar_pcnt.as<uint32_t>();
            pa.a.capw = kCapW;
            pa.a.ng = 1;
            set_dyn_tail(pa.a, (int64_t)ps.nwg * (kScanThreads / 64), ps.ar_dynq.as<uint32_t>());
            pa.st_qfrag = ps.st_qfrag;
            pa.st_mkeys = ps.st_mkeys;
            pa.st_floor = ps.st_floor;
            pa.st_pbuf = ps.st_pbuf;
            pa.st_pcnt = ps.st_pcnt;
            pa.st_dynq = ps.st_dynq;
            pa.ctl = ps.ctl.as<PersistCtl>();
            pa.host_err = ps.host_err;
            pa.e0 = pepoch;
            pa.idle_ticks = ps.idle_ticks;
            if (int rc = launch_persist_post(pa.ctl, pepoch, sp)) return rc;
            ps.epoch = pepoch;  // (an epoch that fails before its post is not consumed)
            HIP_TRY(hipEventRecord(ps.posted[pslot], sp));
            HIP_TRY(hipStreamWaitEvent(ps.pst, ps.posted[pslot], 0));
            ps.launched = true;  // (before the launch: a quiesce after a failed launch still waits on the stream)
            if (int rc = launch_persist(mfma_type(h), scan_dtype(h), pl.P, ps.nwg, pa, scan_lds_bytes(h, pl.QB), ps.pst))
                return rc;
            ps.active = true;
            sc.wtiles_valid = false;
            h->last_scr = &sc;
        } else {
            if (timed) HIP_TRY(hipEventRecord(ev.e[1], sf));
            if (int rc = launch_scan(h, sc, cus, pl, a, groups ? SCAN_FILTER : SCAN_COLLECT, sf)) return rc;
        }
        if (timed) {
            if (!persist) HIP_TRY(hipEventRecord(ev.e[3], sf));
            h->ev_pending.push_back(ev);
            while (h->ev_pending.size() > 4096) {  // nobody is harvesting: recycle the oldest
                h->ev_free.push_back(h->ev_pending.front());
                h->ev_pending.pop_front();
            }
        }
    }
    if (persist) {  // the tail picks the batch up once every workgroup of the instance is through it
        Persist& ps = *h->ps;
        if (int rc = launch_persist_wait(ps.ctl.as<PersistCtl>(), pepoch, (uint32_t)ps.nwg, ps.host_err, st_tail))
            return rc;
    } else if (piped) {  // the tail stream picks the batch up once its FILTER is done
        HIP_TRY(hipEventRecord(sc.scanned, sf));
        HIP_TRY(hipStreamWaitEvent(st_tail, sc.scanned, 0));
    }
    // select
    const int kc_sel = mode == 0 ? kc : cap_out;
    const int sort_cap = kCap;  // power of two
    static bool sel_attr[64] = {};  // per device, set once
    if (!sel_attr[h->device & 63]) {
        HIP_TRY(hipFuncSetAttribute((const void*)k_select, hipFuncAttributeMaxDynamicSharedMemorySize, sort_cap * 8 + 16));
        sel_attr[h->device & 63] = true;
    }
    const bool priv = a.private_bufs && n_vis > 0;
    hipLaunchKernelGGL(k_select, dim3(B), dim3(1024), sort_cap * 8 + 16, st_tail, sc.cnt.as<uint32_t>(), sc.buf.as<float2>(),
                       kCap, priv ? sc.pcnt.as<uint32_t>() : nullptr, priv ? sc.pbuf.as<float2>() : nullptr,
                       (int)sc.last_W, sc.last_capw, pl.QB * 32, Bp, sc.mkeys.as<uint32_t>(), np, sc.floor_q.as<float>(), a.use_groups, B, kc_sel,
                       sc.sel_rows.as<uint32_t>(), sc.sel_cnt.as<int>(), sc.bound_approx.as<float>(),
                       sc.overflow.as<int>(), persist ? &h->ps->ctl.as<PersistCtl>()->slot_fail[pslot] : nullptr);
    HIP_TRY(hipGetLastError());
    // rescore
    const int64_t nw = (int64_t)B * kc_sel;
    int rc = dispatch_dt(h->dtype, [&](auto dt) -> int {
        hipLaunchKernelGGL((k_rescore<decltype(dt)::value>), dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, st_tail, h->rows,
                           h->S, h->dpad, sc.q32.as<float>(), sc.sel_rows.as<uint32_t>(), sc.sel_cnt.as<int>(), B,
                           kc_sel, row_offset, sc.bound_approx.as<float>(), sc.qerr.as<double>(), max_norm,
                           acc_gamma(h), storage_u(h), h->metric, sc.overflow.as<int>(), cand_out, bound_out,
                           h->stripe_G, h->stripe_s);
        HIP_TRY(hipGetLastError());
        return HR_OK;
    });
    if (rc) return rc;
    if (piped) {
        HIP_TRY(hipEventRecord(sc.released, st_tail));
        sc.armed = true;
    }
    if (mode == 1) {
        // collect mode is complete unless the candidate buffer overflowed: bound = -inf, or +inf on overflow
        std::vector<int> ovf((size_t)B), selc((size_t)B);
        HIP_TRY(hipMemcpyAsync(ovf.data(), sc.overflow.p, (size_t)B * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(selc.data(), sc.sel_cnt.p, (size_t)B * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        std::vector<double> bh((size_t)B, -INFINITY);
        for (int b = 0; b < B; ++b) {
            if (!(ovf[(size_t)b] || selc[(size_t)b] >= cap_out)) continue;
            // the window held more rows than the buffer: exact top-cap_out of the whole shard instead
            // (complete by construction, so the bound stays -inf)
            HIP_TRY(h->exh.ensure(exhaustive_scratch_bytes(h->n)));
            double qn2 = 0.0;  // euclidean: the query's |q|^2 (qerr slot 2)
            if (h->metric == L2)
                HIP_TRY(hipMemcpy(&qn2, sc.qerr.as<double>() + 4 * (size_t)b + 2, 8, hipMemcpyDeviceToHost));
            if (int rc2 = exhaustive_topm(h->rows, h->dtype, h->S, h->dpad, sc.q32.as<float>() + (int64_t)b * h->dpad,
                                          h->metric, qn2, h->live, (const uint32_t*)mask_dev, h->n, row_offset, cap_out,
                                          cand_out + (int64_t)b * cap_out, h->exh.p, h->exh.bytes, st, h->stripe_G,
                                          h->stripe_s))
                return set_err(rc2, "exhaustive exact pass failed");
            h->n_exhaustive++;
        }
        HIP_TRY(hipMemcpyAsync(bound_out, bh.data(), (size_t)B * 8, hipMemcpyHostToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    return HR_OK;
}

static int shard_search(hr_index* h, const float* q_dev, int B, int kc, int kj, const uint64_t* mask_dev, int64_t row_offset,
                        Cand* cand_out, double* bound_out, hipStream_t st, hipStream_t st_tail,
                        hipEvent_t q_ready = nullptr) {
    Plan pl;
    if (int rc = make_plan(h, B, &pl)) return rc;
    for (int b0 = 0; b0 < B; b0 += pl.Bp) {
        const int bc = std::min(pl.Bp, B - b0);
        if (int rc = shard_chunk(h, q_dev + (int64_t)b0 * h->dim, bc, kc, kj, mask_dev, row_offset, nullptr, 0, 0,
                                 cand_out + (int64_t)b0 * kc, bound_out + b0, st, st_tail, q_ready))
            return rc;
    }
    return HR_OK;
}

static int validate_search(hr_index* h, int B, int k) {
    if (B <= 0) return set_err(HR_E_INVALID, "B must be positive");
    if (k <= 0 || k > HR_MAX_K) return set_err(HR_E_INVALID, "k must be in [1, HR_MAX_K]");
    return HR_OK;
}

int launch_merge(int device, const Cand* cand, const double* bounds, int G, int B, int kc, int k, float* s_out,
                 int64_t* r_out, double* kth_out, int32_t* fail_out, hipStream_t st, int64_t cstride, int64_t bstride) {
    if (!cstride) cstride = (int64_t)B * kc * (int64_t)sizeof(Cand);
    if (!bstride) bstride = (int64_t)B * 8;
    int p2 = 1;
    while (p2 < G * kc) p2 <<= 1;
    const int lds = p2 * 16 + 16;
    if (lds > 160 * 1024) return set_err(HR_E_INVALID, "too many candidates to merge");
    static bool merge_attr[64] = {};
    if (!merge_attr[device & 63]) {
        HIP_TRY(hipFuncSetAttribute((const void*)k_merge, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        merge_attr[device & 63] = true;
    }
    hipLaunchKernelGGL(k_merge, dim3(B), dim3(256), lds, st, (const uint8_t*)cand, (const uint8_t*)bounds, cstride,
                       bstride, G, B, kc, k, s_out, r_out, kth_out, fail_out);
    HIP_TRY(hipGetLastError());
    return HR_OK;
}


// main pass of a single-shard search on device-resident queries: candidates, merge, guard flags
static int search_main(hr_index* h, const float* q_dev, int B, int k, const uint64_t* mask_dev, float* s_out,
                       int64_t* r_out, hipStream_t st) {
    const int kc = hr_kc_for_k_dim(k, h->dim);
    HIP_TRY(h->cand.ensure((size_t)B * kc * sizeof(Cand)));
    HIP_TRY(h->bound.ensure((size_t)B * 8));
    HIP_TRY(h->kth.ensure((size_t)B * 8));
    HIP_TRY(h->fail.ensure((size_t)B * 4));
    if (int rc = shard_search(h, q_dev, B, kc, hr_rank_for(k, kc, h->dim), mask_dev, 0, h->cand.as<Cand>(),
                              h->bound.as<double>(), st, st))
        return rc;
    return launch_merge(h->device, h->cand.as<Cand>(), h->bound.as<double>(), 1, B, kc, k, s_out, r_out,
                        h->kth.as<double>(), h->fail.as<int32_t>(), st);
}

// exact fallback for the queries whose guard failed: ONE collect re-scan of all of them (every row
// with approx >= kth - E, rescored exactly), merged, then scattered back to their rows of the outputs
static int search_fallback(hr_index* h, const float* q_dev, int k, const uint64_t* mask_dev, float* s_out,
                           int64_t* r_out, const std::vector<int>& failed, const double* kth, hipStream_t st) {
    h->n_guard_fail += (int64_t)failed.size();
    const int nf = (int)failed.size(), kc2 = kFallbackCapMax;
    HIP_TRY(h->fb_q.ensure((size_t)nf * h->dim * 4));
    HIP_TRY(h->fb_cand.ensure((size_t)nf * kc2 * sizeof(Cand)));
    HIP_TRY(h->fb_bound.ensure((size_t)nf * 8));
    HIP_TRY(h->fb_out.ensure((size_t)nf * k * 12 + (size_t)nf * 12 + 64));
    float* fs = h->fb_out.as<float>();
    int64_t* fr = (int64_t*)(h->fb_out.as<uint8_t>() + (((size_t)nf * k * 4 + 7) & ~(size_t)7));
    double* fk = (double*)(fr + (size_t)nf * k);
    int32_t* ff = (int32_t*)(fk + nf);
    std::vector<double> kf((size_t)nf);
    for (int i = 0; i < nf; ++i) {
        kf[(size_t)i] = kth[failed[(size_t)i]];
        HIP_TRY(hipMemcpyAsync(h->fb_q.as<float>() + (int64_t)i * h->dim, q_dev + (int64_t)failed[(size_t)i] * h->dim,
                               (size_t)h->dim * 4, hipMemcpyDeviceToDevice, st));
    }
    Plan pl;
    if (int rc = make_plan(h, nf, &pl)) return rc;
    for (int b0 = 0; b0 < nf; b0 += pl.Bp) {
        const int bc = std::min(pl.Bp, nf - b0);
        if (int rc = shard_chunk(h, h->fb_q.as<float>() + (int64_t)b0 * h->dim, bc, kc2, 0, mask_dev, 0, &kf[(size_t)b0], 1,
                                 kc2, h->fb_cand.as<Cand>() + (int64_t)b0 * kc2, h->fb_bound.as<double>() + b0, st, st))
            return rc;
    }
    if (int rc = launch_merge(h->device, h->fb_cand.as<Cand>(), h->fb_bound.as<double>(), 1, nf, kc2, k, fs, fr, fk, ff,
                              st))
        return rc;
    std::vector<int32_t> ff_h((size_t)nf);
    HIP_TRY(hipMemcpyAsync(ff_h.data(), ff, (size_t)nf * 4, hipMemcpyDeviceToHost, st));
    for (int i = 0; i < nf; ++i) {
        const int b = failed[(size_t)i];
        HIP_TRY(hipMemcpyAsync(s_out + (int64_t)b * k, fs + (int64_t)i * k, (size_t)k * 4, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemcpyAsync(r_out + (int64_t)b * k, fr + (int64_t)i * k, (size_t)k * 8, hipMemcpyDeviceToDevice, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    for (int i = 0; i < nf; ++i)
        if (ff_h[(size_t)i]) return set_err(HR_E_OVERFLOW, "exact fallback overflowed its candidate buffer (massive ties?)");
    return HR_OK;
}

// full single-shard search on device-resident queries, with the exact fallback
static int search_device_impl(hr_index* h, const float* q_dev, int B, int k, const uint64_t* mask_dev, float* s_out,
                              int64_t* r_out, hipStream_t st) {
    if (int rc = validate_search(h, B, k)) return rc;
    if (int rc = search_main(h, q_dev, B, k, mask_dev, s_out, r_out, st)) return rc;
    std::vector<int32_t> fail((size_t)B);
    std::vector<double> kth((size_t)B);
    HIP_TRY(hipMemcpyAsync(fail.data(), h->fail.p, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(kth.data(), h->kth.p, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<int> failed;
    for (int b = 0; b < B; ++b)
        if (fail[(size_t)b]) failed.push_back(b);
    if (failed.empty()) return HR_OK;
    return search_fallback(h, q_dev, k, mask_dev, s_out, r_out, failed, kth.data(), st);
}

// hr_index_search through a captured HIP graph (no mask, k <= HR_MAX_K, untimed): the host work of a
// small search -- ~10 launches, 6 copies, 2 waits -- was most of its latency on small collections.
// Returns HR_E_UNSUPPORTED when the normal path must run instead (a shape's first use, a failed capture).
static int sync_graph_search(hr_index* h, const float* q, int B, int k, float* scores_out, int64_t* rows_out) {
    if (int rc = shadow_update(h)) return rc;  // (a replay reads the shadow as it is now)
    hipStream_t st = h->stream;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t qb = (size_t)B * h->dim * 4, sb = (size_t)B * k * 4, rb = (size_t)B * k * 8;
    const size_t o_s = up(qb), o_r = o_s + up(sb), o_f = o_r + up(rb), o_k = o_f + up((size_t)B * 4);
    const size_t total = o_k + up((size_t)B * 8);
    hr_index::SyncGraph* e = nullptr;
    for (auto& g : h->sync_graphs)
        if (g.B == B && g.k == k) e = &g;
    if (!e) {
        if (h->sync_graphs.size() >= 16) {  // bounded cache: drop the oldest shape
            if (h->sync_graphs.front().exec) (void)hipGraphExecDestroy(h->sync_graphs.front().exec);
            h->sync_graphs.erase(h->sync_graphs.begin());
        }
        h->sync_graphs.push_back({});
        e = &h->sync_graphs.back();
        e->B = B;
        e->k = k;
    }
    if (e->disabled) return HR_E_UNSUPPORTED;
    auto current = [&](const hr_index::SyncGraph& g) {
        return g.exec && g.n == h->n && g.rows == h->rows && g.live == h->live && g.xnorm == h->xnorm &&
               g.max_norm2 == h->max_norm2 && g.pin == h->pin && g.buf_gen == g_buf_gen.load();
    };
    if (!current(*e)) {
        if (e->exec) {  // stale: recapture right away after a buffer moved; after the rows changed
            // (add, compaction) the normal path runs once first, to size the buffers for the new count
            (void)hipGraphExecDestroy(e->exec);
            e->exec = nullptr;
            if (e->n != h->n || e->rows != h->rows || e->live != h->live || e->xnorm != h->xnorm) e->uses = 0;
        }
        // first use of the shape: the normal path runs and sizes every buffer the pass needs, so the
        // capture below allocates nothing (an allocation fails the capture, or bumps g_buf_gen, and
        // the shape then takes the normal path once more)
        if (++e->uses < 2) return HR_E_UNSUPPORTED;
        if (h->pin_bytes < total) {
            if (h->pin) (void)hipHostFree(h->pin);
            h->pin = nullptr;
            h->pin_bytes = 0;
            HIP_TRY(hipHostMalloc(&h->pin, total, hipHostMallocDefault));
            h->pin_bytes = total;
        }
        HIP_TRY(h->q_in.ensure(qb));
        HIP_TRY(h->sync_out.ensure(up(sb) + rb));
        // captured on a stream of its own: a failed capture can leave its stream unusable
        hipStream_t cs = nullptr;
        HIP_TRY(index_stream_create(h, &cs, false));
        const uint64_t gen0 = g_buf_gen.load();
        uint8_t* pin = (uint8_t*)h->pin;
        float* s_dev = h->sync_out.as<float>();
        int64_t* r_dev = (int64_t*)(h->sync_out.as<uint8_t>() + up(sb));
        const int64_t passes0 = h->main_passes;
        const bool began = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal) == hipSuccess;
        int rc = began ? HR_OK : HR_E_HIP;
        if (!rc && hipMemcpyAsync(h->q_in.p, pin, qb, hipMemcpyHostToDevice, cs) != hipSuccess) rc = HR_E_HIP;
        if (!rc) rc = search_main(h, h->q_in.as<float>(), B, k, nullptr, s_dev, r_dev, cs);
        if (!rc && (hipMemcpyAsync(pin + o_s, s_dev, sb, hipMemcpyDeviceToHost, cs) != hipSuccess ||
                    hipMemcpyAsync(pin + o_r, r_dev, rb, hipMemcpyDeviceToHost, cs) != hipSuccess ||
                    hipMemcpyAsync(pin + o_f, h->fail.p, (size_t)B * 4, hipMemcpyDeviceToHost, cs) != hipSuccess ||
                    hipMemcpyAsync(pin + o_k, h->kth.p, (size_t)B * 8, hipMemcpyDeviceToHost, cs) != hipSuccess))
            rc = HR_E_HIP;
        hipGraph_t graph = nullptr;
        const hipError_t ec = began ? hipStreamEndCapture(cs, &graph) : hipErrorUnknown;
        const bool moved = g_buf_gen.load() != gen0;  // a buffer was reallocated while capturing
        if (!rc && ec == hipSuccess && graph && !moved)
            rc = hipGraphInstantiate(&e->exec, graph, nullptr, nullptr, 0) == hipSuccess ? HR_OK : HR_E_HIP;
        else
            rc = HR_E_HIP;
        if (graph) (void)hipGraphDestroy(graph);
        (void)hipStreamDestroy(cs);
        (void)hipGetLastError();
        e->chunks = (int)std::max<int64_t>(1, h->main_passes - passes0);
        h->main_passes = passes0;  // (nothing ran: the replays count their passes)
        if (rc) {
            e->exec = nullptr;
            e->uses = 0;
            if (!moved) e->disabled = true;  // the capture itself failed: this shape keeps the normal path
            return HR_E_UNSUPPORTED;
        }
        e->n = h->n;
        e->rows = h->rows;
        e->live = h->live;
        e->xnorm = h->xnorm;
        e->max_norm2 = h->max_norm2;
        e->pin = h->pin;
        e->buf_gen = gen0;
    }
    uint8_t* pin = (uint8_t*)h->pin;
    std::memcpy(pin, q, qb);
    HIP_TRY(hipGraphLaunch(e->exec, st));
    HIP_TRY(hipStreamSynchronize(st));
    h->main_passes += e->chunks;
    h->n_graph_replays++;
    const int32_t* fail = (const int32_t*)(pin + o_f);
    std::vector<int> failed;
    for (int b = 0; b < B; ++b)
        if (fail[b]) failed.push_back(b);
    if (failed.empty()) {
        std::memcpy(scores_out, pin + o_s, sb);
        std::memcpy(rows_out, pin + o_r, rb);
        return HR_OK;
    }
    float* s_dev = h->sync_out.as<float>();
    int64_t* r_dev = (int64_t*)(h->sync_out.as<uint8_t>() + up(sb));
    if (int rc = search_fallback(h, h->q_in.as<float>(), k, nullptr, s_dev, r_dev, failed, (const double*)(pin + o_k), st))
        return rc;
    HIP_TRY(hipMemcpyAsync(scores_out, s_dev, sb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(rows_out, r_dev, rb, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return HR_OK;
}

extern "C" int hr_index_search_device(hr_index* h, const float* q_dev, int B, int k, const uint64_t* row_mask_dev,
                                      float* scores_out_dev, int64_t* rows_out_dev, void* stream) {
    if (!h || !q_dev || !scores_out_dev || !rows_out_dev) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = set_device(h)) return rc;
    if (int rc = persist_close(h)) return rc;  // a running persistent FILTER leaves the CUs to this search
    hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch's default)
    if (h->G > 1) return group_search_device(h, q_dev, B, k, row_mask_dev, scores_out_dev, rows_out_dev, st);
    return search_device_impl(h, q_dev, B, k, row_mask_dev, scores_out_dev, rows_out_dev, st);
}

// Pipelined search (include/hiprag.h): a group handle keeps two batches in flight, every shard
// submitted by its own host thread (hr_group.hip); a single-device handle runs the batch at once
// (ticket 0; ShardedSearch pipelines single-device shards from Python).
extern "C" int hr_index_search_submit(hr_index* h, const float* q_dev, int B, int k, float* scores_out_dev,
                                      int64_t* rows_out_dev, void* stream, int64_t* ticket_out) {
    if (!h || !q_dev || !scores_out_dev || !rows_out_dev || !ticket_out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = set_device(h)) return rc;
    if (int rc = persist_close(h)) return rc;  // a running persistent FILTER leaves the CUs to this search
    if (int rc = validate_search(h, B, k)) return rc;
    hipStream_t st = (hipStream_t)stream;
    *ticket_out = 0;
    if (h->G > 1) return group_search_submit(h, q_dev, B, k, scores_out_dev, rows_out_dev, st, ticket_out);
    return search_device_impl(h, q_dev, B, k, nullptr, scores_out_dev, rows_out_dev, st);
}

extern "C" int hr_index_search_finalize(hr_index* h, int64_t ticket) {
    if (!h) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return group_search_finalize(h, ticket);
    return HR_OK;
}

// ---- asynchronous host-query search (the drop-in store's event loop; include/hiprag.h)
constexpr int kAsyncPresizeB = 256;  // queries the async slots are sized for at first use (the store's max_batch)
static void notify_fd(void* p) {  // host function on the tail stream: one completion to the caller's eventfd
    auto* sl = (hr_index::AsyncSlot*)p;
    const uint64_t one = 1;
    ssize_t w = write(sl->notify_fd, &one, sizeof one);
    (void)w;
    sl->notify_pending.store(0, std::memory_order_release);  // last access to the slot from this thread
}

// Wait until the slot's notify host function has returned (it runs after `done` completes, on the runtime's
// callback thread).  VERDICT r04 weak #7: `done` alone let a caller collect, close its eventfd and reuse the
// number while the write was still pending.
static int async_wait_notify(hr_index::AsyncSlot& sl) {
    for (int i = 0; sl.notify_pending.load(std::memory_order_acquire); ++i) {
        if (i > 2000000) return set_err(HR_E_HIP, "asynchronous search: the completion host function never ran");
        if (i < 64) std::this_thread::yield();
        else usleep(5);
    }
    return HR_OK;
}

// wait (host) for every asynchronous batch in flight: mutations must not run under a scan that reads the
// rows (a growing corpus is reallocated); the results stay in pinned memory for collect
// A batch whose guard failed for some queries gets its exact fallback HERE, before the mutation: the fallback
// must see the corpus the batch was submitted against (rows removed in between could leave fewer than k rows
// above its bound, rows added in between could be returned).  The slot's pinned flags are then cleared, so
// collect copies the completed results.
static int async_resolve_fallback(hr_index* h, hr_index::AsyncSlot& sl);
static int async_drain(hr_index* h) {
    if (int rc = persist_quiesce(h)) return rc;  // a running instance reads the rows too
    for (auto& sl : h->aslot)
        if (sl.busy && sl.done) {
            HIP_TRY(hipEventSynchronize(sl.done));
            if (int rc = async_resolve_fallback(h, sl)) return rc;
        }
    return HR_OK;
}

static int async_resolve_fallback(hr_index* h, hr_index::AsyncSlot& sl) {
    const int B = sl.B, k = sl.k;
    int32_t* fail = (int32_t*)(sl.pin + sl.off_f);
    const double* kth = (const double*)(sl.pin + sl.off_k);
    std::vector<int> failed;
    for (int b = 0; b < B; ++b)
        if (fail[b]) failed.push_back(b);
    if (failed.empty()) return HR_OK;
    // the exact collect fallback (rare), synchronous, into the slot's device results
    if (int rc = search_fallback(h, sl.q.as<float>(), k, nullptr, sl.s.as<float>(), sl.r.as<int64_t>(), failed, kth,
                                 h->stream))
        return rc;
    HIP_TRY(hipMemcpyAsync(sl.pin + sl.off_s, sl.s.p, (size_t)B * k * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(sl.pin + sl.off_r, sl.r.p, (size_t)B * k * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    for (int b : failed) fail[b] = 0;
    return HR_OK;
}

extern "C" int hr_index_search_submit_host(hr_index* h, const float* q, int B, int k, int notify, int64_t* ticket_out) {
    if (!h || !q || !ticket_out) return set_err(HR_E_INVALID, "null argument");
    // never wait for the handle: the caller is an event loop (another call holding it -- an add waiting
    // for the GPU -- answers HR_E_BUSY and the caller takes its blocking path in a worker thread)
    std::unique_lock<std::mutex> lk(h->mu, std::try_to_lock);
    if (!lk.owns_lock()) return set_err(HR_E_BUSY, "handle busy");
    *ticket_out = 0;
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "asynchronous host search: single-device handles");
    if (int rc = validate_search(h, B, k)) return rc;
    if (h->n_live == 0) return set_err(HR_E_UNSUPPORTED, "empty index: use hr_index_search");
    // any free slot (batches may be collected out of order: one collect can move to a worker thread while
    // the other is collected on the loop); none free: HR_E_BUSY, so the caller takes its blocking path
    hr_index::AsyncSlot* free_slot = nullptr;
    for (auto& s : h->aslot)
        if (!s.busy) {
            free_slot = &s;
            break;
        }
    if (!free_slot) return set_err(HR_E_BUSY, "two batches in flight: collect one first");
    auto& sl = *free_slot;
    if (int rc = set_device(h)) return rc;
    if (int rc = persist_close(h)) return rc;
    if (!h->atail) HIP_TRY(index_stream_create(h, &h->atail, false));
    if (!h->acopy) HIP_TRY(index_stream_create(h, &h->acopy, false));
    if (!sl.done) HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    if (!sl.q_ready) HIP_TRY(hipEventCreateWithFlags(&sl.q_ready, hipEventDisableTiming));
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t qb = (size_t)B * h->dim * 4;
    sl.off_s = up(qb);
    sl.off_r = sl.off_s + up((size_t)B * k * 4);
    sl.off_f = sl.off_r + up((size_t)B * k * 8);
    sl.off_k = sl.off_f + up((size_t)B * 4);
    // The slot's buffers are sized once, for kAsyncPresizeB queries at HR_MAX_K (or the batch, if larger): a
    // later reallocation (hipHostFree / hipFree synchronise the device) would stall the event loop calling this
    const int Bs = std::max(B, kAsyncPresizeB);
    const size_t need = up((size_t)Bs * h->dim * 4) + up((size_t)Bs * HR_MAX_K * 4) + up((size_t)Bs * HR_MAX_K * 8) +
                        up((size_t)Bs * 4) + (size_t)Bs * 8;
    if (sl.off_k + (size_t)B * 8 > sl.pin_bytes) {
        if (sl.pin) HIP_TRY(hipHostFree(sl.pin));
        sl.pin = nullptr;
        sl.pin_bytes = 0;
        HIP_TRY(hipHostMalloc((void**)&sl.pin, need));
        sl.pin_bytes = need;
    }
    const int kc = hr_kc_for_k_dim(k, h->dim);
    HIP_TRY(sl.q.ensure((size_t)Bs * h->dim * 4));
    HIP_TRY(sl.cand.ensure((size_t)Bs * std::max(kc, HR_MAX_KC) * sizeof(Cand)));
    HIP_TRY(sl.bound.ensure((size_t)Bs * 8));
    HIP_TRY(sl.kth.ensure((size_t)Bs * 8));
    HIP_TRY(sl.fail.ensure((size_t)Bs * 4));
    HIP_TRY(sl.s.ensure((size_t)Bs * HR_MAX_K * 4));
    HIP_TRY(sl.r.ensure((size_t)Bs * HR_MAX_K * 8));
    // queries: host -> pinned -> device on a copy stream of their own, so the early query prep + SAMPLE
    // (ready by event) need not queue behind the previous batch's FILTER
    std::memcpy(sl.pin, q, qb);
    HIP_TRY(hipMemcpyAsync(sl.q.p, sl.pin, qb, hipMemcpyHostToDevice, h->acopy));
    HIP_TRY(hipEventRecord(sl.q_ready, h->acopy));
    if (hipEventQuery(sl.q_ready) != hipSuccess) HIP_TRY(hipStreamWaitEvent(h->stream, sl.q_ready, 0));
    if (int rc = shard_search(h, sl.q.as<float>(), B, kc, hr_rank_for(k, kc, h->dim), nullptr, 0, sl.cand.as<Cand>(),
                              sl.bound.as<double>(),
                              h->stream, h->atail, sl.q_ready))
        return rc;
    if (int rc = launch_merge(h->device, sl.cand.as<Cand>(), sl.bound.as<double>(), 1, B, kc, k, sl.s.as<float>(),
                              sl.r.as<int64_t>(), sl.kth.as<double>(), sl.fail.as<int32_t>(), h->atail))
        return rc;
    HIP_TRY(hipMemcpyAsync(sl.pin + sl.off_s, sl.s.p, (size_t)B * k * 4, hipMemcpyDeviceToHost, h->atail));
    HIP_TRY(hipMemcpyAsync(sl.pin + sl.off_r, sl.r.p, (size_t)B * k * 8, hipMemcpyDeviceToHost, h->atail));
    HIP_TRY(hipMemcpyAsync(sl.pin + sl.off_f, sl.fail.p, (size_t)B * 4, hipMemcpyDeviceToHost, h->atail));
    HIP_TRY(hipMemcpyAsync(sl.pin + sl.off_k, sl.kth.p, (size_t)B * 8, hipMemcpyDeviceToHost, h->atail));
    HIP_TRY(hipEventRecord(sl.done, h->atail));
    if (notify >= 0) {
        sl.notify_fd = notify;
        sl.notify_pending.store(1, std::memory_order_release);
        if (hipLaunchHostFunc(h->atail, notify_fd, &sl) != hipSuccess) {
            sl.notify_pending.store(0, std::memory_order_release);
            HIP_TRY(hipGetLastError());
            return set_err(HR_E_HIP, "hipLaunchHostFunc failed");
        }
    }
    sl.busy = true;
    sl.B = B;
    sl.k = k;
    sl.ticket = h->aticket++;
    *ticket_out = sl.ticket;
    return HR_OK;
}

extern "C" int hr_index_search_collect(hr_index* h, int64_t ticket, float* scores_out, int64_t* rows_out) {
    if (!h || !scores_out || !rows_out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    hr_index::AsyncSlot* sp = nullptr;
    for (auto& sl : h->aslot)
        if (sl.busy && sl.ticket == ticket) sp = &sl;
    if (!sp) return set_err(HR_E_INVALID, "unknown or collected ticket");
    auto& sl = *sp;
    struct Free {
        hr_index::AsyncSlot& s;
        ~Free() { s.busy = false; }
    } fr{sl};
    if (int rc = set_device(h)) return rc;
    HIP_TRY(hipEventSynchronize(sl.done));
    if (int rc = async_wait_notify(sl)) return rc;  // the slot is freed only once its host function returned
    const int B = sl.B, k = sl.k;
    if (int rc = async_resolve_fallback(h, sl)) return rc;
    std::memcpy(scores_out, sl.pin + sl.off_s, (size_t)B * k * 4);
    std::memcpy(rows_out, sl.pin + sl.off_r, (size_t)B * k * 8);
    return HR_OK;
}

extern "C" int hr_index_search_poll(hr_index* h, int64_t ticket, int* state_out) {
    if (!h || !state_out) return set_err(HR_E_INVALID, "null argument");
    std::unique_lock<std::mutex> lk(h->mu, std::try_to_lock);
    if (!lk.owns_lock()) return set_err(HR_E_BUSY, "handle busy");
    hr_index::AsyncSlot* sp = nullptr;
    for (auto& sl : h->aslot)
        if (sl.busy && sl.ticket == ticket) sp = &sl;
    if (!sp) return set_err(HR_E_INVALID, "unknown or collected ticket");
    if (hipEventQuery(sp->done) != hipSuccess) {
        *state_out = 0;
        return HR_OK;
    }
    const int32_t* fail = (const int32_t*)(sp->pin + sp->off_f);
    int any = 0;
    for (int b = 0; b < sp->B; ++b) any |= fail[b];
    *state_out = any ? 2 : 1;
    return HR_OK;
}

extern "C" int hr_index_host_us(hr_index* h, double* out) {
    if (!h || !out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return group_host_us(h, out);
    out[0] = out[1] = out[2] = 0.0;
    return HR_OK;
}

// Exact top-m of every query over the whole shard into device records out_dev[B][m] (local row + row_offset;
// -inf / -1 padding past the live, allowed rows): canonical fp64 score of every row + stable radix sort, the same
// arithmetic and (score desc, row asc) order as the scan path.  One corpus pass and one n-row sort per query.
static int index_exact_dev(hr_index* h, const float* q_dev, int B, int m, const uint64_t* mask_dev, int64_t row_offset,
                           Cand* out_dev, hipStream_t st) {
    Scratch& sc = h->scr[kSyncSet];
    const int QB = (B + 31) / 32, Bp = QB * 32;
    HIP_TRY(sc.q32.ensure((size_t)Bp * h->dpad * 4));
    HIP_TRY(sc.qfrag.ensure((size_t)h->S * QB * 1024));
    HIP_TRY(sc.qerr.ensure((size_t)Bp * 4 * 8));
    if (mfma_type(h) == BF16)
        hipLaunchKernelGGL((k_prep_q<BF16>), dim3((Bp + 3) / 4), dim3(256), 0, st, q_dev, B, Bp, h->dim, h->dpad, h->S,
                           QB, h->metric, sc.q32.as<float>(), sc.qfrag.as<uint16_t>(), sc.qerr.as<double>(), nullptr, 1,
                           nullptr, nullptr, nullptr);
    else
        hipLaunchKernelGGL((k_prep_q<F16>), dim3((Bp + 3) / 4), dim3(256), 0, st, q_dev, B, Bp, h->dim, h->dpad, h->S,
                           QB, h->metric, sc.q32.as<float>(), sc.qfrag.as<uint16_t>(), sc.qerr.as<double>(), nullptr, 1,
                           nullptr, nullptr, nullptr);
    HIP_TRY(hipGetLastError());
    std::vector<double> qerr((size_t)Bp * 4);
    HIP_TRY(hipMemcpyAsync(qerr.data(), sc.qerr.p, qerr.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (h->n > 0) HIP_TRY(h->exh.ensure(exhaustive_scratch_bytes(h->n)));
    for (int b = 0; b < B; ++b) {
        if (int rc = exhaustive_topm(h->rows, h->dtype, h->S, h->dpad, sc.q32.as<float>() + (int64_t)b * h->dpad,
                                     h->metric, qerr[4 * (size_t)b + 2], h->live, (const uint32_t*)mask_dev, h->n,
                                     row_offset, m, out_dev + (int64_t)b * m, h->exh.p, h->exh.bytes, st, h->stripe_G,
                                     h->stripe_s))
            return set_err(rc, "exhaustive exact pass failed");
        if (h->n > 0) h->n_exhaustive++;
    }
    return HR_OK;
}

// top-k beyond HR_MAX_K (Chroma's n_results has no cap, chroma_store.py:118-120): the exhaustive exact pass
// (index_exact_dev) into host records out_host[B][m] (global rows; -inf / -1 padding).  For the rare large-k
// call, not the batched hot path.
int index_exact_all(hr_index* h, const float* q_dev, int B, int m, const uint64_t* mask_dev, Cand* out_host,
                    hipStream_t st) {
    HIP_TRY(h->fb_cand.ensure((size_t)B * m * sizeof(Cand)));
    if (int rc = index_exact_dev(h, q_dev, B, m, mask_dev, 0, h->fb_cand.as<Cand>(), st)) return rc;
    HIP_TRY(hipMemcpyAsync(out_host, h->fb_cand.p, (size_t)B * m * sizeof(Cand), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return HR_OK;
}

// Selective filter (kb_file_search's index_type / source where-clauses, kb_search_toolkit.py:530-535):
// when at most half the tiles hold a live, allowed row, the scans visit only those tiles -- a
// filter that keeps one document's chunks reads that document's tiles, not the whole corpus.
// mask_words: the host mask as one u32 per tile of this index.  Sets h->tl / h->tl_n (reset by the caller).
int index_host_tile_list(hr_index* h, const uint32_t* mw, hipStream_t st) {
    h->tl_n = -1;
    if (!mw) return HR_OK;
    const int64_t n_tiles = (h->n + 31) / 32;
    const uint32_t* lw = h->live_host.data();
    // a dense mask (most tiles hold an allowed row) keeps the full scan: decided on every 64th
    // tile first, so a dense mask costs ~n_tiles/64 host checks, not a full list build
    int64_t probe = 0, hit = 0;
    for (int64_t t = 0; t < n_tiles; t += 64, ++probe) hit += (lw[t] & mw[t]) != 0;
    std::vector<uint32_t>& tl = h->tl_host;
    tl.clear();
    bool use = false;
    if (hit * 10 <= probe * 7) {  // not dense: build the list, giving up past half the tiles
        const int64_t limit = n_tiles / 2;
        for (int64_t t = 0; t < n_tiles && (int64_t)tl.size() <= limit; ++t)
            if (lw[t] & mw[t]) tl.push_back((uint32_t)t);
        use = (int64_t)tl.size() <= limit;
    }
    h->tl_n = -2;  // evaluated on the host: full scan unless the list is used below
    if (use) {
        HIP_TRY(h->tl.ensure(std::max<size_t>(4, tl.size() * 4)));
        if (!tl.empty()) HIP_TRY(hipMemcpyAsync(h->tl.p, tl.data(), tl.size() * 4, hipMemcpyHostToDevice, st));
        h->tl_n = (int64_t)tl.size();
    }
    return HR_OK;
}

extern "C" int hr_index_search(hr_index* h, const float* q, int B, int k, const uint64_t* row_mask, float* scores_out,
                               int64_t* rows_out) {
    if (!h || !q || !scores_out || !rows_out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = set_device(h)) return rc;
    if (int rc = persist_close(h)) return rc;  // a running persistent FILTER leaves the CUs to this search
    if (B <= 0) return set_err(HR_E_INVALID, "B must be positive");
    if (k <= 0) return set_err(HR_E_INVALID, "k must be positive");
    if (h->G > 1) return group_search_host(h, q, B, k, row_mask, scores_out, rows_out);
    hipStream_t st = h->stream;
    if (h->n_live == 0) {  // empty index: reference returns [] (faiss_store.py:143-144)
        for (int64_t i = 0; i < (int64_t)B * k; ++i) {
            scores_out[i] = -INFINITY;
            rows_out[i] = -1;
        }
        return HR_OK;
    }
    static const int graph_env = getenv("HIPRAG_SYNC_GRAPH") ? atoi(getenv("HIPRAG_SYNC_GRAPH")) : 1;
    if (graph_env && !row_mask && k <= HR_MAX_K && h->time_every == 0) {
        const int rc = sync_graph_search(h, q, B, k, scores_out, rows_out);
        if (rc != HR_E_UNSUPPORTED) return rc;
    }
    HIP_TRY(h->q_in.ensure((size_t)B * h->dim * 4));
    DevBuf& so = h->stage;
    const size_t words = (size_t)((h->n + 63) / 64);
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t kk = (size_t)std::min(k, HR_MAX_K);  // (k > HR_MAX_K writes the host arrays directly)
    const size_t off_r = up((size_t)B * kk * 4), off_m = off_r + up((size_t)B * kk * 8);
    HIP_TRY(so.ensure(off_m + (row_mask ? words * 8 : 0)));
    float* s_dev = (float*)so.p;
    int64_t* r_dev = (int64_t*)((uint8_t*)so.p + off_r);
    uint64_t* m_dev = row_mask ? (uint64_t*)((uint8_t*)so.p + off_m) : nullptr;
    HIP_TRY(hipMemcpyAsync(h->q_in.p, q, (size_t)B * h->dim * 4, hipMemcpyHostToDevice, st));
    if (row_mask) HIP_TRY(hipMemcpyAsync(m_dev, row_mask, words * 8, hipMemcpyHostToDevice, st));
    if (k > HR_MAX_K) {
        std::vector<Cand> c((size_t)B * k);
        if (int rc = index_exact_all(h, h->q_in.as<float>(), B, k, m_dev, c.data(), st)) return rc;
        for (size_t i = 0; i < c.size(); ++i) {
            scores_out[i] = c[i].row >= 0 ? (float)c[i].score : -INFINITY;
            rows_out[i] = c[i].row;
        }
        return HR_OK;
    }
    struct TileListScope {
        hr_index* h;
        ~TileListScope() { h->tl_n = -1; }
    } tl_scope{h};
    if (int rc = index_host_tile_list(h, (const uint32_t*)row_mask, st)) return rc;
    if (int rc = search_device_impl(h, h->q_in.as<float>(), B, k, m_dev, s_dev, r_dev, st)) return rc;
    HIP_TRY(hipMemcpyAsync(scores_out, s_dev, (size_t)B * k * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(rows_out, r_dev, (size_t)B * k * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return HR_OK;
}

// one shard's exact candidates (group handles, hr_group.hip)
int index_shard_search(hr_index* h, const float* q_dev, int B, int kc, int kj, const uint64_t* mask_dev, Cand* cand_out,
                       double* bound_out, hipStream_t st) {
    return shard_search(h, q_dev, B, kc, kj, mask_dev, 0, cand_out, bound_out, st, st);
}

int index_shard_search_async(hr_index* h, const float* q_dev, int B, int kc, int kj, Cand* cand_out, double* bound_out,
                             hipStream_t st, hipStream_t st_tail, hipEvent_t q_ready) {
    return shard_search(h, q_dev, B, kc, kj, nullptr, 0, cand_out, bound_out, st, st_tail, q_ready);
}

int index_shard_collect(hr_index* h, const float* q_dev, int B, const double* kth_host, int cap,
                        const uint64_t* mask_dev, Cand* cand_out, double* bound_out, hipStream_t st) {
    Plan pl;
    if (int rc = make_plan(h, B, &pl)) return rc;
    for (int b0 = 0; b0 < B; b0 += pl.Bp) {  // one collect scan per chunk of queries
        const int bc = std::min(pl.Bp, B - b0);
        if (int rc = shard_chunk(h, q_dev + (int64_t)b0 * h->dim, bc, cap, 0, mask_dev, 0, kth_host + b0, 1, cap,
                                 cand_out + (int64_t)b0 * cap, bound_out + b0, st, st))
            return rc;
    }
    return HR_OK;
}

extern "C" int hr_index_search_shard(hr_index* h, const float* q_dev, int B, int k, int kc,
                                     const uint64_t* row_mask_dev, int64_t row_offset, void* cand_out_dev,
                                     double* bound_out_dev, void* stream) {
    if (!h || !q_dev || !cand_out_dev || !bound_out_dev) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "per-shard search pieces need a single-device index");
    if (int rc = set_device(h)) return rc;
    if (int rc = persist_close(h)) return rc;  // a running persistent FILTER leaves the CUs to this search
    if (int rc = validate_search(h, B, k)) return rc;
    if (kc < k || kc > HR_MAX_KC) return set_err(HR_E_INVALID, "kc must be in [k, HR_MAX_KC]");
    hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch's default)
    return shard_search(h, q_dev, B, kc, hr_rank_for(k, kc, h->dim), row_mask_dev, row_offset, (Cand*)cand_out_dev,
                        bound_out_dev, st, st);
}

extern "C" int hr_index_search_shard_async_ev(hr_index* h, const float* q_dev, int B, int k, int kc,
                                              const uint64_t* row_mask_dev, int64_t row_offset, void* cand_out_dev,
                                              double* bound_out_dev, void* scan_stream, void* tail_stream,
                                              void* q_ready_event) {
    if (!h || !q_dev || !cand_out_dev || !bound_out_dev) return set_err(HR_E_INVALID, "null argument");
    if (scan_stream == tail_stream) return set_err(HR_E_INVALID, "scan and tail streams must differ");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "per-shard search pieces need a single-device index");
    if (int rc = set_device(h)) return rc;
    if (int rc = validate_search(h, B, k)) return rc;
    if (kc < k || kc > HR_MAX_KC) return set_err(HR_E_INVALID, "kc must be in [k, HR_MAX_KC]");
    return shard_search(h, q_dev, B, kc, hr_rank_for(k, kc, h->dim), row_mask_dev, row_offset, (Cand*)cand_out_dev,
                        bound_out_dev, (hipStream_t)scan_stream, (hipStream_t)tail_stream, (hipEvent_t)q_ready_event);
}

extern "C" int hr_index_search_shard_async(hr_index* h, const float* q_dev, int B, int k, int kc,
                                           const uint64_t* row_mask_dev, int64_t row_offset, void* cand_out_dev,
                                           double* bound_out_dev, void* scan_stream, void* tail_stream) {
    return hr_index_search_shard_async_ev(h, q_dev, B, k, kc, row_mask_dev, row_offset, cand_out_dev, bound_out_dev,
                                          scan_stream, tail_stream, nullptr);
}

extern "C" int hr_index_search_shard_collect(hr_index* h, const float* q_dev, int B, const double* kth_dev, int cap,
                                             const uint64_t* row_mask_dev, int64_t row_offset, void* cand_out_dev,
                                             double* bound_out_dev, void* stream) {
    if (!h || !q_dev || !kth_dev || !cand_out_dev || !bound_out_dev) return set_err(HR_E_INVALID, "null argument");
    if (B <= 0 || cap <= 0 || cap > 2048) return set_err(HR_E_INVALID, "B > 0 and cap in [1, 2048] required");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "per-shard search pieces need a single-device index");
    if (int rc = set_device(h)) return rc;
    if (int rc = persist_close(h)) return rc;  // a running persistent FILTER leaves the CUs to this search
    hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch's default)
    std::vector<double> kth((size_t)B);
    HIP_TRY(hipMemcpyAsync(kth.data(), kth_dev, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    Cand* out = (Cand*)cand_out_dev;
    Plan pl;
    if (int rc = make_plan(h, B, &pl)) return rc;
    for (int b0 = 0; b0 < B; b0 += pl.Bp) {  // one collect scan per chunk of queries
        const int bc = std::min(pl.Bp, B - b0);
        if (int rc = shard_chunk(h, q_dev + (int64_t)b0 * h->dim, bc, cap, 0, row_mask_dev, row_offset, &kth[(size_t)b0], 1,
                                 cap, out + (int64_t)b0 * cap, bound_out_dev + b0, st, st))
            return rc;
    }
    return HR_OK;
}

extern "C" int hr_index_search_shard_exact(hr_index* h, const float* q_dev, int B, int m, const uint64_t* row_mask_dev,
                                           int64_t row_offset, void* cand_out_dev, void* stream) {
    if (!h || !q_dev || !cand_out_dev) return set_err(HR_E_INVALID, "null argument");
    if (B <= 0 || m <= 0) return set_err(HR_E_INVALID, "B > 0 and m > 0 required");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "per-shard search pieces need a single-device index");
    if (int rc = set_device(h)) return rc;
    if (int rc = persist_close(h)) return rc;  // a running persistent FILTER leaves the CUs to this pass
    return index_exact_dev(h, q_dev, B, m, row_mask_dev, row_offset, (Cand*)cand_out_dev, (hipStream_t)stream);
}

extern "C" int hr_merge_sorted(int device, const void* cand_dev, int64_t cand_rank_stride, int G, int B, int m, int k,
                               float* scores_out_dev, int64_t* rows_out_dev, void* stream) {
    if (!cand_dev || !scores_out_dev || !rows_out_dev) return set_err(HR_E_INVALID, "null argument");
    if (G <= 0 || B <= 0 || B > 65535 || m <= 0 || k <= 0) return set_err(HR_E_INVALID, "bad sizes");
    if (!cand_rank_stride) cand_rank_stride = (int64_t)B * m * (int64_t)sizeof(Cand);
    if (cand_rank_stride < (int64_t)B * m * (int64_t)sizeof(Cand) || cand_rank_stride % 8)
        return set_err(HR_E_INVALID, "rank stride smaller than one rank's records or misaligned");
    HIP_TRY(hipSetDevice(device));
    return launch_merge_sorted((const Cand*)cand_dev, cand_rank_stride, G, B, m, k, scores_out_dev, rows_out_dev,
                               (hipStream_t)stream);
}

extern "C" int hr_merge_candidates(int device, const void* cand_dev, const double* bounds_dev, int G, int B, int kc,
                                   int k, float* scores_out_dev, int64_t* rows_out_dev, double* kth_out_dev,
                                   int32_t* fail_out_dev, void* stream) {
    if (!cand_dev || !bounds_dev || !scores_out_dev || !rows_out_dev || !kth_out_dev || !fail_out_dev)
        return set_err(HR_E_INVALID, "null argument");
    if (G <= 0 || B <= 0 || kc <= 0 || k <= 0 || k > kc) return set_err(HR_E_INVALID, "bad sizes");
    HIP_TRY(hipSetDevice(device));
    return launch_merge(device, (const Cand*)cand_dev, bounds_dev, G, B, kc, k, scores_out_dev, rows_out_dev,
                        kth_out_dev, fail_out_dev, (hipStream_t)stream);
}

extern "C" int hr_merge_candidates_strided(int device, const void* cand_dev, const double* bounds_dev,
                                           int64_t cand_rank_stride, int64_t bound_rank_stride, int G, int B, int kc,
                                           int k, float* scores_out_dev, int64_t* rows_out_dev, double* kth_out_dev,
                                           int32_t* fail_out_dev, void* stream) {
    if (!cand_dev || !bounds_dev || !scores_out_dev || !rows_out_dev || !kth_out_dev || !fail_out_dev)
        return set_err(HR_E_INVALID, "null argument");
    if (G <= 0 || B <= 0 || kc <= 0 || k <= 0 || k > kc) return set_err(HR_E_INVALID, "bad sizes");
    if (cand_rank_stride < (int64_t)B * kc * (int64_t)sizeof(Cand) || bound_rank_stride < (int64_t)B * 8 ||
        cand_rank_stride % 8 || bound_rank_stride % 8)
        return set_err(HR_E_INVALID, "rank strides smaller than one rank's records or misaligned");
    HIP_TRY(hipSetDevice(device));
    return launch_merge(device, (const Cand*)cand_dev, bounds_dev, G, B, kc, k, scores_out_dev, rows_out_dev,
                        kth_out_dev, fail_out_dev, (hipStream_t)stream, cand_rank_stride, bound_rank_stride);
}


// diagnostics: approximate scores of every row (Bp×n) and the per-query bound E_q
extern "C" int hr_index_debug_approx(hr_index* h, const float* q, int B, float* approx_out, double* e_out) {
    if (!h || !q || !approx_out || !e_out || B <= 0 || B > 64) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "diagnostics need a single-device index");
    if (int rc = set_device(h)) return rc;
    Plan pl;
    if (int rc = make_plan(h, B, &pl)) return rc;
    hipStream_t st = h->stream;
    Scratch& sc = h->scr[kSyncSet];
    const int Bp = pl.Bp;
    const int64_t n_tiles = (h->n + 31) / 32;
    HIP_TRY(h->q_in.ensure((size_t)B * h->dim * 4));
    HIP_TRY(sc.q32.ensure((size_t)Bp * h->dpad * 4));
    HIP_TRY(sc.qfrag.ensure((size_t)h->S * pl.QB * 1024));
    HIP_TRY(sc.qerr.ensure((size_t)Bp * 4 * 8));
    HIP_TRY(h->stage.ensure((size_t)Bp * n_tiles * 32 * 4 + 16));
    HIP_TRY(hipMemcpyAsync(h->q_in.p, q, (size_t)B * h->dim * 4, hipMemcpyHostToDevice, st));
    const int MT = mfma_type(h);
    if (MT == BF16)
        hipLaunchKernelGGL((k_prep_q<BF16>), dim3((Bp + 3) / 4), dim3(256), 0, st, h->q_in.as<float>(), B, Bp, h->dim,
                           h->dpad, h->S, pl.QB, h->metric, sc.q32.as<float>(), sc.qfrag.as<uint16_t>(), sc.qerr.as<double>(),
                           nullptr, 1, nullptr, nullptr, nullptr);
    else
        hipLaunchKernelGGL((k_prep_q<F16>), dim3((Bp + 3) / 4), dim3(256), 0, st, h->q_in.as<float>(), B, Bp, h->dim,
                           h->dpad, h->S, pl.QB, h->metric, sc.q32.as<float>(), sc.qfrag.as<uint16_t>(), sc.qerr.as<double>(),
                           nullptr, 1, nullptr, nullptr, nullptr);
    HIP_TRY(hipGetLastError());
    const int lds = scan_lds_bytes(h, pl.QB);
    int rc = dispatch_dt(h->dtype, [&](auto dt) -> int {
        constexpr int DT = decltype(dt)::value;
        constexpr int MTc = DT == F16 ? F16 : BF16;
        auto k1 = k_debug_approx<MTc, DT, 1>;
        auto k2 = k_debug_approx<MTc, DT, 2>;
        auto kern = pl.QB == 1 ? k1 : k2;
        if constexpr (DT == F32) {  // the scan's MFMA type for fp32 rows (mfma_type)
            if (mfma_type(h) == F16) kern = pl.QB == 1 ? k_debug_approx<F16, DT, 1> : k_debug_approx<F16, DT, 2>;
        }
        HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        hipLaunchKernelGGL(kern, dim3((unsigned)((n_tiles + 3) / 4)), dim3(256), lds, st, h->rows,
                           sc.qfrag.as<uint16_t>(), h->S, n_tiles, h->metric == L2 ? h->xnorm : nullptr,
                           h->stage.as<float>());
        HIP_TRY(hipGetLastError());
        return HR_OK;
    });
    if (rc) return rc;
    std::vector<float> tmp((size_t)Bp * n_tiles * 32);
    std::vector<double> qerr((size_t)Bp * 4);
    HIP_TRY(hipMemcpyAsync(tmp.data(), h->stage.p, tmp.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(qerr.data(), sc.qerr.p, qerr.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const double max_norm = std::sqrt(h->max_norm2) * (1.0 + 1e-12);
    for (int b = 0; b < B; ++b) {
        std::memcpy(approx_out + (size_t)b * h->n, tmp.data() + (size_t)b * n_tiles * 32, (size_t)h->n * 4);
        e_out[b] = guard_e(&qerr[4 * (size_t)b], max_norm, acc_gamma(h), storage_u(h), h->metric);
    }
    return HR_OK;
}

extern "C" int hr_index_get_rows(hr_index* h, const int64_t* rows, int64_t n, float* out) {
    if (!h || n < 0 || (n > 0 && (!rows || !out))) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (n == 0) return HR_OK;
    for (int64_t i = 0; i < n; ++i)
        if (rows[i] < 0 || rows[i] >= h->n) return set_err(HR_E_INVALID, "row out of range");
    if (h->G > 1) return group_get_rows(h, rows, n, out);
    return index_get_rows(h, rows, n, out);
}

int index_get_rows(hr_index* h, const int64_t* rows, int64_t n, float* out) {
    if (int rc = set_device(h)) return rc;
    HIP_TRY(h->stage.ensure((size_t)n * 8 + (size_t)n * h->dim * 4));
    int64_t* idx = (int64_t*)h->stage.p;
    float* o = (float*)((uint8_t*)h->stage.p + (size_t)n * 8);
    HIP_TRY(hipMemcpyAsync(idx, rows, (size_t)n * 8, hipMemcpyHostToDevice, h->stream));
    int rc = dispatch_dt(h->dtype, [&](auto dt) -> int {
        hipLaunchKernelGGL((k_gather<decltype(dt)::value>), dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream,
                           h->rows, h->S, h->dim, idx, n, o);
        HIP_TRY(hipGetLastError());
        return HR_OK;
    });
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, o, (size_t)n * h->dim * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return HR_OK;
}

// ---------------------------------------------------------------- persistence

extern "C" int hr_index_save(hr_index* h, const char* path) {
    if (!h || !path) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return group_save(h, path);
    if (int rc = set_device(h)) return rc;
    // crash-safe: write <path>.tmp, fsync it, then rename over <path> (a crash leaves the old file)
    const std::string tmp_path = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp_path.c_str(), "wb");
    if (!f) return set_err(HR_E_IO, std::string("cannot open ") + tmp_path);
    FileHeader hd{};
    std::memcpy(hd.magic, "HIPRAG02", 8);  // 02: slot-swizzled tiles
    hd.version = 1;
    hd.dim = h->dim;
    hd.dtype = h->dtype;
    hd.metric = h->metric;
    hd.n = h->n;
    hd.n_live = h->n_live;
    hd.max_norm2 = h->max_norm2;
    bool ok = std::fwrite(&hd, sizeof(hd), 1, f) == 1;
    const int64_t tiles = (h->n + 31) / 32;
    const size_t tb = tile_bytes(h);
    std::vector<uint8_t> tmp;
    const int64_t step = std::max<int64_t>(1, ((int64_t)256 << 20) / (int64_t)tb);
    for (int64_t t = 0; ok && t < tiles; t += step) {
        const int64_t m = std::min(step, tiles - t);
        tmp.resize((size_t)m * tb);
        if (hipMemcpy(tmp.data(), h->rows + (size_t)t * tb, (size_t)m * tb, hipMemcpyDeviceToHost) != hipSuccess) {
            std::fclose(f);
            std::remove(tmp_path.c_str());
            return set_err(HR_E_HIP, "save: device copy failed");
        }
        ok = std::fwrite(tmp.data(), 1, tmp.size(), f) == tmp.size();
    }
    if (ok && tiles > 0) ok = std::fwrite(h->live_host.data(), 4, (size_t)tiles, f) == (size_t)tiles;
    ok = ok && std::fflush(f) == 0 && fsync(fileno(f)) == 0;
    ok = (std::fclose(f) == 0) && ok;
    if (ok) ok = std::rename(tmp_path.c_str(), path) == 0;
    if (!ok) std::remove(tmp_path.c_str());
    return ok ? HR_OK : set_err(HR_E_IO, std::string("write failed: ") + path);
}

extern "C" int hr_index_load(const char* path, int n_dev, const int* dev_ids, hr_index** out) {
    if (!path || !out) return set_err(HR_E_INVALID, "bad arguments");
    FILE* f = std::fopen(path, "rb");
    if (!f) return set_err(HR_E_IO, std::string("cannot open ") + path);
    FileHeader hd{};
    if (std::fread(&hd, sizeof(hd), 1, f) != 1 || std::memcmp(hd.magic, "HIPRAG02", 8) != 0) {
        std::fclose(f);
        return set_err(HR_E_IO, "not a hiprag index file");
    }
    hr_index* h = nullptr;
    if (int rc = hr_index_create(hd.dim, hd.dtype, hd.metric, n_dev, dev_ids, &h)) {
        std::fclose(f);
        return rc;
    }
    if (h->G > 1) {  // the file holds the canonical single-index layout: re-stripe it over the shards
        int rc = group_load_into(h, f, hd.n, hd.n_live, hd.max_norm2);
        std::fclose(f);
        if (rc != HR_OK) {
            hr_index_destroy(h);
            return rc;
        }
        *out = h;
        return HR_OK;
    }
    int rc = index_grow(h, hd.n);  // h is not yet visible to any other thread
    const int64_t tiles = (hd.n + 31) / 32;
    const size_t tb = tile_bytes(h);
    std::vector<uint8_t> tmp;
    const int64_t step = std::max<int64_t>(1, ((int64_t)256 << 20) / (int64_t)tb);
    for (int64_t t = 0; rc == HR_OK && t < tiles; t += step) {
        const int64_t m = std::min(step, tiles - t);
        tmp.resize((size_t)m * tb);
        if (std::fread(tmp.data(), 1, tmp.size(), f) != tmp.size()) rc = set_err(HR_E_IO, "truncated index file");
        else if (hipMemcpy(h->rows + (size_t)t * tb, tmp.data(), tmp.size(), hipMemcpyHostToDevice) != hipSuccess)
            rc = set_err(HR_E_HIP, "load: device copy failed");
    }
    if (rc == HR_OK && tiles > 0) {
        if (std::fread(h->live_host.data(), 4, (size_t)tiles, f) != (size_t)tiles) rc = set_err(HR_E_IO, "truncated index file");
        else if (hipMemcpy(h->live, h->live_host.data(), (size_t)tiles * 4, hipMemcpyHostToDevice) != hipSuccess)
            rc = set_err(HR_E_HIP, "load: device copy failed");
    }
    std::fclose(f);
    if (rc != HR_OK) {
        hr_index_destroy(h);
        return rc;
    }
    h->n = hd.n;
    h->n_live = hd.n_live;
    h->max_norm2 = hd.max_norm2;
    shadow_stale(h, 0);
    if (int rc2 = index_finish_load(h)) {
        hr_index_destroy(h);
        return rc2;
    }
    *out = h;
    return HR_OK;
}

// after rows / live bits / n / max_norm2 were installed: row norms (euclidean) and the device max norm
int index_finish_load(hr_index* h) {
    if (int rc = set_device(h)) return rc;
    if (int rc = index_update_row_norms(h, 0, h->n)) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    unsigned long long bits;
    std::memcpy(&bits, &h->max_norm2, 8);
    HIP_TRY(hipMemcpy(h->norm_bits, &bits, 8, hipMemcpyHostToDevice));
    return HR_OK;
}

extern "C" void hr_index_destroy(hr_index* h) {
    if (!h) return;
    if (h->G > 1) {
        group_destroy(h);
        return;
    }
    (void)hipSetDevice(h->device);
    persist_free(h);  // every persistent FILTER instance exits before the rows go
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->rows) (void)hipFree(h->rows);
    if (h->rows16) (void)hipFree(h->rows16);
    if (h->live) (void)hipFree(h->live);
    if (h->xnorm) (void)hipFree(h->xnorm);
    if (h->norm_bits) (void)hipFree(h->norm_bits);
    (void)hipDeviceSynchronize();  // pipelined batches may still run on caller streams
    for (auto& g : h->sync_graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (h->pin) (void)hipHostFree(h->pin);
    for (DevBuf* b : {&h->q_in, &h->cand, &h->bound, &h->kth, &h->fail, &h->fb_cand, &h->fb_bound, &h->fb_q,
                      &h->fb_out, &h->stage, &h->exh, &h->tl, &h->s_mask, &h->sync_out,
                      &h->ivf_coarse, &h->ivf_probe, &h->ivf_units, &h->ivf_uoff, &h->ivf_out})
        b->release();
    for (auto& sc : h->scr) sc.release_all();
    for (auto* list : {&h->ev_free})
        for (auto& ev : *list)
            for (auto& x : ev.e) (void)hipEventDestroy(x);
    for (auto& ev : h->ev_pending)
        for (auto& x : ev.e) (void)hipEventDestroy(x);
    for (auto& sl : h->aslot) {
        if (sl.done) (void)hipEventSynchronize(sl.done);
        (void)async_wait_notify(sl);  // a host function still pending holds a pointer to the slot
        if (sl.pin) (void)hipHostFree(sl.pin);
        for (DevBuf* b : {&sl.q, &sl.cand, &sl.bound, &sl.kth, &sl.fail, &sl.s, &sl.r}) b->release();
        if (sl.done) (void)hipEventDestroy(sl.done);
        if (sl.q_ready) (void)hipEventDestroy(sl.q_ready);
    }
    if (h->atail) (void)hipStreamDestroy(h->atail);
    if (h->acopy) (void)hipStreamDestroy(h->acopy);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    if (h->pre) (void)hipStreamDestroy(h->pre);
    delete h;
}

// harvest (blocking) the timings of every main-pass scan launched since the last harvest
static int harvest(hr_index* h, float* sample_ms, float* filter_ms, int cap, int* n) {
    int k = 0;
    while (!h->ev_pending.empty() && k < cap) {
        hr_index::ScanEvents ev = h->ev_pending.front();
        h->ev_pending.pop_front();
        float a = 0.f, b = 0.f;
        if (ev.pepoch) {
            // persistent FILTER: the SAMPLE by events; the FILTER's time per batch = from the later of the previous
            // batch's last workgroup arrival and this batch's first workgroup start to this batch's last arrival
            // (device stamps, s_memrealtime at 100 MHz): the period in a steady stream, the batch's own span after a
            // gap (an idle instance is not charged to the batch)
            HIP_TRY(hipEventSynchronize(ev.e[2]));
            HIP_TRY(hipEventElapsedTime(&a, ev.e[0], ev.e[2]));
            const PersistCtl* c = h->ps->ctl.as<PersistCtl>();
            unsigned long long t1 = 0, t0 = 0;
            for (int i = 0; i < 100000 && !t1; ++i) {  // (the batch is normally through already)
                HIP_TRY(hipMemcpy(&t1, &c->t_end[ev.pepoch % kPersistRing], 8, hipMemcpyDeviceToHost));
                if (!t1) usleep(10);
            }
            if (ev.pepoch > 1) HIP_TRY(hipMemcpy(&t0, &c->t_end[(ev.pepoch - 1) % kPersistRing], 8, hipMemcpyDeviceToHost));
            unsigned long long ts = 0;
            HIP_TRY(hipMemcpy(&ts, &c->t_start0[ev.pepoch % kPersistRing], 8, hipMemcpyDeviceToHost));
            if (ts != ~0ull && ts > t0) t0 = ts;
            b = (t1 && t0 && t1 > t0) ? (float)((double)(t1 - t0) * 1e-5) : 0.f;
        } else {
            HIP_TRY(hipEventSynchronize(ev.e[3]));
            if (ev.sampled) HIP_TRY(hipEventElapsedTime(&a, ev.e[0], ev.early ? ev.e[2] : ev.e[1]));
            HIP_TRY(hipEventElapsedTime(&b, ev.e[1], ev.e[3]));
        }
        if (sample_ms) sample_ms[k] = a;
        if (filter_ms) filter_ms[k] = b;
        h->last_sample_ms = a;
        h->last_filter_ms = b;
        h->ev_free.push_back(ev);
        ++k;
    }
    if (n) *n = k;
    return HR_OK;
}

// persistent FILTER (hr_persist.hip) of pipelined shard batches: 0 off, 1 shards of 4.2M-5.1M rows (default: where it
// measured faster),
// 2 every shard size; a change lets every running instance exit first
extern "C" int hr_index_set_persist(hr_index* h, int mode) {
    if (!h || mode < 0 || mode > 2) return set_err(HR_E_INVALID, "mode must be 0, 1 or 2");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "the persistent FILTER serves single-device indexes");
    if (int rc = persist_quiesce(h)) return rc;
    if (!h->ps) h->ps = new Persist();
    h->ps->mode = mode;
    return HR_OK;
}

// Restrict this index's kernels to a set of CUs (include/hiprag.h): every internal stream is recreated on the mask
// and the launch grids are sized for its CU count, so a compute-bound neighbour (the query embedder's forward) can
// own the other CUs instead of contending for all of them.  n_words == 0 lifts the restriction.  The caller's own
// streams (hr_index_search_device / _shard's stream arguments) are the caller's to mask (hr_stream_create_cu_mask).
// forget every captured sync-search graph (their FILTER variant and grid sizes are baked in): a setting that changes
// either must not keep replaying the old form
static void drop_sync_graphs(hr_index* h) {
    for (auto& g : h->sync_graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    h->sync_graphs.clear();
}

extern "C" int hr_index_set_cu_mask(hr_index* h, const uint32_t* mask, int n_words) {
    if (!h || n_words < 0 || n_words > 64 || (n_words > 0 && !mask)) return set_err(HR_E_INVALID, "bad CU mask");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "CU masks: single-device indexes");
    if (int rc = set_device(h)) return rc;
    for (auto& sl : h->aslot)
        if (sl.busy) return set_err(HR_E_BUSY, "asynchronous batches in flight: collect them first");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, h->device));
    int n = 0;
    for (int i = 0; i < n_words; ++i) n += __builtin_popcount(mask[i]);
    if (n_words > 0 && (n < 16 || n > prop.multiProcessorCount)) return set_err(HR_E_INVALID, "a CU mask needs 16..n_cu CUs");
    persist_free(h);  // (quiesces; re-created on the next persistent batch, on the new streams)
    HIP_TRY(hipDeviceSynchronize());
    for (hipStream_t* s : {&h->pre, &h->atail, &h->acopy})
        if (*s) {
            (void)hipStreamDestroy(*s);
            *s = nullptr;
        }
    for (auto& sc : h->scr)
        if (sc.scan) {
            (void)hipStreamDestroy(sc.scan);
            sc.scan = nullptr;
        }
    drop_sync_graphs(h);  // (their grids were sized for the old CU count)
    h->cu_mask.assign(mask, mask + n_words);
    hipStream_t ns = nullptr;
    HIP_TRY(index_stream_create(h, &ns, false));
    if (h->stream) (void)hipStreamDestroy(h->stream);
    h->stream = ns;
    h->n_cu = n_words > 0 ? n : prop.multiProcessorCount;
    return HR_OK;
}

// a stream of `device` whose kernels run on the CUs of `mask` only (bit i of word j: CU 32 j + i); release with
// hr_stream_destroy
extern "C" int hr_stream_create_cu_mask(int device, const uint32_t* mask, int n_words, void** stream_out) {
    if (!mask || n_words <= 0 || n_words > 64 || !stream_out) return set_err(HR_E_INVALID, "bad CU mask");
    HIP_TRY(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, mask));
    *stream_out = (void*)s;
    return HR_OK;
}

extern "C" int hr_stream_destroy(void* stream) {
    if (stream) {
        HIP_TRY(hipStreamSynchronize((hipStream_t)stream));  // (work still queued on it finishes first)
        HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    }
    return HR_OK;
}

// an asynchronous copy of `bytes` on `stream` (any direction: unified addressing), ordered like a kernel on it --
// the row-sharded search's guard-flag copy to pinned host memory without going through torch's pinned-memory
// allocator, which would remember the stream and touch it again when the host block is freed
extern "C" int hr_memcpy_async(void* dst, const void* src, int64_t bytes, void* stream) {
    if (bytes < 0 || (bytes > 0 && (!dst || !src))) return set_err(HR_E_INVALID, "bad copy");
    if (bytes) HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, (hipStream_t)stream));
    return HR_OK;
}

// no further batch for now: a running persistent FILTER instance exits once through the batches it was given
// (instead of after its idle timeout); returns at once
extern "C" int hr_index_persist_close(hr_index* h) {
    if (!h) return set_err(HR_E_INVALID, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return HR_OK;
    return persist_close(h);
}

// persistent FILTER diagnostics: out[0] = batches it served, out[1] = error word (0: none), out[2] = instances that
// ran (a batch admitted to a running instance adds none; an idle exit makes the next batch's instance run)
extern "C" int hr_index_persist_stats(hr_index* h, int64_t out[3]) {
    if (!h || !out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    out[0] = h->ps ? (int64_t)h->ps->epoch : 0;
    out[1] = (h->ps && h->ps->host_err) ? (int64_t)*(volatile uint32_t*)h->ps->host_err : 0;
    if (!out[1] && h->ps && h->ps->timeouts) out[1] = h->ps->last_err;  // (cleared by a quiesce, still reported)
    out[2] = 0;
    if (h->ps && h->ps->ctl.p) {
        if (int rc = set_device(h)) return rc;
        uint32_t runs = 0;
        HIP_TRY(hipMemcpy(&runs, &h->ps->ctl.as<PersistCtl>()->runs, 4, hipMemcpyDeviceToHost));
        out[2] = runs;
    }
    return HR_OK;
}

// persistent FILTER timeline of the last n epochs (through the latest submitted one; n <= 4096), 5 stamps each in
// microseconds relative to the first returned post: post, first workgroup start, last workgroup start, first
// arrival, last arrival (0 where not stamped yet); returns the epochs written in *n_out.  Blocking (device copies).
extern "C" int hr_index_persist_trace(hr_index* h, int n, double* out, int* n_out) {
    if (!h || !out || !n_out || n < 0) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    *n_out = 0;
    if (!h->ps || !h->ps->ctl.p || h->ps->epoch == 0) return HR_OK;
    if (int rc = set_device(h)) return rc;
    const int64_t last = (int64_t)h->ps->epoch;
    const int m = (int)std::min<int64_t>({(int64_t)n, last, (int64_t)kPersistRing});
    std::vector<PersistCtl> c(1);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(c.data(), h->ps->ctl.p, sizeof(PersistCtl), hipMemcpyDeviceToHost));
    const unsigned long long base = c[0].t_post[(last - m + 1) % kPersistRing];
    auto rel = [&](unsigned long long t) { return (t == 0ull || t == ~0ull) ? 0.0 : ((double)t - (double)base) * 1e-2; };
    for (int i = 0; i < m; ++i) {
        const int r = (int)((last - m + 1 + i) % kPersistRing);
        double* o = out + 5 * (size_t)i;
        o[0] = rel(c[0].t_post[r]);
        o[1] = rel(c[0].t_start0[r]);
        o[2] = rel(c[0].t_start1[r]);
        o[3] = rel(c[0].t_end0[r]);
        o[4] = rel(c[0].t_end[r]);
    }
    *n_out = m;
    return HR_OK;
}

extern "C" int hr_index_set_scan_timing(hr_index* h, int every) {
    if (!h || every < 0) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    h->time_every = every;
    if (h->G == 1) h->main_passes = 0;
    for (hr_index* s : h->shards) {  // group: every shard times its own launches (harvested from shard 0)
        s->time_every = every;
        s->main_passes = 0;
    }
    return HR_OK;
}

extern "C" int hr_index_take_scan_times(hr_index* h, float* sample_ms, float* filter_ms, int cap, int* n_out) {
    if (!h || cap < 0) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    hr_index* t = h->G > 1 ? h->shards[0] : h;
    if (int rc = set_device(t)) return rc;
    return harvest(t, sample_ms, filter_ms, cap, n_out);
}

extern "C" int hr_index_last_scan_ms(hr_index* h, float* sample_ms, float* filter_ms) {
    if (!h) return set_err(HR_E_INVALID, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    hr_index* t = h->G > 1 ? h->shards[0] : h;
    if (int rc = set_device(t)) return rc;
    if (int rc = harvest(t, nullptr, nullptr, 1 << 30, nullptr)) return rc;
    if (sample_ms) *sample_ms = t->last_sample_ms;
    if (filter_ms) *filter_ms = t->last_filter_ms;
    return HR_OK;
}


// diagnostics: tiles each wave of the most recent k_scan FILTER launch scanned ([group][wave]; blocking).  Every
// tile is scanned exactly once per query group: the counts sum to groups x units (tiles, or tile-list entries)
extern "C" int hr_index_wave_tiles(hr_index* h, uint32_t* out, int cap, int* n_out) {
    if (!h || !out || !n_out || cap < 0) return set_err(HR_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "single-device indexes");
    const Scratch* sc = h->last_scr;
    *n_out = 0;
    if (!sc || !sc->wtiles.p || !sc->wtiles_valid) return HR_OK;
    if (int rc = set_device(h)) return rc;
    const int n = (int)std::min<int64_t>(cap, (int64_t)sc->last_ng * sc->last_W);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, sc->wtiles.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    *n_out = n;
    return HR_OK;
}

// diagnostics: candidates appended by the last FILTER scan (sum and max over queries)
extern "C" int hr_index_stats(hr_index* h, int64_t out[3]) {
    if (!h || !out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    out[0] = h->main_passes;
    out[1] = h->n_guard_fail;
    out[2] = h->n_exhaustive;
    if (h->G > 1) group_stats(h, out);
    return HR_OK;
}

// diagnostics: 128-query FILTER launches issued by this index (summed over a group's shards)
extern "C" int hr_index_wide_launches(hr_index* h, int64_t* out) {
    if (!h || !out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    *out = h->n_wide;
    for (hr_index* s : h->shards)
        if (s != h) *out += s->n_wide;
    return HR_OK;
}

// 256-query FILTER: on (default) / off (129-256-query batches then take two 128-query FILTER launches)
extern "C" int hr_index_set_q256(hr_index* h, int on) {
    if (!h) return set_err(HR_E_INVALID, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->q256 != (on != 0)) {
        if (int rc = set_device(h)) return rc;
        drop_sync_graphs(h);  // a captured 129-256-query search replays the FILTER variant it was captured with
    }
    h->q256 = on != 0;
    for (hr_index* s : h->shards) s->q256 = on != 0;
    return HR_OK;
}

extern "C" int hr_index_q256_launches(hr_index* h, int64_t* out) {
    if (!h || !out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    int64_t n = h->n_q256;
    for (hr_index* s : h->shards) n += s->n_q256;
    *out = n;
    return HR_OK;
}

extern "C" int hr_index_graph_replays(hr_index* h, int64_t* out) {
    if (!h || !out) return set_err(HR_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    *out = h->n_graph_replays;
    return HR_OK;
}

extern "C" int hr_index_last_candidates(hr_index* h, int64_t* total, int64_t* max_per_query) {
    if (!h) return set_err(HR_E_INVALID, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->G > 1) return set_err(HR_E_UNSUPPORTED, "diagnostics need a single-device index");
    if (int rc = set_device(h)) return rc;
    // private per-wave counts of the last FILTER scan: pcnt[W][Bp]
    const Scratch* sc = h->last_scr;
    // layout [group][W][Bq]
    const int64_t per_group = sc ? sc->last_W * sc->last_Bp : 0, ng = sc ? sc->last_ng : 1;
    const int64_t n = per_group * ng;
    std::vector<uint32_t> c((size_t)n);
    if (n) {
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(c.data(), sc->pcnt.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    }
    std::vector<int64_t> per_q((size_t)(sc ? sc->last_Bp * ng : 0), 0);
    for (int64_t i = 0; i < n; ++i) per_q[(size_t)((i / per_group) * sc->last_Bp + i % sc->last_Bp)] += c[(size_t)i];
    int64_t t = 0, m = 0;
    for (int64_t v : per_q) {
        t += v;
        m = std::max<int64_t>(m, v);
    }
    if (total) *total = t;
    if (max_per_query) *max_per_query = m;
    return HR_OK;
}

extern "C" int hr_device_count(int* n_out) {
    if (!n_out) return set_err(HR_E_INVALID, "null argument");
    HIP_TRY(hipGetDeviceCount(n_out));
    return HR_OK;
}

extern "C" const char* hr_last_error(void) { return g_err.c_str(); }
extern "C" int hr_abi_version(void) { return 2; }

extern "C" int hr_kc_for_k(int k) { return hr_kc_for_k_dim(k, 0); }

static int kc_margin(int k, int dim) {
    const int wide = (dim + 63) / 64 * 64 >= 2048 ? 2 : 1;
    return std::max(wide == 2 ? 20 : 16, wide * k / 2);  // (20: k = 16 lacked margin at 2304 dims)
}

extern "C" int hr_kc_for_k_dim(int k, int dim) {
    // margin beyond k: max(16, k/2), for every k; max(20, k) from 2048 dims on (Youtu-Embedding's
    // 2048 / 2304): the guard's window widens against the score spread (sigma ~ 1/sqrt(D)), and at
    // 2M x 2304 rows k = 64 / 128 with a k/2 margin sent 27 / 20 of 64 queries to the collect pass.  Dense clusters put many rows within the guard's E of
    // the k-th score; at k = 100 a 16-row margin sent half the queries of a clustered corpus to the
    // collect fallback (5.3 ms/batch at 6.25M rows), k/2 sends almost none (2.8 ms).  kc = 32 for every
    // k <= 32 left no margin at k = 32 (every query of a 10M batch failed the guard: 7.2 vs 3.3 ms) and
    // HR_MAX_KC = 160 only 32 rows at k = 128 (83 % failures, 8.2 ms; tools/diag_k.py)
    return std::min(HR_MAX_KC, (k + kc_margin(k, dim) + 31) / 32 * 32);
}

// The order statistic of a query's 32 np group maxima (np = ceil(kc / 32) row parts) that starts the FILTER's
// threshold (k_floor_kth after the SAMPLE): at least kc rows must lie at or above the threshold, and kc is k +
// margin rounded UP to 32 -- the smallest group maximum, the (32 np)-th largest.  The (k + margin)-th largest
// leaves the guard the margin it was sized for and starts higher: the rows above the smallest of 32 group maxima
// number ~32 H(32) = 130 of the rows seen, above the 26th largest (k = 10) ~32 ln(32 / 6) = 54 -- fewer candidates
// appended while the SAMPLE's keys are the threshold (the first tiles of every wave).  Exactness is unchanged:
// every key is the score of a row of its group, so j groups hold a row at or above the j-th largest key, and that
// key only grows (exactness guard).  0: the smallest (k + margin fills every group, or a caller
// asked for a kc of its own -- hr_index_search_shard's kc argument -- and gets kc candidates per shard as before).
int hr_rank_for(int k, int kc, int dim) {
    if (kc != hr_kc_for_k_dim(k, dim)) return 0;
    const int m = (kc + 31) / 32 * 32;
    const int j = std::min(kc, k + kc_margin(k, dim));
    return j < m ? j : 0;
}
