// hr_group.hip -- multi-device index handles: one collection's rows striped over several GPUs
// inside ONE handle (hr_index_create with n_dev > 1).
//
// The reference is one process (FastAPI + agents) holding one cached store per collection
// (base_toolkit.py:79-91); its VectorStoreFactory.create must therefore be able to return a store
// that spans the node's GPUs.  A group handle owns G single-device shard handles (dev_ids may
// repeat: two shards on one GPU exercise the same code on a one-GPU box) and stripes its rows over
// them by 32-row tile -- handle row H lives in shard (H/32) % G at local row ((H/32)/G)*32 + H%32
// (stripe_row, hr_common.hpp) -- so every shard grows by appends, deletes stay local and a
// collection of any size is spread evenly.  A search runs every shard's scan + select + exact
// rescoring on that shard's own stream (all devices at once; the shards' kernels emit global row
// ids), copies each shard's B*kc candidate records and B bounds to the primary device
// (hipMemcpyPeerAsync over xGMI: 16 B per candidate, ~33 KB per shard at B=64 -- latency-bound, no
// collective needed inside one process), and merges them there with the same k_merge and the same
// exactness guard as the single-device path; failing queries take the collect fallback on every
// shard and a second merge.  Results are identical to a single-device index holding the same rows.
// The on-disk format is the single-index layout (tile t = handle tile t, slot swizzle of t), so a
// file loads into any number of devices.
#include <chrono>
#include <condition_variable>
#include <memory>
#include <thread>

#include "hr_internal.hpp"

namespace {

int shard_of(int64_t H, int G) { return (int)((H >> 5) % G); }
int64_t local_of(int64_t H, int G) { return (((H >> 5) / G) << 5) | (H & 31); }

// rows each shard receives from handle rows [H0, H0 + m)
std::vector<int64_t> split_counts(int64_t H0, int64_t m, int G) {
    std::vector<int64_t> c((size_t)G, 0);
    if (m <= 0) return c;
    for (int64_t T = H0 >> 5; T <= (H0 + m - 1) >> 5; ++T) {
        const int64_t lo = std::max(H0, T * 32), hi = std::min(H0 + m, T * 32 + 32);
        c[(size_t)(T % G)] += hi - lo;
    }
    return c;
}

// one tile's k-step chunks with row slots rotated for tile t_from re-laid for tile t_to (host)
void reswizzle_tile(const uint8_t* src, uint8_t* dst, int S, bool f32, int64_t t_from, int64_t t_to) {
    const int rf = tile_rot(t_from), rt = tile_rot(t_to);
    if (rf == rt) {
        std::memcpy(dst, src, (size_t)S * (f32 ? 2048 : 1024));
        return;
    }
    const int halves = f32 ? 2 : 1;
    for (int s = 0; s < S; ++s)
        for (int hv = 0; hv < halves; ++hv) {
            const size_t base = (size_t)s * (f32 ? 2048 : 1024) + (size_t)hv * 1024;
            for (int lane = 0; lane < 64; ++lane) {
                const int slot = lane & 31, h = lane >> 5;
                const int r = (slot - rf) & 31;
                const int nl = ((r + rt) & 31) + 32 * h;
                std::memcpy(dst + base + (size_t)nl * 16, src + base + (size_t)lane * 16, 16);
            }
        }
}

// this shard's u32 tile words of a handle row mask (u64 row bitmap viewed as u32 per handle tile)
void shard_mask_words(const uint32_t* mw, int64_t n_handle, int G, int s, int64_t n_local, std::vector<uint32_t>& out) {
    const int64_t nt_h = (n_handle + 31) / 32, nt_l = (n_local + 31) / 32;
    out.assign((size_t)((nt_l + 1) / 2 * 2 + 2), 0u);  // whole u64 words, + slack
    for (int64_t lt = 0; lt < nt_l; ++lt) {
        const int64_t T = lt * G + s;
        out[(size_t)lt] = T < nt_h ? mw[T] : 0u;
    }
}

struct TileListReset {  // the host tile lists are valid for one group search only
    hr_index* g;
    ~TileListReset() {
        for (hr_index* s : g->shards) s->tl_n = -1;
    }
};

}  // namespace

static void pipe_stop(hr_index* g);

int group_create(int dim, int dtype, int metric, int n_dev, const int* dev_ids, hr_index** out) {
    hr_index* g = new hr_index();
    g->G = n_dev;
    g->dim = dim;
    g->dpad = (dim + 63) / 64 * 64;
    g->S = g->dpad / 16;
    g->dtype = dtype;
    g->metric = metric;
    g->device = dev_ids[0];
    for (int s = 0; s < n_dev; ++s) {
        hr_index* sh = nullptr;
        if (int rc = hr_index_create(dim, dtype, metric, 1, dev_ids + s, &sh)) {
            group_destroy(g);
            return rc;
        }
        sh->stripe_G = n_dev;
        sh->stripe_s = s;
        for (int j = 0; j < n_dev; ++j) sh->shared_dev |= j != s && dev_ids[j] == dev_ids[s];
        g->shards.push_back(sh);
        hipEvent_t ev = nullptr;
        hipError_t e = hipSetDevice(sh->device);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        g->g_ev.push_back(ev);
        if (e != hipSuccess) {
            group_destroy(g);
            return set_err(HR_E_HIP, std::string("group_create: ") + hipGetErrorString(e));
        }
    }
    hipError_t e = hipSetDevice(g->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&g->g_ev_q, hipEventDisableTiming);
    if (e != hipSuccess) {
        group_destroy(g);
        return set_err(HR_E_HIP, std::string("group_create: ") + hipGetErrorString(e));
    }
    g->n_cu = g->shards[0]->n_cu;
    // peer access between the primary and every other device, once per pair (the candidate and query
    // copies then go straight over xGMI; where it is refused hipMemcpyPeerAsync stages, still correct)
    g->g_peer.assign((size_t)n_dev, 1);
    for (int s = 0; s < n_dev; ++s) {
        const int d = dev_ids[s];
        if (d == g->device) continue;
        bool seen = false;
        for (int j = 0; j < s; ++j) seen |= dev_ids[j] == d;
        if (seen) {
            for (int j = 0; j < s; ++j)
                if (dev_ids[j] == d) g->g_peer[(size_t)s] = g->g_peer[(size_t)j];
            continue;
        }
        int a = 0, b = 0;
        bool ok = hipDeviceCanAccessPeer(&a, g->device, d) == hipSuccess &&
                  hipDeviceCanAccessPeer(&b, d, g->device) == hipSuccess && a && b;
        if (ok) {
            hipError_t e1 = hipSetDevice(g->device);
            if (e1 == hipSuccess) e1 = hipDeviceEnablePeerAccess(d, 0);
            hipError_t e2 = hipSetDevice(d);
            if (e2 == hipSuccess) e2 = hipDeviceEnablePeerAccess(g->device, 0);
            ok = (e1 == hipSuccess || e1 == hipErrorPeerAccessAlreadyEnabled) &&
                 (e2 == hipSuccess || e2 == hipErrorPeerAccessAlreadyEnabled);
            (void)hipGetLastError();  // an "already enabled" answer is not an error here
        }
        g->g_peer[(size_t)s] = ok ? 1 : 0;
    }
    if (hipSetDevice(g->device) != hipSuccess) {
        group_destroy(g);
        return set_err(HR_E_HIP, "group_create: hipSetDevice");
    }
    *out = g;
    return HR_OK;
}

void group_destroy(hr_index* g) {
    if (g->pipe) {
        (void)group_drain(g);
        pipe_stop(g);
    }
    for (hr_index* s : g->shards) hr_index_destroy(s);
    for (size_t i = 0; i < g->g_ev.size(); ++i)
        if (g->g_ev[i]) (void)hipEventDestroy(g->g_ev[i]);
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    for (DevBuf* b : {&g->g_cand, &g->g_bound, &g->g_kth, &g->g_fail, &g->g_out, &g->g_q, &g->fb_q, &g->fb_cand,
                      &g->fb_bound, &g->fb_out})
        b->release();
    if (g->g_ev_q) (void)hipEventDestroy(g->g_ev_q);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

int group_reserve(hr_index* g, int64_t rows) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    const int64_t nt = (rows + 31) / 32;
    for (int s = 0; s < g->G; ++s) {
        hr_index* sh = g->shards[(size_t)s];
        const int64_t lt = nt > s ? (nt - s + g->G - 1) / g->G : 0;
        if (int rc = set_device(sh)) return rc;
        if (int rc = index_grow(sh, lt * 32)) return rc;
    }
    return HR_OK;
}

static void refresh_group_totals(hr_index* g) {
    g->max_norm2 = 0.0;
    g->n_live = 0;
    for (hr_index* s : g->shards) {
        g->max_norm2 = std::max(g->max_norm2, s->max_norm2);
        g->n_live += s->n_live;
    }
}

int group_add_host(hr_index* g, const float* rows, int64_t n, int64_t* first) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    const int G = g->G;
    const int64_t H0 = g->n;
    // blocks of whole handle tiles per shard (bounded host staging)
    const int64_t blk = (int64_t)32 * G * std::max<int64_t>(1, ((int64_t)64 << 20) / ((int64_t)32 * G * 4 * g->dim));
    std::vector<std::vector<float>> buf((size_t)G);
    for (int64_t off = 0; off < n;) {
        const int64_t H = H0 + off;
        const int64_t end = std::min(n, off + blk - (H % blk));  // stop on a block boundary of handle rows
        for (auto& b : buf) b.clear();
        for (int64_t i = off; i < end;) {  // one handle tile segment at a time
            const int64_t Hi = H0 + i;
            const int64_t seg = std::min(end - i, 32 - (Hi & 31));
            auto& b = buf[(size_t)shard_of(Hi, G)];
            b.insert(b.end(), rows + i * g->dim, rows + (i + seg) * g->dim);
            i += seg;
        }
        for (int s = 0; s < G; ++s) {
            const int64_t m = (int64_t)buf[(size_t)s].size() / g->dim;
            if (m == 0) continue;
            if (int rc = index_add_host(g->shards[(size_t)s], buf[(size_t)s].data(), m, nullptr)) return rc;
        }
        g->n = H0 + end;
        off = end;
    }
    refresh_group_totals(g);
    if (first) *first = H0;
    return HR_OK;
}

int group_add_synthetic(hr_index* g, uint64_t seed, int64_t global_row0, int64_t n, int64_t* first) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    const int64_t H0 = g->n;
    const std::vector<int64_t> cnt = split_counts(H0, n, g->G);
    for (int s = 0; s < g->G; ++s) {
        if (!cnt[(size_t)s]) continue;
        // shard-local rows continue where the shard ends; handle row H gets generator row global_row0 + (H - H0)
        if (int rc = index_add_synthetic(g->shards[(size_t)s], seed, global_row0 - H0, cnt[(size_t)s])) return rc;
    }
    g->n = H0 + n;
    refresh_group_totals(g);
    if (first) *first = H0;
    return HR_OK;
}

int group_add_device(hr_index* g, const float* rows_dev, int64_t n, int64_t* first, hipStream_t st) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    // rows produced on the caller's device/stream: one D2H, then striped host adds per shard
    std::vector<float> h((size_t)n * g->dim);
    HIP_TRY(hipMemcpyAsync(h.data(), rows_dev, h.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return group_add_host(g, h.data(), n, first);
}

int group_remove(hr_index* g, const int64_t* rows, int64_t n) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    for (int64_t i = 0; i < n; ++i)
        if (rows[i] < 0 || rows[i] >= g->n) return set_err(HR_E_INVALID, "row out of range");
    std::vector<std::vector<int64_t>> loc((size_t)g->G);
    for (int64_t i = 0; i < n; ++i) loc[(size_t)shard_of(rows[i], g->G)].push_back(local_of(rows[i], g->G));
    for (int s = 0; s < g->G; ++s)
        if (!loc[(size_t)s].empty())
            if (int rc = index_remove_local(g->shards[(size_t)s], loc[(size_t)s].data(), (int64_t)loc[(size_t)s].size()))
                return rc;
    refresh_group_totals(g);
    return HR_OK;
}

int group_get_rows(hr_index* g, const int64_t* rows, int64_t n, float* out) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    std::vector<std::vector<int64_t>> loc((size_t)g->G), pos((size_t)g->G);
    for (int64_t i = 0; i < n; ++i) {
        const int s = shard_of(rows[i], g->G);
        loc[(size_t)s].push_back(local_of(rows[i], g->G));
        pos[(size_t)s].push_back(i);
    }
    std::vector<float> tmp;
    for (int s = 0; s < g->G; ++s) {
        const size_t m = loc[(size_t)s].size();
        if (!m) continue;
        tmp.resize(m * g->dim);
        if (int rc = index_get_rows(g->shards[(size_t)s], loc[(size_t)s].data(), (int64_t)m, tmp.data())) return rc;
        for (size_t j = 0; j < m; ++j)
            std::memcpy(out + pos[(size_t)s][j] * g->dim, tmp.data() + j * g->dim, (size_t)g->dim * 4);
    }
    return HR_OK;
}

void group_stats(hr_index* g, int64_t out[3]) {
    out[0] = out[2] = 0;
    for (hr_index* s : g->shards) {
        out[0] += s->main_passes;
        out[2] += s->n_exhaustive;
    }
    out[1] = g->n_guard_fail;
}

// ---------------------------------------------------------------- search
// queries on the primary device (q_dev, ordered on st) -> this shard's copy (or q_dev itself)
static int shard_queries(hr_index* g, hr_index* sh, const float* q_dev, int B, DevBuf& buf, const float** qs) {
    if (sh->device == g->device) {
        *qs = q_dev;
        return HR_OK;
    }
    HIP_TRY(buf.ensure((size_t)B * g->dim * 4));
    HIP_TRY(hipMemcpyPeerAsync(buf.p, sh->device, q_dev, g->device, (size_t)B * g->dim * 4, sh->stream));
    *qs = buf.as<float>();
    return HR_OK;
}

// per-shard masks (device) + host tile lists from a host row mask of the handle
// (words: per-shard host staging that must outlive the search -- the copies are asynchronous)
static int shard_masks(hr_index* g, const uint64_t* mask_host, std::vector<const uint64_t*>& mdev,
                       std::vector<std::vector<uint32_t>>& words) {
    mdev.assign((size_t)g->G, nullptr);
    if (!mask_host) return HR_OK;
    words.resize((size_t)g->G);
    for (int s = 0; s < g->G; ++s) {
        hr_index* sh = g->shards[(size_t)s];
        if (sh->n == 0) continue;
        std::vector<uint32_t>& w = words[(size_t)s];
        shard_mask_words((const uint32_t*)mask_host, g->n, g->G, s, sh->n, w);
        if (int rc = set_device(sh)) return rc;
        HIP_TRY(sh->s_mask.ensure(w.size() * 4));
        HIP_TRY(hipMemcpyAsync(sh->s_mask.p, w.data(), w.size() * 4, hipMemcpyHostToDevice, sh->stream));
        if (int rc = index_host_tile_list(sh, w.data(), sh->stream)) return rc;
        mdev[(size_t)s] = (const uint64_t*)sh->s_mask.p;
    }
    return HR_OK;
}

// gather every shard's [B*kc] candidates + [B] bounds (on the shards' streams) into the primary's
// g_cand / g_bound (on st), after each shard's event
static int gather(hr_index* g, int B, int kc, DevBuf hr_index::*cand, DevBuf hr_index::*bound, DevBuf& gc,
                  DevBuf& gb, hipStream_t st) {
    HIP_TRY(hipSetDevice(g->device));
    HIP_TRY(gc.ensure((size_t)g->G * B * kc * sizeof(Cand)));
    HIP_TRY(gb.ensure((size_t)g->G * B * 8));
    for (int s = 0; s < g->G; ++s) {
        hr_index* sh = g->shards[(size_t)s];
        HIP_TRY(hipStreamWaitEvent(st, g->g_ev[(size_t)s], 0));
        HIP_TRY(hipMemcpyPeerAsync(gc.as<Cand>() + (size_t)s * B * kc, g->device, (sh->*cand).p, sh->device,
                                   (size_t)B * kc * sizeof(Cand), st));
        HIP_TRY(hipMemcpyPeerAsync(gb.as<double>() + (size_t)s * B, g->device, (sh->*bound).p, sh->device,
                                   (size_t)B * 8, st));
    }
    return HR_OK;
}

// exact fallback of the queries whose guard failed: every shard re-scans them in collect mode (every
// row whose approximate score can still reach the k-th exact score), then one more gather + merge;
// the merged rows overwrite the failed queries' rows of s_out / r_out (primary device, on st)
static int group_fallback(hr_index* g, const float* q_dev, int k, const std::vector<int>& failed, const double* kth,
                          const std::vector<const uint64_t*>& mdev, float* s_out, int64_t* r_out, hipStream_t st) {
    g->n_guard_fail += (int64_t)failed.size();
    const int nf = (int)failed.size(), cap = fallback_cap(g->G);
    HIP_TRY(g->fb_q.ensure((size_t)nf * g->dim * 4));
    std::vector<double> kf((size_t)nf);
    for (int i = 0; i < nf; ++i) {
        kf[(size_t)i] = kth[(size_t)failed[(size_t)i]];
        HIP_TRY(hipMemcpyAsync(g->fb_q.as<float>() + (int64_t)i * g->dim, q_dev + (int64_t)failed[(size_t)i] * g->dim,
                               (size_t)g->dim * 4, hipMemcpyDeviceToDevice, st));
    }
    HIP_TRY(hipEventRecord(g->g_ev_q, st));
    for (int s = 0; s < g->G; ++s) {
        hr_index* sh = g->shards[(size_t)s];
        if (int rc = set_device(sh)) return rc;
        HIP_TRY(hipStreamWaitEvent(sh->stream, g->g_ev_q, 0));
        HIP_TRY(sh->fb_cand.ensure((size_t)nf * cap * sizeof(Cand)));
        HIP_TRY(sh->fb_bound.ensure((size_t)nf * 8));
        const float* qs = nullptr;
        if (int rc = shard_queries(g, sh, g->fb_q.as<float>(), nf, sh->fb_q, &qs)) return rc;
        if (sh->n_live == 0) {
            std::vector<Cand> c((size_t)nf * cap, Cand{-INFINITY, -1});
            std::vector<double> b((size_t)nf, -INFINITY);
            HIP_TRY(hipMemcpyAsync(sh->fb_cand.p, c.data(), c.size() * sizeof(Cand), hipMemcpyHostToDevice, sh->stream));
            HIP_TRY(hipMemcpyAsync(sh->fb_bound.p, b.data(), b.size() * 8, hipMemcpyHostToDevice, sh->stream));
            HIP_TRY(hipStreamSynchronize(sh->stream));
        } else if (int rc = index_shard_collect(sh, qs, nf, kf.data(), cap, mdev[(size_t)s], sh->fb_cand.as<Cand>(),
                                                sh->fb_bound.as<double>(), sh->stream)) {
            return rc;
        }
        HIP_TRY(hipEventRecord(g->g_ev[(size_t)s], sh->stream));
    }
    if (int rc = gather(g, nf, cap, &hr_index::fb_cand, &hr_index::fb_bound, g->fb_cand, g->fb_bound, st)) return rc;
    HIP_TRY(g->fb_out.ensure((size_t)nf * k * 12 + (size_t)nf * 12 + 64));
    float* fs = g->fb_out.as<float>();
    int64_t* fr = (int64_t*)(g->fb_out.as<uint8_t>() + (((size_t)nf * k * 4 + 7) & ~(size_t)7));
    double* fk = (double*)(fr + (size_t)nf * k);
    int32_t* ff = (int32_t*)(fk + nf);
    if (int rc = launch_merge(g->device, g->fb_cand.as<Cand>(), g->fb_bound.as<double>(), g->G, nf, cap, k, fs, fr, fk,
                              ff, st))
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


// exact top-k of B queries (q_dev on the primary, ordered on st) over all shards -> s_out / r_out
// (primary device), k <= HR_MAX_K; mask_host: the handle's row bitmap or null
static int group_search_impl(hr_index* g, const float* q_dev, int B, int k, const uint64_t* mask_host, float* s_out,
                             int64_t* r_out, hipStream_t st) {
    const int kc = hr_kc_for_k_dim(k, g->dim);
    TileListReset reset{g};
    std::vector<const uint64_t*> mdev;
    std::vector<std::vector<uint32_t>> words;
    if (int rc = shard_masks(g, mask_host, mdev, words)) return rc;
    HIP_TRY(hipSetDevice(g->device));
    HIP_TRY(hipEventRecord(g->g_ev_q, st));
    for (int s = 0; s < g->G; ++s) {  // every shard's scan + select + rescore, all devices at once
        hr_index* sh = g->shards[(size_t)s];
        if (int rc = set_device(sh)) return rc;
        HIP_TRY(hipStreamWaitEvent(sh->stream, g->g_ev_q, 0));
        HIP_TRY(sh->cand.ensure((size_t)B * kc * sizeof(Cand)));
        HIP_TRY(sh->bound.ensure((size_t)B * 8));
        const float* qs = nullptr;
        if (int rc = shard_queries(g, sh, q_dev, B, sh->g_q, &qs)) return rc;
        if (sh->n_live == 0) {  // nothing here: no candidates, bound -inf
            std::vector<Cand> c((size_t)B * kc, Cand{-INFINITY, -1});
            std::vector<double> b((size_t)B, -INFINITY);
            HIP_TRY(hipMemcpyAsync(sh->cand.p, c.data(), c.size() * sizeof(Cand), hipMemcpyHostToDevice, sh->stream));
            HIP_TRY(hipMemcpyAsync(sh->bound.p, b.data(), b.size() * 8, hipMemcpyHostToDevice, sh->stream));
            HIP_TRY(hipStreamSynchronize(sh->stream));
        } else if (int rc = index_shard_search(sh, qs, B, kc, hr_rank_for(k, kc, g->dim), mdev[(size_t)s], sh->cand.as<Cand>(),
                                               sh->bound.as<double>(), sh->stream)) {
            return rc;
        }
        HIP_TRY(hipEventRecord(g->g_ev[(size_t)s], sh->stream));
    }
    if (int rc = gather(g, B, kc, &hr_index::cand, &hr_index::bound, g->g_cand, g->g_bound, st)) return rc;
    HIP_TRY(g->g_kth.ensure((size_t)B * 8));
    HIP_TRY(g->g_fail.ensure((size_t)B * 4));
    if (int rc = launch_merge(g->device, g->g_cand.as<Cand>(), g->g_bound.as<double>(), g->G, B, kc, k, s_out, r_out,
                              g->g_kth.as<double>(), g->g_fail.as<int32_t>(), st))
        return rc;
    std::vector<int32_t> fail((size_t)B);
    std::vector<double> kth((size_t)B);
    HIP_TRY(hipMemcpyAsync(fail.data(), g->g_fail.p, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(kth.data(), g->g_kth.p, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<int> failed;
    for (int b = 0; b < B; ++b)
        if (fail[(size_t)b]) failed.push_back(b);
    if (failed.empty()) return HR_OK;
    return group_fallback(g, q_dev, k, failed, kth.data(), mdev, s_out, r_out, st);
}

// k > HR_MAX_K: every shard's exhaustive exact top-k, merged on the host (score desc, row asc)
static int group_exact_all(hr_index* g, const float* q_dev, int B, int k, const uint64_t* mask_host, Cand* out,
                           hipStream_t st) {
    TileListReset reset{g};
    std::vector<const uint64_t*> mdev;
    std::vector<std::vector<uint32_t>> words;
    if (int rc = shard_masks(g, mask_host, mdev, words)) return rc;
    HIP_TRY(hipSetDevice(g->device));
    HIP_TRY(hipEventRecord(g->g_ev_q, st));
    std::vector<Cand> all((size_t)g->G * B * k);
    for (int s = 0; s < g->G; ++s) {
        hr_index* sh = g->shards[(size_t)s];
        if (int rc = set_device(sh)) return rc;
        HIP_TRY(hipStreamWaitEvent(sh->stream, g->g_ev_q, 0));
        const float* qs = nullptr;
        if (int rc = shard_queries(g, sh, q_dev, B, sh->g_q, &qs)) return rc;
        if (int rc = index_exact_all(sh, qs, B, k, mdev[(size_t)s], all.data() + (size_t)s * B * k, sh->stream))
            return rc;
    }
    std::vector<Cand> m;
    for (int b = 0; b < B; ++b) {
        m.clear();
        for (int s = 0; s < g->G; ++s)
            for (int i = 0; i < k; ++i) {
                const Cand& c = all[((size_t)s * B + b) * k + i];
                if (c.row >= 0) m.push_back(c);
            }
        const size_t keep = std::min<size_t>(m.size(), (size_t)k);
        std::partial_sort(m.begin(), m.begin() + keep, m.end(), [](const Cand& a, const Cand& c) {
            return a.score > c.score || (a.score == c.score && a.row < c.row);
        });
        for (int i = 0; i < k; ++i) out[(size_t)b * k + i] = (size_t)i < keep ? m[(size_t)i] : Cand{-INFINITY, -1};
    }
    return HR_OK;
}

int group_search_device(hr_index* g, const float* q_dev, int B, int k, const uint64_t* mask_dev, float* s_out,
                        int64_t* r_out, hipStream_t st) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    if (B <= 0) return set_err(HR_E_INVALID, "B must be positive");
    if (k <= 0 || k > HR_MAX_K) return set_err(HR_E_INVALID, "k must be in [1, HR_MAX_K]");
    std::vector<uint64_t> mh;
    if (mask_dev) {  // the handle's row bitmap -> host, split per shard there (a masked batch costs one D2H)
        mh.resize((size_t)((g->n + 63) / 64));
        HIP_TRY(hipMemcpyAsync(mh.data(), mask_dev, mh.size() * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    return group_search_impl(g, q_dev, B, k, mask_dev ? mh.data() : nullptr, s_out, r_out, st);
}

int group_search_host(hr_index* g, const float* q, int B, int k, const uint64_t* mask, float* s_out, int64_t* r_out) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    refresh_group_totals(g);
    if (g->n_live == 0) {  // empty index: reference returns [] (faiss_store.py:143-144)
        for (int64_t i = 0; i < (int64_t)B * k; ++i) {
            s_out[i] = -INFINITY;
            r_out[i] = -1;
        }
        return HR_OK;
    }
    hipStream_t st = g->stream;
    HIP_TRY(hipSetDevice(g->device));
    HIP_TRY(g->g_q.ensure((size_t)B * g->dim * 4));
    HIP_TRY(hipMemcpyAsync(g->g_q.p, q, (size_t)B * g->dim * 4, hipMemcpyHostToDevice, st));
    if (k > HR_MAX_K) {
        std::vector<Cand> c((size_t)B * k);
        if (int rc = group_exact_all(g, g->g_q.as<float>(), B, k, mask, c.data(), st)) return rc;
        for (size_t i = 0; i < c.size(); ++i) {
            s_out[i] = c[i].row >= 0 ? (float)c[i].score : -INFINITY;
            r_out[i] = c[i].row;
        }
        return HR_OK;
    }
    const size_t off_r = ((size_t)B * k * 4 + 255) & ~(size_t)255;
    HIP_TRY(g->g_out.ensure(off_r + (size_t)B * k * 8));
    float* s_dev = g->g_out.as<float>();
    int64_t* r_dev = (int64_t*)(g->g_out.as<uint8_t>() + off_r);
    if (int rc = group_search_impl(g, g->g_q.as<float>(), B, k, mask, s_dev, r_dev, st)) return rc;
    HIP_TRY(hipMemcpyAsync(s_out, s_dev, (size_t)B * k * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(r_out, r_dev, (size_t)B * k * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return HR_OK;
}

// ---------------------------------------------------------------- pipelined search (submit / finalize)
// The synchronous group search submits the G shards one after another from the caller's thread and then
// blocks on the guard flags: ~0.1 ms of host work per shard per batch, so a G = 8 handle spent ~0.9 ms
// of host time per batch against a ~0.42 ms GPU step (1.25M rows per GPU).  The pipelined form gives
// every shard a host thread of its own and keeps two batches in flight:
//   submit   (caller)    records "queries ready" on the caller's stream and hands the batch to the G
//                        shard threads; returns at once with a ticket;
//   shard s  (thread s)  waits for the queries (peer copy if its GPU is not the primary), runs the
//                        pipelined shard search (scan stream + tail stream, two workspaces: batch i's
//                        select/rescore overlaps batch i+1's scan), copies its B*kc candidates + B
//                        bounds to the primary and records "shard done"; the LAST shard thread of a
//                        batch enqueues the merge on the primary's merge stream (waits for every
//                        shard's event), copies the guard flags to pinned host memory, records "merged";
//   finalize (caller)    waits for "merged" and reads the flags; a failing query takes the exact
//                        collect fallback (synchronous, rare) after the shard threads have gone idle.
// Results are identical to the synchronous path (the same kernels on the same data).
namespace {
struct Job {
    int slot;
};

struct WorkerQ {
    std::mutex m;
    std::condition_variable cv;
    std::deque<Job> q;
    bool stop = false;
};
}  // namespace

struct GroupPipe {
    static constexpr int kSlots = 2;
    struct Slot {
        DevBuf cand, bound, kth, fail;                 // primary: gathered candidates, merge outputs
        std::vector<DevBuf> sh_cand, sh_bound, sh_q;   // per shard (shards off the primary device)
        int32_t* fail_h = nullptr;                     // pinned guard flags / k-th exact scores
        double* kth_h = nullptr;
        int cap_B = 0;
        hipEvent_t q_ready = nullptr, merged = nullptr;
        std::vector<hipEvent_t> sh_done, sh_q_ready;   // per shard, on the shard's device
        // the batch in flight
        bool busy = false;
        int64_t ticket = 0;
        const float* q = nullptr;
        int B = 0, k = 0, kc = 0;
        float* s_out = nullptr;
        int64_t* r_out = nullptr;
        int pending = 0;                               // shard threads still enqueuing this batch
        int err = HR_OK;
        std::string errmsg;
    } slot[kSlots];
    std::vector<std::thread> workers;
    std::vector<std::unique_ptr<WorkerQ>> qs;
    std::vector<hipStream_t> tail;                     // per shard: select + rescore + candidate copy
    std::vector<hipStream_t> scan;                     // per shard: prep + SAMPLE + FILTER (null = its own stream)
    std::vector<hipStream_t> owned;                    // streams shared by the shards of one device
    hipStream_t merge = nullptr;                       // primary: merge + flag copy
    std::mutex m;                                      // slot state (pending / err)
    std::condition_variable cv;
    int next = 0;
    int64_t next_ticket = 1;
    // host time (diagnostics, hr_index_host_us): caller submit, shard-thread enqueue per batch
    double submit_us = 0.0, shard_us_max = 0.0;
    int64_t batches = 0;
    std::vector<double> shard_us;
};

static int pipe_merge(hr_index* g, GroupPipe::Slot& sl) {
    GroupPipe* p = g->pipe;
    HIP_TRY(hipSetDevice(g->device));
    for (int s = 0; s < g->G; ++s) HIP_TRY(hipStreamWaitEvent(p->merge, sl.sh_done[(size_t)s], 0));
    HIP_TRY(hipStreamWaitEvent(p->merge, sl.q_ready, 0));  // s_out / r_out: after the caller's earlier work
    if (int rc = launch_merge(g->device, sl.cand.as<Cand>(), sl.bound.as<double>(), g->G, sl.B, sl.kc, sl.k, sl.s_out,
                              sl.r_out, sl.kth.as<double>(), sl.fail.as<int32_t>(), p->merge))
        return rc;
    HIP_TRY(hipMemcpyAsync(sl.fail_h, sl.fail.p, (size_t)sl.B * 4, hipMemcpyDeviceToHost, p->merge));
    HIP_TRY(hipMemcpyAsync(sl.kth_h, sl.kth.p, (size_t)sl.B * 8, hipMemcpyDeviceToHost, p->merge));
    HIP_TRY(hipEventRecord(sl.merged, p->merge));
    return HR_OK;
}

// shard s's part of the batch in slot `si` (runs on shard thread s)
static int pipe_shard(hr_index* g, int s, GroupPipe::Slot& sl) {
    GroupPipe* p = g->pipe;
    hr_index* sh = g->shards[(size_t)s];
    if (int rc = set_device(sh)) return rc;
    const bool local = sh->device == g->device;
    const size_t cb = (size_t)sl.B * sl.kc * sizeof(Cand);
    Cand* cand = local ? sl.cand.as<Cand>() + (size_t)s * sl.B * sl.kc : nullptr;
    double* bound = local ? sl.bound.as<double>() + (size_t)s * sl.B : nullptr;
    if (!local) {
        HIP_TRY(sl.sh_cand[(size_t)s].ensure(cb));
        HIP_TRY(sl.sh_bound[(size_t)s].ensure((size_t)sl.B * 8));
        cand = sl.sh_cand[(size_t)s].as<Cand>();
        bound = sl.sh_bound[(size_t)s].as<double>();
    }
    hipStream_t tail = p->tail[(size_t)s];
    hipStream_t scan = p->scan[(size_t)s] ? p->scan[(size_t)s] : sh->stream;
    if (sh->n_live == 0) {  // nothing here: no candidates, bound -inf (tail stream, after the queries)
        std::vector<Cand> c((size_t)sl.B * sl.kc, Cand{-INFINITY, -1});
        std::vector<double> b((size_t)sl.B, -INFINITY);
        HIP_TRY(hipStreamWaitEvent(tail, sl.q_ready, 0));
        HIP_TRY(hipMemcpyAsync(cand, c.data(), cb, hipMemcpyHostToDevice, tail));
        HIP_TRY(hipMemcpyAsync(bound, b.data(), (size_t)sl.B * 8, hipMemcpyHostToDevice, tail));
        HIP_TRY(hipStreamSynchronize(tail));  // (pageable staging; an empty shard is rare)
    } else {
        const float* qs = sl.q;
        hipEvent_t ready = sl.q_ready;
        if (!local) {  // the queries over xGMI onto this shard's device
            HIP_TRY(sl.sh_q[(size_t)s].ensure((size_t)sl.B * g->dim * 4));
            HIP_TRY(hipStreamWaitEvent(sh->stream, sl.q_ready, 0));
            HIP_TRY(hipMemcpyPeerAsync(sl.sh_q[(size_t)s].p, sh->device, sl.q, g->device, (size_t)sl.B * g->dim * 4,
                                       sh->stream));
            HIP_TRY(hipEventRecord(sl.sh_q_ready[(size_t)s], sh->stream));
            qs = sl.sh_q[(size_t)s].as<float>();
            ready = sl.sh_q_ready[(size_t)s];
        } else if (hipEventQuery(ready) != hipSuccess) {
            HIP_TRY(hipStreamWaitEvent(scan, ready, 0));  // the scan stream's prep reads them
        }
        if (!local && scan != sh->stream) HIP_TRY(hipStreamWaitEvent(scan, ready, 0));
        if (int rc = index_shard_search_async(sh, qs, sl.B, sl.kc, hr_rank_for(sl.k, sl.kc, g->dim), cand, bound, scan,
                                              tail, ready))
            return rc;
        if (!local) {
            HIP_TRY(hipMemcpyPeerAsync(sl.cand.as<Cand>() + (size_t)s * sl.B * sl.kc, g->device, cand, sh->device, cb,
                                       tail));
            HIP_TRY(hipMemcpyPeerAsync(sl.bound.as<double>() + (size_t)s * sl.B, g->device, bound, sh->device,
                                       (size_t)sl.B * 8, tail));
        }
    }
    HIP_TRY(hipEventRecord(sl.sh_done[(size_t)s], tail));
    return HR_OK;
}

static void pipe_worker(hr_index* g, int s) {
    GroupPipe* p = g->pipe;
    WorkerQ& wq = *p->qs[(size_t)s];
    for (;;) {
        Job job;
        {
            std::unique_lock<std::mutex> lk(wq.m);
            wq.cv.wait(lk, [&] { return wq.stop || !wq.q.empty(); });
            if (wq.q.empty()) return;  // stop
            job = wq.q.front();
            wq.q.pop_front();
        }
        GroupPipe::Slot& sl = p->slot[job.slot];
        const auto t0 = std::chrono::steady_clock::now();
        int rc = pipe_shard(g, s, sl);
        std::string msg = rc ? hr_last_error() : std::string();
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        bool last = false;
        {
            std::lock_guard<std::mutex> lk(p->m);
            p->shard_us[(size_t)s] += us;
            if (rc && sl.err == HR_OK) {
                sl.err = rc;
                sl.errmsg = msg;
            }
            last = --sl.pending == 0;
        }
        if (last) {  // every shard has enqueued its part: the merge goes behind all of them
            int mrc = HR_OK;
            std::string mmsg;
            bool ok;
            {
                std::lock_guard<std::mutex> lk(p->m);
                ok = sl.err == HR_OK;
            }
            if (ok && (mrc = pipe_merge(g, sl)) != HR_OK) mmsg = hr_last_error();
            std::lock_guard<std::mutex> lk(p->m);
            if (mrc && sl.err == HR_OK) {
                sl.err = mrc;
                sl.errmsg = mmsg;
            }
            sl.pending = -1;  // merged (or failed): finalize may proceed
            p->cv.notify_all();
        }
    }
}

static void pipe_stop(hr_index* g) {
    GroupPipe* p = g->pipe;
    if (!p) return;
    for (auto& q : p->qs) {
        std::lock_guard<std::mutex> lk(q->m);
        q->stop = true;
        q->cv.notify_all();
    }
    for (auto& t : p->workers)
        if (t.joinable()) t.join();
    for (int i = 0; i < GroupPipe::kSlots; ++i) {
        GroupPipe::Slot& sl = p->slot[i];
        (void)hipSetDevice(g->device);
        if (sl.merged) (void)hipEventSynchronize(sl.merged);
        for (DevBuf* b : {&sl.cand, &sl.bound, &sl.kth, &sl.fail}) b->release();
        if (sl.fail_h) (void)hipHostFree(sl.fail_h);
        if (sl.kth_h) (void)hipHostFree(sl.kth_h);
        if (sl.q_ready) (void)hipEventDestroy(sl.q_ready);
        if (sl.merged) (void)hipEventDestroy(sl.merged);
        for (int s = 0; s < g->G; ++s) {
            (void)hipSetDevice(g->shards[(size_t)s]->device);
            if (sl.sh_done[(size_t)s]) (void)hipEventSynchronize(sl.sh_done[(size_t)s]);
            sl.sh_cand[(size_t)s].release();
            sl.sh_bound[(size_t)s].release();
            sl.sh_q[(size_t)s].release();
            if (sl.sh_done[(size_t)s]) (void)hipEventDestroy(sl.sh_done[(size_t)s]);
            if (sl.sh_q_ready[(size_t)s]) (void)hipEventDestroy(sl.sh_q_ready[(size_t)s]);
        }
    }
    for (int s = 0; s < g->G; ++s) {
        (void)hipSetDevice(g->shards[(size_t)s]->device);
        if (p->tail[(size_t)s]) (void)hipStreamDestroy(p->tail[(size_t)s]);
    }
    for (size_t i = 0; i < p->owned.size(); ++i) {
        for (int s = 0; s < g->G; ++s)
            if (p->scan[(size_t)s] == p->owned[i]) (void)hipSetDevice(g->shards[(size_t)s]->device);
        (void)hipStreamDestroy(p->owned[i]);
    }
    (void)hipSetDevice(g->device);
    if (p->merge) (void)hipStreamDestroy(p->merge);
    delete p;
    g->pipe = nullptr;
}

static int pipe_start(hr_index* g) {
    if (g->pipe) return HR_OK;
    GroupPipe* p = new GroupPipe();
    g->pipe = p;
    const int G = g->G;
    p->tail.assign((size_t)G, nullptr);
    p->scan.assign((size_t)G, nullptr);
    p->shard_us.assign((size_t)G, 0.0);
    for (int i = 0; i < GroupPipe::kSlots; ++i) {
        GroupPipe::Slot& sl = p->slot[i];
        sl.sh_cand.resize((size_t)G);
        sl.sh_bound.resize((size_t)G);
        sl.sh_q.resize((size_t)G);
        sl.sh_done.assign((size_t)G, nullptr);
        sl.sh_q_ready.assign((size_t)G, nullptr);
    }
    auto fail = [&](hipError_t e) {
        pipe_stop(g);
        return set_err(HR_E_HIP, std::string("group pipeline: ") + hipGetErrorString(e));
    };
    hipError_t e = hipSuccess;
    for (int s = 0; s < G && e == hipSuccess; ++s) {
        e = hipSetDevice(g->shards[(size_t)s]->device);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->tail[(size_t)s], hipStreamNonBlocking);
        for (int i = 0; i < GroupPipe::kSlots && e == hipSuccess; ++i) {
            e = hipEventCreateWithFlags(&p->slot[i].sh_done[(size_t)s], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&p->slot[i].sh_q_ready[(size_t)s], hipEventDisableTiming);
        }
    }
    // Shards sharing a device (dev_ids repeated) go on n scan streams of that device, dealt round-robin,
    // instead of one stream each: consecutive shards' FILTERs then overlap pairwise (one's ramp / tail
    // under the other's body, as the dual FILTER streams of one index do) and no hardware queue
    // (GPU_MAX_HW_QUEUES = 4) interleaves many shards' waits.  8 x 1.25M rows on one GPU: 3.73 ms/batch
    // with a stream per shard, 3.88 with n = 1, 3.37 with n = 2, 3.58 with n = 4
    // (profiles/r03_group_scan_streams.log).  HIPRAG_GROUP_SCAN_STREAMS = n (0: a stream per shard)
    static const int gss_env = getenv("HIPRAG_GROUP_SCAN_STREAMS") ? atoi(getenv("HIPRAG_GROUP_SCAN_STREAMS")) : 2;
    if (gss_env > 0) {
        std::vector<std::pair<int, int>> made;  // (device, index) of p->owned
        for (int s = 0; s < G && e == hipSuccess; ++s) {
            hr_index* sh = g->shards[(size_t)s];
            if (!sh->shared_dev) continue;
            int r = 0;
            for (int t = 0; t < s; ++t) r += g->shards[(size_t)t]->device == sh->device;
            const std::pair<int, int> key{sh->device, r % gss_env};
            size_t i = 0;
            while (i < made.size() && made[i] != key) ++i;
            if (i == made.size()) {
                hipStream_t x = nullptr;
                e = hipSetDevice(sh->device);
                if (e == hipSuccess) e = hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
                if (e != hipSuccess) break;
                made.push_back(key);
                p->owned.push_back(x);
            }
            p->scan[(size_t)s] = p->owned[i];
        }
    }
    if (e == hipSuccess) e = hipSetDevice(g->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->merge, hipStreamNonBlocking);
    for (int i = 0; i < GroupPipe::kSlots && e == hipSuccess; ++i) {
        e = hipEventCreateWithFlags(&p->slot[i].q_ready, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->slot[i].merged, hipEventDisableTiming);
    }
    if (e != hipSuccess) return fail(e);
    for (int s = 0; s < G; ++s) p->qs.emplace_back(new WorkerQ());
    for (int s = 0; s < G; ++s) p->workers.emplace_back(pipe_worker, g, s);
    return HR_OK;
}

// wait until slot si's shard threads have enqueued everything (merge included); returns its error
static int pipe_wait_enqueued(GroupPipe* p, GroupPipe::Slot& sl) {
    std::unique_lock<std::mutex> lk(p->m);
    p->cv.wait(lk, [&] { return sl.pending < 0; });
    if (sl.err != HR_OK) return set_err(sl.err, sl.errmsg);
    return HR_OK;
}

static int pipe_finalize_slot(hr_index* g, GroupPipe::Slot& sl) {
    GroupPipe* p = g->pipe;
    struct Done {
        GroupPipe::Slot& sl;
        ~Done() { sl.busy = false; }
    } done{sl};
    if (int rc = pipe_wait_enqueued(p, sl)) return rc;
    HIP_TRY(hipSetDevice(g->device));
    HIP_TRY(hipEventSynchronize(sl.merged));
    std::vector<int> failed;
    for (int b = 0; b < sl.B; ++b)
        if (sl.fail_h[b]) failed.push_back(b);
    if (failed.empty()) return HR_OK;
    // the fallback drives the shards from this thread: every shard thread must be idle first
    for (auto& o : p->slot)
        if (o.busy && &o != &sl)
            if (int rc = pipe_wait_enqueued(p, o)) return rc;
    std::vector<const uint64_t*> mdev((size_t)g->G, nullptr);
    const int rc = group_fallback(g, sl.q, sl.k, failed, sl.kth_h, mdev, sl.s_out, sl.r_out, p->merge);
    return rc;
}

int group_drain(hr_index* g) {
    GroupPipe* p = g->pipe;
    if (!p) return HR_OK;
    int first_rc = HR_OK;
    for (int i = 0; i < GroupPipe::kSlots; ++i) {  // oldest first
        GroupPipe::Slot& sl = p->slot[(p->next + i) % GroupPipe::kSlots];
        if (!sl.busy) continue;
        const int rc = pipe_finalize_slot(g, sl);
        if (rc && first_rc == HR_OK) first_rc = rc;
    }
    return first_rc;
}

int group_search_submit(hr_index* g, const float* q_dev, int B, int k, float* s_out, int64_t* r_out, hipStream_t st,
                        int64_t* ticket) {
    if (int rc = pipe_start(g)) return rc;
    GroupPipe* p = g->pipe;
    GroupPipe::Slot& sl = p->slot[p->next];
    if (sl.busy)  // the slot's previous batch (two submits ago) is finalized first
        if (int rc = pipe_finalize_slot(g, sl)) return rc;
    const auto t0 = std::chrono::steady_clock::now();  // host work of this submit (not the wait above)
    p->next = (p->next + 1) % GroupPipe::kSlots;
    refresh_group_totals(g);
    const int kc = hr_kc_for_k_dim(k, g->dim);
    HIP_TRY(hipSetDevice(g->device));
    if (B > sl.cap_B) {
        if (sl.fail_h) HIP_TRY(hipHostFree(sl.fail_h));
        if (sl.kth_h) HIP_TRY(hipHostFree(sl.kth_h));
        sl.fail_h = nullptr;
        sl.kth_h = nullptr;
        HIP_TRY(hipHostMalloc((void**)&sl.fail_h, (size_t)B * 4));
        HIP_TRY(hipHostMalloc((void**)&sl.kth_h, (size_t)B * 8));
        sl.cap_B = B;
    }
    HIP_TRY(sl.cand.ensure((size_t)g->G * B * kc * sizeof(Cand)));
    HIP_TRY(sl.bound.ensure((size_t)g->G * B * 8));
    HIP_TRY(sl.kth.ensure((size_t)B * 8));
    HIP_TRY(sl.fail.ensure((size_t)B * 4));
    HIP_TRY(hipEventRecord(sl.q_ready, st));
    sl.q = q_dev;
    sl.B = B;
    sl.k = k;
    sl.kc = kc;
    sl.s_out = s_out;
    sl.r_out = r_out;
    sl.err = HR_OK;
    sl.errmsg.clear();
    sl.ticket = p->next_ticket++;
    {
        std::lock_guard<std::mutex> lk(p->m);
        sl.pending = g->G;
    }
    sl.busy = true;
    const int si = (int)(&sl - p->slot);
    for (int s = 0; s < g->G; ++s) {
        WorkerQ& wq = *p->qs[(size_t)s];
        std::lock_guard<std::mutex> lk(wq.m);
        wq.q.push_back(Job{si});
        wq.cv.notify_one();
    }
    *ticket = sl.ticket;
    p->batches++;
    p->submit_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    return HR_OK;
}

int group_search_finalize(hr_index* g, int64_t ticket) {
    GroupPipe* p = g->pipe;
    if (!p || ticket <= 0) return HR_OK;
    for (auto& sl : p->slot)
        if (sl.busy && sl.ticket == ticket) return pipe_finalize_slot(g, sl);
    return HR_OK;  // finalized already (by a later submit or a drain)
}

int group_host_us(hr_index* g, double out[3]) {
    GroupPipe* p = g->pipe;
    out[0] = out[1] = out[2] = 0.0;
    if (!p || !p->batches) return HR_OK;
    std::lock_guard<std::mutex> lk(p->m);
    out[0] = p->submit_us / (double)p->batches;
    double mx = 0.0;
    for (double u : p->shard_us) mx = std::max(mx, u);
    out[1] = mx / (double)p->batches;
    out[2] = (double)p->batches;
    return HR_OK;
}

// ---------------------------------------------------------------- persistence
// The file is the single-index layout (header, handle tiles in order with the slot swizzle of the
// handle tile, live words): written / read in blocks of handle tiles, re-swizzled on the host.
int group_save(hr_index* g, const char* path) {
    if (int rc = group_drain(g)) return rc;  // batches in flight first (they read the rows)
    refresh_group_totals(g);
    const std::string tmp_path = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp_path.c_str(), "wb");
    if (!f) return set_err(HR_E_IO, std::string("cannot open ") + tmp_path);
    FileHeader hd{};
    std::memcpy(hd.magic, "HIPRAG02", 8);
    hd.version = 1;
    hd.dim = g->dim;
    hd.dtype = g->dtype;
    hd.metric = g->metric;
    hd.n = g->n;
    hd.n_live = g->n_live;
    hd.max_norm2 = g->max_norm2;
    bool ok = std::fwrite(&hd, sizeof(hd), 1, f) == 1;
    const int G = g->G;
    const bool f32 = g->dtype == F32;
    const size_t tb = (size_t)g->S * (f32 ? 2048 : 1024);
    const int64_t tiles = (g->n + 31) / 32;
    const int64_t step = std::max<int64_t>(G, (((int64_t)256 << 20) / (int64_t)tb) / G * G);  // handle tiles per block
    std::vector<std::vector<uint8_t>> sb((size_t)G);
    std::vector<uint8_t> out;
    for (int64_t T0 = 0; ok && T0 < tiles; T0 += step) {
        const int64_t T1 = std::min(tiles, T0 + step);
        for (int s = 0; s < G && ok; ++s) {  // this shard's local tiles of [T0, T1): contiguous
            hr_index* sh = g->shards[(size_t)s];
            const int64_t l0 = T0 / G + (T0 % G > s ? 1 : 0), l1 = (T1 - 1 - s) >= 0 ? (T1 - 1 - s) / G + 1 : 0;
            sb[(size_t)s].resize((size_t)std::max<int64_t>(0, l1 - l0) * tb);
            if (l1 > l0 && hipMemcpy(sb[(size_t)s].data(), sh->rows + (size_t)l0 * tb, (size_t)(l1 - l0) * tb,
                                     hipMemcpyDeviceToHost) != hipSuccess)
                ok = false;
        }
        out.resize((size_t)(T1 - T0) * tb);
        for (int64_t T = T0; ok && T < T1; ++T) {
            const int s = (int)(T % G);
            const int64_t lt = T / G, l0 = T0 / G + (T0 % G > s ? 1 : 0);
            reswizzle_tile(sb[(size_t)s].data() + (size_t)(lt - l0) * tb, out.data() + (size_t)(T - T0) * tb, g->S, f32,
                           lt, T);
        }
        if (ok) ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    }
    if (ok && tiles > 0) {
        std::vector<uint32_t> lw((size_t)tiles);
        for (int64_t T = 0; T < tiles; ++T) lw[(size_t)T] = g->shards[(size_t)(T % G)]->live_host[(size_t)(T / G)];
        ok = std::fwrite(lw.data(), 4, lw.size(), f) == lw.size();
    }
    ok = ok && std::fflush(f) == 0 && fsync(fileno(f)) == 0;
    ok = (std::fclose(f) == 0) && ok;
    if (ok) ok = std::rename(tmp_path.c_str(), path) == 0;
    if (!ok) std::remove(tmp_path.c_str());
    return ok ? HR_OK : set_err(HR_E_IO, std::string("write failed: ") + path);
}

int group_load_into(hr_index* g, FILE* f, int64_t n, int64_t n_live, double max_norm2) {
    (void)n_live;
    const int G = g->G;
    const bool f32 = g->dtype == F32;
    const size_t tb = (size_t)g->S * (f32 ? 2048 : 1024);
    const int64_t tiles = (n + 31) / 32;
    if (int rc = group_reserve(g, n)) return rc;
    const std::vector<int64_t> cnt = split_counts(0, n, G);
    const int64_t step = std::max<int64_t>(G, (((int64_t)256 << 20) / (int64_t)tb) / G * G);
    std::vector<uint8_t> in;
    std::vector<std::vector<uint8_t>> sb((size_t)G);
    for (int64_t T0 = 0; T0 < tiles; T0 += step) {
        const int64_t T1 = std::min(tiles, T0 + step);
        in.resize((size_t)(T1 - T0) * tb);
        if (std::fread(in.data(), 1, in.size(), f) != in.size()) return set_err(HR_E_IO, "truncated index file");
        for (int s = 0; s < G; ++s) sb[(size_t)s].clear();
        for (int64_t T = T0; T < T1; ++T) {
            const int s = (int)(T % G);
            auto& b = sb[(size_t)s];
            const size_t at = b.size();
            b.resize(at + tb);
            reswizzle_tile(in.data() + (size_t)(T - T0) * tb, b.data() + at, g->S, f32, T, T / G);
        }
        for (int s = 0; s < G; ++s) {
            if (sb[(size_t)s].empty()) continue;
            hr_index* sh = g->shards[(size_t)s];
            const int64_t l0 = T0 / G + (T0 % G > s ? 1 : 0);
            if (int rc = set_device(sh)) return rc;
            HIP_TRY(hipMemcpy(sh->rows + (size_t)l0 * tb, sb[(size_t)s].data(), sb[(size_t)s].size(), hipMemcpyHostToDevice));
            shadow_stale(sh, l0);
        }
    }
    std::vector<uint32_t> lw((size_t)tiles);
    if (tiles > 0 && std::fread(lw.data(), 4, lw.size(), f) != lw.size()) return set_err(HR_E_IO, "truncated index file");
    for (int s = 0; s < G; ++s) {
        hr_index* sh = g->shards[(size_t)s];
        sh->n = cnt[(size_t)s];
        const int64_t lt_n = (sh->n + 31) / 32;
        int64_t live = 0;
        for (int64_t lt = 0; lt < lt_n; ++lt) {
            const uint32_t w = lw[(size_t)(lt * G + s)];
            sh->live_host[(size_t)lt] = w;
            live += __builtin_popcount(w);
        }
        sh->n_live = live;
        sh->max_norm2 = max_norm2;  // the handle's maximum: an upper bound for every shard's guard
        if (int rc = set_device(sh)) return rc;
        if (lt_n > 0)
            HIP_TRY(hipMemcpy(sh->live, sh->live_host.data(), (size_t)lt_n * 4, hipMemcpyHostToDevice));
        if (int rc = index_finish_load(sh)) return rc;
    }
    g->n = n;
    refresh_group_totals(g);
    return HR_OK;
}
