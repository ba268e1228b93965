// hr_exhaustive.hip -- last-resort exact top-m of one query over a whole shard.
//
// The collect fallback (DESIGN.md "Exactness guard") gathers every row whose approximate
// score is within the error bound of the k-th exact score; when that window holds more rows
// than its buffer (massive exact ties, or an embedding model that maps every chunk to
// nearly the same direction -- a random-init transformer does), this path takes over:
// canonical fp64 score of every live, allowed row (same arithmetic as k_rescore, so the
// same bits as the oracle), then a stable descending radix sort of (score key, row) --
// stability keeps equal scores in row order, i.e. the (score desc, row asc) order of
// the reference (faiss_store.py:139-149 / the oracle).  Cost ~ one exact pass over the
// shard plus the sort; it only runs for queries whose collect window overflowed.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "../../include/hiprag.h"
#include "hr_common.hpp"

namespace {

// one wave per row; key 0 (below d2key(-inf)) marks rows that are deleted or masked out
template <int DT>
__global__ __launch_bounds__(256) void k_exact_all(const uint8_t* __restrict__ rows, int S, int dpad,
                                                   const float* __restrict__ qv, int metric, double qn2,
                                                   const uint32_t* __restrict__ live,
                                                   const uint32_t* __restrict__ mask, int64_t n,
                                                   uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    uint32_t allow = live[r >> 5];
    if (mask) allow &= mask[r >> 5];
    if (!((allow >> (r & 31)) & 1u)) {
        if (lane == 0) {
            keys[r] = 0;
            vals[r] = (uint32_t)r;
        }
        return;
    }
    double p = 0.0, x2 = 0.0;
#pragma unroll 8
    for (int d = lane; d < dpad; d += 64) {
        const double x = (double)hr::load_elem<DT>(rows, S, r, d);
        p = p + x * (double)qv[d];
        if (metric == hr::L2) x2 = x2 + x * x;
    }
    p = hr::wave_butterfly_sum(p);
    if (metric == hr::L2) p = hr::euclid_score(qn2, p, hr::wave_butterfly_sum(x2));
    if (lane == 0) {
        keys[r] = hr::d2key(p);
        vals[r] = (uint32_t)r;
    }
}

__global__ void k_take(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals, int64_t n, int m,
                       int64_t row_offset, int sG, int ss, hr::Cand* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    if (i < n && keys[i] != 0)
        out[i] = hr::Cand{hr::key2d(keys[i]), hr::stripe_row((int64_t)vals[i], sG, ss) + row_offset};
    else
        out[i] = hr::Cand{-__builtin_inf(), -1};
}

}  // namespace

namespace {
// tile t holds at least one live, allowed row
struct TileAllowed {
    const uint32_t* live;
    const uint32_t* mask;
    __device__ bool operator()(uint32_t t) const { return (live[t] & mask[t]) != 0u; }
};
}  // namespace

namespace hr {

// Sorted list of the tiles holding a live, allowed row of a DEVICE row mask (rocPRIM select over
// tile indices; the count lands in device memory).  The host-mask path builds the same list on the
// host (hr_index_search); this one serves device masks (pipelined / distributed search).
size_t tile_list_scratch_bytes(int64_t n_tiles) {
    size_t tmp = 0;
    if (rocprim::select(nullptr, tmp, rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr, (uint32_t*)nullptr,
                        (size_t)n_tiles, TileAllowed{nullptr, nullptr}) != hipSuccess)
        tmp = 0;
    return tmp;
}

int build_tile_list(const uint32_t* live, const uint32_t* mask, int64_t n_tiles, uint32_t* list, uint32_t* count,
                    void* scratch, size_t scratch_bytes, hipStream_t st) {
    return rocprim::select(scratch, scratch_bytes, rocprim::counting_iterator<uint32_t>(0), list, count,
                           (size_t)n_tiles, TileAllowed{live, mask}, st) == hipSuccess
               ? HR_OK
               : HR_E_HIP;
}

// scratch layout: keys_in, keys_out (8n each), vals_in, vals_out (4n each), radix-sort temp
size_t exhaustive_scratch_bytes(int64_t n) {
    size_t tmp = 0;
    if (rocprim::radix_sort_pairs_desc(nullptr, tmp, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                       (uint32_t*)nullptr, (size_t)n, 0, 64) != hipSuccess)
        tmp = 0;  // the sort call below then reports the error
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return up(8 * (size_t)n) * 2 + up(4 * (size_t)n) * 2 + up(tmp);
}

// exact top-m (score desc, row asc) of query qv over rows [0, n) into out[0..m); empty slots -inf / -1;
// returned rows are stripe_row(local row, sG, ss) + row_offset
int exhaustive_topm(const uint8_t* rows, int dtype, int S, int dpad, const float* qv, int metric, double qn2,
                    const uint32_t* live,
                    const uint32_t* mask, int64_t n, int64_t row_offset, int m, Cand* out, void* scratch,
                    size_t scratch_bytes, hipStream_t st, int sG, int ss) {
    if (m <= 0) return HR_E_INVALID;
    if (n <= 0) {  // an empty shard: m padding records
        hipLaunchKernelGGL(k_take, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, (const uint64_t*)nullptr,
                           (const uint32_t*)nullptr, (int64_t)0, m, row_offset, sG, ss, out);
        return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
    }
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    uint8_t* p = (uint8_t*)scratch;
    uint64_t* k_in = (uint64_t*)p;
    uint64_t* k_out = (uint64_t*)(p + up(8 * (size_t)n));
    uint32_t* v_in = (uint32_t*)(p + 2 * up(8 * (size_t)n));
    uint32_t* v_out = (uint32_t*)(p + 2 * up(8 * (size_t)n) + up(4 * (size_t)n));
    uint8_t* tmp = p + 2 * up(8 * (size_t)n) + 2 * up(4 * (size_t)n);
    if (scratch_bytes < exhaustive_scratch_bytes(n)) return HR_E_INVALID;
    size_t tmp_bytes = scratch_bytes - (size_t)(tmp - p);
    const dim3 grid((unsigned)((n + 3) / 4));
    switch (dtype) {
        case HR_F32: hipLaunchKernelGGL(k_exact_all<F32>, grid, dim3(256), 0, st, rows, S, dpad, qv, metric, qn2, live, mask, n, k_in, v_in); break;
        case HR_BF16: hipLaunchKernelGGL(k_exact_all<BF16>, grid, dim3(256), 0, st, rows, S, dpad, qv, metric, qn2, live, mask, n, k_in, v_in); break;
        case HR_F16: hipLaunchKernelGGL(k_exact_all<F16>, grid, dim3(256), 0, st, rows, S, dpad, qv, metric, qn2, live, mask, n, k_in, v_in); break;
        default: return HR_E_INVALID;
    }
    if (hipGetLastError() != hipSuccess) return HR_E_HIP;
    if (rocprim::radix_sort_pairs_desc(tmp, tmp_bytes, k_in, k_out, v_in, v_out, (size_t)n, 0, 64, st) != hipSuccess)
        return HR_E_HIP;
    hipLaunchKernelGGL(k_take, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, k_out, v_out, n, m, row_offset,
                       sG, ss, out);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}

// Merge of G ranks' sorted lists (the exhaustive pass's output: m records per query in (score desc, row asc) order,
// padding (row < 0) at the tail; rank g's lists start at cand + g * cstride bytes, query q's at q * m records) into
// the top-k: element i of rank g lands at position i + (elements of every other rank's list that precede it), found
// by binary search -- the ranks' rows are disjoint, so the order is total and the positions a permutation.  No LDS
// bound on G * m (k_merge's is 8192 candidates): the large-k merge of the row-sharded search.
__global__ __launch_bounds__(256) void k_merge_sorted(const uint8_t* __restrict__ cand, int64_t cstride, int G, int B,
                                                      int m, int k, float* __restrict__ s_out,
                                                      int64_t* __restrict__ r_out) {
    const int q = blockIdx.y;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= B || t >= (int64_t)G * m) return;
    const int g = (int)(t / m), i = (int)(t % m);
    if (i >= k) return;  // at least i elements of its own list precede it
    const Cand e = ((const Cand*)(cand + g * cstride))[(int64_t)q * m + i];
    if (e.row < 0) return;
    const uint64_t ke = d2key(e.score);
    int64_t pos = i;
    for (int h = 0; h < G && pos < k; ++h) {
        if (h == g) continue;
        const Cand* L = (const Cand*)(cand + h * cstride) + (int64_t)q * m;
        int lo = 0, hi = m;  // first index of L that does not precede e
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const Cand x = L[mid];
            const uint64_t kx = d2key(x.score);
            const bool before = x.row >= 0 && (kx > ke || (kx == ke && x.row < e.row));
            if (before) lo = mid + 1;
            else hi = mid;
        }
        pos += lo;
    }
    if (pos < k) {
        s_out[(int64_t)q * k + pos] = (float)e.score;
        r_out[(int64_t)q * k + pos] = e.row;
    }
}

__global__ void k_pad_results(float* __restrict__ s_out, int64_t* __restrict__ r_out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    s_out[i] = -__builtin_inff();
    r_out[i] = -1;
}

int launch_merge_sorted(const Cand* cand, int64_t cstride, int G, int B, int m, int k, float* s_out, int64_t* r_out,
                        hipStream_t st) {
    const int64_t nk = (int64_t)B * k;
    hipLaunchKernelGGL(k_pad_results, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, st, s_out, r_out, nk);
    if (hipGetLastError() != hipSuccess) return HR_E_HIP;
    const int64_t per_q = (int64_t)G * m;
    hipLaunchKernelGGL(k_merge_sorted, dim3((unsigned)((per_q + 255) / 256), (unsigned)B), dim3(256), 0, st,
                       (const uint8_t*)cand, cstride, G, B, m, k, s_out, r_out);
    return hipGetLastError() == hipSuccess ? HR_OK : HR_E_HIP;
}

}  // namespace hr
