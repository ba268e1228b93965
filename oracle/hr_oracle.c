/*
 * hr_oracle.c -- CPU restatement of the youtu-rag KB-search arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker.
 * The product path (youtu-rag_amd/hiprag + libhiprag.so) never links it.
 *
 * What it restates (reference file:line, relative to the youtu-rag tree):
 *   - FAISSVectorStore cosine semantics, the reference's exact store:
 *       normalize_L2 on add        utu/rag/storage/implementations/faiss_store.py:102-108
 *       normalize_L2 on the query  faiss_store.py:148-149
 *       IndexFlatIP exact search   faiss_store.py:103, :154 (similarity = inner product, :179-180)
 *     faiss-cpu 1.12.0 (uv.lock:1286-1287) is a third-party dependency that is
 *     not vendored under the reference; its published IndexFlatIP algorithm is
 *     an exhaustive inner-product scan returning the k largest scores.
 *   - Chroma's hnsw "ip" space for distance_metric="dot" (chroma_store.py:48-53,
 *     similarity = 1 - distance = inner product, :135).
 *   - Chroma's hnsw "l2" space for distance_metric="euclidean" (chroma_store.py:48-53):
 *     distance = squared L2 (hnswlib's l2 space), similarity = 1 - distance (:135);
 *     rows and queries are stored raw.  chromadb 1.3.4 (uv.lock:764-765) is not vendored
 *     and its HNSW is approximate; the exact restatement ranks every row by
 *       score = 1 - ((|q|^2 - 2 q.x) + |x|^2)
 *     with the three terms canonical fp64 sums (below) combined in that order.
 *
 * Canonical arithmetic (shared bit-for-bit with the HIP kernels):
 *   - every dot product / squared norm is an fp64 sum in a fixed order:
 *     64 "lanes", lane l sums terms d = l, l+64, l+128, ... sequentially, then
 *     the 64 partials are combined by the butterfly p[i] += p[i+off] for
 *     off = 32, 16, 8, 4, 2, 1.  Products of fp32/bf16/fp16 operands are exact
 *     in fp64, so FMA contraction cannot change a result.
 *   - normalisation: inv = 1/sqrt(n2) in fp64 (correctly rounded), x' =
 *     (float)(x * inv); rows with n2 == 0 are left unchanged (faiss behaviour).
 *   - storage quantisation: fp32 -> bf16 / fp16 round-to-nearest-even on the
 *     bit pattern.
 *   - result order: exact fp64 score descending, then row ascending.
 *   - synthetic corpus: element (row, d) = sum of the four 16-bit fields of
 *     mix64(seed*K + row*D + d) minus 131070 (an integer, exact in fp32).
 *
 * Parity pin: tests/golden/ holds vectors produced by running the reference's
 * own VectorRetriever (base_retriever.py:42-99) over this restatement; see
 * tests/golden/gen_golden.py and DESIGN.md "Oracle".
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define HRO_F32 0
#define HRO_BF16 1
#define HRO_F16 2

#define HRO_COSINE 0
#define HRO_IP 1
#define HRO_L2 2

uint64_t hro_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline float gen_elem(uint64_t seed, int64_t row, int dim, int d) {
    uint64_t z = hro_mix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)row * (uint64_t)dim + (uint64_t)d);
    int64_t v = (int64_t)(z & 0xFFFF) + (int64_t)((z >> 16) & 0xFFFF) + (int64_t)((z >> 32) & 0xFFFF) +
                (int64_t)(z >> 48) - 131070;
    return (float)v;
}

/* Synthetic corpus rows [row0, row0+n) of dimension dim, fp32 row-major. */
void hro_gen_rows(uint64_t seed, int64_t row0, int64_t n, int dim, float* out) {
    for (int64_t r = 0; r < n; ++r)
        for (int d = 0; d < dim; ++d) out[r * dim + d] = gen_elem(seed, row0 + r, dim, d);
}

/* Canonical fp64 sum of a[d]*b[d] (see header). */
double hro_canon_dot(const double* a, const double* b, int dim) {
    double p[64];
    for (int l = 0; l < 64; ++l) p[l] = 0.0;
    int full = dim & ~63;
    for (int base = 0; base < full; base += 64) /* fixed trip count: vectorises across lanes */
        for (int l = 0; l < 64; ++l) p[l] = p[l] + a[base + l] * b[base + l];
    for (int l = 0; l < dim - full; ++l) p[l] = p[l] + a[full + l] * b[full + l];
    for (int off = 32; off >= 1; off >>= 1)
        for (int i = 0; i < off; ++i) p[i] = p[i] + p[i + off];
    return p[0];
}

static double canon_norm2_f32(const float* x, int dim) {
    double p[64];
    for (int l = 0; l < 64; ++l) p[l] = 0.0;
    for (int base = 0; base < dim; base += 64) {
        int lim = dim - base < 64 ? dim - base : 64;
        for (int l = 0; l < lim; ++l) {
            double v = (double)x[base + l];
            p[l] = p[l] + v * v;
        }
    }
    for (int off = 32; off >= 1; off >>= 1)
        for (int i = 0; i < off; ++i) p[i] = p[i] + p[i + off];
    return p[0];
}

double hro_norm2(const float* x, int dim) { return canon_norm2_f32(x, dim); }

/* Canonical L2 normalisation of n rows (in may alias out). */
void hro_normalize_rows(const float* in, int64_t n, int dim, float* out) {
    for (int64_t r = 0; r < n; ++r) {
        const float* x = in + r * dim;
        float* y = out + r * dim;
        double n2 = canon_norm2_f32(x, dim);
        if (n2 > 0.0) {
            double inv = 1.0 / sqrt(n2);
            for (int d = 0; d < dim; ++d) y[d] = (float)((double)x[d] * inv);
        } else if (y != x) {
            memcpy(y, x, sizeof(float) * (size_t)dim);
        }
    }
}

uint16_t hro_f32_to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (uint16_t)((u >> 16) | 0x40u); /* quiet NaN */
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

float hro_bf16_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

uint16_t hro_f32_to_f16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    uint32_t sign = (u >> 16) & 0x8000u;
    uint32_t a = u & 0x7FFFFFFFu;
    if (a >= 0x7F800000u) return (uint16_t)(sign | 0x7C00u | (a > 0x7F800000u ? 0x200u : 0u));
    if (a >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u); /* rounds to >= 65520 -> inf */
    if (a < 0x38800000u) {                                   /* result is subnormal or zero */
        int e = (int)(a >> 23);
        if (e < 102) return (uint16_t)sign;                  /* < half of the smallest subnormal */
        uint32_t m = (a & 0x7FFFFFu) | 0x800000u;
        int shift = 126 - e;                                 /* 14 .. 24 */
        uint32_t q = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t r = a - 0x38000000u; /* rebias exponent 127 -> 15 */
    r += 0xFFFu + ((r >> 13) & 1u);
    return (uint16_t)(sign | (r >> 13));
}

float hro_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1Fu, m = h & 0x3FFu, u;
    if (e == 0) {
        if (m == 0) {
            u = sign;
        } else {
            float f = (float)m * (1.0f / 16777216.0f);
            memcpy(&u, &f, 4);
            u |= sign;
        }
    } else if (e == 31) {
        u = sign | 0x7F800000u | (m << 13);
    } else {
        u = sign | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* Quantise n×dim fp32 rows into the storage dtype (HRO_F32 copies). */
void hro_quantize(const float* in, int64_t n, int dim, int dtype, void* out) {
    size_t cnt = (size_t)n * (size_t)dim;
    if (dtype == HRO_F32) {
        memcpy(out, in, cnt * 4);
    } else if (dtype == HRO_BF16) {
        uint16_t* o = (uint16_t*)out;
        for (size_t i = 0; i < cnt; ++i) o[i] = hro_f32_to_bf16(in[i]);
    } else {
        uint16_t* o = (uint16_t*)out;
        for (size_t i = 0; i < cnt; ++i) o[i] = hro_f32_to_f16(in[i]);
    }
}

/* Build stored rows for the synthetic corpus: generate, (cosine) normalise, quantise. */
void hro_build_synthetic(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, int metric, void* out,
                         int nthreads) {
    (void)nthreads;
    size_t esz = dtype == HRO_F32 ? 4 : 2;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        float* tmp = (float*)malloc(sizeof(float) * (size_t)dim);
#pragma omp for schedule(static)
        for (int64_t r = 0; r < n; ++r) {
            for (int d = 0; d < dim; ++d) tmp[d] = gen_elem(seed, row0 + r, dim, d);
            if (metric == HRO_COSINE) hro_normalize_rows(tmp, 1, dim, tmp);
            hro_quantize(tmp, 1, dim, dtype, (char*)out + (size_t)r * dim * esz);
        }
        free(tmp);
    }
}

static inline void load_row_f64(const void* stored, int dtype, int64_t r, int dim, double* dst) {
    if (dtype == HRO_F32) {
        const float* x = (const float*)stored + (size_t)r * dim;
        for (int d = 0; d < dim; ++d) dst[d] = (double)x[d];
    } else if (dtype == HRO_BF16) {
        const uint16_t* x = (const uint16_t*)stored + (size_t)r * dim;
        for (int d = 0; d < dim; ++d) dst[d] = (double)hro_bf16_to_f32(x[d]);
    } else {
        const uint16_t* x = (const uint16_t*)stored + (size_t)r * dim;
        for (int d = 0; d < dim; ++d) dst[d] = (double)hro_f16_to_f32(x[d]);
    }
}

/* (score desc, row asc): a ranks before b */
static inline int ranks_before(double sa, int64_t ra, double sb, int64_t rb) {
    return sa > sb || (sa == sb && ra < rb);
}

/* insert (s,r) into the sorted top-k list (length cnt <= k) */
static inline void topk_insert(double* ls, int64_t* lr, int* cnt, int k, double s, int64_t r) {
    int c = *cnt;
    if (c == k && !ranks_before(s, r, ls[k - 1], lr[k - 1])) return;
    int pos = c < k ? c : k - 1;
    while (pos > 0 && ranks_before(s, r, ls[pos - 1], lr[pos - 1])) {
        ls[pos] = ls[pos - 1];
        lr[pos] = lr[pos - 1];
        --pos;
    }
    ls[pos] = s;
    lr[pos] = r;
    if (c < k) *cnt = c + 1;
}

static inline int row_allowed(const uint64_t* mask, int64_t r) {
    return mask == NULL || ((mask[r >> 6] >> (r & 63)) & 1ull);
}

/*
 * Exact top-k over stored rows.  q: B×dim fp32 queries, already processed the
 * way the store processes them (normalised for cosine).  row_offset is added to
 * the returned rows (shards).  Unfilled slots get score -inf and row -1.
 */
typedef void (*row_source_fn)(void* ctx, int64_t r, double* dst);

/* score of one row: inner product (cosine on normalised rows, ip), or the euclidean similarity */
static inline double row_score(const double* xr, const double* qv, int dim, int metric, double qn2) {
    double dot = hro_canon_dot(xr, qv, dim);
    if (metric != HRO_L2) return dot;
    double xn2 = hro_canon_dot(xr, xr, dim);
    return 1.0 - ((qn2 - 2.0 * dot) + xn2);
}

static void search_generic(row_source_fn src, void* ctx, int64_t n, int dim, const float* q, int B, int k,
                           const uint64_t* mask, int64_t row_offset, double* scores_out, int64_t* rows_out,
                           int nthreads, int metric) {
    int nt = nthreads > 0 ? nthreads : 1;
    double* qd = (double*)malloc(sizeof(double) * (size_t)B * dim);
    for (size_t i = 0; i < (size_t)B * dim; ++i) qd[i] = (double)q[i];
    double* qn2 = (double*)malloc(sizeof(double) * (size_t)B);
    for (int b = 0; b < B; ++b) qn2[b] = hro_canon_dot(qd + (size_t)b * dim, qd + (size_t)b * dim, dim);
    double* all_s = (double*)malloc(sizeof(double) * (size_t)nt * B * k);
    int64_t* all_r = (int64_t*)malloc(sizeof(int64_t) * (size_t)nt * B * k);
    int* all_c = (int*)calloc((size_t)nt * B, sizeof(int));
#pragma omp parallel num_threads(nt)
    {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        double* xr = (double*)malloc(sizeof(double) * (size_t)dim);
        double* ls = all_s + (size_t)t * B * k;
        int64_t* lr = all_r + (size_t)t * B * k;
        int* lc = all_c + (size_t)t * B;
#pragma omp for schedule(static)
        for (int64_t r = 0; r < n; ++r) {
            if (!row_allowed(mask, r)) continue;
            src(ctx, r, xr);
            for (int b = 0; b < B; ++b) {
                double s = row_score(xr, qd + (size_t)b * dim, dim, metric, qn2[b]);
                topk_insert(ls + (size_t)b * k, lr + (size_t)b * k, lc + b, k, s, r + row_offset);
            }
        }
        free(xr);
    }
    for (int b = 0; b < B; ++b) {
        double* fs = scores_out + (size_t)b * k;
        int64_t* fr = rows_out + (size_t)b * k;
        int cnt = 0;
        for (int t = 0; t < nt; ++t) {
            int c = all_c[(size_t)t * B + b];
            for (int i = 0; i < c; ++i)
                topk_insert(fs, fr, &cnt, k, all_s[((size_t)t * B + b) * k + i], all_r[((size_t)t * B + b) * k + i]);
        }
        for (int i = cnt; i < k; ++i) {
            fs[i] = -INFINITY;
            fr[i] = -1;
        }
    }
    free(qd);
    free(qn2);
    free(all_s);
    free(all_r);
    free(all_c);
}

typedef struct {
    const void* stored;
    int dtype, dim;
} stored_ctx;

static void stored_src(void* c, int64_t r, double* dst) {
    stored_ctx* s = (stored_ctx*)c;
    load_row_f64(s->stored, s->dtype, r, s->dim, dst);
}

void hro_search(const void* stored, int dtype, int64_t n, int dim, const float* q, int B, int k,
                const uint64_t* mask, int64_t row_offset, double* scores_out, int64_t* rows_out, int nthreads,
                int metric) {
    stored_ctx c = {stored, dtype, dim};
    search_generic(stored_src, &c, n, dim, q, B, k, mask, row_offset, scores_out, rows_out, nthreads, metric);
}

typedef struct {
    uint64_t seed;
    int64_t row0;
    int dim, dtype, metric;
} synth_ctx;

static void synth_src(void* c, int64_t r, double* dst) {
    synth_ctx* s = (synth_ctx*)c;
    float tmp[4096];
    uint16_t h[4096];
    for (int d = 0; d < s->dim; ++d) tmp[d] = gen_elem(s->seed, s->row0 + r, s->dim, d);
    if (s->metric == HRO_COSINE) hro_normalize_rows(tmp, 1, s->dim, tmp);
    if (s->dtype == HRO_F32) {
        for (int d = 0; d < s->dim; ++d) dst[d] = (double)tmp[d];
    } else {
        hro_quantize(tmp, 1, s->dim, s->dtype, h);
        for (int d = 0; d < s->dim; ++d)
            dst[d] = (double)(s->dtype == HRO_BF16 ? hro_bf16_to_f32(h[d]) : hro_f16_to_f32(h[d]));
    }
}

/* Exact top-k over the synthetic corpus rows [row0, row0+n), generated on the fly (dim <= 4096). */
int hro_search_synthetic(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, int metric, const float* q,
                         int B, int k, double* scores_out, int64_t* rows_out, int nthreads) {
    if (dim > 4096) return -1;
    synth_ctx c = {seed, row0, dim, dtype, metric};
    search_generic(synth_src, &c, n, dim, q, B, k, NULL, row0, scores_out, rows_out, nthreads, metric);
    return 0;
}

/* The same restricted to the rows whose bit is set in mask (bit r of word r>>6, r relative to row0):
 * a where-clause bitmap AND the live rows, i.e. a filtered search over a store with tombstones. */
int hro_search_synthetic_masked(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, int metric,
                                const float* q, int B, int k, const uint64_t* mask, double* scores_out,
                                int64_t* rows_out, int nthreads) {
    if (dim > 4096) return -1;
    synth_ctx c = {seed, row0, dim, dtype, metric};
    search_generic(synth_src, &c, n, dim, q, B, k, mask, row0, scores_out, rows_out, nthreads, metric);
    return 0;
}

/* Exact canonical scores of explicit (query, row) pairs against stored rows. */
void hro_score_pairs(const void* stored, int dtype, int dim, const float* q, const int32_t* qidx, const int64_t* rows,
                     int64_t npairs, double* out, int metric) {
    double* xr = (double*)malloc(sizeof(double) * (size_t)dim);
    double* qd = (double*)malloc(sizeof(double) * (size_t)dim);
    for (int64_t i = 0; i < npairs; ++i) {
        load_row_f64(stored, dtype, rows[i], dim, xr);
        for (int d = 0; d < dim; ++d) qd[d] = (double)q[(size_t)qidx[i] * dim + d];
        out[i] = row_score(xr, qd, dim, metric, hro_canon_dot(qd, qd, dim));
    }
    free(xr);
    free(qd);
}

int hro_abi_version(void) { return 2; }
