/*
 * asan_driver.c -- drives every entry point of the CPU restatement (hr_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile target `asan`; TEST
 * INFRASTRUCTURE ONLY, like the restatement itself).  Edge cases: dims that are not multiples of
 * 64, empty and one-row corpora, k larger than the corpus, masks, every dtype and metric, exact
 * duplicates; every synthetic search is cross-checked against the same search over rows built by
 * hro_build_synthetic.  Exit status 0 = consistent (the sanitizers abort on any finding).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void hro_gen_rows(uint64_t seed, int64_t row0, int64_t n, int dim, float* out);
void hro_normalize_rows(const float* in, int64_t n, int dim, float* out);
void hro_quantize(const float* in, int64_t n, int dim, int dtype, void* out);
void hro_build_synthetic(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, int metric, void* out,
                         int nthreads);
void hro_search(const void* stored, int dtype, int64_t n, int dim, const float* q, int B, int k, const uint64_t* mask,
                int64_t row_offset, double* scores_out, int64_t* rows_out, int nthreads, int metric);
int hro_search_synthetic_masked(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, int metric,
                                const float* q, int B, int k, const uint64_t* mask, double* scores_out,
                                int64_t* rows_out, int nthreads);
int hro_search_synthetic(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, int metric, const float* q,
                         int B, int k, double* scores_out, int64_t* rows_out, int nthreads);
void hro_score_pairs(const void* stored, int dtype, int dim, const float* q, const int32_t* qidx, const int64_t* rows,
                     int64_t npairs, double* out, int metric);

static int fail(const char* what, int a, int b, int c) {
    fprintf(stderr, "MISMATCH %s (%d %d %d)\n", what, a, b, c);
    return 1;
}

int main(void) {
    const int dims[] = {1, 7, 64, 100, 130};
    const int64_t ns[] = {0, 1, 33, 257};
    int bad = 0;
    for (int di = 0; di < 5; ++di)
        for (int ni = 0; ni < 4; ++ni)
            for (int dtype = 0; dtype < 3; ++dtype)
                for (int metric = 0; metric < 3; ++metric) {
                    const int dim = dims[di], B = 3, k = 40;
                    const int64_t n = ns[ni];
                    const size_t esz = dtype == 0 ? 4 : 2;
                    void* stored = malloc((size_t)(n > 0 ? n : 1) * dim * esz);
                    hro_build_synthetic(5, 11, n, dim, dtype, metric, stored, 2);
                    float* q = malloc(sizeof(float) * B * dim);
                    hro_gen_rows(77, 0, B, dim, q);
                    if (metric == 0) hro_normalize_rows(q, B, dim, q);
                    uint64_t* mask = calloc((size_t)((n + 63) / 64 + 1), 8);
                    for (int64_t r = 0; r < n; ++r)
                        if ((r * 7) % 3) mask[r >> 6] |= 1ull << (r & 63);
                    double s1[3 * 40], s2[3 * 40];
                    int64_t r1[3 * 40], r2[3 * 40];
                    for (int m = 0; m < 2; ++m) {
                        const uint64_t* mk = m ? mask : NULL;
                        hro_search(stored, dtype, n, dim, q, B, k, mk, 11, s1, r1, 2, metric);
                        if (mk)
                            hro_search_synthetic_masked(5, 11, n, dim, dtype, metric, q, B, k, mk, s2, r2, 2);
                        else
                            hro_search_synthetic(5, 11, n, dim, dtype, metric, q, B, k, s2, r2, 2);
                        for (int i = 0; i < B * k; ++i)
                            if (r1[i] != r2[i] || (r1[i] >= 0 && memcmp(&s1[i], &s2[i], 8))) {  /* bits: f16 ip/l2 overflow to inf/NaN */
                                bad |= fail("synthetic vs stored", dim, (int)n, dtype * 3 + metric);
                                break;
                            }
                    }
                    if (n > 0) {
                        int32_t qi[4] = {0, 1, 2, 0};
                        int64_t rows[4] = {0, n - 1, n / 2, 0};
                        double out[4];
                        hro_score_pairs(stored, dtype, dim, q, qi, rows, 4, out, metric);
                        if (memcmp(&out[0], &out[3], 8)) bad |= fail("score_pairs", dim, (int)n, dtype);
                    }
                    float* raw = malloc(sizeof(float) * (size_t)(n > 0 ? n : 1) * dim);
                    hro_gen_rows(5, 11, n, dim, raw);
                    hro_normalize_rows(raw, n, dim, raw);
                    uint16_t* h = malloc(2 * (size_t)(n > 0 ? n : 1) * dim);
                    hro_quantize(raw, n, dim, 1, h);
                    hro_quantize(raw, n, dim, 2, h);
                    free(h);
                    free(raw);
                    free(mask);
                    free(q);
                    free(stored);
                }
    /* exact duplicates: ties in (score desc, row asc) order */
    {
        const int dim = 48, n = 100;
        float* x = malloc(sizeof(float) * n * dim);
        hro_gen_rows(3, 0, n, dim, x);
        for (int r = 10; r < n; r += 10) memcpy(x + (size_t)r * dim, x, sizeof(float) * dim);
        hro_normalize_rows(x, n, dim, x);
        double s[12];
        int64_t rr[12];
        hro_search(x, 0, n, dim, x, 1, 12, NULL, 0, s, rr, 3, 0);
        for (int i = 0; i < 10; ++i)
            if (rr[i] != 10 * i) bad |= fail("tie order", i, (int)rr[i], 0);
        free(x);
    }
    if (!bad) printf("asan driver: all consistent\n");
    return bad;
}
