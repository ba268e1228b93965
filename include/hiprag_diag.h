/*
 * hiprag_diag.h -- diagnostic and measurement entry points of libhiprag.so (tests, tools/ and bench.py use them to
 * check which kernel served a batch and to time its passes).  They have no counterpart in the reference and are not
 * part of the drop-in boundary (include/hiprag.h); same conventions: 0 or a negative HR_E_* code.
 */
#ifndef HIPRAG_DIAG_H
#define HIPRAG_DIAG_H

#include "hiprag.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostics: tiles each wave of the most recent k_scan FILTER launch scanned ([query group][wave], blocking;
 * up to cap counts, the number in n_out).  Every unit is scanned exactly once per group, so the counts sum to
 * groups x units -- the invariant of the round-robin dealing, its rotation and the dynamic tail. */
int hr_index_wave_tiles(hr_index* h, uint32_t* out, int cap, int* n_out);

/* The persistent FILTER (hr_index_set_persist): out[0] = batches served, out[1] = error word (a bounded wait gave up;
 * 0 = none), out[2] = instances that ran.  persist_trace: per epoch of the last n (oldest first), 5 device stamps in
 * us relative to the first one's post -- post, first / last workgroup start, first / last workgroup arrival
 * (blocking). */
int hr_index_persist_stats(hr_index* h, int64_t out[3]);
int hr_index_persist_trace(hr_index* h, int n, double* out, int* n_out);

/* Scan timing is off by default (each recorded event leaves a ~6 us bubble on the stream);
 * set_scan_timing(h, N) records HIP events around every N-th main pass (0 = off). */
int hr_index_set_scan_timing(hr_index* h, int every);
/* Timing of the main-pass scans (ms, HIP events recorded on the search stream).
 * take_scan_times harvests, in launch order, every (SAMPLE, FILTER) pair launched since the
 * previous harvest (blocking on the pending events; up to cap entries; count in n_out);
 * last_scan_ms harvests everything and reports the most recent pair.  A batch of the persistent FILTER reports
 * as its FILTER time the period between its last workgroup arrival and the previous batch's (device clock). */
int hr_index_take_scan_times(hr_index* h, float* sample_ms, float* filter_ms, int cap, int* n_out);
int hr_index_last_scan_ms(hr_index* h, float* sample_ms, float* filter_ms);

/* Diagnostics: approximate MFMA scores of every row (B <= 64; approx_out B×n) and the
 * per-query error bound E_q that the exactness guard uses (e_out, B). */
int hr_index_debug_approx(hr_index* h, const float* q, int B, float* approx_out, double* e_out);
/* Diagnostics: candidates appended by the most recent FILTER scan (sum, max per query). */
int hr_index_last_candidates(hr_index* h, int64_t* total, int64_t* max_per_query);

/* Diagnostics: hr_index_search calls answered by replaying a captured HIP graph (an unmasked,
 * untimed search with k <= HR_MAX_K, from the second call of a (B, k) shape on; HIPRAG_SYNC_GRAPH=0
 * turns the graphs off).  The results are those of the normal path: the graph is that path, captured. */
int hr_index_graph_replays(hr_index* h, int64_t* out);
/* Diagnostics: 128-query FILTER launches issued so far (65..256-query chunks at D = 256..1024; graph replays
 * not counted) -- tests use it to check which FILTER served a batch. */
int hr_index_wide_launches(hr_index* h, int64_t* out);
/* Diagnostics: 256-query FILTER launches issued so far (graph replays not counted). */
int hr_index_q256_launches(hr_index* h, int64_t* out);

/* Diagnostics of the pipelined search: out[0] = caller host time per submit (us), out[1] = host time
 * per batch of the busiest shard thread (us), out[2] = batches submitted. */
int hr_index_host_us(hr_index* h, double* out);

#ifdef __cplusplus
}
#endif
#endif /* HIPRAG_DIAG_H */
