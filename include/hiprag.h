/*
 * hiprag.h -- C ABI of libhiprag.so, the MI355X-native vector index behind
 * youtu-rag's KB-search plugin interfaces.
 *
 * Every entry point replaces one numeric call of the reference's vector store
 * (paths relative to the youtu-rag tree; the store is a BaseVectorStore,
 * utu/rag/base.py:187-232):
 *
 *   hr_index_create    ChromaVectorStore.__init__ / FAISSVectorStore.__init__
 *                        (chroma_store.py:25-62 get_or_create_collection with hnsw:space;
 *                         faiss_store.py:31-58 IndexFlatIP/IndexFlatL2 choice :102-105)
 *   hr_index_add       add_chunks -> collection.add / normalize_L2 + index.add
 *                        (chroma_store.py:64-88, faiss_store.py:89-127)
 *   hr_index_remove    delete / delete_by_document_id (row tombstones)
 *                        (chroma_store.py:150-183, faiss_store.py:201-254)
 *   hr_index_search    search -> collection.query(n_results=top_k, where=...)
 *                        (chroma_store.py:90-148; exact semantics of faiss_store.py:129-199)
 *   hr_index_search_device  the same on device-resident queries/results (batched
 *                        VectorRetriever.batch_retrieve, base_retriever.py:82-99)
 *   hr_index_size      count (chroma_store.py:249-255, faiss_store.py:283-289)
 *   hr_index_get_rows  get_by_id's stored embedding (chroma_store.py:224-247)
 *   hr_index_save/load PersistentClient dir / faiss write_index+pickle
 *                        (chroma_store.py:41-44, faiss_store.py:61-87)
 *   hr_index_search_shard / hr_index_search_shard_collect / hr_merge_candidates
 *                      row-sharded multi-GPU search (no reference counterpart: the
 *                      reference is single-process)
 *   hr_pool_normalize  the embedding server's masked mean-pool + F.normalize
 *                        (docs/content/docs/en/youtu-embedding/deploying-locally.mdx:75-79, :98-115)
 *
 * Conventions: every int-returning call returns 0 on success or a negative
 * HR_E_* code; hr_last_error() then holds a thread-local message.  Handles are
 * opaque; calls on one handle are serialised by an internal mutex.  Host
 * pointers are caller-owned; "_device"/"_shard"/merge calls take device pointers
 * and run on the given hipStream_t (NULL = the null stream, which is also
 * PyTorch's default stream); host-pointer calls use the handle's own stream and
 * return after synchronising it.  Scores follow the
 * reference's similarity convention (cosine/dot: inner product; euclidean: 1 - |q - x|^2).  Result order:
 * score descending, then row ascending; unfilled slots hold score -inf, row -1.
 * Diagnostic / measurement entry points (kernel counters, scan timing, stamps) are in include/hiprag_diag.h.
 */
#ifndef HIPRAG_H
#define HIPRAG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hr_index hr_index;

enum { HR_F32 = 0, HR_BF16 = 1, HR_F16 = 2 };         /* storage dtype */
/* distance metric (chroma_store.py:48-53): cosine (rows + queries L2-normalised, score = inner
 * product), ip ("dot": raw inner product), l2 ("euclidean": score = 1 - squared distance, Chroma's
 * similarity = 1 - distance, :135) */
enum { HR_COSINE = 0, HR_IP = 1, HR_L2 = 2 };
enum {
    HR_OK = 0,
    HR_E_INVALID = -1,   /* bad argument -> Python ValueError */
    HR_E_HIP = -2,       /* HIP runtime error -> RuntimeError */
    HR_E_UNSUPPORTED = -3,
    HR_E_OVERFLOW = -4,  /* candidate buffer overflow in the exact fallback */
    HR_E_IO = -5,
    HR_E_BUSY = -6       /* hr_index_search_submit_host: another call holds the handle (never waits) */
};

#define HR_MAX_K 128           /* largest top-k (kb_file_search recall 15 x 3, rerank top-100) */
#define HR_MAX_KC 256          /* largest per-shard candidate count kc (k = HR_MAX_K with its margin) */

int hr_index_create(int dim, int dtype, int metric, int n_dev, const int* dev_ids, hr_index** out);
int hr_index_reserve(hr_index* h, int64_t capacity_rows);
int hr_index_add(hr_index* h, const float* rows, int64_t n, int64_t* first_row_out);
int hr_index_add_synthetic(hr_index* h, uint64_t seed, int64_t global_row0, int64_t n, int64_t* first_row_out);
/* Same as hr_index_add for n fp32 rows already in device memory (e.g. the in-process embedder's
 * hr_pool_normalize output): ordered after the work queued on `stream`, no host round trip of the
 * vectors; returns once the rows are stored (rows_dev may then be reused).
 * Replaces embed_texts -> add_chunks in BaseProcessor._chunk_and_store (processors.py:413-418). */
int hr_index_add_device(hr_index* h, const float* rows_dev, int64_t n, int64_t* first_row_out, void* stream);
/* Store n fp32 device rows at explicit positions dest_dev[i] (< n_rows_after, previously unused),
 * e.g. rows placed by list for an IVF index; the index then holds n_rows_after rows, positions
 * never written stay dead.  Ordered after the work queued on `stream`; returns once stored. */
int hr_index_add_device_at(hr_index* h, const float* rows_dev, int64_t n, const int64_t* dest_dev,
                           int64_t n_rows_after, void* stream);
/* The synthetic corpus generator (the one hr_index_add_synthetic and the oracle use) writing n fp32
 * rows of dimension dim, row-major, to device memory on `stream`. */
int hr_gen_rows_device(uint64_t seed, int64_t row0, int64_t n, int dim, float* out_dev, void* stream);
int hr_index_remove(hr_index* h, const int64_t* rows, int64_t n);
/* Host queries and outputs.  1 <= k <= HR_MAX_K: the scan path.  k > HR_MAX_K (Chroma's n_results
 * has no cap, chroma_store.py:118-120): an exhaustive exact pass per query (same scores and order,
 * one corpus pass + one n-row sort per query).  Slots past the live (allowed) rows: -inf / -1. */
int hr_index_search(hr_index* h, const float* q, int B, int k, const uint64_t* row_mask, float* scores_out,
                    int64_t* rows_out);
int hr_index_search_device(hr_index* h, const float* q_dev, int B, int k, const uint64_t* row_mask_dev,
                           float* scores_out_dev, int64_t* rows_out_dev, void* stream);
/* Pipelined form of hr_index_search_device (no mask, k <= HR_MAX_K): enqueue a batch and return a
 * ticket; hr_index_search_finalize(ticket) waits for that batch's exactness-guard flags, runs the exact
 * fallback for queries that need it and returns once scores_out/rows_out hold the final results.  A
 * multi-device handle keeps two batches in flight, every shard submitted by a host thread of its own
 * (so host time per batch does not grow with the number of devices); submitting a third finalizes the
 * oldest.  q_dev and the outputs must stay valid until the batch is finalized; other calls on the handle
 * finalize every batch in flight first.  A single-device handle completes the batch inside submit
 * (ticket 0).  Replaces VectorRetriever.batch_retrieve's sequential search loop (base_retriever.py:82-99)
 * for a store spanning the node's GPUs (one cached store per collection, base_toolkit.py:79-91). */
int hr_index_search_submit(hr_index* h, const float* q_dev, int B, int k, float* scores_out_dev, int64_t* rows_out_dev,
                           void* stream, int64_t* ticket_out);
int hr_index_search_finalize(hr_index* h, int64_t ticket);
/* Asynchronous search of host queries on a single-device handle (the drop-in store's micro-batcher on
 * an asyncio event loop; VectorRetriever.retrieve's store.search, base_retriever.py:58-63): copies the B
 * queries to pinned staging, enqueues the whole pass (query copy, prep, SAMPLE, FILTER, select, rescore,
 * merge, results + guard flags back to pinned memory) and returns a ticket without waiting.  When the
 * batch's results are in host memory a host function writes an 8-byte 1 to notify_fd (an eventfd the
 * caller polls; -1: none).  hr_index_search_collect(ticket) then copies the scores / rows out (after
 * running the exact fallback for queries that need it, synchronously).  At most two batches are in
 * flight, collected in any order (a third submit returns HR_E_BUSY until one is collected); adds, removes
 * and reserve wait for batches in flight first and run their exact fallbacks against the rows the batches
 * were submitted against; submit never blocks on the handle: while another call holds it, it returns
 * HR_E_BUSY at once.  No row mask; 1 <= k <= HR_MAX_K; an empty index or a multi-device handle
 * returns HR_E_UNSUPPORTED (use hr_index_search). */
int hr_index_search_submit_host(hr_index* h, const float* q, int B, int k, int notify_fd, int64_t* ticket_out);
int hr_index_search_collect(hr_index* h, int64_t ticket, float* scores_out, int64_t* rows_out);
/* State of a submitted batch without waiting: *state_out = 0 still running, 1 results ready, 2 ready but some
 * queries need the exact fallback (collect then runs a corpus pass: call it off the event loop).  HR_E_BUSY
 * while another call holds the handle. */
int hr_index_search_poll(hr_index* h, int64_t ticket, int* state_out);
int hr_index_size(hr_index* h, int64_t* n_out, int64_t* n_live_out);
/* Shape of a handle (e.g. one returned by hr_index_load): dim, storage dtype, metric, devices. */
int hr_index_info(hr_index* h, int* dim_out, int* dtype_out, int* metric_out, int* n_dev_out);
int hr_index_get_rows(hr_index* h, const int64_t* rows, int64_t n, float* out);
int hr_index_save(hr_index* h, const char* path);
int hr_index_load(const char* path, int n_dev, const int* dev_ids, hr_index** out);
void hr_index_destroy(hr_index* h);

/* Row-sharded search pieces (one process per GPU; RCCL moves the candidates).
 * Candidate record = {double exact_score; int64 global_row} (16 bytes).
 * kc = candidates per query kept by a shard (k <= kc <= HR_MAX_KC); the scan keeps
 * ceil(kc/32) row parts of group maxima.  hr_kc_for_k gives the kc the single-GPU search
 * uses below 2048 dims: k + max(16, k/2) rounded up to a multiple of 32, at most HR_MAX_KC (margin
 * for the guard; 32 for k <= 16).  hr_kc_for_k_dim(k, dim) is the kc for a given dim (the margin
 * grows to max(20, k) from 2048 dims on); hr_kc_for_k(k) = hr_kc_for_k_dim(k, 0). */
int hr_kc_for_k(int k);
int hr_kc_for_k_dim(int k, int dim);
int hr_index_search_shard(hr_index* h, const float* q_dev, int B, int k, int kc, const uint64_t* row_mask_dev,
                          int64_t row_offset, void* cand_out_dev /* B*kc records */,
                          double* bound_out_dev /* B */, void* stream);
/* Pipelined form of hr_index_search_shard: the scan (query prep, SAMPLE, FILTER) runs on
 * scan_stream over all but a few CUs, select + exact rescoring on tail_stream, which waits for
 * the scan by event; the outputs are ready in tail_stream order.  Consecutive calls alternate
 * between two workspaces, so batch i's tail (and whatever the caller queues after it on
 * tail_stream: the all-gather, the merge) overlaps batch i+1's scan.  Everything the caller
 * enqueued on scan_stream before the call is ordered before the tail-stream work (the tail waits
 * for this batch's scan), so outputs written on scan_stream earlier need no extra sync.  Same
 * results as hr_index_search_shard. */
int hr_index_search_shard_async(hr_index* h, const float* q_dev, int B, int k, int kc, const uint64_t* row_mask_dev,
                                int64_t row_offset, void* cand_out_dev, double* bound_out_dev, void* scan_stream,
                                void* tail_stream);
/* Same, with the event (hipEvent_t, nullable) after which the caller's queries q_dev are ready.
 * With it, a large shard's query prep and SAMPLE pass run early, on the index's own stream over
 * the CUs the previous batch's FILTER scan leaves free, instead of between the two FILTER scans
 * on scan_stream (results identical; only the order of work changes).  Without it: as above. */
int hr_index_search_shard_async_ev(hr_index* h, const float* q_dev, int B, int k, int kc,
                                   const uint64_t* row_mask_dev, int64_t row_offset, void* cand_out_dev,
                                   double* bound_out_dev, void* scan_stream, void* tail_stream,
                                   void* q_ready_event);
int hr_index_search_shard_collect(hr_index* h, const float* q_dev, int B, const double* kth_dev /* B */,
                                  int cap, const uint64_t* row_mask_dev, int64_t row_offset,
                                  void* cand_out_dev /* B*cap records */, double* bound_out_dev, void* stream);
int hr_merge_candidates(int device, const void* cand_dev /* G*B*kc records */, const double* bounds_dev /* G*B */,
                        int G, int B, int kc, int k, float* scores_out_dev, int64_t* rows_out_dev,
                        double* kth_out_dev, int32_t* fail_out_dev, void* stream);
/* The same with explicit per-rank strides (bytes) between the ranks' candidate blocks and bound
 * blocks, so one all-gather can move each rank's packed record [B*kc candidates][B bounds]
 * (cand_rank_stride = bound_rank_stride = B*kc*16 + B*8). */
int hr_merge_candidates_strided(int device, const void* cand_dev, const double* bounds_dev, int64_t cand_rank_stride,
                                int64_t bound_rank_stride, int G, int B, int kc, int k, float* scores_out_dev,
                                int64_t* rows_out_dev, double* kth_out_dev, int32_t* fail_out_dev, void* stream);

/* Exact top-m of every query over the whole shard (the exhaustive pass: canonical fp64 score of every live, allowed
 * row + a stable sort), as B*m candidate records {score, local row + row_offset} on the device in (score desc, row
 * asc) order, (-inf, -1) padding past the shard's rows.  The row-sharded search's path for k above the scan's kc and
 * for collect windows larger than their buffer -- the single index's hr_index_search k > HR_MAX_K pass, per shard
 * (Chroma's n_results has no cap, chroma_store.py:118-120; FAISS returns the exact top-k on ties,
 * faiss_store.py:148-176).  One corpus pass and one n-row sort per query; synchronises `stream`. */
int hr_index_search_shard_exact(hr_index* h, const float* q_dev, int B, int m, const uint64_t* row_mask_dev,
                                int64_t row_offset, void* cand_out_dev, void* stream);
/* Merge of G ranks' sorted exact lists (hr_index_search_shard_exact records, m per query; rank g's block at
 * cand_dev + g * cand_rank_stride bytes, 0 = dense B*m*16) into the top-k (score desc, row asc; -inf / -1 padding).
 * Any G * m (hr_merge_candidates is bounded by its LDS to G * kc <= 8192); ranks' rows must be disjoint. */
int hr_merge_sorted(int device, const void* cand_dev, int64_t cand_rank_stride, int G, int B, int m, int k,
                    float* scores_out_dev, int64_t* rows_out_dev, void* stream);

/* IVF-flat lists search (BASELINE config 5 candidate generation): h holds
 * the rows in list order (list l = tiles [list_tiles_dev[l], list_tiles_dev[l+1]) of 32 rows, pad
 * rows dead), ids_dev the original id of every position (-1 for pads), centroids_dev the nlist
 * processed fp32 centroids (row stride = dim rounded up to 64, zero padded).  Per query: exact top-
 * nprobe lists by canonical fp64 score (ties: lower list first), then the exact top-k of the rows of
 * those lists by canonical score (ties: lower id first), as B*k candidate records (global ids,
 * (-inf, -1) padding) and bound = -inf (nothing unreturned can matter: the same merge as the exact
 * search combines shards).  max_list_tiles: tiles of the largest list (sizes the unit buffer).
 * probes_out_dev (nullable): the B*nprobe probed lists as records {score, list}.  Cosine / dot. */
int hr_ivf_search(hr_index* h, const float* centroids_dev, int nlist, const int64_t* list_tiles_dev,
                  int64_t max_list_tiles, const int64_t* ids_dev, const float* q_dev, int B, int nprobe, int k,
                  const uint64_t* row_mask_dev, void* cand_out_dev, double* bound_out_dev, void* probes_out_dev,
                  void* stream);

/* Exact top-m of B segments of {double score; int64 id} records, order (score desc, id asc), records
 * with id < 0 absent; segment b = [seg_off_records_dev[b], seg_off_records_dev[b+1]) if given, else
 * [b*seg_stride, (b+1)*seg_stride).  Out: B*m records, (-inf, -1) padding; m <= 1024.  The
 * reranker's per-query selection (replaces the reranking service's sort + top_n, openai_reranker.py
 * :92-110 / the /rerank response order). */
int hr_topk_records(const void* in_dev, const int64_t* seg_off_records_dev, int64_t seg_stride, int B, int m,
                    void* out_dev, void* stream);

/* K7: masked mean-pool of the first-dim hidden states with the first n_instr
 * tokens of every sequence masked out, then L2-normalise (fp32 out, B×H). */
int hr_pool_normalize(const void* hidden_dev, int dtype, const int32_t* mask_dev, int B, int T, int H, int n_instr,
                      float* out_dev, void* stream);
/* K7 over packed (unpadded) hidden states: sequence b is rows [cu[b], cu[b+1]) of an N x H matrix (real
 * tokens only, cu: B+1 int32 offsets on the device); same mask rule (first n_instr tokens out), same
 * sums as hr_pool_normalize on the right-padded batch.  The in-process embedder's unpadded forward. */
int hr_pool_normalize_packed(const void* hidden_dev, int dtype, const int32_t* cu_dev, int B, int H, int n_instr,
                             float* out_dev, void* stream);
/* Host (no GPU): the offline tokenizer's word split + crc32 word hash over n_texts ASCII texts (bytes
 * [offsets[i], offsets[i+1]) of `text`): lower-cased \w+ | [^\w\s] tokens -> first_id + crc32 % span,
 * at most `cap` per text (cap < 0: all), wrapped in cls_id ... sep_id when both are >= 0.  ids_out
 * (capacity ids_cap) receives the texts' ids back to back, lengths_out[i] each text's count.
 * HR_E_INVALID for a non-ASCII byte or a full ids_out.  (hiprag.rag.rocm_embedder.HashWordTokenizer) */
int hr_hash_words(const char* text, const int64_t* offsets, int64_t n_texts, int64_t first_id, int64_t span, int64_t cap,
                  int64_t cls_id, int64_t sep_id, int64_t* ids_out, int64_t ids_cap, int64_t* lengths_out);
/* K8: out = LayerNorm(x + r) * gamma + beta over rows x H (H <= 4096), dtype of x, r, gamma, beta and
 * out (HR_F32 / HR_BF16 / HR_F16); the encoder layers' residual add + LayerNorm fused
 * (BertSelfOutput / BertOutput, modeling_bert.py; XLM-R the same).  Ordered on `stream`. */
int hr_add_layernorm(const void* x_dev, const void* r_dev, const void* gamma_dev, const void* beta_dev, void* out_dev,
                     int64_t rows, int H, float eps, int dtype, void* stream);

/* The query embedder's short-sequence attention (hr_attn.hip): for each sequence b (tokens [cu[b], cu[b+1]) of the
 * packed batch, cu: B+1 int32 on the device) and head h, softmax(scale * Q K^T) V over the sequence's own tokens, from
 * the fused QKV projection qkv_dev [N][3][nH][d] (row stride 3 nH d) into out_dev [N][nH][d]: Q K^T and P V on MFMA
 * with fp32 accumulation, the softmax in fp32, P rounded to the input type for the P V product (as the flash
 * kernel), the output rounded once.  BertSelfAttention (modeling_bert.py) on the real tokens, as
 * scaled_dot_product_attention per sequence.  HR_E_UNSUPPORTED outside its scope (d != 64, max_len > 64, fp32,
 * rows not 16-byte aligned): the caller's flash varlen kernel serves those. */
int hr_attn_varlen(const void* qkv_dev, int dtype, const int32_t* cu_dev, int B, int nH, int d, int max_len,
                   float scale, void* out_dev, void* stream);
/* In place: x = 0.5 x (1 + erf(x / sqrt 2)) (BertIntermediate's "gelu", torch.nn.functional.gelu with
 * approximate='none'; fp32 per element, rounded once), n elements of bf16 / f16. */
int hr_gelu_erf(void* x_dev, int dtype, int64_t n, void* stream);

/* The persistent FILTER (pipelined shard batches of <= 64 queries, k <= 16, no mask, early SAMPLE: the per-GPU
 * step of a row-sharded node).  One long-lived launch streams the corpus batch after batch -- no per-batch launch
 * ramp and tail; replaces the per-batch FILTER launch behind hr_index_search_shard_async_ev (same results).
 * set_persist: 0 off, 1 shards of 4.2M-5.1M rows (default: where it measured faster than per-batch launches),
 * 2 every shard size.  persist_close: no further batch
 * for now (the running instance exits once through its batches instead of after its 300 us idle timeout).  (Its
 * counters and stamps: hr_index_persist_stats / _trace, include/hiprag_diag.h.) */
int hr_index_set_persist(hr_index* h, int mode);
int hr_index_persist_close(hr_index* h);
/* CU partitioning (no reference counterpart: the reference's embedder and store are separate services, here the
 * query embedder's forward and the scan share one GPU -- base_retriever.py:57-63 embed_query -> search).
 * set_cu_mask: this index's internal streams run on the CUs of `mask` only (bit i of word j = CU 32 j + i;
 * n_words = 0: all CUs) and its launch grids are sized for that many CUs; blocks while asynchronous batches are
 * in flight (HR_E_BUSY).  stream_create_cu_mask: a stream restricted the same way (the caller's scan / tail /
 * embedder streams), released with hr_stream_destroy. */
int hr_index_set_cu_mask(hr_index* h, const uint32_t* mask, int n_words);
int hr_stream_create_cu_mask(int device, const uint32_t* mask, int n_words, void** stream_out);
/* Waits for the work queued on the stream, then destroys it.  Nothing may use the stream afterwards -- including a
 * framework that remembers it: PyTorch's pinned-host allocator records every stream a non_blocking copy to or from a
 * pinned tensor ran on, and touches those streams again when that tensor is freed, so such tensors must be freed
 * before the stream is destroyed (hiprag's own code copies through hr_memcpy_async instead). */
int hr_stream_destroy(void* stream);
/* Asynchronous copy of `bytes` bytes on `stream` (direction from the pointers: unified addressing). */
int hr_memcpy_async(void* dst, const void* src, int64_t bytes, void* stream);
int hr_device_count(int* n_out);
/* Cumulative counters since creation (the store's metrics) -- out[0] main scan passes, out[1] queries that
 * failed the exactness guard (collect fallback), out[2] queries answered by the exhaustive pass. */
int hr_index_stats(hr_index* h, int64_t out[3]);
/* The 256-query FILTER (hr_q256.hip: 129-256-query batches, bf16 / f16 / fp32 rows, D = 256..1024, k <= 16, no
 * tile list -- one corpus pass for four 64-query groups, VectorRetriever.batch_retrieve / the store's micro-batches of
 * up to 256 single-query calls, base_retriever.py:96-98, chroma_store.py:118-120).  set_q256(h, 0) sends those
 * batches to two 128-query FILTER launches instead (A/B; hr_index_q256_launches in include/hiprag_diag.h counts
 * its launches). */
int hr_index_set_q256(hr_index* h, int on);
const char* hr_last_error(void);
int hr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* HIPRAG_H */
