/*
 * classmate_hip.h — C ABI of libclassmate_hip.so, the MI355X (gfx950) hybrid
 * retrieval engine behind CLASSMATE-RAG's retrieval API.
 *
 * Plain C: pointers + sizes only, no C++/torch types.  Every entry point
 * names the reference interface it replaces (paths relative to the
 * taha-kms/CLASSMATE-RAG tree).  Conventions:
 *   - return 0 (CM_OK) on success, < 0 on error; cm_last_error() gives a
 *     thread-local message.  CM_EINVAL maps to Python ValueError (the
 *     reference's convention for length mismatches, e.g. bm25.py:152-153),
 *     CM_EZERODIV to ZeroDivisionError (rank_bm25 on an empty vocabulary,
 *     SURVEY.md §8a quirk Q7), everything else to RuntimeError.
 *   - "host" functions take caller-owned host arrays, run on the handle's
 *     own HIP stream and return after the results are copied back.
 *   - "_dev" functions take device pointers plus a hipStream_t (as void*;
 *     NULL = the null/default stream, which is torch's default stream too);
 *     they never allocate, never synchronise, and are safe to capture into a
 *     HIP graph.  Handles' private streams (host functions) are blocking, so
 *     they are ordered after work queued on the null stream.
 *   - rows are int64 row indices into the handle's storage; "-1" pads
 *     results that have fewer than k entries.
 *   - allow bitmaps: bit (r & 31) of word r >> 5 set => row r may be
 *     returned (a Chroma `where` / BM25 `_matches_filter` mask).
 */
#ifndef CLASSMATE_HIP_H
#define CLASSMATE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CM_OK 0
#define CM_EINVAL (-1)
#define CM_ENOMEM (-2)
#define CM_EDEVICE (-3)
#define CM_EZERODIV (-4)
#define CM_EUNSUPPORTED (-5)

#define CM_DTYPE_F32 0
#define CM_DTYPE_BF16 1
#define CM_DTYPE_F16 2
#define CM_DTYPE_I32 3
#define CM_DTYPE_I64 4

/* Library ------------------------------------------------------------- */
const char *cm_last_error(void);
int cm_version(void);
int cm_device_count(int *n);
/* A HIP stream restricted to the CUs whose bits are set in cu_mask (n_words
 * 32-bit words; bit i = CU i of the device's enumeration) -- for running a
 * latency-bound stage beside a bandwidth-bound one (bench.py --bm25-cus).
 * Not a reference interface: an engine-side scheduling helper. */
int cm_stream_create_cu_masked(int device, const uint32_t *cu_mask, int n_words, void **out_stream);
int cm_stream_destroy(void *stream);
/* largest k the fused top-k kernels accept (dense and BM25 _dev entries); the
 * host-array searches accept any k >= 1 (beyond it: full order + device sort). */
int cm_max_topk(void);

/* Dense cosine k-NN ---------------------------------------------------
 * Replaces ChromaVectorStore (rag/retrieval/vector_chroma.py:81-278) and
 * the chromadb/hnswlib server it talks to: the corpus lives in HBM as fp32
 * rows, search is exact brute-force cosine (distance = 1 - cos, the
 * `hnsw:space=cosine` metric set at vector_chroma.py:156).               */
typedef struct cm_dense cm_dense;

/* ChromaVectorStore.__init__/_ensure_collection (vector_chroma.py:81-164). */
int cm_dense_create(int device, int32_t dim, int64_t capacity, cm_dense **out);
void cm_dense_destroy(cm_dense *h);
int cm_dense_reserve(cm_dense *h, int64_t capacity);
/* Device bytes of the row arrays (fp32 rows, norms, live bits, f16 plane): now and the most ever
 * held at once, and how many growths went through host memory (cm_dense_set_growth decides when).
 * Not a reference interface (capacity planning for 288 GB). */
int cm_dense_mem_stats(cm_dense *h, int64_t *cur_bytes, int64_t *peak_bytes, int64_t *staged_growths);
/* Growth policy (no reference counterpart: Chroma grows its own collection).  0 = automatic: a
 * growth copies device to device when the new arrays fit in the free device memory next to the old
 * ones, else it stages the rows through host memory; 1 = a store above 1 GiB always stages (peak
 * device footprint = the final allocation, never old + new).  CM_EINVAL for other modes. */
int cm_dense_set_growth(cm_dense *h, int32_t mode);
/* ChromaVectorStore.upsert (vector_chroma.py:168-200): write n fp32 rows
 * (host, n x dim row-major) at the given row indices, marking them live.
 * Rows beyond the current size grow the store. */
int cm_dense_upsert(cm_dense *h, const float *vecs, const int64_t *rows, int64_t n);
/* device variant: n contiguous rows starting at row0 from a device buffer. */
int cm_dense_upsert_dev(cm_dense *h, const float *vecs_dev, int64_t row0, int64_t n, void *stream);
/* col.delete (vector_chroma.py:181-187): clear the live bit of rows. */
int cm_dense_delete(cm_dense *h, const int64_t *rows, int64_t n);
/* ChromaVectorStore.reset_collection (vector_chroma.py:262-269). */
int cm_dense_reset(cm_dense *h);
/* ChromaVectorStore.count (vector_chroma.py:255-260). */
int64_t cm_dense_live_count(cm_dense *h);
int64_t cm_dense_size(cm_dense *h); /* high-water row count */
int32_t cm_dense_dim(cm_dense *h);
/* ChromaVectorStore.query (vector_chroma.py:204-253), batched: for each of
 * nq queries (host, nq x dim) return the k nearest live+allowed rows in
 * ascending (distance, row) order.  out_dist/out_row: nq x k.  out_vec
 * (nullable): nq x k x dim, the stored embeddings (include_embeddings).
 * allow_bits (nullable, host or device memory -- e.g. cm_filter_eval's
 * output, complete before the call): ceil(size/32) words.               */
int cm_dense_search(cm_dense *h, const float *q, int32_t nq, int32_t k, const uint32_t *allow_bits,
                    float *out_dist, int64_t *out_row, float *out_vec);
/* workspace bytes cm_dense_search_dev needs for (nq, k). */
int64_t cm_dense_search_workspace(cm_dense *h, int32_t nq, int32_t k);
/* which scan kernel cm_dense_search[_dev] runs for (nq, k): CM_DENSE_F32
 * (K1, fp32 MFMA, reads 4 B/element: k > 32, other dims, small corpora),
 * CM_DENSE_COARSE (K1c, f16 plane, 2 B/element, 256-query resident passes,
 * certified exact re-rank), CM_DENSE_STREAM (K1s, f16 plane, 2 B/element,
 * nq <= 32, per-wave HBM streams, same re-rank), CM_DENSE_Q8 (K1q, int8 plane
 * with per-row scales, 1 B/element, 256-query resident passes, per-row
 * certified exact re-rank; the automatic choice at dim 768 for nq > 32, unless
 * $CM_DENSE_Q8=0, which keeps K1c / K1s), CM_DENSE_Q8S (below); -1 on error.  Lets callers price the launch against the
 * right roofline.  CM_DENSE_F16X3 (the retired split-plane K1b) is accepted by
 * cm_dense_set_path and means automatic.  */
#define CM_DENSE_F32 1
#define CM_DENSE_F16X3 2
#define CM_DENSE_COARSE 3
#define CM_DENSE_STREAM 4
#define CM_DENSE_Q8 5
/* K1q-s: the int8 plane streamed per wave (register ring, no LDS) for nq <= 32,
 * the same certified re-rank as K1q; the automatic choice at dim 768 for nq <= 32
 * (unless $CM_DENSE_Q8=0, which keeps K1s) */
#define CM_DENSE_Q8S 6
int32_t cm_dense_search_kind(cm_dense *h, int32_t nq, int32_t k);
/* force a scan kernel for this handle (0 = automatic; an ineligible forced
 * kind falls back to the automatic choice).  Results agree within the 1e-4
 * distance tolerance on every path; used for A/B probes and parity tests. */
int cm_dense_set_path(cm_dense *h, int32_t kind);
/* K1c/K1s: number of queries of the search that last used `workspace_dev` whose
 * certificate failed and that were re-run by the exact fp32 pass
 * (synchronous read; 0 for other paths, -1 on error).                    */
int32_t cm_dense_workspace_fallbacks(cm_dense *h, int32_t nq, int32_t k, const void *workspace_dev);
/* same, for the last host-array cm_dense_search on this handle. */
int32_t cm_dense_last_fallbacks(cm_dense *h);
/* K1q/K1q-s: queries of that search whose band overflowed the re-rank's LDS
 * (near-duplicate clusters) and that the wide re-rank finished exactly from
 * the complete candidate buffers instead of the exact scan of every row
 * (ChromaVectorStore.query's result for them is unchanged,
 * rag/retrieval/vector_chroma.py:204-253); 0 for other paths, -1 on error. */
int32_t cm_dense_workspace_wide_reranks(cm_dense *h, int32_t nq, int32_t k, const void *workspace_dev);
int32_t cm_dense_last_wide_reranks(cm_dense *h);
/* kernel timing (bench roofline): while enabled, every search records HIP
 * events on its launch stream around its scan kernel (K1 / K1c / K1s coarse
 * scan); _drain synchronises on them, writes up to cap elapsed ms values and
 * returns how many were recorded (< 0 on error).                         */
int cm_dense_timing(cm_dense *h, int32_t enable);
/* cm_dense_set_seed_event: a hipEvent_t (NULL clears) recorded on the search stream right after K1q's
 * seed pass of every later batched search -- another stream can start work that should not compete
 * with the seed pass for CUs (bench.py --bm25-gate 2).  The caller keeps the event alive. */
int cm_dense_set_seed_event(cm_dense *h, void *event);
int32_t cm_dense_timing_drain(cm_dense *h, float *ms_out, int32_t cap);
int cm_dense_search_dev(cm_dense *h, const float *q_dev, int32_t nq, int32_t k, const uint32_t *allow_dev,
                        float *dist_dev, int64_t *row_dev, void *workspace_dev, int64_t workspace_bytes,
                        void *stream);
/* cm_dense_search_dev in two parts (same arguments, same stream order): the
 * scan + certified re-rank, then the exact fp32 pass for the queries whose
 * certificate failed (gated on the device: every workgroup leaves at once when
 * none did).  A caller enqueues the second part after its concurrent streams'
 * work has joined (ChromaVectorStore.query, vector_chroma.py:204-253, within
 * HybridRetriever.retrieve, fusion.py:124-125): the exact pass's workgroups ask
 * for ~150 KiB of LDS each and would otherwise wait behind the other stream's
 * kernels.  For CM_DENSE_F32 the first part is the whole search and the second
 * does nothing.  The deferred form also runs K1q with its shared LDS footprint
 * (131 KiB instead of 160: room for one BM25 block beside each scan workgroup);
 * results are identical either way.                                        */
int cm_dense_search_dev_deferred(cm_dense *h, const float *q_dev, int32_t nq, int32_t k, const uint32_t *allow_dev,
                                 float *dist_dev, int64_t *row_dev, void *workspace_dev, int64_t workspace_bytes,
                                 void *stream);
int cm_dense_exact_fallback_dev(cm_dense *h, const float *q_dev, int32_t nq, int32_t k, const uint32_t *allow_dev,
                                float *dist_dev, int64_t *row_dev, void *workspace_dev, int64_t workspace_bytes,
                                void *stream);
/* copy rows [row0, row0+n) to host (n x dim fp32) and/or their live bits
 * (row0 % 32 == 0; ceil(n/32) words).  Persistence and verification. */
int cm_dense_export(cm_dense *h, int64_t row0, int64_t n, float *out, uint32_t *live_out);
/* gather stored rows (row < 0 => zeros): out_dev n x dim. */
int cm_dense_gather_dev(cm_dense *h, const int64_t *rows_dev, int64_t n, float *out_dev, void *stream);
/* device pointer of the live bitmap (ceil(size/32) words) for callers that
 * AND their own filters on device. */
const uint32_t *cm_dense_live_bits_dev(cm_dense *h);

/* BM25 Okapi -------------------------------------------------------------
 * Replaces BM25Store's scoring (rag/retrieval/bm25.py:140-212) and the
 * rank_bm25.BM25Okapi it builds per search (k1=1.5, b=0.75, eps=0.25):
 * CSR postings by term in HBM, term-ordered fp64 accumulation, statistics
 * (N, avgdl, df, idf with the eps floor) over the filtered candidate set.  */
typedef struct cm_bm25 cm_bm25;

int cm_bm25_create(int device, cm_bm25 **out);
void cm_bm25_destroy(cm_bm25 *h);
/* BM25Store._rebuild / BM25Okapi.__init__ (bm25.py:140-145): build from
 * doc-major term ids (host): doc d's tokens are term_ids[doc_off[d] ..
 * doc_off[d+1]) in token order, term ids in [0, vocab).  live (nullable):
 * one byte per doc, 0 = tombstone (deleted, keeps insertion order of the
 * others).  Returns CM_EZERODIV when live docs exist but none has a token
 * (the reference raises ZeroDivisionError there). */
int cm_bm25_build(cm_bm25 *h, const int32_t *term_ids, const int64_t *doc_off, int64_t ndocs, int32_t vocab,
                  const uint8_t *live);
/* same from device arrays (K7: device CSR build by radix sort). */
int cm_bm25_build_dev(cm_bm25 *h, const int32_t *term_ids_dev, const int64_t *doc_off_dev, int64_t ndocs,
                      int64_t ntokens, int32_t vocab, void *stream);
int64_t cm_bm25_num_docs(cm_bm25 *h);
int64_t cm_bm25_num_postings(cm_bm25 *h);
/* unfiltered corpus statistics: live docs, total length, avgdl, eps. */
int cm_bm25_stats(cm_bm25 *h, int64_t *n_live, int64_t *sum_len, double *avgdl, double *eps);
/* Dense head-term tiles (K2 fast path): terms with df > ndocs * min_df_frac
 * (highest df first, at most max_bytes of uint8 tf tiles) are scored from a
 * [term][doc] tf tile instead of their postings.  Default 1/64 and 8 GiB;
 * max_bytes = 0 disables.  Results are identical either way. */
int cm_bm25_set_head_policy(cm_bm25 *h, double min_df_frac, int64_t max_bytes);
int32_t cm_bm25_num_head_terms(cm_bm25 *h);
/* Search strategy (results are identical on both):
 *   CM_BM25_FULL   K2 scores every (query, 1024-doc range) pair;
 *   CM_BM25_PRUNED K2a scores the documents holding a tail (non-head) query
 *                  term, then K2 re-scores only the (query, range) pairs whose
 *                  head-only score bound reaches the query's k-th best tail
 *                  score.  0 = automatic (pruned).          */
#define CM_BM25_FULL 1
#define CM_BM25_PRUNED 2
int cm_bm25_set_path(cm_bm25 *h, int32_t kind);
/* (query, range) pairs K2 re-scored by the pruned search that last used
 * `workspace_dev` (synchronous read; -1 on the full path or error), and the
 * same for the last host-array cm_bm25_search on this handle.            */
int32_t cm_bm25_workspace_rescored(cm_bm25 *h, int32_t nq, int32_t total_terms, int32_t k, const void *workspace_dev);
int32_t cm_bm25_last_rescored(cm_bm25 *h);
/* K2b's planned items of the pruned search that last used `workspace_dev` (synchronous read):
 * returns their count (-1 on the full path or error) and copies up to cap items (q << 40 |
 * 1024-doc range << 16 | 64-doc block mask) -- bench.py prices K2b's algorithmic bytes with them. */
int64_t cm_bm25_workspace_items(cm_bm25 *h, int32_t nq, int32_t total_terms, int32_t k, const void *workspace_dev,
                                uint64_t *items_out, int64_t cap);
/* the same items' planned 16-doc sub-blocks (bit 4 b + x = sub-block x of 64-doc block b of the
 * item's range; round 6: K2b scores only these) -- item i's mask is masks_out[i].  New: the planner
 * refines the reference-free block plan above, so no reference interface corresponds to it. */
int64_t cm_bm25_workspace_subblocks(cm_bm25 *h, int32_t nq, int32_t total_terms, int32_t k, const void *workspace_dev,
                                    uint64_t *masks_out, int64_t cap);
/* kernel timing (bench roofline): events around every search's K2 launch;
 * same contract as cm_dense_timing / cm_dense_timing_drain.              */
int cm_bm25_timing(cm_bm25 *h, int32_t enable);
int32_t cm_bm25_timing_drain(cm_bm25 *h, float *ms_out, int32_t cap);
/* the same for K2b (bm25_block_kernel) launches of the pruned search. */
int32_t cm_bm25_timing_drain_block(cm_bm25 *h, float *ms_out, int32_t cap);
/* Sharding support: local df per term and the first posting's
 * (row << 32 | first position) key (0xff..ff when absent), so ranks can
 * all-reduce df (sum) and first keys (min, after offsetting rows) and agree
 * on the reference's dict order; then install the global statistics. */
/* copy the device index to host (any pointer may be NULL): term_off[V+1],
 * post_doc/post_tf/post_pos[P], dl[N]. */
int cm_bm25_export(cm_bm25 *h, int64_t *term_off, int32_t *post_doc, uint16_t *post_tf, uint32_t *post_pos,
                   int32_t *dl);
int cm_bm25_term_stats(cm_bm25 *h, int32_t *df_out, uint64_t *first_out);
int cm_bm25_set_stats(cm_bm25 *h, const double *idf, int32_t vocab, int64_t n_live, int64_t sum_len, double eps);
/* BM25Store.search (bm25.py:175-212) batched: nq queries whose term ids
 * (host, -1 = unknown term) are q_terms[q_off[i] .. q_off[i+1]) in query
 * token order (duplicates count twice).  Candidates = live docs with the
 * allow bit set; statistics are recomputed over them when allow_bits is
 * given (quirk Q2).  Output per query: k (score, row) in descending score,
 * ties -> lower row, zero-score docs padding in row order (quirk Q1);
 * out_n[i] = number of valid entries (min(k, #candidates)).               */
int cm_bm25_search(cm_bm25 *h, const int32_t *q_terms, const int32_t *q_off, int32_t nq, int32_t k,
                   const uint32_t *allow_bits, double *out_score, int64_t *out_row, int32_t *out_n);
/* cm_bm25_search with the caller's statistics instead of this index's: q_idf[total] = every
 * query term's idf (0 for terms outside the candidate vocabulary; ignored for ids outside
 * [0, vocab)), avgdl and n_cand of the candidate set; allow_bits (host or device words,
 * nullable) restricts the scored documents.  A corpus sharded over several devices in one process
 * (classmate_hip/multidev.py, SURVEY §8(b) Threading / §8(e)) scores every shard with the GLOBAL
 * statistics -- for a where-filter the statistics of the filtered candidates of all shards (quirk
 * Q2, rag/retrieval/bm25.py:184-191) -- and merges the shards' lists by (score desc, row asc). */
int cm_bm25_search_idf(cm_bm25 *h, const int32_t *q_terms, const int32_t *q_off, int32_t nq, int32_t k,
                       const uint32_t *allow_bits, const double *q_idf, double avgdl, int64_t n_cand,
                       double *out_score, int64_t *out_row, int32_t *out_n);
/* unfiltered device variant (inputs and outputs device, graph-capturable). */
int64_t cm_bm25_search_workspace(cm_bm25 *h, int32_t nq, int32_t total_terms, int32_t k);
int cm_bm25_search_dev(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int32_t nq,
                       int32_t total_terms, int32_t k, double *score_dev, int64_t *row_dev,
                       void *workspace_dev, int64_t workspace_bytes, void *stream);
/* the same search with its scoring kernels behind gate_event (a hipEvent_t, NULL = none): the
 * query preparation (term descriptors, postings bounds, the seeded threshold) runs at once, beside
 * the caller's producer work (HybridRetriever.retrieve encodes the query first,
 * rag/retrieval/fusion.py:124-125), the tail pass and everything after it wait for the event.
 * Results are identical. */
int cm_bm25_search_dev_gated(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int32_t nq,
                             int32_t total_terms, int32_t k, double *score_dev, int64_t *row_dev,
                             void *workspace_dev, int64_t workspace_bytes, void *stream, void *gate_event);

/* Filtered search on the device (quirk Q2: rank_bm25 statistics over the
 * candidate set, rag/retrieval/bm25.py:184-191), graph-capturable.
 *   cm_bm25_prepare_filtered: host call, once per index (before capture):
 *     uploads L[x] = log(x + 0.5) for x <= max(max_docs, num_docs) (glibc,
 *     CPython's math.log), so the device forms idf = L[Nc - df] - L[df] with
 *     rank_bm25's exact bits.  max_docs = the global corpus size on a shard.
 *   cm_bm25_filter_stats_dev: stats_dev = {Nc, sum of candidate lengths}
 *     (int64[2]), df_dev[i] = candidate df of q_terms_dev[i] (int64).  A
 *     sharded index all-reduces (sums) both before searching.
 *   cm_bm25_filter_term_stats_dev: the same for every term (df int64[V]) plus
 *     each term's first candidate (row << 32 | position) key (uint64[V],
 *     ~0 = none): a shard's share of the epsilon floor's statistics.
 *   cm_bm25_filter_eps: host call; rank_bm25's epsilon (0.25 x the mean idf
 *     of the candidate vocabulary in first-occurrence order) for one filter;
 *     allow_bits host or device words.
 *   cm_bm25_search_stats_dev: cm_bm25_search_dev over the allowed documents
 *     with the given candidate statistics; eps_dev (nullable) is the epsilon
 *     used when an idf is negative.  status_dev (int32, written on stream):
 *     bit 0 an idf was negative and eps_dev was NULL/NaN (compute eps with
 *     cm_bm25_filter_eps and search again), bit 1 candidates without tokens
 *     (the reference's ZeroDivisionError), bit 2 Nc beyond the prepared table.
 *   cm_bm25_search_filtered_dev: filter_stats_dev + search_stats_dev on one
 *     index (workspace: cm_bm25_search_workspace).                          */
int cm_bm25_prepare_filtered(cm_bm25 *h, int64_t max_docs);
int cm_bm25_filter_stats_dev(cm_bm25 *h, const uint32_t *allow_dev, const int32_t *q_terms_dev, int32_t n_terms,
                             int64_t *stats_dev, int64_t *df_dev, void *stream);
int cm_bm25_filter_term_stats_dev(cm_bm25 *h, const uint32_t *allow_dev, int64_t *df_dev, uint64_t *first_dev,
                                  void *stream);
int cm_bm25_filter_eps(cm_bm25 *h, const uint32_t *allow_bits, double *eps_out);
int cm_bm25_search_stats_dev(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int32_t nq,
                             int32_t total_terms, int32_t k, const uint32_t *allow_dev, const int64_t *stats_dev,
                             const int64_t *df_dev, const double *eps_dev, double *score_dev, int64_t *row_dev,
                             int32_t *status_dev, void *workspace_dev, int64_t workspace_bytes, void *stream);
int cm_bm25_search_filtered_dev(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int32_t nq,
                                int32_t total_terms, int32_t k, const uint32_t *allow_dev, const double *eps_dev,
                                double *score_dev, int64_t *row_dev, int32_t *status_dev, void *workspace_dev,
                                int64_t workspace_bytes, void *stream);

/* Where-filters on the device ---------------------------
 * A where clause compiled on the host (classmate_hip/retrieval/filters.py,
 * replacing the per-row _matches_filter of rag/retrieval/bm25.py:79-107
 * and Chroma's where evaluation behind vector_chroma.py:45-78,204-253)
 * into a postfix program: n_ops triples (opcode, a, b) in prog (host).
 *   CM_FOP_EQ / CM_FOP_NE  push cols_dev[a][row] == b  /  != b
 *   CM_FOP_BITS            push bit row of bitmap bits_dev[a]
 *   CM_FOP_TRUE / FALSE    push a constant
 *   CM_FOP_AND / OR        pop two, push the result;  CM_FOP_NOT  negate top
 * cols_dev / bits_dev: host arrays of device pointers (int32 value codes,
 * n_rows each; uint32 bitmaps, ceil(n_rows/32) words).  out_dev receives
 * ceil(n_rows/32) words (bit r & 31 of word r >> 5); count_dev (nullable,
 * device) the number of set bits.  Stack depth <= 32; <= CM_FILTER_MAX_OPS
 * ops and <= CM_FILTER_MAX_SOURCES columns and bitmaps.  Async on stream. */
#define CM_FILTER_MAX_OPS 64
#define CM_FILTER_MAX_SOURCES 16
#define CM_FOP_EQ 1
#define CM_FOP_NE 2
#define CM_FOP_BITS 3
#define CM_FOP_TRUE 4
#define CM_FOP_FALSE 5
#define CM_FOP_AND 6
#define CM_FOP_OR 7
#define CM_FOP_NOT 8
int cm_filter_eval(const int32_t *prog, int32_t n_ops, const int32_t *const *cols_dev, int32_t n_cols,
                   const uint32_t *const *bits_dev, int32_t n_bits, int64_t n_rows, uint32_t *out_dev,
                   unsigned long long *count_dev, void *stream);

/* Fusion -------------------------------------------------------------- */
/* _mmr_order (rag/retrieval/fusion.py:39-61) for nq queries at once:
 * q: nq x dim, cands: nq x pool x dim (fp32), n_valid[i] <= pool rows valid
 * for query i.  out_order: nq x k indices into the pool (-1 pad).         */
int cm_mmr(const float *q, const float *cands, const int32_t *n_valid, int32_t nq, int32_t pool, int32_t dim,
           int32_t k, double lambd, int32_t *out_order);
int cm_mmr_dev(const float *q_dev, const float *cands_dev, const int32_t *n_valid_dev, int32_t nq, int32_t pool,
               int32_t dim, int32_t k, double lambd, int32_t *order_dev, void *stream);
/* rrf_fuse (rag/retrieval/fusion.py:17-36): nl rank lists of int64 keys
 * (host; list i = keys[off[i] .. off[i+1])).  out_keys/out_score receive
 * the distinct keys in first-appearance order (Python dict order) and
 * their fused scores; *out_n = count.  weights nullable (all 1.0).      */
int cm_rrf_fuse(const int64_t *keys, const int32_t *off, int32_t nl, const double *weights, int32_t rrf_k,
                int64_t *out_keys, double *out_score, int32_t *out_n);
/* HybridRetriever.retrieve merge (fusion.py:132-167), batched on device:
 * per query a vector list (<= kv keys with fp32 distance, MMR order) and a
 * BM25 list (<= kb keys with fp64 score); outputs the top_k items sorted by
 * (fused, -distance or -0.0) descending, stable (vector items first).
 * out_flags bit0 = has vector distance, bit1 = has BM25 score.           */
/* Inputs of cm_rrf_merge_dev from the device search outputs (fusion.py:132-153's vec_ids /
 * bm_ids lists): vkeys/vdist[q][i] = pool_keys/pool_dist[q][order[q][i]] for the MMR order
 * (-1 / 0 past the selected count), vn[q] = selected count, bn[q] = valid BM25 rows (>= 0).  */
int cm_rrf_pool_prep_dev(const int64_t *pool_keys, const float *pool_dist, int32_t pool, const int32_t *order,
                         int32_t kv, const int64_t *bkeys, int32_t kb, int32_t nq, int64_t *vkeys, float *vdist,
                         int32_t *vn, int32_t *bn, void *stream);
int cm_rrf_merge_dev(const int64_t *vkeys, const float *vdist, const int32_t *vn, int32_t kv,
                     const int64_t *bkeys, const double *bscore, const int32_t *bn, int32_t kb, int32_t nq,
                     double w_vec, double w_bm25, int32_t rrf_k, int32_t top_k, int64_t *out_keys,
                     double *out_fused, float *out_vdist, double *out_bscore, int32_t *out_flags,
                     int32_t *out_n, void *stream);
int cm_rrf_merge(const int64_t *vkeys, const float *vdist, const int32_t *vn, int32_t kv, const int64_t *bkeys,
                 const double *bscore, const int32_t *bn, int32_t kb, int32_t nq, double w_vec, double w_bm25,
                 int32_t rrf_k, int32_t top_k, int64_t *out_keys, double *out_fused, float *out_vdist,
                 double *out_bscore, int32_t *out_flags, int32_t *out_n);

/* E5 pooling ------------------------------------------------------------
 * sentence-transformers Pooling(mean) + Normalize as used by
 * E5MultilingualEmbedder.encode_* (rag/embeddings/__init__.py:85-105):
 * out[b] = sum_s h[b,s]*m[b,s] / max(sum_s m[b,s], 1e-9), then (if
 * normalize) out[b] /= max(||out[b]||_2, 1e-12).  hidden: B x S x D of
 * hidden_dtype (F32/BF16/F16), mask: B x S of mask_dtype (I32/I64),
 * out: B x D fp32.  All device pointers, torch's stream.                 */
int cm_meanpool_l2norm(const void *hidden_dev, int32_t hidden_dtype, const void *mask_dev, int32_t mask_dtype,
                       int32_t B, int32_t S, int32_t D, int32_t normalize, float *out_dev, void *stream);

/* E5 encoder block epilogue ----------------------------------------------
 * XLM-R "residual add + LayerNorm" (HF XLMRobertaSelfOutput / XLMRobertaOutput /
 * XLMRobertaEmbeddings, run by E5MultilingualEmbedder.encode_*,
 * rag/embeddings/__init__.py:85-105) fused into one pass:
 * out[i] = LN(round(x[i] + r[i % r_rows])) * gamma + beta over D features,
 * fp32 statistics.  r may be NULL (plain LayerNorm); out may alias x.
 * dtype F32 or BF16 for x, r, gamma, beta and out; rows x D row-major.  */
int cm_add_layernorm(const void *x_dev, const void *r_dev, int64_t r_rows, const void *gamma_dev,
                     const void *beta_dev, int64_t rows, int32_t D, float eps, int32_t dtype, void *out_dev,
                     void *stream);

/* Self-attention of an unpadded short batch (HF XLMRobertaSelfAttention with an all-ones
 * mask, as run by E5MultilingualEmbedder.encode_queries): qkv_dev is the fused Q/K/V
 * projection output B x S x 3 x H x head_dim, out_dev receives softmax(q k^T * scale) v as
 * B x S x (H * head_dim).  head_dim must be 64, 0 < S <= 64; dtype F32 or BF16.   */
int cm_short_attention(const void *qkv_dev, int32_t B, int32_t S, int32_t H, int32_t head_dim, float scale,
                       int32_t dtype, void *out_dev, void *stream);

/* fp32-accurate E5 projections on the f16 matrix cores (K10) ------------
 * The XLM-R linear layers y = x W^T + b that E5MultilingualEmbedder.encode_*
 * runs in fp32 (rag/embeddings/__init__.py:85-105, sentence-transformers on
 * torch fp32: nn.Linear in XLMRobertaSelfAttention / SelfOutput /
 * Intermediate / Output), computed as split-precision f16 products: every
 * fp32 operand v = hi + lo (two f16 halves, 22 significant bits), product =
 * lo.hi + hi.lo + hi.hi accumulated in fp32 by v_mfma_f32_16x16x32_f16.
 *
 * "Planes": an M x K fp32 matrix as ONE buffer of 2 KiB split blocks, block
 * (row / 16, k / 32) = [hi halves 1 KiB][lo halves 1 KiB], each in fragment-
 * major order (lane slot c + 16 g = row 16 b + c, k = 32 kb + 8 g .. + 7).
 * A buffer holds cm_f16x3_plane_rows(M) rows (M rounded up to 384, so the
 * GEMM's last tile reads in bounds) x K x 2 halves.  Values are stored times a
 * power-of-two scale with |v * scale| <= 2^15.
 *
 * cm_f16x3_split_rows: fp32 rows (device, M x K row-major) * scale -> planes.
 * cm_f16x3_split_weights: the same for an nn.Linear weight (N x K), once per
 *   model; scale puts max|W| at 2^14..2^15.  N % 16 == 0, K % 32 == 0.
 * cm_linear_f16x3: C = (A planes)(W planes)^T * out_scale + bias, where
 *   out_scale = 1 / (A scale * W scale), bias may be NULL (N <= 4096);
 *   epilogue CM_EPI_BIAS / CM_EPI_BIAS_GELU (exact erf, torch's F.gelu
 *   default) write c_dev (M x N fp32 row-major); CM_EPI_PLANES_GELU writes
 *   GELU(C) * next_scale as planes (c_planes, cm_f16x3_plane_rows(M) x N) for
 *   the next projection (FFN-up -> FFN-down).  K % 64 == 0, N % 64 == 0, any M.
 * cm_add_layernorm_split: cm_add_layernorm (fp32) that also writes its output
 *   rows * a_scale as planes.  D % 32 == 0.
 * cm_short_attention_split: cm_short_attention (fp32) writing the context
 *   * a_scale as planes (B*S x H*64) instead of fp32 rows.
 * cm_short_attention_split_masked: the same for padded batches (S <= 32):
 *   key_mask_dev (B x S int32, nonzero = attend) removes padded keys from
 *   the softmax, as XLM-R's extended attention mask (the reference's HF
 *   forward for a padded query batch, rag/embeddings/__init__.py:85-105).  */
#define CM_EPI_BIAS 0
#define CM_EPI_BIAS_GELU 1
#define CM_EPI_PLANES_GELU 2
/* CM_EPI_PLANES_QKV: the fused QKV projection (N = 3 x H x 64, N % 96 == 0, M > 32) written as planes
 * of C * next_scale for cm_planes_attention: the Q and K thirds in the standard layout, the V third
 * transposed per 32-row unit (the attention's P V operand; see cm_gemm.hip k10_epilogue). */
#define CM_EPI_PLANES_QKV 3
int64_t cm_f16x3_plane_rows(int64_t M);
int cm_f16x3_split_rows(const float *x_dev, int64_t M, int32_t K, float scale, void *planes_dev, void *stream);
int cm_f16x3_split_weights(const float *w_dev, int32_t N, int32_t K, float scale, void *planes_dev, void *stream);
int cm_linear_f16x3(const void *a_planes, int64_t M, int32_t K, const void *w_planes, const float *bias_dev,
                    float out_scale, int32_t N, int32_t epilogue, float *c_dev, float next_scale, void *c_planes,
                    void *stream);
int cm_add_layernorm_split(const float *x_dev, const float *r_dev, int64_t r_rows, const float *gamma_dev,
                           const float *beta_dev, int64_t rows, int32_t D, float eps, float *out_dev, float a_scale,
                           void *planes_dev, void *stream);
int cm_short_attention_split(const float *qkv_dev, int32_t B, int32_t S, int32_t H, int32_t head_dim, float scale,
                             float a_scale, void *planes_dev, void *stream);
int cm_short_attention_split_masked(const float *qkv_dev, int32_t B, int32_t S, int32_t H, int32_t head_dim,
                                    float scale, float a_scale, const int32_t *key_mask_dev, void *planes_dev,
                                    void *stream);
/* cm_long_attention_split: the same context planes for any 0 < S <= 4096 (passages; K9L, a
 * flash-style split-precision MFMA kernel: 64-key chunks through LDS, online softmax in fp32);
 * key_mask_dev (B x S int32, nonzero = attend) may be NULL (every key attends).  Replaces torch
 * SDPA + cm_f16x3_split_rows for the reference's passage encode (rag/embeddings/__init__.py:96-105,
 * truncation at 512 tokens). */
int cm_long_attention_split(const float *qkv_dev, int32_t B, int32_t S, int32_t H, int32_t head_dim, float scale,
                            float a_scale, const int32_t *key_mask_dev, void *planes_dev, void *stream);
/* cm_planes_attention: the same context planes from the CM_EPI_PLANES_QKV output of the QKV
 * projection (qkv_planes = planes of (B*S) x 3*H*64 values times s_qkv, a power of two): K9P, every
 * operand streamed as split blocks by LDS-DMA (the passage encode, S % 64 == 0, S <= 512; the
 * caller pads other lengths with masked keys). */
int cm_planes_attention(const void *qkv_planes, int32_t B, int32_t S, int32_t H, int32_t head_dim, float scale,
                        float s_qkv, float a_scale, const int32_t *key_mask_dev, void *planes_dev, void *stream);

/* The N > 1 step's exchange merge (no reference interface: the reference is single
 * process -- this is the sharded form of ChromaVectorStore.query, vector_chroma.py:204-253, and
 * BM25Store.search's sorted(...)[:top_k], bm25.py:199).  allp_dev: the all-gathered packed shard
 * lists, ws x B x (2P + 2K) int64 (P f32 distance words, P global rows, K f64 score words, K global
 * rows; -1 rows pad).  Writes the global dense top-P (distance asc, row asc) and BM25 top-K
 * (score desc, row asc, -0.0 == 0.0), pads last; device pointers, stream-ordered, no sync.
 * ws x P and ws x K <= 4096. */
int cm_shard_merge_topk_dev(const int64_t *allp_dev, int32_t ws, int32_t B, int32_t P, int32_t K, float *d_out,
                            int64_t *r_out, double *s_out, int64_t *br_out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CLASSMATE_HIP_H */
