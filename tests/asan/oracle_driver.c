/* ASan/UBSan driver for the C oracle (oracle/cm_oracle.c, test infrastructure): a seeded random
 * corpus through every entry point -- CSR build, idf, BM25 top-k (k above the corpus size,
 * duplicate / unknown query terms, empty queries, a filter mask) and the exact fp64 dense top-k --
 * with invariant checks (ranges, ordering). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int orc_bm25_idf(int32_t vocab, const int64_t *df, const uint64_t *first_key, int64_t n_docs, double *idf_out,
                 double *eps_out);
int orc_bm25_csr_topk(int32_t vocab, const int64_t *term_off, const int32_t *post_doc, const uint16_t *post_tf,
                      int64_t ndocs, const int32_t *dl, const uint8_t *allow, const double *idf, double avgdl,
                      int32_t nq, const int32_t *q_terms, const int32_t *q_off, int32_t k, double *out_score,
                      int64_t *out_row);
int64_t orc_count_postings(const int32_t *term_ids, const int64_t *doc_off, int64_t ndocs, int32_t vocab);
int orc_build_csr(const int32_t *term_ids, const int64_t *doc_off, int64_t ndocs, int32_t vocab, int64_t *term_off,
                  int32_t *post_doc, uint16_t *post_tf, int32_t *dl, int64_t *df, uint64_t *first_key);
int orc_dense_topk_f64(int64_t n, int32_t dim, const float *C, int32_t nq, const float *Q, int32_t k,
                       double *out_dist, int64_t *out_row);

static uint64_t rs = 88172645463325252ull;
static uint32_t rnd(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (uint32_t)rs;
}

int main(void) {
  const int64_t nd = 3000;
  const int32_t V = 500, D = 24, K = 4000;
  int64_t *doc_off = malloc((nd + 1) * sizeof(int64_t));
  doc_off[0] = 0;
  for (int64_t d = 0; d < nd; ++d) doc_off[d + 1] = doc_off[d] + 1 + rnd() % 40;
  const int64_t nt = doc_off[nd];
  int32_t *toks = malloc(nt * sizeof(int32_t));
  for (int64_t i = 0; i < nt; ++i) toks[i] = (int32_t)((rnd() % V) * (rnd() % V) / V);
  const int64_t np = orc_count_postings(toks, doc_off, nd, V);
  int64_t *term_off = malloc((V + 1) * sizeof(int64_t));
  int32_t *post_doc = malloc(np * sizeof(int32_t));
  uint16_t *post_tf = malloc(np * sizeof(uint16_t));
  int32_t *dl = malloc(nd * sizeof(int32_t));
  uint64_t *first = malloc(V * sizeof(uint64_t));
  int64_t *df = malloc(V * sizeof(int64_t));
  int bad = 0;
  if (orc_build_csr(toks, doc_off, nd, V, term_off, post_doc, post_tf, dl, df, first)) ++bad;
  for (int t = 0; t < V; ++t)
    if (df[t] != term_off[t + 1] - term_off[t]) ++bad;
  double *idf = malloc(V * sizeof(double)), eps = 0;
  if (orc_bm25_idf(V, df, first, nd, idf, &eps)) ++bad;
  int64_t sl = 0;
  for (int64_t d = 0; d < nd; ++d) sl += dl[d];
  const int32_t nq = 5;
  int32_t q_terms[] = {1, 2, 3, 1, V - 1, -1, 7, 7, 7};
  int32_t q_off[] = {0, 3, 4, 6, 6, 9};          /* dupes, a -1 term, an empty query */
  uint8_t *allow = malloc(nd);
  for (int64_t d = 0; d < nd; ++d) allow[d] = rnd() & 1;
  double *sc = malloc((size_t)nq * K * sizeof(double));
  int64_t *rw = malloc((size_t)nq * K * sizeof(int64_t));
  for (int pass = 0; pass < 2; ++pass) {
    if (orc_bm25_csr_topk(V, term_off, post_doc, post_tf, nd, dl, pass ? allow : NULL, idf, (double)sl / nd, nq,
                          q_terms, q_off, K, sc, rw))
      ++bad;
    for (int q = 0; q < nq; ++q)
      for (int j = 0; j < K; ++j) {
        const int64_t r = rw[(int64_t)q * K + j];
        if (r < -1 || r >= nd) ++bad;
        if (j && r >= 0 && rw[(int64_t)q * K + j - 1] >= 0 && sc[(int64_t)q * K + j] > sc[(int64_t)q * K + j - 1]) ++bad;
      }
  }
  float *C = malloc((size_t)nd * D * sizeof(float)), Q[3 * 24];
  for (int64_t i = 0; i < nd * D; ++i) C[i] = (float)((int)(rnd() % 2001) - 1000) / 1000.f;
  for (int i = 0; i < 3 * D; ++i) Q[i] = (float)((int)(rnd() % 2001) - 1000) / 1000.f;
  double *dd = malloc(3 * 64 * sizeof(double));
  int64_t *dr = malloc(3 * 64 * sizeof(int64_t));
  if (orc_dense_topk_f64(nd, D, C, 3, Q, 64, dd, dr)) ++bad;
  for (int q = 0; q < 3; ++q)
    for (int j = 1; j < 64; ++j)
      if (dd[q * 64 + j] < dd[q * 64 + j - 1] || dr[q * 64 + j] < 0 || dr[q * 64 + j] >= nd) ++bad;
  free(doc_off); free(toks); free(term_off); free(post_doc); free(post_tf); free(dl); free(first);
  free(df); free(idf); free(allow); free(sc); free(rw); free(C); free(dd); free(dr);
  if (bad) {
    fprintf(stderr, "%d invariant failures\n", bad);
    return 1;
  }
  printf("oracle under ASan/UBSan: OK\n");
  return 0;
}
