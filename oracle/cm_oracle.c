/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg).  Never linked into the product library.
 *
 * Plain-C restatement of the BM25 scoring CLASSMATE-RAG does through
 * rank_bm25.BM25Okapi (rag/retrieval/bm25.py:140-212; rank_bm25 0.2.x
 * k1=1.5, b=0.75, epsilon=0.25), for corpora too large for the Python oracle
 * (oracle/ref_semantics.py, which is pinned bit-for-bit to the reference
 * goldens; tests/test_oracle_c.py checks this file against it).
 *
 *   idf_t  = log(N - df_t + 0.5) - log(df_t + 0.5), negative -> eps,
 *   eps    = 0.25 * mean(idf) summed in first-occurrence (dict) order,
 *   K_d    = 1.5 * (0.25 + (0.75 * dl_d) / avgdl),
 *   score  = sum over query tokens (in order, duplicates too) of
 *            idf_q * (tf * 2.5 / (tf + K_d)),
 *   top-k  = stable sort by score descending (ties -> lower row), zero-score
 *            documents included (rank_bm25 scores every candidate).
 * Compiled with -ffp-contract=off so every operation rounds like numpy's.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

typedef struct {
  uint64_t key;
  int32_t t;
} fk_pair;

static int cmp_fk(const void *a, const void *b) {
  const fk_pair *x = (const fk_pair *)a, *y = (const fk_pair *)b;
  if (x->key < y->key) return -1;
  if (x->key > y->key) return 1;
  return 0;
}

/* idf table from df and first-occurrence keys (row << 32 | first position).
 * Returns 0, or -4 when the vocabulary is empty (ZeroDivisionError). */
int orc_bm25_idf(int32_t vocab, const int64_t *df, const uint64_t *first_key, int64_t n_docs, double *idf_out,
                 double *eps_out) {
  fk_pair *order = (fk_pair *)malloc(sizeof(fk_pair) * (size_t)(vocab > 0 ? vocab : 1));
  int32_t m = 0;
  for (int32_t t = 0; t < vocab; ++t) {
    idf_out[t] = 0.0;
    if (df[t] > 0) {
      order[m].key = first_key[t];
      order[m].t = t;
      ++m;
    }
  }
  if (m == 0) {
    free(order);
    return -4;
  }
  qsort(order, (size_t)m, sizeof(fk_pair), cmp_fk);
  double s = 0.0;
  for (int32_t i = 0; i < m; ++i) {
    const int32_t t = order[i].t;
    const double v = log((double)(n_docs - df[t]) + 0.5) - log((double)df[t] + 0.5);
    idf_out[t] = v;
    s = s + v;
  }
  const double eps = 0.25 * (s / (double)m);
  for (int32_t i = 0; i < m; ++i)
    if (idf_out[order[i].t] < 0) idf_out[order[i].t] = eps;
  *eps_out = eps;
  free(order);
  return 0;
}

/* better(a, b): (score desc, row asc) */
static inline int better(double sa, int64_t ra, double sb, int64_t rb) {
  return sa > sb || (sa == sb && ra < rb);
}

/* Score queries over a CSR index (postings sorted by doc within a term) and
 * return the top-k per query over all docs in [0, ndocs) with allow (nullable,
 * 1 byte per doc) set.  idf/avgdl are the statistics of that candidate set.  */
int orc_bm25_csr_topk(int32_t vocab, const int64_t *term_off, const int32_t *post_doc, const uint16_t *post_tf,
                      int64_t ndocs, const int32_t *dl, const uint8_t *allow, const double *idf, double avgdl,
                      int32_t nq, const int32_t *q_terms, const int32_t *q_off, int32_t k, double *out_score,
                      int64_t *out_row) {
  double *kd = (double *)malloc(sizeof(double) * (size_t)(ndocs > 0 ? ndocs : 1));
  for (int64_t d = 0; d < ndocs; ++d) {
    double t = 0.75 * (double)dl[d];
    t = t / avgdl;
    t = 0.25 + t;
    kd[d] = 1.5 * t;
  }
#pragma omp parallel
  {
    double *score = (double *)calloc((size_t)(ndocs > 0 ? ndocs : 1), sizeof(double));
    double *hs = (double *)malloc(sizeof(double) * (size_t)k);
    int64_t *hr = (int64_t *)malloc(sizeof(int64_t) * (size_t)k);
#pragma omp for schedule(dynamic, 1)
    for (int32_t qi = 0; qi < nq; ++qi) {
      memset(score, 0, sizeof(double) * (size_t)ndocs);
      for (int32_t i = q_off[qi]; i < q_off[qi + 1]; ++i) {
        const int32_t t = q_terms[i];
        if (t < 0 || t >= vocab) continue;
        const double w = idf[t];
        for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
          const int32_t d = post_doc[p];
          const double tf = (double)post_tf[p];
          const double num = tf * 2.5;
          const double den = tf + kd[d];
          score[d] = score[d] + w * (num / den);
        }
      }
      /* top-k by insertion into a sorted array (k small) */
      int32_t n = 0;
      for (int64_t d = 0; d < ndocs; ++d) {
        if (allow && !allow[d]) continue;
        const double s = score[d] + 0.0;
        if (n == k && !better(s, d, hs[n - 1], hr[n - 1])) continue;
        int32_t j = n < k ? n++ : k - 1;
        while (j > 0 && better(s, d, hs[j - 1], hr[j - 1])) {
          hs[j] = hs[j - 1];
          hr[j] = hr[j - 1];
          --j;
        }
        hs[j] = s;
        hr[j] = d;
      }
      for (int32_t j = 0; j < k; ++j) {
        out_score[(int64_t)qi * k + j] = j < n ? hs[j] : 0.0;
        out_row[(int64_t)qi * k + j] = j < n ? hr[j] : -1;
      }
    }
    free(score);
    free(hs);
    free(hr);
  }
  free(kd);
  return 0;
}

/* CSR (by term, docs ascending) from doc-major term ids; also dl and the
 * first-occurrence key per term.  Arrays sized by the caller: term_off
 * [vocab+1], post_doc/post_tf [npost] where npost = #distinct (doc, term).
 * Parallel over P contiguous document ranges of about equal token counts: each
 * range counts its postings per term, an exclusive prefix over the ranges (in
 * range order) gives every range its write position inside each term, so the
 * postings of a term stay in ascending document order -- the same arrays as a
 * sequential build (10M documents / 1.2 B tokens: one pass per range instead of
 * minutes on one core; the 10M parity test builds its own CSR with it). */
static int orc_parts(void) {
  const int p = orc_num_threads();
  return p < 1 ? 1 : (p > 64 ? 64 : p);
}

static void orc_split_docs(const int64_t *doc_off, int64_t ndocs, int P, int64_t *bnd) {
  const int64_t tot = doc_off[ndocs] - doc_off[0];
  bnd[0] = 0;
  for (int i = 1; i < P; ++i) {
    const int64_t target = doc_off[0] + tot / P * i;
    int64_t lo = bnd[i - 1], hi = ndocs;
    while (lo < hi) { /* first d with doc_off[d] >= target */
      const int64_t mid = lo + (hi - lo) / 2;
      if (doc_off[mid] < target) lo = mid + 1; else hi = mid;
    }
    bnd[i] = lo;
  }
  bnd[P] = ndocs;
}

int64_t orc_count_postings(const int32_t *term_ids, const int64_t *doc_off, int64_t ndocs, int32_t vocab) {
  const int P = orc_parts();
  int64_t bnd[65];
  orc_split_docs(doc_off, ndocs, P, bnd);
  int64_t np = 0;
#pragma omp parallel for schedule(static, 1) reduction(+ : np) num_threads(P)
  for (int i = 0; i < P; ++i) {
    int64_t *stamp = (int64_t *)malloc(sizeof(int64_t) * (size_t)(vocab > 0 ? vocab : 1));
    for (int32_t t = 0; t < vocab; ++t) stamp[t] = -1;
    for (int64_t d = bnd[i]; d < bnd[i + 1]; ++d)
      for (int64_t p = doc_off[d]; p < doc_off[d + 1]; ++p) {
        const int32_t t = term_ids[p];
        if (stamp[t] != d) {
          stamp[t] = d;
          ++np;
        }
      }
    free(stamp);
  }
  return np;
}

int orc_build_csr(const int32_t *term_ids, const int64_t *doc_off, int64_t ndocs, int32_t vocab, int64_t *term_off,
                  int32_t *post_doc, uint16_t *post_tf, int32_t *dl, int64_t *df, uint64_t *first_key) {
  const int P = orc_parts();
  const size_t V = (size_t)(vocab > 0 ? vocab : 1);
  int64_t bnd[65];
  orc_split_docs(doc_off, ndocs, P, bnd);
  int64_t *cnt = (int64_t *)malloc(sizeof(int64_t) * V * (size_t)P);   /* [range][term] */
  uint64_t *fk = (uint64_t *)malloc(sizeof(uint64_t) * V * (size_t)P);
  /* pass 1: per range, postings per term and the term's first (doc, position) in the range */
#pragma omp parallel for schedule(static, 1) num_threads(P)
  for (int i = 0; i < P; ++i) {
    int64_t *stamp = (int64_t *)malloc(sizeof(int64_t) * V);
    int64_t *c = cnt + (size_t)i * V;
    uint64_t *f = fk + (size_t)i * V;
    for (int32_t t = 0; t < vocab; ++t) {
      stamp[t] = -1;
      c[t] = 0;
      f[t] = ~0ull;
    }
    for (int64_t d = bnd[i]; d < bnd[i + 1]; ++d) {
      dl[d] = (int32_t)(doc_off[d + 1] - doc_off[d]);
      for (int64_t p = doc_off[d]; p < doc_off[d + 1]; ++p) {
        const int32_t t = term_ids[p];
        if (stamp[t] != d) {
          stamp[t] = d;
          if (c[t]++ == 0) f[t] = ((uint64_t)d << 32) | (uint64_t)(p - doc_off[d]);
        }
      }
    }
    free(stamp);
  }
  /* df, first key (the first range holding the term) and each range's offset inside the term */
#pragma omp parallel for schedule(static)
  for (int32_t t = 0; t < vocab; ++t) {
    int64_t s = 0;
    uint64_t first = ~0ull;
    for (int i = 0; i < P; ++i) {
      const int64_t c = cnt[(size_t)i * V + t];
      if (c && first == ~0ull) first = fk[(size_t)i * V + t];
      cnt[(size_t)i * V + t] = s;
      s += c;
    }
    df[t] = s;
    first_key[t] = first;
  }
  free(fk);
  term_off[0] = 0;
  for (int32_t t = 0; t < vocab; ++t) term_off[t + 1] = term_off[t] + df[t];
  /* pass 2: every range writes its documents' postings at its own positions */
#pragma omp parallel for schedule(static, 1) num_threads(P)
  for (int i = 0; i < P; ++i) {
    int64_t *stamp = (int64_t *)malloc(sizeof(int64_t) * V);
    int32_t *tfc = (int32_t *)malloc(sizeof(int32_t) * V);
    int64_t *pos = cnt + (size_t)i * V;
    int32_t *distinct = NULL;
    int64_t cap = 0;
    for (int32_t t = 0; t < vocab; ++t) stamp[t] = -1;
    for (int64_t d = bnd[i]; d < bnd[i + 1]; ++d) {
      const int64_t len = doc_off[d + 1] - doc_off[d];
      if (len > cap) {
        cap = len;
        distinct = (int32_t *)realloc(distinct, sizeof(int32_t) * (size_t)cap);
      }
      int64_t nd = 0;
      for (int64_t p = doc_off[d]; p < doc_off[d + 1]; ++p) {
        const int32_t t = term_ids[p];
        if (stamp[t] != d) {
          stamp[t] = d;
          tfc[t] = 0;
          distinct[nd++] = t;
        }
        tfc[t]++;
      }
      for (int64_t j = 0; j < nd; ++j) {
        const int32_t t = distinct[j];
        const int64_t q = term_off[t] + pos[t]++;
        post_doc[q] = (int32_t)d;
        post_tf[q] = (uint16_t)(tfc[t] > 65535 ? 65535 : tfc[t]);
      }
    }
    free(stamp);
    free(tfc);
    free(distinct);
  }
  free(cnt);
  return 0;
}

/* Exact fp64 cosine top-k (distance = 1 - q.c / (|q||c|)), ties -> lower row. */
int orc_dense_topk_f64(int64_t n, int32_t dim, const float *C, int32_t nq, const float *Q, int32_t k,
                       double *out_dist, int64_t *out_row) {
  double *cn = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < n; ++r) {
    double s = 0.0;
    for (int32_t j = 0; j < dim; ++j) s += (double)C[r * dim + j] * (double)C[r * dim + j];
    cn[r] = sqrt(s);
  }
#pragma omp parallel
  {
    double *hd = (double *)malloc(sizeof(double) * (size_t)k);
    int64_t *hr = (int64_t *)malloc(sizeof(int64_t) * (size_t)k);
#pragma omp for schedule(dynamic, 1)
    for (int32_t qi = 0; qi < nq; ++qi) {
      const float *q = Q + (int64_t)qi * dim;
      double qn = 0.0;
      for (int32_t j = 0; j < dim; ++j) qn += (double)q[j] * (double)q[j];
      qn = sqrt(qn);
      int32_t m = 0;
      for (int64_t r = 0; r < n; ++r) {
        double s = 0.0;
        for (int32_t j = 0; j < dim; ++j) s += (double)q[j] * (double)C[r * dim + j];
        const double dd = (qn > 0 && cn[r] > 0) ? 1.0 - s / qn / cn[r] : 1.0;
        if (m == k && !(dd < hd[m - 1])) continue;
        int32_t j = m < k ? m++ : k - 1;
        while (j > 0 && dd < hd[j - 1]) {
          hd[j] = hd[j - 1];
          hr[j] = hr[j - 1];
          --j;
        }
        hd[j] = dd;
        hr[j] = r;
      }
      for (int32_t j = 0; j < k; ++j) {
        out_dist[(int64_t)qi * k + j] = j < m ? hd[j] : 0.0;
        out_row[(int64_t)qi * k + j] = j < m ? hr[j] : -1;
      }
    }
    free(hd);
    free(hr);
  }
  free(cn);
  return 0;
}
