// BM25 Okapi over HBM-resident postings (replaces BM25Store.search,
// rag/retrieval/bm25.py:175-212, and rank_bm25.BM25Okapi it rebuilds per query).
// See DESIGN.md §K2/K3/K7.
//
// Exactness contract (bit-identical fp64 scores to rank_bm25 0.2.x):
//   contribution(q, d) = idf_q * ((tf*2.5) / (tf + K_d)),
//   K_d = 1.5 * (0.25 + (0.75*dl_d) / avgdl)        [numpy op order, no FMA]
//   score_d = sum over query tokens in order, duplicates included.
// This file is compiled with -ffp-contract=off.  idf values are computed on
// the host with glibc log() (the same libm call CPython's math.log makes),
// including the epsilon floor whose average is summed in the reference's
// dict (first-occurrence) order.
//
// Layout in HBM (per handle): CSR by term, postings sorted by doc row:
//   term_off [V+1] i64, post_doc [P] i32, post_tf [P] u16, post_pos [P] u32
//   (first position of the term in the doc: orders terms by first occurrence),
//   dl [N] i32, live [ceil(N/32)] u32, idf [V] f64 (unfiltered statistics).
//
// Search (K2): grid = (doc ranges of R rows) x (query groups).  A workgroup
// stages K_d for its range in LDS (fp64), then for each query of its group
// accumulates term contributions into an LDS fp64 score tile, term by term
// (barrier between terms keeps the reference's summation order), and selects
// the range's top-k (score desc, row asc) over *all* candidate rows — zero
// scores included, which reproduces the reference's zero-score padding.
// A tournament kernel merges the sorted per-range lists.
#include "cm_common.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <numeric>
#include <vector>

namespace cm {

constexpr int kRange = 1024;                 // docs per range (one wave's LDS score tile)
constexpr int kBmThreads = 256;              // 4 waves = 4 queries per K2 workgroup
constexpr int kBoundsGroup = 8;              // ranges per bounds thread (gallop between them)
constexpr int kMergeThreads = 1024;
constexpr int kMergePer = 16;                // lists per merge thread -> <= 16384 ranges (16.7M docs)
constexpr int kTermLanesQd = 16;             // K2b descriptor slots per query (== kTermLanes)

// Candidate lists, one per (query, range), k slots each: slot 0 of every list of query q lies
// contiguous at [q * nr + r] (the merge's first read of all lists is coalesced), slots 1..k-1 of
// a list contiguous after the heads, at nl + (q * nr + r) * (k - 1) + j - 1 (nl = nq * nr lists).
// A list holds its entries in slots 0..c-1 and, when c < k, the sentinel (kEmptyKey, ~0u) in slot
// c; slots past the sentinel are never written or read (most lists are empty: one 12-B write).
// (Heads in K2a wave order, [q / 4][r][q % 4], so that a wave writes whole lines, measured slower --
// 2.44 vs 2.38 ms per search -- and raised K2a's PMC WRITE_SIZE 0.29 -> 0.34 GB: the list writes
// that count are the entries, not the heads.)
__device__ inline int64_t lhead(int q, int64_t r, int64_t nr) { return (int64_t)q * nr + r; }
// entries of the head region (slots 1..k-1 follow it)
__host__ __device__ inline int64_t lheads_total(int nq, int64_t nr) { return (int64_t)nq * nr; }
__device__ inline int64_t lslot(int q, int64_t r, int64_t nr, int64_t nl, int k, int j) {
  return j == 0 ? lhead(q, r, nr) : nl + ((int64_t)q * nr + r) * (k - 1) + (j - 1);
}

struct PairKey {  // (k, r) lexicographic; smaller is better
  uint64_t k;
  uint32_t r;
};
__device__ inline bool pk_less(uint64_t ka, uint32_t ra, uint64_t kb, uint32_t rb) {
  return ka < kb || (ka == kb && ra < rb);
}

__device__ inline void wave_min_pair(uint64_t &key, uint32_t &row) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t ok = __shfl_xor(key, o);
    const uint32_t orr = __shfl_xor(row, o);
    if (pk_less(ok, orr, key, row)) {
      key = ok;
      row = orr;
    }
  }
}

// Block-wide argmin of (key,row); sk/sr hold one entry per wave. Returns in all threads.
__device__ inline PairKey block_min_pair(uint64_t key, uint32_t row, uint64_t *sk, uint32_t *sr) {
  wave_min_pair(key, row);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sk[w] = key;
    sr[w] = row;
  }
  __syncthreads();
  PairKey best{sk[0], sr[0]};
  const int nw = blockDim.x >> 6;
  for (int i = 1; i < nw; ++i)
    if (pk_less(sk[i], sr[i], best.k, best.r)) best = PairKey{sk[i], sr[i]};
  __syncthreads();
  return best;
}

__device__ inline uint64_t score_key(double s) {
  s = s + 0.0;  // -0.0 -> +0.0 (Python compares them equal)
  return ~f64_order(s);  // ascending key == descending score
}

// q_idf[i] = idf[t] for known terms, 0 otherwise (unfiltered statistics).
__global__ void bm25_qidf_kernel(const int32_t *__restrict__ q_terms, int n, const double *__restrict__ idf,
                                 int32_t vocab, double *__restrict__ q_idf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t t = q_terms[i];
  q_idf[i] = (t >= 0 && t < vocab) ? idf[t] : 0.0;
}

// bounds[i*(nr+1)+r] = first posting of term q_terms[i] with doc >= r*kRange.
// One thread per (term, group of kBoundsGroup ranges): binary search for the
// first range of the group, then gallop forward (bounds are monotone in r).
__device__ inline int64_t lower_bound_doc(const int32_t *__restrict__ post_doc, int64_t lo, int64_t hi, int32_t target) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (post_doc[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// qcand[i] = 1 iff query term i's postings are walked (K2's tail terms, K2a's candidate
// generators): every known non-head term, and — when designate is set and a query has no such
// term — every occurrence of its rarest head term (lowest df, then first in query order), so
// that the pruned search has tail candidates, hence a threshold, for all-head queries too.
// qd_* (when qd_code is set): K2b's per-query term descriptors, so a planned item needs one
// dependent load level instead of q_off -> q_terms -> head_id: qd_code[q][j] = (head id + 1,
// 0 = not a head) | walked << 30 for the first kTermLanes terms (0 past the end), qd_idf the
// term's idf (0 past the end), qd_term the term id (-1 past the end or unknown), qd_tb[q] = q_off[q],
// qd_len[q] = the query's term count.  K2a reads them too.
__global__ void bm25_qcand_kernel(const int32_t *__restrict__ q_terms, const int32_t *__restrict__ q_off, int nq,
                                  int32_t vocab, const int32_t *__restrict__ head_id,
                                  const int64_t *__restrict__ term_off, int designate, uint8_t *__restrict__ qcand,
                                  const double *__restrict__ q_idf, int32_t *__restrict__ qd_code,
                                  double *__restrict__ qd_idf, int32_t *__restrict__ qd_tb,
                                  int32_t *__restrict__ qd_len, int32_t *__restrict__ qd_term) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const int tb = q_off[q], te = q_off[q + 1];
  bool any = false;
  int32_t best_t = -1;
  int64_t best_df = INT64_MAX;
  for (int i = tb; i < te; ++i) {
    const int32_t t = q_terms[i];
    const bool valid = t >= 0 && t < vocab;
    const bool head = valid && head_id && head_id[t] >= 0;
    qcand[i] = (uint8_t)(valid && !head);
    any |= valid && !head;
    if (head) {
      const int64_t df = term_off[t + 1] - term_off[t];
      if (df < best_df) {
        best_df = df;
        best_t = t;
      }
    }
  }
  if (designate && !any && best_t >= 0)
    for (int i = tb; i < te; ++i)
      if (q_terms[i] == best_t) qcand[i] = 1;
  if (!qd_code) return;
  qd_tb[q] = tb;
  qd_len[q] = te - tb;
  for (int j = 0; j < kTermLanesQd; ++j) {
    const int i = tb + j;
    int32_t c = 0, tt = -1;
    double f = 0.0;
    if (i < te) {
      const int32_t t = q_terms[i];
      tt = t < vocab ? t : -1;
      if (t >= 0 && t < vocab) {
        c = (head_id ? head_id[t] : -1) + 1;
        if (qcand[i]) c |= 1 << 30;
      }
      f = q_idf[i];
    }
    qd_code[(int64_t)q * kTermLanesQd + j] = c;
    qd_idf[(int64_t)q * kTermLanesQd + j] = f;
    qd_term[(int64_t)q * kTermLanesQd + j] = tt;
  }
}

__global__ void bm25_bounds_kernel(const int32_t *__restrict__ q_terms, int n_terms, int32_t vocab, int nr,
                                   const int64_t *__restrict__ term_off, const int32_t *__restrict__ post_doc,
                                   const uint8_t *__restrict__ qcand, int64_t *__restrict__ bounds) {
  const int ngroups = (nr + 1 + kBoundsGroup - 1) / kBoundsGroup;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)n_terms * ngroups) return;
  const int i = (int)(gid / ngroups);
  const int g = (int)(gid - (int64_t)i * ngroups);
  const int32_t t = q_terms[i];
  int64_t *out = bounds + (int64_t)i * (nr + 1);
  const int r0 = g * kBoundsGroup;
  const int r1 = min(r0 + kBoundsGroup, nr + 1);
  if (t >= 0 && t < vocab && !qcand[i]) return;  // dense-tile term: no reader looks at its bounds
  if (t < 0 || t >= vocab) {  // unknown term: empty lists (K2 reads them)
    for (int r = r0; r < r1; ++r) out[r] = 0;
    return;
  }
  const int64_t lo_t = term_off[t], hi_t = term_off[t + 1];
  int64_t pos = r0 >= nr ? hi_t : lower_bound_doc(post_doc, lo_t, hi_t, r0 * kRange);
  out[r0] = pos;
  for (int r = r0 + 1; r < r1; ++r) {
    if (r == nr) {
      pos = hi_t;
    } else {
      const int32_t target = r * kRange;
      if (pos < hi_t && post_doc[pos] < target) {
        int64_t lo = pos, step = 1;
        while (lo + step < hi_t && post_doc[lo + step] < target) {
          lo += step;
          step <<= 1;
        }
        pos = lower_bound_doc(post_doc, lo + 1, min(lo + step, hi_t), target);
      }
    }
    out[r] = pos;
  }
}

// K2: one wave per (group of 4 queries, group of consecutive ranges of kRange
// docs); the 4 waves of a workgroup take 4 consecutive query groups over the
// same ranges, and workgroups are remapped so each XCD owns a contiguous run of
// range groups (all queries' head tiles for those ranges share that XCD's L2).
// Waves never synchronise with each other.
//
// Lane l owns docs d0 + 16l .. d0 + 16l + 15 of the current range and keeps
// their K_d (computed once per range, shared by the 4 queries) and the current
// query's fp64 scores in registers.  Lane 16q + j holds the descriptor of term
// j (< 16) of the wave's query q (term, head id, idf, tail postings [lo, hi) of
// the range).  Per range:
//   * the range's tail postings of all 4 queries' tail terms are gathered into
//     the wave's LDS slice with one coalesced pass (query/term-major, doc-sorted);
//   * per query, terms are applied in query order (duplicates twice), so every
//     document sums its contributions in rank_bm25's order:
//       - head term: 16 tf bytes per lane from the dense tile (a 2-deep
//         prefetch ring runs over the (range, query, head term) sequence), 16
//         predicated independent register updates;
//       - tail term: each lane binary-searches its 16-doc window in the
//         term's LDS postings and walks the (usually 0-1) hits slot by slot;
//   * top-k of the (range, query), pruned by the query's global threshold T
//     (atomicMin of every range's k-th best key: any range's k-th best bounds
//     the global k-th best), so most ranges stop after one argmin.
// dl / live / allow words and the tail bounds of range r+1 are loaded while
// range r is scored.
constexpr int kTailCapW = 512;  // tail postings gathered per (wave, range); overflow terms read from global
constexpr int kMaxRangesPerWave = 16;
// Ratio table: tf*2.5 / (tf + K_d) depends on (tf, dl) only, so per search the
// quotients for dl in [lut_dmin, lut_dmin + kLutW) and tf < kLutTF are computed
// once (IEEE division, bit-identical to the per-posting quotient) and K2 reads
// them from LDS; other (dl, tf) pairs divide in place.
constexpr int kLutW = 128;
constexpr int kLutTF = 16;
constexpr int kQPerWave = 4;    // queries per wave; lanes 16q..16q+15 hold query q's first 16 term descriptors
constexpr int kTermLanes = 64 / kQPerWave;
static_assert(kTermLanesQd == kTermLanes, "K2b descriptors cover a wave's term lanes");
#ifndef K2_WAVES_PER_EU
#define K2_WAVES_PER_EU 2
#endif

__device__ inline double bm25_contrib(double idf, uint32_t tfi, double kdv) {
  const double tf = (double)tfi;
  const double num = tf * 2.5;
  const double den = tf + kdv;
  return idf * (num / den);
}
// Same bits as bm25_contrib for every operand K2 can see (tf in [0, 65535], kd in
// [0.375, 2^40)): the quotient is the compiler's IEEE division sequence (rcp, two
// Newton steps, residual correction) without v_div_scale / v_div_fixup, which are
// identities when neither operand is near the exponent range limits.
__device__ inline double bm25_contrib_fast(double idf, uint32_t tfi, double kdv) {
  const double tf = (double)tfi;
  const double num = tf * 2.5;
  const double den = tf + kdv;
  double r = __builtin_amdgcn_rcp(den);
  double e = __builtin_fma(-den, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-den, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q0 = num * r;
  const double rem = __builtin_fma(-den, q0, num);
  return idf * __builtin_fma(rem, r, q0);
}
__device__ inline double kd_of(int32_t dlen, double avgdl) {
  double t = 0.75 * (double)dlen;
  t = t / avgdl;
  t = 0.25 + t;
  return 1.5 * t;
}
__global__ void bm25_lut_kernel(const double *__restrict__ avgdl_p, int dmin, double *__restrict__ lut) {
  const double avgdl = *avgdl_p;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kLutW * kLutTF) return;
  const int tf = i % kLutTF, dl = dmin + i / kLutTF;
  if (tf == 0) {
    lut[i] = 0.0;
    return;
  }
  const double t = (double)tf;
  const double num = t * 2.5;
  const double den = t + kd_of(dl, avgdl);
  lut[i] = num / den;
}
__device__ inline double readlane_f64(double v, int j) {
  const uint64_t b = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, j);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), j);
  return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
__device__ inline uint64_t readlane_u64(uint64_t v, int j) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, j);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), j);
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// first index in [lo, hi) of a doc-sorted posting list with doc >= target
template <typename P>
__device__ inline int first_ge(const P *__restrict__ a, int lo, int hi, int32_t target) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <typename TF>
__global__ void __launch_bounds__(kBmThreads) __attribute__((amdgpu_waves_per_eu(K2_WAVES_PER_EU)))
    bm25_range_kernel(const int32_t *__restrict__ q_terms, const int32_t *__restrict__ q_off, int nq,
                      const double *__restrict__ q_idf, const int64_t *__restrict__ bounds, int nr, int rpw,
                      const int64_t *__restrict__ term_off, const int32_t *__restrict__ post_doc,
                      const TF *__restrict__ post_tf, const int32_t *__restrict__ head_id,
                      const uint8_t *__restrict__ headtf, int64_t npad, const int32_t *__restrict__ dl,
                      const uint32_t *__restrict__ live, const uint32_t *__restrict__ allow, int64_t ndocs,
                      const double *__restrict__ avgdl_p, const double *__restrict__ lut, int lut_dmin, int k,
                      uint64_t *__restrict__ cand_key, uint32_t *__restrict__ cand_row,
                      unsigned long long *__restrict__ thr_key, const uint8_t *__restrict__ need, int32_t vocab,
                      int dbg) {
  __shared__ double s_lut[kLutW * kLutTF];
#ifndef CM_ABLATION
  dbg = 0;  // product build: the ablation branches fold away
#endif
  __shared__ int32_t s_pdoc[kBmThreads / 64][kTailCapW];
  __shared__ uint16_t s_ptf[kBmThreads / 64][kTailCapW];
  __shared__ uint64_t s_keys[kBmThreads / 64][16 * 64];
  const double avgdl = *avgdl_p;
  for (int i = threadIdx.x; i < kLutW * kLutTF; i += kBmThreads) s_lut[i] = lut[i];
  __syncthreads();  // the only block-wide barrier
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // XCD-aware remap: hardware places workgroup b on XCD b % 8
  const int nb = gridDim.x;
  const int b = blockIdx.x;
  const int per = nb >> 3, rem = nb & 7, x = b & 7, y = b >> 3;
  const int lb = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + y;
  const int nqg = (nq + kQPerWave - 1) / kQPerWave;
  const int wid = lb * (kBmThreads / 64) + wave;
  const int qg = wid % nqg;
  const int q0 = qg * kQPerWave;
  const int rg = wid / nqg;
  const int r0 = rg * rpw, r1 = min(r0 + rpw, nr);
  if (r0 >= r1) return;  // whole wave
  const int nqw = min(kQPerWave, nq - q0);
  // re-score mode (need != NULL, pruned search): only (range, query) pairs whose bit is set
  // in need[qg * nr + r] are scored; the others keep the tail pass's lists
  auto need_at = [&](int r) -> uint32_t {
    return need ? (uint32_t)__builtin_amdgcn_readfirstlane((int)need[(int64_t)qg * nr + r]) : 0xfu;
  };
  if (need) {  // nothing to re-score in this wave's ranges (the common case): leave at once
    uint32_t any = 0;
    for (int r = r0; r < r1; ++r) any |= need_at(r);
    if (!any) return;
  }
  int32_t *pdoc = s_pdoc[wave];
  uint16_t *ptf = s_ptf[wave];
  uint64_t *keys = s_keys[wave];
  const int64_t bstride = nr + 1;
  // ---- per-wave term descriptors (lane 16q + j <-> term j of query q0 + q)
  const int my_q = lane / kTermLanes, my_j = lane % kTermLanes;
  int my_tb = 0, my_L = 0;
  if (my_q < nqw) {
    my_tb = q_off[q0 + my_q];
    my_L = q_off[q0 + my_q + 1] - my_tb;
  }
  const bool has_term = my_q < nqw && my_j < my_L;
  const int my_i = my_tb + my_j;
  int32_t my_t = -1, my_h = -1;
  double my_idf = 0.0;
  int64_t my_lo = 0, my_hi = 0;
  if (has_term) {
    my_t = q_terms[my_i];
    if (my_t >= vocab) my_t = -1;
    my_idf = q_idf[my_i];
    my_h = (my_t >= 0 && head_id) ? head_id[my_t] : -1;
    if (my_h < 0) {  // a designated head term (K2a's generator) is read from its tile here
      my_lo = bounds[(int64_t)my_i * bstride + r0];
      my_hi = bounds[(int64_t)my_i * bstride + r0 + 1];
    }
  }
  const bool walk = has_term && my_h < 0;
  const uint64_t headmask = __ballot(has_term && my_t >= 0 && my_h >= 0);
  // ---- head-tile prefetch ring over the (range, scored query, head term) sequence
  auto head_at = [&](int r) -> uint64_t {
    if (!need) return headmask;
    const uint32_t nbits = need_at(r);
    uint64_t qm = 0;
#pragma unroll
    for (int qq = 0; qq < kQPerWave; ++qq)
      if ((nbits >> qq) & 1u) qm |= ((1ull << kTermLanes) - 1) << (kTermLanes * qq);
    return headmask & qm;
  };
  auto tile_at = [&](int r, uint64_t m) -> uint4 {
    if (m == 0 || r >= r1) return uint4{0, 0, 0, 0};
    const int j = __builtin_ctzll(m);
    const int32_t h = __builtin_amdgcn_readlane(my_h, j);
    return *reinterpret_cast<const uint4 *>(headtf + (int64_t)h * npad + (int64_t)r * kRange + 16 * lane);
  };
  auto advance = [&](int &r, uint64_t &m) {
    if (m) m &= m - 1;
    while (m == 0 && r < r1) {
      ++r;
      m = r < r1 ? head_at(r) : 0;
    }
  };
  int c_r = r0;
  uint64_t c_m = head_at(r0);
  if (c_m == 0) advance(c_r, c_m);
  uint4 n1 = tile_at(c_r, c_m);
  advance(c_r, c_m);
  uint4 n2 = tile_at(c_r, c_m);
  advance(c_r, c_m);
  // ---- range words (loaded one range ahead)
  int4 dlq[4];
  uint32_t lw = 0, aw = 0xffffffffu;
  auto load_range_words = [&](int r) {
    const int64_t db = (int64_t)r * kRange + 16 * lane;
    if (db + 16 <= ndocs) {
      const int4 *p4 = reinterpret_cast<const int4 *>(dl + db);
#pragma unroll
      for (int v = 0; v < 4; ++v) dlq[v] = p4[v];
    } else {
      int32_t t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) t[u] = db + u < ndocs ? dl[db + u] : 0;
#pragma unroll
      for (int v = 0; v < 4; ++v) dlq[v] = int4{t[4 * v], t[4 * v + 1], t[4 * v + 2], t[4 * v + 3]};
    }
    const int64_t w = db < ndocs ? db >> 5 : 0;
    lw = live[w];
    aw = allow ? allow[w] : 0xffffffffu;
  };
  if (need_at(r0)) load_range_words(r0);
  for (int r = r0; r < r1; ++r) {
    const uint32_t nbits = need_at(r);
    if (nbits == 0) {  // re-score mode, nothing to score here: keep the tail-bounds chain moving
      int64_t nx_hi = my_hi;
      if (r + 1 < r1) {
        if (need_at(r + 1)) load_range_words(r + 1);
        if (walk) nx_hi = bounds[(int64_t)my_i * bstride + r + 2];
      }
      my_lo = my_hi;
      my_hi = nx_hi;
      continue;
    }
    const int64_t d0 = (int64_t)r * kRange;
    const int64_t db = d0 + 16 * lane;
    // thresholds of the wave's queries (lanes 0..nqw-1); latency hidden behind K_d
    uint64_t Tv = kEmptyKey;
    if (lane < nqw && !(dbg & 2)) Tv = __hip_atomic_load(thr_key + q0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dbg & 2) Tv = 0;
    // LUT row base (dl - lut_dmin) * kLutTF per slot, 0xffff = outside the table (packed 2 x 16 bit)
    uint32_t lbp[8];
    {
      const int32_t dlv[16] = {dlq[0].x, dlq[0].y, dlq[0].z, dlq[0].w, dlq[1].x, dlq[1].y, dlq[1].z, dlq[1].w,
                               dlq[2].x, dlq[2].y, dlq[2].z, dlq[2].w, dlq[3].x, dlq[3].y, dlq[3].z, dlq[3].w};
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const uint32_t r0 = (uint32_t)(dlv[2 * v] - lut_dmin), r1 = (uint32_t)(dlv[2 * v + 1] - lut_dmin);
        const uint32_t b0 = r0 < (uint32_t)kLutW ? r0 * kLutTF : 0xffffu;
        const uint32_t b1 = r1 < (uint32_t)kLutW ? r1 * kLutTF : 0xffffu;
        lbp[v] = b0 | (b1 << 16);
      }
    }
    // contribution of (slot u, tf) from the table, or by division off the table
    auto lut_base = [&](int u) -> uint32_t { return (lbp[u >> 1] >> (16 * (u & 1))) & 0xffffu; };
    auto slow_contrib = [&](int u, double idf, uint32_t tfi) -> double {
      return bm25_contrib_fast(idf, tfi, kd_of(dl[db + u], avgdl));
    };
    uint32_t okmask = 0;
    if (db < ndocs) {
      okmask = ((lw & aw) >> (db & 31)) & 0xffffu;
      const int64_t rm = ndocs - db;
      if (rm < 16) okmask &= (1u << rm) - 1u;
    }
    // this range's tail postings -> LDS; next range's words/bounds in flight
    const int cnt = (int)(my_hi - my_lo);
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    const int excl = incl - cnt;
    const int my_off = (cnt > 0 && incl <= kTailCapW) ? excl : -1;
    const uint64_t inmask = __ballot(cnt > 0 && incl <= kTailCapW);
    const int n_in = inmask ? __builtin_amdgcn_readlane(incl, 63 - __builtin_clzll(inmask)) : 0;
    for (int e0 = 0; e0 < n_in; e0 += 64) {  // wave-uniform trip count: every lane takes part in the shuffles
      const int e = e0 + lane;
      int lo = 0, hi = 63;  // last lane whose exclusive offset <= e (offsets are non-decreasing)
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (__shfl(excl, mid) <= e) lo = mid;
        else hi = mid - 1;
      }
      // several lanes can share an offset (empty terms): the last one is the one with postings
      const int64_t src = __shfl(my_lo, lo) + (e - __shfl(excl, lo));
      if (e < n_in) {
        pdoc[e] = post_doc[src];
        ptf[e] = (uint16_t)post_tf[src];
      }
    }
    int64_t nx_lo = my_hi, nx_hi = my_hi;
    if (r + 1 < r1) {
      if (need_at(r + 1)) load_range_words(r + 1);
      if (walk) nx_hi = bounds[(int64_t)my_i * bstride + r + 2];
    }
    wave_lds_sync();
    const int32_t wlo = (int32_t)(db - d0), whi = wlo + 16;  // this lane's window, range-relative
    for (int qq = 0; qq < nqw; ++qq) {
      if (!((nbits >> qq) & 1u)) continue;  // this pair keeps the tail pass's list
      const int qi = q0 + qq;
      const int base = qq * kTermLanes;
      const int L = __builtin_amdgcn_readlane(my_L, base);
      double sc[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) sc[u] = 0.0;
      if (!(dbg & 1)) {
        for (int j = 0; j < L; ++j) {
          int32_t t, hh;
          double idf;
          int c, off;
          int64_t plo;
          if (j < kTermLanes) {
            const int ln = base + j;
            t = __builtin_amdgcn_readlane(my_t, ln);
            hh = __builtin_amdgcn_readlane(my_h, ln);
            idf = readlane_f64(my_idf, ln);
            c = __builtin_amdgcn_readlane(cnt, ln);
            off = __builtin_amdgcn_readlane(my_off, ln);
            plo = (int64_t)readlane_u64((uint64_t)my_lo, ln);
          } else {  // long query: descriptor, bounds and postings from global
            const int i = __builtin_amdgcn_readlane(my_tb, base) + j;
            t = q_terms[i];
            hh = (t >= 0 && head_id) ? head_id[t] : -1;
            idf = q_idf[i];
            plo = bounds[(int64_t)i * bstride + r];
            c = (int)(bounds[(int64_t)i * bstride + r + 1] - plo);
            off = -1;
          }
          if (t < 0) continue;
          if (hh >= 0) {
            uint4 v;
            if (j < kTermLanes) {
              v = n1;
              n1 = n2;
              n2 = tile_at(c_r, c_m);
              advance(c_r, c_m);
            } else {
              v = *reinterpret_cast<const uint4 *>(headtf + (int64_t)hh * npad + db);
            }
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
            if (__ballot((wv[0] | wv[1] | wv[2] | wv[3]) != 0u) == 0) continue;  // no doc of the range has the term
            // branch-free: tf == 0 (and off-table slots) read the table's 0.0 entry, adding
            // idf * +-0.0, which leaves a (never -0.0) score unchanged
            uint32_t slowm = 0;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const uint32_t tfi = (wv[u >> 2] >> (8 * (u & 3))) & 0xffu;
              const uint32_t b = lut_base(u);
              const bool ok = b != 0xffffu && tfi < (uint32_t)kLutTF;
              sc[u] = sc[u] + idf * s_lut[ok ? b + tfi : 0u];
              if (!ok && tfi != 0u) slowm |= 1u << u;
            }
            if (slowm) {
#pragma unroll
              for (int u = 0; u < 16; ++u)
                if ((slowm >> u) & 1u)
                  sc[u] = sc[u] + slow_contrib(u, idf, (wv[u >> 2] >> (8 * (u & 3))) & 0xffu);
            }
          } else if (c > 0) {
            // lane's window [wlo, whi) of the term's doc-sorted postings (LDS, or global on
            // overflow: one flat-pointer path), walked slot by slot (compile-time register
            // indices; the wave skips the block when no lane has a hit)
            const int32_t *pd = off >= 0 ? pdoc + off : post_doc + plo;
            const TF *pt = off >= 0 ? reinterpret_cast<const TF *>(ptf + off) : post_tf + plo;
            int e = first_ge(pd, 0, c, (int32_t)d0 + wlo);
            int32_t nd = e < c ? pd[e] - (int32_t)d0 : INT32_MAX;
            if (nd < whi) {
#pragma unroll
              for (int u = 0; u < 16; ++u) {
                if (nd == wlo + u) {
                  const uint32_t tfi = (uint32_t)pt[e];
                  const uint32_t b = lut_base(u);
                  sc[u] = sc[u] + ((b != 0xffffu && tfi < (uint32_t)kLutTF) ? idf * s_lut[b + tfi]
                                                                             : slow_contrib(u, idf, tfi));
                  ++e;
                  nd = e < c ? pd[e] - (int32_t)d0 : INT32_MAX;
                }
              }
            }
          }
        }
      } else {  // ablation: keep the ring in step
        uint64_t m = headmask & (((1ull << kTermLanes) - 1) << base);
        for (; m; m &= m - 1) {
          n1 = n2;
          n2 = tile_at(c_r, c_m);
          advance(c_r, c_m);
        }
      }
      // ---- top-k of this (range, query), pruned by the query's global threshold
      // keys -> the wave's LDS key tile (slot-major: conflict-free), lane best in registers;
      // only the lane whose best is taken rescans its 16 keys
      uint64_t bk = kEmptyKey;
      int bu = 0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const uint64_t key = ((okmask >> u) & 1u) ? score_key(sc[u]) : kEmptyKey;
        keys[u * 64 + lane] = key;
        if (key < bk) {  // u ascending == row ascending within the lane
          bk = key;
          bu = u;
        }
      }
      uint32_t br = bk == kEmptyKey ? 0xffffffffu : (uint32_t)db + (uint32_t)bu;
      const uint64_t T = readlane_u64(Tv, qq);
      int i = 0;
      uint64_t last = kEmptyKey;
      for (; i < k; ++i) {
        uint64_t mk = bk;
        uint32_t mr = br;
        wave_min_pair(mk, mr);
        if (mr == 0xffffffffu || mk > T) break;  // nothing left that can enter the global top-k
        if (lane == 0) {
          const int64_t o = lslot(qi, r, nr, lheads_total(nq, nr), k, i);
          cand_key[o] = mk;
          cand_row[o] = mr;
        }
        last = mk;
        if (br == mr && bk == mk) {
          keys[(int)(mr - (uint32_t)db) * 64 + lane] = kEmptyKey;
          bk = kEmptyKey;
          bu = 0;
          for (int u = 0; u < 16; ++u) {
            const uint64_t key = keys[u * 64 + lane];
            if (key < bk) {
              bk = key;
              bu = u;
            }
          }
          br = bk == kEmptyKey ? 0xffffffffu : (uint32_t)db + (uint32_t)bu;
        }
      }
      if (lane == 0 && i < k) {  // list terminator (readers stop at the first empty slot)
        const int64_t o = lslot(qi, r, nr, lheads_total(nq, nr), k, i);
        cand_key[o] = kEmptyKey;
        cand_row[o] = 0xffffffffu;
      }
      if (i == k && lane == 0 && last < T) atomicMin(thr_key + qi, (unsigned long long)last);
    }
    my_lo = nx_lo;
    my_hi = nx_hi;
    wave_lds_sync();  // LDS slice reused by the next range
  }
}

#include "cm_bm25_prune.inc"

// Dense head-term tiles: tf[h][doc] (uint8; heads never have tf >= 255) from the CSR.
__global__ void bm25_head_fill_kernel(const int32_t *__restrict__ head_terms, int nhead,
                                      const int64_t *__restrict__ term_off, const int32_t *__restrict__ post_doc,
                                      const uint16_t *__restrict__ post_tf, uint8_t *__restrict__ headtf,
                                      int64_t npad) {
  const int h = blockIdx.y;
  if (h >= nhead) return;
  const int32_t t = head_terms[h];
  const int64_t lo = term_off[t], hi = term_off[t + 1];
  uint8_t *row = headtf + (int64_t)h * npad;
  for (int64_t p = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < hi; p += (int64_t)gridDim.x * blockDim.x)
    row[post_doc[p]] = (uint8_t)post_tf[p];  // < 255: saturating terms are never heads
}

// Histogram of live document lengths < 65536 (K2 ratio-table window choice).
__global__ void bm25_dl_hist_kernel(const int32_t *__restrict__ dl, int64_t ndocs, uint32_t *__restrict__ hist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ndocs; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = dl[i];
    if (d >= 0 && d < 65536) atomicAdd(hist + d, 1u);
  }
}

// sat[c] != 0 iff candidate head term c has a posting with tf >= 255 (it then stays
// on the postings path: head tiles hold exact tf bytes only).
__global__ void bm25_head_sat_kernel(const int32_t *__restrict__ cand, int ncand, const int64_t *__restrict__ term_off,
                                     const uint16_t *__restrict__ post_tf, int32_t *__restrict__ sat) {
  const int c = blockIdx.y;
  if (c >= ncand) return;
  const int32_t t = cand[c];
  const int64_t lo = term_off[t], hi = term_off[t + 1];
  bool any = false;
  for (int64_t p = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < hi; p += (int64_t)gridDim.x * blockDim.x)
    any |= post_tf[p] >= 255;
  if (__any(any) && (threadIdx.x & 63) == 0) atomicOr(sat + c, 1);
}

// Tournament merge of nr sorted per-range lists per query (one workgroup per query, gridDim.x = nq).
__global__ void __launch_bounds__(kMergeThreads) bm25_merge_kernel(const uint64_t *__restrict__ cand_key,
                                                                   const uint32_t *__restrict__ cand_row, int nr,
                                                                   int k, double *__restrict__ out_score,
                                                                   int64_t *__restrict__ out_row) {
  const int qi = blockIdx.x;
  __shared__ uint64_t sk[kMergeThreads / 64];
  __shared__ uint32_t sr[kMergeThreads / 64];
  int head[kMergePer];
  uint64_t hk[kMergePer];
  uint32_t hr[kMergePer];
  const int64_t nl = lheads_total((int)gridDim.x, nr);
#pragma unroll
  for (int s = 0; s < kMergePer; ++s) {
    const int l = threadIdx.x + kMergeThreads * s;
    head[s] = 0;
    hk[s] = kEmptyKey;
    hr[s] = 0xffffffffu;
    if (l < nr) {
      hk[s] = cand_key[lhead(qi, l, nr)];
      hr[s] = cand_row[lhead(qi, l, nr)];
    }
  }
  for (int i = 0; i < k; ++i) {
    uint64_t mk = kEmptyKey;
    uint32_t mr = 0xffffffffu;
#pragma unroll
    for (int s = 0; s < kMergePer; ++s)
      if (pk_less(hk[s], hr[s], mk, mr)) {
        mk = hk[s];
        mr = hr[s];
      }
    const PairKey best = block_min_pair(mk, mr, sk, sr);
    if (threadIdx.x == 0) {
      const int64_t o = (int64_t)qi * k + i;
      if (best.r == 0xffffffffu) {
        out_score[o] = 0.0;
        out_row[o] = -1;
      } else {
        out_score[o] = f64_unorder(~best.k);
        out_row[o] = (int64_t)best.r;
      }
    }
    if (best.r == 0xffffffffu) continue;
#pragma unroll
    for (int s = 0; s < kMergePer; ++s) {
      if (hr[s] == best.r && hk[s] == best.k) {
        const int l = threadIdx.x + kMergeThreads * s;
        head[s] += 1;
        if (head[s] < k) {
          hk[s] = cand_key[lslot(qi, l, nr, nl, k, head[s])];
          hr[s] = cand_row[lslot(qi, l, nr, nl, k, head[s])];
        } else {
          hk[s] = kEmptyKey;
          hr[s] = 0xffffffffu;
        }
      }
    }
  }
}

// The same merge for k <= kMergeSmallK with a 256-thread workgroup (one wave per SIMD, <= 128 VGPRs,
// 48 B of LDS): it fits beside a K1q workgroup (384 registers per SIMD, <= 131 KiB of LDS), so the
// BM25 chain after K2a runs while the dense scan still streams instead of queueing behind it -- the
// 1024-thread bm25_merge_kernel needs a whole empty CU (4 waves of 128 VGPRs per SIMD) and waited
// for K1q's last workgroup (profiles/r05_headline_timeline.txt).
// Phase 1: each thread reads the heads of its lists l = tid + 256 s (coalesced, merge_batch<K>()
// independent loads in flight) and keeps the K smallest in a sorted register array of (key, row,
// list<<5 | depth).  A list whose head misses its thread's K smallest heads cannot place an entry in
// the top k <= K (K smaller distinct heads precede all its entries), so it is dropped for good.
// Phase 2: k rounds of a block tournament over the threads' array fronts; the owner pops its front
// and re-inserts that list's next entry, which it prefetched the round before (the load latency
// hides behind the reduction).  Same output as bm25_merge_kernel: the k smallest (key, row), 0.0 /
// -1 padding.
constexpr int kMergeSmallK = 12;   // K = 16 needs > 128 VGPRs
constexpr int kMergeSmallThreads = 256;
template <int K>
constexpr int merge_batch() { return K > 8 ? 4 : 8; }   // <= 128 VGPRs
template <int K>
__device__ inline void merge_insert(uint64_t (&lk)[K], uint32_t (&lr)[K], uint32_t (&ll)[K], uint64_t ck,
                                    uint32_t cr, uint32_t cl) {
#pragma unroll
  for (int i = 0; i < K; ++i) {  // sorted insertion, static indices (the last entry falls off)
    if (pk_less(ck, cr, lk[i], lr[i])) {
      const uint64_t tk = lk[i];
      const uint32_t tr = lr[i], tl = ll[i];
      lk[i] = ck;
      lr[i] = cr;
      ll[i] = cl;
      ck = tk;
      cr = tr;
      cl = tl;
    }
  }
}
template <int K>
__global__ void __launch_bounds__(kMergeSmallThreads) bm25_merge_small_kernel(const uint64_t *__restrict__ cand_key,
                                                                               const uint32_t *__restrict__ cand_row,
                                                                               int nr, int k, double *__restrict__ out_score,
                                                                               int64_t *__restrict__ out_row) {
  const int qi = blockIdx.x;
  __shared__ uint64_t sk[kMergeSmallThreads / 64];
  __shared__ uint32_t sr[kMergeSmallThreads / 64];
  uint64_t lk[K];
  uint32_t lr[K], ll[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    lk[i] = kEmptyKey;
    lr[i] = 0xffffffffu;
    ll[i] = 0;
  }
  const int64_t nl = lheads_total((int)gridDim.x, nr);
  constexpr int kMergeBatch = merge_batch<K>();
  for (int l0 = threadIdx.x; l0 < nr; l0 += kMergeSmallThreads * kMergeBatch) {
    uint64_t bk[kMergeBatch];
    uint32_t br[kMergeBatch];
#pragma unroll
    for (int u = 0; u < kMergeBatch; ++u) {
      const int l = l0 + u * kMergeSmallThreads;
      bk[u] = kEmptyKey;
      br[u] = 0xffffffffu;
      if (l < nr) {
        bk[u] = cand_key[lhead(qi, l, nr)];
        br[u] = cand_row[lhead(qi, l, nr)];
      }
    }
#pragma unroll
    for (int u = 0; u < kMergeBatch; ++u)
      if (br[u] != 0xffffffffu && pk_less(bk[u], br[u], lk[K - 1], lr[K - 1]))   // empty list / cannot enter
        merge_insert<K>(lk, lr, ll, bk[u], br[u], (uint32_t)(l0 + u * kMergeSmallThreads) << 5);
  }
  uint64_t nk = kEmptyKey;   // prefetched next entry of the front list
  uint32_t nrow = 0xffffffffu;
  auto prefetch = [&]() {
    nk = kEmptyKey;
    nrow = 0xffffffffu;
    const int d = (int)(ll[0] & 31u) + 1;
    if (lr[0] != 0xffffffffu && d < k) {
      const int64_t o = lslot(qi, ll[0] >> 5, nr, nl, k, d);
      nk = cand_key[o];
      nrow = cand_row[o];
    }
  };
  prefetch();
  for (int i = 0; i < k; ++i) {
    const PairKey best = block_min_pair(lk[0], lr[0], sk, sr);
    if (threadIdx.x == 0) {
      const int64_t o = (int64_t)qi * k + i;
      if (best.r == 0xffffffffu) {
        out_score[o] = 0.0;
        out_row[o] = -1;
      } else {
        out_score[o] = f64_unorder(~best.k);
        out_row[o] = (int64_t)best.r;
      }
    }
    if (best.r == 0xffffffffu) continue;
    if (lr[0] == best.r && lk[0] == best.k) {   // the owner pops its front (entries are unique)
      const uint32_t nxt = ll[0] + 1;
#pragma unroll
      for (int t = 0; t + 1 < K; ++t) {
        lk[t] = lk[t + 1];
        lr[t] = lr[t + 1];
        ll[t] = ll[t + 1];
      }
      lk[K - 1] = kEmptyKey;
      lr[K - 1] = 0xffffffffu;
      if (nrow != 0xffffffffu) merge_insert<K>(lk, lr, ll, nk, nrow, nxt);   // the list's sentinel ends it
      prefetch();
    }
  }
}

// bm25_merge_kernel or, for k <= kMergeSmallK, its small-workgroup form (launch helper)
int launch_bm25_merge(const uint64_t *cand_key, const uint32_t *cand_row, int nq, int nr, int k, double *score,
                      int64_t *row, hipStream_t st) {
  const bool small = env_knob("CM_BM25_MERGE_SMALL", true);   // 0: the 1024-thread kernel for every k (A/B)
  if (small && k <= 8)
    hipLaunchKernelGGL(bm25_merge_small_kernel<8>, dim3(nq), dim3(kMergeSmallThreads), 0, st, cand_key, cand_row, nr, k,
                       score, row);
  else if (small && k <= 10)
    hipLaunchKernelGGL(bm25_merge_small_kernel<10>, dim3(nq), dim3(kMergeSmallThreads), 0, st, cand_key, cand_row, nr,
                       k, score, row);
  else if (small && k <= kMergeSmallK)
    hipLaunchKernelGGL(bm25_merge_small_kernel<kMergeSmallK>, dim3(nq), dim3(kMergeSmallThreads), 0, st, cand_key,
                       cand_row, nr, k, score, row);
  else
    hipLaunchKernelGGL(bm25_merge_kernel, dim3(nq), dim3(kMergeThreads), 0, st, cand_key, cand_row, nr, k, score, row);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

// Filtered statistics: number of candidate docs and their total length.
__global__ void bm25_filtered_stats_kernel(const int32_t *__restrict__ dl, const uint32_t *__restrict__ live,
                                           const uint32_t *__restrict__ allow, int64_t ndocs,
                                           unsigned long long *__restrict__ out /* [2] */) {
  unsigned long long cnt = 0, sum = 0;
  const int64_t nw = ceil_div(ndocs, 32);
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    uint32_t b = live[w] & allow[w];
    while (b) {
      const int bit = __builtin_ctz(b);
      b &= b - 1;
      const int64_t d = w * 32 + bit;
      if (d < ndocs) {
        cnt += 1;
        sum += (unsigned long long)dl[d];
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    sum += __shfl_xor(sum, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (cnt) atomicAdd(&out[0], cnt);
    if (sum) atomicAdd(&out[1], sum);
  }
}

// Per listed term: number of candidate postings and the first candidate
// posting's (doc << 32 | first position) key (terms' dict order).  gridDim.y > 1 (the per-query
// df of a filtered search, out_first unused): block (i, s) counts slice s of the term's postings
// and adds it to out_df[i] (zeroed by the caller) -- one block per term walked a frequent term's
// whole list alone (2.7 ms per single filtered query at 1M documents).
__global__ void __launch_bounds__(256) bm25_term_df_kernel(const int32_t *__restrict__ terms, int n_terms,
                                                           int32_t vocab, const int64_t *__restrict__ term_off,
                                                           const int32_t *__restrict__ post_doc,
                                                           const uint32_t *__restrict__ post_pos,
                                                           const uint32_t *__restrict__ live,
                                                           const uint32_t *__restrict__ allow,
                                                           int64_t *__restrict__ out_df, uint64_t *__restrict__ out_first) {
  const int i = blockIdx.x;
  if (i >= n_terms) return;
  const int32_t t = terms ? terms[i] : i;
  if (t < 0 || t >= vocab) {  // unknown query term: not in the candidate vocabulary
    if (threadIdx.x == 0) {
      out_df[i] = 0;
      if (out_first) out_first[i] = ~0ull;
    }
    return;
  }
  __shared__ unsigned long long red_c[4];
  __shared__ unsigned long long red_m[4];
  unsigned long long c = 0, m = ~0ull;
  const int64_t lo = term_off[t], hi = term_off[t + 1];
  const int64_t stride = 256 * (int64_t)gridDim.y;
  if (gridDim.y > 1 && lo + (int64_t)blockIdx.y * 256 >= hi) return;  // nothing in this slice
  for (int64_t p = lo + (int64_t)blockIdx.y * 256 + threadIdx.x; p < hi; p += stride) {
    const int32_t d = post_doc[p];
    if ((live[d >> 5] & allow[d >> 5]) >> (d & 31) & 1u) {
      c += 1;
      const unsigned long long key = ((unsigned long long)(uint32_t)d << 32) | post_pos[p];
      m = key < m ? key : m;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    const unsigned long long om = __shfl_xor(m, o);
    m = om < m ? om : m;
  }
  if ((threadIdx.x & 63) == 0) {
    red_c[threadIdx.x >> 6] = c;
    red_m[threadIdx.x >> 6] = m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long cc = 0, mm = ~0ull;
    for (int w = 0; w < 4; ++w) {
      cc += red_c[w];
      mm = red_m[w] < mm ? red_m[w] : mm;
    }
    if (gridDim.y > 1) {
      if (cc) atomicAdd(reinterpret_cast<unsigned long long *>(out_df + i), cc);
    } else {
      out_df[i] = (int64_t)cc;
      if (out_first) out_first[i] = mm;
    }
  }
}

// ---------------- K7: device CSR build (radix sort by (term, doc)) ----------------
__global__ void bm25_token_keys_kernel(const int32_t *__restrict__ term_ids, const int64_t *__restrict__ doc_off,
                                       int64_t ndocs, uint64_t *__restrict__ keys, uint32_t *__restrict__ pos,
                                       int32_t *__restrict__ dl, int32_t *__restrict__ bad) {
  const int64_t d = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (d >= ndocs) return;
  const int lane = threadIdx.x & 63;
  const int64_t b = doc_off[d], e = doc_off[d + 1];
  if (lane == 0) dl[d] = (int32_t)(e - b);
  for (int64_t p = b + lane; p < e; p += 64) {
    const int32_t t = term_ids[p];
    if (t < 0) atomicOr(bad, 1);
    keys[p] = ((uint64_t)(uint32_t)t << 32) | (uint64_t)(uint32_t)d;
    pos[p] = (uint32_t)(p - b);
  }
}

__global__ void bm25_postings_from_runs_kernel(const uint64_t *__restrict__ ukeys, const int32_t *__restrict__ counts,
                                               const int64_t *__restrict__ run_start,
                                               const uint32_t *__restrict__ sorted_pos, int64_t nruns,
                                               int32_t *__restrict__ post_doc, uint16_t *__restrict__ post_tf,
                                               uint32_t *__restrict__ post_pos, int64_t *__restrict__ term_off,
                                               int32_t vocab, int32_t *__restrict__ tf_overflow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nruns) return;
  const uint64_t key = ukeys[i];
  const int32_t t = (int32_t)(key >> 32);
  post_doc[i] = (int32_t)(uint32_t)key;
  const int32_t c = counts[i];
  if (c > 65535) atomicOr(tf_overflow, 1);
  post_tf[i] = (uint16_t)min(c, 65535);
  post_pos[i] = sorted_pos[run_start[i]];
  // CSR offsets: the first run of term t starts t's postings; fill skipped terms
  const int32_t tp = i > 0 ? (int32_t)(ukeys[i - 1] >> 32) : -1;
  for (int32_t x = tp + 1; x <= t; ++x) term_off[x] = i;
  if (i == nruns - 1)
    for (int32_t x = t + 1; x <= vocab; ++x) term_off[x] = nruns;
}

__global__ void set_all_bits_kernel(uint32_t *bits, int64_t n) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nw = ceil_div(n, 32);
  if (w >= nw) return;
  const int64_t rem = n - w * 32;
  bits[w] = rem >= 32 ? 0xffffffffu : ((1u << rem) - 1u);
}

__global__ void first_key_kernel(const int64_t *__restrict__ term_off, const int32_t *__restrict__ post_doc,
                                 const uint32_t *__restrict__ post_pos, int32_t vocab,
                                 uint64_t *__restrict__ first) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= vocab) return;
  const int64_t p = term_off[t];
  first[t] = p < term_off[t + 1] ? (((uint64_t)(uint32_t)post_doc[p] << 32) | post_pos[p]) : ~0ull;
}

// k > kMaxTopK (BM25Store.search with a large top_k, rag/retrieval/bm25.py:199): every candidate's
// score.  One launch per query term in query order adds the term's contribution to each of its
// postings' documents (a document appears once per term: no atomics; the sums follow rank_bm25's
// term order, and the quotient is the IEEE division the fused kernels' ratio table / Newton
// sequence reproduce bit for bit); then one key per document for a stable descending sort.
__global__ void bm25_scatter_term_kernel(int64_t lo, int64_t hi, const int32_t *__restrict__ post_doc,
                                         const uint16_t *__restrict__ post_tf, const int32_t *__restrict__ dl,
                                         double idf, double avgdl, double *__restrict__ score) {
  const int64_t p = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= hi) return;
  const int32_t d = post_doc[p];
  score[d] = score[d] + bm25_contrib(idf, (uint32_t)post_tf[p], kd_of(dl[d], avgdl));
}
__global__ void bm25_score_keys_kernel(const double *__restrict__ score, const uint32_t *__restrict__ live,
                                       const uint32_t *__restrict__ allow, int64_t ndocs, uint64_t *__restrict__ keys,
                                       int32_t *__restrict__ rows) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  const uint32_t w = live[d >> 5] & (allow ? allow[d >> 5] : 0xffffffffu);
  keys[d] = ((w >> (d & 31)) & 1u) ? score_key(score[d]) : kEmptyKey;
  rows[d] = (int32_t)d;
}

__global__ void bm25_set_f64_kernel(double v, double *__restrict__ out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *out = v;
}

// Statistics over a filtered candidate set (quirk Q2, rag/retrieval/bm25.py:184-191) on the device:
// stats = {Nc, sum of candidate lengths} (global sums on a sharded index), df[i] = candidate df of
// query term i.  idf = L[Nc - df] - L[df] with L[x] = glibc log(x + 0.5) precomputed on the host
// (cm_bm25_prepare_filtered), i.e. the same two logs and one subtraction as rank_bm25's
// math.log(Nc - df + 0.5) - math.log(df + 0.5): bit-identical to the host path.  A negative idf
// takes the candidate vocabulary's epsilon from *eps_dev (NaN / NULL: status bit 0 -- the caller
// computes it with cm_bm25_filter_eps and searches again).  status bit 1: candidates without
// tokens (rank_bm25's ZeroDivisionError), bit 2: Nc beyond the prepared log table.
__global__ void bm25_stats_idf_kernel(const int32_t *__restrict__ q_terms, int n, int32_t vocab,
                                      const int64_t *__restrict__ stats, const int64_t *__restrict__ df,
                                      const double *__restrict__ logtab, int64_t log_n,
                                      const double *__restrict__ eps_dev, double *__restrict__ q_idf,
                                      double *__restrict__ avgdl, int32_t *__restrict__ status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nc = stats[0], sl = stats[1];
  if (i == 0) {
    *avgdl = nc > 0 ? (double)sl / (double)nc : 1.0;  // Nc == 0: nothing is scored
    if (nc > 0 && sl == 0) atomicOr(status, 2);
    if (nc > log_n) atomicOr(status, 4);
  }
  if (i >= n) return;
  const int32_t t = q_terms[i];
  const int64_t d = df[i];
  double v = 0.0;
  if (t >= 0 && t < vocab && d > 0 && nc <= log_n) {
    v = logtab[nc - d] - logtab[d];
    if (v < 0) {
      const double e = eps_dev ? *eps_dev : __builtin_nan("");
      if (e != e) atomicOr(status, 1);
      v = e;
    }
  }
  q_idf[i] = v;
}

}  // namespace cm

using namespace cm;

struct cm_bm25 {
  int dev = 0;
  hipStream_t stream = nullptr;
  int64_t ndocs = 0, npost = 0;
  int32_t vocab = 0;
  int64_t n_live = 0, sum_len = 0;
  double avgdl = 0.0, eps = 0.0;
  bool empty_vocab = false;  // live docs exist but no tokens (ZeroDivisionError on search)
  DevBuf term_off, post_doc, post_tf, post_pos, dl, live, idf;
  DevBuf headtf, head_id;  // dense tf tiles for high-df terms (K2 fast path)
  DevBuf logtab;           // L[x] = log(x + 0.5), x <= log_n (filtered device statistics)
  int64_t log_n = -1;
  DevBuf head_maxtf, range_mindl;  // pruned search: per-(head, range) max tf, per-range min length
  DevBuf blk_maxtf, blk_mindl;     // the same per 64-doc block
  DevBuf blk_maxr;                 // per (head, 64-doc block): ceil-quantised max ratio tf.2.5/(tf + K_d)
  DevBuf blk16_maxr;               // the same per (head, 16-doc sub-block): the planner's sub-block level
  double maxr_avgdl = 0.0;         // ... at this avgdl: a valid bound for every search avgdl <= it
  int32_t path = 0;                // 0 auto (pruned), 1 full K2 scan, 2 pruned
  int32_t last_rescored = 0;       // (query, range) pairs K2 re-scored in the last host search
  int32_t nhead = 0;
  int64_t npad = 0;
  int32_t lut_dmin = 0;                  // first doc length of K2's ratio table window
  // df > ndocs * frac qualifies.  1/128 (within 8 GiB: 858 tiles at 10M docs) measured 3.20 ms for
  // the pruned search against 3.37 at 1/64 (520 tiles) and 3.67 / 4.2 at 1717 / 3435 tiles: more
  // tiles shorten K2a's postings walks but widen K2b's head-only documents
  double head_min_frac = 1.0 / 128.0;
  int64_t head_max_bytes = 8ll << 30;    // tile memory budget
  std::vector<double> idf_host;
  DevBuf ws, qbuf, obuf, allow_buf, tmp;
  KernelTimer timer;    // K2 events (cm_bm25_timing)
  KernelTimer timer_b;  // K2b events (cm_bm25_timing_drain_block)
};

namespace {

// rank_bm25 idf for one term over a candidate set of n docs.
inline double bm25_idf(int64_t n, int64_t df) {
  return std::log((double)(n - df) + 0.5) - std::log((double)df + 0.5);
}

// Unfiltered statistics from df and the terms' first-occurrence order.
int compute_idf_table(cm_bm25 *h, const std::vector<int32_t> &df, const std::vector<int32_t> &order) {
  h->idf_host.assign(h->vocab, 0.0);
  h->empty_vocab = false;
  h->eps = 0.0;
  h->avgdl = h->n_live ? (double)h->sum_len / (double)h->n_live : 0.0;
  if (h->n_live == 0) return CM_OK;
  if (order.empty()) {
    h->empty_vocab = true;
    return CM_OK;
  }
  double idf_sum = 0.0;
  for (int32_t t : order) {
    const double v = bm25_idf(h->n_live, df[t]);
    h->idf_host[t] = v;
    idf_sum = idf_sum + v;
  }
  const double avg = idf_sum / (double)order.size();
  h->eps = 0.25 * avg;
  for (int32_t t : order)
    if (h->idf_host[t] < 0) h->idf_host[t] = h->eps;
  int rc = h->idf.ensure((size_t)std::max(h->vocab, 1) * 8);
  if (rc) return rc;
  CM_HIP(hipMemcpyAsync(h->idf.ptr, h->idf_host.data(), (size_t)h->vocab * 8, hipMemcpyHostToDevice, h->stream));
  return CM_OK;
}

// Select head terms (df > ndocs * head_min_frac, highest df first, within the
// byte budget) and build their dense uint8 tf tiles on the handle's stream.
// K2 ratio-table window: the kLutW consecutive document lengths holding the most documents.
int choose_lut_window(cm_bm25 *h) {
  h->lut_dmin = 0;
  if (h->ndocs == 0) return CM_OK;
  int rc;
  if ((rc = h->tmp.ensure(65536 * 4))) return rc;
  CM_HIP(hipMemsetAsync(h->tmp.ptr, 0, 65536 * 4, h->stream));
  hipLaunchKernelGGL(bm25_dl_hist_kernel, dim3(1024), dim3(256), 0, h->stream, h->dl.as<int32_t>(), h->ndocs,
                     h->tmp.as<uint32_t>());
  CM_HIP(hipGetLastError());
  std::vector<uint32_t> hist(65536);
  CM_HIP(hipMemcpyAsync(hist.data(), h->tmp.ptr, 65536 * 4, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  uint64_t win = 0, best = 0;
  for (int d = 0; d < kLutW; ++d) win += hist[d];
  best = win;
  for (int d0 = 1; d0 + kLutW <= 65536; ++d0) {
    win += hist[d0 + kLutW - 1];
    win -= hist[d0 - 1];
    if (win > best) {
      best = win;
      h->lut_dmin = d0;
    }
  }
  return CM_OK;
}

int build_head_tiles(cm_bm25 *h, const std::vector<int32_t> &df) {
  h->nhead = 0;
  int rc0 = choose_lut_window(h);
  if (rc0) return rc0;
  h->npad = round_up(std::max<int64_t>(h->ndocs, 1), kRange);
  const double thr = (double)h->ndocs * h->head_min_frac;
  std::vector<int32_t> cand;
  for (int32_t t = 0; t < h->vocab; ++t)
    if ((double)df[t] > thr && df[t] > 0) cand.push_back(t);
  std::sort(cand.begin(), cand.end(), [&](int32_t a, int32_t b) { return df[a] > df[b] || (df[a] == df[b] && a < b); });
  int rc;
  if (!cand.empty()) {  // drop terms whose tf does not fit a byte
    if ((rc = h->tmp.ensure(cand.size() * 8))) return rc;
    int32_t *dcand = h->tmp.as<int32_t>(), *dsat = dcand + cand.size();
    CM_HIP(hipMemcpyAsync(dcand, cand.data(), cand.size() * 4, hipMemcpyHostToDevice, h->stream));
    CM_HIP(hipMemsetAsync(dsat, 0, cand.size() * 4, h->stream));
    hipLaunchKernelGGL(bm25_head_sat_kernel, dim3(16, (unsigned)cand.size()), dim3(256), 0, h->stream, dcand,
                       (int)cand.size(), h->term_off.as<int64_t>(), h->post_tf.as<uint16_t>(), dsat);
    CM_HIP(hipGetLastError());
    std::vector<int32_t> sat(cand.size());
    CM_HIP(hipMemcpyAsync(sat.data(), dsat, cand.size() * 4, hipMemcpyDeviceToHost, h->stream));
    CM_HIP(hipStreamSynchronize(h->stream));
    size_t o = 0;
    for (size_t i = 0; i < cand.size(); ++i)
      if (!sat[i]) cand[o++] = cand[i];
    cand.resize(o);
  }
  const int64_t max_h = h->head_max_bytes / h->npad;
  if ((int64_t)cand.size() > max_h) cand.resize((size_t)std::max<int64_t>(max_h, 0));
  std::vector<int32_t> hid((size_t)std::max(h->vocab, 1), -1);
  for (size_t i = 0; i < cand.size(); ++i) hid[cand[i]] = (int32_t)i;
  if ((rc = h->head_id.ensure((size_t)std::max(h->vocab, 1) * 4))) return rc;
  CM_HIP(hipMemcpyAsync(h->head_id.ptr, hid.data(), (size_t)std::max(h->vocab, 1) * 4, hipMemcpyHostToDevice,
                        h->stream));
  if (!cand.empty()) {
    const size_t bytes = cand.size() * (size_t)h->npad;
    if ((rc = h->headtf.ensure(bytes)) || (rc = h->tmp.ensure(cand.size() * 4))) return rc;
    CM_HIP(hipMemsetAsync(h->headtf.ptr, 0, bytes, h->stream));
    CM_HIP(hipMemcpyAsync(h->tmp.ptr, cand.data(), cand.size() * 4, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(bm25_head_fill_kernel, dim3(64, (unsigned)cand.size()), dim3(256), 0, h->stream,
                       h->tmp.as<int32_t>(), (int)cand.size(), h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(),
                       h->post_tf.as<uint16_t>(), h->headtf.as<uint8_t>(), h->npad);
    CM_HIP(hipGetLastError());
    CM_HIP(hipStreamSynchronize(h->stream));  // tmp is reused by later calls
  }
  h->nhead = (int32_t)cand.size();
  // pruned-search bounds: shortest document per range, largest head tf byte per (head, range)
  const int64_t nr = std::max<int64_t>(1, ceil_div(h->ndocs, kRange));
  if ((rc = h->range_mindl.ensure((size_t)nr * 4))) return rc;
  hipLaunchKernelGGL(bm25_range_mindl_kernel, dim3((unsigned)ceil_div(nr * 64, 256)), dim3(256), 0, h->stream,
                     h->dl.as<int32_t>(), h->ndocs, (int)nr, h->range_mindl.as<int32_t>());
  CM_HIP(hipGetLastError());
  const int64_t nblk = nr * (kRange / 64);
  if ((rc = h->blk_mindl.ensure((size_t)nblk * 4))) return rc;
  hipLaunchKernelGGL(bm25_blk_mindl_kernel, dim3((unsigned)ceil_div(nblk, 256)), dim3(256), 0, h->stream,
                     h->dl.as<int32_t>(), h->ndocs, nblk, h->blk_mindl.as<int32_t>());
  CM_HIP(hipGetLastError());
  if (h->nhead) {
    if ((rc = h->head_maxtf.ensure((size_t)h->nhead * nr)) || (rc = h->blk_maxtf.ensure((size_t)h->nhead * nblk)))
      return rc;
    hipLaunchKernelGGL(bm25_head_max_kernel, dim3((unsigned)ceil_div((int64_t)h->nhead * nr * 64, 256)), dim3(256), 0,
                       h->stream, h->headtf.as<uint8_t>(), h->npad, (int)nr, h->nhead, h->head_maxtf.as<uint8_t>());
    CM_HIP(hipGetLastError());
    hipLaunchKernelGGL(bm25_blk_max_kernel, dim3((unsigned)ceil_div((int64_t)h->nhead * nblk, 256)), dim3(256), 0,
                       h->stream, h->headtf.as<uint8_t>(), h->npad, nblk, h->nhead, h->blk_maxtf.as<uint8_t>());
    CM_HIP(hipGetLastError());
    // the ratio bound per (head, block) at 1.05 x the current avgdl (the ratio grows with avgdl, so
    // it also bounds searches whose avgdl is somewhat larger: other shards' global statistics)
    h->maxr_avgdl = h->avgdl > 0.0 ? h->avgdl * 1.05 : 0.0;
    if (h->maxr_avgdl > 0.0) {
      if ((rc = h->blk_maxr.ensure((size_t)h->nhead * nblk)) || (rc = h->blk16_maxr.ensure((size_t)h->nhead * nblk * 4)))
        return rc;
      hipLaunchKernelGGL(bm25_blk_maxratio_kernel, dim3((unsigned)ceil_div((int64_t)h->nhead * nblk, 256)),
                         dim3(256), 0, h->stream, h->headtf.as<uint8_t>(), h->npad, h->dl.as<int32_t>(), h->ndocs,
                         nblk, h->nhead, h->maxr_avgdl, h->blk_maxr.as<uint8_t>(), 64);
      CM_HIP(hipGetLastError());
      hipLaunchKernelGGL(bm25_blk_maxratio_kernel, dim3((unsigned)ceil_div((int64_t)h->nhead * nblk * 4, 256)),
                         dim3(256), 0, h->stream, h->headtf.as<uint8_t>(), h->npad, h->dl.as<int32_t>(), h->ndocs,
                         nblk * 4, h->nhead, h->maxr_avgdl, h->blk16_maxr.as<uint8_t>(), 16);
      CM_HIP(hipGetLastError());
    }
  }
  CM_HIP(hipStreamSynchronize(h->stream));
  return CM_OK;
}

// CM_BM25_DEBUG (ablation only): K2 bit0 skip scoring, bit1 skip the per-range top-k; bit2 full
// scan instead of the pruned search; K2a bit4 skip candidate scoring, bit5 skip the ranking,
// bit6 no head tf gathers, bit7 no ownership searches, bit8 no tail tf searches, bit9 no dl/live.
// Timing ablations are compiled only into -DCM_ABLATION builds (tools/build_variant.sh); the
// product library ignores CM_BM25_DEBUG, so no bench line can come from a disabled kernel.
#ifdef CM_ABLATION
int bm25_debug_flags() {  // re-read per call so one probe process can sweep the bits
  const char *e = getenv("CM_BM25_DEBUG");
  return e ? atoi(e) : 0;
}
#else
int bm25_debug_flags() { return 0; }
#endif

struct BmWs {
  unsigned long long *thr;
  double *lut;
  double *q_idf;
  int64_t *bounds;
  uint64_t *cand_key;
  uint32_t *cand_row;
  uint8_t *need;  // [query groups][ranges] re-score bits (pruned search)
  uint64_t *items;  // K2b work items (pruned search)
  uint64_t *items_sm;  // per item: its planned 16-doc sub-blocks (bit 4 b + x)
  uint8_t *qcand;   // per query term: postings walked
  int32_t *qd_code;  // [nq][kTermLanes] K2b term descriptors (bm25_qcand_kernel)
  double *qd_idf;
  int32_t *qd_tb;
  int32_t *qd_len;
  int32_t *qd_term;
  uint32_t *item_count;
  double *avgdl;    // the search's avgdl (unfiltered, host-computed or device-computed statistics)
  int64_t *stats;   // filtered entry: {Nc, sum of candidate lengths}
  int64_t *df;      // filtered entry: candidate df per query term
  size_t total;
};

BmWs bm_ws_layout(const cm_bm25 *h, int nq, int total_terms, int k, void *base) {
  BmWs w{};
  char *p = reinterpret_cast<char *>(base);
  const int64_t nr = std::max<int64_t>(1, ceil_div(h->ndocs, kRange));
  size_t off = 0;
  w.thr = reinterpret_cast<unsigned long long *>(p + off);
  off += round_up((int64_t)std::max(nq, 1) * 8, 256);
  w.lut = reinterpret_cast<double *>(p + off);
  off += round_up((int64_t)kLutW * kLutTF * 8, 256);
  w.q_idf = reinterpret_cast<double *>(p + off);
  off += round_up((int64_t)std::max(total_terms, 1) * 8, 256);
  w.bounds = reinterpret_cast<int64_t *>(p + off);
  off += round_up((int64_t)std::max(total_terms, 1) * (nr + 1) * 8, 256);
  const int64_t n_slots = lheads_total(nq, nr) + (int64_t)nq * nr * (k - 1);
  w.cand_key = reinterpret_cast<uint64_t *>(p + off);
  off += round_up(n_slots * 8, 256);
  w.cand_row = reinterpret_cast<uint32_t *>(p + off);
  off += round_up(n_slots * 4, 256);
  w.need = reinterpret_cast<uint8_t *>(p + off);
  off += round_up(ceil_div(std::max(nq, 1), kQPerWave) * nr, 256);
  w.items = reinterpret_cast<uint64_t *>(p + off);  // at most one item per (query, range)
  off += round_up((int64_t)std::max(nq, 1) * nr * 8, 256);
  w.items_sm = reinterpret_cast<uint64_t *>(p + off);
  off += round_up((int64_t)std::max(nq, 1) * nr * 8, 256);
  w.item_count = reinterpret_cast<uint32_t *>(p + off);
  off += 256;
  w.qcand = reinterpret_cast<uint8_t *>(p + off);
  off += round_up(std::max(total_terms, 1), 256);
  w.avgdl = reinterpret_cast<double *>(p + off);
  off += 256;
  w.stats = reinterpret_cast<int64_t *>(p + off);
  off += 256;
  w.df = reinterpret_cast<int64_t *>(p + off);
  off += round_up((int64_t)std::max(total_terms, 1) * 8, 256);
  w.qd_code = reinterpret_cast<int32_t *>(p + off);
  off += round_up((int64_t)std::max(nq, 1) * kTermLanes * 4, 256);
  w.qd_idf = reinterpret_cast<double *>(p + off);
  off += round_up((int64_t)std::max(nq, 1) * kTermLanes * 8, 256);
  w.qd_tb = reinterpret_cast<int32_t *>(p + off);
  off += round_up((int64_t)std::max(nq, 1) * 4, 256);
  w.qd_len = reinterpret_cast<int32_t *>(p + off);
  off += round_up((int64_t)std::max(nq, 1) * 4, 256);
  w.qd_term = reinterpret_cast<int32_t *>(p + off);
  off += round_up((int64_t)std::max(nq, 1) * kTermLanes * 4, 256);
  w.total = off;
  return w;
}

#ifndef K2A_RPW
#define K2A_RPW 4  // K2a ranges per wave (<= kMaxRangesPerWave): 16 -> 4 measured -9 % (CM_ABLATION builds)
#endif
#ifndef K2B_GRID
#define K2B_GRID 2048  // K2b workgroups (grid-stride over the planned items)
#endif
// Launch K2 + merge given q_idf and *avgdl already in the workspace.
int bm25_launch_core(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int nq, int total_terms, int k,
                     const uint32_t *allow_dev, const BmWs &w, double *score_dev, int64_t *row_dev, hipStream_t st,
                     hipEvent_t gate = nullptr) {
  int rc;
  const double *avgdl = w.avgdl;
  const int nr = (int)std::max<int64_t>(1, ceil_div(h->ndocs, kRange));
  if (nr > kMergePer * kMergeThreads) CM_FAIL(CM_EUNSUPPORTED, "BM25 shard too large (> 16.7M docs)");
  const int ngroups = (nr + 1 + kBoundsGroup - 1) / kBoundsGroup;
  const int64_t nb = (int64_t)total_terms * ngroups;
  const bool prune = h->path != 1 && !(bm25_debug_flags() & 4);
  if (nq > 0) {  // also for batches without terms: K2a and K2b read the per-query descriptors
    hipLaunchKernelGGL(bm25_qcand_kernel, dim3((unsigned)ceil_div(nq, 256)), dim3(256), 0, st, q_terms_dev, q_off_dev,
                       nq, h->vocab, h->nhead ? h->head_id.as<int32_t>() : (const int32_t *)nullptr,
                       h->term_off.as<int64_t>(), (int)prune, w.qcand, w.q_idf, prune ? w.qd_code : nullptr,
                       w.qd_idf, w.qd_tb, w.qd_len, w.qd_term);
    CM_HIP(hipGetLastError());
  }
  if (nb > 0) {
    hipLaunchKernelGGL(bm25_bounds_kernel, dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, st, q_terms_dev,
                       total_terms, h->vocab, nr, h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(), w.qcand,
                       w.bounds);
    CM_HIP(hipGetLastError());
  }
  CM_HIP(hipMemsetAsync(w.thr, 0xff, (size_t)nq * 8, st));  // no threshold yet
  if (prune && nq > 0 && env_knob("CM_BM25_TSEED", true)) {   // K2s: a seeded T for the tail pass
    hipLaunchKernelGGL(bm25_tseed_kernel, dim3((unsigned)nq), dim3(kSeedThreads), 0, st, nq, k, w.qd_code,
                       w.qd_idf, w.qd_len, w.qd_term, h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(),
                       h->post_tf.as<uint16_t>(), h->headtf.as<uint8_t>(), h->npad, h->dl.as<int32_t>(),
                       h->live.as<uint32_t>(), allow_dev, avgdl, w.thr);
    CM_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(bm25_lut_kernel, dim3(kLutW * kLutTF / 256), dim3(256), 0, st, (const double *)avgdl, h->lut_dmin,
                     w.lut);
  CM_HIP(hipGetLastError());
  // ranges per wave: enough waves to fill 256 CUs many times over, long runs otherwise
  const int64_t nqg = ceil_div(nq, kQPerWave);
  const int rpw = (int)std::min<int64_t>(kMaxRangesPerWave, std::max<int64_t>(1, nqg * nr / (256 * 4 * 24)));
  const int64_t nwaves = nqg * ceil_div(nr, rpw);
  const int64_t nblk = ceil_div(nwaves, kBmThreads / 64);
  // K2a's own run length (a multiple of its super-range when possible): shorter runs -> more,
  // shorter waves (better balance of the Zipf-skewed work at the end of the grid)
  const int rpw_a = std::max(1, std::min(rpw, (int)K2A_RPW));
  const int64_t nblk_a = ceil_div(nqg * ceil_div(nr, rpw_a), kBmThreads / 64);
  if (nblk > INT32_MAX || nblk_a > INT32_MAX) CM_FAIL(CM_EUNSUPPORTED, "BM25 batch too large");
  const int32_t *head_id = h->nhead ? h->head_id.as<int32_t>() : (const int32_t *)nullptr;
  // the gate: the preparation above (descriptors, postings bounds, seeded threshold) overlaps the
  // caller's producer kernels; the scoring kernels wait for it (cm_bm25_search_dev_gated)
  if (gate) CM_HIP(hipStreamWaitEvent(st, gate, 0));
  h->timer.begin(st);  // the search's dominant scoring kernel: K2a (pruned) or K2 (full)
  if (prune) {
    // K2a: exact scores of the tail candidates -> per-range lists; merged lists give each
    // query's k-th best tail score, against which the head-only bound marks the pairs
    // K2 must re-score (cm_bm25_prune.inc)
    hipLaunchKernelGGL(bm25_tail_kernel<uint16_t>, dim3((unsigned)nblk_a), dim3(kBmThreads), 0, st, q_terms_dev,
                       q_off_dev, nq, h->vocab, w.q_idf, w.bounds, nr, rpw_a, h->post_doc.as<int32_t>(),
                       h->post_tf.as<uint16_t>(), head_id, h->headtf.as<uint8_t>(), h->npad, h->dl.as<int32_t>(),
                       h->live.as<uint32_t>(), allow_dev, avgdl, k, w.cand_key, w.cand_row, w.thr, w.need, w.qd_code,
                       w.qd_term, w.qd_idf, w.qd_tb, w.qd_len,
                       (h->nhead && h->maxr_avgdl > 0.0) ? h->blk_maxr.as<uint8_t>() : (const uint8_t *)nullptr,
                       h->nhead ? h->blk_maxtf.as<uint8_t>() : (const uint8_t *)nullptr, h->blk_mindl.as<int32_t>(),
                       h->maxr_avgdl, (int64_t)nr * (kRange / 64),
                       h->nhead ? h->head_maxtf.as<uint8_t>() : (const uint8_t *)nullptr, h->range_mindl.as<int32_t>(),
                       bm25_debug_flags(),
                       (h->nhead && h->maxr_avgdl > 0.0) ? h->blk16_maxr.as<uint8_t>() : (const uint8_t *)nullptr);
    h->timer.end(st);
    CM_HIP(hipGetLastError());
    if ((rc = launch_bm25_merge(w.cand_key, w.cand_row, nq, nr, k, score_dev, row_dev, st))) return rc;
    CM_HIP(hipMemsetAsync(w.item_count, 0, 4, st));
    hipLaunchKernelGGL(bm25_plan_kernel, dim3((unsigned)ceil_div(nqg * nr, 256)), dim3(256), 0, st, w.qd_code,
                       w.qd_idf, w.qd_len, nq, (int)(head_id != nullptr), h->head_maxtf.as<uint8_t>(),
                       h->range_mindl.as<int32_t>(), h->blk_maxtf.as<uint8_t>(), h->blk_mindl.as<int32_t>(),
                       (h->nhead && h->maxr_avgdl > 0.0) ? h->blk_maxr.as<uint8_t>() : (const uint8_t *)nullptr,
                       h->maxr_avgdl, nr, (int64_t)nr * (kRange / 64), avgdl, k, score_dev, row_dev, w.need, w.items,
                       w.item_count,
                       (h->nhead && h->maxr_avgdl > 0.0 && !env_knob("CM_BM25_SUB16_OFF", false))
                           ? h->blk16_maxr.as<uint8_t>() : (const uint8_t *)nullptr,
                       w.items_sm);
    CM_HIP(hipGetLastError());
    // K2b: head-only documents of the planned blocks, merged into the tail pass's lists
    h->timer_b.begin(st);
    hipLaunchKernelGGL(bm25_block_kernel, dim3(K2B_GRID), dim3(256), 0, st, w.items, w.item_count, w.qd_code,
                       w.qd_idf, w.qd_tb, w.bounds, nr, h->post_doc.as<int32_t>(), h->headtf.as<uint8_t>(), h->npad,
                       h->dl.as<int32_t>(), h->live.as<uint32_t>(), allow_dev, h->ndocs, avgdl, k, score_dev, nq,
                       w.cand_key, w.cand_row, w.items_sm);
    h->timer_b.end(st);
    CM_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(bm25_range_kernel<uint16_t>, dim3((unsigned)nblk), dim3(kBmThreads), 0, st, q_terms_dev,
                     q_off_dev, nq, w.q_idf, w.bounds, nr, rpw, h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(),
                     h->post_tf.as<uint16_t>(), head_id, h->headtf.as<uint8_t>(), h->npad, h->dl.as<int32_t>(),
                     h->live.as<uint32_t>(), allow_dev, h->ndocs, avgdl, w.lut, h->lut_dmin, k, w.cand_key,
                     w.cand_row, w.thr, prune ? (const uint8_t *)w.need : (const uint8_t *)nullptr, h->vocab,
                     bm25_debug_flags());
  if (!prune) h->timer.end(st);
  CM_HIP(hipGetLastError());
  return launch_bm25_merge(w.cand_key, w.cand_row, nq, nr, k, score_dev, row_dev, st);
}

// (query, range) pairs re-scored after the tail pass by the pruned search that last used this
// workspace: whole ranges (K2) plus ranges with planned blocks (K2b).
int32_t count_rescored(cm_bm25 *h, int nq, const BmWs &w, hipStream_t st) {
  const int64_t nr = std::max<int64_t>(1, ceil_div(h->ndocs, kRange));
  const int64_t n = ceil_div(std::max(nq, 1), kQPerWave) * nr;
  std::vector<uint8_t> v((size_t)n);
  uint32_t items = 0;
  if (hipMemcpyAsync(v.data(), w.need, (size_t)n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&items, w.item_count, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return -1;
  int64_t c = items;
  for (uint8_t b : v) c += __builtin_popcount(b);
  return (int32_t)std::min<int64_t>(c, INT32_MAX);
}

void bm25_free(cm_bm25 *h) {
  for (DevBuf *b : {&h->term_off, &h->post_doc, &h->post_tf, &h->post_pos, &h->dl, &h->live, &h->idf, &h->ws,
                    &h->qbuf, &h->obuf, &h->allow_buf, &h->tmp, &h->headtf, &h->head_id, &h->head_maxtf,
                    &h->range_mindl, &h->blk_maxtf, &h->blk_mindl, &h->blk_maxr, &h->blk16_maxr})
    b->release();
}

// Host-array search with k > kMaxTopK: full per-document scores (bm25_scatter_term_kernel, query
// term order), a stable radix sort by (score desc) over the documents in row order (ties keep the
// lower row first, zero scores pad in insertion order: quirk Q1), the first k candidates.
int bm25_search_full(cm_bm25 *h, const int32_t *q_terms, const int32_t *q_off, int nq, int k, const double *q_idf,
                     double avgdl, const uint32_t *allow_dev, int64_t n_cand, double *out_score, int64_t *out_row) {
  const int64_t n = std::max<int64_t>(h->ndocs, 1);
  int rc;
  size_t tmp_bytes = 0;
  CM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                            (const int32_t *)nullptr, (int32_t *)nullptr, (int)n, 0, 64, h->stream));
  const size_t off1 = round_up((int64_t)tmp_bytes, 256);
  const size_t need = off1 + (size_t)round_up(n * 8, 256) * 3 + (size_t)round_up(n * 4, 256) * 2;
  if ((rc = h->ws.ensure(need))) return rc;
  char *base = h->ws.as<char>();
  double *score = reinterpret_cast<double *>(base + off1);
  uint64_t *keys = reinterpret_cast<uint64_t *>(base + off1 + round_up(n * 8, 256));
  uint64_t *skeys = reinterpret_cast<uint64_t *>(base + off1 + 2 * round_up(n * 8, 256));
  int32_t *rows = reinterpret_cast<int32_t *>(base + off1 + 3 * round_up(n * 8, 256));
  int32_t *srows = rows + round_up(n * 4, 256) / 4;
  const int64_t kk = std::min<int64_t>(k, n_cand);
  std::vector<uint64_t> hk((size_t)std::max<int64_t>(kk, 1));
  std::vector<int32_t> hr((size_t)std::max<int64_t>(kk, 1));
  for (int i = 0; i < nq; ++i) {
    CM_HIP(hipMemsetAsync(score, 0, (size_t)n * 8, h->stream));
    for (int32_t j = q_off[i]; j < q_off[i + 1]; ++j) {
      const int32_t t = q_terms[j];
      if (t < 0 || t >= h->vocab || q_idf[j] == 0.0) continue;  // adds idf * ratio = +-0: no change
      int64_t lh[2];
      CM_HIP(hipMemcpyAsync(lh, h->term_off.as<int64_t>() + t, 16, hipMemcpyDeviceToHost, h->stream));
      CM_HIP(hipStreamSynchronize(h->stream));
      if (lh[1] <= lh[0]) continue;
      hipLaunchKernelGGL(bm25_scatter_term_kernel, dim3((unsigned)ceil_div(lh[1] - lh[0], 256)), dim3(256), 0,
                         h->stream, lh[0], lh[1], h->post_doc.as<int32_t>(), h->post_tf.as<uint16_t>(),
                         h->dl.as<int32_t>(), q_idf[j], avgdl, score);
      CM_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(bm25_score_keys_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, h->stream, score,
                       h->live.as<uint32_t>(), allow_dev, h->ndocs, keys, rows);
    CM_HIP(hipGetLastError());
    CM_HIP(hipcub::DeviceRadixSort::SortPairs(base, tmp_bytes, keys, skeys, rows, srows, (int)n, 0, 64, h->stream));
    if (kk > 0) {
      CM_HIP(hipMemcpyAsync(hk.data(), skeys, (size_t)kk * 8, hipMemcpyDeviceToHost, h->stream));
      CM_HIP(hipMemcpyAsync(hr.data(), srows, (size_t)kk * 4, hipMemcpyDeviceToHost, h->stream));
    }
    CM_HIP(hipStreamSynchronize(h->stream));
    for (int j = 0; j < k; ++j) {
      const bool ok = j < kk;
      out_score[(int64_t)i * k + j] = ok ? f64_unorder(~hk[j]) : 0.0;
      out_row[(int64_t)i * k + j] = ok ? (int64_t)hr[j] : -1;
    }
  }
  return CM_OK;
}

// rank_bm25's epsilon over a candidate set: 0.25 x the mean idf of the candidate vocabulary, summed
// in the terms' first-occurrence order (the reference's dict order), glibc logs, host fp64 adds.
// The per-term candidate df and first (doc, position) keys come from one device pass.
int filtered_eps(cm_bm25 *h, const uint32_t *allow_dev, int64_t n_cand, double *eps) {
  const int32_t V = h->vocab;
  int rc;
  if ((rc = h->obuf.ensure((size_t)std::max(V, 1) * 16))) return rc;
  int64_t *dfv = h->obuf.as<int64_t>();
  uint64_t *fkv = reinterpret_cast<uint64_t *>(h->obuf.as<char>() + (size_t)V * 8);
  hipLaunchKernelGGL(bm25_term_df_kernel, dim3((unsigned)V), dim3(256), 0, h->stream, (const int32_t *)nullptr, (int)V,
                     V, h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(), h->post_pos.as<uint32_t>(),
                     h->live.as<uint32_t>(), allow_dev, dfv, fkv);
  CM_HIP(hipGetLastError());
  std::vector<int64_t> dfh((size_t)V);
  std::vector<uint64_t> fkh((size_t)V);
  CM_HIP(hipMemcpyAsync(dfh.data(), dfv, (size_t)V * 8, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipMemcpyAsync(fkh.data(), fkv, (size_t)V * 8, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  std::vector<int32_t> order;
  for (int32_t t = 0; t < V; ++t)
    if (dfh[t] > 0) order.push_back(t);
  if (order.empty()) CM_FAIL(CM_EZERODIV, "float division by zero (candidate documents have no tokens)");
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return fkh[a] < fkh[b]; });
  double sum = 0.0;
  for (int32_t t : order) sum = sum + bm25_idf(n_cand, dfh[t]);
  *eps = 0.25 * (sum / (double)order.size());
  return CM_OK;
}

}  // namespace

extern "C" {

int cm_bm25_create(int device, cm_bm25 **out) {
  if (!out) CM_FAIL(CM_EINVAL, "out is NULL");
  *out = nullptr;
  DeviceGuard dg(device);
  if (!dg.ok) CM_FAIL(CM_EDEVICE, "cannot select device " + std::to_string(device));
  cm_bm25 *h = new cm_bm25();
  h->dev = device;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamDefault) != hipSuccess) {
    delete h;
    CM_FAIL(CM_EDEVICE, "hipStreamCreate failed");
  }
  *out = h;
  return CM_OK;
}

void cm_bm25_destroy(cm_bm25 *h) {
  if (!h) return;
  DeviceGuard dg(h->dev);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  bm25_free(h);
  h->timer.release();
  h->timer_b.release();
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int64_t cm_bm25_num_docs(cm_bm25 *h) { return h ? h->ndocs : -1; }
int64_t cm_bm25_num_postings(cm_bm25 *h) { return h ? h->npost : -1; }

int cm_bm25_stats(cm_bm25 *h, int64_t *n_live, int64_t *sum_len, double *avgdl, double *eps) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (n_live) *n_live = h->n_live;
  if (sum_len) *sum_len = h->sum_len;
  if (avgdl) *avgdl = h->avgdl;
  if (eps) *eps = h->eps;
  return CM_OK;
}

int cm_bm25_build(cm_bm25 *h, const int32_t *term_ids, const int64_t *doc_off, int64_t ndocs, int32_t vocab,
                  const uint8_t *live) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (ndocs < 0 || vocab < 0 || (ndocs > 0 && !doc_off)) CM_FAIL(CM_EINVAL, "bad arguments");
  if (ndocs >= (int64_t)INT32_MAX) CM_FAIL(CM_EINVAL, "too many docs for one shard");
  DeviceGuard dg(h->dev);
  const int64_t ntok = ndocs ? doc_off[ndocs] : 0;
  if (ntok > 0 && !term_ids) CM_FAIL(CM_EINVAL, "term_ids is NULL");
  for (int64_t d = 0; d < ndocs; ++d)
    if (doc_off[d + 1] < doc_off[d]) CM_FAIL(CM_EINVAL, "doc_off must be non-decreasing");
  for (int64_t p = 0; p < ntok; ++p)
    if (term_ids[p] < 0 || term_ids[p] >= vocab) CM_FAIL(CM_EINVAL, "term id out of range");
  // pass 1: df over live docs, first-occurrence order, lengths
  std::vector<int64_t> stamp((size_t)vocab, -1);
  std::vector<int32_t> df((size_t)vocab, 0), order;
  std::vector<int32_t> dlh((size_t)ndocs, 0);
  int64_t n_live = 0, sum_len = 0, npost = 0;
  for (int64_t d = 0; d < ndocs; ++d) {
    const int64_t b = doc_off[d], e = doc_off[d + 1];
    dlh[d] = (int32_t)(e - b);
    if (live && !live[d]) continue;
    n_live++;
    sum_len += e - b;
    for (int64_t p = b; p < e; ++p) {
      const int32_t t = term_ids[p];
      if (stamp[t] != d) {
        stamp[t] = d;
        if (df[t]++ == 0) order.push_back(t);
        npost++;
      }
    }
  }
  // pass 2: postings (sorted by doc within a term because docs are visited in order)
  std::vector<int64_t> toff((size_t)vocab + 1, 0);
  for (int32_t t = 0; t < vocab; ++t) toff[t + 1] = toff[t] + df[t];
  std::vector<int64_t> fill(toff.begin(), toff.end() - 1);
  std::vector<int32_t> pdoc((size_t)npost);
  std::vector<uint16_t> ptf((size_t)npost);
  std::vector<uint32_t> ppos((size_t)npost);
  std::vector<int32_t> tfc((size_t)vocab, 0);
  std::fill(stamp.begin(), stamp.end(), -1);
  std::vector<int32_t> distinct;
  std::vector<uint32_t> firstpos((size_t)vocab, 0);
  for (int64_t d = 0; d < ndocs; ++d) {
    if (live && !live[d]) continue;
    distinct.clear();
    const int64_t b = doc_off[d], e = doc_off[d + 1];
    for (int64_t p = b; p < e; ++p) {
      const int32_t t = term_ids[p];
      if (stamp[t] != d) {
        stamp[t] = d;
        tfc[t] = 0;
        firstpos[t] = (uint32_t)(p - b);
        distinct.push_back(t);
      }
      tfc[t]++;
    }
    for (int32_t t : distinct) {
      if (tfc[t] > 65535) CM_FAIL(CM_EUNSUPPORTED, "term frequency > 65535 in one chunk");
      const int64_t q = fill[t]++;
      pdoc[q] = (int32_t)d;
      ptf[q] = (uint16_t)tfc[t];
      ppos[q] = firstpos[t];
    }
  }
  // live bitmap
  const int64_t nw = std::max<int64_t>(1, ceil_div(ndocs, 32));
  std::vector<uint32_t> lb((size_t)nw, 0);
  for (int64_t d = 0; d < ndocs; ++d)
    if (!live || live[d]) lb[d >> 5] |= 1u << (d & 31);
  int rc;
  if ((rc = h->term_off.ensure(((size_t)vocab + 1) * 8)) || (rc = h->post_doc.ensure(std::max<int64_t>(npost, 1) * 4)) ||
      (rc = h->post_tf.ensure(std::max<int64_t>(npost, 1) * 2)) ||
      (rc = h->post_pos.ensure(std::max<int64_t>(npost, 1) * 4)) ||
      (rc = h->dl.ensure(std::max<int64_t>(ndocs, 1) * 4)) || (rc = h->live.ensure((size_t)nw * 4)))
    return rc;
  CM_HIP(hipMemcpyAsync(h->term_off.ptr, toff.data(), toff.size() * 8, hipMemcpyHostToDevice, h->stream));
  if (npost) {
    CM_HIP(hipMemcpyAsync(h->post_doc.ptr, pdoc.data(), (size_t)npost * 4, hipMemcpyHostToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(h->post_tf.ptr, ptf.data(), (size_t)npost * 2, hipMemcpyHostToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(h->post_pos.ptr, ppos.data(), (size_t)npost * 4, hipMemcpyHostToDevice, h->stream));
  }
  if (ndocs) CM_HIP(hipMemcpyAsync(h->dl.ptr, dlh.data(), (size_t)ndocs * 4, hipMemcpyHostToDevice, h->stream));
  CM_HIP(hipMemcpyAsync(h->live.ptr, lb.data(), (size_t)nw * 4, hipMemcpyHostToDevice, h->stream));
  h->ndocs = ndocs;
  h->npost = npost;
  h->vocab = vocab;
  h->n_live = n_live;
  h->sum_len = sum_len;
  if ((rc = compute_idf_table(h, df, order))) return rc;
  if ((rc = build_head_tiles(h, df))) return rc;
  CM_HIP(hipStreamSynchronize(h->stream));
  if (h->empty_vocab) CM_FAIL(CM_EZERODIV, "float division by zero (every live document has an empty token list)");
  return CM_OK;
}

int cm_bm25_build_dev(cm_bm25 *h, const int32_t *term_ids_dev, const int64_t *doc_off_dev, int64_t ndocs,
                      int64_t ntokens, int32_t vocab, void *stream) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (ndocs <= 0 || ntokens < 0 || vocab <= 0) CM_FAIL(CM_EINVAL, "bad arguments");
  if (ndocs >= (int64_t)INT32_MAX) CM_FAIL(CM_EINVAL, "too many docs for one shard");
  DeviceGuard dg(h->dev);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch default)
  int rc;
  // scratch: keys in/out (u64), pos in/out (u32), flags
  DevBuf keys_a, keys_b, pos_a, pos_b, ukeys, counts, runstart, nruns_d, flags, df_d, cub_tmp, firstk;
  auto cleanup = [&]() {
    for (DevBuf *b : {&keys_a, &keys_b, &pos_a, &pos_b, &ukeys, &counts, &runstart, &nruns_d, &flags, &df_d, &cub_tmp,
                      &firstk})
      b->release();
  };
  const size_t nt = (size_t)std::max<int64_t>(ntokens, 1);
  if ((rc = keys_a.ensure(nt * 8)) || (rc = keys_b.ensure(nt * 8)) || (rc = pos_a.ensure(nt * 4)) ||
      (rc = pos_b.ensure(nt * 4)) || (rc = flags.ensure(16)) || (rc = h->dl.ensure((size_t)ndocs * 4))) {
    cleanup();
    return rc;
  }
  CM_HIP(hipMemsetAsync(flags.ptr, 0, 16, st));
  hipLaunchKernelGGL(bm25_token_keys_kernel, dim3((unsigned)ceil_div(ndocs, 4)), dim3(256), 0, st, term_ids_dev,
                     doc_off_dev, ndocs, keys_a.as<uint64_t>(), pos_a.as<uint32_t>(), h->dl.as<int32_t>(),
                     flags.as<int32_t>());
  CM_HIP(hipGetLastError());
  int tbits = 1;
  while ((1ll << tbits) < (int64_t)vocab) ++tbits;
  hipcub::DoubleBuffer<uint64_t> kbuf(keys_a.as<uint64_t>(), keys_b.as<uint64_t>());
  hipcub::DoubleBuffer<uint32_t> vbuf(pos_a.as<uint32_t>(), pos_b.as<uint32_t>());
  size_t tmp_bytes = 0;
  CM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kbuf, vbuf, ntokens, 0, 32 + tbits, st));
  if ((rc = cub_tmp.ensure(tmp_bytes))) {
    cleanup();
    return rc;
  }
  CM_HIP(hipcub::DeviceRadixSort::SortPairs(cub_tmp.ptr, tmp_bytes, kbuf, vbuf, ntokens, 0, 32 + tbits, st));
  uint64_t *sk = kbuf.Current();
  uint32_t *sp = vbuf.Current();
  // runs of equal (term, doc): unique keys + counts; reuse the free buffers
  uint64_t *uk = kbuf.Alternate();
  int32_t *cnt = reinterpret_cast<int32_t *>(vbuf.Alternate());
  if ((rc = nruns_d.ensure(8))) {
    cleanup();
    return rc;
  }
  size_t tmp2 = 0;
  CM_HIP(hipcub::DeviceRunLengthEncode::Encode(nullptr, tmp2, sk, uk, cnt, nruns_d.as<int64_t>(), ntokens, st));
  if (tmp2 > cub_tmp.bytes) {
    cub_tmp.release();
    if ((rc = cub_tmp.ensure(tmp2))) {
      cleanup();
      return rc;
    }
  }
  CM_HIP(hipcub::DeviceRunLengthEncode::Encode(cub_tmp.ptr, tmp2, sk, uk, cnt, nruns_d.as<int64_t>(), ntokens, st));
  int64_t nruns = 0;
  int32_t hflags[2] = {0, 0};
  CM_HIP(hipMemcpyAsync(&nruns, nruns_d.ptr, 8, hipMemcpyDeviceToHost, st));
  CM_HIP(hipMemcpyAsync(hflags, flags.ptr, 8, hipMemcpyDeviceToHost, st));
  CM_HIP(hipStreamSynchronize(st));
  if (hflags[0]) {
    cleanup();
    CM_FAIL(CM_EINVAL, "term id out of range");
  }
  if ((rc = runstart.ensure((size_t)std::max<int64_t>(nruns, 1) * 8))) {
    cleanup();
    return rc;
  }
  // run_start = exclusive scan of counts (as int64)
  {
    size_t tmp3 = 0;
    auto in = hipcub::TransformInputIterator<int64_t, hipcub::CastOp<int64_t>, int32_t *>(cnt, hipcub::CastOp<int64_t>());
    CM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp3, in, runstart.as<int64_t>(), nruns, st));
    if (tmp3 > cub_tmp.bytes) {
      cub_tmp.release();
      if ((rc = cub_tmp.ensure(tmp3))) {
        cleanup();
        return rc;
      }
    }
    CM_HIP(hipcub::DeviceScan::ExclusiveSum(cub_tmp.ptr, tmp3, in, runstart.as<int64_t>(), nruns, st));
  }
  if ((rc = h->post_doc.ensure((size_t)std::max<int64_t>(nruns, 1) * 4)) ||
      (rc = h->post_tf.ensure((size_t)std::max<int64_t>(nruns, 1) * 2)) ||
      (rc = h->post_pos.ensure((size_t)std::max<int64_t>(nruns, 1) * 4)) ||
      (rc = h->term_off.ensure(((size_t)vocab + 1) * 8))) {
    cleanup();
    return rc;
  }
  if (nruns == 0) CM_HIP(hipMemsetAsync(h->term_off.ptr, 0, ((size_t)vocab + 1) * 8, st));
  hipLaunchKernelGGL(bm25_postings_from_runs_kernel, dim3((unsigned)ceil_div(std::max<int64_t>(nruns, 1), 256)),
                     dim3(256), 0, st, uk, cnt, runstart.as<int64_t>(), sp, nruns, h->post_doc.as<int32_t>(),
                     h->post_tf.as<uint16_t>(), h->post_pos.as<uint32_t>(), h->term_off.as<int64_t>(), vocab,
                     flags.as<int32_t>() + 1);
  CM_HIP(hipGetLastError());
  const int64_t nw = std::max<int64_t>(1, ceil_div(ndocs, 32));
  if ((rc = h->live.ensure((size_t)nw * 4)) || (rc = firstk.ensure((size_t)vocab * 8))) {
    cleanup();
    return rc;
  }
  hipLaunchKernelGGL(set_all_bits_kernel, dim3((unsigned)ceil_div(nw, 256)), dim3(256), 0, st, h->live.as<uint32_t>(),
                     ndocs);
  hipLaunchKernelGGL(first_key_kernel, dim3((unsigned)ceil_div(vocab, 256)), dim3(256), 0, st,
                     h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(), h->post_pos.as<uint32_t>(), vocab,
                     firstk.as<uint64_t>());
  CM_HIP(hipGetLastError());
  std::vector<int32_t> df((size_t)vocab);
  std::vector<int64_t> toff_h((size_t)vocab + 1);
  std::vector<uint64_t> fk((size_t)vocab);
  CM_HIP(hipMemcpyAsync(toff_h.data(), h->term_off.ptr, ((size_t)vocab + 1) * 8, hipMemcpyDeviceToHost, st));
  CM_HIP(hipMemcpyAsync(fk.data(), firstk.ptr, (size_t)vocab * 8, hipMemcpyDeviceToHost, st));
  CM_HIP(hipMemcpyAsync(hflags, flags.ptr, 8, hipMemcpyDeviceToHost, st));
  CM_HIP(hipStreamSynchronize(st));
  cleanup();
  for (int32_t t = 0; t < vocab; ++t) df[t] = (int32_t)(toff_h[t + 1] - toff_h[t]);
  if (hflags[1]) CM_FAIL(CM_EUNSUPPORTED, "term frequency > 65535 in one chunk");
  std::vector<int32_t> order;
  order.reserve((size_t)vocab);
  for (int32_t t = 0; t < vocab; ++t)
    if (df[t] > 0) order.push_back(t);
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return fk[a] < fk[b]; });
  h->ndocs = ndocs;
  h->npost = nruns;
  h->vocab = vocab;
  h->n_live = ndocs;
  h->sum_len = ntokens;
  if ((rc = compute_idf_table(h, df, order))) return rc;
  if ((rc = build_head_tiles(h, df))) return rc;
  CM_HIP(hipStreamSynchronize(h->stream));
  if (h->empty_vocab) CM_FAIL(CM_EZERODIV, "float division by zero (every live document has an empty token list)");
  return CM_OK;
}

int cm_bm25_term_stats(cm_bm25 *h, int32_t *df_out, uint64_t *first_out) {
  if (!h || !df_out || !first_out) CM_FAIL(CM_EINVAL, "NULL argument");
  if (h->vocab <= 0) return CM_OK;
  DeviceGuard dg(h->dev);
  const int32_t V = h->vocab;
  int rc;
  if ((rc = h->obuf.ensure((size_t)V * 16))) return rc;
  uint64_t *fk = h->obuf.as<uint64_t>();
  hipLaunchKernelGGL(first_key_kernel, dim3((unsigned)ceil_div(V, 256)), dim3(256), 0, h->stream,
                     h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(), h->post_pos.as<uint32_t>(), V, fk);
  CM_HIP(hipGetLastError());
  std::vector<int64_t> off((size_t)V + 1);
  CM_HIP(hipMemcpyAsync(off.data(), h->term_off.ptr, ((size_t)V + 1) * 8, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipMemcpyAsync(first_out, fk, (size_t)V * 8, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  for (int32_t t = 0; t < V; ++t) df_out[t] = (int32_t)(off[t + 1] - off[t]);
  return CM_OK;
}

int cm_bm25_export(cm_bm25 *h, int64_t *term_off, int32_t *post_doc, uint16_t *post_tf, uint32_t *post_pos,
                   int32_t *dl) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  DeviceGuard dg(h->dev);
  if (term_off) CM_HIP(hipMemcpyAsync(term_off, h->term_off.ptr, ((size_t)h->vocab + 1) * 8, hipMemcpyDeviceToHost, h->stream));
  if (h->npost) {
    if (post_doc) CM_HIP(hipMemcpyAsync(post_doc, h->post_doc.ptr, (size_t)h->npost * 4, hipMemcpyDeviceToHost, h->stream));
    if (post_tf) CM_HIP(hipMemcpyAsync(post_tf, h->post_tf.ptr, (size_t)h->npost * 2, hipMemcpyDeviceToHost, h->stream));
    if (post_pos) CM_HIP(hipMemcpyAsync(post_pos, h->post_pos.ptr, (size_t)h->npost * 4, hipMemcpyDeviceToHost, h->stream));
  }
  if (dl && h->ndocs) CM_HIP(hipMemcpyAsync(dl, h->dl.ptr, (size_t)h->ndocs * 4, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  return CM_OK;
}

int cm_bm25_set_head_policy(cm_bm25 *h, double min_df_frac, int64_t max_bytes) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (!(min_df_frac >= 0.0) || max_bytes < 0) CM_FAIL(CM_EINVAL, "bad head policy");
  DeviceGuard dg(h->dev);
  h->head_min_frac = min_df_frac;
  h->head_max_bytes = max_bytes;
  if (h->vocab <= 0) return CM_OK;
  std::vector<int64_t> off((size_t)h->vocab + 1);
  CM_HIP(hipMemcpyAsync(off.data(), h->term_off.ptr, off.size() * 8, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  std::vector<int32_t> df((size_t)h->vocab);
  for (int32_t t = 0; t < h->vocab; ++t) df[t] = (int32_t)(off[t + 1] - off[t]);
  return build_head_tiles(h, df);
}

int32_t cm_bm25_num_head_terms(cm_bm25 *h) { return h ? h->nhead : -1; }

int cm_bm25_set_path(cm_bm25 *h, int32_t kind) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (kind < 0 || kind > 2) CM_FAIL(CM_EINVAL, "BM25 path must be 0 (auto), 1 (full scan) or 2 (pruned)");
  h->path = kind;
  return CM_OK;
}

int32_t cm_bm25_workspace_rescored(cm_bm25 *h, int32_t nq, int32_t total_terms, int32_t k, const void *workspace_dev) {
  if (!h || !workspace_dev || nq <= 0 || k <= 0) return -1;
  if (h->path == 1) return -1;
  DeviceGuard dg(h->dev);
  const BmWs w = bm_ws_layout(h, nq, total_terms, k, const_cast<void *>(workspace_dev));
  return count_rescored(h, nq, w, h->stream);
}

int32_t cm_bm25_last_rescored(cm_bm25 *h) { return h ? h->last_rescored : -1; }

int64_t cm_bm25_workspace_items(cm_bm25 *h, int32_t nq, int32_t total_terms, int32_t k, const void *workspace_dev,
                                uint64_t *items_out, int64_t cap) {
  if (!h || !workspace_dev || nq <= 0 || k <= 0 || cap < 0) return -1;
  if (h->path == 1) return -1;
  DeviceGuard dg(h->dev);
  const BmWs w = bm_ws_layout(h, nq, total_terms, k, const_cast<void *>(workspace_dev));
  uint32_t n = 0;
  if (hipMemcpyAsync(&n, w.item_count, 4, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
      hipStreamSynchronize(h->stream) != hipSuccess)
    return -1;
  const int64_t m = std::min<int64_t>(n, cap);
  if (m > 0 && items_out &&
      (hipMemcpyAsync(items_out, w.items, (size_t)m * 8, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
       hipStreamSynchronize(h->stream) != hipSuccess))
    return -1;
  return n;
}

int64_t cm_bm25_workspace_subblocks(cm_bm25 *h, int32_t nq, int32_t total_terms, int32_t k, const void *workspace_dev,
                                    uint64_t *masks_out, int64_t cap) {
  if (!h || !workspace_dev || nq <= 0 || k <= 0 || cap < 0) return -1;
  if (h->path == 1) return -1;
  DeviceGuard dg(h->dev);
  const BmWs w = bm_ws_layout(h, nq, total_terms, k, const_cast<void *>(workspace_dev));
  uint32_t n = 0;
  if (hipMemcpyAsync(&n, w.item_count, 4, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
      hipStreamSynchronize(h->stream) != hipSuccess)
    return -1;
  const int64_t m = std::min<int64_t>(n, cap);
  if (m > 0 && masks_out &&
      (hipMemcpyAsync(masks_out, w.items_sm, (size_t)m * 8, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
       hipStreamSynchronize(h->stream) != hipSuccess))
    return -1;
  return n;
}

int cm_bm25_timing(cm_bm25 *h, int32_t enable) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  h->timer.on = h->timer_b.on = enable != 0;
  h->timer.used = h->timer_b.used = 0;
  return CM_OK;
}

int32_t cm_bm25_timing_drain_block(cm_bm25 *h, float *ms_out, int32_t cap) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  DeviceGuard dg(h->dev);
  const int n = h->timer_b.drain(ms_out, cap);
  if (n < 0) CM_FAIL(CM_EDEVICE, "event query failed");
  return n;
}

int32_t cm_bm25_timing_drain(cm_bm25 *h, float *ms_out, int32_t cap) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  DeviceGuard dg(h->dev);
  const int n = h->timer.drain(ms_out, cap);
  if (n < 0) CM_FAIL(CM_EDEVICE, "event query failed");
  return n;
}

int cm_bm25_set_stats(cm_bm25 *h, const double *idf, int32_t vocab, int64_t n_live, int64_t sum_len, double eps) {
  if (!h || !idf) CM_FAIL(CM_EINVAL, "NULL argument");
  if (vocab != h->vocab) CM_FAIL(CM_EINVAL, "vocab mismatch");
  if (n_live <= 0 || sum_len <= 0) CM_FAIL(CM_EINVAL, "n_live and sum_len must be > 0");
  DeviceGuard dg(h->dev);
  h->idf_host.assign(idf, idf + vocab);
  h->n_live = n_live;
  h->sum_len = sum_len;
  h->avgdl = (double)sum_len / (double)n_live;
  h->eps = eps;
  h->empty_vocab = false;
  int rc = h->idf.ensure((size_t)std::max(vocab, 1) * 8);
  if (rc) return rc;
  CM_HIP(hipMemcpyAsync(h->idf.ptr, idf, (size_t)vocab * 8, hipMemcpyHostToDevice, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  return CM_OK;
}

int64_t cm_bm25_search_workspace(cm_bm25 *h, int32_t nq, int32_t total_terms, int32_t k) {
  if (!h || nq < 0 || total_terms < 0 || k <= 0) return -1;
  return (int64_t)bm_ws_layout(h, nq, total_terms, k, nullptr).total;
}

int cm_bm25_search_dev(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int32_t nq,
                       int32_t total_terms, int32_t k, double *score_dev, int64_t *row_dev, void *workspace_dev,
                       int64_t workspace_bytes, void *stream) {
  return cm_bm25_search_dev_gated(h, q_terms_dev, q_off_dev, nq, total_terms, k, score_dev, row_dev, workspace_dev,
                                  workspace_bytes, stream, nullptr);
}

int cm_bm25_search_dev_gated(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int32_t nq,
                             int32_t total_terms, int32_t k, double *score_dev, int64_t *row_dev, void *workspace_dev,
                             int64_t workspace_bytes, void *stream, void *gate_event) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (k <= 0 || k > kMaxTopK) CM_FAIL(CM_EINVAL, "k must be in [1, " + std::to_string(kMaxTopK) + "]");
  if (h->ndocs == 0) CM_FAIL(CM_EINVAL, "empty BM25 index");
  if (h->empty_vocab) CM_FAIL(CM_EZERODIV, "float division by zero");
  DeviceGuard dg(h->dev);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch default)
  BmWs w = bm_ws_layout(h, nq, total_terms, k, workspace_dev);
  if (!workspace_dev || (int64_t)w.total > workspace_bytes) CM_FAIL(CM_EINVAL, "bm25 workspace too small");
  if (total_terms > 0) {
    hipLaunchKernelGGL(bm25_qidf_kernel, dim3((unsigned)ceil_div(total_terms, 256)), dim3(256), 0, st, q_terms_dev,
                       total_terms, h->idf.as<double>(), h->vocab, w.q_idf);
    CM_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(bm25_set_f64_kernel, dim3(1), dim3(64), 0, st, h->avgdl, w.avgdl);
  CM_HIP(hipGetLastError());
  return bm25_launch_core(h, q_terms_dev, q_off_dev, nq, total_terms, k, nullptr, w, score_dev, row_dev, st,
                          (hipEvent_t)gate_event);
}

static int bm25_search_scored(cm_bm25 *h, const int32_t *q_terms, const int32_t *q_off, int32_t nq, int32_t total,
                              int32_t k, const uint32_t *allow_dev, const double *q_idf_host, double avgdl,
                              int64_t n_cand, double *out_score, int64_t *out_row, int32_t *out_n);

int cm_bm25_search(cm_bm25 *h, const int32_t *q_terms, const int32_t *q_off, int32_t nq, int32_t k,
                   const uint32_t *allow_bits, double *out_score, int64_t *out_row, int32_t *out_n) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (!q_off || !out_score || !out_row) CM_FAIL(CM_EINVAL, "NULL argument");
  if (k <= 0) CM_FAIL(CM_EINVAL, "k must be >= 1");
  const int32_t total = q_off[nq];
  if (total < 0 || (total > 0 && !q_terms)) CM_FAIL(CM_EINVAL, "bad q_off");
  for (int i = 0; i < nq; ++i)
    if (q_off[i + 1] < q_off[i]) CM_FAIL(CM_EINVAL, "q_off must be non-decreasing");
  DeviceGuard dg(h->dev);
  int rc;
  // candidate statistics
  int64_t n_cand = h->n_live, sum_len = h->sum_len;
  const uint32_t *allow_dev = nullptr;
  const int64_t nw = std::max<int64_t>(1, ceil_div(h->ndocs, 32));
  std::vector<double> q_idf((size_t)std::max(total, 1), 0.0);
  if (allow_bits) {
    if ((rc = h->allow_buf.ensure((size_t)nw * 4)) || (rc = h->tmp.ensure(16))) return rc;
    CM_HIP(hipMemcpyAsync(h->allow_buf.ptr, allow_bits, (size_t)nw * 4, hipMemcpyDefault, h->stream));  // host or device
    allow_dev = h->allow_buf.as<uint32_t>();
    CM_HIP(hipMemsetAsync(h->tmp.ptr, 0, 16, h->stream));
    hipLaunchKernelGGL(bm25_filtered_stats_kernel, dim3((unsigned)std::min<int64_t>(1024, ceil_div(nw, 256))),
                       dim3(256), 0, h->stream, h->dl.as<int32_t>(), h->live.as<uint32_t>(), allow_dev, h->ndocs,
                       h->tmp.as<unsigned long long>());
    CM_HIP(hipGetLastError());
    unsigned long long st2[2];
    CM_HIP(hipMemcpyAsync(st2, h->tmp.ptr, 16, hipMemcpyDeviceToHost, h->stream));
    CM_HIP(hipStreamSynchronize(h->stream));
    n_cand = (int64_t)st2[0];
    sum_len = (int64_t)st2[1];
  }
  if (n_cand == 0 || h->ndocs == 0) {
    for (int i = 0; i < nq; ++i) {
      if (out_n) out_n[i] = 0;
      for (int j = 0; j < k; ++j) {
        out_score[(int64_t)i * k + j] = 0.0;
        out_row[(int64_t)i * k + j] = -1;
      }
    }
    return CM_OK;
  }
  if (sum_len == 0) CM_FAIL(CM_EZERODIV, "float division by zero (candidate documents have no tokens)");
  double avgdl = (double)sum_len / (double)n_cand;
  if (!allow_bits) {
    for (int32_t i = 0; i < total; ++i) {
      const int32_t t = q_terms[i];
      q_idf[i] = (t >= 0 && t < h->vocab) ? h->idf_host[t] : 0.0;
    }
  } else {
    // filtered df of the distinct query terms
    std::vector<int32_t> uterms;
    for (int32_t i = 0; i < total; ++i)
      if (q_terms[i] >= 0 && q_terms[i] < h->vocab) uterms.push_back(q_terms[i]);
    std::sort(uterms.begin(), uterms.end());
    uterms.erase(std::unique(uterms.begin(), uterms.end()), uterms.end());
    std::vector<int64_t> udf(uterms.size(), 0);
    bool need_eps = false;
    if (!uterms.empty()) {
      const size_t nu = uterms.size();
      if ((rc = h->qbuf.ensure(nu * 4)) || (rc = h->obuf.ensure(nu * 8))) return rc;
      CM_HIP(hipMemcpyAsync(h->qbuf.ptr, uterms.data(), nu * 4, hipMemcpyHostToDevice, h->stream));
      hipLaunchKernelGGL(bm25_term_df_kernel, dim3((unsigned)nu), dim3(256), 0, h->stream, h->qbuf.as<int32_t>(),
                         (int)nu, h->vocab, h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(), h->post_pos.as<uint32_t>(),
                         h->live.as<uint32_t>(), allow_dev, h->obuf.as<int64_t>(), (uint64_t *)nullptr);
      CM_HIP(hipGetLastError());
      CM_HIP(hipMemcpyAsync(udf.data(), h->obuf.ptr, nu * 8, hipMemcpyDeviceToHost, h->stream));
      CM_HIP(hipStreamSynchronize(h->stream));
      for (size_t u = 0; u < nu; ++u)
        if (udf[u] > 0 && bm25_idf(n_cand, udf[u]) < 0) need_eps = true;
    }
    double eps = 0.0;
    if (need_eps && (rc = filtered_eps(h, allow_dev, n_cand, &eps))) return rc;
    for (int32_t i = 0; i < total; ++i) {
      const int32_t t = q_terms[i];
      if (t < 0 || t >= h->vocab) continue;
      const size_t u = std::lower_bound(uterms.begin(), uterms.end(), t) - uterms.begin();
      const int64_t d = udf[u];
      if (d <= 0) continue;  // not in the candidate vocabulary: idf.get -> None -> 0
      const double v = bm25_idf(n_cand, d);
      q_idf[i] = v < 0 ? eps : v;
    }
  }
  return bm25_search_scored(h, q_terms, q_off, nq, total, k, allow_dev, q_idf.data(), avgdl, n_cand, out_score,
                            out_row, out_n);
}

// The scoring half of the host-array search, given every query term's idf, the candidates' avgdl
// and count: the fused top-k lists (k <= kMaxTopK) or the full order.  allow_dev is device memory.
static int bm25_search_scored(cm_bm25 *h, const int32_t *q_terms, const int32_t *q_off, int32_t nq, int32_t total,
                              int32_t k, const uint32_t *allow_dev, const double *q_idf_host, double avgdl,
                              int64_t n_cand, double *out_score, int64_t *out_row, int32_t *out_n) {
  int rc;
  if (k > kMaxTopK) {  // beyond the fused top-k lists: full scores + one sort per query
    rc = bm25_search_full(h, q_terms, q_off, nq, k, q_idf_host, avgdl, allow_dev, n_cand, out_score, out_row);
    if (rc) return rc;
    if (out_n) {
      const int32_t nv = (int32_t)std::min<int64_t>(k, n_cand);
      for (int i = 0; i < nq; ++i) out_n[i] = nv;
    }
    h->last_rescored = -1;
    return CM_OK;
  }
  // device search
  const int64_t wsb = cm_bm25_search_workspace(h, nq, total, k);
  if ((rc = h->ws.ensure((size_t)wsb))) return rc;
  BmWs w = bm_ws_layout(h, nq, total, k, h->ws.ptr);
  const size_t qb = (size_t)std::max(total, 1) * 4 + (size_t)(nq + 1) * 4;
  if ((rc = h->qbuf.ensure(qb)) || (rc = h->obuf.ensure((size_t)nq * k * 16))) return rc;
  int32_t *d_terms = h->qbuf.as<int32_t>();
  int32_t *d_off = d_terms + std::max(total, 1);
  if (total > 0) CM_HIP(hipMemcpyAsync(d_terms, q_terms, (size_t)total * 4, hipMemcpyHostToDevice, h->stream));
  CM_HIP(hipMemcpyAsync(d_off, q_off, (size_t)(nq + 1) * 4, hipMemcpyHostToDevice, h->stream));
  if (total > 0) CM_HIP(hipMemcpyAsync(w.q_idf, q_idf_host, (size_t)total * 8, hipMemcpyHostToDevice, h->stream));
  double *d_score = h->obuf.as<double>();
  int64_t *d_row = reinterpret_cast<int64_t *>(d_score + (size_t)nq * k);
  hipLaunchKernelGGL(bm25_set_f64_kernel, dim3(1), dim3(64), 0, h->stream, avgdl, w.avgdl);
  CM_HIP(hipGetLastError());
  rc = bm25_launch_core(h, d_terms, d_off, nq, total, k, allow_dev, w, d_score, d_row, h->stream);
  if (rc) return rc;
  h->last_rescored = h->path == 1 ? -1 : count_rescored(h, nq, w, h->stream);
  CM_HIP(hipMemcpyAsync(out_score, d_score, (size_t)nq * k * 8, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipMemcpyAsync(out_row, d_row, (size_t)nq * k * 8, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  if (out_n) {
    const int32_t nv = (int32_t)std::min<int64_t>(k, n_cand);
    for (int i = 0; i < nq; ++i) out_n[i] = nv;
  }
  return CM_OK;
}

int cm_bm25_search_idf(cm_bm25 *h, const int32_t *q_terms, const int32_t *q_off, int32_t nq, int32_t k,
                       const uint32_t *allow_bits, const double *q_idf, double avgdl, int64_t n_cand,
                       double *out_score, int64_t *out_row, int32_t *out_n) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (!q_off || !out_score || !out_row) CM_FAIL(CM_EINVAL, "NULL argument");
  if (k <= 0) CM_FAIL(CM_EINVAL, "k must be >= 1");
  const int32_t total = q_off[nq];
  if (total < 0 || (total > 0 && (!q_terms || !q_idf))) CM_FAIL(CM_EINVAL, "bad q_off / NULL q_idf");
  for (int i = 0; i < nq; ++i)
    if (q_off[i + 1] < q_off[i]) CM_FAIL(CM_EINVAL, "q_off must be non-decreasing");
  if (n_cand < 0) CM_FAIL(CM_EINVAL, "n_cand must be >= 0");
  DeviceGuard dg(h->dev);
  if (n_cand == 0 || h->ndocs == 0) {
    for (int i = 0; i < nq; ++i) {
      if (out_n) out_n[i] = 0;
      for (int j = 0; j < k; ++j) {
        out_score[(int64_t)i * k + j] = 0.0;
        out_row[(int64_t)i * k + j] = -1;
      }
    }
    return CM_OK;
  }
  if (!(avgdl > 0.0)) CM_FAIL(CM_EZERODIV, "float division by zero (candidate documents have no tokens)");
  const uint32_t *allow_dev = nullptr;
  int rc;
  if (allow_bits) {
    const int64_t nw = std::max<int64_t>(1, ceil_div(h->ndocs, 32));
    if ((rc = h->allow_buf.ensure((size_t)nw * 4))) return rc;
    CM_HIP(hipMemcpyAsync(h->allow_buf.ptr, allow_bits, (size_t)nw * 4, hipMemcpyDefault, h->stream));  // host or device
    allow_dev = h->allow_buf.as<uint32_t>();
  }
  std::vector<double> qi((size_t)std::max(total, 1), 0.0);
  for (int32_t i = 0; i < total; ++i)
    qi[(size_t)i] = (q_terms[i] >= 0 && q_terms[i] < h->vocab) ? q_idf[i] : 0.0;
  return bm25_search_scored(h, q_terms, q_off, nq, total, k, allow_dev, qi.data(), avgdl, n_cand, out_score, out_row,
                            out_n);
}

int cm_bm25_prepare_filtered(cm_bm25 *h, int64_t max_docs) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (max_docs < 0 || max_docs >= (int64_t)1 << 40) CM_FAIL(CM_EINVAL, "bad max_docs");
  const int64_t n = std::max(max_docs, h->ndocs);
  if (n <= h->log_n) return CM_OK;
  DeviceGuard dg(h->dev);
  std::vector<double> L((size_t)n + 1);
  for (int64_t x = 0; x <= n; ++x) L[(size_t)x] = std::log((double)x + 0.5);  // glibc, as bm25_idf
  int rc = h->logtab.ensure(L.size() * 8);
  if (rc) return rc;
  CM_HIP(hipMemcpyAsync(h->logtab.ptr, L.data(), L.size() * 8, hipMemcpyHostToDevice, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  h->log_n = n;
  return CM_OK;
}

int cm_bm25_filter_stats_dev(cm_bm25 *h, const uint32_t *allow_dev, const int32_t *q_terms_dev, int32_t n_terms,
                             int64_t *stats_dev, int64_t *df_dev, void *stream) {
  if (!h || !allow_dev || !stats_dev || (n_terms > 0 && (!q_terms_dev || !df_dev))) CM_FAIL(CM_EINVAL, "NULL argument");
  if (n_terms < 0) CM_FAIL(CM_EINVAL, "n_terms must be >= 0");
  DeviceGuard dg(h->dev);
  hipStream_t st = (hipStream_t)stream;
  const int64_t nw = std::max<int64_t>(1, ceil_div(h->ndocs, 32));
  CM_HIP(hipMemsetAsync(stats_dev, 0, 16, st));
  if (h->ndocs > 0) {
    hipLaunchKernelGGL(bm25_filtered_stats_kernel, dim3((unsigned)std::min<int64_t>(1024, ceil_div(nw, 256))),
                       dim3(256), 0, st, h->dl.as<int32_t>(), h->live.as<uint32_t>(), allow_dev, h->ndocs,
                       reinterpret_cast<unsigned long long *>(stats_dev));
    CM_HIP(hipGetLastError());
  }
  if (n_terms > 0) {
    CM_HIP(hipMemsetAsync(df_dev, 0, (size_t)n_terms * 8, st));
    if (h->npost > 0) {
      // slices per term: enough blocks for a single query's few terms, one for big batches
      const unsigned sl = (unsigned)std::max(1, std::min(128, 4096 / n_terms));
      hipLaunchKernelGGL(bm25_term_df_kernel, dim3((unsigned)n_terms, sl), dim3(256), 0, st, q_terms_dev, (int)n_terms,
                         h->vocab, h->term_off.as<int64_t>(), h->post_doc.as<int32_t>(), h->post_pos.as<uint32_t>(),
                         h->live.as<uint32_t>(), allow_dev, df_dev, (uint64_t *)nullptr);
      CM_HIP(hipGetLastError());
    }
  }
  return CM_OK;
}

int cm_bm25_filter_term_stats_dev(cm_bm25 *h, const uint32_t *allow_dev, int64_t *df_dev, uint64_t *first_dev,
                                  void *stream) {
  if (!h || !allow_dev || !df_dev || !first_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (h->vocab <= 0) return CM_OK;
  DeviceGuard dg(h->dev);
  hipLaunchKernelGGL(bm25_term_df_kernel, dim3((unsigned)h->vocab), dim3(256), 0, (hipStream_t)stream,
                     (const int32_t *)nullptr, (int)h->vocab, h->vocab, h->term_off.as<int64_t>(),
                     h->post_doc.as<int32_t>(), h->post_pos.as<uint32_t>(), h->live.as<uint32_t>(), allow_dev, df_dev,
                     first_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int cm_bm25_filter_eps(cm_bm25 *h, const uint32_t *allow_bits, double *eps_out) {
  if (!h || !allow_bits || !eps_out) CM_FAIL(CM_EINVAL, "NULL argument");
  DeviceGuard dg(h->dev);
  int rc;
  const int64_t nw = std::max<int64_t>(1, ceil_div(h->ndocs, 32));
  if ((rc = h->allow_buf.ensure((size_t)nw * 4)) || (rc = h->tmp.ensure(16))) return rc;
  CM_HIP(hipMemcpyAsync(h->allow_buf.ptr, allow_bits, (size_t)nw * 4, hipMemcpyDefault, h->stream));
  CM_HIP(hipMemsetAsync(h->tmp.ptr, 0, 16, h->stream));
  hipLaunchKernelGGL(bm25_filtered_stats_kernel, dim3((unsigned)std::min<int64_t>(1024, ceil_div(nw, 256))), dim3(256),
                     0, h->stream, h->dl.as<int32_t>(), h->live.as<uint32_t>(), h->allow_buf.as<uint32_t>(), h->ndocs,
                     h->tmp.as<unsigned long long>());
  CM_HIP(hipGetLastError());
  unsigned long long st2[2];
  CM_HIP(hipMemcpyAsync(st2, h->tmp.ptr, 16, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  if (st2[0] == 0) {
    *eps_out = 0.0;
    return CM_OK;
  }
  return filtered_eps(h, h->allow_buf.as<uint32_t>(), (int64_t)st2[0], eps_out);
}

int cm_bm25_search_stats_dev(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int32_t nq,
                             int32_t total_terms, int32_t k, const uint32_t *allow_dev, const int64_t *stats_dev,
                             const int64_t *df_dev, const double *eps_dev, double *score_dev, int64_t *row_dev,
                             int32_t *status_dev, void *workspace_dev, int64_t workspace_bytes, void *stream) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (k <= 0 || k > kMaxTopK) CM_FAIL(CM_EINVAL, "k must be in [1, " + std::to_string(kMaxTopK) + "]");
  if (!stats_dev || !status_dev || (total_terms > 0 && !df_dev)) CM_FAIL(CM_EINVAL, "NULL argument");
  if (h->ndocs == 0) CM_FAIL(CM_EINVAL, "empty BM25 index");
  if (h->log_n < 0) CM_FAIL(CM_EINVAL, "cm_bm25_prepare_filtered was not called for this index");
  DeviceGuard dg(h->dev);
  hipStream_t st = (hipStream_t)stream;
  BmWs w = bm_ws_layout(h, nq, total_terms, k, workspace_dev);
  if (!workspace_dev || (int64_t)w.total > workspace_bytes) CM_FAIL(CM_EINVAL, "bm25 workspace too small");
  CM_HIP(hipMemsetAsync(status_dev, 0, 4, st));
  hipLaunchKernelGGL(bm25_stats_idf_kernel, dim3((unsigned)std::max<int64_t>(1, ceil_div(total_terms, 256))), dim3(256),
                     0, st, q_terms_dev, total_terms, h->vocab, stats_dev, df_dev, h->logtab.as<double>(), h->log_n,
                     eps_dev, w.q_idf, w.avgdl, status_dev);
  CM_HIP(hipGetLastError());
  return bm25_launch_core(h, q_terms_dev, q_off_dev, nq, total_terms, k, allow_dev, w, score_dev, row_dev, st);
}

int cm_bm25_search_filtered_dev(cm_bm25 *h, const int32_t *q_terms_dev, const int32_t *q_off_dev, int32_t nq,
                                int32_t total_terms, int32_t k, const uint32_t *allow_dev, const double *eps_dev,
                                double *score_dev, int64_t *row_dev, int32_t *status_dev, void *workspace_dev,
                                int64_t workspace_bytes, void *stream) {
  if (!h || !allow_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (nq <= 0) return CM_OK;
  BmWs w = bm_ws_layout(h, nq, total_terms, k, workspace_dev);
  if (!workspace_dev || (int64_t)w.total > workspace_bytes) CM_FAIL(CM_EINVAL, "bm25 workspace too small");
  int rc = cm_bm25_filter_stats_dev(h, allow_dev, q_terms_dev, total_terms, w.stats, w.df, stream);
  if (rc) return rc;
  return cm_bm25_search_stats_dev(h, q_terms_dev, q_off_dev, nq, total_terms, k, allow_dev, w.stats, w.df, eps_dev,
                                  score_dev, row_dev, status_dev, workspace_dev, workspace_bytes, stream);
}

}  // extern "C"
