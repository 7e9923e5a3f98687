// Device-side fusion: MMR re-ordering (rag/retrieval/fusion.py:39-61) and
// Reciprocal Rank Fusion + HybridRetriever's final sort (fusion.py:17-36,
// 132-167).  Both are tiny per query; they run one workgroup (MMR) or one
// lane (RRF) per query so a batch of queries costs one launch each and the
// pipeline never leaves the device between the k-NN and the final list.
// Compiled with -ffp-contract=off (the fused score must be bit-identical).
#include "cm_common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

namespace cm {

constexpr int kMmrThreads = 256;
constexpr int kMmrMaxPool = 256;
constexpr int kRrfLdsCap = 32;  // kv + kb up to which rrf_merge_kernel keeps its lists in LDS (57 KB)

// fp32 dot computed in fp64 and rounded once (closest fp32 to the exact dot).
__device__ inline float wave_dot(const float *__restrict__ a, const float *__restrict__ b, int dim, int lane) {
  double s = 0.0;
  for (int d = lane; d < dim; d += 64) s += (double)a[d] * (double)b[d];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  return (float)s;
}

// One workgroup per query.  sims_q = C q ; greedy: argmax(sims_q) first, then
// maximise f32(lam*sq[i]) - f32((1-lam)*max_{j in sel} sims_cc[i,j]) with
// strict '>' over remaining i in ascending order (NumPy>=2 float32 scalar
// arithmetic, the reference's set iteration order).  max-diversity is kept
// incrementally, so only pool x k pair dots are computed.
__global__ void __launch_bounds__(kMmrThreads) mmr_kernel(const float *__restrict__ q, const float *__restrict__ cands,
                                                          const int32_t *__restrict__ n_valid, int pool, int dim,
                                                          int k, float lam32, float oml32,
                                                          int32_t *__restrict__ out_order) {
  __shared__ float sq[kMmrMaxPool];
  __shared__ float maxdiv[kMmrMaxPool];
  __shared__ int sel_flag[kMmrMaxPool];
  __shared__ int cur;
  const int qi = blockIdx.x;
  const int n = min(n_valid ? n_valid[qi] : pool, pool);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const float *qv = q + (int64_t)qi * dim;
  const float *cv = cands + (int64_t)qi * pool * dim;
  const int kk = min(k, n);
  for (int i = threadIdx.x; i < k; i += kMmrThreads) out_order[(int64_t)qi * k + i] = -1;
  if (n <= 0) return;
  for (int i = wave; i < n; i += kMmrThreads / 64) {
    const float s = wave_dot(cv + (int64_t)i * dim, qv, dim, lane);
    if (lane == 0) sq[i] = s;
  }
  for (int i = threadIdx.x; i < n; i += kMmrThreads) {
    maxdiv[i] = -INFINITY;
    sel_flag[i] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int best = 0;
    for (int i = 1; i < n; ++i)
      if (sq[i] > sq[best]) best = i;  // np.argmax: first maximum
    cur = best;
    sel_flag[best] = 1;
    out_order[(int64_t)qi * k] = best;
  }
  __syncthreads();
  for (int step = 1; step < kk; ++step) {
    const int s = cur;
    // update max-diversity with the newly selected item
    for (int i = wave; i < n; i += kMmrThreads / 64) {
      if (sel_flag[i]) continue;
      const float sim = wave_dot(cv + (int64_t)i * dim, cv + (int64_t)s * dim, dim, lane);
      if (lane == 0) maxdiv[i] = fmaxf(maxdiv[i], sim);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int best = -1;
      float bs = -1e9f;
      for (int i = 0; i < n; ++i) {
        if (sel_flag[i]) continue;
        const float a = lam32 * sq[i];
        const float b = oml32 * maxdiv[i];
        const float sc = a - b;
        if (sc > bs) {
          bs = sc;
          best = i;
        }
      }
      cur = best;
      sel_flag[best] = 1;
      out_order[(int64_t)qi * k + step] = best;
    }
    __syncthreads();
  }
}

// Same MMR for pools of <= kMmrLdsPool items (the retriever's 24): the pool and the query are
// staged in LDS with all loads in flight, the similarity table's distinct pairs are computed at
// once (one fp64 dot per thread in dimension order, rounded once to fp32 as above, so the values
// are the ones mmr_kernel computes), and one wave runs the greedy loop on registers + shuffles
// with no block barriers: first max wins ties (strict '>' in ascending index order).
// F64 (the rows fit LDS as doubles: pool <= 24 at dim 768): the rows are converted once while
// staged and every product is one v_fma_f64 on two LDS doubles; otherwise the rows stay fp32 and
// each product converts both.  fma(a, b, s) == s + a b here: the product of two fp32 values is
// exact in fp64, so the fused and the separate forms round the same sum once.
constexpr int kMmrLdsPool = 32;
constexpr int kMmrLdsDim = 1024;

constexpr int kMmrLdsThreads = 1024;  // 16 waves: the n (n + 1) / 2 + n distinct pairs (324 at 24) in one pass
template <bool F64>
__global__ void __launch_bounds__(kMmrLdsThreads) mmr_lds_kernel(const float *__restrict__ q, const float *__restrict__ cands,
                                                              const int32_t *__restrict__ n_valid, int pool, int dim,
                                                              int k, float lam32, float oml32,
                                                              int32_t *__restrict__ out_order) {
  extern __shared__ __attribute__((aligned(16))) unsigned char mm_raw[];
  typedef typename std::conditional<F64, double, float>::type R;
  const int ld = dim + 1;                       // row pitch: rows start in different banks
  R *rows = reinterpret_cast<R *>(mm_raw);      // [n + 1][ld]: pool rows, then the query
  const int qi = blockIdx.x;
  const int n = min(n_valid ? n_valid[qi] : pool, pool);
  float *sim = reinterpret_cast<float *>(mm_raw + (size_t)(pool + 1) * ld * sizeof(R));  // [n + 1][kMmrLdsPool]: row n = sims_q
  const int kk = min(k, n);
  for (int i = threadIdx.x; i < k; i += kMmrLdsThreads) out_order[(int64_t)qi * k + i] = -1;
  if (n <= 0) return;  // uniform
  const float *cv = cands + (int64_t)qi * pool * dim;
  const float *qv = q + (int64_t)qi * dim;
  if ((dim & 3) == 0 && ((reinterpret_cast<uintptr_t>(cands) | reinterpret_cast<uintptr_t>(q)) & 15) == 0) {
    // 16-B global loads (every row 16-B aligned), scalar LDS stores (odd pitch)
    const int d4 = dim >> 2;
    for (int t = threadIdx.x; t < (n + 1) * d4; t += kMmrLdsThreads) {
      const int r = t / d4, d = (t - r * d4) * 4;
      const float4 v = *reinterpret_cast<const float4 *>((r < n ? cv + (int64_t)r * dim : qv) + d);
      R *o = rows + r * ld + d;
      o[0] = (R)v.x;
      o[1] = (R)v.y;
      o[2] = (R)v.z;
      o[3] = (R)v.w;
    }
  } else {
    for (int t = threadIdx.x; t < (n + 1) * dim; t += kMmrLdsThreads) {
      const int r = t / dim, d = t - r * dim;
      rows[r * ld + d] = (R)(r < n ? cv[(int64_t)r * dim + d] : qv[d]);
    }
  }
  __syncthreads();
  // the distinct pairs, packed: p < n (n + 1) / 2 -> (i, j), j <= i < n (row-major lower triangle);
  // then the n query pairs (n, j).  Each dot in dimension order with an fp64 accumulator.
  const int ntri = n * (n + 1) / 2;
  for (int p = threadIdx.x; p < ntri + n; p += kMmrLdsThreads) {
    int i, j;
    if (p < ntri) {
      i = (int)((sqrtf(8.f * (float)p + 1.f) - 1.f) * 0.5f);
      while (i * (i + 1) / 2 > p) --i;
      while ((i + 1) * (i + 2) / 2 <= p) ++i;
      j = p - i * (i + 1) / 2;
    } else {
      i = n;
      j = p - ntri;
    }
    const R *a = rows + i * ld;
    const R *b = rows + j * ld;
    double acc = 0.0;
#pragma unroll 8
    for (int d = 0; d < dim; ++d) acc = __builtin_fma((double)a[d], (double)b[d], acc);
    const float v = (float)acc;
    sim[i * kMmrLdsPool + j] = v;
    if (i < n) sim[j * kMmrLdsPool + i] = v;
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const bool have = lane < n;
  const float sq = have ? sim[n * kMmrLdsPool + lane] : -INFINITY;
  bool sel = false;
  float maxdiv = -INFINITY;
  // argmax(sims_q), first maximum
  auto wave_best = [&](float v, bool ok) {
    int bi = ok ? lane : 0x7fffffff;
    float bv = ok ? v : -INFINITY;
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    return bi;
  };
  int cur = wave_best(sq, have);
  if (lane == cur) sel = true;
  if (lane == 0) out_order[(int64_t)qi * k] = cur;
  for (int step = 1; step < kk; ++step) {
    if (have && !sel) maxdiv = fmaxf(maxdiv, sim[lane * kMmrLdsPool + cur]);
    const float a = lam32 * sq;
    const float b = oml32 * maxdiv;
    const float sc = a - b;
    cur = wave_best(sc, have && !sel && sc > -1e9f);
    if (cur == 0x7fffffff) break;  // mmr_kernel would emit -1 here too (no candidate beats -1e9)
    if (lane == cur) sel = true;
    if (lane == 0) out_order[(int64_t)qi * k + step] = cur;
  }
}

// The vector and BM25 lists of cm_rrf_merge_dev straight from the search outputs (one thread per
// query): vkeys/vdist[q][i] = the MMR-ordered pool entries (pool_keys/pool_dist[q][order[q][i]]),
// vn = the selected count (MMR pads its order with -1), bn = the BM25 list's valid count (rows
// padded with -1) -- the gathers and counts the caller would otherwise run as separate ops.
__global__ void rrf_pool_prep_kernel(const int64_t *__restrict__ pool_keys, const float *__restrict__ pool_dist,
                                     int pool, const int32_t *__restrict__ order, int kv,
                                     const int64_t *__restrict__ bkeys, int kb, int nq, int64_t *__restrict__ vkeys,
                                     float *__restrict__ vdist, int32_t *__restrict__ vn, int32_t *__restrict__ bn) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  int n = 0;
  for (int i = 0; i < kv; ++i) {
    const int32_t o = order[(int64_t)q * kv + i];
    const bool ok = o >= 0 && o < pool;
    vkeys[(int64_t)q * kv + i] = ok ? pool_keys[(int64_t)q * pool + o] : -1;
    vdist[(int64_t)q * kv + i] = ok ? pool_dist[(int64_t)q * pool + o] : 0.f;
    n += ok ? 1 : 0;
  }
  vn[q] = n;
  int m = 0;
  for (int i = 0; i < kb; ++i) m += bkeys[(int64_t)q * kb + i] >= 0 ? 1 : 0;
  bn[q] = m;
}

// HybridRetriever.retrieve's merge for one query per lane.
template <bool kLds>
__global__ void rrf_merge_kernel(const int64_t *__restrict__ vkeys, const float *__restrict__ vdist,
                                 const int32_t *__restrict__ vn, int kv, const int64_t *__restrict__ bkeys,
                                 const double *__restrict__ bscore, const int32_t *__restrict__ bn, int kb, int nq,
                                 double w_vec, double w_bm25, int rrf_k, int top_k, int64_t *__restrict__ out_keys,
                                 double *__restrict__ out_fused, float *__restrict__ out_vdist,
                                 double *__restrict__ out_bscore, int32_t *__restrict__ out_flags,
                                 int32_t *__restrict__ out_n, int64_t *__restrict__ scratch_keys,
                                 double *__restrict__ scratch_f, double *__restrict__ scratch_v,
                                 int32_t *__restrict__ scratch_src) {
  // per-query work arrays: this lane's slice of LDS (element j at [j * 64], no global round
  // trips; kv + kb <= kRrfLdsCap) or, for longer lists, the caller's global scratch (stride 1)
  extern __shared__ __attribute__((aligned(16))) unsigned char rrf_lds[];
  const int qi = blockIdx.x * blockDim.x + threadIdx.x;
  if (qi >= nq) return;
  const int nv = vn ? min(vn[qi], kv) : kv;
  const int nb = bn ? min(bn[qi], kb) : kb;
  const int cap = kv + kb;
  const int ln = threadIdx.x;
  constexpr int ST = kLds ? 64 : 1;
  int64_t *key = kLds ? reinterpret_cast<int64_t *>(rrf_lds) + ln : scratch_keys + (int64_t)qi * cap;
  double *fused = kLds ? reinterpret_cast<double *>(rrf_lds + (size_t)cap * 64 * 8) + ln : scratch_f + (int64_t)qi * cap;
  double *vdt = kLds ? reinterpret_cast<double *>(rrf_lds + (size_t)cap * 64 * 16) + ln : scratch_v + (int64_t)qi * cap;
  // bit0: vec index+1 in low 16, bit16..: bm index+1
  int32_t *src = kLds ? reinterpret_cast<int32_t *>(rrf_lds + (size_t)cap * 64 * 24) + ln : scratch_src + (int64_t)qi * cap;
  int m = 0;
  // by_id in insertion order: vector items (MMR order), then BM25-only items.
  for (int r = 0; r < nv; ++r) {
    const int64_t id = vkeys[(int64_t)qi * kv + r];
    key[(m) * ST] = id;
    fused[(m) * ST] = 0.0 + w_vec * (1.0 / (double)(rrf_k + (r + 1)));
    vdt[(m) * ST] = -(double)vdist[(int64_t)qi * kv + r];
    src[(m) * ST] = (r + 1);
    ++m;
  }
  for (int r = 0; r < nb; ++r) {
    const int64_t id = bkeys[(int64_t)qi * kb + r];
    const double c = w_bm25 * (1.0 / (double)(rrf_k + (r + 1)));
    int f = -1;
    for (int j = 0; j < nv; ++j)
      if (key[(j) * ST] == id) {
        f = j;
        break;
      }
    if (f >= 0) {
      fused[(f) * ST] = fused[(f) * ST] + c;
      src[(f) * ST] |= (r + 1) << 16;
    } else {
      key[(m) * ST] = id;
      fused[(m) * ST] = 0.0 + c;
      vdt[(m) * ST] = -0.0;
      src[(m) * ST] = (r + 1) << 16;
      ++m;
    }
  }
  // stable insertion sort by (fused, vd_term) descending
  for (int i = 1; i < m; ++i) {
    const int64_t k0 = key[(i) * ST];
    const double f0 = fused[(i) * ST], v0 = vdt[(i) * ST];
    const int32_t s0 = src[(i) * ST];
    int j = i - 1;
    while (j >= 0 && (fused[(j) * ST] < f0 || (fused[(j) * ST] == f0 && vdt[(j) * ST] < v0))) {
      key[(j + 1) * ST] = key[(j) * ST];
      fused[(j + 1) * ST] = fused[(j) * ST];
      vdt[(j + 1) * ST] = vdt[(j) * ST];
      src[(j + 1) * ST] = src[(j) * ST];
      --j;
    }
    key[(j + 1) * ST] = k0;
    fused[(j + 1) * ST] = f0;
    vdt[(j + 1) * ST] = v0;
    src[(j + 1) * ST] = s0;
  }
  const int n_out = min(m, top_k);
  for (int i = 0; i < top_k; ++i) {
    const int64_t o = (int64_t)qi * top_k + i;
    if (i < n_out) {
      const int vi = (src[(i) * ST] & 0xffff) - 1;
      const int bi = (src[(i) * ST] >> 16) - 1;
      out_keys[o] = key[(i) * ST];
      out_fused[o] = fused[(i) * ST];
      out_vdist[o] = vi >= 0 ? vdist[(int64_t)qi * kv + vi] : 0.f;
      out_bscore[o] = bi >= 0 ? bscore[(int64_t)qi * kb + bi] : 0.0;
      out_flags[o] = (vi >= 0 ? 1 : 0) | (bi >= 0 ? 2 : 0);
    } else {
      out_keys[o] = -1;
      out_fused[o] = 0.0;
      out_vdist[o] = 0.f;
      out_bscore[o] = 0.0;
      out_flags[o] = 0;
    }
  }
  out_n[qi] = n_out;
}

// The same merge with one wave per query (kv + kb <= 64; rrf_merge_kernel above for longer lists):
// lane r holds vector item r and BM25 item r.  A BM25 item's match is the first vector item with
// its id (shuffles over the vector lanes); each vector item adds the contributions of the BM25
// items that matched it in BM25 rank order; unmatched BM25 items take insertion positions nv, nv +
// 1, ... in rank order (ballot prefix).  Every fused value is the same sequence of fp64 operations
// as in rrf_merge_kernel.  The final order: an item's output position is the number of items
// before it in the stable descending (fused, -distance) order -- what the insertion sort yields.
constexpr int kRrfWaveCap = 64;
__global__ void __launch_bounds__(256) rrf_merge_wave_kernel(
    const int64_t *__restrict__ vkeys, const float *__restrict__ vdist, const int32_t *__restrict__ vn, int kv,
    const int64_t *__restrict__ bkeys, const double *__restrict__ bscore, const int32_t *__restrict__ bn, int kb, int nq,
    double w_vec, double w_bm25, int rrf_k, int top_k, int64_t *__restrict__ out_keys, double *__restrict__ out_fused,
    float *__restrict__ out_vdist, double *__restrict__ out_bscore, int32_t *__restrict__ out_flags,
    int32_t *__restrict__ out_n) {
  __shared__ double s_f[4][kRrfWaveCap], s_v[4][kRrfWaveCap];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qi0 = blockIdx.x * 4 + wv;
  const bool act = qi0 < nq;                    // wave-uniform (inactive waves still reach the barrier)
  const int qi = act ? qi0 : 0;
  const int nv = !act ? 0 : vn ? min(vn[qi], kv) : kv;
  const int nb = !act ? 0 : bn ? min(bn[qi], kb) : kb;
  const bool hv = lane < nv, hb = lane < nb;
  const int64_t vid = hv ? vkeys[(int64_t)qi * kv + lane] : -1;
  const int64_t bid = hb ? bkeys[(int64_t)qi * kb + lane] : -1;
  const double bc = w_bm25 * (1.0 / (double)(rrf_k + (lane + 1)));
  int f = -1;                                   // BM25 item lane's first matching vector item
  for (int j = 0; j < nv; ++j) {
    const int64_t kj = __shfl(vid, j);
    if (f < 0 && hb && kj == bid) f = j;
  }
  double fv = 0.0 + w_vec * (1.0 / (double)(rrf_k + (lane + 1)));
  int32_t srcv = lane + 1;
  for (int r = 0; r < nb; ++r) {
    const int fr = __shfl(f, r);
    const double cr = __shfl(bc, r);
    if (fr == lane) {
      fv = fv + cr;
      srcv |= (r + 1) << 16;
    }
  }
  const bool un = hb && f < 0;                  // BM25-only item
  const uint64_t um = __ballot(un);
  const int upos = nv + __popcll(um & ((1ull << lane) - 1ull));
  const int m = nv + __popcll(um);
  const double vdv = hv ? -(double)vdist[(int64_t)qi * kv + lane] : 0.0;
  const double fb = 0.0 + bc, vdb = -0.0;
  if (hv) {
    s_f[wv][lane] = fv;
    s_v[wv][lane] = vdv;
  }
  if (un) {
    s_f[wv][upos] = fb;
    s_v[wv][upos] = vdb;
  }
  __syncthreads();
  if (!act) return;
  auto rank_of = [&](double fx, double vx, int px) {
    int rk = 0;
    for (int e = 0; e < m; ++e) {
      const double fe = s_f[wv][e], ve = s_v[wv][e];
      rk += (fe > fx || (fe == fx && (ve > vx || (ve == vx && e < px)))) ? 1 : 0;
    }
    return rk;
  };
  const int n_out = min(m, top_k);
  auto emit = [&](int rk, int64_t key, double fx, int32_t src) {
    if (rk >= top_k) return;
    const int vi = (src & 0xffff) - 1, bi = (src >> 16) - 1;
    const int64_t o = (int64_t)qi * top_k + rk;
    out_keys[o] = key;
    out_fused[o] = fx;
    out_vdist[o] = vi >= 0 ? vdist[(int64_t)qi * kv + vi] : 0.f;
    out_bscore[o] = bi >= 0 ? bscore[(int64_t)qi * kb + bi] : 0.0;
    out_flags[o] = (vi >= 0 ? 1 : 0) | (bi >= 0 ? 2 : 0);
  };
  if (hv) emit(rank_of(fv, vdv, lane), vid, fv, srcv);
  if (un) emit(rank_of(fb, vdb, upos), bid, fb, (lane + 1) << 16);
  for (int i = n_out + lane; i < top_k; i += 64) {
    const int64_t o = (int64_t)qi * top_k + i;
    out_keys[o] = -1;
    out_fused[o] = 0.0;
    out_vdist[o] = 0.f;
    out_bscore[o] = 0.0;
    out_flags[o] = 0;
  }
  if (lane == 0) out_n[qi] = n_out;
}

// rrf_fuse over arbitrary lists (dict semantics) on one lane.
__global__ void rrf_fuse_kernel(const int64_t *__restrict__ keys, const int32_t *__restrict__ off, int nl,
                                const double *__restrict__ weights, int rrf_k, int64_t *__restrict__ out_keys,
                                double *__restrict__ out_score, int32_t *__restrict__ out_n) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int m = 0;
  for (int li = 0; li < nl; ++li) {
    const double w = weights ? weights[li] : 1.0;
    for (int r = 0; r < off[li + 1] - off[li]; ++r) {
      const int64_t id = keys[off[li] + r];
      const double c = w * (1.0 / (double)(rrf_k + (r + 1)));
      int f = -1;
      for (int j = 0; j < m; ++j)
        if (out_keys[j] == id) {
          f = j;
          break;
        }
      if (f < 0) {
        out_keys[m] = id;
        out_score[m] = 0.0 + c;
        ++m;
      } else {
        out_score[f] = out_score[f] + c;
      }
    }
  }
  *out_n = m;
}

}  // namespace cm

using namespace cm;

namespace {

struct HostStage {
  hipStream_t st = nullptr;
  int dev = -1;
  DevBuf buf;
  ~HostStage() {
    buf.release();
    if (st) (void)hipStreamDestroy(st);
  }
};

// per-thread staging for the host-array fusion entry points
HostStage &stage() {
  static thread_local HostStage s;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (s.dev != dev) {
    s.buf.release();
    if (s.st) (void)hipStreamDestroy(s.st);
    s.st = nullptr;
    (void)hipStreamCreateWithFlags(&s.st, hipStreamDefault);
    s.dev = dev;
  }
  return s;
}

struct Carver {
  char *base;
  size_t off = 0;
  template <typename T>
  T *take(size_t n) {
    T *p = base ? reinterpret_cast<T *>(base + off) : nullptr;  // base == nullptr: sizing pass only
    off += round_up((int64_t)std::max<size_t>(n, 1) * sizeof(T), 256);
    return p;
  }
};

}  // namespace

// Multi-GPU exchange merge: the packed all-gather of every shard's
// dense (distance f32, global row) top-P list and BM25 (score f64, global row) top-K list ->
// the global lists, identical on every rank.  allp[g][b][2P + 2K] int64: P distance words (f32
// bits in the low half), P rows, K score words (f64 bits), K rows.  One 256-thread workgroup per
// query; every entry's rank is the count of entries before it in the merge order -- dense: (f32
// distance asc, row asc), BM25: (score desc, row asc) with -0.0 == 0.0 -- and -1 rows (pads) after
// every real entry in shard-then-position order; ranks < P / K are written.  The same order as
// parallel.merge_dense_topk / merge_bm25_topk (torch sorts); no data-dependent launch, no host sync.
constexpr int kXMax = 4096;  // shard-list entries per query per kind (ws x P, ws x K)
__global__ void __launch_bounds__(256) shard_merge_kernel(const int64_t *__restrict__ allp, int ws, int B, int P,
                                                          int K, float *__restrict__ d_out, int64_t *__restrict__ r_out,
                                                          double *__restrict__ s_out, int64_t *__restrict__ br_out) {
  __shared__ uint64_t s_key[kXMax];
  __shared__ uint32_t s_sub[kXMax];   // tie-break (row for real entries, position for pads)
  const int b = blockIdx.x;
  if (b >= B) return;
  const int W = 2 * P + 2 * K;
  for (int kind = 0; kind < 2; ++kind) {
    const int L = kind == 0 ? P : K, n = ws * L;
    const int c0 = kind == 0 ? 0 : 2 * P;       // value words; rows follow at c0 + L
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
      const int g = e / L, j = e - g * L;
      const int64_t *rec = allp + ((int64_t)g * B + b) * W;
      const int64_t row = rec[c0 + L + j];
      uint64_t key;
      if (row < 0) {
        key = ~0ull;
      } else if (kind == 0) {
        const float dv = __builtin_bit_cast(float, (uint32_t)rec[c0 + j]);
        key = ((uint64_t)f32_order(dv) << 31) | ((uint64_t)row & 0x7fffffffull);
      } else {
        const double sv = __builtin_bit_cast(double, rec[c0 + j]) + 0.0;   // -0.0 -> 0.0
        key = ~f64_order(sv);                                                // score descending
      }
      s_key[e] = key;
      s_sub[e] = row < 0 ? (uint32_t)e : (uint32_t)row;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
      const uint64_t k0 = s_key[e];
      const uint32_t t0 = s_sub[e];
      int rank = 0;
      for (int x = 0; x < n; ++x) {
        const uint64_t kx = s_key[x];
        rank += (kx < k0 || (kx == k0 && s_sub[x] < t0)) ? 1 : 0;
      }
      if (rank < L) {
        const int g = e / L, j = e - g * L;
        const int64_t *rec = allp + ((int64_t)g * B + b) * W;
        if (kind == 0) {
          d_out[(int64_t)b * P + rank] = __builtin_bit_cast(float, (uint32_t)rec[c0 + j]);
          r_out[(int64_t)b * P + rank] = rec[c0 + L + j];
        } else {
          s_out[(int64_t)b * K + rank] = __builtin_bit_cast(double, rec[c0 + j]) + 0.0;
          br_out[(int64_t)b * K + rank] = rec[c0 + L + j];
        }
      }
    }
    __syncthreads();
  }
}

extern "C" {

int cm_mmr_dev(const float *q_dev, const float *cands_dev, const int32_t *n_valid_dev, int32_t nq, int32_t pool,
               int32_t dim, int32_t k, double lambd, int32_t *order_dev, void *stream) {
  if (nq <= 0) return CM_OK;
  if (pool <= 0 || pool > kMmrMaxPool) CM_FAIL(CM_EINVAL, "MMR pool must be in [1, 256]");
  if (dim <= 0 || k <= 0) CM_FAIL(CM_EINVAL, "bad MMR arguments");
  const float lam32 = (float)lambd;
  const float oml32 = (float)(1.0 - lambd);
  if (pool <= kMmrLdsPool && dim <= kMmrLdsDim) {
    constexpr int kMax = 160 * 1024;
    const size_t sim_bytes = (size_t)(kMmrLdsPool + 1) * kMmrLdsPool * 4;
    const size_t lds64 = (size_t)(pool + 1) * (dim + 1) * 8 + sim_bytes;
    static const hipError_t attr = [] {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&mmr_lds_kernel<true>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, kMax);
      return e != hipSuccess ? e
                             : hipFuncSetAttribute(reinterpret_cast<const void *>(&mmr_lds_kernel<false>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, kMax);
    }();
    CM_HIP(attr);
    if (lds64 <= (size_t)kMax)
      hipLaunchKernelGGL(mmr_lds_kernel<true>, dim3(nq), dim3(kMmrLdsThreads), lds64, (hipStream_t)stream, q_dev,
                         cands_dev, n_valid_dev, pool, dim, k, lam32, oml32, order_dev);
    else
      hipLaunchKernelGGL(mmr_lds_kernel<false>, dim3(nq), dim3(kMmrLdsThreads),
                         (size_t)(pool + 1) * (dim + 1) * 4 + sim_bytes, (hipStream_t)stream, q_dev, cands_dev,
                         n_valid_dev, pool, dim, k, lam32, oml32, order_dev);
    CM_HIP(hipGetLastError());
    return CM_OK;
  }
  hipLaunchKernelGGL(mmr_kernel, dim3(nq), dim3(kMmrThreads), 0, (hipStream_t)stream, q_dev, cands_dev, n_valid_dev,
                     pool, dim, k, lam32, oml32, order_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int cm_mmr(const float *q, const float *cands, const int32_t *n_valid, int32_t nq, int32_t pool, int32_t dim,
           int32_t k, double lambd, int32_t *out_order) {
  if (nq <= 0) return CM_OK;
  if (!q || !cands || !out_order) CM_FAIL(CM_EINVAL, "NULL argument");
  if (pool <= 0 || pool > kMmrMaxPool || dim <= 0 || k <= 0) CM_FAIL(CM_EINVAL, "bad MMR arguments");
  HostStage &s = stage();
  Carver c{nullptr};
  const size_t nqs = (size_t)nq;
  c.take<float>(nqs * dim);
  c.take<float>(nqs * pool * dim);
  c.take<int32_t>(nqs);
  c.take<int32_t>(nqs * k);
  int rc = s.buf.ensure(c.off);
  if (rc) return rc;
  Carver d{s.buf.as<char>()};
  float *dq = d.take<float>(nqs * dim);
  float *dc = d.take<float>(nqs * pool * dim);
  int32_t *dn = d.take<int32_t>(nqs);
  int32_t *dout = d.take<int32_t>(nqs * k);
  CM_HIP(hipMemcpyAsync(dq, q, nqs * dim * 4, hipMemcpyHostToDevice, s.st));
  CM_HIP(hipMemcpyAsync(dc, cands, nqs * pool * dim * 4, hipMemcpyHostToDevice, s.st));
  if (n_valid) CM_HIP(hipMemcpyAsync(dn, n_valid, nqs * 4, hipMemcpyHostToDevice, s.st));
  rc = cm_mmr_dev(dq, dc, n_valid ? dn : nullptr, nq, pool, dim, k, lambd, dout, s.st);
  if (rc) return rc;
  CM_HIP(hipMemcpyAsync(out_order, dout, nqs * k * 4, hipMemcpyDeviceToHost, s.st));
  CM_HIP(hipStreamSynchronize(s.st));
  return CM_OK;
}

int cm_rrf_pool_prep_dev(const int64_t *pool_keys, const float *pool_dist, int32_t pool, const int32_t *order,
                         int32_t kv, const int64_t *bkeys, int32_t kb, int32_t nq, int64_t *vkeys, float *vdist,
                         int32_t *vn, int32_t *bn, void *stream) {
  if (nq <= 0) return CM_OK;
  if (pool <= 0 || kv < 0 || kb < 0) CM_FAIL(CM_EINVAL, "bad RRF pool sizes");
  if (!pool_keys || !pool_dist || !order || !bkeys || !vkeys || !vdist || !vn || !bn)
    CM_FAIL(CM_EINVAL, "NULL argument");
  hipLaunchKernelGGL(rrf_pool_prep_kernel, dim3((unsigned)ceil_div(nq, 64)), dim3(64), 0, (hipStream_t)stream,
                     pool_keys, pool_dist, pool, order, kv, bkeys, kb, nq, vkeys, vdist, vn, bn);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int cm_rrf_merge_dev(const int64_t *vkeys, const float *vdist, const int32_t *vn, int32_t kv, const int64_t *bkeys,
                     const double *bscore, const int32_t *bn, int32_t kb, int32_t nq, double w_vec, double w_bm25,
                     int32_t rrf_k, int32_t top_k, int64_t *out_keys, double *out_fused, float *out_vdist,
                     double *out_bscore, int32_t *out_flags, int32_t *out_n, void *stream) {
  // scratch lives after out_* in a caller workspace-free way: carve from a
  // per-thread device buffer (graph capture: call once before capture so the
  // buffer exists; it is reused afterwards).
  if (nq <= 0) return CM_OK;
  if (kv < 0 || kb < 0 || top_k <= 0 || kv + kb > 0xffff) CM_FAIL(CM_EINVAL, "bad RRF sizes");
  static thread_local DevBuf scratch;
  static thread_local int scratch_dev = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (scratch_dev != dev) {
    scratch.release();
    scratch_dev = dev;
  }
  const int cap = std::max(kv + kb, 1);
  const size_t need = (size_t)nq * cap * (8 + 8 + 8 + 4) + 1024;
  if (need > scratch.bytes) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (stream) (void)hipStreamIsCapturing((hipStream_t)stream, &cs);
    if (cs != hipStreamCaptureStatusNone) CM_FAIL(CM_EINVAL, "rrf scratch must be sized before graph capture");
    int rc = scratch.ensure(need);
    if (rc) return rc;
  }
  Carver c{scratch.as<char>()};
  int64_t *sk = c.take<int64_t>((size_t)nq * cap);
  double *sf = c.take<double>((size_t)nq * cap);
  double *sv = c.take<double>((size_t)nq * cap);
  int32_t *ss = c.take<int32_t>((size_t)nq * cap);
  static const bool wave_on = [] {   // CM_RRF_WAVE=0: the lane-per-query kernel (A/B)
    const char *e = getenv("CM_RRF_WAVE");
    return !(e && e[0] == '0');
  }();
  if (wave_on && kv <= kRrfWaveCap && kb <= kRrfWaveCap && kv + kb <= kRrfWaveCap)
    hipLaunchKernelGGL(rrf_merge_wave_kernel, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0, (hipStream_t)stream,
                       vkeys, vdist, vn, kv, bkeys, bscore, bn, kb, nq, w_vec, w_bm25, rrf_k, top_k, out_keys,
                       out_fused, out_vdist, out_bscore, out_flags, out_n);
  else if (cap <= kRrfLdsCap)
    hipLaunchKernelGGL(rrf_merge_kernel<true>, dim3((unsigned)ceil_div(nq, 64)), dim3(64), (size_t)cap * 64 * 28,
                       (hipStream_t)stream, vkeys, vdist, vn, kv, bkeys, bscore, bn, kb, nq, w_vec, w_bm25, rrf_k,
                       top_k, out_keys, out_fused, out_vdist, out_bscore, out_flags, out_n, sk, sf, sv, ss);
  else
    hipLaunchKernelGGL(rrf_merge_kernel<false>, dim3((unsigned)ceil_div(nq, 64)), dim3(64), 0, (hipStream_t)stream,
                       vkeys, vdist, vn, kv, bkeys, bscore, bn, kb, nq, w_vec, w_bm25, rrf_k, top_k, out_keys,
                       out_fused, out_vdist, out_bscore, out_flags, out_n, sk, sf, sv, ss);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int cm_rrf_merge(const int64_t *vkeys, const float *vdist, const int32_t *vn, int32_t kv, const int64_t *bkeys,
                 const double *bscore, const int32_t *bn, int32_t kb, int32_t nq, double w_vec, double w_bm25,
                 int32_t rrf_k, int32_t top_k, int64_t *out_keys, double *out_fused, float *out_vdist,
                 double *out_bscore, int32_t *out_flags, int32_t *out_n) {
  if (nq <= 0) return CM_OK;
  if (top_k <= 0 || kv < 0 || kb < 0) CM_FAIL(CM_EINVAL, "bad RRF sizes");
  HostStage &s = stage();
  const size_t n = (size_t)nq;
  Carver c{nullptr};
  c.take<int64_t>(n * kv);
  c.take<float>(n * kv);
  c.take<int32_t>(n);
  c.take<int64_t>(n * kb);
  c.take<double>(n * kb);
  c.take<int32_t>(n);
  c.take<int64_t>(n * top_k);
  c.take<double>(n * top_k);
  c.take<float>(n * top_k);
  c.take<double>(n * top_k);
  c.take<int32_t>(n * top_k);
  c.take<int32_t>(n);
  int rc = s.buf.ensure(c.off);
  if (rc) return rc;
  Carver d{s.buf.as<char>()};
  int64_t *dvk = d.take<int64_t>(n * kv);
  float *dvd = d.take<float>(n * kv);
  int32_t *dvn = d.take<int32_t>(n);
  int64_t *dbk = d.take<int64_t>(n * kb);
  double *dbs = d.take<double>(n * kb);
  int32_t *dbn = d.take<int32_t>(n);
  int64_t *ok = d.take<int64_t>(n * top_k);
  double *of = d.take<double>(n * top_k);
  float *ov = d.take<float>(n * top_k);
  double *ob = d.take<double>(n * top_k);
  int32_t *ofl = d.take<int32_t>(n * top_k);
  int32_t *on = d.take<int32_t>(n);
  if (kv) {
    CM_HIP(hipMemcpyAsync(dvk, vkeys, n * kv * 8, hipMemcpyHostToDevice, s.st));
    CM_HIP(hipMemcpyAsync(dvd, vdist, n * kv * 4, hipMemcpyHostToDevice, s.st));
  }
  if (kb) {
    CM_HIP(hipMemcpyAsync(dbk, bkeys, n * kb * 8, hipMemcpyHostToDevice, s.st));
    CM_HIP(hipMemcpyAsync(dbs, bscore, n * kb * 8, hipMemcpyHostToDevice, s.st));
  }
  if (vn) CM_HIP(hipMemcpyAsync(dvn, vn, n * 4, hipMemcpyHostToDevice, s.st));
  if (bn) CM_HIP(hipMemcpyAsync(dbn, bn, n * 4, hipMemcpyHostToDevice, s.st));
  rc = cm_rrf_merge_dev(dvk, dvd, vn ? dvn : nullptr, kv, dbk, dbs, bn ? dbn : nullptr, kb, nq, w_vec, w_bm25, rrf_k,
                        top_k, ok, of, ov, ob, ofl, on, s.st);
  if (rc) return rc;
  CM_HIP(hipMemcpyAsync(out_keys, ok, n * top_k * 8, hipMemcpyDeviceToHost, s.st));
  CM_HIP(hipMemcpyAsync(out_fused, of, n * top_k * 8, hipMemcpyDeviceToHost, s.st));
  CM_HIP(hipMemcpyAsync(out_vdist, ov, n * top_k * 4, hipMemcpyDeviceToHost, s.st));
  CM_HIP(hipMemcpyAsync(out_bscore, ob, n * top_k * 8, hipMemcpyDeviceToHost, s.st));
  CM_HIP(hipMemcpyAsync(out_flags, ofl, n * top_k * 4, hipMemcpyDeviceToHost, s.st));
  CM_HIP(hipMemcpyAsync(out_n, on, n * 4, hipMemcpyDeviceToHost, s.st));
  CM_HIP(hipStreamSynchronize(s.st));
  return CM_OK;
}

int cm_rrf_fuse(const int64_t *keys, const int32_t *off, int32_t nl, const double *weights, int32_t rrf_k,
                int64_t *out_keys, double *out_score, int32_t *out_n) {
  if (!out_n || !off) CM_FAIL(CM_EINVAL, "NULL argument");
  *out_n = 0;
  if (nl <= 0) return CM_OK;
  const int32_t total = off[nl];
  for (int i = 0; i < nl; ++i)
    if (off[i + 1] < off[i]) CM_FAIL(CM_EINVAL, "off must be non-decreasing");
  if (total > 0 && (!keys || !out_keys || !out_score)) CM_FAIL(CM_EINVAL, "NULL argument");
  HostStage &s = stage();
  Carver c{nullptr};
  c.take<int64_t>(total);
  c.take<int32_t>(nl + 1);
  c.take<double>(nl);
  c.take<int64_t>(total);
  c.take<double>(total);
  c.take<int32_t>(1);
  int rc = s.buf.ensure(c.off);
  if (rc) return rc;
  Carver d{s.buf.as<char>()};
  int64_t *dk = d.take<int64_t>(total);
  int32_t *doff = d.take<int32_t>(nl + 1);
  double *dw = d.take<double>(nl);
  int64_t *ok = d.take<int64_t>(total);
  double *os = d.take<double>(total);
  int32_t *on = d.take<int32_t>(1);
  if (total) CM_HIP(hipMemcpyAsync(dk, keys, (size_t)total * 8, hipMemcpyHostToDevice, s.st));
  CM_HIP(hipMemcpyAsync(doff, off, (size_t)(nl + 1) * 4, hipMemcpyHostToDevice, s.st));
  if (weights) CM_HIP(hipMemcpyAsync(dw, weights, (size_t)nl * 8, hipMemcpyHostToDevice, s.st));
  hipLaunchKernelGGL(rrf_fuse_kernel, dim3(1), dim3(64), 0, s.st, dk, doff, nl, weights ? dw : nullptr, rrf_k, ok,
                     os, on);
  CM_HIP(hipGetLastError());
  int32_t n = 0;
  CM_HIP(hipMemcpyAsync(&n, on, 4, hipMemcpyDeviceToHost, s.st));
  CM_HIP(hipStreamSynchronize(s.st));
  if (n > 0) {
    CM_HIP(hipMemcpyAsync(out_keys, ok, (size_t)n * 8, hipMemcpyDeviceToHost, s.st));
    CM_HIP(hipMemcpyAsync(out_score, os, (size_t)n * 8, hipMemcpyDeviceToHost, s.st));
    CM_HIP(hipStreamSynchronize(s.st));
  }
  *out_n = n;
  return CM_OK;
}

int cm_shard_merge_topk_dev(const int64_t *allp_dev, int32_t ws, int32_t B, int32_t P, int32_t K, float *d_out,
                            int64_t *r_out, double *s_out, int64_t *br_out, void *stream) {
  if (ws <= 0 || B < 0 || P <= 0 || K <= 0) CM_FAIL(CM_EINVAL, "bad shard merge shape");
  if ((int64_t)ws * P > kXMax || (int64_t)ws * K > kXMax) CM_FAIL(CM_EUNSUPPORTED, "shard lists too long to merge");
  if (B == 0) return CM_OK;
  if (!allp_dev || !d_out || !r_out || !s_out || !br_out) CM_FAIL(CM_EINVAL, "NULL argument");
  hipLaunchKernelGGL(shard_merge_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, allp_dev, ws, B, P, K,
                     d_out, r_out, s_out, br_out);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

}  // extern "C"
