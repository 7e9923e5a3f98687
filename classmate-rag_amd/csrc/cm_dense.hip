// Dense cosine k-NN over an HBM-resident fp32 corpus (replaces Chroma/hnswlib,
// rag/retrieval/vector_chroma.py:204-253).  See DESIGN.md §K1.
//
// Layout in HBM (per handle):
//   C     [rows_alloc][ld] fp32, ld = dim rounded up to 128 (zero padded)
//   invc  [rows_alloc] fp32 = 1 / (||c|| + 1e-30)  (hnswlib cosine normalisation)
//   live  [rows_alloc/32] u32 bitmap (deleted / never-written rows = 0)
// rows_alloc is a multiple of kRowTile*kWaves = 128 so the streaming kernel
// needs no bounds checks.
//
// K1 dense_topk_kernel: one 512-thread workgroup (8 waves) per (corpus range,
// group of QB queries).  Each wave streams 16-row tiles of C straight from HBM
// into VGPRs (float4 per lane, 12 loads/chunk, double-buffered) and feeds
// v_mfma_f32_16x16x4_f32 with the query fragments kept in LDS for the whole
// launch.  Scores never leave the chip: the epilogue turns them into
// (distance,row) keys, filters them against a per-query running threshold and
// appends survivors to an LDS buffer that one wave per query merges into a
// sorted top-k list after every 128-row step.  A second tiny kernel merges the
// per-range lists (sorted) with a tournament.
#include "cm_common.h"

#include <algorithm>
#include <mutex>
#include <vector>

namespace cm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kRowTile = 16;                  // rows per wave step (MFMA M)
constexpr int kStepRows = kRowTile * kWaves;  // rows per workgroup step
constexpr int kCap = kStepRows;               // candidate buffer per query (no overflow per step)

struct DenseLds {
  // byte offsets into the dynamic LDS array
  int qfrag, invq, thr, cnt, len, list, buf, total;
};

__host__ __device__ inline DenseLds dense_lds_layout(int QB, int KMAX, int ld) {
  DenseLds L;
  int off = 0;
  L.qfrag = off;
  off += QB * ld * 4;
  L.invq = off;
  off += QB * 4;
  L.cnt = off;
  off += QB * 4;
  L.len = off;
  off += QB * 4;
  off = (off + 15) & ~15;
  L.thr = off;
  off += QB * 8;
  L.list = off;
  off += QB * KMAX * 8;
  L.buf = off;
  off += QB * kCap * 8;
  L.total = off;
  return L;
}

// Pad queries to ld and compute 1/(||q||+1e-30) (hnswlib normalize_vector).
__global__ void __launch_bounds__(256) dense_prep_queries(const float *__restrict__ q, int nq, int dim, int ld,
                                                          float *__restrict__ qp, float *__restrict__ invq) {
  const int qi = blockIdx.x;
  const float *src = q + (int64_t)qi * dim;
  float *dst = qp + (int64_t)qi * ld;
  float s = 0.f;
  for (int i = threadIdx.x; i < ld; i += 256) {
    float v = (qi < nq && i < dim) ? src[i] : 0.f;
    dst[i] = v;
    s += v * v;
  }
  __shared__ float red[4];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = (red[0] + red[1]) + (red[2] + red[3]);
    invq[qi] = 1.0f / (sqrtf(t) + 1e-30f);
  }
}

template <int QB, int CH, int KMAX>
__global__ void __launch_bounds__(kThreads, 2)
    dense_topk_kernel(const float *__restrict__ C, int ld, const float *__restrict__ invc,
                      const uint32_t *__restrict__ live, const uint32_t *__restrict__ allow, int64_t n_words,
                      const float *__restrict__ qp, const float *__restrict__ invq_g, int nq, int k,
                      int64_t rows_per_block, int64_t rows_end, int n_cblocks, uint64_t *__restrict__ cand) {
  constexpr int QT = QB / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const DenseLds L = dense_lds_layout(QB, KMAX, ld);
  f32x4 *qfrag = reinterpret_cast<f32x4 *>(lds + L.qfrag);
  float *invq = reinterpret_cast<float *>(lds + L.invq);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(lds + L.cnt);
  uint32_t *len = reinterpret_cast<uint32_t *>(lds + L.len);
  uint64_t *thr = reinterpret_cast<uint64_t *>(lds + L.thr);
  uint64_t *list = reinterpret_cast<uint64_t *>(lds + L.list);
  uint64_t *buf = reinterpret_cast<uint64_t *>(lds + L.buf);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int j = lane & 15;
  const int qg = blockIdx.x / n_cblocks;
  const int cb = blockIdx.x % n_cblocks;
  const int KS = ld / 16;  // 16-deep k steps per row

  // Query fragments, MFMA B layout: lane (g,j) of (qt,ks) holds q[qt*16+j][ks*16+4g .. +3].
  for (int idx = tid; idx < QT * KS * 64; idx += kThreads) {
    const int qt = idx / (KS * 64);
    const int rem = idx - qt * KS * 64;
    const int ks = rem >> 6;
    const int ln = rem & 63;
    const int qq = qg * QB + qt * 16 + (ln & 15);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (qq < nq) v = *reinterpret_cast<const f32x4 *>(qp + (int64_t)qq * ld + ks * 16 + 4 * (ln >> 4));
    qfrag[idx] = v;
  }
  for (int q = tid; q < QB; q += kThreads) {
    const int qq = qg * QB + q;
    invq[q] = qq < nq ? invq_g[qq] : 0.f;
    cnt[q] = 0;
    len[q] = 0;
    thr[q] = qq < nq ? kEmptyKey : 0ull;  // padded queries accept nothing
  }
  __syncthreads();

  const int64_t r_begin = (int64_t)cb * rows_per_block;
  const int64_t r_end = min(r_begin + rows_per_block, rows_end);
  const int iters = r_begin < r_end ? (int)((r_end - r_begin) / kStepRows) : 0;
  const int CPT = KS / CH;  // chunks per tile (even, checked on host)
  const int total = iters * CPT;

  // two independent accumulation chains per query tile (even / odd k within a
  // 16-deep step): v_mfma_f32_16x16x4_f32 has a 40-cycle dependent latency vs a
  // 32-cycle issue interval, so back-to-back MFMAs must not share an accumulator.
  f32x4 acc[QT][2];
#pragma unroll
  for (int t = 0; t < QT; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto chunk_ptr = [&](int gc) -> const float * {
    const int it = gc / CPT;
    const int c = gc - it * CPT;
    const int64_t row = r_begin + (int64_t)it * kStepRows + wave * kRowTile + j;
    return C + row * ld + c * CH * 16 + 4 * g;
  };
  auto load = [&](f32x4 (&b)[CH], int gc) {
    const float *p = chunk_ptr(gc);
#pragma unroll
    for (int u = 0; u < CH; ++u) b[u] = *reinterpret_cast<const f32x4 *>(p + u * 16);
  };
  auto compute = [&](const f32x4 (&b)[CH], int gc) {
    const int c = gc % CPT;
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int ks = c * CH + u;
      f32x4 bq[QT];
#pragma unroll
      for (int t = 0; t < QT; ++t) bq[t] = qfrag[(t * KS + ks) * 64 + lane];
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[u].x, bq[t].x, acc[t][0], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[u].y, bq[t].y, acc[t][1], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[u].z, bq[t].z, acc[t][0], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < QT; ++t) acc[t][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[u].w, bq[t].w, acc[t][1], 0, 0, 0);
    }
  };
  // Epilogue operands of a tile are loaded early (before the next chunk's
  // prefetch) so waiting for them never drains the prefetch (vmcnt in order).
  struct EpiOps {
    f32x4 ic;
    uint32_t bits;
  };
  auto epi_load = [&](int it) -> EpiOps {
    const int64_t row0 = r_begin + (int64_t)it * kStepRows + wave * kRowTile;
    const int64_t w = row0 >> 5;
    EpiOps e;
    e.bits = 0;
    if (w < n_words) e.bits = live[w] & (allow ? allow[w] : 0xffffffffu);
    e.ic = *reinterpret_cast<const f32x4 *>(invc + row0 + 4 * g);
    return e;
  };
  // Epilogue of one 16-row tile: distances -> threshold filter -> LDS buffer.
  auto epilogue = [&](int it, const EpiOps &e) {
    const int64_t row0 = r_begin + (int64_t)it * kStepRows + wave * kRowTile;
    const uint32_t bits = e.bits >> ((row0 & 31) + 4 * g);
    const f32x4 ic = e.ic;
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int q = t * 16 + j;
      const float iq = invq[q];
      const uint64_t th = thr[q];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if ((bits >> r) & 1u) {
          const float dist = 1.0f - (acc[t][0][r] + acc[t][1][r]) * iq * ic[r];
          const uint64_t key = ((uint64_t)f32_order(dist) << 32) | (uint64_t)(uint32_t)(row0 + 4 * g + r);
          if (key < th) {
            const uint32_t slot = atomicAdd(&cnt[q], 1u);
            if (slot < (uint32_t)kCap) buf[q * kCap + slot] = key;
          }
        }
      }
      acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // One wave per query: rank-merge the buffer into the sorted list.
  auto merge = [&]() {
    constexpr int T = (KMAX + kCap + 63) / 64;
    for (int q = wave; q < QB; q += kWaves) {
      const uint32_t nn = min(cnt[q], (uint32_t)kCap);
      if (nn == 0) continue;
      const uint32_t Lq = len[q];
      const uint32_t n = Lq + nn;
      uint64_t *lst = list + q * KMAX;
      const uint64_t *bq = buf + q * kCap;
      uint64_t key[T];
      uint32_t rank[T];
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const uint32_t e = lane + 64 * t;
        key[t] = e < Lq ? lst[e] : (e < n ? bq[e - Lq] : kEmptyKey);
        rank[t] = 0;
      }
      for (uint32_t i = 0; i < n; ++i) {
        const uint64_t x = i < Lq ? lst[i] : bq[i - Lq];
#pragma unroll
        for (int t = 0; t < T; ++t) rank[t] += (x < key[t]) ? 1u : 0u;
      }
      const uint32_t newL = min(n, (uint32_t)k);
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const uint32_t e = lane + 64 * t;
        if (e < n && rank[t] < (uint32_t)k) {
          lst[rank[t]] = key[t];
          if (rank[t] == (uint32_t)k - 1) thr[q] = key[t];
        }
      }
      if (lane == 0) {
        len[q] = newL;
        cnt[q] = 0;
      }
    }
  };

  if (total > 0) {
    f32x4 bufA[CH], bufB[CH];
    load(bufA, 0);
    __builtin_amdgcn_sched_barrier(0);
    for (int gc = 0; gc < total; gc += 2) {
      load(bufB, gc + 1);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the MFMAs it overlaps
      compute(bufA, gc);
      const bool tile_end = (gc + 2) % CPT == 0;
      // unconditional (clamped) loads keep one control path, so hipcc can count
      // the in-order vmcnt exactly for compute(bufB)
      const EpiOps eo = epi_load((gc + 1) / CPT);
      load(bufA, min(gc + 2, total - 1));
      __builtin_amdgcn_sched_barrier(0);
      compute(bufB, gc + 1);
      if (tile_end) {
        epilogue((gc + 1) / CPT, eo);
        __syncthreads();
        merge();
        __syncthreads();
      }
    }
  }

  // Emit this range's sorted list per query.
  for (int idx = tid; idx < QB * k; idx += kThreads) {
    const int q = idx / k;
    const int i = idx - q * k;
    const uint64_t v = (uint32_t)i < len[q] ? list[q * KMAX + i] : kEmptyKey;
    cand[((int64_t)blockIdx.x * QB + q) * k + i] = v;
  }
  (void)qg;
}

// ---------------------------------------------------------------------------
// K1b: batched cosine top-k on f16x3 split planes (batches of >= 64 queries,
// k <= 32).  xn.qn = xh.qh + xh.ql + xl.qh (+ xl.ql, dropped: |err| <= 2^-22
// relative per product, products exact in the f32 accumulator), so three
// v_mfma_f32_16x16x32_f16 per 16x16x32 block give f32-grade distances at 16/3x
// the f32-MFMA rate.
//
// One 512-thread workgroup per (corpus range, pass of 256 queries): the whole
// query pass is resident (wave w owns queries 32w..32w+31, fragments streamed
// from L2 one 32-deep k-chunk ahead), so every corpus byte is read from HBM
// once per pass.  Corpus 128-row x 32-k chunks (both planes, 16 KiB) are staged
// through double-buffered LDS (global->VGPR prefetch one chunk ahead).  After
// each 128-row tile every wave filters its 32 x 128 distances against its
// queries' running k-th keys and rank-merges survivors into per-query sorted
// lists in LDS; the per-range lists go to dense_merge_kernel.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int kBRows = 128;                 // corpus rows per tile
constexpr int kBPad = 40;                   // f16 per LDS row (32 + 8 pad: conflict-free b128 reads)
constexpr int kBQPass = 256;                // queries per pass (8 waves x 32)
constexpr int kBQWave = 32;
constexpr int kBSlots = 48;                 // per query: sorted list (len <= k) then unmerged survivors
constexpr int kBMaxK = 32;                  // k <= 32 leaves >= 16 buffer slots (one sub-tile's worst case)
constexpr int kBXBuf = 2 * kBRows * kBPad;  // f16 per LDS stage buffer (2 planes)

struct K1bLds {
  int xs, thr, thrd, cnt, len, list, buf, total;
};
__host__ __device__ inline K1bLds k1b_lds_layout() {
  K1bLds L;
  int off = 0;
  L.xs = off;
  off += 2 * kBXBuf * 2;
  L.thr = off;
  off += kBQPass * 8;
  L.list = off;
  off += kBQPass * kBSlots * 8;
  L.buf = off;
  L.thrd = off;
  off += kBQPass * 4;
  L.cnt = off;
  off += kBQPass * 4;
  L.len = off;
  off += kBQPass * 4;
  L.total = off;
  return L;
}

// Normalise + split queries into Qh/Ql [nq_pad][ld] (zero rows beyond nq).
__global__ void __launch_bounds__(256) dense_prep_planes(const float *__restrict__ q, int nq, int dim, int ld,
                                                         _Float16 *__restrict__ Qh, _Float16 *__restrict__ Ql) {
  const int qi = blockIdx.x;
  const float *src = q + (int64_t)qi * dim;
  float s = 0.f;
  for (int i = threadIdx.x; i < dim; i += 256) {
    const float v = qi < nq ? src[i] : 0.f;
    s += v * v;
  }
  __shared__ float red[4];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float t = (red[0] + red[1]) + (red[2] + red[3]);
  const float inv = 1.0f / (sqrtf(t) + 1e-30f);
  for (int i = threadIdx.x; i < ld; i += 256) {
    const float v = (qi < nq && i < dim) ? src[i] * inv : 0.f;
    const _Float16 hi = (_Float16)v;
    Qh[(int64_t)qi * ld + i] = hi;
    Ql[(int64_t)qi * ld + i] = (_Float16)(v - (float)hi);
  }
}

__global__ void __launch_bounds__(512, 1)
    dense_f16x3_kernel(const _Float16 *__restrict__ Xh, const _Float16 *__restrict__ Xl, int ld,
                       const uint32_t *__restrict__ live, const uint32_t *__restrict__ allow, int64_t n_words,
                       const _Float16 *__restrict__ Qh, const _Float16 *__restrict__ Ql, int nq, int k,
                       int64_t rows_per_wg, int64_t rows_end, int n_wg, uint64_t *__restrict__ cand, int dbg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const K1bLds L = k1b_lds_layout();
  _Float16 *xs = reinterpret_cast<_Float16 *>(lds + L.xs);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int j = lane & 15;
  const int wg = blockIdx.x % n_wg;
  const int qp = blockIdx.x / n_wg;
  const int qw0 = wave * kBQWave;            // wave's first query within the pass
  const int qg0 = qp * kBQPass + qw0;        // ... globally
  uint64_t *thr = reinterpret_cast<uint64_t *>(lds + L.thr) + qw0;
  float *thrd = reinterpret_cast<float *>(lds + L.thrd) + qw0;
  uint32_t *cnt = reinterpret_cast<uint32_t *>(lds + L.cnt) + qw0;
  uint32_t *len = reinterpret_cast<uint32_t *>(lds + L.len) + qw0;
  uint64_t *list = reinterpret_cast<uint64_t *>(lds + L.list) + (int64_t)qw0 * kBSlots;
  if (lane < kBQWave) {
    const bool real = qg0 + lane < nq;
    thr[lane] = real ? kEmptyKey : 0ull;  // padded queries accept nothing
    thrd[lane] = real ? __builtin_inff() : -__builtin_inff();
    cnt[lane] = 0;
    len[lane] = 0;
  }
  const int64_t r_begin = (int64_t)wg * rows_per_wg;
  const int64_t r_end = min(r_begin + rows_per_wg, rows_end);
  const int ntiles = r_begin < r_end ? (int)((r_end - r_begin) / kBRows) : 0;
  const int KC = ld / 32;
  const int total = ntiles * KC;

  // staging pieces of a chunk: 1024 x 16 B (plane, row, 8-f16 part); thread takes tid and tid + 512
  auto xsrc = [&](int gc, int p) -> const f16x8 * {
    const int t = gc / KC, c = gc - t * KC;
    const int plane = p >> 9, row = (p & 511) >> 2, part = p & 3;
    const _Float16 *X = plane ? Xl : Xh;
    return reinterpret_cast<const f16x8 *>(X + (r_begin + (int64_t)t * kBRows + row) * ld + c * 32 + part * 8);
  };
  auto xdst = [&](int b, int p) -> f16x8 * {
    const int plane = p >> 9, row = (p & 511) >> 2, part = p & 3;
    return reinterpret_cast<f16x8 *>(xs + b * kBXBuf + plane * kBRows * kBPad + row * kBPad + part * 8);
  };
  // query fragments (B operand): lane (g, j) of q-tile qt holds q[qt*16 + j][32c + 8g .. +7]
  auto qload = [&](f16x8 (&qh)[2], f16x8 (&ql)[2], int gc) {
    const int c = gc % KC;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int64_t o = (int64_t)(qg0 + qt * 16 + j) * ld + c * 32 + g * 8;
      qh[qt] = *reinterpret_cast<const f16x8 *>(Qh + o);
      ql[qt] = *reinterpret_cast<const f16x8 *>(Ql + o);
    }
  };
  f32x4 acc[8][2];
#pragma unroll
  for (int rt = 0; rt < 8; ++rt) acc[rt][0] = acc[rt][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  // rank-merge query q's slots [0, len + cnt) in place into its sorted list (<= k): one key per lane
  auto merge = [&](int q) {
    uint64_t *sl = list + q * kBSlots;
    const uint32_t n = len[q] + cnt[q];
    const uint64_t key = (uint32_t)lane < n ? sl[lane] : kEmptyKey;
    uint32_t rank = 0;
    for (uint32_t i = 0; i < n; ++i) rank += (sl[i] < key) ? 1u : 0u;
    __builtin_amdgcn_wave_barrier();  // every lane has read the old slots
    if ((uint32_t)lane < n && rank < (uint32_t)k) {
      sl[rank] = key;
      if (rank == (uint32_t)k - 1) {
        thr[q] = key;
        thrd[q] = f32_unorder((uint32_t)(key >> 32));
      }
    }
    if (lane == 0) {
      len[q] = min(n, (uint32_t)k);
      cnt[q] = 0;
    }
  };
  auto wave_lds_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // merge every query of the wave whose free slots could not take another sub-tile (or all
  // queries with anything buffered, at the end)
  auto merge_pending = [&](bool all) {
    wave_lds_sync();
    bool need = false;
    if (lane < kBQWave) {
      const uint32_t c = cnt[lane];
      need = all ? c > 0 : len[lane] + c + 16 > (uint32_t)kBSlots;
    }
    uint64_t m = __ballot(need);
    while (m) {
      const int q = __builtin_ctzll(m);
      m &= m - 1;
      merge(q);
      wave_lds_sync();
    }
  };
  // epilogue of tile t (wave-private queries, no block barrier): survivors of the running
  // k-th key are appended to the query's free slots; a sub-tile adds <= 16 per query (4 lanes
  // x 4 rows), and queries are merged only when fewer than 16 slots remain
  auto epilogue = [&](int t) {
    const int64_t row0 = r_begin + (int64_t)t * kBRows;
    uint32_t bits[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int64_t wi = (row0 >> 5) + w;
      bits[w] = wi < n_words ? (live[wi] & (allow ? allow[wi] : 0xffffffffu)) : 0u;
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int ql_ = qt * 16 + j;
#pragma unroll
      for (int rt = 0; rt < 8; ++rt) {
        const float td = thrd[ql_];
        const uint64_t tk = thr[ql_];
        bool added = false;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = rt * 16 + 4 * g + r;  // row within the tile
          const float dist = 1.0f - acc[rt][qt][r];
          if (((bits[rr >> 5] >> (rr & 31)) & 1u) && dist <= td) {
            const uint64_t key = ((uint64_t)f32_order(dist) << 32) | (uint64_t)(uint32_t)(row0 + rr);
            if (key < tk) {
              list[ql_ * kBSlots + len[ql_] + atomicAdd(&cnt[ql_], 1u)] = key;
              added = true;
            }
          }
        }
        if (__ballot(added)) merge_pending(false);
      }
    }
#pragma unroll
    for (int rt = 0; rt < 8; ++rt) acc[rt][0] = acc[rt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  if (total > 0) {
    // X chunks gc+1..gc+4 in flight in a 4-deep register ring (HBM latency ~ 3-4 chunks of
    // MFMA work); query fragments one chunk ahead (L2).  KC is a multiple of 4 (ld % 128
    // == 0), so a tile is a whole number of ring turns and the epilogue (no vector-memory
    // loads) sits outside the unrolled bodies: every wait is a counted vmcnt, not a drain.
    f16x8 qh[2], ql[2], nqh[2], nql[2];
    f16x8 ra0, ra1, rb0, rb1, rc0, rc1, rd0, rd1;
    auto xload = [&](f16x8 &x0, f16x8 &x1, int gc) {
      const int gl = min(gc, total - 1);  // clamped: one control path
      x0 = *xsrc(gl, tid);
      x1 = *xsrc(gl, tid + 512);
    };
    xload(ra0, ra1, 0);
    *xdst(0, tid) = ra0;
    *xdst(0, tid + 512) = ra1;
    qload(qh, ql, 0);
    xload(ra0, ra1, 1);
    xload(rb0, rb1, 2);
    xload(rc0, rc1, 3);
    xload(rd0, rd1, 4);
    __syncthreads();
    auto body = [&](int gc, f16x8 &x0, f16x8 &x1) {
      qload(nqh, nql, min(gc + 1, total - 1));
      const _Float16 *xb = xs + (gc & 1) * kBXBuf;
      auto frag = [&](int rt, int plane) -> f16x8 {
        return *reinterpret_cast<const f16x8 *>(xb + plane * kBRows * kBPad + (rt * 16 + j) * kBPad + g * 8);
      };
      // LDS fragments one 16-row sub-tile ahead of the MFMAs that use them
      f16x8 xh = frag(0, 0), xl = frag(0, 1);
#pragma unroll
      for (int rt = 0; rt < 8; ++rt) {
        f16x8 nh = xh, nl = xl;
        if (rt < 7) {
          nh = frag(rt + 1, 0);
          nl = frag(rt + 1, 1);
        }
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, qh[qt], acc[rt][qt], 0, 0, 0);
          acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, ql[qt], acc[rt][qt], 0, 0, 0);
          acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, qh[qt], acc[rt][qt], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        xh = nh;
        xl = nl;
      }
      *xdst((gc + 1) & 1, tid) = x0;  // chunk gc+1 (loaded four chunks ago)
      *xdst((gc + 1) & 1, tid + 512) = x1;
      xload(x0, x1, gc + 5);
      __syncthreads();
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        qh[qt] = nqh[qt];
        ql[qt] = nql[qt];
      }
    };
    for (int t = 0; t < ntiles; ++t) {
      for (int c = 0; c < KC; c += 4) {
        const int gc = t * KC + c;
        body(gc, ra0, ra1);
        body(gc + 1, rb0, rb1);
        body(gc + 2, rc0, rc1);
        body(gc + 3, rd0, rd1);
      }
      if (dbg & 1) {  // ablation: consume the accumulators without the top-k epilogue
        float z = 0.f;
#pragma unroll
        for (int rt = 0; rt < 8; ++rt)
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) z += acc[rt][qt][0] + acc[rt][qt][3];
        if (z == 12345.f) thrd[lane & 31] = z;
#pragma unroll
        for (int rt = 0; rt < 8; ++rt) acc[rt][0] = acc[rt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        epilogue(t);
      }
    }
  }
  merge_pending(true);
  // this range's sorted lists (layout of dense_merge_kernel with QB = kBQPass)
  for (int idx = lane; idx < kBQWave * k; idx += 64) {
    const int q = idx / k, i = idx - q * k;
    const uint64_t v = (uint32_t)i < len[q] ? list[q * kBSlots + i] : kEmptyKey;
    cand[(((int64_t)qp * n_wg + wg) * kBQPass + qw0 + q) * k + i] = v;
  }
}

// Tournament merge of n_cblocks sorted lists per query -> final top-k.
__global__ void __launch_bounds__(256) dense_merge_kernel(const uint64_t *__restrict__ cand, int n_cblocks, int QB,
                                                          int k, int nq, float *__restrict__ out_dist,
                                                          int64_t *__restrict__ out_row) {
  const int q = blockIdx.x;
  if (q >= nq) return;
  const int qg = q / QB;
  const int ql = q - qg * QB;
  constexpr int kPer = 8;  // lists per thread (n_cblocks <= 2048)
  int head[kPer];
  uint64_t hk[kPer];
  const uint64_t *base = cand + ((int64_t)qg * n_cblocks * QB + ql) * k;
  const int64_t stride = (int64_t)QB * k;
#pragma unroll
  for (int s = 0; s < kPer; ++s) {
    const int l = threadIdx.x + 256 * s;
    head[s] = 0;
    hk[s] = l < n_cblocks ? base[l * stride] : kEmptyKey;
  }
  __shared__ uint64_t red[4];
  for (int i = 0; i < k; ++i) {
    uint64_t m = kEmptyKey;
#pragma unroll
    for (int s = 0; s < kPer; ++s) m = hk[s] < m ? hk[s] : m;
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t other = __shfl_xor(m, o);
      m = other < m ? other : m;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    uint64_t best = red[0];
    for (int w = 1; w < 4; ++w) best = red[w] < best ? red[w] : best;
    __syncthreads();
    if (threadIdx.x == 0) {
      if (best == kEmptyKey) {
        out_dist[(int64_t)q * k + i] = 0.f;
        out_row[(int64_t)q * k + i] = -1;
      } else {
        out_dist[(int64_t)q * k + i] = f32_unorder((uint32_t)(best >> 32));
        out_row[(int64_t)q * k + i] = (int64_t)(uint32_t)best;
      }
    }
    if (best == kEmptyKey) continue;
#pragma unroll
    for (int s = 0; s < kPer; ++s) {
      if (hk[s] == best) {  // keys are unique (row in the low bits)
        const int l = threadIdx.x + 256 * s;
        head[s] += 1;
        hk[s] = head[s] < k ? base[l * stride + head[s]] : kEmptyKey;
      }
    }
  }
}

// Scatter n rows (staging n x dim) into C at rows[i] (or row0+i), set invc + live,
// and the row's normalised fp16 split planes (K1b): xn = x * invc (hnswlib
// normalize_vector), Xh = f16(xn), Xl = f16(xn - Xh).
__global__ void __launch_bounds__(256) dense_scatter_kernel(const float *__restrict__ src, const int64_t *__restrict__ rows,
                                                            int64_t row0, int64_t n, int dim, int ld,
                                                            float *__restrict__ C, float *__restrict__ invc,
                                                            uint32_t *__restrict__ live, _Float16 *__restrict__ Xh,
                                                            _Float16 *__restrict__ Xl) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int64_t r = rows ? rows[i] : row0 + i;
  const float *s = src + i * dim;
  float *d = C + r * ld;
  float acc = 0.f;
  for (int c = threadIdx.x; c < ld; c += 256) {
    const float v = c < dim ? s[c] : 0.f;
    d[c] = v;
    acc += v * v;
  }
  __shared__ float red[4];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  const float t = (red[0] + red[1]) + (red[2] + red[3]);
  const float inv = 1.0f / (sqrtf(t) + 1e-30f);
  if (threadIdx.x == 0) {
    invc[r] = inv;
    atomicOr(&live[r >> 5], 1u << (r & 31));
  }
  for (int c = threadIdx.x; c < ld; c += 256) {
    const float xn = (c < dim ? s[c] : 0.f) * inv;
    const _Float16 hi = (_Float16)xn;
    Xh[r * ld + c] = hi;
    Xl[r * ld + c] = (_Float16)(xn - (float)hi);
  }
}

__global__ void dense_clear_live_kernel(const int64_t *__restrict__ rows, int64_t n, int64_t size,
                                        uint32_t *__restrict__ live) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  if (r >= 0 && r < size) atomicAnd(&live[r >> 5], ~(1u << (r & 31)));
}

__global__ void dense_gather_kernel(const float *__restrict__ C, int ld, int dim, const int64_t *__restrict__ rows,
                                    int64_t n, int64_t size, float *__restrict__ out) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  float *o = out + i * dim;
  for (int c = threadIdx.x; c < dim; c += blockDim.x) o[c] = (r >= 0 && r < size) ? C[r * ld + c] : 0.f;
}

__global__ void popcount_kernel(const uint32_t *__restrict__ bits, int64_t n_words,
                                unsigned long long *__restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long c = 0;
  for (; i < n_words; i += (int64_t)gridDim.x * blockDim.x) c += __popc(bits[i]);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

}  // namespace cm

using namespace cm;

struct cm_dense {
  int dev = 0;
  int dim = 0;
  int ld = 0;
  int64_t rows_alloc = 0;  // multiple of kStepRows
  int64_t size = 0;        // high-water row count
  float *C = nullptr;
  float *invc = nullptr;
  _Float16 *Xh = nullptr, *Xl = nullptr;  // normalised f16 split planes (K1b)
  uint32_t *live = nullptr;
  hipStream_t stream = nullptr;
  DevBuf staging, rows_buf, allow_buf, ws, out_buf;
  std::vector<float> host_tmp;
};

namespace {

struct DenseCfg {
  int QB, CH, KMAX, n_qgroups, n_cblocks;
  int64_t rows_per_block, rows_end;
  size_t lds;
};

int pick_chunk(int ld) {
  const int KS = ld / 16;
  if (KS % 24 == 0) return 12;
  if (KS % 16 == 0) return 8;
  return 0;
}

int g_num_cus = 0;

int num_cus(int dev) {
  if (g_num_cus == 0) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess) g_num_cus = p.multiProcessorCount;
    if (g_num_cus <= 0) g_num_cus = 256;
  }
  return g_num_cus;
}

DenseCfg dense_config(const cm_dense *h, int nq, int k) {
  DenseCfg c{};
  c.CH = pick_chunk(h->ld);
  c.KMAX = k <= 64 ? 64 : 256;
  c.QB = (nq <= 16 || c.KMAX > 64) ? 16 : 32;
  if (c.QB == 32 && dense_lds_layout(32, c.KMAX, h->ld).total > 163840) c.QB = 16;
  c.n_qgroups = (int)ceil_div(nq, c.QB);
  c.lds = dense_lds_layout(c.QB, c.KMAX, h->ld).total;
  const int per_cu = std::max(1, std::min(2, (int)(163840 / c.lds)));
  const int target = num_cus(h->dev) * per_cu;
  c.rows_end = round_up(std::max<int64_t>(h->size, 1), kStepRows);
  const int64_t steps = c.rows_end / kStepRows;
  int64_t ncb = std::max<int64_t>(1, target / c.n_qgroups);
  if (ncb >= 8) ncb = ncb / 8 * 8;  // same corpus range on one XCD across query groups
  ncb = std::min<int64_t>(ncb, steps);
  c.rows_per_block = ceil_div(steps, ncb) * kStepRows;
  c.n_cblocks = (int)ceil_div(c.rows_end, c.rows_per_block);
  return c;
}

template <int QB, int CH, int KMAX>
int launch_dense_t(const DenseCfg &c, const cm_dense *h, const uint32_t *allow, const float *qp, const float *invq,
                   int nq, int k, uint64_t *cand, hipStream_t st) {
  static std::once_flag once;
  static hipError_t attr_err = hipSuccess;
  std::call_once(once, [] {
    attr_err = hipFuncSetAttribute(reinterpret_cast<const void *>(&dense_topk_kernel<QB, CH, KMAX>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  });
  CM_HIP(attr_err);
  const int64_t n_words = ceil_div(h->size, 32);
  dim3 grid(c.n_cblocks * c.n_qgroups);
  hipLaunchKernelGGL((dense_topk_kernel<QB, CH, KMAX>), grid, dim3(kThreads), c.lds, st, h->C, h->ld, h->invc,
                     h->live, allow, n_words, qp, invq, nq, k, c.rows_per_block, c.rows_end, c.n_cblocks, cand);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int launch_dense(const DenseCfg &c, const cm_dense *h, const uint32_t *allow, const float *qp, const float *invq,
                 int nq, int k, uint64_t *cand, hipStream_t st) {
#define CM_DENSE_CASE(QB_, CH_, KM_) \
  if (c.QB == QB_ && c.CH == CH_ && c.KMAX == KM_) return launch_dense_t<QB_, CH_, KM_>(c, h, allow, qp, invq, nq, k, cand, st);
  CM_DENSE_CASE(16, 12, 64)
  CM_DENSE_CASE(32, 12, 64)
  CM_DENSE_CASE(16, 12, 256)
  CM_DENSE_CASE(16, 8, 64)
  CM_DENSE_CASE(32, 8, 64)
  CM_DENSE_CASE(16, 8, 256)
#undef CM_DENSE_CASE
  CM_FAIL(CM_EUNSUPPORTED, "no dense kernel instance for this configuration");
}

struct DenseWs {
  float *qp;
  float *invq;
  uint64_t *cand;
  size_t total;
};

DenseWs dense_ws_layout(const cm_dense *h, const DenseCfg &c, int nq, int k, void *base) {
  DenseWs w{};
  char *p = reinterpret_cast<char *>(base);
  size_t off = 0;
  const int nq_pad = c.n_qgroups * c.QB;
  w.qp = reinterpret_cast<float *>(p + off);
  off += round_up((int64_t)nq_pad * h->ld * 4, 256);
  w.invq = reinterpret_cast<float *>(p + off);
  off += round_up((int64_t)nq_pad * 4, 256);
  w.cand = reinterpret_cast<uint64_t *>(p + off);
  off += round_up((int64_t)c.n_qgroups * c.n_cblocks * c.QB * k * 8, 256);
  w.total = off;
  (void)nq;
  return w;
}

int dense_grow(cm_dense *h, int64_t need_rows) {
  if (need_rows <= h->rows_alloc) return CM_OK;
  int64_t cap = std::max<int64_t>(need_rows, h->rows_alloc + h->rows_alloc / 2);
  cap = round_up(std::max<int64_t>(cap, kStepRows), kStepRows);
  float *C2 = nullptr, *ic2 = nullptr;
  uint32_t *lv2 = nullptr;
  _Float16 *xh2 = nullptr, *xl2 = nullptr;
  const size_t nel = (size_t)cap * h->ld;
  if (hipMalloc(&C2, nel * 4) != hipSuccess || hipMalloc(&ic2, (size_t)cap * 4) != hipSuccess ||
      hipMalloc(&lv2, (size_t)cap / 8) != hipSuccess || hipMalloc(&xh2, nel * 2) != hipSuccess ||
      hipMalloc(&xl2, nel * 2) != hipSuccess) {
    for (void *p : {(void *)C2, (void *)ic2, (void *)lv2, (void *)xh2, (void *)xl2})
      if (p) (void)hipFree(p);
    CM_FAIL(CM_ENOMEM, "dense: out of device memory");
  }
  CM_HIP(hipMemsetAsync(C2, 0, nel * 4, h->stream));
  CM_HIP(hipMemsetAsync(ic2, 0, (size_t)cap * 4, h->stream));
  CM_HIP(hipMemsetAsync(lv2, 0, (size_t)cap / 8, h->stream));
  CM_HIP(hipMemsetAsync(xh2, 0, nel * 2, h->stream));
  CM_HIP(hipMemsetAsync(xl2, 0, nel * 2, h->stream));
  if (h->rows_alloc) {
    const size_t old = (size_t)h->rows_alloc * h->ld;
    CM_HIP(hipMemcpyAsync(C2, h->C, old * 4, hipMemcpyDeviceToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(ic2, h->invc, (size_t)h->rows_alloc * 4, hipMemcpyDeviceToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(lv2, h->live, (size_t)h->rows_alloc / 8, hipMemcpyDeviceToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(xh2, h->Xh, old * 2, hipMemcpyDeviceToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(xl2, h->Xl, old * 2, hipMemcpyDeviceToDevice, h->stream));
  }
  CM_HIP(hipStreamSynchronize(h->stream));
  for (void *p : {(void *)h->C, (void *)h->invc, (void *)h->live, (void *)h->Xh, (void *)h->Xl})
    if (p) (void)hipFree(p);
  h->C = C2;
  h->invc = ic2;
  h->live = lv2;
  h->Xh = xh2;
  h->Xl = xl2;
  h->rows_alloc = cap;
  return CM_OK;
}

// CM_DENSE_DEBUG (ablation only): bit0 skip K1b's top-k epilogue.
int dense_debug_flags() {
  static const int f = [] {
    const char *e = getenv("CM_DENSE_DEBUG");
    return e ? atoi(e) : 0;
  }();
  return f;
}

// K1b (f16x3 planes, all queries of a pass resident) for large batches.
bool use_k1b(const cm_dense *h, int nq, int k) {
  static const int force = [] {
    const char *e = getenv("CM_DENSE_PATH");  // "f32" / "f16x3": force a path (A/B probes)
    return e ? (e[0] == 'f' && e[1] == '3' ? 1 : (e[0] == 'f' && e[1] == '1' ? 2 : 0)) : 0;
  }();
  if (force == 1) return false;
  if (k > kBMaxK || h->ld % 32) return false;
  if (force == 2) return true;
  return nq >= 64;
}

struct K1bCfg {
  int n_wg, n_pass;
  int64_t rows_per_wg, rows_end;
};
K1bCfg k1b_config(const cm_dense *h, int nq) {
  K1bCfg c{};
  c.n_pass = (int)ceil_div(nq, kBQPass);
  c.rows_end = round_up(std::max<int64_t>(h->size, 1), kBRows);
  const int64_t tiles = c.rows_end / kBRows;
  const int64_t want = std::max(1, num_cus(h->dev) / c.n_pass);
  const int64_t per = ceil_div(tiles, std::min<int64_t>(want, tiles));
  c.rows_per_wg = per * kBRows;
  c.n_wg = (int)ceil_div(tiles, per);
  return c;
}

struct K1bWs {
  _Float16 *qh, *ql;
  uint64_t *cand;
  size_t total;
};
K1bWs k1b_ws_layout(const cm_dense *h, const K1bCfg &c, int k, void *base) {
  K1bWs w{};
  char *p = reinterpret_cast<char *>(base);
  size_t off = 0;
  const int64_t nq_pad = (int64_t)c.n_pass * kBQPass;
  w.qh = reinterpret_cast<_Float16 *>(p + off);
  off += round_up(nq_pad * h->ld * 2, 256);
  w.ql = reinterpret_cast<_Float16 *>(p + off);
  off += round_up(nq_pad * h->ld * 2, 256);
  w.cand = reinterpret_cast<uint64_t *>(p + off);
  off += round_up((int64_t)c.n_pass * c.n_wg * kBQPass * k * 8, 256);
  w.total = off;
  return w;
}

int launch_k1b(cm_dense *h, const float *q_dev, int nq, int k, const uint32_t *allow, float *dist_dev,
               int64_t *row_dev, void *ws, int64_t ws_bytes, hipStream_t st) {
  static std::once_flag once;
  static hipError_t attr_err = hipSuccess;
  std::call_once(once, [] {
    attr_err = hipFuncSetAttribute(reinterpret_cast<const void *>(&dense_f16x3_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, k1b_lds_layout().total);
  });
  CM_HIP(attr_err);
  const K1bCfg c = k1b_config(h, nq);
  const K1bWs w = k1b_ws_layout(h, c, k, ws);
  if ((int64_t)w.total > ws_bytes || !ws) CM_FAIL(CM_EINVAL, "dense workspace too small");
  hipLaunchKernelGGL(dense_prep_planes, dim3(c.n_pass * kBQPass), dim3(256), 0, st, q_dev, nq, h->dim, h->ld, w.qh,
                     w.ql);
  CM_HIP(hipGetLastError());
  hipLaunchKernelGGL(dense_f16x3_kernel, dim3(c.n_wg * c.n_pass), dim3(512), k1b_lds_layout().total, st, h->Xh, h->Xl,
                     h->ld, h->live, allow, ceil_div(h->size, 32), w.qh, w.ql, nq, k, c.rows_per_wg, c.rows_end,
                     c.n_wg, w.cand, dense_debug_flags());
  CM_HIP(hipGetLastError());
  hipLaunchKernelGGL(dense_merge_kernel, dim3(nq), dim3(256), 0, st, w.cand, c.n_wg, kBQPass, k, nq, dist_dev,
                     row_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

}  // namespace

extern "C" {

int cm_max_topk(void) { return kMaxTopK; }

int cm_dense_create(int device, int32_t dim, int64_t capacity, cm_dense **out) {
  if (!out) CM_FAIL(CM_EINVAL, "out is NULL");
  *out = nullptr;
  if (dim <= 0 || dim > 2048) CM_FAIL(CM_EINVAL, "dim must be in [1, 2048]");
  if (capacity < 0) CM_FAIL(CM_EINVAL, "capacity must be >= 0");
  DeviceGuard dg(device);
  if (!dg.ok) CM_FAIL(CM_EDEVICE, "cannot select device " + std::to_string(device));
  cm_dense *h = new cm_dense();
  h->dev = device;
  h->dim = dim;
  int ld = (int)round_up(dim, 128);
  while (!pick_chunk(ld)) ld += 128;
  h->ld = ld;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamDefault) != hipSuccess) {
    delete h;
    CM_FAIL(CM_EDEVICE, "hipStreamCreate failed");
  }
  int rc = dense_grow(h, std::max<int64_t>(capacity, kStepRows));
  if (rc) {
    cm_dense_destroy(h);
    return rc;
  }
  *out = h;
  return CM_OK;
}

void cm_dense_destroy(cm_dense *h) {
  if (!h) return;
  DeviceGuard dg(h->dev);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->C) (void)hipFree(h->C);
  if (h->invc) (void)hipFree(h->invc);
  if (h->live) (void)hipFree(h->live);
  if (h->Xh) (void)hipFree(h->Xh);
  if (h->Xl) (void)hipFree(h->Xl);
  h->staging.release();
  h->rows_buf.release();
  h->allow_buf.release();
  h->ws.release();
  h->out_buf.release();
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int cm_dense_reserve(cm_dense *h, int64_t capacity) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  DeviceGuard dg(h->dev);
  return dense_grow(h, capacity);
}

int cm_dense_upsert(cm_dense *h, const float *vecs, const int64_t *rows, int64_t n) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (n < 0) CM_FAIL(CM_EINVAL, "n must be >= 0");
  if (n == 0) return CM_OK;
  if (!vecs || !rows) CM_FAIL(CM_EINVAL, "vecs/rows are NULL");
  int64_t mx = -1;
  for (int64_t i = 0; i < n; ++i) {
    if (rows[i] < 0 || rows[i] >= (int64_t)0xffffffffll) CM_FAIL(CM_EINVAL, "row index out of range");
    mx = std::max(mx, rows[i]);
  }
  DeviceGuard dg(h->dev);
  int rc = dense_grow(h, mx + 1);
  if (rc) return rc;
  const int64_t batch = 65536;
  for (int64_t s = 0; s < n; s += batch) {
    const int64_t m = std::min(batch, n - s);
    if ((rc = h->staging.ensure((size_t)m * h->dim * 4))) return rc;
    if ((rc = h->rows_buf.ensure((size_t)m * 8))) return rc;
    CM_HIP(hipMemcpyAsync(h->staging.ptr, vecs + s * h->dim, (size_t)m * h->dim * 4, hipMemcpyHostToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(h->rows_buf.ptr, rows + s, (size_t)m * 8, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(dense_scatter_kernel, dim3((unsigned)m), dim3(256), 0, h->stream, h->staging.as<float>(),
                       h->rows_buf.as<int64_t>(), (int64_t)0, m, h->dim, h->ld, h->C, h->invc, h->live, h->Xh, h->Xl);
    CM_HIP(hipGetLastError());
    CM_HIP(hipStreamSynchronize(h->stream));
  }
  h->size = std::max(h->size, mx + 1);
  return CM_OK;
}

int cm_dense_upsert_dev(cm_dense *h, const float *vecs_dev, int64_t row0, int64_t n, void *stream) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (n < 0 || row0 < 0 || row0 + n >= (int64_t)0xffffffffll) CM_FAIL(CM_EINVAL, "bad row range");
  if (n == 0) return CM_OK;
  DeviceGuard dg(h->dev);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch default)
  if (row0 + n > h->rows_alloc) {
    CM_HIP(hipStreamSynchronize(st));
    int rc = dense_grow(h, row0 + n);
    if (rc) return rc;
  }
  const int64_t batch = 1 << 30;
  for (int64_t s = 0; s < n; s += batch) {
    const int64_t m = std::min(batch, n - s);
    hipLaunchKernelGGL(dense_scatter_kernel, dim3((unsigned)m), dim3(256), 0, st, vecs_dev + s * h->dim,
                       (const int64_t *)nullptr, row0 + s, m, h->dim, h->ld, h->C, h->invc, h->live, h->Xh,
                       h->Xl);
    CM_HIP(hipGetLastError());
  }
  h->size = std::max(h->size, row0 + n);
  return CM_OK;
}

int cm_dense_delete(cm_dense *h, const int64_t *rows, int64_t n) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (n <= 0) return CM_OK;
  if (!rows) CM_FAIL(CM_EINVAL, "rows is NULL");
  DeviceGuard dg(h->dev);
  int rc = h->rows_buf.ensure((size_t)n * 8);
  if (rc) return rc;
  CM_HIP(hipMemcpyAsync(h->rows_buf.ptr, rows, (size_t)n * 8, hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(dense_clear_live_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, h->stream,
                     h->rows_buf.as<int64_t>(), n, h->size, h->live);
  CM_HIP(hipGetLastError());
  CM_HIP(hipStreamSynchronize(h->stream));
  return CM_OK;
}

int cm_dense_reset(cm_dense *h) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  DeviceGuard dg(h->dev);
  CM_HIP(hipMemsetAsync(h->live, 0, (size_t)h->rows_alloc / 8, h->stream));
  CM_HIP(hipMemsetAsync(h->invc, 0, (size_t)h->rows_alloc * 4, h->stream));
  CM_HIP(hipMemsetAsync(h->C, 0, (size_t)h->rows_alloc * h->ld * 4, h->stream));
  CM_HIP(hipMemsetAsync(h->Xh, 0, (size_t)h->rows_alloc * h->ld * 2, h->stream));
  CM_HIP(hipMemsetAsync(h->Xl, 0, (size_t)h->rows_alloc * h->ld * 2, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  h->size = 0;
  return CM_OK;
}

int64_t cm_dense_size(cm_dense *h) { return h ? h->size : -1; }
int32_t cm_dense_dim(cm_dense *h) { return h ? h->dim : -1; }
const uint32_t *cm_dense_live_bits_dev(cm_dense *h) { return h ? h->live : nullptr; }

int64_t cm_dense_live_count(cm_dense *h) {
  if (!h) return -1;
  DeviceGuard dg(h->dev);
  if (h->out_buf.ensure(8)) return -1;
  if (hipMemsetAsync(h->out_buf.ptr, 0, 8, h->stream) != hipSuccess) return -1;
  const int64_t nw = ceil_div(h->size, 32);
  if (nw > 0)
    hipLaunchKernelGGL(popcount_kernel, dim3((unsigned)std::min<int64_t>(1024, ceil_div(nw, 256))), dim3(256), 0,
                       h->stream, h->live, nw, h->out_buf.as<unsigned long long>());
  unsigned long long c = 0;
  if (hipMemcpyAsync(&c, h->out_buf.ptr, 8, hipMemcpyDeviceToHost, h->stream) != hipSuccess) return -1;
  if (hipStreamSynchronize(h->stream) != hipSuccess) return -1;
  return (int64_t)c;
}

int64_t cm_dense_search_workspace(cm_dense *h, int32_t nq, int32_t k) {
  if (!h || nq <= 0 || k <= 0 || k > kMaxTopK) return -1;
  if (use_k1b(h, nq, k)) return (int64_t)k1b_ws_layout(h, k1b_config(h, nq), k, nullptr).total;
  DenseCfg c = dense_config(h, nq, k);
  return (int64_t)dense_ws_layout(h, c, nq, k, nullptr).total;
}

int cm_dense_search_dev(cm_dense *h, const float *q_dev, int32_t nq, int32_t k, const uint32_t *allow_dev,
                        float *dist_dev, int64_t *row_dev, void *workspace_dev, int64_t workspace_bytes,
                        void *stream) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (k <= 0 || k > kMaxTopK) CM_FAIL(CM_EINVAL, "k must be in [1, " + std::to_string(kMaxTopK) + "]");
  DeviceGuard dg(h->dev);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch default)
  if (use_k1b(h, nq, k)) return launch_k1b(h, q_dev, nq, k, allow_dev, dist_dev, row_dev, workspace_dev, workspace_bytes, st);
  DenseCfg c = dense_config(h, nq, k);
  if (c.lds > 163840) CM_FAIL(CM_EUNSUPPORTED, "dim/k too large for the LDS-resident query tile");
  DenseWs w = dense_ws_layout(h, c, nq, k, workspace_dev);
  if ((int64_t)w.total > workspace_bytes || !workspace_dev) CM_FAIL(CM_EINVAL, "dense workspace too small");
  const int nq_pad = c.n_qgroups * c.QB;
  hipLaunchKernelGGL(dense_prep_queries, dim3(nq_pad), dim3(256), 0, st, q_dev, nq, h->dim, h->ld, w.qp, w.invq);
  CM_HIP(hipGetLastError());
  int rc = launch_dense(c, h, allow_dev, w.qp, w.invq, nq, k, w.cand, st);
  if (rc) return rc;
  hipLaunchKernelGGL(dense_merge_kernel, dim3(nq), dim3(256), 0, st, w.cand, c.n_cblocks, c.QB, k, nq, dist_dev,
                     row_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int cm_dense_gather_dev(cm_dense *h, const int64_t *rows_dev, int64_t n, float *out_dev, void *stream) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (n <= 0) return CM_OK;
  DeviceGuard dg(h->dev);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch default)
  hipLaunchKernelGGL(dense_gather_kernel, dim3((unsigned)n), dim3(256), 0, st, h->C, h->ld, h->dim, rows_dev, n,
                     h->size, out_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int cm_dense_export(cm_dense *h, int64_t row0, int64_t n, float *out, uint32_t *live_out) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (row0 < 0 || n < 0 || row0 + n > h->size) CM_FAIL(CM_EINVAL, "row range out of bounds");
  if (n == 0) return CM_OK;
  DeviceGuard dg(h->dev);
  if (out) {
    if (h->ld == h->dim) {
      CM_HIP(hipMemcpyAsync(out, h->C + row0 * h->ld, (size_t)n * h->dim * 4, hipMemcpyDeviceToHost, h->stream));
    } else {
      CM_HIP(hipMemcpy2DAsync(out, (size_t)h->dim * 4, h->C + row0 * h->ld, (size_t)h->ld * 4, (size_t)h->dim * 4,
                              (size_t)n, hipMemcpyDeviceToHost, h->stream));
    }
  }
  if (live_out) {
    if (row0 % 32) CM_FAIL(CM_EINVAL, "live export needs row0 % 32 == 0");
    CM_HIP(hipMemcpyAsync(live_out, h->live + row0 / 32, (size_t)ceil_div(n, 32) * 4, hipMemcpyDeviceToHost,
                          h->stream));
  }
  CM_HIP(hipStreamSynchronize(h->stream));
  return CM_OK;
}

int cm_dense_search(cm_dense *h, const float *q, int32_t nq, int32_t k, const uint32_t *allow_bits,
                    float *out_dist, int64_t *out_row, float *out_vec) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (!q || !out_dist || !out_row) CM_FAIL(CM_EINVAL, "NULL argument");
  if (k <= 0 || k > kMaxTopK) CM_FAIL(CM_EINVAL, "k must be in [1, " + std::to_string(kMaxTopK) + "]");
  DeviceGuard dg(h->dev);
  const int64_t wsb = cm_dense_search_workspace(h, nq, k);
  int rc;
  if ((rc = h->ws.ensure((size_t)wsb))) return rc;
  const size_t qbytes = (size_t)nq * h->dim * 4;
  const size_t obytes = (size_t)nq * k * (4 + 8);
  const size_t vbytes = out_vec ? (size_t)nq * k * h->dim * 4 : 0;
  if ((rc = h->staging.ensure(qbytes))) return rc;
  if ((rc = h->out_buf.ensure(round_up(obytes, 256) + vbytes))) return rc;
  const uint32_t *allow_dev = nullptr;
  if (allow_bits) {
    const int64_t nw = ceil_div(h->size, 32);
    if ((rc = h->allow_buf.ensure((size_t)std::max<int64_t>(nw, 1) * 4))) return rc;
    CM_HIP(hipMemcpyAsync(h->allow_buf.ptr, allow_bits, (size_t)nw * 4, hipMemcpyHostToDevice, h->stream));
    allow_dev = h->allow_buf.as<uint32_t>();
  }
  CM_HIP(hipMemcpyAsync(h->staging.ptr, q, qbytes, hipMemcpyHostToDevice, h->stream));
  float *d_dist = h->out_buf.as<float>();
  int64_t *d_row = reinterpret_cast<int64_t *>(h->out_buf.as<char>() + round_up((int64_t)nq * k * 4, 8));
  rc = cm_dense_search_dev(h, h->staging.as<float>(), nq, k, allow_dev, d_dist, d_row, h->ws.ptr, wsb, h->stream);
  if (rc) return rc;
  float *d_vec = nullptr;
  if (out_vec) {
    d_vec = reinterpret_cast<float *>(h->out_buf.as<char>() + round_up(obytes, 256));
    rc = cm_dense_gather_dev(h, d_row, (int64_t)nq * k, d_vec, h->stream);
    if (rc) return rc;
  }
  CM_HIP(hipMemcpyAsync(out_dist, d_dist, (size_t)nq * k * 4, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipMemcpyAsync(out_row, d_row, (size_t)nq * k * 8, hipMemcpyDeviceToHost, h->stream));
  if (out_vec) CM_HIP(hipMemcpyAsync(out_vec, d_vec, vbytes, hipMemcpyDeviceToHost, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  return CM_OK;
}

}  // extern "C"
