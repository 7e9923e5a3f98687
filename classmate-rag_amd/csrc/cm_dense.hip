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
// K1b / K1c: batched cosine top-k on normalised fp16 planes, one template.
//   xn = c * invc (hnswlib normalize_vector), Xh = f16(xn), Xl = f16(xn - Xh).
//   NPL = 2 (K1b, "f16x3"): reads both planes; xn.qn = xh.qh + xh.ql + xl.qh
//       (+ xl.ql dropped, <= 2^-22 relative) -> f32-grade distances.
//   NPL = 1 (K1c, "coarse"): reads only Xh (2 B per element, half of K1/K1b's
//       HBM bytes) and one product xh.qh per block; the lists hold k' = k + 4
//       coarse keys per range and dense_rerank_kernel certifies them with a
//       rigorous error bound before re-ranking the band exactly.
// A chunk is always 1024 x 16 B = 128 rows x 2 sub-blocks x 32 f16 staged
// through double-buffered LDS: for NPL = 2 the sub-blocks are the two planes of
// one 32-deep k slice, for NPL = 1 the two halves of one 64-deep k slice of Xh,
// so both variants share the LDS image, the load pattern and the fragment reads.
//
// One 512-thread workgroup per (corpus range, pass of 256 queries): the whole
// query pass is resident (wave w owns queries 32w..32w+31, fragments streamed
// from L2 one chunk ahead), so every corpus byte is read from HBM once per pass.
// After each 128-row tile every wave filters its 32 x 128 distances against its
// queries' running k-th keys (a per-query max over the lane's 32 values first, so
// tiles without a survivor cost one compare per query) and rank-merges survivors
// into per-query sorted lists in LDS.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// Plane layout (Xh, Xl): tile-major, so every 128-row x 64-f16 chunk the scans stream is one
// contiguous 16 KB block (row-major planes made each chunk 128 row segments 1.5 KB apart and
// reopened every DRAM page once per chunk):  element (row, k) of a plane with row pitch ld lives
// at ((row / 128) * (ld / 64) + k / 64) * 8192 + (row % 128) * 64 + k % 64.
__host__ __device__ inline int64_t plane_off(int64_t row, int k, int ld) {
  return (((row >> 7) * (ld >> 6) + (k >> 6)) << 13) + ((row & 127) << 6) + (k & 63);
}
constexpr int kBRows = 128;                 // corpus rows per tile
constexpr int kBPad = 32;                   // f16 per LDS row (unpadded; 16-B chunks XOR-swizzled, see lds_swz)
constexpr int kBQPass = 256;                // queries per pass (8 waves x 32)
constexpr int kBQWave = 32;
constexpr int kBSlots = 60;                 // per query: sorted list (len <= k) then unmerged survivors
constexpr int kBMaxK = 32;                  // k <= 32 leaves >= 28 buffer slots (one sub-tile adds <= 16)
constexpr int kBXBuf = 2 * kBRows * kBPad;  // f16 per LDS stage buffer (2 sub-blocks)
// 16-B chunk swizzle of an LDS row: chunk c of row r lives at c ^ lds_swz(r).  Conflict-free for
// both the MFMA fragment reads (ds_read_b128: lanes (g, j) read chunk g of row j; gfx950 serves
// lane groups {0-3,12-15,20-27}, ... in one cycle each) and the staging writes (ds_write_b128,
// 8 contiguous lanes = two rows x four chunks), checked exhaustively on the host.
__host__ __device__ inline int lds_swz(int row) { return ((row >> 3) & 1) << 1; }
constexpr int kRerankCap = 1024;            // certified band size per query handled by the re-rank kernel

struct K1bLds {
  int xs, thr, thrd, cnt, len, list, buf, act, total;
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
  L.act = off;
  off += 16;
  L.total = off;
  return L;
}

// Normalise + split queries into Qh/Ql [nq_pad][ld] (zero rows beyond nq) and
// record per query {||q||, ||qh||, ||ql||} (fp32, for K1c's error bound).
__global__ void __launch_bounds__(256) dense_prep_planes(const float *__restrict__ q, int nq, int dim, int ld,
                                                         _Float16 *__restrict__ Qh, _Float16 *__restrict__ Ql,
                                                         float *__restrict__ qnorm) {
  const int qi = blockIdx.x;
  const float *src = q + (int64_t)qi * dim;
  float s = 0.f;
  for (int i = threadIdx.x; i < dim; i += 256) {
    const float v = qi < nq ? src[i] : 0.f;
    s += v * v;
  }
  __shared__ float red[3][4];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = s;
  __syncthreads();
  const float t = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  const float inv = 1.0f / (sqrtf(t) + 1e-30f);
  float sh = 0.f, sl = 0.f;
  for (int i = threadIdx.x; i < ld; i += 256) {
    const float v = (qi < nq && i < dim) ? src[i] * inv : 0.f;
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)hi);
    Qh[(int64_t)qi * ld + i] = hi;
    Ql[(int64_t)qi * ld + i] = lo;
    sh += (float)hi * (float)hi;
    sl += (float)lo * (float)lo;
  }
  for (int o = 32; o > 0; o >>= 1) {
    sh += __shfl_xor(sh, o);
    sl += __shfl_xor(sl, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[1][threadIdx.x >> 6] = sh;
    red[2][threadIdx.x >> 6] = sl;
  }
  __syncthreads();
  if (threadIdx.x == 0 && qnorm) {
    qnorm[4 * qi + 0] = sqrtf(t);
    qnorm[4 * qi + 1] = sqrtf((red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
    qnorm[4 * qi + 2] = sqrtf((red[2][0] + red[2][1]) + (red[2][2] + red[2][3]));
    qnorm[4 * qi + 3] = 0.f;
  }
}

// qmask (nullable): only queries with qmask[q] != 0 are searched (K1c's fallback
// pass); a workgroup whose pass has none exits before touching the corpus.
template <int NPL>
__global__ void __launch_bounds__(512, 1)
    dense_split_kernel(const _Float16 *__restrict__ Xh, const _Float16 *__restrict__ Xl, int ld,
                       const uint32_t *__restrict__ live, const uint32_t *__restrict__ allow, int64_t n_words,
                       const _Float16 *__restrict__ Qh, const _Float16 *__restrict__ Ql, int nq,
                       const int32_t *__restrict__ qmask, int k, int64_t rows_per_wg, int64_t rows_end, int n_wg,
                       uint64_t *__restrict__ cand, int dbg) {
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
  int32_t *act = reinterpret_cast<int32_t *>(lds + L.act);
  if (qmask) {
    if (tid == 0) act[0] = 0;
    __syncthreads();
    const int qq = qp * kBQPass + tid;
    if (tid < kBQPass && qq < nq && qmask[qq]) act[0] = 1;
    __syncthreads();
    if (act[0] == 0) return;  // whole workgroup: no query of this pass is active
  }
  if (lane < kBQWave) {
    const int qq = qg0 + lane;
    const bool real = qq < nq && (!qmask || qmask[qq]);
    thr[lane] = real ? kEmptyKey : 0ull;  // padded / inactive queries accept nothing
    thrd[lane] = real ? __builtin_inff() : -__builtin_inff();
    cnt[lane] = 0;
    len[lane] = 0;
  }
  const int64_t r_begin = (int64_t)wg * rows_per_wg;
  const int64_t r_end = min(r_begin + rows_per_wg, rows_end);
  const int ntiles = r_begin < r_end ? (int)((r_end - r_begin) / kBRows) : 0;
  const int KC = ld / (32 * (3 - NPL));  // chunks per tile: 32-deep (NPL 2) or 64-deep (NPL 1)
  const int total = ntiles * KC;

  // staging pieces of a chunk: 1024 x 16 B (sub-block, row, 8-f16 part); thread takes tid and tid + 512
  auto xsrc = [&](int gc, int p) -> const f16x8 * {
    const int t = gc / KC, c = gc - t * KC;
    const int sb = p >> 9, row = (p & 511) >> 2, part = p & 3;
    const int64_t rg = r_begin + (int64_t)t * kBRows + row;
    if (NPL == 2) return reinterpret_cast<const f16x8 *>((sb ? Xl : Xh) + plane_off(rg, c * 32 + part * 8, ld));
    return reinterpret_cast<const f16x8 *>(Xh + plane_off(rg, c * 64 + sb * 32 + part * 8, ld));
  };
  auto xdst = [&](int b, int p) -> f16x8 * {
    const int sb = p >> 9, row = (p & 511) >> 2, part = p & 3;
    return reinterpret_cast<f16x8 *>(xs + b * kBXBuf + sb * kBRows * kBPad + row * kBPad + (part ^ lds_swz(row)) * 8);
  };
  // query fragments (B operand): lane (g, j) of q-tile qt holds q[qt*16 + j][.. + 8g .. +7] of
  // sub-block 0 (qa) and 1 (qb): NPL 2 -> (Qh, Ql) of the 32-deep slice, NPL 1 -> Qh halves
  auto qload = [&](f16x8 (&qa)[2], f16x8 (&qb)[2], int gc) {
    const int c = gc % KC;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int64_t rb = (int64_t)(qg0 + qt * 16 + j) * ld;
      if (NPL == 2) {
        qa[qt] = *reinterpret_cast<const f16x8 *>(Qh + rb + c * 32 + g * 8);
        qb[qt] = *reinterpret_cast<const f16x8 *>(Ql + rb + c * 32 + g * 8);
      } else {
        qa[qt] = *reinterpret_cast<const f16x8 *>(Qh + rb + c * 64 + g * 8);
        qb[qt] = *reinterpret_cast<const f16x8 *>(Qh + rb + c * 64 + 32 + g * 8);
      }
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
      // quick reject: the lane's best of its 32 rows for this query against the running k-th
      float mx = acc[0][qt][0];
#pragma unroll
      for (int rt = 0; rt < 8; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, acc[rt][qt][r]);
      if (__ballot(1.0f - mx <= thrd[ql_]) == 0) continue;
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
            if (key < tk && !(dbg & 16)) {
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
    // MFMA work); query fragments one chunk ahead (L2).  KC is a multiple of 4 (checked on
    // the host), so a tile is a whole number of ring turns and the epilogue (no vector-memory
    // loads) sits outside the unrolled bodies: every wait is a counted vmcnt, not a drain.
    f16x8 qa[2], qb[2], nqa[2], nqb[2];
    f16x8 ra0, ra1, rb0, rb1, rc0, rc1, rd0, rd1;
    auto xload = [&](f16x8 &x0, f16x8 &x1, int gc) {
      const int gl = min(gc, total - 1);  // clamped: one control path
      x0 = *xsrc(gl, tid);
      x1 = *xsrc(gl, tid + 512);
    };
    xload(ra0, ra1, 0);
    *xdst(0, tid) = ra0;
    *xdst(0, tid + 512) = ra1;
    qload(qa, qb, 0);
    xload(ra0, ra1, 1);
    xload(rb0, rb1, 2);
    xload(rc0, rc1, 3);
    xload(rd0, rd1, 4);
    __syncthreads();
    auto body = [&](int gc, f16x8 &x0, f16x8 &x1) {
      qload(nqa, nqb, min(gc + 1, total - 1));
      const _Float16 *xb = xs + (gc & 1) * kBXBuf;
      auto frag = [&](int rt, int sb) -> f16x8 {
        return *reinterpret_cast<const f16x8 *>(xb + sb * kBRows * kBPad + (rt * 16 + j) * kBPad +
                                                (g ^ lds_swz(j)) * 8);
      };
      // LDS fragments one 16-row sub-tile ahead of the MFMAs that use them
      f16x8 xa = frag(0, 0), xb1 = frag(0, 1);
#pragma unroll
      for (int rt = 0; rt < 8; ++rt) {
        f16x8 na = xa, nb = xb1;
        if (rt < 7) {
          na = frag(rt + 1, 0);
          nb = frag(rt + 1, 1);
        }
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          if (NPL == 2) {
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, qa[qt], acc[rt][qt], 0, 0, 0);
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, qb[qt], acc[rt][qt], 0, 0, 0);
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb1, qa[qt], acc[rt][qt], 0, 0, 0);
          } else {
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, qa[qt], acc[rt][qt], 0, 0, 0);
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb1, qb[qt], acc[rt][qt], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        xa = na;
        xb1 = nb;
      }
      *xdst((gc + 1) & 1, tid) = x0;  // chunk gc+1 (loaded four chunks ago)
      *xdst((gc + 1) & 1, tid + 512) = x1;
      xload(x0, x1, gc + 5);
      __syncthreads();
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        qa[qt] = nqa[qt];
        qb[qt] = nqb[qt];
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

// Waves per K1c workgroup.  4 (one per SIMD) is the measured best: 8 (two per SIMD, 32 queries
// each, 256 VGPRs with 16 spilled at tile boundaries) ran 5.63 vs 4.96 ms on the 10M x 768 scan --
// the second wave did not hide barrier/epilogue time.  Kept selectable for experiments.
#ifndef K1C_WAVES
#define K1C_WAVES 4
#endif
constexpr int kK1cWaves = K1C_WAVES;

// K1c's per-query error bound E (see dense_rerank_kernel).
__device__ inline float coarse_err(const float *qnorm, int qi, const float *row_norms, int dim) {
  const float qh = qnorm[4 * qi + 1], qlo = qnorm[4 * qi + 2];
  const float mxh = row_norms[0], mxl = row_norms[1];
  return (qlo * mxh + mxl * qh + mxl * qlo + (float)dim * 5.9604645e-8f * mxh * qh + 2e-6f) * 1.001f;
}

// ---------------------------------------------------------------------------
// K1c scan (coarse f16, Xh plane only), resident-query form for ld = 64 KC.
// 64 W threads (W = kK1cWaves: 4 -> one wave per SIMD, 8 -> two, so one wave's barrier wait, DMA
// issue and epilogue hide under the other's MFMAs); wave w owns queries 256w/W.. of the 256-query pass and
// keeps their Qh fragments resident -- chunks 0..KC-NQL-1 in registers (32 VGPRs each), the last
// NQL chunks in LDS -- so the corpus is the only memory stream: 64-row x 64-f16 chunks (8 KB; one
// glds wave-instruction = 8 rows x 128 B, full lines) LDS-DMA'd into a kRRing-slot ring, retired
// by a counted vmcnt and published by a raw s_barrier: no vmcnt(0) and no query reloads in the
// loop.  The ring image is 128-B rows with 16-B chunks XOR-swizzled by (row >> 1) & 7 on the glds
// SOURCE address (the DMA writes lane-linearly) and on the ds_read address: conflict-free
// fragment reads (checked exhaustively on the host).  Compute tiles are 64 rows.
//   MINONLY (sample pre-pass): per query, the minimum coarse distance over the workgroup's
//     live+allowed rows -> out_min[pass][wg][q].
//   main pass: every live+allowed row with coarse distance <= seed[q] is appended to the
//     (range, query) candidate buffer out_keys[pass][wg][q][kCBufCap] (LDS slot counter);
//     out_cnt[pass][wg][q] = appended count (> kCBufCap: the buffer overflowed).
#ifndef K1C_RING
#define K1C_RING 8
#endif
constexpr int kRRing = K1C_RING;  // LDS ring slots (8 KB each): kRRing - 1 chunks in flight per CU
constexpr int kRRows = 64;      // rows per compute tile / chunk
constexpr int kCBufCap = 64;    // candidate slots per (range, query)

template <int NQL>
struct K1rLds {
  static constexpr int ring = 0;
  static constexpr int qf = ring + kRRing * 8192;          // [NQL][W waves][32/W frags][64 lanes] x 16 B
  static constexpr int total = qf + NQL * 4 * 8 * 1024;
};
__device__ inline int ring_swz(int row) { return (row >> 1) & 7; }

template <int KC, int NQL, bool MINONLY, int W>
__global__ void __launch_bounds__(64 * W, 1)
    dense_coarse_scan_kernel(const _Float16 *__restrict__ Xh, const uint32_t *__restrict__ live,
                             const uint32_t *__restrict__ allow, int64_t n_words, const _Float16 *__restrict__ Qh,
                             int nq, const float *__restrict__ seed, int64_t rows_per_wg, int64_t rows_end, int n_wg,
                             uint64_t *__restrict__ out_keys, uint32_t *__restrict__ out_cnt,
                             float *__restrict__ out_min, int dbg) {
  constexpr int ld = 64 * KC;
  constexpr int KR = KC - NQL;  // register-resident query chunks
  using LL = K1rLds<NQL>;
  constexpr int QT = 16 / W;        // 16-query tiles per wave
  constexpr int NF = 2 * QT;        // query fragments per wave and chunk
  constexpr int PCS = 8 / W;        // 16-B DMA pieces per thread and chunk
  static_assert(W == 4 || W == 8, "K1c: 4 or 8 waves");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int j = lane & 15;
  const int wg = blockIdx.x % n_wg;
  const int qp = blockIdx.x / n_wg;
  const int64_t r_begin = (int64_t)wg * rows_per_wg;
  const int64_t r_end = min(r_begin + rows_per_wg, rows_end);
  const int ntiles = r_begin < r_end ? (int)((r_end - r_begin) / kRRows) : 0;
  const int total = ntiles * KC;
  const int qc0 = wave * 16 * QT;
  const int qg0 = qp * kBQPass + qc0;

  // resident query fragments (B operand): lane (g, j) of q-tile qt, chunk c, half sb holds
  // q[qt*16 + j][64c + 32sb + 8g .. +7]
  f16x8 qres[KR][QT][2];
  auto qsrc = [&](int c, int qt, int sb) -> const f16x8 * {
    return reinterpret_cast<const f16x8 *>(Qh + (int64_t)(qg0 + qt * 16 + j) * ld + c * 64 + sb * 32 + g * 8);
  };
#pragma unroll
  for (int c = 0; c < KR; ++c)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) qres[c][qt][sb] = *qsrc(c, qt, sb);
#pragma unroll
  for (int c = 0; c < NQL; ++c)
#pragma unroll
    for (int f = 0; f < NF; ++f)
      *reinterpret_cast<f16x8 *>(lds + LL::qf + ((c * W + wave) * NF + f) * 1024 + lane * 16) =
          *qsrc(KR + c, f >> 1, f & 1);
  // per-lane seeds of the lane's QT queries (qt*16 + j)
  float sd[QT], best[QT];
  uint32_t qcnt[QT];  // lanes g == 0: candidates appended for query qt*16 + j
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    best[qt] = __builtin_inff();
    qcnt[qt] = 0u;
    const int qq = qg0 + qt * 16 + j;
    sd[qt] = MINONLY ? 0.f : (qq < nq ? seed[qq] : -__builtin_inff());  // padded queries accept nothing
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // LDS query fragments ready; no DMA in flight yet

  // glds source of wave-instruction i (< PCS) of chunk gc: ring cell o16 = 64 W i + tid holds the
  // 16-B piece (row o16 >> 3, logical chunk (o16 & 7) ^ ring_swz(row)) of the tile-major plane
  auto issue = [&](int gc) __attribute__((always_inline)) {
    const int gl = min(gc, total - 1);  // clamped: one control path past the end
    const int t = gl / KC, c = gl - t * KC;
    const int64_t R0 = r_begin + (int64_t)t * kRRows;
    unsigned char *slot = lds + LL::ring + (gc % kRRing) * 8192;
#pragma unroll
    for (int i = 0; i < PCS; ++i) {
      const int o16 = 64 * W * i + tid;
      const int row = o16 >> 3, lg = (o16 & 7) ^ ring_swz(row);
      const _Float16 *src = Xh + ((((R0 >> 7) * KC + c) << 13) + (((R0 & 127) + row) << 6) + lg * 8);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                       (__attribute__((address_space(3))) void *)(slot + i * W * 1024 + wave * 1024), 16,
                                       0, 0);
    }
  };
  f32x4 acc[4][QT];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) acc[rt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint32_t tile_words = 0;  // lanes 0, 1: live & allow words of the current tile
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int64_t row0 = r_begin + (int64_t)t * kRRows;
    const int64_t w0 = row0 >> 5;  // wave-uniform: scalar loads, outside the DMA's vmcnt queue
    // lane (g, j) holds rows rt*16 + 4g + r: bit (16 rt + 4 g + r) of the 64-bit tile mask, whose
    // two words lanes 0 and 1 loaded when the tile started (tile_words: a vector load that lands
    // during the tile's chunks instead of a scalar load waited for here)
    (void)w0;
    auto tile_mask = [&]() -> uint64_t {
      const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)tile_words, 0);
      const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)tile_words, 1);
      return ((uint64_t)b1 << 32) | b0;
    };
    const uint64_t tmask = MINONLY ? tile_mask() : 0ull;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      if (MINONLY) {
        float m = __builtin_inff();
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if ((tmask >> (rt * 16 + 4 * g + r)) & 1u) m = fminf(m, 1.0f - acc[rt][qt][r]);
        best[qt] = fminf(best[qt], m);
      } else {
        float mx = -__builtin_inff();
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, acc[rt][qt][r]);
        if (__ballot(1.0f - mx <= sd[qt]) == 0) continue;  // no row of the tile under any seed
        const uint64_t tmask = tile_mask();
        // slots by ballot + popcount among the 4 lanes (g = 0..3) sharing query j; the count
        // lives in lane j's register (no LDS atomics: those would wait for the ring's DMAs)
        const int q = qc0 + qt * 16 + j;
        const uint64_t samej = 0x0001000100010001ull << j;
        uint64_t *dst = out_keys + (((int64_t)qp * n_wg + wg) * kBQPass + q) * kCBufCap;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rr = rt * 16 + 4 * g + r;
            const float dist = 1.0f - acc[rt][qt][r];
            const bool pred = ((tmask >> rr) & 1u) && dist <= sd[qt];
            const uint64_t m = __ballot(pred);
            if (m == 0) continue;
            const uint32_t base = __shfl(qcnt[qt], j);
            const uint32_t slot = base + (uint32_t)__popcll(m & samej & ((1ull << lane) - 1ull));
            if (pred && slot < (uint32_t)kCBufCap)
              dst[slot] = ((uint64_t)f32_order(dist) << 32) | (uint64_t)(uint32_t)(row0 + rr);
            if (g == 0) qcnt[qt] += (uint32_t)__popcll(m & samej);
          }
        }
      }
    }
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) acc[rt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  if (total > 0) {
    // Software-pipelined chunk loop.  Chunk gc's 32 MFMAs run in two halves (row tiles 0-1,
    // 2-3); between them the wave waits for chunk gc+1's DMA pieces, the barrier publishes
    // chunk gc+1 and retires every read of chunk gc's slot (each wave drains its LDS reads
    // first), chunk gc + kRRing is issued into that slot and the row fragments 0-1 of chunk gc+1
    // are read into the registers half 1 has just consumed; fragments 2-3 follow half 2.  Every
    // barrier, DMA issue and LDS read thus sits behind >= 16 MFMAs instead of in front of them.
    auto frag = [&](int gc, int rt, int sb) -> f16x8 {
      const unsigned char *slot = lds + LL::ring + (gc % kRRing) * 8192;
      const int row = rt * 16 + j;
      return *reinterpret_cast<const f16x8 *>(slot + row * 128 + (((sb * 4 + g) ^ ring_swz(row)) << 4));
    };
#pragma unroll
    for (int p = 0; p < kRRing - 1; ++p) issue(p);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PCS * (kRRing - 2)) : "memory");
    __builtin_amdgcn_s_barrier();
    issue(kRRing - 1);
    f16x8 xf[4][2];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      xf[rt][0] = frag(0, rt, 0);
      xf[rt][1] = frag(0, rt, 1);
    }
    f16x8 ql[QT][2];  // query fragments of an LDS-resident chunk (c >= KR)
    if (KR == 0) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int sb = 0; sb < 2; ++sb)
          ql[qt][sb] = *reinterpret_cast<const f16x8 *>(lds + LL::qf + ((0 * W + wave) * NF + qt * 2 + sb) * 1024 +
                                                        lane * 16);
    }
    for (int t = 0; t < ntiles; ++t) {
      {
        const int64_t wi = ((r_begin + (int64_t)t * kRRows) >> 5) + (lane & 1);  // lane-split: VMEM, not SMEM
        tile_words = wi < n_words ? (live[wi] & (allow ? allow[wi] : 0xffffffffu)) : 0u;
      }
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const int gc = t * KC + c;
        auto qv = [&](int qt, int sb) -> f16x8 { return c < KR ? qres[c < KR ? c : 0][qt][sb] : ql[qt][sb]; };
        // half 1: row tiles 0, 1
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
          for (int qt = 0; qt < QT; ++qt)
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[rt][0], qv(qt, 0), acc[rt][qt], 0, 0, 0);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt)
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[rt][1], qv(qt, 1), acc[rt][qt], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        // chunk gc+1 landed (this wave's pieces: the PCS (kRRing - 2) younger DMAs may stay in
        // flight); own LDS reads of slot gc done; the barrier makes both true for every wave
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PCS * (kRRing - 2)) : "memory");
        if (!(dbg & 512)) __builtin_amdgcn_s_barrier();  // bit 9: ablation only (races)
        if (!(dbg & 1024)) issue(gc + kRRing);             // bit 10: ablation only (stale data)
#pragma unroll
        for (int rt = 0; rt < ((dbg & 2048) ? 0 : 2); ++rt) {  // bit 11: ablation only (stale fragments)
          xf[rt][0] = frag(gc + 1, rt, 0);
          xf[rt][1] = frag(gc + 1, rt, 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        // half 2: row tiles 2, 3
#pragma unroll
        for (int rt = 2; rt < 4; ++rt) {
#pragma unroll
          for (int qt = 0; qt < QT; ++qt)
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[rt][0], qv(qt, 0), acc[rt][qt], 0, 0, 0);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt)
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[rt][1], qv(qt, 1), acc[rt][qt], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 2; rt < ((dbg & 2048) ? 2 : 4); ++rt) {  // bit 11: ablation only (stale fragments)
          xf[rt][0] = frag(gc + 1, rt, 0);
          xf[rt][1] = frag(gc + 1, rt, 1);
        }
        const int cn = (c + 1) % KC;  // next chunk's query fragments, when LDS-resident
        if (cn >= KR) {
#pragma unroll
          for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int sb = 0; sb < 2; ++sb)
              ql[qt][sb] = *reinterpret_cast<const f16x8 *>(
                  lds + LL::qf + (((cn - KR) * W + wave) * NF + qt * 2 + sb) * 1024 + lane * 16);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (!(dbg & 128)) epilogue(t);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // clamped tail DMAs land before the LDS is released
  }
  if (MINONLY) {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float m = best[qt];
      m = fminf(m, __shfl_xor(m, 16));
      m = fminf(m, __shfl_xor(m, 32));
      if (g == 0) out_min[((int64_t)qp * n_wg + wg) * kBQPass + qc0 + qt * 16 + j] = m;
    }
  } else if (g == 0) {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) out_cnt[((int64_t)qp * n_wg + wg) * kBQPass + qc0 + qt * 16 + j] = qcnt[qt];
  }
}

// K1c seed from the sample pre-pass: the k-th smallest of the n_wg per-workgroup minima bounds the
// k-th smallest coarse distance of the whole corpus (k distinct rows lie at or under it); + 2E.
// +inf when fewer than k groups hold an allowed row.
__global__ void __launch_bounds__(256) dense_seed_kernel(const float *__restrict__ mins, int n_wg, int k, int nq,
                                                         const float *__restrict__ qnorm,
                                                         const float *__restrict__ row_norms, int dim,
                                                         float *__restrict__ seed) {
  const int qi = blockIdx.x;
  if (qi >= nq) return;
  const int qp = qi / kBQPass, ql = qi - qp * kBQPass;
  __shared__ float v[2048];
  const int n = min(n_wg, 2048);
  for (int i = threadIdx.x; i < n; i += 256) v[i] = mins[((int64_t)qp * n_wg + i) * kBQPass + ql];
  __syncthreads();
  // the k-th smallest by rank counting (n <= 2048, ties broken by index)
  __shared__ float kth;
  if (threadIdx.x == 0) kth = __builtin_inff();
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) {
    const float x = v[i];
    if (!(x < __builtin_inff())) continue;
    int rank = 0;
    for (int m = 0; m < n; ++m) rank += (v[m] < x || (v[m] == x && m < i)) ? 1 : 0;
    if (rank == k - 1) kth = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) seed[qi] = kth < __builtin_inff() ? kth + 2.0f * coarse_err(qnorm, qi, row_norms, dim)
                                                           : __builtin_inff();
}

// Block-wide radix select: the k-th smallest (0-based kk) of n u32 values in LDS (4 x 8-bit digits).
__device__ inline uint32_t block_select_u32(const uint32_t *vals, int n, int kk, uint32_t *hist /*[256]*/) {
  __shared__ uint32_t s_prefix, s_rem;
  if (threadIdx.x == 0) {
    s_prefix = 0;
    s_rem = (uint32_t)kk;
  }
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    const uint32_t hmask = shift == 24 ? 0u : (0xffffffffu << (shift + 8));
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t x = vals[i];
      if ((x & hmask) == (prefix & hmask)) atomicAdd(&hist[(x >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t rem = s_rem, b = 0;
      while (hist[b] <= rem) rem -= hist[b++];
      s_prefix = prefix | (b << shift);
      s_rem = rem;
    }
    __syncthreads();
  }
  return s_prefix;
}

// K1c certification + exact re-rank, one 256-thread workgroup per query.
//   For every row |c - d| <= E with
//     E = ||ql|| max||xh|| + max||xl|| ||qh|| + max||xl|| ||ql|| + dim 2^-24 max||xh|| ||qh|| + 2e-6
//   (xn.qn = xh.qh + xh.ql + xl.qh + xl.ql, products exact in f32, accumulation error bounded by
//   the recursive-summation bound, 2e-6 for the normalisations).  With c_k the k-th smallest
//   coarse distance, every row of the exact top-k has c <= T = c_k + 2E <= seed, so it sits in
//   one of the n_wg candidate buffers unless that buffer overflowed (or the band exceeds
//   kRerankCap): then the query is flagged for the exact K1b pass.  Otherwise the band's rows are
//   re-ranked with fp64 dot products of the stored fp32 rows,
//   d = 1 - (c.q) / ((||c|| + 1e-30)(||q|| + 1e-30)), ties -> lower row.
constexpr int kGatherCap = 8192;  // candidates gathered per query
__global__ void __launch_bounds__(256) dense_rerank_kernel(
    const uint64_t *__restrict__ keys, const uint32_t *__restrict__ cnts, int n_wg, int k, int nq,
    const float *__restrict__ C, int ld, int dim, const float *__restrict__ q, const float *__restrict__ qnorm,
    const float *__restrict__ row_norms, float *__restrict__ out_dist, int64_t *__restrict__ out_row,
    int32_t *__restrict__ fb_mask, int32_t *__restrict__ fb_count) {
  const int qi = blockIdx.x;
  if (qi >= nq) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qp = qi / kBQPass, ql = qi - qp * kBQPass;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
  uint64_t *s_keys = reinterpret_cast<uint64_t *>(dyn);                        // [kGatherCap]
  uint32_t *s_dist = reinterpret_cast<uint32_t *>(dyn + kGatherCap * 8);      // [kGatherCap]
  __shared__ uint32_t s_off[2049];
  __shared__ uint32_t hist[256];
  __shared__ float s_q[2048];
  __shared__ int s_flag, s_total, s_band;
  __shared__ uint32_t s_rows[kRerankCap];
  __shared__ uint64_t s_ex[kRerankCap];
  if (tid == 0) {
    s_flag = 0;
    s_band = 0;
  }
  // 1. buffer sizes -> offsets (serial scan by one wave: n_wg <= 2048)
  __syncthreads();
  if (wave == 0) {
    uint32_t run = 0;
    for (int b0 = 0; b0 < n_wg; b0 += 64) {
      const int b = b0 + lane;
      uint32_t c = b < n_wg ? cnts[((int64_t)qp * n_wg + b) * kBQPass + ql] : 0u;
      if (c > (uint32_t)kCBufCap) {
        s_flag = 1;
        c = kCBufCap;
      }
      uint32_t incl = c;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      if (b < n_wg) s_off[b] = run + incl - c;
      run += __shfl(incl, 63);
    }
    if (lane == 0) {
      s_off[n_wg] = run;
      s_total = (int)run;
    }
  }
  __syncthreads();
  const int total = s_total;
  if (s_flag || total > kGatherCap) {
    if (tid == 0) {
      fb_mask[qi] = 1;
      atomicAdd(fb_count, 1);
    }
    return;  // the K1b pass writes this query's results
  }
  // 2. gather the candidates: thread per candidate slot j (its buffer = the last b with
  // s_off[b] <= j; empty buffers share offsets), so every load is independent instead of one
  // global round trip per buffer and wave
  for (int j = tid; j < total; j += 256) {
    int lo = 0, hi = n_wg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_off[mid] <= (uint32_t)j) lo = mid;
      else hi = mid - 1;
    }
    const uint64_t key = keys[(((int64_t)qp * n_wg + lo) * kBQPass + ql) * kCBufCap + (j - s_off[lo])];
    s_keys[j] = key;
    s_dist[j] = (uint32_t)(key >> 32);
  }
  for (int i = tid; i < dim; i += 256) s_q[i] = q[(int64_t)qi * dim + i];
  __syncthreads();
  // 3. band threshold from the k-th smallest coarse distance
  uint32_t tkey = 0xffffffffu;  // fewer than k candidates: all of them
  if (total >= k) {
    const uint32_t ck = block_select_u32(s_dist, total, k - 1, hist);
    tkey = f32_order(f32_unorder(ck) + 2.0f * coarse_err(qnorm, qi, row_norms, dim));
  }
  for (int i = tid; i < total; i += 256) {
    if (s_dist[i] <= tkey) {
      const int p = atomicAdd(&s_band, 1);
      if (p < kRerankCap) s_rows[p] = (uint32_t)s_keys[i];
    }
  }
  __syncthreads();
  const int band = s_band;
  if (band > kRerankCap) {
    if (tid == 0) {
      fb_mask[qi] = 1;
      atomicAdd(fb_count, 1);
    }
    return;
  }
  if (tid == 0) fb_mask[qi] = 0;
  // 4. exact distances, one wave per band row
  const double qnrm = (double)qnorm[4 * qi + 0];
  for (int c = wave; c < band; c += 4) {
    const uint32_t row = s_rows[c];
    const float *cr = C + (int64_t)row * ld;
    double dq = 0.0, dc = 0.0;
    for (int i = lane; i < dim; i += 64) {
      const double x = (double)cr[i];
      dq += x * (double)s_q[i];
      dc += x * x;
    }
    for (int o = 32; o > 0; o >>= 1) {
      dq += __shfl_xor(dq, o);
      dc += __shfl_xor(dc, o);
    }
    if (lane == 0) {
      const float dist = (float)(1.0 - dq / ((sqrt(dc) + 1e-30) * (qnrm + 1e-30)));
      s_ex[c] = ((uint64_t)f32_order(dist) << 32) | row;
    }
  }
  __syncthreads();
  // 5. top-k of the band by rank
  for (int c = tid; c < band; c += 256) {
    const uint64_t key = s_ex[c];
    int rank = 0;
    for (int i = 0; i < band; ++i) rank += s_ex[i] < key ? 1 : 0;
    if (rank < k) {
      out_dist[(int64_t)qi * k + rank] = f32_unorder((uint32_t)(key >> 32));
      out_row[(int64_t)qi * k + rank] = (int64_t)(uint32_t)key;
    }
  }
  for (int i = band + tid; i < k; i += 256) {
    out_dist[(int64_t)qi * k + i] = 0.f;
    out_row[(int64_t)qi * k + i] = -1;
  }
}

// Tournament merge of n_cblocks sorted lists per query -> final top-k.
// qmask (nullable): only queries with qmask[q] != 0 are written.
__global__ void __launch_bounds__(256) dense_merge_kernel(const uint64_t *__restrict__ cand, int n_cblocks, int QB,
                                                          int k, int nq, const int32_t *__restrict__ qmask,
                                                          float *__restrict__ out_dist,
                                                          int64_t *__restrict__ out_row) {
  const int q = blockIdx.x;
  if (q >= nq || (qmask && !qmask[q])) return;
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
                                                            _Float16 *__restrict__ Xl, uint32_t *__restrict__ rnorm) {
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
  float sh = 0.f, sl = 0.f;
  for (int c = threadIdx.x; c < ld; c += 256) {
    const float xn = (c < dim ? s[c] : 0.f) * inv;
    const _Float16 hi = (_Float16)xn;
    const _Float16 lo = (_Float16)(xn - (float)hi);
    Xh[plane_off(r, c, ld)] = hi;
    Xl[plane_off(r, c, ld)] = lo;
    sh += (float)hi * (float)hi;
    sl += (float)lo * (float)lo;
  }
  // running maxima of ||Xh_r|| and ||Xl_r|| (K1c's error bound; non-negative floats order as
  // their bit patterns); never lowered by deletes, so the bound stays conservative
  for (int o = 32; o > 0; o >>= 1) {
    sh += __shfl_xor(sh, o);
    sl += __shfl_xor(sl, o);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = sh;
  }
  __shared__ float red2[4];
  if ((threadIdx.x & 63) == 0) red2[threadIdx.x >> 6] = sl;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float nh = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    const float nl = sqrtf((red2[0] + red2[1]) + (red2[2] + red2[3]));
    atomicMax(&rnorm[0], __float_as_uint(nh));
    atomicMax(&rnorm[1], __float_as_uint(nl));
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
  _Float16 *Xh = nullptr, *Xl = nullptr;  // normalised f16 split planes (K1b/K1c)
  float *rnorm = nullptr;                  // device {max ||Xh_r||, max ||Xl_r||} (K1c bound)
  int path = 0;                            // cm_dense_set_path (0 = automatic)
  int32_t last_fallbacks = -1;             // K1c queries re-run exactly by the last host search
  KernelTimer timer;                       // scan-kernel events (cm_dense_timing)
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

// CM_DENSE_DEBUG (ablation only) for the scan kernels: bit0 skip the top-k epilogue, bit4 filter
// without inserting survivors, bit5 (K1c) no sample pre-pass, bit6 (K1c) no MFMAs, bit7 (K1c) no
// per-tile epilogue, bit9 no chunk barrier, bit10 no DMA issue, bit11 no fragment reads (K1c
// timing ablations only: results are garbage under bits 9-11).
// Timing ablations are compiled only into -DCM_ABLATION builds (tools/build_variant.sh); the
// product library ignores CM_DENSE_DEBUG, so no bench line can come from a disabled kernel.
#ifdef CM_ABLATION
int dense_debug_flags() {
  static const int f = [] {
    const char *e = getenv("CM_DENSE_DEBUG");
    return e ? atoi(e) : 0;
  }();
  return f;
}
#else
int dense_debug_flags() { return 0; }
#endif

// Scan kernel for (nq, k): K1c (coarse f16 + certified re-rank) whenever its list length fits,
// K1b (f16x3) for other batched k <= 32, K1 (fp32) otherwise.  CM_DENSE_PATH=f32|f16x3|coarse
// forces a path (A/B probes; an ineligible forced path falls back to the default rule).
int dense_kind(const cm_dense *h, int nq, int k) {
  static const int env_force = [] {
    const char *e = getenv("CM_DENSE_PATH");
    if (!e) return 0;
    const std::string s(e);
    return s == "f32" ? CM_DENSE_F32 : s == "f16x3" ? CM_DENSE_F16X3 : s == "coarse" ? CM_DENSE_COARSE : 0;
  }();
  const int force = h->path ? h->path : env_force;
  // K1c: resident-query scan instances (ld 768 / 384), a sample of >= 1024 rows for the seed
  const bool coarse_ok = k <= kBMaxK && (h->ld == 768 || h->ld == 384) && h->size >= 16384;
  const bool split_ok = k <= kBMaxK && h->ld % 128 == 0;
  if (force == CM_DENSE_F32) return CM_DENSE_F32;
  if (force == CM_DENSE_F16X3 && split_ok) return CM_DENSE_F16X3;
  if (force == CM_DENSE_COARSE && coarse_ok) return CM_DENSE_COARSE;
  if (coarse_ok) return CM_DENSE_COARSE;
  if (split_ok && nq >= 64) return CM_DENSE_F16X3;
  return CM_DENSE_F32;
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

// K1c sample pre-pass geometry: a prefix of 1/64 of the rows (1/16 below 1M rows) in 64-row
// groups, one group range per workgroup, as many workgroups per pass as the main scan.
struct K1cSample {
  int n_wg;
  int64_t rows_per_wg, rows_end;
};
K1cSample k1c_sample(const cm_dense *h, const K1bCfg &c) {
  K1cSample s{};
  const int64_t frac = c.rows_end >= (1 << 20) ? 64 : 16;
  s.rows_end = round_up(std::max<int64_t>(c.rows_end / frac, 1), kRRows);
  const int64_t tiles = s.rows_end / kRRows;
  const int64_t want = std::max(1, num_cus(h->dev) / c.n_pass);
  const int64_t per = ceil_div(tiles, std::min<int64_t>(want, tiles));
  s.rows_per_wg = per * kRRows;
  s.n_wg = (int)ceil_div(tiles, per);
  return s;
}

struct K1bWs {
  _Float16 *qh, *ql;
  float *qnorm;
  uint64_t *cand;     // K1b lists (k per range) -- K1c: fallback pass
  uint64_t *keys;     // K1c candidate buffers [pass][range][query][kCBufCap]
  uint32_t *cnt;      // K1c buffer fill counts [pass][range][query]
  float *mins;        // K1c sample minima [pass][sample range][query]
  float *seed;        // K1c per-query insertion bound from the sample
  int32_t *fb_mask;   // K1c: queries sent to the fallback pass
  int32_t *fb_count;
  size_t total;
};
K1bWs k1b_ws_layout(const cm_dense *h, const K1bCfg &c, int k, bool coarse, void *base) {
  K1bWs w{};
  char *p = reinterpret_cast<char *>(base);
  size_t off = 0;
  const int64_t nq_pad = (int64_t)c.n_pass * kBQPass;
  auto take = [&](int64_t bytes) -> char * {
    char *r = p + off;
    off += round_up(std::max<int64_t>(bytes, 1), 256);
    return r;
  };
  w.qh = reinterpret_cast<_Float16 *>(take(nq_pad * h->ld * 2));
  w.ql = reinterpret_cast<_Float16 *>(take(nq_pad * h->ld * 2));
  w.qnorm = reinterpret_cast<float *>(take(nq_pad * 16));
  w.cand = reinterpret_cast<uint64_t *>(take((int64_t)c.n_pass * c.n_wg * kBQPass * k * 8));
  if (coarse) {
    w.keys = reinterpret_cast<uint64_t *>(take((int64_t)c.n_pass * c.n_wg * kBQPass * kCBufCap * 8));
    w.cnt = reinterpret_cast<uint32_t *>(take((int64_t)c.n_pass * c.n_wg * kBQPass * 4));
    const K1cSample sm = k1c_sample(h, c);
    w.mins = reinterpret_cast<float *>(take((int64_t)c.n_pass * sm.n_wg * kBQPass * 4));
    w.seed = reinterpret_cast<float *>(take(nq_pad * 4));
    w.fb_mask = reinterpret_cast<int32_t *>(take(nq_pad * 4));
    w.fb_count = reinterpret_cast<int32_t *>(take(4));
  }
  w.total = off;
  return w;
}

template <int NPL>
int set_split_lds() {
  static std::once_flag once;
  static hipError_t err = hipSuccess;
  std::call_once(once, [] {
    err = hipFuncSetAttribute(reinterpret_cast<const void *>(&dense_split_kernel<NPL>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, k1b_lds_layout().total);
  });
  CM_HIP(err);
  return CM_OK;
}

// K1b: f16x3 scan of every query + tournament merge.  K1c: coarse scan -> certification and
// exact re-rank -> f16x3 pass restricted to the queries the certificate rejected (its
// workgroups exit at once when there are none) -> merge of those queries only.
int launch_split(cm_dense *h, const float *q_dev, int nq, int k, bool coarse, const uint32_t *allow,
                 float *dist_dev, int64_t *row_dev, void *ws, int64_t ws_bytes, hipStream_t st) {
  int rc;
  if ((rc = set_split_lds<2>())) return rc;
  if (coarse) {
    static std::once_flag once;
    static hipError_t err = hipSuccess;
    std::call_once(once, [] {
      const std::pair<const void *, int> fs[] = {
          {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<12, 3, false, kK1cWaves>), K1rLds<3>::total},
          {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<12, 3, true, kK1cWaves>), K1rLds<3>::total},
          {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<6, 0, false, kK1cWaves>), K1rLds<0>::total},
          {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<6, 0, true, kK1cWaves>), K1rLds<0>::total},
          {reinterpret_cast<const void *>(&dense_rerank_kernel), kGatherCap * 12}};
      for (const auto &f : fs) {
        const hipError_t e = hipFuncSetAttribute(f.first, hipFuncAttributeMaxDynamicSharedMemorySize, f.second);
        if (e != hipSuccess) err = e;
      }
    });
    CM_HIP(err);
  }
  const K1bCfg c = k1b_config(h, nq);
  const K1bWs w = k1b_ws_layout(h, c, k, coarse, ws);
  if ((int64_t)w.total > ws_bytes || !ws) CM_FAIL(CM_EINVAL, "dense workspace too small");
  const size_t lds = k1b_lds_layout().total;
  const int64_t n_words = ceil_div(h->size, 32);
  const dim3 grid(c.n_wg * c.n_pass);
  hipLaunchKernelGGL(dense_prep_planes, dim3(c.n_pass * kBQPass), dim3(256), 0, st, q_dev, nq, h->dim, h->ld, w.qh,
                     w.ql, w.qnorm);
  CM_HIP(hipGetLastError());
  const int32_t *mask = nullptr;
  if (coarse) {
    CM_HIP(hipMemsetAsync(w.fb_count, 0, 4, st));
    const K1cSample sm = k1c_sample(h, c);
    const bool d768 = h->ld == 768;
    auto scan = [&](bool minonly) {
      if (d768) return minonly ? &dense_coarse_scan_kernel<12, 3, true, kK1cWaves> : &dense_coarse_scan_kernel<12, 3, false, kK1cWaves>;
      return minonly ? &dense_coarse_scan_kernel<6, 0, true, kK1cWaves> : &dense_coarse_scan_kernel<6, 0, false, kK1cWaves>;
    };
    const size_t slds = d768 ? K1rLds<3>::total : K1rLds<0>::total;
    // 1. sample pre-pass (per-group minima) -> seed
    hipLaunchKernelGGL(scan(true), dim3(sm.n_wg * c.n_pass), dim3(64 * kK1cWaves), slds, st, h->Xh, h->live, allow, n_words,
                       w.qh, nq, (const float *)nullptr, sm.rows_per_wg, sm.rows_end, sm.n_wg, (uint64_t *)nullptr,
                       (uint32_t *)nullptr, w.mins, 0);
    CM_HIP(hipGetLastError());
    hipLaunchKernelGGL(dense_seed_kernel, dim3(nq), dim3(256), 0, st, w.mins, sm.n_wg, k, nq, w.qnorm, h->rnorm,
                       h->dim, w.seed);
    CM_HIP(hipGetLastError());
    // 2. coarse scan: rows under the seed -> candidate buffers
    h->timer.begin(st);
    hipLaunchKernelGGL(scan(false), grid, dim3(64 * kK1cWaves), slds, st, h->Xh, h->live, allow, n_words, w.qh, nq,
                       (const float *)w.seed, c.rows_per_wg, c.rows_end, c.n_wg, w.keys, w.cnt, (float *)nullptr,
                       dense_debug_flags());
    h->timer.end(st);
    CM_HIP(hipGetLastError());
    // 3. certificate + exact re-rank (failures -> fb_mask)
    hipLaunchKernelGGL(dense_rerank_kernel, dim3(nq), dim3(256), kGatherCap * 12, st, w.keys, w.cnt, c.n_wg, k, nq,
                       h->C, h->ld, h->dim, q_dev, w.qnorm, h->rnorm, dist_dev, row_dev, w.fb_mask, w.fb_count);
    CM_HIP(hipGetLastError());
    mask = w.fb_mask;
  }
  if (!coarse) h->timer.begin(st);
  hipLaunchKernelGGL(dense_split_kernel<2>, grid, dim3(512), lds, st, h->Xh, h->Xl, h->ld, h->live, allow, n_words,
                     w.qh, w.ql, nq, mask, k, c.rows_per_wg, c.rows_end, c.n_wg, w.cand, dense_debug_flags());
  if (!coarse) h->timer.end(st);
  CM_HIP(hipGetLastError());
  hipLaunchKernelGGL(dense_merge_kernel, dim3(nq), dim3(256), 0, st, w.cand, c.n_wg, kBQPass, k, nq, mask, dist_dev,
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
  if (hipMalloc(&h->rnorm, 8) != hipSuccess || hipMemset(h->rnorm, 0, 8) != hipSuccess) {
    cm_dense_destroy(h);
    CM_FAIL(CM_ENOMEM, "dense: out of device memory");
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
  if (h->rnorm) (void)hipFree(h->rnorm);
  h->timer.release();
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
                       h->rows_buf.as<int64_t>(), (int64_t)0, m, h->dim, h->ld, h->C, h->invc, h->live, h->Xh, h->Xl,
                       reinterpret_cast<uint32_t *>(h->rnorm));
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
                       h->Xl, reinterpret_cast<uint32_t *>(h->rnorm));
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
  CM_HIP(hipMemsetAsync(h->rnorm, 0, 8, h->stream));
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
  const int kind = dense_kind(h, nq, k);
  if (kind != CM_DENSE_F32) return (int64_t)k1b_ws_layout(h, k1b_config(h, nq), k, kind == CM_DENSE_COARSE, nullptr).total;
  DenseCfg c = dense_config(h, nq, k);
  return (int64_t)dense_ws_layout(h, c, nq, k, nullptr).total;
}

int cm_dense_set_path(cm_dense *h, int32_t kind) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (kind < 0 || kind > CM_DENSE_COARSE) CM_FAIL(CM_EINVAL, "unknown dense path");
  h->path = kind;
  return CM_OK;
}

int32_t cm_dense_workspace_fallbacks(cm_dense *h, int32_t nq, int32_t k, const void *workspace_dev) {
  if (!h || !workspace_dev || nq <= 0 || k <= 0 || k > kMaxTopK) return -1;
  if (dense_kind(h, nq, k) != CM_DENSE_COARSE) return 0;
  DeviceGuard dg(h->dev);
  const K1bWs w = k1b_ws_layout(h, k1b_config(h, nq), k, true, const_cast<void *>(workspace_dev));
  int32_t c = -1;
  if (hipMemcpy(&c, w.fb_count, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return c;
}

int32_t cm_dense_last_fallbacks(cm_dense *h) { return h ? h->last_fallbacks : -1; }

int cm_dense_timing(cm_dense *h, int32_t enable) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  DeviceGuard dg(h->dev);
  h->timer.on = enable != 0;
  h->timer.used = 0;
  return CM_OK;
}

int32_t cm_dense_timing_drain(cm_dense *h, float *ms_out, int32_t cap) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  DeviceGuard dg(h->dev);
  const int n = h->timer.drain(ms_out, cap);
  if (n < 0) CM_FAIL(CM_EDEVICE, "event query failed");
  return n;
}

int32_t cm_dense_search_kind(cm_dense *h, int32_t nq, int32_t k) {
  if (!h || nq <= 0 || k <= 0 || k > kMaxTopK) return -1;
  return dense_kind(h, nq, k);
}

int cm_dense_search_dev(cm_dense *h, const float *q_dev, int32_t nq, int32_t k, const uint32_t *allow_dev,
                        float *dist_dev, int64_t *row_dev, void *workspace_dev, int64_t workspace_bytes,
                        void *stream) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (k <= 0 || k > kMaxTopK) CM_FAIL(CM_EINVAL, "k must be in [1, " + std::to_string(kMaxTopK) + "]");
  DeviceGuard dg(h->dev);
  hipStream_t st = (hipStream_t)stream;  // NULL = the null stream (torch default)
  const int kind = dense_kind(h, nq, k);
  if (kind != CM_DENSE_F32)
    return launch_split(h, q_dev, nq, k, kind == CM_DENSE_COARSE, allow_dev, dist_dev, row_dev, workspace_dev,
                        workspace_bytes, st);
  DenseCfg c = dense_config(h, nq, k);
  if (c.lds > 163840) CM_FAIL(CM_EUNSUPPORTED, "dim/k too large for the LDS-resident query tile");
  DenseWs w = dense_ws_layout(h, c, nq, k, workspace_dev);
  if ((int64_t)w.total > workspace_bytes || !workspace_dev) CM_FAIL(CM_EINVAL, "dense workspace too small");
  const int nq_pad = c.n_qgroups * c.QB;
  hipLaunchKernelGGL(dense_prep_queries, dim3(nq_pad), dim3(256), 0, st, q_dev, nq, h->dim, h->ld, w.qp, w.invq);
  CM_HIP(hipGetLastError());
  h->timer.begin(st);
  int rc = launch_dense(c, h, allow_dev, w.qp, w.invq, nq, k, w.cand, st);
  h->timer.end(st);
  if (rc) return rc;
  hipLaunchKernelGGL(dense_merge_kernel, dim3(nq), dim3(256), 0, st, w.cand, c.n_cblocks, c.QB, k, nq,
                     (const int32_t *)nullptr, dist_dev,
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
    CM_HIP(hipMemcpyAsync(h->allow_buf.ptr, allow_bits, (size_t)nw * 4, hipMemcpyDefault, h->stream));  // host or device
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
  h->last_fallbacks = 0;
  if (dense_kind(h, nq, k) == CM_DENSE_COARSE) {
    const K1bWs w = k1b_ws_layout(h, k1b_config(h, nq), k, true, h->ws.ptr);
    CM_HIP(hipMemcpyAsync(&h->last_fallbacks, w.fb_count, 4, hipMemcpyDeviceToHost, h->stream));
  }
  CM_HIP(hipStreamSynchronize(h->stream));
  return CM_OK;
}

}  // extern "C"
