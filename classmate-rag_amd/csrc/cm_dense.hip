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

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
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
                      int64_t rows_per_block, int64_t rows_end, int n_cblocks, const int32_t *__restrict__ qmask,
                      const int32_t *__restrict__ gate, uint64_t *__restrict__ cand) {
  constexpr int QT = QB / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  // gate (the certificate fallback): the number of failed queries -- 0 in the common case, when every
  // workgroup leaves at its first instruction
  if (gate && *gate == 0) return;
  const DenseLds L = dense_lds_layout(QB, KMAX, ld);
  // qmask (K1c/K1s fallback): only queries with qmask[q] != 0 are searched; a workgroup whose
  // query group has none exits before touching the corpus (block-uniform: no barrier skipped)
  if (qmask) {  // (a dynamic-LDS word: __syncthreads_or would add static LDS past the 160 KiB budget)
    uint32_t *flag = reinterpret_cast<uint32_t *>(lds + L.cnt);
    if (threadIdx.x == 0) flag[0] = 0u;
    __syncthreads();
    const int qq = (int)(blockIdx.x / n_cblocks) * QB + (int)threadIdx.x;
    if (threadIdx.x < QB && qq < nq && qmask[qq]) flag[0] = 1u;
    __syncthreads();
    const uint32_t any = flag[0];
    __syncthreads();  // every thread has read the word before the init below reuses it
    if (!any) return;
  }
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
// K1c / K1s: coarse f16 scans + a certified exact re-rank.
//   xn = c * invc (hnswlib normalize_vector), Xh = f16(xn): the only derived plane kept in HBM
//   (2 B per element, half of the fp32 rows).  A scan computes xh.qh on the MFMA f16 pipe and
//   appends every live + allowed row whose coarse distance is under the query's seed to a
//   (range, query) candidate buffer; dense_rerank_kernel certifies the buffers with a rigorous
//   error bound and re-ranks the band in fp64 from the fp32 rows.  Queries whose certificate
//   fails are re-run exactly by K1 (fp32 rows, qmask).
//   K1c dense_coarse_scan_kernel: a whole pass of 256 queries resident per CU (batched search);
//   K1s dense_stream_scan_kernel: <= 32 queries, every wave an independent HBM stream of its own
//     row range (small batches and single queries; no LDS, no barriers).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// Plane layout (Xh): fragment-major.  Rows in 64-row tiles, columns in 64-wide chunks; each
// (tile, chunk) is 8 KB = 8 blocks of 1 KB; block b = 2 rt + sb holds rows 16 rt .. 16 rt + 15 and
// columns 32 sb .. 32 sb + 31 of the chunk in the MFMA A-operand lane order: lane l = 16 g + j owns
// row 16 rt + j, columns 32 sb + 8 g .. + 7 (16 B at byte 16 l of the block).  One wave-instruction
// -- an LDS-DMA piece (K1c) or a 16-B-per-lane load (K1s) -- moves exactly one block, 1 KB
// contiguous, and the LDS image it leaves is read back conflict-free (lane l reads bytes 16 l).
__host__ __device__ inline int64_t plane_off(int64_t row, int k, int ld) {
  const int64_t tile = row >> 6;
  const int rr = (int)(row & 63), rt = rr >> 4, j = rr & 15;
  const int c = k >> 6, cc = k & 63, sb = cc >> 5, g = (cc >> 3) & 3, e = cc & 7;
  return (((tile * (ld >> 6) + c) * 8 + rt * 2 + sb) << 9) + ((j * 4 + g) << 3) + e;
}
// The plane keeps each (row, k-half) of a block as one 64-B run (piece g of row j at (4 j + g) x 16 B),
// so a single row reads as 24 whole sectors (K1q's f16 re-rank stage); the MFMA operand order of
// lane (g, j) is restored by the loads: lane l fetches piece plane_lane(l) of its block.
__device__ inline int plane_lane(int lane) { return ((lane & 15) << 2) | (lane >> 4); }
constexpr int kBQPass = 256;                // K1c: queries per pass (4 waves x 64)
constexpr int kSQ = 32;                     // K1s: queries per launch (<= 2 q-tiles of 16)
constexpr int kBMaxK = 32;                  // coarse paths: k <= 32
constexpr int kRerankCap = 1024;            // certified band size per query handled by the re-rank kernel

// Normalise queries into Qh [nq_pad][ld] (zero rows beyond nq) and record per query
// {||q||, ||qh||, ||ql||} (fp32, ql = qn - qh: K1c/K1s's error bound).
__global__ void __launch_bounds__(256) dense_prep_planes(const float *__restrict__ q, int nq, int dim, int ld,
                                                         _Float16 *__restrict__ Qh, float *__restrict__ qnorm) {
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
    const float lo = v - (float)hi;  // exact residual (the error bound's ||ql||)
    Qh[(int64_t)qi * ld + i] = hi;
    sh += (float)hi * (float)hi;
    sl += lo * lo;
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

// Waves per K1c workgroup.  4 (one per SIMD) is the measured best: 8 (two per SIMD, 32 queries
// each, 256 VGPRs with 16 spilled at tile boundaries) ran 5.63 vs 4.96 ms on the 10M x 768 scan --
// the second wave did not hide barrier/epilogue time.  Kept selectable for experiments.
#ifndef K1C_WAVES
#define K1C_WAVES 4
#endif
constexpr int kK1cWaves = K1C_WAVES;

// K1c/K1s per-query error bound E (see dense_rerank_kernel).
__device__ inline float coarse_err(const float *qnorm, int qi, const float *row_norms, int dim) {
  const float qh = qnorm[4 * qi + 1], qlo = qnorm[4 * qi + 2];
  const float mxh = row_norms[0], mxl = row_norms[1];
  return (qlo * mxh + mxl * qh + mxl * qlo + (float)dim * 5.9604645e-8f * mxh * qh + 2e-6f) * 1.001f;
}

#ifndef K1C_RING
#define K1C_RING 8
#endif
constexpr int kRRing = K1C_RING;  // LDS ring slots (8 KB each): kRRing - 1 chunks in flight per CU
// LDS-resident query chunks of the whole-pass K1c at ld 768 (the rest stay in registers); the ring
// and these share the 160 KiB: (kRRing + 4 kK1cNql) x 8 KiB
#ifndef K1C_NQL
#define K1C_NQL 3
#endif
// cache-policy bits of K1c's corpus DMA (2 = nt: streamed once)
#ifndef K1C_AUX
#define K1C_AUX 2
#endif
// 1: K1s streams the plane with non-temporal loads (read once): 10M x 768, B = 16 2.48 -> 2.22 ms
// (6.9 TB/s, 0.87 of the 8 TB/s peak)
#ifndef K1S_NT
#define K1S_NT 1
#endif
// query chunks whose resident fragments are pinned to AGPRs (see the K1c prologue)
#ifndef K1C_QAGPR
#define K1C_QAGPR 8
#endif
// 1: the interleaved K1c chunk schedule (one non-MFMA step per MFMA); 0: the two-block schedule
#ifndef K1C_SCHED
#define K1C_SCHED 1
#endif
constexpr int kK1cNql = K1C_NQL;
constexpr int kRRows = 64;      // rows per compute tile / chunk
constexpr int kCBufCap = 64;    // candidate slots per (range, query)

// Per-tile candidate epilogue shared by K1c and K1s.  acc[rt][qt][r] is the coarse product of
// row rt*16 + 4g + r of the tile with query qt*16 + j (lane (g, j)); live16 the lane's 16 live &
// allow bits (bit 4 rt + r).  MINONLY: running minimum coarse distance per query.  Otherwise every
// row with coarse distance <= sd[qt] is appended to its query's buffer dst0 + qt * 16 * kCBufCap:
// a per-lane 16-bit hit mask, an exclusive prefix of the hit counts over the 4 lanes (g = 0..3)
// that share query j, then each lane writes its own hits (usually none); the running count lives
// in lane j's register (no LDS atomics: those would wait behind the ring's DMAs).  A q-tile with
// no row under any of its queries' seeds costs one max-reduction and a ballot.
template <int QT, bool MINONLY>
__device__ __attribute__((always_inline)) inline void coarse_epilogue(const f32x4 (&acc)[4][QT], uint32_t live16,
                                                                      int64_t row0, const float (&sd)[QT],
                                                                      float (&best)[QT], uint32_t (&qcnt)[QT],
                                                                      uint64_t *dst0) {
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    if (MINONLY) {
      float m = __builtin_inff();
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if ((live16 >> (rt * 4 + r)) & 1u) m = fminf(m, 1.0f - acc[rt][qt][r]);
      best[qt] = fminf(best[qt], m);
    } else {
      float mx = -__builtin_inff();
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, acc[rt][qt][r]);
      if (__ballot(1.0f - mx <= sd[qt]) == 0) continue;  // no row of the tile under any seed
#ifdef K1C_NOHIT
      if (sd[qt] < 1e30f) continue;  // timing ablation only: never append
#endif
      // Append every live row under the seed, position by position (static register indices):
      // one ballot per position tells which of the 64 lanes hit; the slot of a hit is the query's
      // running count plus the hits of the same query's lower lanes (g' < g) at this position --
      // popcounts of the ballot under per-lane masks, so no cross-lane shuffles (LDS round trips)
      // are needed.  All 4 lanes of query j keep identical copies of its count.
      const uint64_t m_all = 0x0001000100010001ull << j;           // lanes (g', j), g' = 0..3
      const uint64_t m_low = m_all & ((1ull << (16 * g)) - 1ull);  // lanes (g' < g, j)
      uint32_t run = qcnt[qt];
      uint64_t *d = dst0 + (int64_t)qt * 16 * kCBufCap;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const bool hit = (1.0f - acc[i >> 2][qt][i & 3] <= sd[qt]) && ((live16 >> i) & 1u);
        const uint64_t B = __ballot(hit);
        if (B == 0) continue;  // wave-uniform
        const uint32_t slot = run + (uint32_t)__popcll(B & m_low);
        if (hit && slot < (uint32_t)kCBufCap)
          d[slot] = ((uint64_t)f32_order(1.0f - acc[i >> 2][qt][i & 3]) << 32) |
                    (uint64_t)(uint32_t)(row0 + (i >> 2) * 16 + 4 * g + (i & 3));
        run += (uint32_t)__popcll(B & m_all);
      }
      qcnt[qt] = run;
    }
  }
}
// The lane's 16 bits of a tile's 64-bit live & allow mask: bit 4 rt + r = tile row rt*16 + 4g + r.
__device__ inline uint32_t lane_live16(uint64_t tmask, int g) {
  uint32_t v = 0;
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) v |= (uint32_t)((tmask >> (rt * 16 + 4 * g)) & 0xfu) << (rt * 4);
  return v;
}

// ---------------------------------------------------------------------------
// K1c scan (coarse f16, Xh plane only), resident-query form for ld = 64 KC.
// 64 W threads (W = kK1cWaves: 4 -> one wave per SIMD, 8 -> two); wave w owns queries 256w/W.. of
// the 256-query pass and keeps their Qh fragments resident -- chunks 0..KC-NQL-1 in registers (32
// VGPRs each), the last NQL chunks in LDS -- so the corpus is the only memory stream: 64-row x
// 64-f16 chunks (8 KB = 8 fragment blocks; one glds wave-instruction = one 1 KB block) LDS-DMA'd
// into a kRRing-slot ring, retired by a counted vmcnt and published by a raw s_barrier: no
// vmcnt(0) and no query reloads in the loop.  The ring image is the plane's fragment-major block
// order, read back lane-linearly (conflict-free).  Compute tiles are 64 rows.
//   MINONLY (sample pre-pass): per query, the minimum coarse distance over the workgroup's
//     live+allowed rows -> out_min[pass][wg][q].
//   main pass: every live+allowed row with coarse distance <= seed[q] is appended to the
//     (range, query) candidate buffer out_keys[pass][wg][q][kCBufCap];
//     out_cnt[pass][wg][q] = appended count (> kCBufCap: the buffer overflowed).
template <int NQL, int RING = kRRing>
struct K1rLds {
  static constexpr int ring = 0;
  static constexpr int qf = ring + RING * 8192;            // [NQL][W waves][32/W frags][64 lanes] x 16 B
  static constexpr int total = qf + NQL * 4 * 8 * 1024;
};

//   QPASS = 128 (the paired form, K1c2): a workgroup holds half of the pass's queries, all in
//     registers (no LDS-resident query chunks), so the whole 160 KiB LDS is the DMA ring (20 slots,
//     >= 18 chunks = 144 KiB in flight per CU, deep enough to cover the loaded HBM latency); the
//     two workgroups of a (pass, range) are blocks b and b + 8 -- one XCD under round-robin
//     placement -- so the second reader of every chunk finds it in (or on its way into) that XCD's L2
//     and the corpus still crosses HBM about once.  Placement is a speed assumption only.
template <int KC, int NQL, bool MINONLY, int W, int RING = kRRing, int QPASS = kBQPass>
__global__ void __launch_bounds__(64 * W, 1)
    dense_coarse_scan_kernel(const _Float16 *__restrict__ Xh, const uint32_t *__restrict__ live,
                             const uint32_t *__restrict__ allow, int64_t n_words, const _Float16 *__restrict__ Qh,
                             int nq, const float *__restrict__ seed, int64_t rows_per_wg, int64_t rows_end, int n_wg,
                             uint64_t *__restrict__ out_keys, uint32_t *__restrict__ out_cnt,
                             float *__restrict__ out_min, int dbg) {
  constexpr int ld = 64 * KC;
  constexpr int KR = KC - NQL;  // register-resident query chunks
  using LL = K1rLds<NQL, RING>;
  constexpr int QT = QPASS / (16 * W);  // 16-query tiles per wave
  constexpr int NF = 2 * QT;            // query fragments per wave and chunk
  constexpr int PCS = 8 / W;            // 1 KB DMA pieces per wave and chunk
  constexpr int H = kBQPass / QPASS;    // workgroups per (pass, range)
#if defined(K1C_DBG)
  dbg = K1C_DBG;  // compile-time timing ablation (tools/build_dense_variant.sh), folds like the product
#elif !defined(CM_ABLATION)
  dbg = 0;  // product build: the ablation branches fold away (exact lgkmcnt / vmcnt counting)
#endif
  static_assert(W == 4 || W == 8, "K1c: 4 or 8 waves");
  static_assert(LL::total <= 160 * 1024, "K1c: LDS ring + query chunks + mask exceed 160 KiB");
  static_assert(H == 1 || H == 2, "K1c: full or half passes");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int j = lane & 15;
  int lr = blockIdx.x, half = 0;  // linear (pass, range) index and query half
  if (H == 2) {                   // blocks b, b + 8 -> same (pass, range), halves 0 / 1
    const int grp = blockIdx.x >> 3;
    half = grp & 1;
    lr = (grp >> 1) * 8 + (blockIdx.x & 7);
  }
  const int wg = lr % n_wg;
  const int qp = lr / n_wg;
  if (H == 2 && qp * kBQPass >= nq) return;  // grid padding of the paired mapping (whole workgroup)
  const int64_t r_begin = (int64_t)wg * rows_per_wg;
  const int64_t r_end = min(r_begin + rows_per_wg, rows_end);
  const int ntiles = r_begin < r_end ? (int)((r_end - r_begin) / kRRows) : 0;
  const int total = ntiles * KC;
  const int qc0 = half * QPASS + wave * 16 * QT;  // wave's first query within the pass
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
  // pin the first K1C_QAGPR chunks' fragments to AGPRs (the 256 of them hold 8 chunks): the
  // MFMA reads its B operand from an AGPR directly, where a VGPR value the allocator parked
  // in an AGPR is copied back before every use (16 v_accvgpr_read per chunk).  With the
  // accumulators in VGPRs (-mllvm -amdgpu-mfma-vgpr-form, Makefile) nothing is copied.  Pinned
  // after all loads are issued (a pin per load serialised them behind vmcnt(0) waits).
#pragma unroll
  for (int c = 0; c < KR; ++c)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb)
        if (c < K1C_QAGPR) asm volatile("" : "+a"(qres[c][qt][sb]));
#pragma unroll
  for (int c = 0; c < NQL; ++c)
#pragma unroll
    for (int f = 0; f < NF; ++f)
      *reinterpret_cast<f16x8 *>(lds + LL::qf + ((c * W + wave) * NF + f) * 1024 + lane * 16) =
          *qsrc(KR + c, f >> 1, f & 1);
  // per-lane seeds of the lane's QT queries (qt*16 + j)
  float sd[QT], best[QT];
  uint32_t qcnt[QT];  // candidates appended for query qt*16 + j (same value in its 4 lanes)
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    best[qt] = __builtin_inff();
    qcnt[qt] = 0u;
    const int qq = qg0 + qt * 16 + j;
    sd[qt] = MINONLY ? 0.f : (qq < nq ? seed[qq] : -__builtin_inff());  // padded queries accept nothing
  }
  // vmcnt(0) through the builtin (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15), not inline asm: the
  // compiler's wait tracker must see the prologue's query loads retired, or it re-waits for them
  // with a vmcnt(0) inside the chunk loop -- draining the DMA ring once per tile
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();  // LDS query fragments ready; no DMA in flight yet

  // glds of chunk gc: wave-instruction i moves fragment block o = W i + wave (1 KB, lane-linear)
  const __attribute__((address_space(1))) unsigned char *Xb =
      (const __attribute__((address_space(1))) unsigned char *)Xh;
  // the workgroup's chunks are contiguous in the plane: chunk gc = block run (cb + gc) * 8
  const int64_t cb = (r_begin >> 6) * KC;
  auto issue_piece = [&](int gc, int i) __attribute__((always_inline)) {
    int gl = min(gc, total - 1);  // clamped: one control path past the end
    if (dbg & 8192) gl &= 15;     // bit 13: ablation only (L2-resident source: LDS traffic without HBM)
    const int o = W * i + wave;
    __builtin_amdgcn_global_load_lds(Xb + (((cb + gl) * 8 + o) << 10) + plane_lane(lane) * 16,
                                     (__attribute__((address_space(3))) void *)(lds + LL::ring + (gc % RING) * 8192 +
                                                                                o * 1024),
                                     16, 0, K1C_AUX);
  };
  auto issue = [&](int gc) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCS; ++i) issue_piece(gc, i);
  };
  f32x4 acc[4][QT];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) acc[rt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // The live and allow words of a window of 32 tiles (64 words: one per lane) are loaded into
  // two VGPRs when the window starts and read out per tile with a uniform readlane.  The compiler
  // cannot count a VGPR load among the LDS DMAs (it would wait vmcnt(0) at every use), so the
  // window load waits vmcnt(0) itself, where the compiler sees it: the DMA ring drains once per 32
  // tiles instead of once per tile.
  const uint32_t *allw = allow ? allow : live;
  uint32_t lwin = 0u, awin = 0u;
  auto load_window = [&](int t) __attribute__((always_inline)) {
    const int64_t wi = ((r_begin + (int64_t)t * kRRows) >> 5) + lane;
    const int64_t wc = wi < n_words ? wi : n_words - 1;  // n_words >= 1 whenever a tile is scanned
    lwin = live[wc];
    awin = allw[wc];
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the compiler's wait tracking
  };
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int64_t row0 = r_begin + (int64_t)t * kRRows;
    const int64_t w0 = row0 >> 5;
    // lane (g, j) holds rows rt*16 + 4g + r: bit (16 rt + 4 g + r) of the 64-bit tile mask
#ifdef K1C_NOMASK
    const uint32_t b0 = 0xffffffffu, b1 = 0xffffffffu;  // timing ablation only: every row live
#else
    const int wl = 2 * (t & 31);
    const uint32_t m0 = (uint32_t)__builtin_amdgcn_readlane((int)(lwin & awin), wl);
    const uint32_t m1 = (uint32_t)__builtin_amdgcn_readlane((int)(lwin & awin), wl + 1);
    const uint32_t b0 = w0 < n_words ? m0 : 0u;
    const uint32_t b1 = w0 + 1 < n_words ? m1 : 0u;
#endif
    coarse_epilogue<QT, MINONLY>(acc, lane_live16(((uint64_t)b1 << 32) | b0, g), row0, sd, best, qcnt,
                                 out_keys + (((int64_t)qp * n_wg + wg) * kBQPass + qc0 + j) * kCBufCap);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) acc[rt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  if (total > 0) {
    // Software-pipelined chunk loop.  Chunk gc's 32 MFMAs run in two halves (row tiles 0-1,
    // 2-3); between them the wave waits for chunk gc+1's DMA pieces, the barrier publishes
    // chunk gc+1 and retires every read of chunk gc's slot (each wave drains its LDS reads
    // first), chunk gc + RING is issued into that slot and the row fragments 0-1 of chunk gc+1
    // are read into the registers half 1 has just consumed; fragments 2-3 follow half 2.  Every
    // barrier, DMA issue and LDS read thus sits behind >= 16 MFMAs instead of in front of them.
    auto frag = [&](int gc, int rt, int sb) -> f16x8 {
      const unsigned char *slot = lds + LL::ring + (gc % RING) * 8192;
      return *reinterpret_cast<const f16x8 *>(slot + (rt * 2 + sb) * 1024 + lane * 16);
    };
#pragma unroll
    for (int p = 0; p < RING - 1; ++p) issue(p);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PCS * (RING - 2)) : "memory");
    __builtin_amdgcn_s_barrier();
    issue(RING - 1);
    f16x8 xf[4][2];
#pragma unroll
    for (int rt = 0; rt < (K1C_SCHED ? 2 : 4); ++rt) {  // interleaved schedule: chunk 0 reads its own 2-3
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
      if ((t & 31) == 0) load_window(t);
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const int gc = t * KC + c;
#if defined(K1C_QV) && K1C_QV == 1  // timing ablations only: one resident chunk's fragments for all
        auto qv = [&](int qt, int sb) -> f16x8 { return qres[0][qt][sb]; };
#elif defined(K1C_QV) && K1C_QV == 2  // ... register fragments only (no LDS-resident chunks)
        auto qv = [&](int qt, int sb) -> f16x8 { return qres[KR > 0 ? c % KR : 0][qt][sb]; };
#else
        auto qv = [&](int qt, int sb) -> f16x8 { return c < KR ? qres[c < KR ? c : 0][qt][sb] : ql[qt][sb]; };
#endif
        const int cn = (c + 1) % KC;  // next chunk's query fragments come from LDS when cn >= KR
#if K1C_SCHED
        // Interleaved chunk schedule.  With one wave per SIMD nothing hides a non-MFMA instruction
        // but the MFMA issued just before it, so the chunk's LDS reads, counted wait, barrier and
        // DMA pieces are threaded one per MFMA through its 2 x MH MFMAs (sched_barrier-fenced):
        //   half 1 (row tiles 0-1): read row fragments 2-3 of chunk gc (slot certified by the
        //     previous chunk's barrier), then wait for chunk gc+1 (own pieces; PCS (RING - 2) younger
        //     stay in flight) and for the own reads of slot gc, barrier (chunk gc+1 visible, every
        //     read of slot gc retired), DMA chunk gc + RING into slot gc;
        //   half 2 (row tiles 2-3): read row fragments 0-1 of chunk gc+1; the next chunk's LDS
        //     query fragments follow the last MFMA of their q-tile group.
        // MFMA order within a half: q-tile group, k-half, row tile, q-tile (an accumulator recurs
        // every 2 QA MFMAs), so a q-tile group's fragments are free half-way through the half.
        {
          constexpr int QA = QT / 2, MH = 8 * QA;
          auto mf = [&](int h, int m) __attribute__((always_inline)) {
            const int qa = m % QA, rt = 2 * h + (m / QA) % 2, sb = (m / (2 * QA)) % 2, qt = (m / (4 * QA)) * QA + qa;
            if (dbg & 4096) return;  // bit 12: ablation only (no MFMA: the memory side alone)
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[rt][sb], qv(qt, sb), acc[rt][qt], 0, 0, 0);
          };
          auto read_ql = [&](int grp) __attribute__((always_inline)) {
#pragma unroll
            for (int qa = 0; qa < QA; ++qa)
#pragma unroll
              for (int sb = 0; sb < 2; ++sb)
                ql[grp * QA + qa][sb] = *reinterpret_cast<const f16x8 *>(
                    lds + LL::qf + (((cn - KR) * W + wave) * NF + (grp * QA + qa) * 2 + sb) * 1024 + lane * 16);
          };
#pragma unroll
          for (int m = 0; m < MH; ++m) {
            mf(0, m);
            __builtin_amdgcn_sched_barrier(0);
            if (m < 4 && !(dbg & 2048)) xf[2 + m / 2][m % 2] = frag(gc, 2 + m / 2, m % 2);  // bit 11: ablation
            const int w0 = MH - PCS - 2;
            if (m == w0) {
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PCS * (RING - 2)) : "memory");
              if (!(dbg & 512)) __builtin_amdgcn_s_barrier();  // bit 9: ablation only (races)
            }
            if (m > w0 && m <= w0 + PCS && !(dbg & 1024))  // bit 10: ablation only (stale data)
              issue_piece(gc + RING, m - w0 - 1);
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int m = 0; m < MH; ++m) {
            mf(1, m);
            __builtin_amdgcn_sched_barrier(0);
            if (m < 4 && !(dbg & 2048)) xf[m / 2][m % 2] = frag(gc + 1, m / 2, m % 2);
            if (cn >= KR && m == MH / 2 - 1) read_ql(0);
            if (cn >= KR && m == MH - 1) read_ql(1);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
#else
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
        // chunk gc+1 landed (this wave's pieces: the PCS (RING - 2) younger DMAs may stay in
        // flight); own LDS reads of slot gc done; the barrier makes both true for every wave
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PCS * (RING - 2)) : "memory");
        if (!(dbg & 512)) __builtin_amdgcn_s_barrier();  // bit 9: ablation only (races)
        if (!(dbg & 1024)) issue(gc + RING);             // bit 10: ablation only (stale data)
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
        if (cn >= KR) {
#pragma unroll
          for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int sb = 0; sb < 2; ++sb)
              ql[qt][sb] = *reinterpret_cast<const f16x8 *>(
                  lds + LL::qf + (((cn - KR) * W + wave) * NF + qt * 2 + sb) * 1024 + lane * 16);
        }
        __builtin_amdgcn_sched_barrier(0);
#endif
      }
#ifdef K1C_EPI0  // timing ablation only: keep the MFMAs alive with a trivial epilogue
      {
        float z = 0.f;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) z += acc[rt][qt][0];
        best[0] = fminf(best[0], z);
        qcnt[0] += z == 12345.f ? 1u : 0u;  // observable: out_cnt / out_min
      }
#else
      if (!(dbg & 128)) epilogue(t);
#endif
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

// ---------------------------------------------------------------------------
// K1s: coarse f16 scan for nq <= 16 QT queries (single queries, small batches: SURVEY §8d C2'
// at B = 16), HBM streaming.  Every wave is an independent "virtual group" vg owning a contiguous
// run of 64-row tiles; its queries' Qh fragments stay in registers for the whole launch, the
// plane's fragment blocks go straight to registers (each load instruction = one contiguous 1 KB
// block, 16 B per lane) through a ring of R chunks (R - 1 in flight: 24 KB per wave, 96 KB per
// CU) and feed v_mfma_f32_16x16x32_f16 without any LDS round trip, barrier or cross-wave
// hand-off.  Output layout = K1c's with n_wg = n_vg groups and a pass of qs queries, so the seed
// and re-rank kernels are shared.
template <int KC, int QT, bool MINONLY>
__global__ void __launch_bounds__(256, 1)
    dense_stream_scan_kernel(const _Float16 *__restrict__ Xh, const uint32_t *__restrict__ live,
                             const uint32_t *__restrict__ allow, int64_t n_words, const _Float16 *__restrict__ Qh,
                             int nq, const float *__restrict__ seed, int64_t rows_per_vg, int64_t rows_end, int n_vg,
                             int qs, uint64_t *__restrict__ out_keys, uint32_t *__restrict__ out_cnt,
                             float *__restrict__ out_min) {
  constexpr int ld = 64 * KC;
  constexpr int R = (KC % 4 == 0) ? 4 : 3;  // register ring (chunks), KC % R == 0 keeps indices static
  static_assert(KC % R == 0, "K1s: ring must divide the chunks per tile");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int vg = blockIdx.x * 4 + wave;
  if (vg >= n_vg) return;  // wave-uniform; the kernel has no barriers
  const int64_t r_begin = (int64_t)vg * rows_per_vg;
  const int64_t r_end = min(r_begin + rows_per_vg, rows_end);
  const int ntiles = r_begin < r_end ? (int)((r_end - r_begin) / kRRows) : 0;
  const int total = ntiles * KC;

  f16x8 qf[KC][2][QT];
#pragma unroll
  for (int c = 0; c < KC; ++c)
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
        qf[c][sb][qt] = *reinterpret_cast<const f16x8 *>(Qh + (int64_t)(qt * 16 + j) * ld + c * 64 + sb * 32 + g * 8);
  float sd[QT], best[QT];
  uint32_t qcnt[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    best[qt] = __builtin_inff();
    qcnt[qt] = 0u;
    const int qq = qt * 16 + j;
    sd[qt] = MINONLY ? 0.f : (qq < nq ? seed[qq] : -__builtin_inff());
  }
  f32x4 acc[4][QT];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) acc[rt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (total > 0) {
    const f16x8 *Xv = reinterpret_cast<const f16x8 *>(Xh);
    const int64_t tile0 = r_begin >> 6;
    f16x8 xb[R][8];
    auto load = [&](f16x8 (&b)[8], int gc) __attribute__((always_inline)) {
      const int gl = min(gc, total - 1);  // clamped: one control path past the end
      const f16x8 *p = Xv + (tile0 * KC + gl) * 512 + plane_lane(lane);  // the wave's chunks are contiguous
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = K1S_NT ? __builtin_nontemporal_load(p + i * 64) : p[i * 64];
    };
#pragma unroll
    for (int p = 0; p < R - 1; ++p) load(xb[p], p);
    for (int t = 0; t < ntiles; ++t) {
      uint32_t lw, aw;  // branch-free loads, combined at the epilogue (see K1c)
      bool w_ok;
      {
        const int64_t wi = ((r_begin + (int64_t)t * kRRows) >> 5) + (lane & 1);
        w_ok = wi < n_words;
        const int64_t wc = w_ok ? wi : n_words - 1;
        lw = __builtin_nontemporal_load(live + wc);
        aw = __builtin_nontemporal_load((allow ? allow : live) + wc);
      }
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const int gc = t * KC + c;
        load(xb[(c + R - 1) % R], gc + R - 1);  // into the slot chunk gc - 1 used
        __builtin_amdgcn_sched_barrier(0);
        const int s = c % R;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int sb = 0; sb < 2; ++sb)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
              acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb[s][rt * 2 + sb], qf[c][sb][qt], acc[rt][qt], 0,
                                                                  0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      const int64_t row0 = r_begin + (int64_t)t * kRRows;
      const uint32_t tile_words = w_ok ? (lw & aw) : 0u;
      const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)tile_words, 0);
      const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)tile_words, 1);
      coarse_epilogue<QT, MINONLY>(acc, lane_live16(((uint64_t)b1 << 32) | b0, g), row0, sd, best, qcnt,
                                   out_keys + ((int64_t)vg * qs + j) * kCBufCap);
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) acc[rt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (MINONLY) {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float m = best[qt];
      m = fminf(m, __shfl_xor(m, 16));
      m = fminf(m, __shfl_xor(m, 32));
      if (g == 0) out_min[(int64_t)vg * qs + qt * 16 + j] = m;
    }
  } else if (g == 0) {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) out_cnt[(int64_t)vg * qs + qt * 16 + j] = qcnt[qt];
  }
}

// K1c seed from the sample pre-pass: the k-th smallest of the n_wg per-workgroup minima bounds the
// k-th smallest coarse distance of the whole corpus (k distinct rows lie at or under it); + 2E.
// +inf when fewer than k groups hold an allowed row.
// qs = queries per pass in the buffer layout (K1c: kBQPass, K1s: kSQ).
#include "cm_dense_q8.inc"

// Block-wide radix select: the k-th smallest (0-based kk) of n u32 values in LDS (4 x 8-bit digits).
__device__ inline uint32_t block_select_u32(const uint32_t *vals, int n, int kk, uint32_t *hist /*[256]*/) {
  return block_select_fn([&](int i) { return vals[i]; }, n, kk, hist);
}

// seed[q] = the k-th smallest per-group minimum + add_err x E: K1c / K1s add 2E (their minima are
// coarse f16 distances and their scans test the coarse distance against the seed), K1q seeded from
// the same f16 sample adds E (its scan tests a lower bound of the true distance), K1q seeded from
// its own int8 sample adds nothing (those minima already carry their rows' bounds)
__global__ void __launch_bounds__(256) dense_seed_kernel(const float *__restrict__ mins, int n_wg, int qs, int k,
                                                         int nq, const float *__restrict__ qnorm,
                                                         const float *__restrict__ row_norms, int dim,
                                                         float *__restrict__ seed, int add_err) {
  const int qi = blockIdx.x;
  if (qi >= nq) return;
  const int qp = qi / qs, ql = qi - qp * qs;
  __shared__ uint32_t v[2048];
  __shared__ uint32_t hist[256];
  const int n = min(n_wg, 2048);
  for (int i = threadIdx.x; i < n; i += 256) v[i] = f32_order(mins[((int64_t)qp * n_wg + i) * qs + ql]);
  __syncthreads();
  // the k-th smallest minimum (radix select; +inf when fewer than k groups hold a finite one --
  // the O(n^2) rank count it replaces took ~0.1 ms per single-query search)
  const float kth = n >= k ? f32_unorder(block_select_u32(v, n, k - 1, hist)) : __builtin_inff();
  if (threadIdx.x == 0)
    seed[qi] = kth < __builtin_inff() ? (add_err ? kth + (float)add_err * coarse_err(qnorm, qi, row_norms, dim) : kth)
                                      : __builtin_inff();
}

// K1c certification + exact re-rank, one 256-thread workgroup per query.
//   For every row |c - d| <= E with
//     E = ||ql|| max||xh|| + max||xl|| ||qh|| + max||xl|| ||ql|| + dim 2^-24 max||xh|| ||qh|| + 2e-6
//   (xn.qn = xh.qh + xh.ql + xl.qh + xl.ql, products exact in f32, accumulation error bounded by
//   the recursive-summation bound, 2e-6 for the normalisations).  With c_k the k-th smallest
//   coarse distance, every row of the exact top-k has c <= T = c_k + 2E <= seed, so it sits in
//   one of the n_wg candidate buffers unless that buffer overflowed (or the band exceeds
//   kRerankCap): then the query is flagged for the exact fp32 K1 pass.  Otherwise the band's rows are
//   re-ranked with fp64 dot products of the stored fp32 rows,
//   d = 1 - (c.q) / ((||c|| + 1e-30)(||q|| + 1e-30)), ties -> lower row.
constexpr int kGatherCap = 8192;  // candidates gathered per query
__global__ void __launch_bounds__(256) dense_rerank_kernel(
    const uint64_t *__restrict__ keys, const uint32_t *__restrict__ cnts, int n_wg, int qs, int k, int nq,
    const float *__restrict__ C, int ld, int dim, const float *__restrict__ q, const float *__restrict__ qnorm,
    const float *__restrict__ row_norms, float *__restrict__ out_dist, int64_t *__restrict__ out_row,
    int32_t *__restrict__ fb_mask, int32_t *__restrict__ fb_count) {
  const int qi = blockIdx.x;
  if (qi >= nq) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qp = qi / qs, ql = qi - qp * qs;
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
      uint32_t c = b < n_wg ? cnts[((int64_t)qp * n_wg + b) * qs + ql] : 0u;
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
    return;  // the exact K1 pass writes this query's results
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
    const uint64_t key = keys[(((int64_t)qp * n_wg + lo) * qs + ql) * kCBufCap + (j - s_off[lo])];
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

// Scatter n rows (staging n x dim) into C at rows[i] (or row0+i), set invc + live, and the
// row's normalised f16 plane (K1c/K1s): xn = x * invc (hnswlib normalize_vector), Xh = f16(xn).
// The residual xl = xn - Xh is not stored (the exact passes read the fp32 rows); only its
// norm enters the running maximum of K1c's error bound.
__global__ void __launch_bounds__(256) dense_scatter_kernel(const float *__restrict__ src, const int64_t *__restrict__ rows,
                                                            int64_t row0, int64_t n, int dim, int ld,
                                                            float *__restrict__ C, float *__restrict__ invc,
                                                            uint32_t *__restrict__ live, _Float16 *__restrict__ Xh,
                                                            int64_t xh_rows, uint32_t *__restrict__ rnorm) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int64_t r = rows ? rows[i] : row0 + i;
  const bool in_plane = r < xh_rows;   // the f16 plane holds every row, or only the seed-sample prefix
  const float *s = src + i * dim;
  float *d = C + r * ld;
  float acc = 0.f;
  for (int c = threadIdx.x; c < ld; c += 256) {
    const float v = c < dim ? s[c] : 0.f;
    d[c] = v;
    acc += v * v;
  }
  __shared__ float red[4];
  __shared__ float red2[4];
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
    const _Float16 hi = (_Float16)xn;  // subnormal halves included: the matrix cores keep them
    const float lo = xn - (float)hi;    // exact residual (||xl|| of the bound E; tools/denorm_probe.hip)
    if (in_plane) Xh[plane_off(r, c, ld)] = hi;
    sh += (float)hi * (float)hi;
    sl += lo * lo;
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
    red2[threadIdx.x >> 6] = sl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float nh = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    const float nl = sqrtf((red2[0] + red2[1]) + (red2[2] + red2[3]));
    atomicMax(&rnorm[0], __float_as_uint(nh));
    atomicMax(&rnorm[1], __float_as_uint(nl));
  }
}  // the int8 plane of K1q follows per row group (dense_q8_group_kernel, launched after the scatter)

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

// k > kMaxTopK (a Chroma n_results beyond the fused top-k lists, vector_chroma.py:225-229): the
// exact distance of every live + allowed row to one query, with the re-rank kernel's formula
// d = 1 - (c.q) / ((||c|| + 1e-30)(||q|| + 1e-30)) in fp64, as a sortable (f32 distance, row) key
// (~0 for rows that cannot be returned).  One wave per 4 rows, lanes across the dims (coalesced
// 1 KB per load instruction), fp64 butterfly reduction.
__global__ void __launch_bounds__(256) dense_all_keys_kernel(const float *__restrict__ C, int ld,
                                                             const uint32_t *__restrict__ live,
                                                             const uint32_t *__restrict__ allow, int64_t size,
                                                             const float *__restrict__ qp, double qnorm,
                                                             uint64_t *__restrict__ keys) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = (((int64_t)blockIdx.x * 4) + (threadIdx.x >> 6)) * 4;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t r = r0 + u;
    if (r >= size) return;  // wave-uniform
    const float *cr = C + r * ld;
    double dq = 0.0, dc = 0.0;
    for (int c = lane * 4; c < ld; c += 256) {
      const float4 x = *reinterpret_cast<const float4 *>(cr + c);
      const float4 y = *reinterpret_cast<const float4 *>(qp + c);
      dq += (double)x.x * y.x + (double)x.y * y.y + (double)x.z * y.z + (double)x.w * y.w;
      dc += (double)x.x * x.x + (double)x.y * x.y + (double)x.z * x.z + (double)x.w * x.w;
    }
    for (int o = 32; o > 0; o >>= 1) {
      dq += __shfl_xor(dq, o);
      dc += __shfl_xor(dc, o);
    }
    if (lane == 0) {
      const uint32_t w = live[r >> 5] & (allow ? allow[r >> 5] : 0xffffffffu);
      const float dist = (float)(1.0 - dq / ((sqrt(dc) + 1e-30) * (qnorm + 1e-30)));
      keys[r] = ((w >> (r & 31)) & 1u) ? (((uint64_t)f32_order(dist) << 32) | (uint64_t)(uint32_t)r) : kEmptyKey;
    }
  }
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
  _Float16 *Xh = nullptr;                 // normalised f16 plane, fragment-major (K1c/K1s)
  int64_t xh_rows = 0;                     // rows Xh holds: all of rows_alloc, or the seed-sample prefix
  int8_t *Xq = nullptr;                    // normalised int8 plane, fragment-major (K1q)
  float2 *rmeta = nullptr;                 // per row {s_r, e_r} of the int8 plane (K1q bound)
  float *rnorm = nullptr;                  // device {max ||Xh_r||, max ||xn_r - Xh_r||, max ||s_r q8_r||, 0}
  int path = 0;                            // cm_dense_set_path (0 = automatic)
  int32_t last_fallbacks = -1;             // K1c queries re-run exactly by the last host search
  int32_t last_wide = -1;                  // K1q queries finished by the wide re-rank in the last host search
  KernelTimer timer;                       // scan-kernel events (cm_dense_timing)
  hipEvent_t seed_event = nullptr;         // cm_dense_set_seed_event: recorded after K1q's seed pass
  uint32_t *live = nullptr;
  hipStream_t stream = nullptr;
  int64_t mem_cur = 0, mem_peak = 0;       // device bytes of the four row arrays (cm_dense_mem_stats)
  int64_t staged_growths = 0;              // growths that went through host memory
  int32_t grow_mode = 0;                   // cm_dense_set_growth: 0 auto, 1 always staged (> 1 GiB)
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

// fallback: the geometry of the certificate's exact pass -- every query group spread over the whole
// chip (ranges = target), because only the groups holding a failed query run (usually one): at
// target / n_qgroups ranges a lone failing group of a 256-query batch used 32 of 256 CUs (~40 ms at
// 10M rows)
DenseCfg dense_config(const cm_dense *h, int nq, int k, bool fallback = false) {
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
  int64_t ncb = std::max<int64_t>(1, fallback ? target : target / c.n_qgroups);
  if (ncb >= 8) ncb = ncb / 8 * 8;  // same corpus range on one XCD across query groups
  ncb = std::min<int64_t>(ncb, steps);
  c.rows_per_block = ceil_div(steps, ncb) * kStepRows;
  c.n_cblocks = (int)ceil_div(c.rows_end, c.rows_per_block);
  return c;
}

template <int QB, int CH, int KMAX>
int launch_dense_t(const DenseCfg &c, const cm_dense *h, const uint32_t *allow, const float *qp, const float *invq,
                   int nq, int k, const int32_t *qmask, const int32_t *gate, uint64_t *cand, hipStream_t st) {
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
                     h->live, allow, n_words, qp, invq, nq, k, c.rows_per_block, c.rows_end, c.n_cblocks, qmask,
                     gate, cand);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int launch_dense(const DenseCfg &c, const cm_dense *h, const uint32_t *allow, const float *qp, const float *invq,
                 int nq, int k, const int32_t *qmask, const int32_t *gate, uint64_t *cand, hipStream_t st) {
#define CM_DENSE_CASE(QB_, CH_, KM_) \
  if (c.QB == QB_ && c.CH == CH_ && c.KMAX == KM_)   \
    return launch_dense_t<QB_, CH_, KM_>(c, h, allow, qp, invq, nq, k, qmask, gate, cand, st);
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

// The f16 plane (round 6).  Above kXhFullRows rows a dim-768 store searches with the
// int8 plane (K1q / K1q-s) and reads its f16 plane only for the seed pass, over a prefix of 1/16 of
// the rows: the plane then holds that prefix alone (10M x 768: 0.96 instead of 15.4 GB), the
// re-rank's middle stage reads the band rows' fp32 data directly (dense_rerank_q8_kernel with Xh =
// nullptr: every band row gets its exact fp64 distance), and the K1c / K1s scans, which read every
// row of the plane, are not eligible (dense_kind).  CM_DENSE_F16=full keeps the whole plane,
// =prefix forces the prefix at any size (tests).
constexpr int64_t kXhFullRows = 4ll << 20;
constexpr int64_t kXhPrefixFrac = 16;
int xh_mode() {   // read at every allocation (a store's policy is fixed by its arrays, not re-read per search)
  const char *e = getenv("CM_DENSE_F16");
  if (!e) return 0;
  const std::string v(e);
  return v == "full" ? 1 : v == "prefix" ? 2 : 0;
}
int64_t xh_rows_for(const cm_dense *h, int64_t cap) {
  const int m = xh_mode();
  if (h->ld != 768 || m == 1 || (m == 0 && cap <= kXhFullRows)) return cap;
  return std::min<int64_t>(cap, round_up(ceil_div(cap, kXhPrefixFrac), kStepRows));
}
// true when the f16 plane holds every written row (the K1c / K1s scans and the f16 band stage)
bool xh_full(const cm_dense *h) { return round_up(std::max<int64_t>(h->size, 1), kStepRows) <= h->xh_rows; }

// Bytes of the row arrays at `rows` rows (C fp32, invc, live bits, Xh f16 plane, Xq int8 plane + rmeta).
int64_t dense_row_bytes(const cm_dense *h, int64_t rows) {
  return rows * h->ld * 5 + xh_rows_for(h, rows) * h->ld * 2 + rows * 12 + rows / 8;
}

// Growth (dense_grow).  The arrays are reallocated at max(need, 1.5 x rows_alloc) rows.  When the
// new arrays fit in the device's free memory next to the old ones (hipMemGetInfo, with kGrowSlack to
// spare), the rows are copied device to device.  Otherwise -- or always above kStageBytes under
// grow_mode 1 (cm_dense_set_growth) -- the store moves through host memory: its written rows' fp32
// data, norms and live bits go to an uninitialised host buffer (through a pinned bounce buffer of
// kBounceBytes, so no pageable copies), the old arrays are freed, the new ones allocated and the
// rows copied back; the f16 plane is recomputed on the device from them (dense_replane_kernel,
// bit-identical to the upsert's).  The device then never holds the old and the new arrays at once:
// a store growing to hundreds of GB of HBM peaks at its final size, not 2.5 x it.
constexpr int64_t kStageBytes = 1ll << 30;
constexpr int64_t kGrowSlack = 1ll << 30;
constexpr size_t kBounceBytes = 64ull << 20;

// Host <-> device through one pinned bounce buffer (chunks of kBounceBytes, stream-synchronous).
int staged_copy(cm_dense *h, char *host, char *dev, size_t bytes, bool to_host, char *bounce) {
  for (size_t o = 0; o < bytes; o += kBounceBytes) {
    const size_t n = std::min(kBounceBytes, bytes - o);
    if (to_host) {
      CM_HIP(hipMemcpyAsync(bounce, dev + o, n, hipMemcpyDeviceToHost, h->stream));
      CM_HIP(hipStreamSynchronize(h->stream));
      memcpy(host + o, bounce, n);
    } else {
      memcpy(bounce, host + o, n);
      CM_HIP(hipMemcpyAsync(dev + o, bounce, n, hipMemcpyHostToDevice, h->stream));
      CM_HIP(hipStreamSynchronize(h->stream));
    }
  }
  return CM_OK;
}

__global__ void __launch_bounds__(256) dense_replane_kernel(const float *__restrict__ C, const float *__restrict__ invc,
                                                            int64_t r0, int64_t n, int dim, int ld,
                                                            _Float16 *__restrict__ Xh) {
  const int64_t r = r0 + blockIdx.x;
  if (r >= r0 + n) return;
  const float inv = invc[r];
  for (int c = threadIdx.x; c < ld; c += 256) {
    const float xn = (c < dim ? C[r * ld + c] : 0.f) * inv;  // == dense_scatter_kernel's
    Xh[plane_off(r, c, ld)] = (_Float16)xn;
  }
}

struct RowArrays {
  float *C = nullptr, *invc = nullptr;
  uint32_t *live = nullptr;
  _Float16 *Xh = nullptr;
  int64_t xh_rows = 0;
  int8_t *Xq = nullptr;
  float2 *rmeta = nullptr;
};

int dense_alloc_rows(cm_dense *h, int64_t cap, RowArrays &a) {
  a = RowArrays{};
  const size_t nel = (size_t)cap * h->ld;
  a.xh_rows = xh_rows_for(h, cap);
  const size_t nel_h = (size_t)a.xh_rows * h->ld;
  if (hipMalloc(&a.C, nel * 4) != hipSuccess || hipMalloc(&a.invc, (size_t)cap * 4) != hipSuccess ||
      hipMalloc(&a.live, (size_t)cap / 8) != hipSuccess || hipMalloc(&a.Xh, nel_h * 2) != hipSuccess ||
      hipMalloc(&a.Xq, nel) != hipSuccess || hipMalloc(&a.rmeta, (size_t)cap * 8) != hipSuccess) {
    for (void *p : {(void *)a.C, (void *)a.invc, (void *)a.live, (void *)a.Xh, (void *)a.Xq, (void *)a.rmeta})
      if (p) (void)hipFree(p);
    a = RowArrays{};
    CM_FAIL(CM_ENOMEM, "dense: out of device memory");
  }
  CM_HIP(hipMemsetAsync(a.C, 0, nel * 4, h->stream));
  CM_HIP(hipMemsetAsync(a.invc, 0, (size_t)cap * 4, h->stream));
  CM_HIP(hipMemsetAsync(a.live, 0, (size_t)cap / 8, h->stream));
  CM_HIP(hipMemsetAsync(a.Xh, 0, nel_h * 2, h->stream));
  CM_HIP(hipMemsetAsync(a.Xq, 0, nel, h->stream));
  CM_HIP(hipMemsetAsync(a.rmeta, 0, (size_t)cap * 8, h->stream));
  return CM_OK;
}

void dense_set_rows(cm_dense *h, const RowArrays &a) {
  h->C = a.C, h->invc = a.invc, h->live = a.live, h->Xh = a.Xh, h->Xq = a.Xq, h->rmeta = a.rmeta;
  h->xh_rows = a.xh_rows;
}

void dense_free_rows(cm_dense *h) {
  for (void *p : {(void *)h->C, (void *)h->invc, (void *)h->live, (void *)h->Xh, (void *)h->Xq, (void *)h->rmeta})
    if (p) (void)hipFree(p);
  dense_set_rows(h, RowArrays{});
}

int dense_grow(cm_dense *h, int64_t need_rows) {
  if (need_rows <= h->rows_alloc) return CM_OK;
  int64_t cap = std::max<int64_t>(need_rows, h->rows_alloc + h->rows_alloc / 2);
  cap = round_up(std::max<int64_t>(cap, kStepRows), kStepRows);
  const int64_t keep = std::min<int64_t>(round_up(h->size, kStepRows), h->rows_alloc);  // rows holding data
  RowArrays a;
  int rc;
  bool staged = keep > 0 && h->mem_cur > kStageBytes;
  if (staged && h->grow_mode == 0) {   // auto: copy on the device when old + new fit with slack
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
        (int64_t)free_b >= dense_row_bytes(h, cap) + kGrowSlack)
      staged = false;
  }
  if (staged) {
    // host-staged: fp32 rows + norms + live bits out, old arrays freed, new ones in
    const size_t cb = (size_t)keep * h->ld * 4, ib = (size_t)keep * 4, lb = (size_t)keep / 8;
    std::unique_ptr<char, void (*)(void *)> host_p(static_cast<char *>(malloc(cb + ib + lb)), free);
    char *bounce = nullptr;
    if (!host_p) CM_FAIL(CM_ENOMEM, "dense: no host memory to stage the growth");
    if (hipHostMalloc(reinterpret_cast<void **>(&bounce), kBounceBytes, hipHostMallocDefault) != hipSuccess)
      CM_FAIL(CM_ENOMEM, "dense: no pinned host memory to stage the growth");
    std::unique_ptr<char, hipError_t (*)(void *)> bounce_p(bounce, hipHostFree);
    char *host = host_p.get();
    CM_HIP(hipStreamSynchronize(h->stream));
    if ((rc = staged_copy(h, host, reinterpret_cast<char *>(h->C), cb, true, bounce))) return rc;
    if ((rc = staged_copy(h, host + cb, reinterpret_cast<char *>(h->invc), ib, true, bounce))) return rc;
    if ((rc = staged_copy(h, host + cb + ib, reinterpret_cast<char *>(h->live), lb, true, bounce))) return rc;
    dense_free_rows(h);
    h->rows_alloc = 0;
    h->mem_cur = 0;
    if ((rc = dense_alloc_rows(h, cap, a))) {
      // put the old rows back (the size just freed, so this allocation fits where the larger failed)
      cap = keep;
      if (dense_alloc_rows(h, cap, a) != CM_OK) {
        // nothing fits any more: an empty minimal store (never a handle without arrays)
        if (dense_alloc_rows(h, kStepRows, a) != CM_OK)
          CM_FAIL(CM_ENOMEM, "dense: out of device memory; the handle is unusable");
        CM_HIP(hipStreamSynchronize(h->stream));
        dense_set_rows(h, a);
        h->rows_alloc = kStepRows;
        h->size = 0;
        h->mem_cur = dense_row_bytes(h, kStepRows);
        CM_FAIL(CM_ENOMEM, "dense: out of device memory while growing; the store was emptied");
      }
      rc = CM_ENOMEM;
    }
    // (cap may now be keep: the old rows go back into an array of their old size)
    int rc2;
    if ((rc2 = staged_copy(h, host, reinterpret_cast<char *>(a.C), cb, false, bounce)) ||
        (rc2 = staged_copy(h, host + cb, reinterpret_cast<char *>(a.invc), ib, false, bounce)) ||
        (rc2 = staged_copy(h, host + cb + ib, reinterpret_cast<char *>(a.live), lb, false, bounce))) {
      dense_set_rows(h, a);
      h->rows_alloc = cap;
      h->mem_cur = dense_row_bytes(h, cap);
      return rc2;
    }
    // both coarse planes recomputed from the fp32 rows, bit-identical to the upserts'
    const int64_t kh = std::min(keep, a.xh_rows);   // the plane's rows (all, or the sample prefix)
    if (kh > 0)
      hipLaunchKernelGGL(dense_replane_kernel, dim3((unsigned)kh), dim3(256), 0, h->stream, a.C, a.invc, (int64_t)0, kh,
                         h->dim, h->ld, a.Xh);
    CM_HIP(hipGetLastError());
    hipLaunchKernelGGL(dense_q8_group_kernel, dim3((unsigned)(keep / 16)), dim3(256), 0, h->stream, a.C, a.invc,
                       (const int64_t *)nullptr, (int64_t)0, keep / 16, h->dim, h->ld, a.Xq, a.rmeta,
                       reinterpret_cast<uint32_t *>(h->rnorm));
    CM_HIP(hipGetLastError());
    CM_HIP(hipStreamSynchronize(h->stream));
    ++h->staged_growths;
    dense_set_rows(h, a);
    h->rows_alloc = cap;
    h->mem_cur = dense_row_bytes(h, cap);
    h->mem_peak = std::max(h->mem_peak, h->mem_cur);
    if (rc) CM_FAIL(CM_ENOMEM, "dense: out of device memory");
    return CM_OK;
  }
  if ((rc = dense_alloc_rows(h, cap, a))) return rc;
  h->mem_peak = std::max(h->mem_peak, h->mem_cur + dense_row_bytes(h, cap));  // old + new at once
  if (keep > 0) {
    // the planes are tile-major (64-row tiles, keep a multiple of 128): prefix copies keep them
    const size_t old = (size_t)keep * h->ld;
    CM_HIP(hipMemcpyAsync(a.C, h->C, old * 4, hipMemcpyDeviceToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(a.invc, h->invc, (size_t)keep * 4, hipMemcpyDeviceToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(a.live, h->live, (size_t)keep / 8, hipMemcpyDeviceToDevice, h->stream));
    const int64_t kh_old = std::min(keep, std::min(h->xh_rows, a.xh_rows));   // plane rows both hold
    if (kh_old > 0)
      CM_HIP(hipMemcpyAsync(a.Xh, h->Xh, (size_t)kh_old * h->ld * 2, hipMemcpyDeviceToDevice, h->stream));
    const int64_t kh_new = std::min(keep, a.xh_rows);   // a longer prefix: its new rows from the fp32 data
    if (kh_new > kh_old)
      hipLaunchKernelGGL(dense_replane_kernel, dim3((unsigned)(kh_new - kh_old)), dim3(256), 0, h->stream, a.C,
                         a.invc, kh_old, kh_new - kh_old, h->dim, h->ld, a.Xh);
    CM_HIP(hipMemcpyAsync(a.Xq, h->Xq, old, hipMemcpyDeviceToDevice, h->stream));
    CM_HIP(hipMemcpyAsync(a.rmeta, h->rmeta, (size_t)keep * 8, hipMemcpyDeviceToDevice, h->stream));
  }
  CM_HIP(hipStreamSynchronize(h->stream));
  dense_free_rows(h);
  dense_set_rows(h, a);
  h->rows_alloc = cap;
  h->mem_cur = dense_row_bytes(h, cap);
  return CM_OK;
}

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

// Scan kernel for (nq, k), the "search kind":
//   CM_DENSE_Q8S   (K1q-s) dim-768, nq <= kSQ: per-wave HBM streams of the int8 plane + re-rank;
//   CM_DENSE_Q8    (K1q)   dim-768 batches nq > kSQ: int8 plane, 256-query resident passes + re-rank;
//   CM_DENSE_STREAM (K1s)  nq <= kSQ queries, other dims (384) or CM_DENSE_Q8=0: f16 plane streams;
//   CM_DENSE_COARSE (K1c)  larger batches at dim 384 (or CM_DENSE_Q8=0): f16 resident passes;
//   CM_DENSE_F32   (K1)    exact fp32 scan: k > 32, dims other than 384 / 768, corpora under
//                          16384 rows (and the certificate's fallback).
// CM_DENSE_PATH=f32|coarse|stream|q8|q8s (or cm_dense_set_path) forces a kind for A/B probes; an
// ineligible forced kind falls back to the automatic rule.  The retired K1b (f16x3 split planes,
// kind 2) maps to the automatic rule.
int dense_kind(const cm_dense *h, int nq, int k) {
  static const int env_force = [] {
    const char *e = getenv("CM_DENSE_PATH");
    if (!e) return 0;
    const std::string s(e);
    return s == "f32" ? CM_DENSE_F32 : s == "coarse" ? CM_DENSE_COARSE : s == "stream" ? CM_DENSE_STREAM
         : s == "q8" ? CM_DENSE_Q8 : s == "q8s" ? CM_DENSE_Q8S : 0;
  }();
  static const bool q8_auto = [] {  // K1q / K1q-s automatic at dim 768 (CM_DENSE_Q8=0: K1c / K1s)
    const char *e = getenv("CM_DENSE_Q8");
    return !(e && e[0] == '0');
  }();
  const int force = h->path ? h->path : env_force;
  // coarse scans: resident-query instances for ld 768 / 384, a sample of >= 1024 rows for the seed
  const bool coarse_ok = k <= kBMaxK && (h->ld == 768 || h->ld == 384) && h->size >= 16384;
  const bool q8_ok = coarse_ok && h->ld == 768;  // K1q / K1q-s: the 6-chunk (ld 768) instances
  if (force == CM_DENSE_F32 || !coarse_ok) return CM_DENSE_F32;
  if (!xh_full(h)) {   // the f16 plane holds only the seed-sample prefix: the int8 scans (xh_rows_for)
    if (force == CM_DENSE_Q8) return CM_DENSE_Q8;
    return nq <= kSQ ? CM_DENSE_Q8S : CM_DENSE_Q8;
  }
  if (force == CM_DENSE_COARSE) return CM_DENSE_COARSE;
  if (force == CM_DENSE_STREAM && nq <= kSQ) return CM_DENSE_STREAM;
  if (force == CM_DENSE_Q8 && q8_ok) return CM_DENSE_Q8;
  if (force == CM_DENSE_Q8S && q8_ok && nq <= kSQ) return CM_DENSE_Q8S;
  // small batches: the int8 stream (half K1s's bytes; round 4 ran them on the batched K1q from 4M
  // rows, whose 256-slot MFMA work and LDS ring are waste at <= 32 queries)
  if (nq <= kSQ) return (q8_ok && q8_auto) ? CM_DENSE_Q8S : CM_DENSE_STREAM;
  return (q8_ok && q8_auto) ? CM_DENSE_Q8 : CM_DENSE_COARSE;
}

// Coarse-scan geometry.  K1c: a pass of kBQPass queries per workgroup, one workgroup per CU and
// pass; K1s: one pass of kSQ queries, n_wg = "virtual groups" = waves (4 per CU).  The sample
// pre-pass runs the same kernel over a prefix of 1/64 of the rows (1/16 below 1M rows).
// K1c form: whole passes (QPASS 256, LDS ring + LDS-resident query chunks; default) or paired
// half passes (QPASS 128, 20-slot ring, CM_K1C_PAIRED=1).  Measured at 10M x 768, B = 256:
// 4.5 vs 6.0 ms -- the ring depth is not what limits the scan (4 slots run as fast as 8).
bool k1c_paired() {
  static const bool p = [] {
    const char *e = getenv("CM_K1C_PAIRED");
    return e && e[0] == '1';
  }();
  return p;
}

// K1q's seed: by default the K1c MINONLY scan over a 1/16 row sample of the f16 plane (its bound E is
// ~30x tighter than the int8 plane's, so the seed lands near the sample's k-th distance and the scan
// appends ~3x fewer candidates: 4-14k -> ~3k per query at 10M, profiles/r04b_k1q_abl.txt);
// CM_K1Q_SEED=q8 keeps the int8 MINONLY pass over a 1/8 sample (A/B).
bool k1q_seed_q8() {
  static const bool v = [] {
    const char *e = getenv("CM_K1Q_SEED");
    return e && std::string(e) == "q8";
  }();
  return v;
}
int64_t k1qs_sample_frac() {
  // K1q-s's f16 seed sample: 1/32 of the rows (10M x 768, k = 24: B = 1 1.48 / B = 16 1.61 ms per search
  // vs 1.54 / 1.64 at 1/16 and 1.47 / 1.76 at 1/64 -- a thinner sample's looser seed costs the 16-query
  // batch more candidates than its pass saves, profiles/r05_q8s_sample_sweep.txt)
  static const int64_t v = [] {   // $CM_K1QS_SAMPLE = 1/fraction of the rows in K1q-s's seed sample (A/B knob)
    const char *e = getenv("CM_K1QS_SAMPLE");
    const int64_t f = e ? atoll(e) : 0;
    return f >= 2 && f <= 256 ? f : (int64_t)32;
  }();
  return v;
}
int64_t k1q_sample_frac() {
  static const int64_t v = [] {   // $CM_K1Q_SAMPLE = 1/fraction of the rows in the seed sample (A/B knob)
    const char *e = getenv("CM_K1Q_SAMPLE");
    const int64_t f = e ? atoll(e) : 0;
    return f >= 2 && f <= 256 ? f : (k1q_seed_q8() ? (int64_t)kQSampleFrac : 16);
  }();
  return v;
}

struct CoarseCfg {
  bool stream, paired, q8, q8s;
  int qs, n_pass, n_wg, n_wg_sample;
  int64_t rows_per_wg, rows_end, rows_per_wg_sample, rows_end_sample;
  // blocks of a K1c launch over n_wg ranges: the paired form maps blocks b, b + 8 to one (pass,
  // range) and pads the grid to whole groups of 16
  unsigned grid(int ranges) const {
    const int64_t m = (int64_t)n_pass * ranges;
    return (unsigned)(paired ? round_up(2 * m, 16) : m);
  }
};
CoarseCfg coarse_config(const cm_dense *h, int nq, int kind) {
  CoarseCfg c{};
  const bool stream = kind == CM_DENSE_STREAM || kind == CM_DENSE_Q8S;   // per-wave stream geometry
  c.stream = stream;
  c.q8s = kind == CM_DENSE_Q8S;
  c.q8 = kind == CM_DENSE_Q8 || c.q8s;                                    // int8 buffers + re-rank
  c.paired = !stream && !c.q8 && k1c_paired();
  c.qs = stream ? kSQ : kBQPass;
  c.n_pass = stream ? 1 : (int)ceil_div(nq, kBQPass);
  c.rows_end = round_up(std::max<int64_t>(h->size, 1), kStepRows);
  // row groups per pass: one pass fills the CUs; many passes (nq > 256) keep >= kMinGroups groups each
  // (more workgroups than CUs) -- fewer, longer groups would overflow the 128-slot (group, query)
  // buffers and send the whole batch to the exact pass
  constexpr int64_t kMinGroups = 64;
  int64_t groups = stream ? (int64_t)num_cus(h->dev) * 4
                          : std::max<int64_t>(kMinGroups, std::max(1, num_cus(h->dev) / c.n_pass));
  if (c.paired) groups = std::max<int64_t>(1, groups / 2);
  auto split = [&](int64_t rows_end, int64_t g, int64_t &per, int &n) {
    const int64_t tiles = rows_end / kRRows;
    per = ceil_div(tiles, std::min<int64_t>(g, tiles)) * kRRows;
    n = (int)ceil_div(rows_end, per);
  };
  split(c.rows_end, groups, c.rows_per_wg, c.n_wg);
  // K1q's per-row bounds widen the candidate set: a denser seed sample keeps it near ~4k per query
  const int64_t frac = c.q8s ? k1qs_sample_frac() : c.q8 ? k1q_sample_frac() : c.rows_end >= (1 << 20) ? 64 : 16;
  c.rows_end_sample = round_up(std::max<int64_t>(c.rows_end / frac, 1), kRRows);
  if (c.rows_end_sample > h->xh_rows)   // the sample stays inside the f16 plane's prefix (xh_rows_for)
    c.rows_end_sample = std::max<int64_t>(kRRows, h->xh_rows / kRRows * kRRows);
  // the seed is the k-th smallest of the sample groups' minima: >= kMaxTopK groups whenever the sample
  // has that many tiles, so no k <= kMaxTopK gets an infinite seed at any batch size
  split(c.rows_end_sample, std::max<int64_t>(groups, kMaxTopK), c.rows_per_wg_sample, c.n_wg_sample);
  return c;
}

struct CoarseWs {
  int8_t *qq;         // [nq_pad][ld] int8 query fragments (K1q)
  float4 *qsc;        // [nq_pad] {s_q, a_q, b_q, ||q||} (K1q)
  _Float16 *qh;       // [nq_pad][ld] normalised f16 queries
  float *qnorm;       // [nq_pad][4]
  uint64_t *keys;     // candidate buffers [pass][group][qs][kCBufCap]
  uint32_t *cnt;      // buffer fill counts [pass][group][qs]
  float *ups;         // K1q: d~ + E_r beside every candidate key [pass][group][qs][kQCap]
  float *mins;        // sample minima [pass][sample group][qs]
  float *seed;        // per-query insertion bound from the sample
  int32_t *fb_mask;   // queries sent to the exact K1 pass (K1q: 2 = the wide re-rank first)
  int32_t *fb_count;
  uint32_t *fb_bound; // K1q: kth_up of a query sent to the wide re-rank
  int32_t *wide_ctr;  // K1q wide re-rank: [0] slot allocator, [1] queries it finished
  uint32_t *wide_rows;   // [kWideSlots][kWideCap]
  uint64_t *wide_keys;   // [kWideSlots][kWideCap]
  DenseWs k1;         // the exact K1 pass's own workspace (used only for fb_mask queries)
  size_t total;
};
CoarseWs coarse_ws_layout(const cm_dense *h, const CoarseCfg &c, int nq, int k, void *base) {
  CoarseWs w{};
  char *p = reinterpret_cast<char *>(base);
  size_t off = 0;
  const int64_t nq_pad = (int64_t)c.n_pass * c.qs;
  auto take = [&](int64_t bytes) -> char * {
    char *r = p + off;
    off += round_up(std::max<int64_t>(bytes, 1), 256);
    return r;
  };
  const int cap = c.q8 ? kQCap : kCBufCap;
  if (c.q8) {
    w.qq = reinterpret_cast<int8_t *>(take(nq_pad * h->ld));
    w.qsc = reinterpret_cast<float4 *>(take(nq_pad * 16));
  }
  w.qh = reinterpret_cast<_Float16 *>(take(nq_pad * h->ld * 2));
  w.qnorm = reinterpret_cast<float *>(take(nq_pad * 16));
  w.keys = reinterpret_cast<uint64_t *>(take((int64_t)c.n_pass * c.n_wg * c.qs * cap * 8));
  if (c.q8) w.ups = reinterpret_cast<float *>(take((int64_t)c.n_pass * c.n_wg * c.qs * cap * 4));
  w.cnt = reinterpret_cast<uint32_t *>(take((int64_t)c.n_pass * c.n_wg * c.qs * 4));
  w.mins = reinterpret_cast<float *>(take((int64_t)c.n_pass * c.n_wg_sample * c.qs * 4));
  w.seed = reinterpret_cast<float *>(take(nq_pad * 4));
  w.fb_mask = reinterpret_cast<int32_t *>(take(nq_pad * 4));
  w.fb_count = reinterpret_cast<int32_t *>(take(4));
  if (c.q8) {
    w.fb_bound = reinterpret_cast<uint32_t *>(take(nq_pad * 4));
    w.wide_ctr = reinterpret_cast<int32_t *>(take(8));
    w.wide_rows = reinterpret_cast<uint32_t *>(take((int64_t)kWideSlots * kWideCap * 4));
    w.wide_keys = reinterpret_cast<uint64_t *>(take((int64_t)kWideSlots * kWideCap * 8));
  }
  const DenseCfg kc = dense_config(h, nq, k, true);
  w.k1 = dense_ws_layout(h, kc, nq, k, p ? p + off : nullptr);
  off += w.k1.total;
  w.total = off;
  return w;
}

int set_coarse_attrs() {
  static std::once_flag once;
  static hipError_t err = hipSuccess;
  std::call_once(once, [] {
    const std::pair<const void *, int> fs[] = {
        {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<12, kK1cNql, false, kK1cWaves>), K1rLds<kK1cNql>::total},
        {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<12, kK1cNql, true, kK1cWaves>), K1rLds<kK1cNql>::total},
        {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<6, 0, false, kK1cWaves>), K1rLds<0>::total},
        {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<6, 0, true, kK1cWaves>), K1rLds<0>::total},
        {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<12, 0, false, 4, 20, 128>), K1rLds<0, 20>::total},
        {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<12, 0, true, 4, 20, 128>), K1rLds<0, 20>::total},
        {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<6, 0, false, 4, 20, 128>), K1rLds<0, 20>::total},
        {reinterpret_cast<const void *>(&dense_coarse_scan_kernel<6, 0, true, 4, 20, 128>), K1rLds<0, 20>::total},
        {reinterpret_cast<const void *>(&dense_rerank_kernel), kGatherCap * 12},
        {reinterpret_cast<const void *>(&dense_q8_scan_kernel<false>), kQLds},
        {reinterpret_cast<const void *>(&dense_q8_scan_kernel<true>), kQLds},
        {reinterpret_cast<const void *>(&dense_q8_scan_kernel<true, K1Q_LDS_SHARED>), kQLdsShared},
        {reinterpret_cast<const void *>(&dense_q8_scan_kernel<false, K1Q_LDS_SHARED>), kQLdsShared},
        {reinterpret_cast<const void *>(&dense_rerank_q8_kernel), kQRerankLds}};
    for (const auto &f : fs) {
      const hipError_t e = hipFuncSetAttribute(f.first, hipFuncAttributeMaxDynamicSharedMemorySize, f.second);
      if (e != hipSuccess) err = e;
    }
  });
  CM_HIP(err);
  return CM_OK;
}

using StreamFn = void (*)(const _Float16 *, const uint32_t *, const uint32_t *, int64_t, const _Float16 *, int,
                          const float *, int64_t, int64_t, int, int, uint64_t *, uint32_t *, float *);
StreamFn stream_kernel(int ld, int nq, bool minonly) {
  const bool two = nq > 16;
  if (ld == 768)
    return two ? (minonly ? &dense_stream_scan_kernel<12, 2, true> : &dense_stream_scan_kernel<12, 2, false>)
               : (minonly ? &dense_stream_scan_kernel<12, 1, true> : &dense_stream_scan_kernel<12, 1, false>);
  return two ? (minonly ? &dense_stream_scan_kernel<6, 2, true> : &dense_stream_scan_kernel<6, 2, false>)
             : (minonly ? &dense_stream_scan_kernel<6, 1, true> : &dense_stream_scan_kernel<6, 1, false>);
}

// K1c / K1s: sample pre-pass -> seed -> coarse scan -> certificate + exact re-rank; the queries
// whose certificate fails (fb_mask) are re-searched by the exact fp32 K1 and merged (every
// workgroup of those launches exits at once when there are none: graph-capturable, no host sync).
int launch_exact_fallback(cm_dense *h, const float *q_dev, int nq, int k, int kind, const uint32_t *allow,
                          float *dist_dev, int64_t *row_dev, void *ws, int64_t ws_bytes, hipStream_t st);
int launch_coarse(cm_dense *h, const float *q_dev, int nq, int k, int kind, const uint32_t *allow,
                  float *dist_dev, int64_t *row_dev, void *ws, int64_t ws_bytes, hipStream_t st,
                  bool run_exact = true) {
  int rc;
  if ((rc = set_coarse_attrs())) return rc;
  const bool stream = kind == CM_DENSE_STREAM;
  const CoarseCfg c = coarse_config(h, nq, kind);
  const CoarseWs w = coarse_ws_layout(h, c, nq, k, ws);
  if ((int64_t)w.total > ws_bytes || !ws) CM_FAIL(CM_EINVAL, "dense workspace too small");
  const int64_t n_words = ceil_div(h->size, 32);
  hipLaunchKernelGGL(dense_prep_planes, dim3(c.n_pass * c.qs), dim3(256), 0, st, q_dev, nq, h->dim, h->ld, w.qh,
                     w.qnorm);
  CM_HIP(hipGetLastError());
  CM_HIP(hipMemsetAsync(w.fb_count, 0, 4, st));
  if (c.q8) CM_HIP(hipMemsetAsync(w.wide_ctr, 0, 8, st));
  if (c.q8) {
    // K1q: int8 queries -> seed from a row sample -> scan -> certified re-rank (int8 band -> f16 band
    // -> fp64)
    hipLaunchKernelGGL(dense_prep_q8, dim3(c.n_pass * c.qs), dim3(256), 0, st, q_dev, nq, h->dim, h->ld, w.qq, w.qsc,
                       reinterpret_cast<const uint32_t *>(h->rnorm));
    CM_HIP(hipGetLastError());
    if (c.q8s) {   // K1q-s: K1s's MINONLY stream over the f16 plane's sample, then the int8 stream
      hipLaunchKernelGGL(stream_kernel(h->ld, nq, true), dim3((unsigned)ceil_div(c.n_wg_sample, 4)), dim3(256), 0, st,
                         h->Xh, h->live, allow, n_words, w.qh, nq, (const float *)nullptr, c.rows_per_wg_sample,
                         c.rows_end_sample, c.n_wg_sample, c.qs, (uint64_t *)nullptr, (uint32_t *)nullptr, w.mins);
      CM_HIP(hipGetLastError());
      hipLaunchKernelGGL(dense_seed_kernel, dim3(nq), dim3(256), 0, st, w.mins, c.n_wg_sample, c.qs, k, nq, w.qnorm,
                         h->rnorm, h->dim, w.seed, 1);
      CM_HIP(hipGetLastError());
      h->timer.begin(st);
      if (nq > 16)
        hipLaunchKernelGGL((dense_q8_stream_kernel<2, K1QS_RING>), dim3((unsigned)ceil_div(c.n_wg, 4)), dim3(256), 0, st,
                           h->Xq, h->rmeta, h->live, allow, n_words, w.qq, w.qsc, nq, (const float *)w.seed,
                           c.rows_per_wg, c.rows_end, c.n_wg, w.keys, w.ups, w.cnt);
      else
        hipLaunchKernelGGL((dense_q8_stream_kernel<1, K1QS_RING>), dim3((unsigned)ceil_div(c.n_wg, 4)), dim3(256), 0, st,
                           h->Xq, h->rmeta, h->live, allow, n_words, w.qq, w.qsc, nq, (const float *)w.seed,
                           c.rows_per_wg, c.rows_end, c.n_wg, w.keys, w.ups, w.cnt);
      h->timer.end(st);
      CM_HIP(hipGetLastError());
    } else {
    if (k1q_seed_q8()) {   // (deferred search: the shared LDS footprint, beside the BM25 blocks)
      if (run_exact || !env_knob("CM_K1Q_SHARED_LDS", true))
        hipLaunchKernelGGL(dense_q8_scan_kernel<true>, dim3(c.n_pass * c.n_wg_sample), dim3(256), kQLds, st, h->Xq,
                           h->rmeta, h->live, allow, n_words, w.qq, w.qsc, nq, (const float *)nullptr,
                           c.rows_per_wg_sample, c.rows_end_sample, c.n_wg_sample, (uint64_t *)nullptr,
                           (float *)nullptr, (uint32_t *)nullptr, w.mins);
      else
        hipLaunchKernelGGL((dense_q8_scan_kernel<true, K1Q_LDS_SHARED>), dim3(c.n_pass * c.n_wg_sample), dim3(256),
                           kQLdsShared, st, h->Xq, h->rmeta, h->live, allow, n_words, w.qq, w.qsc, nq,
                           (const float *)nullptr, c.rows_per_wg_sample, c.rows_end_sample, c.n_wg_sample,
                           (uint64_t *)nullptr, (float *)nullptr, (uint32_t *)nullptr, w.mins);
    } else {   // K1c MINONLY over the f16 plane's sample (dim 768: the resident-query instance)
      hipLaunchKernelGGL((dense_coarse_scan_kernel<12, kK1cNql, true, kK1cWaves>), dim3(c.grid(c.n_wg_sample)),
                         dim3(64 * kK1cWaves), K1rLds<kK1cNql>::total, st, h->Xh, h->live, allow, n_words, w.qh, nq,
                         (const float *)nullptr, c.rows_per_wg_sample, c.rows_end_sample, c.n_wg_sample,
                         (uint64_t *)nullptr, (uint32_t *)nullptr, w.mins, 0);
    }
    CM_HIP(hipGetLastError());
    hipLaunchKernelGGL(dense_seed_kernel, dim3(nq), dim3(256), 0, st, w.mins, c.n_wg_sample, c.qs, k, nq, w.qnorm,
                       h->rnorm, h->dim, w.seed, k1q_seed_q8() ? 0 : 1);
    CM_HIP(hipGetLastError());
    if (h->seed_event) CM_HIP(hipEventRecord(h->seed_event, st));
    h->timer.begin(st);
    // deferred search (!run_exact): the caller runs other work beside it -> the shared LDS footprint
    // (CM_K1Q_SHARED_LDS=0: the full one, A/B)
    if (run_exact || !env_knob("CM_K1Q_SHARED_LDS", true))
      hipLaunchKernelGGL(dense_q8_scan_kernel<false>, dim3(c.n_pass * c.n_wg), dim3(256), kQLds, st, h->Xq,
                         h->rmeta, h->live, allow, n_words, w.qq, w.qsc, nq, (const float *)w.seed, c.rows_per_wg,
                         c.rows_end, c.n_wg, w.keys, w.ups, w.cnt, (float *)nullptr);
    else
      hipLaunchKernelGGL((dense_q8_scan_kernel<false, K1Q_LDS_SHARED>), dim3(c.n_pass * c.n_wg), dim3(256), kQLdsShared,
                         st, h->Xq, h->rmeta, h->live, allow, n_words, w.qq, w.qsc, nq, (const float *)w.seed,
                         c.rows_per_wg, c.rows_end, c.n_wg, w.keys, w.ups, w.cnt, (float *)nullptr);
    h->timer.end(st);
    CM_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(dense_rerank_q8_kernel, dim3(nq), dim3(kQRT), kQRerankLds, st, w.keys, w.ups, w.cnt, c.n_wg, c.qs, k,
                       nq, h->C, h->ld, h->dim, q_dev, w.qsc, xh_full(h) ? h->Xh : nullptr, w.qh, w.qnorm, h->rnorm,
                       dist_dev, row_dev,
                       w.fb_mask, w.fb_count, w.fb_bound);
    CM_HIP(hipGetLastError());
    // band overflow with complete candidate buffers: the wide re-rank (gated; ~5 us when none failed;
    // CM_K1Q_WIDE=0: the exact scan takes every failing query, A/B)
    if (env_knob("CM_K1Q_WIDE", true))
      hipLaunchKernelGGL(dense_rerank_wide_kernel, dim3(nq), dim3(kWideThreads), 0, st, w.keys, w.cnt, c.n_wg, c.qs, k,
                         nq, h->C, h->ld, h->dim, q_dev, w.qsc, xh_full(h) ? h->Xh : nullptr, w.qh, w.qnorm, h->rnorm,
                         h->Xq, h->rmeta, w.qq, h->live, allow,
                         n_words, c.rows_per_wg, c.rows_end, dist_dev, row_dev, w.fb_mask, w.fb_count, w.fb_bound, w.wide_ctr,
                         w.wide_rows, w.wide_keys);
    CM_HIP(hipGetLastError());
  } else {
  const bool d768 = h->ld == 768;
  const size_t slds = c.paired ? K1rLds<0, 20>::total : d768 ? K1rLds<kK1cNql>::total : K1rLds<0>::total;
  const int k1c_threads = c.paired ? 256 : 64 * kK1cWaves;
  auto k1c = [&](bool minonly) {
    if (c.paired) {
      if (d768)
        return minonly ? &dense_coarse_scan_kernel<12, 0, true, 4, 20, 128>
                       : &dense_coarse_scan_kernel<12, 0, false, 4, 20, 128>;
      return minonly ? &dense_coarse_scan_kernel<6, 0, true, 4, 20, 128>
                     : &dense_coarse_scan_kernel<6, 0, false, 4, 20, 128>;
    }
    if (d768) return minonly ? &dense_coarse_scan_kernel<12, kK1cNql, true, kK1cWaves> : &dense_coarse_scan_kernel<12, kK1cNql, false, kK1cWaves>;
    return minonly ? &dense_coarse_scan_kernel<6, 0, true, kK1cWaves> : &dense_coarse_scan_kernel<6, 0, false, kK1cWaves>;
  };
  // 1. sample pre-pass (per-group minima) -> seed
  if (stream) {
    hipLaunchKernelGGL(stream_kernel(h->ld, nq, true), dim3((unsigned)ceil_div(c.n_wg_sample, 4)), dim3(256), 0, st,
                       h->Xh, h->live, allow, n_words, w.qh, nq, (const float *)nullptr, c.rows_per_wg_sample,
                       c.rows_end_sample, c.n_wg_sample, c.qs, (uint64_t *)nullptr, (uint32_t *)nullptr, w.mins);
  } else {
    hipLaunchKernelGGL(k1c(true), dim3(c.grid(c.n_wg_sample)), dim3(k1c_threads), slds, st, h->Xh, h->live,
                       allow, n_words, w.qh, nq, (const float *)nullptr, c.rows_per_wg_sample, c.rows_end_sample,
                       c.n_wg_sample, (uint64_t *)nullptr, (uint32_t *)nullptr, w.mins, 0);
  }
  CM_HIP(hipGetLastError());
  hipLaunchKernelGGL(dense_seed_kernel, dim3(nq), dim3(256), 0, st, w.mins, c.n_wg_sample, c.qs, k, nq, w.qnorm,
                     h->rnorm, h->dim, w.seed, 2);
  CM_HIP(hipGetLastError());
  // 2. coarse scan: rows under the seed -> candidate buffers
  h->timer.begin(st);
  if (stream) {
    hipLaunchKernelGGL(stream_kernel(h->ld, nq, false), dim3((unsigned)ceil_div(c.n_wg, 4)), dim3(256), 0, st, h->Xh,
                       h->live, allow, n_words, w.qh, nq, (const float *)w.seed, c.rows_per_wg, c.rows_end, c.n_wg,
                       c.qs, w.keys, w.cnt, (float *)nullptr);
  } else {
    hipLaunchKernelGGL(k1c(false), dim3(c.grid(c.n_wg)), dim3(k1c_threads), slds, st, h->Xh, h->live, allow,
                       n_words, w.qh, nq, (const float *)w.seed, c.rows_per_wg, c.rows_end, c.n_wg, w.keys, w.cnt,
                       (float *)nullptr, dense_debug_flags());
  }
  h->timer.end(st);
  CM_HIP(hipGetLastError());
  // 3. certificate + exact re-rank (failures -> fb_mask)
  hipLaunchKernelGGL(dense_rerank_kernel, dim3(nq), dim3(256), kGatherCap * 12, st, w.keys, w.cnt, c.n_wg, c.qs, k,
                     nq, h->C, h->ld, h->dim, q_dev, w.qnorm, h->rnorm, dist_dev, row_dev, w.fb_mask, w.fb_count);
  CM_HIP(hipGetLastError());
  }
  return run_exact ? launch_exact_fallback(h, q_dev, nq, k, kind, allow, dist_dev, row_dev, ws, ws_bytes, st) : CM_OK;
}

// 4. the certificate's fallback: exact fp32 K1 for the rejected queries only (fb_mask), merged into
// their rows of the output.  Gated on the device by fb_count (every workgroup of the K1 grid leaves at
// once when nothing failed: no host sync, graph-capturable).  cm_dense_search_dev runs it right
// after the re-rank; cm_dense_search_dev_deferred leaves it to cm_dense_exact_fallback_dev, so a
// caller can enqueue it behind other streams' work -- the K1 grid asks for ~150 KiB of LDS per
// workgroup, and even workgroups that leave at once wait for CUs whose LDS other kernels hold
// (0.5 ms per step beside the BM25 stream).
int launch_exact_fallback(cm_dense *h, const float *q_dev, int nq, int k, int kind, const uint32_t *allow,
                          float *dist_dev, int64_t *row_dev, void *ws, int64_t ws_bytes, hipStream_t st) {
  const CoarseCfg c = coarse_config(h, nq, kind);
  const CoarseWs w = coarse_ws_layout(h, c, nq, k, ws);
  if ((int64_t)w.total > ws_bytes || !ws) CM_FAIL(CM_EINVAL, "dense workspace too small");
  const DenseCfg kc = dense_config(h, nq, k, true);
  if (kc.lds > 163840) CM_FAIL(CM_EUNSUPPORTED, "dim/k too large for the LDS-resident query tile");
  hipLaunchKernelGGL(dense_prep_queries, dim3(kc.n_qgroups * kc.QB), dim3(256), 0, st, q_dev, nq, h->dim, h->ld,
                     w.k1.qp, w.k1.invq);
  CM_HIP(hipGetLastError());
  int rc;
  if ((rc = launch_dense(kc, h, allow, w.k1.qp, w.k1.invq, nq, k, w.fb_mask, w.fb_count, w.k1.cand, st))) return rc;
  hipLaunchKernelGGL(dense_merge_kernel, dim3(nq), dim3(256), 0, st, w.k1.cand, kc.n_cblocks, kc.QB, k, nq,
                     (const int32_t *)w.fb_mask, dist_dev, row_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

// Host-array search with k > kMaxTopK: every row's exact key, one device radix sort per query, the
// first k keys (ascending (distance, row), -1 padding past the live + allowed rows).
int dense_search_full(cm_dense *h, const float *q, int nq, int k, const uint32_t *allow_bits, float *out_dist,
                      int64_t *out_row, float *out_vec) {
  const int64_t n = std::max<int64_t>(h->size, 1);
  int rc;
  size_t tmp_bytes = 0;
  CM_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                           (int)n, 0, 64, h->stream));
  const size_t keys_off = round_up((int64_t)tmp_bytes, 256);
  const size_t q_off = keys_off + round_up(n * 16, 256);
  if ((rc = h->ws.ensure(q_off + (size_t)h->ld * 4))) return rc;
  char *base = h->ws.as<char>();
  uint64_t *keys = reinterpret_cast<uint64_t *>(base + keys_off), *sorted = keys + n;
  float *qp = reinterpret_cast<float *>(base + q_off);
  const uint32_t *allow_dev = nullptr;
  const int64_t nw = ceil_div(h->size, 32);
  if (allow_bits) {
    if ((rc = h->allow_buf.ensure((size_t)std::max<int64_t>(nw, 1) * 4))) return rc;
    CM_HIP(hipMemcpyAsync(h->allow_buf.ptr, allow_bits, (size_t)nw * 4, hipMemcpyDefault, h->stream));
    allow_dev = h->allow_buf.as<uint32_t>();
  }
  CM_HIP(hipMemsetAsync(keys, 0xff, (size_t)n * 8, h->stream));  // rows past size (empty store) sort last
  const int kk = (int)std::min<int64_t>(k, n);
  std::vector<uint64_t> top((size_t)kk);
  std::vector<float> qpad((size_t)h->ld, 0.f);
  for (int i = 0; i < nq; ++i) {
    double qn = 0.0;
    for (int c = 0; c < h->dim; ++c) {
      qpad[c] = q[(int64_t)i * h->dim + c];
      qn += (double)qpad[c] * qpad[c];
    }
    CM_HIP(hipMemcpyAsync(qp, qpad.data(), (size_t)h->ld * 4, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(dense_all_keys_kernel, dim3((unsigned)ceil_div(n, 16)), dim3(256), 0, h->stream, h->C, h->ld,
                       h->live, allow_dev, h->size, qp, std::sqrt(qn), keys);
    CM_HIP(hipGetLastError());
    CM_HIP(hipcub::DeviceRadixSort::SortKeys(base, tmp_bytes, keys, sorted, (int)n, 0, 64, h->stream));
    CM_HIP(hipMemcpyAsync(top.data(), sorted, (size_t)kk * 8, hipMemcpyDeviceToHost, h->stream));
    CM_HIP(hipStreamSynchronize(h->stream));
    for (int j = 0; j < k; ++j) {
      const uint64_t key = j < kk ? top[j] : kEmptyKey;
      out_dist[(int64_t)i * k + j] = key == kEmptyKey ? 0.f : f32_unorder((uint32_t)(key >> 32));
      out_row[(int64_t)i * k + j] = key == kEmptyKey ? -1 : (int64_t)(uint32_t)key;
    }
  }
  if (out_vec) {  // stored fp32 rows of the results (include_embeddings)
    const size_t nr = (size_t)nq * k;
    if ((rc = h->rows_buf.ensure(nr * 8)) || (rc = h->out_buf.ensure(nr * h->dim * 4))) return rc;
    CM_HIP(hipMemcpyAsync(h->rows_buf.ptr, out_row, nr * 8, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(dense_gather_kernel, dim3((unsigned)nr), dim3(256), 0, h->stream, h->C, h->ld, h->dim,
                       h->rows_buf.as<int64_t>(), (int64_t)nr, h->size, h->out_buf.as<float>());
    CM_HIP(hipGetLastError());
    CM_HIP(hipMemcpyAsync(out_vec, h->out_buf.ptr, nr * h->dim * 4, hipMemcpyDeviceToHost, h->stream));
    CM_HIP(hipStreamSynchronize(h->stream));
  }
  h->last_fallbacks = 0;
  h->last_wide = 0;
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
  if (hipMalloc(&h->rnorm, 16) != hipSuccess || hipMemset(h->rnorm, 0, 16) != hipSuccess) {
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
  dense_free_rows(h);
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
                       h->rows_buf.as<int64_t>(), (int64_t)0, m, h->dim, h->ld, h->C, h->invc, h->live, h->Xh,
                       h->xh_rows, reinterpret_cast<uint32_t *>(h->rnorm));
    CM_HIP(hipGetLastError());
    // the int8 plane: every row group the batch touched, once (stream-ordered after the scatter)
    std::vector<int64_t> gs((size_t)m);
    for (int64_t i = 0; i < m; ++i) gs[(size_t)i] = q8_group_of(rows[s + i]);
    std::sort(gs.begin(), gs.end());
    gs.erase(std::unique(gs.begin(), gs.end()), gs.end());
    CM_HIP(hipMemcpyAsync(h->rows_buf.ptr, gs.data(), gs.size() * 8, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(dense_q8_group_kernel, dim3((unsigned)gs.size()), dim3(256), 0, h->stream, h->C, h->invc,
                       h->rows_buf.as<int64_t>(), (int64_t)0, (int64_t)gs.size(), h->dim, h->ld, h->Xq, h->rmeta,
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
                       h->xh_rows, reinterpret_cast<uint32_t *>(h->rnorm));
    CM_HIP(hipGetLastError());
  }
  // the int8 plane of every row group in the written tiles (rows_alloc is a multiple of 128)
  const int64_t g_lo = (row0 >> 6) * 4, g_hi = ((row0 + n - 1) >> 6) * 4 + 4;
  hipLaunchKernelGGL(dense_q8_group_kernel, dim3((unsigned)(g_hi - g_lo)), dim3(256), 0, st, h->C, h->invc,
                     (const int64_t *)nullptr, g_lo, g_hi - g_lo, h->dim, h->ld, h->Xq, h->rmeta,
                     reinterpret_cast<uint32_t *>(h->rnorm));
  CM_HIP(hipGetLastError());
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
  CM_HIP(hipMemsetAsync(h->Xh, 0, (size_t)h->xh_rows * h->ld * 2, h->stream));
  CM_HIP(hipMemsetAsync(h->Xq, 0, (size_t)h->rows_alloc * h->ld, h->stream));
  CM_HIP(hipMemsetAsync(h->rmeta, 0, (size_t)h->rows_alloc * 8, h->stream));
  CM_HIP(hipMemsetAsync(h->rnorm, 0, 16, h->stream));
  CM_HIP(hipStreamSynchronize(h->stream));
  h->size = 0;
  return CM_OK;
}

int cm_dense_set_growth(cm_dense *h, int32_t mode) {
  if (!h) CM_FAIL(CM_EINVAL, "cm_dense_set_growth: null handle");
  if (mode != 0 && mode != 1) CM_FAIL(CM_EINVAL, "cm_dense_set_growth: mode must be 0 (auto) or 1 (staged)");
  h->grow_mode = mode;
  return CM_OK;
}

int cm_dense_mem_stats(cm_dense *h, int64_t *cur_bytes, int64_t *peak_bytes, int64_t *staged_growths) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (cur_bytes) *cur_bytes = h->mem_cur;
  if (peak_bytes) *peak_bytes = h->mem_peak;
  if (staged_growths) *staged_growths = h->staged_growths;
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
  if (kind != CM_DENSE_F32)
    return (int64_t)coarse_ws_layout(h, coarse_config(h, nq, kind), nq, k, nullptr).total;
  DenseCfg c = dense_config(h, nq, k);
  return (int64_t)dense_ws_layout(h, c, nq, k, nullptr).total;
}

int cm_dense_set_path(cm_dense *h, int32_t kind) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (kind < 0 || kind > CM_DENSE_Q8S) CM_FAIL(CM_EINVAL, "unknown dense path");
  h->path = kind;
  return CM_OK;
}

int32_t cm_dense_workspace_fallbacks(cm_dense *h, int32_t nq, int32_t k, const void *workspace_dev) {
  if (!h || !workspace_dev || nq <= 0 || k <= 0 || k > kMaxTopK) return -1;
  const int kind = dense_kind(h, nq, k);
  if (kind == CM_DENSE_F32) return 0;
  DeviceGuard dg(h->dev);
  const CoarseWs w = coarse_ws_layout(h, coarse_config(h, nq, kind), nq, k,
                                      const_cast<void *>(workspace_dev));
  int32_t c = -1;
  if (hipMemcpy(&c, w.fb_count, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return c;
}

int32_t cm_dense_last_fallbacks(cm_dense *h) { return h ? h->last_fallbacks : -1; }

int32_t cm_dense_workspace_wide_reranks(cm_dense *h, int32_t nq, int32_t k, const void *workspace_dev) {
  if (!h || !workspace_dev || nq <= 0 || k <= 0 || k > kMaxTopK) return -1;
  const int kind = dense_kind(h, nq, k);
  if (kind != CM_DENSE_Q8 && kind != CM_DENSE_Q8S) return 0;
  DeviceGuard dg(h->dev);
  const CoarseWs w = coarse_ws_layout(h, coarse_config(h, nq, kind), nq, k, const_cast<void *>(workspace_dev));
  int32_t c[2] = {-1, -1};
  if (hipMemcpy(c, w.wide_ctr, 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return c[1];
}

int32_t cm_dense_last_wide_reranks(cm_dense *h) { return h ? h->last_wide : -1; }

int cm_dense_set_seed_event(cm_dense *h, void *event) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  h->seed_event = (hipEvent_t)event;
  return CM_OK;
}

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
    return launch_coarse(h, q_dev, nq, k, kind, allow_dev, dist_dev, row_dev, workspace_dev, workspace_bytes, st);
  DenseCfg c = dense_config(h, nq, k);
  if (c.lds > 163840) CM_FAIL(CM_EUNSUPPORTED, "dim/k too large for the LDS-resident query tile");
  DenseWs w = dense_ws_layout(h, c, nq, k, workspace_dev);
  if ((int64_t)w.total > workspace_bytes || !workspace_dev) CM_FAIL(CM_EINVAL, "dense workspace too small");
  const int nq_pad = c.n_qgroups * c.QB;
  hipLaunchKernelGGL(dense_prep_queries, dim3(nq_pad), dim3(256), 0, st, q_dev, nq, h->dim, h->ld, w.qp, w.invq);
  CM_HIP(hipGetLastError());
  h->timer.begin(st);
  int rc = launch_dense(c, h, allow_dev, w.qp, w.invq, nq, k, (const int32_t *)nullptr, (const int32_t *)nullptr,
                        w.cand, st);
  h->timer.end(st);
  if (rc) return rc;
  hipLaunchKernelGGL(dense_merge_kernel, dim3(nq), dim3(256), 0, st, w.cand, c.n_cblocks, c.QB, k, nq,
                     (const int32_t *)nullptr, dist_dev,
                     row_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

int cm_dense_search_dev_deferred(cm_dense *h, const float *q_dev, int32_t nq, int32_t k, const uint32_t *allow_dev,
                                 float *dist_dev, int64_t *row_dev, void *workspace_dev, int64_t workspace_bytes,
                                 void *stream) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (k <= 0 || k > kMaxTopK) CM_FAIL(CM_EINVAL, "k must be in [1, " + std::to_string(kMaxTopK) + "]");
  const int kind = dense_kind(h, nq, k);
  if (kind == CM_DENSE_F32)   // the exact scan: nothing to defer
    return cm_dense_search_dev(h, q_dev, nq, k, allow_dev, dist_dev, row_dev, workspace_dev, workspace_bytes, stream);
  DeviceGuard dg(h->dev);
  return launch_coarse(h, q_dev, nq, k, kind, allow_dev, dist_dev, row_dev, workspace_dev, workspace_bytes,
                       (hipStream_t)stream, false);
}

int cm_dense_exact_fallback_dev(cm_dense *h, const float *q_dev, int32_t nq, int32_t k, const uint32_t *allow_dev,
                                float *dist_dev, int64_t *row_dev, void *workspace_dev, int64_t workspace_bytes,
                                void *stream) {
  if (!h) CM_FAIL(CM_EINVAL, "null handle");
  if (nq <= 0) return CM_OK;
  if (k <= 0 || k > kMaxTopK) CM_FAIL(CM_EINVAL, "k must be in [1, " + std::to_string(kMaxTopK) + "]");
  const int kind = dense_kind(h, nq, k);
  if (kind == CM_DENSE_F32) return CM_OK;
  DeviceGuard dg(h->dev);
  return launch_exact_fallback(h, q_dev, nq, k, kind, allow_dev, dist_dev, row_dev, workspace_dev, workspace_bytes,
                               (hipStream_t)stream);
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
  if (k <= 0) CM_FAIL(CM_EINVAL, "k must be >= 1");
  DeviceGuard dg(h->dev);
  if (k > kMaxTopK) return dense_search_full(h, q, nq, k, allow_bits, out_dist, out_row, out_vec);
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
  h->last_wide = 0;
  const int kind = dense_kind(h, nq, k);
  if (kind != CM_DENSE_F32) {
    const CoarseWs w = coarse_ws_layout(h, coarse_config(h, nq, kind), nq, k, h->ws.ptr);
    CM_HIP(hipMemcpyAsync(&h->last_fallbacks, w.fb_count, 4, hipMemcpyDeviceToHost, h->stream));
    if (w.wide_ctr) CM_HIP(hipMemcpyAsync(&h->last_wide, w.wide_ctr + 1, 4, hipMemcpyDeviceToHost, h->stream));
  }
  CM_HIP(hipStreamSynchronize(h->stream));
  return CM_OK;
}

}  // extern "C"

