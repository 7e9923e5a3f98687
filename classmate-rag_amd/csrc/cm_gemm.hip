// K10: fp32-accurate linear layers of the E5 (XLM-R) forward on the f16 matrix cores.
//
// The reference encodes in fp32 (sentence-transformers on torch fp32,
// rag/embeddings/__init__.py:85-105): every projection of XLM-R is y = x W^T + b with fp32
// operands and fp32 accumulation.  gfx950's fp32 MFMA runs at the fp32 vector rate (157 TF),
// 1/16 of the f16 rate, and has no reduced-precision xf32 form.  Here each fp32 operand is
// split into two f16 halves, v = hi + lo (hi = f16(v), lo = f16(v - hi): 22 significant bits),
// and the product is accumulated from three f16 MFMAs, lo.hi + hi.lo + hi.hi, in fp32
// (v_mfma_f32_16x16x32_f16 multiplies exactly and accumulates in fp32).  The dropped lo.lo
// term and the rounding of the lo halves are each <= 2^-22 relative per product, below the
// 2^-24 rounding of one fp32 accumulation step times the sqrt(K) growth of a K = 768 / 3072
// reduction -- the result is as accurate as the fp32 GEMM it replaces (tests/test_gpu_gemm.py
// holds it to 2x torch's fp32 GEMM error against fp64), at 16/3 of its peak rate.
//
// Range: f16 has a 5-bit exponent.  Weights are split once (cm_f16x3_split_weights) after a
// power-of-two scale that puts max|W| at 2^14..2^15, so no weight's lo half is subnormal
// except where its absolute error is < 2^-39 max|W|.  Activations are split by their
// producers after a power-of-two a_scale that the host derives from a rigorous bound on |x|
// (the LayerNorm / attention / GELU bounds in classmate_hip/embeddings) with |x| a_scale <=
// 2^15; an activation below 2^-14 / a_scale contributes an absolute error < 2^-25 / a_scale.
// Both scales are exact powers of two, undone exactly in the epilogue (out_scale).
//
// Split-plane layout ("planes", HBM): a row-major M x K fp32 matrix becomes one buffer of 2 KiB
// split blocks [row / 16][k / 32] = [hi 1 KiB][lo 1 KiB]; each 1 KiB half is fragment-major:
// lane slot (c, g) = c + 16 g holds the 8 halves of row 16 b + c, k = 32 kb + 8 g .. + 7, which
// is exactly what lane c + 16 g feeds to v_mfma_f32_16x16x32_f16 as its A (row) or B (column)
// operand.  Weights W (N x K, nn.Linear layout) use the same order with N as the row index.
// Every operand load of the GEMM is one global_load_lds_dwordx4 wave-instruction per 1 KiB
// (8 full 128-B lines), read back with a conflict-free ds_read_b128 at lane*16; a k-step of a
// row block is one contiguous 2 KiB run.  Buffers hold f16x3_plane_rows(M) rows (a multiple of
// 384, every tile height): rows >= M hold whatever the producer left and only reach output rows
// >= M, which are never stored as fp32 (planes outputs carry them along as padding).
//
// Producers of planes: cm_f16x3_split_rows (any fp32 matrix), cm_add_layernorm_split (the
// XLM-R residual + LayerNorm, also writing the fp32 rows the next residual needs),
// cm_short_attention_split (query-batch attention) and this GEMM's own GELU epilogue
// (FFN-up -> FFN-down: the intermediate exists only as planes).
//
// GEMM (linear_f16x3_kernel): a persistent grid of one workgroup (4 waves, 2 x 2) per CU; each
// runs its output tiles' k-steps as one stream through an S-stage LDS ring (stage = the tile's
// BM/16 A split blocks then its BN/16 weight split blocks of one 32-wide k-step), all filled by
// LDS-DMA.  Per step: the first row tile's MFMAs, a counted vmcnt wait for the next stage + one
// raw s_barrier (publishes it, retires every read of this step's slot), then the remaining
// MFMAs with the next step's 18 fragment reads and this wave's DMA pieces of stage g + S
// threaded between them (sched_group_barrier).  No VGPR staging and no address arithmetic in
// the loop beyond one scalar add: per-piece offsets are fixed, per-tile bases change once per
// tile.  Tile order: XCD x takes a contiguous chunk of a grouped (8 row tiles per column
// sweep) order, so concurrently running tiles share A rows and weight columns in its L2.
#include "cm_common.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>

namespace cm {

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float g32x4 __attribute__((ext_vector_type(4)));
// fragments travel as 4 dwords (a loop-carried vector of halves gets split into 16-bit pieces and
// re-packed with v_perm at every loop back-edge); reinterpreted as 8 halves at the MFMA
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ h16x8 as_h8(i32x4 v) { return __builtin_bit_cast(h16x8, v); }

#ifndef K10_SMALL_S
#define K10_SMALL_S 6          // ring stages of the 64 x 32 tile (M <= 32): 6 vs 4 = 1.03 vs 1.08 ms batch-1 encode
#endif
#ifndef K10S_DEPTH
#define K10S_DEPTH 8           // k-steps in flight per wave of the skinny (M <= 32) kernel
#endif
#ifndef K10_S6
#define K10_S6 0              // ring stages of the 96 x 192 tile (0: 4 at 12 waves, 3 at 8; A/B knob)
#endif
#ifndef K10_W6
#define K10_W6 12              // waves per workgroup at the 96 x 192 tile (2 x 6: three per SIMD)
#endif

// Timing ablations for variant builds only (tools/build_k10_variant.sh; the product build has
// K10_ABL = 0): bit 0 no MFMA, bit 1 no DMA, bit 2 every DMA reads k-step 0 of the tile (an
// L2-resident source), bit 3 no epilogue stores.  Results are wrong in every ablated build.
#ifndef K10_ABL
#define K10_ABL 0
#endif


// Experiment knobs (variant builds, tools/build_k10_variant.sh; product values are the defaults):
// K10_SCHED 1 = spread the second half's fragment reads and DMA pieces evenly over its MFMAs for
// any counts (the default threads them only when they divide evenly); K10_PRIO 1 = s_setprio 1
// for the second half of the waves (the arbitration losers of a lockstep workgroup); K10_H1 > 0
// overrides the row tiles issued before the mid-step barrier.
#ifndef K10_SCHED
#define K10_SCHED 0
#endif
#ifndef K10_PRIO
#define K10_PRIO 0
#endif
#ifndef K10_H1
#define K10_H1 0
#endif
#ifndef K10_H1_6
#define K10_H1_6 0           // > 0: row tiles before the mid-step barrier of the 96-row tiles only (A/B knob)
#endif
#ifndef K10_SPREAD_ALL
#define K10_SPREAD_ALL 0     // 1: every tile whose counts do not divide gets the spread schedule (A/B knob)
#endif

// one MFMA slot of the spread schedule: the MFMA, then its share of reads and DMA pieces (EARLY:
// one read after each of the first NR MFMAs instead of an even spread)
template <int NM, int NR, int ND, bool EARLY, int M>
__device__ __forceinline__ void k10_slot() {
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  constexpr int r = EARLY ? (M < NR ? 1 : 0) : (M + 1) * NR / NM - M * NR / NM;
  if constexpr (r > 0) __builtin_amdgcn_sched_group_barrier(0x100, r, 0);
  constexpr int d = (M + 1) * ND / NM - M * ND / NM;
  if constexpr (d > 0) __builtin_amdgcn_sched_group_barrier(0x020, d, 0);
}
template <int NM, int NR, int ND, bool EARLY, int... I>
__device__ __forceinline__ void k10_spread(std::integer_sequence<int, I...>) {
  (k10_slot<NM, NR, ND, EARLY, I>(), ...);
}

// GELU(x) = x Phi(x) (torch's exact-erf F.gelu) in one branch-free form: Phi(x) = 1 - h for x >= 0, h
// for x < 0, h = erfc(u) / 2 = 2^P(u), u = |x| / sqrt 2, P a degree-9 least-squares fit of
// log2(erfc(u) / 2) on [0, 3.92] (beyond, erf rounds to +-1 in fp32 and h is 0, as in torch).  Against
// an fp64 GELU on a 700k-point grid over [-7, 7] (fp32 arithmetic, fma): max abs error 3.8e-7 and
// relative 3.2e-6 for |x| < 5.5, where 0.5 x (1 + erff(x / sqrt 2)) in fp32 has 4.5e-7 and, through
// its cancellation at negative x, 0.57 (tools/gelu_fit.py).  19 VALU operations instead of ~37 for
// ocml's two-branch erff + the product: the FFN-up epilogue applies it to 72 outputs per lane and tile.
#ifndef K10_GELU_OCML
#define K10_GELU_OCML 0   // 1: 0.5 x (1 + erff(x / sqrt 2)) (variant builds, A/B)
#endif
__device__ inline float gelu_erf(float x) {
  if (K10_GELU_OCML) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  const float u = fminf(fabsf(x) * 0.70710678118654752f, 3.92f);
  float p = 1.5919721363388817e-06f;
  p = fmaf(p, u, -2.9504877602448687e-05f);
  p = fmaf(p, u, 0.00020694537670351565f);
  p = fmaf(p, u, -0.0004535108746495098f);
  p = fmaf(p, u, -0.002977503463625908f);
  p = fmaf(p, u, 0.03079916536808014f);
  p = fmaf(p, u, -0.1500696986913681f);
  p = fmaf(p, u, -0.9179301261901855f);
  p = fmaf(p, u, -1.6279653310775757f);
  p = fmaf(p, u, -0.999998927116394f);
  const float h = u >= 3.92f ? 0.f : __builtin_amdgcn_exp2f(p);
  return x * (x >= 0.f ? 1.f - h : h);
}

// one 8-element segment: fp32 -> (hi, lo) f16 halves after the exact power-of-two scale
__device__ inline void split8(const float (&x)[8], float s, h16x8 &hi, h16x8 &lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    _Float16 h, l;
    f16x3_split1(x[e] * s, h, l);
    hi[e] = h;
    lo[e] = l;
  }
}

enum { kEpiF32 = 0, kEpiF32Gelu = 1, kEpiPlanesGelu = 2, kEpiPlanesQKV = 3 };

// Tile order of the persistent schedule: 8 row tiles per column sweep ("grouped").
__device__ __forceinline__ void k10_tile(int L, int tiles_m, int tiles_n, int &tm, int &tn) {
  const int per_group = 8 * tiles_n;
  const int first_m = (L / per_group) * 8;
  const int gsz = min(tiles_m - first_m, 8);
  const int rem = L % per_group;
  tm = first_m + rem % gsz;
  tn = rem / gsz;
}

// Epilogue of one tile for one wave, straight from the accumulators (no LDS: the ring keeps
// all of it).  fp32 rows: lane (g, c) stores rows 4 g + r of column c (16 consecutive floats per
// row and store).  Planes: lanes c and c ^ 1 swap half their halves (DPP quad_perm 1,0,3,2) so
// that each lane stores 4-byte column pairs (c even: rows 0-1, c odd: rows 2-3 of its group).
template <int BMB, int BNB, int NW, int EPI>
__device__ __forceinline__ void k10_epilogue(g32x4 (&acc)[BMB / 2][BNB / (NW / 2)], int tm, int tn, int wr, int wc,
                                             int lane, const float *btab, float out_scale, float next_scale,
                                             int64_t M, int N, float *__restrict__ Cout, _Float16 *__restrict__ Cp) {
  constexpr int WMT = BMB / 2, WNT = BNB / (NW / 2);
  const int g4 = lane >> 4, c16 = lane & 15;
  const int64_t rb0 = (int64_t)tm * BMB + wr * WMT;    // this wave's first row block
  const int cbase = (tn * BNB + wc * WNT) * 16;        // its first column
  const bool odd = c16 & 1;
#pragma unroll
  for (int j = 0; j < WNT; ++j) {
    const int col = cbase + 16 * j + c16;
    const float bv = btab[col];
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
      if constexpr (EPI == kEpiF32 || EPI == kEpiF32Gelu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = (rb0 + i) * 16 + 4 * g4 + r;
          float y = acc[i][j][r] * out_scale + bv;
          if (EPI == kEpiF32Gelu) y = gelu_erf(y);
          if (row < M) Cout[row * N + col] = y;
        }
      } else {
        float y[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          y[r] = acc[i][j][r] * out_scale + bv;
          if constexpr (EPI == kEpiPlanesGelu) y[r] = gelu_erf(y[r]);
          y[r] *= next_scale;
        }
        uint32_t h01, l01, h23, l23;                  // rows 0-1 / 2-3 as packed (low, high) halves
        f16x3_split2(y[0], y[1], h01, l01);
        f16x3_split2(y[2], y[3], h23, l23);
        // QKV: the V third (columns >= 2N/3, whole 16-column blocks) goes out transposed for the
        // P V operand of planes_attention_kernel: per 32-row unit u and 16-column block d, a 2 KiB
        // block [hi][lo] whose lane slot (c, g) holds rows 4 g .. + 3 (e 0-3) and 16 + 4 g .. + 3
        // (e 4-7) of column c -- the key order of the P fragment.  It occupies the 2 x (N/96)
        // split blocks of the standard layout's V region of those 32 rows (d / (N/96) picks the row
        // block, d % (N/96) the block within it), so the buffer keeps the standard size.
        if constexpr (EPI == kEpiPlanesQKV) {
          const int vcol0 = (N / 3) * 2, nkbv = N / 96;
          if (cbase + 16 * j >= vcol0) {
            const int64_t rb16 = rb0 + i;
            const int dblk = (col - vcol0) >> 4;
            const int64_t rb = 2 * (rb16 >> 1) + dblk / nkbv;
            const int kb = 2 * nkbv + dblk % nkbv;
            const int64_t off = ((rb * (N >> 5) + kb) * 128 + c16 + 16 * g4) * 8 + 4 * (rb16 & 1);
            *reinterpret_cast<uint2 *>(Cp + off) = make_uint2(h01, h23);
            *reinterpret_cast<uint2 *>(Cp + off + 512) = make_uint2(l01, l23);
            acc[i][j] = g32x4{0.f, 0.f, 0.f, 0.f};
            continue;
          }
        }
        // even lane keeps rows 0-1 and sends 2-3; odd lane keeps 2-3 and sends 0-1
        const uint32_t sh = odd ? h01 : h23, sl = odd ? l01 : l23;
        const uint32_t kh = odd ? h23 : h01, kl = odd ? l23 : l01;
        const uint32_t rh = (uint32_t)__builtin_amdgcn_mov_dpp((int)sh, 0xB1, 0xF, 0xF, false);
        const uint32_t rl = (uint32_t)__builtin_amdgcn_mov_dpp((int)sl, 0xB1, 0xF, 0xF, false);
        const int r0 = odd ? 2 : 0;
        const int c0 = col & ~1;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint32_t mine_h = (kh >> (16 * q)) & 0xffffu, mine_l = (kl >> (16 * q)) & 0xffffu;
          const uint32_t oth_h = (rh >> (16 * q)) & 0xffffu, oth_l = (rl >> (16 * q)) & 0xffffu;
          // column c0 (even) in the low half, c0 + 1 in the high half
          const uint32_t wh = odd ? (oth_h | mine_h << 16) : (mine_h | oth_h << 16);
          const uint32_t wl = odd ? (oth_l | mine_l << 16) : (mine_l | oth_l << 16);
          const int64_t off = f16x3_plane_off((rb0 + i) * 16 + 4 * g4 + r0 + q, c0, N >> 5);
          *reinterpret_cast<uint32_t *>(Cp + off) = wh;
          *reinterpret_cast<uint32_t *>(Cp + off + 512) = wl;
        }
      }
      acc[i][j] = g32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// BMB x BNB fragment blocks (16 x 16 outputs each) per tile, NW waves (2 x NW/2), S-stage ring.
template <int BMB, int BNB, int S, int NW, int EPI>
__global__ void __launch_bounds__(64 * NW)
    linear_f16x3_kernel(const _Float16 *__restrict__ Ap, int64_t M, int K, const _Float16 *__restrict__ Wp,
                        const float *__restrict__ bias, float out_scale, int N, float *__restrict__ Cout,
                        float next_scale, _Float16 *__restrict__ Cp) {
  constexpr int WGN = NW / 2;                         // waves: 2 rows x WGN columns
  constexpr int WMT = BMB / 2, WNT = BNB / WGN;       // 16x16 tiles per wave
  constexpr int NBLK = 2 * (BMB + BNB);               // 1 KiB blocks per stage
  constexpr int PCS = (NBLK + NW - 1) / NW;           // DMA pieces per wave per stage (uniform count:
                                                      // pieces past NBLK re-load block 0 into a pad)
  constexpr int STAGE = PCS * NW * 1024;
  constexpr int H1 = (BMB == 6 && K10_H1_6 > 0 && K10_H1_6 < WMT) ? K10_H1_6   // row tiles before the mid-step barrier
                     : (K10_H1 > 0 && K10_H1 < WMT) ? K10_H1 : WMT / 2;
  constexpr int NMF2 = 3 * (WMT - H1) * WNT;          // MFMAs after it
  constexpr int NRD = 2 * (WMT + WNT);                // fragment reads per step
  static_assert(BMB % 2 == 0 && BNB % WGN == 0, "tile must split over the waves");
  static_assert(S >= 3, "the ring needs one stage in use, one landing, one in flight");
  static_assert(H1 >= 1, "a row tile before the barrier");
  // threaded schedule of the second half: PCS groups of (NMF2 / PCS MFMAs, NRD / PCS reads, 1 DMA piece)
  constexpr bool THREAD = NMF2 % PCS == 0 && NRD % PCS == 0 && NMF2 / PCS >= NRD / PCS + 1;
  // the 96 x 288 tile's counts do not divide (18 MFMAs, 12 reads, 4 pieces): spread them evenly
  constexpr bool SPREAD = !THREAD && (BNB == 18 || K10_SPREAD_ALL);
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: piece choice and M0 stay scalar
  const int wr = wave / WGN, wc = wave % WGN;
  const int kb32 = K >> 5, nk = kb32;
  const int64_t rstride = (int64_t)kb32 * 2048;       // bytes per row block of a split buffer
  const int tiles_m = (int)((M + 16 * BMB - 1) / (16 * BMB)), tiles_n = N / (16 * BNB);
  const int n_tiles = tiles_m * tiles_n;
  float *btab = reinterpret_cast<float *>(lds + S * STAGE);                    // bias[N]

  // ---- tile schedule: XCD x (= blockIdx % 8 under round-robin dispatch) takes a contiguous
  //      chunk of the grouped tile order and its sx workgroups step through it together (a
  //      placement guess for L2 sharing only: any mapping is correct)
  const int w = blockIdx.x, nwg = gridDim.x, xcd = w & 7, slot = w >> 3;
  const int sx = nwg / 8 + (xcd < (nwg & 7));
  const int q8 = n_tiles / 8, r8 = n_tiles % 8;
  const int c0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int cn = q8 + (xcd < r8);
  const int my_n = slot < cn ? (cn - slot + sx - 1) / sx : 0;
  if (my_n == 0) return;                              // whole workgroup: no barrier is left waiting
  if (K10_PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  // bias of every column into LDS once (no global load may sit between the counted DMA waits)
  for (int i = tid; i < N; i += 64 * NW) btab[i] = bias ? bias[i] : 0.f;
  __syncthreads();

  // ---- DMA: piece i of this wave = stage block o = 4 i + wave; its source is a fixed offset
  //      (block's row within the tile, hi/lo half, lane) from the tile's A or W base + k-step
  uint32_t voff[PCS];
#pragma unroll
  for (int i = 0; i < PCS; ++i) {
    const int o = NW * i + wave;
    const int ob = o >= NBLK ? 0 : o < 2 * BMB ? o : o - 2 * BMB;
    voff[i] = (uint32_t)((ob >> 1) * rstride + (ob & 1) * 1024 + lane * 16);
  }
  const unsigned char *is_a, *is_w;                   // issue cursor: tile bases
  int is_kt = 0, is_ti = 0;
#define K10_TILE_BASES(ti)                                                                                 \
  do {                                                                                                     \
    int tm_, tn_;                                                                                          \
    k10_tile(c0 + (ti) * sx, tiles_m, tiles_n, tm_, tn_);                                                  \
    is_a = reinterpret_cast<const unsigned char *>(Ap) + (int64_t)tm_ * BMB * rstride;                     \
    is_w = reinterpret_cast<const unsigned char *>(Wp) + (int64_t)tn_ * BNB * rstride;                     \
  } while (0)
  K10_TILE_BASES(0);
#define K10_ISSUE(slotidx)                                                                                 \
  do {                                                                                                     \
    unsigned char *st_ = lds + (slotidx) * STAGE;                                                          \
    const int64_t ko_ = (K10_ABL & 4) ? 0 : (int64_t)is_kt * 2048;                                         \
    _Pragma("unroll") for (int i = 0; i < PCS; ++i) {                                                      \
      const unsigned char *src_ = (NW * i + wave < 2 * BMB || NW * i + wave >= NBLK ? is_a : is_w) + ko_ + voff[i]; \
      if (!(K10_ABL & 2))                                                                                  \
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src_,             \
                                         (__attribute__((address_space(3))) void *)(st_ + (NW * i + wave) * 1024), \
                                         16, 0, 0);                                                        \
    }                                                                                                      \
  } while (0)
#define K10_ADVANCE()                                                                                      \
  do {                                                                                                     \
    if (++is_kt == nk) {                                                                                   \
      if (is_ti + 1 < my_n) {                                                                              \
        is_kt = 0;                                                                                         \
        ++is_ti;                                                                                           \
        K10_TILE_BASES(is_ti);                                                                             \
      } else {                                                                                             \
        is_kt = nk - 1;                              /* clamped: the last stage repeats past the end */    \
      }                                                                                                    \
    }                                                                                                      \
  } while (0)

  i32x4 ah0[WMT], al0[WMT], bh0[WNT], bl0[WNT];
  i32x4 ah1[WMT], al1[WMT], bh1[WNT], bl1[WNT];
#define K10_READ(slotidx, AH, AL, BH, BL)                                                                    \
  do {                                                                                                       \
    const unsigned char *st_ = lds + (slotidx) * STAGE + lane * 16;                                          \
    _Pragma("unroll") for (int j = 0; j < WNT; ++j) {                                                        \
      BH[j] = *reinterpret_cast<const i32x4 *>(st_ + (2 * BMB + 2 * (wc * WNT + j)) * 1024);                 \
      BL[j] = *reinterpret_cast<const i32x4 *>(st_ + (2 * BMB + 2 * (wc * WNT + j) + 1) * 1024);             \
    }                                                                                                        \
    _Pragma("unroll") for (int i = 0; i < WMT; ++i) {                                                        \
      AH[i] = *reinterpret_cast<const i32x4 *>(st_ + (2 * (wr * WMT + i)) * 1024);                           \
      AL[i] = *reinterpret_cast<const i32x4 *>(st_ + (2 * (wr * WMT + i) + 1) * 1024);                       \
    }                                                                                                        \
  } while (0)

  g32x4 acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) acc[i][j] = g32x4{0.f, 0.f, 0.f, 0.f};
#define K10_MFMA(I0, I1, AH, AL, BH, BL)                                                       \
  if (!(K10_ABL & 1)) _Pragma("unroll") for (int i = (I0); i < (I1); ++i) _Pragma("unroll") for (int j = 0; j < WNT; ++j) { \
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(AL[i]), as_h8(BH[j]), acc[i][j], 0, 0, 0); \
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(AH[i]), as_h8(BL[j]), acc[i][j], 0, 0, 0); \
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(AH[i]), as_h8(BH[j]), acc[i][j], 0, 0, 0); \
  }

  // ---- the stream.  Prologue: stages 0 .. S-1 in flight, wait for stage 0, read its fragments.
  //      Step g (slot g % S): MFMAs of the first H1 row tiles; wait (counted: stages g+2 ..
  //      g+S-1 may stay in flight) + barrier: stage g+1 is published, every read of slot g % S
  //      is retired; then the rest of the MFMAs with the next step's fragment reads (slot
  //      (g+1) % S) and the DMA of stage g+S into slot g % S threaded between them.  Past the
  //      end the DMA repeats the last stage and the reads fetch unused data: every step runs
  //      the same uniform code.
#pragma unroll
  for (int p = 0; p < S; ++p) {
    K10_ISSUE(p);
    K10_ADVANCE();
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PCS * (S - 1)) : "memory");
  __builtin_amdgcn_s_barrier();
  K10_READ(0, ah0, al0, bh0, bl0);

#define K10_STEP(g, AH, AL, BH, BL, NAH, NAL, NBH, NBL)                                                      \
  do {                                                                                                       \
    const int cs_ = (g) % S, ns_ = ((g) + 1) % S;                                                            \
    K10_MFMA(0, H1, AH, AL, BH, BL)                                                                          \
    if constexpr (K10_SCHED >= 2) __builtin_amdgcn_sched_barrier(0);   /* part-1 MFMAs stay before the wait */ \
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(%0)" ::"n"(PCS * (S - 2)) : "memory");             \
    __builtin_amdgcn_s_barrier();                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                                       \
    K10_READ(ns_, NAH, NAL, NBH, NBL);                                                                       \
    K10_ISSUE(cs_);                                                                                          \
    K10_MFMA(H1, WMT, AH, AL, BH, BL)                                                                        \
    if constexpr (K10_SCHED == 1) {                                                                          \
      k10_spread<NMF2, NRD, PCS, false>(std::make_integer_sequence<int, NMF2>{});                            \
    } else if constexpr (K10_SCHED == 2) {   /* every read first: they have the whole half-step to land */  \
      __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);                                                   \
      k10_spread<NMF2, 0, PCS, false>(std::make_integer_sequence<int, NMF2>{});                              \
    } else if constexpr (K10_SCHED == 3) {                                                                   \
      k10_spread<NMF2, NRD, PCS, true>(std::make_integer_sequence<int, NMF2>{});                             \
    } else if constexpr (SPREAD) {                                                                           \
      k10_spread<NMF2, NRD, PCS, false>(std::make_integer_sequence<int, NMF2>{});                            \
    } else if constexpr (THREAD) {                                                                           \
      _Pragma("unroll") for (int q_ = 0; q_ < PCS; ++q_) {                                                   \
        _Pragma("unroll") for (int r_ = 0; r_ < NRD / PCS; ++r_) {                                           \
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                                 \
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                                 \
        }                                                                                                    \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                                   \
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                                   \
        __builtin_amdgcn_sched_group_barrier(0x008, NMF2 / PCS - NRD / PCS - 1, 0);                          \
      }                                                                                                      \
    }                                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                                       \
    K10_ADVANCE();                                                                                           \
  } while (0)

  for (int ti = 0; ti < my_n; ++ti) {
    for (int kt = 0; kt < nk; kt += 2) {              // nk is even (K % 64 == 0)
      const int g = ti * nk + kt;
      K10_STEP(g, ah0, al0, bh0, bl0, ah1, al1, bh1, bl1);
      K10_STEP(g + 1, ah1, al1, bh1, bl1, ah0, al0, bh0, bl0);
    }
    int tm, tn;
    k10_tile(c0 + ti * sx, tiles_m, tiles_n, tm, tn);
    if (!(K10_ABL & 8))
      k10_epilogue<BMB, BNB, NW, EPI>(acc, tm, tn, wr, wc, lane, btab, out_scale, next_scale, M, N, Cout, Cp);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail DMAs landed before the LDS is released
#undef K10_TILE_BASES
#undef K10_ISSUE
#undef K10_ADVANCE
#undef K10_READ
#undef K10_MFMA
#undef K10_STEP
}

// K10s: the skinny form for M <= 32 rows (one short query: a retrieve() call).  The GEMM is then a
// weight stream, and the tiled kernel's N / 32 workgroups (24 at N = 768) are too few to keep it
// in flight (FFN-down 21 us for 9.4 MB at batch 1, profiles/r05_e5_b1_kernels.txt).  Here one
// wave per 16 output columns (N / 16 workgroups of one wave, each on its own CU) streams its
// column block's split blocks -- one contiguous run of K / 32 x 2 KiB -- and the RB row blocks of A
// (L2-resident: every wave reads the same <= 2 x 2 KiB per k-step) straight into registers, D
// k-steps in flight.  Per k-step the same three MFMAs in the same order as linear_f16x3_kernel
// (lo.hi, hi.lo, hi.hi into the fp32 accumulator, k ascending), so every output bit equals the
// tiled kernel's: a query embeds the same alone or batched (tests/test_gpu_gemm.py).
template <int RB, int D, int EPI>
__global__ void __launch_bounds__(64)
    linear_f16x3_skinny_kernel(const _Float16 *__restrict__ Ap, int64_t M, int K, const _Float16 *__restrict__ Wp,
                               const float *__restrict__ bias, float out_scale, int N, float *__restrict__ Cout,
                               float next_scale, _Float16 *__restrict__ Cp) {
  const int lane = threadIdx.x, cb = blockIdx.x;
  const int nk = K >> 5;                               // k-steps (a multiple of D: checked by the launcher)
  const int64_t rstride = (int64_t)nk * 2048;          // bytes per row block of a split buffer
  const unsigned char *wp = reinterpret_cast<const unsigned char *>(Wp) + (int64_t)cb * rstride + lane * 16;
  const unsigned char *ap = reinterpret_cast<const unsigned char *>(Ap) + lane * 16;
  i32x4 wh[D], wl[D], ah[D][RB], al[D][RB];
#define K10S_LOAD(slot, step)                                                                       \
  do {                                                                                              \
    const int64_t o_ = (int64_t)(step) * 2048;                                                      \
    wh[slot] = *reinterpret_cast<const i32x4 *>(wp + o_);                                           \
    wl[slot] = *reinterpret_cast<const i32x4 *>(wp + o_ + 1024);                                    \
    _Pragma("unroll") for (int r = 0; r < RB; ++r) {                                                \
      ah[slot][r] = *reinterpret_cast<const i32x4 *>(ap + r * rstride + o_);                        \
      al[slot][r] = *reinterpret_cast<const i32x4 *>(ap + r * rstride + o_ + 1024);                 \
    }                                                                                               \
  } while (0)
#define K10S_MFMA(slot)                                                                                       \
  _Pragma("unroll") for (int r = 0; r < RB; ++r) {                                                            \
    acc[r][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(al[slot][r]), as_h8(wh[slot]), acc[r][0], 0, 0, 0); \
    acc[r][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(ah[slot][r]), as_h8(wl[slot]), acc[r][0], 0, 0, 0); \
    acc[r][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(ah[slot][r]), as_h8(wh[slot]), acc[r][0], 0, 0, 0); \
  }
  g32x4 acc[RB][1];
#pragma unroll
  for (int r = 0; r < RB; ++r) acc[r][0] = g32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int d = 0; d < D; ++d) K10S_LOAD(d, d);
  for (int s0 = 0; s0 + D < nk; s0 += D) {             // steady state: consume step s0 + d, refill its slot
#pragma unroll
    for (int d = 0; d < D; ++d) {
      K10S_MFMA(d)
      K10S_LOAD(d, s0 + D + d);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) K10S_MFMA(d)             // the last D steps
#undef K10S_LOAD
#undef K10S_MFMA
  k10_epilogue<2 * RB, 1, 2, EPI>(acc, 0, cb, 0, 0, lane, bias, out_scale, next_scale, M, N, Cout, Cp);
}

template <int RB, int D>
static int launch_skinny(const _Float16 *A, int64_t M, int K, const _Float16 *W, const float *bias, float out_scale,
                         int N, int epi, float *C, float next_scale, _Float16 *Cp, hipStream_t st) {
  const dim3 grid((unsigned)(N / 16)), block(64);
  switch (epi) {
    case kEpiF32:
      hipLaunchKernelGGL((linear_f16x3_skinny_kernel<RB, D, kEpiF32>), grid, block, 0, st, A, M, K, W, bias, out_scale,
                         N, C, next_scale, Cp);
      break;
    case kEpiF32Gelu:
      hipLaunchKernelGGL((linear_f16x3_skinny_kernel<RB, D, kEpiF32Gelu>), grid, block, 0, st, A, M, K, W, bias,
                         out_scale, N, C, next_scale, Cp);
      break;
    case kEpiPlanesGelu:
      hipLaunchKernelGGL((linear_f16x3_skinny_kernel<RB, D, kEpiPlanesGelu>), grid, block, 0, st, A, M, K, W, bias,
                         out_scale, N, C, next_scale, Cp);
      break;
    default: CM_FAIL(CM_EINVAL, "unknown epilogue");
  }
  CM_HIP(hipGetLastError());
  return CM_OK;
}

// fp32 rows [N][K] (weights or activations) -> split blocks of rows * scale
__global__ void split_rows_kernel(const float *__restrict__ W, int64_t N, int K, float scale, _Float16 *__restrict__ P) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one 8-element segment
  const int64_t nseg = N * (K / 8);
  if (t >= nseg) return;
  const int64_t n = t / (K / 8);
  const int k = (int)(t % (K / 8)) * 8;
  const float4 *p = reinterpret_cast<const float4 *>(W + n * K + k);
  const float4 u = p[0], v = p[1];
  const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
  h16x8 h, l;
  split8(x, scale, h, l);
  const int64_t off = f16x3_plane_off(n, k, K >> 5);
  *reinterpret_cast<h16x8 *>(P + off) = h;
  *reinterpret_cast<h16x8 *>(P + off + 512) = l;
}

struct TileCfg {
  int bmb, bnb;
};

// Pick the tile minimising (rounds of one-workgroup-per-CU waves) x (tile area + perimeter):
// the 96 x 192 tile divides M = 6144 (the 256 x 24 query batch) x N in {768, 2304, 3072} into
// exact multiples of 256 tiles; 128 x 128, 64 x 128 and 64 x 64 cover the other shapes.
static TileCfg pick_tile(int64_t M, int N, int n_cu) {
  // CM_K10_TILE=RxC (fragment blocks, e.g. 12x12) forces a tile for A/B timing
  static const TileCfg forced = [] {
    TileCfg f{0, 0};
    if (const char *e = getenv("CM_K10_TILE")) (void)sscanf(e, "%dx%d", &f.bmb, &f.bnb);
    return f;
  }();
  if (forced.bmb && N % (16 * forced.bnb) == 0) return forced;
  // FFN-up (N = 3072): 192 x 192 measured 98.3 -> 90.5 us at M = 6144 (tools/k10_tiles.sh); the
  // other E5 shapes are faster at 96 x 192 (qkv 67 vs 75 us, o 25 vs 34, down 73 vs 95)
  if (N >= 3072 && N % 192 == 0 && ceil_div(M, 192) * (N / 192) >= n_cu) return TileCfg{12, 12};
  // large batches (the passage encode, M = 65536 at the ingest shape): 192 x 192 for every projection
  // once each CU has >= 4 tiles -- qkv 696 -> 667, o + down 485 -> 475 us per call there, ingest
  // 6.96k -> 7.1k chunks/s (profiles/r05_k10_ingest_tile_ab.txt); the query batch (M = 6144) keeps
  // 96 x 192
  if (N % 192 == 0 && ceil_div(M, 192) * (N / 192) >= 4 * (int64_t)n_cu) return TileCfg{12, 12};
  // single short queries (M <= 32 rows, e.g. one retrieve() call): the GEMM is a weight stream spread
  // over N / (tile width) workgroups, so a 64 x 32 tile puts twice the CUs of 64 x 64 on it (the
  // per-element k order, hence every output bit, does not depend on the tile)
  if (M <= 32 && N % 32 == 0) return TileCfg{4, 2};
  // 96 x 288 (the query batch's QKV projection, N = 2304 at M = 6144: 512 tiles = two per CU instead
  // of three 96 x 192 ones; fewer fragment reads per MFMA and operand bytes per flop)
  static const bool t288 = [] {
    const char *e = getenv("CM_K10_T288");
    return !(e && e[0] == '0');
  }();
  const TileCfg cands[5] = {{6, 12}, {8, 8}, {4, 8}, {4, 4}, {6, 18}};
  TileCfg best = {0, 0};
  double best_cost = 0;
  for (const TileCfg &c : cands) {
    if (c.bnb == 18 && !t288) continue;
    if (N % (16 * c.bnb)) continue;
    const int64_t tiles = ceil_div(M, 16 * c.bmb) * (N / (16 * c.bnb));
    const double cost = (double)ceil_div(tiles, n_cu) * (c.bmb * c.bnb + 2 * (c.bmb + c.bnb));
    if (best.bmb == 0 || cost < best_cost) {
      best = c;
      best_cost = cost;
    }
  }
  return best;
}

template <int BMB, int BNB, int S, int NW>
static int launch_tile(const _Float16 *A, int64_t M, int K, const _Float16 *W, const float *bias, float out_scale,
                       int N, int epi, float *C, float next_scale, _Float16 *Cp, int n_cu, hipStream_t st) {
  const int64_t tiles = ceil_div(M, 16 * BMB) * (N / (16 * BNB));
  if (tiles > INT32_MAX / 2) CM_FAIL(CM_EINVAL, "too many tiles");
  const int lds_bytes = S * ((2 * (BMB + BNB) + NW - 1) / NW) * NW * 1024 + ((N * 4 + 15) & ~15);
  if (lds_bytes > 160 * 1024) CM_FAIL(CM_EINVAL, "N too large for the LDS bias table");
  const dim3 grid((unsigned)std::min<int64_t>(tiles, n_cu)), block(64 * NW);
  static int attr_set[4] = {0, 0, 0, 0};  // > 64 KiB of dynamic LDS: opt in once per kernel
  switch (epi) {
#define CM_K10_CASE(E)                                                                                             \
  case E:                                                                                                          \
    if (!attr_set[E]) {                                                                                            \
      CM_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&linear_f16x3_kernel<BMB, BNB, S, NW, E>),         \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));                         \
      attr_set[E] = 1;                                                                                             \
    }                                                                                                              \
    hipLaunchKernelGGL((linear_f16x3_kernel<BMB, BNB, S, NW, E>), grid, block, lds_bytes, st, A, M, K, W, bias,   \
                       out_scale, N, C, next_scale, Cp);                                                           \
    break;
    CM_K10_CASE(kEpiF32)
    CM_K10_CASE(kEpiF32Gelu)
    CM_K10_CASE(kEpiPlanesGelu)
    CM_K10_CASE(kEpiPlanesQKV)
#undef CM_K10_CASE
    default: CM_FAIL(CM_EINVAL, "unknown epilogue");
  }
  CM_HIP(hipGetLastError());
  return CM_OK;
}

static int g_n_cu = 0;

}  // namespace cm

using namespace cm;

extern "C" int64_t cm_f16x3_plane_rows(int64_t M) { return M <= 0 ? 0 : f16x3_plane_rows(M); }

extern "C" int cm_f16x3_split_rows(const float *x_dev, int64_t M, int32_t K, float scale, void *planes_dev,
                                   void *stream) {
  if (M <= 0) return CM_OK;
  if (!x_dev || !planes_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (K <= 0 || K % 32) CM_FAIL(CM_EINVAL, "K must be a positive multiple of 32");
  if (((uintptr_t)x_dev & 15) || ((uintptr_t)planes_dev & 15)) CM_FAIL(CM_EINVAL, "x and planes must be 16-byte aligned");
  const int64_t nseg = M * (K / 8);
  hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)ceil_div(nseg, 256)), dim3(256), 0, (hipStream_t)stream, x_dev,
                     M, K, scale, (_Float16 *)planes_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

extern "C" int cm_f16x3_split_weights(const float *w_dev, int32_t N, int32_t K, float scale, void *planes_dev,
                                      void *stream) {
  if (N <= 0 || K <= 0) return CM_OK;
  if (N % 16) CM_FAIL(CM_EINVAL, "need N % 16 == 0");
  return cm_f16x3_split_rows(w_dev, N, K, scale, planes_dev, stream);
}

extern "C" int cm_linear_f16x3(const void *a_planes, int64_t M, int32_t K, const void *w_planes, const float *bias_dev,
                               float out_scale, int32_t N, int32_t epilogue, float *c_dev, float next_scale,
                               void *c_planes, void *stream) {
  if (M <= 0) return CM_OK;
  if (!a_planes || !w_planes) CM_FAIL(CM_EINVAL, "NULL argument");
  if (K <= 0 || K % 64) CM_FAIL(CM_EINVAL, "K must be a positive multiple of 64");
  if (N <= 0 || N % 64) CM_FAIL(CM_EINVAL, "N must be a positive multiple of 64");
  const bool planes_out = epilogue == CM_EPI_PLANES_GELU || epilogue == CM_EPI_PLANES_QKV;
  if (planes_out ? !c_planes : !c_dev) CM_FAIL(CM_EINVAL, "NULL output");
  if (epilogue != CM_EPI_BIAS && epilogue != CM_EPI_BIAS_GELU && epilogue != CM_EPI_PLANES_GELU &&
      epilogue != CM_EPI_PLANES_QKV)
    CM_FAIL(CM_EINVAL, "unknown epilogue");
  // the QKV planes epilogue: three equal parts of whole 16-column blocks, 32-row units of V (the
  // tiled kernel: every tile height is a multiple of 32, and M > 32 keeps it off the skinny form)
  if (epilogue == CM_EPI_PLANES_QKV && (N % 96 || M <= 32)) CM_FAIL(CM_EINVAL, "QKV planes: need N % 96 == 0, M > 32");
  if (!g_n_cu) {
    int dev = 0, n = 0;
    CM_HIP(hipGetDevice(&dev));
    CM_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    g_n_cu = n > 0 ? n : 256;
  }
  const _Float16 *A = (const _Float16 *)a_planes, *W = (const _Float16 *)w_planes;
  _Float16 *Cp = (_Float16 *)c_planes;
  hipStream_t st = (hipStream_t)stream;
  // K10s for M <= 32 with a bias (every XLM-R projection has one); CM_K10_SKINNY=0 forces the tiled kernel
  static const bool skinny_on = [] {
    const char *e = getenv("CM_K10_SKINNY");
    return !(e && e[0] == '0');
  }();
  if (skinny_on && M <= 32 && bias_dev && (K / 32) % K10S_DEPTH == 0) {
    if (M <= 16)
      return launch_skinny<1, K10S_DEPTH>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, st);
    return launch_skinny<2, K10S_DEPTH>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, st);
  }
  const TileCfg t = pick_tile(M, N, g_n_cu);
  // waves per workgroup: two or three per SIMD, so one wave's MFMAs cover another's waits
  if (t.bmb == 12 && t.bnb == 12)  // 192 x 192: half the operand bytes per MFMA of 96 x 192 (L2 -> LDS bound)
    return launch_tile<12, 12, 3, 8>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, g_n_cu, st);
  if (t.bmb == 8 && t.bnb == 16)
    return launch_tile<8, 16, 3, 8>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, g_n_cu, st);
  if (t.bmb == 6 && t.bnb == 18)
    return launch_tile<6, 18, 3, 12>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, g_n_cu, st);
  if (t.bmb == 6)
    return launch_tile<6, 12, K10_S6 ? K10_S6 : (K10_W6 == 8 ? 3 : 4), K10_W6>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev,
                                                           next_scale, Cp, g_n_cu, st);
  if (t.bmb == 8)
    return launch_tile<8, 8, 4, 8>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, g_n_cu, st);
  if (t.bnb == 8)
    return launch_tile<4, 8, 4, 8>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, g_n_cu, st);
  if (t.bmb == 4 && t.bnb == 2)
    return launch_tile<4, 2, K10_SMALL_S, 4>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, g_n_cu, st);
  return launch_tile<4, 4, 4, 8>(A, M, K, W, bias_dev, out_scale, N, epilogue, c_dev, next_scale, Cp, g_n_cu, st);
}
