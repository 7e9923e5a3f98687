// Metadata where-filters evaluated on the device.
//
// The host compiles a where clause -- Chroma semantics (rag/retrieval/vector_chroma.py:45-78 via
// Chroma's $and/$or/$eq/$ne/$in/$nin) or the BM25 store's _matches_filter (rag/retrieval/
// bm25.py:79-107, quirk Q4) -- into a postfix program over row-aligned int32 value-code columns
// (one code per distinct metadata value, classmate_hip/retrieval/filters.py) and precomputed
// row bitmaps (live rows, tag sets, range predicates).  One lane evaluates one row with its
// operand stack in a 32-bit register (top = bit 0); a wave ballot packs 64 row results into two
// words of the allow bitmap the scan kernels read.  HBM-bound: 4 B per referenced column and
// 1/8 B per referenced bitmap per row, plus 1/8 B written.
#include "cm_common.h"

namespace cm {

constexpr int kFilterMaxOps = CM_FILTER_MAX_OPS;
constexpr int kFilterMaxSrc = CM_FILTER_MAX_SOURCES;

struct FilterProg {
  int32_t op[kFilterMaxOps];
  int32_t a[kFilterMaxOps];
  int32_t b[kFilterMaxOps];
  const int32_t *cols[kFilterMaxSrc];
  const uint32_t *bits[kFilterMaxSrc];
  int32_t n_ops;
};

__global__ void __launch_bounds__(256) filter_eval_kernel(const FilterProg p, int64_t n_rows, uint32_t *__restrict__ out,
                                                          unsigned long long *__restrict__ count) {
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool in = row < n_rows;
  uint32_t st = 0;  // operand stack, top at bit 0
  for (int i = 0; i < p.n_ops; ++i) {  // the program is kernel-argument (scalar) data: uniform branches
    const int op = p.op[i];
    if (op == CM_FOP_EQ || op == CM_FOP_NE) {
      const uint32_t v = in ? (uint32_t)(p.cols[p.a[i]][row] == p.b[i]) : 0u;
      st = (st << 1) | (op == CM_FOP_EQ ? v : v ^ 1u);
    } else if (op == CM_FOP_BITS) {
      const uint32_t v = in ? (p.bits[p.a[i]][row >> 5] >> (row & 31)) & 1u : 0u;
      st = (st << 1) | v;
    } else if (op == CM_FOP_TRUE || op == CM_FOP_FALSE) {
      st = (st << 1) | (op == CM_FOP_TRUE ? 1u : 0u);
    } else if (op == CM_FOP_AND) {
      st = ((st >> 2) << 1) | (st & (st >> 1) & 1u);
    } else if (op == CM_FOP_OR) {
      st = ((st >> 2) << 1) | ((st | (st >> 1)) & 1u);
    } else {  // CM_FOP_NOT
      st ^= 1u;
    }
  }
  const uint64_t m = __ballot(in && (st & 1u));
  const int lane = threadIdx.x & 63;
  const int64_t w = row >> 5;  // lanes 0 and 32 own the wave's two words
  if ((lane & 31) == 0 && in) out[w] = (uint32_t)(lane ? (m >> 32) : m);
  if (count && lane == 0 && m) atomicAdd(count, (unsigned long long)__popcll(m));
}

}  // namespace cm

using namespace cm;

extern "C" int cm_filter_eval(const int32_t *prog, int32_t n_ops, const int32_t *const *cols_dev, int32_t n_cols,
                              const uint32_t *const *bits_dev, int32_t n_bits, int64_t n_rows, uint32_t *out_dev,
                              unsigned long long *count_dev, void *stream) {
  if (n_rows < 0) CM_FAIL(CM_EINVAL, "cm_filter_eval: n_rows < 0");
  if (n_ops < 1 || n_ops > kFilterMaxOps || !prog) CM_FAIL(CM_EINVAL, "cm_filter_eval: program length out of range");
  if (n_cols < 0 || n_cols > kFilterMaxSrc || n_bits < 0 || n_bits > kFilterMaxSrc)
    CM_FAIL(CM_EINVAL, "cm_filter_eval: too many columns or bitmaps");
  if (!out_dev) CM_FAIL(CM_EINVAL, "cm_filter_eval: out_dev is NULL");
  FilterProg p{};
  p.n_ops = n_ops;
  int depth = 0;
  for (int i = 0; i < n_ops; ++i) {
    const int op = prog[3 * i], a = prog[3 * i + 1];
    p.op[i] = op;
    p.a[i] = a;
    p.b[i] = prog[3 * i + 2];
    switch (op) {
      case CM_FOP_EQ:
      case CM_FOP_NE:
        if (a < 0 || a >= n_cols || !cols_dev[a]) CM_FAIL(CM_EINVAL, "cm_filter_eval: bad column operand");
        ++depth;
        break;
      case CM_FOP_BITS:
        if (a < 0 || a >= n_bits || !bits_dev[a]) CM_FAIL(CM_EINVAL, "cm_filter_eval: bad bitmap operand");
        ++depth;
        break;
      case CM_FOP_TRUE:
      case CM_FOP_FALSE:
        ++depth;
        break;
      case CM_FOP_AND:
      case CM_FOP_OR:
        if (depth < 2) CM_FAIL(CM_EINVAL, "cm_filter_eval: stack underflow");
        --depth;
        break;
      case CM_FOP_NOT:
        if (depth < 1) CM_FAIL(CM_EINVAL, "cm_filter_eval: stack underflow");
        break;
      default:
        CM_FAIL(CM_EINVAL, "cm_filter_eval: unknown opcode");
    }
    if (depth > 32) CM_FAIL(CM_EINVAL, "cm_filter_eval: stack deeper than 32");
  }
  if (depth != 1) CM_FAIL(CM_EINVAL, "cm_filter_eval: program must leave exactly one value");
  for (int i = 0; i < n_cols; ++i) p.cols[i] = cols_dev[i];
  for (int i = 0; i < n_bits; ++i) p.bits[i] = bits_dev[i];
  hipStream_t st = (hipStream_t)stream;
  if (count_dev) CM_HIP(hipMemsetAsync(count_dev, 0, sizeof(unsigned long long), st));
  if (n_rows == 0) return CM_OK;
  hipLaunchKernelGGL(filter_eval_kernel, dim3((unsigned)ceil_div(n_rows, 256)), dim3(256), 0, st, p, n_rows, out_dev,
                     count_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}
