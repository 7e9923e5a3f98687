/* ASan/UBSan driver for libclassmate_hip's host side (tools/asan_check.sh builds the library's host
 * halves with -fsanitize=address,undefined and links this program against them).  No GPU in the
 * build container: it exercises every entry point's argument validation and error reporting
 * (cm_last_error's thread-local string), the host-only helpers, and the device-less paths of the
 * constructors -- the code that runs before any kernel.  Exit 0 = every call returned the
 * expected code; ASan aborts on any memory error. */
#include <stdio.h>
#include <string.h>

#include "classmate_hip.h"

static int fails = 0;
#define EXPECT(call, want)                                                                     \
  do {                                                                                         \
    int rc_ = (int)(call);                                                                     \
    const char *m_ = cm_last_error();                                                          \
    if (rc_ != (want)) {                                                                       \
      fprintf(stderr, "%s: got %d want %d (%s)\n", #call, rc_, (want), m_ ? m_ : "");         \
      ++fails;                                                                                 \
    }                                                                                          \
    if (m_ && strlen(m_) > 4096) ++fails;                                                      \
  } while (0)

int main(void) {
  if (cm_version() <= 0) ++fails;
  if (cm_max_topk() < 10) ++fails;
  EXPECT(cm_device_count(NULL), CM_EINVAL);
  int n = -1;
  (void)cm_device_count(&n); /* no GPU here: an error or 0, never a crash */
  EXPECT(cm_stream_create_cu_masked(0, NULL, 0, NULL), CM_EINVAL);
  EXPECT(cm_stream_destroy(NULL), CM_OK);
  /* dense */
  cm_dense *dh = NULL;
  EXPECT(cm_dense_create(0, 0, 0, &dh), CM_EINVAL);
  EXPECT(cm_dense_create(0, 4096, 0, &dh), CM_EINVAL);
  EXPECT(cm_dense_create(0, 768, -1, &dh), CM_EINVAL);
  EXPECT(cm_dense_create(0, 768, 0, NULL), CM_EINVAL);
  /* bm25 */
  EXPECT(cm_bm25_create(0, NULL), CM_EINVAL);
  /* fusion (host arrays) */
  int32_t on = 7;
  EXPECT(cm_rrf_fuse(NULL, NULL, 2, NULL, 60, NULL, NULL, &on), CM_EINVAL);
  int32_t off0[3] = {0, 0, 0};
  (void)cm_rrf_fuse(NULL, off0, 2, NULL, 60, NULL, NULL, &on); /* reaches the device: an error here */
  if (on != 0) ++fails;
  int32_t offbad[3] = {0, 2, 1};
  EXPECT(cm_rrf_fuse(NULL, offbad, 2, NULL, 60, NULL, NULL, &on), CM_EINVAL);
  /* encoder / pooling / K10: validation happens before any device call */
  EXPECT(cm_meanpool_l2norm(NULL, CM_DTYPE_F32, NULL, CM_DTYPE_I32, 2, 3, 4, 1, NULL, NULL), CM_EINVAL);
  EXPECT(cm_add_layernorm(NULL, NULL, 0, NULL, NULL, 0, 768, 1e-5f, CM_DTYPE_F32, NULL, NULL), CM_OK);
  EXPECT(cm_add_layernorm(NULL, NULL, 0, NULL, NULL, 4, 768, 1e-5f, CM_DTYPE_F32, NULL, NULL), CM_EINVAL);
  EXPECT(cm_short_attention(NULL, 1, 8, 12, 64, 0.125f, CM_DTYPE_F32, NULL, NULL), CM_EINVAL);
  float dummy[64];
  EXPECT(cm_short_attention(dummy, 1, 8, 12, 32, 0.125f, CM_DTYPE_F32, dummy, NULL), CM_EINVAL);
  EXPECT(cm_short_attention(dummy, 1, 65, 12, 64, 0.125f, CM_DTYPE_F32, dummy, NULL), CM_EINVAL);
  if (cm_f16x3_plane_rows(0) != 0 || cm_f16x3_plane_rows(1) != 384 || cm_f16x3_plane_rows(385) != 768) ++fails;
  EXPECT(cm_f16x3_split_rows(NULL, 4, 768, 1.f, NULL, NULL), CM_EINVAL);
  EXPECT(cm_f16x3_split_rows(dummy, 4, 100, 1.f, dummy, NULL), CM_EINVAL);
  EXPECT(cm_f16x3_split_weights(dummy, 15, 64, 1.f, dummy, NULL), CM_EINVAL);
  EXPECT(cm_linear_f16x3(NULL, 8, 768, NULL, NULL, 1.f, 768, CM_EPI_BIAS, NULL, 0.f, NULL, NULL), CM_EINVAL);
  EXPECT(cm_linear_f16x3(dummy, 8, 96, dummy, NULL, 1.f, 768, CM_EPI_BIAS, dummy, 0.f, NULL, NULL), CM_EINVAL);
  EXPECT(cm_linear_f16x3(dummy, 8, 768, dummy, NULL, 1.f, 100, CM_EPI_BIAS, dummy, 0.f, NULL, NULL), CM_EINVAL);
  EXPECT(cm_linear_f16x3(dummy, 8, 768, dummy, NULL, 1.f, 768, CM_EPI_PLANES_GELU, dummy, 0.f, NULL, NULL), CM_EINVAL);
  EXPECT(cm_linear_f16x3(dummy, 8, 768, dummy, NULL, 1.f, 768, 9, dummy, 0.f, NULL, NULL), CM_EINVAL);
  EXPECT(cm_add_layernorm_split(NULL, NULL, 0, NULL, NULL, 4, 768, 1e-5f, NULL, 1.f, NULL, NULL), CM_EINVAL);
  EXPECT(cm_short_attention_split(NULL, 1, 8, 12, 64, 0.125f, 1.f, NULL, NULL), CM_EINVAL);
  /* filters */
  EXPECT(cm_filter_eval(NULL, 0, NULL, 0, NULL, 0, 10, NULL, NULL, NULL), CM_EINVAL);
  if (fails) {
    fprintf(stderr, "%d unexpected results\n", fails);
    return 1;
  }
  printf("host ABI validation paths: OK\n");
  return 0;
}
