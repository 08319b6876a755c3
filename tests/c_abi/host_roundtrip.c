/* A plain-C caller of libgsync's C ABI (include/gsync.h), no Python, no torch:
 * host plans (GS_DEV_HOST) pack three ragged tensors with the fused 1/ws
 * scale, unpack them back, run one SGD step, compute Σg², and draw a
 * DistributedSampler index list.  Prints "ok" or the first failure.
 * Built and run by tests/test_c_abi.py. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gsync.h"

#define CHECK(x)                                                              \
  do {                                                                        \
    int rc_ = (x);                                                            \
    if (rc_ < 0) {                                                            \
      printf("FAIL %s -> %d: %s\n", #x, rc_, gs_last_error());                \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(void) {
  const int64_t numels[3] = {5, 1000, 3};
  float a[5], b[1000], c[3], ga[5], gb[1000], gc[3], ba[5], bb[1000], bc[3];
  for (int i = 0; i < 5; ++i) { a[i] = (float)i; ga[i] = 0.5f * i; ba[i] = 0.f; }
  for (int i = 0; i < 1000; ++i) { b[i] = 1.f / (i + 1); gb[i] = -0.25f; bb[i] = 0.f; }
  for (int i = 0; i < 3; ++i) { c[i] = -1.f; gc[i] = 2.f; bc[i] = 0.f; }
  gs_plan* plan = NULL;
  CHECK(gs_plan_create(GS_DEV_HOST, 0, 3, numels, 64, &plan));
  const int64_t flat_n = gs_plan_flat_numel(plan);
  float* flat = calloc((size_t)flat_n, sizeof(float));
  void* src[3] = {ga, gb, gc};
  CHECK(gs_plan_set_ptrs(plan, 1, src, NULL));
  CHECK(gs_pack(plan, 1, GS_F32, flat, GS_F32, 0.5f, GS_SCALE_MUL, NULL));
  int64_t offs[3];
  CHECK(gs_plan_offsets(plan, offs));
  if (flat[offs[1] + 7] != -0.125f || flat[offs[0] + 4] != 1.0f) { printf("FAIL pack values\n"); return 1; }
  float ua[5], ub[1000], uc[3];
  void* dst[3] = {ua, ub, uc};
  CHECK(gs_plan_set_ptrs(plan, 2, dst, NULL));
  float sq = 0.f;
  CHECK(gs_unpack(plan, flat, GS_F32, 2, GS_F32, &sq, 0, NULL));
  for (int i = 0; i < 5; ++i) if (ua[i] != 0.25f * i) { printf("FAIL unpack\n"); return 1; }
  /* Σ (g/2)² = Σ ga²/4 + 1000·(1/8)² + 3·1² */
  double want = 0.0;
  for (int i = 0; i < 5; ++i) want += (0.25 * i) * (0.25 * i);
  want += 1000 * 0.125 * 0.125 + 3.0;
  if (fabs(sq - want) > 1e-4 * want) { printf("FAIL sqnorm %f vs %f\n", sq, want); return 1; }
  /* one SGD step, momentum 0.9, wd 0, lr 0.1, first step: p -= 0.1 * g */
  void* ps[3] = {a, b, c};
  void* bufs[3] = {ba, bb, bc};
  CHECK(gs_plan_set_ptrs(plan, 0, ps, NULL));
  CHECK(gs_plan_set_ptrs(plan, 1, src, NULL));
  CHECK(gs_plan_set_ptrs(plan, 2, bufs, NULL));
  CHECK(gs_sgd_step(plan, GS_F32, -1, 0.1, 0.9, 0.0, 0.0, 0, 0, 1, NULL, NULL, NULL));
  if (fabsf(c[1] - (-1.2f)) > 1e-6f || bc[2] != 2.f) { printf("FAIL sgd %f %f\n", c[1], bc[2]); return 1; }
  /* DistributedSampler(n=10, ws=3, rank=1, shuffle=False): [1, 4, 7, 0] (padded) */
  int64_t idx[8], cnt = 0;
  CHECK(gs_distributed_sampler_indices(10, 3, 1, 0, 0, 0, 0, idx, 8, &cnt));
  if (cnt != 4 || idx[0] != 1 || idx[1] != 4 || idx[2] != 7 || idx[3] != 0) { printf("FAIL sampler\n"); return 1; }
  /* errors come back as codes + message, never as a crash */
  if (gs_plan_create(GS_DEV_HOST, 0, 1, numels, 3, &plan) != GS_EINVAL) { printf("FAIL error path\n"); return 1; }
  CHECK(gs_plan_destroy(plan));
  free(flat);
  printf("ok gsync %d\n", gs_version());
  return 0;
}
