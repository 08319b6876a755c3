/* A plain-C caller of libgsync's C ABI (include/gsync.h), no Python, no torch:
 * host plans (GS_DEV_HOST) pack three ragged tensors with the fused 1/ws
 * scale, unpack them back, run one SGD step, compute Σg², run a clipped step
 * on sharded group sums (the ZeRO world > 1 form: gs_sqnorm_partial_out +
 * gs_plan_set_clip_groups, two "ranks" summed by hand), and draw a
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
  /* sharded clip: each "rank" leaves its shard's Σg² as group sums, the sums are
   * added element-wise (the all-reduce), every rank's update folds them */
  {
    const int64_t shard_n[1] = {4};
    float g0[4] = {3.f, 0.f, 0.f, 0.f}, g1[4] = {0.f, 4.f, 0.f, 0.f};  /* ‖g‖ = 5 over both shards */
    float p0[4] = {0.f, 0.f, 0.f, 0.f}, m0[4] = {0.f, 0.f, 0.f, 0.f};
    gs_plan *s0 = NULL, *s1 = NULL;
    CHECK(gs_plan_create(GS_DEV_HOST, 0, 1, shard_n, 0, &s0));
    CHECK(gs_plan_create(GS_DEV_HOST, 0, 1, shard_n, 0, &s1));
    void* gp0[1] = {g0};
    void* gp1[1] = {g1};
    CHECK(gs_plan_set_ptrs(s0, 1, gp0, NULL));
    CHECK(gs_plan_set_ptrs(s1, 1, gp1, NULL));
    float grp0[GS_RED_PARTIALS], grp1[GS_RED_PARTIALS];  /* the buffer the call requires */
    int32_t n0 = 0, n1 = 0;
    CHECK(gs_sqnorm_partial_out(s0, 1, GS_F32, grp0, &n0, NULL));
    CHECK(gs_sqnorm_partial_out(s1, 1, GS_F32, grp1, &n1, NULL));
    if (n0 != n1 || n0 < 1) { printf("FAIL group counts %d %d\n", n0, n1); return 1; }
    for (int k = 0; k < n0; ++k) grp0[k] += grp1[k];
    void* pp[1] = {p0};
    void* mp[1] = {m0};
    CHECK(gs_plan_set_ptrs(s0, 0, pp, NULL));
    CHECK(gs_plan_set_ptrs(s0, 2, mp, NULL));
    float out[3];
    CHECK(gs_plan_set_clip_groups(s0, grp0, n0, 1.f, 1e-6f, 1.f, 1.f, out));
    CHECK(gs_sgd_step(s0, GS_F32, -1, 1.0, 0.0, 0.0, 0.0, 0, 0, 1, NULL, NULL, NULL));
    /* Σg² = 25, coef = 1/(5 + 1e-6): p = -3·coef on the first element */
    if (out[0] != 25.f || fabsf(out[2] - 5.f) > 1e-6f || fabsf(p0[0] + 3.f / 5.f) > 1e-6f) {
      printf("FAIL clip groups %f %f %f\n", out[0], out[2], p0[0]);
      return 1;
    }
    if (gs_plan_set_clip_groups(s0, grp0, GS_RED_PARTIALS + 1, 1.f, 1e-6f, 1.f, 1.f, out) != GS_EINVAL) {
      printf("FAIL clip groups range\n");
      return 1;
    }
    CHECK(gs_plan_destroy(s0));
    CHECK(gs_plan_destroy(s1));
  }
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
