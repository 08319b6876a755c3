/* A plain-C caller of libgsync's C ABI on the GPU, no Python, no torch — the
 * Reducer replacement as a non-Python host would bind it:
 *   gs_comm_get_unique_id / gs_comm_create (RCCL, world 1)
 *   gs_compute_bucket_assignment (torch's greedy caps, gradient-ready order)
 *   gs_bucketer_create + per-bucket buffers, prepare, mark_ready per grad on a
 *   HIP stream (pack x 1/div_factor -> RCCL all-reduce -> unpack + fused Σg²),
 *   finalize
 *   gs_plan_create + gs_sgd_step (two steps, momentum + weight decay)
 * checked against the oracle (oracle/gs_oracle.c, linked as the checker):
 * averaged grads == g * float(1/div) bit for bit (world 1: the collective is
 * the identity), Σg² within 1e-5 relative of the fp64 sum, weights and
 * momentum buffers == or_sgd bit for bit.  Prints "ok" or the first failure.
 * Built and run by tests/test_gpu_c_abi.py. */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gsync.h"

/* the checker (oracle/gs_oracle.c) */
void or_sgd(int64_t n, float* p, const void* g, int gdt, float* buf, double lr, double mom, double damp,
            double wd, int nesterov, int maximize, int first, const float* gscale, void* lowp, int ldt);
double or_sqnorm(int n, const void* const* xs, const int64_t* numels, int dt);

#define CHECK(x)                                                              \
  do {                                                                        \
    int rc_ = (x);                                                            \
    if (rc_ < 0) {                                                            \
      printf("FAIL %s -> %d: %s\n", #x, rc_, gs_last_error());                \
      return 1;                                                               \
    }                                                                         \
  } while (0)
#define HIPCHECK(x)                                                           \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("FAIL %s -> %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                               \
    }                                                                         \
  } while (0)

enum { NP = 6 };

static uint32_t lcg = 12345u;
static float rnd(void) {
  lcg = lcg * 1664525u + 1013904223u;
  return ((float)(lcg >> 8) / 16777216.f - 0.5f) * 0.02f;
}

int main(void) {
  /* ragged sizes: tails, a tiny tensor, one > 1 Mi elements */
  const int64_t numels[NP] = {5, 3000, 1, 70001, 1 << 20, 257};
  float* hg[NP];
  float* hp[NP];
  float* hb[NP];
  void* dg[NP];
  void* dp[NP];
  void* db[NP];
  HIPCHECK(hipSetDevice(0));
  hipStream_t s;
  HIPCHECK(hipStreamCreate(&s));
  for (int i = 0; i < NP; ++i) {
    const size_t nb = (size_t)numels[i] * sizeof(float);
    hg[i] = malloc(nb);
    hp[i] = malloc(nb);
    hb[i] = malloc(nb);
    for (int64_t k = 0; k < numels[i]; ++k) {
      hg[i][k] = rnd();
      hp[i][k] = 50.f * rnd();
      hb[i][k] = 0.f;
    }
    HIPCHECK(hipMalloc(&dg[i], nb));
    HIPCHECK(hipMalloc(&dp[i], nb));
    HIPCHECK(hipMalloc(&db[i], nb));
    HIPCHECK(hipMemcpy(dp[i], hp[i], nb, hipMemcpyHostToDevice));
    HIPCHECK(hipMemset(db[i], 0, nb));
  }

  /* buckets in gradient-ready order (last layer first), torch's caps 1 MiB / 25 MiB */
  int64_t nbytes[NP];
  int32_t keys[NP], order[NP], bucket_of[NP], members[NP], counts[NP];
  for (int i = 0; i < NP; ++i) {
    nbytes[i] = numels[i] * 4;
    keys[i] = 0;
    order[i] = NP - 1 - i;
  }
  const int64_t limits[2] = {1 << 20, 25 << 20};
  const int nb_ = gs_compute_bucket_assignment(NP, nbytes, keys, order, 2, limits, bucket_of, members, counts);
  CHECK(nb_);
  if (nb_ < 2) {
    printf("FAIL expected >= 2 buckets, got %d\n", nb_);
    return 1;
  }

  uint8_t uid[128];
  if (gs_comm_unique_id_bytes() > (int)sizeof uid) {
    printf("FAIL unique id size\n");
    return 1;
  }
  CHECK(gs_comm_get_unique_id(uid));
  gs_comm* comm = NULL;
  CHECK(gs_comm_create(0, 1, uid, 0, &comm));
  const float div = 4.f; /* a world of 4's prescale: grads arrive as g * float(1/4) */
  gs_bucketer* bk = NULL;
  CHECK(gs_bucketer_create(comm, GS_DEV_HIP, 0, NP, numels, GS_F32, nb_, counts, members, GS_F32, 64, div,
                           GS_BKT_AUTO_COLLECTIVE, &bk));
  void* bufs[NP];
  for (int b = 0; b < nb_; ++b) {
    int64_t n = 0;
    CHECK(gs_bucketer_bucket_numel(bk, b, &n));
    HIPCHECK(hipMalloc(&bufs[b], (size_t)n * 4));
    CHECK(gs_bucketer_set_bucket_buffer(bk, b, bufs[b]));
  }
  float* dsq = NULL;
  HIPCHECK(hipMalloc((void**)&dsq, 4));

  gs_plan* plan = NULL;
  CHECK(gs_plan_create(GS_DEV_HIP, 0, NP, numels, 4, &plan));
  CHECK(gs_plan_set_ptrs(plan, 0, dp, s));
  CHECK(gs_plan_set_ptrs(plan, 1, dg, s));
  CHECK(gs_plan_set_ptrs(plan, 2, db, s));

  for (int step = 0; step < 2; ++step) {
    for (int i = 0; i < NP; ++i) {
      for (int64_t k = 0; k < numels[i]; ++k) hg[i][k] = rnd();
      HIPCHECK(hipMemcpy(dg[i], hg[i], (size_t)numels[i] * 4, hipMemcpyHostToDevice));
    }
    CHECK(gs_bucketer_prepare(bk, dsq));
    for (int r = 0; r < NP; ++r) { /* autograd hooks, in ready order */
      int32_t ready[NP], n_ready = 0;
      CHECK(gs_bucketer_mark_ready(bk, order[r], dg[order[r]], s, ready, &n_ready));
    }
    CHECK(gs_bucketer_finalize(bk, s));
    CHECK(gs_sgd_step(plan, GS_F32, -1, 0.1, 0.9, 0.0, 1e-4, 0, 0, step == 0, NULL, NULL, s));
    HIPCHECK(hipStreamSynchronize(s));

    /* averaged grads: g * float(1/div), bit for bit */
    const float inv = 1.f / div;
    const void* avg[NP];
    float* hav[NP];
    for (int i = 0; i < NP; ++i) {
      hav[i] = malloc((size_t)numels[i] * 4);
      HIPCHECK(hipMemcpy(hav[i], dg[i], (size_t)numels[i] * 4, hipMemcpyDeviceToHost));
      for (int64_t k = 0; k < numels[i]; ++k) {
        const float want = hg[i][k] * inv;
        if (memcmp(&want, &hav[i][k], 4) != 0) {
          printf("FAIL step %d grad %d[%lld]: %.9g vs %.9g\n", step, i, (long long)k, hav[i][k], want);
          return 1;
        }
      }
      avg[i] = hav[i];
    }
    float sq = 0.f;
    HIPCHECK(hipMemcpy(&sq, dsq, 4, hipMemcpyDeviceToHost));
    const double want_sq = or_sqnorm(NP, avg, numels, GS_F32);
    if (fabs(sq - want_sq) > 1e-5 * want_sq) {
      printf("FAIL step %d sqnorm %.9g vs %.9g\n", step, sq, want_sq);
      return 1;
    }
    /* the oracle's SGD on the same averaged grads */
    for (int i = 0; i < NP; ++i) {
      or_sgd(numels[i], hp[i], hav[i], GS_F32, hb[i], 0.1, 0.9, 0.0, 1e-4, 0, 0, step == 0, NULL, NULL, 0);
      float* got = malloc((size_t)numels[i] * 4);
      HIPCHECK(hipMemcpy(got, dp[i], (size_t)numels[i] * 4, hipMemcpyDeviceToHost));
      if (memcmp(got, hp[i], (size_t)numels[i] * 4) != 0) {
        printf("FAIL step %d weights %d\n", step, i);
        return 1;
      }
      HIPCHECK(hipMemcpy(got, db[i], (size_t)numels[i] * 4, hipMemcpyDeviceToHost));
      if (memcmp(got, hb[i], (size_t)numels[i] * 4) != 0) {
        printf("FAIL step %d momentum %d\n", step, i);
        return 1;
      }
      free(got);
      free(hav[i]);
    }
  }
  CHECK(gs_plan_destroy(plan));
  CHECK(gs_bucketer_destroy(bk));
  CHECK(gs_comm_destroy(comm));
  for (int b = 0; b < nb_; ++b) HIPCHECK(hipFree(bufs[b]));
  for (int i = 0; i < NP; ++i) {
    HIPCHECK(hipFree(dg[i]));
    HIPCHECK(hipFree(dp[i]));
    HIPCHECK(hipFree(db[i]));
    free(hg[i]);
    free(hp[i]);
    free(hb[i]);
  }
  HIPCHECK(hipFree(dsq));
  HIPCHECK(hipStreamDestroy(s));
  printf("ok %d buckets\n", nb_);
  return 0;
}
