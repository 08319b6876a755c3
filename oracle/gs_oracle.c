/*
 * gs_oracle.c — CPU restatement of the reference's gradient-synchronisation
 * arithmetic.  TEST INFRASTRUCTURE ONLY: it is the checker that libgsync's HIP
 * kernels and host backend are compared against; no product code links it.
 *
 * The reference (R: = /root/reference) is Python; its hot path is torch's
 * DDP Reducer + ATen foreach optimizers (T: = torch 2.10 under
 * /usr/local/lib/python3.10/dist-packages/torch).  Each function cites the
 * torch code it restates.  The oracle is pinned by tests/golden/ fixtures
 * produced by running the reference's own train step
 * (R:resnet/pytorch_ddp/ddp_train.py:52-75) under torch DDP + gloo.
 *
 * Plain C99, built with `gcc -O2 -ffp-contract=off` so no multiply-add is
 * fused unless written as fmaf().
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define OR_F32 0
#define OR_BF16 1
#define OR_F16 2

/* ---- bf16: c10::BFloat16 round_to_nearest_even (c10/util/BFloat16.h) ---- */
float or_bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint16_t or_f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7FC0;
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

/* ---- fp16: IEEE binary16 round-to-nearest-even (c10::Half fp16_ieee_from_fp32_value) ---- */
float or_f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1fu, man = h & 0x3ffu, u;
  if (exp == 0) {
    if (man == 0) {
      u = sign;
    } else { /* subnormal */
      exp = 127 - 15 + 1;
      while (!(man & 0x400u)) { man <<= 1; exp--; }
      man &= 0x3ffu;
      u = sign | (exp << 23) | (man << 13);
    }
  } else if (exp == 31) {
    u = sign | 0x7f800000u | (man << 13);
  } else {
    u = sign | ((exp + 127 - 15) << 23) | (man << 13);
  }
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint16_t or_f32_to_f16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint16_t sign = (uint16_t)((u >> 16) & 0x8000u);
  const uint32_t au = u & 0x7fffffffu;
  if (au > 0x7f800000u) return sign | 0x7e00u; /* NaN */
  if (au >= 0x477ff000u) return sign | 0x7c00u; /* overflow -> inf (>= 65520) */
  if (au < 0x38800000u) {                        /* subnormal or zero */
    /* exact RNE: value * 2^24 rounded to integer */
    float a;
    memcpy(&a, &au, 4);
    const float r = nearbyintf(a * 16777216.0f);
    return sign | (uint16_t)r;
  }
  uint32_t mant = au & 0x7fffffu;
  int32_t e = (int32_t)(au >> 23) - 127 + 15;
  uint32_t h = ((uint32_t)e << 10) | (mant >> 13);
  const uint32_t rest = mant & 0x1fffu;
  if (rest > 0x1000u || (rest == 0x1000u && (h & 1u))) h += 1;
  return sign | (uint16_t)h;
}

static float ld(const void* p, int dt, int64_t i) {
  if (dt == OR_F32) return ((const float*)p)[i];
  if (dt == OR_BF16) return or_bf16_to_f32(((const uint16_t*)p)[i]);
  return or_f16_to_f32(((const uint16_t*)p)[i]);
}
static void st(void* p, int dt, int64_t i, float v) {
  if (dt == OR_F32) ((float*)p)[i] = v;
  else if (dt == OR_BF16) ((uint16_t*)p)[i] = or_f32_to_bf16(v);
  else ((uint16_t*)p)[i] = or_f32_to_f16(v);
}
static float round_to(int dt, float v) {
  if (dt == OR_F32) return v;
  if (dt == OR_BF16) return or_bf16_to_f32(or_f32_to_bf16(v));
  return or_f16_to_f32(or_f32_to_f16(v));
}

/* Reducer pack (upstream reducer.cpp mark_variable_ready_dense, declared at
 * T:include/torch/csrc/distributed/c10d/reducer.hpp:275):
 *   mode 0: bucket_view.copy_(grad)                       (comm hook registered)
 *   mode 1: at::mul_out(bucket_view, grad, 1/div_factor)  (default; scale = float(1/ws))
 *   mode 2: bucket_view = grad.to(bucket dtype).div_(s)   (bf16_compress_hook order,
 *           T:distributed/algorithms/ddp_comm_hooks/default_hooks.py:116; also the
 *           gradient_as_bucket_view bucket_view.div_(div_factor)) */
void or_pack(int n, const void* const* srcs, const int64_t* numels, const int64_t* offsets,
             int src_dt, void* flat, int flat_dt, float scale, int mode) {
  const int fsz = flat_dt == OR_F32 ? 4 : 2;
  for (int t = 0; t < n; ++t) {
    char* dst = (char*)flat + offsets[t] * fsz;
    for (int64_t i = 0; i < numels[t]; ++i) {
      float v = srcs[t] ? ld(srcs[t], src_dt, i) : 0.f;
      if (mode == 1) v = v * scale;
      else if (mode == 2) v = round_to(flat_dt, v) / scale;
      st(dst, flat_dt, i, v);
    }
  }
}

/* Reducer unpack: copy_bucket_to_grad grad.copy_(bucket_view) (reducer.hpp:329);
 * _unflatten_dense_tensors (T:_utils.py:578). */
void or_unpack(int n, void* const* dsts, const int64_t* numels, const int64_t* offsets,
               const void* flat, int flat_dt, int dst_dt) {
  const int fsz = flat_dt == OR_F32 ? 4 : 2;
  for (int t = 0; t < n; ++t) {
    if (!dsts[t]) continue;
    const char* src = (const char*)flat + offsets[t] * fsz;
    for (int64_t i = 0; i < numels[t]; ++i) st(dsts[t], dst_dt, i, ld(src, flat_dt, i));
  }
}

/* SUM all-reduce across `ws` rank buffers, left to right (rank 0 + rank 1 + ...).
 * For ws <= 2 this is exactly NCCL/RCCL/gloo's result (a+b is commutative);
 * for more ranks the collective's order differs and callers use a tolerance. */
void or_allreduce_sum(int ws, const void* const* bufs, int64_t count, int dt, void* out) {
  for (int64_t i = 0; i < count; ++i) {
    float acc = ld(bufs[0], dt, i);
    for (int r = 1; r < ws; ++r) acc = round_to(dt, acc + ld(bufs[r], dt, i));
    st(out, dt, i, acc);
  }
}

/* torch.optim.SGD (T:optim/sgd.py:322-381 _single_tensor_sgd):
 *   g = g*gscale; if maximize g = -g; if wd: g = g.add(p, alpha=wd)
 *   buf = first ? clone(g) : buf.mul_(mom).add_(g, alpha=1-damp)
 *   d = nesterov ? g.add(buf, alpha=mom) : buf;  p.add_(d, alpha=-lr)
 * Scalars are Python doubles rounded to fp32 at use; 1-damp is formed in double.
 * `a.add(b, alpha=s)` is evaluated as fmaf(s, b, a) (ATen's vectorised fmadd). */
void or_sgd(int64_t n, float* p, const void* g, int gdt, float* buf, double lr, double mom,
            double damp, double wd, int nesterov, int maximize, int first, const float* gscale,
            void* lowp, int ldt) {
  const float lr_f = (float)lr, mom_f = (float)mom, omd = (float)(1.0 - damp), wd_f = (float)wd;
  for (int64_t i = 0; i < n; ++i) {
    float gi = ld(g, gdt, i);
    if (gscale) gi = gi * gscale[0];
    if (maximize) gi = -gi;
    if (wd_f != 0.f) gi = fmaf(wd_f, p[i], gi);
    float d = gi;
    if (mom_f != 0.f) {
      const float b = first ? gi : fmaf(omd, gi, buf[i] * mom_f);
      buf[i] = b;
      d = nesterov ? fmaf(mom_f, b, gi) : b;
    }
    p[i] = fmaf(-lr_f, d, p[i]);
    if (lowp) st(lowp, ldt, i, p[i]);
  }
}

/* torch.optim.Adam / AdamW foreach arithmetic (T:optim/adam.py:554-800):
 *   adamw: p.mul_(1 - lr*wd)  |  adam: g = g.add(p, alpha=wd)
 *   m.lerp_(g, 1-b1)                 (ATen lerp, weight < 0.5: m + w*(g-m))
 *   v.mul_(b2).addcmul_(g, g, 1-b2)
 *   denom = v.sqrt() / bc2_sqrt + eps
 *   p.addcdiv_(m, denom, step_size)  (step_size = -lr/bc1, bc in double) */
void or_adam(int64_t n, float* p, const void* g, int gdt, float* m, float* v, double lr,
             double b1, double b2, double eps, double wd, int adamw, int maximize,
             double step_size, double bc2_sqrt, const float* gscale, void* lowp, int ldt) {
  const float w1 = (float)(1.0 - b1), b2f = (float)b2, w2 = (float)(1.0 - b2);
  const float eps_f = (float)eps, wd_f = (float)wd, decay = (float)(1.0 - lr * wd);
  const float ss = (float)step_size, bc2s = (float)bc2_sqrt;
  for (int64_t i = 0; i < n; ++i) {
    float gi = ld(g, gdt, i);
    if (gscale) gi = gi * gscale[0];
    if (maximize) gi = -gi;
    float x = p[i];
    if (wd_f != 0.f) {
      if (adamw) x = x * decay;
      else gi = fmaf(wd_f, x, gi);
    }
    const float mi = fmaf(w1, gi - m[i], m[i]);
    const float vi = fmaf(w2 * gi, gi, v[i] * b2f);
    const float denom = sqrtf(vi) / bc2s + eps_f;
    x = fmaf(ss, mi / denom, x);
    p[i] = x;
    m[i] = mi;
    v[i] = vi;
    if (lowp) st(lowp, ldt, i, x);
  }
}

/* Σ x² in double (the reference computes per-tensor fp32 norms then the norm
 * of norms, T:nn/utils/clip_grad.py:96-103; compared with a tolerance). */
double or_sqnorm(int n, const void* const* xs, const int64_t* numels, int dt) {
  double acc = 0.0;
  for (int t = 0; t < n; ++t)
    for (int64_t i = 0; i < numels[t]; ++i) {
      const double x = ld(xs[t], dt, i);
      acc += x * x;
    }
  return acc;
}

/* clip_coef = max_norm / (total_norm + 1e-6), clamped to 1 (T:nn/utils/clip_grad.py:165-174) */
float or_clip_coef(float total_norm, float max_norm, float eps) {
  const float c = max_norm / (total_norm + eps);
  return c < 1.f ? c : 1.f;
}

/* compute_bucket_assignment_by_size (upstream reducer.cpp; declared at
 * T:include/torch/csrc/distributed/c10d/reducer.hpp:590-595).  Returns the
 * number of buckets; members are written bucket after bucket. */
int or_bucket_assignment(int n, const int64_t* nbytes, const int32_t* keys, const int32_t* order,
                         int n_limits, const int64_t* limits, int32_t* members, int32_t* counts) {
  enum { MAXK = 16 };
  int32_t key_of[MAXK];
  int nkeys = 0;
  int64_t size[MAXK];
  int lim[MAXK];
  /* open bucket member lists live in a scratch area per key: at most n each */
  static int32_t open_idx[MAXK][4096];
  int open_n[MAXK];
  int nb = 0, pos = 0;
  int32_t bstart[4096];
  if (n > 4096) return -1;
  for (int i = 0; i < n; ++i) {
    const int32_t t = order ? order[i] : i;
    const int32_t key = keys ? keys[t] : 0;
    int k = 0;
    while (k < nkeys && key_of[k] != key) ++k;
    if (k == nkeys) {
      if (nkeys == MAXK) return -1;
      key_of[k] = key;
      size[k] = 0;
      lim[k] = 0;
      open_n[k] = 0;
      ++nkeys;
    }
    open_idx[k][open_n[k]++] = t;
    size[k] += nbytes[t];
    if (size[k] >= limits[lim[k]]) {
      bstart[nb] = pos;
      counts[nb++] = open_n[k];
      for (int j = 0; j < open_n[k]; ++j) members[pos++] = open_idx[k][j];
      open_n[k] = 0;
      size[k] = 0;
      if (lim[k] + 1 < n_limits) ++lim[k];
    }
  }
  for (int k = 0; k < nkeys; ++k)
    if (open_n[k]) {
      bstart[nb] = pos;
      counts[nb++] = open_n[k];
      for (int j = 0; j < open_n[k]; ++j) members[pos++] = open_idx[k][j];
    }
  if (!order) { /* sort buckets by their smallest member (stable insertion sort) */
    int32_t tmp[4096];
    int32_t mins[4096], perm[4096];
    for (int b = 0; b < nb; ++b) {
      int32_t mn = members[bstart[b]];
      for (int j = 1; j < counts[b]; ++j)
        if (members[bstart[b] + j] < mn) mn = members[bstart[b] + j];
      mins[b] = mn;
      perm[b] = b;
    }
    for (int a = 1; a < nb; ++a) {
      int32_t x = perm[a];
      int c = a - 1;
      while (c >= 0 && mins[perm[c]] > mins[x]) { perm[c + 1] = perm[c]; --c; }
      perm[c + 1] = x;
    }
    int32_t newcounts[4096];
    int q = 0;
    for (int b = 0; b < nb; ++b) {
      const int src = perm[b];
      newcounts[b] = counts[src];
      for (int j = 0; j < counts[src]; ++j) tmp[q++] = members[bstart[src] + j];
    }
    memcpy(members, tmp, sizeof(int32_t) * q);
    memcpy(counts, newcounts, sizeof(int32_t) * nb);
  }
  return nb;
}
