// Host implementation of the plan ops, used for CPU tensors (the CPU/gloo
// configuration: BASELINE config 1).  Same arithmetic as gs_kernels.hip,
// element for element (explicit fmaf, -ffp-contract=off), so a CPU run and a
// GPU run of the engine agree bit for bit on the pack / unpack / optimizer
// math.  A HIP plan never reaches this file.
#include <cmath>

#include "gs_common.h"

namespace gs {
namespace {

inline float bf16_to_f32(uint16_t h) {
  uint32_t u = static_cast<uint32_t>(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7FC0;
  return static_cast<uint16_t>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
inline float f16_to_f32(uint16_t h) {
  _Float16 x;
  std::memcpy(&x, &h, 2);
  return static_cast<float>(x);
}
inline uint16_t f32_to_f16(float f) {
  _Float16 x = static_cast<_Float16>(f);
  uint16_t h;
  std::memcpy(&h, &x, 2);
  return h;
}

inline float ld(const void* base, int dt, int64_t i) {
  switch (dt) {
    case GS_F32: return static_cast<const float*>(base)[i];
    case GS_BF16: return bf16_to_f32(static_cast<const uint16_t*>(base)[i]);
    default: return f16_to_f32(static_cast<const uint16_t*>(base)[i]);
  }
}
inline void st(void* base, int dt, int64_t i, float v) {
  switch (dt) {
    case GS_F32: static_cast<float*>(base)[i] = v; break;
    case GS_BF16: static_cast<uint16_t*>(base)[i] = f32_to_bf16(v); break;
    default: static_cast<uint16_t*>(base)[i] = f32_to_f16(v); break;
  }
}
inline float round_to(int dt, float v) {
  if (dt == GS_F32) return v;
  if (dt == GS_BF16) return bf16_to_f32(f32_to_bf16(v));
  return f16_to_f32(f32_to_f16(v));
}
inline void* slot(gs_plan* p, int s, int t) { return p->h_ptrs[static_cast<size_t>(s) * p->n + t]; }

int check_float(int dt) {
  if (!is_float_dtype(dt)) return fail(GS_EINVAL, "unsupported floating dtype");
  return GS_OK;
}

}  // namespace

int host_pack(gs_plan* p, int src_slot, int src_dt, void* flat, int flat_dt, float s, int mode) {
  GS_TRY_RET(check_float(src_dt));
  GS_TRY_RET(check_float(flat_dt));
  const int fsz = dtype_size(flat_dt);
  for (int t = 0; t < p->n; ++t) {
    const void* src = slot(p, src_slot, t);
    void* dst = static_cast<char*>(flat) + p->off[t] * fsz;
    for (int64_t i = 0; i < p->numel[t]; ++i) {
      float v = src ? ld(src, src_dt, i) : 0.f;
      if (mode == GS_SCALE_MUL) v = v * s;
      else if (mode == GS_SCALE_DIV) v = round_to(flat_dt, v) / s;
      st(dst, flat_dt, i, v);
    }
  }
  return GS_OK;
}

int host_unpack(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* sq,
                int acc) {
  GS_TRY_RET(check_float(flat_dt));
  GS_TRY_RET(check_float(dst_dt));
  const int fsz = dtype_size(flat_dt);
  double total = 0.0;
  for (int t = 0; t < p->n; ++t) {
    const void* src = static_cast<const char*>(flat) + p->off[t] * fsz;
    void* dst = slot(p, dst_slot, t);
    if (dst == nullptr) continue;
    for (int64_t i = 0; i < p->numel[t]; ++i) {
      const float v = ld(src, flat_dt, i);
      st(dst, dst_dt, i, v);
      if (sq) {
        const float r = round_to(dst_dt, v);
        total += static_cast<double>(r) * r;
      }
    }
  }
  if (sq) sq[0] = acc ? sq[0] + static_cast<float>(total) : static_cast<float>(total);
  return GS_OK;
}

int host_unpack_check(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* found) {
  GS_TRY_RET(check_float(flat_dt));
  GS_TRY_RET(check_float(dst_dt));
  const int fsz = dtype_size(flat_dt);
  float f = found[0];
  for (int t = 0; t < p->n; ++t) {
    const void* src = static_cast<const char*>(flat) + p->off[t] * fsz;
    void* dst = slot(p, dst_slot, t);
    if (dst == nullptr) continue;
    for (int64_t i = 0; i < p->numel[t]; ++i) {
      const float v = ld(src, flat_dt, i);
      st(dst, dst_dt, i, v);
      if (!std::isfinite(round_to(dst_dt, v))) f = 1.f;
    }
  }
  found[0] = f;
  return GS_OK;
}

int host_scale(gs_plan* p, int s_, int dt, float s, int mode) {
  GS_TRY_RET(check_float(dt));
  for (int t = 0; t < p->n; ++t) {
    void* x = slot(p, s_, t);
    for (int64_t i = 0; i < p->numel[t]; ++i) {
      const float v = ld(x, dt, i);
      st(x, dt, i, mode == GS_SCALE_DIV ? v / s : v * s);
    }
  }
  return GS_OK;
}

int host_sqnorm(gs_plan* p, int s_, int dt, float* sq, int acc) {
  GS_TRY_RET(check_float(dt));
  double total = 0.0;
  for (int t = 0; t < p->n; ++t) {
    const void* x = slot(p, s_, t);
    for (int64_t i = 0; i < p->numel[t]; ++i) {
      const double v = ld(x, dt, i);
      total += v * v;
    }
  }
  sq[0] = acc ? sq[0] + static_cast<float>(total) : static_cast<float>(total);
  return GS_OK;
}

int host_clip_coef(const float* sq, float max_norm, float eps, float* coef, float* norm) {
  const float nrm = std::sqrt(sq[0]);
  if (norm) norm[0] = nrm;
  const float c = max_norm / (nrm + eps);
  coef[0] = c < 1.f ? c : 1.f;
  return GS_OK;
}

int host_unscale_check(gs_plan* p, int s_, int dt, const float* inv, float* found) {
  GS_TRY_RET(check_float(dt));
  float f = found[0];
  for (int t = 0; t < p->n; ++t) {
    void* x = slot(p, s_, t);
    for (int64_t i = 0; i < p->numel[t]; ++i) {
      const float v = ld(x, dt, i);
      if (!std::isfinite(v)) f = 1.f;
      if (inv && inv[0] != 1.f) st(x, dt, i, v * inv[0]);
    }
  }
  found[0] = f;
  return GS_OK;
}

int host_sgd(gs_plan* p, int gdt, int ldt, const SgdHyper& h, const float* gsc, const float* fi) {
  GS_TRY_RET(check_float(gdt));
  if (fi && fi[0] != 0.f) return GS_OK;
  for (int t = 0; t < p->n; ++t) {
    float* pp = static_cast<float*>(slot(p, 0, t));
    const void* gp = slot(p, 1, t);
    float* bp = static_cast<float*>(slot(p, 2, t));
    void* lp = slot(p, 3, t);
    for (int64_t i = 0; i < p->numel[t]; ++i) {
      float g = ld(gp, gdt, i);
      if (gsc) g = g * gsc[0];
      if (h.maximize) g = -g;
      if (h.wd != 0.f) g = std::fmaf(h.wd, pp[i], g);
      float d = g;
      if (h.mom != 0.f) {
        const float b = h.first ? g : std::fmaf(h.omd, g, bp[i] * h.mom);
        bp[i] = b;
        d = h.nesterov ? std::fmaf(h.mom, b, g) : b;
      }
      pp[i] = std::fmaf(-h.lr, d, pp[i]);
      if (ldt >= 0) st(lp, ldt, i, pp[i]);
    }
  }
  return GS_OK;
}

int host_adam(gs_plan* p, int gdt, int ldt, const AdamHyper& h, const float* gsc,
              const float* fi) {
  GS_TRY_RET(check_float(gdt));
  if (fi && fi[0] != 0.f) return GS_OK;
  for (int t = 0; t < p->n; ++t) {
    float* pp = static_cast<float*>(slot(p, 0, t));
    const void* gp = slot(p, 1, t);
    float* mp = static_cast<float*>(slot(p, 2, t));
    float* vp = static_cast<float*>(slot(p, 3, t));
    void* lp = slot(p, 4, t);
    for (int64_t i = 0; i < p->numel[t]; ++i) {
      float g = ld(gp, gdt, i);
      if (gsc) g = g * gsc[0];
      if (h.maximize) g = -g;
      float x = pp[i];
      if (h.wd != 0.f) {
        if (h.adamw) x = x * h.decay;
        else g = std::fmaf(h.wd, x, g);
      }
      const float m = std::fmaf(h.w1, g - mp[i], mp[i]);
      const float v = std::fmaf(h.w2 * g, g, vp[i] * h.b2);
      const float denom = std::sqrt(v) / h.bc2s + h.eps;
      x = std::fmaf(h.step_size, m / denom, x);
      pp[i] = x;
      mp[i] = m;
      vp[i] = v;
      if (ldt >= 0) st(lp, ldt, i, x);
    }
  }
  return GS_OK;
}

}  // namespace gs
