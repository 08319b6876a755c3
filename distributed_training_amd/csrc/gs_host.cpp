// Host implementation of the plan ops, used for CPU tensors (the CPU/gloo
// configuration: BASELINE config 1).  Same arithmetic as gs_kernels.hip,
// element for element (explicit fmaf, -ffp-contract=off), so a CPU run and a
// GPU run of the engine agree bit for bit on the pack / unpack / optimizer
// math.  A HIP plan never reaches this file.
//
// Speed: loops are instantiated per dtype combination (no per-element type
// switch) so the compiler vectorises them (built with -mavx2 -mfma: std::fmaf
// is one vfmadd, bit-identical to the software fmaf), and large plans are
// split over gs_set_host_threads() threads (torch's intra-op thread count).
// Elementwise results do not depend on the split; the Σg² reductions stay
// serial (their double-precision order is the oracle's).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <thread>

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


template <int DT>
inline float ldT(const void* base, int64_t i) {
  if constexpr (DT == GS_F32) return static_cast<const float*>(base)[i];
  else if constexpr (DT == GS_BF16) return bf16_to_f32(static_cast<const uint16_t*>(base)[i]);
  else return f16_to_f32(static_cast<const uint16_t*>(base)[i]);
}
template <int DT>
inline void stT(void* base, int64_t i, float v) {
  if constexpr (DT == GS_F32) static_cast<float*>(base)[i] = v;
  else if constexpr (DT == GS_BF16) static_cast<uint16_t*>(base)[i] = f32_to_bf16(v);
  else static_cast<uint16_t*>(base)[i] = f32_to_f16(v);
}
template <int DT>
inline float roundT(float v) {
  if constexpr (DT == GS_F32) return v;
  else if constexpr (DT == GS_BF16) return bf16_to_f32(f32_to_bf16(v));
  else return f16_to_f32(f32_to_f16(v));
}
inline void* slot(gs_plan* p, int s, int t) { return p->h_ptrs[static_cast<size_t>(s) * p->n + t]; }

int check_float(int dt) {
  if (!is_float_dtype(dt)) return fail(GS_EINVAL, "unsupported floating dtype");
  return GS_OK;
}

std::atomic<int> g_threads{1};
constexpr int64_t kChunk = int64_t(1) << 16;     // elements per work item
constexpr int64_t kParallelMin = int64_t(1) << 19;  // below this, one thread

// fn(t, i0, i1) over every tensor's element range, split into chunks and
// spread over the host threads (static round-robin: deterministic, and the
// elementwise results do not depend on it anyway)
template <class F>
void for_ranges(const gs_plan* p, F&& fn) {
  int64_t total = 0;
  for (int t = 0; t < p->n; ++t) total += p->numel[t];
  const int nt = std::max(1, std::min<int>(g_threads.load(), static_cast<int>(total / kChunk) + 1));
  if (nt == 1 || total < kParallelMin) {
    for (int t = 0; t < p->n; ++t)
      if (p->numel[t]) fn(t, int64_t(0), p->numel[t]);
    return;
  }
  std::vector<std::tuple<int, int64_t, int64_t>> items;
  for (int t = 0; t < p->n; ++t)
    for (int64_t i = 0; i < p->numel[t]; i += kChunk) items.emplace_back(t, i, std::min(p->numel[t], i + kChunk));
  auto work = [&](int k) {
    for (size_t j = k; j < items.size(); j += nt) fn(std::get<0>(items[j]), std::get<1>(items[j]), std::get<2>(items[j]));
  };
  std::vector<std::thread> pool;
  for (int k = 1; k < nt; ++k) pool.emplace_back(work, k);
  work(0);
  for (auto& th : pool) th.join();
}

#define GS_HOST_FLOAT(DT, NAME, ...)                                    \
  switch (DT) {                                                         \
    case GS_F32: { constexpr int NAME = GS_F32; __VA_ARGS__; break; }   \
    case GS_BF16: { constexpr int NAME = GS_BF16; __VA_ARGS__; break; } \
    case GS_F16: { constexpr int NAME = GS_F16; __VA_ARGS__; break; }   \
    default: return fail(GS_EINVAL, "unsupported floating dtype");      \
  }
#define GS_HOST_LOWP(DT, NAME, ...)                                      \
  switch (DT) {                                                          \
    case -1: { constexpr int NAME = -1; __VA_ARGS__; break; }            \
    case GS_BF16: { constexpr int NAME = GS_BF16; __VA_ARGS__; break; }  \
    case GS_F16: { constexpr int NAME = GS_F16; __VA_ARGS__; break; }    \
    default: return fail(GS_EINVAL, "unsupported low-precision dtype");  \
  }

}  // namespace

int host_pack(gs_plan* p, int src_slot, int src_dt, void* flat, int flat_dt, float s, int mode) {
  GS_HOST_FLOAT(src_dt, SD, GS_HOST_FLOAT(flat_dt, FD, {
    const int fsz = dtype_size(FD);
    for_ranges(p, [&](int t, int64_t i0, int64_t i1) {
      const void* src = slot(p, src_slot, t);
      void* dst = static_cast<char*>(flat) + p->off[t] * fsz;
      if (!src) {
        const float z = mode == GS_SCALE_MUL ? 0.f * s : (mode == GS_SCALE_DIV ? 0.f / s : 0.f);
        for (int64_t i = i0; i < i1; ++i) stT<FD>(dst, i, z);  // unused parameter: zeros, as the kernel
      } else if (mode == GS_SCALE_MUL) {
        for (int64_t i = i0; i < i1; ++i) stT<FD>(dst, i, ldT<SD>(src, i) * s);
      } else if (mode == GS_SCALE_DIV) {
        for (int64_t i = i0; i < i1; ++i) stT<FD>(dst, i, roundT<FD>(ldT<SD>(src, i)) / s);
      } else {
        for (int64_t i = i0; i < i1; ++i) stT<FD>(dst, i, ldT<SD>(src, i));
      }
    });
  }));
  return GS_OK;
}

int host_unpack(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* sq,
                int acc) {
  GS_HOST_FLOAT(flat_dt, FD, GS_HOST_FLOAT(dst_dt, DD, {
    const int fsz = dtype_size(FD);
    if (sq) {  // serial: the double-precision Σ order is the oracle's
      double total = 0.0;
      for (int t = 0; t < p->n; ++t) {
        const void* src = static_cast<const char*>(flat) + p->off[t] * fsz;
        void* dst = slot(p, dst_slot, t);
        if (dst == nullptr) continue;
        for (int64_t i = 0; i < p->numel[t]; ++i) {
          const float v = ldT<FD>(src, i);
          stT<DD>(dst, i, v);
          const float r = roundT<DD>(v);
          total += static_cast<double>(r) * r;
        }
      }
      sq[0] = acc ? sq[0] + static_cast<float>(total) : static_cast<float>(total);
    } else {
      for_ranges(p, [&](int t, int64_t i0, int64_t i1) {
        const void* src = static_cast<const char*>(flat) + p->off[t] * fsz;
        void* dst = slot(p, dst_slot, t);
        if (dst == nullptr) return;
        for (int64_t i = i0; i < i1; ++i) stT<DD>(dst, i, ldT<FD>(src, i));
      });
    }
  }));
  return GS_OK;
}

int host_unpack_check(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* found) {
  std::atomic<int> bad{found[0] != 0.f ? 1 : 0};
  GS_HOST_FLOAT(flat_dt, FD, GS_HOST_FLOAT(dst_dt, DD, {
    const int fsz = dtype_size(FD);
    for_ranges(p, [&](int t, int64_t i0, int64_t i1) {
      const void* src = static_cast<const char*>(flat) + p->off[t] * fsz;
      void* dst = slot(p, dst_slot, t);
      if (dst == nullptr) return;
      int b = 0;
      for (int64_t i = i0; i < i1; ++i) {
        const float v = ldT<FD>(src, i);
        stT<DD>(dst, i, v);
        b |= !std::isfinite(roundT<DD>(v));
      }
      if (b) bad.store(1);
    });
  }));
  found[0] = bad.load() ? 1.f : 0.f;
  return GS_OK;
}

int host_scale(gs_plan* p, int s_, int dt, float s, int mode) {
  GS_HOST_FLOAT(dt, DT, {
    for_ranges(p, [&](int t, int64_t i0, int64_t i1) {
      void* x = slot(p, s_, t);
      if (mode == GS_SCALE_DIV)
        for (int64_t i = i0; i < i1; ++i) stT<DT>(x, i, ldT<DT>(x, i) / s);
      else
        for (int64_t i = i0; i < i1; ++i) stT<DT>(x, i, ldT<DT>(x, i) * s);
    });
  });
  return GS_OK;
}

int host_clip_scale(gs_plan* p, int s_, int dt, const ClipArgs& clip) {
  const float cf = host_clip_factor(clip, nullptr);
  if (cf == 1.f) return GS_OK;  // x * 1 == x: nothing to write (the device grid exits too)
  return host_scale(p, s_, dt, cf, GS_SCALE_MUL);
}

int host_sqnorm(gs_plan* p, int s_, int dt, float* sq, int acc) {
  GS_HOST_FLOAT(dt, DT, {
    double total = 0.0;
    for (int t = 0; t < p->n; ++t) {
      const void* x = slot(p, s_, t);
      for (int64_t i = 0; i < p->numel[t]; ++i) {
        const double v = ldT<DT>(x, i);
        total += v * v;
      }
    }
    sq[0] = acc ? sq[0] + static_cast<float>(total) : static_cast<float>(total);
  });
  return GS_OK;
}

int host_sum(gs_plan* p, int s_, int dt, float* out, int acc) {
  GS_HOST_FLOAT(dt, DT, {
    double total = 0.0;
    for (int t = 0; t < p->n; ++t) {
      const void* x = slot(p, s_, t);
      for (int64_t i = 0; i < p->numel[t]; ++i) total += ldT<DT>(x, i);
    }
    out[0] = acc ? out[0] + static_cast<float>(total) : static_cast<float>(total);
  });
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
  std::atomic<int> bad{found[0] != 0.f ? 1 : 0};
  const bool scale = inv && inv[0] != 1.f;
  const float sc = scale ? inv[0] : 1.f;
  GS_HOST_FLOAT(dt, DT, {
    for_ranges(p, [&](int t, int64_t i0, int64_t i1) {
      void* x = slot(p, s_, t);
      int b = 0;
      for (int64_t i = i0; i < i1; ++i) {
        const float v = ldT<DT>(x, i);
        b |= !std::isfinite(v);
        if (scale) stT<DT>(x, i, v * sc);
      }
      if (b) bad.store(1);
    });
  });
  found[0] = bad.load() ? 1.f : 0.f;
  return GS_OK;
}

// gs_kernels.hip wave_reduce<false>: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror, row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3; lane 63.
// A lane a step does not write adds 0 (the DPP `old` operand is the identity).
float host_wave_sum(const float* x, int n, int stride) {
  float v[64], t[64];
  // lane l first adds x[l], x[l + 64], ... in order (clip_multiplier's fold of up to
  // GS_RED_PARTIALS partials), then the tree
  for (int l = 0; l < 64; ++l) {
    float a = 0.f;
    for (int j = l; j < n; j += 64) a = a + x[static_cast<int64_t>(j) * stride];
    v[l] = 0.f + a;
  }
  auto step = [&](auto src, unsigned row_mask) {
    for (int l = 0; l < 64; ++l) t[l] = ((row_mask >> (l >> 4)) & 1u) ? v[src(l)] : 0.f;
    for (int l = 0; l < 64; ++l) v[l] = v[l] + t[l];
  };
  static const int q1[4] = {1, 0, 3, 2}, q2[4] = {2, 3, 0, 1};
  step([](int l) { return (l & ~3) | q1[l & 3]; }, 0xFu);
  step([](int l) { return (l & ~3) | q2[l & 3]; }, 0xFu);
  step([](int l) { return (l & ~7) | (7 - (l & 7)); }, 0xFu);
  step([](int l) { return (l & ~15) | (15 - (l & 15)); }, 0xFu);
  step([](int l) { return (l & ~15) - 1; }, 0xAu);  // rows 1, 3 <- lane 15 of the row below
  step([](int) { return 31; }, 0xCu);                // rows 2, 3 <- lane 31
  return v[63];
}

float host_clip_factor(const ClipArgs& c, const float* gsc) {
  float sq = c.groups > 0 ? host_wave_sum(c.sq, c.groups, c.stride) : c.sq[0];
  const float s = gsc ? gsc[0] : 1.f;
  if (gsc) sq = sq * (s * s);
  sq = sq * c.sq_mul;
  const float nrm = std::sqrt(sq);
  float coef = c.max_norm / (nrm + c.eps);
  coef = c.torch_clamp ? (coef >= 1.f ? 1.f : coef) : (coef < 1.f ? coef : 1.f);
  if (gsc) coef = coef * s;
  coef = coef * c.coef_mul;
  if (c.out) {
    c.out[0] = sq;
    c.out[1] = coef;
    c.out[2] = nrm;
  }
  return coef;
}

int host_sgd(gs_plan* p, int gdt, int ldt, const SgdHyper& h, const float* gsc, const float* fi,
             const ClipArgs* clip) {
  const float cf = clip ? host_clip_factor(*clip, gsc) : 1.f;  // published even on a skipped step
  if (fi && fi[0] != 0.f) {
    GS_TRY_RET(check_float(gdt));
    return GS_OK;
  }
  const bool has_gs = gsc != nullptr || clip != nullptr;
  const float gs = clip ? cf : (gsc ? gsc[0] : 1.f);
  GS_HOST_FLOAT(gdt, GD, GS_HOST_LOWP(ldt, LD, {
    for_ranges(p, [&](int t, int64_t i0, int64_t i1) {
      float* pp = static_cast<float*>(slot(p, 0, t));
      const void* gp = slot(p, 1, t);
      float* bp = static_cast<float*>(slot(p, 2, t));
      void* lp = slot(p, 3, t);
      for (int64_t i = i0; i < i1; ++i) {
        float g = ldT<GD>(gp, i);
        if (has_gs) g = g * gs;
        if (h.maximize) g = -g;
        if (h.wd != 0.f) g = std::fmaf(h.wd, pp[i], g);
        float d = g;
        if (h.mom != 0.f) {
          const float b = h.first ? g : std::fmaf(h.omd, g, bp[i] * h.mom);
          bp[i] = b;
          d = h.nesterov ? std::fmaf(h.mom, b, g) : b;
        }
        pp[i] = std::fmaf(-h.lr, d, pp[i]);
        if constexpr (LD >= 0) stT<LD>(lp, i, pp[i]);
      }
    });
  }));
  return GS_OK;
}

int host_adam(gs_plan* p, int gdt, int ldt, const AdamHyper& h, const float* gsc,
              const float* fi, const ClipArgs* clip) {
  const float cf = clip ? host_clip_factor(*clip, gsc) : 1.f;  // published even on a skipped step
  if (fi && fi[0] != 0.f) {
    GS_TRY_RET(check_float(gdt));
    return GS_OK;
  }
  const bool has_gs = gsc != nullptr || clip != nullptr;
  const float gs = clip ? cf : (gsc ? gsc[0] : 1.f);
  GS_HOST_FLOAT(gdt, GD, GS_HOST_LOWP(ldt, LD, {
    for_ranges(p, [&](int t, int64_t i0, int64_t i1) {
      float* pp = static_cast<float*>(slot(p, 0, t));
      const void* gp = slot(p, 1, t);
      float* mp = static_cast<float*>(slot(p, 2, t));
      float* vp = static_cast<float*>(slot(p, 3, t));
      void* lp = slot(p, 4, t);
      for (int64_t i = i0; i < i1; ++i) {
        float g = ldT<GD>(gp, i);
        if (has_gs) g = g * gs;
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
        if constexpr (LD >= 0) stT<LD>(lp, i, x);
      }
    });
  }));
  return GS_OK;
}

}  // namespace gs

extern "C" int gs_set_host_threads(int n) {
  gs::g_threads.store(n < 1 ? 1 : (n > 256 ? 256 : n));
  return GS_OK;
}
