// gfx950 (CDNA4) fused SGD / Adam(W) updates of libgsync (gs_sgd_step / gs_adam_step):
// the chunk-map engine of gs_engine.h with SgdOp / AdamOp, the load policy per launch.

#include "gs_engine.h"

namespace gs {

// non-temporal loads of the update's state streams (GS_NT_STATE, gs_engine.h): never,
// always, or when p + the fp32 states (state_streams of them) exceed 256 MiB
static bool nt_state(const gs_plan* p, int state_streams) {
  static const int policy = [] {
    const char* e = std::getenv("GS_NT_STATE");
    return e ? std::atoi(e) : GS_NT_STATE_DEFAULT;
  }();
  if (policy != 2) return policy != 0;
  return p->elems * 4 * (1 + state_streams) > kInfinityCacheBytes;
}

// grads a Σg² pass of this plan read just before (the clip path) stay in the caches
// when they fit in the Infinity Cache: cached loads then, non-temporal otherwise
// (the flag is consumed by the update)
static bool nt_grad(gs_plan* p, int gdt) {
  const bool hot = p->grads_read && p->elems * dtype_bytes(gdt) <= kInfinityCacheBytes;
  p->grads_read = false;
  return GS_NT_LOAD_GRAD != 0 && !hot;
}

template <bool NTG, bool NTS>
static int sgd_nt(gs_plan* p, int gdt, int ldt, const SgdHyper& h, const float* gsc, const float* fi,
                  const ClipArgs* clip, void* stream) {
  GS_DISPATCH_FLOAT(gdt, GD, GS_DISPATCH_LOWP(ldt, LD, {
    SgdOp<GS_OPT_N, GD, LD, NTG, NTS> op;
    op.h = h; op.gscale = gsc; op.found_inf = fi; op.hyper = p->hyper;
    if (clip) { op.clip = *clip; op.clip_on = true; }
    return launch<GS_OPT_ILP>(p, op, stream);
  }));
  return GS_OK;
}

int hip_sgd(gs_plan* p, int gdt, int ldt, const SgdHyper& h, const float* gsc, const float* fi,
            const ClipArgs* clip, void* stream) {
  DeviceGuard g(p->device);
  const bool ntg = nt_grad(p, gdt), nts = nt_state(p, h.mom != 0.f ? 1 : 0);
  if (ntg) return nts ? sgd_nt<true, true>(p, gdt, ldt, h, gsc, fi, clip, stream)
                      : sgd_nt<true, false>(p, gdt, ldt, h, gsc, fi, clip, stream);
  return nts ? sgd_nt<false, true>(p, gdt, ldt, h, gsc, fi, clip, stream)
             : sgd_nt<false, false>(p, gdt, ldt, h, gsc, fi, clip, stream);
}

template <bool NTG, bool NTS>
static int adam_nt(gs_plan* p, int gdt, int ldt, const AdamHyper& h, const float* gsc, const float* fi,
                   const ClipArgs* clip, void* stream) {
  GS_DISPATCH_FLOAT(gdt, GD, GS_DISPATCH_LOWP(ldt, LD, {
    AdamOp<GS_OPT_N, GD, LD, NTG, NTS> op;
    op.h = h; op.gscale = gsc; op.found_inf = fi; op.hyper = p->hyper;
    if (clip) { op.clip = *clip; op.clip_on = true; }
    return launch<GS_OPT_ILP>(p, op, stream);
  }));
  return GS_OK;
}

int hip_adam(gs_plan* p, int gdt, int ldt, const AdamHyper& h, const float* gsc, const float* fi,
             const ClipArgs* clip, void* stream) {
  DeviceGuard g(p->device);
  const bool ntg = nt_grad(p, gdt), nts = nt_state(p, 2);
  if (ntg) return nts ? adam_nt<true, true>(p, gdt, ldt, h, gsc, fi, clip, stream)
                      : adam_nt<true, false>(p, gdt, ldt, h, gsc, fi, clip, stream);
  return nts ? adam_nt<false, true>(p, gdt, ldt, h, gsc, fi, clip, stream)
             : adam_nt<false, false>(p, gdt, ldt, h, gsc, fi, clip, stream);
}

}  // namespace gs
