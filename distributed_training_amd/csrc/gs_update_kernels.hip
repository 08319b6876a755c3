// gfx950 (CDNA4) fused SGD / Adam(W) updates of libgsync (gs_sgd_step / gs_adam_step):
// the chunk-map engine of gs_engine.h with SgdOp / AdamOp, the grad-load policy per launch.

#include "gs_engine.h"

namespace gs {

// grads a Σg² pass of this plan read just before (the clip path) stay in the caches
// when they fit in the Infinity Cache: cached loads then, non-temporal otherwise
// (the flag is consumed by the update)
static bool nt_grad(gs_plan* p, int gdt) {
  const bool hot = p->grads_read && p->elems * dtype_bytes(gdt) <= kInfinityCacheBytes;
  p->grads_read = false;
  return !hot;
}

template <bool NTG>
static int sgd_nt(gs_plan* p, int gdt, int ldt, const SgdHyper& h, const float* gsc, const float* fi,
                  const ClipArgs* clip, void* stream) {
  GS_DISPATCH_FLOAT(gdt, GD, GS_DISPATCH_LOWP(ldt, LD, {
    SgdOp<kUnit, GD, LD, NTG> op;
    op.h = h; op.gscale = gsc; op.found_inf = fi; op.hyper = p->hyper;
    if (clip) { op.clip = *clip; op.clip_on = true; }
    return launch(p, op, stream);
  }));
  return GS_OK;
}

int hip_sgd(gs_plan* p, int gdt, int ldt, const SgdHyper& h, const float* gsc, const float* fi,
            const ClipArgs* clip, void* stream) {
  DeviceGuard g(p->device);
  return nt_grad(p, gdt) ? sgd_nt<true>(p, gdt, ldt, h, gsc, fi, clip, stream)
                         : sgd_nt<false>(p, gdt, ldt, h, gsc, fi, clip, stream);
}

template <bool NTG>
static int adam_nt(gs_plan* p, int gdt, int ldt, const AdamHyper& h, const float* gsc, const float* fi,
                   const ClipArgs* clip, void* stream) {
  GS_DISPATCH_FLOAT(gdt, GD, GS_DISPATCH_LOWP(ldt, LD, {
    AdamOp<kUnit, GD, LD, NTG> op;
    op.h = h; op.gscale = gsc; op.found_inf = fi; op.hyper = p->hyper;
    if (clip) { op.clip = *clip; op.clip_on = true; }
    return launch(p, op, stream);
  }));
  return GS_OK;
}

int hip_adam(gs_plan* p, int gdt, int ldt, const AdamHyper& h, const float* gsc, const float* fi,
             const ClipArgs* clip, void* stream) {
  DeviceGuard g(p->device);
  return nt_grad(p, gdt) ? adam_nt<true>(p, gdt, ldt, h, gsc, fi, clip, stream)
                         : adam_nt<false>(p, gdt, ldt, h, gsc, fi, clip, stream);
}

}  // namespace gs
