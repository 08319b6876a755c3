// libgsync: error plumbing, multi-tensor plans and the plan-op entry points,
// plus the bucket-assignment restatement of torch's Reducer.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <new>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "gs_common.h"

namespace gs {

static thread_local std::string g_last_error;

bool roctx_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("GSYNC_ROCTX");
    return e && std::atoi(e) != 0;
  }();
  return on;
}
void roctx_push(const char* name) { roctxRangePushA(name); }
void roctx_pop() { roctxRangePop(); }

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

}  // namespace gs

using namespace gs;

gs::PlanArgs gs_plan::args() const {
  PlanArgs a{};
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  char* base = static_cast<char*>(d_static);
  size_t o = 0;
  a.segs = reinterpret_cast<const Seg*>(base + o);
  o += al(sizeof(Seg) * segs.size());
  a.task_begin = reinterpret_cast<const int32_t*>(base + o);
  o += al(sizeof(int32_t) * task_begin.size());
  a.numel = reinterpret_cast<const int64_t*>(base + o);
  o += al(sizeof(int64_t) * n);
  a.off = reinterpret_cast<const int64_t*>(base + o);
  o += al(sizeof(int64_t) * n);
  a.chunks = reinterpret_cast<const ChunkDesc*>(base + o);
  o += al(sizeof(ChunkDesc) * chunks.size());
  a.voff = reinterpret_cast<const int64_t*>(base + o);
  o += al(sizeof(int64_t) * n);
  a.ticket = nullptr;  // the launch points it at the sync words after d_partials
  a.red_out = nullptr;
  a.red_acc = 0;
  a.red_fuse = 0;
  a.red_groups_only = 0;
  a.red_raw = 0;
  a.ptrs = static_cast<void* const*>(d_table);
  a.align = reinterpret_cast<const uint32_t*>(static_cast<char*>(d_table) +
                                              sizeof(void*) * GS_PLAN_SLOTS * n);
  a.n = n;
  a.n_tasks = static_cast<int32_t>(task_begin.size()) - 1;
  a.n_chunks = static_cast<int32_t>(chunks.size());
  return a;
}

// Chunk map of the chunk-map engine (gs_common.h): virtual offsets and one
// descriptor per kChunkElems elements of the virtual space.
static void build_chunk_map(gs_plan* p) {
  const int n = p->n;
  p->voff.assign(n, 0);
  int64_t cur = 0;
  for (int t = 0; t < n; ++t) {
    const int64_t m = p->numel[t];
    const int64_t a = m >= kGroupElems ? kGroupElems : (m >= kChunkElems ? kChunkElems : kUnit);
    cur = (cur + a - 1) / a * a;
    p->voff[t] = cur;
    cur += m;
  }
  const int64_t n_chunks = (cur + kChunkElems - 1) / kChunkElems;
  p->chunks.assign(static_cast<size_t>(n_chunks), ChunkDesc{-1, -1});
  int t = 0;
  for (int64_t c = 0; c < n_chunks; ++c) {
    const int64_t lo = c * kChunkElems, hi = lo + kChunkElems;
    // skip tensors that end at or before this chunk (and empty ones)
    while (t < n && p->voff[t] + p->numel[t] <= lo) ++t;
    if (t >= n || p->voff[t] >= hi) continue;  // gap: empty chunk
    // span = tensor indices [t, t + span) whose ranges may intersect the chunk
    // (empty tensors inside the run are harmless: a lane's search picks the
    // LAST index with voff <= e, which is the non-empty one holding e)
    int span = 0;
    for (int u = t; u < n && p->voff[u] < hi; ++u) span = u - t + 1;
    ChunkDesc& d = p->chunks[static_cast<size_t>(c)];
    d.t0 = t;
    const bool full = p->voff[t] <= lo && p->voff[t] + p->numel[t] >= hi;
    d.code = full ? 0 : span;
  }
}

// Task size (units) of a plan.  Every task is one workgroup's work; 256 CUs
// hold 2048 resident workgroups (256 CUs x 8).  Plans up to
// ~1920 x 16 Ki elements are cut into ~kTargetTasks tasks: one wave of
// workgroups evenly spread over the CUs (no second partial round), rounded to
// whole 256-lane iterations.  Larger plans keep 16 Ki-element tasks
// (kSegUnits): the interleaved sweep (profiles/r1d_sweep_tasks_nt.jsonl)
// puts 64 Ki-element tasks 20-25 % below 8-16 Ki-element ones on pack/unpack
// of 120 M-element plans, while a second round of tasks costs little there.
// Optimizer-update plans ask for 512-unit tasks instead (gs_plan_create_ex,
// multi_tensor.UPDATE_TASK_UNITS): five streams per element make the
// per-task descriptor prologue cheap relative to the data, and a short task
// per workgroup streams +2-8 % faster (profiles/r1r_grid_sweep.jsonl).
int64_t plan_task_units(int64_t total_units) {
  const int64_t target = kTargetTasks;
  int64_t u = (total_units + target - 1) / target;
  u = (u + kBlock - 1) / kBlock * kBlock;
  return std::max<int64_t>(kMinTaskUnits, std::min<int64_t>(kSegUnits, u));
}

extern "C" {

int gs_version(void) { return GSYNC_VERSION; }
const char* gs_last_error(void) { return gs::g_last_error.c_str(); }
int gs_device_count(void) { return hip_device_count(); }

int gs_plan_create(int device_kind, int device, int n_tensors, const int64_t* numels,
                   int64_t align_elems, gs_plan** out) {
  return gs_plan_create_ex(device_kind, device, n_tensors, numels, align_elems, 0, out);
}

int gs_plan_create_ex(int device_kind, int device, int n_tensors, const int64_t* numels,
                      int64_t align_elems, int64_t task_units_req, gs_plan** out) {
  GS_CHECK_ARG(task_units_req >= 0 && task_units_req <= (int64_t(1) << 20),
               "gs_plan_create_ex: task_units out of [0, 2^20]");
  GS_CHECK_ARG(out != nullptr, "gs_plan_create: out is NULL");
  GS_CHECK_ARG(n_tensors >= 0, "gs_plan_create: n_tensors < 0");
  GS_CHECK_ARG(n_tensors == 0 || numels != nullptr, "gs_plan_create: numels is NULL");
  GS_CHECK_ARG(device_kind == GS_DEV_HOST || device_kind == GS_DEV_HIP,
               "gs_plan_create: bad device_kind");
  GS_CHECK_ARG(align_elems >= 0 && (align_elems == 0 || align_elems % kUnit == 0),
               "gs_plan_create: align_elems must be 0 or a multiple of 4");
  if (device_kind == GS_DEV_HIP && hip_device_count() <= device)
    return fail(GS_ENODEV, "gs_plan_create: HIP device " + std::to_string(device) +
                               " not available");
  gs_plan* p = new (std::nothrow) gs_plan();
  if (!p) return fail(GS_ENOMEM, "gs_plan_create: out of host memory");
  p->kind = device_kind;
  p->device = device;
  p->n = n_tensors;
  p->align_elems = align_elems;
  p->numel.assign(numels, numels + n_tensors);
  p->off.resize(n_tensors);
  int64_t cur = 0;
  auto rup = [&](int64_t x) { return align_elems ? (x + align_elems - 1) / align_elems * align_elems : x; };
  for (int t = 0; t < n_tensors; ++t) {
    if (numels[t] < 0) {
      delete p;
      return fail(GS_EINVAL, "gs_plan_create: negative numel");
    }
    cur = rup(cur);
    p->off[t] = cur;
    cur += numels[t];
    p->elems += numels[t];
  }
  p->flat_numel = rup(cur);
  // segments and tasks
  int64_t total_units = 0;
  for (int t = 0; t < n_tensors; ++t) total_units += (numels[t] + kUnit - 1) / kUnit;
  int64_t task_units =
      task_units_req > 0 ? std::max<int64_t>(kUnit, task_units_req) : plan_task_units(total_units);
  task_units += task_units & 1;  // even (see the segment padding below)
  p->task_units = task_units;
  for (int t = 0; t < n_tensors; ++t) {
    int64_t units = (numels[t] + kUnit - 1) / kUnit;
    if (units == 0) continue;
    // even unit counts: an 8-element lane-step (two units) never straddles
    // segments; the padding unit lies past the tensor's end and is masked
    units += units & 1;
    if (units > task_units) {
      // a tensor larger than a task is shared by M single-segment tasks in
      // interleaved chunks (part i takes lane-step chunks i, i+M, i+2M, ...):
      // the M workgroups sweep the tensor front to back together instead of M
      // far-apart streams (DRAM / Infinity-Cache locality; a torch-copy-like
      // access pattern) — Seg.pad = M, unit_begin = i, units = the tensor's
      const int64_t parts = (units + task_units - 1) / task_units;
      for (int64_t i = 0; i < parts; ++i) {
        Seg s{};
        s.unit_begin = i;
        s.tensor = t;
        s.units = static_cast<int32_t>(units);
        s.pad = static_cast<int32_t>(parts);
        p->segs.push_back(s);
      }
      continue;
    }
    for (int64_t u = 0; u < units; u += task_units) {
      Seg s{};
      s.unit_begin = u;
      s.tensor = t;
      s.units = static_cast<int32_t>(std::min<int64_t>(task_units, units - u));
      p->segs.push_back(s);
    }
  }
  p->task_begin.push_back(0);
  int64_t tu = 0;
  int32_t tc = 0;
  for (size_t i = 0; i < p->segs.size(); ++i) {
    Seg& s = p->segs[i];
    const bool alone = s.pad > 0;  // interleaved parts always own a task
    if (tc > 0 && (alone || tu + s.units > task_units || tc == kMaxSegPerTask)) {
      p->task_begin.push_back(static_cast<int32_t>(i));
      tu = 0;
      tc = 0;
    }
    s.task_off = static_cast<int32_t>(tu);
    tu += alone ? task_units : s.units;  // a part fills its task
    ++tc;
  }
  if (!p->segs.empty()) p->task_begin.push_back(static_cast<int32_t>(p->segs.size()));
  const int n_tasks = static_cast<int>(p->task_begin.size()) - 1;
  const int grid_cap = kMaxGrid;
  p->grid = std::max(1, std::min(n_tasks, grid_cap));
  build_chunk_map(p);
  p->grid_cap = grid_cap;
  p->h_ptrs.assign(static_cast<size_t>(GS_PLAN_SLOTS) * n_tensors, nullptr);
  p->h_align.assign(n_tensors, 0u);
  if (device_kind == GS_DEV_HIP) {
    int rc = hip_plan_upload_static(p);
    if (rc != GS_OK) {
      hip_plan_release(p);
      delete p;
      return rc;
    }
  }
  *out = p;
  return GS_OK;
}

int gs_plan_destroy(gs_plan* p) {
  if (!p) return GS_OK;
  if (p->kind == GS_DEV_HIP) {
    comm_forget_consumer(p);
    hip_plan_release(p);
  }
  delete p;
  return GS_OK;
}

int64_t gs_plan_flat_numel(gs_plan* p) { return p ? p->flat_numel : -1; }

int gs_plan_offsets(gs_plan* p, int64_t* out) {
  GS_CHECK_ARG(p && out, "gs_plan_offsets: NULL argument");
  std::copy(p->off.begin(), p->off.end(), out);
  return GS_OK;
}

int gs_plan_n_tasks(gs_plan* p) { return p ? static_cast<int>(p->task_begin.size()) - 1 : -1; }

int64_t gs_plan_task_units(gs_plan* p) { return p ? p->task_units : -1; }

int gs_plan_timer_enable(gs_plan* p, int n_slots) {
  GS_CHECK_ARG(p != nullptr, "gs_plan_timer_enable: NULL plan");
  GS_CHECK_ARG(n_slots >= 0 && n_slots <= 4096, "gs_plan_timer_enable: n_slots out of [0, 4096]");
  if (p->kind != GS_DEV_HIP) return fail(GS_EINVAL, "gs_plan_timer_enable: host plans have no launch timer");
  return hip_plan_timer_enable(p, n_slots);
}

int gs_plan_timer_read(gs_plan* p, float* ms_out, int32_t* kind_out, int cap) {
  GS_CHECK_ARG(p != nullptr && (cap == 0 || ms_out != nullptr), "gs_plan_timer_read: NULL argument");
  if (p->kind != GS_DEV_HIP) return fail(GS_EINVAL, "gs_plan_timer_read: host plans have no launch timer");
  return hip_plan_timer_read(p, ms_out, kind_out, cap);
}

int gs_plan_set_ptrs(gs_plan* p, int slot, void* const* ptrs, void* /*stream*/) {
  GS_CHECK_ARG(p != nullptr, "gs_plan_set_ptrs: NULL plan");
  GS_CHECK_ARG(slot >= 0 && slot < GS_PLAN_SLOTS, "gs_plan_set_ptrs: slot out of range");
  GS_CHECK_ARG(p->n == 0 || ptrs != nullptr, "gs_plan_set_ptrs: NULL ptrs");
  void** row = p->h_ptrs.data() + static_cast<size_t>(slot) * p->n;
  for (int t = 0; t < p->n; ++t) {
    if (row[t] != ptrs[t]) {
      row[t] = ptrs[t];
      const uint32_t bit = 1u << slot;
      const bool al = (reinterpret_cast<uintptr_t>(ptrs[t]) & 15u) == 0;
      p->h_align[t] = al ? (p->h_align[t] | bit) : (p->h_align[t] & ~bit);
      p->dirty = true;
    }
  }
  return GS_OK;
}

#define PLAN_OK(p) GS_CHECK_ARG((p) != nullptr, "NULL plan")
#define SLOT_OK(s) GS_CHECK_ARG((s) >= 0 && (s) < GS_PLAN_SLOTS, "slot out of range")

int gs_pack(gs_plan* p, int src_slot, int src_dtype, void* flat, int flat_dtype, float scale,
            int scale_mode, void* stream) {
  GsRange range("gs_pack");
  PLAN_OK(p);
  SLOT_OK(src_slot);
  GS_CHECK_ARG(flat != nullptr || p->flat_numel == 0, "gs_pack: NULL flat buffer");
  GS_CHECK_ARG(scale_mode >= GS_SCALE_NONE && scale_mode <= GS_SCALE_DIV, "gs_pack: bad scale_mode");
  if (p->kind == GS_DEV_HOST) return host_pack(p, src_slot, src_dtype, flat, flat_dtype, scale, scale_mode);
  return hip_pack(p, src_slot, src_dtype, flat, flat_dtype, scale, scale_mode, stream);
}

int gs_unpack(gs_plan* p, const void* flat, int flat_dtype, int dst_slot, int dst_dtype,
              float* sqnorm_dev, int accumulate, void* stream) {
  GsRange range("gs_unpack");
  PLAN_OK(p);
  SLOT_OK(dst_slot);
  GS_CHECK_ARG(flat != nullptr || p->flat_numel == 0, "gs_unpack: NULL flat buffer");
  if (p->kind == GS_DEV_HOST)
    return host_unpack(p, flat, flat_dtype, dst_slot, dst_dtype, sqnorm_dev, accumulate);
  return hip_unpack(p, flat, flat_dtype, dst_slot, dst_dtype, sqnorm_dev, accumulate, stream);
}

int gs_unpack_check(gs_plan* p, const void* flat, int flat_dtype, int dst_slot, int dst_dtype,
                    float* found_inf, void* stream) {
  GsRange range("gs_unpack_check");
  PLAN_OK(p);
  SLOT_OK(dst_slot);
  GS_CHECK_ARG(flat != nullptr || p->flat_numel == 0, "gs_unpack_check: NULL flat buffer");
  GS_CHECK_ARG(found_inf != nullptr, "gs_unpack_check: NULL found_inf");
  if (p->kind == GS_DEV_HOST) return host_unpack_check(p, flat, flat_dtype, dst_slot, dst_dtype, found_inf);
  return hip_unpack_check(p, flat, flat_dtype, dst_slot, dst_dtype, found_inf, stream);
}

int gs_scale(gs_plan* p, int slot, int dtype, float s, int scale_mode, void* stream) {
  GsRange range("gs_scale");
  PLAN_OK(p);
  SLOT_OK(slot);
  GS_CHECK_ARG(scale_mode == GS_SCALE_MUL || scale_mode == GS_SCALE_DIV, "gs_scale: bad scale_mode");
  if (p->kind == GS_DEV_HOST) return host_scale(p, slot, dtype, s, scale_mode);
  return hip_scale(p, slot, dtype, s, scale_mode, stream);
}

int gs_sqnorm(gs_plan* p, int slot, int dtype, float* sqnorm_dev, int accumulate, void* stream) {
  GsRange range("gs_sqnorm");
  PLAN_OK(p);
  SLOT_OK(slot);
  GS_CHECK_ARG(sqnorm_dev != nullptr, "gs_sqnorm: NULL output");
  p->grads_read = slot == 1;
  if (p->kind == GS_DEV_HOST) return host_sqnorm(p, slot, dtype, sqnorm_dev, accumulate);
  return hip_sqnorm(p, slot, dtype, sqnorm_dev, accumulate, stream);
}

int gs_sqnorm_partial(gs_plan* p, int slot, int dtype, void* stream) {
  GsRange range("gs_sqnorm_partial");
  PLAN_OK(p);
  SLOT_OK(slot);
  p->red_valid = true;
  p->grads_read = slot == 1;
  if (p->kind == GS_DEV_HOST) {
    p->red_groups = 0;
    return host_sqnorm(p, slot, dtype, &p->h_red, 0);
  }
  return hip_sqnorm_partial(p, slot, dtype, nullptr, nullptr, stream);
}

int gs_sqnorm_partial_out(gs_plan* p, int slot, int dtype, float* groups_out, int32_t* n_groups,
                          void* stream) {
  GsRange range("gs_sqnorm_partial_out");
  PLAN_OK(p);
  SLOT_OK(slot);
  GS_CHECK_ARG(groups_out != nullptr && n_groups != nullptr, "gs_sqnorm_partial_out: NULL argument");
  p->red_valid = true;
  p->grads_read = slot == 1;
  if (p->kind == GS_DEV_HOST) {
    p->red_groups = 0;
    GS_TRY_RET(host_sqnorm(p, slot, dtype, &p->h_red, 0));
    groups_out[0] = p->h_red;
    std::fill(groups_out + 1, groups_out + GS_RED_PARTIALS, 0.f);
    *n_groups = 1;
    return GS_OK;
  }
  return hip_sqnorm_partial(p, slot, dtype, groups_out, n_groups, stream);
}

int gs_plan_set_read_hint(gs_plan* p, int hint) {
  PLAN_OK(p);
  GS_CHECK_ARG(hint >= 0 && hint <= 2, "gs_plan_set_read_hint: hint 0, 1 or 2");
  p->read_hint = hint;
  return GS_OK;
}

int gs_plan_set_clip(gs_plan* p, const float* sqnorm_dev, float max_norm, float eps, float sq_mul,
                     float coef_mul, float* out_dev) {
  PLAN_OK(p);
  if (!(max_norm > 0.f)) {
    p->clip_on = false;
    return GS_OK;
  }
  GS_CHECK_ARG(eps >= 0.f, "gs_plan_set_clip: eps < 0");
  p->clip_on = true;
  p->clip_own = sqnorm_dev == nullptr;
  p->clip = ClipArgs{sqnorm_dev, 0, 1, max_norm, eps, sq_mul, coef_mul, out_dev};
  return GS_OK;
}

int gs_plan_set_clip_groups(gs_plan* p, const float* groups_dev, int32_t n_groups, float max_norm,
                            float eps, float sq_mul, float coef_mul, float* out_dev) {
  PLAN_OK(p);
  if (!(max_norm > 0.f)) {
    p->clip_on = false;
    return GS_OK;
  }
  GS_CHECK_ARG(groups_dev != nullptr, "gs_plan_set_clip_groups: NULL group sums");
  GS_CHECK_ARG(n_groups >= 1 && n_groups <= GS_RED_PARTIALS, "gs_plan_set_clip_groups: n_groups out of 1..GS_RED_PARTIALS");
  GS_CHECK_ARG(eps >= 0.f, "gs_plan_set_clip_groups: eps < 0");
  p->clip_on = true;
  p->clip_own = false;
  p->clip = ClipArgs{groups_dev, n_groups, 1, max_norm, eps, sq_mul, coef_mul, out_dev};
  return GS_OK;
}

// the clip of the next update on plan p (nullptr: none)
static int plan_clip(gs_plan* p, ClipArgs* c, const ClipArgs** out) {
  *out = nullptr;
  if (!p->clip_on) return GS_OK;
  *c = p->clip;
  if (p->clip_own) {
    // the plan's own partial sums serve ONE update: a later update without a fresh
    // gs_sqnorm_partial fails instead of clipping with stale sums (and any other
    // fused reduction on the plan in between overwrote them: gs_kernels.hip launch)
    if (!p->red_valid)
      return fail(GS_ESTATE, "clipped update from the plan's own Σg²: call gs_sqnorm_partial first "
                             "(once per update; a fused reduction on the plan in between overwrites it)");
    p->red_valid = false;
    if (p->kind == GS_DEV_HOST) {
      c->sq = &p->h_red;
      c->groups = 0;
    } else {
      if (p->red_groups > kRedMaxGroups)
        return fail(GS_ESTATE, "clipped update from the plan's own Σg²: more group sums than the plan keeps");
      c->groups = p->red_groups;
      c->stride = 1;  // the contiguous copy (hip_plan_red_groups)
      c->sq = p->red_groups > 0 ? hip_plan_red_groups(p) : hip_plan_red_scalar(p);
    }
  }
  *out = c;
  return GS_OK;
}

int gs_clip_scale(gs_plan* p, int slot, int dtype, void* stream) {
  GsRange r("gs_clip_scale");
  PLAN_OK(p);
  SLOT_OK(slot);
  GS_CHECK_ARG(p->clip_on, "gs_clip_scale: no clip set on the plan (gs_plan_set_clip / gs_plan_set_clip_groups)");
  ClipArgs cs;
  const ClipArgs* clip;
  GS_TRY_RET(plan_clip(p, &cs, &clip));
  cs = *clip;
  cs.torch_clamp = 1;  // torch.clamp(coef, max=1): a NaN norm scales every grad by NaN, as torch
  if (p->kind == GS_DEV_HOST) return host_clip_scale(p, slot, dtype, cs);
  return hip_clip_scale(p, slot, dtype, cs, stream);
}

int gs_sum(gs_plan* p, int slot, int dtype, float* sum_dev, int accumulate, void* stream) {
  PLAN_OK(p);
  SLOT_OK(slot);
  GS_CHECK_ARG(sum_dev != nullptr, "gs_sum: NULL output");
  GsRange r("gs_sum");
  if (p->kind == GS_DEV_HOST) return host_sum(p, slot, dtype, sum_dev, accumulate);
  return hip_sum(p, slot, dtype, sum_dev, accumulate, stream);
}

int gs_clip_coef(int device_kind, const float* sqnorm_dev, float max_norm, float eps,
                 float* coef_dev, float* norm_dev, void* stream) {
  GS_CHECK_ARG(sqnorm_dev && coef_dev, "gs_clip_coef: NULL argument");
  if (device_kind == GS_DEV_HOST)
    return host_clip_coef(sqnorm_dev, max_norm, eps, coef_dev, norm_dev);
  return hip_clip_coef(sqnorm_dev, max_norm, eps, coef_dev, norm_dev, stream);
}

int gs_adam_hyper(int device_kind, double* step, const double* lr, double beta1, double beta2,
                  double weight_decay, const float* found_inf, float* hyper, void* stream) {
  GS_CHECK_ARG(step && lr && hyper, "gs_adam_hyper: NULL argument");
  if (device_kind == GS_DEV_HOST) {
    adam_hyper_update(step, lr, beta1, beta2, weight_decay, found_inf, hyper);
    return GS_OK;
  }
  return hip_adam_hyper(step, lr, beta1, beta2, weight_decay, found_inf, hyper, stream);
}

int gs_unscale_check(gs_plan* p, int slot, int dtype, const float* inv_scale_dev,
                     float* found_inf_dev, void* stream) {
  GsRange range("gs_unscale_check");
  PLAN_OK(p);
  SLOT_OK(slot);
  GS_CHECK_ARG(found_inf_dev != nullptr, "gs_unscale_check: NULL found_inf");
  if (p->kind == GS_DEV_HOST) return host_unscale_check(p, slot, dtype, inv_scale_dev, found_inf_dev);
  return hip_unscale_check(p, slot, dtype, inv_scale_dev, found_inf_dev, stream);
}

int gs_sgd_step(gs_plan* p, int grad_dtype, int lowp_dtype, double lr, double momentum,
                double dampening, double weight_decay, int nesterov, int maximize, int first_step,
                const float* grad_scale_dev, const float* found_inf_dev, void* stream) {
  GsRange range("gs_sgd_step");
  PLAN_OK(p);
  GS_CHECK_ARG(!nesterov || (momentum > 0 && dampening == 0),
               "Nesterov momentum requires a momentum and zero dampening");
  GS_CHECK_ARG(first_step >= 0 || (first_step == -1 && p->hyper != nullptr),
               "gs_sgd_step: first_step = -1 (device flag) needs a hyper source");
  SgdHyper h = make_sgd(lr, momentum, dampening, weight_decay, nesterov, maximize, first_step);
  if (p->kind == GS_DEV_HOST && p->hyper) {
    h.lr = p->hyper[0];
    if (h.first < 0) h.first = p->hyper[1] != 0.f;
  }
  ClipArgs cs;
  const ClipArgs* clip;
  GS_TRY_RET(plan_clip(p, &cs, &clip));
  if (p->kind == GS_DEV_HOST) return host_sgd(p, grad_dtype, lowp_dtype, h, grad_scale_dev, found_inf_dev, clip);
  return hip_sgd(p, grad_dtype, lowp_dtype, h, grad_scale_dev, found_inf_dev, clip, stream);
}

int gs_adam_step(gs_plan* p, int grad_dtype, int lowp_dtype, double lr, double beta1,
                 double beta2, double eps, double weight_decay, int adamw, int maximize,
                 double step_size, double bias_correction2_sqrt, const float* grad_scale_dev,
                 const float* found_inf_dev, void* stream) {
  GsRange range("gs_adam_step");
  PLAN_OK(p);
  GS_CHECK_ARG(bias_correction2_sqrt > 0, "gs_adam_step: bias_correction2_sqrt must be > 0");
  AdamHyper h = make_adam(lr, beta1, beta2, eps, weight_decay, adamw, maximize, step_size,
                          bias_correction2_sqrt);
  if (p->kind == GS_DEV_HOST && p->hyper) {
    h.step_size = p->hyper[0];
    h.bc2s = p->hyper[1];
    h.decay = p->hyper[2];
  }
  ClipArgs cs;
  const ClipArgs* clip;
  GS_TRY_RET(plan_clip(p, &cs, &clip));
  if (p->kind == GS_DEV_HOST) return host_adam(p, grad_dtype, lowp_dtype, h, grad_scale_dev, found_inf_dev, clip);
  return hip_adam(p, grad_dtype, lowp_dtype, h, grad_scale_dev, found_inf_dev, clip, stream);
}

int gs_plan_set_hyper_source(gs_plan* p, const float* hyper) {
  PLAN_OK(p);
  p->hyper = hyper;
  return GS_OK;
}

int gs_stream_wait(void* waiter, void* signaler) { return hip_stream_wait(waiter, signaler); }

// Restatement of compute_bucket_assignment_by_size (torch c10d reducer.cpp,
// declared at T:include/torch/csrc/distributed/c10d/reducer.hpp:590-595):
// per (dtype, device) key a bucket accumulates tensors until its byte size
// reaches the current limit (>=, so a bucket may exceed it); each key then
// advances to the next limit.  Leftover buckets are appended; without an
// explicit order the result is sorted by the smallest tensor index.
int gs_compute_bucket_assignment(int n, const int64_t* nbytes, const int32_t* dtype_keys,
                                 const int32_t* order, int n_limits, const int64_t* limits,
                                 int32_t* bucket_of, int32_t* bucket_members,
                                 int32_t* bucket_counts) {
  GS_CHECK_ARG(n >= 0 && nbytes && n_limits > 0 && limits, "gs_compute_bucket_assignment: bad args");
  struct Acc {
    std::vector<int32_t> idx;
    int64_t size = 0;
    int lim = 0;
  };
  std::map<int32_t, Acc> acc;  // key -> open bucket
  std::vector<int32_t> key_order;
  std::vector<std::vector<int32_t>> result;
  for (int i = 0; i < n; ++i) {
    const int32_t t = order ? order[i] : i;
    GS_CHECK_ARG(t >= 0 && t < n, "gs_compute_bucket_assignment: order out of range");
    const int32_t key = dtype_keys ? dtype_keys[t] : 0;
    auto it = acc.find(key);
    if (it == acc.end()) {
      it = acc.emplace(key, Acc{}).first;
      key_order.push_back(key);
    }
    Acc& b = it->second;
    b.idx.push_back(t);
    b.size += nbytes[t];
    if (b.size >= limits[b.lim]) {
      result.push_back(std::move(b.idx));
      b.idx.clear();
      b.size = 0;
      if (b.lim + 1 < n_limits) ++b.lim;
    }
  }
  for (int32_t key : key_order) {
    Acc& b = acc[key];
    if (!b.idx.empty()) result.push_back(std::move(b.idx));
  }
  if (!order) {
    std::stable_sort(result.begin(), result.end(),
                     [](const std::vector<int32_t>& a, const std::vector<int32_t>& b) {
                       return *std::min_element(a.begin(), a.end()) <
                              *std::min_element(b.begin(), b.end());
                     });
  }
  int pos = 0;
  for (size_t bi = 0; bi < result.size(); ++bi) {
    if (bucket_counts) bucket_counts[bi] = static_cast<int32_t>(result[bi].size());
    for (int32_t t : result[bi]) {
      if (bucket_of) bucket_of[t] = static_cast<int32_t>(bi);
      if (bucket_members) bucket_members[pos] = t;
      ++pos;
    }
  }
  return static_cast<int>(result.size());
}

}  // extern "C"
