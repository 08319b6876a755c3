// gfx950 (CDNA4) kernels of libgsync: multi-tensor pack / unpack / scale / sq-norm /
// unscale, the plan's device memory and pointer-table uploads.  The engine and the
// ops live in gs_engine.h; the fused updates in gs_update_kernels.hip.

#include "gs_engine.h"

namespace gs {

// ------------------------------------------------------------- plan memory
int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int hip_memset_async(void* dst, int value, size_t bytes, void* stream) {
  HIP_RET(hipMemsetAsync(dst, value, bytes, static_cast<hipStream_t>(stream)));
  return GS_OK;
}

int hip_stream_wait(void* waiter, void* signaler) {
  if (waiter == signaler) return GS_OK;
  hipEvent_t ev;
  HIP_RET(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  hipError_t e1 = hipEventRecord(ev, static_cast<hipStream_t>(signaler));
  hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(static_cast<hipStream_t>(waiter), ev, 0)
                                   : e1;
  (void)hipEventDestroy(ev);  // destruction is deferred until the event completes
  if (e2 != hipSuccess) return fail(GS_EHIP, std::string("stream wait: ") + hipGetErrorString(e2));
  return GS_OK;
}

static size_t table_bytes(const gs_plan* p) {
  return sizeof(void*) * GS_PLAN_SLOTS * p->n + sizeof(uint32_t) * p->n;
}

int hip_plan_upload_static(gs_plan* p) {
  DeviceGuard g(p->device);
  const size_t sz_segs = sizeof(Seg) * p->segs.size();
  const size_t sz_tb = sizeof(int32_t) * p->task_begin.size();
  const size_t sz_n = sizeof(int64_t) * p->n;
  const size_t sz_ch = sizeof(ChunkDesc) * p->chunks.size();
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  // segs | task_begin | numel | off | chunks | voff (layout of gs_plan::args)
  const size_t total = al(sz_segs) + al(sz_tb) + al(sz_n) * 3 + al(sz_ch);
  HIP_RET(hipMalloc(&p->d_static, total));
  char* base = static_cast<char*>(p->d_static);
  std::vector<char> h(total, 0);
  size_t o = 0;
  if (sz_segs) std::memcpy(h.data() + o, p->segs.data(), sz_segs);
  o += al(sz_segs);
  std::memcpy(h.data() + o, p->task_begin.data(), sz_tb);
  o += al(sz_tb);
  if (sz_n) std::memcpy(h.data() + o, p->numel.data(), sz_n);
  o += al(sz_n);
  if (sz_n) std::memcpy(h.data() + o, p->off.data(), sz_n);
  o += al(sz_n);
  if (sz_ch) std::memcpy(h.data() + o, p->chunks.data(), sz_ch);
  o += al(sz_ch);
  if (sz_n) std::memcpy(h.data() + o, p->voff.data(), sz_n);
  HIP_RET(hipMemcpy(base, h.data(), total, hipMemcpyHostToDevice));
  const size_t tb = table_bytes(p) + 16;
  HIP_RET(hipMalloc(&p->d_table, tb));
  HIP_RET(hipMemset(p->d_table, 0, tb));
  // per-workgroup partials + the fused reduction's counters / group sums (zeroed once;
  // every fused launch leaves them at zero)
  // (+ one more line: the Σg² scalar of gs_sqnorm_partial when the chunk engine is off,
  // + the contiguous copy of its group sums that a clipped launch folds)
  HIP_RET(hipMalloc(reinterpret_cast<void**>(&p->d_partials),
                    sizeof(float) * (kGridLimit + kRedSyncWords + kRedSyncStride + GS_RED_PARTIALS)));
  HIP_RET(hipMemset(p->d_partials + kGridLimit, 0, sizeof(float) * kRedSyncWords));
  HIP_RET(hipHostMalloc(&p->pinned, tb * 4, hipHostMallocDefault));
  for (int i = 0; i < 4; ++i) {
    hipEvent_t ev;
    HIP_RET(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    p->ring_events[i] = ev;
  }
  hipEvent_t ev;
  HIP_RET(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  p->last_event = ev;
  return GS_OK;
}

int hip_plan_timer_enable(gs_plan* p, int n_slots) {
  DeviceGuard g(p->device);
  for (void* ev : p->timer_ev) {
    (void)hipEventSynchronize(static_cast<hipEvent_t>(ev));
    (void)hipEventDestroy(static_cast<hipEvent_t>(ev));
  }
  p->timer_ev.clear();
  p->timer_kind.assign(n_slots, 0);
  p->timer_next = p->timer_count = 0;
  for (int i = 0; i < 2 * n_slots; ++i) {
    hipEvent_t ev;
    HIP_RET(hipEventCreate(&ev));
    p->timer_ev.push_back(ev);
  }
  return GS_OK;
}

int hip_plan_timer_read(gs_plan* p, float* ms_out, int32_t* kind_out, int cap) {
  DeviceGuard g(p->device);
  const int nslots = static_cast<int>(p->timer_ev.size() / 2);
  if (nslots == 0) return 0;
  const int n = std::min(p->timer_count, cap);
  // oldest recorded pair first
  const int first = (p->timer_next - p->timer_count + nslots) % nslots;
  for (int i = 0; i < n; ++i) {
    const int k = (first + i) % nslots;
    hipEvent_t a = static_cast<hipEvent_t>(p->timer_ev[2 * k]);
    hipEvent_t b = static_cast<hipEvent_t>(p->timer_ev[2 * k + 1]);
    HIP_RET(hipEventSynchronize(b));
    float ms = 0.f;
    HIP_RET(hipEventElapsedTime(&ms, a, b));
    ms_out[i] = ms;
    if (kind_out) kind_out[i] = p->timer_kind[k];
  }
  p->timer_count = 0;
  return n;
}

int hip_plan_release(gs_plan* p) {
  DeviceGuard g(p->device);
  (void)hip_plan_timer_enable(p, 0);
  // make sure nothing in flight still reads the tables: an event behind the plan's
  // last launch (hipFree below synchronises the device as well, hip_runtime_api.h)
  if (p->last_event && p->last_stream != nullptr && !stream_destroyed(p->last_stream) && !p->last_captured &&
      !stream_capturing(p->last_stream) &&
      hipEventRecord(static_cast<hipEvent_t>(p->last_event), static_cast<hipStream_t>(p->last_stream)) ==
          hipSuccess)
    (void)hipEventSynchronize(static_cast<hipEvent_t>(p->last_event));
  for (int i = 0; i < 4; ++i) {
    if (p->ring_events[i]) {
      (void)hipEventSynchronize(static_cast<hipEvent_t>(p->ring_events[i]));
      (void)hipEventDestroy(static_cast<hipEvent_t>(p->ring_events[i]));
    }
  }
  if (p->last_event) (void)hipEventDestroy(static_cast<hipEvent_t>(p->last_event));
  if (p->d_static) (void)hipFree(p->d_static);
  if (p->d_table) (void)hipFree(p->d_table);
  if (p->d_partials) (void)hipFree(p->d_partials);
  if (p->pinned) (void)hipHostFree(p->pinned);
  return GS_OK;
}

// Table upload while the stream is being captured into a hipGraph: the table
// travels in kernel arguments (captured by value), ~3 KiB per launch, so the
// graph carries no reference to host staging memory and no host sync is
// needed; a replay rewrites the same (static) pointers.
constexpr int kTableWordsPerLaunch = 384;  // 3 KiB of 8-byte words
struct TableChunk {
  uint64_t words[kTableWordsPerLaunch];
  int64_t first;  // first 8-byte word of the table this chunk writes
  int32_t count;
};
__global__ void __launch_bounds__(128) table_write_kernel(uint64_t* table, TableChunk c) {
  for (int i = threadIdx.x; i < c.count; i += blockDim.x) table[c.first + i] = c.words[i];
}

bool stream_capturing(void* stream) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(static_cast<hipStream_t>(stream), &st) == hipSuccess &&
         st == hipStreamCaptureStatusActive;
}

// Pointer-table upload before a launch.  Eager: staged through a pinned ring
// and copied on the launch stream.  Under hipGraph capture: written by
// table_write_kernel launches (once per plan per capture), so every replay
// restores the table the captured kernels were recorded against even if eager
// launches changed it in between; the plan then re-uploads before its next
// eager launch, since a replay may have overwritten the eager table.
int hip_plan_flush(gs_plan* p, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  if (hipStreamGetCaptureInfo(s, &st, &cid) != hipSuccess) st = hipStreamCaptureStatusNone;
  const bool capturing = st == hipStreamCaptureStatusActive;
  // a launch on a new stream is ordered after the plan's previous launch when
  // both are eager or both belong to the capture (an event recorded inside a
  // capture cannot order eager work: graph replays are ordered by the caller,
  // as torch.cuda.graph requires)
  // The event is recorded on the previous stream now, not after every launch (a packet
  // per launch cost ~4.7 µs of stream time, scripts/micro/event_chain.hip): it
  // follows everything enqueued there so far, the plan's last launch included.  A
  // previous stream that entered or left a capture since cannot order this launch.
  if (p->last_stream != nullptr && stream_destroyed(p->last_stream)) p->last_stream = nullptr;  // nothing pending there
  if (p->last_stream != nullptr && p->last_stream != stream && capturing == p->last_captured &&
      (!capturing || cid == p->table_capture_id) &&
      stream_capturing(p->last_stream) == p->last_captured) {
    HIP_RET(hipEventRecord(static_cast<hipEvent_t>(p->last_event), static_cast<hipStream_t>(p->last_stream)));
    HIP_RET(hipStreamWaitEvent(s, static_cast<hipEvent_t>(p->last_event), 0));
  }
  const size_t ptr_bytes = sizeof(void*) * GS_PLAN_SLOTS * p->n;
  const size_t tb = table_bytes(p);
  if (capturing) {
    if (!p->dirty && p->table_capture_id == cid) return GS_OK;
    std::vector<uint64_t> words((tb + 7) / 8, 0);
    std::memcpy(words.data(), p->h_ptrs.data(), ptr_bytes);
    std::memcpy(reinterpret_cast<char*>(words.data()) + ptr_bytes, p->h_align.data(),
                sizeof(uint32_t) * p->n);
    for (size_t w = 0; w < words.size(); w += kTableWordsPerLaunch) {
      TableChunk c{};
      c.first = static_cast<int64_t>(w);
      c.count = static_cast<int32_t>(std::min<size_t>(kTableWordsPerLaunch, words.size() - w));
      std::memcpy(c.words, words.data() + w, sizeof(uint64_t) * c.count);
      hipLaunchKernelGGL(table_write_kernel, dim3(1), dim3(128), 0, s,
                         static_cast<uint64_t*>(p->d_table), c);
      HIP_RET(hipGetLastError());
    }
    p->table_capture_id = cid;
    p->in_graph = true;
    p->dirty = false;
    return GS_OK;
  }
  if (!p->dirty && !p->in_graph) return GS_OK;
  const int k = p->ring;
  HIP_RET(hipEventSynchronize(static_cast<hipEvent_t>(p->ring_events[k])));
  char* stage = static_cast<char*>(p->pinned) + k * (tb + 16);
  std::memcpy(stage, p->h_ptrs.data(), ptr_bytes);
  std::memcpy(stage + ptr_bytes, p->h_align.data(), sizeof(uint32_t) * p->n);
  HIP_RET(hipMemcpyAsync(p->d_table, stage, tb, hipMemcpyHostToDevice, s));
  HIP_RET(hipEventRecord(static_cast<hipEvent_t>(p->ring_events[k]), s));
  p->ring = (k + 1) & 3;
  p->dirty = false;
  return GS_OK;
}

// ------------------------------------------------------------- dispatchers
// An fp32 bucket whose plan fits one resident wave at groups of 2 chunks (<= 4 Ki
// chunks, 16 MB of fp32: the exposed last DDP bucket, ResNet-50's 9.7 MB) takes
// groups of 2 — half the workgroups, two accesses in flight per lane — where the
// large buckets keep one chunk per workgroup (the dispatcher refills CUs faster
// than a resident grid loops).  Level-2 tail, two rounds: pack 7.6-7.8 -> 7.0-7.2
// µs, the tail 35.9-36.8 -> 34.8-34.9 µs (profiles/r5/r5c_rows.jsonl, variant gpack2).
constexpr int64_t kPackG2MaxChunks = 4096;

template <int SD, int FD, int MODE, bool NT>
static int pack_mode(gs_plan* p, int src_slot, void* flat, float s, void* stream) {
  if constexpr (FD == GS_F32) {
    if (static_cast<int64_t>(p->chunks.size()) <= kPackG2MaxChunks) {
      PackOp<kUnit, SD, FD, MODE, NT, true> op;
      op.slot = src_slot; op.flat = flat; op.flat_vec = flat_aligned(flat); op.s = s;
      return launch(p, op, stream);
    }
  }
  PackOp<kUnit, SD, FD, MODE, NT> op;
  op.slot = src_slot; op.flat = flat; op.flat_vec = flat_aligned(flat); op.s = s;
  return launch(p, op, stream);
}

template <bool NT>
static int pack_nt(gs_plan* p, int src_slot, int src_dt, void* flat, int flat_dt, float s, int mode,
                   void* stream) {
  GS_DISPATCH_FLOAT(src_dt, SD, GS_DISPATCH_FLOAT(flat_dt, FD, {
    switch (mode) {
      case GS_SCALE_NONE: return pack_mode<SD, FD, GS_SCALE_NONE, NT>(p, src_slot, flat, s, stream);
      case GS_SCALE_MUL: return pack_mode<SD, FD, GS_SCALE_MUL, NT>(p, src_slot, flat, s, stream);
      case GS_SCALE_DIV: return pack_mode<SD, FD, GS_SCALE_DIV, NT>(p, src_slot, flat, s, stream);
      default: return fail(GS_EINVAL, "gs_pack: unknown scale mode");
    }
  }));
  return GS_OK;
}

// the source grads are read once: non-temporal loads above the cache size (nt_read_once)
int hip_pack(gs_plan* p, int src_slot, int src_dt, void* flat, int flat_dt, float s, int mode,
             void* stream) {
  DeviceGuard g(p->device);
  return nt_read_once(p->elems * dtype_bytes(src_dt))
             ? pack_nt<true>(p, src_slot, src_dt, flat, flat_dt, s, mode, stream)
             : pack_nt<false>(p, src_slot, src_dt, flat, flat_dt, s, mode, stream);
}

// RED = 1: Σ dst² into sq (nullable); RED = 2: the non-finite flag, accumulated
template <int RED, bool NT>
static int unpack_nt(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* red, int acc,
                     void* stream) {
  GS_DISPATCH_FLOAT(flat_dt, FD, GS_DISPATCH_FLOAT(dst_dt, DD, {
    UnpackOp<kUnit, FD, DD, RED, NT> op;
    op.want_red = red != nullptr; op.flat = flat; op.flat_vec = flat_aligned(flat); op.slot = dst_slot;
    return launch(p, op, stream, red, acc);
  }));
  return GS_OK;
}

// the flat buffer is read once: non-temporal loads above the cache size (nt_read_once)
int hip_unpack(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* sq,
               int acc, void* stream) {
  DeviceGuard g(p->device);
  return nt_read_once(p->flat_numel * dtype_bytes(flat_dt))
             ? unpack_nt<1, true>(p, flat, flat_dt, dst_slot, dst_dt, sq, acc, stream)
             : unpack_nt<1, false>(p, flat, flat_dt, dst_slot, dst_dt, sq, acc, stream);
}

int hip_unpack_check(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* found,
                     void* stream) {
  DeviceGuard g(p->device);
  // the flag accumulates (max), as torch's non-finite check does
  return nt_read_once(p->flat_numel * dtype_bytes(flat_dt))
             ? unpack_nt<2, true>(p, flat, flat_dt, dst_slot, dst_dt, found, 1, stream)
             : unpack_nt<2, false>(p, flat, flat_dt, dst_slot, dst_dt, found, 1, stream);
}

int hip_scale(gs_plan* p, int slot, int dt, float s, int mode, void* stream) {
  DeviceGuard g(p->device);
  GS_DISPATCH_FLOAT(dt, DT, {
    ScaleOp<kUnit, DT> op;
    op.slot = slot; op.s = s; op.mode = mode;
    return launch(p, op, stream);
  });
  return GS_OK;
}

template <bool NT>
static int sqnorm_nt(gs_plan* p, int slot, int dt, float* sq, int acc, int groups_only, void* stream) {
  GS_DISPATCH_FLOAT(dt, DT, {
    SqnormOp<kUnit, DT, NT> op;
    op.slot = slot;
    return launch(p, op, stream, sq, acc, groups_only);
  });
  return GS_OK;
}
// the slot is read once: non-temporal loads beyond the Infinity Cache (nt_read_once),
// or as the caller's hint says (who wrote the grads: gs_plan_set_read_hint);
// a non-temporal Σg² leaves the grads out of the caches, so the update that
// follows loads them non-temporally too (grads_read cleared)
static int sqnorm_launch(gs_plan* p, int slot, int dt, float* sq, int acc, int groups_only, void* stream) {
  if (!nt_read_once(p->elems * dtype_bytes(dt), true, p->read_hint))
    return sqnorm_nt<false>(p, slot, dt, sq, acc, groups_only, stream);
  p->grads_read = false;
  return sqnorm_nt<true>(p, slot, dt, sq, acc, groups_only, stream);
}

int hip_sqnorm(gs_plan* p, int slot, int dt, float* sq, int acc, void* stream) {
  DeviceGuard g(p->device);
  return sqnorm_launch(p, slot, dt, sq, acc, 0, stream);
}

// Σ x² of one slot left in the plan for a clipped update (gs_sqnorm_partial):
// the chunk kernel with the in-kernel combine stopped at its 64 group sums
// (no combine launch, no top-level hand-off); the update's workgroups fold them
// (clip_multiplier).  A reduction without the in-kernel combine (GS_RED_FUSE=0)
// or an empty plan writes the finished Σ into the plan's scalar word instead
// (red_groups = 0).
// The group sums as a clipped launch folds them: contiguous, one 256-B run for up to
// 64 groups (the fused reduction's own copies sit one per 128-B line, beside their
// counters: a fold over those took 64 lines per workgroup, every workgroup)
const float* hip_plan_red_groups(const gs_plan* p) {
  return p->d_partials + kGridLimit + kRedSyncWords + kRedSyncStride;
}
float* hip_plan_red_scalar(const gs_plan* p) { return p->d_partials + kGridLimit + kRedSyncWords; }

// Groups exactly when gs_sqnorm would run the in-kernel combine (same grid, same
// R: GS_RED_FUSE / GS_RED_GRID overrides apply to both), so the clipped update's
// fold equals gs_sqnorm's last step bit for bit; otherwise the combine launch
// writes the finished Σ (red_groups = 0).  groups_out (nullable): the group sums
// also contiguous in caller memory, or the finished Σ in groups_out[0].
int hip_sqnorm_partial(gs_plan* p, int slot, int dt, float* groups_out, int32_t* n_groups, void* stream) {
  DeviceGuard g(p->device);
  // NULL groups_out: the plan's own sums (gs_sqnorm_partial), written contiguously
  // by the group leaders beside their fused-reduction copies; never the raw form (the
  // fold must equal gs_sqnorm's combine bit for bit)
  const bool own = groups_out == nullptr;
  if (own) groups_out = const_cast<float*>(hip_plan_red_groups(p));
  // caller memory on a small plan (<= 4 Ki chunks: a ZeRO shard at N = 8): one partial per
  // workgroup of a balanced grid, no counters and no combine — the kernel ends with its
  // last store (groups of 8 chunks, one per workgroup, measured 0.7 µs slower: r5f)
  if (!own && !p->chunks.empty() && p->n > 0 && !p->segs.empty() &&
      static_cast<int64_t>(p->chunks.size()) <= kRawChunksMax) {
    GS_TRY_RET(sqnorm_launch(p, slot, dt, groups_out, 0, 2, stream));
    if (n_groups) *n_groups = p->red_groups;
    // the partials live only in the caller's buffer: the plan's own group sums were not
    // written, so a clip from them (gs_plan_set_clip(sqnorm = NULL)) fails with GS_ESTATE
    // instead of folding stale or out-of-range slots
    p->red_valid = false;
    p->red_groups = 0;
    return GS_OK;
  }
  const int cap = std::min(p->grid_cap, red_grid_cap(SqnormOp<kUnit, GS_F32>::kRedGrid));
  const bool groups = !p->chunks.empty() && p->n > 0 && !p->segs.empty() &&
                      red_fuse_groups() > 0 && cap <= kRedFuseMaxGrid;
  if (groups) {
    GS_TRY_RET(sqnorm_launch(p, slot, dt, groups_out, 0, 1, stream));
    if (n_groups) *n_groups = p->red_groups;
    return GS_OK;
  }
  p->red_groups = 0;
  if (n_groups) *n_groups = 1;
  GS_TRY_RET(sqnorm_launch(p, slot, dt, hip_plan_red_scalar(p), 0, 0, stream));
  if (!own) {  // the finished Σ in slot 0, the rest of the buffer 0
    HIP_RET(hipMemsetAsync(groups_out, 0, GS_RED_PARTIALS * sizeof(float), static_cast<hipStream_t>(stream)));
    HIP_RET(hipMemcpyAsync(groups_out, hip_plan_red_scalar(p), sizeof(float), hipMemcpyDeviceToDevice,
                           static_cast<hipStream_t>(stream)));
  }
  return GS_OK;
}

int hip_sum(gs_plan* p, int slot, int dt, float* out, int acc, void* stream) {
  DeviceGuard g(p->device);
  GS_DISPATCH_FLOAT(dt, DT, {
    SumOp<kUnit, DT> op;
    op.slot = slot;
    return launch(p, op, stream, out, acc);
  });
  return GS_OK;
}

int hip_clip_coef(const float* sq, float max_norm, float eps, float* coef, float* norm,
                  void* stream) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                     sq, max_norm, eps, coef, norm);
  HIP_RET(hipGetLastError());
  return GS_OK;
}

__global__ void adam_hyper_kernel(double* step, const double* lr, double beta1, double beta2, double wd,
                                  const float* found_inf, float* hyper) {
  if (threadIdx.x == 0) adam_hyper_update(step, lr, beta1, beta2, wd, found_inf, hyper);
}

int hip_adam_hyper(double* step, const double* lr, double beta1, double beta2, double wd,
                   const float* found_inf, float* hyper, void* stream) {
  hipLaunchKernelGGL(adam_hyper_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), step, lr,
                     beta1, beta2, wd, found_inf, hyper);
  HIP_RET(hipGetLastError());
  return GS_OK;
}

template <bool NT>
static int clip_scale_nt(gs_plan* p, int slot, int dt, const ClipArgs& clip, void* stream) {
  GS_DISPATCH_FLOAT(dt, DT, {
    ClipScaleOp<kUnit, DT, NT> op;
    op.slot = slot;
    op.clip = clip;
    return launch(p, op, stream);
  });
  return GS_OK;
}

int hip_clip_scale(gs_plan* p, int slot, int dt, const ClipArgs& clip, void* stream) {
  DeviceGuard g(p->device);
  return nt_read_once(p->elems * dtype_bytes(dt)) ? clip_scale_nt<true>(p, slot, dt, clip, stream)
                                                   : clip_scale_nt<false>(p, slot, dt, clip, stream);
}

int hip_unscale_check(gs_plan* p, int slot, int dt, const float* inv, float* found,
                      void* stream) {
  DeviceGuard g(p->device);
  GS_DISPATCH_FLOAT(dt, DT, {
    UnscaleOp<kUnit, DT> op;
    op.slot = slot; op.inv = inv;
    // found_inf accumulates (max) into the caller's flag, as torch's kernel does
    return launch(p, op, stream, found, 1);
  });
  return GS_OK;
}

}  // namespace gs
