// Internal declarations shared by the libgsync translation units.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gsync.h"

namespace gs {

// ---- roctx ranges (SURVEY.md §5 tracing): host-side ranges around every
// pack / collective / unpack / update enqueue, visible in
// `rocprofv3 --marker-trace`; off unless GSYNC_ROCTX=1 (one cached getenv)
bool roctx_enabled();
void roctx_push(const char* name);
void roctx_pop();
struct GsRange {
  bool on;
  explicit GsRange(const char* name) : on(roctx_enabled()) {
    if (on) roctx_push(name);
  }
  ~GsRange() {
    if (on) roctx_pop();
  }
  GsRange(const GsRange&) = delete;
  GsRange& operator=(const GsRange&) = delete;
};

// ---- error plumbing: thread-local message, int codes across the ABI ----
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define GS_CHECK_ARG(cond, msg)                                   \
  do {                                                            \
    if (!(cond)) return ::gs::fail(GS_EINVAL, std::string(msg));  \
  } while (0)

#define GS_TRY_RET(expr)          \
  do {                            \
    int _rc = (expr);             \
    if (_rc != GS_OK) return _rc; \
  } while (0)

inline int dtype_size(int dt) {
  switch (dt) {
    case GS_F32: return 4;
    case GS_BF16: return 2;
    case GS_F16: return 2;
    case GS_F64: return 8;
    case GS_I64: return 8;
    case GS_I32: return 4;
    case GS_U8: return 1;
    default: return 0;
  }
}
inline bool is_float_dtype(int dt) { return dt == GS_F32 || dt == GS_BF16 || dt == GS_F16; }

// ---- multi-tensor work decomposition ----
// A tensor is cut into segments of <= task_units units (1 unit = 4 elements;
// plan_task_units() sizes them per plan, at most kSegUnits).
// Consecutive segments are grouped into tasks of <= task_units units and
// <= kMaxSegPerTask segments; one workgroup processes one task at a time
// (small tensors share a task; their descriptors are staged in LDS).
constexpr int kUnit = 4;
constexpr int kSegUnits = 4096;   // max task: 16Ki elements = 64 KiB fp32 per stream
constexpr int kMinTaskUnits = 256;        // one unit per lane of a 256-thread workgroup
constexpr int kTargetTasks = 1920;  // < 2048 resident: ragged tensor ends add tasks
constexpr int kMaxSegPerTask = 64;
constexpr int kBlock = 256;         // 4 waves of 64
// default grid: one workgroup per task up to kGridLimit (the dispatcher refills
// CUs faster than a resident grid loops: profiles/r1r_copy_micro.jsonl,
// r1r_grid_sweep.jsonl)
constexpr int kMaxGrid = 65536;
constexpr int kGridLimit = 65536;   // hard cap (partials buffer)
// fused reductions: at most kRedMaxGroups group sums (one per lane of the
// folding wave), each counter / group sum on its own 128-B line
constexpr int kRedMaxGroups = GS_RED_GROUPS;
constexpr int kRedSyncStride = 32;

struct Seg {
  int64_t unit_begin;  // first unit inside the tensor (interleaved part: the part index)
  int32_t tensor;
  int32_t units;       // (interleaved part: the tensor's units)
  int32_t task_off;    // unit offset of this segment inside its task
  int32_t pad;         // 0 = contiguous segment; M > 0 = one of M interleaved parts
};
static_assert(sizeof(Seg) == 24, "Seg layout");

// ---- chunk-map engine (streaming ops) ----
// The plan's tensors are laid end to end in a VIRTUAL element space (voff):
// a tensor of >= kGroupElems elements starts on a kGroupElems boundary, one of
// >= kChunkElems on a kChunkElems boundary, a smaller one on a 4-element
// boundary.  The space is cut into chunks of kChunkElems (one 16-B access per
// lane of a 256-lane workgroup); a workgroup takes G consecutive chunks per
// iteration (G per op, gs_kernels.hip) and grid-strides.  A group of chunks
// that lies wholly inside one tensor is streamed with no per-lane lookup and
// no bounds checks: a wave-uniform base pointer (SGPRs) plus a 32-bit lane
// offset, G accesses per stream in flight; the rest (tensor tails, runs of
// small tensors) go chunk by chunk, resolving each lane's tensor by binary
// search over voff.
constexpr int kChunkElems = 256 * kUnit;    // 1 Ki elements
constexpr int kGroupElems = 4 * kChunkElems;  // largest group (G = 4)
struct ChunkDesc {
  int32_t t0;    // first tensor intersecting the chunk
  int32_t code;  // 0: full chunk inside t0; k > 0: k tensors intersect; -1: empty
};
static_assert(sizeof(ChunkDesc) == 8, "ChunkDesc layout");

// Arguments handed to a device kernel (by value).
struct PlanArgs {
  const Seg* segs;
  const int32_t* task_begin;  // [n_tasks + 1]
  const int64_t* numel;       // [n]
  const int64_t* off;         // [n] flat offsets (elements)
  void* const* ptrs;          // [GS_PLAN_SLOTS * n]
  const uint32_t* align;      // [n] bit s = slot s pointer is 16-B aligned
  const ChunkDesc* chunks;    // [n_chunks]
  const int64_t* voff;        // [n] virtual offsets (chunk-map engine)
  uint32_t* ticket;           // arrival counters of the fused reduction (0 between launches)
  float* red_out;             // fused reduction target (chunk engine), NULL = none
  int32_t red_acc;            // accumulate into red_out
  int32_t red_fuse;           // R > 0: combine in-kernel (two-level ticket, R groups), no combine launch
  int32_t red_groups_only;    // stop after the group level: the R group sums stay for a clipped update
  int32_t red_raw;            // one partial per workgroup straight to red_out (no counters, no combine)
  int32_t n;
  int32_t n_tasks;
  int32_t n_chunks;
};

// optimizer hyper-parameters, rounded to fp32 where torch rounds them
struct SgdHyper {
  float lr, mom, omd, wd;  // omd = float(1 - dampening) formed in double
  int nesterov, maximize, first;
};
struct AdamHyper {
  float b2, w1, w2, eps, wd, step_size, bc2s, decay;  // w1 = float(1-b1), decay = float(1-lr*wd)
  int adamw, maximize;
};
// Gradient-norm clip folded into an update launch (gs_plan_set_clip): the
// update's workgroups form the coefficient themselves, so no coefficient
// launch (and, with the plan's own group sums, no combine launch) sits between
// the Σg² kernel and the update.  Same arithmetic as the separate path
// (sq *= gscale², sq *= sq_mul; norm = sqrt(sq); coef = min(1, max/(norm+eps))
// * gscale * coef_mul, T:nn/utils/clip_grad.py:165-174), so it is bit-identical.
struct ClipArgs {
  const float* sq;     // a finished Σg² (groups == 0) or `groups` group sums, `stride` floats apart
  int32_t groups;
  int32_t stride;      // floats between consecutive group sums (1: contiguous; the plan's own copy and a caller's buffer)
  float max_norm, eps;
  float sq_mul, coef_mul;  // host multipliers (ZeRO's loss scale): 1 = none
  float* out;          // [sq, coef, norm] written by workgroup 0 (nullable)
  // 0: DeepSpeed's `if coef < 1: clip` (a NaN coefficient clips nothing); 1: torch's
  // clamp(coef, max=1) (clip_grad_norm_, T:nn/utils/clip_grad.py:172 — NaN stays NaN)
  int32_t torch_clamp;
};

inline SgdHyper make_sgd(double lr, double mom, double damp, double wd, int nest, int maxi,
                         int first) {
  return SgdHyper{static_cast<float>(lr), static_cast<float>(mom),
                  static_cast<float>(1.0 - damp), static_cast<float>(wd), nest, maxi, first};
}
inline AdamHyper make_adam(double lr, double b1, double b2, double eps, double wd, int adamw,
                           int maxi, double step_size, double bc2s) {
  return AdamHyper{static_cast<float>(b2), static_cast<float>(1.0 - b1),
                   static_cast<float>(1.0 - b2), static_cast<float>(eps),
                   static_cast<float>(wd), static_cast<float>(step_size),
                   static_cast<float>(bc2s), static_cast<float>(1.0 - lr * wd), adamw, maxi};
}

}  // namespace gs

// The opaque plan (visible to every TU of the library).
struct gs_plan {
  int kind = GS_DEV_HOST;
  int device = 0;
  int n = 0;
  int64_t align_elems = 0;
  int64_t flat_numel = 0;
  int64_t elems = 0;                   // Σ numel (the load policy's stream sizes)
  std::vector<int64_t> numel, off;
  std::vector<gs::Seg> segs;
  std::vector<int32_t> task_begin;
  std::vector<int64_t> voff;           // chunk-map engine: virtual offsets
  std::vector<gs::ChunkDesc> chunks;   // chunk-map engine: one per kChunkElems elements of voff space
  int grid = 0;
  int grid_cap = gs::kMaxGrid;         // the streaming ops' grid cap
  int64_t task_units = 0;
  // host shadow of the pointer table
  std::vector<void*> h_ptrs;       // [SLOTS * n]
  std::vector<uint32_t> h_align;   // [n]
  bool dirty = true;
  // device side (HIP plans only)
  void* d_static = nullptr;  // segs | task_begin | numel | off | chunks | voff
  void* d_table = nullptr;   // ptrs | align
  float* d_partials = nullptr;  // [kGridLimit] partials + the fused reduction's sync words
  void* pinned = nullptr;       // staging ring for table uploads
  int ring = 0;
  void* ring_events[4] = {nullptr, nullptr, nullptr, nullptr};
  void* last_stream = nullptr;
  void* last_event = nullptr;   // recorded on last_stream only when a launch moves to another stream
  bool last_captured = false;   // the last launch was recorded into a stream capture
  // one-shot HIP events for the next launch (the bucketer's timeline): written by
  // that kernel's own dispatch (hipExtLaunchKernel start / stop), not as packets
  void* once_start = nullptr;
  void* once_stop = nullptr;
  // a collective's watchdog mark rides on this plan's next eager launch (its stop event):
  // the communicator that deferred it there (gs_allreduce_marked & co.), or NULL
  void* watch_comm = nullptr;
  unsigned long long table_capture_id = 0;  // capture that last recorded a table write
  bool in_graph = false;        // a graph holds a table write: re-upload before eager launches
  const float* hyper = nullptr; // device hyper-parameter source of sgd/adam (gs_plan_set_hyper_source)
  // clip folded into sgd/adam (gs_plan_set_clip); clip_own: Σg² from this plan's
  // group sums, left by its last gs_sqnorm_partial (red_groups of them)
  bool clip_on = false, clip_own = false;
  gs::ClipArgs clip{};
  int red_groups = 0;
  bool red_valid = false;       // a gs_sqnorm_partial has run on this plan
  bool grads_read = false;      // a Σg² pass read slot 1 since the last update (load policy)
  int read_hint = 0;            // Σg² loads: 0 the size rule, 1 non-temporal, 2 cached (gs_plan_set_read_hint)
  float h_red = 0.f;            // host plans: the Σg² of gs_sqnorm_partial
  // launch timer ring (gs_plan_timer_enable)
  std::vector<void*> timer_ev;  // [2 * slots]: start, stop
  std::vector<int32_t> timer_kind;  // [slots]: GS_OP_* of the timed launch
  int timer_next = 0, timer_count = 0;
  gs::PlanArgs args() const;
};

namespace gs {
// ---- input step (gs_data.cpp / gs_data_kernels.hip) ----
#ifdef __HIPCC__
#define GS_HD __host__ __device__
#else
#define GS_HD
#endif
struct ImageAugArgs {
  const uint8_t* src;     // [n_src, H, W, C] uint8
  const int64_t* labels;  // [n_src] or NULL
  int64_t n_src;
  int H, W, C, pad, out_h, out_w;
  const int32_t* params;  // [B, 4] = (sample index, flip, top, left)
  int64_t B;
  void* out;              // [B, C, out_h, out_w] (NCHW) or [B, out_h, out_w, C] (NHWC)
  int out_dtype, layout;
  int64_t* out_labels;    // [B] or NULL
};
// Pad(pad, fill 0) -> hflip (of the padded image) -> crop(top, left) -> x/255
// for one output element (c, y, x) of sample idx; the same expression on the
// host and the device (IEEE division on both).
GS_HD inline float aug_pixel(const uint8_t* src, int64_t idx, int H, int W, int C, int pad, int flip,
                             int top, int left, int c, int y, int x) {
  const int wp = W + 2 * pad;
  const int px = flip ? (wp - 1 - (x + left)) : (x + left);
  const int sy = y + top - pad, sx = px - pad;
  if (sy < 0 || sy >= H || sx < 0 || sx >= W) return 0.f;
  return static_cast<float>(src[((idx * H + sy) * W + sx) * C + c]) / 255.f;
}
int hip_image_augment(int device, const ImageAugArgs& a, void* stream);

// Adam's step-varying hyper-parameters from a device step counter (torch's
// capturable=True): step += 1 unless found_inf; then, in double as the host
// path forms them, hyper = [-(lr/bc1), sqrt(bc2), 1 - lr*wd] rounded to fp32.
GS_HD inline void adam_hyper_update(double* step, const double* lr, double beta1, double beta2,
                                    double wd, const float* found_inf, float* hyper) {
  double s = step[0];
  if (found_inf == nullptr || found_inf[0] == 0.f) s += 1.0;
  step[0] = s;
  const double bc1 = 1.0 - pow(beta1, s), bc2 = 1.0 - pow(beta2, s);
  hyper[0] = static_cast<float>((lr[0] / bc1) * -1.0);
  hyper[1] = static_cast<float>(sqrt(bc2));
  hyper[2] = static_cast<float>(1.0 - lr[0] * wd);
}
int hip_adam_hyper(double* step, const double* lr, double beta1, double beta2, double wd,
                   const float* found_inf, float* hyper, void* stream);

// Deferred watchdog marks (gs_comm.cpp): a consumer plan's launch carries the mark of
// the collectives deferred to it.  comm_mark_take: 0 = nothing to do (the
// communicator is gone or not watching), 1 = carry *ev as the launch's stop event
// (*ev NULL: every mark of the ring is still pending — comm_mark_commit then records a
// pooled packet after the launch instead).  comm_mark_commit hands the carried event
// (or that packet) to the watchdog.
int comm_mark_take(gs_comm* c, void** ev);
// a destroyed communicator's stream (its work finished before the destroy, which
// synchronises it): a plan whose last launch ran there records nothing on it
bool stream_destroyed(void* stream);
// consumer: the launching plan — the collectives deferred to it are covered by its mark,
// timed from the oldest one's enqueue (a deferral whose consumer has not launched within
// about a second gets a packet from the watchdog instead)
int comm_mark_commit(gs_comm* c, void* ev, void* stream, const gs_plan* consumer);
// a plan being destroyed: collectives deferred to it keep only the watchdog's packet
void comm_forget_consumer(const gs_plan* consumer);

// HIP-side implementations (gs_kernels.hip)
int hip_plan_upload_static(gs_plan* p);
int hip_plan_release(gs_plan* p);
int hip_plan_flush(gs_plan* p, void* stream);
bool stream_capturing(void* stream);  // hipStreamIsCapturing: recording into a hipGraph
int hip_plan_timer_enable(gs_plan* p, int n_slots);
int hip_plan_timer_read(gs_plan* p, float* ms_out, int32_t* kind_out, int cap);
int hip_pack(gs_plan* p, int src_slot, int src_dt, void* flat, int flat_dt, float s, int mode,
             void* stream);
int hip_unpack(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* sq,
               int acc, void* stream);
int hip_unpack_check(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* found,
                     void* stream);
int hip_scale(gs_plan* p, int slot, int dt, float s, int mode, void* stream);
int hip_sqnorm(gs_plan* p, int slot, int dt, float* sq, int acc, void* stream);
int hip_sum(gs_plan* p, int slot, int dt, float* out, int acc, void* stream);
int hip_clip_coef(const float* sq, float max_norm, float eps, float* coef, float* norm,
                  void* stream);
int hip_unscale_check(gs_plan* p, int slot, int dt, const float* inv, float* found,
                      void* stream);
int hip_clip_scale(gs_plan* p, int slot, int dt, const ClipArgs& clip, void* stream);
int hip_sqnorm_partial(gs_plan* p, int slot, int dt, float* groups_out, int32_t* n_groups, void* stream);
const float* hip_plan_red_groups(const gs_plan* p);  // the <= 64 group sums of gs_sqnorm_partial, contiguous
float* hip_plan_red_scalar(const gs_plan* p);        // its finished Σ when red_groups == 0
int hip_sgd(gs_plan* p, int gdt, int ldt, const SgdHyper& h, const float* gs, const float* fi,
            const ClipArgs* clip, void* stream);
int hip_adam(gs_plan* p, int gdt, int ldt, const AdamHyper& h, const float* gs, const float* fi,
             const ClipArgs* clip, void* stream);
int hip_device_count();
int hip_memset_async(void* dst, int value, size_t bytes, void* stream);
int hip_stream_wait(void* waiter, void* signaler);

// host-side implementations (gs_host.cpp)
int host_pack(gs_plan* p, int src_slot, int src_dt, void* flat, int flat_dt, float s, int mode);
int host_unpack(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* sq,
                int acc);
int host_unpack_check(gs_plan* p, const void* flat, int flat_dt, int dst_slot, int dst_dt, float* found);
int host_scale(gs_plan* p, int slot, int dt, float s, int mode);
int host_clip_scale(gs_plan* p, int slot, int dt, const ClipArgs& clip);
int host_sqnorm(gs_plan* p, int slot, int dt, float* sq, int acc);
int host_sum(gs_plan* p, int slot, int dt, float* out, int acc);
int host_clip_coef(const float* sq, float max_norm, float eps, float* coef, float* norm);
int host_unscale_check(gs_plan* p, int slot, int dt, const float* inv, float* found);
int host_sgd(gs_plan* p, int gdt, int ldt, const SgdHyper& h, const float* gs, const float* fi,
             const ClipArgs* clip);
int host_adam(gs_plan* p, int gdt, int ldt, const AdamHyper& h, const float* gs, const float* fi,
              const ClipArgs* clip);
// the clip coefficient of ClipArgs on the host (groups == 0: *sq is final)
float host_clip_factor(const ClipArgs& c, const float* gs);
// the device's 64-lane DPP fold (gs_kernels.hip wave_reduce) restated on the
// host: lane l holds x[l * stride] (l < n), zeros elsewhere
float host_wave_sum(const float* x, int n, int stride);
}  // namespace gs
