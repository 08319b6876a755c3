/*
 * gsync.h — C-ABI of libgsync, the MI355X-native data-parallel
 * gradient-synchronisation engine (bucketer + RCCL collectives + fused
 * multi-tensor optimizer) behind the reference's DDP / ZeRO training wrappers.
 *
 * Every entry point replaces a native piece of the reference's path (the
 * reference itself is Python; its hot path lives in torch's c10d Reducer,
 * ProcessGroupNCCL and the ATen foreach/fused optimizer kernels — see
 * SURVEY.md §2.4 / §8a).  The "replaces:" line on each declaration names the
 * reference-side interface (file:line; R: = /root/reference,
 * T: = torch 2.10 under dist-packages/torch).
 *
 * Conventions
 *   - every function returns int: 0 = ok, <0 = error (GS_E*); the message is
 *     in gs_last_error() (thread-local).  No C++ exception crosses the ABI.
 *   - device memory is owned by the caller (torch caching allocator); the
 *     library only receives raw pointers.  The library owns communicators,
 *     streams, events and its own small metadata tables.
 *   - `stream` arguments are hipStream_t passed as void* (NULL = legacy
 *     default stream).  No entry point synchronises the host with the device
 *     except *_destroy and gs_comm_create.
 *   - device_kind GS_DEV_HIP runs hand-written gfx950 kernels; GS_DEV_HOST
 *     runs the host implementation used for CPU tensors (the gloo/CPU
 *     config).  A HIP plan never falls back to the host implementation.
 */
#ifndef GSYNC_H
#define GSYNC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSYNC_VERSION 1000 /* 0.1.0 */

/* ---- error codes ---- */
#define GS_OK 0
#define GS_EINVAL (-1)   /* bad argument (TORCH_CHECK equivalent) */
#define GS_EHIP (-2)     /* HIP runtime error */
#define GS_ERCCL (-3)    /* RCCL error */
#define GS_ESTATE (-4)   /* call out of protocol order (Reducer REDUCER_CHECK equivalent) */
#define GS_ENOMEM (-5)
#define GS_ENODEV (-6)   /* HIP requested but no device / library built without it */

/* ---- dtypes ---- */
#define GS_F32 0
#define GS_BF16 1
#define GS_F16 2
#define GS_F64 3
#define GS_I64 4
#define GS_I32 5
#define GS_U8 6

/* threads the host implementation (GS_DEV_HOST plans) may use; torch's
 * intra-op thread count is passed by the Python layer (default 1) */
int gs_set_host_threads(int n);

/* ---- device kinds ---- */
#define GS_DEV_HOST 0
#define GS_DEV_HIP 1

/* ---- reduce ops (ncclRedOp_t order) ---- */
#define GS_SUM 0
#define GS_PROD 1
#define GS_MAX 2
#define GS_MIN 3
#define GS_AVG 4

/* ---- scale modes for pack / scale ---- */
#define GS_SCALE_NONE 0
#define GS_SCALE_MUL 1 /* x * s  — Reducer pack: at::mul_out(bucket_view, grad, 1/div_factor) */
#define GS_SCALE_DIV 2 /* x / s  — Reducer view mode: bucket_view.div_(div_factor) */

typedef struct gs_comm gs_comm;
typedef struct gs_plan gs_plan;
typedef struct gs_bucketer gs_bucketer;

/* ======================================================================
 * library
 * ==================================================================== */
int gs_version(void);
const char* gs_last_error(void);
/* number of HIP devices visible (0 on a CPU-only host) */
int gs_device_count(void);

/* ======================================================================
 * communicator: RCCL over xGMI with a library-owned stream
 * replaces: T:include/torch/csrc/distributed/c10d/ProcessGroupNCCL.hpp:849
 *           (allreduce), :836 (broadcast), :872 (_allgather_base),
 *           :887-892 (reduce_scatter / _reduce_scatter_base),
 *           per-device NCCL streams ncclStreams_ :1398
 * ==================================================================== */
int gs_comm_unique_id_bytes(void); /* 128 */
int gs_comm_get_unique_id(uint8_t* out /* [gs_comm_unique_id_bytes()] */);
int gs_comm_create(int rank, int world, const uint8_t* uid, int device, gs_comm** out);
/* The same with RCCL's per-collective workgroup (CTA) cap (ncclConfig_t
 * maxCTAs; <= 0: RCCL's default): fewer CUs taken from the backward kernels the
 * in-step collectives overlap.  Replaces ProcessGroupNCCL's Options::config
 * (an ncclConfig_t handed to ncclCommInitRankConfig,
 * T:include/torch/csrc/distributed/c10d/ProcessGroupNCCL.hpp:531). */
int gs_comm_create_ex(int rank, int world, const uint8_t* uid, int device, int max_ctas, gs_comm** out);
int gs_comm_destroy(gs_comm* c);
/* ncclCommAbort: for the failure path (timeout / peer death) */
int gs_comm_abort(gs_comm* c);
/* failure detection: with timeout_ms > 0 a watchdog thread aborts the
 * communicator (ncclCommAbort) when a collective enqueued through it has been
 * in flight longer than timeout_ms, or RCCL reports an asynchronous error;
 * later calls then fail with GS_ERCCL.  0 disables the timeout.  A
 * collective called through this API is followed by an event on its stream
 * for the watchdog to poll; the bucketer's collectives are instead watched
 * through the stop event their unpack kernel carries (no event packet between
 * a bucket's collective and its unpack).
 * replaces: ProcessGroupNCCL's watchdog / TORCH_NCCL_ASYNC_ERROR_HANDLING
 *           (T:include/torch/csrc/distributed/c10d/ProcessGroupNCCL.hpp:59-68, :156) */
int gs_comm_set_timeout(gs_comm* c, int64_t timeout_ms);
/* Pause (1) / resume (0) every communicator's watchdog event polling,
 * process-wide and counted: bracket a global-mode hipGraph capture with it,
 * since event queries from the watchdog thread are illegal while another
 * thread records (collectives recorded into a graph are not tracked).
 * replaces: ProcessGroupNCCL's capture-time watchdog exclusion
 *           (T:.../c10d/ProcessGroupNCCL.cpp, "graph capture" handling) */
int gs_watchdog_pause(int pause);
/* 1 if aborted (reason copied into `reason`, NUL-terminated), 0 if live */
int gs_comm_status(gs_comm* c, char* reason, int cap);
int gs_comm_rank(gs_comm* c);
int gs_comm_world(gs_comm* c);
/* the dedicated collective stream (hipStream_t) */
int gs_comm_stream(gs_comm* c, void** stream_out);
/* make `waiter` wait for all work queued so far on `signaler` (event edge) */
int gs_stream_wait(void* waiter, void* signaler);

/* collectives on `stream` (NULL = the legacy default stream, like every
 * stream argument; gs_comm_stream() gives the communicator's own stream).
 * count in elements. */
int gs_allreduce(gs_comm* c, const void* send, void* recv, int64_t count, int dtype, int op,
                 void* stream);
int gs_reduce_scatter(gs_comm* c, const void* send, void* recv, int64_t recv_count, int dtype,
                      int op, void* stream);
int gs_all_gather(gs_comm* c, const void* send, void* recv, int64_t send_count, int dtype,
                  void* stream);
/* The same collectives with their watchdog mark deferred to a consumer kernel:
 * with a watchdog running, no event packet follows the collective (~4.7 µs of
 * stream time on the step's end each); `consumer`'s next launch
 * carries the communicator's mark as its own stop event instead and hands it
 * to the watchdog.  The caller guarantees that launch is stream-ordered after
 * the collective (ZeRO: the partials all-reduce before the clipped update on the
 * same stream; the parameter all-gather before the next backward's first pack).
 * If that launch has not come within half the timeout (at most 1 s), the watchdog
 * records a packet on `stream` itself and times the collective from its enqueue, so
 * `stream` must outlive that window (as a plan's last stream, gs_plan_destroy).
 * NULL consumer (or an empty plan, a capture): a packet, as the entry points above.
 * replaces: ProcessGroupNCCL's per-work end event (T:.../ProcessGroupNCCL.hpp:424
 *           ncclEndEvent_), recorded after every collective */
int gs_allreduce_marked(gs_comm* c, const void* send, void* recv, int64_t count, int dtype, int op,
                        void* stream, gs_plan* consumer);
int gs_all_gather_marked(gs_comm* c, const void* send, void* recv, int64_t send_count, int dtype,
                         void* stream, gs_plan* consumer);
int gs_broadcast(gs_comm* c, const void* send, void* recv, int64_t count, int dtype, int root,
                 void* stream);

/* ======================================================================
 * multi-tensor plan: a static list of tensor shapes laid out in one flat
 * buffer (per-tensor offsets aligned to `align_elems`, 0 = packed back to
 * back like torch's _flatten_dense_tensors / Reducer bucket), plus up to
 * GS_PLAN_SLOTS per-tensor pointer tables (param / grad / state...).
 * The work decomposition (segments + tasks) is built once on the host and
 * uploaded once; pointer tables are re-uploaded only when they change.
 * replaces: T:include/ATen/native/cuda/MultiTensorApply.cuh:14-21 launch
 *           geometry (kILP 4, 64Ki-element chunks, <=110 tensors/launch)
 * ==================================================================== */
#define GS_PLAN_SLOTS 5
int gs_plan_create(int device_kind, int device, int n_tensors, const int64_t* numels,
                   int64_t align_elems, gs_plan** out);
/* as gs_plan_create, with the work decomposition's task size pinned
 * (task_units units of 4 elements per workgroup task; 0 = automatic:
 * ~1920 tasks, one resident wave of workgroups) */
int gs_plan_create_ex(int device_kind, int device, int n_tensors, const int64_t* numels,
                      int64_t align_elems, int64_t task_units, gs_plan** out);
/* Stream lifetime: a plan orders a launch on a new stream after its previous
 * launch by recording an event on the PREVIOUS launch's stream at that point
 * (no packet after every launch), and gs_plan_destroy synchronises on it.  So
 * the stream of a plan's last launch must stay alive until the plan's next
 * launch on another stream, or until gs_plan_destroy. */
int gs_plan_destroy(gs_plan* p);
int64_t gs_plan_flat_numel(gs_plan* p);
int gs_plan_offsets(gs_plan* p, int64_t* out /* [n_tensors] */);
int gs_plan_n_tasks(gs_plan* p);
/* units (4 elements) per task of the plan's work decomposition */
int64_t gs_plan_task_units(gs_plan* p);
/* launch timer: when enabled (n_slots > 0) every kernel launched through the
 * plan is bracketed by a pair of timing HIP events recorded on the launch
 * stream, immediately around the kernel (after any pointer-table upload), in
 * a ring of n_slots pairs; n_slots = 0 disables and frees them.
 * gs_plan_timer_read waits for the recorded pairs and writes up to `cap`
 * durations (ms, oldest first) and, if kind_out is not NULL, the GS_OP_* of
 * each timed launch; returns how many it wrote, then clears.
 * (bench.py's roofline.avg_launch_ms; no torch counterpart.) */
#define GS_OP_PACK 1
#define GS_OP_UNPACK 2
#define GS_OP_SCALE 3
#define GS_OP_SQNORM 4
#define GS_OP_UNSCALE 5
#define GS_OP_SGD 6
#define GS_OP_ADAM 7
#define GS_OP_SUM 8
int gs_plan_timer_enable(gs_plan* p, int n_slots);
int gs_plan_timer_read(gs_plan* p, float* ms_out, int32_t* kind_out, int cap);
/* register the per-tensor pointers of one slot (uploads on change, ordered on `stream`) */
int gs_plan_set_ptrs(gs_plan* p, int slot, void* const* ptrs, void* stream);

/* flatten + fused scale + dtype cast: flat[off_t + i] = cast(src_t[i] (*|/) scale)
 * replaces: Reducer::mark_variable_ready_dense (T:.../c10d/reducer.hpp:275,
 *           upstream at::mul_out(bucket_view, grad, 1/div_factor_));
 *           T:_utils.py:558 _flatten_dense_tensors */
int gs_pack(gs_plan* p, int src_slot, int src_dtype, void* flat, int flat_dtype, float scale,
            int scale_mode, void* stream);
/* unflatten + cast: dst_t[i] = cast(flat[off_t + i]); if sqnorm_dev != NULL,
 * Σ dst² (fp32) is written (accumulate=0) or added (accumulate=1) to sqnorm_dev[0]
 * replaces: Reducer::copy_bucket_to_grad / finalize_bucket_dense (T:reducer.hpp:283,329);
 *           T:_utils.py:578 _unflatten_dense_tensors */
int gs_unpack(gs_plan* p, const void* flat, int flat_dtype, int dst_slot, int dst_dtype,
              float* sqnorm_dev, int accumulate, void* stream);
/* unflatten + cast with the AMP non-finite check of the written grads fused:
 * found_inf[0] = max(found_inf[0], any dst non-finite ? 1 : 0)
 * replaces: copy_bucket_to_grad + GradScaler's _amp_foreach_non_finite_check_and_unscale_
 *           check pass (T:amp/grad_scaler.py:280) over the same grads */
int gs_unpack_check(gs_plan* p, const void* flat, int flat_dtype, int dst_slot, int dst_dtype,
                    float* found_inf, void* stream);
/* in-place x = x (*|/) s on one slot (view-mode bucket_view.div_(div_factor)) */
int gs_scale(gs_plan* p, int slot, int dtype, float s, int scale_mode, void* stream);
/* Σ x² over all tensors of one slot into sqnorm_dev[0] (fp32, deterministic order)
 * replaces: T:nn/utils/clip_grad.py:96 torch._foreach_norm (+ vector_norm of norms) */
int gs_sqnorm(gs_plan* p, int slot, int dtype, float* sqnorm_dev, int accumulate, void* stream);
/* Σ x over every tensor of a slot (fp32 accumulation, deterministic order):
 * the bucket checksum of the GSYNC_DEBUG mode (gs_bucketer_set_debug) */
int gs_sum(gs_plan* p, int slot, int dtype, float* sum_dev, int accumulate, void* stream);
/* Σ x² of one slot left inside the plan as partial sums (no combine launch,
 * nothing written to caller memory), for the next clipped gs_sgd_step /
 * gs_adam_step on the same plan and stream (gs_plan_set_clip with
 * sqnorm_dev = NULL): the update's workgroups fold the partials themselves.
 * replaces: T:nn/utils/clip_grad.py:96-109 (_foreach_norm + the norm of norms)
 *           when the norm only feeds the clip */
int gs_sqnorm_partial(gs_plan* p, int slot, int dtype, void* stream);
/* Gradient-norm clip folded into every later gs_sgd_step / gs_adam_step on
 * this plan (max_norm <= 0 turns it off).  The update forms, in every workgroup,
 *   sq   = sqnorm_dev[0]   (sqnorm_dev = NULL: the plan's gs_sqnorm_partial sums)
 *   sq  *= grad_scale² (if grad_scale_dev) * sq_mul;  norm = sqrt(sq)
 *   coef = min(1, max_norm/(norm + eps)) * grad_scale * coef_mul
 * and multiplies the grads by coef — the arithmetic of gs_clip_coef plus the
 * caller's scale multiplies, bit for bit, without the coefficient launch.
 * out_dev (nullable, fp32[3]) receives [sq, coef, norm] (written even when
 * found_inf skips the step).  sq_mul / coef_mul: host-side loss-scale factors
 * (ZeRO: (1/scale)², 1/scale), 1 = none.
 * replaces: T:nn/utils/clip_grad.py:165-174 (clip_coef, clamp, _foreach_mul_)
 *           DeepSpeed gradient_clipping (R:resnet/deepspeed/deepspeed_train.py:195) */
/* How the plan's Σg² kernels (gs_sqnorm, gs_sqnorm_partial, gs_sqnorm_partial_out)
 * load their slot: 0 (default) cached below the 256 MiB Infinity Cache and
 * non-temporal above it; 1 non-temporal (the grads were just written by
 * non-temporal stores — libgsync's unpack — or by backward, and are read once);
 * 2 cached (e.g. a shard RCCL's reduce-scatter just wrote).  Bits never change.
 * GS_NT_SQNORM in the environment overrides.  No reference counterpart (a load
 * policy of this implementation). */
int gs_plan_set_read_hint(gs_plan* p, int hint);
int gs_plan_set_clip(gs_plan* p, const float* sqnorm_dev, float max_norm, float eps, float sq_mul,
                     float coef_mul, float* out_dev);
/* The partial sums of Σx² over the plan, written out for a sharded optimizer:
 * groups_out (device memory of the plan's kind) must hold GS_RED_PARTIALS
 * floats; *n_groups (host) receives how many are valid, 1..GS_RED_PARTIALS,
 * and the call sets the slots past them to 0.
 * A plan of at most 4 Ki chunks (a ZeRO shard at N = 8: 3.2 M elements)
 * writes one partial per workgroup of a balanced grid (<= 1024 workgroups) —
 * no arrival counters, no in-kernel combine, nothing after the
 * streaming but one store per workgroup; a larger plan writes the fused
 * reduction's <= 64 group sums (gs_sqnorm_partial's kernel); 1 = a finished Σ
 * (host plans, a reduction without the in-kernel combine).  A sharded
 * optimizer SUM-all-reduces the whole GS_RED_PARTIALS-float buffer across its
 * ranks (a rank's n follows its own chunk map, so only a fixed length is the
 * same on every rank; the zero slots past a rank's n add nothing) and hands it
 * to gs_plan_set_clip_groups
 * (n_groups = GS_RED_PARTIALS): the global ‖g‖
 * of every shard with no combine launch and no scalar coefficient launch on the
 * step's exposed end.
 * replaces: DeepSpeed stage_1_and_2 get_grad_norm_direct (per-rank Σg² of the
 *           partition, all_reduce of the scalar, U) for gradient_clipping
 *           (R:resnet/deepspeed/deepspeed_train.py:195) */
#define GS_RED_GROUPS 64
#define GS_RED_PARTIALS 1024
int gs_sqnorm_partial_out(gs_plan* p, int slot, int dtype, float* groups_out, int32_t* n_groups,
                          void* stream);
/* gs_plan_set_clip with ‖g‖² = the fold of n_groups (<= GS_RED_PARTIALS)
 * partial sums at groups_dev (contiguous; typically gs_sqnorm_partial_out's,
 * summed over ranks): every update workgroup folds them in a fixed order —
 * lane l of one wave adds partials l, l + 64, l + 128, ..., then the fused
 * reduction's own 64-lane tree — so every rank forms the same coefficient. */
int gs_plan_set_clip_groups(gs_plan* p, const float* groups_dev, int32_t n_groups, float max_norm,
                            float eps, float sq_mul, float coef_mul, float* out_dev);
/* clip_grad_norm_'s scale pass: slot `slot` (dtype) *= the clip coefficient of
 * the plan's clip (gs_plan_set_clip / gs_plan_set_clip_groups, consumed as by a
 * clipped update), torch.clamp(max_norm / (‖g‖ + eps), max = 1): every
 * workgroup folds the Σg² partial sums itself, workgroup 0 publishes
 * [Σg², coef, norm] to the clip's out; a coefficient of exactly 1 writes
 * nothing (x * 1 == x).  With gs_sqnorm_partial before it, clip_grad_norm_ is
 * two launches: no combine, no coefficient kernel, no flag fill.
 * replaces: T:nn/utils/clip_grad.py:165-174 (clip_coef, clamp, _foreach_mul_) */
int gs_clip_scale(gs_plan* p, int slot, int dtype, void* stream);
/* coef_dev[0] = min(1, max_norm / (sqrt(sqnorm_dev[0]) + eps)); norm_dev (nullable) = sqrt
 * replaces: T:nn/utils/clip_grad.py:165-174 clip_coef / clamp */
int gs_clip_coef(int device_kind, const float* sqnorm_dev, float max_norm, float eps,
                 float* coef_dev, float* norm_dev, void* stream);
/* found_inf_dev[0] = 1.0 if any non-finite in slot, and (if inv_scale_dev) x *= inv_scale
 * replaces: T:amp/grad_scaler.py:280 _amp_foreach_non_finite_check_and_unscale_ */
int gs_unscale_check(gs_plan* p, int slot, int dtype, const float* inv_scale_dev,
                     float* found_inf_dev, void* stream);

/* fused SGD momentum / weight decay, one pass over (p, g, buf[, p_lowp]):
 *   g' = g*gscale (+ wd*p);  buf = first ? g' : mom*buf + (1-damp)*g';
 *   d = nesterov ? g' + mom*buf : buf;  p -= lr*d;  p_lowp = cast(p)
 * slots: 0 = param (f32), 1 = grad (grad_dtype), 2 = momentum buffer (f32, unused if mom==0),
 *        3 = optional low-precision param copy (lowp_dtype, -1 = none)
 * grad_scale_dev (nullable): multiplies g (clip coefficient / AMP unscale);
 * found_inf_dev (nullable): skip the whole step when *found_inf != 0.
 * replaces: T:optim/sgd.py:322-381 _single_tensor_sgd, :383-470 _multi_tensor_sgd */
int gs_sgd_step(gs_plan* p, int grad_dtype, int lowp_dtype, double lr, double momentum,
                double dampening, double weight_decay, int nesterov, int maximize, int first_step,
                const float* grad_scale_dev, const float* found_inf_dev, void* stream);
/* fused Adam / AdamW, one pass over (p, g, m, v[, p_lowp]) with torch's foreach arithmetic:
 *   (adamw) p *= 1 - lr*wd  |  (adam) g += wd*p
 *   m = lerp(m, g, 1-b1);  v = b2*v + (1-b2)*g*g;
 *   p += step_size * m / (sqrt(v)/bc2_sqrt + eps)       (step_size = -lr/bc1)
 * slots: 0 = p, 1 = g, 2 = exp_avg, 3 = exp_avg_sq, 4 = optional low-precision copy
 * Hyper-parameters are Python floats (double) and are rounded to fp32 exactly
 * where torch rounds them: 1-b1, 1-b2, 1-lr*wd are formed in double first.
 * replaces: T:optim/adam.py:554-800 _multi_tensor_adam (reference GPU default);
 *           T:include/ATen/native/cuda/fused_adam_utils.cuh:11-88 */
int gs_adam_step(gs_plan* p, int grad_dtype, int lowp_dtype, double lr, double beta1,
                 double beta2, double eps, double weight_decay, int adamw, int maximize,
                 double step_size, double bias_correction2_sqrt, const float* grad_scale_dev,
                 const float* found_inf_dev, void* stream);
/* Step-varying hyper-parameters from memory instead of the arguments: with a
 * non-NULL source, every later gs_sgd_step / gs_adam_step on this plan reads
 *   SGD:  hyper[0] = lr; hyper[1] = "first step" flag (buf = g) when gs_sgd_step
 *         is called with first_step = -1 — the AMP path keeps it on the device
 *         (cleared by the caller after a step that was not skipped)
 *   Adam: hyper[0] = step_size (-lr/bc1), hyper[1] = bias_correction2_sqrt,
 *         hyper[2] = 1 - lr*wd (AdamW decay)
 * (fp32, device memory for HIP plans, host memory for host plans) when the
 * kernel runs, so a step recorded into a hipGraph follows an LR schedule and
 * Adam's bias corrections on replay; the argument values are then ignored.
 * NULL restores argument hyper-parameters.  The buffer must outlive its use.
 * replaces: T:optim/adam.py capturable=True (device step / tensor lr) */
int gs_plan_set_hyper_source(gs_plan* p, const float* hyper);
/* Adam hyper source update on the stream (one thread; graph-capturable):
 *   if (!found_inf || *found_inf == 0) *step += 1;
 *   hyper = [-(lr/bc1), sqrt(bc2), 1 - lr*wd]  with bcK = 1 - betaK^step, in double
 * step, lr: fp64 scalars; hyper: fp32[3] (the plan's hyper source).
 * replaces: T:optim/adam.py:640-668 (capturable branch: device step, bias corrections) */
int gs_adam_hyper(int device_kind, double* step, const double* lr, double beta1, double beta2,
                  double weight_decay, const float* found_inf, float* hyper, void* stream);

/* ======================================================================
 * bucket assignment (greedy by size per dtype, first-bucket cap)
 * replaces: T:.../c10d/reducer.hpp:590-595 compute_bucket_assignment_by_size
 *           (dist._compute_bucket_assignment_by_size)
 * order: NULL -> tensors in index order and buckets sorted by min index;
 *        else the gradient-ready order (no sort), as Reducer::rebuild_buckets.
 * Writes bucket_of[n] (bucket id per tensor position in `order`/index order) and
 * returns the bucket count (>=0) or an error.
 * ==================================================================== */
int gs_compute_bucket_assignment(int n, const int64_t* nbytes, const int32_t* dtype_keys,
                                 const int32_t* order, int n_limits, const int64_t* limits,
                                 int32_t* bucket_of /* [n], indexed by tensor id */,
                                 int32_t* bucket_members /* [n] concatenated, bucket order */,
                                 int32_t* bucket_counts /* [n] */);

/* ======================================================================
 * bucketer: the Reducer state machine
 * replaces: T:.../c10d/reducer.hpp:52-63 Reducer ctor, :73 autograd_hook,
 *           :275 mark_variable_ready_dense, :111-116 run_comm_hook,
 *           :283 finalize_bucket_dense, :346-402 Bucket
 * ==================================================================== */
#define GS_BKT_AUTO_COLLECTIVE 1 /* library launches the collective itself (needs comm) */
#define GS_BKT_GRAD_VIEW 2       /* grads already alias the bucket: scale in place, no unpack */
#define GS_BKT_NO_SCALE 4        /* a comm hook owns the averaging: copy without 1/ws */
#define GS_BKT_REDUCE_SCATTER 8  /* ZeRO-2: reduce-scatter into shard buffers instead of allreduce */
#define GS_BKT_NO_UNPACK 16      /* caller consumes the bucket directly (ZeRO / fused step) */

int gs_bucketer_create(gs_comm* comm, int device_kind, int device, int n_params,
                       const int64_t* numels, int grad_dtype, int n_buckets,
                       const int32_t* bucket_counts, const int32_t* bucket_members,
                       int bucket_dtype, int64_t align_elems, float div_factor, int flags,
                       gs_bucketer** out);
int gs_bucketer_destroy(gs_bucketer* b);
int gs_bucketer_bucket_numel(gs_bucketer* b, int bucket, int64_t* out);
/* padded numel of the reduce-scatter output shard for a bucket (ZeRO-2) */
int gs_bucketer_shard_numel(gs_bucketer* b, int bucket, int64_t* out);
int gs_bucketer_param_location(gs_bucketer* b, int param, int32_t* bucket, int64_t* offset);
/* per-bucket dtypes (torch's Reducer buckets per dtype: a model with params of
 * several floating dtypes gets buckets of each; create() sets the defaults) */
int gs_bucketer_set_bucket_dtype(gs_bucketer* b, int bucket, int grad_dtype, int bucket_dtype);
/* storage for bucket `bucket` (torch-owned, bucket_numel elements of its bucket dtype) */
int gs_bucketer_set_bucket_buffer(gs_bucketer* b, int bucket, void* ptr);
/* ZeRO-2 output shard storage for bucket */
int gs_bucketer_set_shard_buffer(gs_bucketer* b, int bucket, void* ptr);
/* start of a backward pass that will synchronise (Reducer::prepare_for_backward).
 * sqnorm_dev (nullable): receives Σ g² of the averaged grads, fused into unpack. */
int gs_bucketer_prepare(gs_bucketer* b, float* sqnorm_dev);
/* autograd hook: param's grad (grad_ptr) is final for this backward.
 * ready_out[*n_ready] receives the buckets that became launchable, in launch
 * order; with GS_BKT_AUTO_COLLECTIVE their collectives are already enqueued. */
int gs_bucketer_mark_ready(gs_bucketer* b, int param, const void* grad, void* stream,
                           int32_t* ready_out, int32_t* n_ready);
/* mark every not-yet-ready param as unused (zero its slot) — find_unused_parameters */
int gs_bucketer_mark_unused(gs_bucketer* b, void* stream, int32_t* ready_out, int32_t* n_ready);
/* end of backward: unpack (unless view / no-unpack) and order `stream` after
 * the collectives (Reducer::finalize_backward). */
int gs_bucketer_finalize(gs_bucketer* b, void* stream);
/* unpack one bucket (external-collective mode: after the caller's collective) */
/* AMP: fuse the non-finite check of the averaged grads into each bucket's
 * unpack (found_inf[0] = max(found_inf[0], non-finite ? 1 : 0); the caller
 * zeroes it before backward); NULL disables.  Replaces the check pass of
 * GradScaler._unscale_grads_ (T:amp/grad_scaler.py:280) for these grads. */
int gs_bucketer_set_found_inf(gs_bucketer* b, float* found_inf);
/* The divisor of the next backward's packs (grad x float(1/div_factor)),
 * between backwards: DDP.join(divide_by_initial_world_size=False) divides by
 * the ranks still training, as the Reducer's div_factor_ set from the forward
 * pass work handle (T:include/torch/csrc/distributed/c10d/reducer.hpp:499,
 * _set_forward_pass_work_handle). */
int gs_bucketer_set_div_factor(gs_bucketer* b, float div_factor);
int gs_bucketer_unpack_bucket(gs_bucketer* b, int bucket, void* stream);
/* Sharded buckets (NO_UNPACK / REDUCE_SCATTER, the ZeRO engine): the
 * bucket collectives' watchdog marks ride on `consumer`'s next launch (the
 * sharded update, stream-ordered after finalize) instead of a packet after
 * each collective; NULL restores the packets.  GS_EINVAL on unpacking buckets
 * (their unpack kernels already carry the marks).
 * replaces: ProcessGroupNCCL's per-work end event, as gs_allreduce_marked */
int gs_bucketer_set_mark_consumer(gs_bucketer* b, gs_plan* consumer);
/* the plan of bucket 0's pack — the first libgsync kernel of the next
 * synchronising backward, a consumer for collectives issued after a step
 * (ZeRO's parameter all-gather) */
int gs_bucketer_first_pack_plan(gs_bucketer* b, gs_plan** out);
/* timing of the library's own collective launches (ms of the last iteration, via events) */
int gs_bucketer_last_comm_ms(gs_bucketer* b, int bucket, float* ms);
/* per-bucket timeline of the last iteration (HIP events; -1 where untimed:
 * host buckets, external collectives, hipGraph capture), ms:
 *   out[0] queue      bucket ready on the producer -> its pack kernel starts
 *   out[1] pack       out[2] collective (pack end -> unpack start)
 *   out[3] unpack (+ fused checks)
 *   out[4] ready -> every bucket finished: for the last bucket this is the
 *          exposed end-of-backward tail */
int gs_bucketer_last_timing(gs_bucketer* b, int bucket, float* out /* [5] */);
/* which timing marks the bucketer takes: 0 none; 1 (default) the last bucket's
 * ready event + the "every chain done" mark — out[4] of the last bucket, the
 * tail; 2 every bucket's full timeline (and gs_bucketer_last_comm_ms).  The
 * ready mark is an event packet (~4.7 µs of stream time on the exposed chain);
 * every other mark rides on the chain's own kernels (hipExtLaunchKernel start /
 * stop events, ~2.4 µs) and becomes a packet only where no kernel runs */
int gs_bucketer_set_timeline(gs_bucketer* b, int level);
/* the HIP stream bucket `bucket`'s chain (pack -> collective -> unpack) was
 * enqueued on in this backward (the comm stream, or the producer stream for the
 * last bucket); NULL before its launch, on the host and with external
 * collectives.  Work enqueued there after the chain sees the averaged grads —
 * the overlapped optimizer (DDP._register_fused_optim) steps each bucket so.
 * replaces: the Future of run_comm_hook that _hook_then_optimizer chains on
 *           (T:distributed/algorithms/ddp_comm_hooks/optimizer_overlap_hooks.py) */
int gs_bucketer_bucket_stream(gs_bucketer* b, int bucket, void** stream);
/* Debug mode (checksum each bucket before and after the
 * collective): with a non-NULL device (host, for host buckets) buffer of
 * 3 * n_buckets floats, every backward writes sums[3b] = Σx of bucket b after
 * its pack (before the collective), sums[3b+1] = Σx after the collective
 * (before the unpack) and sums[3b+2] = Σx² after the pack.  Across ranks
 * Σ_r sums_r[3b] must equal sums[3b+1] up to fp32 rounding and sums[3b+1]
 * must be identical on every rank
 * (distributed_training_amd.ddp.DistributedDataParallel.verify_bucket_checksums).
 * NULL disables. */
int gs_bucketer_set_debug(gs_bucketer* b, float* sums);

/* ====================================================================
 * Input step of the CIFAR configuration
 * replaces: torch.utils.data.DistributedSampler.__iter__
 *           (T:utils/data/distributed.py:107-138) and the per-sample
 *           torchvision 0.15.2 transforms Pad(4) / RandomHorizontalFlip /
 *           RandomCrop(32) / ToTensor + default_collate, driven by
 *           DataLoader(num_workers=0) (R:resnet/pytorch_ddp/ddp_train.py:25-48)
 * ==================================================================== */
#define GS_LAYOUT_NCHW 0
#define GS_LAYOUT_NHWC 1
/* size of torch.get_rng_state() for a CPU generator (MT19937 + caches) */
int gs_rng_state_bytes(void);
/* n raw 32-bit MT19937 outputs from torch's serialized CPU generator state,
 * advancing the state in place exactly as n torch draws would */
int gs_rng_draw_u32(uint8_t* state, int64_t state_bytes, int64_t n, uint32_t* out);
/* torch.randperm(n, generator=torch.Generator().manual_seed(seed)) */
int gs_randperm(uint64_t seed, int64_t n, int64_t* out);
/* DistributedSampler(n, num_replicas, rank, shuffle, seed, drop_last) with
 * set_epoch(epoch): this rank's indices (out = NULL: *count only) */
int gs_distributed_sampler_indices(int64_t n, int num_replicas, int rank, int shuffle, uint64_t seed,
                                   int64_t epoch, int drop_last, int64_t* out, int64_t cap,
                                   int64_t* count);
/* per-sample (index, flip, top, left) for a batch, consuming torch's global
 * generator state in the reference's order: flip draw (if flip), then the
 * crop's two draws (unless the padded image equals the crop) per sample */
int gs_crop_flip_params(const int64_t* indices, int64_t B, int in_h, int in_w, int pad, int out_h,
                        int out_w, int flip, uint8_t* rng_state, int64_t state_bytes,
                        int32_t* params /* [B,4] */);
/* one batch: gather + pad + flip + crop + uint8->float /255 (+ bf16 cast),
 * labels gathered alongside; device_kind HIP runs one gfx950 kernel on
 * `stream` (src, labels, params, out in device memory) */
int gs_image_augment(int device_kind, int device, const uint8_t* src, const int64_t* labels, int64_t n_src,
                     int H, int W, int C, int pad, int out_h, int out_w, const int32_t* params, int64_t B,
                     void* out, int out_dtype, int out_layout, int64_t* out_labels, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSYNC_H */
