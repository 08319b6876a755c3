// libgsync bucketer: the Reducer state machine of torch DDP restated for
// MI355X (T:include/torch/csrc/distributed/c10d/reducer.hpp:52-63 ctor,
// :73 autograd_hook, :275 mark_variable_ready_dense, :111-116 run_comm_hook,
// :283 finalize_bucket_dense, :346-402 Bucket).
//
// Differences in HOW (not WHAT):
//  - a bucket is packed by ONE multi-tensor launch when its last gradient is
//    ready (torch: one elementwise launch per parameter, 161 for ResNet-50);
//  - pack, collective and unpack all run on the communicator's own stream,
//    ordered after the producer (autograd) stream by one event, so the whole
//    per-bucket chain overlaps the rest of backward and only the last
//    bucket's chain is exposed;
//  - per-parameter offsets inside a bucket are padded to `align_elems` so
//    every access is a full 16-B vector access; padding is zero and is
//    reduced as zero.
// Buckets launch strictly in index order (next_bucket_), so every rank issues
// the same collective sequence, as Reducer::mark_bucket_ready does.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <functional>
#include <mutex>

#include "gs_common.h"

namespace gs {
ncclComm_t comm_handle(gs_comm* c);
hipStream_t comm_stream(gs_comm* c);
int comm_dtype(int dt, ncclDataType_t* out);
int comm_enqueue(gs_comm* c, hipStream_t stream, const std::function<ncclResult_t()>& fn, const char* what,
                 bool track = true, gs_plan* consumer = nullptr);
int comm_track_event(gs_comm* c, hipEvent_t ev);
bool comm_watching(gs_comm* c);
void comm_forget_event(gs_comm* c, hipEvent_t ev);
}  // namespace gs

using namespace gs;

namespace {

#define HIPB_RET(expr)                                                               \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess)                                                            \
      return fail(GS_EHIP, std::string(#expr " failed: ") + hipGetErrorString(_e));  \
  } while (0)

constexpr int kWdRing = 8;

struct Bucket {
  std::vector<int32_t> params;  // global parameter ids, bucket order
  gs_plan* plan = nullptr;      // layout of the params inside the flat bucket
  gs_plan* flat = nullptr;      // the whole flat bucket as one tensor (in-place ops)
  int64_t numel = 0;            // padded flat numel
  int gdt = GS_F32, bdt = GS_F32;  // grad / bucket dtype of this bucket (torch buckets per dtype)
  void* buf = nullptr;          // torch-owned flat storage
  void* shard = nullptr;        // torch-owned reduce-scatter output
  int pending = 0;
  bool launched = false;
  bool unpacked = false;
  void* stream = nullptr;       // the stream this iteration's chain ran on (gs_bucketer_bucket_stream)
  // timing (all on the comm stream but ev_ready, recorded on the producer):
  // ready -> pk0 (queue) -> t0 (pack) -> t1 (collective) -> u1 (unpack)
  hipEvent_t ev_ready = nullptr, ev_pk0 = nullptr, ev_t0 = nullptr, ev_t1 = nullptr, ev_u1 = nullptr;
  hipEvent_t ev_sync = nullptr;  // untimed ready event (a comm-stream chain waits on it)
  // the watchdog's marks of the collective, carried by the unpack kernel: a ring, so a
  // host queueing steps ahead re-records an event only after its previous record
  // completed (comm_track_event); timing-enabled, as the level-1 tail's done mark
  hipEvent_t ev_wd[kWdRing] = {};
  int wd_next = 0;
  bool timed = false;            // pk0 / t0 / t1 / u1 recorded (level 2)
  bool pk0_is_ready = false;     // the producer-side tail: its pack follows the ready mark on the same
                                 // stream with nothing between, so ready doubles as pk0 (queue 0)
  bool ready_timed = false;      // ev_ready recorded
};

// End marks ride on the chain's own kernels (hipExtLaunchKernel's stop event,
// written by the dispatch) instead of event packets of their own: a packet costs
// ~4.7 µs of stream time on the exposed chain, a kernel-carried stop event ~2.4 µs,
// a kernel-carried START event ~7.4 µs (scripts/micro/event_chain.hip,
// profiles/r5/r5a_event_chain.jsonl, r5f_event_chain.jsonl) — so start marks stay
// packets.  arm() hands the events to the plan's next launch; settle() records
// whatever no launch took (an empty plan, a grad-view bucket that needs no scaling)
// at that point instead.
void arm(gs_plan* p, hipEvent_t start, hipEvent_t stop) {
  p->once_start = start;
  p->once_stop = stop;
}
int settle(gs_plan* p, hipStream_t s) {
  hipEvent_t a = static_cast<hipEvent_t>(p->once_start), b = static_cast<hipEvent_t>(p->once_stop);
  p->once_start = p->once_stop = nullptr;
  if (a && hipEventRecord(a, s) != hipSuccess) return fail(GS_EHIP, "timeline event record failed");
  if (b && hipEventRecord(b, s) != hipSuccess) return fail(GS_EHIP, "timeline event record failed");
  return GS_OK;
}

}  // namespace

struct gs_bucketer {
  gs_comm* comm = nullptr;
  int kind = GS_DEV_HOST;
  int device = 0;
  int n_params = 0;
  int grad_dtype = GS_F32;
  int bucket_dtype = GS_F32;
  int64_t align = 0;
  float div = 1.f;
  int flags = 0;
  std::vector<Bucket> buckets;
  std::vector<int32_t> loc_bucket, loc_intra;
  std::vector<int64_t> numel;
  std::vector<char> ready;
  int next_bucket = 0;
  bool prepared = false;
  float* sqnorm = nullptr;
  int sq_count = 0;
  float* found_inf = nullptr;  // AMP non-finite flag of the averaged grads (fused into unpack)
  float* dbg = nullptr;        // GSYNC_DEBUG: [3 * n_buckets] Σx after pack, Σx after collective, Σx² after pack
  void* producer = nullptr;
  hipEvent_t ev_done = nullptr;
  hipEvent_t ev_done_sync = nullptr;  // untimed finalize event (timeline level 0)
  // timeline level (gs_bucketer_set_timeline): 0 none, 1 the tail only (the
  // last bucket's ready event + the finalize event, default), 2 every bucket's
  // queue / pack / collective / unpack.  Each timing event is a packet on the
  // stream; at level 2 they stretch the exposed chain by ~10 µs apiece.
  int timeline = 1;
  hipEvent_t ev_comm = nullptr;     // comm stream's earlier buckets, joined before a producer-side tail's collective
  bool done_timed = false;
  hipEvent_t done_ev = nullptr;     // this iteration's "every chain done" mark: ev_done, or the stop
                                    // event of the producer-side tail's last kernel (done_on_chain)
  bool done_on_chain = false;
  bool tail_ran_on_producer = false;
  // sharded buckets (no unpack): the plan whose next launch consumes the shards (ZeRO's
  // update) carries the collectives' watchdog marks (gs_bucketer_set_mark_consumer)
  gs_plan* mark_consumer = nullptr;
  std::mutex mu;

  bool hip() const { return kind == GS_DEV_HIP; }
  bool auto_coll() const { return (flags & GS_BKT_AUTO_COLLECTIVE) != 0; }
  bool do_unpack() const {
    return (flags & (GS_BKT_GRAD_VIEW | GS_BKT_NO_UNPACK | GS_BKT_REDUCE_SCATTER)) == 0;
  }
};

namespace {

void plan_set_one(gs_plan* p, int slot, int t, void* ptr) {
  void*& cur = p->h_ptrs[static_cast<size_t>(slot) * p->n + t];
  if (cur == ptr) return;
  cur = ptr;
  const uint32_t bit = 1u << slot;
  const bool al = (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0;
  p->h_align[t] = al ? (p->h_align[t] | bit) : (p->h_align[t] & ~bit);
  p->dirty = true;
}

int bucket_index(gs_bucketer* b, const Bucket& bk) { return static_cast<int>(&bk - b->buckets.data()); }

// GSYNC_DEBUG checksums: Σ bucket after the pack (which = 0, before the
// collective) / after the collective (which = 1, before the unpack)
int debug_sum(gs_bucketer* b, Bucket& bk, int which, void* stream) {
  if (!b->dbg) return GS_OK;
  float* d = b->dbg + 3 * bucket_index(b, bk);
  GS_TRY_RET(gs_sum(bk.flat, 0, bk.bdt, d + which, 0, stream));
  // the packed bucket's Σx² sets the scale of the cross-rank comparison
  return which == 0 ? gs_sqnorm(bk.flat, 0, bk.bdt, d + 2, 0, stream) : GS_OK;
}

// after the collective: unpack into the grads (with the fused Σg² or the fused
// non-finite check), or, when the grads ARE the bucket, just the check.  e0 / e1:
// timing events carried by the first / last kernel of this step (nullable).
int unpack_one(gs_bucketer* b, Bucket& bk, void* stream, int accumulate_sq, hipEvent_t e0 = nullptr,
               hipEvent_t e1 = nullptr) {
  float* sq = b->sqnorm;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (b->do_unpack()) {
    if (b->found_inf && !sq) {
      arm(bk.plan, e0, e1);
      GS_TRY_RET(gs_unpack_check(bk.plan, bk.buf, bk.bdt, 1, bk.gdt, b->found_inf, stream));
      GS_TRY_RET(settle(bk.plan, s));
    } else {
      const int acc = (b->sq_count > 0 || accumulate_sq) ? 1 : 0;
      arm(bk.plan, e0, b->found_inf ? nullptr : e1);
      GS_TRY_RET(gs_unpack(bk.plan, bk.buf, bk.bdt, 1, bk.gdt, sq, acc, stream));
      GS_TRY_RET(settle(bk.plan, s));
      if (sq) ++b->sq_count;
      if (b->found_inf) {
        arm(bk.flat, nullptr, e1);
        GS_TRY_RET(gs_unscale_check(bk.flat, 0, bk.bdt, nullptr, b->found_inf, stream));
        GS_TRY_RET(settle(bk.flat, s));
      }
    }
  } else if (b->found_inf) {
    arm(bk.flat, e0, e1);
    GS_TRY_RET(gs_unscale_check(bk.flat, 0, bk.bdt, nullptr, b->found_inf, stream));
    GS_TRY_RET(settle(bk.flat, s));
  } else {
    if (e0) HIPB_RET(hipEventRecord(e0, s));
    if (e1) HIPB_RET(hipEventRecord(e1, s));
  }
  bk.unpacked = true;
  return GS_OK;
}

// pack (or scale in place) bucket bk on `stream`
int pack_raw(gs_bucketer* b, Bucket& bk, void* stream) {
  const bool no_scale = (b->flags & GS_BKT_NO_SCALE) != 0;
  if (b->flags & GS_BKT_GRAD_VIEW) {
    // grads alias the bucket (gradient_as_bucket_view): bucket_view.div_(div_factor)
    bool all_alias = true;
    const int es = dtype_size(bk.bdt);
    for (size_t i = 0; i < bk.params.size(); ++i) {
      const void* g = bk.plan->h_ptrs[static_cast<size_t>(1) * bk.plan->n + i];
      if (g != static_cast<char*>(bk.buf) + bk.plan->off[i] * es) { all_alias = false; break; }
    }
    if (all_alias) {
      if (no_scale || b->div == 1.f) return GS_OK;
      return gs_scale(bk.flat, 0, bk.bdt, b->div, GS_SCALE_DIV, stream);
    }
  }
  if (no_scale) return gs_pack(bk.plan, 1, bk.gdt, bk.buf, bk.bdt, 1.f, GS_SCALE_NONE, stream);
  // at::mul_out(bucket_view, grad, 1/div_factor): the scalar is float(1.0/div)
  const float inv = static_cast<float>(1.0 / static_cast<double>(b->div));
  return gs_pack(bk.plan, 1, bk.gdt, bk.buf, bk.bdt, inv, GS_SCALE_MUL, stream);
}

int pack_one(gs_bucketer* b, Bucket& bk, void* stream) {
  GS_TRY_RET(pack_raw(b, bk, stream));
  return debug_sum(b, bk, 0, stream);
}

// track = false: the caller hands the collective to the watchdog through an event
// of its own that the stream records after it (comm_track_event)
// consumer (nullable): the plan whose next launch carries the collective's mark instead
int launch_collective(gs_bucketer* b, Bucket& bk, hipStream_t cs, bool track = true, gs_plan* consumer = nullptr) {
  ncclDataType_t dt;
  GS_TRY_RET(comm_dtype(bk.bdt, &dt));
  if (b->flags & GS_BKT_REDUCE_SCATTER) {
    const int w = gs_comm_world(b->comm);
    return comm_enqueue(b->comm, cs, [&] {
      return ncclReduceScatter(bk.buf, bk.shard, static_cast<size_t>(bk.numel / w), dt, ncclSum,
                               comm_handle(b->comm), cs);
    }, "bucket reduce-scatter", track, consumer);
  }
  return comm_enqueue(b->comm, cs, [&] {
    return ncclAllReduce(bk.buf, bk.buf, static_cast<size_t>(bk.numel), dt, ncclSum, comm_handle(b->comm), cs);
  }, "bucket all-reduce", track, consumer);
}

int launch_bucket(gs_bucketer* b, int bi) {
  GsRange range("gsync.bucket");
  Bucket& bk = b->buckets[bi];
  if (!bk.buf) return fail(GS_ESTATE, "bucket " + std::to_string(bi) + " has no storage");
  if (!b->hip()) {
    GS_TRY_RET(pack_one(b, bk, nullptr));
  } else if (b->auto_coll()) {
    // The last bucket's chain is the exposed end-of-backward tail: nothing is
    // left to overlap it with, so it runs on the producer stream itself — no
    // cross-stream hop to start it (its "queue") and none back at finalize.
    // The producer joins the comm stream's earlier buckets after its pack, right
    // before its collective, so the communicator's collectives stay in issue
    // order on the GPU while the pack overlaps the previous bucket's chain.
    // (Joining only the previous collective there and the rest of the comm
    // stream before the unpack measured 5 µs longer: r5j.)
    const bool last = bi == static_cast<int>(b->buckets.size()) - 1;
    const bool on_producer = last;
    hipStream_t ps = static_cast<hipStream_t>(b->producer);
    hipStream_t cs = on_producer ? ps : comm_stream(b->comm);
    // timing events stay out of a hipGraph capture (the timeline then reports -1)
    const bool capturing = stream_capturing(cs);
    bk.ready_timed = !capturing && (b->timeline >= 2 || (b->timeline == 1 && last));
    // the ready mark: a comm-stream chain waits on it; a producer-side tail needs
    // it only as the start of the timed tail (no packet otherwise)
    if (bk.ready_timed) {
      HIPB_RET(hipEventRecord(bk.ev_ready, ps));
    } else if (!on_producer) {
      HIPB_RET(hipEventRecord(bk.ev_sync, ps));
    }
    if (on_producer) {
      if (bi > 0) HIPB_RET(hipEventRecord(b->ev_comm, comm_stream(b->comm)));
      b->tail_ran_on_producer = true;
    } else {
      HIPB_RET(hipStreamWaitEvent(cs, bk.ready_timed ? bk.ev_ready : bk.ev_sync, 0));
    }
    const bool timed = !capturing && b->timeline >= 2;
    bk.timed = timed;
    // the producer-side tail at timeline >= 1: its last kernel marks "every chain
    // done" itself (finalize then records nothing) — level 2: ev_u1, level 1: ev_done
    const bool chain_end = !capturing && on_producer && b->timeline >= 1 && (b->do_unpack() || b->found_inf);
    hipEvent_t end_ev = chain_end ? (timed ? bk.ev_u1 : b->ev_done) : (timed ? bk.ev_u1 : nullptr);
    b->done_on_chain = chain_end;
    if (chain_end) b->done_ev = end_ev;
    // pack: pk0 an event packet before it (a kernel-carried START event costs more
    // stream time than a packet: 7.4 against 4.6 µs, profiles/r5/r5f_event_chain.jsonl),
    // t0 the kernel's own stop event (the pack or the grad-view scaling, whichever runs)
    // (the producer-side tail: no pk0 packet, ready is its pack's start)
    bk.pk0_is_ready = timed && on_producer;
    if (timed) {
      if (!on_producer) HIPB_RET(hipEventRecord(bk.ev_pk0, cs));
      arm(bk.plan, nullptr, bk.ev_t0);
      arm(bk.flat, nullptr, bk.ev_t0);
    }
    GS_TRY_RET(pack_raw(b, bk, cs));
    if (timed) {
      // the launch consumed the event of the plan it ran on; the other plan's is dropped,
      // and one left unconsumed on both (no kernel ran) is recorded here
      const bool taken = bk.plan->once_stop == nullptr || bk.flat->once_stop == nullptr;
      if (taken) {
        arm(bk.plan, nullptr, nullptr);
        arm(bk.flat, nullptr, nullptr);
      } else {
        arm(bk.flat, nullptr, nullptr);
        GS_TRY_RET(settle(bk.plan, cs));
      }
    }
    GS_TRY_RET(debug_sum(b, bk, 0, cs));
    if (on_producer && bi > 0) HIPB_RET(hipStreamWaitEvent(ps, b->ev_comm, 0));
    // The watchdog learns of the collective's completion through the stop event its
    // unpack kernel carries (the done mark, u1, or ev_wd), not through an event packet
    // after the collective: a packet costs ~4.7 µs of stream time, a kernel-carried
    // stop ~2.4 (scripts/micro/event_chain.hip) — the whole gap between the tail's
    // pack and unpack at N = 1 (scripts/tail_trace.py)
    // The event stands for one record (comm_track_event): the ring's next slot, or u1
    // at level 2, only once its previous record completed — a host that runs a whole
    // ring of steps ahead of the GPU gets a pooled packet after the collective instead.
    // At level 1 the producer-side tail's slot is also this step's done mark.
    const bool unpacks = b->do_unpack() || b->found_inf;
    hipEvent_t wd_ev = nullptr;
    if (!capturing && unpacks && comm_watching(b->comm)) {
      hipEvent_t cand = timed ? bk.ev_u1 : bk.ev_wd[bk.wd_next];
      if (hipEventQuery(cand) == hipSuccess) {
        wd_ev = cand;
        if (!timed) bk.wd_next = (bk.wd_next + 1) % kWdRing;
        if (chain_end) end_ev = b->done_ev = wd_ev;
      }
    }
    // no unpack (sharded buckets): the shards' consumer, when named, carries the mark
    GS_TRY_RET(launch_collective(b, bk, cs, wd_ev == nullptr, unpacks ? nullptr : b->mark_consumer));
    GS_TRY_RET(debug_sum(b, bk, 1, cs));
    // unpack: t1 a packet before it, its stop = u1 or the done mark; the collective lies
    // between t0 and t1
    if (unpacks) {
      if (timed) HIPB_RET(hipEventRecord(bk.ev_t1, cs));
      GS_TRY_RET(unpack_one(b, bk, cs, 0, nullptr, wd_ev ? wd_ev : end_ev));
      if (wd_ev) GS_TRY_RET(comm_track_event(b->comm, wd_ev));
    } else if (timed) {
      HIPB_RET(hipEventRecord(bk.ev_t1, cs));
      HIPB_RET(hipEventRecord(bk.ev_u1, cs));
    }
    bk.stream = cs;
  } else {
    GS_TRY_RET(pack_one(b, bk, b->producer));
  }
  bk.launched = true;
  return GS_OK;
}

int drain_ready(gs_bucketer* b, int32_t* ready_out, int32_t* n_ready) {
  int nr = 0;
  while (b->next_bucket < static_cast<int>(b->buckets.size()) &&
         b->buckets[b->next_bucket].pending == 0) {
    GS_TRY_RET(launch_bucket(b, b->next_bucket));
    if (ready_out) ready_out[nr] = b->next_bucket;
    ++nr;
    ++b->next_bucket;
  }
  if (n_ready) *n_ready = nr;
  return GS_OK;
}

}  // namespace

extern "C" {

int gs_bucketer_create(gs_comm* comm, int device_kind, int device, int n_params,
                       const int64_t* numels, int grad_dtype, int n_buckets,
                       const int32_t* bucket_counts, const int32_t* bucket_members,
                       int bucket_dtype, int64_t align_elems, float div_factor, int flags,
                       gs_bucketer** out) {
  GS_CHECK_ARG(out && numels && bucket_counts && bucket_members, "gs_bucketer_create: NULL argument");
  GS_CHECK_ARG(n_params >= 0 && n_buckets >= 0, "gs_bucketer_create: negative count");
  GS_CHECK_ARG(is_float_dtype(grad_dtype) && is_float_dtype(bucket_dtype),
               "gs_bucketer_create: grad and bucket dtypes must be floating");
  GS_CHECK_ARG(div_factor > 0.f, "gs_bucketer_create: div_factor must be > 0");
  GS_CHECK_ARG(!(flags & GS_BKT_AUTO_COLLECTIVE) || (comm && device_kind == GS_DEV_HIP),
               "gs_bucketer_create: AUTO_COLLECTIVE needs a HIP communicator");
  GS_CHECK_ARG(!(flags & GS_BKT_REDUCE_SCATTER) || comm,
               "gs_bucketer_create: REDUCE_SCATTER needs a communicator");
  auto* b = new gs_bucketer();
  b->comm = comm;
  b->kind = device_kind;
  b->device = device;
  b->n_params = n_params;
  b->grad_dtype = grad_dtype;
  b->bucket_dtype = bucket_dtype;
  b->align = align_elems;
  b->div = div_factor;
  b->flags = flags;
  b->numel.assign(numels, numels + n_params);
  b->loc_bucket.assign(n_params, -1);
  b->loc_intra.assign(n_params, -1);
  b->ready.assign(n_params, 0);
  b->buckets.resize(n_buckets);
  int pos = 0;
  auto bail = [&](int rc) {
    gs_bucketer_destroy(b);
    return rc;
  };
  // div_factor is the world size (DDP / ZeRO divide by it); without a
  // communicator (host / external collectives) it is the only source of it
  const int world = comm ? gs_comm_world(comm) : std::max(1, static_cast<int>(div_factor + 0.5f));
  for (int bi = 0; bi < n_buckets; ++bi) {
    Bucket& bk = b->buckets[bi];
    std::vector<int64_t> nm;
    for (int k = 0; k < bucket_counts[bi]; ++k) {
      const int32_t p = bucket_members[pos++];
      if (p < 0 || p >= n_params || b->loc_bucket[p] != -1)
        return bail(fail(GS_EINVAL, "gs_bucketer_create: bad or duplicate member " + std::to_string(p)));
      b->loc_bucket[p] = bi;
      b->loc_intra[p] = k;
      bk.params.push_back(p);
      nm.push_back(numels[p]);
    }
    int rc = gs_plan_create(device_kind, device, static_cast<int>(nm.size()), nm.data(), align_elems, &bk.plan);
    if (rc != GS_OK) return bail(rc);
    bk.numel = bk.plan->flat_numel;
    if (flags & (GS_BKT_REDUCE_SCATTER | GS_BKT_NO_UNPACK)) {
      // sharded consumers (ZeRO): pad so the bucket splits into `world` equal, aligned shards
      const int64_t q = static_cast<int64_t>(world) * (align_elems > 0 ? align_elems : 1);
      bk.numel = (bk.numel + q - 1) / q * q;
    }
    rc = gs_plan_create(device_kind, device, 1, &bk.numel, 0, &bk.flat);
    if (rc != GS_OK) return bail(rc);
    bk.pending = static_cast<int>(bk.params.size());
    bk.gdt = grad_dtype;
    bk.bdt = bucket_dtype;
    if (device_kind == GS_DEV_HIP) {
      if (hipEventCreate(&bk.ev_ready) != hipSuccess || hipEventCreate(&bk.ev_pk0) != hipSuccess ||
          hipEventCreate(&bk.ev_t0) != hipSuccess || hipEventCreate(&bk.ev_t1) != hipSuccess ||
          hipEventCreate(&bk.ev_u1) != hipSuccess ||
          hipEventCreateWithFlags(&bk.ev_sync, hipEventDisableTiming) != hipSuccess)
        return bail(fail(GS_EHIP, "gs_bucketer_create: event creation failed"));
      for (hipEvent_t& ev : bk.ev_wd)
        if (hipEventCreate(&ev) != hipSuccess) return bail(fail(GS_EHIP, "gs_bucketer_create: event creation failed"));
    }
  }
  for (int p = 0; p < n_params; ++p)
    if (b->loc_bucket[p] < 0)
      return bail(fail(GS_EINVAL, "gs_bucketer_create: parameter " + std::to_string(p) + " is in no bucket"));
  if (device_kind == GS_DEV_HIP &&
      (hipEventCreateWithFlags(&b->ev_comm, hipEventDisableTiming) != hipSuccess ||
       hipEventCreate(&b->ev_done) != hipSuccess ||
       hipEventCreateWithFlags(&b->ev_done_sync, hipEventDisableTiming) != hipSuccess))
    return bail(fail(GS_EHIP, "gs_bucketer_create: event creation failed"));
  *out = b;
  return GS_OK;
}

int gs_bucketer_destroy(gs_bucketer* b) {
  if (!b) return GS_OK;
  if (b->hip() && b->comm) (void)hipStreamSynchronize(comm_stream(b->comm));
  if (b->hip() && b->comm) {  // the watchdog may still hold the tail's marks (comm_track_event)
    comm_forget_event(b->comm, b->ev_done);
    for (Bucket& bk : b->buckets) {
      comm_forget_event(b->comm, bk.ev_u1);
      for (hipEvent_t ev : bk.ev_wd) comm_forget_event(b->comm, ev);
    }
  }
  for (Bucket& bk : b->buckets) {
    gs_plan_destroy(bk.plan);
    gs_plan_destroy(bk.flat);
    for (hipEvent_t ev : {bk.ev_ready, bk.ev_pk0, bk.ev_t0, bk.ev_t1, bk.ev_u1, bk.ev_sync})
      if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : bk.ev_wd)
      if (ev) (void)hipEventDestroy(ev);
  }
  if (b->ev_done) (void)hipEventDestroy(b->ev_done);
  if (b->ev_done_sync) (void)hipEventDestroy(b->ev_done_sync);
  if (b->ev_comm) (void)hipEventDestroy(b->ev_comm);
  delete b;
  return GS_OK;
}

int gs_bucketer_bucket_numel(gs_bucketer* b, int bucket, int64_t* out) {
  GS_CHECK_ARG(b && out && bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "bad bucket");
  *out = b->buckets[bucket].numel;
  return GS_OK;
}

int gs_bucketer_shard_numel(gs_bucketer* b, int bucket, int64_t* out) {
  GS_CHECK_ARG(b && out && bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "bad bucket");
  const int w = b->comm ? gs_comm_world(b->comm) : 1;
  *out = b->buckets[bucket].numel / w;
  return GS_OK;
}

int gs_bucketer_param_location(gs_bucketer* b, int param, int32_t* bucket, int64_t* offset) {
  GS_CHECK_ARG(b && param >= 0 && param < b->n_params, "gs_bucketer_param_location: bad param");
  const int bi = b->loc_bucket[param];
  if (bucket) *bucket = bi;
  if (offset) *offset = b->buckets[bi].plan->off[b->loc_intra[param]];
  return GS_OK;
}

int gs_bucketer_set_bucket_dtype(gs_bucketer* b, int bucket, int grad_dtype, int bucket_dtype) {
  GS_CHECK_ARG(b && bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "bad bucket");
  GS_CHECK_ARG(is_float_dtype(grad_dtype) && is_float_dtype(bucket_dtype),
               "gs_bucketer_set_bucket_dtype: grad and bucket dtypes must be floating");
  std::lock_guard<std::mutex> lk(b->mu);
  if (b->prepared) return fail(GS_ESTATE, "gs_bucketer_set_bucket_dtype inside a backward");
  b->buckets[bucket].gdt = grad_dtype;
  b->buckets[bucket].bdt = bucket_dtype;
  return GS_OK;
}

int gs_bucketer_set_bucket_buffer(gs_bucketer* b, int bucket, void* ptr) {
  GS_CHECK_ARG(b && bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "bad bucket");
  GS_CHECK_ARG(ptr != nullptr, "gs_bucketer_set_bucket_buffer: NULL storage");
  Bucket& bk = b->buckets[bucket];
  bk.buf = ptr;
  void* one[1] = {ptr};
  return gs_plan_set_ptrs(bk.flat, 0, one, nullptr);
}

int gs_bucketer_set_shard_buffer(gs_bucketer* b, int bucket, void* ptr) {
  GS_CHECK_ARG(b && bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "bad bucket");
  b->buckets[bucket].shard = ptr;
  return GS_OK;
}

int gs_bucketer_prepare(gs_bucketer* b, float* sqnorm_dev) {
  GS_CHECK_ARG(b != nullptr, "gs_bucketer_prepare: NULL bucketer");
  std::lock_guard<std::mutex> lk(b->mu);
  std::fill(b->ready.begin(), b->ready.end(), 0);
  for (Bucket& bk : b->buckets) {
    bk.pending = static_cast<int>(bk.params.size());
    bk.launched = false;
    bk.unpacked = false;
  }
  b->next_bucket = 0;
  b->tail_ran_on_producer = false;
  b->prepared = true;
  b->sqnorm = sqnorm_dev;
  b->sq_count = 0;
  b->producer = nullptr;
  return GS_OK;
}

int gs_bucketer_mark_ready(gs_bucketer* b, int param, const void* grad, void* stream,
                           int32_t* ready_out, int32_t* n_ready) {
  GS_CHECK_ARG(b != nullptr, "gs_bucketer_mark_ready: NULL bucketer");
  std::lock_guard<std::mutex> lk(b->mu);
  if (n_ready) *n_ready = 0;
  if (!b->prepared)
    return fail(GS_ESTATE, "mark_ready called outside of a synchronising backward (prepare not called)");
  GS_CHECK_ARG(param >= 0 && param < b->n_params, "gs_bucketer_mark_ready: param out of range");
  if (b->ready[param])
    return fail(GS_ESTATE, "Expected to mark a variable ready only once. Parameter " +
                               std::to_string(param) + " was marked twice in one backward.");
  b->ready[param] = 1;
  if (b->producer == nullptr) b->producer = stream;
  Bucket& bk = b->buckets[b->loc_bucket[param]];
  plan_set_one(bk.plan, 1, b->loc_intra[param], const_cast<void*>(grad));
  bk.pending -= 1;
  return drain_ready(b, ready_out, n_ready);
}

int gs_bucketer_mark_unused(gs_bucketer* b, void* stream, int32_t* ready_out, int32_t* n_ready) {
  GS_CHECK_ARG(b != nullptr, "gs_bucketer_mark_unused: NULL bucketer");
  std::lock_guard<std::mutex> lk(b->mu);
  if (!b->prepared) return fail(GS_ESTATE, "mark_unused outside of a synchronising backward");
  if (b->producer == nullptr) b->producer = stream;
  for (int p = 0; p < b->n_params; ++p) {
    if (b->ready[p]) continue;
    b->ready[p] = 1;
    Bucket& bk = b->buckets[b->loc_bucket[p]];
    // a NULL source packs zeros and a NULL destination is skipped by unpack
    plan_set_one(bk.plan, 1, b->loc_intra[p], nullptr);
    bk.pending -= 1;
  }
  return drain_ready(b, ready_out, n_ready);
}

int gs_bucketer_finalize(gs_bucketer* b, void* stream) {
  GS_CHECK_ARG(b != nullptr, "gs_bucketer_finalize: NULL bucketer");
  GsRange range("gsync.finalize");
  std::lock_guard<std::mutex> lk(b->mu);
  if (!b->prepared) return fail(GS_ESTATE, "finalize without prepare");
  if (b->next_bucket != static_cast<int>(b->buckets.size())) {
    std::string missing;
    int shown = 0;
    for (int p = 0; p < b->n_params && shown < 16; ++p)
      if (!b->ready[p]) { missing += (shown ? ", " : "") + std::to_string(p); ++shown; }
    return fail(GS_ESTATE,
                "Expected to have finished reduction in the prior iteration before starting a new "
                "one. Parameter indices which did not receive grad: " + missing);
  }
  if (b->hip() && b->auto_coll()) {
    hipStream_t ps = static_cast<hipStream_t>(stream);
    const bool on_ps = b->tail_ran_on_producer && ps == static_cast<hipStream_t>(b->producer);
    hipStream_t ds = on_ps ? ps : comm_stream(b->comm);
    b->done_timed = b->timeline >= 1 && !stream_capturing(ds);
    hipEvent_t done = b->done_timed ? b->ev_done : b->ev_done_sync;
    // the last bucket ran on the producer after joining the comm stream:
    // everything is already ordered before this point; otherwise join the comm stream.
    // A producer-side tail whose last kernel carried the done mark records nothing.
    const bool marked = on_ps && b->done_on_chain;
    if (!on_ps || (b->done_timed && !marked)) {
      HIPB_RET(hipEventRecord(done, ds));
      b->done_ev = done;
    }
    b->done_on_chain = false;
    if (!on_ps) HIPB_RET(hipStreamWaitEvent(ps, done, 0));
  } else {
    // external collectives (comm hook / process group) are done by now
    for (Bucket& bk : b->buckets) {
      if (bk.unpacked) continue;
      GS_TRY_RET(debug_sum(b, bk, 1, stream));
      if (b->do_unpack() || b->found_inf) GS_TRY_RET(unpack_one(b, bk, stream, 0));
    }
  }
  b->prepared = false;
  return GS_OK;
}

int gs_bucketer_set_div_factor(gs_bucketer* b, float div_factor) {
  GS_CHECK_ARG(b != nullptr, "gs_bucketer_set_div_factor: NULL bucketer");
  GS_CHECK_ARG(div_factor > 0.f, "gs_bucketer_set_div_factor: div_factor must be > 0");
  std::lock_guard<std::mutex> lk(b->mu);
  b->div = div_factor;
  return GS_OK;
}

int gs_bucketer_set_found_inf(gs_bucketer* b, float* found_inf) {
  GS_CHECK_ARG(b != nullptr, "gs_bucketer_set_found_inf: NULL bucketer");
  GS_CHECK_ARG(!(b->flags & (GS_BKT_REDUCE_SCATTER | GS_BKT_NO_UNPACK)) || found_inf == nullptr,
               "gs_bucketer_set_found_inf: sharded (ZeRO) buckets check their shard in the optimizer");
  std::lock_guard<std::mutex> lk(b->mu);
  b->found_inf = found_inf;
  return GS_OK;
}

int gs_bucketer_set_debug(gs_bucketer* b, float* sums) {
  GS_CHECK_ARG(b != nullptr, "gs_bucketer_set_debug: NULL bucketer");
  GS_CHECK_ARG(!(b->flags & GS_BKT_REDUCE_SCATTER) || sums == nullptr,
               "gs_bucketer_set_debug: reduce-scatter buckets keep only a shard after the collective");
  std::lock_guard<std::mutex> lk(b->mu);
  b->dbg = sums;
  return GS_OK;
}

int gs_bucketer_unpack_bucket(gs_bucketer* b, int bucket, void* stream) {
  GS_CHECK_ARG(b && bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "bad bucket");
  std::lock_guard<std::mutex> lk(b->mu);
  Bucket& bk = b->buckets[bucket];
  if (!bk.launched) return fail(GS_ESTATE, "unpack of a bucket that was never launched");
  return unpack_one(b, bk, stream, 0);
}

int gs_bucketer_last_timing(gs_bucketer* b, int bucket, float* out) {
  GS_CHECK_ARG(b && out && bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "bad bucket");
  for (int i = 0; i < 5; ++i) out[i] = -1.f;
  Bucket& bk = b->buckets[bucket];
  if (!b->hip() || !b->auto_coll()) return GS_OK;
  if (bk.timed && bk.ready_timed) {
    HIPB_RET(hipEventSynchronize(bk.ev_u1));
    hipEvent_t pk0 = bk.pk0_is_ready ? bk.ev_ready : bk.ev_pk0;
    HIPB_RET(hipEventElapsedTime(&out[0], bk.ev_ready, pk0));
    HIPB_RET(hipEventElapsedTime(&out[1], pk0, bk.ev_t0));
    HIPB_RET(hipEventElapsedTime(&out[2], bk.ev_t0, bk.ev_t1));
    HIPB_RET(hipEventElapsedTime(&out[3], bk.ev_t1, bk.ev_u1));
  }
  if (bk.ready_timed && b->done_timed && b->done_ev) {
    HIPB_RET(hipEventSynchronize(b->done_ev));
    HIPB_RET(hipEventElapsedTime(&out[4], bk.ev_ready, b->done_ev));
  }
  return GS_OK;
}

int gs_bucketer_bucket_stream(gs_bucketer* b, int bucket, void** stream) {
  GS_CHECK_ARG(b != nullptr && stream != nullptr, "gs_bucketer_bucket_stream: NULL argument");
  std::lock_guard<std::mutex> lk(b->mu);
  GS_CHECK_ARG(bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "gs_bucketer_bucket_stream: bad bucket");
  const Bucket& bk = b->buckets[bucket];
  *stream = (b->hip() && b->auto_coll() && bk.launched) ? bk.stream : nullptr;
  return GS_OK;
}

int gs_bucketer_set_timeline(gs_bucketer* b, int level) {
  GS_CHECK_ARG(b != nullptr && level >= 0 && level <= 2, "gs_bucketer_set_timeline: level 0, 1 or 2");
  std::lock_guard<std::mutex> lk(b->mu);
  if (b->prepared) return fail(GS_ESTATE, "gs_bucketer_set_timeline inside a backward");
  b->timeline = level;
  return GS_OK;
}

int gs_bucketer_set_mark_consumer(gs_bucketer* b, gs_plan* consumer) {
  GS_CHECK_ARG(b != nullptr, "gs_bucketer_set_mark_consumer: NULL bucketer");
  std::lock_guard<std::mutex> lk(b->mu);
  GS_CHECK_ARG(consumer == nullptr || !b->do_unpack(),
               "gs_bucketer_set_mark_consumer: only sharded (NO_UNPACK / REDUCE_SCATTER) buckets hand marks on");
  b->mark_consumer = consumer;
  return GS_OK;
}

int gs_bucketer_first_pack_plan(gs_bucketer* b, gs_plan** out) {
  GS_CHECK_ARG(b != nullptr && out != nullptr, "gs_bucketer_first_pack_plan: NULL argument");
  *out = b->buckets.empty() ? nullptr : b->buckets[0].plan;
  return GS_OK;
}

int gs_bucketer_last_comm_ms(gs_bucketer* b, int bucket, float* ms) {
  GS_CHECK_ARG(b && ms && bucket >= 0 && bucket < static_cast<int>(b->buckets.size()), "bad bucket");
  Bucket& bk = b->buckets[bucket];
  *ms = -1.f;
  if (!bk.timed) return GS_OK;
  HIPB_RET(hipEventSynchronize(bk.ev_t1));
  HIPB_RET(hipEventElapsedTime(ms, bk.ev_t0, bk.ev_t1));
  return GS_OK;
}

}  // extern "C"
