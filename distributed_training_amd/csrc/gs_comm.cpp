// libgsync communicator: one RCCL communicator per process (one process per
// GPU) with a library-owned non-blocking, high-priority stream, so that
// gradient collectives run beside the backward kernels instead of behind
// them.  The unique id is exchanged by the caller (torch.distributed store).
//
// replaces: torch ProcessGroupNCCL (T:include/torch/csrc/distributed/c10d/
// ProcessGroupNCCL.hpp:849 allreduce, :836 broadcast, :872 _allgather_base,
// :887-892 reduce_scatter; dedicated ncclStreams_ :1398).
//
// Failure detection ("RCCL error checking plus ncclCommAbort on
// a timeout"; torch's ProcessGroupNCCL watchdog, T:.../ProcessGroupNCCL.hpp:59-68,
// 156): with a timeout set, every collective enqueued through the
// communicator records a completion event; a watchdog thread polls the oldest
// in-flight one and ncclCommGetAsyncError, and aborts the communicator
// (ncclCommAbort) when a collective has been in flight longer than the
// timeout or RCCL reports an asynchronous error.  Every later call on the
// communicator then fails with the reason (gs_comm_status).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <algorithm>
#include <chrono>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>

#include "gs_common.h"

struct gs_comm {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int rank = 0, world = 1, device = 0;
  std::atomic<bool> aborted{false};
  std::string abort_reason;  // written once, by the winner of `aborted`, under reason_mu
  std::mutex reason_mu;
  std::mutex mu;  // enqueue (comm_enqueue) vs abort vs the watchdog's bookkeeping
  // steady-clock ns at which the enqueue now holding `mu` started (0: none):
  // the watchdog times a blocked enqueue from here, not from when it noticed
  std::atomic<int64_t> enq_since{0};
  // watchdog
  int64_t timeout_ms = 0;
  std::thread wd;
  std::atomic<bool> wd_stop{false};
  struct Inflight {
    hipEvent_t ev;
    std::chrono::steady_clock::time_point t0;
    bool from_pool = false;  // a caller-list entry whose event the pool owns (a lapsed deferral)
  };
  // collectives whose mark waits for a consumer plan's next launch (comm_enqueue with a
  // consumer): untracked until that launch commits its mark — or, if it has not come
  // within kDeferLimitMs (the host blocked or idle between the collective and its
  // consumer, e.g. a loss.item() before the next backward), the watchdog records a
  // packet on the collective's stream itself and times it from the enqueue
  struct Deferred {
    const gs_plan* consumer;  // nullptr once that plan is destroyed
    hipStream_t stream;
    std::chrono::steady_clock::time_point t0;
  };
  std::vector<Deferred> deferred;
  // packets recorded after a collective (comm_track_locked), in enqueue order: retired
  // from the front, so each poll queries the entries it retires and one pending one
  std::deque<Inflight> pooled;
  // the callers' own events (comm_track_event: the bucketer's unpack-carried marks), one
  // entry per event, each standing for one record; a few of them are queried per poll
  std::vector<Inflight> caller;
  size_t caller_next = 0;  // rotation cursor over `caller`
  // marks carried by consumer plans' launches (comm_mark_take): a ring, each slot
  // re-recorded only after its previous record completed
  std::vector<hipEvent_t> mark_ring;
  size_t mark_next = 0;
  std::vector<hipEvent_t> ev_pool;
};

namespace gs {
namespace {

// live communicators: a consumer plan holds its deferring communicator's address
// until its next launch, which checks here first (comm_mark_take), so a
// communicator destroyed in between is never touched
std::mutex g_live_mu;
std::vector<gs_comm*> g_live;
bool comm_live_locked(gs_comm* c) { return std::find(g_live.begin(), g_live.end(), c) != g_live.end(); }
// the streams of destroyed communicators (until a new stream reuses the handle): a plan
// whose last launch ran on one must not record its ordering event there (stream_destroyed)
std::vector<void*> g_dead_streams;

int rccl_fail(ncclResult_t r, const char* what) {
  return fail(GS_ERCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

#define RCCL_RET(expr)                          \
  do {                                          \
    ncclResult_t _r = (expr);                   \
    if (_r != ncclSuccess) return rccl_fail(_r, #expr); \
  } while (0)

#define HIPC_RET(expr)                                                               \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess)                                                            \
      return fail(GS_EHIP, std::string(#expr " failed: ") + hipGetErrorString(_e));  \
  } while (0)

int to_nccl_dtype(int dt, ncclDataType_t* out) {
  switch (dt) {
    case GS_F32: *out = ncclFloat32; return GS_OK;
    case GS_BF16: *out = ncclBfloat16; return GS_OK;
    case GS_F16: *out = ncclFloat16; return GS_OK;
    case GS_F64: *out = ncclFloat64; return GS_OK;
    case GS_I64: *out = ncclInt64; return GS_OK;
    case GS_I32: *out = ncclInt32; return GS_OK;
    case GS_U8: *out = ncclUint8; return GS_OK;
    default: return fail(GS_EINVAL, "unsupported collective dtype");
  }
}

int to_nccl_op(int op, ncclRedOp_t* out) {
  switch (op) {
    case GS_SUM: *out = ncclSum; return GS_OK;
    case GS_PROD: *out = ncclProd; return GS_OK;
    case GS_MAX: *out = ncclMax; return GS_OK;
    case GS_MIN: *out = ncclMin; return GS_OK;
    case GS_AVG: *out = ncclAvg; return GS_OK;
    default: return fail(GS_EINVAL, "unsupported reduce op");
  }
}

// NULL is HIP's legacy default stream, as everywhere in the ABI: torch's
// default stream has handle 0, and mapping it to the (non-blocking) comm
// stream would drop the order with the work the caller queued before the
// collective (a pack, a fill).  gs_comm_stream() hands out the comm stream.
hipStream_t pick(gs_comm*, void* stream) { return static_cast<hipStream_t>(stream); }

// First caller wins (compare-exchange on `aborted`), so the reason is written
// once even when the watchdog aborts a blocked enqueue without c->mu; every
// other caller holds c->mu.
void abort_locked(gs_comm* c, const std::string& why) {
  {
    std::lock_guard<std::mutex> lk(c->reason_mu);
    bool expected = false;
    if (!c->aborted.compare_exchange_strong(expected, true)) return;
    c->abort_reason = why;
  }
  if (c->comm) (void)ncclCommAbort(c->comm);
}

std::string abort_reason(gs_comm* c) {
  std::lock_guard<std::mutex> lk(c->reason_mu);
  return c->abort_reason;
}

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// how long a deferred mark may wait for its consumer's launch before the watchdog
// records a packet for it (at most half the timeout)
constexpr int64_t kDeferLimitMs = 1000;

// > 0 while a graph capture is being recorded (gs_watchdog_pause): event
// queries from the watchdog thread are not allowed during a global-mode capture
std::atomic<int> g_wd_pause{0};

void watchdog_loop(gs_comm* c) {
  (void)hipSetDevice(c->device);
  using clk = std::chrono::steady_clock;
  while (!c->wd_stop.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    if (g_wd_pause.load() > 0) continue;
    // enqueues hold c->mu for the few microseconds of an RCCL enqueue, so the
    // abort never frees the communicator under a concurrent enqueue; only an
    // enqueue that itself hangs (holding the lock past the timeout, measured
    // from the enqueue's own start) is aborted without it — that enqueue is
    // what the abort has to break.  A first collective that blocks in RCCL's
    // lazy connection setup while a peer is late counts against the timeout
    // too (as ProcessGroupNCCL's watchdog counts it): set the timeout above the
    // slowest expected start-up.
    std::unique_lock<std::mutex> lk(c->mu, std::try_to_lock);
    if (!lk.owns_lock()) {
      const int64_t t0 = c->enq_since.load();
      const int64_t held_ms = t0 ? (now_ns() - t0) / 1000000 : 0;
      if (c->timeout_ms > 0 && held_ms > c->timeout_ms)
        abort_locked(c, "watchdog: an RCCL enqueue has been blocked for " + std::to_string(held_ms) +
                            " ms (timeout " + std::to_string(c->timeout_ms) + " ms); communicator aborted");
      continue;
    }
    if (c->aborted.load()) continue;
    ncclResult_t async = ncclSuccess;
    if (c->comm && ncclCommGetAsyncError(c->comm, &async) == ncclSuccess && async != ncclSuccess &&
        async != ncclInProgress) {
      abort_locked(c, std::string("RCCL asynchronous error: ") + ncclGetErrorString(async));
      continue;
    }
    // Pooled packets: retired from the front while complete (at most kRetire a poll, so
    // the lock is never held for a long backlog), the front's age decides a timeout —
    // every later packet was enqueued after it.  The lock is held for the queries of
    // one poll: an enqueue waiting on it (the exposed tail's collective at the end of
    // backward) waits for them.
    constexpr int kRetire = 64;
    const auto now = clk::now();
    auto age_ms = [&](const gs_comm::Inflight& f) {
      return std::chrono::duration_cast<std::chrono::milliseconds>(now - f.t0).count();
    };
    bool front_pending = false;
    for (int n = 0; n < kRetire && !c->pooled.empty(); ++n) {
      const gs_comm::Inflight& f = c->pooled.front();
      if (hipEventQuery(f.ev) != hipSuccess) {
        front_pending = true;
        break;
      }
      c->ev_pool.push_back(f.ev);
      c->pooled.pop_front();
    }
    if (front_pending && c->timeout_ms > 0 && age_ms(c->pooled.front()) > c->timeout_ms) {
      abort_locked(c, "watchdog: a collective has been in flight for " + std::to_string(age_ms(c->pooled.front())) +
                          " ms (timeout " + std::to_string(c->timeout_ms) + " ms); communicator aborted");
      continue;
    }
    // Deferred marks whose consumer has not launched within kDeferLimitMs: a packet on
    // the collective's stream now (stream order: it completes only after the
    // collective), watched from the collective's enqueue like any caller entry
    if (!c->deferred.empty()) {
      const int64_t limit = std::min<int64_t>(kDeferLimitMs, c->timeout_ms > 0 ? c->timeout_ms / 2 : kDeferLimitMs);
      size_t w = 0;
      for (size_t i = 0; i < c->deferred.size(); ++i) {
        const gs_comm::Deferred& d = c->deferred[i];
        const int64_t age = std::chrono::duration_cast<std::chrono::milliseconds>(now - d.t0).count();
        hipEvent_t ev = nullptr;
        if (age > limit && !stream_capturing(d.stream)) {
          if (!c->ev_pool.empty()) {
            ev = c->ev_pool.back();
            c->ev_pool.pop_back();
          } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            ev = nullptr;
          }
          if (ev && hipEventRecord(ev, d.stream) != hipSuccess) {
            c->ev_pool.push_back(ev);
            ev = nullptr;
          }
        }
        if (ev) c->caller.push_back({ev, d.t0, true});
        else c->deferred[w++] = d;
      }
      c->deferred.resize(w);
    }
    // The callers' events: every entry past the timeout is queried, of the others
    // kQueries a poll in rotation; a completed entry leaves the list.
    constexpr size_t kQueries = 4;
    const size_t n = c->caller.size();
    if (n == 0) continue;
    std::vector<char> done(n, 0);
    size_t queried = 0;
    bool aborted = false;
    for (size_t k = 0; k < n; ++k) {
      const size_t i = (c->caller_next + k) % n;
      const gs_comm::Inflight& f = c->caller[i];
      const int64_t age = age_ms(f);
      const bool overdue = c->timeout_ms > 0 && age > c->timeout_ms;
      if (!overdue && queried >= kQueries) continue;
      if (!overdue) ++queried;
      if (hipEventQuery(f.ev) == hipSuccess) {
        done[i] = 1;
      } else if (overdue) {
        abort_locked(c, "watchdog: a collective has been in flight for " + std::to_string(age) + " ms (timeout " +
                            std::to_string(c->timeout_ms) + " ms); communicator aborted");
        aborted = true;
        break;
      }
    }
    if (aborted) continue;
    size_t w = 0;
    for (size_t i = 0; i < n; ++i) {
      if (!done[i]) c->caller[w++] = c->caller[i];
      else if (c->caller[i].from_pool) c->ev_pool.push_back(c->caller[i].ev);
    }
    c->caller.resize(w);
    c->caller_next = w ? (c->caller_next + kQueries) % w : 0;
  }
}

}  // namespace

// used by the bucketer
ncclComm_t comm_handle(gs_comm* c) { return c->comm; }
hipStream_t comm_stream(gs_comm* c) { return c->stream; }
int comm_dtype(int dt, ncclDataType_t* out) { return to_nccl_dtype(dt, out); }

// caller holds c->mu: hand the completion of the collective just enqueued on
// `stream` to the watchdog
int comm_track_locked(gs_comm* c, hipStream_t stream) {
  // a collective recorded into a hipGraph runs at replay, not now: not tracked
  if (c->timeout_ms <= 0 || stream_capturing(stream)) return GS_OK;
  hipEvent_t ev;
  if (!c->ev_pool.empty()) {
    ev = c->ev_pool.back();
    c->ev_pool.pop_back();
  } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    return fail(GS_EHIP, "watchdog: event creation failed");
  }
  if (hipEventRecord(ev, stream) != hipSuccess) {
    c->ev_pool.push_back(ev);
    return fail(GS_EHIP, "watchdog: event record failed");
  }
  c->pooled.push_back({ev, std::chrono::steady_clock::now()});
  return GS_OK;
}

// A collective enqueued untracked (comm_enqueue track = false) handed to the
// watchdog through an event of the caller's that its stream records after it —
// the bucketer: each bucket's unpack kernel carries the stop event, so no event
// packet sits between a collective and its unpack (~4.7 µs of stream time each,
// scripts/micro/event_chain.hip).  The caller keeps the event and calls
// comm_forget_event before destroying it.
// One entry per event, standing for ONE record: the caller re-records an event only
// after its previous record completed (the bucketer queries it first and rotates
// through a ring of them, falling back to a pooled packet when the host runs that far
// ahead), so restarting the entry's clock here never hides a pending collective.
int comm_track_event(gs_comm* c, hipEvent_t ev) {
  if (!c || !ev) return GS_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->timeout_ms <= 0) return GS_OK;
  const auto now = std::chrono::steady_clock::now();
  for (auto& f : c->caller)
    if (f.ev == ev) {
      f.t0 = now;
      return GS_OK;
    }
  c->caller.push_back({ev, now});
  return GS_OK;
}

bool comm_watching(gs_comm* c) {
  if (!c) return false;
  std::lock_guard<std::mutex> lk(c->mu);
  return c->timeout_ms > 0;
}

void comm_forget_event(gs_comm* c, hipEvent_t ev) {
  if (!c || !ev) return;
  std::lock_guard<std::mutex> lk(c->mu);
  c->caller.erase(std::remove_if(c->caller.begin(), c->caller.end(),
                                 [ev](const gs_comm::Inflight& f) { return f.ev == ev; }),
                  c->caller.end());
}

// Enqueue one RCCL collective under c->mu: liveness check, enqueue and
// watchdog tracking are atomic with respect to the watchdog's abort.
// consumer (nullable): the plan whose next launch is stream-ordered after this
// collective; with a watchdog running (and not under capture) the collective's
// mark is deferred to that launch's stop event instead of a packet after it.
int comm_enqueue(gs_comm* c, hipStream_t stream, const std::function<ncclResult_t()>& fn, const char* what,
                 bool track = true, gs_plan* consumer = nullptr) {
  if (!c) return fail(GS_EINVAL, "no communicator");
  GsRange range(what);
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->aborted.load()) return fail(GS_ERCCL, "communicator aborted: " + abort_reason(c));
  c->enq_since.store(now_ns());
  const ncclResult_t r = fn();
  c->enq_since.store(0);
  if (r != ncclSuccess) return rccl_fail(r, what);
  if (!track) return GS_OK;
  if (consumer && consumer->kind == GS_DEV_HIP && consumer->n > 0 && !consumer->segs.empty() &&
      c->timeout_ms > 0 && !stream_capturing(stream)) {
    consumer->watch_comm = c;
    c->deferred.push_back({consumer, stream, std::chrono::steady_clock::now()});
    return GS_OK;
  }
  return comm_track_locked(c, stream);
}

bool stream_destroyed(void* stream) {
  if (!stream) return false;
  std::lock_guard<std::mutex> live(g_live_mu);
  return std::find(g_dead_streams.begin(), g_dead_streams.end(), stream) != g_dead_streams.end();
}

int comm_mark_take(gs_comm* c, void** ev) {
  *ev = nullptr;
  std::lock_guard<std::mutex> live(g_live_mu);
  if (!c || !comm_live_locked(c)) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->timeout_ms <= 0 || c->aborted.load()) return 0;
  constexpr size_t kRing = 16;
  if (c->mark_ring.empty()) {
    for (size_t i = 0; i < kRing; ++i) {
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) break;
      c->mark_ring.push_back(e);
    }
    if (c->mark_ring.empty()) return 1;  // no event: a pooled packet after the launch
  }
  hipEvent_t e = c->mark_ring[c->mark_next];
  if (hipEventQuery(e) != hipSuccess) return 1;  // its previous record is still pending
  c->mark_next = (c->mark_next + 1) % c->mark_ring.size();
  *ev = e;
  return 1;
}

int comm_mark_commit(gs_comm* c, void* ev, void* stream, const gs_plan* consumer) {
  std::lock_guard<std::mutex> live(g_live_mu);
  if (!c || !comm_live_locked(c)) return GS_OK;
  hipEvent_t e = static_cast<hipEvent_t>(ev);
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->timeout_ms <= 0) return GS_OK;
  // the collectives deferred to this consumer: its launch is stream-ordered after them,
  // so its mark covers them; the clock runs from the oldest one's enqueue
  auto t0 = std::chrono::steady_clock::now();
  bool any = false;
  size_t w = 0;
  for (size_t i = 0; i < c->deferred.size(); ++i) {
    if (c->deferred[i].consumer == consumer) {
      t0 = std::min(t0, c->deferred[i].t0);
      any = true;
    } else {
      c->deferred[w++] = c->deferred[i];
    }
  }
  c->deferred.resize(w);
  if (!any) return GS_OK;  // the watchdog already recorded their packets
  if (!e) {
    // the packet joins the FIFO behind younger entries with its older clock: it is timed
    // once it reaches the front, at most the deferral window (<= 1 s) late
    const size_t before = c->pooled.size();
    GS_TRY_RET(comm_track_locked(c, static_cast<hipStream_t>(stream)));
    if (c->pooled.size() > before) c->pooled.back().t0 = t0;
    return GS_OK;
  }
  for (auto& f : c->caller)
    if (f.ev == e) {
      f.t0 = t0;
      return GS_OK;
    }
  c->caller.push_back({e, t0});
  return GS_OK;
}

void comm_forget_consumer(const gs_plan* consumer) {
  std::lock_guard<std::mutex> live(g_live_mu);
  for (gs_comm* c : g_live) {
    std::lock_guard<std::mutex> lk(c->mu);
    for (auto& d : c->deferred)
      if (d.consumer == consumer) d.consumer = nullptr;  // the watchdog's packet covers it
  }
}

}  // namespace gs

using namespace gs;

extern "C" {

int gs_comm_unique_id_bytes(void) { return static_cast<int>(sizeof(ncclUniqueId)); }

int gs_comm_get_unique_id(uint8_t* out) {
  GS_CHECK_ARG(out != nullptr, "gs_comm_get_unique_id: NULL out");
  ncclUniqueId id;
  RCCL_RET(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
  return GS_OK;
}

int gs_comm_create(int rank, int world, const uint8_t* uid, int device, gs_comm** out) {
  return gs_comm_create_ex(rank, world, uid, device, 0, out);
}

int gs_comm_create_ex(int rank, int world, const uint8_t* uid, int device, int max_ctas, gs_comm** out) {
  GS_CHECK_ARG(out && uid, "gs_comm_create: NULL argument");
  GS_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "gs_comm_create: bad rank/world");
  if (hip_device_count() <= device) return fail(GS_ENODEV, "gs_comm_create: no HIP device");
  HIPC_RET(hipSetDevice(device));
  gs_comm* c = new gs_comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  hipError_t e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi);
  if (e != hipSuccess) {
    delete c;
    return fail(GS_EHIP, std::string("hipStreamCreateWithPriority: ") + hipGetErrorString(e));
  }
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  ncclResult_t r;
  if (max_ctas > 0) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.maxCTAs = max_ctas;
    cfg.minCTAs = 1;
    r = ncclCommInitRankConfig(&c->comm, world, id, rank, &cfg);
  } else {
    r = ncclCommInitRank(&c->comm, world, id, rank);
  }
  if (r != ncclSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return rccl_fail(r, "ncclCommInitRank");
  }
  {
    std::lock_guard<std::mutex> live(g_live_mu);
    g_live.push_back(c);
    g_dead_streams.erase(std::remove(g_dead_streams.begin(), g_dead_streams.end(), static_cast<void*>(c->stream)),
                         g_dead_streams.end());
  }
  *out = c;
  return GS_OK;
}

int gs_comm_destroy(gs_comm* c) {
  if (!c) return GS_OK;
  {
    std::lock_guard<std::mutex> live(g_live_mu);
    g_live.erase(std::remove(g_live.begin(), g_live.end(), c), g_live.end());
  }
  if (c->wd.joinable()) {
    c->wd_stop.store(true);
    c->wd.join();
  }
  (void)hipSetDevice(c->device);
  if (c->stream && !c->aborted.load()) (void)hipStreamSynchronize(c->stream);
  for (auto& f : c->pooled) (void)hipEventDestroy(f.ev);  // the caller's events stay the caller's
  for (auto& f : c->caller)
    if (f.from_pool) (void)hipEventDestroy(f.ev);  // ... but a lapsed deferral's packet is ours
  for (hipEvent_t ev : c->ev_pool) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : c->mark_ring) (void)hipEventDestroy(ev);
  if (c->comm && !c->aborted.load()) (void)ncclCommDestroy(c->comm);
  if (c->stream) {
    {
      std::lock_guard<std::mutex> live(g_live_mu);
      g_dead_streams.push_back(c->stream);
    }
    (void)hipStreamDestroy(c->stream);
  }
  delete c;
  return GS_OK;
}

int gs_comm_abort(gs_comm* c) {
  GS_CHECK_ARG(c != nullptr, "gs_comm_abort: NULL comm");
  std::lock_guard<std::mutex> lk(c->mu);
  abort_locked(c, "aborted by the caller (gs_comm_abort)");
  return GS_OK;
}

int gs_watchdog_pause(int pause) {
  const int v = pause ? g_wd_pause.fetch_add(1) + 1 : g_wd_pause.fetch_sub(1) - 1;
  if (v < 0) {
    g_wd_pause.store(0);
    return fail(GS_ESTATE, "gs_watchdog_pause: resume without a pause");
  }
  return GS_OK;
}

int gs_comm_set_timeout(gs_comm* c, int64_t timeout_ms) {
  GS_CHECK_ARG(c != nullptr && timeout_ms >= 0, "gs_comm_set_timeout: bad argument");
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->timeout_ms = timeout_ms;
  }
  if (timeout_ms > 0 && !c->wd.joinable()) c->wd = std::thread(watchdog_loop, c);
  return GS_OK;
}

int gs_comm_status(gs_comm* c, char* reason, int cap) {
  GS_CHECK_ARG(c != nullptr, "gs_comm_status: NULL comm");
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->aborted.load()) {
    ncclResult_t async = ncclSuccess;
    if (c->comm && ncclCommGetAsyncError(c->comm, &async) == ncclSuccess && async != ncclSuccess &&
        async != ncclInProgress)
      abort_locked(c, std::string("RCCL asynchronous error: ") + ncclGetErrorString(async));
  }
  if (reason && cap > 0) {
    const std::string r = abort_reason(c);
    const size_t n = std::min(r.size(), static_cast<size_t>(cap - 1));
    std::memcpy(reason, r.data(), n);
    reason[n] = 0;
  }
  return c->aborted.load() ? 1 : 0;
}

int gs_comm_rank(gs_comm* c) { return c ? c->rank : -1; }
int gs_comm_world(gs_comm* c) { return c ? c->world : -1; }

int gs_comm_stream(gs_comm* c, void** stream_out) {
  GS_CHECK_ARG(c && stream_out, "gs_comm_stream: NULL argument");
  *stream_out = c->stream;
  return GS_OK;
}

int gs_allreduce(gs_comm* c, const void* send, void* recv, int64_t count, int dtype, int op,
                 void* stream) {
  GS_CHECK_ARG(c != nullptr, "gs_allreduce: NULL communicator");
  ncclDataType_t dt;
  ncclRedOp_t o;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  GS_TRY_RET(to_nccl_op(op, &o));
  hipStream_t s = pick(c, stream);
  return comm_enqueue(c, s, [&] { return ncclAllReduce(send, recv, static_cast<size_t>(count), dt, o, c->comm, s); },
                      "ncclAllReduce");
}

int gs_allreduce_marked(gs_comm* c, const void* send, void* recv, int64_t count, int dtype, int op, void* stream,
                        gs_plan* consumer) {
  GS_CHECK_ARG(c != nullptr, "gs_allreduce_marked: NULL communicator");
  ncclDataType_t dt;
  ncclRedOp_t o;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  GS_TRY_RET(to_nccl_op(op, &o));
  hipStream_t s = pick(c, stream);
  return comm_enqueue(c, s, [&] { return ncclAllReduce(send, recv, static_cast<size_t>(count), dt, o, c->comm, s); },
                      "ncclAllReduce", true, consumer);
}

int gs_all_gather_marked(gs_comm* c, const void* send, void* recv, int64_t send_count, int dtype, void* stream,
                         gs_plan* consumer) {
  GS_CHECK_ARG(c != nullptr, "gs_all_gather_marked: NULL communicator");
  ncclDataType_t dt;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  hipStream_t s = pick(c, stream);
  return comm_enqueue(c, s, [&] { return ncclAllGather(send, recv, static_cast<size_t>(send_count), dt, c->comm, s); },
                      "ncclAllGather", true, consumer);
}

int gs_reduce_scatter(gs_comm* c, const void* send, void* recv, int64_t recv_count, int dtype,
                      int op, void* stream) {
  GS_CHECK_ARG(c != nullptr, "gs_reduce_scatter: NULL communicator");
  ncclDataType_t dt;
  ncclRedOp_t o;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  GS_TRY_RET(to_nccl_op(op, &o));
  hipStream_t s = pick(c, stream);
  return comm_enqueue(
      c, s, [&] { return ncclReduceScatter(send, recv, static_cast<size_t>(recv_count), dt, o, c->comm, s); },
      "ncclReduceScatter");
}

int gs_all_gather(gs_comm* c, const void* send, void* recv, int64_t send_count, int dtype,
                  void* stream) {
  GS_CHECK_ARG(c != nullptr, "gs_all_gather: NULL communicator");
  ncclDataType_t dt;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  hipStream_t s = pick(c, stream);
  return comm_enqueue(c, s, [&] { return ncclAllGather(send, recv, static_cast<size_t>(send_count), dt, c->comm, s); },
                      "ncclAllGather");
}

int gs_broadcast(gs_comm* c, const void* send, void* recv, int64_t count, int dtype, int root,
                 void* stream) {
  GS_CHECK_ARG(c != nullptr, "gs_broadcast: NULL communicator");
  GS_CHECK_ARG(root >= 0 && root < c->world, "gs_broadcast: bad root");
  ncclDataType_t dt;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  hipStream_t s = pick(c, stream);
  return comm_enqueue(
      c, s, [&] { return ncclBroadcast(send, recv, static_cast<size_t>(count), dt, root, c->comm, s); },
      "ncclBroadcast");
}

}  // extern "C"
