// libgsync communicator: one RCCL communicator per process (one process per
// GPU) with a library-owned non-blocking, high-priority stream, so that
// gradient collectives run beside the backward kernels instead of behind
// them.  The unique id is exchanged by the caller (torch.distributed store).
//
// replaces: torch ProcessGroupNCCL (T:include/torch/csrc/distributed/c10d/
// ProcessGroupNCCL.hpp:849 allreduce, :836 broadcast, :872 _allgather_base,
// :887-892 reduce_scatter; dedicated ncclStreams_ :1398).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "gs_common.h"

struct gs_comm {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int rank = 0, world = 1, device = 0;
  bool aborted = false;
};

namespace gs {
namespace {

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

hipStream_t pick(gs_comm* c, void* stream) {
  return stream ? static_cast<hipStream_t>(stream) : c->stream;
}

}  // namespace

// used by the bucketer
ncclComm_t comm_handle(gs_comm* c) { return c->comm; }
hipStream_t comm_stream(gs_comm* c) { return c->stream; }
int comm_dtype(int dt, ncclDataType_t* out) { return to_nccl_dtype(dt, out); }

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
  ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
  if (r != ncclSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return rccl_fail(r, "ncclCommInitRank");
  }
  *out = c;
  return GS_OK;
}

int gs_comm_destroy(gs_comm* c) {
  if (!c) return GS_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm && !c->aborted) (void)ncclCommDestroy(c->comm);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GS_OK;
}

int gs_comm_abort(gs_comm* c) {
  GS_CHECK_ARG(c != nullptr, "gs_comm_abort: NULL comm");
  if (!c->aborted && c->comm) RCCL_RET(ncclCommAbort(c->comm));
  c->aborted = true;
  return GS_OK;
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
  GS_CHECK_ARG(c && !c->aborted, "gs_allreduce: no live communicator");
  ncclDataType_t dt;
  ncclRedOp_t o;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  GS_TRY_RET(to_nccl_op(op, &o));
  RCCL_RET(ncclAllReduce(send, recv, static_cast<size_t>(count), dt, o, c->comm, pick(c, stream)));
  return GS_OK;
}

int gs_reduce_scatter(gs_comm* c, const void* send, void* recv, int64_t recv_count, int dtype,
                      int op, void* stream) {
  GS_CHECK_ARG(c && !c->aborted, "gs_reduce_scatter: no live communicator");
  ncclDataType_t dt;
  ncclRedOp_t o;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  GS_TRY_RET(to_nccl_op(op, &o));
  RCCL_RET(ncclReduceScatter(send, recv, static_cast<size_t>(recv_count), dt, o, c->comm,
                             pick(c, stream)));
  return GS_OK;
}

int gs_all_gather(gs_comm* c, const void* send, void* recv, int64_t send_count, int dtype,
                  void* stream) {
  GS_CHECK_ARG(c && !c->aborted, "gs_all_gather: no live communicator");
  ncclDataType_t dt;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  RCCL_RET(ncclAllGather(send, recv, static_cast<size_t>(send_count), dt, c->comm, pick(c, stream)));
  return GS_OK;
}

int gs_broadcast(gs_comm* c, const void* send, void* recv, int64_t count, int dtype, int root,
                 void* stream) {
  GS_CHECK_ARG(c && !c->aborted, "gs_broadcast: no live communicator");
  GS_CHECK_ARG(root >= 0 && root < c->world, "gs_broadcast: bad root");
  ncclDataType_t dt;
  GS_TRY_RET(to_nccl_dtype(dtype, &dt));
  RCCL_RET(ncclBroadcast(send, recv, static_cast<size_t>(count), dt, root, c->comm, pick(c, stream)));
  return GS_OK;
}

}  // extern "C"
