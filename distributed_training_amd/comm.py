"""RCCL communicator owned by libgsync (one per process / GPU).

The unique id is created on rank 0 and handed to the other ranks through the
caller's ``torch.distributed`` process group (the same rendezvous the
reference uses: ``init_process_group`` at R:resnet/pytorch_ddp/ddp_train.py:84),
after which all gradient traffic goes through this communicator on its own
high-priority stream.  The id travels through the rendezvous store, not a
process-group collective, so torch's ProcessGroupNCCL never has to bring up a
second RCCL communicator on the rank.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from . import _lib as L

_REDUCE_OPS = {"sum": L.GS_SUM, "prod": L.GS_PROD, "max": L.GS_MAX, "min": L.GS_MIN, "avg": L.GS_AVG}


DEFAULT_TIMEOUT_MS = 600_000  # torch's default process-group timeout (10 min)


class Communicator:
    def __init__(self, process_group=None, device: torch.device | None = None, timeout_ms: int | None = None,
                 max_ctas: int = 0):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if device.type != "cuda":
            raise ValueError("Communicator needs a HIP device; CPU tensors use the gloo process group")
        self.device = device
        self.pg = process_group
        self.rank = dist.get_rank(process_group)
        self.world = dist.get_world_size(process_group)
        lib = L.lib()
        nbytes = lib.gs_comm_unique_id_bytes()
        uid = (ctypes.c_uint8 * nbytes)()
        if self.rank == 0:
            L.check(lib.gs_comm_get_unique_id(uid), "gs_comm_get_unique_id")
        uid = (ctypes.c_uint8 * nbytes).from_buffer_copy(self._exchange_uid(bytes(uid)))
        h = ctypes.c_void_p()
        torch.cuda.set_device(device)
        self.max_ctas = int(max_ctas)
        L.check(lib.gs_comm_create_ex(self.rank, self.world, uid, device.index, self.max_ctas, ctypes.byref(h)),
                "gs_comm_create_ex")
        self.handle = h
        import weakref

        # bucketers built on this communicator: closed first when it closes (they
        # synchronise its stream at destruction — a freed communicator there was a
        # use-after-free once the comm went before a bucketer still awaiting GC)
        self._users = weakref.WeakSet()
        s = ctypes.c_void_p()
        L.check(lib.gs_comm_stream(h, ctypes.byref(s)), "gs_comm_stream")
        self.stream_ptr = s.value
        self.stream = torch.cuda.ExternalStream(self.stream_ptr, device=device)
        if timeout_ms is None:
            timeout_ms = int(os.environ.get("GSYNC_TIMEOUT_MS", DEFAULT_TIMEOUT_MS))
        self.set_timeout(timeout_ms)

    def set_timeout(self, timeout_ms: int):
        """Watchdog: abort the communicator when a collective is in flight longer
        than timeout_ms or RCCL reports an asynchronous error (0 disables)."""
        L.check(L.lib().gs_comm_set_timeout(self.handle, int(timeout_ms)), "gs_comm_set_timeout")
        self.timeout_ms = int(timeout_ms)

    def status(self):
        """(aborted, reason) — a host-side flag read, no device synchronisation."""
        buf = ctypes.create_string_buffer(512)
        rc = L.check(L.lib().gs_comm_status(self.handle, buf, 512), "gs_comm_status")
        return bool(rc), buf.value.decode(errors="replace")

    def check(self):
        aborted, why = self.status()
        if aborted:
            raise L.GsyncError(f"libgsync communicator (rank {self.rank}/{self.world}) aborted: {why}")

    def _exchange_uid(self, uid: bytes) -> bytes:
        """Rank 0's RCCL unique id to every rank through the rendezvous store
        (the TCP store torch.distributed.init_process_group already holds) —
        not a collective on the process group: with the nccl backend that would
        bring up torch's own RCCL communicator beside this one (two sets of
        channels and proxy threads per rank).  Keys are namespaced by group
        and by creation count, which every rank advances in the same order."""
        store = None
        try:
            store = dist.distributed_c10d._get_default_store()
        except Exception:  # pragma: no cover - a torch without the private accessor
            store = None
        if store is None:
            obj = [uid]
            src = dist.get_global_rank(self.pg, 0) if self.pg is not None else 0
            backend = dist.get_backend(self.pg)
            dev = self.device if backend in ("nccl", "rccl") else torch.device("cpu")
            dist.broadcast_object_list(obj, src=src, group=self.pg, device=dev)
            return obj[0]
        name = getattr(self.pg if self.pg is not None else dist.group.WORLD, "group_name", "world")
        gen = _UID_GEN[name] = _UID_GEN.get(name, -1) + 1
        key = f"gsync/uid/{name}/{gen}"
        if self.rank == 0:
            store.set(key, uid)
            return uid
        return bytes(store.get(key))

    def add_user(self, obj):
        """`obj` (with a close()) holds library objects bound to this communicator."""
        self._users.add(obj)

    def close(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            for u in list(getattr(self, "_users", ())):
                u.close()
            L.destroy("gs_comm_destroy", h)
            self.handle = None

    def abort(self):
        if self.handle is not None:
            L.check(L.lib().gs_comm_abort(self.handle), "gs_comm_abort")

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    # ------------------------------------------------------------ collectives
    def _s(self, stream):
        return self.stream_ptr if stream is None else stream

    def all_reduce(self, t: torch.Tensor, op="sum", stream=None, out: torch.Tensor | None = None, consumer=None):
        """consumer: a plan handle (c_void_p) whose next launch, stream-ordered after
        this collective, carries its watchdog mark instead of an event packet
        (gs_allreduce_marked)."""
        out = t if out is None else out
        if consumer is not None:
            L.check(L.lib().gs_allreduce_marked(self.handle, t.data_ptr(), out.data_ptr(), t.numel(),
                                                L.gs_dtype(t.dtype), _REDUCE_OPS[op], self._s(stream), consumer),
                    "gs_allreduce_marked")
            return out
        L.check(L.lib().gs_allreduce(self.handle, t.data_ptr(), out.data_ptr(), t.numel(), L.gs_dtype(t.dtype),
                                     _REDUCE_OPS[op], self._s(stream)), "gs_allreduce")
        return out

    def reduce_scatter(self, send: torch.Tensor, recv: torch.Tensor, op="sum", stream=None):
        L.check(L.lib().gs_reduce_scatter(self.handle, send.data_ptr(), recv.data_ptr(), recv.numel(),
                                          L.gs_dtype(send.dtype), _REDUCE_OPS[op], self._s(stream)),
                "gs_reduce_scatter")
        return recv

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor, stream=None, consumer=None):
        if consumer is not None:  # the mark rides on `consumer`'s next launch (gs_all_gather_marked)
            L.check(L.lib().gs_all_gather_marked(self.handle, send.data_ptr(), recv.data_ptr(), send.numel(),
                                                 L.gs_dtype(send.dtype), self._s(stream), consumer),
                    "gs_all_gather_marked")
            return recv
        L.check(L.lib().gs_all_gather(self.handle, send.data_ptr(), recv.data_ptr(), send.numel(),
                                      L.gs_dtype(send.dtype), self._s(stream)), "gs_all_gather")
        return recv

    def broadcast(self, t: torch.Tensor, root=0, stream=None):
        L.check(L.lib().gs_broadcast(self.handle, t.data_ptr(), t.data_ptr(), t.numel(), L.gs_dtype(t.dtype),
                                     root, self._s(stream)), "gs_broadcast")
        return t

    def wait_on_current(self):
        """comm stream waits for everything queued on torch's current stream."""
        L.check(L.lib().gs_stream_wait(self.stream_ptr, L.stream_ptr(self.device)), "gs_stream_wait")

    def current_waits(self):
        """torch's current stream waits for everything queued on the comm stream."""
        L.check(L.lib().gs_stream_wait(L.stream_ptr(self.device), self.stream_ptr), "gs_stream_wait")


_COMMS: dict = {}
_UID_GEN: dict = {}  # group name -> communicators created for it so far (store key namespace)


def get_communicator(process_group=None, device=None) -> Communicator:
    """Process-wide cache: one communicator per (group, device)."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (id(process_group) if process_group is not None else None, device.index)
    c = _COMMS.get(key)
    if c is None:
        c = Communicator(process_group, device)
        _COMMS[key] = c
    return c


def destroy_communicators():
    for c in list(_COMMS.values()):
        c.close()
    _COMMS.clear()
