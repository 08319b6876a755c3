"""Drop-in ``DistributedDataParallel`` on the libgsync gradient-sync engine.

Same constructor, attribute and call surface as torch's
``torch.nn.parallel.DistributedDataParallel`` (T:nn/parallel/distributed.py:653-953)
as the reference scripts use it (``DDP(model)`` at
R:resnet/pytorch_ddp/ddp_train.py:95; colossal ``TorchDDPPlugin`` at
R:resnet/colossal/colossal_train.py:131-132,159): ``.module``, ``forward``,
``no_sync()``, ``register_comm_hook``, ``state_dict`` with the ``module.``
prefix, ``_get_ddp_logging_data()``.

What changes is underneath:

* the c10d Reducer is replaced by the libgsync bucketer (C++), driven by one
  ``register_post_accumulate_grad_hook`` per parameter;
* a bucket is packed (fused 1/world_size scale + cast) by one gfx950
  multi-tensor kernel when its last gradient arrives, all-reduced by RCCL on
  libgsync's own stream and unpacked there, overlapped with the rest of
  backward (torch: one ATen launch per parameter for pack and for unpack);
* BN buffers are broadcast from rank 0 before every forward through the same
  pack kernel + one RCCL broadcast (T:nn/parallel/distributed.py:2178-2221).

Bucketing semantics follow torch: first iteration one bucket (sys.maxsize,
:1199-1200), then buckets rebuilt once in gradient-ready order with a
1 MiB first bucket and ``bucket_cap_mb`` (25 MiB) caps, rank 0's layout
broadcast to all ranks (Reducer::rebuild_buckets / sync_bucket_indices).

On CPU tensors (the CPU/gloo configuration) the same bucketer runs its host
backend and the collective is torch's gloo all-reduce.
"""
from __future__ import annotations

import ctypes
import os
import sys
from contextlib import contextmanager
from dataclasses import dataclass
from enum import Enum, auto
from typing import Any, Callable

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.distributed.algorithms.join import Join, Joinable, JoinHook

from . import _lib as L
from .comm import get_communicator
from .multi_tensor import TensorListPlan, dense_like_param, is_dense

DEFAULT_FIRST_BUCKET_BYTES = getattr(dist, "_DEFAULT_FIRST_BUCKET_BYTES", 1024 * 1024)
BUCKET_ALIGN_ELEMS = 64  # 256 B (fp32) per-parameter alignment inside a bucket


def compute_bucket_assignment_by_size(tensors, size_limits, order=None):
    """Restatement of dist._compute_bucket_assignment_by_size (libgsync C++).

    Returns a list of buckets, each a list of tensor indices.  ``order``
    (gradient-ready order) disables the final sort, as Reducer::rebuild_buckets.
    """
    n = len(tensors)
    nbytes = L.i64_array([t.numel() * t.element_size() for t in tensors])
    keys = []
    key_ids: dict = {}
    for t in tensors:
        k = (t.dtype, t.device)
        keys.append(key_ids.setdefault(k, len(key_ids)))
    limits = [int(min(x, 2**62)) for x in size_limits]
    bucket_of = (ctypes.c_int32 * max(1, n))()
    members = (ctypes.c_int32 * max(1, n))()
    counts = (ctypes.c_int32 * max(1, n))()
    nb = L.check(
        L.lib().gs_compute_bucket_assignment(
            n, nbytes, L.i32_array(keys), None if order is None else L.i32_array(order), len(limits),
            L.i64_array(limits), bucket_of, members, counts),
        "gs_compute_bucket_assignment",
    )
    out, pos = [], 0
    for b in range(nb):
        out.append([int(members[pos + k]) for k in range(counts[b])])
        pos += counts[b]
    return out


def split_last_bucket(buckets, nbytes, cap):
    """Cap the LAST bucket in gradient-ready order (the conv1 / layer1 end of
    backward, whose pack -> collective -> unpack chain is exposed) at `cap`
    bytes: its last-ready members up to `cap` form a new final bucket, the
    rest stay a bucket of their own (torch's first_bucket_bytes_cap idea,
    T:include/torch/csrc/distributed/c10d/reducer.hpp:30-31, applied to the
    other end).  Bucket membership changes no element's sum."""
    if not buckets:
        return buckets
    last = list(buckets[-1])
    tail, size = [], 0
    while last and (not tail or size + nbytes[last[-1]] <= cap):
        i = last.pop()
        tail.insert(0, i)
        size += nbytes[i]
    out = [list(b) for b in buckets[:-1]]
    if last:
        out.append(last)
    out.append(tail)
    return out


def xgmi_bucket_caps(allreduce_time, world: int, sizes_mib=(1, 4, 16, 64), efficiency: float = 0.85) -> dict:
    """Bucket caps for point-to-point xGMI from the live all-reduce curve.

    Fits t(S) = alpha + S*f/B (f = 2(n-1)/n, B = bus bandwidth) to the measured
    times of `sizes_mib` and picks
      * bucket cap C: the smallest bucket whose all-reduce runs at `efficiency`
        of B, i.e. S*f/B >= efficiency * t(S)  <=>  C = efficiency/(1-efficiency) * alpha*B/f,
        clamped to [4, 256] MiB — fewer, larger collectives while each bucket
        still overlaps the backward that follows it;
      * last-bucket cap L: the bucket whose transfer costs one alpha
        (L = alpha*B/f, clamped to [256 KiB, C]) — bounds the exposed tail to
        ~2*alpha + the pack/unpack of L.
    allreduce_time(nbytes) -> seconds (identical on every rank)."""
    f = 2.0 * (world - 1) / world
    pts = [(m * 1024 * 1024, allreduce_time(m * 1024 * 1024)) for m in sizes_mib]
    # least-squares line t = alpha + S * beta
    n = len(pts)
    sx = sum(p[0] for p in pts)
    sy = sum(p[1] for p in pts)
    sxx = sum(p[0] * p[0] for p in pts)
    sxy = sum(p[0] * p[1] for p in pts)
    beta = (n * sxy - sx * sy) / max(1e-30, n * sxx - sx * sx)
    alpha = max(0.0, (sy - beta * sx) / n)
    if beta <= 0:  # degenerate curve: keep torch's caps
        beta = pts[-1][1] / pts[-1][0]
    bus = f / beta  # bytes/s
    cap = efficiency / (1 - efficiency) * alpha * bus / f
    cap = int(min(256 * 2**20, max(4 * 2**20, cap)))
    last = int(min(cap, max(256 * 1024, alpha * bus / f)))
    return {"points": [{"bytes": b, "ms": t * 1e3, "bus_GBps": b * f / t / 1e9} for b, t in pts],
            "alpha_us": alpha * 1e6, "bus_GBps": bus / 1e9, "bucket_cap_bytes": cap, "last_bucket_cap_bytes": last,
            "efficiency": efficiency}


def _as_words(t: torch.Tensor):
    """A view of buffer `t` the multi-tensor kernels can move bit for bit:
    fp32 / bf16 / fp16 as they are; 4- and 8-byte integer or fp64 tensors as
    fp32 words (pure loads and stores, no arithmetic); None otherwise."""
    if not t.is_contiguous():
        return None
    if t.dtype in (torch.float32, torch.bfloat16, torch.float16):
        return t
    if t.element_size() in (4, 8) and t.dtype != torch.complex64:
        return t.reshape(-1).view(torch.float32)
    return None


class GradBucket:
    """Mirror of torch.distributed.GradBucket (T:include/torch/csrc/distributed/c10d/comm.hpp:20-98)."""

    def __init__(self, index, buffer, params, offsets, is_last):
        self._index = index
        self._buffer = buffer
        self._params = params
        self._offsets = offsets
        self._is_last = is_last

    def index(self):
        return self._index

    def buffer(self):
        return self._buffer

    def set_buffer(self, t):
        self._buffer.copy_(t)

    def parameters(self):
        return list(self._params)

    def gradients(self):
        buf = self._buffer
        return [
            buf.as_strided(p.size(), p.stride(), buf.storage_offset() + off)
            for p, off in zip(self._params, self._offsets)
        ]

    def is_last(self):
        return self._is_last


class _Bucketer:
    """Python owner of one gs_bucketer + its torch-allocated bucket storage."""

    def __init__(self, ddp, buckets, flags):
        import weakref

        self._ddp_ref = weakref.ref(ddp)  # no DDP <-> bucketer cycle: freed when the DDP goes
        params = ddp._params
        self.buckets = buckets
        self.flags = flags
        kind = L.GS_DEV_HIP if ddp.device.type == "cuda" else L.GS_DEV_HOST
        counts = [len(b) for b in buckets]
        members = [i for b in buckets for i in b]
        h = ctypes.c_void_p()
        comm = ddp._comm.handle if (ddp._comm is not None) else None
        # torch buckets per dtype (compute_bucket_assignment_by_size keys on it):
        # every bucket holds params of one dtype; its buffer has that dtype
        # unless bucket_dtype overrides it
        self.grad_dtypes = [params[b[0]].dtype for b in buckets]
        self.bucket_dtypes = [ddp._bucket_dtype_override or gdt for gdt in self.grad_dtypes]
        L.check(
            L.lib().gs_bucketer_create(
                comm, kind, ddp._dev_index, len(params), L.i64_array([p.numel() for p in params]),
                L.gs_dtype(params[0].dtype), len(buckets), L.i32_array(counts), L.i32_array(members),
                L.gs_dtype(ddp._bucket_dtype_override or params[0].dtype), BUCKET_ALIGN_ELEMS,
                float(ddp.world_size), flags, ctypes.byref(h)),
            "gs_bucketer_create",
        )
        self.handle = h
        if ddp._comm is not None:
            ddp._comm.add_user(self)
        self.buffers = []
        for b in range(len(buckets)):
            if any(params[i].dtype != self.grad_dtypes[b] for i in buckets[b]):
                raise RuntimeError(f"bucket {b} mixes parameter dtypes")
            L.check(L.lib().gs_bucketer_set_bucket_dtype(h, b, L.gs_dtype(self.grad_dtypes[b]),
                                                         L.gs_dtype(self.bucket_dtypes[b])),
                    "gs_bucketer_set_bucket_dtype")
            n = ctypes.c_int64()
            L.check(L.lib().gs_bucketer_bucket_numel(h, b, ctypes.byref(n)), "gs_bucketer_bucket_numel")
            buf = torch.zeros(n.value, dtype=self.bucket_dtypes[b], device=ddp.device)
            L.check(L.lib().gs_bucketer_set_bucket_buffer(h, b, buf.data_ptr()), "gs_bucketer_set_bucket_buffer")
            self.buffers.append(buf)
        self.loc = []
        for i in range(len(params)):
            bi, off = ctypes.c_int32(), ctypes.c_int64()
            L.check(L.lib().gs_bucketer_param_location(h, i, ctypes.byref(bi), ctypes.byref(off)),
                    "gs_bucketer_param_location")
            self.loc.append((bi.value, off.value))
        self.offsets_in_bucket = [[self.loc[i][1] for i in b] for b in buckets]
        self._ready = (ctypes.c_int32 * max(1, len(buckets)))()
        self._n_ready = ctypes.c_int32()
        # the per-gradient hook's call, bound once (it runs ~160 times a backward)
        self._mark = L.lib().gs_bucketer_mark_ready
        self._n_ready_ref = ctypes.byref(self._n_ready)

    @property
    def ddp(self):
        return self._ddp_ref()

    def bucket_view(self, i):
        b, off = self.loc[i]
        p = self.ddp._params[i]
        buf = self.buffers[b]
        return buf.as_strided(p.size(), p.stride(), off)

    def logical_bytes(self):
        params = self.ddp._params
        return [sum(params[i].numel() for i in b) * torch.tensor([], dtype=dt).element_size()
                for b, dt in zip(self.buckets, self.bucket_dtypes)]

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            nat = getattr(self.ddp, "_native", None)
            if nat is not None:
                nat.set_bucketer(0, 0)  # the C++ hooks must not reach a destroyed bucketer
            L.destroy("gs_bucketer_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass


class _BufferCommHookLocation(Enum):
    """Where a buffer comm hook runs (T:nn/parallel/distributed.py:226-228)."""
    PRE_FORWARD = auto()
    POST_FORWARD = auto()


@dataclass
class _BufferCommHook:
    buffer_comm_hook: Callable
    buffer_comm_hook_state: Any
    buffer_comm_hook_location: _BufferCommHookLocation


def _make_native_hooks(owner, params=None, release: bool = False):
    """The C++ hook object for a DDP (or, `release`, a ZeRO engine) — None when
    GSYNC_NATIVE_HOOK=0 or the extension is not built.  Its end-of-backward
    callback holds the owner weakly (the hooks live as long as the owner, not
    the other way round) and calls owner._native_finalized()."""
    if os.environ.get("GSYNC_NATIVE_HOOK", "1") == "0":
        return None
    mod = L.hook_module()
    if mod is None:
        return None
    import weakref

    ref = weakref.ref(owner)

    def on_finalize():
        d = ref()
        if d is not None:
            d._native_finalized()

    return mod.Hooks(owner._params if params is None else params, owner._dev_index, on_finalize, release)


class DistributedDataParallel(nn.Module, Joinable):
    def __init__(self, module, device_ids=None, output_device=None, dim=0, broadcast_buffers=True,
                 init_sync=True, process_group=None, bucket_cap_mb=None, find_unused_parameters=False,
                 check_reduction=False, gradient_as_bucket_view=False, static_graph=False,
                 delay_all_reduce_named_params=None, param_to_hook_all_reduce=None, mixed_precision=None,
                 device_mesh=None, skip_all_reduce_unused_params=False, *, bucket_dtype=None,
                 collective: str = "auto", bucket_policy: str = "torch", last_bucket_cap_mb=None,
                 rccl_max_ctas: int | None = None):
        super().__init__()
        Joinable.__init__(self)  # the join config (disabled until a Join context enables it)
        self._divide_by_initial_world_size = True
        if delay_all_reduce_named_params is not None or param_to_hook_all_reduce is not None:
            raise NotImplementedError("delay_all_reduce_named_params is outside the gradient-sync path")
        if mixed_precision is not None or device_mesh is not None:
            raise NotImplementedError("DDP mixed_precision / device_mesh are outside the gradient-sync path")
        if not dist.is_initialized():
            raise RuntimeError("Default process group has not been initialized, please make sure to call "
                               "init_process_group.")
        self.module = module
        self.process_group = process_group if process_group is not None else dist.group.WORLD
        self.world_size = dist.get_world_size(self.process_group)
        self.rank = dist.get_rank(self.process_group)
        self.dim = dim
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.gradient_as_bucket_view = gradient_as_bucket_view
        self.static_graph = static_graph
        self.require_backward_grad_sync = True
        self.require_forward_param_sync = True
        self.bucket_bytes_cap_default = bucket_cap_mb is None
        self.bucket_bytes_cap = int((25 if bucket_cap_mb is None else bucket_cap_mb) * 1024 * 1024)
        self.first_bucket_bytes_cap = DEFAULT_FIRST_BUCKET_BYTES if self.bucket_bytes_cap_default else self.bucket_bytes_cap

        # parameters handed to the bucketer: module order, requires_grad, no duplicates,
        # minus the names _set_params_and_buffers_to_ignore_for_model listed (torch's
        # ``parameters_to_ignore``: neither synchronised nor broadcast)
        self.parameters_to_ignore = set(getattr(module, "_ddp_params_and_buffers_to_ignore", ()))
        self.buffer_hook = None  # _register_buffer_comm_hook
        self._post_bwd_futs = []
        seen = set()
        self._params, self._param_names = [], []
        for name, p in module.named_parameters():
            if name in self.parameters_to_ignore:
                continue
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                self._params.append(p)
                self._param_names.append(name)
        if not self._params:
            raise RuntimeError("DistributedDataParallel is not needed when a module doesn't have any "
                               "parameter that requires a gradient.")
        devices = {p.device for p in self._params}
        if len(devices) != 1:
            raise ValueError(f"DDP module parameters must live on one device, found {devices}")
        self.device = next(iter(devices))
        self.device_type = self.device.type
        self.device_ids = device_ids if device_ids is None else [torch.device(d).index if not isinstance(d, int) else d for d in device_ids]
        self.output_device = output_device
        dtypes = {p.dtype for p in self._params}
        if not all(dt.is_floating_point for dt in dtypes):
            raise NotImplementedError(f"gradient sync needs floating parameters, got {dtypes}")
        # several dtypes -> buckets per dtype (torch's Reducer does the same)
        self._bucket_dtype_override = bucket_dtype
        self._grad_dtype = self._params[0].dtype if len(dtypes) == 1 else None
        self._bucket_dtype = bucket_dtype if bucket_dtype is not None else self._grad_dtype
        if self.device.type == "cuda":
            self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
            if not L.available():
                raise L.GsyncUnavailable(L._load_error)
        else:
            self._dev_index = 0
        self._backend = dist.get_backend(self.process_group)

        # library-owned RCCL communicator for CUDA tensors over an nccl (=RCCL) group
        self._comm = None
        self._own_comm = False
        if self.device.type == "cuda" and collective != "process_group" and self._backend == "nccl":
            pg = None if self.process_group is dist.group.WORLD else self.process_group
            if rccl_max_ctas:
                # RCCL's per-collective workgroup cap (ncclConfig_t maxCTAs): a communicator
                # of this DDP's own, closed with it (the shared one keeps RCCL's default)
                from .comm import Communicator

                self._comm = Communicator(pg, torch.device("cuda", self._dev_index), max_ctas=int(rccl_max_ctas))
                self._own_comm = True
            else:
                self._comm = get_communicator(pg, torch.device("cuda", self._dev_index))
        self._comm_hook: tuple[Any, Callable] | None = None
        self._buffers_plan = None
        self._sqnorm_target: torch.Tensor | None = None
        self._sqnorm_valid = False  # the last synchronising backward's unpacks filled _sqnorm_target
        self._sqnorm_versions = None  # _grad_versions() when they did
        self._found_inf_target: torch.Tensor | None = None
        self._found_inf_valid = False

        # GSYNC_DEBUG=1: checksum every bucket before and after its collective
        self._debug_sums = None
        if os.environ.get("GSYNC_DEBUG", "0") not in ("", "0"):
            self._debug_sums = torch.zeros(0)

        if init_sync:
            self._verify_param_shape_across_processes()
            self._sync_module_states()

        # bucket policy: "torch" = torch's caps (1 MiB first bucket, bucket_cap_mb);
        # "xgmi" = caps from the live all-reduce curve of this group (xgmi_bucket_caps)
        if bucket_policy not in ("torch", "xgmi"):
            raise ValueError(f"bucket_policy must be 'torch' or 'xgmi', got {bucket_policy!r}")
        self.bucket_policy = bucket_policy
        self._last_bucket_cap = None if last_bucket_cap_mb is None else int(last_bucket_cap_mb * 1024 * 1024)
        self._xgmi_calibration = None
        if bucket_policy == "xgmi" and self.world_size > 1:
            cal = xgmi_bucket_caps(self._calib_allreduce, self.world_size)
            self._xgmi_calibration = cal
            if bucket_cap_mb is None:
                self.bucket_bytes_cap = cal["bucket_cap_bytes"]
            if last_bucket_cap_mb is None:
                self._last_bucket_cap = cal["last_bucket_cap_bytes"]

        if static_graph or not find_unused_parameters:
            limits = [sys.maxsize]
        elif self.bucket_bytes_cap_default:
            limits = [DEFAULT_FIRST_BUCKET_BYTES, self.bucket_bytes_cap]
        else:
            limits = [self.bucket_bytes_cap]
        buckets = compute_bucket_assignment_by_size(self._params, limits)
        # "reverse list of buckets because we want to approximate the order in
        # which their gradients are produced" (T:nn/parallel/distributed.py:1222)
        self._bucketer = self._make_bucketer(list(reversed(buckets)))
        self._has_rebuilt_buckets = False
        self._ready_order: list[int] = []
        self._in_backward = False
        self._finalize_queued = False
        self._stream = None
        self._pending: dict[int, Any] = {}
        self._num_iterations = 0
        self._capture_local: dict | None = None  # parity.py: {param index: local grad copy}
        # find_unused_parameters: torch's local-used map — a parameter counts as used if its
        # grad was produced in any backward since the last synchronising one (no_sync included)
        self._used_local = [0] * len(self._params) if find_unused_parameters else None
        self._ready_now: list = []
        self._overlap: dict | None = None  # _register_fused_optim state
        self._param_index = {id(p): i for i, p in enumerate(self._params)}
        self._hook_handles = []
        # C++ gradient hooks (_gshook: AccumulateGrad post-hooks calling
        # gs_bucketer_mark_ready, as torch's Reducer) on the fast path; the Python
        # hooks below serve every other configuration.  _set_native switches.
        self._native = _make_native_hooks(self) if self.device.type == "cuda" else None
        self._native_on = False
        if self._native is not None:
            self._native.set_bucketer(self._bucketer.handle.value, len(self._bucketer.buckets))
            # static_graph: the C++ finalize marks never-used parameters ready first,
            # as _finalize_backward's static_graph branch does on the Python hooks
            self._native.set_mark_unused(bool(self.static_graph))
        self._set_native(self._native_ok())

    # ------------------------------------------------------------------ setup
    def _flags(self):
        flags = 0
        if self._comm is not None and self._comm_hook is None:
            flags |= L.GS_BKT_AUTO_COLLECTIVE
        if self.gradient_as_bucket_view:
            flags |= L.GS_BKT_GRAD_VIEW
        if self._comm_hook is not None:
            flags |= L.GS_BKT_NO_SCALE
        return flags

    def _make_bucketer(self, buckets):
        old = getattr(self, "_bucketer", None)
        if old is not None:
            old.close()
        b = _Bucketer(self, buckets, self._flags())
        self._div_factor = float(self.world_size)  # a new bucketer divides by the world size
        t = getattr(self, "_found_inf_target", None)
        if t is not None:
            L.check(L.lib().gs_bucketer_set_found_inf(b.handle, t.data_ptr()), "gs_bucketer_set_found_inf")
        if getattr(self, "_debug_sums", None) is not None:
            self._debug_sums = torch.zeros(3 * len(buckets), dtype=torch.float32, device=self.device)
            L.check(L.lib().gs_bucketer_set_debug(b.handle, self._debug_sums.data_ptr()), "gs_bucketer_set_debug")
        lvl = getattr(self, "_timeline", None)
        if lvl is not None:
            L.check(L.lib().gs_bucketer_set_timeline(b.handle, lvl), "gs_bucketer_set_timeline")
        if getattr(self, "_overlap", None) is not None:
            self._overlap["per_bucket"] = {}  # bucket membership changed
        if getattr(self, "_native", None) is not None:
            self._native.set_bucketer(b.handle.value, len(buckets))
        return b

    # ---- which hooks run: C++ (_gshook) on the fast path, Python otherwise
    def _native_ok(self) -> bool:
        return (self._native is not None and bool(self._bucketer.flags & L.GS_BKT_AUTO_COLLECTIVE)
                and not self.find_unused_parameters and self._overlap is None and self._comm_hook is None
                and self._capture_local is None)

    def _set_native(self, on: bool):
        if on:
            for h in self._hook_handles:
                h.remove()
            self._hook_handles = []
            self._native.attach()
        else:
            if self._native is not None:
                self._native.detach()
            if not self._hook_handles:
                self._hook_handles = [p.register_post_accumulate_grad_hook(self._make_hook(i))
                                      for i, p in enumerate(self._params)]
        self._native_on = on

    def _native_finalized(self):
        """End of a backward whose hooks and gs_bucketer_finalize ran in C++:
        the Python side of _finalize_backward (once per backward)."""
        if self._record_order:
            self._ready_order = list(self._native.order())
        if self._post_bwd_futs:
            self._wait_post_backward_futures()
        self._found_inf_valid = self._found_inf_target is not None
        self._sqnorm_valid = self._sqnorm_fusable()
        self._sqnorm_versions = self._grad_versions() if self._sqnorm_valid else None
        if self.gradient_as_bucket_view:
            b = self._bucketer
            for i, p in enumerate(self._params):
                if p.grad is not None:
                    view = b.bucket_view(i)
                    if p.grad.data_ptr() != view.data_ptr():
                        p.grad = view
        self._in_backward = False
        self._finalize_queued = False
        self._num_iterations += 1

    def _calib_allreduce(self, nbytes: int, iters: int = 4) -> float:
        """Median time (s, MAX over ranks) of one SUM all-reduce of nbytes of
        fp32 through this DDP's collective (libgsync RCCL on its stream, or the
        process group)."""
        import time

        n = max(1, nbytes // 4)
        on_dev = self._comm is not None or self._backend == "nccl"
        buf = torch.zeros(n, dtype=torch.float32, device=self.device if on_dev else "cpu")
        ts = []
        for it in range(iters + 1):
            if on_dev:
                torch.cuda.synchronize(self.device)
            self._ctl_barrier()
            t0 = time.perf_counter()
            if self._comm is not None:
                self._comm.all_reduce(buf, stream=L.stream_ptr(self.device))
                torch.cuda.synchronize(self.device)
            else:
                dist.all_reduce(buf, group=self.process_group)
                if on_dev:
                    torch.cuda.synchronize(self.device)
            if it:
                ts.append(time.perf_counter() - t0)
        ts.sort()
        return float(self._ctl_all_reduce(torch.tensor([ts[len(ts) // 2]], dtype=torch.float64), "max").item())

    # ---- control-plane collectives (shape check, layout broadcast, checksums,
    # calibration): on the libgsync communicator when there is one, so a rank
    # runs ONE RCCL communicator — torch's ProcessGroupNCCL then issues nothing
    # between wrap and training (T:nn/parallel/distributed.py:860-870 uses the
    # process group for the same checks); the process group otherwise (gloo).
    _CTL_OPS = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}

    def _ctl_device(self):
        return self.device if (self._comm is not None or self._backend == "nccl") else torch.device("cpu")

    def _ctl_all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        t = t.to(self._ctl_device())
        if self._comm is not None:
            self._comm.all_reduce(t, op=op, stream=L.stream_ptr(self.device))
        else:
            dist.all_reduce(t, op=self._CTL_OPS[op], group=self.process_group)
        return t

    def _ctl_broadcast(self, t: torch.Tensor) -> torch.Tensor:
        t = t.to(self._ctl_device())
        if self._comm is not None:
            self._comm.broadcast(t, root=0, stream=L.stream_ptr(self.device))
        else:
            dist.broadcast(t, src=dist.get_global_rank(self.process_group, 0)
                           if self.process_group is not dist.group.WORLD else 0, group=self.process_group)
        return t

    def _ctl_barrier(self):
        if self._comm is not None:
            self._ctl_all_reduce(torch.zeros(1, dtype=torch.int32))
            torch.cuda.synchronize(self.device)
        else:
            dist.barrier(group=self.process_group)

    def _verify_param_shape_across_processes(self):
        if self.world_size == 1:
            return
        meta = torch.tensor([len(self._params), sum(p.numel() for p in self._params),
                             hash(tuple(tuple(p.shape) for p in self._params)) % (2**61)], dtype=torch.int64)
        lo = self._ctl_all_reduce(meta.clone(), "min")
        hi = self._ctl_all_reduce(meta.clone(), "max")
        if not torch.equal(lo, hi):
            raise RuntimeError("DDP expects same model across all ranks, but the parameter shapes differ "
                               f"(rank {self.rank}: {meta.tolist()})")

    def _module_buffers(self):
        # collected once at wrap time, as torch's DDP does (``self.modules_buffers``):
        # walking the module tree every forward costs ~0.3 ms of host time a step
        bufs = getattr(self, "_modules_buffers", None)
        if bufs is None:
            named = [(n, b) for n, b in self.module.named_buffers() if n not in self.parameters_to_ignore]
            self._named_module_buffers = dict(named)
            bufs = self._modules_buffers = [b for _, b in named]
        return bufs

    @property
    def named_module_buffers(self):
        """{name: buffer} of the synchronised buffers (torch's attribute of the same
        name, T:nn/parallel/distributed.py:1125-1133) — what a buffer comm hook gets."""
        self._module_buffers()
        return self._named_module_buffers

    def _register_buffer_comm_hook(self, state, hook, comm_hook_location=None):
        """torch's buffer comm hook (T:nn/parallel/distributed.py:1909-1951):
        ``hook(state, named_module_buffers)`` replaces the rank-0 buffer broadcast,
        before the forward (``_BufferCommHookLocation.PRE_FORWARD``) or after it
        (``POST_FORWARD``, the default).  Futures it returns are awaited at the end
        of the next backward, as the Reducer's ``_install_post_backward_futures``."""
        if not callable(hook):
            raise TypeError("buffer comm hook must be callable")
        if comm_hook_location is None:
            comm_hook_location = _BufferCommHookLocation.POST_FORWARD
        # torch's own enum (torch.nn.parallel.distributed._BufferCommHookLocation) is accepted too
        comm_hook_location = _BufferCommHookLocation[getattr(comm_hook_location, "name", comm_hook_location)]
        self.buffer_hook = _BufferCommHook(hook, state, comm_hook_location)

    def _run_buffer_hook(self):
        bh = self.buffer_hook
        futs = bh.buffer_comm_hook(bh.buffer_comm_hook_state, self.named_module_buffers)
        if futs is not None:
            self._post_bwd_futs = list(futs)

    def _wait_post_backward_futures(self):
        futs, self._post_bwd_futs = self._post_bwd_futs, []
        for f in futs:
            f.wait()

    def _broadcast_tensors(self, tensors, root: int = 0):
        """Broadcast tensors from group rank `root` (0 but under join): floating
        tensors go through the libgsync pack kernel + one broadcast + unpack;
        others through a cat."""
        if self.world_size == 1 or not tensors:
            return
        floats = [t for t in tensors if t.is_floating_point() and is_dense(t)]
        others = [t for t in tensors if not (t.is_floating_point() and is_dense(t))]
        by_dtype: dict = {}
        for t in floats:
            by_dtype.setdefault(t.dtype, []).append(t)
        for dt, ts in by_dtype.items():
            plan = TensorListPlan([t.numel() for t in ts], self.device, align=BUCKET_ALIGN_ELEMS)
            plan.set_ptrs(0, ts)
            flat = torch.zeros(plan.flat_numel, dtype=dt, device=self.device)
            if self.rank == root:
                plan.pack(0, dt, flat)
            self._bcast_flat(flat, root)
            if self.rank != root:
                plan.unpack(flat, 0, dt)
        if others:
            flat = torch.cat([t.reshape(-1) for t in others])
            self._bcast_flat(flat, root)
            if self.rank != root:
                off = 0
                for t in others:
                    t.copy_(flat[off:off + t.numel()].view_as(t))
                    off += t.numel()

    def _bcast_flat(self, flat, root: int = 0):
        if self._comm is not None:
            self._comm.broadcast(flat, root=root, stream=L.stream_ptr(self.device))
            return
        src = dist.get_global_rank(self.process_group, root) if self.process_group is not dist.group.WORLD else root
        if flat.is_cuda and self._backend == "gloo":
            # a device tensor over gloo (ranks sharing a GPU: the rehearsal path) is staged
            # through host memory, as the bucket all-reduces are (_launch_external): no
            # collective of gloo's CUDA path runs on the rehearsal
            host = flat.cpu()
            dist.broadcast(host, src=src, group=self.process_group)
            flat.copy_(host)
        else:
            dist.broadcast(flat, src=src, group=self.process_group)

    @torch.no_grad()
    def _sync_module_states(self):
        """_sync_module_states: params + buffers from rank 0 (T:nn/parallel/distributed.py:860-870).
        Every parameter, frozen ones included (torch's ``module_states`` walks
        ``named_parameters()`` without a requires_grad filter)."""
        seen, params = set(), []
        for n, p in self.module.named_parameters():
            if n in self.parameters_to_ignore:
                continue
            if id(p) not in seen:
                seen.add(id(p))
                params.append(p.detach())
        self._broadcast_tensors(params + self._module_buffers())

    @torch.no_grad()
    def _sync_buffers(self, root: int = 0):
        """Per-forward BN buffer broadcast (T:nn/parallel/distributed.py:2178-2221):
        one pack launch + one RCCL broadcast + one unpack launch per word size,
        plan cached across steps.  Integer buffers (BN num_batches_tracked,
        int64) travel as fp32 words — the kernels move them bit for bit."""
        if self.buffer_hook is not None:
            self._run_buffer_hook()  # the hook decides how buffers agree (torch: _sync_module_buffers)
            return
        bufs = self._module_buffers()
        if self.world_size == 1 or not bufs:
            return
        key = tuple(id(t) for t in bufs)
        if self._buffers_plan is None or self._buffers_plan[0] != key:
            groups: dict = {}
            others = []
            for t in bufs:
                w = _as_words(t)
                if w is None:
                    others.append(t)
                else:
                    groups.setdefault(w.dtype, []).append(w)
            plans = []
            for dt, ws in groups.items():
                plan = TensorListPlan([w.numel() for w in ws], self.device, align=BUCKET_ALIGN_ELEMS)
                flat = torch.zeros(plan.flat_numel, dtype=dt, device=self.device)
                plan.set_ptrs(0, ws)
                plans.append((plan, ws, dt, flat))
            self._buffers_plan = (key, plans, others)
        _, plans, others = self._buffers_plan
        for plan, ws, dt, flat in plans:
            plan.set_ptrs(0, ws)
            if self.rank == root:
                plan.pack(0, dt, flat)
            self._bcast_flat(flat, root)
            if self.rank != root:
                plan.unpack(flat, 0, dt)
        if others:
            flat = torch.cat([t.reshape(-1) for t in others])
            self._bcast_flat(flat, root)
            if self.rank != root:
                off = 0
                for t in others:
                    t.copy_(flat[off:off + t.numel()].view_as(t))
                    off += t.numel()

    # ------------------------------------------------------------------ forward
    def _will_sync_module_buffers(self):
        return ((self.world_size > 1 or self.buffer_hook is not None) and self.require_forward_param_sync
                and self.broadcast_buffers and len(self._module_buffers()) != 0)

    def forward(self, *inputs, **kwargs):
        L.flush_deferred()
        if self._comm is not None:
            self._comm.check()  # watchdog / RCCL async error surfaces here, like ProcessGroupNCCL's
        grad_sync = torch.is_grad_enabled() and self.require_backward_grad_sync
        # under ddp.join(): tell the joined ranks this one is still training (their
        # Join context counts these), as torch's forward does
        work = Join.notify_join_context(self)
        if grad_sync:
            self._maybe_rebuild_buckets()
        if work is not None and not self._divide_by_initial_world_size:
            # divide by the ranks still training (torch: the Reducer waits on this work
            # for its div_factor_); a host read, in join mode only
            work.wait()
            self._set_div_factor(float(work.result()[0].item()))
        elif self._div_factor != self.world_size and not self._join_config.enable:
            self._set_div_factor(float(self.world_size))
        joining = self._join_config.enable
        bh = self.buffer_hook
        sync_bufs = self._will_sync_module_buffers()
        post_fwd = bh is not None and bh.buffer_comm_hook_location == _BufferCommHookLocation.POST_FORWARD
        if sync_bufs and not post_fwd:
            # under join rank 0 may have stopped: the highest still-training rank is the source
            self._sync_buffers(self._find_common_rank(self.rank, True) if joining else 0)
        if joining:
            self._check_global_requires_backward_grad_sync(is_joined_rank=False)
        if self.device_ids:
            dev = torch.device(self.device_type, self.device_ids[0])
            inputs = tuple(x.to(dev, non_blocking=True) if isinstance(x, torch.Tensor) else x for x in inputs)
            kwargs = {k: (v.to(dev, non_blocking=True) if isinstance(v, torch.Tensor) else v) for k, v in kwargs.items()}
        output = self.module(*inputs, **kwargs)
        if sync_bufs and post_fwd:
            self._sync_buffers()
        if grad_sync:
            self.require_forward_param_sync = True
            self._prepare_for_backward()
        else:
            self.require_forward_param_sync = False
            self._found_inf_valid = False  # grads will change without a synchronising unpack
            self._sqnorm_valid = False
        return output

    def _prepare_for_backward(self):
        want = self._native_ok()
        if want != self._native_on:
            self._set_native(want)
        if self._native_on and self._in_backward and self._native.finalize_queued():
            self._finalize_queued = True
        if self._in_backward and self._finalize_queued:
            raise RuntimeError(
                "Expected to have finished reduction in the prior iteration before starting a new one. "
                "This error indicates that your module has parameters that were not used in producing loss.")
        sq = self._sqnorm_target
        if self._found_inf_target is not None:
            self._found_inf_target.zero_()  # on the producer stream, before any bucket is launched
        self._found_inf_valid = False
        self._sqnorm_valid = False
        L.check(L.lib().gs_bucketer_prepare(self._bucketer.handle, None if sq is None else sq.data_ptr()),
                "gs_bucketer_prepare")
        self._in_backward = True
        self._finalize_queued = False
        self._pending = {}
        self._record_order = not self._has_rebuilt_buckets and (self.static_graph or not self.find_unused_parameters)
        self._ready_now = []
        if self._record_order:
            self._ready_order = []
        if self._native_on:
            self._native.prepare(self._record_order)

    @contextmanager
    def no_sync(self):
        """Gradients accumulate locally; synchronised on the first backward after exit."""
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    # ------------------------------------------------------------------ hooks
    def _make_hook(self, idx):
        dense_strides = [None]  # strides of this parameter once seen dense (grads in the same layout are too)

        def hook(param):
            if not self._in_backward:
                if self._used_local is not None:
                    self._used_local[idx] = 1  # a no_sync backward: used for the next sync
                return
            if not self._finalize_queued:
                self._finalize_queued = True
                self._stream = L.stream_ptr(self.device)
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)
            if self._record_order:
                self._ready_order.append(idx)
            if self._used_local is not None:
                self._used_local[idx] = 1
                self._ready_now.append(idx)
            g = param.grad
            ps = param.stride()
            # fast path: the grad has the strides of a parameter already seen to be dense
            if g.stride() != ps or dense_strides[0] != ps:
                if not dense_like_param(g, param):
                    dense = torch.empty_like(param)
                    dense.copy_(g)
                    param.grad = g = dense
                elif is_dense(param):
                    dense_strides[0] = ps
            cap = self._capture_local
            if cap is not None and idx in cap:
                cap[idx] = g.detach().clone()  # on the producer stream, before the pack
            b = self._bucketer
            rc = b._mark(b.handle, idx, g.data_ptr(), self._stream, b._ready, b._n_ready_ref)
            if rc < 0:
                L.check(rc, "gs_bucketer_mark_ready")
            if b._n_ready.value:
                ready = [b._ready[k] for k in range(b._n_ready.value)]
                if not (b.flags & L.GS_BKT_AUTO_COLLECTIVE):
                    self._launch_external(ready)
                elif self._overlap is not None:
                    self._overlap_step(ready)

        return hook

    def _launch_external(self, bucket_ids):
        b = self._bucketer
        nb = len(b.buckets)
        for bi in bucket_ids:
            buf = b.buffers[bi]
            if self._comm_hook is not None:
                state, hook = self._comm_hook
                gb = GradBucket(bi, buf, [self._params[i] for i in b.buckets[bi]], b.offsets_in_bucket[bi],
                                bi == nb - 1)
                self._pending[bi] = ("fut", hook(state, gb))
            elif self._comm is not None:
                self._comm.all_reduce(buf, stream=L.stream_ptr(self.device))
                self._pending[bi] = ("done", None)
            elif buf.is_cuda and self._backend == "gloo":
                # gloo over device buckets (ranks sharing a GPU: the rehearsal path).  Not
                # gloo's own CUDA path: its async all-reduce of a device tensor issued from
                # the autograd thread deadlocks at 4 ranks on one GPU in the second
                # iteration (reproduced without libgsync: scripts/gloo_cuda_repro.py
                # MODE=hook) — stage through host memory here instead
                host = buf.to("cpu")  # waits for this bucket's pack on the producer stream
                self._pending[bi] = ("host", (host, dist.all_reduce(host, group=self.process_group,
                                                                    async_op=True)))
            else:
                self._pending[bi] = ("work", dist.all_reduce(buf, group=self.process_group, async_op=True))

    def _finalize_backward(self):
        b = self._bucketer
        if self.find_unused_parameters:
            # a parameter unused in this backward that still holds a grad (accumulated
            # under no_sync) contributes that grad, as torch's mark_variable_ready_dense
            # copies a defined grad of an unused variable into its bucket; the rest
            # contribute zeros
            fired = set(self._ready_now)
            for i, p in enumerate(self._params):
                if i not in fired and p.grad is not None:
                    g = p.grad
                    if not dense_like_param(g, p):
                        dense = torch.empty_like(p)
                        dense.copy_(g)
                        p.grad = g = dense
                    L.check(L.lib().gs_bucketer_mark_ready(b.handle, i, g.data_ptr(), self._stream, b._ready,
                                                           ctypes.byref(b._n_ready)), "gs_bucketer_mark_ready")
                    self._dispatch_ready(b)
            L.check(L.lib().gs_bucketer_mark_unused(b.handle, self._stream, b._ready, ctypes.byref(b._n_ready)),
                    "gs_bucketer_mark_unused")
            self._dispatch_ready(b)
        elif self.static_graph:
            # static_graph: parameters the (fixed) graph never uses are marked ready at
            # the end of backward, as torch's static-graph Reducer does; their slots
            # reduce as zeros and, unused on every rank, their grads stay None
            L.check(L.lib().gs_bucketer_mark_unused(b.handle, self._stream, b._ready, ctypes.byref(b._n_ready)),
                    "gs_bucketer_mark_unused")
            self._dispatch_ready(b)
        for bi in sorted(self._pending):
            kind, obj = self._pending[bi]
            if kind == "work":
                obj.wait()
            elif kind == "host":
                host, work = obj
                work.wait()
                b.buffers[bi].copy_(host)
            elif kind == "fut":
                res = obj.wait()
                if isinstance(res, (list, tuple)):
                    res = res[0]
                if res is not None and res.data_ptr() != b.buffers[bi].data_ptr():
                    b.buffers[bi].copy_(res.reshape(-1)[: b.buffers[bi].numel()])
        self._pending = {}
        if self._post_bwd_futs:
            self._wait_post_backward_futures()
        L.check(L.lib().gs_bucketer_finalize(b.handle, self._stream), "gs_bucketer_finalize")
        if self._overlap is not None and not (b.flags & L.GS_BKT_AUTO_COLLECTIVE):
            # external collectives (gloo, host buckets): the grads exist once the
            # bucketer has unpacked them at finalize — step every bucket then
            self._overlap_step(range(len(b.buckets)))
        self._found_inf_valid = self._found_inf_target is not None
        self._sqnorm_valid = self._sqnorm_fusable()
        self._sqnorm_versions = self._grad_versions() if self._sqnorm_valid else None
        if self.find_unused_parameters:
            if self.world_size > 1:
                self._grads_of_locally_unused()
            self._used_local = [0] * len(self._params)  # torch resets the map after each sync
        if self.gradient_as_bucket_view:
            for i, p in enumerate(self._params):
                if p.grad is not None:
                    view = b.bucket_view(i)
                    if p.grad.data_ptr() != view.data_ptr():
                        p.grad = view
        self._in_backward = False
        self._finalize_queued = False
        self._num_iterations += 1

    def _dispatch_ready(self, b):
        if b._n_ready.value:
            ready = [b._ready[k] for k in range(b._n_ready.value)]
            if not (b.flags & L.GS_BKT_AUTO_COLLECTIVE):
                self._launch_external(ready)
            elif self._overlap is not None:
                self._overlap_step(ready)

    def _grads_of_locally_unused(self):
        """find_unused_parameters: a parameter unused on this rank but used on
        another gets the averaged grad from its bucket, as torch's
        ``copy_bucket_to_grad`` creates it (T:.../reducer.cpp finalize_bucket_dense:
        ``global_unused`` from the all-reduced local-used map; globally unused
        parameters keep their grad untouched).  One MAX all-reduce of the used
        map per iteration and a host read of it — torch's Reducer does the same."""
        glob = self._ctl_all_reduce(torch.tensor(self._used_local, dtype=torch.int32), "max").tolist()
        b = self._bucketer
        made = []
        for i, p in enumerate(self._params):
            if glob[i] and not self._used_local[i]:
                view = b.bucket_view(i)
                if view.dtype != p.dtype:  # bf16/fp16 buckets: the grad keeps the parameter's dtype
                    p.grad = view.to(p.dtype, memory_format=torch.preserve_format)
                elif self.gradient_as_bucket_view:
                    p.grad = view
                else:
                    p.grad = view.clone(memory_format=torch.preserve_format)
                made.append(p.grad)
        if made:
            self._check_extra_grads(made)

    def _check_extra_grads(self, grads):
        """The fused checks of the bucket unpack (AMP non-finite flag, Σg²)
        over grads created outside it — those of parameters unused on this rank
        (their slots are not unpacked): every rank's flag then covers the same
        averaged grads, so every rank takes the same skip decision."""
        if self._found_inf_target is None and self._sqnorm_target is None:
            return
        by_dtype: dict = {}
        for g in grads:
            by_dtype.setdefault(g.dtype, []).append(g)
        cache = self.__dict__.setdefault("_extra_plans", {})
        for dt, gs in by_dtype.items():
            key = (dt,) + tuple(g.numel() for g in gs)
            plan = cache.get(key)
            if plan is None:
                plan = cache[key] = TensorListPlan([g.numel() for g in gs], self.device)
            plan.set_ptrs(0, gs)
            if self._found_inf_target is not None:
                plan.unscale_check(0, dt, None, self._found_inf_target)
            if self._sqnorm_target is not None:
                plan.sqnorm(0, dt, self._sqnorm_target, accumulate=True)

    def _maybe_rebuild_buckets(self):
        if self._has_rebuilt_buckets or not (self.static_graph or not self.find_unused_parameters):
            return
        if len(self._ready_order) != len(self._params) or self._num_iterations == 0:
            return
        limits = [self.first_bucket_bytes_cap, self.bucket_bytes_cap]
        buckets = compute_bucket_assignment_by_size(self._params, limits, order=self._ready_order)
        if self._last_bucket_cap is not None:
            buckets = split_last_bucket(buckets, [p.numel() * p.element_size() for p in self._params],
                                        self._last_bucket_cap)
        buckets = self._sync_bucket_indices(buckets)
        if self.gradient_as_bucket_view:
            for p in self._params:  # grads must not alias the old buckets once they are freed
                if p.grad is not None:
                    p.grad = p.grad.clone()
        self._bucketer = self._make_bucketer(buckets)
        self._has_rebuilt_buckets = True
        self._ready_order = []

    def _sync_bucket_indices(self, buckets):
        """Broadcast rank 0's rebuilt layout (Reducer::sync_bucket_indices)."""
        if self.world_size == 1:
            return buckets
        n = len(self._params)
        flat = [len(buckets)] + [len(b) for b in buckets] + [i for b in buckets for i in b]
        flat += [0] * (2 * n + 1 - len(flat))
        v = self._ctl_broadcast(torch.tensor(flat, dtype=torch.int64)).tolist()
        nb = v[0]
        counts = v[1:1 + nb]
        out, pos = [], 1 + nb
        for c in counts:
            out.append(v[pos:pos + c])
            pos += c
        return out

    def _overlap_step(self, bucket_ids):
        """The overlapped optimizer's update of buckets `bucket_ids`: one fused
        kernel per bucket on the stream its chain ran on, behind its unpack."""
        ov = self._overlap
        main = ov["opt"]
        hyper = {k: v for k, v in main.param_groups[0].items() if k != "params"}
        for bi in bucket_ids:
            bo = ov["per_bucket"].get(bi)
            if bo is None:
                members = [self._params[i] for i in self._bucketer.buckets[bi] if id(self._params[i]) in ov["ids"]]
                bo = ov["cls"](members, *ov["args"], **ov["kwargs"]) if members else False
                ov["per_bucket"][bi] = bo
            if not bo:
                continue
            # one optimizer state across the buckets, held by the main optimizer (its
            # state_dict / load_state_dict, which may replace the dict); lr schedules
            # act on the main optimizer's group
            bo.state = main.state
            bo.param_groups[0].update(hyper)
            ptr = ctypes.c_void_p()
            L.check(L.lib().gs_bucketer_bucket_stream(self._bucketer.handle, bi, ctypes.byref(ptr)),
                    "gs_bucketer_bucket_stream")
            if ptr.value:
                st = ov["streams"].get(ptr.value)
                if st is None:
                    st = ov["streams"][ptr.value] = torch.cuda.ExternalStream(ptr.value, device=self.device)
                with torch.cuda.stream(st):
                    self._step_bucket(bi, bo)
            else:
                self._step_bucket(bi, bo)

    def _step_bucket(self, bi, bo):
        """One overlapped update of bucket bi.  As torch's _hook_then_optimizer
        (T:distributed/algorithms/ddp_comm_hooks/optimizer_overlap_hooks.py), every
        bucket parameter steps with its bucket gradient — a parameter unused on
        this rank (find_unused_parameters / static_graph: no grad yet) with the
        averaged one from the bucket view (zeros when unused everywhere), so weight
        decay and momentum apply on every rank alike.  Runs on the bucket's stream,
        behind its chain; the temporary grads are dropped after the launch
        (_grads_of_locally_unused creates the kept ones at finalize)."""
        tmp = []
        for p in bo.param_groups[0]["params"]:
            if p.grad is None:
                i = self._param_index[id(p)]
                view = self._bucketer.bucket_view(i)
                p.grad = view if view.dtype == p.dtype else view.to(p.dtype, memory_format=torch.preserve_format)
                tmp.append(p)
        bo.step()
        for p in tmp:
            p.grad = None

    # ------------------------------------------------------------------ API
    def _register_fused_optim(self, optim: type, *args, optim_params=None, **kwargs):
        """Overlapped optimizer (T:nn/parallel/distributed.py ``_register_fused_optim``,
        T:distributed/algorithms/_optimizer_overlap/optimizer_overlap.py and
        ddp_comm_hooks/optimizer_overlap_hooks.py ``_hook_then_optimizer``):
        each bucket's parameters are updated as soon as its averaged grads
        exist, so the update runs under the rest of backward instead of after it.
        torch chains a functional per-parameter ``step_param`` on the bucket's
        future; here ONE fused SGD / Adam(W) kernel per bucket is enqueued on the
        stream the bucket's pack -> collective -> unpack chain ran on
        (``gs_bucketer_bucket_stream``), right behind its unpack.  As in torch:
        call once, the caller no longer calls ``optimizer.step()``, no comm hook,
        and ``no_sync`` accumulation updates at the next synchronising backward.
        ``optim``: torch.optim.SGD / Adam / AdamW or FusedSGD / FusedAdam(W)
        (same arguments); the optimizer holding the state is
        ``ddp._overlapped_optimizer`` (state_dict, lr schedules)."""
        import inspect

        from .optim import FusedAdam, FusedAdamW, FusedSGD

        if self._overlap is not None:
            raise RuntimeError("_register_fused_optim should only be called once on a DDP instance")
        if self._comm_hook is not None:
            raise RuntimeError("_register_fused_optim and register_comm_hook do not compose (as in torch)")
        table = {torch.optim.SGD: FusedSGD, torch.optim.Adam: FusedAdam, torch.optim.AdamW: FusedAdamW,
                 FusedSGD: FusedSGD, FusedAdam: FusedAdam, FusedAdamW: FusedAdamW}
        cls = next((table[c] for c in inspect.getmro(optim) if c in table), None)
        if cls is None:
            raise RuntimeError(f"{optim} does not support overlapped DDP (SGD, Adam, AdamW)")
        if kwargs.get("max_grad_norm"):
            raise RuntimeError("overlapped optimizer: a global-norm clip needs every bucket before any update")
        if self._found_inf_target is not None:
            raise RuntimeError("overlapped optimizer: AMP loss scaling needs the overflow check of every bucket "
                               "before any update (torch's overlapped optimizer has no GradScaler path either)")
        params = list(optim_params) if optim_params is not None else list(self._params)
        opt = cls(params, *args, **kwargs)
        self._overlap = {"cls": cls, "args": args, "kwargs": kwargs, "opt": opt, "ids": {id(p) for p in params},
                         "per_bucket": {}, "streams": {}}
        self._overlapped_optimizer = opt

    def register_comm_hook(self, state: object, hook: Callable):
        """hook(state, GradBucket) -> torch.futures.Future[Tensor] (T:nn/parallel/distributed.py:1953)."""
        if self._comm_hook is not None:
            raise RuntimeError("register_comm_hook or register_builtin_comm_hook can only be called once.")
        if self._overlap is not None:
            raise RuntimeError("register_comm_hook and _register_fused_optim do not compose (as in torch)")
        if not callable(hook):
            raise TypeError("Communication hook must be callable.")
        self._comm_hook = (state, hook)
        self._bucketer = self._make_bucketer(self._bucketer.buckets)

    def set_found_inf_target(self, t: torch.Tensor | None):
        """Fuse GradScaler's non-finite check of the averaged grads into the
        bucket unpack (fp32 1-element device tensor, zeroed by every
        synchronising backward; ``_found_inf_valid`` tells whether the last
        backward filled it)."""
        if t is not None and (t.numel() != 1 or t.dtype != torch.float32 or t.device != self.device):
            raise ValueError("found_inf target must be a 1-element float32 tensor on the DDP device")
        if t is not None and self._overlap is not None:
            raise RuntimeError("AMP loss scaling and the overlapped optimizer do not compose")
        self._found_inf_target = t
        self._found_inf_valid = False
        L.check(L.lib().gs_bucketer_set_found_inf(self._bucketer.handle, None if t is None else t.data_ptr()),
                "gs_bucketer_set_found_inf")

    def set_grad_sqnorm_target(self, t: torch.Tensor | None):
        """Fuse Σg² of the averaged grads into the bucket unpack (fp32 1-element
        device tensor; the first bucket's unpack writes it, the others add, in
        bucket order); ``_sqnorm_valid`` tells whether the last synchronising
        backward filled it (not in ``gradient_as_bucket_view`` mode: no unpack)."""
        if t is not None and (t.numel() != 1 or t.dtype != torch.float32 or t.device != self.device):
            raise ValueError("Σg² target must be a 1-element float32 tensor on the DDP device")
        self._sqnorm_target = t
        self._sqnorm_valid = False

    def _sqnorm_fusable(self) -> bool:
        return self._sqnorm_target is not None and not self.gradient_as_bucket_view

    def _grad_versions(self) -> int:
        """Σ of the grads' autograd version counters when the unpacks formed Σg²:
        any in-place change of a grad after that (torch ops bump the counter;
        libgsync's own in-place grad kernels — GradScaler.unscale_, clip_grad_norm_
        — bump it explicitly) makes the fused Σg² stale (a scaled Σg²
        folded after ``scaler.unscale_``)."""
        return sum(p.grad._version for p in self._params if p.grad is not None)

    def set_timeline(self, level: int):
        """Which HIP timing events the bucket chains record
        (gs_bucketer_set_timeline): 0 none; 1 (default) the tail total only
        (:meth:`tail_ms` ``total``); 2 every bucket's queue / pack / collective /
        unpack (:meth:`bucket_timeline_ms`, :meth:`bucket_comm_ms`).  Each event is
        a packet on its stream (~10 µs on the exposed tail at level 2), so timed
        runs stay at level ≤ 1 and read the split from a separate step."""
        self._timeline = int(level)
        L.check(L.lib().gs_bucketer_set_timeline(self._bucketer.handle, self._timeline), "gs_bucketer_set_timeline")

    def bucket_comm_ms(self):
        """Per-bucket collective time of the last iteration (HIP events on the
        comm stream; -1 unless :meth:`set_timeline` is 2)."""
        out = []
        for bi in range(len(self._bucketer.buckets)):
            ms = ctypes.c_float()
            L.check(L.lib().gs_bucketer_last_comm_ms(self._bucketer.handle, bi, ctypes.byref(ms)),
                    "gs_bucketer_last_comm_ms")
            out.append(ms.value)
        return out

    def enable_bucket_checksums(self, on: bool = True):
        """Debug mode (GSYNC_DEBUG=1 at construction does the
        same): every synchronising backward writes Σ of each bucket after its
        pack and after its collective (gs_bucketer_set_debug);
        :meth:`verify_bucket_checksums` checks them across ranks."""
        if on:
            self._debug_sums = torch.zeros(3 * len(self._bucketer.buckets), dtype=torch.float32, device=self.device)
            ptr = self._debug_sums.data_ptr()
        else:
            self._debug_sums, ptr = None, None
        L.check(L.lib().gs_bucketer_set_debug(self._bucketer.handle, ptr), "gs_bucketer_set_debug")

    def bucket_checksums(self):
        """[(Σx after pack, Σx after collective, Σx² after pack)] per bucket of the last backward."""
        if self._debug_sums is None or self._debug_sums.numel() == 0:
            raise RuntimeError("bucket checksums are off (GSYNC_DEBUG=1 or enable_bucket_checksums())")
        return [tuple(x) for x in self._debug_sums.view(-1, 3).cpu().tolist()]

    def verify_bucket_checksums(self, rtol: float = 1e-4):
        """Collective over the DDP group, after a synchronising backward:
        * the all-reduced bucket is identical on every rank (Σx MIN == MAX);
        * Σ_r (Σx after pack)_r == Σx after the collective within
          rtol·sqrt(numel·Σ_r Σx²_r) (an fp32-rounding scale: >= rtol·Σ|x|/…
          by Cauchy-Schwarz; a wrong or missing contribution is O(1) off).
        Raises RuntimeError naming the first bad bucket; returns per bucket
        (Σ_r pre, post, tolerance)."""
        sums = self._debug_sums.view(-1, 3).double()
        pre, post, sq = sums[:, 0].contiguous(), sums[:, 1].contiguous(), sums[:, 2].contiguous()
        tot = self._ctl_all_reduce(pre.clone(), "sum")
        sqt = self._ctl_all_reduce(sq.clone(), "sum")
        lo = self._ctl_all_reduce(post.clone(), "min")
        hi = self._ctl_all_reduce(post.clone(), "max")
        out = []
        for bi, buf in enumerate(self._bucketer.buffers):
            tol = rtol * (buf.numel() * float(sqt[bi])) ** 0.5 + 1e-30
            if float(lo[bi]) != float(hi[bi]):
                raise RuntimeError(f"bucket {bi}: the all-reduced bucket differs across ranks "
                                   f"(checksum {float(lo[bi])} vs {float(hi[bi])})")
            if abs(float(tot[bi]) - float(post[bi])) > tol:
                raise RuntimeError(f"bucket {bi}: sum over ranks of the packed bucket {float(tot[bi])} != "
                                   f"the all-reduced bucket {float(post[bi])} (tolerance {tol})")
            out.append((float(tot[bi]), float(post[bi]), tol))
        return out

    def bucket_timeline_ms(self):
        """Per-bucket timeline of the last iteration (gs_bucketer_last_timing):
        list of dicts queue / pack / collective / unpack / ready_to_done, ms
        (None where untimed: host buckets, external collectives, hipGraph replays)."""
        out = []
        buf = (ctypes.c_float * 5)()
        for bi in range(len(self._bucketer.buckets)):
            L.check(L.lib().gs_bucketer_last_timing(self._bucketer.handle, bi, buf), "gs_bucketer_last_timing")
            v = [float(buf[k]) if buf[k] >= 0 else None for k in range(5)]
            out.append(dict(zip(("queue", "pack", "collective", "unpack", "ready_to_done"), v)))
        return out

    def tail_ms(self):
        """The exposed end-of-backward tail of the last iteration: from the
        last bucket's ready event (its last gradient produced) to the
        finalize event every bucket's chain has passed, split into the last
        bucket's queue / pack / collective / unpack (HIP events; the split is
        None below timeline level 2)."""
        tl = self.bucket_timeline_ms()
        if not tl or tl[-1]["ready_to_done"] is None:
            return None
        last = tl[-1]
        return {"total": last["ready_to_done"], "queue": last["queue"], "pack": last["pack"],
                "collective": last["collective"], "unpack": last["unpack"],
                "last_bucket_bytes": self._bucketer.buffers[-1].numel() * self._bucketer.buffers[-1].element_size()}

    def _get_ddp_logging_data(self):
        b = self._bucketer
        return {
            "world_size": self.world_size,
            "rank": self.rank,
            "backend_name": "rccl(libgsync)" if self._comm is not None else self._backend,
            "bucket_cap_bytes": self.bucket_bytes_cap,
            "find_unused_parameters": int(self.find_unused_parameters),
            "gradient_as_bucket_view": int(self.gradient_as_bucket_view),
            "static_graph": int(self.static_graph),
            "comm_hook": "" if self._comm_hook is None else getattr(self._comm_hook[1], "__qualname__", "hook"),
            "has_rebuilt_buckets": int(self._has_rebuilt_buckets),
            "bucket_sizes": b.logical_bytes(),
            "rebuilt_bucket_sizes": b.logical_bytes() if self._has_rebuilt_buckets else [],
            "padded_bucket_numels": [buf.numel() for buf in b.buffers],
            "bucket_dtype": str(self._bucket_dtype) if self._bucket_dtype is not None else
            ",".join(sorted({str(d) for d in b.bucket_dtypes})),
            "bucket_policy": self.bucket_policy,
            "rccl_max_ctas": self._comm.max_ctas if self._comm is not None else None,
            "last_bucket_cap_bytes": self._last_bucket_cap,
            "xgmi_calibration": self._xgmi_calibration,
            "num_parameter_tensors": len(self._params),
            "total_parameter_size_bytes": sum(p.numel() * p.element_size() for p in self._params),
        }

    # ---- uneven inputs: torch's DDP.join() (T:nn/parallel/distributed.py join /
    # _DDPJoinHook, T:distributed/algorithms/join.py).  Ranks that run out of
    # batches shadow every collective of a training iteration — the forward's
    # buffer broadcast (from the highest still-training rank), the grad-sync flag,
    # one all-reduce of zeros per bucket in bucket order (the same count, dtype
    # and communicator as the bucketer's), the find-unused map — until all have
    # joined; then the last joiner's parameters and buffers are broadcast.
    def join(self, divide_by_initial_world_size: bool = True, enable: bool = True,
             throw_on_early_termination: bool = False):
        if self._overlap is not None:
            raise NotImplementedError("join() with the overlapped optimizer")
        return Join([self], enable, throw_on_early_termination,
                    divide_by_initial_world_size=divide_by_initial_world_size)

    def join_hook(self, **kwargs) -> JoinHook:
        self._divide_by_initial_world_size = kwargs.get("divide_by_initial_world_size", True)
        return _DDPJoinHook(self)

    def _set_div_factor(self, div: float):
        """The packs' divisor for the next backward (gs_bucketer_set_div_factor)."""
        if div != self._div_factor:
            L.check(L.lib().gs_bucketer_set_div_factor(self._bucketer.handle, float(div)),
                    "gs_bucketer_set_div_factor")
            self._div_factor = div

    @property
    def join_device(self) -> torch.device:
        return self.device

    @property
    def join_process_group(self):
        return self.process_group

    def _find_common_rank(self, input_rank: int, rank_cond: bool) -> int:
        r = self._ctl_all_reduce(torch.tensor([input_rank if rank_cond else -1], dtype=torch.int64), "max")
        v = int(r.item())
        if v < 0:
            raise ValueError("join: no rank qualified as the common rank")
        return v

    def _check_global_requires_backward_grad_sync(self, is_joined_rank: bool):
        t = torch.tensor([1.0 if (not is_joined_rank and self.require_backward_grad_sync) else 0.0])
        t = self._ctl_all_reduce(t, "sum")
        return bool(t.item() != 0) if is_joined_rank else None

    def _match_all_reduce_for_bwd_pass(self):
        """A joined rank's side of one backward: an all-reduce of zeros per bucket,
        in bucket order, through the path the training ranks' buckets take."""
        b = self._bucketer
        nb = len(b.buckets)
        for bi, buf in enumerate(b.buffers):
            z = torch.zeros_like(buf)
            if self._comm_hook is not None:
                state, hook = self._comm_hook
                hook(state, GradBucket(bi, z, [self._params[i] for i in b.buckets[bi]], b.offsets_in_bucket[bi],
                                       bi == nb - 1)).wait()
            elif self._comm is not None:
                self._comm.all_reduce(z, stream=L.stream_ptr(self.device))
            elif z.is_cuda and self._backend == "gloo":
                dist.all_reduce(z.cpu(), group=self.process_group)  # as _launch_external stages it
            else:
                dist.all_reduce(z, group=self.process_group)

    def _sync_final_model(self, is_last_joiner: bool):
        """After every rank joined: the last joiner's parameters (and buffers)
        to all ranks (torch: _sync_module_states from the authoritative rank)."""
        root = self._find_common_rank(self.rank, is_last_joiner)
        seen, ts = set(), []
        for n, p in self.module.named_parameters():
            if n not in self.parameters_to_ignore and id(p) not in seen:
                seen.add(id(p))
                ts.append(p.detach())
        if self.broadcast_buffers:
            ts += self._module_buffers()
        with torch.no_grad():
            self._broadcast_tensors(ts, root)

    @staticmethod
    def _set_params_and_buffers_to_ignore_for_model(module, params_and_buffers_to_ignore):
        """torch's static helper (T:nn/parallel/distributed.py): names (as in
        ``named_parameters`` / ``named_buffers``) that a DDP wrapping `module`
        neither synchronises nor broadcasts.  Call before wrapping."""
        module._ddp_params_and_buffers_to_ignore = params_and_buffers_to_ignore
        for name, param in module.named_parameters():
            if name in params_and_buffers_to_ignore:
                param._ddp_ignored = True
        for name, buffer in module.named_buffers():
            if name in params_and_buffers_to_ignore:
                buffer._ddp_ignored = True

    def bucket_indices(self):
        return [list(b) for b in self._bucketer.buckets]

    def close(self):
        """Detach from the module: remove the gradient hooks and free the
        buckets (the module can then be wrapped again, e.g. with another
        bucket policy).  Not collective."""
        for h in getattr(self, "_hook_handles", []):
            try:
                h.remove()
            except Exception:  # pragma: no cover
                pass
        self._hook_handles = []
        if getattr(self, "_native", None) is not None:
            self._native.detach()
            self._native_on = False
        b = getattr(self, "_bucketer", None)
        if b is not None:
            if self.gradient_as_bucket_view:
                for p in self._params:  # grads must not alias the buckets about to be freed
                    if p.grad is not None:
                        p.grad = p.grad.clone()
            b.close()
        if getattr(self, "_own_comm", False) and self._comm is not None:
            self._comm.close()
            self._own_comm = False

    def __del__(self):
        for h in getattr(self, "_hook_handles", []):
            try:
                h.remove()
            except Exception:  # pragma: no cover
                pass
        nat = getattr(self, "_native", None)
        if nat is not None:
            nat.detach()


class _DDPJoinHook(JoinHook):
    """A joined rank's shadow of one DDP iteration (torch's _DDPJoinHook)."""

    def __init__(self, ddp):
        self.ddp = ddp
        super().__init__()

    def main_hook(self):
        d = self.ddp
        d._maybe_rebuild_buckets()
        # the training ranks' forward, collective for collective: the buffer sync before
        # the module (common-rank pick + broadcast, or a PRE_FORWARD buffer comm hook),
        # the sync flag, then a POST_FORWARD buffer comm hook after the module (torch
        # leaves buffer comm hooks under join unsupported, pytorch#65436)
        bh = d.buffer_hook
        post_fwd = bh is not None and bh.buffer_comm_hook_location == _BufferCommHookLocation.POST_FORWARD
        sync_bufs = d._will_sync_module_buffers()
        if sync_bufs and not post_fwd:
            d._sync_buffers(d._find_common_rank(d.rank, False))
        should_sync = d._check_global_requires_backward_grad_sync(is_joined_rank=True)
        if sync_bufs and post_fwd:
            d._sync_buffers()
            d._wait_post_backward_futures()  # no backward here to await the hook's futures
        d.require_forward_param_sync = should_sync
        if not should_sync:
            return
        d._match_all_reduce_for_bwd_pass()
        if d.find_unused_parameters:
            d._ctl_all_reduce(torch.zeros(len(d._params), dtype=torch.int32), "max")  # the used map

    def post_hook(self, is_last_joiner: bool):
        self.ddp._sync_final_model(is_last_joiner)


DDP = DistributedDataParallel
