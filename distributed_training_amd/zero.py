"""ZeRO-1/2 data parallelism on libgsync (the DeepSpeed / ColossalAI
LowLevelZero path; configured at
R:resnet/deepspeed/deepspeed_train.py:210-219 and R:resnet/colossal/colossal_train.py:135-136).

Layout (per bucket of <= reduce_bucket_size elements, DeepSpeed default 5e7 —
one bucket for ResNet-18/50):

  param flat (model dtype)  [ rank0 shard | rank1 shard | ... ]   params are views of it
  grad bucket (model dtype) same layout; packed with the fused 1/ws scale
  master (fp32)             this rank's shard only, plus exp_avg / exp_avg_sq

backward: hooks pack each bucket and RCCL reduce-scatters it (stage 2) or
          all-reduces it (stage 1) on libgsync's stream, under backward;
step:     (fp16) non-finite check of the shard + MAX all-reduce of the flag,
          (clip) Σg² partial sums of the shard + one SUM all-reduce of
          them (<= 1 Ki floats), folded into the update (no combine / coefficient
          launch); ONE fused Adam/SGD launch over all shards
          that also writes the low-precision params into this rank's slice
          of the param flat buffer; in-place all-gather of each bucket.
No host synchronisation except the fp16 loss-scale bookkeeping (DeepSpeed
reads its overflow flag on the host too).

Parity: ZeRO-1/2 == DDP + the same optimizer (reduction order aside); the
DeepSpeed/Colossal-specific numerics (AdamW mode, clip epsilon, loss scaling
schedule) are restated from their published algorithms — DeepSpeed and
ColossalAI are not installed here, so that part is "parity unpinned"
(SURVEY.md §8c).
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.distributed as dist

from . import _lib as L
from .comm import get_communicator
from .ddp import BUCKET_ALIGN_ELEMS, compute_bucket_assignment_by_size
from .multi_tensor import TensorListPlan, clip_coef, dense_like_param, update_task_units
from . import optim as _optim


class DynamicLossScaler:
    """DeepSpeed DynamicLossScaler semantics (loss_scale 0 = dynamic):
    overflow -> (hysteresis) halve, floor at min_scale, skip the step;
    `scale_window` clean steps -> double."""

    def __init__(self, init_scale=2.0 ** 15, scale_window=500, hysteresis=2, min_scale=1.0, scale_factor=2.0,
                 dynamic=True):
        self.scale = float(init_scale)
        self.scale_window = scale_window
        self.hysteresis = hysteresis
        self.cur_hysteresis = hysteresis
        self.min_scale = min_scale
        self.scale_factor = scale_factor
        self.dynamic = dynamic
        self.last_overflow_iter = -1
        self.iter = 0

    def update(self, overflow: bool):
        if not self.dynamic:
            self.iter += 1
            return
        if overflow:
            if self.cur_hysteresis > 1:
                self.cur_hysteresis -= 1
            else:
                self.scale = max(self.scale / self.scale_factor, self.min_scale)
            self.last_overflow_iter = self.iter
        elif (self.iter - self.last_overflow_iter) % self.scale_window == 0:
            self.scale *= self.scale_factor
            self.cur_hysteresis = self.hysteresis
        self.iter += 1

    def state_dict(self):
        return dict(self.__dict__)

    def load_state_dict(self, sd):
        self.__dict__.update(sd)


class ZeroDataParallel:
    def __init__(self, module: torch.nn.Module, *, stage: int = 2, optimizer: str = "adamw", lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, momentum: float = 0.0,
                 process_group=None, reduce_bucket_size: int = int(5e7), gradient_clipping: float = 0.0,
                 loss_scaler: DynamicLossScaler | None = None, broadcast_params: bool = True,
                 capturable: bool = False, overlap_allgather: bool = False,
                 allgather_bucket_size: int | None = None, communicator=None):
        if stage not in (1, 2):
            raise NotImplementedError(f"ZeRO stage {stage}: only 1 and 2 are on the gradient-sync path")
        if not dist.is_initialized():
            raise RuntimeError("ZeroDataParallel needs an initialised process group")
        self.module = module
        self.stage = stage
        self.pg = process_group if process_group is not None else dist.group.WORLD
        self.world = dist.get_world_size(self.pg)
        self.rank = dist.get_rank(self.pg)
        self.params = [p for p in module.parameters() if p.requires_grad]
        dts = {p.dtype for p in self.params}
        if len(dts) != 1:
            raise NotImplementedError(f"ZeRO: one parameter dtype expected, got {dts}")
        self.dtype = next(iter(dts))
        self.device = self.params[0].device
        self.is_cuda = self.device.type == "cuda"
        self.kind = optimizer
        self.hp = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, momentum=momentum)
        self.param_groups = [dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, momentum=momentum,
                                  params=self.params)]
        self.clip = float(gradient_clipping or 0.0)
        self.scaler = loss_scaler
        self.step_count = 0
        # capturable (CapturedStep): Adam's step counter, lr and bias corrections live on
        # the device (gs_adam_hyper advances them per launch, also on graph replays)
        self.capturable = bool(capturable)
        if self.capturable and (loss_scaler is not None or optimizer == "sgd"):
            raise NotImplementedError("capturable ZeRO: Adam/AdamW without a dynamic loss scaler "
                                      "(DeepSpeed's overflow check reads the flag on the host)")
        self.require_backward_grad_sync = True
        backend = dist.get_backend(self.pg)
        self._comm = None
        if communicator is not None:  # a caller-owned libgsync Communicator over this group
            self._comm = communicator
        elif self.is_cuda and backend == "nccl":
            self._comm = get_communicator(None if self.pg is dist.group.WORLD else self.pg, self.device)
        self._dev_index = self.device.index if self.device.index is not None else (
            torch.cuda.current_device() if self.is_cuda else 0)

        if broadcast_params and self.world > 1:
            with torch.no_grad():
                for t in list(self.params) + list(module.buffers()):
                    self._bcast(t.data if t.is_floating_point() else t)

        # buckets in gradient-ready (reverse module) order, <= reduce_bucket_size elements.
        # overlap_allgather (opt-in; DeepSpeed's ZeRO-2 gathers everything at the end of
        # step, R:resnet/deepspeed/deepspeed_train.py:210-216, and stays the default):
        # buckets of <= allgather_bucket_size elements whose parameter all-gathers run on
        # the communicator's stream behind the update, first layers first, each awaited
        # by the first forward of a module holding its parameters (wait_allgather())
        self.overlap_allgather = bool(overlap_allgather)
        if self.overlap_allgather and self.capturable:
            raise NotImplementedError("overlap_allgather: eager steps only (not with capturable)")
        cap = int(reduce_bucket_size)
        if self.overlap_allgather:
            cap = min(cap, int(allgather_bucket_size or 5_000_000))
        n = len(self.params)
        order = list(reversed(range(n)))
        esz = self.params[0].element_size()
        self.buckets = compute_bucket_assignment_by_size(self.params, [cap * esz], order=order)
        self._make_bucketer()
        self._build_flat_state()
        self._bind_marks(True)
        self._hooks = []
        self._in_backward = False
        self._queued = False
        self._pending = {}
        # [found_inf, Σg² (all-reduced), 1/scale, -, clip out: Σg²·s², coefficient, ‖g‖]
        self._scratch = torch.zeros(8, dtype=torch.float32, device=self.device)
        # world > 1 folded clip: this rank's Σg² partial sums, then their SUM over ranks
        self._red_groups = torch.zeros(L.GS_RED_PARTIALS, dtype=torch.float32, device=self.device)
        self._capture_local: dict | None = None  # parity.py: {param index: local grad copy}
        # the per-gradient hook in C++ (_gshook, release mode: the grad is freed once its
        # pack is enqueued) on the library-collective path; Python hooks otherwise
        from .ddp import _make_native_hooks

        self._native = _make_native_hooks(self, self.params, release=True) if self._comm is not None else None
        self._native_on = False
        if self._native is not None:
            self._native_bind()
        self._set_native(self._native_ok())
        self._ag_pending: set = set()
        self._ag_hooks = []
        self._ag_time = None  # (start, end) timing events around the step's all-gathers (time_allgather)
        if self.overlap_allgather:
            self._ag_ev = [torch.cuda.Event() if self.is_cuda else None for _ in self.buckets]
            index = {id(p): i for i, p in enumerate(self.params)}
            for m in module.modules():
                bs = sorted({self.loc[index[id(p)]][0] for p in m.parameters(recurse=False) if id(p) in index})
                if bs:
                    self._ag_hooks.append(m.register_forward_pre_hook(
                        lambda mod, inp, bs=tuple(bs): self._wait_buckets(bs)))

    # ------------------------------------------------------------------ setup
    # Without the library communicator the collectives go through the process
    # group; device tensors over gloo (ranks sharing a GPU: the rehearsal path)
    # are staged through host memory, as the bucket all-reduces are — no
    # collective of gloo's CUDA path runs
    def _host_staged(self, t) -> bool:
        return self._comm is None and t.is_cuda and dist.get_backend(self.pg) == "gloo"

    def _bcast(self, t):
        if self._comm is not None:
            self._comm.broadcast(t, 0, stream=L.stream_ptr(self.device))
        elif self._host_staged(t):
            host = t.cpu()
            dist.broadcast(host, src=dist.get_global_rank(self.pg, 0) if self.pg is not dist.group.WORLD else 0,
                           group=self.pg)
            t.copy_(host)
        else:
            dist.broadcast(t, src=dist.get_global_rank(self.pg, 0) if self.pg is not dist.group.WORLD else 0,
                           group=self.pg)

    def _make_bucketer(self):
        flags = L.GS_BKT_NO_UNPACK
        if self._comm is not None:
            flags |= L.GS_BKT_AUTO_COLLECTIVE
            if self.stage == 2:
                flags |= L.GS_BKT_REDUCE_SCATTER
        kind = L.GS_DEV_HIP if self.is_cuda else L.GS_DEV_HOST
        counts = [len(b) for b in self.buckets]
        members = [i for b in self.buckets for i in b]
        h = ctypes.c_void_p()
        comm = self._comm.handle if self._comm is not None else None
        # host / external-collective buckets are padded like reduce-scatter ones
        L.check(L.lib().gs_bucketer_create(
            comm, kind, self._dev_index, len(self.params), L.i64_array([p.numel() for p in self.params]),
            L.gs_dtype(self.dtype), len(self.buckets), L.i32_array(counts), L.i32_array(members),
            L.gs_dtype(self.dtype), BUCKET_ALIGN_ELEMS, float(self.world), flags, ctypes.byref(h)),
            "gs_bucketer_create")
        self.handle = h
        if self.is_cuda:
            # no tail timing on the ZeRO engine: its end-of-backward chain records no
            # event packets (~4.7 µs of stream time each)
            L.check(L.lib().gs_bucketer_set_timeline(h, 0), "gs_bucketer_set_timeline")
        if self._comm is not None:
            self._comm.add_user(self)
        self._ready = (ctypes.c_int32 * max(1, len(self.buckets)))()
        self._n_ready = ctypes.c_int32()
        q = self.world * BUCKET_ALIGN_ELEMS
        self.bucket_numel, self.grad_bufs, self.grad_shards, self.loc = [], [], [], []
        for b in range(len(self.buckets)):
            nb = ctypes.c_int64()
            L.check(L.lib().gs_bucketer_bucket_numel(h, b, ctypes.byref(nb)), "gs_bucketer_bucket_numel")
            numel = nb.value
            if numel % q:
                raise RuntimeError("internal: bucket not padded to world*align")
            buf = torch.zeros(numel, dtype=self.dtype, device=self.device)
            L.check(L.lib().gs_bucketer_set_bucket_buffer(h, b, buf.data_ptr()), "set_bucket_buffer")
            shard_n = numel // self.world
            if flags & L.GS_BKT_REDUCE_SCATTER:
                shard = torch.zeros(shard_n, dtype=self.dtype, device=self.device)
                L.check(L.lib().gs_bucketer_set_shard_buffer(h, b, shard.data_ptr()), "set_shard_buffer")
            else:
                shard = buf[self.rank * shard_n:(self.rank + 1) * shard_n]
            self.bucket_numel.append(numel)
            self.grad_bufs.append(buf)
            self.grad_shards.append(shard)
        for i in range(len(self.params)):
            bi, off = ctypes.c_int32(), ctypes.c_int64()
            L.check(L.lib().gs_bucketer_param_location(h, i, ctypes.byref(bi), ctypes.byref(off)), "param_location")
            self.loc.append((bi.value, off.value))

    @torch.no_grad()
    def _build_flat_state(self):
        """params become views of per-bucket flat buffers; fp32 master shard + states."""
        self.param_flats = []
        for b, members in enumerate(self.buckets):
            flat = torch.zeros(self.bucket_numel[b], dtype=self.dtype, device=self.device)
            for i in members:
                p = self.params[i]
                _, off = self.loc[i]
                view = flat.as_strided(p.size(), p.stride(), off)
                view.copy_(p.data)
                p.data = view
            self.param_flats.append(flat)
        shard_sizes = [n // self.world for n in self.bucket_numel]
        self.shard_sizes = shard_sizes
        self.param_shards = [f[self.rank * s:(self.rank + 1) * s] for f, s in zip(self.param_flats, shard_sizes)]
        self.lowp = self.dtype != torch.float32
        if self.lowp:
            self.master = [ps.float().clone() for ps in self.param_shards]
        else:
            self.master = self.param_shards  # fp32 model: the shard IS the master copy
        self.state1 = [torch.zeros(s, dtype=torch.float32, device=self.device) for s in shard_sizes]
        self.state2 = [torch.zeros(s, dtype=torch.float32, device=self.device) for s in shard_sizes]
        self.plan = TensorListPlan(shard_sizes, self.device, task_units=update_task_units(self.device))
        self.plan.set_ptrs(0, self.master)
        self.plan.set_ptrs(1, self.grad_shards)
        self.plan.set_ptrs(2, self.state1)
        if self.kind == "sgd":
            self.plan.set_ptrs(3, self.param_shards if self.lowp else [0] * len(shard_sizes))
        else:
            self.plan.set_ptrs(3, self.state2)
            self.plan.set_ptrs(4, self.param_shards if self.lowp else [0] * len(shard_sizes))

    # ---- watchdog marks of the step-end collectives: the reduce-scatters
    # and the clip's / overflow check's all-reduces hand their marks to the update's
    # launch, the parameter all-gathers to the next backward's first pack — no event
    # packet after each (~4.7 µs of stream time apiece on the step's end).
    # mark_packets = True restores the packets (round 5's form, the zero2 leg's A/B).
    def _bind_marks(self, on: bool):
        self.mark_packets = not on
        if self._comm is None or not self.is_cuda:
            self._mark_update = self._mark_next_pack = None
            return
        L.check(L.lib().gs_bucketer_set_mark_consumer(self.handle, self.plan.handle if on else None),
                "gs_bucketer_set_mark_consumer")
        first = ctypes.c_void_p()
        L.check(L.lib().gs_bucketer_first_pack_plan(self.handle, ctypes.byref(first)), "gs_bucketer_first_pack_plan")
        self._mark_update = self.plan.handle if on else None
        self._mark_next_pack = first if on and first.value else None

    def set_mark_packets(self, packets: bool):
        """True: an event packet after every step-end collective (round 5's form);
        False (default): the marks ride on the consuming kernels."""
        self._bind_marks(not packets)

    # ------------------------------------------------------------------ backward
    # ---- which hooks run: C++ (_gshook) on the library-collective path, Python otherwise
    def _native_ok(self) -> bool:
        return self._native is not None and self._capture_local is None

    def _native_bind(self):
        self._native.set_bucketer(self.handle.value, len(self.buckets), [bi for bi, _ in self.loc],
                                  self._comm.stream_ptr)

    def _set_native(self, on: bool):
        if on:
            for h in self._hooks:
                h.remove()
            self._hooks = []
            self._native.attach()
        else:
            if self._native is not None:
                self._native.detach()
            if not self._hooks:
                self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i))
                               for i, p in enumerate(self.params)]
        self._native_on = on

    def _native_finalized(self):
        self._in_backward = False

    def prepare_backward(self):
        """Start a synchronising backward (called by the engine's backward())."""
        want = self._native_ok()
        if want != self._native_on:
            self._set_native(want)
        if not self.require_backward_grad_sync:
            self._in_backward = False
            return
        L.check(L.lib().gs_bucketer_prepare(self.handle, None), "gs_bucketer_prepare")
        self._in_backward = True
        self._queued = False
        self._pending = {}
        self._held = {}
        if self._native_on:
            self._native.prepare(False)

    def _make_hook(self, idx):
        def hook(param):
            if not self._in_backward:
                return
            if not self._queued:
                self._queued = True
                self._stream = L.stream_ptr(self.device)
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            g = param.grad
            if not dense_like_param(g, param):
                dense = torch.empty_like(param)
                dense.copy_(g)
                g = dense
            cap = self._capture_local
            if cap is not None and idx in cap:
                cap[idx] = g.detach().clone()  # on the producer stream, before the pack
            # hold the grad until its bucket's pack is enqueued; param.grad is
            # released now (DeepSpeed frees it too)
            self._held.setdefault(self.loc[idx][0], []).append(g)
            param.grad = None
            L.check(L.lib().gs_bucketer_mark_ready(self.handle, idx, g.data_ptr(), self._stream, self._ready,
                                                   ctypes.byref(self._n_ready)), "gs_bucketer_mark_ready")
            for k in range(self._n_ready.value):
                b = self._ready[k]
                if self._comm is None and self.grad_bufs[b].is_cuda:
                    # device buckets over gloo (the rehearsal path): staged through host
                    # memory, as DDP does (gloo's async CUDA path deadlocks from the
                    # autograd thread at 4 ranks on one GPU)
                    host = self.grad_bufs[b].to("cpu")
                    self._pending[b] = (host, dist.all_reduce(host, group=self.pg, async_op=True))
                elif self._comm is None:
                    self._pending[b] = (None, dist.all_reduce(self.grad_bufs[b], group=self.pg, async_op=True))
                for held in self._held.pop(b, []):
                    if self._comm is not None:
                        # the pack on the comm stream is enqueued: the allocator may
                        # reuse this memory only after it has run
                        held.record_stream(self._comm.stream)

        return hook

    def _finalize(self):
        for b in sorted(self._pending):
            host, work = self._pending[b]
            work.wait()
            if host is not None:
                self.grad_bufs[b].copy_(host)
        self._pending = {}
        L.check(L.lib().gs_bucketer_finalize(self.handle, self._stream), "gs_bucketer_finalize")
        self._in_backward = False

    # ------------------------------------------------------------------ step
    def _allreduce_scalar(self, t, op, consumer=None):
        if self._comm is not None:
            self._comm.all_reduce(t, op=op, stream=L.stream_ptr(self.device), consumer=consumer)
            return
        rop = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
        if self._host_staged(t):
            host = t.cpu()
            dist.all_reduce(host, op=rop, group=self.pg)
            t.copy_(host)
        else:
            dist.all_reduce(t, op=rop, group=self.pg)

    # ---- overlapped parameter all-gather (opt-in, overlap_allgather)
    def _launch_allgathers(self):
        """Each bucket's in-place all-gather behind the update, last bucket (the
        model's first layers, needed first by the next forward) first; on the
        communicator's stream when there is one, so the next forward's early layers
        run while the later buckets travel."""
        order = list(reversed(range(len(self.param_flats))))
        if self._comm is not None:
            cs = self._comm.stream
            cs.wait_stream(torch.cuda.current_stream(self.device))  # the update wrote this rank's slices
            for b in order:
                flat = self.param_flats[b]
                shard = flat[self.rank * self.shard_sizes[b]:(self.rank + 1) * self.shard_sizes[b]]
                self._comm.all_gather(shard, flat, stream=self._comm.stream_ptr, consumer=self._mark_next_pack)
                self._ag_ev[b].record(cs)
        else:
            for b in order:  # the process group: synchronous, the events mark the same points
                self._all_gather_flat(b, self.param_flats[b])
                if self._ag_ev[b] is not None:
                    self._ag_ev[b].record()
        self._ag_pending = set(order)

    def _wait_buckets(self, buckets):
        if not self._ag_pending:
            return
        for b in buckets:
            if b in self._ag_pending:
                self._ag_pending.discard(b)
                if self._ag_ev[b] is not None:
                    torch.cuda.current_stream(self.device).wait_event(self._ag_ev[b])

    def wait_allgather(self):
        """Order the current stream after every pending parameter all-gather
        (overlap_allgather): what a module's forward pre-hook does for its own
        parameters; call it before reading parameters outside a forward."""
        self._wait_buckets(sorted(self._ag_pending))

    def time_allgather(self, on: bool = True):
        """HIP events around the end-of-step all-gathers on the step's stream
        (the exposed all-gather: all of it by default, the issue cost with
        overlap_allgather); :meth:`last_allgather_ms` reads the last step's."""
        self._ag_time = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) \
            if on and self.is_cuda else None

    def last_allgather_ms(self):
        t = self._ag_time
        if t is None:
            return None
        t[1].synchronize()
        return t[0].elapsed_time(t[1])

    @torch.no_grad()
    def step(self):
        self.wait_allgather()  # the update writes this rank's slice of the parameter buffers
        s = self._scratch
        found_inf = None
        grad_scale = None
        inv_scale = 1.0
        if self.scaler is not None:
            inv_scale = 1.0 / self.scaler.scale
            found_inf = s[0:1]
            found_inf.zero_()
            self.plan.unscale_check(1, self.dtype, None, found_inf)
            self._allreduce_scalar(found_inf, "max", consumer=self._mark_update)
        if self.clip > 0 and _optim.CLIP_FUSED:
            # DeepSpeed gradient_clipping (R:resnet/deepspeed/deepspeed_train.py:195) folded
            # into the update: its workgroups form min(1, c/(‖g‖+1e-6))·(1/scale) themselves
            # (gs_plan_set_clip) — no combine launch, no coefficient launch
            if self.world == 1:
                # Σg² stays as the plan's partial sums
                self.plan.sqnorm_partial(1, self.dtype)
                self.plan.set_clip(self.clip, 1e-6, None, inv_scale * inv_scale, inv_scale, out=s[4:7])
            else:
                # this shard's Σg² partial sums (a small shard, e.g. ResNet-50 at N=8: one per
                # workgroup of a <= 1024-workgroup grid, no in-kernel combine) SUM-all-reduced
                # over the ranks (one message, identical bits everywhere), folded by every
                # update workgroup: Σg² kernel -> collective -> update, nothing in between
                # (DeepSpeed: per-rank Σ, scalar all_reduce, coefficient, U).  The message
                # length never depends on a rank's own chunk map or reduction settings
                # (ADVICE r4): slots past a rank's count stay zero and add nothing
                gr = self._red_groups
                self.plan.sqnorm_partial_out(1, self.dtype, gr)
                # the whole buffer travels and is folded: a rank's partial count follows
                # its shard's chunk map (tensor pieces split at shard edges differ from
                # rank to rank), so no count-dependent length is safe to send
                self._allreduce_scalar(gr, "sum", consumer=self._mark_update)
                self.plan.set_clip_groups(self.clip, 1e-6, gr, gr.numel(), inv_scale * inv_scale, inv_scale,
                                          out=s[4:7])
        elif self.clip > 0:
            self.plan.set_clip(None)
            sq = s[1:2]
            self.plan.sqnorm(1, self.dtype, sq)
            self._allreduce_scalar(sq, "sum")
            if inv_scale != 1.0:
                sq.mul_(inv_scale * inv_scale)
            clip_coef(sq, self.clip, 1e-6, s[5:6], s[6:7])
            grad_scale = s[5:6]
            if inv_scale != 1.0:
                grad_scale.mul_(inv_scale)
        elif inv_scale != 1.0:
            grad_scale = s[2:3]
            grad_scale.fill_(inv_scale)
        g0 = self.param_groups[0]
        lowp = self.dtype if self.lowp else None
        self.step_count += 1
        if self.kind == "sgd":
            self.plan.sgd(self.dtype, g0["lr"], g0["momentum"], 0.0, g0["weight_decay"], False, False,
                          self.step_count == 1, lowp_dtype=lowp, grad_scale=grad_scale, found_inf=found_inf)
        elif self.capturable:
            # device hyper-parameters: advance the step, form [step_size, bc2_sqrt, 1 - lr*wd]
            # (the same double arithmetic as the host branch, T:optim/adam.py), the kernel reads them
            b1, b2 = g0["betas"]
            h = self._hyper_state()
            L.check(L.lib().gs_adam_hyper(L.GS_DEV_HIP if self.is_cuda else L.GS_DEV_HOST, h["step"].data_ptr(),
                                          h["lr"].data_ptr(), float(b1), float(b2), float(g0["weight_decay"]), None,
                                          h["hyper"].data_ptr(), L.stream_ptr(self.device) if self.is_cuda else None),
                    "gs_adam_hyper")
            self.plan.adam(self.dtype, g0["lr"], b1, b2, g0["eps"], g0["weight_decay"], self.kind == "adamw", False,
                           -1.0, 1.0, lowp_dtype=lowp, grad_scale=grad_scale, found_inf=found_inf)
        else:
            b1, b2 = g0["betas"]
            bc1 = 1 - b1 ** self.step_count
            bc2 = 1 - b2 ** self.step_count
            self.plan.adam(self.dtype, g0["lr"], b1, b2, g0["eps"], g0["weight_decay"], self.kind == "adamw", False,
                           (g0["lr"] / bc1) * -1, bc2 ** 0.5, lowp_dtype=lowp, grad_scale=grad_scale,
                           found_inf=found_inf)
        # re-replicate the updated parameters: in-place all-gather per bucket
        t = self._ag_time
        if t is not None:
            t[0].record()
        if self.overlap_allgather:
            self._launch_allgathers()
        else:
            for b, flat in enumerate(self.param_flats):
                self._all_gather_flat(b, flat, consumer=self._mark_next_pack)
        if t is not None:
            t[1].record()
        overflow = False
        if self.scaler is not None:
            overflow = bool(found_inf.item() != 0)  # DeepSpeed reads the overflow flag on the host
            if overflow:
                self.step_count -= 1
            self.scaler.update(overflow)
        return not overflow

    def _hyper_state(self):
        """Device step counter (fp64), lr (fp64) and the kernel's hyper source
        (fp32 [step_size, bc2_sqrt, 1 - lr*wd]) of the capturable mode."""
        h = getattr(self, "_dev_hyper", None)
        if h is None:
            h = self._dev_hyper = {
                "step": torch.full((1,), float(self.step_count - 1), dtype=torch.float64, device=self.device),
                "lr": torch.full((1,), float(self.param_groups[0]["lr"]), dtype=torch.float64, device=self.device),
                "hyper": torch.zeros(3, dtype=torch.float32, device=self.device), "lr_host": self.param_groups[0]["lr"]}
            self.plan.set_hyper_source(h["hyper"])
        return h

    def refresh_hyper(self):
        """Write a changed host lr (a WarmupLR step) into the device buffer —
        outside a capture; CapturedStep calls it before every replay."""
        h = getattr(self, "_dev_hyper", None)
        lr = self.param_groups[0]["lr"]
        if h is not None and h["lr_host"] != lr:
            h["lr"].fill_(float(lr))
            h["lr_host"] = lr

    def device_step_count(self) -> int:
        """The step count (capturable: read from the device counter, which graph
        replays advance; a host read)."""
        h = getattr(self, "_dev_hyper", None)
        return int(h["step"].item()) if h is not None else self.step_count

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def grad_norm(self):
        """‖g‖ of the unscaled averaged grads at the last clipped step (device tensor)."""
        return self._scratch[6:7]

    def state_dict(self):
        """This rank's optimizer shard (fp32 master + states): DeepSpeed's
        zero_pp_rank_<r>_mp_rank_00_optim_states layout, one file per rank."""
        return {"step": self.device_step_count(), "rank": self.rank, "world": self.world, "stage": self.stage,
                "bucket_numel": list(self.bucket_numel), "kind": self.kind,
                "master": [m.detach().float().cpu().clone() for m in self.master],
                "exp_avg": [t.cpu() for t in self.state1], "exp_avg_sq": [t.cpu() for t in self.state2],
                "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups],
                "loss_scaler": None if self.scaler is None else self.scaler.state_dict()}

    @torch.no_grad()
    def load_state_dict(self, sd):
        """Restore this rank's shard (same world size and bucket layout)."""
        self.wait_allgather()
        if sd["world"] != self.world or sd["rank"] != self.rank or list(sd["bucket_numel"]) != self.bucket_numel:
            raise RuntimeError(f"ZeRO checkpoint shard is for rank {sd['rank']}/{sd['world']} with buckets "
                               f"{sd['bucket_numel']}; this engine is rank {self.rank}/{self.world} with "
                               f"{self.bucket_numel}")
        self.step_count = int(sd["step"])
        self._dev_hyper = None  # re-derived from the loaded step count on the next step
        for m, v in zip(self.master, sd["master"]):
            m.copy_(v.to(m.device, m.dtype))
        for t, v in zip(self.state1, sd["exp_avg"]):
            t.copy_(v.to(t.device))
        for t, v in zip(self.state2, sd["exp_avg_sq"]):
            t.copy_(v.to(t.device))
        for g, saved in zip(self.param_groups, sd["param_groups"]):
            g.update({k: v for k, v in saved.items() if k in g})
        if self.scaler is not None and sd.get("loss_scaler") is not None:
            self.scaler.load_state_dict(sd["loss_scaler"])
        if self.lowp:  # the model copy follows the master
            for shard, m in zip(self.param_shards, self.master):
                shard.copy_(m.to(shard.dtype))
        # every rank's parameters from the loaded shards (fp32: the master IS this rank's
        # slice of the flats, the other slices come from the gather, not from whatever the
        # module held — a module load_state_dict may have run before this)
        for b, flat in enumerate(self.param_flats):
            self._all_gather_flat(b, flat)

    def _all_gather_flat(self, b, flat, consumer=None):
        shard = flat[self.rank * self.shard_sizes[b]:(self.rank + 1) * self.shard_sizes[b]]
        if self._comm is not None:
            self._comm.all_gather(shard, flat, stream=L.stream_ptr(self.device), consumer=consumer)
        elif self._host_staged(flat):
            host = torch.empty(flat.numel(), dtype=flat.dtype)
            dist.all_gather(list(host.chunk(self.world)), shard.cpu(), group=self.pg)
            flat.copy_(host)
        else:
            chunks = list(flat.chunk(self.world))
            dist.all_gather(chunks, shard.clone(), group=self.pg)

    @torch.no_grad()
    def consolidated_state_dict(self) -> dict:
        """The full model ``state_dict`` (torchvision keys, module order) with the
        fp32 master values for the parameters, gathered from every rank's shard
        (DeepSpeed ``zero_to_fp32`` / ``get_fp32_state_dict_from_zero_checkpoint``;
        Colossal ``save_model(shard=False)``).  Collective: every rank calls it
        and every rank gets it.  Buffers are this rank's."""
        self.wait_allgather()
        fulls = []
        for b, m in enumerate(self.master):
            full = torch.empty(self.bucket_numel[b], dtype=torch.float32, device=self.device)
            if self._comm is not None:
                self._comm.all_gather(m.contiguous(), full, stream=L.stream_ptr(self.device))
            elif self._host_staged(full):
                host = torch.empty(full.numel(), dtype=full.dtype)
                dist.all_gather(list(host.chunk(self.world)), m.contiguous().cpu(), group=self.pg)
                full.copy_(host)
            else:
                dist.all_gather(list(full.chunk(self.world)), m.contiguous(), group=self.pg)
            fulls.append(full)
        by_id = {}
        for i, p in enumerate(self.params):
            b, off = self.loc[i]
            by_id[id(p)] = fulls[b].as_strided(p.size(), p.stride(), off)
        out = {}
        names = {id(p): n for n, p in self.module.named_parameters()}
        pn = {names[id(p)]: id(p) for p in self.params}
        for k, v in self.module.state_dict().items():
            out[k] = by_id[pn[k]].detach().cpu().clone() if k in pn else v.detach().cpu().clone()
        return out

    @torch.no_grad()
    def load_consolidated_state_dict(self, sd: dict):
        """Inverse of :meth:`consolidated_state_dict`: fp32 values into the master
        shards and the (low-precision) model, buffers into the module.  No
        collective: every rank reads the full dict."""
        self.wait_allgather()
        names = {id(p): n for n, p in self.module.named_parameters()}
        fulls = [torch.zeros(n, dtype=torch.float32, device=self.device) for n in self.bucket_numel]
        for i, p in enumerate(self.params):
            b, off = self.loc[i]
            fulls[b].as_strided(p.size(), p.stride(), off).copy_(sd[names[id(p)]].to(self.device, torch.float32))
        for b, full in enumerate(fulls):
            s = self.shard_sizes[b]
            if self.lowp:
                self.master[b].copy_(full[self.rank * s:(self.rank + 1) * s])
            self.param_flats[b].copy_(full.to(self.dtype))
        param_keys = {names[id(p)] for p in self.params}
        bufs = {k: v for k, v in sd.items() if k not in param_keys}
        missing, unexpected = self.module.load_state_dict(bufs, strict=False)
        if unexpected or set(missing) - param_keys:
            raise RuntimeError(f"state_dict mismatch: missing {sorted(set(missing) - param_keys)}, "
                               f"unexpected {unexpected}")

    def close(self):
        self.wait_allgather()
        if getattr(self, "handle", None) is not None and self.handle.value and self._comm is not None:
            self._bind_marks(False)  # no mark left on the update plan's or the pack plan's next launch
        for h in self._hooks + getattr(self, "_ag_hooks", []):
            h.remove()
        self._hooks = []
        self._ag_hooks = []
        nat = getattr(self, "_native", None)
        if nat is not None:
            nat.detach()
            nat.set_bucketer(0, 0)
            self._native_on = False
        if getattr(self, "handle", None) is not None and self.handle.value:
            L.destroy("gs_bucketer_destroy", self.handle)
            self.handle = None


def warmup_lr(step: int, min_lr: float, max_lr: float, warmup_num_steps: int, warmup_type: str = "log") -> float:
    """DeepSpeed WarmupLR (R:resnet/deepspeed/deepspeed_train.py:187-194): log (default) or linear
    ramp from warmup_min_lr to warmup_max_lr over warmup_num_steps, then constant."""
    if step < warmup_num_steps:
        if warmup_type == "log":
            gamma = math.log(step + 1) / math.log(warmup_num_steps) if warmup_num_steps > 1 else 1.0
        else:
            gamma = step / warmup_num_steps
    else:
        gamma = 1.0
    return min_lr + (max_lr - min_lr) * gamma
