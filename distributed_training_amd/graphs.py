"""Whole training step as one hipGraph ("hipGraph capture").

The reference's step — forward, backward with DDP's bucketed all-reduce, the
optimizer update (R:resnet/pytorch_ddp/ddp_train.py:104-111) — is a few
hundred small kernel launches per iteration; at the reference's own CIFAR
shape (ResNet-18, batch 100 per GPU) the GPU finishes them faster than Python
and the HIP runtime can enqueue them.  :class:`CapturedStep` records the step
once (torch.cuda.graph over libgsync's capture-safe plans, bucketer and RCCL
collectives) and replays it: one launch per iteration.

    step = CapturedStep(lambda x, y: train_step(x, y), optimizers=[opt])
    for x, y in loader:
        loss = step(x, y)          # a real training step on every call

Every call performs exactly one training step: the first ``warmup`` calls run
eagerly on a side stream (DDP bucket rebuild, optimizer state creation, lazy
init), the next call records the graph and replays it once, later calls copy
their inputs into the recorded input buffers and replay.  The recorded
outputs are returned (overwritten by the next call: clone what you keep).

What stays correct across replays:
* LR schedules and Adam's bias corrections — the optimizers must be
  ``capturable=True`` (libgsync FusedSGD / FusedAdam): their step-varying
  hyper-parameters are read from device memory, refreshed here before each
  replay (``refresh_hyper``);
* AMP: libgsync ``GradScaler`` keeps scale, growth tracker and skip flag on
  the device;
* any other host-side change to a hyper-parameter (momentum, betas, weight
  decay, eps, a param group added): the step runs eagerly once and the graph
  is recorded again on the next call.

Requirements are torch.cuda.graph's: static shapes (the same batch size on
every call — a ragged last batch runs eagerly), no host synchronisation inside
the step (``loss.item()`` belongs outside), and a ``zero_grad`` inside the
step so that recorded grads are reused: `zero_grad(set_to_none=True)` at the
start of the step is the cheap form (the recorded backward then writes fresh
grads in the graph pool; `set_to_none=False` records a fill + an accumulate
per parameter).
DDP with ``find_unused_parameters=True`` or a comm hook that waits on the host
is not capturable.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch

from . import _lib as L
from .optim import _FusedBase


def _hyper_key(optimizers):
    """Everything a recorded step bakes in (libgsync optimizers: all but lr,
    which they read from device memory)."""
    key = []
    for opt in optimizers:
        # libgsync optimizers and the capturable ZeRO engine read lr from device memory
        skip = ("params", "lr") if (isinstance(opt, _FusedBase) or hasattr(opt, "refresh_hyper")) else ("params",)
        for g in opt.param_groups:
            key.append(tuple(sorted((k, repr(v)) for k, v in g.items() if k not in skip)))
            key.append(tuple(id(p) for p in g["params"]))
    return tuple(key)


class CapturedStep:
    def __init__(self, step_fn: Callable, optimizers: Sequence[torch.optim.Optimizer] = (), warmup: int = 3,
                 pool=None):
        for opt in optimizers:
            if (isinstance(opt, _FusedBase) or hasattr(opt, "refresh_hyper")) and not getattr(opt, "capturable", True):
                raise ValueError(f"{type(opt).__name__} must be created with capturable=True to be recorded")
        self.step_fn = step_fn
        self.optimizers = list(optimizers)
        self.warmup = int(warmup)
        self.pool = pool
        self.graph: torch.cuda.CUDAGraph | None = None
        self.calls = 0
        self.captures = 0
        self.replays = 0
        self._inputs: list | None = None
        self._out = None
        self._key = None
        self._prev_key = None
        self._side = None

    # ------------------------------------------------------------------ helpers
    def _refresh(self):
        for opt in self.optimizers:
            if isinstance(opt, _FusedBase) or hasattr(opt, "refresh_hyper"):
                opt.refresh_hyper()

    def _signature(self, args):
        return tuple((a.shape, a.dtype, a.device) if isinstance(a, torch.Tensor) else ("py", repr(a))
                     for a in args)

    def _eager(self, args):
        self._refresh()
        if self._side is None:
            self._side = torch.cuda.Stream()
        self._side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self._side):
            out = self.step_fn(*args)
        torch.cuda.current_stream().wait_stream(self._side)
        return out

    def _capture(self, args):
        self.graph = None
        self._inputs = [a.clone() if isinstance(a, torch.Tensor) else a for a in args]
        self._sig = self._signature(args)
        self._refresh()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        L.check(L.lib().gs_watchdog_pause(1), "gs_watchdog_pause")
        try:
            with torch.cuda.graph(g, pool=self.pool):
                self._out = self.step_fn(*self._inputs)
        finally:
            L.check(L.lib().gs_watchdog_pause(0), "gs_watchdog_pause")
            L.flush_deferred()  # destroys the garbage collector requested mid-recording
        self.graph = g
        self.captures += 1

    # ------------------------------------------------------------------ call
    def __call__(self, *args):
        self.calls += 1
        key = _hyper_key(self.optimizers)
        stable = key == self._prev_key
        self._prev_key = key
        if self.calls <= self.warmup or (self.graph is None and not stable):
            return self._eager(args)
        if self.graph is not None and (key != self._key or self._signature(args) != self._sig):
            if self._signature(args) != self._sig:  # e.g. a ragged last batch: this call only
                return self._eager(args)
            self.graph = None  # a baked-in hyper-parameter changed: record again once stable
            return self._eager(args)
        if self.graph is None:
            self._capture(args)
            self._key = key
        else:
            for dst, src in zip(self._inputs, args):
                if isinstance(dst, torch.Tensor):
                    dst.copy_(src, non_blocking=True)
            self._refresh()
        self.graph.replay()
        self.replays += 1
        return self._out
