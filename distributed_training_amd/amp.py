"""Mixed-precision loss scaling on libgsync kernels.

``GradScaler`` keeps torch.amp.GradScaler's API and semantics
(T:amp/grad_scaler.py: scale / unscale_ / step / update; init 2**16,
growth 2.0 every 2000 clean steps, backoff 0.5) but replaces
``_amp_foreach_non_finite_check_and_unscale_`` (:280) with one libgsync
multi-tensor pass, and for libgsync fused optimizers folds the 1/scale into
the update kernel and skips the step ON THE DEVICE when a non-finite grad was
found: SGD's first-step flag and Adam's step counter live on the device and
advance only on a clean step, so a scale/backward/step/update iteration does
no host synchronisation (tests/test_gpu_amp_nosync.py).  Foreign optimizers
keep torch's host read of the flag (T:amp/grad_scaler.py _maybe_opt_step).  Reached from the Colossal
``torch_ddp_fp16`` plugin (R:resnet/colossal/colossal_train.py:129-130).
"""
from __future__ import annotations

import torch
from torch.autograd.graph import increment_version

from .multi_tensor import TensorListPlan


class GradScaler:
    def __init__(self, device="cuda", init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5,
                 growth_interval=2000, enabled=True):
        self._device = torch.device(device) if not isinstance(device, torch.device) else device
        self._init_scale = init_scale
        self._growth_factor = growth_factor
        self._backoff_factor = backoff_factor
        self._growth_interval = growth_interval
        self._enabled = enabled
        self._scale = None
        self._growth_tracker = None
        self._per_opt = {}
        self._plans = {}
        self._ddp = None
        self._ddp_found = None
        self.fused_checks = 0  # steps whose inf check came from the DDP unpack (no extra pass)

    def is_enabled(self):
        return self._enabled

    def fuse_check_into(self, ddp):
        """Let ``ddp`` (libgsync DistributedDataParallel) compute the non-finite
        check of the averaged grads inside its bucket unpack (SURVEY.md §8f-2:
        "fuse it into pack/unpack"): for a libgsync fused optimizer over exactly
        the DDP parameters, step() then skips its own check pass."""
        self._ddp = ddp
        dev = next(iter(ddp.parameters())).device
        self._ddp_found = torch.zeros(1, dtype=torch.float32, device=dev)
        ddp.set_found_inf_target(self._ddp_found)
        self._ddp_param_ids = frozenset(id(p) for p in ddp._params)

    def _ddp_flag_for(self, optimizer):
        d = self._ddp
        if d is None or not d._found_inf_valid:
            return None
        ids = frozenset(id(p) for g in optimizer.param_groups for p in g["params"] if p.grad is not None)
        return self._ddp_found if ids == self._ddp_param_ids else None

    def _lazy_init(self, dev):
        if self._scale is None:
            self._scale = torch.full((1,), self._init_scale, dtype=torch.float32, device=dev)
            self._growth_tracker = torch.zeros((1,), dtype=torch.int32, device=dev)

    def scale(self, outputs):
        if not self._enabled:
            return outputs
        self._lazy_init(outputs.device)
        # as torch: the 0-dim fp32 scale multiplies without a cast (an fp16 loss
        # is promoted to fp32 — the default 2**16 does not fit fp16 — and keeps its shape)
        return outputs * self._scale.view(()).to(device=outputs.device, non_blocking=True)

    def get_scale(self):
        return self._init_scale if self._scale is None else float(self._scale.item())

    def _state(self, optimizer):
        st = self._per_opt.get(id(optimizer))
        if st is None:
            dev = self._scale.device
            st = {"found_inf": torch.zeros(1, dtype=torch.float32, device=dev),
                  "inv_scale": torch.ones(1, dtype=torch.float32, device=dev), "stage": "ready"}
            self._per_opt[id(optimizer)] = st
        return st

    def _grads(self, optimizer):
        by_dtype = {}
        for group in optimizer.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    by_dtype.setdefault(p.grad.dtype, []).append(p.grad)
        return by_dtype

    def _check(self, optimizer, unscale: bool):
        st = self._state(optimizer)
        st["inv_scale"].copy_(self._scale.reciprocal())
        st["found_inf"].zero_()
        for dt, grads in self._grads(optimizer).items():
            # a plan depends only on the sizes and the device (grads are
            # short-lived: ids are reused after zero_grad(set_to_none))
            key = (id(optimizer), dt, grads[0].device, tuple(g.numel() for g in grads))
            plan = self._plans.get(key)
            if plan is None:
                plan = TensorListPlan([g.numel() for g in grads], grads[0].device)
                self._plans = {k: v for k, v in self._plans.items() if k[0] != id(optimizer) or k[1] != dt}
                self._plans[key] = plan
            plan.set_ptrs(0, grads)
            plan.unscale_check(0, dt, st["inv_scale"] if unscale else None, st["found_inf"])
            if unscale:
                # grads multiplied in place by the kernel: bump their version counters
                # as torch's in-place unscale does (a DDP's fused Σg² of them is stale)
                increment_version(grads)
        return st

    def unscale_(self, optimizer):
        if not self._enabled:
            return
        st = self._state(optimizer)
        if st["stage"] == "unscaled":
            raise RuntimeError("unscale_() has already been called on this optimizer since the last update().")
        self._check(optimizer, unscale=True)
        st["stage"] = "unscaled"

    def step(self, optimizer, *args, **kwargs):
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        st = self._state(optimizer)
        fused = hasattr(optimizer, "found_inf") and hasattr(optimizer, "grad_scale")
        if st["stage"] != "unscaled":
            if fused:
                flag = self._ddp_flag_for(optimizer)
                if flag is not None:  # the check already ran inside DDP's unpack
                    st["inv_scale"].copy_(self._scale.reciprocal())
                    st["found_inf"].copy_(flag)
                    self._ddp._found_inf_valid = False
                    self.fused_checks += 1
                else:
                    self._check(optimizer, unscale=False)  # check only; 1/scale folded into the update
                optimizer.grad_scale = st["inv_scale"]
            else:
                self._check(optimizer, unscale=True)
        elif fused:
            optimizer.grad_scale = None
        if fused:
            optimizer.found_inf = st["found_inf"]  # the kernel skips the step on the device
            try:
                ret = optimizer.step(*args, **kwargs)
            finally:
                optimizer.found_inf = None
                optimizer.grad_scale = None
        else:
            ret = None if st["found_inf"].item() != 0 else optimizer.step(*args, **kwargs)
        st["stage"] = "stepped"
        return ret

    def update(self, new_scale=None):
        if not self._enabled or self._scale is None:
            return
        if new_scale is not None:
            self._scale.fill_(float(new_scale))
        else:
            found = torch.zeros_like(self._scale)
            for st in self._per_opt.values():
                found = torch.maximum(found, st["found_inf"])
            # torch._amp_update_scale_ semantics, on the device
            bad = found > 0
            tracker = torch.where(bad, torch.zeros_like(self._growth_tracker), self._growth_tracker + 1)
            grow = tracker >= self._growth_interval
            self._scale.copy_(torch.where(bad, self._scale * self._backoff_factor,
                                          torch.where(grow, self._scale * self._growth_factor, self._scale)))
            self._growth_tracker.copy_(torch.where(grow, torch.zeros_like(tracker), tracker))
        for st in self._per_opt.values():
            st["stage"] = "ready"

    def state_dict(self):
        return {"scale": self.get_scale(), "growth_factor": self._growth_factor,
                "backoff_factor": self._backoff_factor, "growth_interval": self._growth_interval,
                "_growth_tracker": 0 if self._growth_tracker is None else int(self._growth_tracker.item())}

    def load_state_dict(self, sd):
        self._init_scale = sd["scale"]
        if self._scale is not None:
            self._scale.fill_(sd["scale"])
            self._growth_tracker.fill_(sd.get("_growth_tracker", 0))
