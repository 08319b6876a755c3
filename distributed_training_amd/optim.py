"""Fused multi-tensor optimizers on libgsync kernels (drop-ins for torch.optim).

* :class:`FusedSGD`  — ``torch.optim.SGD`` semantics (T:optim/sgd.py:322-381
  ``_single_tensor_sgd``; :383-470 ``_multi_tensor_sgd``): one HIP pass over
  (param, grad, momentum_buffer) = 20 B/param fp32 instead of >=3 foreach passes.
* :class:`FusedAdam` — ``torch.optim.Adam`` / ``AdamW`` semantics
  (T:optim/adam.py:554-800 ``_multi_tensor_adam``, the reference's default on
  GPU, ``R:resnet/pytorch_ddp/ddp_train.py:97``): one pass over
  (p, g, m, v) = 28 B/param instead of the ~72 B/param of 7 foreach passes.
* :func:`clip_grad_norm_` — ``torch.nn.utils.clip_grad_norm_``
  (T:nn/utils/clip_grad.py:50-186) with a wave-level Σg² reduction and the
  clip coefficient kept on the device (no host sync).

``state_dict`` layouts are torch's (``momentum_buffer``; ``step`` /
``exp_avg`` / ``exp_avg_sq``), so checkpoints move between the two.

Extras used by the engine: ``grad_scale`` (a 1-element device tensor the
update multiplies grads by — clip coefficient or AMP 1/scale), ``found_inf``
(skip the step when non-zero) and ``max_grad_norm`` (DeepSpeed-style
``gradient_clipping``: Σg² + coefficient computed on device, folded into the
update kernel).

``capturable=True`` (torch's Adam flag, also offered on SGD) makes ``step()``
safe to record into a hipGraph (see :mod:`.graphs`): the step-varying
hyper-parameters live in a small device buffer the update kernel reads when it
runs (``gs_plan_set_hyper_source``) — SGD's lr; Adam's step_size, sqrt(bc2)
and 1-lr·wd, produced on the device from a device step counter that does not
advance on an AMP overflow (``gs_adam_hyper``, T:optim/adam.py capturable
branch).  :meth:`refresh_hyper` copies a changed ``group["lr"]`` into that
buffer outside the graph, so LR schedulers keep working across replays.
"""
from __future__ import annotations

import math
import os
from typing import Iterable

import torch
from torch.autograd.graph import increment_version

from . import _lib as L
from .multi_tensor import TensorListPlan, clip_coef, is_dense, update_task_units


# the gradient-norm clip folded into the update kernels (gs_plan_set_clip);
# GSYNC_CLIP_FUSED=0 keeps the separate Σg² / coefficient launches (A/B runs)
CLIP_FUSED = os.environ.get("GSYNC_CLIP_FUSED", "1") not in ("", "0")


def _capturing() -> bool:
    """Is torch's current stream recording a graph (False without a GPU)?"""
    return torch.cuda.is_initialized() and torch.cuda.is_current_stream_capturing()


class _PlanCache:
    """One TensorListPlan per (param list, grad dtype) signature."""

    def __init__(self):
        self._plans: dict = {}
        self.timer_slots = 0

    def get(self, params):
        key = tuple(id(p) for p in params) + (params[0].device,)
        plan = self._plans.get(key)
        if plan is None:
            plan = TensorListPlan([p.numel() for p in params], params[0].device,
                                  task_units=update_task_units(params[0].device))
            if self.timer_slots and plan.kind == L.GS_DEV_HIP:
                plan.timer_enable(self.timer_slots)
            self._plans[key] = plan
        return plan

    def plans(self):
        return list(self._plans.values())


def _check_dense(p: torch.Tensor, g: torch.Tensor, what: str, seen: dict | None = None):
    """p dense and g in p's layout.  ``seen`` (id(p) -> strides found dense)
    skips the walk over the dims for a parameter already checked — a grad with
    the same strides (and shape) is then dense too."""
    ps = p.stride()
    if g.stride() != ps:
        raise RuntimeError(f"{what}: grad layout must match its parameter's (param {ps}, grad {g.stride()})")
    if seen is not None and seen.get(id(p)) == ps:
        return
    if not is_dense(p):
        raise RuntimeError(f"{what}: parameters must be dense (got strides {ps})")
    if seen is not None:
        seen[id(p)] = ps


class _FusedBase(torch.optim.Optimizer):
    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._plans = _PlanCache()
        self.grad_scale: torch.Tensor | None = None
        self.found_inf: torch.Tensor | None = None
        self._clip_buf: dict = {}
        self._norm_ddp = None  # fuse_grad_norm_into: (ddp, its parameter ids)
        self._dev_hyper: dict = {}  # param-group index -> device hyper-parameter buffers
        self._dense_seen: dict = {}  # id(param) -> strides already checked dense

    @property
    def capturable(self) -> bool:
        return bool(self.defaults.get("capturable"))

    def _group_hyper(self, gi, group, device):
        """Device buffers of group `gi` (capturable mode): ``hyper`` fp32[3]
        read by the update kernel, ``lr`` fp64[1] (Adam's hyper producer)."""
        h = self._dev_hyper.get(gi)
        if h is None or h["hyper"].device != device:
            if _capturing():
                raise RuntimeError("capturable optimizer: take one step outside the graph before capturing it")
            h = {"hyper": torch.zeros(3, dtype=torch.float32, device=device),
                 "lr": torch.zeros(1, dtype=torch.float64, device=device), "lr_host": None}
            self._dev_hyper[gi] = h
        return h

    def refresh_hyper(self):
        """Write each group's host ``lr`` into its device buffer when it changed
        (an eager fill, never recorded: call it outside a capture, before a
        replay — graphs.CapturedStep does)."""
        if _capturing():
            return
        for gi, group in enumerate(self.param_groups):
            h = self._dev_hyper.get(gi)
            if h is not None and h["lr_host"] != group["lr"]:
                lr = float(group["lr"])
                h["lr"].fill_(lr)
                h["hyper"][0:1].fill_(lr)  # SGD reads hyper[0] = fp32(lr); Adam overwrites it
                h["lr_host"] = group["lr"]

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dev_hyper = {}  # device step counters are re-derived from the loaded state

    def enable_kernel_timer(self, n_slots: int = 256):
        """Time every update-kernel launch with HIP events recorded on its
        launch stream right around the kernel (bench.py's roofline)."""
        self._plans.timer_slots = int(n_slots)
        for plan in self._plans.plans():
            if plan.kind == L.GS_DEV_HIP:
                plan.timer_enable(n_slots)

    def kernel_ms(self) -> list:
        """Update-kernel durations (ms) since the last call, all plans (the
        Σg² launches of max_grad_norm are left out)."""
        kind = L.GS_OP_ADAM if isinstance(self, FusedAdam) else L.GS_OP_SGD
        return [ms for plan in self._plans.plans() if plan.kind == L.GS_DEV_HIP
                for ms in plan.timer_read(kind=kind)]

    def _device_state(self) -> bool:
        """Step-varying state on the device: capturable mode, the AMP path
        (``found_inf`` set: torch skips ``optimizer.step()`` entirely on an
        overflow, T:amp/grad_scaler.py ``_maybe_opt_step`` — here the kernels
        skip on the device and SGD's first-step flag / Adam's step counter
        advance only on a clean step, so nothing is read on the host), or once
        a group already keeps its counters there."""
        return self.capturable or self.found_inf is not None or bool(self._dev_hyper)

    def fuse_grad_norm_into(self, ddp):
        """Let ``ddp`` (libgsync DistributedDataParallel over exactly this
        optimizer's parameters) compute Σg² of the averaged grads inside its
        bucket unpacks ("partial ‖g‖² fused into unpack"); the
        clipped step then folds that scalar and runs no Σg² pass of its own —
        the clip path's exposed end is the update alone.  The sum runs in bucket
        order instead of the plan's, so the coefficient equals the unfused one
        to fp32 rounding.  Steps without a fresh synchronising backward (no_sync
        accumulation, ``gradient_as_bucket_view``, another parameter set) take
        the unfused path."""
        if not self.defaults.get("max_grad_norm"):
            raise ValueError("fuse_grad_norm_into: the optimizer has no max_grad_norm")
        dev = ddp.device
        buf = self._clip_buf.get(dev)
        if buf is None:
            buf = self._clip_buf[dev] = torch.zeros(4, dtype=torch.float32, device=dev)
        ddp.set_grad_sqnorm_target(buf[3:4])
        self._norm_ddp = (ddp, frozenset(id(p) for p in ddp._params))

    def _ddp_sqnorm(self, device):
        """The DDP's fused Σg² when it covers this step's grads, unchanged since
        the unpacks formed it (consumed).  A grad changed in place after backward
        (``GradScaler.unscale_``, ``clip_grad_norm_``, any torch in-place op: the
        grads' version counters moved) leaves the optimizer's own Σg² pass to run."""
        if self._norm_ddp is None:
            return None
        ddp, ids = self._norm_ddp
        if not ddp._sqnorm_valid or ddp.device != device:
            return None
        mine, ver = set(), 0
        for g in self.param_groups:
            for p in g["params"]:
                gr = p.grad
                if gr is not None:
                    mine.add(id(p))
                    ver += gr._version
        ddp._sqnorm_valid = False
        if mine != ids or ver != ddp._sqnorm_versions:
            return None
        return self._clip_buf[device][3:4]

    def _clip_scale(self, device, all_plans):
        """DeepSpeed-style gradient_clipping folded into the update: returns the
        grad multiplier the update launches get.

        Folded path (default): the coefficient min(1, max_norm/(‖g‖+1e-6))
        (times grad_scale) is formed by the update kernel's own workgroups
        (gs_plan_set_clip) — one plan: from the plan's Σg² partial sums
        (gs_sqnorm_partial), so Σg² -> update is two launches with no combine
        and no coefficient launch between them; several plans (grad dtypes):
        Σg² accumulated into one scalar first.  Those two forms are
        bit-identical to the separate path (GSYNC_CLIP_FUSED=0: Σg² + combine,
        gs_clip_coef, mul_ launches).  The DDP-fed form (fuse_grad_norm_into,
        ``last_clip_source == "ddp_unpack"``) sums the same squares in bucket
        order: its coefficient equals the others only to fp32 rounding."""
        max_norm = self.defaults.get("max_grad_norm")
        if not max_norm:
            for plan, _ in all_plans:
                if getattr(plan, "_clip_on", False):
                    plan.set_clip(None)
                    plan._clip_on = False
            return self.grad_scale
        buf = self._clip_buf.get(device)
        if buf is None:
            # [published Σg², coef, norm | accumulated raw Σg² (several plans)]
            buf = torch.zeros(4, dtype=torch.float32, device=device)
            self._clip_buf[device] = buf
        sq, coef, norm = buf[0:1], buf[1:2], buf[2:3]
        self.last_grad_norm = norm
        if CLIP_FUSED:
            fused = self._ddp_sqnorm(device)
            if fused is not None:
                # Σg² already formed by the DDP's unpacks: no pass over the grads here
                for plan, _ in all_plans:
                    plan.set_clip(float(max_norm), 1e-6, fused, out=buf[0:3])
                    plan._clip_on = True
                self.last_clip_source = "ddp_unpack"
                return self.grad_scale
            self.last_clip_source = "optimizer"
            if len(all_plans) == 1:
                plan, gdt = all_plans[0]
                plan.sqnorm_partial(1, gdt)
                plan.set_clip(float(max_norm), 1e-6, None, out=buf[0:3])
                plan._clip_on = True
            else:
                # the raw sum lives apart from the published triple: every update
                # launch reads it while workgroup 0 of each writes the (scaled) Σg²
                raw = buf[3:4]
                for i, (plan, gdt) in enumerate(all_plans):
                    plan.sqnorm(1, gdt, raw, accumulate=i > 0)
                for plan, _ in all_plans:
                    plan.set_clip(float(max_norm), 1e-6, raw, out=buf[0:3])
                    plan._clip_on = True
            return self.grad_scale  # the kernels fold it into the coefficient
        for plan, _ in all_plans:
            if getattr(plan, "_clip_on", False):
                plan.set_clip(None)
                plan._clip_on = False
        for i, (plan, gdt) in enumerate(all_plans):
            plan.sqnorm(1, gdt, sq, accumulate=i > 0)
        if self.grad_scale is not None:
            # norm of the unscaled grads: ‖g·s‖² = s²‖g‖²
            sq.mul_(self.grad_scale * self.grad_scale)
        clip_coef(sq, float(max_norm), 1e-6, coef, norm)
        if self.grad_scale is not None:
            coef.mul_(self.grad_scale)
        return coef


class FusedSGD(_FusedBase):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 *, maximize=False, foreach=None, differentiable=False, fused=None, max_grad_norm=None,
                 capturable=False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        if differentiable:
            raise ValueError("FusedSGD does not support differentiable=True")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, maximize=maximize, foreach=foreach, differentiable=False,
                        fused=fused, max_grad_norm=max_grad_norm, capturable=bool(capturable))
        super().__init__(params, defaults)

    def _collect(self, group):
        out = {}  # (grad dtype, has_buf) -> lists
        for p in group["params"]:
            if p.grad is None:
                continue
            if p.grad.is_sparse:
                raise RuntimeError("FusedSGD does not support sparse gradients")
            _check_dense(p, p.grad, "FusedSGD", self._dense_seen)
            if p.dtype != torch.float32:
                raise RuntimeError("FusedSGD expects fp32 parameters (keep a fp32 master copy)")
            st = self.state[p]
            buf = st.get("momentum_buffer")
            first = group["momentum"] != 0 and buf is None
            if group["momentum"] != 0 and buf is None:
                buf = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["momentum_buffer"] = buf
            key = (p.grad.dtype, first)
            out.setdefault(key, ([], [], []))
            ps, gs, bs = out[key]
            ps.append(p)
            gs.append(p.grad)
            bs.append(buf)
        return out

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        new_bufs = any(group["momentum"] != 0 and p.grad is not None and "momentum_buffer" not in self.state[p]
                       for group in self.param_groups for p in group["params"])
        if new_bufs and _capturing():
            raise RuntimeError("FusedSGD: momentum buffers must exist before capture (take an eager step first)")
        dev_state = self._device_state()
        work = []
        for gi, group in enumerate(self.param_groups):
            for (gdt, first), (ps, gs, bs) in self._collect(group).items():
                plan = self._plans.get(ps)
                plan.set_ptrs(0, ps)
                plan.set_ptrs(1, gs)
                plan.set_ptrs(2, [b.data_ptr() if b is not None else 0 for b in bs])
                flag = None
                if dev_state:
                    h = self._group_hyper(gi, group, ps[0].device)
                    if getattr(plan, "_hyper", None) is not h["hyper"]:
                        plan.set_hyper_source(h["hyper"])
                    if group["momentum"] != 0:
                        # first-step flag on the device (hyper[1]): set when this
                        # step creates the buffers, cleared after a step that ran
                        flag = h.setdefault("first_flags", {}).setdefault(
                            id(plan), torch.zeros(1, dtype=torch.float32, device=ps[0].device))
                        if first:
                            flag.fill_(1.0)
                work.append((group, plan, gdt, first, h if dev_state else None, flag))
        if dev_state:
            self.refresh_hyper()
        if not work:
            return loss
        scale = self._clip_scale(work[0][1].device, [(w[1], w[2]) for w in work])
        for group, plan, gdt, first, h, flag in work:
            if flag is not None:
                h["hyper"][1:2].copy_(flag)
            plan.sgd(gdt, group["lr"], group["momentum"], group["dampening"], group["weight_decay"],
                     group["nesterov"], group["maximize"], -1 if flag is not None else first,
                     grad_scale=scale, found_inf=self.found_inf)
            if flag is not None:
                if self.found_inf is not None:
                    flag.mul_(self.found_inf)  # kept only when the step was skipped
                else:
                    flag.zero_()
        return loss


class FusedAdam(_FusedBase):
    """Adam (``adamw=False``) or AdamW (``adamw=True`` / ``decoupled_weight_decay=True``)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 *, foreach=None, maximize=False, capturable=False, differentiable=False, fused=None,
                 decoupled_weight_decay=False, adamw=None, max_grad_norm=None):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        if amsgrad:
            raise NotImplementedError("FusedAdam: amsgrad is not on the reference path")
        if differentiable:
            raise ValueError("FusedAdam does not support differentiable=True")
        adamw = bool(decoupled_weight_decay if adamw is None else adamw)
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        foreach=foreach, maximize=maximize, capturable=bool(capturable), differentiable=False,
                        fused=fused, decoupled_weight_decay=adamw, max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)

    # ---- device step counters (capturable / AMP): one fp64 counter per cohort of
    # parameters that have advanced together so far.  torch keeps one step per
    # parameter (T:optim/adam.py: state_steps[i] += 1 only for params with a
    # grad); a cohort shares one counter while all its members get grads, and is
    # split (its counter cloned on the device, no host read) the first step some
    # members have none — so every parameter's bias correction is its own.
    def _adopt_cohorts(self, h, group):
        """Give every stateful parameter of `group` without a device counter one:
        parameters whose (host) step values are equal share a new cohort."""
        cohorts = h.setdefault("cohorts", {})
        by_value: dict = {}
        for p in group["params"]:
            st = self.state.get(p)
            if not st or "exp_avg" not in st:
                continue
            t = st.get("step")
            if t is not None and id(t) in cohorts:
                continue
            if _capturing():
                raise RuntimeError("FusedAdam: state must exist before capture (take an eager step first)")
            v = 0.0 if t is None else float(t)
            c = by_value.get(v)
            if c is None:
                c = by_value[v] = {"step": torch.full((1,), v, dtype=torch.float64, device=p.device),
                                   "hyper": torch.zeros(3, dtype=torch.float32, device=p.device),
                                   "members": set()}
                cohorts[id(c["step"])] = c
            c["members"].add(id(p))
            st["step"] = c["step"]

    def _split_cohort(self, h, c, ps):
        """Members `ps` (with grads) leave cohort `c` (some of whose members have
        none this step) for a new one starting at the same count."""
        if _capturing():
            raise RuntimeError("FusedAdam: the set of parameters with grads changed inside a capture")
        n = {"step": c["step"].clone(), "hyper": torch.zeros_like(c["hyper"]), "members": {id(p) for p in ps}}
        c["members"] -= n["members"]
        h["cohorts"][id(n["step"])] = n
        for p in ps:
            self.state[p]["step"] = n["step"]
        return n

    def state_dict(self):
        """torch's layout: one ``step`` tensor per parameter (fp32; on the CPU,
        or on the device when capturable, as torch's Adam keeps it) — device
        counters shared by a cohort are read out here (host read, checkpoint time)."""
        sd = super().state_dict()
        vals: dict = {}
        for k, st in list(sd["state"].items()):
            t = st.get("step")
            if torch.is_tensor(t) and t.dtype == torch.float64:
                v = vals.get(id(t))
                if v is None:
                    v = vals[id(t)] = float(t.item())
                dev = t.device if self.capturable else torch.device("cpu")
                sd["state"][k] = dict(st, step=torch.tensor(v, dtype=torch.float32, device=dev))
        return sd

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        cap = self._device_state()  # device step counters: capturable or AMP (no host read of found_inf)
        work = []
        for gi, group in enumerate(self.param_groups):
            buckets = {}
            by_cohort: dict = {}
            h = None
            live = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                _check_dense(p, p.grad, "FusedAdam", self._dense_seen)
                if p.dtype != torch.float32:
                    raise RuntimeError("FusedAdam expects fp32 parameters (keep a fp32 master copy)")
                st = self.state[p]
                if len(st) == 0 or "exp_avg" not in st:
                    if _capturing():
                        raise RuntimeError("FusedAdam: state must exist before capture (take an eager step first)")
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                live.append(p)
            # every state of this step exists before cohorts are formed: parameters
            # whose state starts together share one cohort (one counter, one plan)
            for p in live:
                st = self.state[p]
                if cap:
                    if h is None:
                        h = self._group_hyper(gi, group, p.device)
                    if id(st["step"]) not in h.get("cohorts", {}):
                        self._adopt_cohorts(h, group)
                    by_cohort.setdefault(id(st["step"]), []).append(p)
                else:
                    st["step"] += 1
                    lists = buckets.setdefault((p.grad.dtype, float(st["step"].item())), ([], [], [], []))
                    lists[0].append(p)
                    lists[1].append(p.grad)
                    lists[2].append(st["exp_avg"])
                    lists[3].append(st["exp_avg_sq"])
            for cid, ps in by_cohort.items():
                c = h["cohorts"][cid]
                if len(ps) < len(c["members"]):
                    c = self._split_cohort(h, c, ps)
                work.append((group, None, gi, (h, c)))  # advance the cohort's counter, form its hyper source
                for p in ps:
                    st = self.state[p]
                    lists = buckets.setdefault((p.grad.dtype, id(c["step"])), ([], [], [], []))
                    lists[0].append(p)
                    lists[1].append(p.grad)
                    lists[2].append(st["exp_avg"])
                    lists[3].append(st["exp_avg_sq"])
            cohort_hyper = {id(c["step"]): c["hyper"] for c in h["cohorts"].values()} if h is not None else {}
            for (gdt, step), (ps, gs, ms, vs) in buckets.items():
                plan = self._plans.get(ps)
                plan.set_ptrs(0, ps)
                plan.set_ptrs(1, gs)
                plan.set_ptrs(2, ms)
                plan.set_ptrs(3, vs)
                if cap:
                    hyper = cohort_hyper[step]
                    if getattr(plan, "_hyper", None) is not hyper:
                        plan.set_hyper_source(hyper)
                    work.append((group, plan, gdt, None))
                else:
                    work.append((group, plan, gdt, step))
        if not work:
            return loss
        if cap:
            self.refresh_hyper()
        plans = [(w[1], w[2]) for w in work if w[1] is not None]
        if not plans:
            return loss
        scale = self._clip_scale(plans[0][0].device, plans)
        for group, plan, gdt, step in work:
            beta1, beta2 = group["betas"]
            if plan is None:  # device counters: advance the cohort's step, form its hyper source
                h, c = step
                L.check(L.lib().gs_adam_hyper(
                    L.GS_DEV_HIP if c["step"].is_cuda else L.GS_DEV_HOST, c["step"].data_ptr(), h["lr"].data_ptr(),
                    float(beta1), float(beta2), float(group["weight_decay"]),
                    None if self.found_inf is None else self.found_inf.data_ptr(), c["hyper"].data_ptr(),
                    L.stream_ptr(c["step"].device) if c["step"].is_cuda else None), "gs_adam_hyper")
                continue
            if step is None:  # the kernel reads step_size / bc2 / decay from the hyper source
                plan.adam(gdt, group["lr"], beta1, beta2, group["eps"], group["weight_decay"],
                          group["decoupled_weight_decay"], group["maximize"], -1.0, 1.0,
                          grad_scale=scale, found_inf=self.found_inf)
                continue
            lr = group["lr"]
            # python-double bias corrections, as torch's foreach path computes them
            bias_correction1 = 1 - beta1 ** step
            bias_correction2 = 1 - beta2 ** step
            step_size = (lr / bias_correction1) * -1
            bias_correction2_sqrt = bias_correction2 ** 0.5
            plan.adam(gdt, lr, beta1, beta2, group["eps"], group["weight_decay"],
                      group["decoupled_weight_decay"], group["maximize"], step_size, bias_correction2_sqrt,
                      grad_scale=scale, found_inf=self.found_inf)
        return loss


class FusedAdamW(FusedAdam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, **kw):
        kw.pop("decoupled_weight_decay", None)
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw=True, **kw)


_NORM_PLANS: dict = {}


@torch.no_grad()
def clip_grad_norm_(parameters: torch.Tensor | Iterable[torch.Tensor], max_norm: float, norm_type: float = 2.0,
                    error_if_nonfinite: bool = False, foreach=None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ for the L2 norm on libgsync kernels.

    total_norm = ‖concat(g)‖₂ ; coef = clamp(max_norm / (total_norm + 1e-6), max=1);
    grads *= coef (T:nn/utils/clip_grad.py:165-174).  Everything stays on the
    device; only error_if_nonfinite forces a host read, as in torch.

    One grad dtype (the common case) is two launches: the Σg² partial sums
    (gs_sqnorm_partial, left in the plan), then the scale pass whose every
    workgroup folds them into the coefficient itself (gs_clip_scale; it writes
    nothing when the coefficient is 1).  No combine launch, no coefficient
    launch, no flag fill.  Several grad dtypes: Σg² accumulated over the groups
    (gs_sqnorm), then each group's scale pass folds that scalar.
    """
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    grads = [p.grad for p in parameters if p.grad is not None]
    if float(norm_type) != 2.0:
        raise NotImplementedError("clip_grad_norm_: only norm_type=2 is on the gradient-sync path")
    if len(grads) == 0:
        return torch.tensor(0.0)
    dev = grads[0].device
    groups: dict = {}
    for g in grads:
        if not is_dense(g):
            raise RuntimeError("clip_grad_norm_: grads must be dense")
        groups.setdefault(g.dtype, []).append(g)
    # [Σg², coef, norm | accumulated Σg² (several dtypes)]: written by the kernels before
    # any read (workgroup 0 of the scale pass publishes the first three), so no fill
    buf = torch.empty(4, dtype=torch.float32, device=dev)
    plans = []
    for dt, gl in groups.items():
        key = tuple(g.numel() for g in gl) + (dev,)  # sizes + device: grad ids are reused after zero_grad
        plan = _NORM_PLANS.get(key)
        if plan is None:
            plan = TensorListPlan([g.numel() for g in gl], dev)
            if len(_NORM_PLANS) > 64:
                _NORM_PLANS.clear()
            _NORM_PLANS[key] = plan
        plan.set_ptrs(0, gl)
        plans.append((plan, dt))
    if len(plans) == 1 and not error_if_nonfinite:
        plan, dt = plans[0]
        plan.sqnorm_partial(0, dt)
        plan.set_clip(float(max_norm), 1e-6, None, out=buf[0:3])
    else:
        raw = buf[3:4]
        for i, (plan, dt) in enumerate(plans):
            plan.sqnorm(0, dt, raw, accumulate=i > 0)
        # torch raises before touching the grads (T:nn/utils/clip_grad.py:96-109)
        if error_if_nonfinite and not torch.isfinite(raw).item():
            raise RuntimeError(
                f"The total norm of order {float(norm_type)} for gradients from `parameters` is non-finite, "
                "so it cannot be clipped. To disable this error and scale the gradients by the non-finite "
                "norm anyway, set `error_if_nonfinite=False`")
        for plan, _ in plans:
            plan.set_clip(float(max_norm), 1e-6, raw, out=buf[0:3])
    for plan, dt in plans:
        plan.clip_scale(0, dt)
        plan.set_clip(None)
    norm = buf[2:3]
    # the kernel wrote the grads in place: tell autograd's version counters, as a
    # torch in-place op would (a DDP's fused Σg² of these grads is stale now)
    increment_version(grads)
    return norm.reshape(())
