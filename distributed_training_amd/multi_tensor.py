"""Python handle on a libgsync multi-tensor plan (``gs_plan``).

A plan is a static list of tensor sizes laid out in one flat buffer, with the
chunk map the device kernels stream through built once; only the per-tensor
pointer tables change from call to call, and they are re-uploaded only when
they do.
It plays the role of ATen's ``multi_tensor_apply`` launch machinery
(T:include/ATen/native/cuda/MultiTensorApply.cuh:14-21) for every op on the
gradient-sync path.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from . import _lib as L

# Task size (units of 4 elements) of an optimizer-update plan's segment table on
# the GPU (gs_plan_create_ex task_units).  The device kernels stream through the
# chunk map (gs_engine.h) whatever the task size; the segment table stays the
# plan's public work decomposition (gs_plan_n_tasks / gs_plan_task_units).
UPDATE_TASK_UNITS = 512


def update_task_units(device) -> int:
    """task_units for an optimizer-update plan on ``device`` (0 = library default)."""
    return UPDATE_TASK_UNITS if torch.device(device).type == "cuda" else 0


class TensorListPlan:
    def __init__(self, numels: Sequence[int], device: torch.device, align: int = 0, task_units: int = 0):
        self.device = torch.device(device)
        self.kind = L.GS_DEV_HIP if self.device.type == "cuda" else L.GS_DEV_HOST
        self.numels = [int(n) for n in numels]
        self.n = len(self.numels)
        dev_index = self.device.index if self.device.index is not None else (
            torch.cuda.current_device() if self.kind == L.GS_DEV_HIP else 0
        )
        self.dev_index = dev_index
        h = ctypes.c_void_p()
        lib = L.lib()
        L.check(
            lib.gs_plan_create_ex(self.kind, dev_index, self.n, L.i64_array(self.numels), int(align),
                                  int(task_units), ctypes.byref(h)),
            "gs_plan_create_ex",
        )
        self.handle = h
        self.flat_numel = int(lib.gs_plan_flat_numel(h))
        offs = (ctypes.c_int64 * max(1, self.n))()
        L.check(lib.gs_plan_offsets(h, offs), "gs_plan_offsets")
        self.offsets = [int(offs[i]) for i in range(self.n)]
        self._slot_cache: dict[int, tuple] = {}

    # ------------------------------------------------------------------
    def close(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                L.destroy("gs_plan_destroy", h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self.handle = None

    def __del__(self):
        self.close()

    def _stream(self, stream):
        if stream is not None:
            return stream
        if self.kind == L.GS_DEV_HOST:  # host backend: torch's intra-op threads
            L.lib().gs_set_host_threads(torch.get_num_threads())
        return L.stream_ptr(self.device)

    def set_ptrs(self, slot: int, tensors_or_ptrs):
        ptrs = tuple(
            (t if isinstance(t, int) or t is None else t.data_ptr()) for t in tensors_or_ptrs
        )
        if len(ptrs) != self.n:
            raise ValueError(f"plan has {self.n} tensors, got {len(ptrs)} pointers")
        if self._slot_cache.get(slot) == ptrs:
            return
        for t, n in zip(tensors_or_ptrs, self.numels):  # new pointers: the sizes must be the plan's
            if isinstance(t, torch.Tensor) and t.numel() != n:
                raise ValueError(f"plan tensor of {n} elements bound to a tensor of {t.numel()}")
        L.check(L.lib().gs_plan_set_ptrs(self.handle, slot, L.ptr_array(ptrs), None), "gs_plan_set_ptrs")
        self._slot_cache[slot] = ptrs

    @property
    def n_tasks(self) -> int:
        return int(L.lib().gs_plan_n_tasks(self.handle))

    @property
    def task_units(self) -> int:
        return int(L.lib().gs_plan_task_units(self.handle))

    def set_hyper_source(self, hyper: torch.Tensor | None):
        """Later sgd()/adam() launches read their step-varying hyper-parameters
        from ``hyper`` (fp32, on the plan's device) when they run — SGD [lr];
        Adam [step_size, bias_correction2_sqrt, 1 - lr*wd] — instead of their
        arguments (gs_plan_set_hyper_source).  The plan keeps a reference."""
        if hyper is not None:
            if hyper.dtype != torch.float32 or not hyper.is_contiguous() or hyper.numel() < 3:
                raise ValueError("hyper source: contiguous fp32 tensor of >= 3 elements")
            if (hyper.device.type == "cuda") != (self.kind == L.GS_DEV_HIP):
                raise ValueError("hyper source must live where the plan runs")
        L.check(L.lib().gs_plan_set_hyper_source(self.handle, None if hyper is None else hyper.data_ptr()),
                "gs_plan_set_hyper_source")
        self._hyper = hyper

    def timer_enable(self, n_slots: int = 256):
        """Bracket every launch of this plan with HIP timing events on its
        launch stream (ring of n_slots); 0 disables."""
        L.check(L.lib().gs_plan_timer_enable(self.handle, int(n_slots)), "gs_plan_timer_enable")

    def timer_read(self, cap: int = 4096, kind: int | None = None) -> list:
        """Kernel durations (ms) recorded since the last read, oldest first
        (only launches of op `kind` = L.GS_OP_* when given)."""
        out = (ctypes.c_float * max(1, cap))()
        kinds = (ctypes.c_int32 * max(1, cap))()
        n = L.check(L.lib().gs_plan_timer_read(self.handle, out, kinds, int(cap)), "gs_plan_timer_read")
        return [float(out[i]) for i in range(n) if kind is None or kinds[i] == kind]

    def timer_read_by_kind(self, cap: int = 4096) -> dict:
        """{GS_OP_* kind: [durations (ms)]} of the launches recorded since the last read."""
        out = (ctypes.c_float * max(1, cap))()
        kinds = (ctypes.c_int32 * max(1, cap))()
        n = L.check(L.lib().gs_plan_timer_read(self.handle, out, kinds, int(cap)), "gs_plan_timer_read")
        by: dict = {}
        for i in range(n):
            by.setdefault(int(kinds[i]), []).append(float(out[i]))
        return by

    # ------------------------------------------------------------------ ops
    def pack(self, src_slot, src_dtype, flat: torch.Tensor, scale=1.0, mode=L.GS_SCALE_NONE, stream=None):
        L.check(
            L.lib().gs_pack(self.handle, src_slot, L.gs_dtype(src_dtype), flat.data_ptr(),
                            L.gs_dtype(flat.dtype), float(scale), mode, self._stream(stream)),
            "gs_pack",
        )

    def unpack(self, flat: torch.Tensor, dst_slot, dst_dtype, sqnorm: torch.Tensor | None = None,
               accumulate=False, stream=None):
        L.check(
            L.lib().gs_unpack(self.handle, flat.data_ptr(), L.gs_dtype(flat.dtype), dst_slot,
                              L.gs_dtype(dst_dtype), None if sqnorm is None else sqnorm.data_ptr(),
                              int(bool(accumulate)), self._stream(stream)),
            "gs_unpack",
        )

    def scale(self, slot, dtype, s, mode=L.GS_SCALE_MUL, stream=None):
        L.check(L.lib().gs_scale(self.handle, slot, L.gs_dtype(dtype), float(s), mode, self._stream(stream)),
                "gs_scale")

    def sqnorm(self, slot, dtype, out: torch.Tensor, accumulate=False, stream=None):
        L.check(
            L.lib().gs_sqnorm(self.handle, slot, L.gs_dtype(dtype), out.data_ptr(), int(bool(accumulate)),
                              self._stream(stream)),
            "gs_sqnorm",
        )

    def sqnorm_partial(self, slot, dtype, stream=None):
        """Σ x² of the slot left inside the plan (gs_sqnorm_partial): no combine
        launch; the next clipped sgd()/adam() on this plan folds it."""
        L.check(L.lib().gs_sqnorm_partial(self.handle, slot, L.gs_dtype(dtype), self._stream(stream)),
                "gs_sqnorm_partial")

    def sqnorm_partial_out(self, slot, dtype, groups: torch.Tensor, stream=None) -> int:
        """:meth:`sqnorm_partial` whose partial sums land contiguously in
        ``groups`` (fp32, >= GS_RED_PARTIALS elements, where the plan runs;
        gs_sqnorm_partial_out: one per workgroup of a balanced grid on a small
        plan, else the <= 64 group sums); returns how many are valid.  Sharded
        optimizers SUM-all-reduce the whole buffer across ranks (the slots past
        n stay zero), then :meth:`set_clip_groups`."""
        if groups.dtype != torch.float32 or groups.numel() < L.GS_RED_PARTIALS or not groups.is_contiguous() or \
                (groups.device.type == "cuda") != (self.kind == L.GS_DEV_HIP):
            raise ValueError(f"partial sums: contiguous fp32[>= {L.GS_RED_PARTIALS}] where the plan runs")
        n = ctypes.c_int32()
        L.check(L.lib().gs_sqnorm_partial_out(self.handle, slot, L.gs_dtype(dtype), groups.data_ptr(),
                                              ctypes.byref(n), self._stream(stream)), "gs_sqnorm_partial_out")
        return n.value

    def set_clip_groups(self, max_norm: float | None, eps: float, groups: torch.Tensor, n_groups: int,
                        sq_mul: float = 1.0, coef_mul: float = 1.0, out: torch.Tensor | None = None):
        """:meth:`set_clip` with ‖g‖² = the fold of ``groups[:n_groups]``
        (<= GS_RED_PARTIALS; gs_plan_set_clip_groups), the update's workgroups
        folding them in a fixed order."""
        for t in (groups, out):
            if t is not None and (t.dtype != torch.float32 or (t.device.type == "cuda") != (self.kind == L.GS_DEV_HIP)):
                raise ValueError("clip tensors: fp32, where the plan runs")
        if out is not None and out.numel() < 3:
            raise ValueError("clip out: 3 elements")
        if not groups.is_contiguous() or groups.numel() < int(n_groups):
            raise ValueError(f"partial sums: {n_groups} contiguous floats expected, got {groups.numel()}")
        L.check(L.lib().gs_plan_set_clip_groups(self.handle, groups.data_ptr(), int(n_groups), float(max_norm or 0.0),
                                                float(eps), float(sq_mul), float(coef_mul),
                                                None if out is None else out.data_ptr()), "gs_plan_set_clip_groups")
        self._clip_refs = (groups, out)

    def set_read_hint(self, hint: int):
        """How this plan's Σg² kernels load their slot (gs_plan_set_read_hint): 0 the
        size rule, 1 non-temporal, 2 cached."""
        L.check(L.lib().gs_plan_set_read_hint(self.handle, int(hint)), "gs_plan_set_read_hint")

    def set_clip(self, max_norm: float | None, eps: float = 1e-6, sqnorm: torch.Tensor | None = None,
                 sq_mul: float = 1.0, coef_mul: float = 1.0, out: torch.Tensor | None = None):
        """Fold the clip coefficient min(1, max_norm/(‖g‖+eps)) into the later
        sgd()/adam() launches of this plan (gs_plan_set_clip): ‖g‖² from
        ``sqnorm`` (a 1-element fp32 tensor) or, when None, from this plan's last
        :meth:`sqnorm_partial`; ``out`` (fp32[3], optional) receives
        [‖g‖², coef, ‖g‖].  ``max_norm`` None/0 turns it off."""
        for t in (sqnorm, out):
            if t is not None and (t.dtype != torch.float32 or (t.device.type == "cuda") != (self.kind == L.GS_DEV_HIP)):
                raise ValueError("clip tensors: fp32, where the plan runs")
        if out is not None and out.numel() < 3:
            raise ValueError("clip out: 3 elements")
        L.check(L.lib().gs_plan_set_clip(self.handle, None if sqnorm is None else sqnorm.data_ptr(),
                                         float(max_norm or 0.0), float(eps), float(sq_mul), float(coef_mul),
                                         None if out is None else out.data_ptr()), "gs_plan_set_clip")
        self._clip_refs = (sqnorm, out)

    def sum(self, slot, dtype, out: torch.Tensor, accumulate=False, stream=None):
        """out[0] = Σ x over the slot's tensors (fp32, deterministic order)."""
        L.check(
            L.lib().gs_sum(self.handle, slot, L.gs_dtype(dtype), out.data_ptr(), int(bool(accumulate)),
                           self._stream(stream)),
            "gs_sum",
        )

    def clip_scale(self, slot, dtype, stream=None):
        """slot *= torch.clamp(max_norm/(‖g‖+eps), max=1) from this plan's clip
        (:meth:`set_clip`, consumed like a clipped update's); nothing written when
        the coefficient is 1 (gs_clip_scale)."""
        L.check(L.lib().gs_clip_scale(self.handle, slot, L.gs_dtype(dtype), self._stream(stream)), "gs_clip_scale")

    def unscale_check(self, slot, dtype, inv_scale: torch.Tensor | None, found_inf: torch.Tensor, stream=None):
        L.check(
            L.lib().gs_unscale_check(self.handle, slot, L.gs_dtype(dtype),
                                     None if inv_scale is None else inv_scale.data_ptr(),
                                     found_inf.data_ptr(), self._stream(stream)),
            "gs_unscale_check",
        )

    def sgd(self, grad_dtype, lr, momentum, dampening, weight_decay, nesterov, maximize, first_step,
            lowp_dtype=None, grad_scale=None, found_inf=None, stream=None):
        L.check(
            L.lib().gs_sgd_step(
                self.handle, L.gs_dtype(grad_dtype), -1 if lowp_dtype is None else L.gs_dtype(lowp_dtype),
                float(lr), float(momentum), float(dampening), float(weight_decay), int(bool(nesterov)),
                int(bool(maximize)), -1 if first_step == -1 else int(bool(first_step)),
                None if grad_scale is None else grad_scale.data_ptr(),
                None if found_inf is None else found_inf.data_ptr(), self._stream(stream)),
            "gs_sgd_step",
        )

    def adam(self, grad_dtype, lr, beta1, beta2, eps, weight_decay, adamw, maximize, step_size,
             bias_correction2_sqrt, lowp_dtype=None, grad_scale=None, found_inf=None, stream=None):
        L.check(
            L.lib().gs_adam_step(
                self.handle, L.gs_dtype(grad_dtype), -1 if lowp_dtype is None else L.gs_dtype(lowp_dtype),
                float(lr), float(beta1), float(beta2), float(eps), float(weight_decay), int(bool(adamw)),
                int(bool(maximize)), float(step_size), float(bias_correction2_sqrt),
                None if grad_scale is None else grad_scale.data_ptr(),
                None if found_inf is None else found_inf.data_ptr(), self._stream(stream)),
            "gs_adam_step",
        )


def clip_coef(sqnorm: torch.Tensor, max_norm: float, eps: float, coef: torch.Tensor,
              norm: torch.Tensor | None = None, stream=None):
    kind = L.GS_DEV_HIP if sqnorm.device.type == "cuda" else L.GS_DEV_HOST
    if stream is None:
        stream = L.stream_ptr(sqnorm.device)
    L.check(
        L.lib().gs_clip_coef(kind, sqnorm.data_ptr(), float(max_norm), float(eps), coef.data_ptr(),
                             None if norm is None else norm.data_ptr(), stream),
        "gs_clip_coef",
    )


def is_dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense: the elements fill exactly numel() consecutive
    slots starting at data_ptr() (any dim order, e.g. channels_last)."""
    if t.is_contiguous():
        return True
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.size()) if sz != 1)
    expected = 1
    for st, sz in dims:
        if st != expected:
            return False
        expected *= sz
    return True


def dense_like_param(grad: torch.Tensor, param: torch.Tensor) -> bool:
    """grad's memory is one dense block in the same element order as param's."""
    return grad.shape == param.shape and grad.stride() == param.stride() and is_dense(grad)
