"""Flat-buffer helpers on libgsync kernels.

Drop-ins for ``torch._utils._flatten_dense_tensors`` /
``_unflatten_dense_tensors`` (T:_utils.py:558-608), the flatten / unflatten
DeepSpeed and ColossalAI use around their flat ZeRO buffers, plus the copy
back into the original tensors they do after an all-gather
(``for t, v in zip(ts, unflatten(flat, ts)): t.copy_(v)``):

* :func:`flatten_dense_tensors` — one multi-tensor pack launch instead of
  ``torch.cat``; same result (elements in each tensor's contiguous order,
  tensors back to back, no padding);
* :func:`unflatten_dense_tensors` — views of the flat buffer, no copy (as torch);
* :func:`copy_flat_to` — one multi-tensor unpack launch instead of one
  ``copy_`` per tensor.
"""
from __future__ import annotations

from typing import Sequence

import torch

from .multi_tensor import TensorListPlan

_PLANS: dict = {}


def _plan(tensors: Sequence[torch.Tensor]) -> TensorListPlan:
    key = (tensors[0].device, tuple(t.numel() for t in tensors))
    plan = _PLANS.get(key)
    if plan is None:
        if len(_PLANS) > 64:
            _PLANS.clear()
        plan = TensorListPlan([t.numel() for t in tensors], tensors[0].device)
        _PLANS[key] = plan
    return plan


def _check(tensors):
    if len(tensors) == 0:
        raise ValueError("expected a non-empty list of tensors")
    dt, dev = tensors[0].dtype, tensors[0].device
    for t in tensors:
        if t.dtype != dt or t.device != dev:
            raise TypeError("all tensors must share one dtype and device (torch.cat would promote or fail)")
        if t.is_sparse:
            raise TypeError("dense tensors only")


def flatten_dense_tensors(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """torch._utils._flatten_dense_tensors: 1-D concatenation of each tensor's
    contiguous-order elements."""
    tensors = list(tensors)
    _check(tensors)
    src = [t if t.is_contiguous() else t.contiguous() for t in tensors]
    plan = _plan(src)
    flat = torch.empty(plan.flat_numel, dtype=src[0].dtype, device=src[0].device)
    plan.set_ptrs(0, src)
    plan.pack(0, src[0].dtype, flat)
    return flat


def unflatten_dense_tensors(flat: torch.Tensor, tensors: Sequence[torch.Tensor]):
    """torch._utils._unflatten_dense_tensors: views of `flat` shaped like `tensors`."""
    out, off = [], 0
    for t in tensors:
        n = t.numel()
        out.append(flat.narrow(0, off, n).view_as(t))
        off += n
    return tuple(out)


def copy_flat_to(flat: torch.Tensor, tensors: Sequence[torch.Tensor]) -> None:
    """``t.copy_(v)`` for every (t, v) in zip(tensors, unflatten(flat, tensors)),
    as one launch.  Tensors must be contiguous (as the flat layout is)."""
    tensors = list(tensors)
    _check(tensors)
    if any(not t.is_contiguous() for t in tensors):
        for t, v in zip(tensors, unflatten_dense_tensors(flat, tensors)):
            t.copy_(v)
        return
    plan = _plan(tensors)
    if flat.numel() < plan.flat_numel or flat.dtype != tensors[0].dtype or flat.device != tensors[0].device:
        raise ValueError("flat buffer does not match the tensors (numel, dtype, device)")
    plan.set_ptrs(0, tensors)
    plan.unpack(flat, 0, tensors[0].dtype)
