"""numpy front-end of the C oracle (gs_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker; never by the product package.
Every function restates a piece of the reference path (torch DDP Reducer +
optimizers, cited in gs_oracle.c) and is pinned against tests/golden/
fixtures produced by running the reference's own train step under torch DDP.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libgsoracle.so")
F32, BF16, F16 = 0, 1, 2

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, i64, i32, f, d, c_int = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float,
                                    ctypes.c_double, ctypes.c_int)
        L.or_pack.argtypes = [c_int, ctypes.POINTER(vp), ctypes.POINTER(i64), ctypes.POINTER(i64), c_int, vp, c_int, f, c_int]
        L.or_unpack.argtypes = [c_int, ctypes.POINTER(vp), ctypes.POINTER(i64), ctypes.POINTER(i64), vp, c_int, c_int]
        L.or_allreduce_sum.argtypes = [c_int, ctypes.POINTER(vp), i64, c_int, vp]
        L.or_sgd.argtypes = [i64, vp, vp, c_int, vp, d, d, d, d, c_int, c_int, c_int, vp, vp, c_int]
        L.or_adam.argtypes = [i64, vp, vp, c_int, vp, vp, d, d, d, d, d, c_int, c_int, d, d, vp, vp, c_int]
        L.or_sqnorm.argtypes = [c_int, ctypes.POINTER(vp), ctypes.POINTER(i64), c_int]
        L.or_sqnorm.restype = d
        L.or_clip_coef.argtypes = [f, f, f]
        L.or_clip_coef.restype = f
        L.or_bucket_assignment.argtypes = [c_int, ctypes.POINTER(i64), ctypes.POINTER(i32), ctypes.POINTER(i32), c_int,
                                           ctypes.POINTER(i64), ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.or_f32_to_bf16.argtypes = [f]
        L.or_f32_to_bf16.restype = ctypes.c_uint16
        _lib = L
    return _lib


def _dt(a: np.ndarray) -> int:
    if a.dtype == np.float32:
        return F32
    if a.dtype == np.uint16:  # bf16 bit patterns unless told otherwise
        return BF16
    if a.dtype == np.float16:
        return F16
    raise TypeError(a.dtype)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _vparr(arrs):
    return (ctypes.c_void_p * len(arrs))(*[None if a is None else a.ctypes.data for a in arrs])


def aligned_offsets(numels, align):
    offs, cur = [], 0
    for n in numels:
        if align:
            cur = (cur + align - 1) // align * align
        offs.append(cur)
        cur += n
    total = ((cur + align - 1) // align * align) if align else cur
    return offs, total


def f32_to_bf16(x: np.ndarray) -> np.ndarray:
    """round-to-nearest-even bf16 bit patterns (uint16), NaN -> 0x7FC0."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(x)
    r[nan] = 0x7FC0
    return r


def bf16_to_f32(h: np.ndarray) -> np.ndarray:
    return (h.astype(np.uint32) << 16).view(np.float32)


def pack(srcs, flat_dtype="f32", scale=1.0, mode=0, align=0, src_dtype=None):
    """Flatten + scale + cast; returns the flat buffer (float32 or uint16 bf16 bits)."""
    srcs = [np.ascontiguousarray(s).reshape(-1) if s is not None else None for s in srcs]
    numels = [s.size if s is not None else 0 for s in srcs]
    offs, total = aligned_offsets(numels, align)
    fdt = {"f32": F32, "bf16": BF16, "f16": F16}[flat_dtype]
    flat = np.zeros(total, dtype=np.float32 if fdt == F32 else (np.uint16 if fdt == BF16 else np.float16))
    sdt = src_dtype if src_dtype is not None else _dt(next(s for s in srcs if s is not None))
    lib().or_pack(len(srcs), _vparr(srcs), (ctypes.c_int64 * len(numels))(*numels),
                  (ctypes.c_int64 * len(offs))(*offs), sdt, _ptr(flat), fdt, float(scale), int(mode))
    return flat


def unpack(flat, shapes, dst_dtype=np.float32, align=0, flat_dtype=None):
    numels = [int(np.prod(s)) for s in shapes]
    offs, _ = aligned_offsets(numels, align)
    outs = [np.zeros(n, dtype=dst_dtype) for n in numels]
    fdt = flat_dtype if flat_dtype is not None else _dt(flat)
    ddt = _dt(outs[0]) if outs else F32
    lib().or_unpack(len(outs), _vparr(outs), (ctypes.c_int64 * len(numels))(*numels),
                    (ctypes.c_int64 * len(offs))(*offs), _ptr(flat), fdt, ddt)
    return [o.reshape(s) for o, s in zip(outs, shapes)]


def allreduce_sum(bufs):
    bufs = [np.ascontiguousarray(b) for b in bufs]
    out = np.empty_like(bufs[0])
    lib().or_allreduce_sum(len(bufs), _vparr(bufs), bufs[0].size, _dt(bufs[0]), _ptr(out))
    return out


def ddp_average(local_grads_per_rank, bucket_dtype="f32", align=0):
    """The reference's averaged gradient: Σ_r (g_r · float(1/ws)) per tensor
    (pack with mul_out scale, SUM all-reduce, unpack).  Returns a list of arrays."""
    ws = len(local_grads_per_rank)
    scale = np.float32(1.0 / ws)
    shapes = [g.shape for g in local_grads_per_rank[0]]
    flats = [pack(gs, bucket_dtype, scale, 1, align) for gs in local_grads_per_rank]
    summed = allreduce_sum(flats)
    return unpack(summed, shapes, np.float32, align)


def sgd(p, g, buf, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, maximize=False,
        first=False, gscale=None):
    p = np.array(p, dtype=np.float32, copy=True).reshape(-1)
    buf = np.zeros_like(p) if buf is None else np.array(buf, dtype=np.float32, copy=True).reshape(-1)
    g = np.ascontiguousarray(g).reshape(-1)
    gs = None if gscale is None else np.array([gscale], dtype=np.float32)
    lib().or_sgd(p.size, _ptr(p), _ptr(g), _dt(g), _ptr(buf), lr, momentum, dampening, weight_decay,
                 int(nesterov), int(maximize), int(first), _ptr(gs), None, 0)
    return p, buf


def adam(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, adamw=False,
         maximize=False, gscale=None):
    p = np.array(p, dtype=np.float32, copy=True).reshape(-1)
    m = np.array(m, dtype=np.float32, copy=True).reshape(-1)
    v = np.array(v, dtype=np.float32, copy=True).reshape(-1)
    g = np.ascontiguousarray(g).reshape(-1)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = (lr / bc1) * -1
    gs = None if gscale is None else np.array([gscale], dtype=np.float32)
    lib().or_adam(p.size, _ptr(p), _ptr(g), _dt(g), _ptr(m), _ptr(v), lr, beta1, beta2, eps, weight_decay,
                  int(adamw), int(maximize), step_size, bc2 ** 0.5, _ptr(gs), None, 0)
    return p, m, v


def sqnorm(xs):
    xs = [np.ascontiguousarray(x).reshape(-1) for x in xs]
    return lib().or_sqnorm(len(xs), _vparr(xs), (ctypes.c_int64 * len(xs))(*[x.size for x in xs]), _dt(xs[0]))


def clip_coef(total_norm, max_norm, eps=1e-6):
    return lib().or_clip_coef(float(total_norm), float(max_norm), float(eps))


def bucket_assignment(nbytes, limits, order=None, keys=None):
    n = len(nbytes)
    members = (ctypes.c_int32 * n)()
    counts = (ctypes.c_int32 * n)()
    nb = lib().or_bucket_assignment(
        n, (ctypes.c_int64 * n)(*nbytes), None if keys is None else (ctypes.c_int32 * n)(*keys),
        None if order is None else (ctypes.c_int32 * n)(*order), len(limits),
        (ctypes.c_int64 * len(limits))(*[min(int(x), 2**62) for x in limits]), members, counts)
    if nb < 0:
        raise ValueError("or_bucket_assignment: too many tensors / keys")
    out, pos = [], 0
    for b in range(nb):
        out.append([members[pos + k] for k in range(counts[b])])
        pos += counts[b]
    return out
