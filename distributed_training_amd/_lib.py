"""ctypes binding of libgsync (``include/gsync.h``).

The library is the product: every pack / unpack / optimizer / collective on a
GPU tensor goes through it.  If it cannot be loaded the import of this module
still succeeds (so CPU-only tooling can introspect), but every call raises
:class:`GsyncUnavailable` — there is no silent fallback.

``torch`` is imported first on purpose: torch-ROCm ships its own
``libamdhip64.so`` (soname ``libamdhip64.so.7``) and ``librccl.so``
(``librccl.so.1``); loading torch first makes the dynamic loader bind
libgsync's DT_NEEDED entries to those same copies, so one HIP runtime and one
RCCL live in the process (SURVEY.md §5 "RCCL library identity").
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = os.environ.get(
    "GSYNC_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libgsync.so")
)

# ---- constants mirrored from include/gsync.h ----
GS_OK = 0
GS_EINVAL, GS_EHIP, GS_ERCCL, GS_ESTATE, GS_ENOMEM, GS_ENODEV = -1, -2, -3, -4, -5, -6
GS_F32, GS_BF16, GS_F16, GS_F64, GS_I64, GS_I32, GS_U8 = 0, 1, 2, 3, 4, 5, 6
GS_DEV_HOST, GS_DEV_HIP = 0, 1
GS_SUM, GS_PROD, GS_MAX, GS_MIN, GS_AVG = 0, 1, 2, 3, 4
GS_SCALE_NONE, GS_SCALE_MUL, GS_SCALE_DIV = 0, 1, 2
GS_PLAN_SLOTS = 5
GS_RED_GROUPS = 64  # the fused reduction's group sums (one per lane of the folding wave)
GS_RED_PARTIALS = 1024  # gs_sqnorm_partial_out: the caller's buffer, at most this many partial sums
GS_BKT_AUTO_COLLECTIVE = 1
GS_BKT_GRAD_VIEW = 2
GS_BKT_NO_SCALE = 4
GS_BKT_REDUCE_SCATTER = 8
GS_BKT_NO_UNPACK = 16
GS_LAYOUT_NCHW, GS_LAYOUT_NHWC = 0, 1
GS_OP_PACK, GS_OP_UNPACK, GS_OP_SCALE, GS_OP_SQNORM, GS_OP_UNSCALE, GS_OP_SGD, GS_OP_ADAM, GS_OP_SUM = 1, 2, 3, 4, 5, 6, 7, 8

_TORCH_TO_GS = {
    torch.float32: GS_F32,
    torch.bfloat16: GS_BF16,
    torch.float16: GS_F16,
    torch.float64: GS_F64,
    torch.int64: GS_I64,
    torch.int32: GS_I32,
    torch.uint8: GS_U8,
}

_c_int, _c_i64, _c_f, _c_d, _vp = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_void_p
_p_i64 = ctypes.POINTER(ctypes.c_int64)
_p_i32 = ctypes.POINTER(ctypes.c_int32)
_p_u8 = ctypes.POINTER(ctypes.c_uint8)
_p_vp = ctypes.POINTER(ctypes.c_void_p)
_p_f = ctypes.POINTER(ctypes.c_float)

# name -> (restype, argtypes); every symbol declared in include/gsync.h
SIGNATURES = {
    "gs_version": (_c_int, []),
    "gs_last_error": (ctypes.c_char_p, []),
    "gs_device_count": (_c_int, []),
    "gs_set_host_threads": (_c_int, [_c_int]),
    "gs_comm_unique_id_bytes": (_c_int, []),
    "gs_comm_get_unique_id": (_c_int, [_p_u8]),
    "gs_comm_create": (_c_int, [_c_int, _c_int, _p_u8, _c_int, _p_vp]),
    "gs_comm_create_ex": (_c_int, [_c_int, _c_int, _p_u8, _c_int, _c_int, _p_vp]),
    "gs_comm_destroy": (_c_int, [_vp]),
    "gs_comm_abort": (_c_int, [_vp]),
    "gs_comm_set_timeout": (_c_int, [_vp, _c_i64]),
    "gs_comm_status": (_c_int, [_vp, ctypes.c_char_p, _c_int]),
    "gs_comm_rank": (_c_int, [_vp]),
    "gs_comm_world": (_c_int, [_vp]),
    "gs_comm_stream": (_c_int, [_vp, _p_vp]),
    "gs_stream_wait": (_c_int, [_vp, _vp]),
    "gs_allreduce": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _c_int, _vp]),
    "gs_reduce_scatter": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _c_int, _vp]),
    "gs_all_gather": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _vp]),
    "gs_broadcast": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _c_int, _vp]),
    "gs_allreduce_marked": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _c_int, _vp, _vp]),
    "gs_all_gather_marked": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _vp, _vp]),
    "gs_plan_create": (_c_int, [_c_int, _c_int, _c_int, _p_i64, _c_i64, _p_vp]),
    "gs_plan_create_ex": (_c_int, [_c_int, _c_int, _c_int, _p_i64, _c_i64, _c_i64, _p_vp]),
    "gs_plan_destroy": (_c_int, [_vp]),
    "gs_plan_flat_numel": (_c_i64, [_vp]),
    "gs_plan_offsets": (_c_int, [_vp, _p_i64]),
    "gs_plan_n_tasks": (_c_int, [_vp]),
    "gs_plan_task_units": (_c_i64, [_vp]),
    "gs_plan_set_hyper_source": (_c_int, [_vp, _vp]),
    "gs_watchdog_pause": (_c_int, [_c_int]),
    "gs_adam_hyper": (_c_int, [_c_int, _vp, _vp, _c_d, _c_d, _c_d, _vp, _vp, _vp]),
    "gs_plan_timer_enable": (_c_int, [_vp, _c_int]),
    "gs_plan_timer_read": (_c_int, [_vp, _p_f, _p_i32, _c_int]),
    "gs_plan_set_ptrs": (_c_int, [_vp, _c_int, _p_vp, _vp]),
    "gs_pack": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _c_f, _c_int, _vp]),
    "gs_unpack": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _vp]),
    "gs_unpack_check": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "gs_scale": (_c_int, [_vp, _c_int, _c_int, _c_f, _c_int, _vp]),
    "gs_sqnorm": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _vp]),
    "gs_sum": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _vp]),
    "gs_sqnorm_partial": (_c_int, [_vp, _c_int, _c_int, _vp]),
    "gs_plan_set_clip": (_c_int, [_vp, _vp, _c_f, _c_f, _c_f, _c_f, _vp]),
    "gs_plan_set_read_hint": (_c_int, [_vp, _c_int]),
    "gs_sqnorm_partial_out": (_c_int, [_vp, _c_int, _c_int, _vp, _p_i32, _vp]),
    "gs_plan_set_clip_groups": (_c_int, [_vp, _vp, ctypes.c_int32, _c_f, _c_f, _c_f, _c_f, _vp]),
    "gs_clip_scale": (_c_int, [_vp, _c_int, _c_int, _vp]),
    "gs_rng_state_bytes": (_c_int, []),
    "gs_rng_draw_u32": (_c_int, [_vp, _c_i64, _c_i64, _vp]),
    "gs_randperm": (_c_int, [ctypes.c_uint64, _c_i64, _vp]),
    "gs_distributed_sampler_indices": (_c_int, [_c_i64, _c_int, _c_int, _c_int, ctypes.c_uint64, _c_i64, _c_int,
                                                _vp, _c_i64, _p_i64]),
    "gs_crop_flip_params": (_c_int, [_vp, _c_i64, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_i64,
                                     _vp]),
    "gs_image_augment": (_c_int, [_c_int, _c_int, _vp, _vp, _c_i64, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                  _vp, _c_i64, _vp, _c_int, _c_int, _vp, _vp]),
    "gs_clip_coef": (_c_int, [_c_int, _vp, _c_f, _c_f, _vp, _vp, _vp]),
    "gs_unscale_check": (_c_int, [_vp, _c_int, _c_int, _vp, _vp, _vp]),
    "gs_sgd_step": (
        _c_int,
        [_vp, _c_int, _c_int, _c_d, _c_d, _c_d, _c_d, _c_int, _c_int, _c_int, _vp, _vp, _vp],
    ),
    "gs_adam_step": (
        _c_int,
        [_vp, _c_int, _c_int, _c_d, _c_d, _c_d, _c_d, _c_d, _c_int, _c_int, _c_d, _c_d, _vp, _vp, _vp],
    ),
    "gs_compute_bucket_assignment": (
        _c_int,
        [_c_int, _p_i64, _p_i32, _p_i32, _c_int, _p_i64, _p_i32, _p_i32, _p_i32],
    ),
    "gs_bucketer_create": (
        _c_int,
        [_vp, _c_int, _c_int, _c_int, _p_i64, _c_int, _c_int, _p_i32, _p_i32, _c_int, _c_i64, _c_f, _c_int, _p_vp],
    ),
    "gs_bucketer_destroy": (_c_int, [_vp]),
    "gs_bucketer_bucket_numel": (_c_int, [_vp, _c_int, _p_i64]),
    "gs_bucketer_shard_numel": (_c_int, [_vp, _c_int, _p_i64]),
    "gs_bucketer_param_location": (_c_int, [_vp, _c_int, _p_i32, _p_i64]),
    "gs_bucketer_set_bucket_buffer": (_c_int, [_vp, _c_int, _vp]),
    "gs_bucketer_set_shard_buffer": (_c_int, [_vp, _c_int, _vp]),
    "gs_bucketer_prepare": (_c_int, [_vp, _vp]),
    "gs_bucketer_mark_ready": (_c_int, [_vp, _c_int, _vp, _vp, _p_i32, _p_i32]),
    "gs_bucketer_mark_unused": (_c_int, [_vp, _vp, _p_i32, _p_i32]),
    "gs_bucketer_finalize": (_c_int, [_vp, _vp]),
    "gs_bucketer_unpack_bucket": (_c_int, [_vp, _c_int, _vp]),
    "gs_bucketer_set_found_inf": (_c_int, [_vp, _vp]),
    "gs_bucketer_set_div_factor": (_c_int, [_vp, _c_f]),
    "gs_bucketer_set_debug": (_c_int, [_vp, _vp]),
    "gs_bucketer_set_bucket_dtype": (_c_int, [_vp, _c_int, _c_int, _c_int]),
    "gs_bucketer_last_comm_ms": (_c_int, [_vp, _c_int, _p_f]),
    "gs_bucketer_last_timing": (_c_int, [_vp, _c_int, _p_f]),
    "gs_bucketer_set_timeline": (_c_int, [_vp, _c_int]),
    "gs_bucketer_bucket_stream": (_c_int, [_vp, _c_int, ctypes.POINTER(_vp)]),
    "gs_bucketer_set_mark_consumer": (_c_int, [_vp, _vp]),
    "gs_bucketer_first_pack_plan": (_c_int, [_vp, _p_vp]),
}


class GsyncError(RuntimeError):
    """A libgsync entry point returned an error (message from gs_last_error)."""


class GsyncUnavailable(GsyncError):
    """libgsync.so is missing or failed to load."""


_lock = threading.Lock()
_lib = None
_load_error: str | None = None


def _load():
    global _lib, _load_error
    with _lock:
        if _lib is not None or _load_error is not None:
            return
        if not os.path.exists(LIB_PATH):
            _load_error = (
                f"libgsync not built: {LIB_PATH} is missing "
                "(run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C distributed_training_amd/csrc`)"
            )
            return
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the host
            _load_error = f"failed to load {LIB_PATH}: {e}"
            return
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib


def lib():
    """The loaded CDLL; raises GsyncUnavailable (never falls back)."""
    if _lib is None:
        _load()
        if _lib is None:
            raise GsyncUnavailable(_load_error)
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except GsyncUnavailable:
        return False


# the hooks beside the loaded library: lib/, or a variant directory holding its own
# libgsync.so + _gshook.so (A/B runs; _gshook's rpath $ORIGIN resolves its libgsync there)
HOOK_PATH = os.path.join(os.path.dirname(os.path.abspath(LIB_PATH)), "_gshook.so")
if not os.path.exists(HOOK_PATH):
    HOOK_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "_gshook.so")
_hook_mod = None
_hook_error: str | None = None


def hook_module():
    """The _gshook extension (C++ DDP gradient hooks, csrc/gs_torch_hook.cpp),
    or None when it is not built — DDP then keeps its Python hooks, which call
    the same library.  It links the libgsync.so of its own directory, so a
    GSYNC_LIB variant without a _gshook.so beside it disables it."""
    global _hook_mod, _hook_error
    if _hook_mod is not None or _hook_error is not None:
        return _hook_mod
    lib()  # libgsync first: _gshook resolves its symbols from the loaded copy
    if os.path.realpath(LIB_PATH) != os.path.realpath(os.path.join(os.path.dirname(HOOK_PATH), "libgsync.so")):
        _hook_error = f"GSYNC_LIB={LIB_PATH} is not the library _gshook links"
        return None
    if not os.path.exists(HOOK_PATH):
        _hook_error = f"{HOOK_PATH} is not built"
        return None
    import importlib.util

    spec = importlib.util.spec_from_file_location("_gshook", HOOK_PATH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    _hook_mod = mod
    return mod


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = lib().gs_last_error().decode(errors="replace")
        raise GsyncError(f"{what or 'libgsync'} failed ({rc}): {msg}")
    return rc


def gs_dtype(dtype: torch.dtype) -> int:
    try:
        return _TORCH_TO_GS[dtype]
    except KeyError:
        raise TypeError(f"libgsync: unsupported dtype {dtype}") from None


def device_kind(t: torch.Tensor) -> int:
    if t.device.type == "cuda":
        return GS_DEV_HIP
    if t.device.type == "cpu":
        return GS_DEV_HOST
    raise TypeError(f"libgsync: unsupported device {t.device}")


def i64_array(vals):
    arr = (ctypes.c_int64 * max(1, len(vals)))(*vals)
    return arr


def i32_array(vals):
    return (ctypes.c_int32 * max(1, len(vals)))(*vals)


def ptr_array(vals):
    return (ctypes.c_void_p * max(1, len(vals)))(*vals)


def stream_ptr(device: torch.device) -> int | None:
    """hipStream_t of torch's current stream on `device` (None for CPU)."""
    if device.type != "cuda":
        return None
    return torch.cuda.current_stream(device).cuda_stream


# ---- capture-safe destruction.  Freeing a plan / bucketer / communicator
# synchronises streams and frees device memory, which is illegal while a
# stream of this thread records a hipGraph (the recording is invalidated and
# capture_end faults).  Python's garbage collector can run at any allocation,
# including inside a capture (an old DDP / optimizer in a reference cycle): a
# destroy requested then is parked and run at the next safe point.
_deferred: list = []


def _capturing() -> bool:
    try:
        return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    except Exception:  # pragma: no cover - no device / interpreter teardown
        return False


def destroy(fn_name: str, handle) -> None:
    """lib().<fn_name>(handle) now, or after the current capture ends."""
    if _capturing():
        _deferred.append((fn_name, handle))
        return
    getattr(lib(), fn_name)(handle)


def flush_deferred() -> None:
    """Run the destroys parked during a capture (no-op while still capturing)."""
    if not _deferred or _capturing():
        return
    while _deferred:
        fn_name, h = _deferred.pop(0)
        getattr(lib(), fn_name)(h)

