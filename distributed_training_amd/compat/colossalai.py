"""ColossalAI API subset used by R:resnet/colossal/colossal_train.py, on libgsync.

Covered surface:
  colossalai.launch_from_torch(config={})                      :110
  DistCoordinator(): world_size, is_master(), priority_execution()  :65,88,111,122
  Booster(plugin=..., mixed_precision='fp16')                  :138
  booster.boost(model, optimizer, criterion=...)               :159-161
  booster.backward(loss, optimizer)                            :100
  plugin.prepare_dataloader(ds, batch_size, shuffle, drop_last) :76-77
  TorchDDPPlugin(), LowLevelZeroPlugin(initial_scale=2**5)     :132,136
  HybridAdam(params, lr); optimizer.step() / zero_grad()       :153, :101-102

TorchDDPPlugin -> libgsync DistributedDataParallel (+ fp16 autocast and the
libgsync GradScaler for mixed_precision='fp16', the run.sh default).
LowLevelZeroPlugin -> libgsync ZeRO (stage 1 default, fp16 params, fp32
master, dynamic loss scale).  HybridAdam -> libgsync FusedAdam (AdamW mode,
Colossal's default).  ColossalAI is not installed here: its numerics are
restated from the published algorithm, parity unpinned.
"""
from __future__ import annotations

import contextlib
import os
import random

import torch
import torch.distributed as dist
import torch.nn as nn

from ..amp import GradScaler
from ..ddp import DistributedDataParallel
from ..optim import FusedAdam
from ..zero import DynamicLossScaler, ZeroDataParallel


def launch_from_torch(config=None, seed: int = 1024, verbose: bool = True, backend=None):
    """torchrun env -> process group (nccl = RCCL on GPUs, gloo on CPU), device, seed."""
    if not dist.is_initialized():
        backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend, rank=int(os.environ.get("RANK", "0")),
                                world_size=int(os.environ.get("WORLD_SIZE", "1")))
    random.seed(seed)
    torch.manual_seed(seed)


def get_current_device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class DistCoordinator:
    def __init__(self):
        if not dist.is_initialized():
            raise RuntimeError("launch_from_torch() first")
        self.rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    def is_master(self):
        return self.rank == 0

    @contextlib.contextmanager
    def priority_execution(self):
        """Master runs the block first (e.g. a dataset download), then the others."""
        if not self.is_master():
            dist.barrier()
        yield
        if self.is_master():
            dist.barrier()

    def print_on_master(self, *a, **k):
        if self.is_master():
            print(*a, **k)


class HybridAdam(FusedAdam):
    def __init__(self, model_params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, adamw_mode=True, nvme_offload_fraction=0.0, nvme_offload_dir=None, **kw):
        if not bias_correction:
            raise NotImplementedError("bias_correction=False")
        # capturable (not a Colossal argument): device step counters / lr, for CapturedStep
        super().__init__(model_params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw=adamw_mode,
                         capturable=bool(kw.pop("capturable", False)))
        self.colossal_kwargs = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw_mode=adamw_mode)


class _DPPluginBase:
    def prepare_dataloader(self, dataset, batch_size, shuffle=False, seed=1024, drop_last=False, pin_memory=False,
                           num_workers=0, **kwargs):
        sampler = torch.utils.data.distributed.DistributedSampler(dataset, shuffle=shuffle, seed=seed,
                                                                  drop_last=drop_last)
        return torch.utils.data.DataLoader(dataset, batch_size=batch_size, sampler=sampler, drop_last=drop_last,
                                           pin_memory=pin_memory, num_workers=num_workers, **kwargs)


class _AutocastModule(nn.Module):
    def __init__(self, module, dtype):
        super().__init__()
        self.module = module
        self.dtype = dtype

    def forward(self, *a, **k):
        with torch.autocast(get_current_device().type, dtype=self.dtype):
            return self.module(*a, **k)


class _OptimizerWrapper:
    """Booster's OptimizerWrapper: backward / step / zero_grad, optional GradScaler."""

    def __init__(self, optim, scaler: GradScaler | None = None):
        self.optim = optim
        self.scaler = scaler

    @property
    def param_groups(self):
        return self.optim.param_groups

    def backward(self, loss):
        (self.scaler.scale(loss) if self.scaler is not None else loss).backward()

    def step(self, *a, **k):
        if self.scaler is None:
            return self.optim.step(*a, **k)
        out = self.scaler.step(self.optim, *a, **k)
        self.scaler.update()
        return out

    def zero_grad(self, set_to_none=True):
        self.optim.zero_grad(set_to_none=set_to_none)

    def state_dict(self):
        sd = {"optim": self.optim.state_dict()}
        if self.scaler is not None:
            sd["scaler"] = self.scaler.state_dict()
        return sd

    def load_state_dict(self, sd):
        self.optim.load_state_dict(sd["optim"])
        if self.scaler is not None and "scaler" in sd:
            self.scaler.load_state_dict(sd["scaler"])


def _unwrap(model):
    """The user's nn.Module under the booster's wrappers (autocast / cast / DDP)."""
    m = model
    while hasattr(m, "module") and isinstance(m.module, nn.Module):
        m = m.module
    return m


class TorchDDPPlugin(_DPPluginBase):
    def __init__(self, broadcast_buffers=True, bucket_cap_mb=25, find_unused_parameters=False,
                 check_reduction=False, gradient_as_bucket_view=False, static_graph=False):
        self.ddp_kwargs = dict(broadcast_buffers=broadcast_buffers, bucket_cap_mb=bucket_cap_mb,
                               find_unused_parameters=find_unused_parameters,
                               gradient_as_bucket_view=gradient_as_bucket_view, static_graph=static_graph)

    def configure(self, model, optimizer, mixed_precision):
        model = model.to(get_current_device())
        ddp = DistributedDataParallel(model, **self.ddp_kwargs)
        wrapped = ddp
        scaler = None
        if mixed_precision == "fp16":
            wrapped = _AutocastModule(ddp, torch.float16)
            scaler = GradScaler(device=get_current_device())
            if isinstance(optimizer, FusedAdam):
                scaler.fuse_check_into(ddp)  # inf check inside the bucket unpack
        elif mixed_precision == "bf16":
            wrapped = _AutocastModule(ddp, torch.bfloat16)
        return wrapped, _OptimizerWrapper(optimizer, scaler)


class _ZeroOptimizerWrapper:
    def __init__(self, zero: ZeroDataParallel):
        self.zero = zero

    @property
    def param_groups(self):
        return self.zero.param_groups

    def backward(self, loss):
        self.zero.prepare_backward()
        scale = self.zero.scaler.scale if self.zero.scaler is not None else 1.0
        (loss.float() * scale).backward()

    def step(self):
        return self.zero.step()

    def zero_grad(self, set_to_none=True):
        self.zero.zero_grad()

    def state_dict(self):
        return self.zero.state_dict()

    def load_state_dict(self, sd):
        self.zero.load_state_dict(sd)


class _CastInputs(nn.Module):
    def __init__(self, module, dtype):
        super().__init__()
        self.module = module
        self.dtype = dtype

    def forward(self, *a, **k):
        a = tuple(x.to(self.dtype) if torch.is_tensor(x) and x.is_floating_point() else x for x in a)
        out = self.module(*a, **k)
        return out.float() if torch.is_tensor(out) else out


class LowLevelZeroPlugin(_DPPluginBase):
    def __init__(self, stage=1, precision="fp16", initial_scale=2 ** 32, min_scale=1, growth_factor=2,
                 backoff_factor=0.5, growth_interval=1000, hysteresis=2, max_scale=2 ** 32, max_norm=0.0,
                 reduce_bucket_size_in_m=12, **kwargs):
        self.stage = stage
        self.precision = precision
        self.scaler_kw = dict(init_scale=float(initial_scale), scale_window=growth_interval, hysteresis=hysteresis,
                              min_scale=float(min_scale), scale_factor=float(growth_factor))
        self.max_norm = max_norm
        self.bucket = int(reduce_bucket_size_in_m * 1024 * 1024)

    def configure(self, model, optimizer, mixed_precision):
        dtype = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[self.precision]
        model = model.to(get_current_device()).to(dtype)
        hp = getattr(optimizer, "colossal_kwargs", None) or dict(
            lr=optimizer.param_groups[0]["lr"], betas=optimizer.param_groups[0].get("betas", (0.9, 0.999)),
            eps=optimizer.param_groups[0].get("eps", 1e-8), weight_decay=optimizer.param_groups[0].get("weight_decay", 0.0),
            adamw_mode=True)
        scaler = DynamicLossScaler(**self.scaler_kw) if dtype == torch.float16 else None
        zero = ZeroDataParallel(model, stage=self.stage, optimizer="adamw" if hp["adamw_mode"] else "adam",
                                lr=hp["lr"], betas=hp["betas"], eps=hp["eps"], weight_decay=hp["weight_decay"],
                                reduce_bucket_size=self.bucket, gradient_clipping=self.max_norm, loss_scaler=scaler)
        return _CastInputs(model, dtype), _ZeroOptimizerWrapper(zero)


class GeminiPlugin(_DPPluginBase):  # referenced but unreachable in the reference (R:colossal_train.py:133-134)
    def __init__(self, *a, **k):
        raise NotImplementedError("Gemini is outside the gradient-sync path (unreachable in the reference)")


class Booster:
    def __init__(self, device=None, mixed_precision=None, plugin=None):
        self.plugin = plugin if plugin is not None else TorchDDPPlugin()
        self.mixed_precision = mixed_precision

    def boost(self, model, optimizer=None, criterion=None, dataloader=None, lr_scheduler=None):
        model, optimizer = self.plugin.configure(model, optimizer, self.mixed_precision)
        self._zero = optimizer.zero if isinstance(optimizer, _ZeroOptimizerWrapper) else None
        amp = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(self.mixed_precision)
        if criterion is not None and amp is not None and isinstance(self.plugin, TorchDDPPlugin):
            # Colossal's FP16TorchMixedPrecision.configure wraps the criterion in
            # the autocast module too: the loss is computed in fp32 under autocast
            criterion = _AutocastModule(criterion, amp)
        return model, optimizer, criterion, dataloader, lr_scheduler

    def backward(self, loss, optimizer):
        optimizer.backward(loss)

    # ---- checkpoint I/O (Booster.save_model / load_model / save_optimizer / load_optimizer).
    # The reference parses -c/--checkpoint but never saves (R:colossal_train.py:40-42); the
    # layout kept is the model's torchvision-keyed state_dict, unsharded (shard=False):
    # for LowLevelZero the fp32 master values gathered from every rank's shard.
    def save_model(self, model, checkpoint: str, shard: bool = False, **kw):
        if shard:
            raise NotImplementedError("sharded model checkpoints are not on the reference path")
        zero = getattr(self, "_zero", None)
        sd = zero.consolidated_state_dict() if zero is not None else {
            k: v.detach().cpu() for k, v in _unwrap(model).state_dict().items()}
        if not dist.is_initialized() or dist.get_rank() == 0:
            torch.save(sd, checkpoint)
        if dist.is_initialized():
            dist.barrier()

    def load_model(self, model, checkpoint: str, strict: bool = True):
        sd = torch.load(checkpoint, map_location="cpu", weights_only=True)
        zero = getattr(self, "_zero", None)
        if zero is not None:
            zero.load_consolidated_state_dict(sd)
        else:
            target = _unwrap(model)
            target.load_state_dict({k: v.to(target.state_dict()[k].dtype) for k, v in sd.items()}, strict=strict)

    def save_optimizer(self, optimizer, checkpoint: str, shard: bool = False, **kw):
        """One file per rank for ZeRO (its shard), one file from rank 0 otherwise."""
        rank = dist.get_rank() if dist.is_initialized() else 0
        if getattr(self, "_zero", None) is not None:
            torch.save(optimizer.state_dict(), f"{checkpoint}.rank{rank}")
        elif rank == 0:
            torch.save(optimizer.state_dict(), checkpoint)
        if dist.is_initialized():
            dist.barrier()

    def load_optimizer(self, optimizer, checkpoint: str):
        rank = dist.get_rank() if dist.is_initialized() else 0
        path = f"{checkpoint}.rank{rank}" if getattr(self, "_zero", None) is not None else checkpoint
        optimizer.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
