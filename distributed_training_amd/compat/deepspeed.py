"""DeepSpeed API subset used by R:resnet/deepspeed/deepspeed_train.py, on libgsync.

Covered surface:
  deepspeed.init_distributed()                             :168
  deepspeed.add_config_arguments(parser)                    :125
  deepspeed.initialize(args, model, model_parameters, training_data, config)
      -> (engine, optimizer, dataloader, lr_scheduler)      :236-237
  engine.backward(loss) / engine.step() / engine.local_rank :154-155, :241
  engine.bfloat16_enabled() / fp16_enabled()                :245-248
  deepspeed.accelerator.get_accelerator().device_name(i)    :240
  the config keys of :172-220 (train_batch_size, optimizer Adam/AdamW/SGD,
  WarmupLR, gradient_clipping, bf16 / fp16 (dynamic loss scale), zero_optimization
  stage 0-2 with reduce_bucket_size / allgather_bucket_size / overlap_comm).
  engine.save_checkpoint / load_checkpoint (DeepSpeed's directory layout) and
  consolidated_fp32_state_dict (zero_to_fp32), for resume — the reference
  itself never saves.

Mapping: stage 0 in fp32 -> libgsync DDP (bucketed RCCL all-reduce + fused
optimizer); stage 0 with bf16/fp16 (DeepSpeed's BF16_Optimizer / FP16
optimizer keep a DP-partitioned fp32 master) and stage 1 -> ZeRO-1; stage 2 ->
ZeRO-2 (reduce-scatter).  DeepSpeed's "Adam" is its FusedAdam in AdamW mode.
DeepSpeed itself is not installed here: its numerics are restated from the
published algorithm, parity unpinned.
"""
from __future__ import annotations

import argparse
import json
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ddp import DistributedDataParallel
from ..optim import FusedAdam, FusedSGD
from ..zero import DynamicLossScaler, ZeroDataParallel, warmup_lr


def _env_int(name, default):
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


def init_distributed(dist_backend=None, auto_mpi_discovery=True, distributed_port=29500, verbose=True,
                     timeout=None, init_method=None, dist_init_required=None, config=None, rank=-1,
                     world_size=-1):
    """Initialise torch.distributed from the launcher's env (RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT / LOCAL_RANK); nccl (= RCCL) on GPUs, gloo on CPU."""
    if dist.is_initialized():
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(distributed_port))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    if dist_backend is None:
        dist_backend = "nccl" if torch.cuda.is_available() else "gloo"
    if dist_backend == "nccl":
        torch.cuda.set_device(_env_int("LOCAL_RANK", 0))
    kw = {}
    if timeout is not None:
        kw["timeout"] = timeout
    dist.init_process_group(dist_backend, init_method=init_method,
                            rank=rank if rank >= 0 else _env_int("RANK", 0),
                            world_size=world_size if world_size >= 0 else _env_int("WORLD_SIZE", 1), **kw)


def add_config_arguments(parser: argparse.ArgumentParser):
    group = parser.add_argument_group("DeepSpeed", "DeepSpeed configurations")
    group.add_argument("--deepspeed", default=False, action="store_true", help="Enable DeepSpeed")
    group.add_argument("--deepspeed_config", default=None, type=str, help="DeepSpeed json configuration file.")
    group.add_argument("--deepscale", default=False, action="store_true", help=argparse.SUPPRESS)
    group.add_argument("--deepscale_config", default=None, type=str, help=argparse.SUPPRESS)
    return parser


class _Accelerator:
    def device_name(self, device_index=None):
        if not torch.cuda.is_available():
            return "cpu"
        return "cuda" if device_index is None else f"cuda:{device_index}"

    def current_device_name(self):
        return self.device_name(torch.cuda.current_device() if torch.cuda.is_available() else None)

    def device_count(self):
        return torch.cuda.device_count()

    def is_available(self):
        return torch.cuda.is_available()

    def communication_backend_name(self):
        return "nccl" if torch.cuda.is_available() else "gloo"


_ACCEL = _Accelerator()


def get_accelerator():
    return _ACCEL


class WarmupLR:
    """DeepSpeed WarmupLR (config :187-194); stepped once per optimizer step."""

    def __init__(self, optimizer, warmup_min_lr=0.0, warmup_max_lr=0.001, warmup_num_steps=1000,
                 warmup_type="log", last_batch_iteration=-1):
        self.optimizer = optimizer
        self.min_lr = warmup_min_lr
        self.max_lr = warmup_max_lr
        self.warmup_num_steps = max(2, warmup_num_steps)
        self.warmup_type = warmup_type
        # DeepSpeed's published schedule: construction leaves warmup_min_lr in the
        # optimizer; step() (after each optimizer step) sets last_batch_iteration
        # += 1 and lr = min + (max - min) * gamma(last_batch_iteration) with
        # gamma(i) = log(i + 1) / log(N) — lrs of steps 1, 2, 3: min, min, gamma(1)
        self.last_batch_iteration = last_batch_iteration
        self._set(self.min_lr if last_batch_iteration < 0 else self.get_lr()[0])

    def get_lr(self):
        if self.last_batch_iteration < 0:  # DeepSpeed warns "before it has started" and returns [0.0]
            return [0.0]
        return [warmup_lr(self.last_batch_iteration, self.min_lr, self.max_lr, self.warmup_num_steps,
                          self.warmup_type)]

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def _set(self, lr):
        for g in self.optimizer.param_groups:
            g["lr"] = lr

    def step(self, last_batch_iteration=None):
        self.last_batch_iteration = self.last_batch_iteration + 1 if last_batch_iteration is None else last_batch_iteration
        self._set(self.get_lr()[0])

    def state_dict(self):
        return {"last_batch_iteration": self.last_batch_iteration}

    def load_state_dict(self, sd):
        self.last_batch_iteration = sd["last_batch_iteration"]
        self._set(self.min_lr if self.last_batch_iteration < 0 else self.get_lr()[0])


class DeepSpeedEngine(nn.Module):
    def __init__(self, model: nn.Module, config: dict, model_parameters=None, training_data=None, args=None):
        super().__init__()
        if not dist.is_initialized():
            init_distributed()
        self.config = config
        self.world_size = dist.get_world_size()
        self.global_rank = dist.get_rank()
        self.local_rank = _env_int("LOCAL_RANK", getattr(args, "local_rank", 0) if args is not None else 0)
        if self.local_rank < 0:
            self.local_rank = 0
        self.device = torch.device("cuda", self.local_rank) if torch.cuda.is_available() else torch.device("cpu")
        self._bf16 = bool(config.get("bf16", {}).get("enabled", False))
        fp16cfg = config.get("fp16", {})
        self._fp16 = bool(fp16cfg.get("enabled", False))
        dtype = torch.bfloat16 if self._bf16 else (torch.float16 if self._fp16 else torch.float32)
        self.module = model.to(self.device).to(dtype)
        # batch bookkeeping: train_batch_size = micro * gas * world
        tbs = config.get("train_batch_size")
        micro = config.get("train_micro_batch_size_per_gpu")
        gas = config.get("gradient_accumulation_steps")
        if micro is None and gas is None:
            gas = 1
            micro = tbs // self.world_size
        elif micro is None:
            micro = tbs // (self.world_size * gas)
        elif gas is None:
            gas = max(1, (tbs or micro * self.world_size) // (micro * self.world_size))
        self._micro, self._gas = int(micro), int(gas)
        self._tbs = self._micro * self._gas * self.world_size
        self.micro_steps = 0
        self.global_steps = 0
        self.skipped_steps = 0
        self.clip = float(config.get("gradient_clipping", 0.0) or 0.0)
        opt_cfg = config.get("optimizer", {"type": "Adam", "params": {}})
        otype = opt_cfg.get("type", "Adam").lower()
        p = dict(opt_cfg.get("params", {}))
        lr = p.get("lr", 1e-3)
        zcfg = config.get("zero_optimization", {})
        stage = int(zcfg.get("stage", 0)) if isinstance(zcfg, dict) else int(zcfg)
        if stage == 3:
            raise NotImplementedError("ZeRO stage 3 is outside the gradient-sync path (SURVEY.md §2.3)")
        self.zero_stage = stage
        scaler = None
        if self._fp16:
            ls = float(fp16cfg.get("loss_scale", 0))
            scaler = DynamicLossScaler(init_scale=2.0 ** fp16cfg.get("initial_scale_power", 16) if ls == 0 else ls,
                                       scale_window=fp16cfg.get("loss_scale_window", 1000),
                                       hysteresis=fp16cfg.get("hysteresis", 2),
                                       min_scale=fp16cfg.get("min_loss_scale", 1), dynamic=ls == 0)
        self.loss_scaler = scaler
        if otype in ("adam", "adamw", "fusedadam"):
            # DeepSpeed "Adam" = FusedAdam(adam_w_mode=True) unless torch_adam / adam_w_mode False
            adamw = otype == "adamw" or p.get("adam_w_mode", True)
            kind = "adamw" if adamw else "adam"
        elif otype == "sgd":
            kind = "sgd"
        else:
            raise NotImplementedError(f"optimizer type {opt_cfg.get('type')} is not on the gradient-sync path")
        betas = tuple(p.get("betas", (0.9, 0.999)))
        eps = p.get("eps", 1e-8)
        wd = p.get("weight_decay", 0.0)
        use_zero = stage in (1, 2) or dtype != torch.float32
        self._ddp = None
        self._zero = None
        if use_zero:
            self._zero = ZeroDataParallel(
                self.module, stage=max(1, stage), optimizer=kind, lr=lr, betas=betas, eps=eps, weight_decay=wd,
                momentum=p.get("momentum", 0.0), reduce_bucket_size=int(zcfg.get("reduce_bucket_size", 5e8)
                                                                      if isinstance(zcfg, dict) else 5e8),
                gradient_clipping=self.clip, loss_scaler=scaler,
                # libgsync extension keys (DeepSpeed ignores unknown ones): per-bucket parameter
                # all-gathers under the next forward instead of DeepSpeed's end-of-step gather
                overlap_allgather=bool(isinstance(zcfg, dict) and zcfg.get("overlap_allgather", False)),
                allgather_bucket_size=(zcfg.get("overlap_allgather_bucket_size") if isinstance(zcfg, dict)
                                       else None))
            self.optimizer = self._zero
        else:
            self._ddp = DistributedDataParallel(self.module, broadcast_buffers=False)
            if kind == "sgd":
                self.optimizer = FusedSGD(self.module.parameters(), lr=lr, momentum=p.get("momentum", 0.0),
                                          weight_decay=wd, max_grad_norm=self.clip or None)
            else:
                self.optimizer = FusedAdam(self.module.parameters(), lr=lr, betas=betas, eps=eps, weight_decay=wd,
                                           adamw=kind == "adamw", max_grad_norm=self.clip or None)
        sched = config.get("scheduler")
        self.lr_scheduler = None
        if sched is not None:
            if sched.get("type") != "WarmupLR":
                raise NotImplementedError(f"scheduler {sched.get('type')} not provided")
            self.lr_scheduler = WarmupLR(self.optimizer, **sched.get("params", {}))
        self.training_dataloader = None
        if training_data is not None:
            sampler = torch.utils.data.distributed.DistributedSampler(training_data)
            self.training_dataloader = torch.utils.data.DataLoader(training_data, batch_size=self._micro,
                                                                   sampler=sampler)

    # ---- DeepSpeedEngine surface
    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def is_gradient_accumulation_boundary(self):
        return (self.micro_steps + 1) % self._gas == 0

    def backward(self, loss, retain_graph=False):
        boundary = self.is_gradient_accumulation_boundary()
        if self._gas > 1:
            loss = loss / self._gas
        if self.loss_scaler is not None:
            loss = loss.float() * self.loss_scaler.scale
        if self._zero is not None:
            self._zero.require_backward_grad_sync = boundary
            self._zero.prepare_backward()
        else:
            d = self._ddp
            d.require_backward_grad_sync = boundary
            if boundary:
                # the reference calls the raw module (R:deepspeed_train.py:150), so the
                # wrapper's forward-side bookkeeping runs here
                d._maybe_rebuild_buckets()
                d._prepare_for_backward()
        loss.backward(retain_graph=retain_graph)
        return loss

    def step(self, lr_kwargs=None):
        boundary = self.is_gradient_accumulation_boundary()
        self.micro_steps += 1
        if not boundary:
            return
        if self._zero is not None:
            ok = self._zero.step()
            self._zero.zero_grad()
        else:
            self.optimizer.step()
            self.optimizer.zero_grad(set_to_none=True)
            ok = True
        if ok:
            self.global_steps += 1
            if self.lr_scheduler is not None:
                self.lr_scheduler.step(**(lr_kwargs or {}))
        else:
            self.skipped_steps += 1

    def bfloat16_enabled(self):
        return self._bf16

    def fp16_enabled(self):
        return self._fp16

    def train_batch_size(self):
        return self._tbs

    def train_micro_batch_size_per_gpu(self):
        return self._micro

    def gradient_accumulation_steps(self):
        return self._gas

    def get_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def zero_optimization_stage(self):
        return self.zero_stage

    # ---- checkpoints (DeepSpeed's directory layout; the reference never saves,
    # R:resnet/deepspeed/deepspeed_train.py:252 start_epoch = 0)
    #   <dir>/<tag>/mp_rank_00_model_states.pt             rank 0: module state_dict (model dtype,
    #                                                       torchvision keys) + engine counters
    #   <dir>/<tag>/zero_pp_rank_<r>_mp_rank_00_optim_states.pt   every rank: its ZeRO shard
    #                                                       (fp32 master + moments)   [ZeRO]
    #   <dir>/<tag>/optim_states.pt                        rank 0: optimizer state_dict  [no ZeRO]
    #   <dir>/latest                                        the tag
    def save_checkpoint(self, save_dir, tag=None, client_state=None, save_latest=True):
        tag = f"global_step{self.global_steps}" if tag is None else str(tag)
        path = os.path.join(save_dir, tag)
        rank = self.global_rank
        if self._zero is not None:
            # overlap_allgather: the last step's parameter all-gathers may still run on the
            # communicator's stream; the module state read below must follow them
            self._zero.wait_allgather()
        if rank == 0:
            os.makedirs(path, exist_ok=True)
        dist.barrier()
        if rank == 0:
            torch.save({"module": {k: v.detach().cpu() for k, v in self.module.state_dict().items()},
                        "global_steps": self.global_steps, "skipped_steps": self.skipped_steps,
                        "micro_steps": self.micro_steps,
                        "lr_scheduler": None if self.lr_scheduler is None else self.lr_scheduler.state_dict(),
                        "client_state": client_state or {}, "dp_world_size": self.world_size,
                        "zero_stage": self.zero_stage}, os.path.join(path, "mp_rank_00_model_states.pt"))
        if self._zero is not None:
            torch.save(self._zero.state_dict(), os.path.join(path, f"zero_pp_rank_{rank}_mp_rank_00_optim_states.pt"))
        elif rank == 0:
            torch.save(self.optimizer.state_dict(), os.path.join(path, "optim_states.pt"))
        dist.barrier()
        if save_latest and rank == 0:
            with open(os.path.join(save_dir, "latest"), "w") as f:
                f.write(tag)
        dist.barrier()
        return True

    def load_checkpoint(self, load_dir, tag=None, load_optimizer_states=True, load_lr_scheduler_states=True):
        if tag is None:
            latest = os.path.join(load_dir, "latest")
            if not os.path.exists(latest):
                return None, None
            with open(latest) as f:
                tag = f.read().strip()
        path = os.path.join(load_dir, str(tag))
        if self._zero is not None:
            self._zero.wait_allgather()  # a pending all-gather must not land on the loaded parameters
        ms = torch.load(os.path.join(path, "mp_rank_00_model_states.pt"), map_location="cpu", weights_only=True)
        if ms["dp_world_size"] != self.world_size and self._zero is not None:
            raise RuntimeError(f"checkpoint has {ms['dp_world_size']} ZeRO shards, this job {self.world_size}")
        with torch.no_grad():
            self.module.load_state_dict(ms["module"])
        self.global_steps, self.skipped_steps = ms["global_steps"], ms["skipped_steps"]
        self.micro_steps = ms.get("micro_steps", 0)
        if load_lr_scheduler_states and self.lr_scheduler is not None and ms.get("lr_scheduler") is not None:
            self.lr_scheduler.load_state_dict(ms["lr_scheduler"])
        if load_optimizer_states:
            if self._zero is not None:
                f = os.path.join(path, f"zero_pp_rank_{self.global_rank}_mp_rank_00_optim_states.pt")
                self._zero.load_state_dict(torch.load(f, map_location="cpu", weights_only=True))
            else:
                self.optimizer.load_state_dict(torch.load(os.path.join(path, "optim_states.pt"),
                                                          map_location="cpu", weights_only=True))
        return path, ms.get("client_state", {})

    def consolidated_fp32_state_dict(self):
        """zero_to_fp32: the full fp32 model state_dict (collective under ZeRO)."""
        if self._zero is not None:
            return self._zero.consolidated_state_dict()  # waits for pending all-gathers itself
        return {k: v.detach().float().cpu() if v.is_floating_point() else v.detach().cpu()
                for k, v in self.module.state_dict().items()}


def initialize(args=None, model=None, optimizer=None, model_parameters=None, training_data=None, lr_scheduler=None,
               distributed_port=29500, mpu=None, dist_init_required=None, collate_fn=None, config=None,
               config_params=None, **kw):
    if config is None:
        config = config_params
    if config is None and args is not None and getattr(args, "deepspeed_config", None):
        with open(args.deepspeed_config) as f:
            config = json.load(f)
    if isinstance(config, str):
        with open(config) as f:
            config = json.load(f)
    if config is None:
        raise ValueError("DeepSpeed config required")
    if optimizer is not None or lr_scheduler is not None:
        raise NotImplementedError("client optimizers / schedulers: use the config's optimizer section")
    engine = DeepSpeedEngine(model, config, model_parameters, training_data, args)
    return engine, engine.optimizer, engine.training_dataloader, engine.lr_scheduler
