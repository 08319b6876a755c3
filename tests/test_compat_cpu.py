"""DeepSpeed / ColossalAI API shims on CPU/gloo (world_size 2), driven the way
R:resnet/deepspeed/deepspeed_train.py:142-158 and
R:resnet/colossal/colossal_train.py:87-105 drive the real libraries.
DeepSpeed / ColossalAI are not installed here, so their own numerics are
parity-unpinned; these tests pin the plumbing and the identities that hold
(replicas agree, ZeRO stages agree with the DDP path, schedule shape)."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

from tests.test_ddp_cpu import _micro, _run

SHIMS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed_training_amd",
                     "compat", "shims")

# the reference's ds_config (R:resnet/deepspeed/deepspeed_train.py:172-220), CPU-sized batch
DS_CONFIG = {
    "train_batch_size": 8,
    "steps_per_print": 2000,
    "optimizer": {"type": "Adam", "params": {"lr": 0.001, "betas": [0.8, 0.999], "eps": 1e-8, "weight_decay": 3e-7}},
    "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0, "warmup_max_lr": 0.001, "warmup_num_steps": 1000}},
    "gradient_clipping": 1.0,
    "prescale_gradients": False,
    "bf16": {"enabled": False},
    "fp16": {"enabled": False},
    "wall_clock_breakdown": False,
    "zero_optimization": {"stage": 0, "allgather_partitions": True, "reduce_scatter": True,
                          "allgather_bucket_size": 50000000, "reduce_bucket_size": 50000000,
                          "overlap_comm": True, "contiguous_gradients": True, "cpu_offload": False},
}


def _dataset(n=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.utils.data.TensorDataset(torch.rand(n, 3, 32, 32, generator=g), torch.randint(0, 10, (n,), generator=g))


def _ds_run(rank, ws, stage, bf16, overlap=False):
    sys.path.insert(0, SHIMS)
    import copy

    import deepspeed
    from deepspeed.accelerator import get_accelerator

    deepspeed.init_distributed()  # already initialised: no-op
    cfg = copy.deepcopy(DS_CONFIG)
    cfg["zero_optimization"]["stage"] = stage
    cfg["bf16"]["enabled"] = bf16
    if overlap:  # libgsync's opt-in keys: per-bucket all-gathers under the next forward
        cfg["zero_optimization"]["overlap_allgather"] = True
        cfg["zero_optimization"]["overlap_allgather_bucket_size"] = 2000
    torch.manual_seed(123)
    model = _micro()
    params = filter(lambda p: p.requires_grad, model.parameters())
    engine, opt, loader, sched = deepspeed.initialize(args=None, model=model, model_parameters=params,
                                                      training_data=_dataset(), config=cfg)
    if overlap:
        assert engine._zero.overlap_allgather and len(engine._zero.buckets) > 2
    assert get_accelerator().device_name(engine.local_rank) in ("cpu", f"cuda:{engine.local_rank}")
    assert engine.train_micro_batch_size_per_gpu() == 8 // ws
    target = torch.bfloat16 if engine.bfloat16_enabled() else None
    crit = nn.CrossEntropyLoss()
    lrs = []
    before = [p.detach().clone() for p in model.parameters()]
    for i, (images, labels) in enumerate(loader):
        if target is not None:
            images = images.to(target)
        outputs = model(images)  # the raw module, as the reference does
        loss = crit(outputs, labels)
        engine.backward(loss)
        engine.step()
        lrs.append(engine.get_lr()[0])
        assert torch.isfinite(loss.float()).item()
        if i == 2:
            break
    # WarmupLR (DeepSpeed schedule): the lr after steps 1..3 is gamma(0) = 0, gamma(1), gamma(2)
    assert lrs[0] == 0.0 and 0 < lrs[1] < lrs[2] < 1e-3
    changed = sum(int(not torch.equal(a, b)) for a, b in zip(before, model.parameters()))
    assert changed > 0
    w = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()])
    allw = [torch.zeros_like(w) for _ in range(ws)]
    dist.all_gather(allw, w)
    assert torch.equal(allw[0], allw[1]), "replicas diverged"
    return w


@pytest.mark.parametrize("stage,bf16", [(0, False), (1, False), (2, False), (2, True), (0, True)])
def test_deepspeed_shim(stage, bf16):
    _run(_ds_run, 2, stage, bf16)


def _ds_overlap_vs_default(rank, ws):
    a = _ds_run(rank, ws, 2, False)
    b = _ds_run(rank, ws, 2, False, overlap=True)
    # the reference's gradient_clipping 1.0: its Σg² is summed per bucket layout, so the two
    # engines agree to fp32 rounding (bit for bit with the clip off, tests/test_zero_ds_step.py)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


def test_deepspeed_shim_overlap_allgather():
    """zero_optimization.overlap_allgather (libgsync's opt-in key) through the
    DeepSpeed shim: the reference's loop, per-bucket gathers awaited by each
    module's forward, the same weights as the default engine."""
    _run(_ds_overlap_vs_default, 2)


def _col_run(rank, ws, plugin_name, mp):
    sys.path.insert(0, SHIMS)
    import colossalai
    from colossalai.booster import Booster
    from colossalai.booster.plugin import LowLevelZeroPlugin, TorchDDPPlugin
    from colossalai.cluster import DistCoordinator
    from colossalai.nn.optimizer import HybridAdam

    colossalai.launch_from_torch(config={})
    coordinator = DistCoordinator()
    lr = 1e-3 * coordinator.world_size
    kwargs = {}
    if mp:
        kwargs["mixed_precision"] = mp
    if plugin_name == "torch_ddp":
        plugin = TorchDDPPlugin()
    else:
        plugin = LowLevelZeroPlugin(initial_scale=2 ** 5, precision="fp32")
    booster = Booster(plugin=plugin, **kwargs)
    with coordinator.priority_execution():
        ds = _dataset()
    loader = plugin.prepare_dataloader(ds, batch_size=4, shuffle=False, drop_last=True)
    model = _micro()
    crit = nn.CrossEntropyLoss()
    optimizer = HybridAdam(model.parameters(), lr=lr)
    model, optimizer, crit, _, _ = booster.boost(model, optimizer, criterion=crit)
    model.train()
    for i, (images, labels) in enumerate(loader):
        outputs = model(images)
        loss = crit(outputs, labels)
        booster.backward(loss, optimizer)
        optimizer.step()
        optimizer.zero_grad()
        assert torch.isfinite(loss.float()).item()
        if i == 2:
            break
    w = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()])
    allw = [torch.zeros_like(w) for _ in range(ws)]
    dist.all_gather(allw, w)
    assert torch.equal(allw[0], allw[1])


@pytest.mark.parametrize("plugin,mp", [("torch_ddp", None), ("torch_ddp", "bf16"), ("low_level_zero", None)])
def test_colossal_shim(plugin, mp):
    _run(_col_run, 2, plugin, mp)


def test_warmup_lr_schedule_matches_deepspeed():
    """DeepSpeed WarmupLR (R:resnet/deepspeed/deepspeed_train.py:187-194): the lrs
    the first three optimizer steps run with are [min, min, min + (max-min)*log2/logN]
    (construction sets min; each scheduler.step() after an optimizer step
    advances last_batch_iteration and sets gamma(last_batch_iteration))."""
    import math

    sys.path.insert(0, SHIMS)
    from distributed_training_amd.compat.deepspeed import WarmupLR

    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=123.0)
    sch = WarmupLR(opt, warmup_min_lr=0.0, warmup_max_lr=1e-3, warmup_num_steps=1000)
    used = []
    for _ in range(4):
        used.append(opt.param_groups[0]["lr"])  # the lr this optimizer step runs with
        sch.step()
    assert used[0] == 0.0 and used[1] == 0.0
    assert abs(used[2] - 1e-3 * math.log(2) / math.log(1000)) < 1e-15
    assert abs(used[3] - 1e-3 * math.log(3) / math.log(1000)) < 1e-15
    assert sch.get_lr()[0] == opt.param_groups[0]["lr"]
    sch2 = WarmupLR(opt, warmup_min_lr=0.0, warmup_max_lr=1e-3, warmup_num_steps=1000)
    sch2.load_state_dict(sch.state_dict())
    assert opt.param_groups[0]["lr"] == sch.get_lr()[0]
