"""Checkpoint layout and resume, CPU / gloo, world_size 2.

* ZeRO shard consolidation: the gathered fp32 master state_dict has the
  model's torchvision keys and equals the trained parameters (fp32 model) or
  rounds to them (bf16 model).
* Resume is exact: train 2 steps, save, rebuild a fresh engine from another
  seed, load, train step 3  ==  3 uninterrupted steps, bit for bit, for the
  DeepSpeed shim (ZeRO-0/1/2, fp32 / bf16) and the ColossalAI booster
  (TorchDDP, LowLevelZero).
"""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

from tests.test_compat_cpu import DS_CONFIG, SHIMS
from tests.test_ddp_cpu import _micro, _run


def _batch(rank, it, dtype=torch.float32):
    g = torch.Generator().manual_seed(1000 * it + rank)
    return torch.rand(4, 3, 32, 32, generator=g).to(dtype), torch.randint(0, 10, (4,), generator=g)


def _ds_engine(stage, bf16, seed):
    import copy

    import deepspeed

    cfg = copy.deepcopy(DS_CONFIG)
    cfg["zero_optimization"]["stage"] = stage
    cfg["zero_optimization"]["reduce_bucket_size"] = 20000  # several buckets
    cfg["bf16"]["enabled"] = bf16
    torch.manual_seed(seed)
    model = _micro()
    engine, _, _, _ = deepspeed.initialize(model=model, model_parameters=model.parameters(), config=cfg)
    return engine, model


def _ds_steps(engine, model, rank, its, bf16):
    crit = nn.CrossEntropyLoss()
    for it in its:
        x, y = _batch(rank, it, torch.bfloat16 if bf16 else torch.float32)
        engine.backward(crit(model(x).float(), y))
        engine.step()


def _ds_resume(rank, ws, stage, bf16, tmp):
    sys.path.insert(0, SHIMS)
    e1, m1 = _ds_engine(stage, bf16, seed=1)
    _ds_steps(e1, m1, rank, [0, 1], bf16)
    e1.save_checkpoint(tmp, client_state={"epoch": 7})
    _ds_steps(e1, m1, rank, [2], bf16)
    e2, m2 = _ds_engine(stage, bf16, seed=99)  # different init: everything must come from the checkpoint
    path, client = e2.load_checkpoint(tmp)
    assert client == {"epoch": 7} and path.endswith("global_step2") and e2.global_steps == 2
    _ds_steps(e2, m2, rank, [2], bf16)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a, b), n
    sd = e1.consolidated_fp32_state_dict()
    assert list(sd) == list(m1.state_dict())  # torchvision keys, module order
    for n, p in m1.named_parameters():
        assert sd[n].dtype == torch.float32
        assert torch.equal(sd[n].to(p.dtype), p.detach()), n  # master rounds to the model copy
    if stage and bf16:
        assert any(not torch.equal(sd[n], p.detach().float()) for n, p in m1.named_parameters())  # real fp32 master


@pytest.mark.parametrize("stage,bf16", [(0, False), (1, False), (2, False), (2, True)])
def test_deepspeed_checkpoint_resume(stage, bf16, tmp_path):
    _run(_ds_resume, 2, stage, bf16, str(tmp_path))


def _col_build(plugin_name, seed):
    import colossalai  # noqa: F401
    from colossalai.booster import Booster
    from colossalai.booster.plugin import LowLevelZeroPlugin, TorchDDPPlugin
    from colossalai.nn.optimizer import HybridAdam

    torch.manual_seed(seed)
    model = _micro()
    plugin = TorchDDPPlugin() if plugin_name == "torch_ddp" else LowLevelZeroPlugin(stage=2, precision="fp32")
    booster = Booster(plugin=plugin)
    opt = HybridAdam(model.parameters(), lr=2e-3)
    wrapped, opt, crit, _, _ = booster.boost(model, opt, criterion=nn.CrossEntropyLoss())
    return booster, wrapped, opt, crit, model


def _col_steps(booster, wrapped, opt, crit, rank, its):
    for it in its:
        x, y = _batch(rank, it)
        booster.backward(crit(wrapped(x), y), opt)
        opt.step()
        opt.zero_grad()


def _col_resume(rank, ws, plugin_name, tmp):
    sys.path.insert(0, SHIMS)
    import colossalai

    colossalai.launch_from_torch(config={})
    b1, w1, o1, c1, m1 = _col_build(plugin_name, 1)
    _col_steps(b1, w1, o1, c1, rank, [0, 1])
    b1.save_model(w1, os.path.join(tmp, "model.pt"))
    b1.save_optimizer(o1, os.path.join(tmp, "optim.pt"))
    _col_steps(b1, w1, o1, c1, rank, [2])
    b2, w2, o2, c2, m2 = _col_build(plugin_name, 99)
    b2.load_model(w2, os.path.join(tmp, "model.pt"))
    b2.load_optimizer(o2, os.path.join(tmp, "optim.pt"))
    _col_steps(b2, w2, o2, c2, rank, [2])
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a, b), n
    sd = torch.load(os.path.join(tmp, "model.pt"), weights_only=True)
    assert list(sd) == [k for k in m1.state_dict()]


@pytest.mark.parametrize("plugin", ["torch_ddp", "low_level_zero"])
def test_colossal_checkpoint_resume(plugin, tmp_path):
    _run(_col_resume, 2, plugin, str(tmp_path))
