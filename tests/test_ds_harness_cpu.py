"""The DeepSpeed shim replayed against the fixture the reference's OWN harness
produced (tests/golden/make_ds_golden.py: R:resnet/deepspeed/deepspeed_train.py
add_argument() :27-129 and train_epoch() :133-158 imported and run unchanged
against the shim, CPU/gloo world size 2, ZeRO stage 0/2 x fp32/bf16).

This test never reads /root/reference: it restates the harness loop (as
tests/test_compat_cpu.py does) and must reproduce, per rank and step, the
losses the reference's train_epoch computed, its WarmupLR schedule, and the
final weights — so a change in the shim's call surface or numerics that the
reference harness would see shows here.  DeepSpeed itself is not installed:
its own numerics stay parity-unpinned."""
import os
import sys

import numpy as np
import pytest
import torch

from tests.golden.make_ds_golden import N_SAMPLES, SHIMS, dataset, ds_config, micro, RecordingCE
from tests.test_ddp_cpu import _run

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ds_harness_ws2.npz")


def _replay(rank, ws, stage, dtype):
    sys.path.insert(0, SHIMS)
    import argparse

    import deepspeed

    torch.set_num_threads(2)  # as the generator
    z = np.load(GOLDEN, allow_pickle=False)
    key = f"stage{stage}_{dtype}"
    parser = deepspeed.add_config_arguments(argparse.ArgumentParser())
    parser.add_argument("--stage", type=int, default=0)
    parser.add_argument("--dtype", default="bf16")
    args, _ = parser.parse_known_args(["--deepspeed", "--stage", str(stage), "--dtype", dtype])
    torch.manual_seed(0)
    model = micro()
    engine, _, loader, _ = deepspeed.initialize(args=args, model=model,
                                                model_parameters=filter(lambda p: p.requires_grad, model.parameters()),
                                                training_data=dataset(), config=ds_config(stage, dtype))
    target = torch.bfloat16 if engine.bfloat16_enabled() else None
    crit = RecordingCE()
    lrs = []
    model.train()
    for images, labels in loader:  # R:deepspeed_train.py:142-158, restated
        if target is not None:
            images = images.to(target)
        loss = crit(model(images), labels)
        engine.backward(loss)
        engine.step()
        lrs.append(engine.get_lr()[0])
    assert len(crit.losses) == N_SAMPLES // 96
    np.testing.assert_array_equal(np.array(crit.losses), z[f"r{rank}_{key}_losses"], err_msg=f"{key} losses")
    np.testing.assert_array_equal(np.array(lrs), z[f"r{rank}_{key}_lrs"], err_msg=f"{key} lr schedule")
    w = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).numpy()
    np.testing.assert_array_equal(w, z[f"r0_{key}_weights"], err_msg=f"{key} weights")


@pytest.mark.parametrize("stage,dtype", [(0, "fp32"), (0, "bf16"), (2, "fp32"), (2, "bf16")])
def test_shim_replays_the_reference_harness(stage, dtype):
    _run(_replay, 2, stage, dtype)
