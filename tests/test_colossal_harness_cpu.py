"""The Colossal shim replayed against the fixture the reference's OWN harness
produced (tests/golden/make_colossal_golden.py: R:resnet/colossal/colossal_train.py
add_argument() :30-50 and train_epoch() :81-105 compiled from the reference file
and run unchanged against the shim, the plugin choice of :127-138, CPU/gloo
world size 2, plugins torch_ddp / torch_ddp_fp16 / low_level_zero).

This test never reads /root/reference: it restates the harness loop and must
reproduce, per rank and step, the losses the reference's train_epoch computed,
the final weights and the fp16 loss scale — so a change in the shim's call
surface or numerics that the reference harness would see shows here.
ColossalAI itself is not installed: its own numerics stay parity-unpinned
(SURVEY.md §8c)."""
import os
import sys

import numpy as np
import pytest
import torch

from tests.golden.make_colossal_golden import (BATCH, N_SAMPLES, SHIMS, WS, HostLoader, RecordingCE, dataset,
                                               loss_scale, make_plugin, micro)
from tests.test_ddp_cpu import _run

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "colossal_harness_ws2.npz")


def _replay(rank, ws, plugin_name):
    sys.path.insert(0, SHIMS)
    import colossalai
    from colossalai.booster import Booster
    from colossalai.cluster import DistCoordinator
    from colossalai.nn.optimizer import HybridAdam

    torch.set_num_threads(2)  # as the generator
    z = np.load(GOLDEN, allow_pickle=False)
    colossalai.launch_from_torch(config={})
    coordinator = DistCoordinator()
    plugin, kw = make_plugin(colossalai, plugin_name)
    booster = Booster(plugin=plugin, **kw)
    loader = plugin.prepare_dataloader(dataset(), batch_size=BATCH, shuffle=False, drop_last=True)
    torch.manual_seed(0)
    model = micro()
    criterion = RecordingCE()
    optimizer = HybridAdam(model.parameters(), lr=1e-3 * coordinator.world_size)
    model, optimizer, criterion, _, _ = booster.boost(model, optimizer, criterion=criterion)
    inner = criterion.module if hasattr(criterion, "module") else criterion
    model.train()
    for images, labels in HostLoader(loader):  # R:colossal_train.py:87-105, restated
        images = images.cuda()
        labels = labels.cuda()
        outputs = model(images)
        loss = criterion(outputs, labels)
        booster.backward(loss, optimizer)
        optimizer.step()
        optimizer.zero_grad()
    assert len(inner.losses) == N_SAMPLES // (WS * BATCH)
    key = plugin_name
    np.testing.assert_array_equal(np.array(inner.losses), z[f"r{rank}_{key}_losses"], err_msg=f"{key} losses")
    w = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).numpy()
    np.testing.assert_array_equal(w, z[f"r0_{key}_weights"], err_msg=f"{key} weights")
    assert loss_scale(optimizer) == float(z[f"r{rank}_{key}_scale"][0]), key


@pytest.mark.parametrize("plugin", ["torch_ddp", "torch_ddp_fp16", "low_level_zero"])
def test_shim_replays_the_reference_colossal_harness(plugin):
    _run(_replay, 2, plugin)
