"""Generate tests/golden/colossal_harness_ws2.npz by driving the Colossal shim with
the REFERENCE's own Colossal harness (run in the build container, which has
/root/reference; the output is plain data — no reference source is stored).

What runs unchanged from R:resnet/colossal/colossal_train.py, taken out of the
file at run time (its module body launches a job and downloads CIFAR-10, so the
module is not imported: its import statements and three function definitions
are compiled from the parsed source):
  * add_argument() (:30-50) — the `-p/--plugin {torch_ddp, torch_ddp_fp16,
    low_level_zero}` argparse surface;
  * train_epoch() (:81-105) — model.train(), the tqdm loop, `images.cuda()`,
    `model(images)`, criterion, booster.backward(loss, optimizer) against the
    module-global `optimizer`, optimizer.step() / zero_grad().
What is restated: the script body (:110-165): launch_from_torch, the
coordinator, LEARNING_RATE = 1e-3 * world_size (:117-122), the plugin choice
exactly as :127-138 (torch_ddp_fp16 -> mixed_precision 'fp16'; torch_ddp* ->
TorchDDPPlugin(); low_level_zero -> LowLevelZeroPlugin(initial_scale=2**5)),
HybridAdam(model.parameters(), lr) (:153) and booster.boost(model, optimizer,
criterion=criterion) (:159-161); plugin.prepare_dataloader(..., batch_size=100,
shuffle=False, drop_last=True) as build_dataloader (:76) does, over a synthetic
CIFAR-shaped dataset (the download needs the network); the width-4
BasicBlock[1,1,1,1] ResNet of the other fixtures instead of resnet18 (:149) so
the weights fit a fixture; CPU/gloo world size 2.  On the CPU the harness's
`.cuda()` calls (:90-91) return the host tensor: the loader yields a tensor
subclass whose cuda() is the identity.  `colossalai` / `torchvision` resolve
to libgsync's shims (distributed_training_amd/compat/shims, tests/golden/_shim):
ColossalAI is not installed, so this pins the reference harness's CALL SURFACE
and the shim's numerics as driven by it (ColossalAI's own numerics stay
unpinned).

Recorded per plugin: every step's loss on each rank (through the criterion the
harness calls), the final fp32 weights of rank 0 (the replicas must agree) and,
for the fp16 plugins, the loss scale after the epoch.
tests/test_colossal_harness_cpu.py replays the shim against it without the
reference.

Usage: python tests/golden/make_colossal_golden.py
"""
from __future__ import annotations

import ast
import os
import sys
import types

import numpy as np
import torch
import torch.multiprocessing as mp
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_COL = "/root/reference/resnet/colossal/colossal_train.py"
SHIMS = os.path.join(REPO, "distributed_training_amd", "compat", "shims")
OUT = os.path.join(HERE, "colossal_harness_ws2.npz")
WS = 2
PLUGINS = ["torch_ddp", "torch_ddp_fp16", "low_level_zero"]
BATCH = 100  # R:colossal_train.py:143 build_dataloader(100, ...)
STEPS = 3
N_SAMPLES = WS * BATCH * STEPS


def micro():
    from distributed_training_amd.resnet import BasicBlock, ResNet

    return ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, width=4)


class HostTensor(torch.Tensor):
    """A host tensor whose .cuda() is the identity: the harness's `images.cuda()` /
    `labels.cuda()` (R:colossal_train.py:90-91) on the CPU rehearsal."""

    def cuda(self, *a, **k):
        return self.as_subclass(torch.Tensor)


class HostLoader:
    """The plugin's DataLoader, yielding HostTensor batches."""

    def __init__(self, loader):
        self.loader = loader

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for images, labels in self.loader:
            yield images.as_subclass(HostTensor), labels.as_subclass(HostTensor)


def dataset():
    g = torch.Generator().manual_seed(2025)
    return torch.utils.data.TensorDataset(torch.rand(N_SAMPLES, 3, 32, 32, generator=g),
                                          torch.randint(0, 10, (N_SAMPLES,), generator=g))


class RecordingCE(nn.CrossEntropyLoss):
    """The harness's criterion, recording each step's loss."""

    def __init__(self):
        super().__init__()
        self.losses = []

    def forward(self, x, y):
        loss = super().forward(x, y)
        self.losses.append(float(loss.detach().float()))
        return loss


def make_plugin(colossalai_mod, name):
    """R:colossal_train.py:127-138, restated: (plugin, booster kwargs)."""
    from colossalai.booster.plugin import LowLevelZeroPlugin, TorchDDPPlugin

    kw = {}
    if name == "torch_ddp_fp16":
        kw["mixed_precision"] = "fp16"
    if name.startswith("torch_ddp"):
        plugin = TorchDDPPlugin()
    elif name == "low_level_zero":
        plugin = LowLevelZeroPlugin(initial_scale=2 ** 5)
    else:
        raise ValueError(name)
    return plugin, kw


def loss_scale(optimizer) -> float:
    """The fp16 loss scale after the epoch (0: no scaler): the TorchDDPPlugin's
    GradScaler or the LowLevelZero engine's DynamicLossScaler."""
    sc = getattr(optimizer, "scaler", None)
    if sc is not None:
        return float(sc.get_scale())
    zs = getattr(getattr(optimizer, "zero", None), "scaler", None)
    return float(zs.scale) if zs is not None else 0.0


def load_reference_functions():
    """The reference file's import statements and its add_argument / build_dataloader /
    train_epoch definitions, compiled into a fresh module (the script body is left out)."""
    with open(REF_COL) as f:
        tree = ast.parse(f.read(), filename=REF_COL)
    keep = [n for n in tree.body if isinstance(n, (ast.Import, ast.ImportFrom))
            or (isinstance(n, ast.FunctionDef) and n.name in ("add_argument", "build_dataloader", "train_epoch"))]
    mod = types.ModuleType("ref_colossal_train")
    exec(compile(ast.Module(body=keep, type_ignores=[]), REF_COL, "exec"), mod.__dict__)
    return mod


def worker(rank, ws, port, q):
    sys.path[:0] = [SHIMS, os.path.join(HERE, "_shim"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    import colossalai
    from colossalai.booster import Booster
    from colossalai.cluster import DistCoordinator
    from colossalai.nn.optimizer import HybridAdam

    colossalai.launch_from_torch(config={})  # R:colossal_train.py:110 (gloo on the CPU)
    coordinator = DistCoordinator()  # :111
    ref = load_reference_functions()
    out = {}
    for name in PLUGINS:
        sys.argv = ["colossal_train.py", "-p", name]
        args = ref.add_argument()  # :30-50, unchanged
        lr = 1e-3 * coordinator.world_size  # :117-122
        plugin, kw = make_plugin(colossalai, args.plugin)
        booster = Booster(plugin=plugin, **kw)  # :138
        loader = plugin.prepare_dataloader(dataset(), batch_size=BATCH, shuffle=False, drop_last=True)  # :76
        torch.manual_seed(0)
        model = micro()
        criterion = RecordingCE()
        optimizer = HybridAdam(model.parameters(), lr=lr)  # :153
        model, optimizer, criterion, _, _ = booster.boost(model, optimizer, criterion=criterion)  # :159-161
        ref.NUM_EPOCHS = 1
        ref.optimizer = optimizer  # train_epoch steps the module-global optimizer (:100-102)
        inner = criterion.module if hasattr(criterion, "module") else criterion
        ref.train_epoch(0, model, criterion, HostLoader(loader), booster, coordinator)  # :81-105, unchanged
        params = list(model.parameters())
        out[f"{name}_losses"] = np.array(inner.losses, dtype=np.float64)
        out[f"{name}_weights"] = torch.cat([p.detach().float().reshape(-1) for p in params]).numpy()
        out[f"{name}_scale"] = np.array([loss_scale(optimizer)])
        out[f"{name}_plugin"] = np.array([PLUGINS.index(args.plugin)])
    q.put((rank, out))


def main():
    sys.path.insert(0, REPO)
    from tests._dist_util import free_port

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    ps = [ctx.Process(target=worker, args=(r, WS, port, q)) for r in range(WS)]
    for p in ps:
        p.start()
    res = dict(q.get() for _ in range(WS))
    for p in ps:
        p.join(600)
    blob = {}
    for rank, out in sorted(res.items()):
        for k, v in out.items():
            if k.endswith("_weights") and rank != 0:
                assert np.array_equal(v, res[0][k]), f"{k}: replicas diverged"
                continue
            blob[f"r{rank}_{k}"] = v
    np.savez_compressed(OUT, **blob)
    print(f"wrote {OUT}: {sorted(blob)}")


if __name__ == "__main__":
    main()
