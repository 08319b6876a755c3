"""examples/ddp_train.py (the reference's DDP trainer on libgsync: DDP + fused
Adam + device-resident input step) vs the reference's own pipeline (torch DDP
+ torch Adam + torch DataLoader/DistributedSampler with torchvision's
transforms restated), CPU / gloo, world_size 2, same seed and data.

Batches are bit-identical (tests/test_data_cpu.py), averaged grads are
bit-identical at ws=2 (tests/test_ddp_cpu.py); Adam's update differs from
torch's in the last bits.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from tests._dist_util import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _synthetic(n, seed):
    g = torch.Generator().manual_seed(seed)
    imgs = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (n,), generator=g)
    return imgs.numpy(), labels.numpy()


def _reference(rank, ws, port, steps, batch, n, q):
    sys.path.insert(0, REPO)
    from distributed_training_amd.resnet import MODELS
    from oracle.input_pipeline import reference_loader

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    torch.set_num_threads(1)
    torch.manual_seed(0)
    model = torch.nn.parallel.DistributedDataParallel(MODELS["resnet18"](num_classes=10))
    imgs, labels = _synthetic(n, 0)
    loader = reference_loader(imgs, labels, batch, ws, rank, train=True, drop_last=True)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3 * ws)
    crit = nn.CrossEntropyLoss()
    loader.sampler.set_epoch(0)
    grads = {}
    for k, (x, y) in enumerate(loader):
        if k >= steps:
            break
        loss = crit(model(x), y)
        loss.backward()
        for name, p in model.module.named_parameters():  # the averaged grads Adam sees
            grads[f"grad/{k}/{name}"] = p.grad.detach().numpy().copy()
        opt.step()
        opt.zero_grad()
    if rank == 0:
        out = {k: v.detach().numpy().copy() for k, v in model.module.state_dict().items()}
        out.update(grads)
        q.put(out)
    import gc

    gc.collect()  # as tests/test_ddp_cpu.py::_wrap: no gloo work outlives the interpreter
    dist.destroy_process_group()


def _mine(rank, ws, port, steps, batch, n, q):
    sys.path.insert(0, REPO)
    torch.set_num_threads(1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import importlib.util

    spec = importlib.util.spec_from_file_location("ddp_train_example", os.path.join(REPO, "examples", "ddp_train.py"))
    ex = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ex)
    ex.ddp(rank, ws, 1, 1e-3 * ws, batch, "cpu", max_steps=steps, synthetic_n=n, port=port, result=q)


def _run(fn, ws, steps, batch, n):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    ps = [ctx.Process(target=fn, args=(r, ws, port, steps, batch, n, q)) for r in range(ws)]
    for p in ps:
        p.start()
    out = q.get()
    for p in ps:
        p.join(300)
        assert p.exitcode == 0
    return {k: torch.from_numpy(v) for k, v in out.items()}


def _adam_close(ref, mine, steps, lr, eps=1e-8):
    """SURVEY.md §8c Adam tolerance on the parameters: |Δ| <= steps·lr·1e-3,
    excluding elements whose averaged grad had |ĝ| < 1e3·eps at some step (the
    normalised update m/(√v+eps) can flip sign there).  Returns (worst, excluded
    fraction)."""
    worst, excl, total, over = 0.0, 0, 0, 0
    tol = steps * lr * 1e-3
    for name in [k[len("grad/0/"):] for k in ref if k.startswith("grad/0/")]:
        keep = np.ones(ref[name].shape, dtype=bool)
        for s in range(steps):
            keep &= np.abs(ref[f"grad/{s}/{name}"].numpy()) >= 1e3 * eps
        d = (ref[name].double() - mine[name].double()).abs().numpy()
        if keep.any():
            worst = max(worst, float(d[keep].max()))
            over += int((d[keep] > tol).sum())
        excl += int((~keep).sum())
        total += keep.size
    return worst, excl / total, over / total


def _compare(ref, mine):
    ref = {k: v for k, v in ref.items() if not k.startswith("grad/")}
    assert ref.keys() == mine.keys()
    fl = [k for k in ref if ref[k].is_floating_point()]
    for k in ref:
        if k not in fl:
            assert torch.equal(ref[k], mine[k]), k  # num_batches_tracked
    init = _init()
    worst = max((ref[k].double() - mine[k].double()).abs().max().item() for k in fl)
    diff = sum(((ref[k].double() - mine[k].double()) ** 2).sum().item() for k in fl) ** 0.5
    moved = sum(((ref[k].double() - init[k].double()) ** 2).sum().item() for k in fl) ** 0.5
    big = sum(((ref[k].double() - mine[k].double()).abs() > 1e-5).sum().item() for k in fl)
    total = sum(ref[k].numel() for k in fl)
    return worst, diff / moved, big / total


def test_example_trainer_one_step_matches_reference():
    """One step: same batches, bit-identical averaged grads, Adam within last bits."""
    ws, batch, n = 2, 16, 400
    ref, mine = _run(_reference, ws, 1, batch, n), _run(_mine, ws, 1, batch, n)
    worst, rel, frac = _compare(ref, mine)
    assert worst <= 1e-7 and rel <= 1e-6, (worst, rel)
    worst, _, over = _adam_close(ref, mine, 1, 1e-3 * ws)
    assert over == 0, (worst, over)  # one step: every kept element within lr·1e-3


def test_example_trainer_three_steps_track_reference():
    """Three steps.  After step 1 the weights differ in the last bits, so the
    step-2/3 grads carry backprop round-off, which Adam's normalised update
    m/(√v+eps) turns into a relative change for small |g| — an element-wise
    one-step bound cannot hold along a trajectory.  Checked: of the elements
    with |ĝ| >= 1e3·eps at every step (SURVEY.md §8c's exclusion; 37 % of
    ResNet-18's elements at batch 16), <= 0.01 % beyond steps·lr·1e-3 and none
    beyond 0.1·lr (observed: 0.003 % and 0.05·lr); the whole trajectory within
    1e-4 relative L2 of the distance travelled.  The one-step test holds every
    kept element to lr·1e-3."""
    ws, batch, n = 2, 16, 400
    ref, mine = _run(_reference, ws, 3, batch, n), _run(_mine, ws, 3, batch, n)
    worst, rel, frac = _compare(ref, mine)
    assert rel <= 1e-4 and frac <= 1e-4, (worst, rel, frac)
    lr = 1e-3 * ws
    worst, excluded, over = _adam_close(ref, mine, 3, lr)  # SURVEY §8c off the |g|<1e-5 set
    assert over <= 1e-4 and worst <= 0.1 * lr, (worst, excluded, over)


def _init():
    sys.path.insert(0, REPO)
    from distributed_training_amd.resnet import MODELS

    torch.manual_seed(0)
    return MODELS["resnet18"](num_classes=10).state_dict()
