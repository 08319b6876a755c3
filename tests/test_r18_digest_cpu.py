"""BASELINE configs[0] at full size against the reference's own train step:
ResNet-18 / CIFAR shape, 100 images per rank, world size 2, Adam(lr=1e-3·ws)
(R:resnet/pytorch_ddp/ddp_train.py:95,97,110-111), two steps of the
reference's ``train_epoch`` body (:59-72).

``tests/golden/r18_digest_ws2.json`` was recorded by ``make_golden.py`` running
the reference's ``train_epoch`` on torch's DDP over gloo (per-tensor digests:
Σx, Σx², max|x| and 64 evenly spaced samples, in fp64).  Here libgsync DDP +
FusedAdam runs the same steps from the same seeds (model seed 0, data seed
1234 + rank, 4 threads per rank as the generator):

* step-1 averaged grads: every sample bit-identical (Σ g_r·½ is exact at
  ws = 2 and the local grads come from the same CPU kernels), Σ / Σ² / max
  equal to fp64 round-off;
* step-1 post-step weights: SURVEY.md §8c's Adam tolerance, |Δ| <= lr·1e-3
  on every sample (ĝ is never below 1e3·eps on the sampled elements here);
* step-2 grads and weights: step 1's last-bit weight differences flip the
  sign of Adam's lr·g/(|g|+eps) on elements with |g| ~ eps, which then move
  the step-2 grads for real; samples within 1e-2 of the tensor's max |g| and
  weights within 0.2·lr (observed 5.6e-3 and 0.12·lr).
"""
import json
import os

import numpy as np
import torch
import torch.nn as nn

from tests.test_ddp_cpu import _run

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "r18_digest_ws2.json")


def _digest(t):
    x = t.detach().double().reshape(-1)
    idx = torch.linspace(0, x.numel() - 1, steps=min(64, x.numel())).long()
    return {"sum": x.sum().item(), "sumsq": (x * x).sum().item(), "maxabs": x.abs().max().item(),
            "samples": x[idx].tolist()}


def _worker(rank, ws, out_path):
    import distributed_training_amd as D
    from distributed_training_amd.resnet import resnet18

    torch.manual_seed(0)
    model = resnet18(num_classes=10)
    ddp = D.DistributedDataParallel(model)
    opt = D.FusedAdam(ddp.parameters(), lr=1e-3 * ws)  # R:ddp_train.py:97,110
    crit = nn.CrossEntropyLoss()
    g = torch.Generator().manual_seed(1234 + rank)
    batches = [(torch.rand(100, 3, 32, 32, generator=g), torch.randint(0, 10, (100,), generator=g))
               for _ in range(2)]
    params = list(model.parameters())
    grads, weights = [], []
    model.train()
    for x, y in batches:  # R:ddp_train.py:61-72
        loss = crit(ddp(x), y)
        loss.backward()
        grads.append([_digest(p.grad) for p in params])
        opt.step()
        weights.append([_digest(p) for p in params])
        opt.zero_grad()
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"grads": grads, "params": weights}, f)


def test_resnet18_cifar_ws2_matches_reference_digests(tmp_path):
    out = str(tmp_path / "mine.json")
    _run(_worker, 2, out)
    with open(GOLDEN) as f:
        ref = json.load(f)
    with open(out) as f:
        mine = json.load(f)
    assert ref["ws"] == 2 and ref["batch"] == 100 and len(ref["param_names"]) == len(mine["grads"][0])
    lr = 1e-3 * 2
    n_exact, worst_g, worst_p = 0, 0.0, 0.0
    for i, name in enumerate(ref["param_names"]):
        # step 1: averaged grads bit-identical
        rg, mg = ref["grads"][0][i], mine["grads"][0][i]
        assert mg["samples"] == rg["samples"], f"step-1 grad samples of {name}"
        for k in ("sum", "sumsq", "maxabs"):
            assert abs(mg[k] - rg[k]) <= 1e-9 * max(1.0, abs(rg[k])), (name, k, mg[k], rg[k])
        n_exact += 1
        # step 1: post-step weights within lr·1e-3
        rp, mp_ = ref["params"][0][i], mine["params"][0][i]
        d = np.abs(np.array(mp_["samples"]) - np.array(rp["samples"]))
        assert d.max() <= lr * 1e-3, (name, float(d.max()))
        # step 2: after one Adam step whose last-bit differences flip the
        # sign of lr·g/(|g|+eps) where |g| ~ eps, off the samples
        r, m = ref["grads"][1][i], mine["grads"][1][i]
        worst_g = max(worst_g, float(np.abs(np.array(m["samples"]) - np.array(r["samples"])).max()) / r["maxabs"])
        r, m = ref["params"][1][i], mine["params"][1][i]
        worst_p = max(worst_p, float(np.abs(np.array(m["samples"]) - np.array(r["samples"])).max()))
    assert n_exact == 62
    print(f"step 2: grads worst |d|/max|g| {worst_g:.2e}, weights worst |d| {worst_p:.2e}")
    assert worst_g <= 1e-2, worst_g
    assert worst_p <= 0.2 * lr, worst_p
