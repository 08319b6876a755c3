"""The clipped AdamW update on configs[3]'s N = 8 shard (ResNet-50 / 8 = 3.19 M
elements; bf16 grads, fp32 master / moments, bf16 param write), its kernel
alone (plan launch timer), folding n partial sums at its start
(gs_plan_set_clip_groups, n = 1 ... GS_RED_PARTIALS) against the scalar form
(gs_plan_set_clip on a finished Σg²) and no clip: what the fold costs and how
it grows with n.  Two interleaved rounds, one JSON line per (round, form).

    python scripts/fold_cost.py > rows.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_training_amd import _lib as L  # noqa: E402
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402

dev = torch.device("cuda", 0)
shard = 3194688
g = torch.Generator(device=dev).manual_seed(11)
master = torch.randn(shard, device=dev, generator=g)
grads = (torch.randn(shard, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
m = torch.randn(shard, device=dev, generator=g) * 1e-3
v = torch.rand(shard, device=dev, generator=g) * 1e-6
p16 = master.to(torch.bfloat16)
plan = TensorListPlan([shard], dev, task_units=update_task_units(dev))
for k, t in enumerate((master, grads, m, v, p16)):
    plan.set_ptrs(k, [t])
groups = torch.rand(L.GS_RED_PARTIALS, device=dev, generator=g) * 1e-3
sq = torch.full((1,), 0.5, device=dev)
out = torch.zeros(3, device=dev)
ITERS = 50


def adam():
    plan.adam(torch.bfloat16, 1e-3, 0.8, 0.999, 1e-8, 3e-7, True, False, -1e-3, 0.5, lowp_dtype=torch.bfloat16)


def timed():
    for _ in range(3):
        adam()
    plan.timer_enable(4 * ITERS)
    for _ in range(ITERS):
        adam()
    ts = plan.timer_read()
    plan.timer_enable(0)
    return sum(ts) / ITERS


forms = [("no_clip", None), ("scalar", 0)] + [(f"fold_{n}", n) for n in (1, 64, 256, 512, 780, L.GS_RED_PARTIALS)]
for rnd in range(2):
    for name, n in forms:
        if n is None:
            plan.set_clip(None)
        elif n == 0:
            plan.set_clip(1.0, 1e-6, sq, out=out)
        else:
            plan.set_clip_groups(1.0, 1e-6, groups, n, out=out)
        us = timed() * 1e3
        print(json.dumps({"round": rnd, "form": name, "n": n, "update_us": us}), flush=True)
plan.set_clip(None)
