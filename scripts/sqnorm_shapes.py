"""Σg² (gs_sqnorm) at ResNet-50 size on three layouts of the same 25.56 M fp32
elements, plan launch timer (the kernel's own start / end), to separate the
chunk engine's per-tensor costs from its streaming: ResNet-50's 161 tensors in
the DDP bucket layout (64-element alignment: tensor boundaries inside chunks,
~161 mixed chunks), the same tensors 1 Ki-aligned (every tensor starts a chunk;
its tail chunk is still partial), and one tensor of the same size.  Also the
partial-sums form (gs_sqnorm_partial: no top-level hand-off).  One JSON line
per (layout, op, round).

    python scripts/sqnorm_shapes.py > rows.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_training_amd.multi_tensor import TensorListPlan  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
shapes = [tuple(p.shape) for p in MODELS["resnet50"](num_classes=1000).parameters()]
numels = [int(torch.Size(s).numel()) for s in shapes]
n = sum(numels)
g = torch.Generator(device=dev).manual_seed(7)
ITERS = 50


def timed(plan, fn):
    for _ in range(3):
        fn()
    plan.timer_enable(4 * ITERS)
    for _ in range(ITERS):
        fn()
    ts = plan.timer_read()
    plan.timer_enable(0)
    return sum(ts) / ITERS


layouts = {
    "r50_align64": (numels, 64),
    "r50_align1024": (numels, 1024),
    "one_tensor": ([n], 64),
}
for rnd in range(2):
    for name, (ns, align) in layouts.items():
        ts = [torch.randn(k, device=dev, generator=g) * 0.01 for k in ns]
        plan = TensorListPlan(ns, dev, align=align)
        plan.set_ptrs(1, ts)
        sq = torch.zeros(1, device=dev)
        for op, fn in (("sqnorm", lambda: plan.sqnorm(1, torch.float32, sq)),
                       ("sqnorm_partial", lambda: plan.sqnorm_partial(1, torch.float32))):
            ms = timed(plan, fn)
            print(json.dumps({"layout": name, "op": op, "round": rnd, "tensors": len(ns), "elems": n,
                              "avg_us": ms * 1e3, "frac": 4 * n / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
        plan.close()
        del ts
