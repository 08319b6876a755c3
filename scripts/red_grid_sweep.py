"""The reductions alone under GS_RED_GRID (the reduction grid cap, which also
decides whether the unpack's fused Σg² combines in-kernel — caps <= 8 Ki — or
through a second launch): unpack + Σg², Σg², Σg² partials, on ResNet-50's
parameter shapes and ResNet-152's x 2; plan launch timer (the kernels' own
start / end).  One JSON line per row (scripts/r4l_red_grid.sh)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
cap = os.environ.get("GS_RED_GRID", "default")
for model, reps in (("resnet50", 1), ("resnet152", 2)):
    with torch.device("meta"):
        m = MODELS[model](num_classes=1000)
    shapes = [tuple(p.shape) for p in m.parameters()] * reps
    numels = [int(torch.Size(s).numel()) for s in shapes]
    n = sum(numels)
    g = torch.Generator(device=dev).manual_seed(3)
    grads = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
    plan = TensorListPlan(numels, dev, align=64)
    plan.set_ptrs(1, grads)
    flat = torch.randn(plan.flat_numel, device=dev, generator=g) * 0.01
    sq = torch.zeros(1, device=dev)
    for name, nbytes, fn in (("unpack_f32+sqnorm", 8 * n, lambda: plan.unpack(flat, 1, torch.float32, sqnorm=sq)),
                             ("sqnorm_f32", 4 * n, lambda: plan.sqnorm(1, torch.float32, sq)),
                             ("sqnorm_partial_f32", 4 * n, lambda: plan.sqnorm_partial(1, torch.float32))):
        for _ in range(3):
            fn()
        plan.timer_enable(128)
        for _ in range(30):
            fn()
        ts = plan.timer_read()
        plan.timer_enable(0)
        ms = sum(ts) / 30
        print(json.dumps({"GS_RED_GRID": cap, "model": model, "replicas": reps, "kernel": name, "avg_ms": ms,
                          "frac": nbytes / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
    del grads, flat, plan
    torch.cuda.empty_cache()
