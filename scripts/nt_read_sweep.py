"""Σg² and the clip path under GS_NT_READ_ONCE (non-temporal loads of the read-once
gradient stream: 0 never, 1 always, 2 when it is larger than the Infinity Cache,
the default): Σg², Σg² partials, the clip path (partials + the clipped SGD) and
the SGD alone, and the bucket pack / unpack (the read-once source grads / flat
buffer), on ResNet-50's parameter shapes (102 MB of grads), ResNet-152's
(241 MB) and ResNet-152's x 2 (482 MB); plan launch timer (the kernels' own
start / end).  One JSON line per row, with the Σg² value (scripts/r4q_nt_read.sh)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
pol = os.environ.get("GS_NT_READ_ONCE", "default")
for model, reps in (("resnet50", 1), ("resnet152", 1), ("resnet152", 2)):
    with torch.device("meta"):
        m = MODELS[model](num_classes=1000)
    shapes = [tuple(p.shape) for p in m.parameters()] * reps
    numels = [int(torch.Size(s).numel()) for s in shapes]
    n = sum(numels)
    g = torch.Generator(device=dev).manual_seed(3)
    grads = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
    ps = [torch.randn(s, device=dev, generator=g) for s in shapes]
    bufs = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
    plan = TensorListPlan(numels, dev, task_units=update_task_units(dev))
    for k, ts in enumerate((ps, grads, bufs)):
        plan.set_ptrs(k, ts)
    sq = torch.zeros(1, device=dev)
    out = torch.zeros(3, device=dev)

    def clip_path():
        plan.sqnorm_partial(1, torch.float32)
        plan.set_clip(1.0, 1e-6, None, 1.0, 1.0, out=out)
        plan.sgd(torch.float32, 1e-9, 0.9, 0.0, 1e-4, False, False, False)

    def sgd():
        plan.set_clip(None)
        plan.sgd(torch.float32, 1e-9, 0.9, 0.0, 1e-4, False, False, False)

    for name, nbytes, fn, launches in (("sqnorm_f32", 4 * n, lambda: plan.sqnorm(1, torch.float32, sq), 1),
                                       ("sqnorm_partial_f32", 4 * n, lambda: plan.sqnorm_partial(1, torch.float32), 1),
                                       ("clip_path_sgd", 24 * n, clip_path, 2),
                                       ("sgd_momentum_wd", 20 * n, sgd, 1)):
        for _ in range(3):
            fn()
        plan.timer_enable(128)
        for _ in range(30):
            fn()
        ts = plan.timer_read()
        plan.timer_enable(0)
        ms = sum(ts) / 30  # per call: the timer holds every launch of the call
        row = {"GS_NT_READ_ONCE": pol, "model": model, "replicas": reps, "grad_MB": 4 * n / 1e6, "kernel": name,
               "avg_ms": ms, "frac": nbytes / (ms * 1e-3) / 1e9 / 8000.0}
        if name == "sqnorm_f32":
            row["sqnorm"] = float(sq.item())
        print(json.dumps(row), flush=True)
    bplan = TensorListPlan(numels, dev, align=64)
    bplan.set_ptrs(1, grads)
    flat = torch.randn(bplan.flat_numel, device=dev, generator=g) * 0.01
    flat16 = torch.zeros(bplan.flat_numel, device=dev, dtype=torch.bfloat16)
    for name, nbytes, fn in (("pack_f32", 8 * n, lambda: bplan.pack(1, torch.float32, flat, 0.125, 1)),
                             ("pack_f32_to_bf16", 6 * n, lambda: bplan.pack(1, torch.float32, flat16, 0.125, 1)),
                             ("unpack_f32", 8 * n, lambda: bplan.unpack(flat, 1, torch.float32)),
                             ("unpack_f32+sqnorm", 8 * n, lambda: bplan.unpack(flat, 1, torch.float32, sqnorm=sq))):
        for _ in range(3):
            fn()
        bplan.timer_enable(128)
        for _ in range(30):
            fn()
        ts = bplan.timer_read()
        bplan.timer_enable(0)
        ms = sum(ts) / 30
        print(json.dumps({"GS_NT_READ_ONCE": pol, "model": model, "replicas": reps, "grad_MB": 4 * n / 1e6,
                          "kernel": name, "avg_ms": ms, "frac": nbytes / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
    del grads, ps, bufs, plan, bplan, flat, flat16
    torch.cuda.empty_cache()
