"""Σg² where the clip path runs it: right after the grads were written (a bucket
unpack into the grads, then the Σg² partials, then the clipped SGD), per kernel
by the plan launch timer, under GS_NT_SQNORM (the Σg² kernels' load policy:
0 cached, 1 non-temporal, 2 the size rule = default; GS_NT_SQ_HOT=1: the SGD
keeps cached grad loads after a non-temporal Σg², "/hot" in the label).  ResNet-50 / ResNet-152 /
ResNet-152 x 2 parameter shapes, fp32.  One JSON line per kernel and size
(scripts/r4s_sqnorm_chain.sh)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
pol = os.environ.get("GS_NT_SQNORM", "default") + ("/hot" if os.environ.get("GS_NT_SQ_HOT") == "1" else "")
for model, reps in (("resnet50", 1), ("resnet152", 1), ("resnet152", 2)):
    with torch.device("meta"):
        m = MODELS[model](num_classes=1000)
    shapes = [tuple(p.shape) for p in m.parameters()] * reps
    numels = [int(torch.Size(s).numel()) for s in shapes]
    n = sum(numels)
    g = torch.Generator(device=dev).manual_seed(3)
    grads = [torch.zeros(s, device=dev) for s in shapes]
    ps = [torch.randn(s, device=dev, generator=g) for s in shapes]
    bufs = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
    bplan = TensorListPlan(numels, dev, align=64)
    bplan.set_ptrs(1, grads)
    flat = torch.randn(bplan.flat_numel, device=dev, generator=g) * 0.01
    plan = TensorListPlan(numels, dev, task_units=update_task_units(dev))
    for k, ts in enumerate((ps, grads, bufs)):
        plan.set_ptrs(k, ts)
    out = torch.zeros(3, device=dev)

    def step():
        bplan.unpack(flat, 1, torch.float32)
        plan.sqnorm_partial(1, torch.float32)
        plan.set_clip(1.0, 1e-6, None, 1.0, 1.0, out=out)
        plan.sgd(torch.float32, 1e-9, 0.9, 0.0, 1e-4, False, False, False)

    for _ in range(3):
        step()
    bplan.timer_enable(128)
    plan.timer_enable(128)
    for _ in range(30):
        step()
    upd = plan.timer_read()  # one read (it drains the ring); the launches alternate partials, SGD
    rows = {"unpack_f32": (bplan.timer_read(), 8 * n),
            "sqnorm_partial_f32": (upd[0::2], 4 * n),
            "clipped_sgd": (upd[1::2], 20 * n)}
    bplan.timer_enable(0)
    plan.timer_enable(0)
    rows["clip_path_total"] = ([a + b for a, b in zip(upd[0::2], upd[1::2])], 24 * n)
    for name, (ts, nbytes) in rows.items():
        ms = sum(ts) / len(ts)
        print(json.dumps({"GS_NT_SQNORM": pol, "model": model, "replicas": reps, "kernel": name, "launches": len(ts),
                          "avg_ms": ms, "frac": nbytes / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
    del grads, ps, bufs, plan, bplan, flat
    torch.cuda.empty_cache()
