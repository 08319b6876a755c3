"""The exposed tail's pack / unpack (ResNet-50's last DDP bucket: conv1, bn1, layer1,
layer2 and the start of layer3, ~2.43 M fp32 elements, 9.7 MB) by the plan launch
timer (the kernel's own start / end), to split the ~7 µs a launch takes there
 into the layout's cost and the stream's: the bucket's own tensors
(64-element alignment, as the bucketer lays them out) against one tensor of the same
size, each warm (back to back: the 19 MB a launch moves fit the XCDs' L2s) and cold
(a 512 MB fill between launches, as the backward's own traffic leaves the caches).
One JSON line per (layout, op, cache, round).

    python scripts/tail_pack_shapes.py > rows.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_training_amd.multi_tensor import TensorListPlan  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402
from distributed_training_amd import _lib as L  # noqa: E402

dev = torch.device("cuda", 0)
numels = []
for p in MODELS["resnet50"](num_classes=1000).parameters():  # model order = the last bucket's first
    if sum(numels) >= 2_431_040:
        break
    numels.append(p.numel())
n = sum(numels)
g = torch.Generator(device=dev).manual_seed(7)
ITERS = 40
junk = torch.empty(128 * 1024 * 1024, device=dev)  # 512 MB: evicts the L2s and the Infinity Cache


def timed(plan, fn, cold):
    for _ in range(3):
        fn()
    plan.timer_enable(4 * ITERS)
    for _ in range(ITERS):
        if cold:
            junk.fill_(1.0)
        fn()
    ts = plan.timer_read()
    plan.timer_enable(0)
    return sum(ts) / len(ts)


layouts = {"last_bucket_align64": (numels, 64), "one_tensor": ([n], 64)}
for rnd in range(2):
    for name, (ns, align) in layouts.items():
        ts = [torch.randn(k, device=dev, generator=g) * 0.01 for k in ns]
        plan = TensorListPlan(ns, dev, align=align)
        plan.set_ptrs(1, ts)
        flat = torch.zeros(plan.flat_numel, device=dev)
        for op, fn in (("pack", lambda: plan.pack(1, torch.float32, flat, 0.125, L.GS_SCALE_MUL)),
                       ("unpack", lambda: plan.unpack(flat, 1, torch.float32))):
            for cold in (False, True):
                ms = timed(plan, fn, cold)
                print(json.dumps({"layout": name, "op": op, "cache": "cold" if cold else "warm", "round": rnd,
                                  "tensors": len(ns), "elems": n, "avg_us": ms * 1e3,
                                  "frac": 8 * n / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
        plan.close()
        del ts, flat
