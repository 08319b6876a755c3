"""Small-tensor-heavy plans: pack ×1/ws, unpack and fused SGD over K tensors
of random size in [lo, hi] elements (≈ N elements in all) against one tensor
of the same N — plan launch timer, average of `iters` launches.  One JSON line
per (case, op).  Run with GS_ENGINE=0 for the task engine (LDS-staged
descriptors) beside the default chunk-map engine.
    python scripts/small_tensors.py [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)


def sizes(lo, hi, total):
    out, s = [], 0
    while s < total:
        n = int(torch.randint(lo, hi + 1, (1,), generator=g))
        out.append(n)
        s += n
    return out


N = 16 << 20
cases = {"one_tensor": [N], "bn_like_64_2k": sizes(64, 2048, N), "tiny_1_256": sizes(1, 256, 4 << 20),
         "mixed_r50_like": sizes(1, 2048, N // 2) + [N // 2]}


def rate(plan, fn):
    for _ in range(3):
        fn()
    plan.timer_enable(iters)
    for _ in range(iters):
        fn()
    ts = plan.timer_read()
    plan.timer_enable(0)
    return sum(ts) / len(ts)


for name, numels in cases.items():
    n = sum(numels)
    xs = [torch.randn(k, device=dev) for k in numels]
    plan = TensorListPlan(numels, dev, align=64)
    plan.set_ptrs(1, xs)
    flat = torch.zeros(plan.flat_numel, device=dev)
    outs = [torch.empty_like(x) for x in xs]
    plan.set_ptrs(2, outs)
    rows = {"pack": (8 * n, lambda: plan.pack(1, torch.float32, flat, 0.5, 1)),
            "unpack": (8 * n, lambda: plan.unpack(flat, 2, torch.float32))}
    for op, (nbytes, fn) in rows.items():
        ms = rate(plan, fn)
        print(json.dumps({"case": name, "tensors": len(numels), "elements": n, "op": op,
                          "engine": os.environ.get("GS_ENGINE", "default"), "avg_us": ms * 1e3,
                          "GBps": nbytes / (ms * 1e-3) / 1e9}), flush=True)
    up = TensorListPlan(numels, dev, task_units=update_task_units(dev))
    bufs = [torch.zeros_like(x) for x in xs]
    up.set_ptrs(0, outs)
    up.set_ptrs(1, xs)
    up.set_ptrs(2, bufs)
    ms = rate(up, lambda: up.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False))
    print(json.dumps({"case": name, "tensors": len(numels), "elements": n, "op": "sgd",
                      "engine": os.environ.get("GS_ENGINE", "default"), "avg_us": ms * 1e3,
                      "GBps": 20 * n / (ms * 1e-3) / 1e9}), flush=True)
    del xs, outs, bufs, flat
