"""Interleaved task-size sweep of the grad-sync kernels, timed with the plan
launch timer (HIP events around each kernel on its stream).

    python scripts/sweep_tasks.py --model resnet50 --replicas 1 --rounds 5

For each task size (0 = automatic) one plan over the model's real parameter
shapes; every round times `--launches` back-to-back launches of each op for
every plan in turn, so box drift hits all configurations alike.  Prints one
JSON row per (task size, op): median kernel ms and GB/s (algorithmic bytes).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--replicas", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--tasks", default="0,1024,2048,3072,4096,6144,8192,16384")
    ap.add_argument("--ops", default="pack,unpack,sgd,adam,pack16,sgd16")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from distributed_training_amd.multi_tensor import TensorListPlan
    from distributed_training_amd.resnet import MODELS

    dev = torch.device("cuda", 0)
    shapes = [p.shape for p in MODELS[args.model]().parameters()] * args.replicas
    numels = [torch.Size(s).numel() for s in shapes]
    n = sum(numels)
    g = torch.Generator(device=dev).manual_seed(0)
    mk = lambda scale=1.0: [torch.randn(s, device=dev, generator=g) * scale for s in shapes]  # noqa: E731
    params, grads, bufs, ms = mk(), mk(0.01), mk(0.01), mk(0.01)
    vs = [x.abs() for x in mk(1e-4)]
    sizes = [int(x) for x in args.tasks.split(",")]
    plans = {}
    for tu in sizes:
        p = TensorListPlan(numels, dev, align=64, task_units=tu)
        for slot, ts in enumerate((params, grads, bufs, vs)):
            p.set_ptrs(slot, ts)
        p.timer_enable(args.launches)
        plans[tu] = p
    flat = torch.zeros(plans[sizes[0]].flat_numel, device=dev)
    flat16 = torch.zeros(plans[sizes[0]].flat_numel, device=dev, dtype=torch.bfloat16)
    g16 = [x.to(torch.bfloat16) for x in grads]
    lp16 = [x.to(torch.bfloat16) for x in params]
    sq = torch.zeros(1, device=dev)
    plans16 = {}
    for tu in sizes:
        q = TensorListPlan(numels, dev, align=64, task_units=tu)
        for slot, ts in enumerate((params, g16, bufs, lp16)):
            q.set_ptrs(slot, ts)
        q.timer_enable(args.launches)
        plans16[tu] = q
    ops = {
        "pack": (8, lambda p: p.pack(1, torch.float32, flat, 0.125, 1)),
        "unpack": (8, lambda p: p.unpack(flat, 2, torch.float32)),
        "sgd": (20, lambda p: p.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False)),
        "adam": (28, lambda p: p.adam(torch.float32, 1e-6, 0.9, 0.999, 1e-8, 0.0, False, False, -1e-6, 0.5)),
        # 16-bit streams: fp32 -> bf16 bucket pack (6 B/param); ZeRO-style SGD with bf16 grads
        # and a bf16 parameter copy (p 8 + g 2 + buf 8 + lowp 2 = 20 B/param)
        "sqnorm": (4, lambda p: p.sqnorm(1, torch.float32, sq)),
        "pack16": (6, lambda p: p.pack(0, torch.float32, flat16, 0.125, 1)),
        "sgd16": (20, lambda p: p.sgd(torch.bfloat16, 1e-6, 0.9, 0.0, 1e-4, False, False, False,
                                      lowp_dtype=torch.bfloat16)),
    }
    sel = args.ops.split(",")
    res = {(tu, op): [] for tu in sizes for op in sel}
    for r in range(args.rounds + 1):  # round 0 = warmup
        for op in sel:
            for tu in sizes:
                p = plans16[tu] if op.endswith("16") else plans[tu]
                for _ in range(args.launches):
                    ops[op][1](p)
                t = p.timer_read()
                if r > 0:
                    res[(tu, op)].extend(t)
    for (tu, op), t in res.items():
        med = statistics.median(t)
        bpp = ops[op][0]
        print(json.dumps({"tag": args.tag, "model": args.model, "replicas": args.replicas, "op": op,
                          "task_units": plans[tu].task_units, "n_tasks": plans[tu].n_tasks, "req": tu,
                          "median_ms": med, "min_ms": min(t), "GBps": bpp * n / (med * 1e-3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
