"""Practical streaming ceiling at the grad-sync sizes: torch's own copy_ (one
fp32 tensor, read + write) vs libgsync pack (same bytes, 161-tensor R50 plan or
one tensor) at 25.6 M ... 240 M elements, HIP events around each launch.

    python scripts/copy_ceiling.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n=30):
    for _ in range(5):
        fn()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in evs)


def main():
    from distributed_training_amd.multi_tensor import TensorListPlan

    dev = torch.device("cuda", 0)
    for n in (25_557_032, 60_192_808, 120_385_616, 240_771_232):
        src = torch.randn(n, device=dev)
        dst = torch.empty_like(src)
        t_copy = timed(lambda: dst.copy_(src))
        plans = {}
        for tu in [int(x) for x in os.environ.get("CC_TASKS", "0,4096,8192").split(",")]:
            p = TensorListPlan([n], dev, task_units=tu)
            p.set_ptrs(0, [src])
            plans[tu] = (p.task_units, p.n_tasks, timed(lambda p=p: p.pack(0, torch.float32, dst, 0.5, 1)))
        row = {"elements": n, "bytes": 8 * n, "torch_copy_GBps": 8 * n / (t_copy * 1e-3) / 1e9}
        for tu, (u, k, t) in plans.items():
            row[f"pack_tu{tu}"] = {"task_units": u, "tasks": k, "GBps": 8 * n / (t * 1e-3) / 1e9}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
