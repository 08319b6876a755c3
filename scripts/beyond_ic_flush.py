"""The beyond-cache update rows back to back (each launch pays the write-back of
the previous launch's dirty lines) against the same launches with a 1 GiB read
between them (the previous launch's lines written back and evicted outside the
timed kernel, as in the training step, where ~40 ms of forward / backward
separate two updates).  ResNet-152 x 2 shapes; plan launch timer (the kernel's
own start / end, the flush never inside).  One JSON line per row and mode
(scripts/r4x_beyond_ic_flush.sh)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402

dev = torch.device("cuda", 0)
shapes = bench._beyond_ic_shapes()
numels = [int(torch.Size(s).numel()) for s in shapes]
n = sum(numels)
g = torch.Generator(device=dev).manual_seed(7)
grads = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
ps = [torch.randn(s, device=dev, generator=g) for s in shapes]
bs = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
vs = [torch.rand(s, device=dev, generator=g) * 1e-4 for s in shapes]
up = TensorListPlan(numels, dev, task_units=update_task_units(dev))
for k, ts in enumerate((ps, grads, bs, vs)):
    up.set_ptrs(k, ts)
scratch = torch.ones(256 * 1024 * 1024, device=dev)  # 1 GiB
acc = torch.zeros(1, device=dev)


def sgd():
    up.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False)


def adam():
    up.adam(torch.float32, 1e-6, 0.9, 0.999, 1e-8, 0.0, False, False, -1e-6, 0.5)


for rnd in range(2):
    for name, fn, bpe in (("sgd_momentum_wd", sgd, 20), ("adam", adam, 28)):
        for mode in ("back_to_back", "flushed"):
            for _ in range(3):
                fn()
            up.timer_enable(64)
            for _ in range(20):
                if mode == "flushed":
                    torch.sum(scratch, dim=0, out=acc[0])
                fn()
            ts = up.timer_read()
            up.timer_enable(0)
            ms = sum(ts) / len(ts)
            print(json.dumps({"round": rnd, "kernel": name, "mode": mode, "avg_ms": ms,
                              "frac": bpe * n / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
