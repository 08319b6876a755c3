"""Runs only the libgsync fused SGD (or Adam) kernel over a model's parameter
set (ResNet-50: 25.56M params in 161 tensors), N launches — the unit the PMC
traffic pass measures (bench.py's roofline kernel).
    python scripts/sgd_only.py [model] [launches] [sgd|adam]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
op = sys.argv[3] if len(sys.argv) > 3 else "sgd"
dev = torch.device("cuda", 0)
shapes = [p.shape for p in MODELS[model]().parameters()]
ps = [torch.randn(s, device=dev) for s in shapes]
gs = [torch.randn(s, device=dev) * 0.01 for s in shapes]
bs = [torch.randn(s, device=dev) * 0.01 for s in shapes]
vs = [torch.rand(s, device=dev) * 1e-4 for s in shapes] if op == "adam" else None
plan = TensorListPlan([p.numel() for p in ps], dev, task_units=update_task_units(dev))  # as FusedSGD/FusedAdam
for k, ts in enumerate((ps, gs, bs) + ((vs,) if vs is not None else ())):
    plan.set_ptrs(k, ts)
for _ in range(iters):
    if op == "adam":
        plan.adam(torch.float32, 1e-6, 0.9, 0.999, 1e-8, 0.0, False, False, -1e-6, 0.5)
    else:
        plan.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False)
torch.cuda.synchronize()
print("params", sum(p.numel() for p in ps), "launches", iters)
