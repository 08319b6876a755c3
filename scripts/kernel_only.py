"""Runs only one libgsync grad-sync kernel over a model's parameter set, N
launches — the unit a rocprofv3 PMC pass (FETCH_SIZE / WRITE_SIZE) measures.
    python scripts/kernel_only.py <model> <launches> <op> [replicas]
op: sgd | adam (update plan, as FusedSGD / FusedAdam build it), clipsgd (the folded clip
    path on the update plan: gs_sqnorm_partial + the clipped SGD, max_norm 1.0),
    pack | pack16 | pack16b | unpack | unpacksq | sqnorm | sqpart (bucket-layout plan, align 64;
    pack16 = fp32 grads -> bf16 bucket, pack16b = bf16 grads -> bf16 bucket (ZeRO-2's pack);
    sqpart = gs_sqnorm_partial, the folded clip's Σg² launch; clipscale = clip_grad_norm_'s scale
    pass, gs_clip_scale, at a fixed coefficient 0.1 so every launch writes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
op = sys.argv[3] if len(sys.argv) > 3 else "sgd"
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
dev = torch.device("cuda", 0)
shapes = [p.shape for p in MODELS[model]().parameters()] * reps
n = [torch.Size(s).numel() for s in shapes]
gdt = torch.bfloat16 if op == "pack16b" else torch.float32
gs = [(torch.randn(s, device=dev) * 0.01).to(gdt) for s in shapes]
if op in ("sgd", "adam", "clipsgd"):
    ps = [torch.randn(s, device=dev) for s in shapes]
    bs = [torch.randn(s, device=dev) * 0.01 for s in shapes]
    vs = [torch.rand(s, device=dev) * 1e-4 for s in shapes] if op == "adam" else None
    plan = TensorListPlan(n, dev, task_units=update_task_units(dev))
    for k, ts in enumerate((ps, gs, bs) + ((vs,) if vs is not None else ())):
        plan.set_ptrs(k, ts)
else:
    plan = TensorListPlan(n, dev, align=64)
    plan.set_ptrs(1, gs)
    flat = torch.zeros(plan.flat_numel, device=dev, dtype=torch.bfloat16 if op in ("pack16", "pack16b") else torch.float32)
    sq = torch.zeros(1, device=dev)
    sq100 = torch.full((1,), 100.0, device=dev)  # clipscale: ||g|| = 10, max_norm 1 -> coefficient ~0.1
for _ in range(iters):
    if op == "adam":
        plan.adam(torch.float32, 1e-6, 0.9, 0.999, 1e-8, 0.0, False, False, -1e-6, 0.5)
    elif op == "sgd":
        plan.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False)
    elif op == "clipsgd":
        plan.sqnorm_partial(1, torch.float32)
        plan.set_clip(1.0)
        plan.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False)
    elif op in ("pack", "pack16", "pack16b"):
        plan.pack(1, gdt, flat, 0.125, 1)
    elif op == "unpack":
        plan.unpack(flat, 1, torch.float32)
    elif op == "unpacksq":
        plan.unpack(flat, 1, torch.float32, sqnorm=sq)
    elif op == "sqnorm":
        plan.sqnorm(1, torch.float32, sq)
    elif op == "sqpart":
        plan.sqnorm_partial(1, torch.float32)
    elif op == "clipscale":
        plan.set_clip(1.0, 1e-6, sq100)
        plan.clip_scale(1, torch.float32)
torch.cuda.synchronize()
print("params", sum(n), "launches", iters, "op", op)
