"""The 16-bit packs alone (ZeRO's bf16 grads -> bf16 bucket x 1/ws; fp32 -> bf16),
plan launch timer, on ResNet-50's parameter shapes and ResNet-152's x 2 (beyond
the Infinity Cache); the library picked by GSYNC_LIB (variants of the group size,
scripts/r4k_pack16.sh).  One JSON line per row."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_amd.multi_tensor import TensorListPlan  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
tag = os.environ.get("GSYNC_LIB", "libgsync").split("/")[-1]
for model, reps in (("resnet50", 1), ("resnet152", 2)):
    with torch.device("meta"):
        m = MODELS[model](num_classes=1000)
    shapes = [tuple(p.shape) for p in m.parameters()] * reps
    numels = [int(torch.Size(s).numel()) for s in shapes]
    n = sum(numels)
    g = torch.Generator(device=dev).manual_seed(3)
    for src_dt, nbytes in ((torch.bfloat16, 4), (torch.float32, 6)):
        grads = [(torch.randn(s, device=dev, generator=g) * 0.01).to(src_dt) for s in shapes]
        plan = TensorListPlan(numels, dev, align=64)
        plan.set_ptrs(1, grads)
        flat = torch.zeros(plan.flat_numel, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            plan.pack(1, src_dt, flat, 0.125, 1)
        plan.timer_enable(64)
        for _ in range(30):
            plan.pack(1, src_dt, flat, 0.125, 1)
        ts = plan.timer_read()
        plan.timer_enable(0)
        ms = sum(ts) / len(ts)
        print(json.dumps({"lib": tag, "model": model, "replicas": reps, "src": str(src_dt), "elems": n,
                          "avg_ms": ms, "frac": nbytes * n / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
        del grads, flat, plan
        torch.cuda.empty_cache()
