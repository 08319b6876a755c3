"""The fused SGD and Adam back to back at ResNet-50 and ResNet-152 x 2 sizes
(plan launch timer), labelled with this process's ROWS_LABEL (a library
variant) or GS_UPD_CONTIG (the update grid: one group per workgroup, or a capped
grid of contiguous group ranges).
One JSON line per row (scripts/r4y_upd_contig.sh)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
label = os.environ.get("ROWS_LABEL", os.environ.get("GS_UPD_CONTIG", "0"))
with torch.device("meta"):
    r50 = [tuple(p.shape) for p in MODELS["resnet50"](num_classes=1000).parameters()]
for setname, shapes in (("resnet50", r50), ("resnet152x2", bench._beyond_ic_shapes())):
    numels = [int(torch.Size(s).numel()) for s in shapes]
    n = sum(numels)
    g = torch.Generator(device=dev).manual_seed(7)
    ts = [[torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes] for _ in range(4)]
    up = TensorListPlan(numels, dev, task_units=update_task_units(dev))
    for k in range(4):
        up.set_ptrs(k, ts[k])
    for name, bpe, fn in (("sgd_momentum_wd", 20, lambda: up.sgd(torch.float32, 1e-6, 0.9, 0.0, 1e-4, False, False, False)),
                          ("adam", 28, lambda: up.adam(torch.float32, 1e-6, 0.9, 0.999, 1e-8, 0.0, False, False, -1e-6, 0.5))):
        for _ in range(3):
            fn()
        up.timer_enable(64)
        for _ in range(20):
            fn()
        t = up.timer_read()
        up.timer_enable(0)
        ms = sum(t) / len(t)
        print(json.dumps({"GS_UPD_CONTIG": os.environ.get("GS_UPD_CONTIG", "0"), "variant": label, "set": setname,
                          "kernel": name, "avg_ms": ms, "frac": bpe * n / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
    del ts, up
    torch.cuda.empty_cache()
