"""bench.py's grad_sync_kernel_rates on a model's parameter set, alone, one
JSON line per call: for A/B runs of library variants (GSYNC_LIB=...).

    python scripts/kernel_rates.py [resnet50] [label]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(os.environ.get("GSYNC_LIB", "libgsync.so"))
dev = torch.device("cuda", 0)
params = list(MODELS[name]().to(dev).parameters())
r = bench.grad_sync_kernel_rates(params, dev, iters=50)
print(json.dumps({"label": label, "model": name,
                  "frac": {k: round(v["frac"], 4) for k, v in r["kernels"].items()},
                  "us": {k: round(v["avg_ms"] * 1e3, 2) for k, v in r["kernels"].items()}}), flush=True)
