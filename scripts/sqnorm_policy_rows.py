"""bench.py's own kernel rows (ResNet-50 shapes, `_kernel_rows`) and configs[3]'s
N=8-shard ZeRO clip path (`zero_clip_path_rows`, one-rank RCCL) plus the clip
chain (scripts/sqnorm_chain.py's unpack -> Σg² partials -> clipped SGD at
ResNet-50), under the GS_NT_SQNORM of this process; one JSON line per row
(scripts/r4u_sqnorm_policy.sh)."""
import json
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from distributed_training_amd.comm import get_communicator  # noqa: E402
from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

pol = os.environ.get("GS_NT_SQNORM", "default")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % int(sys.argv[1]), rank=0, world_size=1)
with torch.device("meta"):
    m = MODELS["resnet50"](num_classes=1000)
shapes = [tuple(p.shape) for p in m.parameters()]
n, rows = bench._kernel_rows(shapes, dev, 20)
for k in ("sqnorm_f32", "sqnorm_partial_f32", "clip_path_sgd", "sgd_momentum_wd", "unpack_f32+sqnorm"):
    print(json.dumps({"GS_NT_SQNORM": pol, "row": k, "frac": rows[k]["frac"], "avg_ms": rows[k]["avg_ms"]}), flush=True)
z = bench.zero_clip_path_rows(n, dev, get_communicator(None, dev))
for k, r in z.items():
    print(json.dumps({"GS_NT_SQNORM": pol, "row": k, "avg_ms": r["avg_ms"], "kernels_ms": r["kernels_ms"]}), flush=True)
# the chain: the grads just written by an unpack
numels = [int(torch.Size(s).numel()) for s in shapes]
g = torch.Generator(device=dev).manual_seed(3)
grads = [torch.zeros(s, device=dev) for s in shapes]
ps = [torch.randn(s, device=dev, generator=g) for s in shapes]
bufs = [torch.randn(s, device=dev, generator=g) * 0.01 for s in shapes]
bplan = TensorListPlan(numels, dev, align=64)
bplan.set_ptrs(1, grads)
flat = torch.randn(bplan.flat_numel, device=dev, generator=g) * 0.01
plan = TensorListPlan(numels, dev, task_units=update_task_units(dev))
for k, ts in enumerate((ps, grads, bufs)):
    plan.set_ptrs(k, ts)
out = torch.zeros(3, device=dev)


def step():
    bplan.unpack(flat, 1, torch.float32)
    plan.sqnorm_partial(1, torch.float32)
    plan.set_clip(1.0, 1e-6, None, 1.0, 1.0, out=out)
    plan.sgd(torch.float32, 1e-9, 0.9, 0.0, 1e-4, False, False, False)


for _ in range(3):
    step()
plan.timer_enable(128)
for _ in range(30):
    step()
upd = plan.timer_read()
plan.timer_enable(0)
tot = sum(upd) / 30
print(json.dumps({"GS_NT_SQNORM": pol, "row": "chain_clip_path_total", "frac": 24 * n / (tot * 1e-3) / 1e9 / 8000.0,
                  "avg_ms": tot}), flush=True)
dist.destroy_process_group()
