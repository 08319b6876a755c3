"""configs[3]'s end of step in the training step itself: ResNet-50 bf16 under
ZeroDataParallel (stage 2, AdamW betas (0.8, 0.999), wd 3e-7, clip 1.0, one
5e7-element bucket), one-rank RCCL; the shard plan's kernels (Σg² partials,
then the clipped AdamW) timed by the plan launch timer inside real steps, under
the GS_NT_SQNORM / GS_RED_GRID of this process.  One JSON line (scripts/r4v_zero_instep.sh)."""
import json
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import DS_ADAM  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402
from distributed_training_amd.zero import ZeroDataParallel  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % int(sys.argv[1]), rank=0, world_size=1)
torch.backends.cudnn.benchmark = False
model = MODELS["resnet50"](num_classes=1000).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
zero = ZeroDataParallel(model, stage=2, optimizer="adamw", reduce_bucket_size=int(5e7), gradient_clipping=1.0,
                        **DS_ADAM)
g = torch.Generator(device=dev).manual_seed(1)
x = torch.rand(64, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last).to(torch.bfloat16)
y = torch.randint(0, 1000, (64,), device=dev, generator=g)
crit = torch.nn.CrossEntropyLoss()


def step():
    zero.prepare_backward()
    loss = crit(model(x).float(), y)
    loss.backward()
    zero.step()


for _ in range(5):
    step()
torch.cuda.synchronize()
zero.plan.timer_enable(64)
for _ in range(10):
    step()
torch.cuda.synchronize()
ts = zero.plan.timer_read()
zero.plan.timer_enable(0)
sq, upd = ts[0::2], ts[1::2]
n = sum(zero.shard_sizes)
print(json.dumps({"GS_NT_SQNORM": os.environ.get("GS_NT_SQNORM", "default"),
                  "GS_RED_GRID": os.environ.get("GS_RED_GRID", "default"), "shard_elems": n,
                  "sqnorm_partial_us": 1e3 * sum(sq) / len(sq), "adamw_us": 1e3 * sum(upd) / len(upd),
                  "sqnorm_frac": 2 * n / (sum(sq) / len(sq) * 1e-3) / 1e9 / 8000.0,
                  "adamw_frac": 28 * n / (sum(upd) / len(upd) * 1e-3) / 1e9 / 8000.0}), flush=True)
dist.destroy_process_group()
