"""Host-side profile of small training steps on the GPU (where a launch-bound
step spends its CPU time): cProfile over N steps of ResNet-18 x8 with libgsync
DDP + FusedSGD, top functions by internal time (ctypes calls count to their
Python caller)."""
import cProfile
import os
import pstats
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29571")
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
import distributed_training_amd as D  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

impl = sys.argv[1] if len(sys.argv) > 1 else "libgsync"
model = MODELS["resnet18"](num_classes=1000).to(dev).to(memory_format=torch.channels_last)
if impl == "libgsync":
    ddp = D.DistributedDataParallel(model)
    opt = D.FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
else:
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0])
    opt = torch.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, foreach=True)
x = torch.rand(8, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (8,), device=dev)
crit = torch.nn.CrossEntropyLoss()


def step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = crit(ddp(x), y)
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)


for _ in range(10):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
