"""Do the gradients of the exposed last DDP bucket keep their addresses from step
to step (bench.py's step: zero_grad(set_to_none=True), the caching allocator
hands out fresh grads)?  If they move, the bucket's pointer table is
re-uploaded (a staged H2D copy + an event) on the exposed tail every step.
Prints one JSON line: per step, how many of the last bucket's grads moved."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_training_amd as D  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"file:///tmp/gptr_{os.getpid()}")
torch.manual_seed(0)
model = MODELS["resnet50"](num_classes=1000).to(dev).to(memory_format=torch.channels_last)
ddp = D.DistributedDataParallel(model)
opt = D.FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
x = torch.rand(256, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (256,), device=dev)
crit = torch.nn.CrossEntropyLoss()
params = ddp._params
moved, prev = [], None
for it in range(8):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = crit(ddp(x), y)
    loss.backward()
    last = ddp._bucketer.buckets[-1]
    ptrs = [params[i].grad.data_ptr() for i in last]
    if prev is not None:
        moved.append(sum(a != b for a, b in zip(ptrs, prev)))
    prev = ptrs
    opt.step()
    opt.zero_grad(set_to_none=True)
torch.cuda.synchronize()
print(json.dumps({"last_bucket_params": len(prev), "moved_per_step": moved}), flush=True)
dist.destroy_process_group()
