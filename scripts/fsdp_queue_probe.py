"""Why torch FSDP's configs[3] step read 108 ms inside the bench process against
81.5 ms standalone (DESIGN §5, r6d / r6f against r6e): the same FSDP(SHARD_GRAD_OP,
bf16) + clip + fused AdamW step on ResNet-50 x 256, timed fresh, then after the
process has created more HIP streams — torch pool streams with a kernel each, then
libgsync communicators (one high-priority stream each), as the bench's earlier legs
leave them.  HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues
(4 on the box); streams that share one run in submission order.  `--lazy-pg`: the
process group without device_id (lazy communicator, as the libgsync bench process
creates it), then a libgsync DDP step run before FSDP as the headline does.  One JSON
line per phase.

    python scripts/fsdp_queue_probe.py [--lazy-pg] > rows.jsonl
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_training_amd.resnet import MODELS  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29655")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
LAZY = "--lazy-pg" in sys.argv
dist.init_process_group("nccl", rank=0, world_size=1, **({} if LAZY else dict(device_id=dev)))
DS_ADAM = dict(lr=1e-3, betas=(0.8, 0.999), eps=1e-8, weight_decay=3e-7)


def fsdp_time(label, steps=10, warmup=4):
    from torch.distributed.fsdp import FullyShardedDataParallel as FSDP, MixedPrecision, ShardingStrategy

    torch.manual_seed(0)
    bf = torch.bfloat16
    model = MODELS["resnet50"](num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    fsdp = FSDP(model, sharding_strategy=ShardingStrategy.SHARD_GRAD_OP, device_id=dev,
                mixed_precision=MixedPrecision(param_dtype=bf, reduce_dtype=bf, buffer_dtype=bf))
    opt = torch.optim.AdamW(fsdp.parameters(), fused=True, **DS_ADAM)
    g = torch.Generator(device=dev).manual_seed(4321)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last).to(bf)
    y = torch.randint(0, 1000, (256,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()

    def one():
        crit(fsdp(x).float(), y).backward()
        fsdp.clip_grad_norm_(1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(json.dumps({"phase": label, "ms_per_step": round(ms, 2), "images_per_sec": round(256e3 / ms, 1),
                      "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "lazy_pg": LAZY}), flush=True)
    del fsdp, opt, model
    torch.cuda.empty_cache()


fsdp_time("fresh")
keep = []
for k in range(6):
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        keep.append(torch.ones(16, device=dev).add_(1))
    keep.append(s)
torch.cuda.synchronize()
fsdp_time("after 6 torch pool streams")
from distributed_training_amd.comm import Communicator  # noqa: E402

comms = [Communicator(None, dev) for _ in range(3)]
for c in comms:
    c.all_reduce(torch.ones(4, device=dev))
torch.cuda.synchronize()
fsdp_time("after 3 libgsync communicators")
if LAZY:
    import distributed_training_amd as D

    torch.manual_seed(0)
    m = MODELS["resnet50"](num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    ddp = D.DistributedDataParallel(m)
    opt = D.FusedSGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    xx = torch.rand(256, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    yy = torch.randint(0, 1000, (256,), device=dev)
    for _ in range(6):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = torch.nn.functional.cross_entropy(ddp(xx), yy)
        loss.backward()
        opt.step()
        opt.zero_grad()
    torch.cuda.synchronize()
    ddp.close()
    del ddp, opt, m, xx, yy
    torch.cuda.empty_cache()
    fsdp_time("after a libgsync DDP ResNet-50 run")
for c in comms:
    c.close()
dist.destroy_process_group()
