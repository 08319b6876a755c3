"""The reference's own workload on one MI355X: ResNet-18 / CIFAR-10 shape,
batch 100, Adam(lr=1e-3*ws), DDP (R:resnet/pytorch_ddp/ddp_train.py:94-111),
ws=1 over RCCL.  Times a step (forward, backward + grad sync, optimizer) for

  torch      torch DDP + torch.optim.Adam (the reference path)
  libgsync   libgsync DDP + FusedAdam
  graph      libgsync DDP + FusedAdam(capturable) with the step replayed as one hipGraph
and the input step per batch (torch DataLoader + transforms + H2D vs the
device-resident loader) — images/s for each.

    python scripts/bench_cifar.py [--steps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=100)
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import distributed_training_amd as D
    from distributed_training_amd.resnet import MODELS

    x = torch.rand(args.batch, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (args.batch,), device=dev)
    crit = nn.CrossEntropyLoss()
    rows = []
    for impl in ("torch", "libgsync", "graph", "torch", "libgsync", "graph"):
        torch.manual_seed(0)
        model = MODELS["resnet18"](num_classes=10).to(dev)
        if impl == "torch":
            ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0])
            opt = torch.optim.Adam(ddp.parameters(), lr=1e-3)
        else:
            ddp = D.DistributedDataParallel(model)
            opt = D.FusedAdam(ddp.parameters(), lr=1e-3, capturable=impl == "graph")

        def train(xb, yb):
            opt.zero_grad(set_to_none=True)
            loss = crit(ddp(xb), yb)
            loss.backward()
            opt.step()
            return loss

        run = D.CapturedStep(train, optimizers=[opt]) if impl == "graph" else train

        def step():
            run(x, y)

        for _ in range(10):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        rows.append({"impl": impl, "ms_per_step": dt * 1e3, "images_per_s": args.batch / dt})
        print(json.dumps(rows[-1]), flush=True)
        del ddp, opt, model
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
