"""The reference's DeepSpeed workload on one MI355X: ResNet-18 / CIFAR-10
shape, bf16 model, ZeRO-2, AdamW, gradient_clipping 1.0, train_batch_size 96
(R:resnet/deepspeed/deepspeed_train.py:170-223), ws=1 over RCCL — a
host-bound step.  Times (synchronised every step, as the reference reads
loss.item()) and splits the host time:

  zero2   libgsync ZeroDataParallel stage 2 (GSYNC_NATIVE_HOOK decides the hook)
  floor   the same bf16 model's forward + backward alone (no optimizer, no
          gradient sync): what any ZeRO engine adds its step on top of

    python scripts/zero_host.py [--steps 100] [--out file.jsonl]
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
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=96)
    ap.add_argument("--impls", default="zero2,floor")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29617")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import distributed_training_amd as D
    from distributed_training_amd.resnet import MODELS
    from distributed_training_amd.zero import ZeroDataParallel

    x = torch.rand(args.batch, 3, 32, 32, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 10, (args.batch,), device=dev)
    crit = nn.CrossEntropyLoss()
    out = open(args.out, "a") if args.out else None
    for rnd in range(args.rounds):
        for impl in args.impls.split(","):
            torch.manual_seed(0)
            model = MODELS["resnet18"](num_classes=10).to(dev).to(torch.bfloat16)
            t = {"fwd": 0.0, "bwd": 0.0, "step": 0.0}
            if impl == "zero2":
                eng = ZeroDataParallel(model, stage=2, optimizer="adamw", lr=1e-3, weight_decay=3e-7,
                                       reduce_bucket_size=int(5e7), gradient_clipping=1.0)

                def one(acc):
                    pc = time.perf_counter
                    a = pc()
                    eng.prepare_backward()
                    loss = crit(model(x).float(), y)
                    b = pc()
                    loss.backward()
                    c = pc()
                    eng.step()
                    d = pc()
                    if acc:
                        t["fwd"] += b - a
                        t["bwd"] += c - b
                        t["step"] += d - c
            else:
                def one(acc):  # the model alone: forward + backward, grads dropped
                    pc = time.perf_counter
                    a = pc()
                    loss = crit(model(x).float(), y)
                    b = pc()
                    loss.backward()
                    c = pc()
                    for p in model.parameters():
                        p.grad = None
                    d = pc()
                    if acc:
                        t["fwd"] += b - a
                        t["bwd"] += c - b
                        t["step"] += d - c

            for _ in range(15):
                one(False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                one(True)
                torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / args.steps * 1e3
            row = {"impl": impl, "round": rnd, "native_hook": os.environ.get("GSYNC_NATIVE_HOOK", "1") != "0",
                   "ms_per_step_synced": wall, "images_per_s": args.batch / wall * 1e3,
                   "host_ms": {k: v / args.steps * 1e3 for k, v in t.items()}}
            print(json.dumps(row), flush=True)
            if out:
                out.write(json.dumps(row) + "\n")
                out.flush()
            if impl == "zero2":
                eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
