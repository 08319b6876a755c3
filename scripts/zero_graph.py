"""The reference's DeepSpeed CIFAR step (ResNet-18, bf16 model, ZeRO-2,
AdamW, gradient_clipping 1.0, train_batch_size 96,
R:resnet/deepspeed/deepspeed_train.py:170-223) on ZeroDataParallel(capturable=True):
eager vs recorded as one hipGraph with CapturedStep (lr schedule stepped
outside the graph).  Losses over the same batches and ms/step.

    python scripts/zero_graph.py [--steps 100] [--deterministic 0]
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
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--batch", type=int, default=96)
    ap.add_argument("--deterministic", type=int, default=1,
                    help="1: deterministic MIOpen (losses comparable bit for bit); 0: the default kernels (timing)")
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29621")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import distributed_training_amd as D
    from distributed_training_amd.resnet import MODELS
    from distributed_training_amd.zero import ZeroDataParallel

    torch.backends.cudnn.deterministic = bool(args.deterministic)
    g = torch.Generator(device=dev).manual_seed(1)
    xs = [torch.rand(args.batch, 3, 32, 32, device=dev, generator=g).to(torch.bfloat16) for _ in range(8)]
    ys = [torch.randint(0, 10, (args.batch,), device=dev, generator=g) for _ in range(8)]
    res = {}
    for mode in ("eager", "graph"):
        torch.manual_seed(0)
        model = MODELS["resnet18"](num_classes=10).to(dev).to(torch.bfloat16)
        eng = ZeroDataParallel(model, stage=2, optimizer="adamw", lr=1e-3, weight_decay=3e-7,
                               reduce_bucket_size=int(5e7), gradient_clipping=1.0, capturable=True)
        crit = nn.CrossEntropyLoss()

        def step(x, y):
            eng.prepare_backward()
            loss = crit(model(x).float(), y)
            loss.backward()
            eng.step()
            eng.zero_grad()
            return loss.detach()

        run = D.CapturedStep(step, optimizers=[eng], warmup=3) if mode == "graph" else step
        losses = []
        for i in range(12):
            losses.append(float(run(xs[i % 8], ys[i % 8])))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            run(xs[i % 8], ys[i % 8])
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        res[mode] = {"losses": losses, "ms_per_step": ms,
                     "captures": getattr(run, "captures", None), "replays": getattr(run, "replays", None)}
        print(json.dumps({"mode": mode, **res[mode]}), flush=True)
    le, lg = res["eager"]["losses"], res["graph"]["losses"]
    print(json.dumps({"deterministic": bool(args.deterministic), "max_loss_diff": max(abs(a - b) for a, b in zip(le, lg)),
                      "speedup": res["eager"]["ms_per_step"] / res["graph"]["ms_per_step"]}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
