"""CPU baseline: the reference's DDP training path on host cores.

TEST / MEASUREMENT INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).  It
restates R:resnet/pytorch_ddp/ddp_train.py:79-114 with the two changes
BASELINE.md prescribes: backend "gloo" and no .cuda(); the model is wrapped
in torch's own DistributedDataParallel and stepped with the reference's
Adam(lr=1e-3*ws) through the reference's train-step body (:62-72), on
synthetic data (seed 1234+rank).

Prints one JSON line: {"images_per_sec": ..., "cores": ..., ...}
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def worker(rank, args, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(args.port)
    dist.init_process_group("gloo", rank=rank, world_size=args.ws)  # :84 with gloo
    torch.set_num_threads(max(1, args.cores // args.ws))
    from torch.nn.parallel import DistributedDataParallel as DDP

    from distributed_training_amd.resnet import MODELS

    hw = 32 if args.model == "resnet18" else 224
    classes = 10 if args.model == "resnet18" else 1000
    torch.manual_seed(0)
    model = DDP(MODELS[args.model](num_classes=classes))  # :95 without .cuda()
    optimizer = torch.optim.Adam(model.parameters(), lr=1e-3 * args.ws)  # :97, :110
    criterion = nn.CrossEntropyLoss()
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.rand(args.batch, 3, hw, hw, generator=g)
    y = torch.randint(0, classes, (args.batch,), generator=g)
    model.train()
    times = []
    for it in range(args.warmup + args.steps):
        dist.barrier()
        t0 = time.perf_counter()
        outputs = model(x)                       # :66
        loss = criterion(outputs, y)             # :67
        loss.backward()                          # :70
        optimizer.step()                         # :71
        optimizer.zero_grad()                    # :72
        loss.item()                              # :75
        dist.barrier()
        if it >= args.warmup:
            times.append(time.perf_counter() - t0)
        if rank == 0:
            print(f"[cpu_baseline] step {it}: {time.perf_counter() - t0:.2f}s", file=sys.stderr, flush=True)
    # gloo all-reduce bus bandwidth at the model's fp32 grad size (BASELINE.md CPU plan)
    nparam = sum(p.numel() for p in model.parameters())
    buf = torch.ones(nparam)
    dist.all_reduce(buf)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.ar_iters):
        dist.all_reduce(buf)
    dist.barrier()
    ar_s = (time.perf_counter() - t0) / args.ar_iters
    if rank == 0:
        q.put((times, ar_s, nparam * 4))
    # torch's DDP here sits in a reference cycle that holds the process group: free it
    # before the teardown, so no gloo worker thread drops a Python tensor during
    # interpreter finalization (std::terminate)
    del model, optimizer, buf
    import gc

    gc.collect()
    dist.barrier()
    dist.destroy_process_group()


def cpu_model_name() -> str:
    """The host CPU model (lscpu's "Model name", read from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def run(model="resnet50", batch=16, ws=2, cores=None, steps=3, warmup=1, port=29777, ar_iters=3):
    if cores is None:
        cores = min(16, os.cpu_count() or 1)
    args = argparse.Namespace(model=model, batch=batch, ws=ws, cores=cores, steps=steps, warmup=warmup, port=port,
                              ar_iters=ar_iters)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=worker, args=(r, args, q)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
    times, ar_s, ar_bytes = q.get()
    mean = sum(times) / len(times)
    return {
        "gloo_allreduce_bytes": ar_bytes,
        "gloo_allreduce_ms": ar_s * 1e3,
        "gloo_allreduce_busbw_GBps": ar_bytes / ar_s * 2 * (ws - 1) / ws / 1e9,
        "images_per_sec": ws * batch / mean,
        "step_s": mean,
        "cores": cores,
        "ws": ws,
        "batch_per_rank": batch,
        "steps": steps,
        "model": model,
        "cpu_model": cpu_model_name(),
    }


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--ws", type=int, default=2)
    ap.add_argument("--cores", type=int, default=None)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--port", type=int, default=29777)
    a = ap.parse_args()
    print(json.dumps(run(a.model, a.batch, a.ws, a.cores, a.steps, a.warmup, a.port)))
