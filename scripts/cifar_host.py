"""Where an eager step of the reference's own workload spends its time on one
MI355X: ResNet-18 / CIFAR-10 shape, batch 100, Adam(lr=1e-3)
(R:resnet/pytorch_ddp/ddp_train.py:94-111), ws=1 over RCCL.

Variants (interleaved, two rounds each), per step: wall ms (synchronised
every step), and the host time spent issuing forward / backward / step /
zero_grad (no synchronisation inside the step, so these are enqueue costs as
long as the GPU queue does not fill):

  torch        torch DDP + torch.optim.Adam (foreach; the reference path)
  torch_fused  torch DDP + torch.optim.Adam(fused=True)
  gsync        libgsync DDP + FusedAdam (GSYNC_NATIVE_HOOK decides the hook)
  nodpp        no DDP + FusedAdam (the floor for gradient-sync host cost)
  colossal     the reference's Colossal step: Booster(TorchDDPPlugin, fp16) + HybridAdam (shim)
  torch_amp    the same fp16 step on torch: DDP + autocast + GradScaler + torch.optim.Adam

    python scripts/cifar_host.py [--steps 100] [--out file.jsonl]
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
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--impls", default="torch,torch_fused,gsync,nodpp")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29613")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import distributed_training_amd as D
    from distributed_training_amd.resnet import MODELS

    x = torch.rand(args.batch, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (args.batch,), device=dev)
    crit = nn.CrossEntropyLoss()
    out = open(args.out, "a") if args.out else None
    for rnd in range(args.rounds):
        for impl in args.impls.split(","):
            torch.manual_seed(0)
            model = MODELS["resnet18"](num_classes=10).to(dev)
            if impl in ("torch", "torch_fused"):
                ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0])
                opt = torch.optim.Adam(ddp.parameters(), lr=1e-3, fused=impl == "torch_fused")
            elif impl == "gsync":
                ddp = D.DistributedDataParallel(model)
                opt = D.FusedAdam(ddp.parameters(), lr=1e-3)
            elif impl == "colossal":
                # the reference's Colossal run (R:resnet/colossal/colossal_train.py:118-161,
                # run.sh torch_ddp_fp16): Booster(TorchDDPPlugin, fp16) + HybridAdam on the shim
                from distributed_training_amd.compat import colossalai as C

                booster = C.Booster(plugin=C.TorchDDPPlugin(), mixed_precision="fp16")
                hopt = C.HybridAdam(model.parameters(), lr=1e-3)
                cmodel, copt, ccrit, _, _ = booster.boost(model, hopt, criterion=crit)
                ddp = next(m for m in cmodel.modules() if isinstance(m, D.DistributedDataParallel))

                class _Step:  # booster.backward + step, behind the loop's zero_grad/ddp/step calls
                    def zero_grad(self, set_to_none=True):
                        copt.zero_grad()

                    def step(self):
                        copt.step()

                opt = _Step()
            elif impl == "torch_amp":
                # the same fp16 step on torch alone: DDP + autocast + GradScaler + torch.optim.Adam
                ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0])
                tadam = torch.optim.Adam(ddp.parameters(), lr=1e-3)
                scaler = torch.amp.GradScaler("cuda")
            else:
                ddp = model
                opt = D.FusedAdam(model.parameters(), lr=1e-3)
            t = {"fwd": 0.0, "bwd": 0.0, "step": 0.0, "zero": 0.0}

            def one(acc):
                pc = time.perf_counter
                a = pc()
                if impl == "torch_amp":
                    tadam.zero_grad(set_to_none=True)
                    b = pc()
                    with torch.autocast("cuda", dtype=torch.float16):
                        loss = crit(ddp(x), y)
                    c = pc()
                    scaler.scale(loss).backward()
                    d = pc()
                    scaler.step(tadam)
                    scaler.update()
                    e = pc()
                elif impl == "colossal":
                    opt.zero_grad()
                    b = pc()
                    loss = ccrit(cmodel(x), y)
                    c = pc()
                    booster.backward(loss, copt)
                    d = pc()
                    opt.step()
                    e = pc()
                else:
                    opt.zero_grad(set_to_none=True)
                    b = pc()
                    loss = crit(ddp(x), y)
                    c = pc()
                    loss.backward()
                    d = pc()
                    opt.step()
                    e = pc()
                if acc:
                    t["zero"] += b - a
                    t["fwd"] += c - b
                    t["bwd"] += d - c
                    t["step"] += e - d

            for _ in range(15):
                one(False)
            torch.cuda.synchronize()
            # wall: synchronised per step (the reference's loop reads loss.item())
            t0 = time.perf_counter()
            for _ in range(args.steps):
                one(True)
                torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / args.steps * 1e3
            # pipelined: no sync inside (host-bound vs GPU-bound shows here)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                one(False)
            torch.cuda.synchronize()
            piped = (time.perf_counter() - t1) / args.steps * 1e3
            row = {"impl": impl, "round": rnd, "native_hook": getattr(ddp, "_native", None) is not None,
                   "ms_per_step_synced": wall, "ms_per_step_pipelined": piped,
                   "images_per_s_synced": args.batch / wall * 1e3,
                   "host_ms": {k: v / args.steps * 1e3 for k, v in t.items()}}
            print(json.dumps(row), flush=True)
            if out:
                out.write(json.dumps(row) + "\n")
                out.flush()
            del ddp, model
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
