"""The reference's DDP trainer (R:resnet/pytorch_ddp/ddp_train.py) on libgsync.

Same structure and hyper-parameters as the reference — ResNet-18 / CIFAR-10,
``DDP(model)`` (:95), ``Adam(lr=1e-3 * world_size)`` (:97, :110), batch 100
(:111), ``sampler.set_epoch(epoch)`` every epoch (:102), the train-step body
(:62-72) — with libgsync's DDP, fused Adam and device-resident input step.
There is no download: ``$DATA`` (default ../data) is read as the CIFAR-10
binary distribution when present, otherwise a seeded synthetic set of the
same shape is used.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/ddp_train.py        # one GPU per rank (RCCL)
    python examples/ddp_train.py --device cpu --world-size 2                            # CPU / gloo (config 1)
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_training_amd import DDP, FusedAdam as Adam  # noqa: E402
from distributed_training_amd import data as D  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402


def build_dataloader(batch_size: int, device, synthetic_n: int = 50000):
    """R:ddp_train.py:25-48 on device-resident data."""
    data_path = os.environ.get("DATA", "../data")
    try:
        train = D.ImageDataset.cifar10_bin(data_path, train=True, device=device)
        test = D.ImageDataset.cifar10_bin(data_path, train=False, device=device)
    except FileNotFoundError:
        train = D.ImageDataset.synthetic(synthetic_n, seed=0, device=device)
        test = D.ImageDataset.synthetic(max(1, synthetic_n // 5), seed=1, device=device)
    return D.build_dataloader(batch_size, train, test)


def train_epoch(epoch, num_epochs, model, optimizer, criterion, train_dataloader, max_steps=None):
    """R:ddp_train.py:52-75 (tqdm progress bar omitted); returns the last loss."""
    model.train()
    loss = None
    for k, (images, labels) in enumerate(train_dataloader):
        if max_steps is not None and k >= max_steps:
            break
        outputs = model(images)
        loss = criterion(outputs, labels)
        loss.backward()
        optimizer.step()
        optimizer.zero_grad()
    return None if loss is None else loss.item()


def ddp(rank, world_size, num_epochs, learning_rate, batch_size, device_type="cuda", max_steps=None,
        synthetic_n=50000, port=12355, result=None, local_rank=None):
    """R:ddp_train.py:94-105 (ddp_setup :79-85 with the backend chosen by device)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(port))
    if device_type == "cuda":
        device = torch.device("cuda", rank if local_rank is None else local_rank)
        torch.cuda.set_device(device)
        dist.init_process_group("nccl", rank=rank, world_size=world_size, device_id=device)
    else:
        device = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world_size)
    torch.manual_seed(0)
    model = DDP(MODELS["resnet18"](num_classes=10).to(device))
    train_dataloader, _ = build_dataloader(batch_size, device, synthetic_n)
    optimizer = Adam(model.parameters(), lr=learning_rate)
    criterion = nn.CrossEntropyLoss()
    last = None
    for epoch in range(num_epochs):
        train_dataloader.sampler.set_epoch(epoch)
        last = train_epoch(epoch, num_epochs, model, optimizer, criterion, train_dataloader, max_steps)
        if rank == 0:
            print(f"epoch {epoch + 1}/{num_epochs} loss {last:.4f}", flush=True)
    if result is not None and rank == 0:
        result.put({k: v.detach().cpu().numpy().copy() for k, v in model.module.state_dict().items()})
    dist.destroy_process_group()
    return last


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--world-size", type=int, default=2, help="processes to spawn when not under torchrun")
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=100)
    ap.add_argument("--max-steps", type=int, default=None)
    a = ap.parse_args()
    if "RANK" in os.environ:  # torchrun
        ws = int(os.environ["WORLD_SIZE"])
        ddp(int(os.environ["RANK"]), ws, a.epochs, 1e-3 * ws, a.batch_size, a.device, a.max_steps,
            local_rank=int(os.environ.get("LOCAL_RANK", "0")))
    else:
        ws = a.world_size
        mp.spawn(ddp, args=(ws, a.epochs, 1e-3 * ws, a.batch_size, a.device, a.max_steps), nprocs=ws)


if __name__ == "__main__":
    main()
