"""Input step measurement: libgsync's device-resident CIFAR
loader vs the reference pipeline (torch DataLoader + per-sample transforms +
H2D, R:resnet/pytorch_ddp/ddp_train.py:25-48,62).

    python scripts/bench_input.py [--batches 64]

Rows (JSON, one per line):
  kernel     gs_image_augment alone, HIP events on its stream, at batch
             256 / 4096 / 16384: algorithmic bytes = per sample C*h*w*(1 + 4)
             (uint8 read, f32 write) + 32 B (params, label read/write)
  loader     whole libgsync loader per batch (host param draws from torch's
             generator, 16 B/sample H2D, kernel), images/s
  reference  oracle/input_pipeline.py (torch's DataLoader + DistributedSampler,
             numpy restatement of torchvision's transforms) + .to(device),
             images/s on the host, bounded sample
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=64)
    ap.add_argument("--ref-batches", type=int, default=8)
    args = ap.parse_args()
    from distributed_training_amd import _lib as L
    from distributed_training_amd import data as D

    dev = torch.device("cuda", 0)
    ds = D.ImageDataset.synthetic(50000, device=dev, seed=0)
    per = 3 * 32 * 32
    for B in (256, 4096, 16384):
        g = torch.Generator().manual_seed(B)
        idx = torch.randint(0, ds.n, (B,), generator=g)
        params = torch.stack([idx, torch.randint(0, 2, (B,), generator=g), torch.randint(0, 9, (B,), generator=g),
                              torch.randint(0, 9, (B,), generator=g)], 1).to(torch.int32).to(dev)
        out = torch.empty(B, 3, 32, 32, device=dev)
        lab = torch.empty(B, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream(dev)

        def launch():
            L.check(L.lib().gs_image_augment(L.GS_DEV_HIP, 0, ds.images.data_ptr(), ds.labels.data_ptr(), ds.n, 32,
                                              32, 3, 4, 32, 32, params.data_ptr(), B, out.data_ptr(), L.GS_F32,
                                              L.GS_LAYOUT_NCHW, lab.data_ptr(), s.cuda_stream), "gs_image_augment")

        for _ in range(5):
            launch()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
        for a, b in evs:
            a.record(s)
            launch()
            b.record(s)
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in evs)[25]
        nbytes = B * (per * 5 + 32)
        print(json.dumps({"row": "kernel", "batch": B, "median_ms": ms, "alg_bytes": nbytes,
                          "GBps": nbytes / (ms * 1e-3) / 1e9, "images_per_s": B / (ms * 1e-3)}), flush=True)

    ld = D.DeviceDataLoader(ds, batch_size=256, drop_last=True, transform=D.TRAIN_TRANSFORM,
                            sampler=D.DistributedSampler(ds, num_replicas=1, rank=0))
    it = iter(ld)
    next(it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for _ in range(args.batches):
        x, y = next(it)
        n += x.shape[0]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"row": "loader", "batch": 256, "batches": args.batches, "images_per_s": n / dt,
                      "ms_per_batch": dt / args.batches * 1e3}), flush=True)

    from oracle import input_pipeline as R

    imgs, labels = ds.images.cpu().numpy(), ds.labels.cpu().numpy()
    ref = R.reference_loader(imgs, labels, 256, 1, 0, train=True, drop_last=True)
    it = iter(ref)
    next(it)
    t0 = time.perf_counter()
    n = 0
    for _ in range(args.ref_batches):
        x, y = next(it)
        x, y = x.to(dev), y.to(dev)
        n += x.shape[0]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"row": "reference", "batch": 256, "batches": args.ref_batches, "images_per_s": n / dt,
                      "ms_per_batch": dt / args.ref_batches * 1e3, "cores": 1,
                      "note": "torch DataLoader num_workers=0 (as R:ddp_train.py:46), numpy transforms, H2D"}),
          flush=True)


if __name__ == "__main__":
    main()
