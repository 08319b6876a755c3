"""Input step on the GPU: the gfx950 gather/pad/flip/crop/
ToTensor kernel vs the host backend (itself pinned to the reference pipeline
in tests/test_data_cpu.py), bit for bit, every layout and dtype."""
import numpy as np
import pytest
import torch

from distributed_training_amd import data as D
from oracle import input_pipeline as R

pytestmark = pytest.mark.gpu


def _images(n, seed=0):
    g = np.random.default_rng(seed)
    return g.integers(0, 256, (n, 32, 32, 3), dtype=np.uint8), g.integers(0, 10, n)


@pytest.mark.parametrize("transform", ["train", "test"])
@pytest.mark.parametrize("fmt", ["nchw", "nhwc"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_device_loader_equals_host_loader(cuda_device, transform, fmt, dtype):
    imgs, labels = _images(1000)
    tf = D.TRAIN_TRANSFORM if transform == "train" else D.TEST_TRANSFORM
    mf = torch.channels_last if fmt == "nhwc" else torch.contiguous_format
    out = {}
    for dev in ("cpu", cuda_device):
        ds = D.ImageDataset(imgs, labels, dev)
        ld = D.DeviceDataLoader(ds, batch_size=100, drop_last=True, transform=tf, out_dtype=dtype, memory_format=mf,
                                sampler=D.DistributedSampler(ds, num_replicas=2, rank=1))
        ld.sampler.set_epoch(1)
        torch.manual_seed(3)
        out[str(dev)] = [(x.cpu(), y.cpu()) for x, y in ld]
    a, b = out["cpu"], out[str(cuda_device)]
    assert len(a) == len(b) == 5
    for (ax, ay), (bx, by) in zip(a, b):
        assert torch.equal(ax, bx) and torch.equal(ay, by)


def test_device_loader_equals_reference_pipeline(cuda_device):
    imgs, labels = _images(300, seed=7)
    ref = R.reference_loader(imgs, labels, 32, 2, 0, train=True, drop_last=True)
    ds = D.ImageDataset(imgs, labels, cuda_device)
    mine = D.DeviceDataLoader(ds, batch_size=32, drop_last=True, transform=D.TRAIN_TRANSFORM,
                              sampler=D.DistributedSampler(ds, num_replicas=2, rank=0))
    torch.manual_seed(21)
    want = list(ref)
    torch.manual_seed(21)
    got = [(x.cpu(), y.cpu()) for x, y in mine]
    assert len(got) == len(want)
    for (gx, gy), (wx, wy) in zip(got, want):
        assert torch.equal(gx, wx) and torch.equal(gy, wy)


def test_full_cifar_shape_epoch(cuda_device):
    """50,000 resident images, batch 256, one epoch: every batch matches the host backend
    on a sample of batches; labels are the gathered ones."""
    ds = D.ImageDataset.synthetic(50000, device=cuda_device, seed=1)
    host = D.ImageDataset(ds.images.cpu(), ds.labels.cpu(), "cpu")
    kw = dict(batch_size=256, drop_last=True, transform=D.TRAIN_TRANSFORM)
    ld = D.DeviceDataLoader(ds, sampler=D.DistributedSampler(ds, num_replicas=1, rank=0), **kw)
    lh = D.DeviceDataLoader(host, sampler=D.DistributedSampler(host, num_replicas=1, rank=0), **kw)
    torch.manual_seed(0)
    dev_batches = [(x.cpu(), y.cpu()) if i % 37 == 0 else None for i, (x, y) in enumerate(ld)]
    torch.manual_seed(0)
    n = 0
    for i, (x, y) in enumerate(lh):
        if dev_batches[i] is not None:
            assert torch.equal(dev_batches[i][0], x) and torch.equal(dev_batches[i][1], y)
            n += 1
    assert len(dev_batches) == 195 and n == 6


@pytest.mark.parametrize("H,W,pad,crop,fmt", [
    (64, 64, 0, 56, "nchw"),     # LDS path, non-CIFAR geometry
    (130, 130, 2, 128, "nchw"),  # 50.7 KB image: global-gather path
    (130, 130, 2, 128, "nhwc"),
    (9, 7, 1, 5, "nchw"),        # 75 outputs per sample (not a multiple of 4): global-gather path
    (9, 7, 1, 5, "nhwc"),
])
def test_kernel_paths_equal_host(cuda_device, H, W, pad, crop, fmt):
    g = np.random.default_rng(H * W)
    imgs = g.integers(0, 256, (37, H, W, 3), dtype=np.uint8)
    labels = g.integers(0, 10, 37)
    mf = torch.channels_last if fmt == "nhwc" else torch.contiguous_format
    tf = D.PadFlipCrop(pad, True, crop)
    out = {}
    for dev in ("cpu", cuda_device):
        ds = D.ImageDataset(imgs, labels, dev)
        ld = D.DeviceDataLoader(ds, batch_size=6, drop_last=False, transform=tf, memory_format=mf,
                                sampler=D.DistributedSampler(ds, num_replicas=1, rank=0))
        torch.manual_seed(4)
        out[str(dev)] = [(x.cpu(), y.cpu()) for x, y in ld]
    for (ax, ay), (bx, by) in zip(out["cpu"], out[str(cuda_device)]):
        assert torch.equal(ax, bx) and torch.equal(ay, by)
