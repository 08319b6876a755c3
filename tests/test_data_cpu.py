"""Input step on the host backend vs the reference pipeline.

The checker is oracle/input_pipeline.py: torch's own DataLoader +
DistributedSampler, torchvision 0.15.2's Pad/RandomHorizontalFlip/RandomCrop/
ToTensor restated in numpy, random draws from torch's global generator.
Everything here is bit-exact (integer indices, byte gathers, x/255 in fp32).
"""
import numpy as np
import pytest
import torch
import torch.utils.data as tud

from distributed_training_amd import _lib as L
from distributed_training_amd import data as D
from oracle import input_pipeline as R


def _images(n=103, seed=0, H=32, W=32):
    g = np.random.default_rng(seed)
    return g.integers(0, 256, (n, H, W, 3), dtype=np.uint8), g.integers(0, 10, n)


@pytest.mark.parametrize("n", [0, 1, 5, 7, 103, 50000])
@pytest.mark.parametrize("ws", [1, 2, 3, 8])
@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("drop_last", [True, False])
def test_sampler_matches_torch(n, ws, shuffle, drop_last):
    ds = list(range(n))
    for rank in range(ws) if n < 1000 else (0, ws - 1):
        for epoch in (0, 3):
            a = tud.DistributedSampler(ds, num_replicas=ws, rank=rank, shuffle=shuffle, seed=11, drop_last=drop_last)
            b = D.DistributedSampler(ds, num_replicas=ws, rank=rank, shuffle=shuffle, seed=11, drop_last=drop_last)
            a.set_epoch(epoch)
            b.set_epoch(epoch)
            assert len(a) == len(b)
            assert list(a) == list(b)


def test_sampler_errors():
    with pytest.raises(ValueError, match="Invalid rank"):
        D.DistributedSampler(list(range(4)), num_replicas=2, rank=2)


@pytest.mark.parametrize("n", [0, 1, 2, 17, 1000, 50000])
@pytest.mark.parametrize("seed", [0, 1, 12345, 2**32 + 5])
def test_randperm_matches_torch(n, seed):
    g = torch.Generator().manual_seed(seed)
    assert D.randperm(n, seed).tolist() == torch.randperm(n, generator=g).tolist()


def test_rng_draws_advance_torch_state():
    torch.manual_seed(77)
    want = [(torch.rand(1).item(), torch.randint(0, 9, (1,)).item()) for _ in range(700)]  # crosses a twist
    after = torch.rand(3)
    torch.manual_seed(77)
    st = torch.get_rng_state()
    raw = np.empty(1400, dtype=np.uint32)
    L.check(L.lib().gs_rng_draw_u32(st.data_ptr(), st.numel(), raw.size, raw.ctypes.data))
    torch.set_rng_state(st)
    got = [(float(np.float32(int(raw[2 * k]) & 0xFFFFFF) * np.float32(2.0 ** -24)), int(raw[2 * k + 1]) % 9)
           for k in range(700)]
    assert got == want
    assert torch.equal(torch.rand(3), after)
    bad = torch.zeros(100, dtype=torch.uint8)
    with pytest.raises(L.GsyncError, match="5056"):
        L.check(L.lib().gs_rng_draw_u32(bad.data_ptr(), bad.numel(), 1, raw.ctypes.data))


@pytest.mark.parametrize("ws,rank", [(1, 0), (2, 0), (2, 1), (3, 2)])
@pytest.mark.parametrize("batch", [1, 10, 32])
def test_train_loader_matches_reference_pipeline(ws, rank, batch):
    imgs, labels = _images(103)
    ref = R.reference_loader(imgs, labels, batch, ws, rank, train=True, drop_last=True)
    ds = D.ImageDataset(imgs, labels, "cpu")
    mine = D.DeviceDataLoader(ds, batch_size=batch, shuffle=False, drop_last=True,
                              sampler=D.DistributedSampler(ds, num_replicas=ws, rank=rank),
                              transform=D.TRAIN_TRANSFORM)
    assert len(mine) == len(ref)
    for epoch in range(2):
        ref.sampler.set_epoch(epoch)
        mine.sampler.set_epoch(epoch)
        torch.manual_seed(100 + epoch)
        want = [(x.clone(), y.clone()) for x, y in ref]
        st_ref = torch.get_rng_state()
        torch.manual_seed(100 + epoch)
        got = [(x.clone(), y.clone()) for x, y in mine]
        assert torch.equal(torch.get_rng_state(), st_ref)  # generator left exactly where the reference leaves it
        assert len(got) == len(want)
        for (gx, gy), (wx, wy) in zip(got, want):
            assert gx.dtype == torch.float32 and gx.shape == wx.shape
            assert torch.equal(gx, wx)
            assert torch.equal(gy, wy)


def test_test_loader_matches_reference_pipeline():
    imgs, labels = _images(53, seed=3)
    ref = R.reference_loader(imgs, labels, 8, 2, 1, train=False, drop_last=False)
    ds = D.ImageDataset(imgs, labels, "cpu")
    mine = D.DeviceDataLoader(ds, batch_size=8, drop_last=False,
                              sampler=D.DistributedSampler(ds, num_replicas=2, rank=1), transform=D.TEST_TRANSFORM)
    torch.manual_seed(5)
    want = list(ref)
    torch.manual_seed(5)
    got = list(mine)
    assert len(got) == len(want) == 4  # 27 samples -> 3 full + 1 partial
    for (gx, gy), (wx, wy) in zip(got, want):
        assert torch.equal(gx, wx) and torch.equal(gy, wy)


def test_layouts_and_bf16():
    imgs, labels = _images(40, seed=4)
    ds = D.ImageDataset(imgs, labels, "cpu")
    kw = dict(batch_size=16, drop_last=False, sampler=D.DistributedSampler(ds, num_replicas=1, rank=0),
              transform=D.TRAIN_TRANSFORM)
    torch.manual_seed(9)
    base = [x for x, _ in D.DeviceDataLoader(ds, **kw)]
    torch.manual_seed(9)
    cl = [x for x, _ in D.DeviceDataLoader(ds, memory_format=torch.channels_last, **kw)]
    torch.manual_seed(9)
    bf = [x for x, _ in D.DeviceDataLoader(ds, out_dtype=torch.bfloat16, **kw)]
    for a, b, c in zip(base, cl, bf):
        assert b.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(a, b)
        assert torch.equal(a.to(torch.bfloat16), c)  # same RNE rounding as torch's cast


def test_geometry_errors():
    imgs, labels = _images(4)
    ds = D.ImageDataset(imgs, labels, "cpu")
    big = D.DeviceDataLoader(ds, batch_size=2, sampler=D.DistributedSampler(ds, num_replicas=1, rank=0),
                             transform=D.PadFlipCrop(0, True, 40))
    with pytest.raises(L.GsyncError, match="larger than"):
        next(iter(big))
    params = torch.tensor([[7, 0, 0, 0]], dtype=torch.int32)
    out = torch.empty(1, 3, 32, 32)
    with pytest.raises(L.GsyncError, match="index out of range"):
        L.check(L.lib().gs_image_augment(L.GS_DEV_HOST, 0, ds.images.data_ptr(), ds.labels.data_ptr(), ds.n, 32, 32,
                                         3, 0, 32, 32, params.data_ptr(), 1, out.data_ptr(), L.GS_F32,
                                         L.GS_LAYOUT_NCHW, None, None))
    with pytest.raises(NotImplementedError):
        D.DeviceDataLoader(ds, batch_size=2, shuffle=True)


def test_cifar10_binary_reader(tmp_path):
    g = np.random.default_rng(0)
    rec = g.integers(0, 256, (7, 3073), dtype=np.uint8)
    rec[:, 0] %= 10
    rec.tofile(tmp_path / "test_batch.bin")
    ds = D.ImageDataset.cifar10_bin(str(tmp_path), train=False)
    assert len(ds) == 7 and ds.labels.tolist() == rec[:, 0].tolist()
    # record = label | R plane | G plane | B plane (32x32 row-major) -> HWC
    assert np.array_equal(ds.images[2].numpy(), rec[2, 1:].reshape(3, 32, 32).transpose(1, 2, 0))
    with pytest.raises(FileNotFoundError):
        D.ImageDataset.cifar10_bin(str(tmp_path), train=True)
