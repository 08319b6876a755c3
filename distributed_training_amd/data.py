"""Input step of the CIFAR configuration on libgsync.

The reference builds its batches with torchvision + a torch DataLoader
(R:resnet/pytorch_ddp/ddp_train.py:25-48):

    transform_train = Compose([Pad(4), RandomHorizontalFlip(), RandomCrop(32), ToTensor()])
    DataLoader(CIFAR10(...), batch_size, shuffle=False, drop_last=True,
               sampler=DistributedSampler(train_dataset))
    ... images.to(device)                                           (:62)

Here the uint8 image set is resident on the device (HBM: CIFAR-10's 50,000
train images are 153.6 MB) and every batch is ONE libgsync kernel that
gathers the sampled images, pads, flips, crops and converts to float
(x / 255) straight into the training tensor, labels gathered alongside —
no per-sample PIL work, no collate, no H2D of pixels.  Only the per-sample
(index, flip, top, left) table (16 B/sample) crosses PCIe.

Parity with the reference pipeline is exact, not statistical:

* :class:`DistributedSampler` yields torch's indices (randperm(n) under
  ``manual_seed(seed + epoch)``, head-repeat padding, ``[rank::ws]`` stride;
  T:utils/data/distributed.py:107-138), computed by libgsync's C++ restatement
  of torch's MT19937 / randperm.
* the per-sample random flip / crop offsets consume torch's *global* CPU
  generator in torchvision 0.15.2's order (flip draw, then the crop's two
  draws, per sample in sampler order, after the DataLoader iterator's one
  int64 base-seed draw), so a script that seeds torch gets the same
  augmentations as with the reference's DataLoader, and the generator is left
  in the same state.

There is no dataset download (no network): :meth:`ImageDataset.cifar10_bin`
reads the CIFAR-10 *binary* distribution from disk when present;
:meth:`ImageDataset.synthetic` makes a seeded stand-in of the same shape.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Iterator, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L


def _sampler_indices(n, num_replicas, rank, shuffle, seed, epoch, drop_last) -> np.ndarray:
    lib = L.lib()
    count = ctypes.c_int64()
    L.check(lib.gs_distributed_sampler_indices(n, num_replicas, rank, int(bool(shuffle)), int(seed), int(epoch),
                                               int(bool(drop_last)), None, 0, ctypes.byref(count)),
            "gs_distributed_sampler_indices")
    out = np.empty(max(1, count.value), dtype=np.int64)
    L.check(lib.gs_distributed_sampler_indices(n, num_replicas, rank, int(bool(shuffle)), int(seed), int(epoch),
                                               int(bool(drop_last)), out.ctypes.data, out.size,
                                               ctypes.byref(count)),
            "gs_distributed_sampler_indices")
    return out[: count.value]


def randperm(n: int, seed: int) -> np.ndarray:
    """torch.randperm(n, generator=torch.Generator().manual_seed(seed)), in C++."""
    out = np.empty(max(1, n), dtype=np.int64)
    L.check(L.lib().gs_randperm(int(seed), int(n), out.ctypes.data), "gs_randperm")
    return out[:n]


class DistributedSampler(torch.utils.data.Sampler):
    """Drop-in for torch.utils.data.DistributedSampler (same arguments, errors,
    ``set_epoch``, ``__len__``), indices from libgsync."""

    def __init__(self, dataset, num_replicas: int | None = None, rank: int | None = None, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if num_replicas is None:
            if not dist.is_available():
                raise RuntimeError("Requires distributed package to be available")
            num_replicas = dist.get_world_size()
        if rank is None:
            if not dist.is_available():
                raise RuntimeError("Requires distributed package to be available")
            rank = dist.get_rank()
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if self.drop_last and n % self.num_replicas != 0:
            self.num_samples = math.ceil((n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def indices(self) -> np.ndarray:
        return _sampler_indices(len(self.dataset), self.num_replicas, self.rank, self.shuffle, self.seed,
                                self.epoch, self.drop_last)

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch


class ImageDataset:
    """A uint8 image set ``[N, H, W, C]`` (HWC, as CIFAR10.data) + int64 labels,
    resident on one device (HBM for a HIP device)."""

    def __init__(self, images, labels, device="cpu"):
        images = torch.as_tensor(images)
        labels = torch.as_tensor(labels)
        if images.dtype != torch.uint8 or images.dim() != 4:
            raise ValueError("images must be uint8 [N, H, W, C]")
        if labels.dim() != 1 or labels.numel() != images.shape[0]:
            raise ValueError("labels must be [N]")
        self.device = torch.device(device)
        self.images = images.contiguous().to(self.device)
        self.labels = labels.to(torch.int64).contiguous().to(self.device)
        self.n, self.H, self.W, self.C = (int(x) for x in images.shape)

    def __len__(self) -> int:
        return self.n

    @classmethod
    def synthetic(cls, n=50000, H=32, W=32, C=3, classes=10, seed=0, device="cpu"):
        g = torch.Generator().manual_seed(seed)
        imgs = torch.randint(0, 256, (n, H, W, C), dtype=torch.uint8, generator=g)
        labels = torch.randint(0, classes, (n,), generator=g)
        return cls(imgs, labels, device)

    @classmethod
    def cifar10_bin(cls, root, train=True, device="cpu"):
        """CIFAR-10 binary version (cifar-10-batches-bin/{data_batch_1..5,test_batch}.bin:
        records of 1 label byte + 3,072 bytes R|G|B planes of 32x32, row-major)."""
        d = os.path.join(root, "cifar-10-batches-bin") if not os.path.exists(os.path.join(root, "test_batch.bin")) else root
        names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
        recs = []
        for nm in names:
            path = os.path.join(d, nm)
            if not os.path.exists(path):
                raise FileNotFoundError(f"{path} (CIFAR-10 binary version; there is no download here)")
            raw = np.fromfile(path, dtype=np.uint8)
            if raw.size % 3073:
                raise ValueError(f"{path}: size is not a multiple of 3073-byte records")
            recs.append(raw.reshape(-1, 3073))
        rec = np.concatenate(recs)
        labels = rec[:, 0].astype(np.int64)
        imgs = rec[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy()
        return cls(imgs, labels, device)


class PadFlipCrop:
    """Compose([Pad(pad), RandomHorizontalFlip(), RandomCrop(crop), ToTensor()])
    (R:resnet/pytorch_ddp/ddp_train.py:27-31); pad=0, flip=False, crop=None is
    the test transform ToTensor() (:32)."""

    def __init__(self, pad=4, flip=True, crop=32):
        self.pad, self.flip, self.crop = int(pad), bool(flip), crop

    def out_hw(self, H, W):
        if self.crop is None:
            return H + 2 * self.pad, W + 2 * self.pad
        c = self.crop
        return (c, c) if isinstance(c, int) else (int(c[0]), int(c[1]))


TRAIN_TRANSFORM = PadFlipCrop(4, True, 32)
TEST_TRANSFORM = PadFlipCrop(0, False, None)


class DeviceDataLoader:
    """``DataLoader(dataset, batch_size, shuffle=False, sampler=..., drop_last=...)``
    over an :class:`ImageDataset`, yielding ``(images, labels)`` on the
    dataset's device: images float32 (or ``out_dtype``) ``[B, C, h, w]`` in
    ``memory_format``, labels int64 ``[B]``."""

    def __init__(self, dataset: ImageDataset, batch_size: int = 1, shuffle: bool = False, sampler=None,
                 drop_last: bool = False, transform: PadFlipCrop = TEST_TRANSFORM,
                 out_dtype: torch.dtype = torch.float32, memory_format=torch.contiguous_format,
                 generator: torch.Generator | None = None):
        if shuffle and sampler is not None:
            raise ValueError("sampler option is mutually exclusive with shuffle")
        if shuffle:
            raise NotImplementedError("shuffle=True (RandomSampler) is not on the reference path; "
                                      "pass sampler=DistributedSampler(...)")
        if out_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("out_dtype must be float32 or bfloat16")
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.sampler = sampler
        self.drop_last = drop_last
        self.transform = transform
        self.out_dtype = out_dtype
        self.memory_format = memory_format
        self.generator = generator
        self.device = dataset.device
        self._kind = L.GS_DEV_HIP if self.device.type == "cuda" else L.GS_DEV_HOST
        if self._kind == L.GS_DEV_HIP and not L.available():
            raise L.GsyncUnavailable(L._load_error)
        self.oh, self.ow = transform.out_hw(dataset.H, dataset.W)

    def _indices(self) -> list:
        if self.sampler is None:
            return list(range(len(self.dataset)))
        if hasattr(self.sampler, "indices"):
            return self.sampler.indices().tolist()
        return list(iter(self.sampler))

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def _rng_get(self):
        if self.generator is not None:
            return self.generator.get_state()
        return torch.get_rng_state()

    def _rng_set(self, st):
        if self.generator is not None:
            self.generator.set_state(st)
        else:
            torch.set_rng_state(st)

    def _draw_params(self, idx: np.ndarray) -> torch.Tensor:
        B = idx.size
        t = self.transform
        # a fresh pinned block per batch: torch's host caching allocator keeps it
        # from reuse until the non_blocking H2D copy that reads it has run
        params = torch.empty((B, 4), dtype=torch.int32, pin_memory=self._kind == L.GS_DEV_HIP)
        st = self._rng_get()
        nbytes = st.numel()
        L.check(L.lib().gs_crop_flip_params(idx.ctypes.data, B, self.dataset.H, self.dataset.W, t.pad, self.oh,
                                            self.ow, int(t.flip), st.data_ptr(), nbytes, params.data_ptr()),
                "gs_crop_flip_params")
        self._rng_set(st)
        return params

    def __iter__(self):
        order = np.asarray(self._indices(), dtype=np.int64)
        if order.size and (order.min() < 0 or order.max() >= len(self.dataset)):
            raise IndexError("sampler produced an index outside the dataset")
        # _BaseDataLoaderIter.__init__: one int64 draw for the workers' base seed
        torch.empty((), dtype=torch.int64).random_(generator=self.generator)
        bs = self.batch_size
        nb = len(self)
        ds = self.dataset
        for k in range(nb):
            idx = np.ascontiguousarray(order[k * bs:(k + 1) * bs])
            B = idx.size
            params = self._draw_params(idx)
            if self._kind == L.GS_DEV_HIP:
                dparams = params.to(self.device, non_blocking=True)
                stream = L.stream_ptr(self.device)
            else:
                dparams, stream = params, None
            out = torch.empty((B, ds.C, self.oh, self.ow), dtype=self.out_dtype, device=self.device,
                              memory_format=self.memory_format)
            layout = L.GS_LAYOUT_NHWC if (self.memory_format == torch.channels_last and B > 0) else L.GS_LAYOUT_NCHW
            labels = torch.empty(B, dtype=torch.int64, device=self.device)
            L.check(L.lib().gs_image_augment(self._kind, self.device.index or 0, ds.images.data_ptr(),
                                              ds.labels.data_ptr(), ds.n, ds.H, ds.W, ds.C, self.transform.pad,
                                              self.oh, self.ow, dparams.data_ptr(), B, out.data_ptr(),
                                              L.gs_dtype(self.out_dtype), layout, labels.data_ptr(), stream),
                    "gs_image_augment")
            yield out, labels


def build_dataloader(batch_size: int, dataset_train: ImageDataset, dataset_test: ImageDataset | None = None,
                     **kw):
    """build_dataloader of R:resnet/pytorch_ddp/ddp_train.py:25-48 on device-resident data."""
    train = DeviceDataLoader(dataset_train, batch_size=batch_size, shuffle=False, drop_last=True,
                             sampler=DistributedSampler(dataset_train), transform=TRAIN_TRANSFORM, **kw)
    test = None
    if dataset_test is not None:
        test = DeviceDataLoader(dataset_test, batch_size=batch_size, shuffle=False, drop_last=False,
                                sampler=DistributedSampler(dataset_test), transform=TEST_TRANSFORM, **kw)
    return train, test
