"""Reference input pipeline of the CIFAR configuration, restated on torch's own
DataLoader + DistributedSampler with torchvision 0.15.2's transforms in numpy.

TEST INFRASTRUCTURE ONLY — the checker for distributed_training_amd/data.py;
never imported by the product package.

The reference (R:resnet/pytorch_ddp/ddp_train.py:25-48) runs

    Compose([Pad(4), RandomHorizontalFlip(), RandomCrop(32), ToTensor()])
    DataLoader(CIFAR10(...), batch_size, shuffle=False, drop_last=True,
               sampler=DistributedSampler(train_dataset))

torchvision (pinned 0.15.2 in R:resnet/pytorch_ddp/requirements.txt) is not
installed here; its published algorithm for these four transforms on a
uint8 RGB PIL image is restated below (torchvision/transforms/transforms.py
``Pad.forward`` -> F.pad(fill=0, 'constant'); ``RandomHorizontalFlip.forward``:
``if torch.rand(1) < self.p: return F.hflip(img)``; ``RandomCrop.get_params``:
``if w == tw and h == th: return 0, 0, h, w``; ``i = torch.randint(0, h - th + 1,
size=(1,)).item(); j = torch.randint(0, w - tw + 1, size=(1,)).item()``;
``ToTensor`` -> ``F.to_tensor``: HWC uint8 -> CHW, ``.to(float32).div(255)``).
The random draws are torch's real global-generator calls, and the DataLoader,
sampler and collate are torch's own — so this is the reference pipeline with
PIL's pixel copies done by numpy.
"""
from __future__ import annotations

import numpy as np
import torch


def pad_flip_crop_to_tensor(img_hwc: np.ndarray, pad: int, flip: bool, top: int, left: int, oh: int, ow: int):
    """F.pad -> F.hflip (if flip) -> F.crop -> F.to_tensor on one HWC uint8 image."""
    p = np.pad(img_hwc, ((pad, pad), (pad, pad), (0, 0)), mode="constant", constant_values=0)
    if flip:
        p = p[:, ::-1, :]
    c = p[top:top + oh, left:left + ow, :]
    return torch.from_numpy(np.ascontiguousarray(c.transpose(2, 0, 1))).to(torch.float32).div(255)


class TorchvisionCifarTransform:
    """Compose([Pad(pad), RandomHorizontalFlip(p), RandomCrop(crop), ToTensor()])."""

    def __init__(self, pad=4, flip=True, crop=32, p=0.5):
        self.pad, self.flip, self.crop, self.p = pad, flip, crop, p

    def __call__(self, img_hwc: np.ndarray):
        h, w = img_hwc.shape[0] + 2 * self.pad, img_hwc.shape[1] + 2 * self.pad
        f = False
        if self.flip:
            f = bool(torch.rand(1) < self.p)
        th = tw = self.crop if self.crop is not None else None
        if th is None:
            th, tw = h, w
        if h < th or w < tw:
            raise ValueError(f"Required crop size {(th, tw)} is larger than input image size {(h, w)}")
        if w == tw and h == th:
            i = j = 0
        else:
            i = torch.randint(0, h - th + 1, size=(1,)).item()
            j = torch.randint(0, w - tw + 1, size=(1,)).item()
        return pad_flip_crop_to_tensor(img_hwc, self.pad, f, i, j, th, tw)


class NumpyImageDataset(torch.utils.data.Dataset):
    """CIFAR10-like dataset: ``data`` uint8 [N, H, W, C], ``targets`` list of int."""

    def __init__(self, images: np.ndarray, labels: np.ndarray, transform):
        self.data = images
        self.targets = [int(x) for x in labels]
        self.transform = transform

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        return self.transform(self.data[index]), self.targets[index]


def reference_loader(images, labels, batch_size, num_replicas, rank, train=True, drop_last=True, seed=0):
    """build_dataloader (R:resnet/pytorch_ddp/ddp_train.py:25-48) with explicit
    num_replicas/rank (no process group needed)."""
    tf = TorchvisionCifarTransform(4, True, 32) if train else TorchvisionCifarTransform(0, False, None)
    ds = NumpyImageDataset(images, labels, tf)
    sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=num_replicas, rank=rank, seed=seed)
    return torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=False, drop_last=drop_last,
                                       sampler=sampler)
