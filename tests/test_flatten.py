"""flatten / unflatten drop-ins vs torch._utils, bit for bit,
on the host backend and (-m gpu) on the HIP kernels."""
import pytest
import torch
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from distributed_training_amd.flatten import copy_flat_to, flatten_dense_tensors, unflatten_dense_tensors

SHAPES = [(3,), (64, 3, 3, 3), (1,), (7, 5), (0,), (2, 3, 4, 5), (1000,)]


def _tensors(device, dtype, channels_last=False):
    g = torch.Generator().manual_seed(0)
    ts = [torch.randn(s, generator=g).to(dtype).to(device) for s in SHAPES]
    if channels_last:
        ts = [t.to(memory_format=torch.channels_last) if t.dim() == 4 else t for t in ts]
    return ts


def _check(device, dtype, channels_last):
    ts = _tensors(device, dtype, channels_last)
    ref = _flatten_dense_tensors(ts)
    flat = flatten_dense_tensors(ts)
    assert flat.dtype == ref.dtype and torch.equal(flat, ref)
    for a, b in zip(unflatten_dense_tensors(flat, ts), _unflatten_dense_tensors(ref, ts)):
        assert a.shape == b.shape and torch.equal(a, b)
        assert a.numel() == 0 or a.data_ptr() >= flat.data_ptr()  # views, no copy
    dst = [torch.zeros_like(t) for t in ts]
    copy_flat_to(flat * 2, dst)
    for t, d in zip(ts, dst):
        assert torch.equal(d, t * 2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("channels_last", [False, True])
def test_flatten_cpu(dtype, channels_last):
    _check(torch.device("cpu"), dtype, channels_last)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("channels_last", [False, True])
def test_flatten_gpu(cuda_device, dtype, channels_last):
    _check(cuda_device, dtype, channels_last)


def test_flatten_errors():
    with pytest.raises(TypeError):
        flatten_dense_tensors([torch.zeros(2), torch.zeros(2, dtype=torch.float64)])
    with pytest.raises(ValueError):
        flatten_dense_tensors([])
