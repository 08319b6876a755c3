"""libgsync GradScaler + fused optimizers vs torch.amp.GradScaler + torch.optim.

Both sides step on the SAME gradients (model 1's backward, copied into model
2's ``.grad``), so MIOpen's run-to-run backward differences never enter: what
is compared is the scaler (unscale, overflow detection, skip, scale update)
and the optimizer arithmetic only.  Overflows are injected on the first step
(SGD momentum buffers must not be created by a skipped step; Adam's step count
must not advance) and mid-run.

Tolerances: SGD rtol 1e-6 / atol 1e-7 (fp32, fma placement may differ from
ATen's in the last bit); Adam atol lr*1e-3 (its sign can flip
where |g| ~ eps).
"""
import copy

import pytest
import torch
import torch.nn as nn

from distributed_training_amd.amp import GradScaler
from distributed_training_amd.optim import FusedAdam, FusedSGD


def _micro():
    from distributed_training_amd.resnet import ResNet, BasicBlock

    return ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, width=8)


def _run(dev, kind, poison_at, iters=5, drop=None):
    torch.manual_seed(0)
    m1, m2 = _micro().to(dev), _micro().to(dev)
    m2.load_state_dict(m1.state_dict())
    if kind == "sgd":
        o1 = FusedSGD(m1.parameters(), lr=1e-2, momentum=0.9, weight_decay=1e-4)
        o2 = torch.optim.SGD(m2.parameters(), lr=1e-2, momentum=0.9, weight_decay=1e-4)
        tol = dict(rtol=1e-6, atol=1e-7)
    else:
        o1 = FusedAdam(m1.parameters(), lr=1e-3)
        o2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
        tol = dict(rtol=0, atol=1e-3 * 1e-3)
    s1 = GradScaler(dev.type, init_scale=2.0 ** 10, growth_interval=2)
    s2 = torch.amp.GradScaler(dev.type, init_scale=2.0 ** 10, growth_interval=2)
    g = torch.Generator(device=dev).manual_seed(7)
    for it in range(iters):
        x = torch.rand(4, 3, 32, 32, device=dev, generator=g)
        y = torch.randint(0, 10, (4,), device=dev, generator=g)
        loss = nn.functional.cross_entropy(m1(x), y)
        s1.scale(loss).backward()
        s2.scale(loss.detach())  # lazy-inits torch's scale on the device
        if it in poison_at:
            next(m1.parameters()).grad.view(-1)[3] = float("inf")
        for p1, p2 in zip(m1.parameters(), m2.parameters()):
            p2.grad = p1.grad.detach().clone()
        for k in (drop or {}).get(it, ()):  # a parameter without a grad this step
            list(m1.parameters())[k].grad = None
            list(m2.parameters())[k].grad = None
        s1.step(o1)
        s1.update()
        s2.step(o2)
        s2.update()
        o1.zero_grad()
        o2.zero_grad()
        assert s1.get_scale() == s2.get_scale(), (it, s1.get_scale(), s2.get_scale())
        for k, (p1, p2) in enumerate(zip(m1.parameters(), m2.parameters())):
            torch.testing.assert_close(p1, p2, **tol, msg=lambda m: f"iter {it} param {k}: {m}")
    # optimizer state layout and content follow torch's
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        st1, st2 = o1.state[p1], o2.state[p2]
        assert set(st1) == set(st2)
        if kind == "sgd":
            torch.testing.assert_close(st1["momentum_buffer"], st2["momentum_buffer"], rtol=1e-6, atol=1e-7)
        else:
            assert float(st1["step"]) == float(st2["step"])
    if kind == "adam":
        # state_dict: one fp32 step tensor per parameter, as torch's (no shared device counter)
        sd1, sd2 = o1.state_dict(), o2.state_dict()
        steps = [st["step"] for st in sd1["state"].values()]
        assert len({id(t) for t in steps}) == len(steps)
        for k in sd2["state"]:
            t1, t2 = sd1["state"][k]["step"], sd2["state"][k]["step"]
            assert t1.dtype == torch.float32 and t1.device.type == "cpu" and float(t1) == float(t2)


# parameters that get no grad on some steps keep their own
# Adam step count (torch advances state["step"] per parameter, only with a grad)
DROPS = {1: (0, 5), 2: (5,), 3: (1,)}


@pytest.mark.parametrize("poison_at", [(), (2,)])
def test_scaler_cpu_intermittent_grads(poison_at):
    _run(torch.device("cpu"), "adam", poison_at, iters=6, drop=DROPS)


@pytest.mark.gpu
@pytest.mark.parametrize("poison_at", [(), (2,)])
def test_scaler_gpu_intermittent_grads(cuda_device, poison_at):
    _run(cuda_device, "adam", poison_at, iters=6, drop=DROPS)


def test_adam_device_counters_from_loaded_state():
    """A torch Adam state_dict whose parameters are at different steps, loaded
    into FusedAdam on the AMP (device-counter) path: each parameter continues
    from its own step, bit-for-bit with torch.optim.Adam continuing the same."""
    torch.manual_seed(0)
    ps_t = [torch.nn.Parameter(torch.randn(n)) for n in (10, 33, 7)]
    ps_f = [torch.nn.Parameter(p.detach().clone()) for p in ps_t]
    ot = torch.optim.Adam(ps_t, lr=1e-2)
    g = torch.Generator().manual_seed(1)
    for it in range(4):  # param 1 skips two steps: steps 4 / 2 / 4
        for k, p in enumerate(ps_t):
            p.grad = None if (k == 1 and it in (1, 2)) else torch.randn(p.shape, generator=g)
        ot.step()
    of = FusedAdam(ps_f, lr=1e-2)
    of.load_state_dict(copy.deepcopy(ot.state_dict()))  # torch's state_dict shares its step tensors
    of.found_inf = torch.zeros(1)  # the AMP path: device counters
    for p, q in zip(ps_f, ps_t):
        p.data.copy_(q.data)
    for it in range(3):
        for p, q in zip(ps_t, ps_f):
            p.grad = torch.randn(p.shape, generator=g)
            q.grad = p.grad.clone()
        ot.step()
        of.step()
        for k, (p, q) in enumerate(zip(ps_t, ps_f)):
            torch.testing.assert_close(q, p, rtol=0, atol=1e-2 * 1e-3, msg=lambda m: f"it {it} param {k}: {m}")
    sd = of.state_dict()
    assert [float(sd["state"][k]["step"]) for k in range(3)] == [7.0, 5.0, 7.0]


@pytest.mark.parametrize("kind", ["sgd", "adam"])
@pytest.mark.parametrize("poison_at", [(0,), (2,), (0, 1, 3)])
def test_scaler_cpu_host_backend(kind, poison_at):
    _run(torch.device("cpu"), kind, poison_at)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sgd", "adam"])
@pytest.mark.parametrize("poison_at", [(0,), (2,), (0, 1, 3)])
def test_scaler_gpu(cuda_device, kind, poison_at):
    _run(cuda_device, kind, poison_at)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_scale_matches_torch_for_low_precision_loss(dtype):
    """scale() multiplies by the fp32 scale tensor without casting it
    (T:amp/grad_scaler.py scale()): an fp16 loss at the default init_scale
    2**16 (> fp16 max 65504) stays finite and equals torch's bit for bit, in
    dtype and shape."""
    loss = torch.tensor(1.2345, dtype=dtype)
    for shape in ((), (3,)):
        x = loss.expand(shape).clone() if shape else loss
        a = GradScaler("cpu").scale(x)
        b = torch.amp.GradScaler("cpu").scale(x)
        assert a.dtype == b.dtype and a.shape == b.shape
        assert torch.equal(a, b)
        if not shape:  # a scalar loss is promoted to fp32 (a 1-D fp16 tensor is not, in torch too)
            assert a.dtype == torch.float32 and bool(torch.isfinite(a))
