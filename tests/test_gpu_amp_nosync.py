"""The Colossal ``torch_ddp_fp16`` step (R:resnet/colossal/run.sh:1,
R:resnet/colossal/colossal_train.py:100-102,129-130: TorchDDPPlugin + fp16
mixed precision + HybridAdam) runs without a host synchronisation.

GradScaler.scale -> backward (libgsync DDP, inf check fused into the bucket
unpack) -> scaler.step (fused Adam: 1/scale folded into the update, the step
skipped ON THE DEVICE when found_inf, the device step counter advanced only
on a clean step) -> scaler.update (on the device) -> zero_grad: under
``torch.cuda.set_sync_debug_mode("error")`` any host read raises.  The same
for FusedSGD (device first-step flag).  An injected overflow is then skipped
exactly as torch skips it: the weights do not move and Adam's step count does
not advance.
"""
import pytest
import torch
import torch.distributed as dist

from tests._dist_util import free_port, init_pg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg(cuda_device):
    owned = False
    if not dist.is_initialized():
        init_pg("nccl", 0, 1, free_port())
        owned = True
    yield
    if owned:
        from distributed_training_amd.comm import destroy_communicators

        destroy_communicators()
        dist.destroy_process_group()


def _booster_step(model, optimizer, criterion, booster, x, y):
    outputs = model(x)                      # R:colossal_train.py:97
    loss = criterion(outputs, y)            # :98
    booster.backward(loss, optimizer)       # :100
    optimizer.step()                        # :101
    optimizer.zero_grad()                   # :102
    return loss


@pytest.mark.parametrize("opt_kind", ["hybrid_adam", "sgd"])
def test_torch_ddp_fp16_step_has_no_host_sync(cuda_device, pg, opt_kind):
    from distributed_training_amd import FusedSGD
    from distributed_training_amd.compat import colossalai as C
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device)
    if opt_kind == "hybrid_adam":
        optimizer = C.HybridAdam(model.parameters(), lr=1e-3)
    else:
        optimizer = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    booster = C.Booster(plugin=C.TorchDDPPlugin(), mixed_precision="fp16")
    model, optimizer, criterion, _, _ = booster.boost(model, optimizer, criterion=torch.nn.CrossEntropyLoss())
    g = torch.Generator(device=cuda_device).manual_seed(5)
    xs = [torch.rand(8, 3, 32, 32, device=cuda_device, generator=g) for _ in range(6)]
    ys = [torch.randint(0, 10, (8,), device=cuda_device, generator=g) for _ in range(6)]
    for k in range(3):  # bucket rebuild, optimizer state and plans are created here
        _booster_step(model, optimizer, criterion, booster, xs[k], ys[k])
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for k in range(3, 6):
            loss = _booster_step(model, optimizer, criterion, booster, xs[k], ys[k])
    finally:
        torch.cuda.set_sync_debug_mode(0)
    assert torch.isfinite(loss).item()
    assert loss.dtype == torch.float32  # the criterion runs under autocast (Colossal wraps it)

    # an overflow is skipped on the device: weights unchanged, Adam's step not advanced
    params = [p for p in model.parameters()]
    before = [p.detach().clone() for p in params]
    inner = optimizer.optim
    st = inner.state[params[0]]
    step_before = float(st["step"]) if "step" in st else None
    outputs = model(xs[0])
    loss = criterion(outputs, ys[0]) * float("inf")
    booster.backward(loss, optimizer)
    optimizer.step()
    optimizer.zero_grad()
    torch.cuda.synchronize()
    for a, b in zip(before, params):
        assert torch.equal(a, b.detach())
    if step_before is not None:
        assert float(st["step"]) == step_before
