"""AMP non-finite check fused into the DDP bucket unpack (SURVEY.md §8f-2:
"fuse it into pack/unpack") == the separate check pass, bit for bit:
GradScaler.fuse_check_into(ddp) + FusedAdam vs the same without fusion, an
inf injected into ONE rank's local grad (so only the all-reduced grads carry
it to the other rank) on one iteration; CPU/gloo ws=2 and (-m gpu) RCCL ws=1."""
import pytest
import torch
import torch.nn as nn

from tests.test_ddp_cpu import _micro, _run


def _train(dev, rank, fused, poison_rank, iters=4):
    import distributed_training_amd as D
    from distributed_training_amd.amp import GradScaler

    torch.manual_seed(0)
    model = _micro().to(dev)
    first = next(model.parameters())
    state = {"it": 0}

    def poison(p):  # runs before DDP's hook: the local grad, ahead of the pack
        if state["it"] == 2 and rank == poison_rank:
            p.grad.view(-1)[1] = float("inf")

    first.register_post_accumulate_grad_hook(poison)
    ddp = D.DistributedDataParallel(model)
    opt = D.FusedAdam(ddp.parameters(), lr=1e-3)
    scaler = GradScaler(dev.type, init_scale=2.0 ** 8, growth_interval=2)
    if fused:
        scaler.fuse_check_into(ddp)
    g = torch.Generator(device=dev).manual_seed(10 + rank)
    scales = []
    for it in range(iters):
        state["it"] = it
        x = torch.rand(4, 3, 32, 32, device=dev, generator=g)
        y = torch.randint(0, 10, (4,), device=dev, generator=g)
        scaler.scale(nn.functional.cross_entropy(ddp(x), y)).backward()
        scaler.step(opt)
        scaler.update()
        opt.zero_grad()
        scales.append(scaler.get_scale())
    return [p.detach().clone() for p in model.parameters()], scales, scaler.fused_checks


def _compare(dev, rank, poison_rank):
    w_ref, s_ref, n_ref = _train(dev, rank, False, poison_rank)
    w_fus, s_fus, n_fus = _train(dev, rank, True, poison_rank)
    assert n_ref == 0 and n_fus == 4  # every step took the DDP flag, no extra pass
    assert s_ref == s_fus and s_ref[2] == s_ref[1] / 2  # iteration 2 overflowed on every rank
    for a, b in zip(w_ref, w_fus):
        assert torch.equal(a, b)


def _cpu_case(rank, ws):
    _compare(torch.device("cpu"), rank, poison_rank=1)


def test_fused_inf_check_cpu_ws2():
    _run(_cpu_case, 2)


@pytest.mark.gpu
def test_fused_inf_check_gpu_ws1(cuda_device):
    """On the GPU two training runs are not bit-reproducible (MIOpen's backward),
    so the property is checked on ONE run: after every backward the flag the
    bucket unpack produced equals a separate check pass over the same grads,
    and it is set exactly on the poisoned iteration; the scaler then backs off."""
    import torch.distributed as dist

    from tests._dist_util import free_port, init_pg

    created = not dist.is_initialized()
    if created:
        init_pg("nccl", 0, 1, free_port())
    try:
        _gpu_body(cuda_device)
    finally:
        if created:
            from distributed_training_amd.comm import destroy_communicators

            destroy_communicators()
            dist.destroy_process_group()


def _gpu_body(cuda_device):
    import distributed_training_amd as D
    from distributed_training_amd.amp import GradScaler
    from distributed_training_amd.multi_tensor import TensorListPlan

    dev = cuda_device
    torch.manual_seed(0)
    model = _micro().to(dev)
    state = {"it": 0}

    def poison(p):
        if state["it"] == 2:
            p.grad.view(-1)[1] = float("inf")

    next(model.parameters()).register_post_accumulate_grad_hook(poison)
    ddp = D.DistributedDataParallel(model)
    opt = D.FusedAdam(ddp.parameters(), lr=1e-3)
    scaler = GradScaler("cuda", init_scale=2.0 ** 8, growth_interval=2)
    scaler.fuse_check_into(ddp)
    params = list(model.parameters())
    plan = TensorListPlan([p.numel() for p in params], dev)
    ref = torch.zeros(1, device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    for it in range(4):
        state["it"] = it
        x = torch.rand(4, 3, 32, 32, device=dev, generator=g)
        y = torch.randint(0, 10, (4,), device=dev, generator=g)
        scaler.scale(nn.functional.cross_entropy(ddp(x), y)).backward()
        ref.zero_()
        plan.set_ptrs(0, [p.grad for p in params])
        plan.unscale_check(0, torch.float32, None, ref)
        assert ddp._found_inf_valid
        assert scaler._ddp_found.item() == ref.item() == (1.0 if it == 2 else 0.0), it
        before = scaler.get_scale()
        scaler.step(opt)
        scaler.update()
        opt.zero_grad()
        if it == 2:
            assert scaler.get_scale() == before / 2
    assert scaler.fused_checks == 4
