"""ZeRO-1/2 (libgsync ZeroDataParallel) on CPU/gloo, world_size 2 and 3:
ZeRO == DDP + the same fused optimizer (SURVEY.md §8c pins the DeepSpeed /
Colossal variants to this identity; reduction order is the same here, so it
holds bit for bit), including gradient clipping and a bf16 model."""
import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

from tests.test_ddp_cpu import _micro, _run


def _zero_vs_ddp(rank, ws, stage, kind, clip, dtype):
    import distributed_training_amd as D
    from distributed_training_amd.zero import ZeroDataParallel

    torch.manual_seed(0)
    m1, m2 = _micro(), _micro()
    m2.load_state_dict(m1.state_dict())
    if dtype == "bf16":
        m1 = m1.to(torch.bfloat16)
    z = ZeroDataParallel(m1, stage=stage, optimizer=kind, lr=1e-2 if kind != "sgd" else 0.1, momentum=0.9,
                         weight_decay=1e-4, gradient_clipping=clip, reduce_bucket_size=5000)
    assert len(z.buckets) > 1  # several buckets at this cap
    d = D.DistributedDataParallel(m2)
    if kind == "sgd":
        opt = D.FusedSGD(d.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, max_grad_norm=clip or None)
    else:
        opt = D.FusedAdam(d.parameters(), lr=1e-2, weight_decay=1e-4, adamw=kind == "adamw",
                          max_grad_norm=clip or None)
    g = torch.Generator().manual_seed(5 + rank)
    for it in range(3):
        x = torch.rand(4, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (4,), generator=g)
        z.prepare_backward()
        nn.functional.cross_entropy(m1(x.to(m1.conv1.weight.dtype)).float(), y).backward()
        z.step()
        nn.functional.cross_entropy(d(x), y).backward()
        opt.step()
        opt.zero_grad()
        for (n1, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
            if dtype == "bf16":
                continue
            if clip:
                # Σg² is summed per shard then across ranks (vs whole-model in DDP):
                # the clip coefficient may differ in the last bit
                # (Adam tolerance of SURVEY §8c: atol = lr * 1e-3)
                torch.testing.assert_close(p1.detach(), p2.detach(), rtol=0, atol=1e-2 * 1e-3)
            else:
                assert torch.equal(p1.detach(), p2.detach()), f"stage {stage} {kind} it {it} {n1}"
    # every rank holds the full, identical parameters after the all-gather
    w = torch.cat([p.detach().float().reshape(-1) for p in m1.parameters()])
    allw = [torch.zeros_like(w) for _ in range(ws)]
    dist.all_gather(allw, w)
    for other in allw[1:]:
        assert torch.equal(allw[0], other)
    z.close()


@pytest.mark.parametrize("stage", [1, 2])
@pytest.mark.parametrize("kind", ["adamw", "sgd"])
def test_zero_equals_ddp_fp32(stage, kind):
    _run(_zero_vs_ddp, 2, stage, kind, 0.0, "fp32")


def test_zero_with_clipping_ws3():
    _run(_zero_vs_ddp, 3, 2, "adamw", 0.5, "fp32")


def test_zero_bf16_model_replicas_agree():
    _run(_zero_vs_ddp, 2, 2, "adamw", 1.0, "bf16")


def _zero_overflow(rank, ws, device="cpu", dtype=torch.float32):
    """DeepSpeed-style dynamic loss scaling through ZeRO-2 (R:resnet/deepspeed/
    deepspeed_train.py:200-208, loss_scale 0 = dynamic, hysteresis 2): an
    overflow on ONE rank skips the step on every rank (the reduce-scattered
    shards carry it; the found-inf flag is all-reduced), leaves params, fp32
    masters and the step count untouched; the first overflow only spends the
    hysteresis, the second in a row halves the scale; clean steps update."""
    from distributed_training_amd.zero import DynamicLossScaler, ZeroDataParallel

    torch.manual_seed(0)
    m = _micro().to(device).to(dtype)
    scaler = DynamicLossScaler(init_scale=2.0 ** 8, scale_window=1000, hysteresis=2)
    z = ZeroDataParallel(m, stage=2, optimizer="adamw", lr=1e-3, loss_scaler=scaler)
    g = torch.Generator(device=device).manual_seed(7 + rank)
    want = [  # (poison on, step taken, scale after, step count after)
        ("none", True, 256.0, 1), ("rank0", False, 256.0, 1), ("all", False, 128.0, 1), ("none", True, 128.0, 2)]
    for it, (poison, taken, scale_after, steps_after) in enumerate(want):
        x = torch.rand(4, 3, 32, 32, device=device, generator=g).to(dtype)
        y = torch.randint(0, 10, (4,), device=device, generator=g)
        before = [p.detach().clone() for p in m.parameters()]
        master_before = torch.cat([t.detach().reshape(-1) for t in z.master]).clone()
        z.prepare_backward()
        loss = nn.functional.cross_entropy(m(x).float(), y)
        if poison == "all" or (poison == "rank0" and rank == 0):
            loss = loss * float("inf")
        (loss * scaler.scale).backward()
        ok = z.step()
        z.zero_grad()
        master_after = torch.cat([t.detach().reshape(-1) for t in z.master])
        changed = any(not torch.equal(a, p.detach()) for a, p in zip(before, m.parameters()))
        assert ok == taken and changed == taken, (it, ok, changed)
        assert torch.equal(master_before, master_after) != taken, it
        assert scaler.scale == scale_after and z.step_count == steps_after, (it, scaler.scale, z.step_count)
    w = torch.cat([p.detach().float().reshape(-1) for p in m.parameters()])
    if ws > 1:
        allw = [torch.zeros_like(w) for _ in range(ws)]
        dist.all_gather(allw, w)
        assert all(torch.equal(allw[0], o) for o in allw[1:])
    z.close()


def test_zero2_dynamic_loss_scaling_overflow_skip_ws2():
    _run(_zero_overflow, 2)


def _zero_capturable(rank, ws):
    """capturable=True (device step counter, lr and bias corrections through
    gs_adam_hyper, the kernel reading them) equals the host-hyper engine bit
    for bit over steps with lr changes (refresh_hyper) and clipping; the device
    step count is the truth for state_dict."""
    from tests.test_ddp_cpu import _micro
    from distributed_training_amd.zero import ZeroDataParallel

    res = []
    for capt in (False, True):
        torch.manual_seed(0)
        m = _micro().to(torch.bfloat16)
        eng = ZeroDataParallel(m, stage=2, optimizer="adamw", lr=1e-3, weight_decay=1e-2, gradient_clipping=0.5,
                               capturable=capt)
        g = torch.Generator().manual_seed(7 + rank)
        for it in range(5):
            eng.param_groups[0]["lr"] = 1e-3 * (1 + it)  # a warm-up schedule, stepped by the caller
            eng.refresh_hyper()
            x = torch.rand(4, 3, 32, 32, generator=g).to(torch.bfloat16)
            y = torch.randint(0, 10, (4,), generator=g)
            eng.prepare_backward()
            torch.nn.functional.cross_entropy(m(x).float(), y).backward()
            eng.step()
            eng.zero_grad()
        assert eng.state_dict()["step"] == 5
        res.append([t.detach().clone() for t in eng.master] + [t.clone() for t in eng.state1 + eng.state2])
        eng.close()
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_zero_capturable_equals_host_hyper_ws2():
    from tests.test_ddp_cpu import _run

    _run(_zero_capturable, 2)
