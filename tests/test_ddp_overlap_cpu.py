"""The overlapped optimizer (DDP._register_fused_optim, T:nn/parallel/distributed.py
``_register_fused_optim``; torch/distributed/algorithms/_optimizer_overlap) on
CPU / gloo, world size 2:

* libgsync DDP + ``_register_fused_optim(SGD | Adam)`` == libgsync DDP +
  an explicit fused ``optimizer.step()`` after backward, bit for bit (the same
  elementwise update, launched per bucket instead of once);
* == torch's DDP + its own ``_register_fused_optim`` (functional per-parameter
  ``step_param``) within SURVEY.md §8c's tolerances (SGD rtol 1e-6 / atol 1e-7,
  fma placement; Adam atol lr·1e-3);
* the API contract: one registration, no comm hook beside it, lr changes on
  ``ddp._overlapped_optimizer`` reach the per-bucket updates, ``no_sync``
  accumulates and the next synchronising backward updates once."""
import pytest
import torch
import torch.nn as nn

from tests.test_ddp_cpu import _micro, _run

STEPS = 3


def _batches(rank, n):
    g = torch.Generator().manual_seed(1234 + rank)
    return [(torch.rand(4, 3, 32, 32, generator=g), torch.randint(0, 10, (4,), generator=g)) for _ in range(n)]


def _train(rank, kind, impl, overlap):
    import distributed_training_amd as D

    torch.manual_seed(0)
    model = _micro()
    opt_cls = {"sgd": torch.optim.SGD, "adam": torch.optim.Adam}[kind]
    kw = dict(lr=0.05, momentum=0.9, weight_decay=1e-4) if kind == "sgd" else dict(lr=1e-3)
    if impl == "torch":
        ddp = torch.nn.parallel.DistributedDataParallel(model)
    else:
        ddp = D.DistributedDataParallel(model)
    opt = None
    if overlap:
        ddp._register_fused_optim(opt_cls, **kw)
    else:
        opt = (D.FusedSGD if kind == "sgd" else D.FusedAdam)(ddp.parameters(), **kw)
    for x, y in _batches(rank, STEPS):
        nn.functional.cross_entropy(ddp(x), y).backward()
        if opt is not None:
            opt.step()
        for p in model.parameters():
            p.grad = None
    return [p.detach().clone() for p in model.parameters()], ddp


def _compare(rank, ws, kind):
    ref, _ = _train(rank, kind, "libgsync", overlap=False)
    got, ddp = _train(rank, kind, "libgsync", overlap=True)
    for i, (a, b) in enumerate(zip(ref, got)):
        assert torch.equal(a, b), f"{kind} param {i}: overlapped != explicit step"
    tor, _ = _train(rank, kind, "torch", overlap=True)
    tol = dict(rtol=1e-6, atol=1e-7) if kind == "sgd" else dict(rtol=0, atol=1e-3 * 1e-3)
    for i, (a, b) in enumerate(zip(tor, got)):
        torch.testing.assert_close(b, a, **tol, msg=lambda m: f"{kind} param {i} vs torch overlap: {m}")
    st = ddp._overlapped_optimizer.state
    assert len(st) == len(got)  # one state for every parameter, held by the main optimizer
    if kind == "adam":
        assert all(float(s["step"]) == STEPS for s in st.values())


def _contract(rank, ws):
    import distributed_training_amd as D

    torch.manual_seed(0)
    model = _micro()
    ddp = D.DistributedDataParallel(model)
    ddp._register_fused_optim(torch.optim.SGD, lr=0.0)
    with pytest.raises(RuntimeError):
        ddp._register_fused_optim(torch.optim.SGD, lr=0.1)
    with pytest.raises(RuntimeError):
        ddp.register_comm_hook(None, lambda s, b: None)
    (x, y), (x2, y2) = _batches(rank, 2)
    w0 = [p.detach().clone() for p in model.parameters()]
    nn.functional.cross_entropy(ddp(x), y).backward()  # lr 0: nothing moves
    assert all(torch.equal(a, p) for a, p in zip(w0, model.parameters()))
    for p in model.parameters():
        p.grad = None
    ddp._overlapped_optimizer.param_groups[0]["lr"] = 0.1  # a schedule acts on the main optimizer
    with ddp.no_sync():
        nn.functional.cross_entropy(ddp(x), y).backward()
    assert all(torch.equal(a, p) for a, p in zip(w0, model.parameters()))  # no update without sync
    nn.functional.cross_entropy(ddp(x2), y2).backward()
    moved = sum(not torch.equal(a, p) for a, p in zip(w0, model.parameters()))
    assert moved == len(w0)
    # a checkpoint round trip through the main optimizer reaches the per-bucket updates
    sd = ddp._overlapped_optimizer.state_dict()
    ddp._overlapped_optimizer.load_state_dict(sd)
    w1 = [p.detach().clone() for p in model.parameters()]
    for p in model.parameters():
        p.grad = None
    nn.functional.cross_entropy(ddp(x), y).backward()
    per_bucket = [o for o in ddp._overlap["per_bucket"].values() if o]
    assert per_bucket and all(o.state is ddp._overlapped_optimizer.state for o in per_bucket)
    assert all(not torch.equal(a, p) for a, p in zip(w1, model.parameters()))
    with pytest.raises(RuntimeError):
        D.DistributedDataParallel(_micro())._register_fused_optim(torch.optim.RMSprop, lr=0.1)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_overlapped_optimizer_matches_explicit_step_and_torch(kind):
    _run(_compare, 2, kind)


def test_overlapped_optimizer_contract():
    _run(_contract, 2)


class _Branchy(nn.Module):
    """A trunk plus three heads: head a is used on rank 0, head b on rank 1,
    head c on no rank (find_unused_parameters with rank-dependent usage)."""

    def __init__(self):
        super().__init__()
        self.trunk = nn.Linear(12, 16)
        self.a = nn.Linear(16, 5)
        self.b = nn.Linear(16, 5)
        self.c = nn.Linear(16, 5)

    def forward(self, x, which):
        h = torch.relu(self.trunk(x))
        return self.a(h) if which == 0 else self.b(h)


def _unused_train(rank, kind, impl, bucket_cap_mb):
    import distributed_training_amd as D

    torch.manual_seed(0)
    model = _Branchy()
    kw = dict(lr=0.05, momentum=0.9, weight_decay=1e-2) if kind == "sgd" else dict(lr=1e-2, weight_decay=1e-2)
    cls = torch.optim.SGD if kind == "sgd" else torch.optim.AdamW
    if impl == "torch":
        ddp = torch.nn.parallel.DistributedDataParallel(model, find_unused_parameters=True,
                                                        bucket_cap_mb=bucket_cap_mb)
    else:
        ddp = D.DistributedDataParallel(model, find_unused_parameters=True, bucket_cap_mb=bucket_cap_mb)
    ddp._register_fused_optim(cls, **kw)
    g = torch.Generator().manual_seed(77 + rank)
    grads = []
    for step in range(3):
        x = torch.randn(6, 12, generator=g)
        ddp(x, rank % 2).square().mean().backward()
        grads.append([None if p.grad is None else p.grad.clone() for p in model.parameters()])
        for p in model.parameters():
            p.grad = None
    return [p.detach().clone() for p in model.parameters()], grads


def _unused_compare(rank, ws, kind, bucket_cap_mb):
    ref, ref_g = _unused_train(rank, kind, "torch", bucket_cap_mb)
    got, got_g = _unused_train(rank, kind, "libgsync", bucket_cap_mb)
    w0 = _Branchy()
    names = [n for n, _ in w0.named_parameters()]
    tol = dict(rtol=1e-6, atol=1e-7) if kind == "sgd" else dict(rtol=1e-6, atol=1e-6)
    for n, a, b in zip(names, ref, got):
        torch.testing.assert_close(b, a, **tol, msg=lambda m: f"{kind} {n} vs torch overlap: {m}")
    # the never-used head moved (weight decay + momentum on zero grads), as torch's
    torch.manual_seed(0)
    init = dict(_Branchy().named_parameters())
    assert not torch.equal(got[names.index("c.weight")], init["c.weight"].detach())
    for step, (gr, gg) in enumerate(zip(ref_g, got_g)):
        for n, a, b in zip(names, gr, gg):
            assert (a is None) == (b is None), f"step {step} {n}: grad presence differs from torch"
            if a is not None:
                torch.testing.assert_close(b, a, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("kind", ["sgd", "adamw"])
@pytest.mark.parametrize("bucket_cap_mb", [None, 0.0005])
def test_overlapped_optimizer_with_rank_dependent_unused_parameters(kind, bucket_cap_mb):
    """a parameter unused on this rank but used on another —
    and one unused everywhere — must be stepped by the overlapped optimizer on
    every rank, as torch's _hook_then_optimizer steps every bucket parameter
    with bucket.gradients()."""
    _run(_unused_compare, 2, kind, bucket_cap_mb)
