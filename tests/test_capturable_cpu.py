"""Capturable fused optimizers (device hyper-parameter source) on the host
backend: the same update as the default path, step for step, across an LR
schedule and an AMP overflow skip (T:optim/adam.py capturable branch)."""
import pytest
import torch

import distributed_training_amd as D


def _model(seed):
    torch.manual_seed(seed)
    return [torch.randn(n) for n in (7, 64, 1000, 3)]


def _run(opt_cls, capturable, steps=5, **kw):
    ps = [p.clone().requires_grad_(False) for p in _model(0)]
    opt = opt_cls(ps, capturable=capturable, **kw)
    gen = torch.Generator().manual_seed(1)
    found = torch.zeros(1)
    for i in range(steps):
        for p in ps:
            p.grad = torch.randn(p.shape, generator=gen) * 0.1
        if i == 2:
            for g in opt.param_groups:
                g["lr"] = g["lr"] * 0.5  # scheduler between steps
        if i == 3:  # overflow: device-skipped step (AMP)
            found.fill_(1.0)
            opt.found_inf = found
            if not capturable:
                opt.step()  # host path reads the flag and skips
                opt.found_inf = None
                continue
        opt.step()
        opt.found_inf = None
        found.zero_()
    return ps, opt


@pytest.mark.parametrize("adamw,wd", [(False, 0.0), (False, 0.01), (True, 0.05)])
def test_capturable_adam_matches_default(adamw, wd):
    ref, ro = _run(D.FusedAdam, False, lr=1e-2, weight_decay=wd, adamw=adamw)
    got, co = _run(D.FusedAdam, True, lr=1e-2, weight_decay=wd, adamw=adamw)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    # the device counter did not advance on the skipped step, as torch's host count
    p0 = ro.param_groups[0]["params"][0]
    assert float(co.state[co.param_groups[0]["params"][0]]["step"]) == float(ro.state[p0]["step"]) == 4.0


@pytest.mark.parametrize("nesterov", [False, True])
def test_capturable_sgd_matches_default(nesterov):
    ref, _ = _run(D.FusedSGD, False, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=nesterov)
    got, _ = _run(D.FusedSGD, True, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=nesterov)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_adam_hyper_vs_oracle_formula():
    """gs_adam_hyper's fp32 outputs equal the host-double formula rounded once."""
    import numpy as np
    ps = [torch.zeros(4)]
    opt = D.FusedAdam(ps, lr=3e-3, betas=(0.8, 0.95), weight_decay=0.1, adamw=True, capturable=True)
    for k in range(1, 6):
        ps[0].grad = torch.ones(4)
        opt.step()
        (cohort,) = opt._dev_hyper[0]["cohorts"].values()  # one device step counter: every param has a grad
        h = cohort["hyper"]
        bc1, bc2 = 1 - 0.8 ** k, 1 - 0.95 ** k
        exp = np.array([(3e-3 / bc1) * -1, bc2 ** 0.5, 1 - 3e-3 * 0.1], dtype=np.float32)
        assert np.array_equal(h.numpy(), exp)


def test_capturable_state_dict_roundtrip():
    ps, opt = _run(D.FusedAdam, True, lr=1e-2)
    import copy
    sd = copy.deepcopy(opt.state_dict())  # as a checkpoint file would (no aliasing)
    ps2 = [p.clone() for p in ps]
    opt2 = D.FusedAdam(ps2, lr=1e-2, capturable=True)
    opt2.load_state_dict(sd)
    gen = torch.Generator().manual_seed(9)
    grads = [torch.randn(p.shape, generator=gen) for p in ps]
    for p, q, g in zip(ps, ps2, grads):
        p.grad, q.grad = g.clone(), g.clone()
    opt.step()
    opt2.step()
    for a, b in zip(ps, ps2):
        assert torch.equal(a, b)
