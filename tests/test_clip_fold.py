"""The gradient-norm clip folded into the update kernels (gs_plan_set_clip /
gs_sqnorm_partial) against the separate path it replaces (Σg² + combine,
gs_clip_coef, the mul_ launches; optim.CLIP_FUSED = False): bit-identical
parameters, optimizer state and published norm, for SGD and Adam, with and
without an AMP grad scale, a skipped (found_inf) step, and ZeRO's loss-scale
multipliers.  Reference arithmetic: T:nn/utils/clip_grad.py:165-174 (coef),
DeepSpeed gradient_clipping R:resnet/deepspeed/deepspeed_train.py:195.

CPU tests run the host backend; the `gpu` ones the gfx950 kernels, where the
folded coefficient comes from the Σg² kernel's 64 group sums."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import distributed_training_amd as D
from distributed_training_amd import optim as O

SIZES = [1000, 64, 4099, 3, 70001, 17, 2 ** 16, 1]


def _params(dev, seed=0, sizes=SIZES):
    g = torch.Generator().manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(n, generator=g).to(dev)) for n in sizes]
    for p in ps:
        p.grad = (torch.randn(p.shape, generator=g) * 0.3).to(dev)
    return ps


def _run(dev, fused, opt_cls, kw, gscale=None, found_inf=None, steps=3):
    old = O.CLIP_FUSED
    O.CLIP_FUSED = fused
    try:
        ps = _params(dev)
        opt = opt_cls(ps, max_grad_norm=1.0, **kw)
        if gscale is not None:
            opt.grad_scale = torch.tensor([gscale], device=dev)
        if found_inf is not None:
            opt.found_inf = torch.tensor([found_inf], device=dev)
        norms = []
        for s in range(steps):
            for i, p in enumerate(ps):
                p.grad.mul_(1.0 + 0.25 * s)  # a different norm every step
            opt.step()
            norms.append(opt.last_grad_norm.clone())
        if dev.type == "cuda":
            torch.cuda.synchronize()
        state = [(k, v.clone()) for p in ps for k, v in sorted(opt.state[p].items()) if torch.is_tensor(v)]
        return [p.detach().clone() for p in ps], state, torch.cat(norms)
    finally:
        O.CLIP_FUSED = old


def _assert_same(a, b):
    pa, sa, na = a
    pb, sb, nb = b
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)
    for (k1, x), (k2, y) in zip(sa, sb):
        assert k1 == k2 and torch.equal(x.float().cpu(), y.float().cpu()), k1
    assert torch.equal(na, nb)


CASES = [
    (D.FusedSGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
    (D.FusedAdam, dict(lr=1e-3)),
    (D.FusedAdamW, dict(lr=1e-3, weight_decay=0.01)),
]


@pytest.mark.parametrize("opt_cls,kw", CASES)
@pytest.mark.parametrize("gscale", [None, 0.125])
def test_folded_clip_equals_separate_path_cpu(opt_cls, kw, gscale):
    dev = torch.device("cpu")
    _assert_same(_run(dev, True, opt_cls, kw, gscale), _run(dev, False, opt_cls, kw, gscale))


def test_folded_clip_skipped_step_cpu():
    dev = torch.device("cpu")
    fused = _run(dev, True, D.FusedSGD, CASES[0][1], 0.5, found_inf=1.0)
    sep = _run(dev, False, D.FusedSGD, CASES[0][1], 0.5, found_inf=1.0)
    _assert_same(fused, sep)
    assert torch.equal(fused[0][0], _params(dev)[0].detach())  # nothing moved


@pytest.mark.parametrize("opt_cls,kw", CASES)
@pytest.mark.parametrize("gscale", [None, 0.5, 0.125])
@pytest.mark.parametrize("found_inf", [0.0, 1.0])
def test_folded_clip_amp_device_state_cpu(opt_cls, kw, gscale, found_inf):
    """The AMP path (found_inf set: device step counters / first-step flags)
    with an unscale multiplier: the folded clip equals the separate one."""
    dev = torch.device("cpu")
    _assert_same(_run(dev, True, opt_cls, kw, gscale, found_inf=found_inf),
                 _run(dev, False, opt_cls, kw, gscale, found_inf=found_inf))


def test_folded_clip_several_plans_cpu():
    """Two grad dtypes -> two plans: Σg² accumulated into one scalar that every
    update launch reads while each publishes the scaled Σg² (kept apart)."""
    dev = torch.device("cpu")
    res = []
    for fused in (True, False):
        O.CLIP_FUSED = fused
        try:
            ps = _params(dev)
            ps[1].grad_dtype = None  # torch 2.10: a grad of another dtype needs this
            ps[1].grad = ps[1].grad.bfloat16()
            opt = D.FusedSGD(ps, lr=0.1, momentum=0.9, max_grad_norm=1.0)
            opt.grad_scale = torch.tensor([0.25])
            for _ in range(2):
                opt.step()
            res.append(([p.detach().clone() for p in ps], opt.last_grad_norm.clone()))
        finally:
            O.CLIP_FUSED = True
    for x, y in zip(res[0][0], res[1][0]):
        assert torch.equal(x, y)
    assert torch.equal(res[0][1], res[1][1])


def test_amp_adam_first_step_one_cohort_cpu():
    """Parameters whose Adam state starts in the same step share one device
    step counter and one update plan (they got one each: a launch per tensor)."""
    ps = _params(torch.device("cpu"))
    opt = D.FusedAdam(ps, lr=1e-3)
    opt.found_inf = torch.zeros(1)
    opt.step()
    assert len(list(opt._plans.plans())) == 1
    assert len({id(opt.state[p]["step"]) for p in ps}) == 1


def test_plan_clip_needs_partial_first():
    plan = D.multi_tensor.TensorListPlan([8], torch.device("cpu"), task_units=0)
    p, g, b = torch.zeros(8), torch.ones(8), torch.zeros(8)
    plan.set_ptrs(0, [p])
    plan.set_ptrs(1, [g])
    plan.set_ptrs(2, [b])
    plan.set_clip(1.0)
    with pytest.raises(D._lib.GsyncError, match="gs_sqnorm_partial"):
        plan.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)
    plan.sqnorm_partial(1, torch.float32)
    out = torch.zeros(3)
    plan.set_clip(1.0, out=out)
    plan.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)
    # ‖g‖ = sqrt(8): coef = 1/(sqrt(8)+1e-6); p = -0.1 * coef
    nrm = torch.tensor(8.0).sqrt()
    coef = torch.clamp(1.0 / (nrm + 1e-6), max=1.0)
    assert torch.equal(out, torch.stack([torch.tensor(8.0), coef, nrm]))
    assert torch.equal(p, torch.full((8,), 1.0) * coef * -0.1)


def test_plan_clip_partial_is_single_use():
    """the plan's own Σg² partial feeds ONE clipped update; a second
    update without a fresh gs_sqnorm_partial fails (GS_ESTATE) instead of
    clipping with stale sums."""
    plan = D.multi_tensor.TensorListPlan([8], torch.device("cpu"), task_units=0)
    p, g, b = torch.zeros(8), torch.ones(8), torch.zeros(8)
    for k, t in enumerate((p, g, b)):
        plan.set_ptrs(k, [t])
    plan.sqnorm_partial(1, torch.float32)
    plan.set_clip(1.0)
    plan.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)
    with pytest.raises(D._lib.GsyncError, match="gs_sqnorm_partial"):
        plan.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)
    plan.sqnorm_partial(1, torch.float32)
    plan.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)


def _dpp_wave_sum(x):
    """The update kernel's fold of up to 512 partial sums (gs_engine.h
    clip_multiplier), restated independently: lane l first adds partials l,
    l + 64, ... in order (fp32), then the 64-lane tree of wave_reduce —
    quad_perm [1,0,3,2] / [2,3,0,1] and the half-row / row mirrors are lane XORs
    1 / 2 / 7 / 15; row_bcast:15 adds lane 15 of the row below into rows 1 and 3,
    row_bcast:31 adds lane 31 into rows 2 and 3."""
    lanes = np.arange(64)
    v = np.zeros(64, np.float32)
    x = np.asarray(x, np.float32)
    for lane in range(64):
        a = np.float32(0.0)
        for j in range(lane, len(x), 64):
            a = np.float32(a + x[j])
        v[lane] = a

    def step(v, src, rows):
        t = np.zeros(64, np.float32)
        m = np.isin(lanes // 16, rows)
        t[m] = v[src[m]]
        return (v + t).astype(np.float32)

    for mask in (1, 2, 7, 15):
        v = step(v, lanes ^ mask, [0, 1, 2, 3])
    v = step(v, (lanes // 16) * 16 - 1, [1, 3])
    v = step(v, np.full(64, 31), [2, 3])
    return v[63]


@pytest.mark.parametrize("n", [1, 5, 64, 65, 200, 512])
def test_clip_groups_fold_host(n):
    """gs_plan_set_clip_groups on a host plan: the published Σg² is the device
    fold of the partial sums (restated above), coefficient and update follow."""
    g0 = torch.Generator().manual_seed(n)
    groups = torch.rand(D._lib.GS_RED_PARTIALS, generator=g0) * 100.0
    plan = D.multi_tensor.TensorListPlan([16], torch.device("cpu"), task_units=0)
    p, g, b = torch.zeros(16), torch.ones(16), torch.zeros(16)
    for k, t in enumerate((p, g, b)):
        plan.set_ptrs(k, [t])
    out = torch.zeros(3)
    plan.set_clip_groups(1.0, 1e-6, groups, n, out=out)
    plan.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)
    sq = np.float32(_dpp_wave_sum(groups[:n].numpy()))
    assert out[0].item() == float(sq)
    nrm = np.sqrt(sq, dtype=np.float32)
    coef = min(np.float32(1.0) / (nrm + np.float32(1e-6)), np.float32(1.0))
    assert out[1].item() == float(coef) and out[2].item() == float(nrm)
    want = np.float32(-0.1) * np.float32(np.float32(1.0) * coef)  # fmaf(-lr, g·coef, 0)
    assert torch.equal(p, torch.full((16,), float(want)))
    with pytest.raises(D._lib.GsyncError, match="n_groups"):
        plan.set_clip_groups(1.0, 1e-6, torch.zeros(D._lib.GS_RED_PARTIALS + 1), D._lib.GS_RED_PARTIALS + 1)
    with pytest.raises(ValueError, match="partial sums"):
        plan.set_clip_groups(1.0, 1e-6, groups[:8], 9)


def test_sqnorm_partial_out_host():
    """Host plans: one group, the finished Σg² (what gs_sqnorm gives); the slots
    past it are zeroed (a sharded caller all-reduces the whole buffer)."""
    xs = [torch.randn(n, generator=torch.Generator().manual_seed(n)) for n in (7, 1000, 33)]
    plan = D.multi_tensor.TensorListPlan([x.numel() for x in xs], torch.device("cpu"), task_units=0)
    plan.set_ptrs(1, xs)
    gr = torch.full((D._lib.GS_RED_PARTIALS,), 7.0)
    n = plan.sqnorm_partial_out(1, torch.float32, gr)
    ref = torch.zeros(1)
    plan.sqnorm(1, torch.float32, ref)
    assert n == 1 and gr[0].item() == ref.item() and not gr[1:].any()
    with pytest.raises(ValueError, match="partial sums"):
        plan.sqnorm_partial_out(1, torch.float32, torch.zeros(64))


@pytest.mark.gpu
@pytest.mark.parametrize("opt_cls,kw", CASES)
@pytest.mark.parametrize("gscale", [None, 0.125])
def test_folded_clip_equals_separate_path_gpu(opt_cls, kw, gscale):
    dev = torch.device("cuda", 0)
    _assert_same(_run(dev, True, opt_cls, kw, gscale), _run(dev, False, opt_cls, kw, gscale))


@pytest.mark.gpu
@pytest.mark.parametrize("opt_cls,kw", CASES)
@pytest.mark.parametrize("found_inf", [0.0, 1.0])
def test_folded_clip_amp_device_state_gpu(opt_cls, kw, found_inf):
    dev = torch.device("cuda", 0)
    _assert_same(_run(dev, True, opt_cls, kw, 0.5, found_inf=found_inf),
                 _run(dev, False, opt_cls, kw, 0.5, found_inf=found_inf))


@pytest.mark.gpu
@pytest.mark.parametrize("mixed", [False, True])
def test_folded_clip_large_plan_gpu(mixed):
    """ResNet-50-sized single plan (25.6 M elements: the Σg² kernel's full 64
    groups), and with one bf16 grad (two plans: the accumulated-scalar form)."""
    dev = torch.device("cuda", 0)
    sizes = [2048 * 1000, 1000, 512 * 2048, 2048, 2048 * 512 * 9, 64 * 3 * 49, 7, 2048 * 4096]
    res = []
    try:
        for fused in (True, False):
            O.CLIP_FUSED = fused
            g = torch.Generator(device=dev).manual_seed(3)
            ps = [torch.nn.Parameter(torch.randn(n, device=dev, generator=g)) for n in sizes]
            for p in ps:
                p.grad = torch.randn(p.shape, device=dev, generator=g) * 0.01
            if mixed:
                ps[1].grad_dtype = None  # torch 2.10: a grad of another dtype needs this
                ps[1].grad = ps[1].grad.bfloat16()
            opt = D.FusedSGD(ps, lr=0.1, momentum=0.9, max_grad_norm=0.5)
            opt.step()
            opt.step()
            torch.cuda.synchronize()
            res.append(([p.detach().clone() for p in ps], opt.last_grad_norm.clone()))
    finally:
        O.CLIP_FUSED = True
    for x, y in zip(res[0][0], res[1][0]):
        assert torch.equal(x, y)
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.gpu
def test_clip_groups_fold_gpu_equals_host_and_sqnorm():
    """The device fold of gs_plan_set_clip_groups == the host restatement bit for
    bit (512, 200, 65, 64, 5 and 1 random partial sums); gs_sqnorm_partial_out's
    64 group sums of a large slot folded == gs_sqnorm's Σg² bit for bit; on a
    small plan (a ZeRO N=8 shard) its raw per-workgroup partials, folded, equal
    the restated fold of the same partials and the double Σ to fp32 rounding."""
    dev = torch.device("cuda", 0)
    for n in (512, 200, 65, 64, 5, 1):
        groups = torch.rand(D._lib.GS_RED_PARTIALS, generator=torch.Generator().manual_seed(n)) * 100.0
        outs = []
        for d in (dev, torch.device("cpu")):
            plan = D.multi_tensor.TensorListPlan([4096], d, task_units=0)
            p, g, b = (torch.zeros(4096, device=d), torch.ones(4096, device=d), torch.zeros(4096, device=d))
            for k, t in enumerate((p, g, b)):
                plan.set_ptrs(k, [t])
            out = torch.zeros(3, device=d)
            plan.set_clip_groups(1.0, 1e-6, groups.to(d), n, out=out)
            plan.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)
            outs.append((out.cpu(), p.cpu()))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), n
        assert outs[1][0][0].item() == float(np.float32(_dpp_wave_sum(groups[:n].numpy())))
    sizes = [2048 * 1000, 1000, 512 * 2048, 2048, 2048 * 512 * 9, 64 * 3 * 49, 7, 2048 * 4096]
    gen = torch.Generator(device=dev).manual_seed(9)
    xs = [torch.randn(k, device=dev, generator=gen) * 0.01 for k in sizes]
    plan = D.multi_tensor.TensorListPlan(sizes, dev)
    plan.set_ptrs(1, xs)
    gr = torch.full((D._lib.GS_RED_PARTIALS,), 7.0, device=dev)  # stale slots: zeroed by the call
    n = plan.sqnorm_partial_out(1, torch.float32, gr)
    ref = torch.zeros(1, device=dev)
    plan.sqnorm(1, torch.float32, ref)
    torch.cuda.synchronize()
    assert n == 64 and not gr[n:].any()
    assert float(np.float32(_dpp_wave_sum(gr.cpu().numpy()[:n]))) == ref.item()
    # the raw form: 3.2 M bf16 elements (ResNet-50 / 8), one partial per workgroup
    shard = (torch.randn(3194688, device=dev, generator=gen) * 1e-3).to(torch.bfloat16)
    small = D.multi_tensor.TensorListPlan([shard.numel()], dev)
    small.set_ptrs(1, [shard])
    gr.fill_(7.0)
    n = small.sqnorm_partial_out(1, torch.bfloat16, gr)
    torch.cuda.synchronize()
    parts = gr.cpu().numpy()
    assert 64 < n <= D._lib.GS_RED_PARTIALS and not parts[n:].any(), n
    exact = float((shard.double() ** 2).sum())
    assert abs(float(parts[:n].astype(np.float64).sum()) - exact) <= 1e-5 * exact
    p1, g1, b1 = (torch.zeros(8, device=dev), torch.ones(8, device=dev), torch.zeros(8, device=dev))
    up = D.multi_tensor.TensorListPlan([8], dev)
    for k, t in enumerate((p1, g1, b1)):
        up.set_ptrs(k, [t])
    out = torch.zeros(3, device=dev)
    up.set_clip_groups(1.0, 1e-6, gr, n, out=out)
    up.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)
    assert out[0].item() == float(np.float32(_dpp_wave_sum(parts[:n])))


@pytest.mark.gpu
def test_sharded_partials_with_different_counts_gpu():
    """ZeRO's world > 1 clip when two ranks' shards have different chunk maps (the
    same element count split into different tensor pieces): their raw partial
    counts differ, so the whole GS_RED_PARTIALS buffer travels and is folded.
    Buffers start stale (the call zeroes the slots past its count); their sum (the
    all-reduce) folded over all GS_RED_PARTIALS slots gives the exact Σg² of both
    shards to fp32 rounding, bit-equal to the restated fold, on a second call too."""
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(13)
    total = 3194688
    a = (torch.randn(total, device=dev, generator=gen) * 1e-3).to(torch.bfloat16)
    pieces = [999] * (total // 999) + [total % 999]  # 64-aligned: ~one chunk per piece
    b_flat = (torch.randn(total, device=dev, generator=gen) * 1e-3).to(torch.bfloat16)
    b = list(b_flat.split(pieces))
    pa = D.multi_tensor.TensorListPlan([total], dev)
    pa.set_ptrs(1, [a])
    pb = D.multi_tensor.TensorListPlan(pieces, dev, align=64)
    pb.set_ptrs(1, b)
    exact = float((a.double() ** 2).sum() + (b_flat.double() ** 2).sum())
    P = D._lib.GS_RED_PARTIALS
    for _ in range(2):
        ga = torch.full((P,), 5.0, device=dev)
        gb = torch.full((P,), 3.0, device=dev)
        na = pa.sqnorm_partial_out(1, torch.bfloat16, ga)
        nb = pb.sqnorm_partial_out(1, torch.bfloat16, gb)
        torch.cuda.synchronize()
        assert na != nb and 64 < min(na, nb) and max(na, nb) <= P, (na, nb)
        assert not ga[na:].any() and not gb[nb:].any()
        tot = ga + gb  # the SUM all-reduce of two ranks
        p1, g1, b1 = (torch.zeros(8, device=dev), torch.ones(8, device=dev), torch.zeros(8, device=dev))
        up = D.multi_tensor.TensorListPlan([8], dev)
        for k, t in enumerate((p1, g1, b1)):
            up.set_ptrs(k, [t])
        out = torch.zeros(3, device=dev)
        up.set_clip_groups(1.0, 1e-6, tot, P, out=out)
        up.sgd(torch.float32, 0.1, 0.0, 0.0, 0.0, False, False, True)
        torch.cuda.synchronize()
        assert out[0].item() == float(np.float32(_dpp_wave_sum(tot.cpu().numpy())))
        assert abs(out[0].item() - exact) <= 1e-5 * exact


_RED_FUSE_CHILD = r"""
import sys, torch
sys.path.insert(0, {repo!r})
from tests.test_clip_fold import _run, _assert_same, CASES
dev = torch.device("cuda", 0)
for opt_cls, kw in CASES:
    _assert_same(_run(dev, True, opt_cls, kw, None), _run(dev, False, opt_cls, kw, None))
print("OK")
"""


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"GS_RED_FUSE": "16"}, {"GS_RED_FUSE": "0"}, {"GS_RED_GRID": "512"}])
def test_folded_clip_equals_separate_path_reduction_overrides_gpu(env):
    """the folded clip follows the reduction settings gs_sqnorm uses
    (GS_RED_FUSE groups, or the combine launch at GS_RED_FUSE=0; GS_RED_GRID), so
    it stays bit-identical to the separate path under the A/B sweeps' overrides
    (read once per process: a child process per setting)."""
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _RED_FUSE_CHILD.format(repo=repo)], env={**os.environ, **env},
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


_NT_READ_CHILD = r"""
import hashlib, sys, torch
sys.path.insert(0, {repo!r})
import distributed_training_amd as D
dev = torch.device("cuda", 0)
sizes = [48 * 1024 * 1024, 1000, 24 * 1024 * 1024 + 7, 2048]  # 288 MiB of fp32 grads: above the cache
gen = torch.Generator(device=dev).manual_seed(5)
gs = [torch.randn(k, device=dev, generator=gen) * 0.01 for k in sizes]
ps = [torch.randn(k, device=dev, generator=gen) for k in sizes]
bs = [torch.randn(k, device=dev, generator=gen) * 0.01 for k in sizes]
plan = D.multi_tensor.TensorListPlan(sizes, dev)
for k, ts in enumerate((ps, gs, bs)):
    plan.set_ptrs(k, ts)
sq = torch.zeros(1, device=dev)
plan.sqnorm(1, torch.float32, sq)
out = torch.zeros(3, device=dev)
plan.sqnorm_partial(1, torch.float32)
plan.set_clip(0.5, 1e-6, None, 1.0, 1.0, out=out)
plan.sgd(torch.float32, 0.1, 0.9, 0.0, 1e-4, False, False, False)
torch.cuda.synchronize()
h = hashlib.sha256()
for t in ps + bs:
    h.update(t.cpu().numpy().tobytes())
print("RES", sq.item().hex(), out.cpu().numpy().tobytes().hex(), h.hexdigest())
"""


@pytest.mark.gpu
def test_nt_read_once_policy_changes_no_bits_gpu():
    """Σg², the folded clip's partials and the clipped SGD over a 288 MiB gradient
    slot (above the Infinity Cache: the size rule's non-temporal loads) give the
    same bits under GS_NT_READ_ONCE = 0 (cached), 1 (always NT) and the default
    rule: the load policy moves the bytes differently, never the sum's order
    (a child process per setting: the policy is read once per process)."""
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for pol in ("0", "1", None):
        env = {k: v for k, v in os.environ.items() if k != "GS_NT_READ_ONCE"}
        if pol is not None:
            env["GS_NT_READ_ONCE"] = pol
        r = subprocess.run([sys.executable, "-c", _NT_READ_CHILD.format(repo=repo)], env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        res.append([ln for ln in r.stdout.splitlines() if ln.startswith("RES")][0])
    assert res[0] == res[1] == res[2], res


def test_read_hint_setter_cpu():
    """gs_plan_set_read_hint takes 0 / 1 / 2 (a host plan keeps it and ignores it)."""
    plan = D.multi_tensor.TensorListPlan([1000, 7], torch.device("cpu"))
    for h in (1, 2, 0):
        plan.set_read_hint(h)
    with pytest.raises(D._lib.GsyncError, match="hint"):
        plan.set_read_hint(3)


@pytest.mark.gpu
def test_read_hint_changes_no_bits_gpu():
    """Σg², its group sums and its raw partials (a small plan) below the cache size
    give the same bits with the default rule (cached there), the non-temporal hint
    and the cached hint: the hint moves the bytes differently, never the order."""
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(21)
    sizes = [2048 * 1000, 1000, 512 * 2048, 64 * 3 * 49, 7, 2048 * 4096]
    xs = [torch.randn(k, device=dev, generator=gen) * 0.01 for k in sizes]
    small = (torch.randn(3194688, device=dev, generator=gen) * 1e-3).to(torch.bfloat16)
    res = []
    for h in (0, 1, 2):
        plan = D.multi_tensor.TensorListPlan(sizes, dev)
        plan.set_ptrs(1, xs)
        plan.set_read_hint(h)
        sq = torch.zeros(1, device=dev)
        plan.sqnorm(1, torch.float32, sq)
        gr = torch.zeros(D._lib.GS_RED_PARTIALS, device=dev)
        plan.sqnorm_partial_out(1, torch.float32, gr)
        sp = D.multi_tensor.TensorListPlan([small.numel()], dev)
        sp.set_ptrs(1, [small])
        sp.set_read_hint(h)
        gs = torch.zeros(D._lib.GS_RED_PARTIALS, device=dev)
        sp.sqnorm_partial_out(1, torch.bfloat16, gs)
        torch.cuda.synchronize()
        res.append((sq.cpu(), gr.cpu(), gs.cpu()))
    for r in res[1:]:
        assert all(torch.equal(a, b) for a, b in zip(res[0], r))


def _ddp_fused_norm(rank, ws, device="cpu", steps=4):
    """FusedSGD.fuse_grad_norm_into(ddp): Σg² of the averaged grads formed inside
    the DDP's bucket unpacks (several buckets, accumulated in bucket order), the
    clipped update folding that scalar — against the same DDP + clipped FusedSGD
    whose Σg² pass runs in the optimizer: published norms within fp32 rounding
    (rtol 1e-6: the two sums add the same squares in another order), weights within
    SURVEY §8c's SGD bound (rtol 1e-5, atol 1e-7), with a no_sync accumulation step
    (synchronised by the next backward) and the ranks' weights identical."""
    import torch.distributed as dist

    from tests.test_ddp_cpu import _micro

    dev = torch.device(device)
    torch.manual_seed(0)
    m1, m2 = _micro().to(dev), _micro().to(dev)
    m2.load_state_dict(m1.state_dict())
    a = D.DistributedDataParallel(m1, bucket_cap_mb=0.05)
    b = D.DistributedDataParallel(m2, bucket_cap_mb=0.05)
    oa = D.FusedSGD(a.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, max_grad_norm=0.5)
    ob = D.FusedSGD(b.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, max_grad_norm=0.5)
    oa.fuse_grad_norm_into(a)
    g = torch.Generator().manual_seed(7 + rank)
    for it in range(steps):
        xs = [torch.rand(4, 3, 32, 32, generator=g).to(dev) for _ in range(2)]
        ys = [torch.randint(0, 10, (4,), generator=g).to(dev) for _ in range(2)]
        if it == 2:
            for model in (a, b):
                with model.no_sync():
                    torch.nn.functional.cross_entropy(model(xs[0]), ys[0]).backward()
        for model in (a, b):
            torch.nn.functional.cross_entropy(model(xs[1]), ys[1]).backward()
        oa.step()
        ob.step()
        assert oa.last_clip_source == "ddp_unpack" and ob.last_clip_source == "optimizer", it
        na, nb = oa.last_grad_norm.item(), ob.last_grad_norm.item()
        assert abs(na - nb) <= 1e-6 * nb, (it, na, nb)
        for (n, pa), pb in zip(m1.named_parameters(), m2.parameters()):
            torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-7, msg=f"it {it} {n}")
        oa.zero_grad()
        ob.zero_grad()
    # a step without a fresh synchronising backward falls back to the optimizer's own pass
    torch.nn.functional.cross_entropy(a(xs[1]), ys[1]).backward()
    oa.step()
    oa.step()
    assert oa.last_clip_source == "optimizer"
    if ws > 1:
        w = torch.cat([p.detach().reshape(-1).cpu() for p in m1.parameters()])
        allw = [None] * ws
        dist.all_gather_object(allw, w)
        assert all(torch.equal(allw[0], x) for x in allw[1:])


def test_ddp_fused_grad_norm_cpu_ws2():
    from tests.test_ddp_cpu import _run

    _run(_ddp_fused_norm, 2)


def _gpu_fused_norm_worker(rank, ws, backend, port, errq):
    try:
        from tests._dist_util import init_pg

        init_pg(backend, rank, ws, port)
        torch.cuda.set_device(0)
        # both models must see the same grads: MIOpen's default backward is not
        # run-to-run deterministic (that alone moved the norms by 3e-6)
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
        _ddp_fused_norm(rank, ws, "cuda")
        import torch.distributed as dist

        dist.barrier()
        if backend == "nccl":
            from distributed_training_amd.comm import destroy_communicators

            destroy_communicators()
        import gc

        gc.collect()  # as tests/test_ddp_cpu.py::_wrap: no gloo work outlives the interpreter
        dist.destroy_process_group()
    except BaseException as e:
        import traceback

        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


@pytest.mark.gpu
@pytest.mark.parametrize("backend,ws", [("nccl", 1), ("gloo", 2)])
def test_ddp_fused_grad_norm_gpu(backend, ws):
    """The same on the GPU: RCCL at ws=1 (the bucketer's own collective and
    unpacks) and two ranks sharing the GPU over gloo (host-staged buckets)."""
    import torch.multiprocessing as mp

    from tests._dist_util import free_port

    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_gpu_fused_norm_worker, args=(r, ws, backend, port, errq)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
