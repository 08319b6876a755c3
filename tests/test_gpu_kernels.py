"""Parity of libgsync's gfx950 kernels (through the C ABI) with the oracle.

Bit-exact for pack / unpack / scale / SGD / Adam (the oracle restates the
same fp32 expression, explicit fmaf, no contraction); sq-norm within
rtol 1e-5 (reduction order differs: per-workgroup partials vs double sum).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

RAGGED = [1, 3, 4, 5, 63, 64, 65, 1000, 16383, 16384, 16385, 70001] + [1 + (i % 7) for i in range(100)]


def to_np(t: torch.Tensor) -> np.ndarray:
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16).reshape(-1)
    return t.numpy().reshape(-1)


def rand_list(sizes, dtype, device, seed=0, scale=1.0, offset=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for n in sizes:
        base = torch.randn(n + offset, generator=g) * scale
        out.append(base.to(dtype).to(device)[offset:])
    return out


def plan_for(ts, device, align=0):
    from distributed_training_amd.multi_tensor import TensorListPlan

    return TensorListPlan([t.numel() for t in ts], device, align=align)


CASES = [
    (torch.float32, torch.float32, 1.0 / 2, 1, "f32"),
    (torch.float32, torch.float32, float(np.float32(1.0 / 3)), 1, "f32"),
    (torch.float32, torch.bfloat16, 0.125, 1, "bf16"),
    (torch.bfloat16, torch.bfloat16, 0.25, 1, "bf16"),
    (torch.float32, torch.bfloat16, 3.0, 2, "bf16"),
    (torch.float32, torch.float32, 1.0, 0, "f32"),
]


@pytest.mark.parametrize("align", [0, 64])
@pytest.mark.parametrize("offset", [0, 1])
@pytest.mark.parametrize("src_dt,flat_dt,scale,mode,fname", CASES)
def test_pack_unpack_bitwise(cuda_device, align, offset, src_dt, flat_dt, scale, mode, fname):
    from distributed_training_amd import _lib as L

    ts = rand_list(RAGGED, src_dt, cuda_device, seed=1, offset=offset)
    plan = plan_for(ts, cuda_device, align)
    plan.set_ptrs(1, ts)
    flat = torch.full((plan.flat_numel,), 7.0, dtype=flat_dt, device=cuda_device)
    flat.zero_()
    plan.pack(1, src_dt, flat, scale, mode)
    torch.cuda.synchronize()
    srcs = [to_np(t) for t in ts]
    src_code = O.BF16 if src_dt == torch.bfloat16 else O.F32
    ref = O.pack(srcs, fname, scale, mode, align, src_dtype=src_code)
    assert np.array_equal(to_np(flat), ref)
    # unpack back into fresh tensors, with the fused sq-norm
    outs = [torch.empty_like(t, dtype=torch.float32) for t in ts]
    plan.set_ptrs(2, outs)
    sq = torch.zeros(1, dtype=torch.float32, device=cuda_device)
    plan.unpack(flat, 2, torch.float32, sqnorm=sq)
    torch.cuda.synchronize()
    ref_out = O.unpack(ref, [t.shape for t in ts], np.float32, align,
                       flat_dtype=O.BF16 if flat_dt == torch.bfloat16 else O.F32)
    for o, r in zip(outs, ref_out):
        assert np.array_equal(to_np(o), r.reshape(-1))
    want = sum(float((r.astype(np.float64) ** 2).sum()) for r in ref_out)
    assert abs(sq.item() - want) <= 1e-5 * want + 1e-30
    assert L.GS_SCALE_MUL == 1


def test_empty_and_zero_sized(cuda_device):
    ts = [torch.zeros(0, device=cuda_device), torch.ones(5, device=cuda_device), torch.zeros(0, device=cuda_device)]
    plan = plan_for(ts, cuda_device, 64)
    plan.set_ptrs(1, ts)
    flat = torch.zeros(plan.flat_numel, device=cuda_device)
    plan.pack(1, torch.float32, flat, 0.5, 1)
    torch.cuda.synchronize()
    assert flat[:5].tolist() == [0.5] * 5
    empty = plan_for([], cuda_device)
    out = torch.full((1,), 3.0, device=cuda_device)
    empty.sqnorm(0, torch.float32, out)
    torch.cuda.synchronize()
    assert out.item() == 0.0


SGD_CASES = [
    dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=False, first=True),
    dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=False, first=False),
    dict(lr=0.05, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=True, first=False),
    dict(lr=0.05, momentum=0.8, dampening=0.3, weight_decay=0.0, nesterov=False, first=False),
    dict(lr=0.3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, first=False),
]


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", SGD_CASES)
@pytest.mark.parametrize("gscale", [None, 0.37])
def test_sgd_bitwise(cuda_device, gdt, case, gscale):
    sizes = RAGGED
    ps = rand_list(sizes, torch.float32, cuda_device, seed=2)
    gs = rand_list(sizes, gdt, cuda_device, seed=3, scale=0.1)
    bs = rand_list(sizes, torch.float32, cuda_device, seed=4, scale=0.01)
    ref = []
    for p, g, b in zip(ps, gs, bs):
        ref.append(O.sgd(to_np(p), to_np(g), to_np(b), case["lr"], case["momentum"], case["dampening"],
                         case["weight_decay"], case["nesterov"], False, case["first"], gscale))
    plan = plan_for(ps, cuda_device)
    plan.set_ptrs(0, ps)
    plan.set_ptrs(1, gs)
    plan.set_ptrs(2, bs)
    gsc = None if gscale is None else torch.tensor([gscale], dtype=torch.float32, device=cuda_device)
    plan.sgd(gdt, case["lr"], case["momentum"], case["dampening"], case["weight_decay"], case["nesterov"], False,
             case["first"], grad_scale=gsc)
    torch.cuda.synchronize()
    for p, b, (rp, rb) in zip(ps, bs, ref):
        assert np.array_equal(to_np(p), rp)
        if case["momentum"] != 0:
            assert np.array_equal(to_np(b), rb)


@pytest.mark.parametrize("adamw", [False, True])
@pytest.mark.parametrize("wd", [0.0, 3e-7, 1e-2])
@pytest.mark.parametrize("step", [1, 7])
def test_adam_bitwise(cuda_device, adamw, wd, step):
    sizes = RAGGED
    ps = rand_list(sizes, torch.float32, cuda_device, seed=5)
    gs = rand_list(sizes, torch.float32, cuda_device, seed=6, scale=0.1)
    ms = rand_list(sizes, torch.float32, cuda_device, seed=7, scale=0.01)
    vs = [torch.abs(v) for v in rand_list(sizes, torch.float32, cuda_device, seed=8, scale=1e-4)]
    lr, b1, b2, eps = 2e-3, 0.8, 0.999, 1e-8
    ref = [O.adam(to_np(p), to_np(g), to_np(m), to_np(v), step, lr, b1, b2, eps, wd, adamw)
           for p, g, m, v in zip(ps, gs, ms, vs)]
    plan = plan_for(ps, cuda_device)
    for s, ts in enumerate((ps, gs, ms, vs)):
        plan.set_ptrs(s, ts)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    plan.adam(torch.float32, lr, b1, b2, eps, wd, adamw, False, (lr / bc1) * -1, bc2 ** 0.5)
    torch.cuda.synchronize()
    for p, m, v, (rp, rm, rv) in zip(ps, ms, vs, ref):
        assert np.array_equal(to_np(p), rp)
        assert np.array_equal(to_np(m), rm)
        assert np.array_equal(to_np(v), rv)


def test_found_inf_skips_step(cuda_device):
    ps = rand_list([1000, 5], torch.float32, cuda_device, seed=9)
    before = [p.clone() for p in ps]
    gs = rand_list([1000, 5], torch.float32, cuda_device, seed=10)
    plan = plan_for(ps, cuda_device)
    plan.set_ptrs(0, ps)
    plan.set_ptrs(1, gs)
    plan.set_ptrs(2, [torch.zeros_like(p) for p in ps])
    found = torch.ones(1, device=cuda_device)
    plan.sgd(torch.float32, 0.1, 0.9, 0, 0, False, False, True, found_inf=found)
    torch.cuda.synchronize()
    for a, b in zip(ps, before):
        assert torch.equal(a, b)


def test_unscale_check(cuda_device):
    gs = rand_list([100, 7, 3000], torch.float32, cuda_device, seed=11)
    plan = plan_for(gs, cuda_device)
    plan.set_ptrs(0, gs)
    inv = torch.tensor([0.5], device=cuda_device)
    found = torch.zeros(1, device=cuda_device)
    ref = [to_np(g) * np.float32(0.5) for g in gs]
    plan.unscale_check(0, torch.float32, inv, found)
    torch.cuda.synchronize()
    assert found.item() == 0.0
    for g, r in zip(gs, ref):
        assert np.array_equal(to_np(g), r)
    gs[1][3] = float("inf")
    plan.unscale_check(0, torch.float32, None, found)
    torch.cuda.synchronize()
    assert found.item() == 1.0


def test_sqnorm_and_clip(cuda_device):
    from distributed_training_amd.multi_tensor import clip_coef

    gs = rand_list(RAGGED, torch.float32, cuda_device, seed=12, scale=3.0)
    plan = plan_for(gs, cuda_device)
    plan.set_ptrs(0, gs)
    buf = torch.zeros(3, device=cuda_device)
    plan.sqnorm(0, torch.float32, buf[0:1])
    clip_coef(buf[0:1], 1.0, 1e-6, buf[1:2], buf[2:3])
    torch.cuda.synchronize()
    want = O.sqnorm([to_np(g) for g in gs])
    assert abs(buf[0].item() - want) <= 1e-5 * want
    assert abs(buf[2].item() - want ** 0.5) <= 1e-5 * want ** 0.5
    assert abs(buf[1].item() - O.clip_coef(want ** 0.5, 1.0)) <= 1e-6


def test_clip_grad_norm_matches_torch(cuda_device):
    from distributed_training_amd.optim import clip_grad_norm_

    ps = [torch.nn.Parameter(torch.zeros(n, device=cuda_device)) for n in (10, 3000, 7)]
    qs = [torch.nn.Parameter(torch.zeros(n, device=cuda_device)) for n in (10, 3000, 7)]
    for p, q, g in zip(ps, qs, rand_list([10, 3000, 7], torch.float32, cuda_device, seed=13, scale=5.0)):
        p.grad = g.clone()
        q.grad = g.clone()
    n1 = clip_grad_norm_(ps, 1.0)
    n2 = torch.nn.utils.clip_grad_norm_(qs, 1.0)
    torch.cuda.synchronize()
    assert abs(n1.item() - n2.item()) <= 1e-5 * n2.item()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("case", ["clip", "no_clip", "nan", "bf16"])
def test_clip_grad_norm_two_launches(cuda_device, case):
    """The drop-in clip_grad_norm_ is two launches on one grad dtype:
    the Σg² partial sums, then the scale pass whose workgroups fold them into the
    coefficient themselves — no combine, no coefficient launch, no flag fill.  The
    published [Σg², coef, norm] follow torch's arithmetic (coef = clamp(max/(norm +
    1e-6), max=1) in fp32), the grads are g * coef bit for bit; a coefficient of 1
    leaves them untouched, a NaN norm makes them NaN (torch.clamp keeps NaN)."""
    from distributed_training_amd import _lib as L
    from distributed_training_amd import optim as OPT

    dt = torch.bfloat16 if case == "bf16" else torch.float32
    sizes = [10, 3000, 7, 70_000, 1 << 20]
    gs = rand_list(sizes, dt, cuda_device, seed=21, scale=5.0)
    if case == "nan":
        gs[1][5] = float("nan")
    ps = [torch.nn.Parameter(torch.zeros(n, device=cuda_device, dtype=dt)) for n in sizes]
    for p, g in zip(ps, gs):
        p.grad = g.clone()
    max_norm = 1e9 if case == "no_clip" else 1.0
    OPT.clip_grad_norm_(ps, max_norm)  # builds the cached plan
    plan = OPT._NORM_PLANS[tuple(sizes) + (cuda_device,)]
    for p, g in zip(ps, gs):
        p.grad.copy_(g)
    torch.cuda.synchronize()
    plan.timer_enable(8)
    norm = OPT.clip_grad_norm_(ps, max_norm)
    torch.cuda.synchronize()
    kinds = plan.timer_read_by_kind()
    plan.timer_enable(0)
    assert sorted((k, len(v)) for k, v in kinds.items()) == [(L.GS_OP_SCALE, 1), (L.GS_OP_SQNORM, 1)], kinds
    want_sq = O.sqnorm([to_np(g.float()) for g in gs])
    if case == "nan":
        assert torch.isnan(norm).item()
        assert all(torch.isnan(p.grad.float()).all().item() for p in ps)
        return
    assert abs(norm.item() - want_sq ** 0.5) <= 1e-5 * want_sq ** 0.5
    buf_norm = norm.reshape(1)
    nrm = torch.tensor([norm.item()], dtype=torch.float32)
    coef = torch.clamp(torch.tensor([max_norm], dtype=torch.float32) / (nrm + 1e-6), max=1.0)
    for p, g in zip(ps, gs):
        want = g if coef.item() == 1.0 else (g.float() * coef.item()).to(dt)
        assert torch.equal(p.grad, want)
    assert buf_norm.device == cuda_device


def test_large_sgd_property(cuda_device):
    """ResNet-152-sized flat step (60.2M params, > Infinity Cache): bit-exact vs the oracle."""
    n = 60_192_808
    g = torch.Generator(device=cuda_device).manual_seed(0)
    p = torch.randn(n, device=cuda_device, generator=g)
    gr = torch.randn(n, device=cuda_device, generator=g) * 0.01
    b = torch.randn(n, device=cuda_device, generator=g) * 0.01
    rp, rb = O.sgd(to_np(p), to_np(gr), to_np(b), 0.1, 0.9, 0.0, 1e-4, False, False, False)
    plan = plan_for([p], cuda_device)
    plan.set_ptrs(0, [p])
    plan.set_ptrs(1, [gr])
    plan.set_ptrs(2, [b])
    plan.sgd(torch.float32, 0.1, 0.9, 0.0, 1e-4, False, False, False)
    torch.cuda.synchronize()
    assert np.array_equal(to_np(p), rp)
    assert np.array_equal(to_np(b), rb)


def test_resnet50_shaped_sgd_bitwise(cuda_device):
    """The real ResNet-50 parameter list (161 tensors, 108 of them <= 16 KiB) under the
    balanced task sizing: every segment boundary / shared task lands bit-exact."""
    from distributed_training_amd.resnet import MODELS

    sizes = [p.numel() for p in MODELS["resnet50"]().parameters()]
    ps = rand_list(sizes, torch.float32, cuda_device, seed=1)
    gs = rand_list(sizes, torch.float32, cuda_device, seed=2, scale=0.01)
    bs = rand_list(sizes, torch.float32, cuda_device, seed=3, scale=0.01)
    ref = [O.sgd(to_np(p), to_np(g), to_np(b), 0.1, 0.9, 0.0, 1e-4, False, False, False)
           for p, g, b in zip(ps, gs, bs)]
    plan = plan_for(ps, cuda_device)
    assert plan.n_tasks <= 2048 and plan.task_units % 256 == 0
    plan.set_ptrs(0, ps)
    plan.set_ptrs(1, gs)
    plan.set_ptrs(2, bs)
    plan.sgd(torch.float32, 0.1, 0.9, 0.0, 1e-4, False, False, False)
    torch.cuda.synchronize()
    for (rp, rb), p, b in zip(ref, ps, bs):
        assert np.array_equal(to_np(p), rp)
        assert np.array_equal(to_np(b), rb)


def test_plan_launch_timer(cuda_device):
    n = 1 << 22
    p, g, b = (torch.randn(n, device=cuda_device) for _ in range(3))
    plan = plan_for([p], cuda_device)
    plan.set_ptrs(0, [p])
    plan.set_ptrs(1, [g])
    plan.set_ptrs(2, [b])
    assert plan.timer_read() == []  # disabled: nothing recorded
    plan.timer_enable(4)
    for _ in range(6):
        plan.sgd(torch.float32, 1e-3, 0.9, 0.0, 0.0, False, False, False)
    ms = plan.timer_read()
    assert len(ms) == 4 and all(0 < t < 100 for t in ms)  # ring keeps the last 4
    assert plan.timer_read() == []  # read clears
    from distributed_training_amd import _lib as L

    sq = torch.zeros(1, device=cuda_device)
    plan.sgd(torch.float32, 1e-3, 0.9, 0.0, 0.0, False, False, False)
    plan.sqnorm(1, torch.float32, sq)
    plan.sgd(torch.float32, 1e-3, 0.9, 0.0, 0.0, False, False, False)
    assert len(plan.timer_read(kind=L.GS_OP_SGD)) == 2  # the Σg² launch is tagged apart
    plan.timer_enable(0)
    plan.sgd(torch.float32, 1e-3, 0.9, 0.0, 0.0, False, False, False)
    assert plan.timer_read() == []


def test_fp16_outputs_round_the_fp32_value(cuda_device):
    """Every fp16 output is the round-to-nearest-even of the fp32 result, as
    torch's opmath-then-cast: pack ×s into an fp16 bucket == (x * s).half(),
    the in-place fp16 unscale == (g.float() * inv).half(), the fused update's
    fp16 param copy == the fp32 master's .half().  (LLVM folded the producing
    fma / mul into v_fma_mixlo_f16 — one rounding, straight to fp16 — which
    differs wherever the fp32 value is an fp16 tie: ~1e-4 of random inputs.)"""
    from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units

    dev = cuda_device
    n = 1 << 20
    g = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn(n, device=dev, generator=g)
    s = float(np.float32(1.0 / 3.0))
    plan = TensorListPlan([n], dev, align=64)
    plan.set_ptrs(1, [x])
    flat = torch.zeros(plan.flat_numel, dtype=torch.float16, device=dev)
    plan.pack(1, torch.float32, flat, s, 1)
    torch.cuda.synchronize()
    assert torch.equal(flat[:n], (x * s).half())

    g16 = (torch.randn(n, device=dev, generator=g) * 100).half()
    inv = torch.tensor([s], device=dev)
    want = (g16.float() * inv).half()
    p2 = TensorListPlan([n], dev)
    p2.set_ptrs(1, [g16])
    found = torch.zeros(1, device=dev)
    p2.unscale_check(1, torch.float16, inv, found)
    torch.cuda.synchronize()
    assert found.item() == 0.0 and torch.equal(g16, want)

    for kind in ("adam", "sgd"):
        up = TensorListPlan([n], dev, task_units=update_task_units(dev))
        p = torch.randn(n, device=dev, generator=g)
        gr = torch.randn(n, device=dev, generator=g) * 1e-2
        m = torch.zeros(n, device=dev)
        v = torch.zeros(n, device=dev)
        p16 = torch.zeros(n, device=dev, dtype=torch.float16)
        up.set_ptrs(0, [p])
        up.set_ptrs(1, [gr])
        up.set_ptrs(2, [m])
        if kind == "adam":
            up.set_ptrs(3, [v])
            up.set_ptrs(4, [p16])
            up.adam(torch.float32, 1e-3, 0.9, 0.999, 1e-8, 0.0, True, False, -1e-3 / 0.1, 0.001 ** 0.5,
                    lowp_dtype=torch.float16)
        else:
            up.set_ptrs(3, [p16])
            up.sgd(torch.float32, 0.1, 0.9, 0.0, 1e-4, False, False, True, lowp_dtype=torch.float16)
        torch.cuda.synchronize()
        assert torch.equal(p16, p.half()), f"{kind}: {(p16 != p.half()).sum().item()} of {n}"
