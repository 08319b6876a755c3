"""Maximum sizes: one tensor of 2^31 + 1029 fp32 elements (8.6 GB — beyond
32-bit element indexing) between two small ones, on the MI355X's 288 GB.

Every grad-sync op on a plan that holds it — pack ×0.5 into a 64-element-
aligned fp32 bucket, unpack back, Σg², the fused SGD first step, pack into a
bf16 bucket — against torch on the same device: bitwise where the arithmetic
is exact or elementwise-identical, Σg² within fp32 summation error.  Guards
the 64-bit offsets of the chunk map (virtual offsets, chunk indices, the
per-lane search) and the tails of the last chunk."""
import pytest
import torch

pytestmark = pytest.mark.gpu

BIG = (1 << 31) + 1029


def test_plan_ops_beyond_2g_elements(cuda_device):
    from distributed_training_amd.multi_tensor import TensorListPlan, update_task_units

    dev = cuda_device
    free, _ = torch.cuda.mem_get_info(dev)
    if free < 80 * 2**30:
        pytest.skip(f"needs ~80 GB free device memory ({free / 2**30:.0f} GB free)")
    g = torch.Generator(device=dev).manual_seed(21)
    small_a = torch.randn(5, device=dev, generator=g)
    small_b = torch.randn(3, device=dev, generator=g)
    big = torch.empty(BIG, device=dev)
    big.uniform_(-1.0, 1.0, generator=g)
    ts = [small_a, big, small_b]
    plan = TensorListPlan([t.numel() for t in ts], dev, align=64)
    plan.set_ptrs(1, ts)
    offs = [0, 64, 64 + (BIG + 63) // 64 * 64]
    assert plan.flat_numel == offs[2] + 64
    flat = torch.zeros(plan.flat_numel, device=dev)
    plan.pack(1, torch.float32, flat, 0.5, 1)
    torch.cuda.synchronize()
    for t, o in zip(ts, offs):
        assert torch.equal(flat[o:o + t.numel()], t * 0.5)
    assert int(torch.count_nonzero(flat[offs[1] + BIG:offs[2]])) == 0  # padding stays zero

    # unpack into fresh tensors (slot 2), with the fused Σg²
    outs = [torch.empty_like(t) for t in ts]
    plan.set_ptrs(2, outs)
    sq = torch.zeros(1, device=dev)
    plan.unpack(flat, 2, torch.float32, sqnorm=sq)
    torch.cuda.synchronize()
    for t, o in zip(ts, outs):
        assert torch.equal(o, t * 0.5)
    del outs
    want = sum(float(torch.sum((t.double() * 0.5) ** 2)) for t in (small_a, small_b))
    for k in range(0, BIG, 1 << 28):  # fp64 reference in slices (no 17 GB temporary)
        want += float(torch.sum((big[k:k + (1 << 28)].double() * 0.5) ** 2))
    assert abs(sq.item() - want) <= 1e-5 * want
    sq2 = torch.zeros(1, device=dev)
    plan.sqnorm(1, torch.float32, sq2)
    torch.cuda.synchronize()
    assert abs(sq2.item() - 4.0 * want) <= 1e-5 * 4.0 * want

    # pack into a bf16 bucket: the cast of x·0.5 (exact in fp32) is torch's RNE
    flat16 = torch.zeros(plan.flat_numel, device=dev, dtype=torch.bfloat16)
    plan.pack(1, torch.float32, flat16, 0.5, 1)
    torch.cuda.synchronize()
    for t, o in zip(ts, offs):
        assert torch.equal(flat16[o:o + t.numel()], (t * 0.5).bfloat16())
    del flat, flat16

    # the fused SGD first step (buf = g; p -= lr·g, no momentum history) on an update plan
    up = TensorListPlan([t.numel() for t in ts], dev, task_units=update_task_units(dev))
    ps = [t.clone() for t in ts]
    bufs = [torch.empty_like(t) for t in ts]
    grads = [torch.full_like(t, 0.25) for t in ts]
    up.set_ptrs(0, ps)
    up.set_ptrs(1, grads)
    up.set_ptrs(2, bufs)
    up.sgd(torch.float32, 0.5, 0.9, 0.0, 0.0, False, False, True)
    torch.cuda.synchronize()
    for t, p, b in zip(ts, ps, bufs):
        assert torch.equal(b, torch.full_like(t, 0.25))
        assert torch.equal(p, t - 0.125)  # fmaf(-0.5, 0.25, x): one rounding of x - 0.125, as torch
