"""Grad-norm clipping folded into the fused update, on the
GPU: FusedSGD / FusedAdam(max_grad_norm=c) — Σg² (chunk kernel + combine),
the device clip coefficient min(1, c/(‖g‖+1e-6)) and the update reading it —
against torch's own `clip_grad_norm_(c)` + `torch.optim.SGD` / `Adam` on the
same inputs, over three steps with the clip active (‖g‖ ≫ c) and inactive.

Tolerances: SGD rtol 1e-5 / atol 1e-7; Adam lr·1e-3 outside
the |ĝ| < 1e3·eps exclusion (as tests/test_example_cpu.py).
The coefficient itself may differ in the last bits (torch: Σ of per-tensor
norms, here one fp32 Σg² in a fixed order), hence tolerances, not bits."""
import pytest
import torch

import distributed_training_amd as D

pytestmark = pytest.mark.gpu

SHAPES = [(64, 3, 7, 7), (64,), (1000, 2048), (1000,), (5,), (33, 17), (256, 256, 3, 3)]


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw"])
@pytest.mark.parametrize("gscale", [3.0, 1e-4])  # clip active / inactive at max_norm 1
def test_fused_update_with_max_grad_norm_matches_torch(cuda_device, kind, gscale):
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(3)
    p0 = [torch.randn(s, device=dev, generator=g) for s in SHAPES]
    mine = [p.clone().requires_grad_() for p in p0]
    ref = [p.clone().requires_grad_() for p in p0]
    if kind == "sgd":
        lr = 0.1
        o1 = D.FusedSGD(mine, lr=lr, momentum=0.9, weight_decay=1e-4, max_grad_norm=1.0)
        o2 = torch.optim.SGD(ref, lr=lr, momentum=0.9, weight_decay=1e-4, foreach=False)
    else:
        lr = 1e-3
        cls1 = D.FusedAdamW if kind == "adamw" else D.FusedAdam
        cls2 = torch.optim.AdamW if kind == "adamw" else torch.optim.Adam
        o1 = cls1(mine, lr=lr, weight_decay=1e-2, max_grad_norm=1.0)
        o2 = cls2(ref, lr=lr, weight_decay=1e-2, foreach=False)
    for it in range(3):
        grads = [torch.randn(s, device=dev, generator=g) * gscale for s in SHAPES]
        for a, b, gr in zip(mine, ref, grads):
            a.grad = gr.clone()
            b.grad = gr.clone()
        o1.step()
        total = torch.nn.utils.clip_grad_norm_(ref, 1.0)
        o2.step()
        torch.cuda.synchronize()
        assert o1.last_grad_norm is not None
        torch.testing.assert_close(o1.last_grad_norm.reshape(()), total.reshape(()), rtol=1e-5, atol=0)
        for i, (a, b) in enumerate(zip(mine, ref)):
            if kind == "sgd":
                torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-7,
                                           msg=lambda m: f"it {it} tensor {i}: {m}")
            else:
                # SURVEY §8c's Adam bound, with its exclusion: where the update's
                # input ĝ (clipped grad + wd·p) is within ~eps of 0, lr·ĝ/(|ĝ|+eps)
                # turns a last-bit difference of the coefficient into up to ~lr —
                # at most 0.01 % of elements beyond (it+1)·lr·1e-3, none beyond 0.1·lr
                d = (a.detach() - b.detach()).abs()
                frac = (d > (it + 1) * lr * 1e-3).float().mean().item()
                assert frac <= 1e-4, f"it {it} tensor {i}: {frac:.2e} of elements beyond (it+1)*lr*1e-3"
                assert d.max().item() <= 0.1 * lr, f"it {it} tensor {i}: max|Δ| {d.max().item()}"
