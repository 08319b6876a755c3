"""Known-answer test of the gradient average (torch's ``_test_ddp_hook_parity``
pattern, T:testing/_internal/distributed/distributed_test.py:5072-5133: with
input = rank, the grad equals the mean of ranks), CPU / gloo at world sizes 2,
3 and 4, through the default path, torch's ``allreduce_hook`` and
``bf16_compress_hook``, and several bucket layouts.

Rank r feeds a constant batch x = r + 1 into bias-free Linear layers with
all-ones weights and sums the output, so every weight-grad element is
4·(r + 1)·(fan-in chain) — the averaged grad is known in closed form:
mean_r 4(r + 1) = 2(ws + 1) for the first layer.  Exact at ws = 2 and 4
(1/ws is a power of two and every term is an integer multiple of it); at
ws = 3 within SURVEY.md §8c's 4(n−1)·2⁻²⁴·Σ_r|g_r|/n; bf16 buckets within
2⁻⁷·max|g|."""
import pytest
import torch
import torch.nn as nn

from tests.test_ddp_cpu import _run


class Chain(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(8, 16, bias=False)
        self.b = nn.Linear(16, 300, bias=False)  # a second bucket at a small cap
        for m in (self.a, self.b):
            nn.init.ones_(m.weight)

    def forward(self, x):
        return self.b(self.a(x))


def _known(rank, ws, hook, cap_mb):
    import distributed_training_amd as D
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks as H

    model = Chain()
    ddp = D.DistributedDataParallel(model, bucket_cap_mb=cap_mb)
    if hook == "allreduce":
        ddp.register_comm_hook(None, H.allreduce_hook)
    elif hook == "bf16":
        ddp.register_comm_hook(None, H.bf16_compress_hook)
    for it in range(2):  # before and after the bucket rebuild
        x = torch.full((4, 8), float(rank + 1))
        ddp(x).sum().backward()
        # d/dA of sum(B A x) = (Bᵀ 1) xᵀ summed over the batch: 300 · 4(r+1) per element;
        # d/dB = 1 (A x)ᵀ: 8 · 4(r+1) per element (A = ones, x = r+1)
        want_a = 300.0 * 2.0 * (ws + 1)
        want_b = 8.0 * 2.0 * (ws + 1)
        for p, want, fan in ((model.a.weight, want_a, 300.0), (model.b.weight, want_b, 8.0)):
            g = p.grad
            if hook == "bf16":
                tol = 2.0 ** -7 * fan * 4 * ws
            elif ws in (2, 4):
                tol = 0.0
            else:
                tol = 4 * (ws - 1) * 2.0 ** -24 * sum(fan * 4 * (r + 1) for r in range(ws)) / ws
            err = float((g - want).abs().max())
            assert err <= tol, (it, hook, ws, err, tol)
        for p in model.parameters():
            p.grad = None


@pytest.mark.parametrize("ws", [2, 3, 4])
@pytest.mark.parametrize("hook,cap_mb", [(None, None), (None, 0.001), ("allreduce", 0.001), ("bf16", None)])
def test_grad_is_the_mean_of_ranks(ws, hook, cap_mb):
    _run(_known, ws, hook, cap_mb)
