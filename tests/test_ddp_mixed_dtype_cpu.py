"""Parameters of several floating dtypes: torch's Reducer buckets per dtype
(compute_bucket_assignment_by_size keys on (dtype, device),
T:include/torch/csrc/distributed/c10d/reducer.hpp:590-595); so does the
libgsync bucketer (per-bucket grad / bucket dtypes).  CPU / gloo, world size 2:
averaged grads bit-identical to torch's DDP on the same model and data, and
the bucket layout (per dtype, rebuilt in ready order) identical to torch's."""
import torch
import torch.distributed as dist
import torch.nn as nn

from tests.test_ddp_cpu import _micro, _run


class Mixed(nn.Module):
    """fp32 ResNet body + a bf16 projection head + an fp16 bias term."""

    def __init__(self):
        super().__init__()
        self.body = _micro()
        self.head = nn.Linear(10, 7).to(torch.bfloat16)
        self.bias16 = nn.Parameter(torch.zeros(7, dtype=torch.float16))

    def forward(self, x):
        h = self.head(self.body(x).to(torch.bfloat16)).float()
        return h + self.bias16.float()


def _mixed(rank, ws):
    import distributed_training_amd as D

    out = {}
    for impl in ("torch", "libgsync"):
        torch.manual_seed(0)
        model = Mixed()
        ddp = (torch.nn.parallel.DistributedDataParallel(model) if impl == "torch"
               else D.DistributedDataParallel(model))
        g = torch.Generator().manual_seed(1234 + rank)
        grads = []
        for it in range(3):  # iteration 0: one bucket per dtype; then rebuilt in ready order
            x = torch.rand(4, 3, 32, 32, generator=g)
            y = torch.randint(0, 7, (4,), generator=g)
            for p in model.parameters():
                p.grad = None
            nn.functional.cross_entropy(ddp(x), y).backward()
            grads.append([p.grad.clone() for p in model.parameters()])
        out[impl] = (grads, ddp._get_ddp_logging_data()["rebuilt_bucket_sizes"], ddp)
    tg, tsizes, _ = out["torch"]
    mg, msizes, mddp = out["libgsync"]
    for it, (a, b) in enumerate(zip(tg, mg)):
        for i, (x, y) in enumerate(zip(a, b)):
            assert x.dtype == y.dtype and torch.equal(x, y), f"iter {it} param {i} ({x.dtype})"
    tsizes = [int(v) for v in str(tsizes).split(",")] if isinstance(tsizes, str) else list(tsizes)
    assert sorted(tsizes) == sorted(msizes), (tsizes, msizes)
    assert set(mddp._bucketer.bucket_dtypes) == {torch.float32, torch.bfloat16, torch.float16}
    for b, dt in zip(mddp._bucketer.buffers, mddp._bucketer.bucket_dtypes):
        assert b.dtype == dt


def test_mixed_dtype_buckets_match_torch_ddp():
    _run(_mixed, 2)
