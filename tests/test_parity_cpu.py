"""The cross-rank self-check bench.py runs after its timed region
(distributed_training_amd/parity.py), the xGMI bucket policy and the
last-bucket split — on CPU tensors over gloo (world sizes 1-3).

* a correct step passes: averaged grads == Σ_r g_r·float(1/ws) bitwise at
  ws ≤ 2 and within SURVEY.md §8c's bound at ws = 3; post-step weights and
  BN buffers identical on every rank (DDP and ZeRO-2);
* a broken step is caught: one rank's gradient perturbed after the sync makes
  that rank's averaged-grad check and every rank's weight check fail;
* bucket_policy="xgmi" / last_bucket_cap_mb change only the bucket
  membership, never an element's sum: grads bit-identical to the torch policy.
"""
import pytest
import torch
import torch.distributed as dist

from tests.test_ddp_cpu import _micro, _run


def _step_fn(ddp, x, y):
    def fwd_bwd():
        torch.nn.functional.cross_entropy(ddp(x), y).backward()

    return fwd_bwd


def _ddp_parity(rank, ws, perturb):
    import distributed_training_amd as D
    from distributed_training_amd import parity as PC

    torch.manual_seed(0)
    model = _micro()
    ddp = D.DistributedDataParallel(model)
    opt = D.FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.rand(4, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (4,), generator=g)
    fb = _step_fn(ddp, x, y)
    for _ in range(2):  # bucket rebuild happens on the second iteration
        fb()
        opt.step()
        opt.zero_grad(set_to_none=True)
    if perturb and rank == ws - 1:
        inner = fb

        def fb():
            inner()
            with torch.no_grad():
                ddp._params[0].grad.add_(1e-3)  # a broken sync on one rank

    res = PC.ddp_parity_step(ddp, opt, fb)
    assert res["collective"] == "gloo" and res["world"] == ws
    grads = res["averaged_grads"]
    if not perturb:
        assert res["ok"], res
        assert grads["bitwise_equal"] == (ws <= 2) or grads["bitwise_equal"], res
        if ws <= 2:
            assert grads["bitwise_equal"], res
        assert res["weights_identical"] and res["buffers_identical"], res
    else:
        assert not res["weights_identical"], res
        assert not res["ok"], res
        if rank == ws - 1:
            assert not grads["ok"] and grads["max_abs_err"] >= 9e-4, res


@pytest.mark.parametrize("ws", [1, 2, 3])
def test_ddp_parity_step_passes(ws):
    _run(_ddp_parity, ws, False)


def test_ddp_parity_step_catches_a_broken_sync():
    _run(_ddp_parity, 2, True)


def _zero_parity(rank, ws, channels_last=False):
    from distributed_training_amd import parity as PC
    from distributed_training_amd.zero import ZeroDataParallel

    torch.manual_seed(0)
    model = _micro()
    mf = torch.channels_last if channels_last else torch.contiguous_format
    model = model.to(memory_format=mf)  # bench.py's layout: the bucket holds grads in memory order
    zero = ZeroDataParallel(model, stage=2, optimizer="adamw", lr=1e-3, weight_decay=3e-7, gradient_clipping=1.0)
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.rand(4, 3, 32, 32, generator=g).to(memory_format=mf)
    y = torch.randint(0, 10, (4,), generator=g)

    def fb():
        torch.nn.functional.cross_entropy(model(x), y).backward()

    zero.prepare_backward()
    fb()
    zero.step()
    res = PC.zero_parity_step(zero, fb)
    assert res["ok"] and res["weights_identical"], res
    if ws <= 2:
        assert res["averaged_grads"]["bitwise_equal"], res


@pytest.mark.parametrize("channels_last", [False, True])
@pytest.mark.parametrize("ws", [2, 3])
def test_zero_parity_step_passes(ws, channels_last):
    _run(_zero_parity, ws, channels_last)


def test_split_last_bucket():
    from distributed_training_amd.ddp import split_last_bucket

    nbytes = [100, 400, 50, 30, 20, 700]
    # ready order: bucket 0 = [5], bucket 1 = [4, 3, 2, 1, 0] (last ready = 0)
    out = split_last_bucket([[5], [4, 3, 2, 1, 0]], nbytes, 160)
    assert out == [[5], [4, 3, 2, 1], [0]]  # 100 fits, +400 would not
    out = split_last_bucket([[5], [4, 3, 2]], nbytes, 1000)
    assert out == [[5], [4, 3, 2]]  # already under the cap: unchanged (no empty bucket)
    out = split_last_bucket([[1, 0]], nbytes, 10)
    assert out == [[1], [0]]  # a tensor above the cap still forms the last bucket alone


def test_xgmi_bucket_caps_formula():
    from distributed_training_amd.ddp import xgmi_bucket_caps

    alpha, bus, n = 20e-6, 500e9, 8
    f = 2 * (n - 1) / n
    cal = xgmi_bucket_caps(lambda b: alpha + b * f / bus, n)
    assert abs(cal["alpha_us"] - 20.0) < 1e-6 and abs(cal["bus_GBps"] - 500.0) < 1e-6
    want = 0.85 / 0.15 * alpha * bus / f
    assert abs(cal["bucket_cap_bytes"] - int(want)) <= 1
    assert abs(cal["last_bucket_cap_bytes"] - int(alpha * bus / f)) <= 1
    for pt in cal["points"]:
        assert pt["bus_GBps"] < 500.0
    # a latency-free link: caps clamp to their floors
    cal = xgmi_bucket_caps(lambda b: b * f / bus, n)
    assert cal["bucket_cap_bytes"] == 4 * 2**20 and cal["last_bucket_cap_bytes"] == 256 * 1024


def _policy_grads(rank, ws):
    import distributed_training_amd as D

    grads = {}
    for policy, last in (("torch", None), ("xgmi", None), ("torch", 0.0001)):
        torch.manual_seed(0)
        model = _micro()
        ddp = D.DistributedDataParallel(model, bucket_policy=policy, last_bucket_cap_mb=last)
        g = torch.Generator().manual_seed(1234 + rank)
        x = torch.rand(4, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (4,), generator=g)
        for _ in range(3):
            for p in model.parameters():
                p.grad = None
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
        grads[(policy, last)] = [p.grad.clone() for p in model.parameters()]
        log = ddp._get_ddp_logging_data()
        assert log["bucket_policy"] == policy
        if policy == "xgmi":
            cal = log["xgmi_calibration"]
            assert cal is not None and len(cal["points"]) == 4 and cal["bucket_cap_bytes"] >= 4 * 2**20
        if last is not None:
            last_bucket = ddp.bucket_indices()[-1]
            assert sum(ddp._params[i].numel() * 4 for i in last_bucket) <= 105 or len(last_bucket) == 1
    base = grads[("torch", None)]
    for k, gs in grads.items():
        for a, b in zip(base, gs):
            assert torch.equal(a, b), k


def test_bucket_policies_change_no_sum():
    _run(_policy_grads, 2)


def _debug_checksums(rank, ws, corrupt):
    import os

    os.environ["GSYNC_DEBUG"] = "1"
    import distributed_training_amd as D

    torch.manual_seed(0)
    model = _micro()
    ddp = D.DistributedDataParallel(model)
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.rand(4, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (4,), generator=g)
    for it in range(3):  # iteration 0: one bucket; then the rebuilt layout
        if it == 2 and corrupt and rank == 1:
            inner = ddp._launch_external

            def bad(bucket_ids, inner=inner):
                for bi in bucket_ids:
                    if corrupt == "before":
                        ddp._bucketer.buffers[bi].add_(1.0)  # a wrong contribution enters the sum
                inner(bucket_ids)
                if corrupt == "after":
                    for bi in bucket_ids:
                        ddp._pending[bi][1].wait()
                        ddp._bucketer.buffers[bi].add_(1.0)  # one rank's result diverges
            ddp._launch_external = bad
        for p in model.parameters():
            p.grad = None
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        sums = ddp.bucket_checksums()
        assert len(sums) == len(ddp.bucket_indices())
        if it < 2 or not corrupt:
            out = ddp.verify_bucket_checksums()
            assert all(abs(t - p) <= tol for t, p, tol in out)
        else:
            with pytest.raises(RuntimeError, match="bucket"):
                ddp.verify_bucket_checksums()


@pytest.mark.parametrize("corrupt", [None, "before", "after"])
def test_debug_bucket_checksums(corrupt):
    _run(_debug_checksums, 2, corrupt)
