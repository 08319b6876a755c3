"""``FusedSGD.fuse_grad_norm_into(ddp)`` under AMP loss scaling, pinned to the
oracle.

DDP + FusedSGD(max_grad_norm) + GradScaler, Σg² formed inside the DDP's bucket
unpacks (on the SCALED averaged grads: the update folds s² into it, s = 1/scale)
and the non-finite check fused there too.  Every step is checked against the
oracle chain on the same averaged grads:
``O.sqnorm`` -> ``O.clip_coef(‖g‖·s)`` -> ``O.sgd(gscale = coef·s)``
(oracle/oracle.py -> gs_oracle.c, restating T:nn/utils/clip_grad.py:165-174,
T:amp/grad_scaler.py, T:optim/sgd.py:322-381):
* the published coefficient / norm within rtol 1e-5 of the oracle's (double Σ;
  the unpacks add the same squares in bucket order);
* weights and momentum buffers bit-exact given the published coefficient;
* an overflow step (an inf in ONE rank's local grad) leaves weights and momentum
  untouched and halves the scale;
* a step after an explicit ``scaler.unscale_(opt)`` must NOT fold the stale
  scaled Σg² from the unpacks (the grads changed in place after backward): the
  optimizer runs its own pass (``last_clip_source == "optimizer"``) and the
  result matches the oracle on the unscaled grads.
CPU/gloo ws=2 (host backend) and, with -m gpu, RCCL ws=1 (HIP kernels).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from tests.test_ddp_cpu import _micro, _run

MAX_NORM = 0.5
LR, MOM, WD = 0.1, 0.9, 1e-4


def _np(t):
    return t.detach().float().cpu().numpy().copy()


def _body(dev, rank, steps=6, poison_it=2):
    import distributed_training_amd as D
    from distributed_training_amd.amp import GradScaler
    from oracle import oracle as O

    torch.manual_seed(0)
    model = _micro().to(dev)
    state = {"it": -1}

    def poison(p):  # runs before DDP's hook: this rank's local grad, ahead of the pack
        if state["it"] == poison_it and rank == 0:
            p.grad.view(-1)[1] = float("inf")

    next(model.parameters()).register_post_accumulate_grad_hook(poison)
    ddp = D.DistributedDataParallel(model, bucket_cap_mb=0.05)  # several buckets: Σg² accumulated in bucket order
    opt = D.FusedSGD(ddp.parameters(), lr=LR, momentum=MOM, weight_decay=WD, max_grad_norm=MAX_NORM)
    opt.fuse_grad_norm_into(ddp)
    scaler = GradScaler(dev.type, init_scale=2.0 ** 8, growth_interval=3)
    scaler.fuse_check_into(ddp)
    params = list(model.parameters())
    g = torch.Generator(device=dev).manual_seed(10 + rank)
    sources = []
    for it in range(steps):
        state["it"] = it
        x = torch.rand(4, 3, 32, 32, device=dev, generator=g)
        y = torch.randint(0, 10, (4,), device=dev, generator=g)
        scaler.scale(nn.functional.cross_entropy(ddp(x), y)).backward()
        unscale_first = it == steps - 1  # the ADVICE r4 case
        scale = scaler.get_scale()
        if unscale_first:
            scaler.unscale_(opt)
        grads = [_np(p.grad) for p in params]
        p0 = [_np(p) for p in params]
        b0 = [None if "momentum_buffer" not in opt.state[p] else _np(opt.state[p]["momentum_buffer"])
              for p in params]
        scaler.step(opt)
        scaler.update()
        sources.append(opt.last_clip_source)
        if it == poison_it:
            assert not all(np.isfinite(gr).all() for gr in grads), "the poisoned step carries an inf"
            for p, a in zip(params, p0):
                assert np.array_equal(_np(p), a), "an overflow step changed a weight"
            for p, b in zip(params, b0):
                if b is not None:
                    assert np.array_equal(_np(opt.state[p]["momentum_buffer"]), b), "momentum moved on overflow"
            assert scaler.get_scale() == scale / 2
            opt.zero_grad()
            continue
        # the oracle chain on the averaged grads the optimizer saw
        s = np.float32(1.0) if unscale_first else np.float32(1.0) / np.float32(scale)
        sq = O.sqnorm(grads)  # double Σ of the (scaled, or already unscaled) grads
        norm_o = float(np.sqrt(sq)) * float(s)
        coef_o = O.clip_coef(norm_o, MAX_NORM) * float(s)
        pub = _np(opt._clip_buf[params[0].device][0:3])  # [Σg²·s², coef·s, ‖g‖]
        assert abs(pub[2] - norm_o) <= 1e-5 * norm_o, (it, pub, norm_o)
        assert abs(pub[1] - coef_o) <= 1e-5 * coef_o, (it, pub, coef_o)
        assert coef_o < float(s), "the clip must be active for the test to mean something"
        for i, p in enumerate(params):
            pe, be = O.sgd(p0[i], grads[i], b0[i], LR, MOM, 0.0, WD, first=b0[i] is None, gscale=float(pub[1]))
            assert np.array_equal(_np(p).reshape(-1), pe), (it, i)
            assert np.array_equal(_np(opt.state[p]["momentum_buffer"]).reshape(-1), be), (it, i)
        opt.zero_grad()
    # every backward fed the optimizer from its unpacks, except after unscale_
    assert sources[-1] == "optimizer", sources
    assert all(src == "ddp_unpack" for i, src in enumerate(sources[:-1]) if i != poison_it), sources
    assert scaler.fused_checks == steps - 1  # the unscale_ step ran its own check
    return [_np(p) for p in params]


def _cpu_case(rank, ws):
    import torch.distributed as dist

    w = _body(torch.device("cpu"), rank)
    allw = [None] * ws
    dist.all_gather_object(allw, np.concatenate([a.reshape(-1) for a in w]))
    assert all(np.array_equal(allw[0], a) for a in allw[1:])


def test_fused_norm_amp_cpu_ws2():
    _run(_cpu_case, 2)


def test_unscale_invalidates_fused_norm_cpu():
    """Unit level, one process: the version counters a DDP records at finalize
    move when GradScaler.unscale_ or libgsync's clip_grad_norm_ rewrite grads
    in place (their kernels bump them as torch's in-place ops do)."""
    import distributed_training_amd as D
    from distributed_training_amd.amp import GradScaler

    ps = [torch.nn.Parameter(torch.randn(5)) for _ in range(3)]
    for p in ps:
        p.grad = torch.randn(5)
    v0 = [p.grad._version for p in ps]
    opt = torch.optim.SGD(ps, lr=0.1)
    sc = GradScaler("cpu", init_scale=4.0)
    sc._lazy_init(torch.device("cpu"))
    sc.unscale_(opt)
    assert all(p.grad._version > v for p, v in zip(ps, v0))
    v1 = [p.grad._version for p in ps]
    D.clip_grad_norm_(ps, 1e-3)
    assert all(p.grad._version > v for p, v in zip(ps, v1))


def _gpu_worker(rank, ws, port, errq):
    try:
        from tests._dist_util import init_pg

        init_pg("nccl", rank, ws, port)
        torch.cuda.set_device(0)
        _body(torch.device("cuda", 0), rank)
        import torch.distributed as dist

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
def test_fused_norm_amp_gpu_ws1(cuda_device):
    import torch.multiprocessing as mp

    from tests._dist_util import free_port

    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    p = ctx.Process(target=_gpu_worker, args=(0, 1, free_port(), errq))
    p.start()
    p.join(180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert p.exitcode == 0, p.exitcode
