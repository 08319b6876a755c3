"""The DDP drop-in on CPU tensors over gloo (world_size 2 and 4): the
configuration-1 plumbing path (BASELINE.json configs[0]), compared with the
golden fixtures of the reference's own DDP train step and with torch's DDP
run side by side."""
import gc
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from tests._dist_util import free_port, init_pg

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _micro():
    from distributed_training_amd.resnet import ResNet, BasicBlock

    return ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, width=4)


def _run(fn, ws, *args):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_wrap, args=(fn, r, ws, port, errq) + args) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _wrap(fn, rank, ws, port, errq, *args):
    import faulthandler

    faulthandler.enable(all_threads=True)
    if os.environ.get("GSYNC_TERMINATE_TRACE"):  # diagnosis: native backtrace of an exit-time abort
        import ctypes

        ctypes.CDLL(os.environ["GSYNC_TERMINATE_TRACE"])
    try:
        init_pg("gloo", rank, ws, port)
        torch.set_num_threads(max(1, 8 // ws))  # as make_golden.py: CPU conv sums depend on it
        fn(rank, ws, *args)
        # Free the test's objects (a DDP in a reference cycle holds the process group)
        # while the interpreter is whole: a gloo worker thread that drops the last
        # reference to a Python-owned tensor during interpreter finalization cannot
        # take the GIL and ends in std::terminate (ProcessGroupGloo::runLoop ->
        # TensorImpl::decref_pyobject -> pthread_exit under a noexcept frame; native
        # backtrace with GSYNC_TERMINATE_TRACE)
        gc.collect()
        dist.barrier()  # no rank tears gloo down while a peer is still talking
        dist.destroy_process_group()
        gc.collect()
    except BaseException as e:
        import traceback

        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def _golden_run(rank, ws, name, use_torch_opt, hook):
    import distributed_training_amd as D

    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    n = len(z["param_names"])
    torch.manual_seed(500 + rank)
    model = _micro()
    if rank == 0:
        with torch.no_grad():
            for i, p in enumerate(model.parameters()):
                p.copy_(torch.from_numpy(z[f"init/{i}"]))
    ddp = D.DistributedDataParallel(model)
    if hook:
        from torch.distributed.algorithms.ddp_comm_hooks.default_hooks import bf16_compress_hook

        ddp.register_comm_hook(None, bf16_compress_hook)  # torch's own hook on our GradBucket
    for i, p in enumerate(model.parameters()):  # init broadcast from rank 0
        assert np.array_equal(p.detach().numpy(), z[f"init/{i}"])
    adam = "adam" in name
    if use_torch_opt:
        opt = (torch.optim.Adam(ddp.parameters(), lr=1e-3 * ws, foreach=False) if adam else
               torch.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, foreach=False))
    else:
        opt = (D.FusedAdam(ddp.parameters(), lr=1e-3 * ws) if adam else
               D.FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4))
    crit = nn.CrossEntropyLoss()
    model.train()
    for s in range(int(z["steps"])):
        x = torch.from_numpy(z[f"x/{rank}/{s}"])
        y = torch.from_numpy(z[f"y/{rank}/{s}"])
        crit(ddp(x), y).backward()
        for i, p in enumerate(model.parameters()):
            ref = z[f"grad/{s}/{i}"]
            if ws <= 2:
                assert np.array_equal(p.grad.numpy(), ref), f"step {s} grad {i}"
            else:
                np.testing.assert_allclose(p.grad.numpy(), ref, rtol=1e-5, atol=1e-7, err_msg=f"step {s} grad {i}")
        opt.step()
        opt.zero_grad()
        for i, p in enumerate(model.parameters()):
            ref = z[f"param/{s}/{i}"]
            if use_torch_opt and ws <= 2:
                assert np.array_equal(p.detach().numpy(), ref), f"step {s} param {i}"
            elif adam:
                assert np.max(np.abs(p.detach().numpy() - ref)) <= 1e-3 * ws * 1e-3
            else:
                np.testing.assert_allclose(p.detach().numpy(), ref, rtol=1e-5, atol=1e-6, err_msg=f"step {s} param {i}")
            if not use_torch_opt:
                # teacher forcing: continue from the reference weights so the next
                # step's averaged grads stay comparable bit for bit
                with torch.no_grad():
                    p.copy_(torch.from_numpy(ref))
    if not hook:
        for i, b in enumerate(model.buffers()):
            assert np.array_equal(b.numpy(), z[f"buf/{rank}/{i}"]), f"buffer {i}"
    assert ddp._get_ddp_logging_data()["has_rebuilt_buckets"] == 1
    assert n == len(list(model.parameters()))


@pytest.mark.parametrize("name,torch_opt", [("ddp_sgd_ws2.npz", True), ("ddp_sgd_ws2.npz", False),
                                            ("ddp_adam_ws2.npz", True), ("ddp_adam_ws2.npz", False)])
def test_golden_ws2(name, torch_opt):
    _run(_golden_run, 2, name, torch_opt, False)


def test_golden_ws4():
    _run(_golden_run, 4, "ddp_sgd_ws4.npz", False, False)


def test_golden_bf16_compress_hook_ws2():
    _run(_golden_run, 2, "ddp_bf16hook_ws2.npz", True, True)


def _side_by_side(rank, ws, mode):
    """Our DDP and torch's DDP on identical replicas, same batches."""
    import distributed_training_amd as D
    from torch.nn.parallel import DistributedDataParallel as TDDP

    class WithUnused(nn.Module):
        def __init__(self):
            super().__init__()
            self.body = _micro()
            self.unused = nn.Linear(3, 3)

        def forward(self, x):
            return self.body(x)

    torch.manual_seed(0)
    make = WithUnused if mode == "find_unused" else _micro
    m1, m2 = make(), make()
    m2.load_state_dict(m1.state_dict())
    kw = {}
    if mode == "find_unused":
        kw["find_unused_parameters"] = True
    if mode == "view":
        kw["gradient_as_bucket_view"] = True
    if mode == "small_buckets":
        kw["bucket_cap_mb"] = 0.01
    a = D.DistributedDataParallel(m1, **kw)
    b = TDDP(m2, **kw)
    g = torch.Generator().manual_seed(77 + rank)
    for it in range(3):
        xs = [torch.rand(3, 3, 32, 32, generator=g) for _ in range(3)]
        ys = [torch.randint(0, 10, (3,), generator=g) for _ in range(3)]
        for model in (a, b):
            if mode == "no_sync":
                with model.no_sync():
                    for x, y in zip(xs[:2], ys[:2]):
                        nn.functional.cross_entropy(model(x), y).backward()
            nn.functional.cross_entropy(model(xs[2]), ys[2]).backward()
        for (na, pa), (nb, pb) in zip(a.module.named_parameters(), b.module.named_parameters()):
            assert (pa.grad is None) == (pb.grad is None), na
            if pa.grad is not None:
                if ws <= 2:
                    assert torch.equal(pa.grad, pb.grad), f"{mode} it {it} {na}"
                else:  # gloo's ring sums in a chunk order that depends on the bucket layout
                    torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-5, atol=1e-6,
                                               msg=f"{mode} it {it} {na}")
        if mode == "view":
            for p in a.module.parameters():
                p.grad.zero_()
            b.module.zero_grad(set_to_none=False)
        else:
            a.module.zero_grad()
            b.module.zero_grad()
    if mode == "small_buckets":
        assert len(a.bucket_indices()) > 3


@pytest.mark.parametrize("mode", ["no_sync", "view", "small_buckets", "find_unused"])
def test_side_by_side_with_torch_ddp(mode):
    _run(_side_by_side, 2, mode)


def test_side_by_side_ws4_many_buckets_rebuild():
    """4 ranks, more than 3 buckets, the rebuild after the first iteration and
    the rank-0 layout broadcast (Reducer::sync_bucket_indices): the step-1 code
    of the 4-rank rehearsal against torch's DDP."""
    _run(_side_by_side, 4, "small_buckets")


def _ignored(rank, ws):
    """_set_params_and_buffers_to_ignore_for_model: the listed parameter keeps its
    local grad and its own init, the listed buffer is not broadcast — as torch."""
    import distributed_training_amd as D
    from torch.nn.parallel import DistributedDataParallel as TDDP

    torch.manual_seed(1 + rank)  # rank-dependent init: broadcast (or not) shows
    m1 = _micro()
    m2 = _micro()
    m2.load_state_dict(m1.state_dict())
    ignore = ["fc.weight", "bn1.running_mean"]
    for m in (m1, m2):
        D.DistributedDataParallel._set_params_and_buffers_to_ignore_for_model(m, ignore)
    a = D.DistributedDataParallel(m1, broadcast_buffers=False)
    b = TDDP(m2, broadcast_buffers=False)
    assert "fc.weight" not in a._param_names and len(a._params) == len(b._module_parameters)
    for (n, x), y in zip(m1.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(x, y), n  # the same init broadcast (or kept) as torch
    g = torch.Generator().manual_seed(9 + rank)
    for it in range(2):
        x = torch.rand(3, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (3,), generator=g)
        for model in (a, b):
            nn.functional.cross_entropy(model(x), y).backward()
        for (n, pa), pb in zip(m1.named_parameters(), m2.parameters()):
            assert torch.equal(pa.grad, pb.grad), f"it {it} {n}"
        m1.zero_grad()
        m2.zero_grad()


def test_params_and_buffers_to_ignore_match_torch():
    _run(_ignored, 2)


def _buffer_hook(rank, ws, where):
    """_register_buffer_comm_hook (T:nn/parallel/distributed.py:1909-1951): a hook
    that sums every buffer across ranks with async all-reduces replaces the
    rank-0 broadcast, before the forward (waiting itself) or after it
    (returning the futures, awaited by the end of backward).  Buffers and grads equal torch's
    DDP with the same hook, torch's own enum passed to both."""
    import distributed_training_amd as D
    from torch.nn.parallel import DistributedDataParallel as TDDP
    from torch.nn.parallel.distributed import _BufferCommHookLocation as Loc

    torch.manual_seed(3)
    m1 = _micro()
    m2 = _micro()
    m2.load_state_dict(m1.state_dict())
    a = D.DistributedDataParallel(m1)
    b = TDDP(m2)
    calls = {"a": [], "b": []}

    def hook(state, named):
        calls[state].append(sorted(named))
        futs = [dist.all_reduce(t, async_op=True).get_future() for t in named.values()]
        if where == "PRE_FORWARD":  # the forward is about to use them (torch's docstring: sync yourself)
            torch.futures.wait_all(futs)
            return None
        return futs

    a._register_buffer_comm_hook("a", hook, getattr(Loc, where))
    b._register_buffer_comm_hook("b", hook, getattr(Loc, where))
    assert sorted(a.named_module_buffers) == sorted(n for n, _ in m1.named_buffers())
    g = torch.Generator().manual_seed(20 + rank)
    for it in range(3):
        x = torch.rand(3, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (3,), generator=g)
        for model in (a, b):
            nn.functional.cross_entropy(model(x), y).backward()
        for (n, pa), pb in zip(m1.named_parameters(), m2.parameters()):
            assert torch.equal(pa.grad, pb.grad), f"{where} it {it} {n}"
        for (n, x1), x2 in zip(m1.named_buffers(), m2.buffers()):
            assert torch.equal(x1, x2), f"{where} it {it} {n}"
        m1.zero_grad()
        m2.zero_grad()
    assert calls["a"] == calls["b"] and len(calls["a"]) == 3
    # the hook replaces the broadcast: ranks saw different batches, yet after a
    # post-forward hook (summed after the last update) the buffers agree
    mine = torch.cat([t.float().reshape(-1) for t in m1.buffers()])
    both = [torch.empty_like(mine) for _ in range(ws)]
    dist.all_gather(both, mine)
    assert torch.equal(both[0], both[1]) == (where == "POST_FORWARD")


@pytest.mark.parametrize("where", ["PRE_FORWARD", "POST_FORWARD"])
def test_buffer_comm_hook_matches_torch(where):
    _run(_buffer_hook, 2, where)


def _join_buffer_hook(rank, ws, where):
    """ddp.join() with uneven inputs and a buffer comm hook (the joined
    ranks' shadow of a forward must issue the training ranks' collectives in the
    same order; a POST_FORWARD hook used to leave them mismatched).  Rank r runs
    2 + 2r batches; the run completes, the hook runs once per iteration of the
    longest rank on every rank, and the final model is the same on every rank."""
    import distributed_training_amd as D
    from torch.nn.parallel.distributed import _BufferCommHookLocation as Loc

    torch.manual_seed(0)
    m = _micro()
    a = D.DistributedDataParallel(m, bucket_cap_mb=0.01)
    calls = []

    def hook(state, named):
        calls.append(len(named))
        # in place, outside autograd's version counter (BN saved its stats for backward)
        futs = [dist.all_reduce(t, async_op=True).get_future() for t in named.values() if t.is_floating_point()]
        if where == "PRE_FORWARD":
            torch.futures.wait_all(futs)
            return None
        return futs

    a._register_buffer_comm_hook(None, hook, getattr(Loc, where))
    opt = torch.optim.SGD(a.parameters(), lr=0.05)
    g = torch.Generator().manual_seed(40 + rank)
    batches = [(torch.rand(3, 3, 32, 32, generator=g), torch.randint(0, 10, (3,), generator=g))
               for _ in range(2 + 2 * rank)]
    with a.join():
        for x, y in batches:
            opt.zero_grad()
            nn.functional.cross_entropy(a(x), y).backward()
            opt.step()
    # the longest rank ran 2 + 2(ws-1) iterations and every rank called the hook once per
    # iteration (joined ranks shadowing the rest)
    assert len(calls) == 2 + 2 * (ws - 1), calls
    for t in m.state_dict().values():
        lo, hi = t.double().clone(), t.double().clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        assert torch.equal(lo, hi)


@pytest.mark.parametrize("where", ["PRE_FORWARD", "POST_FORWARD"])
def test_join_with_buffer_comm_hook(where):
    _run(_join_buffer_hook, 2, where)


def _uneven(rank, ws, opt_name, divide_initial=True):
    """ddp.join() with uneven inputs (rank r has 2 + 2r batches): the same
    weights, BN buffers and per-iteration grads as torch's DDP under its own
    join, on every rank (the last joiner's model broadcast at the end)."""
    import distributed_training_amd as D
    from torch.nn.parallel import DistributedDataParallel as TDDP

    torch.manual_seed(0)
    m1, m2 = _micro(), _micro()
    m2.load_state_dict(m1.state_dict())
    kw = dict(bucket_cap_mb=0.01)  # several buckets: the joined ranks shadow each in order
    a = D.DistributedDataParallel(m1, **kw)
    b = TDDP(m2, **kw)
    mk = {"sgd": lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9),
          "adam": lambda ps: torch.optim.Adam(ps, lr=1e-3),
          # ws=3 is compared within a tolerance: a small plain step keeps the
          # rounding differences from being amplified over six iterations
          "sgd_small": lambda ps: torch.optim.SGD(ps, lr=1e-3)}[opt_name]
    oa, ob = mk(a.parameters()), mk(b.parameters())
    g = torch.Generator().manual_seed(40 + rank)
    batches = [(torch.rand(3, 3, 32, 32, generator=g), torch.randint(0, 10, (3,), generator=g))
               for _ in range(2 + 2 * rank)]
    grads = {}
    for tag, model, opt in (("a", a, oa), ("b", b, ob)):
        with model.join(divide_by_initial_world_size=divide_initial):
            for it, (x, y) in enumerate(batches):
                opt.zero_grad()
                nn.functional.cross_entropy(model(x), y).backward()
                grads[(tag, it)] = [p.grad.clone() for p in model.module.parameters()]
                opt.step()
    # ws > 2: x(1/ws) before the sum (not exact for 3) and gloo's ring order
    same = torch.equal if ws <= 2 else (lambda u, v: torch.allclose(u.double(), v.double(), rtol=1e-5, atol=1e-6))
    for it in range(len(batches)):
        for i, (u, v) in enumerate(zip(grads[("a", it)], grads[("b", it)])):
            assert same(u, v), f"it {it} grad {i}"
    for (n, x), y in zip(m1.state_dict().items(), m2.state_dict().values()):
        assert same(x, y), n
    # the final broadcast: every rank ends with the last joiner's model, bit for bit
    for t in m1.state_dict().values():
        lo, hi = t.double().clone(), t.double().clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        assert torch.equal(lo, hi)
    assert a._has_rebuilt_buckets


@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_join_uneven_inputs_match_torch(opt_name):
    _run(_uneven, 2, opt_name)


def test_join_uneven_inputs_ws3():
    _run(_uneven, 3, "sgd_small")


@pytest.mark.parametrize("ws", [2, 3])
def test_join_divide_by_remaining_ranks(ws):
    """divide_by_initial_world_size=False: the grads are averaged over the ranks
    still training (the packs' divisor set per iteration from the join count)."""
    _run(_uneven, ws, "sgd" if ws == 2 else "sgd_small", False)


def _state_dict_keys(rank, ws):
    import distributed_training_amd as D

    m = _micro()
    d = D.DistributedDataParallel(m)
    keys = list(d.state_dict().keys())
    assert keys[0] == "module.conv1.weight" and all(k.startswith("module.") for k in keys)
    assert len(keys) == len(m.state_dict())
    # rccl_max_ctas only shapes a libgsync RCCL communicator: on CPU/gloo there is
    # none to own, the DDP works as without it and close() leaves the group alone
    c = D.DistributedDataParallel(_micro(), rccl_max_ctas=8)
    assert c._comm is None and not c._own_comm
    assert c._get_ddp_logging_data()["rccl_max_ctas"] is None
    c(torch.rand(2, 3, 32, 32)).sum().backward()
    c.close()


def test_state_dict_has_module_prefix():
    _run(_state_dict_keys, 1)


def _zero_sized(rank, ws):
    """A zero-element parameter (used in the forward) rides in a bucket as an
    empty slot: grads equal torch's DDP bit for bit, fused SGD equals torch's."""
    import distributed_training_amd as D
    from torch.nn.parallel import DistributedDataParallel as TDDP

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.l = nn.Linear(6, 5)
            self.z = nn.Parameter(torch.empty(0))
            self.l2 = nn.Linear(5, 3)

        def forward(self, x):
            return self.l2(torch.relu(self.l(x) + self.z.sum()))

    torch.manual_seed(0)
    m1, m2 = M(), M()
    m2.load_state_dict(m1.state_dict())
    a, b = D.DistributedDataParallel(m1), TDDP(m2)
    oa = D.FusedSGD(a.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    ob = torch.optim.SGD(b.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, foreach=False)
    g = torch.Generator().manual_seed(40 + rank)
    for it in range(3):
        x = torch.rand(4, 6, generator=g)
        for mod in (a, b):
            mod(x).square().sum().backward()
        for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
            assert (p.grad is None) == (q.grad is None) and (p.grad is None or torch.equal(p.grad, q.grad)), \
                f"it {it} {n}"
        oa.step()
        ob.step()
        oa.zero_grad()
        ob.zero_grad()
        for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7, msg=f"it {it} {n}")


def test_zero_sized_parameter_matches_torch():
    _run(_zero_sized, 2)


def _tied(rank, ws):
    """A weight shared by two layers (one parameter, two uses): one bucket slot,
    its grad the sum of both uses, averaged once — as torch's DDP, which keeps
    the parameter once (T:nn/parallel/distributed.py _build_params_for_reducer
    dedups by identity)."""
    import distributed_training_amd as D
    from torch.nn.parallel import DistributedDataParallel as TDDP

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(6, 6)
            self.b = nn.Linear(6, 6)
            self.b.weight = self.a.weight
            self.c = nn.Linear(6, 2)

        def forward(self, x):
            return self.c(self.b(torch.tanh(self.a(x))))

    torch.manual_seed(0)
    m1, m2 = M(), M()
    m2.load_state_dict(m1.state_dict())
    a, b = D.DistributedDataParallel(m1), TDDP(m2)
    assert len(a._params) == len(list(m1.parameters())) == 5
    g = torch.Generator().manual_seed(60 + rank)
    for it in range(3):
        x = torch.rand(4, 6, generator=g)
        for mod in (a, b):
            mod(x).square().sum().backward()
        for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
            assert torch.equal(p.grad, q.grad), f"it {it} {n}"
        m1.zero_grad()
        m2.zero_grad()
    assert m1.a.weight is m1.b.weight


def test_tied_weights_match_torch():
    _run(_tied, 2)


def _eval_interleaved(rank, ws):
    """Validation forwards between training steps (model.eval() under no_grad,
    then back to train()): outputs, BN buffers and grads equal torch's DDP at
    every step — including torch's rule that a forward after a no-grad forward
    skips the buffer broadcast (require_forward_param_sync)."""
    import distributed_training_amd as D
    from torch.nn.parallel import DistributedDataParallel as TDDP

    torch.manual_seed(2)
    m1, m2 = _micro(), _micro()
    m2.load_state_dict(m1.state_dict())
    a, b = D.DistributedDataParallel(m1), TDDP(m2)
    g = torch.Generator().manual_seed(80 + rank)
    for it in range(4):
        x = torch.rand(3, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (3,), generator=g)
        xv = torch.rand(2, 3, 32, 32, generator=g)
        for mod in (a, b):
            mod.train()
            nn.functional.cross_entropy(mod(x), y).backward()
        for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
            assert torch.equal(p.grad, q.grad), f"it {it} {n}"
        outs = []
        for mod in (a, b):
            mod.eval()
            with torch.no_grad():
                outs.append(mod(xv))
        assert torch.equal(outs[0], outs[1]), f"it {it} eval output"
        for (n, x1), x2 in zip(m1.named_buffers(), m2.buffers()):
            assert torch.equal(x1, x2), f"it {it} {n}"
        m1.zero_grad()
        m2.zero_grad()


def test_eval_forwards_between_steps_match_torch():
    _run(_eval_interleaved, 2)


def _frozen(rank, ws):
    """A frozen layer (requires_grad=False): torch's DDP leaves it out of the
    buckets but still broadcasts it from rank 0 at wrap time; grads of the
    trainable ones equal torch DDP's bit for bit."""
    import distributed_training_amd as D

    out = {}
    for impl in ("torch", "libgsync"):
        torch.manual_seed(0)
        model = _micro()
        torch.manual_seed(100 + rank)  # ranks start with different frozen weights
        with torch.no_grad():
            model.conv1.weight.normal_()
        model.conv1.weight.requires_grad_(False)
        ddp = (torch.nn.parallel.DistributedDataParallel(model) if impl == "torch"
               else D.DistributedDataParallel(model))
        g = torch.Generator().manual_seed(1234 + rank)
        x = torch.rand(4, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (4,), generator=g)
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        out[impl] = (model.conv1.weight.detach().clone(),
                     [p.grad.clone() if p.grad is not None else None for p in model.parameters()])
    (tw, tg), (mw, mg) = out["torch"], out["libgsync"]
    assert torch.equal(tw, mw)  # rank 0's frozen weights on every rank
    w = [torch.zeros_like(mw) for _ in range(ws)]
    dist.all_gather(w, mw)
    assert all(torch.equal(w[0], o) for o in w[1:])
    for a, b in zip(tg, mg):
        assert (a is None) == (b is None) and (a is None or torch.equal(a, b))


def test_frozen_parameters_broadcast_and_grads_match_torch():
    _run(_frozen, 2)


class _Branchy(torch.nn.Module):
    """`extra` is used on rank 0 only; `dead` on no rank."""

    def __init__(self):
        super().__init__()
        self.body = _micro()
        self.extra = torch.nn.Linear(10, 10)
        self.dead = torch.nn.Linear(10, 10)

    def forward(self, x, use_extra):
        h = self.body(x)
        return self.extra(h) if use_extra else h


def _unused_across_ranks(rank, ws):
    """find_unused_parameters with a parameter unused on one rank but used on
    another: torch's Reducer gives that rank the averaged grad (it creates the
    grad from the bucket); a parameter unused everywhere keeps grad None.
    Three iterations, grads bit-identical to torch DDP's on every rank."""
    import distributed_training_amd as D

    out = {}
    for impl in ("torch", "libgsync"):
        torch.manual_seed(0)
        model = _Branchy()
        kw = dict(find_unused_parameters=True)
        ddp = torch.nn.parallel.DistributedDataParallel(model, **kw) if impl == "torch" else \
            D.DistributedDataParallel(model, **kw)
        g = torch.Generator().manual_seed(1234 + rank)
        grads = []
        for _ in range(3):
            for p in model.parameters():
                p.grad = None
            x = torch.rand(4, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (4,), generator=g)
            torch.nn.functional.cross_entropy(ddp(x, rank == 0), y).backward()
            grads.append([None if p.grad is None else p.grad.clone() for p in model.parameters()])
        out[impl] = grads
    for it, (a, b) in enumerate(zip(out["torch"], out["libgsync"])):
        for i, (u, v) in enumerate(zip(a, b)):
            assert (u is None) == (v is None), f"iter {it} param {i}: torch {u is None} libgsync {v is None}"
            assert u is None or torch.equal(u, v), f"iter {it} param {i}"
    names = [n for n, _ in _Branchy().named_parameters()]
    last = out["libgsync"][-1]
    assert all(last[i] is None for i, n in enumerate(names) if n.startswith("dead."))
    assert all(last[i] is not None for i, n in enumerate(names) if n.startswith("extra."))


def test_find_unused_parameters_used_on_another_rank():
    _run(_unused_across_ranks, 2)


def _unused_bf16_buckets(rank, ws):
    """with bf16 buckets, the grad created for a parameter
    unused on this rank keeps the parameter's dtype (fp32; torch refuses a
    grad of another dtype), equals bit for bit the grad the using rank
    unpacked from the same bucket, and the fused AMP non-finite check covers
    it — an inf in rank 0's `extra` grad flags found_inf on rank 1 as well, so
    both ranks take the same skip decision."""
    import distributed_training_amd as D

    torch.manual_seed(0)
    model = _Branchy()
    ddp = D.DistributedDataParallel(model, find_unused_parameters=True, bucket_dtype=torch.bfloat16)
    found = torch.zeros(1)
    ddp.set_found_inf_target(found)
    names = [n for n, _ in model.named_parameters()]
    ix = names.index("extra.weight")
    g = torch.Generator().manual_seed(1234 + rank)
    for it in range(3):
        for p in model.parameters():
            p.grad = None
        x = torch.rand(4, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (4,), generator=g)
        loss = torch.nn.functional.cross_entropy(ddp(x, rank == 0), y)
        if it == 2 and rank == 0:
            model.extra.weight.register_hook(lambda gr: gr.index_fill(0, torch.tensor([0]), float("inf")))
        loss.backward()
        grads = [None if p.grad is None else p.grad for p in model.parameters()]
        assert all(gr is None or gr.dtype == torch.float32 for gr in grads)
        w = grads[ix].clone()
        allw = [torch.zeros_like(w) for _ in range(ws)]
        dist.all_gather(allw, w)
        if it < 2:
            assert torch.equal(allw[0], allw[1]), f"iter {it}: unused rank's grad != using rank's"
            assert found.item() == 0.0
        else:
            assert found.item() == 1.0, f"rank {rank}: the non-finite averaged grad was not flagged"


def test_find_unused_parameters_bf16_buckets_and_amp_check():
    _run(_unused_bf16_buckets, 2)


def _unused_after_no_sync(rank, ws):
    """find_unused_parameters + no_sync: a parameter used only in an
    accumulation (no_sync) backward on one rank counts as used for the next
    synchronising backward, and its accumulated grad is what it contributes
    there (torch's local-used map spans the no_sync steps; an unused variable
    with a defined grad is copied into its bucket).  Grads bit-identical to
    torch DDP on both ranks, two rounds."""
    import distributed_training_amd as D

    out = {}
    for impl in ("torch", "libgsync"):
        torch.manual_seed(0)
        m = _Branchy()
        kw = dict(find_unused_parameters=True)
        ddp = torch.nn.parallel.DistributedDataParallel(m, **kw) if impl == "torch" else \
            D.DistributedDataParallel(m, **kw)
        g = torch.Generator().manual_seed(1234 + rank)
        res = []
        for _ in range(2):
            for p in m.parameters():
                p.grad = None
            with ddp.no_sync():
                x = torch.rand(4, 3, 32, 32, generator=g)
                y = torch.randint(0, 10, (4,), generator=g)
                torch.nn.functional.cross_entropy(ddp(x, rank == 1), y).backward()
            x = torch.rand(4, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (4,), generator=g)
            torch.nn.functional.cross_entropy(ddp(x, False), y).backward()
            res.append([None if p.grad is None else p.grad.clone() for p in m.parameters()])
        out[impl] = res
    for it, (a, b) in enumerate(zip(out["torch"], out["libgsync"])):
        for i, (u, v) in enumerate(zip(a, b)):
            assert (u is None) == (v is None), f"iter {it} param {i}"
            assert u is None or torch.equal(u, v), f"iter {it} param {i}"


def test_find_unused_parameters_used_under_no_sync():
    _run(_unused_after_no_sync, 2)


def _static_graph_dead_layer(rank, ws):
    """static_graph=True with a parameter the graph never uses: torch's
    static-graph Reducer marks it ready at the end of backward (grad stays None);
    libgsync did not and raised at finalize.  Three iterations, grads
    bit-identical to torch DDP."""
    import distributed_training_amd as D

    out = {}
    for impl in ("torch", "libgsync"):
        torch.manual_seed(0)
        m = _Branchy()
        ddp = torch.nn.parallel.DistributedDataParallel(m, static_graph=True) if impl == "torch" else \
            D.DistributedDataParallel(m, static_graph=True)
        g = torch.Generator().manual_seed(1234 + rank)
        res = []
        for _ in range(3):
            for p in m.parameters():
                p.grad = None
            x = torch.rand(4, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (4,), generator=g)
            torch.nn.functional.cross_entropy(ddp(x, True), y).backward()
            res.append([None if p.grad is None else p.grad.clone() for p in m.parameters()])
        out[impl] = res
    for it, (a, b) in enumerate(zip(out["torch"], out["libgsync"])):
        for i, (u, v) in enumerate(zip(a, b)):
            assert (u is None) == (v is None) and (u is None or torch.equal(u, v)), f"iter {it} param {i}"


def test_static_graph_with_a_never_used_parameter():
    _run(_static_graph_dead_layer, 2)


def _torch_hooks(rank, ws):
    """torch's own comm hooks registered on libgsync DDP give torch DDP's grads
    bit for bit: fp16_compress_hook, and the stateful PowerSGD hook (rank-1
    compression after 2 plain iterations, error feedback, warm start) that
    reads GradBucket.index / buffer / gradients / parameters / is_last."""
    import distributed_training_amd as D
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks as dh
    from torch.distributed.algorithms.ddp_comm_hooks import powerSGD_hook as ps

    cases = {"fp16": lambda: (None, dh.fp16_compress_hook),
             "powerSGD": lambda: (ps.PowerSGDState(process_group=None, matrix_approximation_rank=1,
                                                   start_powerSGD_iter=2, min_compression_rate=0.5,
                                                   use_error_feedback=True, warm_start=True, random_seed=0),
                                  ps.powerSGD_hook)}
    for name, make in cases.items():
        out = {}
        for impl in ("torch", "libgsync"):
            torch.manual_seed(0)
            m = _micro()
            ddp = torch.nn.parallel.DistributedDataParallel(m) if impl == "torch" else D.DistributedDataParallel(m)
            ddp.register_comm_hook(*make())
            g = torch.Generator().manual_seed(1234 + rank)
            res = []
            for _ in range(4):
                for p in m.parameters():
                    p.grad = None
                x = torch.rand(4, 3, 32, 32, generator=g)
                y = torch.randint(0, 10, (4,), generator=g)
                torch.nn.functional.cross_entropy(ddp(x), y).backward()
                res.append([p.grad.clone() for p in m.parameters()])
            out[impl] = res
        for it, (a, b) in enumerate(zip(out["torch"], out["libgsync"])):
            for i, (u, v) in enumerate(zip(a, b)):
                assert torch.equal(u, v), f"{name} iter {it} param {i}"


def test_torch_comm_hooks_fp16_and_powersgd_match_torch():
    _run(_torch_hooks, 2)
