"""The C++ gradient hooks (_gshook, csrc/gs_torch_hook.cpp: AccumulateGrad
post-hooks calling gs_bucketer_mark_ready, end-of-backward gs_bucketer_finalize,
as torch's Reducer hooks T:include/torch/csrc/distributed/c10d/reducer.hpp:73)
driven on the CPU: the hook object is pointed at the DDP's host bucketer
(device -1: no stream) at world size 1, where the averaged grad is the local
grad bit for bit.  Checks the grads through the first-iteration single bucket,
the rebuild in the ready order the C++ hooks recorded, no_sync accumulation,
non-dense grads, and the switch back to the Python hooks."""
import weakref

import pytest
import torch
import torch.nn as nn

from tests.test_ddp_cpu import _micro, _run

pytestmark = pytest.mark.skipif(
    __import__("distributed_training_amd")._lib.hook_module() is None, reason="_gshook not built")


def _force_native(ddp):
    from distributed_training_amd import _lib as L

    ref = weakref.ref(ddp)
    ddp._native = L.hook_module().Hooks(ddp._params, -1, lambda: ref()._native_finalized())
    ddp._native.set_bucketer(ddp._bucketer.handle.value, len(ddp._bucketer.buckets))
    ddp._native.set_mark_unused(bool(ddp.static_graph))
    ddp._native_ok = lambda: ddp._capture_local is None  # host bucketer: no library collective
    ddp._set_native(True)


def _native_vs_plain(rank, ws):
    import distributed_training_amd as D

    torch.manual_seed(0)
    m1, m2 = _micro(), _micro()
    m2.load_state_dict(m1.state_dict())
    a = D.DistributedDataParallel(m1)
    _force_native(a)
    assert a._native_on and not a._hook_handles
    g = torch.Generator().manual_seed(5)
    for it in range(4):
        xs = [torch.rand(4, 3, 32, 32, generator=g) for _ in range(2)]
        ys = [torch.randint(0, 10, (4,), generator=g) for _ in range(2)]
        if it == 2:  # accumulation under no_sync, synchronised by the next backward
            with a.no_sync():
                nn.functional.cross_entropy(a(xs[0]), ys[0]).backward()
            nn.functional.cross_entropy(m2(xs[0]), ys[0]).backward()
        nn.functional.cross_entropy(a(xs[1]), ys[1]).backward()
        nn.functional.cross_entropy(m2(xs[1]), ys[1]).backward()
        for (n, pa), pb in zip(m1.named_parameters(), m2.parameters()):
            assert torch.equal(pa.grad, pb.grad), f"it {it} {n}"
        if it == 0:
            assert len(a._ready_order) == len(a._params)  # recorded by the C++ hooks
        m1.zero_grad()
        m2.zero_grad()
    assert a._has_rebuilt_buckets and a._num_iterations == 4
    assert a._native_on
    # a non-dense grad is copied into the parameter's layout before the pack
    w = m1.fc.weight
    x = torch.rand(4, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (4,), generator=g)
    w.grad = torch.zeros(w.shape[1], w.shape[0]).t()  # transposed strides: not dense-like
    nn.functional.cross_entropy(a(x), y).backward()
    assert w.grad.stride() == w.stride()
    # parity capture switches to the Python hooks, and back
    a._capture_local = {0: None}
    m1.zero_grad()
    nn.functional.cross_entropy(a(x), y).backward()
    assert not a._native_on and a._hook_handles and a._capture_local[0] is not None
    a._capture_local = None
    nn.functional.cross_entropy(a(x), y).backward()
    assert a._native_on and not a._hook_handles


def test_native_hooks_match_plain_grads_ws1():
    _run(_native_vs_plain, 1)


def test_native_hooks_attach_detach():
    from distributed_training_amd import _lib as L

    p = nn.Parameter(torch.zeros(3))
    calls = []
    h = L.hook_module().Hooks([p], -1, lambda: calls.append(1))
    h.attach()
    assert h.attached()
    h.detach()
    assert not h.attached()
    (p * 2).sum().backward()  # detached: nothing fires
    assert calls == [] and torch.equal(p.grad, torch.full((3,), 2.0))


def _zero_native_vs_python(rank, ws):
    """The ZeRO engine's release mode of the C++ hooks (grad freed once marked
    ready, held until its bucket's pack is enqueued) on the host bucketer at
    world size 1: weights after several AdamW steps with clipping equal the
    Python-hook engine's bit for bit, and grads are released."""
    from distributed_training_amd import _lib as L
    from distributed_training_amd.zero import ZeroDataParallel

    res = []
    for native in (True, False):
        torch.manual_seed(0)
        m = _micro()
        eng = ZeroDataParallel(m, stage=2, optimizer="adamw", lr=1e-3, weight_decay=1e-2, gradient_clipping=0.5)
        if native:
            ref = weakref.ref(eng)
            eng._native = L.hook_module().Hooks(eng.params, -1, lambda: ref()._native_finalized(), True)
            eng._native.set_bucketer(eng.handle.value, len(eng.buckets), [bi for bi, _ in eng.loc], 0)
            eng._native_ok = lambda: eng._capture_local is None
        g = torch.Generator().manual_seed(3)
        for it in range(4):
            x = torch.rand(4, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (4,), generator=g)
            eng.prepare_backward()  # before the forward, as the engines call it
            nn.functional.cross_entropy(m(x), y).backward()
            assert all(p.grad is None for p in eng.params)  # released into the buckets
            eng.step()
        assert eng._native_on == native and not eng._in_backward
        res.append([p.detach().clone() for p in m.parameters()])
        eng.close()
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_native_hooks_zero_release_mode_ws1():
    _run(_zero_native_vs_python, 1)


def _native_static_graph(rank, ws):
    """static_graph=True with a never-used layer on the C++ hooks: their finalize
    marks it ready (gs_bucketer_mark_unused) as the Python _finalize_backward does;
    grads equal torch's static-graph DDP bit for bit, the dead layer's stay None."""
    import distributed_training_amd as D
    from tests.test_ddp_cpu import _Branchy

    out = {}
    for impl in ("torch", "native"):
        torch.manual_seed(0)
        m = _Branchy()
        if impl == "torch":
            ddp = torch.nn.parallel.DistributedDataParallel(m, static_graph=True)
        else:
            ddp = D.DistributedDataParallel(m, static_graph=True)
            _force_native(ddp)
        g = torch.Generator().manual_seed(7)
        res = []
        for _ in range(3):
            for p in m.parameters():
                p.grad = None
            x = torch.rand(4, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (4,), generator=g)
            nn.functional.cross_entropy(ddp(x, True), y).backward()
            res.append([None if p.grad is None else p.grad.clone() for p in m.parameters()])
        if impl == "native":
            assert ddp._native_on
        out[impl] = res
    for it, (a, b) in enumerate(zip(out["torch"], out["native"])):
        for i, (u, v) in enumerate(zip(a, b)):
            assert (u is None) == (v is None) and (u is None or torch.equal(u, v)), f"iter {it} param {i}"


def test_native_hooks_static_graph_ws1():
    _run(_native_static_graph, 1)
