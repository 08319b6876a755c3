"""DDP drop-in on the GPU: averaged gradients and post-step weights vs the oracle.

* world_size 1 over RCCL (libgsync's own communicator, AUTO collective on
  the comm stream): averaged grad == local grad bit for bit, before and after
  the bucket rebuild; FusedSGD / FusedAdam steps == oracle bit for bit.
* world_size 2 on the single GPU of the box (two processes sharing cuda:0,
  gloo carries the collective; pack / unpack / optimizer are the HIP kernels):
  averaged grads == oracle Σ_r g_r·float(1/2) bit for bit; BN buffers agree
  across ranks at the start of every forward (rank-0 broadcast).
"""
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from tests._dist_util import free_port, init_pg

pytestmark = pytest.mark.gpu


def _snap_hooks(params, store):
    for i, p in enumerate(params):
        p.register_post_accumulate_grad_hook(lambda q, i=i: store.__setitem__(i, q.grad.detach().clone()))


def to_np(t):
    return t.detach().float().cpu().numpy()


@pytest.fixture(scope="module")
def rccl_pg(cuda_device):
    if dist.is_initialized():  # another module's group is still up
        yield
        return
    init_pg("nccl", 0, 1, free_port())
    yield
    from distributed_training_amd.comm import destroy_communicators

    destroy_communicators()
    dist.destroy_process_group()


def test_ddp_ws1_rccl_grads_and_sgd(cuda_device, rccl_pg):
    from distributed_training_amd import DistributedDataParallel, FusedSGD
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device).to(memory_format=torch.channels_last)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    ddp = DistributedDataParallel(model)
    ddp.set_timeline(2)  # every bucket's HIP events (bucket_comm_ms below)
    assert ddp._comm is not None  # RCCL path, not a fallback
    opt = FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device=cuda_device).manual_seed(1)
    bufs = {}
    for it in range(4):
        x = torch.rand(8, 3, 32, 32, device=cuda_device, generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), device=cuda_device, generator=g)
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            assert torch.equal(p.grad, local[i]), f"iter {it} param {i}"
        # optimizer vs oracle
        ref = []
        for i, p in enumerate(params):
            b = bufs.get(i)
            ref.append(O.sgd(to_np(p).reshape(-1), to_np(p.grad).reshape(-1), None if b is None else b,
                             0.1, 0.9, 0.0, 1e-4, False, False, b is None))
        opt.step()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            assert np.array_equal(to_np(p).reshape(-1), ref[i][0]), f"iter {it} param {i} weights"
            bufs[i] = ref[i][1]
        opt.zero_grad()
    log = ddp._get_ddp_logging_data()
    assert log["has_rebuilt_buckets"] == 1
    assert all(ms >= 0 for ms in ddp.bucket_comm_ms())


@pytest.mark.parametrize("model_name", ["resnet50", "resnet152"])
def test_ddp_full_size_ws1(cuda_device, rccl_pg, model_name):
    """BASELINE sizes (ResNet-50: 25.6 M params in 5 rebuilt buckets; ResNet-152:
    60.2 M in 10), bf16 autocast + channels_last as in bench.py: after the
    rebuild, every averaged grad == the local grad (ws=1 identity through pack ->
    RCCL -> unpack) and the fused SGD step == the oracle, bit for bit."""
    from distributed_training_amd import DistributedDataParallel, FusedSGD
    from distributed_training_amd.resnet import MODELS

    torch.manual_seed(0)
    model = MODELS[model_name]().to(cuda_device).to(memory_format=torch.channels_last)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    ddp = DistributedDataParallel(model)
    opt = FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device=cuda_device).manual_seed(3)
    for it in range(2):  # iteration 0: one bucket; iteration 1: rebuilt buckets
        x = torch.rand(4, 3, 224, 224, device=cuda_device, generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (4,), device=cuda_device, generator=g)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = torch.nn.functional.cross_entropy(ddp(x), y)
        loss.backward()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            assert torch.equal(p.grad, local[i]), f"iter {it} param {i}"
        if it == 1:
            ref = [O.sgd(to_np(p).reshape(-1), to_np(p.grad).reshape(-1), None, 0.1, 0.9, 0.0, 1e-4, False, False,
                         True) for p in params]
            opt.step()
            torch.cuda.synchronize()
            for i, p in enumerate(params):
                assert np.array_equal(to_np(p).reshape(-1), ref[i][0]), f"param {i}"
        opt.zero_grad()
    assert ddp._get_ddp_logging_data()["has_rebuilt_buckets"] == 1
    assert len(ddp.bucket_indices()) == (5 if model_name == "resnet50" else 10)


@pytest.mark.parametrize("div", [3.0, 8.0])
def test_ddp_full_size_in_step_scale(cuda_device, rccl_pg, div):
    """The fused 1/world_size scale inside the real step (at ws=1 the
    pack multiplies by 1.0): ResNet-50 at BASELINE size through the C++ hooks, pack ->
    RCCL -> unpack on the comm / producer streams, with the packs' divisor set to 3 and
    8 (what ws=3 / ws=8 pack with, gs_bucketer_set_div_factor): every averaged grad ==
    local grad * float(1/div) bit for bit (torch's at::mul_out(bucket, grad,
    1/div_factor) in fp32), and the fused SGD step on those grads == the oracle."""
    from distributed_training_amd import DistributedDataParallel, FusedSGD
    from distributed_training_amd.resnet import MODELS

    torch.manual_seed(0)
    model = MODELS["resnet50"]().to(cuda_device).to(memory_format=torch.channels_last)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    ddp = DistributedDataParallel(model)
    opt = FusedSGD(ddp.parameters(), lr=0.1, momentum=0.0, weight_decay=1e-4)
    g = torch.Generator(device=cuda_device).manual_seed(5)
    inv = float(np.float32(1.0 / div))
    for it in range(3):  # iteration 0: one bucket; then the rebuilt layout
        x = torch.rand(4, 3, 224, 224, device=cuda_device, generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (4,), device=cuda_device, generator=g)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = torch.nn.functional.cross_entropy(ddp(x), y)
        # the forward sets the divisor for its backward (world size, or the ranks still
        # training under join): override it between the forward and the backward
        ddp._set_div_factor(div if it > 0 else 1.0)
        loss.backward()
        torch.cuda.synchronize()
        if it > 0:
            assert ddp._native_on  # the C++ hooks, the production path
            for i, p in enumerate(params):
                want = local[i] * torch.tensor(inv, dtype=torch.float32, device=cuda_device)
                assert torch.equal(p.grad, want), f"iter {it} param {i}"
            ref = [O.sgd(to_np(p).reshape(-1), to_np(p.grad).reshape(-1), None, 0.1, 0.0, 0.0, 1e-4, False, False,
                         True) for p in params]
            saved = [p.detach().clone() for p in params]
            opt.step()
            torch.cuda.synchronize()
            for i, p in enumerate(params):
                assert np.array_equal(to_np(p).reshape(-1), ref[i][0]), f"iter {it} param {i} weights"
                p.data.copy_(saved[i])  # keep the weights: the next iteration's grads stay comparable
        opt.zero_grad()
    assert len(ddp.bucket_indices()) == 5
    ddp.close()


def test_ddp_ws1_adam_matches_torch_adam(cuda_device, rccl_pg):
    from distributed_training_amd import DistributedDataParallel, FusedAdam
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device)
    ddp = DistributedDataParallel(model)
    params = list(model.parameters())
    ref_params = [p.detach().clone().requires_grad_(True) for p in params]
    opt = FusedAdam(ddp.parameters(), lr=2e-3)  # the reference's Adam(lr=1e-3*ws), ws=2
    ref_opt = torch.optim.Adam(ref_params, lr=2e-3, foreach=True)
    g = torch.Generator(device=cuda_device).manual_seed(2)
    for it in range(3):
        x = torch.rand(8, 3, 32, 32, device=cuda_device, generator=g)
        y = torch.randint(0, 10, (8,), device=cuda_device, generator=g)
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        for p, q in zip(params, ref_params):
            q.grad = p.grad.clone()
        opt.step()
        ref_opt.step()
        opt.zero_grad()
        ref_opt.zero_grad()
        # Adam tolerance: atol = lr*1e-3 (sign flips where |g|~eps aside)
        for p, q in zip(params, ref_params):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=0, atol=2e-3 * 1e-3)


def test_ddp_bf16_bucket_ws1(cuda_device, rccl_pg):
    """fp32 grads, bf16 buckets: pack casts (x*1.0 -> bf16), unpack widens."""
    from distributed_training_amd import DistributedDataParallel
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    ddp = DistributedDataParallel(model, bucket_dtype=torch.bfloat16)
    x = torch.rand(8, 3, 32, 32, device=cuda_device)
    ddp(x).sum().backward()
    torch.cuda.synchronize()
    for i, p in enumerate(params):
        want = O.bf16_to_f32(O.f32_to_bf16(to_np(local[i]).reshape(-1)))
        assert np.array_equal(to_np(p.grad).reshape(-1), want)


def test_ddp_rccl_max_ctas_ws1(cuda_device, rccl_pg):
    """rccl_max_ctas: the DDP owns a communicator built with ncclConfig_t
    maxCTAs; grads stay the local grads (ws=1, x*1.0 exact) and close() frees it."""
    from distributed_training_amd import DistributedDataParallel
    from distributed_training_amd.comm import get_communicator
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    ddp = DistributedDataParallel(model, rccl_max_ctas=4)
    assert ddp._own_comm and ddp._comm.max_ctas == 4
    assert ddp._comm is not get_communicator(None, cuda_device)
    assert ddp._get_ddp_logging_data()["rccl_max_ctas"] == 4
    x = torch.rand(8, 3, 32, 32, device=cuda_device)
    for _ in range(2):
        for p in params:
            p.grad = None
        ddp(x).sum().backward()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            assert torch.equal(p.grad, local[i])
    comm = ddp._comm
    ddp.close()
    assert not ddp._own_comm and comm.handle is None


def test_ddp_zero_sized_parameter_ws1(cuda_device, rccl_pg):
    """A zero-element parameter in the model (an empty bucket slot, a NULL grad
    pointer) on the C++-hook RCCL path: every grad equals the local grad and the
    fused SGD step equals the oracle."""
    from distributed_training_amd import DistributedDataParallel, FusedSGD

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.l = torch.nn.Linear(64, 32)
            self.z = torch.nn.Parameter(torch.empty(0))
            self.l2 = torch.nn.Linear(32, 8)

        def forward(self, x):
            return self.l2(torch.relu(self.l(x) + self.z.sum()))

    torch.manual_seed(0)
    model = M().to(cuda_device)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    ddp = DistributedDataParallel(model)
    opt = FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    bufs = {}
    for it in range(3):
        x = torch.rand(16, 64, device=cuda_device)
        ddp(x).square().sum().backward()
        torch.cuda.synchronize()
        assert ddp._native_on
        for i, p in enumerate(params):
            assert torch.equal(p.grad, local[i]), f"iter {it} param {i}"
        ref = []
        for i, p in enumerate(params):
            b = bufs.get(i)
            ref.append(O.sgd(to_np(p).reshape(-1), to_np(p.grad).reshape(-1), b, 0.1, 0.9, 0.0, 1e-4,
                             False, False, b is None))
        opt.step()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            assert np.array_equal(to_np(p).reshape(-1), ref[i][0]), f"iter {it} param {i} weights"
            bufs[i] = ref[i][1]
        opt.zero_grad()


def test_ddp_buffer_comm_hook_native_ws1(cuda_device, rccl_pg):
    """A post-forward buffer comm hook on the C++-hook path: called once per
    forward with the named buffers, its futures drained by the end of backward
    (the native finalize), grads unchanged."""
    from distributed_training_amd import DistributedDataParallel
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    ddp = DistributedDataParallel(model)
    seen = []

    def hook(state, named):
        seen.append(len(named))
        fut = torch.futures.Future()
        fut.set_result(None)
        return [fut]

    ddp._register_buffer_comm_hook(None, hook)
    x = torch.rand(8, 3, 32, 32, device=cuda_device)
    for it in range(3):
        for p in params:
            p.grad = None
        ddp(x).sum().backward()
        torch.cuda.synchronize()
        assert ddp._native_on and ddp._post_bwd_futs == []
        for i, p in enumerate(params):
            assert torch.equal(p.grad, local[i]), f"iter {it} param {i}"
    assert seen == [len(list(model.buffers()))] * 3


def _ws2_worker(rank, ws, port, errq):
    try:
        import distributed_training_amd as D
        from distributed_training_amd.resnet import micro_resnet

        init_pg("gloo", rank, ws, port)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.manual_seed(10 + rank)  # different per rank: init broadcast must fix it
        model = micro_resnet().to(dev)
        params = list(model.parameters())
        local = {}
        _snap_hooks(params, local)
        ddp = D.DistributedDataParallel(model, collective="process_group")
        opt = D.FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        seen_bufs = []
        model.register_forward_pre_hook(lambda m, a: seen_bufs.append([b.detach().cpu().clone() for b in m.buffers()]))
        g = torch.Generator(device=dev).manual_seed(100 + rank)
        for it in range(3):
            x = torch.rand(6, 3, 32, 32, device=dev, generator=g)
            y = torch.randint(0, 10, (6,), device=dev, generator=g)
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
            torch.cuda.synchronize()
            mine = [to_np(local[i]) for i in range(len(params))]
            allg = [None] * ws
            dist.all_gather_object(allg, mine)
            avg = O.ddp_average(allg)
            for i, p in enumerate(params):
                assert np.array_equal(to_np(p.grad), avg[i]), f"rank {rank} iter {it} param {i}"
            opt.step()
            opt.zero_grad()
            allb = [None] * ws
            dist.all_gather_object(allb, seen_bufs[-1])
            for a, b in zip(allb[0], allb[1]):
                assert torch.equal(a, b), "BN buffers differ across ranks at forward start"
        w = [to_np(p) for p in params]
        allw = [None] * ws
        dist.all_gather_object(allw, w)
        for a, b in zip(allw[0], allw[1]):
            assert np.array_equal(a, b), "weights diverged across ranks"
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent
        import traceback

        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def test_ddp_ws2_one_gpu_gloo_collective(cuda_device):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_ws2_worker, args=(r, 2, port, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.mark.parametrize("mode", ["no_sync", "view", "small_buckets", "find_unused", "bf16_model", "mixed_dtype",
                                  "debug_checksums", "last_bucket_cap"])
def test_ddp_ws1_modes(cuda_device, rccl_pg, mode):
    """torch-DDP options on the RCCL path; at ws=1 the averaged grad must equal
    the (accumulated) local grad bit for bit."""
    from distributed_training_amd import DistributedDataParallel
    from distributed_training_amd.resnet import micro_resnet

    class WithUnused(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.body = micro_resnet()
            self.unused = torch.nn.Linear(3, 3)

        def forward(self, x):
            return self.body(x)

    class Mixed(torch.nn.Module):  # fp32 body, bf16 head: per-dtype buckets
        def __init__(self):
            super().__init__()
            self.body = micro_resnet()
            self.head = torch.nn.Linear(10, 5).to(torch.bfloat16)

        def forward(self, x):
            return self.head(self.body(x).to(torch.bfloat16)).float()

    torch.manual_seed(0)
    model = (WithUnused() if mode == "find_unused" else Mixed() if mode == "mixed_dtype" else micro_resnet())
    model = model.to(cuda_device)
    if mode == "bf16_model":
        model = model.to(torch.bfloat16)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    kw = {"find_unused_parameters": mode == "find_unused", "gradient_as_bucket_view": mode == "view"}
    if mode == "small_buckets":
        kw["bucket_cap_mb"] = 0.02
    if mode == "last_bucket_cap":
        kw["last_bucket_cap_mb"] = 0.001
    ddp = DistributedDataParallel(model, **kw)
    if mode == "last_bucket_cap":
        ddp.set_timeline(2)  # the tail split below
    if mode == "debug_checksums":
        ddp.enable_bucket_checksums()
    dt = torch.bfloat16 if mode == "bf16_model" else torch.float32
    g = torch.Generator(device=cuda_device).manual_seed(3)
    for it in range(3):
        local.clear()
        xs = [torch.rand(4, 3, 32, 32, device=cuda_device, generator=g).to(dt) for _ in range(3)]
        if mode == "no_sync":
            with ddp.no_sync():
                for x in xs[:2]:
                    ddp(x).float().sum().backward()
        ddp(xs[2]).float().sum().backward()
        torch.cuda.synchronize()
        if mode == "debug_checksums":
            for tot, post, tol in ddp.verify_bucket_checksums():
                assert tot == post  # ws=1: the collective is the identity
        if mode == "mixed_dtype":
            assert set(ddp._bucketer.bucket_dtypes) == {torch.float32, torch.bfloat16}
        for i, p in enumerate(params):
            if mode == "find_unused" and i >= len(params) - 2:
                assert p.grad is None
                continue
            assert torch.equal(p.grad, local[i]), f"{mode} it {it} param {i}"
        if mode == "view":
            for i, p in enumerate(params):
                assert p.grad.data_ptr() == ddp._bucketer.bucket_view(i).data_ptr()
                p.grad.zero_()
        else:
            ddp.zero_grad(set_to_none=True)
    if mode == "small_buckets":
        assert len(ddp.bucket_indices()) > 3
    if mode == "last_bucket_cap":
        last = ddp.bucket_indices()[-1]
        assert len(last) == 1 or sum(params[i].numel() * 4 for i in last) <= 1048
        t = ddp.tail_ms()
        assert t is not None and t["total"] >= t["pack"] >= 0
        ddp.set_timeline(1)  # default: the tail total only, no split
        run_one = params[0].grad is None
        x = torch.rand(8, 3, 32, 32, device=cuda_device)
        torch.nn.functional.cross_entropy(ddp(x), torch.zeros(8, dtype=torch.long, device=cuda_device)).backward()
        t = ddp.tail_ms()
        assert run_one and t is not None and t["total"] >= 0 and t["pack"] is None
        assert all(ms < 0 for ms in ddp.bucket_comm_ms())


def test_communicator_watchdog_and_abort(cuda_device):
    """Failure detection: a live communicator with a short watchdog
    timeout never trips on completing collectives; after an abort every call fails
    with the reason instead of hanging."""
    import time

    import torch.distributed as dist

    from distributed_training_amd import _lib as L
    from distributed_training_amd.comm import Communicator
    from tests._dist_util import free_port

    if not dist.is_initialized():
        import os

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(free_port())
        dist.init_process_group("gloo", rank=0, world_size=1)
    c = Communicator(None, cuda_device, timeout_ms=500)
    t = torch.ones(1 << 20, device=cuda_device)
    for _ in range(200):
        c.all_reduce(t)
    torch.cuda.synchronize()
    time.sleep(0.7)  # > timeout: completed collectives must not count as hung
    assert c.status() == (False, "")
    c.abort()
    aborted, why = c.status()
    assert aborted and "gs_comm_abort" in why
    with pytest.raises(L.GsyncError, match="aborted"):
        c.all_reduce(t)
    with pytest.raises(L.GsyncError, match="aborted"):
        c.check()
    c.close()


def test_ddp_watchdog_marks_on_unpacks(cuda_device, rccl_pg):
    """The bucketer hands each collective to the RCCL watchdog through the stop
    event its unpack kernel carries (no event packet after the collective): with
    a 400 ms timeout, steps queued back to back at timeline levels 0, 1 and 2
    (each bucket's mark re-recorded before its last record completed) complete,
    and after a wait longer than the timeout nothing counts as hung; closing the DDP drops
    the bucketer's events from the watchdog; the grads equal the hooks' own at
    world size 1."""
    import time

    from distributed_training_amd import DistributedDataParallel
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device).to(memory_format=torch.channels_last)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)
    ddp = DistributedDataParallel(model)
    comm = ddp._comm
    saved = comm.timeout_ms
    comm.set_timeout(400)
    g = torch.Generator(device=cuda_device).manual_seed(3)
    x = torch.rand(8, 3, 32, 32, device=cuda_device, generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda_device, generator=g)
    for level in (0, 1, 2, 1):
        ddp.set_timeline(level)
        # steps queued back to back (the host ahead of the GPU re-records each bucket's
        # mark before the last record completed), then one checked step
        for _ in range(8):
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
        for p in params:
            p.grad = None
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            assert torch.equal(p.grad, local[i]), f"level {level} param {i}"
    time.sleep(0.6)
    assert comm.status() == (False, "")
    own = getattr(ddp, "_own_comm", False)
    ddp.close()  # drops the bucketer's events from the watchdog before destroying them
    if not own:  # a shared communicator lives on: its watchdog must not trip on them
        time.sleep(0.6)
        assert comm.status() == (False, "")
        comm.set_timeout(saved)


@pytest.mark.parametrize("kind", ["sgd", "adamw"])
def test_overlapped_optimizer_ws1_rccl(cuda_device, rccl_pg, kind):
    """DDP._register_fused_optim on the AUTO-collective path: each bucket's
    fused update is enqueued behind its unpack on the stream its chain ran on
    (the comm stream; the producer stream for the last bucket), under the rest
    of backward.  Every iteration (bucket rebuild included), against the oracle
    on the same run's data (MIOpen's backward is not bitwise run-to-run, so two
    runs are not compared): the grads the hooks saw == the averaged grads
    (ws=1) and the weights after backward == oracle SGD / AdamW of the weights
    before it with those grads, bit for bit — no update read a partial unpack
    or a weight the backward still used."""
    import ctypes

    from distributed_training_amd import DistributedDataParallel
    from distributed_training_amd import _lib as L
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device).to(memory_format=torch.channels_last)
    params = list(model.parameters())
    local = {}
    _snap_hooks(params, local)  # before DDP's hooks: the local grad, ahead of the chain
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.02)  # several buckets after the rebuild
    if kind == "sgd":
        ddp._register_fused_optim(torch.optim.SGD, lr=0.05, momentum=0.9, weight_decay=1e-4)
    else:
        ddp._register_fused_optim(torch.optim.AdamW, lr=1e-3, weight_decay=1e-2)
    g = torch.Generator(device=cuda_device).manual_seed(5)
    state = {}
    for it in range(4):
        x = torch.rand(8, 3, 32, 32, device=cuda_device, generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), device=cuda_device, generator=g)
        out = ddp(x)  # the forward reads the weights: snapshot them after it (same stream)
        before = [to_np(p).reshape(-1).copy() for p in params]
        torch.nn.functional.cross_entropy(out, y).backward()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            gl = to_np(local[i]).reshape(-1)
            assert np.array_equal(to_np(p.grad).reshape(-1), gl), f"iter {it} param {i} grad"
            if kind == "sgd":
                st = state.get(i)
                w, buf = O.sgd(before[i], gl, st, 0.05, 0.9, 0.0, 1e-4, False, False, st is None)
                state[i] = buf
            else:
                m, v = state.get(i, (np.zeros_like(gl), np.zeros_like(gl)))
                w, m, v = O.adam(before[i], gl, m, v, it + 1, 1e-3, weight_decay=1e-2, adamw=True)
                state[i] = (m, v)
            assert np.array_equal(to_np(p).reshape(-1), w), f"{kind} iter {it} param {i} weights"
        for p in params:
            p.grad = None
    nb = len(ddp.bucket_indices())
    assert nb > 2 and ddp._get_ddp_logging_data()["has_rebuilt_buckets"] == 1
    comm = ctypes.c_void_p()
    L.check(L.lib().gs_comm_stream(ddp._comm.handle, ctypes.byref(comm)), "gs_comm_stream")
    streams = []
    for bi in range(nb):
        s = ctypes.c_void_p()
        L.check(L.lib().gs_bucketer_bucket_stream(ddp._bucketer.handle, bi, ctypes.byref(s)), "stream")
        streams.append(s.value)
    assert all(s == comm.value for s in streams[:-1])  # updates under backward, on the comm stream
    # the tail runs on the producer stream (here the default stream, handle 0)
    assert (streams[-1] or 0) == (torch.cuda.current_stream(cuda_device).cuda_stream or 0)


def test_mixed_dtype_buckets_ws1_rccl(cuda_device, rccl_pg):
    """fp32 body + bf16 head + fp16 bias on the GPU (RCCL ws=1): the HIP path
    of per-dtype buckets (pack / all-reduce / unpack per bucket dtype, rebuilt
    in ready order) gives the same grads as torch's own DDP bit for bit, and
    the same rebuilt bucket sizes (tests/test_ddp_mixed_dtype_cpu.py on CPU).
    MIOpen in deterministic mode so both see identical local grads."""
    from distributed_training_amd import DistributedDataParallel
    from tests.test_ddp_mixed_dtype_cpu import Mixed

    det, bench = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        out = {}
        for impl in ("torch", "libgsync"):
            torch.manual_seed(0)
            model = Mixed().to(cuda_device)
            ddp = (torch.nn.parallel.DistributedDataParallel(model, device_ids=[cuda_device.index])
                   if impl == "torch" else DistributedDataParallel(model))
            g = torch.Generator(device=cuda_device).manual_seed(1234)
            grads = []
            for _ in range(3):  # iteration 0: one bucket per dtype; then rebuilt in ready order
                x = torch.rand(4, 3, 32, 32, device=cuda_device, generator=g)
                y = torch.randint(0, 7, (4,), device=cuda_device, generator=g)
                for p in model.parameters():
                    p.grad = None
                torch.nn.functional.cross_entropy(ddp(x), y).backward()
                torch.cuda.synchronize()
                grads.append([p.grad.clone() for p in model.parameters()])
            sizes = ddp._get_ddp_logging_data()["rebuilt_bucket_sizes"]
            out[impl] = (grads, sizes, ddp)
        (tg, ts, _), (mg, ms, mddp) = out["torch"], out["libgsync"]
        for it, (a, b) in enumerate(zip(tg, mg)):
            for i, (u, v) in enumerate(zip(a, b)):
                assert u.dtype == v.dtype and torch.equal(u, v), f"iter {it} param {i} ({u.dtype})"
        ts = [int(v) for v in str(ts).split(",")] if isinstance(ts, str) else list(ts)
        assert sorted(ts) == sorted(ms), (ts, ms)
        assert set(mddp._bucketer.bucket_dtypes) == {torch.float32, torch.bfloat16, torch.float16}
        assert all(b.is_cuda for b in mddp._bucketer.buffers)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, bench


def _join_worker(rank, ws, port, errq):
    """ddp.join() on the GPU (two ranks sharing cuda:0 over gloo, device buckets
    staged through the host): rank 0 has 2 batches, rank 1 has 4.  While both
    train, the averaged grads equal the oracle's Σ_r g_r·float(1/2); after rank 0
    joined, rank 1's grads are its local grads ·float(1/2) (the joined rank's
    zeros, divide_by_initial_world_size); afterwards both hold the last joiner's
    weights."""
    try:
        import distributed_training_amd as D
        from distributed_training_amd.resnet import micro_resnet

        init_pg("gloo", rank, ws, port)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.manual_seed(10 + rank)
        model = micro_resnet().to(dev)
        params = list(model.parameters())
        local = {}
        _snap_hooks(params, local)
        ddp = D.DistributedDataParallel(model, collective="process_group", bucket_cap_mb=0.05)
        opt = D.FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9)
        g = torch.Generator(device=dev).manual_seed(100 + rank)
        n = 2 + 2 * rank
        with ddp.join():
            for it in range(n):
                x = torch.rand(6, 3, 32, 32, device=dev, generator=g)
                y = torch.randint(0, 10, (6,), device=dev, generator=g)
                torch.nn.functional.cross_entropy(ddp(x), y).backward()
                torch.cuda.synchronize()
                mine = [to_np(local[i]) for i in range(len(params))]
                if it < 2:  # both ranks still training
                    allg = [None] * ws
                    dist.all_gather_object(allg, mine)
                    avg = O.ddp_average(allg)
                else:
                    avg = O.ddp_average([[np.zeros_like(m) for m in mine], mine])
                for i, p in enumerate(params):
                    assert np.array_equal(to_np(p.grad), avg[i]), f"rank {rank} iter {it} param {i}"
                opt.step()
                opt.zero_grad()
        w = [to_np(p) for p in params]
        allw = [None] * ws
        dist.all_gather_object(allw, w)
        for a, b in zip(allw[0], allw[1]):
            assert np.array_equal(a, b), "weights differ across ranks after join"
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent
        import traceback

        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def test_ddp_join_uneven_inputs_ws2_one_gpu(cuda_device):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_join_worker, args=(r, 2, port, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
