"""The C++ gradient hooks (_gshook) on the GPU fast path (RCCL ws=1, library
collective): the DDP picks them by default and the library that ran is the
in-tree extension.  At world size 1 the averaged grad is the local grad bit for
bit, so every step's grads (bf16 autocast, channels_last, the first-iteration
single bucket, the rebuild in the ready order the C++ hooks recorded, a
no_sync accumulation) are checked against the local grads snapshotted before
the pack (MIOpen's backward is not run-to-run deterministic, so two trainings
are not compared with each other).  Also: the Python hooks take over for the
parity capture and hand back."""
import pytest
import torch
import torch.distributed as dist

from tests._dist_util import free_port, init_pg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_pg(cuda_device):
    if dist.is_initialized():
        yield
        return
    init_pg("nccl", 0, 1, free_port())
    yield
    from distributed_training_amd.comm import destroy_communicators

    destroy_communicators()
    dist.destroy_process_group()


def _train(dev, opt_name: str, steps=5):
    import distributed_training_amd as D
    from distributed_training_amd.resnet import MODELS

    torch.manual_seed(0)
    model = MODELS["resnet18"](num_classes=10).to(dev).to(memory_format=torch.channels_last)
    params = list(model.parameters())
    local = {}
    for i, p in enumerate(params):  # the local (pre-pack) grads, on the producer stream
        p.register_post_accumulate_grad_hook(lambda q, i=i: local.__setitem__(i, q.grad.detach().clone()))
    ddp = D.DistributedDataParallel(model)
    assert ddp._comm is not None and ddp._native is not None
    opt = (D.FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4) if opt_name == "sgd"
           else D.FusedAdam(ddp.parameters(), lr=1e-3))
    g = torch.Generator(device=dev).manual_seed(3)
    crit = torch.nn.CrossEntropyLoss()
    for s in range(steps):
        x = torch.rand(16, 3, 32, 32, device=dev, generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (16,), device=dev, generator=g)
        if s == 3:
            with ddp.no_sync():
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    crit(ddp(x), y).backward()
        local.clear()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            crit(ddp(x), y).backward()
        assert ddp._native_on and not ddp._hook_handles
        assert len(local) == len(params)
        for i, p in enumerate(params):
            assert torch.equal(p.grad, local[i]), f"step {s} grad {i}"
        if s == 0:
            assert sorted(ddp._ready_order) == list(range(len(params)))
        opt.step()
        opt.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    assert ddp._has_rebuilt_buckets and ddp._num_iterations == steps
    # the parity capture runs on the Python hooks, then the C++ hooks return
    ddp._capture_local = {0: None}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        crit(ddp(x), y).backward()
    assert not ddp._native_on and ddp._capture_local[0] is not None
    ddp._capture_local = None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        crit(ddp(x), y).backward()
    assert ddp._native_on
    torch.cuda.synchronize()


@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_native_hooks_grads_equal_local_grads(cuda_device, rccl_pg, opt_name):
    from distributed_training_amd import _lib as L

    assert L.hook_module() is not None, "the _gshook extension is not built"
    _train(cuda_device, opt_name)
    import collections

    maps = collections.OrderedDict((ln.split()[-1], 1) for ln in open("/proc/self/maps") if "_gshook" in ln)
    assert any(m.endswith("distributed_training_amd/lib/_gshook.so") for m in maps), list(maps)


def test_native_hooks_static_graph_never_used_parameter(cuda_device, rccl_pg):
    """static_graph=True with a module the graph never uses, on the C++ hooks
    (their finalize skipped gs_bucketer_mark_unused and raised
    'Expected to have finished reduction'): three iterations; grads equal the
    local grads snapshotted before the pack (ws=1) and torch DDP's None for the
    never-used layer; the Python-hook path gives the same."""
    import distributed_training_amd as D
    from tests.test_ddp_cpu import _Branchy

    for native in (True, False):
        torch.manual_seed(0)
        m = _Branchy().to(cuda_device)
        params = list(m.parameters())
        local = {}
        for i, p in enumerate(params):
            p.register_post_accumulate_grad_hook(lambda q, i=i: local.__setitem__(i, q.grad.detach().clone()))
        ddp = D.DistributedDataParallel(m, static_graph=True)
        if not native:
            ddp._native = None
            ddp._set_native(False)
        g = torch.Generator(device=cuda_device).manual_seed(11)
        for it in range(3):
            for p in params:
                p.grad = None
            local.clear()
            x = torch.rand(4, 3, 32, 32, device=cuda_device, generator=g)
            y = torch.randint(0, 10, (4,), device=cuda_device, generator=g)
            torch.nn.functional.cross_entropy(ddp(x, True), y).backward()
            assert ddp._native_on == native
            for i, p in enumerate(params):
                if i in local:
                    assert torch.equal(p.grad, local[i]), f"native={native} it {it} param {i}"
                else:
                    assert p.grad is None, f"native={native} it {it} param {i}: never used"
        assert m.dead.weight.grad is None and m.extra.weight.grad is not None
        torch.cuda.synchronize()
