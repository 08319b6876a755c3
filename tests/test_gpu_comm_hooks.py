"""Comm-hook path of the DDP drop-in on the GPU (the
Colossal torch_ddp plugin is torch DDP, R:resnet/colossal/colossal_train.py:131-132,
so torch's hook API is part of the drop-in).

torch's own ``allreduce_hook`` and ``bf16_compress_hook``
(T:distributed/algorithms/ddp_comm_hooks/default_hooks.py:18-54, 57-93) are
registered on libgsync DDP.  The bucketer then packs WITHOUT the 1/ws scale
(GS_BKT_NO_SCALE) on the producer stream, the hook owns the averaging and the
collective, and its future's tensor is unpacked into the grads.  The averaged
grads must equal the oracle bit for bit:

  allreduce_hook:      Σ_r (g_r / ws)                 O.pack(f32, ws, DIV) -> sum -> unpack
  bf16_compress_hook:  Σ_r bf16(bf16(g_r) / ws) -> f32  O.pack(bf16, ws, DIV) -> bf16 sum -> unpack

at world size 1 over the RCCL process group and world size 2 over gloo (two
processes sharing the box's one GPU).
"""
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from tests._dist_util import free_port, init_pg

pytestmark = pytest.mark.gpu


def _expected(local_per_rank, hook_name):
    ws = len(local_per_rank)
    shapes = [g.shape for g in local_per_rank[0]]
    if hook_name == "allreduce":
        flats = [O.pack(gs, "f32", float(ws), 2) for gs in local_per_rank]
        return O.unpack(O.allreduce_sum(flats), shapes, np.float32)
    flats = [O.pack(gs, "bf16", float(ws), 2) for gs in local_per_rank]
    return O.unpack(O.allreduce_sum(flats), shapes, np.float32, flat_dtype=O.BF16)


def _hook(name):
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks

    return default_hooks.allreduce_hook if name == "allreduce" else default_hooks.bf16_compress_hook


def _run_steps(rank, ws, dev, hook_name, steps=3):
    import distributed_training_amd as D
    from distributed_training_amd import _lib as L
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(dev)
    params = list(model.parameters())
    local = {}
    for i, p in enumerate(params):
        p.register_post_accumulate_grad_hook(lambda q, i=i: local.__setitem__(i, q.grad.detach().clone()))
    ddp = D.DistributedDataParallel(model)
    ddp.register_comm_hook(None, _hook(hook_name))
    assert ddp._bucketer.flags & L.GS_BKT_NO_SCALE
    assert not (ddp._bucketer.flags & L.GS_BKT_AUTO_COLLECTIVE)
    g = torch.Generator(device=dev).manual_seed(50 + rank)
    for it in range(steps):  # iteration 0: one bucket; then the rebuilt layout
        x = torch.rand(6, 3, 32, 32, device=dev, generator=g)
        y = torch.randint(0, 10, (6,), device=dev, generator=g)
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        mine = [local[i].float().cpu().numpy() for i in range(len(params))]
        if ws > 1:
            allg = [None] * ws
            dist.all_gather_object(allg, mine)
        else:
            allg = [mine]
        want = _expected(allg, hook_name)
        for i, p in enumerate(params):
            got = p.grad.float().cpu().numpy()
            assert np.array_equal(got, want[i]), f"{hook_name} rank {rank} iter {it} param {i}"
        ddp.zero_grad(set_to_none=True)
    assert ddp._get_ddp_logging_data()["has_rebuilt_buckets"] == 1


@pytest.mark.parametrize("hook_name", ["allreduce", "bf16_compress"])
def test_comm_hook_ws1_rccl(cuda_device, hook_name):
    owned = False
    if not dist.is_initialized():
        init_pg("nccl", 0, 1, free_port())
        owned = True
    try:
        if dist.get_backend() != "nccl":
            pytest.skip("another module left a non-RCCL default group")
        _run_steps(0, 1, cuda_device, hook_name)
    finally:
        if owned:
            from distributed_training_amd.comm import destroy_communicators

            destroy_communicators()
            dist.destroy_process_group()


def _ws2_worker(rank, ws, port, hook_name, errq):
    try:
        init_pg("gloo", rank, ws, port)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        _run_steps(rank, ws, dev, hook_name)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent
        import traceback

        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


@pytest.mark.parametrize("hook_name", ["allreduce", "bf16_compress"])
def test_comm_hook_ws2_one_gpu_gloo(cuda_device, hook_name):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_ws2_worker, args=(r, 2, port, hook_name, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
