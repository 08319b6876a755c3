"""libgsync's RCCL communicator API at world size 1 (the only RCCL world a
one-GPU box can hold): every collective wrapper the N>1 paths call — the
per-forward BN broadcast (DDP._bcast_flat), the ZeRO reduce-scatter /
all-gather, the parity step's all-gather and MIN/MAX checksum all-reduces,
bench.py's standalone collective leg — on every dtype they carry, on an
explicit stream and on the comm stream.  At world 1 each is the identity, so
a wrong count unit, dtype or op mapping shows as a changed or untouched
output.  The calls go on torch's DEFAULT stream (handle 0): the entry points
once read a NULL stream as the communicator's own (non-blocking) stream, so
the collective ran unordered with the fill queued before it — visible at
4 Mi elements.  Also DDP's N>1-only helpers (_broadcast_tensors / _sync_buffers),
run through the communicator by faking the world size on the root rank."""
import pytest
import torch
import torch.distributed as dist

from tests._dist_util import free_port, init_pg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(cuda_device):
    own = not dist.is_initialized()
    if own:
        init_pg("nccl", 0, 1, free_port())
    from distributed_training_amd.comm import destroy_communicators, get_communicator

    yield get_communicator(None, cuda_device)
    if own:
        destroy_communicators()
        dist.destroy_process_group()


def _data(dt, n, dev):
    g = torch.Generator(device=dev).manual_seed(n)
    if dt == torch.int64:
        return torch.randint(-2**40, 2**40, (n,), device=dev, generator=g)
    return torch.randn(n, device=dev, generator=g).to(dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.float64])
@pytest.mark.parametrize("n", [1, 1000, 1 << 20, 1 << 22])  # 4 Mi: large enough to lose a stream race
def test_collectives_identity_at_world_1(comm, cuda_device, dt, n):
    x = _data(dt, n, cuda_device)
    cur = torch.cuda.current_stream(cuda_device).cuda_stream
    for op in ("sum", "min", "max"):
        out = torch.full_like(x, 7)
        comm.all_reduce(x, op=op, stream=cur, out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, x), op
    y = x.clone()
    comm.all_reduce(y)  # in place, on the comm stream
    comm.current_waits()
    assert torch.equal(y, x)
    rs = torch.full_like(x, 3)
    comm.reduce_scatter(x, rs, stream=cur)
    ag = torch.full_like(x, 5)
    comm.all_gather(x, ag, stream=cur)
    b = x.clone()
    comm.broadcast(b, root=0, stream=cur)
    torch.cuda.synchronize()
    assert torch.equal(rs, x) and torch.equal(ag, x) and torch.equal(b, x)


def test_ddp_broadcast_helpers_through_the_communicator(comm, cuda_device):
    """_broadcast_tensors (init sync) and _sync_buffers (per-forward BN buffers)
    are skipped at world 1; run them with the world size faked to 2 on rank 0:
    the pack kernel + RCCL broadcast (the identity on one rank) must leave params
    and buffers — fp32 BN statistics and int64 counters — bit-identical."""
    from distributed_training_amd import DistributedDataParallel
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device)
    ddp = DistributedDataParallel(model)
    assert ddp._comm is not None
    model(torch.rand(4, 3, 32, 32, device=cuda_device))  # non-trivial running stats, counters = 1
    before = [t.detach().clone() for t in list(model.parameters()) + list(model.buffers())]
    ddp.world_size = 2  # rank 0 of a pretend world of two: the broadcast paths run
    try:
        ddp._sync_module_states()
        ddp._sync_buffers()
        ddp._sync_buffers()  # the cached plan
    finally:
        ddp.world_size = 1
    torch.cuda.synchronize()
    after = list(model.parameters()) + list(model.buffers())
    for i, (a, b) in enumerate(zip(before, after)):
        assert a.dtype == b.dtype and torch.equal(a, b.detach()), i


def test_xgmi_calibration_through_the_communicator(comm, cuda_device):
    """bucket_policy="xgmi" (N>1 only) times all-reduces on the DDP's own
    communicator and fits the caps: the same code at world 1 (the fit fed a
    pretend world of 8) runs RCCL on the default stream and returns caps inside
    their clamps."""
    from distributed_training_amd import DistributedDataParallel
    from distributed_training_amd.ddp import xgmi_bucket_caps
    from distributed_training_amd.resnet import micro_resnet

    ddp = DistributedDataParallel(micro_resnet().to(cuda_device))
    cal = xgmi_bucket_caps(ddp._calib_allreduce, 8)
    assert [p["bytes"] for p in cal["points"]] == [m * 2**20 for m in (1, 4, 16, 64)]
    assert all(p["ms"] > 0 for p in cal["points"])
    assert 4 * 2**20 <= cal["bucket_cap_bytes"] <= 256 * 2**20
    assert 256 * 1024 <= cal["last_bucket_cap_bytes"] <= cal["bucket_cap_bytes"]
