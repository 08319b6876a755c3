"""One RCCL communicator per rank: with libgsync's
communicator in place, DDP's control-plane collectives — the wrap-time shape
check and module-state broadcast (T:nn/parallel/distributed.py:860-870), the
rank-0 bucket-layout broadcast after the first iteration (Reducer
sync_bucket_indices), the per-forward buffer broadcast, the
find_unused_parameters used-map all-reduce, the bucket-checksum debug check and
the xGMI calibration — and the communicator's own unique-id bootstrap go
through libgsync, never through torch.distributed.  Checked at world 1 (the only
RCCL world a one-GPU box holds) with the world size faked to 2 on rank 0 so the
N>1 branches run, and every torch.distributed collective patched to raise."""
import pytest
import torch
import torch.distributed as dist

from tests._dist_util import free_port, init_pg

pytestmark = pytest.mark.gpu

COLLECTIVES = ("all_reduce", "broadcast", "barrier", "all_gather", "all_gather_into_tensor", "reduce_scatter",
               "reduce_scatter_tensor", "broadcast_object_list", "all_gather_object", "gather", "scatter")


@pytest.fixture
def no_torch_collectives(monkeypatch):
    calls = []

    def make(name):
        def refuse(*a, **k):
            calls.append(name)
            raise AssertionError(f"torch.distributed.{name} called on the RCCL path")
        return refuse

    for name in COLLECTIVES:
        monkeypatch.setattr(dist, name, make(name))
    return calls


@pytest.fixture(scope="module")
def pg(cuda_device):
    own = not dist.is_initialized()
    if own:
        init_pg("nccl", 0, 1, free_port())
    yield
    if own:
        from distributed_training_amd.comm import destroy_communicators

        destroy_communicators()
        dist.destroy_process_group()


def test_communicator_bootstrap_uses_the_store(pg, cuda_device, no_torch_collectives):
    from distributed_training_amd.comm import Communicator

    c = Communicator(None, cuda_device)
    t = torch.arange(10, dtype=torch.float32, device=cuda_device)
    c.all_reduce(t, stream=torch.cuda.current_stream(cuda_device).cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(10, dtype=torch.float32, device=cuda_device))
    c.close()
    assert not no_torch_collectives


@pytest.mark.parametrize("find_unused", [False, True])
def test_ddp_control_plane_through_the_communicator(pg, cuda_device, no_torch_collectives, find_unused):
    from distributed_training_amd import DistributedDataParallel, FusedSGD
    from distributed_training_amd.ddp import xgmi_bucket_caps
    from distributed_training_amd.resnet import micro_resnet

    torch.manual_seed(0)
    model = micro_resnet().to(cuda_device)
    ddp = DistributedDataParallel(model, find_unused_parameters=find_unused)
    assert ddp._comm is not None
    ddp.enable_bucket_checksums()
    opt = FusedSGD(ddp.parameters(), lr=0.05, momentum=0.9)
    ddp.world_size = 2  # rank 0 of a pretend world of two: the N>1 branches run
    try:
        ddp._verify_param_shape_across_processes()
        ddp._sync_module_states()
        g = torch.Generator(device=cuda_device).manual_seed(1)
        for step in range(3):  # step 1: the rebuild + rank-0 layout broadcast
            x = torch.rand(4, 3, 32, 32, device=cuda_device, generator=g)
            y = torch.randint(0, 10, (4,), device=cuda_device, generator=g)
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
            ddp.verify_bucket_checksums()
            opt.step()
            opt.zero_grad(set_to_none=True)
        assert ddp._has_rebuilt_buckets or find_unused
        cal = xgmi_bucket_caps(ddp._calib_allreduce, 8)
        assert cal["bus_GBps"] > 0
    finally:
        ddp.world_size = 1
    torch.cuda.synchronize()
    assert not no_torch_collectives
    ddp.close()
