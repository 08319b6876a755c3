"""The RCCL watchdog (SURVEY.md §5 failure detection) on the GPU: marks that ride
on kernels instead of event packets, and stalls that must still abort.

* ZeRO-2's step-end collectives hand their marks to the consuming kernels
  (gs_allreduce_marked / gs_all_gather_marked / gs_bucketer_set_mark_consumer):
  steps queued back to back with a short timeout complete without a false abort,
  with the same weights as the packet form (round 5's).
* A collective stalled behind a long kernel while the host keeps queueing is
  aborted within the timeout — ZeRO (its reduce-scatter's mark on the update)
  and DDP with more buckets than the watchdog queries per poll (the overdue
  entry is found while the others rotate), each on a private communicator.
* A deferred mark whose consumer never launches gets the watchdog's own packet
  after half the timeout (at most 1 s), so a stall there still aborts.

The stall is a spin kernel (torch.cuda._sleep) ahead of the step on its stream;
with one rank RCCL's collectives touch only the caller's buffers, and the
communicator's resources are freed only once the device is idle.
"""
import time

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

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


def _micro(dtype=torch.float32):
    from distributed_training_amd.resnet import BasicBlock, ResNet

    return ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, width=8).to(dtype)


def _spin_cycles(seconds):
    """torch.cuda._sleep cycles for about `seconds` of GPU time (calibrated here)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    torch.cuda._sleep(2_000_000)
    b.record()
    torch.cuda.synchronize()
    per_ms = 2_000_000 / max(a.elapsed_time(b), 1e-3)
    return int(per_ms * seconds * 1e3)


def _zero(dev, comm, **kw):
    from distributed_training_amd.zero import ZeroDataParallel

    torch.manual_seed(0)
    m = _micro(torch.bfloat16).to(dev)
    z = ZeroDataParallel(m, stage=2, optimizer="adamw", lr=1e-3, gradient_clipping=1.0, reduce_bucket_size=30000,
                         communicator=comm, **kw)
    return m, z


def test_zero_marks_on_consumers_queued_steps(cuda_device, rccl_pg):
    """Eight steps queued back to back with a 400 ms timeout: the reduce-scatters'
    marks on the update, the all-gathers' on the next backward's first pack — no
    false abort after waiting past the timeout, and the weights equal the packet
    form's (the marks change no arithmetic)."""
    from distributed_training_amd.comm import Communicator

    comm = Communicator(None, cuda_device, timeout_ms=400)
    g = torch.Generator(device=cuda_device).manual_seed(1)
    x = torch.rand(8, 3, 32, 32, device=cuda_device, generator=g).to(torch.bfloat16)
    y = torch.randint(0, 10, (8,), device=cuda_device, generator=g)
    finals = []
    for packets in (False, True):
        m, z = _zero(cuda_device, comm)
        z.set_mark_packets(packets)
        assert z.mark_packets is packets and len(z.buckets) > 1
        for _ in range(8):
            z.prepare_backward()
            nn.functional.cross_entropy(m(x).float(), y).backward()
            z.step()
        torch.cuda.synchronize()
        time.sleep(0.6)
        assert comm.status() == (False, ""), packets
        finals.append([p.detach().clone() for p in m.parameters()])
        z.close()
    # backward is not bitwise run to run on MIOpen; the update path is: compare loosely
    for a, b in zip(*finals):
        assert torch.allclose(a.float(), b.float(), rtol=0, atol=5e-2)
    comm.close()


def test_zero_stalled_collective_aborts(cuda_device, rccl_pg):
    """A step queued behind a 2 s kernel with a 300 ms timeout: the reduce-scatter's
    mark (on the update kernel) is overdue and the watchdog aborts the communicator;
    later calls fail with the reason."""
    from distributed_training_amd import _lib as L
    from distributed_training_amd.comm import Communicator

    comm = Communicator(None, cuda_device, timeout_ms=300)
    m, z = _zero(cuda_device, comm)
    x = torch.rand(8, 3, 32, 32, device=cuda_device).to(torch.bfloat16)
    y = torch.randint(0, 10, (8,), device=cuda_device)
    z.prepare_backward()
    nn.functional.cross_entropy(m(x).float(), y).backward()
    z.step()
    torch.cuda.synchronize()
    cycles = _spin_cycles(2.0)
    torch.cuda._sleep(cycles)  # the stall: everything below queues behind it
    z.prepare_backward()
    nn.functional.cross_entropy(m(x).float(), y).backward()
    z.step()
    time.sleep(1.0)
    aborted, why = comm.status()
    assert aborted and "in flight" in why, why
    torch.cuda.synchronize()
    with pytest.raises(L.GsyncError, match="aborted"):
        comm.all_reduce(torch.ones(4, device=cuda_device))
    z.close()
    comm.close()


def test_deferred_mark_without_consumer_launch_aborts(cuda_device, rccl_pg):
    """A collective whose mark is deferred to a consumer plan that never launches
    (the host blocked or idle between them — a loss.item() before the next
    backward) is still watched: past about half the timeout the watchdog records
    a packet on the collective's stream itself, timed from the enqueue, and a
    stall aborts within the timeout.  Without a stall the packet completes and
    nothing aborts."""
    from distributed_training_amd import _lib as L
    from distributed_training_amd.comm import Communicator
    from distributed_training_amd.multi_tensor import TensorListPlan

    plan = TensorListPlan([4096], cuda_device)
    buf = torch.ones(1024, device=cuda_device)
    stream = torch.cuda.current_stream(cuda_device).cuda_stream
    # no stall: the lapsed deferral's packet completes, no abort
    ok = Communicator(None, cuda_device, timeout_ms=400)
    ok.all_reduce(buf, stream=stream, consumer=plan.handle)
    torch.cuda.synchronize()
    time.sleep(1.0)
    assert ok.status() == (False, "")
    ok.close()
    # the stall: the collective queued behind a 2 s kernel, its consumer never launched
    comm = Communicator(None, cuda_device, timeout_ms=400)
    torch.cuda._sleep(_spin_cycles(2.0))
    comm.all_reduce(buf, stream=stream, consumer=plan.handle)
    time.sleep(1.2)
    aborted, why = comm.status()
    assert aborted and "in flight" in why, why
    torch.cuda.synchronize()
    with pytest.raises(L.GsyncError, match="aborted"):
        comm.all_reduce(buf)
    comm.close()
    del plan


def test_ddp_stall_many_buckets_aborts(cuda_device, rccl_pg):
    """DDP with more buckets than the watchdog queries per poll (its unpack-carried
    marks rotate through the query budget), three steps queued behind a 2 s kernel:
    an overdue mark is still found and the communicator aborted within the timeout."""
    from distributed_training_amd import DistributedDataParallel

    torch.manual_seed(0)
    m = _micro().to(cuda_device)
    # rccl_max_ctas: the DDP's own communicator (aborting it leaves the shared one alone)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.004, rccl_max_ctas=8)
    assert ddp._own_comm and len(ddp.bucket_indices()) >= 1
    x = torch.rand(8, 3, 32, 32, device=cuda_device)
    y = torch.randint(0, 10, (8,), device=cuda_device)
    for _ in range(2):  # the first step rebuilds the buckets in ready order
        nn.functional.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    n_buckets = len(ddp.bucket_indices())
    assert n_buckets > 4, n_buckets
    comm = ddp._comm
    comm.set_timeout(300)
    cycles = _spin_cycles(2.0)
    torch.cuda._sleep(cycles)
    for _ in range(3):
        nn.functional.cross_entropy(ddp(x), y).backward()
    time.sleep(1.0)
    aborted, why = comm.status()
    assert aborted and "in flight" in why, (n_buckets, why)
    torch.cuda.synchronize()
    ddp.close()
