"""bench.py's self-checked step on the real RCCL path with N >= 2 GPUs
(skipped on a one-GPU box: RCCL refuses two ranks on one device).

The driver's N = 2/4/8 runs launch bench.py exactly like this; after the timed
region every rank runs one step whose averaged grads (libgsync's RCCL
all-reduce, or reduce-scatter + all-gather for ZeRO-2) are checked against
Σ_r g_r·float(1/ws) gathered through the same communicator, and whose
post-step weights / BN buffers are checked identical across ranks
(distributed_training_amd/parity.py).  Reference: R:resnet/pytorch_ddp/
ddp_train.py:84,95,109-114 (NCCL DDP, world size 2) and
R:resnet/deepspeed/deepspeed_train.py:210-219 (ZeRO reduce-scatter)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = min(torch.cuda.device_count(), 8)  # device_count() does not initialise the GPU


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.skipif(N < 2, reason="needs >= 2 GPUs (RCCL: one rank per device)")
@pytest.mark.parametrize("engine", ["ddp", "zero2"])
def test_bench_rccl_parity_multi_gpu(engine):
    env = {k: v for k, v in os.environ.items()
           if k not in ("MASTER_PORT", "RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK")}
    env["MASTER_ADDR"] = "127.0.0.1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(N),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(N),
           "--model", "resnet18", "--batch", "16", "--steps", "3", "--warmup", "2", "--engine", engine,
           "--cpu-baseline", "0", "--collective-bench", "0"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    par = lines[0]["parity"]
    assert par["collective"] == "rccl(libgsync)" and par["world"] == N, par
    assert par["ok"] and par["weights_identical"], par
    if N == 2 and engine == "ddp":
        assert par["averaged_grads"]["bitwise_equal"], par
    g = lines[0]["grad_sync"]
    if engine == "ddp":
        assert g["allreduce_bus_GBps"] > 0 and g["xgmi_peak_GBps"] == (N - 1) * 153.0
        # the same run times BASELINE configs[3] and [4] on its ranks (bench.py legs)
        for leg in ("zero2", "colossal"):
            assert lines[0][leg]["parity"]["ok"] is True, (leg, lines[0][leg]["parity"])
            assert lines[0][leg]["parity"]["collective"] == "rccl(libgsync)"
        assert "leg_errors" not in lines[0], lines[0].get("leg_errors")
