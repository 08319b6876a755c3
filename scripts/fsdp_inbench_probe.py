"""Which earlier leg of the bench process leaves torch FSDP's configs[3] step slow
(108 ms a step in-process, r6d / r6f, against 81.5 ms standalone, r6e; a fresh
process with libgsync streams, communicators and a libgsync DDP run stays at
80-81 ms, scripts/fsdp_queue_probe.py): runs `bench.py`'s default N=1 flow with
every leg function wrapped so that the same FSDP(SHARD_GRAD_OP, bf16) + clip +
fused AdamW step (ResNet-50 x 256) is timed right after it.  The bench line goes
to stdout as usual; one "[fsdp-probe]" JSON line per leg to stderr.

    python scripts/fsdp_inbench_probe.py 2> probe.err > bench.json
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from distributed_training_amd.resnet import MODELS  # noqa: E402


def fsdp_time(label, steps=10, warmup=4):
    from torch.distributed.fsdp import FullyShardedDataParallel as FSDP, MixedPrecision, ShardingStrategy

    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(0)
    bf = torch.bfloat16
    model = MODELS["resnet50"](num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    fsdp = FSDP(model, sharding_strategy=ShardingStrategy.SHARD_GRAD_OP, device_id=dev,
                mixed_precision=MixedPrecision(param_dtype=bf, reduce_dtype=bf, buffer_dtype=bf))
    opt = torch.optim.AdamW(fsdp.parameters(), fused=True, **bench.DS_ADAM)
    g = torch.Generator(device=dev).manual_seed(4321)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last).to(bf)
    y = torch.randint(0, 1000, (256,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()

    parts = {"forward": [], "backward": [], "clip": [], "step": []}

    def one(timed=False):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if timed else None
        if timed:
            ev[0].record()
        loss = crit(fsdp(x).float(), y)
        if timed:
            ev[1].record()
        loss.backward()
        if timed:
            ev[2].record()
        fsdp.clip_grad_norm_(1.0)
        if timed:
            ev[3].record()
        opt.step()
        opt.zero_grad(set_to_none=True)
        if timed:
            ev[4].record()
            return ev

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    st0 = torch.cuda.memory_stats()
    t0 = time.perf_counter()
    evs = [one(timed=True) for _ in range(steps)]
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    for ev in evs:
        for k, name in enumerate(parts):
            parts[name].append(ev[k].elapsed_time(ev[k + 1]))
    st = torch.cuda.memory_stats()
    print("[fsdp-probe] " + json.dumps({"after": label, "ms_per_step": round(ms, 2),
                                        "parts_ms": {k: round(sum(v) / len(v), 2) for k, v in parts.items()},
                                        "device_allocs_in_timed": st.get("num_device_alloc", 0) - st0.get("num_device_alloc", 0),
                                        "device_frees_in_timed": st.get("num_device_free", 0) - st0.get("num_device_free", 0),
                                        "reserved_GB": round(st.get("reserved_bytes.all.current", 0) / 1e9, 2),
                                        "segments": st.get("segment.all.current"),
                                        "alloc_retries": st.get("num_alloc_retries")}), file=sys.stderr, flush=True)
    del fsdp, opt, model
    torch.cuda.empty_cache()


def wrap(name, before=False):
    orig = getattr(bench, name)

    def f(*a, **k):
        if before:
            fsdp_time("the headline (before " + name + ")")
        out = orig(*a, **k)
        fsdp_time(name)
        return out

    setattr(bench, name, f)


wrap("grad_sync_kernel_rates", before=True)
for name in ("zero2_leg", "colossal_leg", "torch_ddp_leg", "torch_colossal_leg"):
    wrap(name)
sys.argv = ["bench.py", "--cpu-baseline", "0"]
bench.main()
